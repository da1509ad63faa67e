#!/usr/bin/env python3
"""Time the packed gate GEMM alone (kcm_bench_gemm_packed) on the train
step's shapes: split-fp16 (configs[1]) and bf16 (configs[4]).  TF/s are of
the 2MNK product (fp32-class for x3; the f16 issue rate is 3x that)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge

k = ge.load_package()
L = k.lib()
torch.zeros(1, device="cuda:0")
SHAPES = [  # (name, M, N, K, bf16, split)
    ("c1_proj0", 32000, 4096, 40, 0, 1),     # layer 0 (D = 40): output-bound
    ("c1_fwd_proj", 32000, 2048, 1024, 0, 1),
    ("c1_bwd_data", 32000, 1024, 2048, 0, 1),
    ("c1_bwd_w", 2048, 1024, 32000, 0, 8),
    ("c1_bwd_r", 2048, 512, 32000, 0, 16),
    ("c4_proj0", 64000, 6144, 40, 1, 1),
    ("c4_fwd_proj", 64000, 3072, 2048, 1, 1),
    ("c4_bwd_data", 64000, 2048, 3072, 1, 1),
    ("c4_bwd_w", 3072, 2048, 64000, 1, 4),
    ("c4_bwd_r", 3072, 1024, 64000, 1, 8),
    ("sq8192_bf16", 8192, 8192, 8192, 1, 1),
    ("sq8192_x3", 8192, 8192, 8192, 0, 1),
]
pick = sys.argv[1:]  # shape names (default: all)
for name, M, N, K, bf, sp in SHAPES:
    if pick and name not in pick:
        continue
    ms = L.kcm_bench_gemm_packed(None, M, N, K, bf, 10, sp)
    tf = 2.0 * M * N * K / ms / 1e9 if ms > 0 else 0.0
    f16 = tf * (1 if bf else 3)
    print(f"{name:12s} {'bf16' if bf else 'x3  '} M={M} N={N} K={K} split={sp}: {ms:.3f} ms  {tf:.1f} TF "
          f"(MFMA issue {f16:.0f} TF = {f16 / 2500:.3f} of 2.5 PF)", flush=True)
