#!/usr/bin/env python3
"""Time the fp32 and split-fp16 (x3) GEMMs on the train step's shapes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import __graft_entry__ as ge

k = ge.load_package()
dev = torch.device("cuda:0")
SHAPES = [  # (name, transA, transB, M, N, K)
    ("fwd_proj", 0, 1, 32000, 2048, 1024),
    ("bwd_data", 0, 0, 32000, 1024, 2048),
    ("bwd_w", 1, 0, 2048, 1024, 32000),
    ("bwd_r", 1, 0, 2048, 512, 32000),
]
for name, ta, tb, M, N, K in SHAPES:
    A = torch.randn((K, M) if ta else (M, K), device=dev)
    B = torch.randn((N, K) if tb else (K, N), device=dev)
    C = torch.empty((M, N), device=dev)
    for fn, lab in ((k.add_mat_mat, "f32"), (k.add_mat_mat_x3, "x3")):
        for _ in range(2):
            fn(C, A, B, bool(ta), bool(tb))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        n = 10
        for _ in range(n):
            fn(C, A, B, bool(ta), bool(tb))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        print(f"{name:9s} {lab:4s} M={M} N={N} K={K}: {ms:.3f} ms  {2.0*M*N*K/ms/1e9:.1f} TF(fp32-equiv)", flush=True)
