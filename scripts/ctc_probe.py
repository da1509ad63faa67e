"""CTC alpha/beta timing probe at the configs[1] shape (T=2000, N=16, A=41,
L = T/8): compute_ctc_loss with and without gradients (alpha+beta with the
column spill vs alpha alone), for rocprofv3 --kernel-trace --stats; also
prints the event-timed mean per call."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

pkg = g.load_package()
rng = np.random.default_rng(3)
T, N, A = 2000, 16, 41
lens = np.array([T - int(u * 0.1 * T) for u in rng.uniform(size=N)], np.int32)
ll = (lens // 8).astype(np.int32)
fl = np.concatenate([rng.integers(1, A, size=l) for l in ll]).astype(np.int32)
acts = torch.randn(T, N, A, device="cuda")
ws = torch.empty(pkg.ctc_workspace_size(ll, lens, A), dtype=torch.uint8, device="cuda")
for win, want in ((1, True), (0, True), (1, False), (0, False)):
    pkg.ctc_window_kernel(win)
    for _ in range(3):
        pkg.compute_ctc_loss(acts, fl, ll, lens, want_grad=want, workspace=ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        pkg.compute_ctc_loss(acts, fl, ll, lens, want_grad=want, workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    print(f"compute_ctc_loss {'window' if win else 'halo'} kernel, want_grad={want}: "
          f"{e0.elapsed_time(e1) / 20:.4f} ms per call (host launch gaps included)")
print("ctc probe done")
