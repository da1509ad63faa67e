"""Localise a parameter-gradient mismatch of a CuDNNRecurrentComponent: the
central difference of objf along a random direction confined to one lin-layer
region (W / R / bW / bR of each pseudo-layer) vs the gradient holder's dot."""
import sys
import numpy as np
import torch
sys.path.insert(0, "tests")
from conftest import load_kctc

k = load_kctc()
T, N = int(sys.argv[1]), int(sys.argv[2])
D, H, mode = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 2
line = (f"CuDNNRecurrentComponent input-dim={D} output-dim={H} bidirectional=true max-seq-length=2000 "
        f"learning-rate=0.0005 rnn-mode={mode} num-layers=1 param-stddev=0.02 bias-stddev=0.2 clip-gradient=1e30")
gpu = torch.device("cuda:0")
comp = k.Component(line, seed=7)
g = torch.Generator(device=gpu)
g.manual_seed(11)
x = torch.randn((T * N, D), generator=g, device=gpu)
v = torch.randn((2 * H,), generator=g, device=gpu)
f = lambda c: float((c.Propagate(T, N, x).double() @ v.double()).sum())
y = comp.Propagate(T, N, x)
grad = comp.Copy()
grad.SetZero(True)
comp.Backprop(T, N, x, y, v.expand(T * N, -1).contiguous(), grad, torch.empty_like(x))
gv = grad.Vectorize().astype(np.float64)
p0 = comp.Vectorize()
r = k.Rnn(mode, D, H, 1, True)
nlin = 8 if mode == 2 else 6
rng = np.random.default_rng(3)
for pl in range(2):
    for lin in range(nlin):
        for isb in (0, 1):
            off, (a, b) = r.lin_offset(pl, lin, isb)
            n = a * b
            d = np.zeros_like(p0)
            d[off:off + n] = rng.standard_normal(n) * 1e-3
            comp.UnVectorize(p0 + d); fp = f(comp)
            comp.UnVectorize(p0 - d); fm = f(comp)
            obs = (fp - fm) / 2
            pred = float(d.astype(np.float64) @ gv)
            print(f"pl {pl} lin {lin} bias {isb}: pred {pred:+.6e} obs {obs:+.6e} rel {abs(pred-obs)/max(abs(obs),1e-30):.2e}")
comp.UnVectorize(p0)
