#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/*.npz.

The reference's arithmetic for this path lives in warp-ctc and cuDNN, neither
of which is in /root/reference nor installable offline, and
the reference holds no golden vectors for it.  The fixtures are
therefore produced by torch 2.10 on the CPU in float64 -- an independent
implementation of the same published equations:

  * CTC: F.ctc_loss(log_softmax(acts), blank=0, reduction='none') with autograd
    back to the un-normalised activations == warp-ctc compute_ctc_loss's
    cost and gradient (src/ctc/ctc-nnet-update.cc:224-231).
  * RNN: nn.LSTM / nn.GRU / nn.RNN(relu|tanh), whose gate orders (i,f,g,o) /
    (r,z,n) and GRU r*(W_hn h + b_hn) form are the cuDNN-v5 equations; weights
    are mapped to the cuDNN opaque layout used by CuDNNRecurrentComponent
    (src/nnet2/nnet-cudnn-component.cc:327-413).
  * The cfg0 train step (1 x uni-LSTM-256, N=2, T_max=200, D=40, A=41):
    Splice -> LSTM -> ClipGradient(norm, 30) -> Affine -> CTC, backprop,
    RNN dW clipped to +-5, SGD at lr 5e-4 (NnetCtcUpdater::ComputeForMinibatch).

Inputs are stored as float32 (the dtype the path consumes), outputs as
float64.  Run:  python tests/golden/make_golden.py
"""
import os

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
torch.set_default_dtype(torch.float64)

MODES = {"relu": 0, "tanh": 1, "lstm": 2, "gru": 3}
NW = {0: 1, 1: 1, 2: 4, 3: 3}


def ctc_torch(acts, labels_list, in_lens):
    """acts [T,N,A] float64 -> (costs [N], grads [T,N,A])."""
    x = torch.tensor(acts, requires_grad=True)
    lp = F.log_softmax(x, dim=-1)
    flat = torch.tensor([l for ls in labels_list for l in ls], dtype=torch.long)
    tl = torch.tensor([len(ls) for ls in labels_list], dtype=torch.long)
    il = torch.tensor(in_lens, dtype=torch.long)
    loss = F.ctc_loss(lp, flat, il, tl, blank=0, reduction="none", zero_infinity=False)
    loss.sum().backward()
    return loss.detach().numpy(), x.grad.detach().numpy()


def make_labels(rng, L, A, repeats):
    out = []
    for i in range(L):
        if repeats and i > 0 and rng.random() < 0.3:
            out.append(out[-1])
            continue
        while True:
            v = int(rng.integers(1, A))
            if repeats or not out or v != out[-1]:
                break
        out.append(v)
    return out


def ctc_cases(rng):
    cases = []
    # (name, T_max, N, A, per-utt (T_n, L_n), repeats)
    specs = [
        ("basic", 30, 3, 6, [(30, 5), (25, 8), (12, 3)], False),
        ("repeats", 40, 3, 5, [(40, 10), (33, 6), (20, 7)], True),
        ("empty_label", 10, 2, 4, [(10, 0), (7, 2)], False),
        ("tight", 21, 2, 8, [(21, 10), (9, 4)], False),       # T = 2L+1 exactly
        ("tight_repeat", 12, 1, 3, [(12, 6)], True),
        ("a41", 120, 4, 41, [(120, 15), (110, 12), (64, 8), (1, 0)], False),
        ("long", 400, 2, 41, [(400, 50), (377, 47)], True),
    ]
    for name, T, N, A, per, rep in specs:
        acts = rng.standard_normal((T, N, A)).astype(np.float32) * 2.0
        labels, in_lens = [], []
        for (tn, ln) in per:
            labels.append(make_labels(rng, ln, A, rep))
            in_lens.append(tn)
        costs, grads = ctc_torch(acts.astype(np.float64), labels, in_lens)
        cases.append(dict(name=name, acts=acts,
                          flat_labels=np.array([l for ls in labels for l in ls], dtype=np.int32),
                          label_lengths=np.array([len(l) for l in labels], dtype=np.int32),
                          input_lengths=np.array(in_lens, dtype=np.int32),
                          costs=costs, grads=grads))
    return cases


def torch_rnn(mode, D, H, layers, bidir):
    kw = dict(input_size=D, hidden_size=H, num_layers=layers, bidirectional=bidir, batch_first=False)
    if mode == 2:
        return torch.nn.LSTM(**kw)
    if mode == 3:
        return torch.nn.GRU(**kw)
    return torch.nn.RNN(nonlinearity="relu" if mode == 0 else "tanh", **kw)


def cudnn_flat(m, mode, layers, dirs):
    """torch params -> cuDNN-v5 opaque layout: per pseudo-layer
    [W (nW*H x Din) | R (nW*H x H) | bW (nW*H) | bR (nW*H)]."""
    parts = []
    for l in range(layers):
        for d in range(dirs):
            sfx = f"_l{l}" + ("_reverse" if d == 1 else "")
            parts += [getattr(m, "weight_ih" + sfx).detach().reshape(-1),
                      getattr(m, "weight_hh" + sfx).detach().reshape(-1),
                      getattr(m, "bias_ih" + sfx).detach().reshape(-1),
                      getattr(m, "bias_hh" + sfx).detach().reshape(-1)]
    return torch.cat(parts)


def cudnn_flat_grad(m, layers, dirs):
    parts = []
    for l in range(layers):
        for d in range(dirs):
            sfx = f"_l{l}" + ("_reverse" if d == 1 else "")
            parts += [getattr(m, n + sfx).grad.reshape(-1)
                      for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    return torch.cat(parts)


def rnn_case(rng, name, mode, T, N, D, H, layers, bidir):
    dirs = 2 if bidir else 1
    m = torch_rnn(mode, D, H, layers, bidir)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.tensor(rng.standard_normal(tuple(p.shape)).astype(np.float32) * 0.3))
    x32 = rng.standard_normal((T, N, D)).astype(np.float32)
    dy32 = rng.standard_normal((T, N, dirs * H)).astype(np.float32)
    x = torch.tensor(x32.astype(np.float64), requires_grad=True)
    y, _ = m(x)
    (y * torch.tensor(dy32.astype(np.float64))).sum().backward()
    w = cudnn_flat(m, mode, layers, dirs).numpy().astype(np.float32)
    return dict(name=name, mode=mode, T=T, N=N, D=D, H=H, layers=layers, dirs=dirs,
                x=x32, w=w, dy=dy32, y=y.detach().numpy(), dx=x.grad.numpy(),
                dw=cudnn_flat_grad(m, layers, dirs).numpy())


class ClipGrad(torch.autograd.Function):
    """ClipGradientComponent, norm-based (nnet-cudnn-component.cc:921-970)."""

    @staticmethod
    def forward(ctx, x, thr):
        ctx.thr = thr
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        ss = (g * g).sum(dim=-1, keepdim=True) / (ctx.thr ** 2)
        scale = torch.where(ss < 1.0, torch.ones_like(ss), ss.rsqrt())
        return g * scale, None


def cfg0_step(rng):
    """configs[0]: 1 x uni-LSTM-256, N=2, T_max=200, D=40, A=41, T_n = {200, 180}."""
    T, N, D, H, A = 200, 2, 40, 256, 41
    lens = [200, 180]
    m = torch_rnn(2, D, H, 1, False)
    with torch.no_grad():   # reference init: W ~ N(0, 0.02^2), biases 0.2
        for name, p in m.named_parameters():
            if name.startswith("weight"):
                p.copy_(torch.tensor(rng.standard_normal(tuple(p.shape)).astype(np.float32) * 0.02))
            else:
                p.fill_(0.2)
    Wa32 = (rng.standard_normal((A, H)) / np.sqrt(H)).astype(np.float32)
    ba32 = rng.standard_normal(A).astype(np.float32)
    feats = rng.standard_normal((T, N, D)).astype(np.float32)
    for n, tn in enumerate(lens):
        feats[tn:, n, :] = 0.0      # FormatNnetInput zero padding
    labels = [make_labels(rng, tn // 8, A, False) for tn in lens]
    w0 = cudnn_flat(m, 2, 1, 1).numpy().astype(np.float32)
    Wa = torch.tensor(Wa32.astype(np.float64), requires_grad=True)
    ba = torch.tensor(ba32.astype(np.float64), requires_grad=True)
    y, _ = m(torch.tensor(feats.astype(np.float64)))
    yc = ClipGrad.apply(y, 30.0)
    logits = yc @ Wa.T + ba
    lp = F.log_softmax(logits, dim=-1)
    flat = torch.tensor([l for ls in labels for l in ls], dtype=torch.long)
    costs = F.ctc_loss(lp, flat, torch.tensor(lens), torch.tensor([len(l) for l in labels]),
                       blank=0, reduction="none")
    costs.sum().backward()
    lr = 5e-4
    dw = -cudnn_flat_grad(m, 1, 1)                    # deriv is -grad (ctc-nnet-update.cc:323)
    # parameter deltas of the SGD update (stored float32: w1 = w0 + delta)
    w_delta = (lr * dw.clamp(-5.0, 5.0)).numpy().astype(np.float32)
    Wa_delta = (-lr * Wa.grad).numpy().astype(np.float32)
    ba_delta = (-lr * ba.grad).numpy().astype(np.float32)
    return dict(name="cfg0", T=T, N=N, D=D, H=H, A=A, feats=feats,
                num_frames=np.array(lens, dtype=np.int32),
                flat_labels=np.array([l for ls in labels for l in ls], dtype=np.int32),
                label_lengths=np.array([len(l) for l in labels], dtype=np.int32),
                w0=w0, Wa0=Wa32, ba0=ba32, logits=logits.detach().numpy(),
                costs=costs.detach().numpy(), w_delta=w_delta, Wa_delta=Wa_delta, ba_delta=ba_delta,
                lr=np.float64(lr))


def save(name, d):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in d.items()})
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    rng = np.random.default_rng(20161015)
    for c in ctc_cases(rng):
        save("ctc_" + c["name"], c)
    rnn_specs = [
        ("lstm_bi", 2, 9, 3, 5, 8, 1, True),
        ("lstm_uni", 2, 7, 2, 4, 6, 1, False),
        ("lstm_bi_2layer", 2, 6, 2, 3, 5, 2, True),
        ("gru_bi", 3, 8, 3, 5, 7, 1, True),
        ("gru_uni_2layer", 3, 6, 2, 4, 5, 2, False),
        ("relu_bi", 0, 7, 2, 4, 6, 1, True),
        ("tanh_bi", 1, 7, 3, 5, 6, 1, True),
        ("lstm_bi_h32", 2, 20, 4, 24, 32, 1, True),
    ]
    for (name, mode, T, N, D, H, layers, bidir) in rnn_specs:
        save("rnn_" + name, rnn_case(rng, name, mode, T, N, D, H, layers, bidir))
    save("step_cfg0", cfg0_step(rng))


if __name__ == "__main__":
    main()
