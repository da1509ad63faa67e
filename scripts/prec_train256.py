#!/usr/bin/env python3
"""Diagnostic: H=256 train-step parameter/delta errors vs the fp64 oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, ROOT)
import numpy as np, torch
import oracle_lib as oracle
from conftest import load_kctc, rel_err
from test_train_gpu import splitmix_uniforms, _oracle_spec
kctc = load_kctc()
gpu = torch.device("cuda:0")
for mode, H, pstd in ((2, 256, 0.1), (3, 256, 0.1), (2, 256, 0.05)):
    R, D, A, T, N, lr, thr, steps = 2, 24, 11, 30, 4, 0.02, 30.0, 2
    cfg = kctc.recipe_config(num_rnn=R, input_dim=D, hidden=H, num_targets=A, rnn_mode=mode,
                             learning_rate=lr, clipping_threshold=thr, param_stddev=pstd)
    net = kctc.Nnet(cfg, seed=5)
    net.set_repair_seed(99)
    draws = splitmix_uniforms(99, steps * R)
    upd = [c for c in range(net.num_components) if net.num_params(c) > 0]
    params = [net.get_params(c).astype(np.float64) for c in upd]
    init = [p.copy() for p in params]
    spec = _oracle_spec(oracle, R, mode, H, 2, D, A, thr, lr)
    cnc, cc = np.zeros(R), np.zeros(R)
    for step in range(steps):
        feats, nf, fl, ll = kctc.synth_minibatch(1000 + step, T, N, D, A, 0.2)
        objf, acc, wt = net.train_step(torch.from_numpy(feats).to(gpu), T, N, nf, fl, ll)
        d = draws[step * R:(step + 1) * R][::-1]
        aff = params[-1]
        Wa = aff[:-A].reshape(A, -1).copy(); ba = aff[-A:].copy()
        robjf, racc, rwt = oracle.train_step(spec, params[:-1], Wa, ba, feats.reshape(T, N, D).astype(np.float64),
                                             nf, fl, ll, repair_draws=np.array(d, np.float32),
                                             clip_num_clipped=cnc, clip_count=cc)
        params[-1] = np.concatenate([Wa.ravel(), ba])
        print(f"mode {mode} H {H} step {step}: objf rel {abs(objf - robjf) / abs(robjf):.2e}")
    for c, p, p0 in zip(upd, params, init):
        got = net.get_params(c).astype(np.float64)
        print(f"  comp {c}: params {rel_err(got, p):.2e}  deltas {rel_err(got - p0, p - p0):.2e}  |delta|/|p| {np.linalg.norm(p - p0) / np.linalg.norm(p):.2e}")
