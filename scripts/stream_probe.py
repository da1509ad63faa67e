"""One train step of a small 2 x BLSTM-256 net (streamed GEMM diagnostics)."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
import importlib
kctc = importlib.import_module("kaldi-ctc_amd")
T, N, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cfg = kctc.recipe_config(num_rnn=2, input_dim=24, hidden=H, num_targets=11, learning_rate=0.02, param_stddev=0.1)
net = kctc.Nnet(cfg, seed=5)
feats, nf, fl, ll = kctc.synth_minibatch(1000, T, N, 24, 11, 0.2)
f = torch.from_numpy(feats).cuda()
t0 = time.time()
print("objf", net.compute_objf(f, T, N, nf, fl, ll), time.time() - t0, flush=True)
t0 = time.time()
print("step", net.train_step(f, T, N, nf, fl, ll), time.time() - t0, flush=True)
