"""Where bf16 direct packing differs from the pack path: per-component max |diff| after 1 step."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
kctc = importlib.import_module("kaldi-ctc_amd")
import torch

mode, H, N, T = int(os.environ.get("BP_MODE", "3")), 1024, 32, 120
cfg = kctc.recipe_config(num_rnn=2, input_dim=40, hidden=H, num_targets=41, learning_rate=5e-4, max_seq_length=T, rnn_mode=mode)
feats, nf, fl, ll = kctc.synth_minibatch(17 + N, T, N, 40, 41, 0.125)
f = torch.from_numpy(feats).to("cuda:0")
res = {}
for tag, env in [("off", {"KCTC_BF16_DIRECT": "0"}), ("direct", {"KCTC_BF16_DIRECT": "1", "KCTC_BF16_IO": "0"}),
                 ("io", {"KCTC_BF16_DIRECT": "1", "KCTC_BF16_IO": "1"})]:
    os.environ.update(env)
    net = kctc.Nnet(cfg, seed=3)
    net.set_precision("bf16")
    st = net.train_step(f, T, N, nf, fl, ll)
    res[tag] = (st, [net.get_params(c) for c in range(net.num_components) if net.num_params(c)])
    net.close()
    if tag != "off":
        d = [float(np.max(np.abs(a - b))) for a, b in zip(res[tag][1], res["off"][1])]
        print(tag, "stats equal", st == res["off"][0], "max|diff| per component", ["%.3g" % x for x in d], flush=True)
