"""One gated-projection train step per setting, under the caller's timeout:
prints the step's wall time and whether the parameters equal the ungated run."""
import faulthandler, os, sys, time
faulthandler.enable()
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib
kctc = importlib.import_module("kaldi-ctc_amd")
import torch

mode, N, T, R = 2, 16, int(os.environ.get("GP_T", "64")), 2
cfg = kctc.recipe_config(num_rnn=R, input_dim=40, hidden=512, num_targets=41, learning_rate=5e-4,
                         max_seq_length=T, rnn_mode=mode)
feats, nf, fl, ll = kctc.synth_minibatch(3, T, N, 40, 41, 0.125)
f = torch.from_numpy(feats).to("cuda:0")
res = {}
for tag in sys.argv[1:]:
    os.environ["KCTC_FWD_GATE"] = "0" if tag == "off" else "1"
    os.environ["KCTC_GATE_DIAG"] = {"d1": "1", "d2": "2", "d4": "4", "d5": "5"}.get(tag, "0")
    print("start", tag, flush=True)
    net = kctc.Nnet(cfg, seed=5)
    t0 = time.time()
    try:
        st = net.train_step(f, T, N, nf, fl, ll)
        torch.cuda.synchronize()
    except Exception as e:
        print(tag, "FAILED", repr(e), flush=True)
        net.close()
        continue
    res[tag] = [net.get_params(c) for c in range(net.num_components) if net.num_params(c)]
    same = all(np.array_equal(a, b) for a, b in zip(res[tag], res["off"])) if "off" in res else None
    print(tag, f"{time.time() - t0:.2f}s", "same_as_off", same, flush=True)
    net.close()
