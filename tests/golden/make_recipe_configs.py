"""Generate tests/golden/recipe_configs.json: the component config lines the
reference's own generator writes for the CTC recipe.

Runs in the build container only (it imports the reference's
egs/wsj/s5/steps/ctc/nnet2/components.py, stdlib-only, from /root/reference);
the committed JSON is text data and is all that travels.

The call sequence restates MakeConfigs (egs/wsj/s5/steps/ctc/nnet2/make_configs.py:
237-358) for model_type "google", rnn_first, no LDA, splice_indexes "0 0 0 ...":
  init.config   = AddInputLayer + AddRnnLayer(first: default learning-rate /
                  param-stddev / bias-stddev) + AddAffineLayer(num_targets)
  layer{i}.config (i = 1 .. rnn_layers-1) = AddRnnLayer(param/bias stddev passed)
  softmax.config = "SoftmaxComponent dim={num_targets}"
with the argument values of egs/wsj/s5/steps/ctc/train.sh:46-66 and its
make_configs.py call (:204-218): clipping_threshold is the float argparse
gives (30.0), norm_based_clipping the bool StrToBoolAction gives (True).
Configurations: BASELINE.json configs[0] (1 x uni-LSTM-256, max-seq-length
200), configs[1] (5 x BLSTM-512, max-seq-length 2000) and configs[4]
(5 x BGRU-1024, rnn-mode 3).
"""
import importlib.util
import json
import os
import sys

REF = "/root/reference/egs/wsj/s5/steps/ctc/nnet2/components.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "recipe_configs.json")


def load_components():
    spec = importlib.util.spec_from_file_location("ref_ctc_nnet2_components", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def make_configs(nodes, feat_dim, num_targets, rnn_layers, cell_dim, rnn_mode, bidirectional, max_seq_length,
                 cudnn_layers=1, param_stddev=0.02, bias_stddev=0.2, clipping_threshold=30.0,
                 norm_based_clipping=True, dropout_proportion=0.0):
    files = {}
    init = {"components": []}
    prev = nodes.AddInputLayer(init, feat_dim, [0], 0)
    first = nodes.AddRnnLayer(init, prev, cell_dim, num_layers=cudnn_layers, max_seq_length=max_seq_length,
                              bidirectional=bidirectional, rnn_mode=rnn_mode,
                              clipping_threshold=clipping_threshold, dropout_proportion=dropout_proportion,
                              norm_based_clipping=norm_based_clipping, self_repair_scale_clipgradient=None)
    nodes.AddAffineLayer(init, first, num_targets)
    files["init.config"] = init["components"]
    out = first
    for i in range(rnn_layers - 1):
        lines = {"components": []}
        out = nodes.AddRnnLayer(lines, out, cell_dim, num_layers=cudnn_layers, max_seq_length=max_seq_length,
                                bidirectional=bidirectional, rnn_mode=rnn_mode, param_stddev=param_stddev,
                                bias_stddev=bias_stddev, clipping_threshold=clipping_threshold,
                                dropout_proportion=dropout_proportion, norm_based_clipping=norm_based_clipping,
                                self_repair_scale_clipgradient=None)
        files[f"layer{i + 1}.config"] = lines["components"]
    files["softmax.config"] = [f"SoftmaxComponent dim={num_targets}"]
    return files


def main():
    nodes = load_components()
    cases = {
        "configs0": dict(feat_dim=40, num_targets=41, rnn_layers=1, cell_dim=256, rnn_mode=2, bidirectional=False,
                         max_seq_length=200),
        "configs1": dict(feat_dim=40, num_targets=41, rnn_layers=5, cell_dim=512, rnn_mode=2, bidirectional=True,
                         max_seq_length=2000),
        "configs4": dict(feat_dim=40, num_targets=41, rnn_layers=5, cell_dim=1024, rnn_mode=3, bidirectional=True,
                         max_seq_length=2000),
    }
    out = {"generator": "egs/wsj/s5/steps/ctc/nnet2/components.py via tests/golden/make_recipe_configs.py",
           "args": cases,
           "configs": {k: make_configs(nodes, **v) for k, v in cases.items()}}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
