"""Full-size parity by sketches (TEST INFRASTRUCTURE).

The fp64 oracle needs minutes for a configs[1]-sized layer or train step, so
it runs once, here in the build container (tests/golden/make_sketch.py), and
only a SKETCH of each output tensor is committed (tests/golden/sketch_*.npz):
its norm, 4 projections onto fixed Gaussian vectors and 256 sampled entries.
The GPU tests regenerate the identical inputs (numpy PCG64 streams and the
library's host-side synthetic generator are deterministic across machines),
run the HIP path and compare sketches.

Why projections: for r ~ N(0, I), E[(r.a - r.b)^2] = |a - b|^2, so
|r.(y_gpu - y_ref)| / |y_ref| estimates the norm-wise relative error that
north_star bounds (1e-4), while a localised fault (one wrong row of 2H
entries among T*N) moves a projection by ~sqrt(2H / (T*N)) >> 1e-4.
"""
import numpy as np

NPROJ = 4
NSAMP = 256
# sampled entries: max |diff| / rms(ref) over NSAMP entries may exceed the
# norm-wise bar by this factor -- an entry's error scales with its own
# magnitude, and the largest of 256 sampled |entries| of a gradient runs to
# several times the rms (measured on the fp32 configs[1] step: the sampled
# error at most 0.56x the norm-wise bar, profiles/r02b_fullsize_parity.log)
SAMP_FACTOR = 10.0


def proj_vectors(n, seed):
    """The k-th projection vector of a tensor of n entries (float32 N(0,1))."""
    return [np.random.default_rng([seed, k, n]).standard_normal(n, dtype=np.float32) for k in range(NPROJ)]


def sample_index(n, seed):
    return np.random.default_rng([seed, 99, n]).integers(0, n, NSAMP)


def sketch(a, seed):
    """dict(norm, proj[NPROJ], idx[NSAMP], val[NSAMP]) of a flattened tensor."""
    a = np.ascontiguousarray(a).ravel()
    a64 = a.astype(np.float64)
    idx = sample_index(a.size, seed)
    return {"norm": float(np.linalg.norm(a64)),
            "proj": np.array([float(np.dot(r.astype(np.float64), a64)) for r in proj_vectors(a.size, seed)]),
            "idx": idx, "val": a64[idx]}


def save(prefix, sk, out):
    for k, v in sk.items():
        out[f"{prefix}.{k}"] = np.asarray(v)


def load(g, prefix):
    return {k: g[f"{prefix}.{k}"] for k in ("norm", "proj", "idx", "val")}


def compare(a, ref, seed, tol):
    """Max relative sketch error of tensor a vs the committed sketch ref:
    max(|norm diff|, max_k |proj diff|) / |ref| (bar: tol), and the sampled
    entries' max |diff| / rms(ref) (bar: SAMP_FACTOR * tol); ok = all three
    below their bars."""
    s = sketch(a, seed)
    n = np.asarray(a).size
    den = float(ref["norm"]) or 1.0
    e_norm = abs(s["norm"] - float(ref["norm"])) / den
    e_proj = float(np.max(np.abs(s["proj"] - ref["proj"]))) / den
    rms = den / np.sqrt(n)
    e_samp = float(np.max(np.abs(s["val"] - ref["val"]))) / rms
    return {"norm": e_norm, "proj": e_proj, "samp": e_samp,
            "ok": e_norm < tol and e_proj < tol and e_samp < SAMP_FACTOR * tol}


# ---- the two workloads --------------------------------------------------------
# (i) one BLSTM-512 layer at the configs[1] shape, D = 40 (first layer) and
#     D = 1024 (layers 2-5): recipe init (matrices N(0, 0.02^2), biases 0.2,
#     nnet-cudnn-component.cc:336-407), x = the synthetic features (D = 40) or
#     tanh(N(0,1)) (D = 1024, a bounded LSTM output), dy ~ N(0, 1e-2^2).
LAYER_CASES = {"lstm512_d40": dict(mode=2, T=2000, N=16, D=40, H=512, seed=11),
               "lstm512_d1024": dict(mode=2, T=2000, N=16, D=1024, H=512, seed=12),
               # configs[2]: frame_subsampling_factor 3 -> T_max 667, minibatch 64
               "lstm512_d1024_n64": dict(mode=2, T=667, N=64, D=1024, H=512, seed=13),
               # configs[4]: BGRU-1024 layers 2-5 (D = 2H), minibatch 32, run in bf16
               "gru1024_d2048_n32": dict(mode=3, T=2000, N=32, D=2048, H=1024, seed=14, prec="bf16")}


class ProductLayout:
    """params_size / lin_offset (the cuDNN-v5 opaque layout) through the
    library's own krnn ABI, for callers that must not load the oracle
    (bench.py's loss match); equal to the oracle's (tests/test_abi.py)."""

    def __init__(self, kctc):
        self.k, self._rnns = kctc, {}

    def _rnn(self, mode, D, H, layers, dirs):
        key = (mode, D, H, layers, dirs)
        if key not in self._rnns:
            self._rnns[key] = self.k.Rnn(mode, D, H, layers, dirs == 2)
        return self._rnns[key]

    def params_size(self, mode, D, H, layers, dirs):
        return self._rnn(mode, D, H, layers, dirs).num_params

    def lin_offset(self, mode, D, H, layers, dirs, pl, lin, isb):
        return self._rnn(mode, D, H, layers, dirs).lin_offset(pl, lin, isb)[0]


def recipe_rnn_params(oracle, mode, D, H, seed, stddev=0.02, bias=0.2):
    P = oracle.params_size(mode, D, H, 1, 2)
    w = (np.random.default_rng([seed, 1]).standard_normal(P) * stddev).astype(np.float32)
    nlin = 2 * (4 if mode == 2 else 3 if mode == 3 else 1)
    for pl in range(2):
        for lin in range(nlin):
            off = oracle.lin_offset(mode, D, H, 1, 2, pl, lin, 1)
            w[off:off + H] = bias
    return w


def layer_inputs(kctc, oracle, case):
    c = LAYER_CASES[case]
    T, N, D, H = c["T"], c["N"], c["D"], c["H"]
    w = recipe_rnn_params(oracle, c["mode"], D, H, c["seed"])
    if D == 40:
        feats, _, _, _ = kctc.synth_minibatch(c["seed"], T, N, D, 41, 0.125)
        x = feats.reshape(T, N, D)
    else:
        x = np.tanh(np.random.default_rng([c["seed"], 2]).standard_normal((T, N, D))).astype(np.float32)
    dy = (np.random.default_rng([c["seed"], 3]).standard_normal((T, N, 2 * H)) * 1e-2).astype(np.float32)
    return w, x, dy


# (ii) one whole train step of bench.py's first minibatch (seed 20161015) per
#      BASELINE config, lr 5e-4; recipe init, affine N(0, 1/2H) / N(0, 1)
#      (nnet-component.cc:1169-1174):
#      cfg1  configs[1]: 5 x BLSTM-512, N=16, T_max=2000 (fixture sketch_step.npz)
#      cfg2  configs[2]: 5 x BLSTM-512, fs=3: N=64, T_max=667, 3/8 labels per frame
#      cfg4  configs[4]: 5 x BGRU-1024, N=32, T_max=2000, run in bf16 on the GPU
STEPS = {"cfg1": dict(T=2000, N=16, D=40, H=512, A=41, R=5, mode=2, lr=5e-4, seed=20161015, pseed=77,
                      ratio=0.125, file="sketch_step"),
         "cfg2": dict(T=667, N=64, D=40, H=512, A=41, R=5, mode=2, lr=5e-4, seed=20161015, pseed=78,
                      ratio=0.375, file="sketch_step_cfg2"),
         "cfg4": dict(T=2000, N=32, D=40, H=1024, A=41, R=5, mode=3, lr=5e-4, seed=20161015, pseed=79,
                      ratio=0.125, file="sketch_step_cfg4", prec="bf16")}
STEP = STEPS["cfg1"]


def step_params(oracle, case="cfg1"):
    s = STEPS[case]
    rnn = [recipe_rnn_params(oracle, s["mode"], s["D"] if c == 0 else 2 * s["H"], s["H"], s["pseed"] + c)
           for c in range(s["R"])]
    rng = np.random.default_rng([s["pseed"], 9])
    Wa = (rng.standard_normal((s["A"], 2 * s["H"])) / np.sqrt(2 * s["H"])).astype(np.float32)
    ba = rng.standard_normal(s["A"]).astype(np.float32)
    return rnn, Wa, ba


def step_inputs(kctc, case="cfg1"):
    s = STEPS[case]
    return kctc.synth_minibatch(s["seed"], s["T"], s["N"], s["D"], s["A"], s["ratio"])


# ---- bf16 error model (configs[4]) ---------------------------------------------
BF16_EPS = 2.0 ** -9  # relative rounding of a bf16 operand: 8 significant bits, half an ulp
# variance units of one stage:
#   a GEMM of bf16-rounded operands (fp32 accumulation)                       1
#   a recurrence: h (or dh) is re-rounded every step and the earlier steps'
#   errors are carried forward through the gates, an AR(1) process whose
#   stationary error is 1/sqrt(1 - lam^2) times one step's; lam ~ 0.87
#   (update / forget gates ~ 0.5 plus the R h feedback at the recipe init)
#   gives a factor 2, i.e. 4 variance units                                  4
GEMM, REC = 1, 4


def bf16_tol(units, k=3.0):
    """Tolerance on the sketch error (tests/sketch_common.compare: the max of
    4 random projections of the difference, each ~ N(0, |a - b|^2)) of a
    result computed through stages of bf16-rounded products with fp32
    accumulation.  Each operand rounding is uniform in +-2^-9 relative (rms
    2^-9/sqrt(3)), so a product of two rounded operands carries rms
    sqrt(2/3) 2^-9, and a K-term fp32 sum of such products keeps that
    norm-wise (independent errors: both the error and the sum grow like
    sqrt(K); the fp32 accumulation adds ~sqrt(K) 2^-24, negligible).  Chained
    stages add in quadrature (`units` variance units, see GEMM / REC), which
    gives the expected norm-wise relative error; k = 3 covers the projection
    estimator (P(max of 4 |N(0,1)| > 3) ~ 1 %)."""
    return k * np.sqrt(units) * np.sqrt(2.0 / 3.0) * BF16_EPS


def layer_stages(what, layers=1):
    """Variance units behind the outputs of `layers` stacked layers: forward
    x W then the recurrence per layer; dx adds, per layer, the backward
    recurrence and the dx GEMM; dW the backward recurrence and its GEMM."""
    fwd = (GEMM + REC) * layers
    return {"y": fwd, "dx": fwd + (REC + GEMM) * layers, "dw": fwd + (REC + GEMM) * layers}[what]


def step_stages(R, what, c=0):
    """Variance units behind a whole train step's outputs (R stacked layers):
    the logits and the costs see the forward path; component c's gradient (0
    = bottom) also the backward (recurrence + dx GEMM) of the R-1-c layers
    above it, its own backward recurrence and its dW GEMM."""
    fwd = (GEMM + REC) * R
    if what in ("logits", "costs", "affine"):
        return fwd
    return fwd + (REC + GEMM) * (R - 1 - c) + REC + GEMM
