"""Generate the full-size sketch fixtures (tests/golden/sketch_*.npz) from the
fp64 oracle.  TEST INFRASTRUCTURE: run once in the build container
(`python tests/golden/make_sketch.py [layers|step|step_cfg2|step_cfg4|<layer case>]`,
~5 min on 8 cores for the layers and the configs[1] step; step_cfg4 ~30 min); the GPU tests in
tests/test_fullsize_gpu.py regenerate the same inputs and compare sketches
(tests/sketch_common.py).  Nothing here reads /root/reference.
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_lib as O  # noqa: E402
import sketch_common as S  # noqa: E402
import __graft_entry__ as ge  # noqa: E402


def layers(kctc, only=None):
    path = os.path.join(HERE, "sketch_layers.npz")
    out = {}
    if only and os.path.exists(path):  # add / refresh some cases, keep the others
        with np.load(path, allow_pickle=False) as z:
            out = {k: z[k] for k in z.files}
    for case, c in S.LAYER_CASES.items():
        if only and case not in only:
            continue
        t0 = time.time()
        w, x, dy = S.layer_inputs(kctc, O, case)
        H = c["H"]
        y, res = O.rnn_forward(c["mode"], x.astype(np.float64), w.astype(np.float64), H, 1, 2)
        dx, dw = O.rnn_backward(c["mode"], x.astype(np.float64), w.astype(np.float64), y,
                                dy.astype(np.float64), res, H, 1, 2)
        del res
        seed = c["seed"]
        S.save(f"{case}.y", S.sketch(y, seed), out)
        S.save(f"{case}.dx", S.sketch(dx, seed + 1), out)
        S.save(f"{case}.dw", S.sketch(dw, seed + 2), out)
        # per-region norms of dW (W, R, biases of both directions)
        nlin = 8 if c["mode"] == 2 else 6
        regs = []
        for pl in range(2):
            for lin in range(nlin):
                for isb in (0, 1):
                    off = O.lin_offset(c["mode"], c["D"], H, 1, 2, pl, lin, isb)
                    sz = H if isb else H * (c["D"] if lin < nlin // 2 else H)
                    regs.append(np.linalg.norm(dw[off:off + sz]))
        out[f"{case}.dw_region_norms"] = np.array(regs)
        out[f"{case}.y_t0_fwd"] = y[0, :, :H].copy()           # t=0 forward outputs, exact check
        print(f"{case}: {time.time() - t0:.1f}s |y| {np.linalg.norm(y):.6g} |dx| {np.linalg.norm(dx):.6g} "
              f"|dw| {np.linalg.norm(dw):.6g}", flush=True)
    np.savez_compressed(path, **out)


def step(kctc, case="cfg1"):
    s = S.STEPS[case]
    t0 = time.time()
    rnn, Wa, ba = S.step_params(O, case)
    feats, nf, fl, ll = S.step_inputs(kctc, case)
    spec = O.NnetSpec()
    spec.num_rnn, spec.mode, spec.hidden, spec.dirs, spec.layers_per_rnn = s["R"], s["mode"], s["H"], 2, 1
    spec.input_dim, spec.num_targets = s["D"], s["A"]
    spec.clip_threshold, spec.repair_threshold, spec.repair_scale, spec.repair_target = 30.0, 0.01, 1.0, 0.0
    spec.rnn_clip_gradient, spec.lr_rnn, spec.lr_affine = 5.0, s["lr"], s["lr"]
    p = [w.astype(np.float64) for w in rnn]
    Wd, bd = Wa.astype(np.float64), ba.astype(np.float64)
    cnc, cc = np.zeros(s["R"]), np.zeros(s["R"])
    # the first rand() of srand(0) decides self-repair; with threshold 30 nothing
    # is clipped at init, so the repair never fires and the draws do not matter
    ex = {}
    tot, acc, wt = O.train_step(spec, p, Wd, bd, feats.reshape(s["T"], s["N"], s["D"]).astype(np.float64),
                                nf, fl, ll, repair_draws=np.ones(s["R"], np.float32), clip_num_clipped=cnc,
                                clip_count=cc, extras=ex)
    out = {"costs": ex["costs"], "tot_objf": tot, "tot_accuracy": acc, "tot_weight": wt,
           "clip_num_clipped": cnc, "clip_count": cc, "ids": ex["ids"]}
    S.save("logits", S.sketch(ex["logits"], 500), out)
    # the applied gradient of every component: (W_after - W_before) / lr in
    # fp64 = the +-5-clipped dW of an RNN (nnet-cudnn-component.cc:602-614),
    # the plain gradient of the affine layer (UpdateSimple)
    for c in range(s["R"]):
        S.save(f"g{c}", S.sketch((p[c] - rnn[c].astype(np.float64)) / s["lr"], 600 + c), out)
    daff = np.concatenate([(Wd - Wa.astype(np.float64)).ravel(), bd - ba.astype(np.float64)]) / s["lr"]
    S.save("gaff", S.sketch(daff, 700), out)
    np.savez_compressed(os.path.join(HERE, s["file"] + ".npz"), **out)
    print(f"step {case}: {time.time() - t0:.1f}s objf {tot:.8g} acc {acc} weight {wt} clipped {cnc}", flush=True)


if __name__ == "__main__":
    kctc = ge.load_package()
    what = sys.argv[1:] or ["layers", "step"]
    cases = [w for w in what if w in S.LAYER_CASES]
    if "layers" in what or cases:
        layers(kctc, cases or None)
    if "step" in what:
        step(kctc)
    for case in ("cfg2", "cfg4"):
        if "step_" + case in what:
            step(kctc, case)
