"""kctc_nnet_copy_features_async: minibatches staged from pinned host memory
on the trainer's copy stream, one ahead of the queued steps (the bench's
H2D-inclusive pass), train exactly as the same minibatches already resident
in HBM -- the copy is ordered before the step that reads it and never
overwrites a buffer a queued step still uses (three staging buffers, two
steps in flight)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_copy_stream_steps_match_resident(kctc, gpu):
    import torch
    T, N, D, H, A = 60, 8, 40, 256, 41
    cfg = kctc.recipe_config(num_rnn=2, input_dim=D, hidden=H, num_targets=A, learning_rate=1e-3,
                             max_seq_length=T, rnn_mode=2)
    mbs = [kctc.synth_minibatch(31 + i, T, N, D, A, 0.125) for i in range(5)]

    def run(staged):
        net = kctc.Nnet(cfg, seed=5)
        stats = []
        if staged:
            host = [torch.from_numpy(m[0]).pin_memory() for m in mbs]
            buf = [torch.empty(host[0].shape, dtype=torch.float32, device=gpu) for _ in range(3)]
            net.copy_features_async(buf[0], host[0])
            for i, (_, nf, fl, ll) in enumerate(mbs):
                r = net.train_step_async(buf[i % 3], T, N, nf, fl, ll)
                if r is not None:
                    stats.append(r)
                if i + 1 < len(mbs):
                    net.copy_features_async(buf[(i + 1) % 3], host[i + 1])
        else:
            dev = [torch.from_numpy(m[0]).to(gpu) for m in mbs]
            for i, (_, nf, fl, ll) in enumerate(mbs):
                r = net.train_step_async(dev[i], T, N, nf, fl, ll)
                if r is not None:
                    stats.append(r)
        stats += net.train_flush()
        params = [net.get_params(c) for c in range(net.num_components) if net.num_params(c) > 0]
        net.close()
        return stats, params

    a, pa = run(False)
    b, pb = run(True)
    assert a == b
    for x, y in zip(pa, pb):
        np.testing.assert_array_equal(x, y)
