"""bench.py's own rank launcher: `bench.py --gpus N`
without WORLD_SIZE starts N rank processes with torchrun-style environments
before anything touches the GPU.  CPU-only: the environments, the
rank -> device map of both transports and the process handling (exit status
of a failed rank, the others stopped)."""
import json
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_rank_envs():
    envs = bench.rank_envs(4, 29999, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"


def test_device_map():
    # RCCL: one device per rank, refused when the node has fewer
    assert [bench.device_of(r, 8, 8, "rccl") for r in range(8)] == [(r, 0, 1) for r in range(8)]
    with pytest.raises(SystemExit):
        bench.device_of(1, 2, 1, "rccl")
    # host transport: ranks wrap around the devices and split a shared one's CUs
    assert [bench.device_of(r, 2, 1, "host") for r in range(2)] == [(0, 0, 2), (0, 1, 2)]
    assert [bench.device_of(r, 3, 2, "host") for r in range(3)] == [(0, 0, 2), (1, 0, 1), (0, 1, 2)]
    assert [bench.device_of(r, 4, 8, "host") for r in range(4)] == [(r, 0, 1) for r in range(4)]


def test_args_defaults():
    a = bench.parse_args([])
    assert (a.gpus, a.steps, a.warmup, a.config, a.dp_transport) == (1, 100, 3, 1, "rccl")
    a = bench.parse_args(["--gpus", "2", "--dp-transport", "host"])
    assert (a.gpus, a.dp_transport) == (2, "host")


CHILD = r'''
import json, os, sys, time
out = sys.argv[1]
r = int(os.environ["RANK"])
with open(os.path.join(out, "rank%d.json" % r), "w") as f:
    json.dump({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT")}, f)
if len(sys.argv) > 2 and r == int(sys.argv[2]):
    sys.exit(5)
if len(sys.argv) > 2:
    time.sleep(60)
'''


def test_spawn_ranks_ok(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    assert bench.spawn_ranks(3, [str(tmp_path)], script=str(script)) == 0
    got = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"]
    assert len({g["MASTER_PORT"] for g in got}) == 1 and all(g["WORLD_SIZE"] == "3" for g in got)


def test_spawn_ranks_failure_stops_the_rest(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    t0 = time.time()
    assert bench.spawn_ranks(3, [str(tmp_path), "1"], script=str(script)) == 5
    assert time.time() - t0 < 30  # the sleeping ranks were terminated
