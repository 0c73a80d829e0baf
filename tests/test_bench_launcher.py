"""bench.py's own multi-GPU launcher on CPU (SHINE_BENCH_STUB=1: each rank joins a gloo group instead of using a GPU).

`python bench.py --gpus N` without torchrun must start N rank processes itself (a torch.distributed.run child; the
parent never touches the GPU), run the sharded leg over the same N GPUs in a child of rank 0, and print ONE merged
JSON line whose n_gpus is N.  `python bench.py --gpus 1` stays a single process with no sharded leg.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["SHINE_BENCH_STUB"] = "1"
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True, env=env,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    return json.loads(lines[0])


def test_gpus_2_spawns_two_ranks_and_merges_the_sharded_leg():
    line = _bench("--gpus", "2")
    assert line["n_gpus"] == 2
    assert line["ranks_seen"] == 2  # an all-reduce over the two rank processes
    assert "launcher" in line
    assert line["sharded"]["stub"] is True
    assert line["sharded"]["n_gpus"] == 2 and line["sharded"]["gpu_slots"] == 2
    assert line["config"]["parallelism"] == "replica2"


def test_gpus_1_is_one_process_without_a_sharded_leg():
    line = _bench("--gpus", "1")
    assert line["n_gpus"] == 1 and line["ranks_seen"] == 1
    assert "launcher" not in line and "sharded" not in line


def test_sharded_leg_can_be_forced_at_one_gpu_and_switched_off_at_two():
    assert _bench("--gpus", "1", "--sharded-leg", "on")["sharded"]["n_gpus"] == 1
    assert "sharded" not in _bench("--gpus", "2", "--sharded-leg", "off")


def test_forwarded_args_round_trip():
    sys.path.insert(0, str(ROOT))
    import argparse
    import bench
    a = argparse.Namespace(gpus=4, steps=7, no_cpu=True, no_host=False, ef_sweep="", cache_frac=0.05)
    out = bench.forwarded_args(a)
    assert "--gpus" not in out
    assert out[out.index("--steps") + 1] == "7"
    assert "--no-cpu" in out and "--no-host" not in out
    assert out[out.index("--ef-sweep") + 1] == ""
