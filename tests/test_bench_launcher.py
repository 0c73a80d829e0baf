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


def _bench(*args, timeout=240, **extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["SHINE_BENCH_STUB"] = "1"
    env.update(extra_env)
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


def test_line_explains_itself_at_two_ranks():
    """The keys the 8-GPU record needs to be read without the node (bench.py rank_report / peer_access / run_sharded):
    how many ranks the collective saw, every rank's own rate, the peer-access matrix, and per slot of the sharded leg
    its span and read classes.  The real line carries the same keys (bench.py main)."""
    line = _bench("--gpus", "2", "--steps", "10", "--batch", "100")
    assert line["ranks_seen"] == 2
    assert [r["rank"] for r in line["per_rank"]] == [0, 1]
    # the stub ranks "took" 1.0 and 1.1 s for 10 x 100 queries
    assert abs(line["per_rank"][0]["value"] - 1000.0) < 1e-6 and abs(line["per_rank"][1]["value"] - 1000 / 1.1) < 1e-6
    assert set(line["peer_access"]) >= {"devices", "can_access"}
    slots = line["sharded"]["per_slot"]
    assert [p["slot"] for p in slots] == [0, 1]
    assert all(set(p) >= {"gpu", "span_ms_per_step", "reads"} for p in slots)


def test_failing_sharded_child_keeps_the_replica_line():
    line = _bench("--gpus", "2", SHINE_BENCH_STUB_FAIL_SHARDED="1")
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2
    assert "error" in line["sharded"]


def test_real_line_carries_the_stub_keys():
    """bench.py's real rank-0 line builds the same self-explaining keys the stub emits (checked on the source: the
    real line needs a GPU)."""
    src = (ROOT / "bench.py").read_text()
    for key in ('"ranks_seen": ranks_seen', '"per_rank": per_rank', '"peer_access": peer_access(torch)',
                '"per_slot": per_slot'):
        assert key in src, key
