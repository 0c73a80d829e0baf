"""The N>1 path of bench.py on CPU: two ranks over gloo (127.0.0.1), driving the real protocol functions.

bench.py under torchrun does the following; each step is exercised here with world_size 2:
* rank 0 builds the memory-node dumps once and the others read them after a barrier (`prepare_dumps`);
* every rank answers the queries with id ≡ rank (mod world) (`rank_queries`, read_data.hh:57-58);
* the job's wall time is the max over ranks (`max_over_ranks`).
The GPU search is replaced by the CPU oracle, so the check is that the union of the two ranks' answers equals a
single-process run over the whole query pool, and that no rank reads a dump before rank 0 wrote it.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, tmp):
    for p in (ROOT, ROOT / "dm-hnsw-reference_amd", ROOT / "oracle"):
        sys.path.insert(0, str(p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    import oracle as O
    import shine_amd
    from shine_amd import datasets as D

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tmp = Path(tmp)
        paths = [tmp / "dump" / shine_amd.dump_name(8, 32, i, 2) for i in range(2)]
        base = D.sift_like(1200, seed=21)

        def build():
            assert rank == 0, "only rank 0 builds"
            return shine_amd.build(base, 8, 32, shine_amd.METRIC_L2, 2, seed=5, threads=2)[0]

        bench.prepare_dumps(paths, rank, dist, build)
        assert all(p.exists() for p in paths)  # after the barrier every rank sees complete dumps
        dumps = [np.fromfile(p, dtype=np.uint8) for p in paths]
        pool = D.sift_like(30, seed=22)
        q = bench.rank_queries(pool, rank, world, 15)
        ids, _, _ = O.OracleIndex(dumps, 128, 8, 0).knn(q, 10, 32)
        mine = {int(i): ids[j].tolist() for j, i in enumerate(range(rank, 30, world))}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        slowest = bench.max_over_ranks(0.5 + rank, dist, "cpu")
        if rank == 0:
            merged = {}
            for g in gathered:
                assert not (set(g) & set(merged)), "a query was answered by two ranks"
                merged.update(g)
            ref, _, _ = O.OracleIndex(dumps, 128, 8, 0).knn(pool, 10, 32)
            ok = sorted(merged) == list(range(30)) and all(merged[i] == ref[i].tolist() for i in range(30))
            (tmp / "result.txt").write_text(f"{ok} {slowest}")
    finally:
        dist.destroy_process_group()


def test_two_rank_bench_protocol_over_gloo(tmp_path):
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    ok, slowest = (tmp_path / "result.txt").read_text().split()
    assert ok == "True"
    assert float(slowest) == 1.5  # max over ranks of 0.5 + rank


def test_rank_queries_partition():
    sys.path.insert(0, str(ROOT))
    import bench
    pool = np.arange(40, dtype=np.float32).reshape(20, 2)
    parts = [bench.rank_queries(pool, r, 3, 100) for r in range(3)]
    rows = sorted(int(x) for p in parts for x in p[:, 0] // 2)
    assert rows == list(range(20))
    assert all((p[:, 0] // 2 % 3 == r).all() for r, p in enumerate(parts))


@pytest.mark.parametrize("slots,ndev", [(8, 8), (8, 1), (4, 2), (3, 8), (1, 1)])
def test_sharded_leg_slot_plan(slots, ndev):
    """bench.py --placement sharded: slot s runs on device s % ndev (N slots over N GPUs = one per GPU; more slots
    than GPUs repeat devices), and every batch's queries are split by id % slots, each exactly once."""
    sys.path.insert(0, str(ROOT))
    import bench
    gpus, rows = bench.sharded_plan(slots, ndev, 1024, 3)
    assert gpus == [s % ndev for s in range(slots)]
    assert len(set(gpus)) == min(slots, ndev)
    for b in range(3):
        allq = np.sort(np.concatenate(rows[b]))
        np.testing.assert_array_equal(allq, np.arange(b * 1024, (b + 1) * 1024))
        for s in range(slots):
            assert (rows[b][s] % slots == s).all()


def test_sharded_leg_refuses_torchrun_and_empty_plans(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench
    with pytest.raises(SystemExit):
        bench.sharded_plan(0, 8, 1024, 1)
    monkeypatch.setenv("WORLD_SIZE", "2")

    class A:
        pass
    with pytest.raises(SystemExit):
        bench.run_sharded(A())
