"""The product's parallel builder (restating HNSW::insert, hnsw.hh:40-251) against the oracle's single-threaded
build: byte-identical dumps with one thread; valid, high-recall dumps with many."""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import datasets as D


@pytest.mark.parametrize("n,dim,M,efc,metric,shards,gen", [
    (3000, 128, 16, 100, 0, 1, D.sift_like),
    (3000, 128, 16, 100, 0, 3, D.sift_like),
    (2000, 96, 12, 60, 1, 2, D.deep_like),
    (1500, 200, 8, 40, 1, 1, D.tti_like),
    (1200, 100, 32, 80, 0, 4, D.deep_like),
])
def test_single_thread_build_is_byte_identical_to_oracle(n, dim, M, efc, metric, shards, gen):
    base = gen(n, seed=3, d=dim)
    ref, ref_dc, _ = O.build(base, M, efc, metric, shards, seed=99)
    got, dc = shine_amd.build(base, M, efc, metric, shards, seed=99, threads=1)
    assert dc == ref_dc
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert a.size == b.size and np.array_equal(a, b)


def test_parallel_build_is_a_valid_index_with_high_recall():
    base = D.sift_like(20000, seed=5)
    q = D.sift_like(100, seed=6)
    dumps, _ = shine_amd.build(base, 16, 100, 0, 2, seed=1, threads=8)
    gt, _ = D.brute_force_knn(base, q, 10)
    ids, _, qs = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 64)
    assert D.recall_at_k(ids, gt, 10) >= 0.95
    # every record reachable: the uids found in the dumps are exactly 0..n-1
    assert sum(int(np.frombuffer(d[:8], np.uint64)[0]) for d in dumps) == sum(d.size for d in dumps)


@pytest.mark.parametrize("threads,metric,gen,dim", [(1, 0, D.sift_like, 128), (8, 0, D.sift_like, 128),
                                                    (8, 1, D.deep_like, 96)])
def test_parallel_build_reaches_every_record(threads, metric, gen, dim):
    """Reachability from the entry point along level-0 lists (shine_graph_stats_buffers): a race in the parallel
    insert (lost list updates, a list published before its node) would leave records no search can return."""
    base = gen(30000, seed=8, d=dim)
    dumps, _ = shine_amd.build(base, 16, 100, metric, 2, seed=2, threads=threads)
    st = shine_amd.graph_stats(dumps, dim, 16)
    assert st["num_nodes"] == 30000
    assert st["reachable_l0"] >= 30000 - 3, st
    assert st["reachable_any"] >= st["reachable_l0"]
    assert 8.0 <= st["mean_degree_l0"] <= 32.0


def test_graph_stats_sees_a_cut_graph():
    """Emptying the entry point's level-0 list (and every upper list) leaves only the entry point reachable."""
    base = D.sift_like(300, seed=9)
    dumps, _, _ = O.build(base, 4, 16, 0, 1, seed=1)
    d = dumps[0].copy()
    free = int(np.frombuffer(d[:8].tobytes(), np.uint64)[0])
    off = 16
    while off < free:  # zero every list count (node.hh:10-19 record walk)
        level = int(np.frombuffer(d[off + 12:off + 16].tobytes(), np.uint32)[0])
        lo = off + 16 + 4 * 128
        d[lo:lo + 4] = 0
        for l in range(1, level + 1):
            p = lo + 4 + 8 * 8 + (l - 1) * (4 + 8 * 4)
            d[p:p + 4] = 0
        size = 16 + 4 * 128 + 4 + 8 * 8 + level * (4 + 8 * 4)
        off += size + (-size) % 8
    st = shine_amd.graph_stats([d], 128, 4)
    assert st["reachable_l0"] == 1 and st["reachable_any"] == 1 and st["zero_indegree_l0"] == 299


def test_build_write_uses_reference_dump_names(tmp_path):
    import ctypes as C
    base = D.sift_like(500, seed=7)
    L = shine_amd._lib
    b = np.ascontiguousarray(base)
    h = C.c_void_p()
    L.check(L.lib().shine_build(b.ctypes.data_as(C.c_void_p), 500, 128, 8, 40, 0, 2, 1, 2, C.byref(h)))
    try:
        L.check(L.lib().shine_build_write(h, str(tmp_path).encode(), 8, 40))
    finally:
        L.lib().shine_build_free(h)
    names = sorted(p.name for p in (tmp_path / "dump").iterdir())
    assert names == ["index_m8_efc40_node1_of2.dat", "index_m8_efc40_node2_of2.dat"]  # compute_node.cc:428-430


def test_build_rejects_bad_parameters():
    base = D.sift_like(10, seed=1)
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.build(base, 1, 10)  # M < 2: 1/ln(M) undefined (hnsw.hh:30)
    assert e.value.code == 1
