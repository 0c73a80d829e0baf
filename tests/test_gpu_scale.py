"""Parity at the size the bench times: BASELINE.json configs[1] exactly as bench.py builds and searches it.

1M SIFT-shaped records (datasets.sift_like(1M, seed=1)), M=16, efC=200, built on the GPU by shine_gpu_build with the
bench's seed (1234), searched at ef=128, k=10, batch 1,024 (the bench's first query batch, sift_like(seed=2)).
Size-independent checks:
* exact mode equals the oracle's knn (hnsw.hh:253-307, 406-476) on the GPU-built dump: ids in heap order, distances
  bitwise, every counter, on a 64-query sample;
* fast mode equals exact mode on every query of the batch without a tie event (same id set, same distances in
  ascending order, same counters);
* recall@10 against a float64 brute-force ground truth is at least 0.95 in both modes (the metric's bar), and the two
  modes' recalls agree within 1e-3 (the north-star bar over the whole batch, ties included).
"""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def test_bench_index_at_1m(gpu_available):
    import torch
    n, dim, M, efc, ef, k, batch = 1_000_000, 128, 16, 200, 128, 10, 1024
    base = D.sift_like(n, seed=1, d=dim)
    q = D.sift_like(batch * 12, seed=2, d=dim)[:batch]
    with shine_amd.GpuBuild(base, M, efc, L.METRIC_L2, seed=1234) as gb:
        st = gb.stats()
        assert st["num_nodes"] == n and st["search_failures"] == 0
        dumps = gb.dumps(1)
        with gb.open() as idx:
            ex = idx.knn(q, k, ef)
            idx.set_search_mode(L.MODE_FAST)
            fa = idx.knn(q, k, ef)
    assert (ex.qstats[:, L.QS_STATUS] == 0).all() and (fa.qstats[:, L.QS_STATUS] == 0).all()
    # exact mode against the oracle on the dump, 64 queries spread over the batch
    sample = np.arange(0, batch, batch // 64)
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, dim, M, L.METRIC_L2).knn(q[sample], k, ef, threads=8)
    del dumps
    np.testing.assert_array_equal(ex.ids[sample], ref_ids)
    np.testing.assert_array_equal(ex.dists[sample].view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(ex.qstats[sample, :5], ref_qs[:, :5])
    # fast mode against exact mode on every tie-free query of the batch
    clean = fa.qstats[:, L.QS_TIES] == 0
    assert clean.mean() > 0.3, clean.mean()
    np.testing.assert_array_equal(np.sort(fa.ids[clean], 1), np.sort(ex.ids[clean], 1))
    np.testing.assert_array_equal(fa.dists[clean].view(np.uint32), np.sort(ex.dists[clean], 1).view(np.uint32))
    np.testing.assert_array_equal(fa.qstats[clean][:, :5], ex.qstats[clean][:, :5])
    # ground truth in float64 (an f32 GEMM reorders near neighbours: DESIGN §3)
    bt = torch.from_numpy(base).cuda().double()
    bn = (bt * bt).sum(1)
    qt = torch.from_numpy(q).cuda().double()
    d = (qt * qt).sum(1)[:, None] + bn[None, :] - 2.0 * (qt @ bt.T)
    gt = torch.topk(d, k, largest=False).indices.cpu().numpy()
    del bt, bn, qt, d
    torch.cuda.empty_cache()
    r_ex, r_fa = D.recall_at_k(ex.ids, gt, k), D.recall_at_k(fa.ids, gt, k)
    assert r_ex >= 0.95 and r_fa >= 0.95, (r_ex, r_fa)
    assert abs(r_fa - r_ex) <= 1e-3
