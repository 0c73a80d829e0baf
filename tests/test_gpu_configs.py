"""The BASELINE.json configs through the HIP path, each against the oracle on the same dumps and queries.

  cfg1     the committed golden fixtures (tests/golden: siftsmall-shaped L2 and the DEEP-shaped IP case) through
           exact mode, bitwise against expected_*.npz (the oracle's answers, pinned by sha256 of its dumps).
  cfg3     DEEP-shaped 96-d inner product, M=16, ef=256, one launch of 4,096 queries: search_fast_kernel<96, IP,
           f32, R=4> and the exact heap kernel at the bench launch shape (16 wavefronts wanted per CU).
  cfg4     DEEP-shaped 96-d L2, M=16, ef=128, eight memory-node dumps over eight GPU slots (sharded placement;
           repeated device ids on a one-GPU box: eight stripes, eight id ranges, the per-slot query split).
  cfg5     TTI-shaped 200-d inner product with fp16 records, a Zipf-skewed query mix (skew.py, alpha 1), ef=250.
Bars: exact mode bit-exact (ids in heap order, distances, counters); fast mode bit-exact on tie-free queries and
|recall_fast - recall_oracle| <= 1e-3 over the batch (north star); fp16 records (cfg 5) by recall within 1e-3 of the
f32 oracle.
"""
import json

import numpy as np
import pytest

import oracle as O
import shine_amd
from conftest import GOLDEN
from shine_amd import _lib as L
from shine_amd import datasets as D
from shine_amd import formats as F

pytestmark = pytest.mark.gpu

META = json.loads((GOLDEN / "meta.json").read_text())


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _check_exact(r, ref):
    ref_ids, ref_d, ref_qs = ref
    assert (r.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, [0, 1, 2, 3, 4, 5, 7]], ref_qs[:, [0, 1, 2, 3, 4, 5, 7]])


def _check_fast(r, ref, gt, k, min_clean):
    ref_ids, ref_d, ref_qs = ref
    assert (r.qstats[:, L.QS_STATUS] == 0).all()
    clean = r.qstats[:, L.QS_TIES] == 0
    assert clean.mean() >= min_clean, clean.mean()
    order = np.argsort(ref_d, axis=1, kind="stable")
    s_d = np.take_along_axis(ref_d, order, 1)
    s_ids = np.take_along_axis(ref_ids, order, 1)
    np.testing.assert_array_equal(r.dists[clean].view(np.uint32), s_d[clean].view(np.uint32))
    np.testing.assert_array_equal(np.sort(r.ids[clean], 1), np.sort(s_ids[clean], 1))
    np.testing.assert_array_equal(r.qstats[clean][:, [0, 1, 2, 3, 4, 7]], ref_qs[clean][:, [0, 1, 2, 3, 4, 7]])
    rf, ro = D.recall_at_k(r.ids, gt, k), D.recall_at_k(ref_ids, gt, k)
    assert abs(rf - ro) <= 1e-3, (rf, ro)


def _device_knn(idx, q, k, ef, slot=0):
    """One launch of the whole batch through shine_knn_batch_device (the bench's entry point)."""
    import torch
    nq = q.shape[0]
    qt = torch.from_numpy(np.ascontiguousarray(q)).cuda()
    ids = torch.empty((nq, k), dtype=torch.int32, device="cuda")
    dd = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    qs = torch.empty((nq, L.QS_WORDS), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    idx.knn_device(qt.data_ptr(), nq, k, ef, ids.data_ptr(), dd.data_ptr(), qs.data_ptr(), stream=s.cuda_stream,
                   gpu_slot=slot)
    torch.cuda.synchronize()
    return shine_amd.KnnResult(ids.cpu().numpy().view(np.uint32).copy(), dd.cpu().numpy().copy(),
                               qs.cpu().numpy().view(np.uint32).copy(), {})


# ---- cfg 1: the committed golden fixtures --------------------------------------------------------------------
def test_golden_cfg1_l2_through_hip_is_bitwise(gpu_available):
    c = META["cfg1"]
    _, base = F.read_vectors(GOLDEN / "base.u8bin")
    _, q = F.read_vectors(GOLDEN / "query.u8bin")
    dumps, _, _ = O.build(base, c["M"], c["efc"], 0, 1, c["seed"])
    assert [_sha(d) for d in dumps] == META["dumps"]["l2_1"]["sha256"]  # the exact dump the fixture was made on
    exp = np.load(GOLDEN / "expected_l2.npz")
    with shine_amd.Index.from_buffers(dumps, c["dim"], c["M"], 0, gpus=[0]) as idx:
        r = idx.knn(q, c["k"], c["ef"])
        d = _device_knn(idx, q, c["k"], c["ef"])
    for got in (r, d):
        np.testing.assert_array_equal(got.ids, exp["ids"])
        np.testing.assert_array_equal(got.dists.view(np.uint32), exp["dists"].view(np.uint32))
        np.testing.assert_array_equal(got.qstats[:, :8], exp["qstats"])


def test_golden_ip_through_hip_is_bitwise(gpu_available):
    c = META["ip"]
    _, base = F.read_vectors(GOLDEN / "ip_base.fbin")
    _, q = F.read_vectors(GOLDEN / "ip_query.fbin")
    dumps, _, _ = O.build(base, c["M"], c["efc"], 1, c["shards"][0], c["seed"])
    assert [_sha(d) for d in dumps] == META["dumps"]["ip_2"]["sha256"]
    exp = np.load(GOLDEN / "expected_ip.npz")
    with shine_amd.Index.from_buffers(dumps, c["dim"], c["M"], 1, gpus=[0]) as idx:
        r = idx.knn(q, c["k"], c["ef"])
    np.testing.assert_array_equal(r.ids, exp["ids"])
    np.testing.assert_array_equal(r.dists.view(np.uint32), exp["dists"].view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :8], exp["qstats"])


# ---- cfg 3: DEEP-shaped IP, ef=256, batch 4096 ---------------------------------------------------------------
@pytest.fixture(scope="module")
def cfg3():
    base = D.deep_like(12000, seed=301, d=96)
    q = D.deep_like(4096, seed=302, d=96)
    dumps, _, _ = O.build(base, 16, 100, 1, 1, seed=31)
    ref = O.OracleIndex(dumps, 96, 16, 1).knn(q, 10, 256, threads=8)
    gt, _ = D.brute_force_knn(base, q, 10, metric=1)
    return dict(base=base, q=q, dumps=dumps, ref=ref, gt=gt)


def test_cfg3_batch4096_exact_mode(cfg3, gpu_available):
    with shine_amd.Index.from_buffers(cfg3["dumps"], 96, 16, 1, gpus=[0]) as idx:
        r = _device_knn(idx, cfg3["q"], 10, 256)
    _check_exact(r, cfg3["ref"])


def test_cfg3_batch4096_fast_mode_r4(cfg3, gpu_available):
    with shine_amd.Index.from_buffers(cfg3["dumps"], 96, 16, 1, gpus=[0]) as idx:
        idx.set_search_mode(L.MODE_FAST)
        r = _device_knn(idx, cfg3["q"], 10, 256)
    _check_fast(r, cfg3["ref"], cfg3["gt"], 10, 0.95)


# ---- cfg 4: DEEP-shaped L2, 8 memory nodes over 8 GPU slots --------------------------------------------------
@pytest.fixture(scope="module")
def cfg4():
    base = D.deep_like(12000, seed=401, d=96)
    q = D.deep_like(1024, seed=402, d=96)
    dumps, _, _ = O.build(base, 16, 100, 0, 8, seed=41)
    ref = O.OracleIndex(dumps, 96, 16, 0).knn(q, 10, 128, threads=8)
    gt, _ = D.brute_force_knn(base, q, 10, metric=0)
    return dict(q=q, dumps=dumps, ref=ref, gt=gt)


@pytest.mark.parametrize("cache", [0.0, 0.25])
def test_cfg4_eight_slots_sharded_exact(cfg4, cache, gpu_available):
    with shine_amd.Index.from_buffers(cfg4["dumps"], 96, 16, 0, gpus=[0] * 8, placement="sharded",
                                      cache=cache) as idx:
        info = idx.info()
        r = idx.knn(cfg4["q"], 10, 128)
    assert info["n_gpus"] == 8 and info["n_shards"] == 8
    _check_exact(r, cfg4["ref"])
    # 8 stripes: most reads leave the answering slot's stripe (7/8 for random placement)
    off = r.qstats[:, [8, 9, 10, 11]].sum(1)
    assert 0.6 < off.sum() / (r.qstats[:, 0].sum() + r.qstats[:, 4].sum()) < 0.95
    if cache == 0.0:
        assert r.stats["cache_hits"] == 0 and r.stats["cache_misses"] == off.sum()
    else:
        assert r.stats["cache_hits"] > 0


def test_cfg4_eight_slots_sharded_fast(cfg4, gpu_available):
    with shine_amd.Index.from_buffers(cfg4["dumps"], 96, 16, 0, gpus=[0] * 8, placement="sharded") as idx:
        idx.set_search_mode(L.MODE_FAST)
        r = idx.knn(cfg4["q"], 10, 128)
    _check_fast(r, cfg4["ref"], cfg4["gt"], 10, 0.95)


# ---- cfg 5: TTI-shaped fp16 records, Zipf-skewed mix ---------------------------------------------------------
def test_cfg5_fp16_zipf_mix_recall(gpu_available):
    base = D.tti_like(10000, seed=501)
    pool = D.tti_like(600, seed=502)
    q, _, src = D.zipf_query_mix(pool, 2000, 1.0, seed=5)
    assert np.bincount(src).max() > 50  # the mix is skewed: the head query repeats
    dumps, _, _ = O.build(base, 16, 100, 1, 2, seed=51)
    ref_ids, _, _ = O.OracleIndex(dumps, 200, 16, 1).knn(q, 10, 250, threads=8)
    gt, _ = D.brute_force_knn(base, q, 10, metric=1)
    ro = D.recall_at_k(ref_ids, gt, 10)
    for mode in (L.MODE_EXACT, L.MODE_FAST):
        with shine_amd.Index.from_buffers(dumps, 200, 16, 1, elem=L.ELEM_F16, gpus=[0]) as idx:
            idx.set_search_mode(mode)
            r = idx.knn(q, 10, 250)
        assert (r.qstats[:, L.QS_STATUS] == 0).all()
        rf = D.recall_at_k(r.ids, gt, 10)
        assert abs(rf - ro) <= 1e-3, (mode, rf, ro)
        # a repeated query gets the same answer every time (the pool index decides the result)
        first = {}
        for i, s in enumerate(src):
            if s in first:
                np.testing.assert_array_equal(r.ids[i], r.ids[first[s]])
            else:
                first[s] = i


@pytest.mark.parametrize("policy", ["warmup", "dynamic"])
def test_cfg5_fp16_eight_slots_cached_skewed_stream(policy, gpu_available):
    """cfg 5 as one workload: fp16 records, eight memory-node dumps over eight GPU slots, a 5 % cache of the other
    stripes (ranked by a warmup split, shine_cache_warmup, or run by the reference's admission / cooling policy
    between calls, SHINE_CACHE_DYNAMIC), a Zipf alpha=1 stream (skew.py).  Recall within 1e-3 of the f32 oracle on
    the same dumps; the cache changes where records are read from, never the answers."""
    base = D.tti_like(12000, seed=511)
    pool = D.tti_like(800, seed=512)
    q, warm, _ = D.zipf_query_mix(pool, 2048 + 512, 1.0, split=512, seed=7)
    dumps, _, _ = O.build(base, 16, 100, 1, 8, seed=52)
    ref_ids, _, _ = O.OracleIndex(dumps, 200, 16, 1).knn(q, 10, 250, threads=8)
    gt, _ = D.brute_force_knn(base, q, 10, metric=1)
    ro = D.recall_at_k(ref_ids, gt, 10)
    qid = np.arange(q.shape[0], dtype=np.uint32)
    with shine_amd.Index.from_buffers(dumps, 200, 16, 1, elem=L.ELEM_F16, gpus=[0] * 8, placement="sharded") as plain:
        plain.set_search_mode(L.MODE_FAST)
        want = plain.knn(q, 10, 250, query_ids=qid)
    cache = 0.05 if policy == "warmup" else 0.0
    with shine_amd.Index.from_buffers(dumps, 200, 16, 1, elem=L.ELEM_F16, gpus=[0] * 8, placement="sharded",
                                      cache=cache) as idx:
        idx.set_search_mode(L.MODE_FAST)
        if policy == "warmup":
            idx.cache_warmup(warm, 10, 250, query_ids=np.arange(warm.shape[0], dtype=np.uint32))
            r = idx.knn(q, 10, 250, query_ids=qid)
            hit = r.stats["node_cache_hits"] / r.stats["node_reads"]
        else:
            idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=3)
            idx.knn(warm, 10, 250, query_ids=np.arange(warm.shape[0], dtype=np.uint32))  # fills the cache
            parts = [idx.knn(q[b:b + 512], 10, 250, query_ids=qid[b:b + 512]) for b in range(0, q.shape[0], 512)]
            r = shine_amd.KnnResult(np.concatenate([p.ids for p in parts]), np.concatenate([p.dists for p in parts]),
                                    np.concatenate([p.qstats for p in parts]), parts[-1].stats)
            hit = parts[-1].stats["node_cache_hits"] / parts[-1].stats["node_reads"]
    assert (r.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(r.ids, want.ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), want.dists.view(np.uint32))
    assert abs(D.recall_at_k(r.ids, gt, 10) - ro) <= 1e-3
    assert hit > 0.0


def test_cfg4_eight_slots_dynamic_cache_exact(cfg4, gpu_available):
    """cfg 4 under the reference's runtime cache (5 %): exact mode stays the oracle's search call after call while
    the cache fills and evicts."""
    with shine_amd.Index.from_buffers(cfg4["dumps"], 96, 16, 0, gpus=[0] * 8, placement="sharded") as idx:
        idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=11)
        parts = [idx.knn(cfg4["q"][b:b + 256], 10, 128, query_ids=np.arange(b, b + 256, dtype=np.uint32))
                 for b in range(0, 1024, 256)]
    r = shine_amd.KnnResult(np.concatenate([p.ids for p in parts]), np.concatenate([p.dists for p in parts]),
                            np.concatenate([p.qstats for p in parts]), {})
    _check_exact(r, cfg4["ref"])
    assert parts[-1].stats["node_cache_hits"] > 0
