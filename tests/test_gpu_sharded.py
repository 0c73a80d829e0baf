"""Sharded placement (SHINE_PLACE_SHARDED) against the oracle and against the replica placement.

Memory node s lives on GPU slot s % G only and every slot reads the others' records through one virtual range
(include/shine_gpu.h).  On a one-GPU box the slots are repeated device ids (gpus=[0, 0, ...]): each slot still
owns a separate physical stripe and a separate id range, so the id renumbering, the holes between stripes, the
replicated upper levels / uids and the per-slot query split are all exercised; only the xGMI hop is not.
Bar: identical ids, bitwise distances and counters to the oracle (exact mode), and identical output to the
replica placement in every mode.
"""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def four_shards():
    base = D.sift_like(4000, seed=61)
    q = D.sift_like(150, seed=62)
    dumps, _, _ = O.build(base, 8, 48, 0, 4, seed=5)
    return base, q, dumps


@pytest.mark.parametrize("gpus", [[0], [0, 0], [0, 0, 0], [0, 0, 0, 0, 0]])
def test_sharded_exact_matches_oracle(four_shards, gpus, gpu_available):
    base, q, dumps = four_shards
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 128, 8, 0).knn(q, k=10, ef=48)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement="sharded") as idx:
        info = idx.info()
        r = idx.knn(q, 10, 48)
    assert info["placement"] == L.PLACE_SHARDED and info["n_gpus"] == len(gpus)
    assert info["num_nodes"] == 4000 and info["id_space"] % len(gpus) == 0 and info["id_space"] >= 4000
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :5], ref_qs[:, :5])
    np.testing.assert_array_equal(r.qstats[:, 7], ref_qs[:, 7])


@pytest.mark.parametrize("gpus", [[0, 0], [0, 0, 0]])
def test_sharded_fast_equals_replica_fast(four_shards, gpus, gpu_available):
    _, q, dumps = four_shards
    out = {}
    for placement in ("replica", "sharded"):
        with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement=placement) as idx:
            idx.set_search_mode(L.MODE_FAST)
            out[placement] = idx.knn(q, 10, 64)
    a, b = out["replica"], out["sharded"]
    np.testing.assert_array_equal(a.ids, b.ids)
    np.testing.assert_array_equal(a.dists.view(np.uint32), b.dists.view(np.uint32))
    np.testing.assert_array_equal(a.qstats[:, :8], b.qstats[:, :8])  # words 8-11 depend on placement


@pytest.mark.parametrize("start_mode", ["1", "2"])
def test_sharded_fixup_passes(four_shards, start_mode, monkeypatch, gpu_available):
    """Mode 2 keeps the visited set as a bitmap over the device id space (holes included)."""
    _, q, dumps = four_shards
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 128, 8, 0).knn(q[:40], k=10, ef=32)
    monkeypatch.setenv("SHINE_DEBUG_START_MODE", start_mode)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement="sharded") as idx:
        r = idx.knn(q[:40], 10, 32)
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.qstats[:, :5], ref_qs[:, :5])


def test_sharded_ip_f16_equals_replica(gpu_available):
    base = D.tti_like(2500, seed=71)
    q = D.tti_like(80, seed=72)
    dumps, _, _ = O.build(base, 8, 40, 1, 3, seed=9)
    out = {}
    for placement in ("replica", "sharded"):
        with shine_amd.Index.from_buffers(dumps, 200, 8, 1, elem=L.ELEM_F16, gpus=[0, 0],
                                          placement=placement) as idx:
            out[placement] = idx.knn(q, 10, 40)
    np.testing.assert_array_equal(out["replica"].ids, out["sharded"].ids)
    np.testing.assert_array_equal(out["replica"].dists.view(np.uint32), out["sharded"].dists.view(np.uint32))


def test_sharded_distance_kernel(four_shards, gpu_available):
    import torch
    base, q, dumps = four_shards
    rng = np.random.default_rng(3)
    uids = rng.integers(0, 4000, (16, 50)).astype(np.uint32)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement="sharded") as idx:
        for slot in (0, 1):
            qt = torch.from_numpy(q[:16]).cuda()
            ut = torch.from_numpy(uids.view(np.int32)).cuda()
            out = torch.empty((16, 50), dtype=torch.float32, device="cuda")
            idx.distance_device(qt.data_ptr(), 16, ut.data_ptr(), 50, out.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream, gpu_slot=slot)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            for i in range(16):
                for j in range(50):
                    ref = O.distance(0, q[i], base[uids[i, j]])
                    assert np.float32(ref).view(np.uint32) == got[i, j].view(np.uint32), (slot, i, j)


def test_sharded_device_entry_point_per_slot(four_shards, gpu_available):
    import torch
    _, q, dumps = four_shards
    ref_ids, _, _ = O.OracleIndex(dumps, 128, 8, 0).knn(q[:64], k=10, ef=48)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement="sharded") as idx:
        for slot in (0, 1):
            qt = torch.from_numpy(q[:64]).cuda()
            ids = torch.empty((64, 10), dtype=torch.int32, device="cuda")
            idx.knn_device(qt.data_ptr(), 64, 10, 48, ids.data_ptr(), None, None,
                           stream=torch.cuda.current_stream().cuda_stream, gpu_slot=slot)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), ref_ids)


@pytest.mark.parametrize("gpus,cache", [([0, 0], 0.5), ([0, 0, 0], 1.0), ([0, 0, 0], 0.2)])
def test_sharded_cache_changes_nothing_but_placement(four_shards, gpus, cache, gpu_available):
    """Local copies of the other slots' hottest records (SHINE cache row): same ids, distances and counters."""
    _, q, dumps = four_shards
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 128, 8, 0).knn(q, k=10, ef=48)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement="sharded", cache=cache) as idx:
        info = idx.info()
        r = idx.knn(q, 10, 48)
        idx.set_search_mode(L.MODE_FAST)
        f = idx.knn(q, 10, 48)
    assert 0.0 < info["cache_fraction"] <= 1.0
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :5], ref_qs[:, :5])
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement="replica") as idx:
        idx.set_search_mode(L.MODE_FAST)
        g = idx.knn(q, 10, 48)
    np.testing.assert_array_equal(f.ids, g.ids)
    np.testing.assert_array_equal(f.qstats[:, :8], g.qstats[:, :8])


def test_sharded_partial_cache_on_a_larger_index(gpu_available):
    """80K records over 2 slots (M=8: a page step is 32768 rows), so each stripe spans two steps and a 0.5 cache
    maps a hot prefix from local copies and the cold rest from the owner, both kinds of piece in one view.  Must
    equal the replica exactly."""
    base = D.sift_like(80000, seed=81)
    q = D.sift_like(200, seed=82)
    dumps, _ = shine_amd.build(base, 8, 40, 0, 2, seed=6, threads=8)
    out = {}
    for placement, cache in (("replica", 0.0), ("sharded", 0.5)):
        with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement=placement, cache=cache) as idx:
            if placement == "sharded":
                assert idx.info()["cache_fraction"] == 0.5
            out[placement] = idx.knn(q, 10, 40)
    a, b = out["replica"], out["sharded"]
    np.testing.assert_array_equal(a.ids, b.ids)
    np.testing.assert_array_equal(a.dists.view(np.uint32), b.dists.view(np.uint32))
    np.testing.assert_array_equal(a.qstats[:, :8], b.qstats[:, :8])  # words 8-11 depend on placement


@pytest.mark.parametrize("gpus", [[0, 0], [0, 0, 0, 0]])
def test_region_placement_matches_oracle_and_routes_locally(four_shards, gpus, gpu_available):
    """SHINE_PLACE_SHARDED_REGIONS: slot o owns region o; queries are routed to their region.  Results must not
    change; the routed slot should own most of a query's results (locality the xGMI path is meant to exploit)."""
    base, q, dumps = four_shards
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 128, 8, 0).knn(q, k=10, ef=48)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement="regions", cache=0.5) as idx:
        assert idx.info()["placement"] == L.PLACE_SHARDED_REGIONS
        r = idx.knn(q, 10, 48)
        slots = idx.route(q)
        idx.set_search_mode(L.MODE_FAST)
        f = idx.knn(q, 10, 48)
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :5], ref_qs[:, :5])
    k = len(gpus)
    # the router's per-batch limits (LIMIT_PER_CN = 200 per slot, query_router.hh:361-364) bound every window
    assert np.bincount(slots, minlength=k).max() <= 200 * (len(q) // (200 * k) + 2)
    _, region, _ = shine_amd.plan_regions(dumps, 128, 8, 0, k)
    local = (region[r.ids] == slots[:, None]).mean()
    assert local > 1.5 / k, local  # well above the 1/k of an unrouted split
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=gpus, placement="replica") as idx:
        idx.set_search_mode(L.MODE_FAST)
        g = idx.knn(q, 10, 48)
    np.testing.assert_array_equal(f.ids, g.ids)
    np.testing.assert_array_equal(f.qstats[:, :8], g.qstats[:, :8])


def test_read_accounting_replica_is_all_local(four_shards, gpu_available):
    _, q, dumps = four_shards
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0], placement="replica") as idx:
        r = idx.knn(q, 10, 48)
    assert (r.qstats[:, 8:12] == 0).all()
    assert r.stats["cache_hits"] == 0 and r.stats["cache_misses"] == 0 and r.stats["remote_reads_in_bytes"] == 0


@pytest.mark.parametrize("mode", [L.MODE_EXACT, L.MODE_FAST])
def test_read_accounting_splits_the_same_reads_between_cache_and_xgmi(four_shards, mode, gpu_available):
    """The search reads the same records whatever the cache holds, so per query remote + cached reads at any cache
    fraction equal the remote reads without a cache; a full cache leaves nothing on xGMI."""
    _, q, dumps = four_shards
    out = {}
    for cache in (0.0, 0.5, 1.0):
        with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0, 0, 0], placement="sharded", cache=cache) as idx:
            idx.set_search_mode(mode)
            out[cache] = idx.knn(q, 10, 48)
    none, half, full = out[0.0].qstats, out[0.5].qstats, out[1.0].qstats
    assert (none[:, 10:12] == 0).all()
    assert (full[:, 8:10] == 0).all()
    for qs in (half, full):
        np.testing.assert_array_equal(qs[:, 8] + qs[:, 10], none[:, 8])
        np.testing.assert_array_equal(qs[:, 9] + qs[:, 11], none[:, 9])
    # off-stripe reads: about 2/3 of the vector reads over three stripes, never more than all of them
    assert (none[:, 8] <= none[:, 0]).all() and (none[:, 9] <= none[:, 4]).all()
    share = none[:, 8].sum() / none[:, 0].sum()
    assert 0.45 < share < 0.85, share
    s = out[0.5].stats
    assert s["cache_hits"] == half[:, 10:12].sum() and s["cache_misses"] == half[:, 8:10].sum()
    assert s["remote_reads_in_bytes"] == half[:, 8].sum() * 128 * 4 + half[:, 9].sum() * 4 * 16


def test_query_ids_route_to_slot_id_mod_g(four_shards, gpu_available):
    """shine_knn_batch answers query i on slot query_ids[i] % G (read_data.hh:57-58): its read accounting equals
    that slot's answer through the device entry point."""
    import torch
    _, q, dumps = four_shards
    G = 3
    qids = np.arange(len(q), dtype=np.uint32) * 7 + 5
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0] * G, placement="sharded") as idx:
        r = idx.knn(q, 10, 48, query_ids=qids)
        per_slot = []
        qt = torch.from_numpy(q).cuda()
        for s in range(G):
            qs = torch.zeros((len(q), L.QS_WORDS), dtype=torch.int32, device="cuda")
            ids = torch.empty((len(q), 10), dtype=torch.int32, device="cuda")
            idx.knn_device(qt.data_ptr(), len(q), 10, 48, ids.data_ptr(), None, qs.data_ptr(),
                           stream=torch.cuda.current_stream().cuda_stream, gpu_slot=s)
            torch.cuda.synchronize()
            per_slot.append(qs.cpu().numpy().view(np.uint32).copy())
    want = np.stack([per_slot[int(i) % G][j] for j, i in enumerate(qids)])
    np.testing.assert_array_equal(r.qstats, want)
    assert len({tuple(p[:, 8]) for p in per_slot}) == G  # the slots really differ in what is remote


def test_release_stream_then_reuse(four_shards, gpu_available):
    import torch
    _, q, dumps = four_shards
    ref_ids, _, _ = O.OracleIndex(dumps, 128, 8, 0).knn(q[:32], k=10, ef=48)
    qt = torch.from_numpy(q[:32]).cuda()
    ids = torch.empty((32, 10), dtype=torch.int32, device="cuda")
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0]) as idx:
        for _ in range(3):
            s = torch.cuda.Stream()
            idx.knn_device(qt.data_ptr(), 32, 10, 48, ids.data_ptr(), None, None, stream=s.cuda_stream)
            idx.release_stream(s.cuda_stream)  # waits for the stream, then drops its scratch
            np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), ref_ids)
            del s


@pytest.fixture(scope="module")
def skew_index():
    """200K DEEP-shaped records in 8 memory-node dumps: two slots of ~100K records (stripes of 114,688 ids), so a 0.15
    cache (each array's share rounded up to whole 2 MiB pages: 21,845 vector rows) holds under a fifth of each
    stripe."""
    base = D.deep_like(200_000, seed=111, d=96)
    dumps, _ = shine_amd.build(base, 16, 100, 0, 8, seed=7, threads=16)
    pool = D.deep_like(3000, seed=112, d=96)
    return dumps, pool


def test_cache_warmup_hit_rate_rises_with_skew_and_results_do_not_change(skew_index, gpu_available):
    """The skew grid of exp_cache_size_and_skew.py on the sharded layout: the warmup split (skew.py's last `split`
    queries) ranks every stripe's cached prefix by its reads (shine_cache_warmup, the admission of hnsw.hh:447-448);
    the measured queries then hit the cache more as the Zipf alpha grows, more than with the static ranking, and
    return exactly what the oracle returns."""
    dumps, pool = skew_index
    hit = {}
    for alpha in (0.0, 1.0, 1.5):
        q, warm, _ = D.zipf_query_mix(pool, 3000, alpha, split=1000, seed=9)
        with shine_amd.Index.from_buffers(dumps, 96, 16, 0, gpus=[0, 0], placement="sharded", cache=0.15) as idx:
            assert 0.15 <= idx.info()["cache_fraction"] < 0.25
            static = idx.knn(q, 10, 128)
            idx.cache_warmup(warm, 10, 128)
            warmed = idx.knn(q, 10, 128)
        np.testing.assert_array_equal(warmed.ids, static.ids)
        np.testing.assert_array_equal(warmed.qstats[:, :8], static.qstats[:, :8])
        rate = lambda r: r.stats["cache_hits"] / (r.stats["cache_hits"] + r.stats["cache_misses"])
        hit[alpha] = (rate(static), rate(warmed))
        if alpha == 1.0:
            ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 96, 16, 0).knn(q, 10, 128, threads=8)
            np.testing.assert_array_equal(warmed.ids, ref_ids)
            np.testing.assert_array_equal(warmed.dists.view(np.uint32), ref_d.view(np.uint32))
    print("cache hit rate (static, warmed) by alpha:", hit)
    assert hit[0.0][1] < hit[1.0][1] < hit[1.5][1], hit
    assert hit[1.5][1] > hit[1.5][0] + 0.05, hit  # the warmup ranking beats the static one on a skewed mix


def test_cache_warmup_is_a_noop_for_a_replica(four_shards, gpu_available):
    _, q, dumps = four_shards
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0], placement="replica") as idx:
        before = idx.knn(q, 10, 48)
        idx.cache_warmup(q[:50], 10, 48)
        after = idx.knn(q, 10, 48)
    np.testing.assert_array_equal(before.ids, after.ids)
