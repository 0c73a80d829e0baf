"""The dynamic record cache (SHINE_CACHE_DYNAMIC, include/shine_gpu.h) against its restatement (oracle/cache_ref.py).

The reference's compute-node cache (cache.hh:24-311, cooling_table.hh:52-98, hnsw.hh:447-448, 524-548) admits a node
record on a miss — upper levels always, level 0 while not full and then with probability 0.01 — evicts by random
cooling through the cooling table and rescues a cooling entry that is hit.  The GPU applies it between calls, by
default one call later (the host replays a call's logs while the next call runs).  In exact
mode a query reads exactly the records the oracle reads (oracle_knn_trace), so from the same starting state the
restatement predicts, call after call, every query's cache hits (qstats word SHINE_QS_CACHED_VEC) and each GPU's cache
contents after the call.  Results never change.
"""
import numpy as np
import pytest

import cache_ref as CR
import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def _stream(idx, trace_index, batches, slots, seed, k, ef, capacity, lag=False):
    """Run every batch through the GPU handle and the restatement side by side; returns per-call hit rates.
    lag: the pipelined policy (capi.cc replay): call n's logs are replayed during call n + 1, so call n searches the
    cache as calls <= n - 2 left it, and the engine holds calls <= n - 1 when call n returns."""
    caches = [CR.RefCache(capacity, seed + s) for s in range(slots)]
    pending = None
    rates = []
    for call, (q, ids) in enumerate(batches):
        r = idx.knn(q, k, ef, query_ids=ids)
        assert (r.qstats[:, L.QS_STATUS] == 0).all()
        (ref_ids, _, _), (uids, always, nodes, off) = trace_index.knn_trace(q, k, ef)
        np.testing.assert_array_equal(r.ids, ref_ids)  # exact mode: the oracle's search
        dev = idx.device_ids(uids)
        hits = np.zeros(q.shape[0], np.int64)
        rescued = [[] for _ in range(slots)]
        cands = [[] for _ in range(slots)]
        local = np.zeros(q.shape[0], np.int64)
        seen = [0] * slots
        for i in range(q.shape[0]):
            s = int(ids[i]) % slots
            local[i] = seen[s]
            seen[s] += 1
        for i in range(q.shape[0]):
            s = int(ids[i]) % slots
            c = caches[s]
            for j in range(off[i], off[i + 1]):
                if int(nodes[j]) % slots == s:
                    continue  # own stripe: local memory, not a cache lookup of this GPU
                u = int(uids[j])
                if u in c:
                    hits[i] += 1
                    if c.cooling[u]:
                        rescued[s].append(u)
                else:
                    cands[s].append((int(local[i]), u, bool(always[j]),
                                     CR.admission_coin(seed + s, call, int(local[i]), int(dev[j]))))
        np.testing.assert_array_equal(r.qstats[:, L.QS_CACHED_VEC].astype(np.int64), hits)
        apply, pending = (pending, (rescued, cands)) if lag else ((rescued, cands), None)
        for s in range(slots):
            if apply is not None:
                caches[s].apply_call(apply[0][s], apply[1][s])
            np.testing.assert_array_equal(idx.cache_keys(s), np.array(sorted(caches[s].keys()), np.uint32))
        rates.append(r.stats["node_cache_hits"] / max(1, r.stats["node_reads"]))
    return rates, caches


@pytest.mark.parametrize("lag", [True, False], ids=["pipelined", "synchronous"])
def test_dynamic_cache_matches_the_restatement_call_by_call(lag, gpu_available, monkeypatch):
    monkeypatch.setenv("SHINE_CACHE_LAG", "1" if lag else "0")
    base = D.deep_like(6000, seed=401, d=96)
    pool = D.deep_like(400, seed=402, d=96)
    dumps, _, _ = O.build(base, 12, 64, 0, 4, seed=5)
    slots, seed, k, ef = 2, 77, 10, 48
    q, _, _ = D.zipf_query_mix(pool, 6 * 96, 1.0, seed=3)
    batches = [(q[b * 96:(b + 1) * 96], np.arange(b * 96, (b + 1) * 96, dtype=np.uint32)) for b in range(6)]
    oi = O.OracleIndex(dumps, 96, 12, 0)
    with shine_amd.Index.from_buffers(dumps, 96, 12, 0, gpus=[0] * slots, placement="sharded") as idx:
        idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=seed)
        rates, caches = _stream(idx, oi, batches, slots, seed, k, ef, CR.capacity(6000, 12, 96, 5.0), lag)
    assert caches[0].is_full() and caches[1].is_full()  # the stream went past the fill phase
    assert sum(c.evicted for c in caches) > 0 and rates[-1] > rates[0]


def test_dynamic_cache_rejects_static_fraction_and_replicas(gpu_available):
    base = D.deep_like(500, seed=1, d=96)
    dumps, _, _ = O.build(base, 8, 20, 0, 2, seed=1)
    with shine_amd.Index.from_buffers(dumps, 96, 8, 0, gpus=[0]) as idx:
        with pytest.raises(shine_amd.ShineError):
            idx.set_cache_policy(L.CACHE_DYNAMIC)
    with shine_amd.Index.from_buffers(dumps, 96, 8, 0, gpus=[0, 0], placement="sharded", cache=0.5) as idx:
        with pytest.raises(shine_amd.ShineError):
            idx.set_cache_policy(L.CACHE_DYNAMIC)


def test_dynamic_cache_recovers_after_the_zipf_head_moves(gpu_available):
    """A Zipf-skewed stream (skew.py) whose head moves to other queries mid-stream: the hit rate drops, then climbs back
    with no warmup, as admissions and cooling replace the old head's records.  Results stay the fast kernel's with and
    without the cache."""
    base = D.deep_like(20000, seed=411, d=96)
    pool = D.deep_like(2000, seed=412, d=96)
    dumps, _, _ = O.build(base, 16, 64, 0, 8, seed=6)
    slots = 4
    qa, _, _ = D.zipf_query_mix(pool, 12 * 512, 1.25, seed=1)
    qb, _, _ = D.zipf_query_mix(pool[::-1].copy(), 12 * 512, 1.25, seed=2)  # another head
    stream = np.concatenate([qa, qb])
    with shine_amd.Index.from_buffers(dumps, 96, 16, 0, gpus=[0] * slots, placement="sharded") as plain, \
            shine_amd.Index.from_buffers(dumps, 96, 16, 0, gpus=[0] * slots, placement="sharded") as idx:
        plain.set_search_mode(L.MODE_FAST)
        idx.set_search_mode(L.MODE_FAST)
        idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=9)
        rates = []
        for b in range(24):
            qq = stream[b * 512:(b + 1) * 512]
            ids = np.arange(b * 512, (b + 1) * 512, dtype=np.uint32)
            r = idx.knn(qq, 10, 64, query_ids=ids)
            ref = plain.knn(qq, 10, 64, query_ids=ids)
            np.testing.assert_array_equal(r.ids, ref.ids)
            np.testing.assert_array_equal(r.dists.view(np.uint32), ref.dists.view(np.uint32))
            rates.append(r.stats["node_cache_hits"] / r.stats["node_reads"])
    before, after, end = rates[11], rates[12], rates[23]
    assert after < before          # the head moved: the cached records no longer serve it
    assert end > after + 0.02      # and the cache follows it without a new warmup


@pytest.mark.parametrize("lag", [True, False], ids=["pipelined", "synchronous"])
def test_dynamic_cache_with_device_api_searches_between_calls(lag, gpu_available, monkeypatch):
    """Device-API searches (shine_knn_batch_device on a caller stream) between host calls of a handle under the dynamic
    policy: they read and log through the same arena, so the host waits for the device before it fetches the logs or
    uploads an update (capi.cc dev_api_dirty) and shine_cache_update replays what they logged.  Every result equals a
    cache-less handle's, and the cache still fills."""
    import torch
    monkeypatch.setenv("SHINE_CACHE_LAG", "1" if lag else "0")
    base = D.deep_like(8000, seed=421, d=96)
    pool = D.deep_like(600, seed=422, d=96)
    dumps, _, _ = O.build(base, 12, 64, 0, 4, seed=8)
    slots, k, ef, B = 2, 10, 48, 128
    q, _, _ = D.zipf_query_mix(pool, 10 * B, 1.0, seed=4)
    stream = torch.cuda.Stream()
    with shine_amd.Index.from_buffers(dumps, 96, 12, 0, gpus=[0] * slots, placement="sharded") as plain, \
            shine_amd.Index.from_buffers(dumps, 96, 12, 0, gpus=[0] * slots, placement="sharded") as idx:
        idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=13)
        qd = torch.from_numpy(q).cuda()
        ids_d = torch.empty((B, k), dtype=torch.int32, device="cuda")
        for b in range(10):
            qq = q[b * B:(b + 1) * B]
            qid = np.arange(b * B, (b + 1) * B, dtype=np.uint32)
            if b % 2:  # a device-API batch on slot b % slots, then the host API
                idx.knn_device(qd[b * B:(b + 1) * B].data_ptr(), B, k, ef, ids_d.data_ptr(), None, None,
                               stream=stream.cuda_stream, gpu_slot=b % slots)
                stream.synchronize()
                ref_slot = plain.knn(qq, k, ef, query_ids=np.full(B, b % slots, dtype=np.uint32))
                np.testing.assert_array_equal(ids_d.cpu().numpy().view(np.uint32), ref_slot.ids)
            r = idx.knn(qq, k, ef, query_ids=qid)
            ref = plain.knn(qq, k, ef, query_ids=qid)
            np.testing.assert_array_equal(r.ids, ref.ids)
            assert (r.qstats[:, L.QS_STATUS] == 0).all()
        idx.cache_update()  # the device-API searches' logs too
        assert sum(len(idx.cache_keys(s)) for s in range(slots)) > 0
        idx.release_stream(stream.cuda_stream)


def test_dynamic_cache_device_api_batch_in_flight_across_a_host_call(gpu_available, monkeypatch):
    """A device-API batch still running on a caller stream when a pipelined host call starts: the host call
    copies its log counts behind its own searches, the update it uploads drains the device first, and the counts are
    then copied again, so nothing the device-API batch logged after the early copy is lost.  The same sequence with the
    caller stream synchronized before every host call leaves the same cache contents, slot by slot."""
    import torch
    monkeypatch.setenv("SHINE_CACHE_LAG", "1")
    base = D.deep_like(8000, seed=431, d=96)
    pool = D.deep_like(600, seed=432, d=96)
    dumps, _, _ = O.build(base, 12, 64, 0, 4, seed=8)
    slots, k, ef, B = 2, 10, 48, 256
    q, _, _ = D.zipf_query_mix(pool, 8 * B, 1.0, seed=5)
    keys = {}
    for sync in (True, False):
        stream = torch.cuda.Stream()
        with shine_amd.Index.from_buffers(dumps, 96, 12, 0, gpus=[0] * slots, placement="sharded") as idx:
            idx.set_cache_policy(L.CACHE_DYNAMIC, ratio_percent=5.0, seed=17)
            qd = torch.from_numpy(q).cuda()
            ids_d = torch.empty((B, k), dtype=torch.int32, device="cuda")
            for b in range(8):
                qq = q[b * B:(b + 1) * B]
                qid = np.arange(b * B, (b + 1) * B, dtype=np.uint32)
                idx.knn_device(qd[b * B:(b + 1) * B].data_ptr(), B, k, ef, ids_d.data_ptr(), None, None,
                               stream=stream.cuda_stream, gpu_slot=b % slots)
                if sync:
                    stream.synchronize()
                r = idx.knn(qq, k, ef, query_ids=qid)
                assert (r.qstats[:, L.QS_STATUS] == 0).all()
                assert r.stats["cache_log_dropped"] == 0
            stream.synchronize()
            idx.cache_update()
            keys[sync] = [np.asarray(idx.cache_keys(s)) for s in range(slots)]
            idx.release_stream(stream.cuda_stream)
    for s in range(slots):
        assert keys[True][s].size > 0
        np.testing.assert_array_equal(keys[False][s], keys[True][s])
