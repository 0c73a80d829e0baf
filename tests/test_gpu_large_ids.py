"""Visited sets at a 27-bit id space (the cfg 4 / cfg 5 sizes): an index of 2^26 + 2^20 records.

At more than 32M ids the spill target of an overflowing LDS visited table is the hash table in HBM (kernels_impl.h
SpillSet; the id-space bitmap would be 8.5 MB, beyond an XCD's L2), chosen by the library itself (no override here).
The records are 16-d (DEEP-shaped, GPU-generated) and the graph sparse (M = 8, efC = 24, the GPU batch builder) so the
build and the dump images stay small; 64-entry LDS tables (SHINE_DEBUG_VISCAP) make every query spill.  Exact mode
equals the oracle's knn on the dump bit for bit (ids in heap order, distances, counters); fast mode equals it on every
tie-free query, with the forced tables and with the library's own learned u32 table for this id space.
"""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def test_spill_to_hash_at_27_bit_ids(gpu_available, monkeypatch, capfd):
    import sys
    import time

    import torch
    t0 = time.time()

    def step(what):  # progress (visible with pytest -s): the phases' cost at this size
        print(f"[large ids {time.time() - t0:6.1f}s] {what}", file=sys.stderr, flush=True)

    n, dim, M, efc, ef, k = (1 << 26) + (1 << 16), 16, 8, 24, 64, 10
    base_t = D.generate_device("deep_like", n, seed=61, d=dim)
    q = D.generate_device("deep_like", 64, seed=62, d=dim).cpu().numpy()
    step("rows generated")
    with shine_amd.GpuBuild(base_t.data_ptr(), M, efc, L.METRIC_L2, seed=7, n=n, dim=dim) as gb:
        step("built")
        del base_t
        torch.cuda.empty_cache()
        assert gb.stats()["search_failures"] == 0
        dumps = gb.dumps(1, copy=False)
        step("dump images")
        ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, dim, M, L.METRIC_L2).knn(q, k, ef, threads=8)
        del dumps
        step("oracle")
        monkeypatch.setenv("SHINE_DEBUG_VISCAP", "64")
        monkeypatch.setenv("SHINE_DEBUG_VIS16", "0")
        monkeypatch.setenv("SHINE_DEBUG_SHAPE", "1")
        out = {}
        with gb.open() as idx:  # the build's device arrays move into the handle
            assert idx.info()["id_space"] >= 1 << 26
            for mode in (L.MODE_EXACT, L.MODE_FAST):
                idx.set_search_mode(mode)
                capfd.readouterr()
                out[mode] = idx.knn(q, k, ef)
                err = capfd.readouterr().err
                assert " spill_hash 16384" in err, err  # the library chose the hash-table spill target
            # the library's own fast table at this id space once a call has been seen: two-choice u32 buckets
            # (kernels_impl.h VisitedLds<3>; capi.cc learned_max_table at SHINE_VT3_LOAD, grown to its residency level)
            monkeypatch.delenv("SHINE_DEBUG_VISCAP")
            monkeypatch.delenv("SHINE_DEBUG_VIS16")
            idx.set_search_mode(L.MODE_FAST)
            for _ in range(3):
                capfd.readouterr()
                out["learned"] = idx.knn(q, k, ef)
            err = capfd.readouterr().err
            shape = [ln for ln in err.splitlines() if ln.startswith("shape: pass 4")][-1].split()
            table, vis16, learned = int(shape[shape.index("table") + 1]), int(shape[shape.index("vis16") + 1]), \
                int(shape[shape.index("learned_fast") + 1])
            assert vis16 == 3 and learned >= 1024 and table % 4 == 0, shape  # two-choice u32 buckets, a learned size
            # and the exact pass's (the same load rule on the recent calls' mean query): bit for bit the oracle's
            idx.set_search_mode(L.MODE_EXACT)
            for _ in range(3):
                capfd.readouterr()
                out["learned_exact"] = idx.knn(q, k, ef)
            err = capfd.readouterr().err
            shape = [ln for ln in err.splitlines() if ln.startswith("shape: pass")][0].split()
            assert int(shape[shape.index("vis16") + 1]) == 3, shape
        step("searched")
    ex, fa = out[L.MODE_EXACT], out[L.MODE_FAST]
    assert ex.stats["overflow_retries"] == 0 and (ex.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(ex.ids, ref_ids)
    np.testing.assert_array_equal(ex.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(ex.qstats[:, :5], ref_qs[:, :5])
    assert (ex.qstats[:, L.QS_VISITED_L0] > 64).all()  # every query outgrew its 64-entry table
    clean = fa.qstats[:, L.QS_TIES] == 0
    assert clean.mean() >= 0.9
    order = np.argsort(ref_d, axis=1, kind="stable")
    s_ids, s_d = np.take_along_axis(ref_ids, order, 1), np.take_along_axis(ref_d, order, 1)
    np.testing.assert_array_equal(fa.dists[clean].view(np.uint32), s_d[clean].view(np.uint32))
    np.testing.assert_array_equal(np.sort(fa.ids[clean], 1), np.sort(s_ids[clean], 1))
    np.testing.assert_array_equal(fa.qstats[clean][:, :5], ref_qs[clean][:, :5])
    lx = out["learned_exact"]
    assert (lx.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(lx.ids, ref_ids)
    np.testing.assert_array_equal(lx.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(lx.qstats[:, :5], ref_qs[:, :5])
    le = out["learned"]
    clean = le.qstats[:, L.QS_TIES] == 0
    assert clean.mean() >= 0.9 and (le.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(le.dists[clean].view(np.uint32), s_d[clean].view(np.uint32))
    np.testing.assert_array_equal(np.sort(le.ids[clean], 1), np.sort(s_ids[clean], 1))
    np.testing.assert_array_equal(le.qstats[clean][:, :5], ref_qs[clean][:, :5])
