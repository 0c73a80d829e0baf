"""GPU parity: the HIP search / distance kernels through the C ABI vs the CPU oracle, on identical dumps.

Bar (north star): identical neighbour ids.  Here the bar is stricter — the kernels reproduce the oracle's FP
order and libstdc++'s heap algorithms, so ids (in heap-array order), distances (bitwise) and every per-query
counter must be identical, ties included.
"""
import os

import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def _check_same(r, ref_ids, ref_d, ref_qs):
    assert (r.qstats[:, shine_amd.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    # distcomps, visited (upper, L0), lists (upper, L0), peak next size, n results
    np.testing.assert_array_equal(r.qstats[:, [0, 1, 2, 3, 4, 5, 7]], ref_qs[:, [0, 1, 2, 3, 4, 5, 7]])


CASES = [
    # name, generator, n, nq, dim, M, efc, metric, shards, k, ef
    ("sift_l2_m16", D.sift_like, 6000, 200, 128, 16, 100, 0, 1, 10, 64),
    ("sift_l2_m16_3shards", D.sift_like, 6000, 200, 128, 16, 100, 0, 3, 10, 128),
    ("sift_l2_m8_ef256", D.sift_like, 4000, 100, 128, 8, 64, 0, 2, 10, 256),
    ("deep_ip_d96", D.deep_like, 5000, 150, 96, 16, 100, 1, 1, 10, 100),
    ("deep_l2_d96", D.deep_like, 4000, 100, 96, 12, 80, 0, 4, 5, 40),
    ("tti_ip_d200_tail", D.tti_like, 3000, 100, 200, 16, 80, 1, 2, 10, 64),
    ("m32_lists64", D.sift_like, 3000, 100, 128, 32, 100, 0, 1, 10, 64),
    ("k_eq_ef", D.sift_like, 2000, 64, 128, 16, 64, 0, 1, 20, 20),
]


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request):
    name, gen, n, nq, dim, M, efc, metric, shards, k, ef = request.param
    base = gen(n, seed=101, d=dim)
    q = gen(nq, seed=202, d=dim)
    dumps, _, _ = O.build(base, M, efc, metric, shards, seed=5)
    ref = O.OracleIndex(dumps, dim, M, metric).knn(q, k, ef)
    return dict(base=base, q=q, dumps=dumps, dim=dim, M=M, metric=metric, k=k, ef=ef, ref=ref)


def test_knn_parity(case, gpu_available):
    with shine_amd.Index.from_buffers(case["dumps"], case["dim"], case["M"], case["metric"], gpus=[0]) as idx:
        r = idx.knn(case["q"], case["k"], case["ef"])
    _check_same(r, *case["ref"])


def test_knn_parity_u16_visited(case, gpu_available, monkeypatch):
    """The exact kernel with the u16 quotient visited table (VisitedLds<1>; chosen on large batches, where it lets
    more wavefronts share a CU), forced here on every case: same bar."""
    monkeypatch.setenv("SHINE_DEBUG_VIS16", "1")
    with shine_amd.Index.from_buffers(case["dumps"], case["dim"], case["M"], case["metric"], gpus=[0]) as idx:
        r = idx.knn(case["q"], case["k"], case["ef"])
    _check_same(r, *case["ref"])


def test_exact_large_batch_picks_u16_and_matches(gpu_available):
    """2,048 queries want 8 wavefronts per CU: the u16 table (7 fit) beats the u32 one (4 fit), so the exact pass
    runs VisitedLds<1> without any hook.  Every query must still match the oracle bitwise."""
    base = D.sift_like(20000, seed=41)
    q = D.sift_like(2048, seed=42)
    dumps, _ = shine_amd.build(base, 16, 100, 0, 1, seed=6, threads=8)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 128)
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        r = idx.knn(q, 10, 128)
    _check_same(r, *ref)


def test_knn_device_entry(case, gpu_available):
    import torch
    q = torch.from_numpy(case["q"]).cuda()
    nq, k = q.shape[0], case["k"]
    ids = torch.empty((nq, k), dtype=torch.int32, device="cuda")
    dd = torch.empty((nq, k), dtype=torch.float32, device="cuda")
    qs = torch.empty((nq, shine_amd.QS_WORDS), dtype=torch.int32, device="cuda")
    with shine_amd.Index.from_buffers(case["dumps"], case["dim"], case["M"], case["metric"], gpus=[0]) as idx:
        idx.knn_device(q.data_ptr(), nq, k, case["ef"], ids.data_ptr(), dd.data_ptr(), qs.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    ref_ids, ref_d, ref_qs = case["ref"]
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), ref_ids)
    np.testing.assert_array_equal(dd.cpu().numpy().view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(qs.cpu().numpy().view(np.uint32)[:, :5], ref_qs[:, :5])


def test_overflow_rerun_path(gpu_available, monkeypatch):
    """A first pass with a 24-entry next_candidates queue overflows; the re-run must give identical results."""
    base = D.sift_like(4000, seed=7)
    q = D.sift_like(64, seed=8)
    dumps, _, _ = O.build(base, 16, 100, 0, 1, seed=3)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 128)
    assert ref[2][:, 5].max() > 24
    monkeypatch.setenv("SHINE_DEBUG_CAP", "24")
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        r = idx.knn(q, 10, 128)
    assert r.stats["overflow_retries"] > 0
    _check_same(r, *ref)


def test_tight_next_room_hands_on_and_matches(gpu_available, capfd, monkeypatch):
    """ef = 400 and 2,048 queries: the fixed next_candidates room (5 ef) leaves 5 wavefronts per CU, so the exact pass
    reserves 3 ef (capi.cc pick_shape, 7 per CU) and its capacity is what that LDS share leaves; queries that outgrow it
    are handed on to the next pass.  The shape line shows the pick; every query must still equal the oracle bit for
    bit."""
    monkeypatch.setenv("SHINE_DEBUG_SHAPE", "1")
    base = D.sift_like(3000, seed=51)
    q = D.sift_like(2048, seed=52)
    dumps, _, _ = O.build(base, 16, 100, 0, 1, seed=7)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 400)
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        for _ in range(2):  # (the second call's table is learned from the first)
            r = idx.knn(q, 10, 400)
            _check_same(r, *ref)
    shapes = [ln for ln in capfd.readouterr().err.splitlines() if ln.startswith("shape: pass 0")]
    assert shapes
    f = shapes[-1].split()
    waves, cap = int(f[f.index("waves") + 1]), int(f[f.index("cap") + 1])
    assert 5 < waves <= 16 and cap < 5 * 400  # the 3 ef room was taken: more wavefronts, a capacity below 5 ef


def test_repeated_batches_keep_visited_clean(gpu_available):
    """The visited bitmaps are cleared per query from the visited log: re-running must not change anything."""
    base = D.sift_like(5000, seed=21)
    q = D.sift_like(300, seed=22)
    dumps, _, _ = O.build(base, 16, 100, 0, 1, seed=4)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 64)
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        for _ in range(3):
            _check_same(idx.knn(q, 10, 64), *ref)
        # a batch with fewer queries than slots, then a single query
        r = idx.knn(q[:7], 10, 64)
        np.testing.assert_array_equal(r.ids, ref[0][:7])
        r = idx.knn(q[5:6], 10, 64)
        np.testing.assert_array_equal(r.ids, ref[0][5:6])


def test_duplicate_vectors_ties(gpu_available):
    """Many exactly-equal distances (duplicated base vectors): tie order must follow libstdc++'s heaps."""
    rng = np.random.default_rng(3)
    uniq = np.rint(rng.uniform(0, 4, (300, 16))).astype(np.float32)
    base = uniq[rng.integers(0, 300, 3000)]
    q = np.rint(rng.uniform(0, 4, (100, 16))).astype(np.float32)
    dumps, _, _ = O.build(base, 8, 40, 0, 2, seed=9)
    ref = O.OracleIndex(dumps, 16, 8, 0).knn(q, 10, 50)
    with shine_amd.Index.from_buffers(dumps, 16, 8, 0, gpus=[0]) as idx:
        _check_same(idx.knn(q, 10, 50), *ref)


@pytest.mark.parametrize("n", [1, 2, 17])
def test_tiny_graphs(n, gpu_available):
    base = D.sift_like(n, seed=31)
    q = D.sift_like(9, seed=32)
    dumps, _, _ = O.build(base, 4, 16, 0, 1, seed=1)
    ref = O.OracleIndex(dumps, 128, 4, 0).knn(q, 10, 16)
    with shine_amd.Index.from_buffers(dumps, 128, 4, 0, gpus=[0]) as idx:
        r = idx.knn(q, 10, 16)
    np.testing.assert_array_equal(r.ids, ref[0])
    np.testing.assert_array_equal(r.qstats[:, 7], ref[2][:, 7])


def test_distance_kernel_parity(gpu_available):
    import torch
    for dim, metric, gen in [(128, 0, D.sift_like), (96, 1, D.deep_like), (200, 1, D.tti_like), (100, 0, D.deep_like)]:
        base = gen(500, seed=41, d=dim)
        q = gen(33, seed=42, d=dim)
        dumps, _, _ = O.build(base, 8, 32, metric, 1, seed=2)
        rng = np.random.default_rng(dim)
        uids = rng.integers(0, 500, (33, 77)).astype(np.uint32)
        uids[0, 3] = 10_000  # unknown uid → NaN
        with shine_amd.Index.from_buffers(dumps, dim, 8, metric, gpus=[0]) as idx:
            qt = torch.from_numpy(q).cuda()
            ut = torch.from_numpy(uids.view(np.int32)).cuda()
            out = torch.empty((33, 77), dtype=torch.float32, device="cuda")
            idx.distance_device(qt.data_ptr(), 33, ut.data_ptr(), 77, out.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
        for i in range(33):
            for j in range(77):
                if i == 0 and j == 3:
                    assert np.isnan(got[i, j])
                    continue
                ref = O.distance(metric, q[i], base[uids[i, j]])
                assert np.float32(ref).view(np.uint32) == got[i, j].view(np.uint32), (dim, metric, i, j)


def test_open_from_files_and_errors(tmp_path, gpu_available):
    base = D.sift_like(1500, seed=51)
    q = D.sift_like(20, seed=52)
    dumps, _, _ = O.build(base, 16, 60, 0, 2, seed=6)
    paths = []
    for i, d in enumerate(dumps):
        p = tmp_path / shine_amd.dump_name(16, 60, i, 2)
        d.tofile(p)
        paths.append(p)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 32)
    with shine_amd.Index.open(paths, 128, 16, 0, gpus=[0]) as idx:
        info = idx.info()
        assert info["num_nodes"] == 1500 and info["n_shards"] == 2
        r = idx.knn(q, 10, 32)
        np.testing.assert_array_equal(r.ids, ref[0])
        with pytest.raises(shine_amd.ShineError) as e:
            idx.knn(q, 10, 5)  # ef < k (hnsw.hh:36)
        assert e.value.code == 1
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.open([tmp_path / "missing.dat"], 128, 16, 0, gpus=[0])
    assert e.value.code == 2


@pytest.mark.skipif(os.environ.get("SHINE_SKIP_F16") == "1", reason="disabled")
def test_fp16_records_recall(gpu_available):
    """Config 5 converts records to fp16 at load: ids cannot be bit-exact; recall must match the f32 path."""
    base = D.tti_like(6000, seed=61)
    q = D.tti_like(200, seed=62)
    dumps, _, _ = O.build(base, 16, 100, 1, 2, seed=8)
    gt, _ = D.brute_force_knn(base, q, 10, metric=1)
    with shine_amd.Index.from_buffers(dumps, 200, 16, 1, elem=shine_amd.ELEM_F32, gpus=[0]) as i32, \
            shine_amd.Index.from_buffers(dumps, 200, 16, 1, elem=shine_amd.ELEM_F16, gpus=[0]) as i16:
        r32 = D.recall_at_k(i32.knn(q, 10, 128).ids, gt, 10)
        r16 = D.recall_at_k(i16.knn(q, 10, 128).ids, gt, 10)
    assert r16 >= r32 - 0.02, (r16, r32)


def _heap_ops(rng, n_ops, ties):
    ops = rng.choice([0, 0, 0, 1, 2], n_ops).astype(np.int32)
    vals = (rng.integers(0, 6, n_ops) if ties else rng.permutation(n_ops)).astype(np.float32)
    ids = np.arange(n_ops, dtype=np.uint32)
    return ops, vals, ids


@pytest.mark.parametrize("general", [False, True])
@pytest.mark.parametrize("is_max", [True, False])
@pytest.mark.parametrize("ties", [True, False])
def test_device_heaps_match_libstdcxx(is_max, ties, general, gpu_available):
    """The wave-parallel push/pop the kernel uses must leave the exact heap array libstdc++ leaves."""
    import ctypes as C
    L = shine_amd._lib
    rng = np.random.default_rng(17 + is_max + 2 * ties)
    for n_ops, k in [(1, 1), (2, 1), (7, 3), (100, 8), (600, 40), (3000, 128), (5000, 5000)]:
        ops, vals, ids = _heap_ops(rng, n_ops, ties)
        ref_d, ref_i = O.heap_replay(is_max, ops, vals, ids, k)
        od = np.empty(n_ops + 1, np.float32)
        oi = np.empty(n_ops + 1, np.uint32)
        on = np.zeros(1, np.uint32)
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        kk = k | (0x80000000 if general else 0)  # high bit: the general (NaN-safe) pop
        L.check(L.lib().shine_selftest_heap(int(is_max), p(ops), p(vals), p(ids), n_ops, kk, p(od), p(oi), p(on)))
        n = int(on[0])
        assert n == ref_d.size, (n_ops, k)
        np.testing.assert_array_equal(oi[:n], ref_i)
        np.testing.assert_array_equal(od[:n], ref_d)


@pytest.mark.parametrize("env", [{"SHINE_DEBUG_VISCAP": "1024", "SHINE_DEBUG_NO_SPILL": "1"},
                                 {"SHINE_DEBUG_START_MODE": "1"},
                                 {"SHINE_DEBUG_START_MODE": "2"}, {"SHINE_DEBUG_START_MODE": "3"},
                                 {"SHINE_DEBUG_VISCAP": "1024", "SHINE_DEBUG_LIGHT_CAP": "16", "SHINE_DEBUG_NO_SPILL": "1"}])
def test_visited_modes(env, gpu_available, monkeypatch):
    """Every pass of the chain alone or handed overflowing queries: the whole-CU LDS pass (start mode 1), the
    light pass (HBM visited bitmap, 16 KiB LDS heaps; start mode 2), the global-heap pass (bitmap and both heaps in
    HBM; start mode 3), and a light pass too small for most queries: identical results."""
    base = D.sift_like(8000, seed=71)
    q = D.sift_like(128, seed=72)
    dumps, _, _ = O.build(base, 16, 100, 0, 1, seed=3)
    ref = O.OracleIndex(dumps, 128, 16, 0).knn(q, 10, 200)
    for k_, v in env.items():
        monkeypatch.setenv(k_, v)
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        r = idx.knn(q, 10, 200)
        if "SHINE_DEBUG_VISCAP" in env:
            assert r.stats["overflow_retries"] > 0
        _check_same(r, *ref)
        _check_same(idx.knn(q, 10, 200), *ref)


@pytest.mark.parametrize("vis16", ["0", "1"])
@pytest.mark.parametrize("gen,dim,metric,ef", [(D.sift_like, 128, 0, 128), (D.deep_like, 96, 1, 256)])
def test_exact_mode_spills_in_place(gen, dim, metric, ef, vis16, gpu_available, monkeypatch):
    """Exact mode with a 256-entry visited table: every query outgrows it, spills it into an HBM bitmap mid-search
    and goes on there (the in-place spill the fast kernel has); more queries than the 64 bitmaps spill at once, so
    the rest are handed to the light pass.  Both paths: ids, distances and every counter identical to the oracle."""
    base = gen(6000, seed=311, d=dim)
    q = gen(300, seed=312, d=dim)
    dumps, _, _ = O.build(base, 16, 100, metric, 1, seed=6)
    ref = O.OracleIndex(dumps, dim, 16, metric).knn(q, 10, ef, threads=8)
    monkeypatch.setenv("SHINE_DEBUG_VISCAP", "256")
    monkeypatch.setenv("SHINE_DEBUG_VIS16", vis16)
    with shine_amd.Index.from_buffers(dumps, dim, 16, metric, gpus=[0]) as idx:
        r = idx.knn(q, 10, ef)
        assert r.stats["overflow_retries"] < q.shape[0]  # some queries went on in place instead of being re-run
        _check_same(r, *ref)
        for i in range(0, 32, 8):  # a few queries at a time: every spill finds a free bitmap, none is handed on
            one = idx.knn(q[i:i + 8], 10, ef)
            assert one.stats["overflow_retries"] == 0
            np.testing.assert_array_equal(one.ids, ref[0][i:i + 8])
            np.testing.assert_array_equal(one.dists.view(np.uint32), ref[1][i:i + 8].view(np.uint32))
            np.testing.assert_array_equal(one.qstats[:, :5], ref[2][i:i + 8, :5])


@pytest.mark.parametrize("viscap,vis_bits", [("4096", "24"), ("1024", "22")], ids=["24bit_ids", "22bit_ids_spill"])
def test_exact_mode_two_choice_tables(viscap, vis_bits, gpu_available, monkeypatch, capfd):
    """Exact mode on two-choice u16 tables (VisitedLds<2>, SHINE_DEBUG_VIS16=2) with the id space widened to 22-24
    bits: 4,096 entries at 24 bits (cfg 3's shape), and 1,024 entries at 22 bits, which every query outgrows (the
    table spills, decoded into the HBM bitmap).  Ids in heap-array order, distances and every counter equal the
    oracle's."""
    base = D.deep_like(6000, seed=313, d=96)
    q = D.deep_like(200, seed=314, d=96)
    dumps, _, _ = O.build(base, 16, 100, 1, 1, seed=6)
    ref = O.OracleIndex(dumps, 96, 16, 1).knn(q, 10, 128, threads=8)
    monkeypatch.setenv("SHINE_DEBUG_VISCAP", viscap)
    monkeypatch.setenv("SHINE_DEBUG_VIS_BITS", vis_bits)
    monkeypatch.setenv("SHINE_DEBUG_VIS16", "2")
    monkeypatch.setenv("SHINE_DEBUG_SHAPE", "1")
    with shine_amd.Index.from_buffers(dumps, 96, 16, 1, gpus=[0]) as idx:
        capfd.readouterr()
        r = idx.knn(q, 10, 128)
        err = capfd.readouterr().err
        assert " vis16 2 " in err, err
        _check_same(r, *ref)


def test_global_heap_capacity_overflow_is_reported(gpu_available, monkeypatch):
    """The last pass's capacity is the only hard limit: a query that outgrows it fails with SHINE_ERR_OVERFLOW in
    its status word and shine_knn_batch returns that status (no silent truncation)."""
    base = D.sift_like(3000, seed=95)
    q = D.sift_like(8, seed=96)
    dumps, _, _ = O.build(base, 8, 40, 0, 1, seed=2)
    monkeypatch.setenv("SHINE_DEBUG_START_MODE", "3")
    monkeypatch.setenv("SHINE_DEBUG_GLOBAL_CAP", "4")
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0]) as idx:
        with pytest.raises(shine_amd.ShineError) as e:
            idx.knn(q, 10, 64)
    assert e.value.code == shine_amd._lib.ERR_OVERFLOW


def test_nan_distances_follow_reference(gpu_available):
    """NaN components give NaN distances: comparisons with NaN are false in the reference too, so the search
    still has one exact outcome; the kernel switches to its general heap routine and must reproduce it."""
    base = D.sift_like(3000, seed=81)
    base[::97, 5] = np.nan
    q = D.sift_like(64, seed=82)
    q[3, 7] = np.nan
    dumps, _, _ = O.build(base, 8, 40, 0, 1, seed=2)
    ref = O.OracleIndex(dumps, 128, 8, 0).knn(q, 10, 48)
    with shine_amd.Index.from_buffers(dumps, 128, 8, 0, gpus=[0]) as idx:
        r = idx.knn(q, 10, 48)
    np.testing.assert_array_equal(r.ids, ref[0])
    nan = np.isnan(ref[1])
    np.testing.assert_array_equal(np.isnan(r.dists), nan)  # NaN sign/payload is not specified by IEEE 754
    np.testing.assert_array_equal(r.dists[~nan].view(np.uint32), ref[1][~nan].view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :5], ref[2][:, :5])


def test_device_api_zero_copy_pinned_host_buffers(gpu_available):
    """shine_knn_batch_device on pinned host memory (queries read and results written by the kernels over PCIe,
    bench.py value_host_to_host): the oracle's answers, bitwise, in exact mode."""
    import torch
    base = D.sift_like(3000, seed=61)
    qn = D.sift_like(200, seed=62)
    dumps, _, _ = O.build(base, 16, 80, 0, 1, seed=6)
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, 128, 16, 0).knn(qn, 10, 64)
    with shine_amd.Index.from_buffers(dumps, 128, 16, 0, gpus=[0]) as idx:
        qh = torch.from_numpy(qn).pin_memory()
        ids = torch.empty((200, 10), dtype=torch.int32).pin_memory()
        dd = torch.empty((200, 10), dtype=torch.float32).pin_memory()
        qs = torch.empty((200, shine_amd.QS_WORDS), dtype=torch.int32).pin_memory()
        st = torch.cuda.Stream()
        idx.knn_device(qh.data_ptr(), 200, 10, 64, ids.data_ptr(), dd.data_ptr(), qs.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        idx.release_stream(st.cuda_stream)
    np.testing.assert_array_equal(ids.numpy().view(np.uint32), ref_ids)
    np.testing.assert_array_equal(dd.numpy().view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(qs.numpy().view(np.uint32)[:, :8], ref_qs[:, :8])
