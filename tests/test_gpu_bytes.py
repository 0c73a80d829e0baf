"""Byte rows (SHINE_ELEM_U8 / _I8, include/shine_gpu.h) through the HIP path.

The reference reads .u8bin / .i8bin bases and widens every component to f32 (read_data.hh:21-28,
deserializer.hh:24-44), so its records hold byte values as floats.  A byte-row index stores those records as the
bytes they were and widens them in the kernels; the distance arithmetic is the f32 path's, so everything must be
bitwise what the f32 rows give: exact mode against the oracle (ids in heap order, distances, counters), fast mode
against fast mode on f32 rows (same ids, distances and counters, tie events included), the batched distance
kernel against the oracle's distance, and the sharded layout against the replica.
"""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def i8_like(n, seed=1, d=100):
    """SPACEV-shaped signed bytes: a clustered float set scaled and rounded into [-128, 127]."""
    x = np.rint(D.deep_like(n, seed=seed, d=d) * np.float32(300.0))
    np.clip(x, -128.0, 127.0, out=x)
    x += np.float32(0.0)  # no -0.0: it is not the f32 image of a byte
    return x.astype(np.float32)


CASES = [
    # name, generator, n, nq, dim, M, efc, metric, shards, k, ef, elem
    ("sift_u8_l2_d128", D.sift_like, 6000, 300, 128, 16, 100, 0, 1, 10, 128, L.ELEM_U8),
    ("sift_u8_ip_d128_2shards", D.sift_like, 4000, 200, 128, 8, 64, 1, 2, 10, 64, L.ELEM_U8),
    ("spacev_i8_l2_d100_2shards", i8_like, 5000, 300, 100, 16, 100, 0, 2, 10, 96, L.ELEM_I8),
    ("spacev_i8_ip_d100", i8_like, 4000, 200, 100, 16, 100, 1, 1, 10, 200, L.ELEM_I8),
]


@pytest.fixture(scope="module", params=CASES, ids=[c[0] for c in CASES])
def case(request):
    name, gen, n, nq, dim, M, efc, metric, shards, k, ef, elem = request.param
    base = gen(n, seed=71, d=dim)
    q = gen(nq, seed=72, d=dim)
    dumps, _, _ = O.build(base, M, efc, metric, shards, seed=7)
    ref = O.OracleIndex(dumps, dim, M, metric).knn(q, k, ef, threads=8)
    return dict(base=base, q=q, dumps=dumps, ref=ref, dim=dim, M=M, metric=metric, k=k, ef=ef, elem=elem)


def _knn(c, elem, mode, **kw):
    with shine_amd.Index.from_buffers(c["dumps"], c["dim"], c["M"], c["metric"], elem=elem, gpus=kw.pop("gpus", [0]),
                                      **kw) as idx:
        idx.set_search_mode(mode)
        info = idx.info()
        return idx.knn(c["q"], c["k"], c["ef"]), info


def test_byte_rows_exact_mode_is_the_oracle_bitwise(case, gpu_available):
    r, info = _knn(case, case["elem"], L.MODE_EXACT)
    assert info["elem"] == case["elem"]
    ref_ids, ref_d, ref_qs = case["ref"]
    assert (r.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(r.ids, ref_ids)
    np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(r.qstats[:, :8], ref_qs[:, :8])


def test_byte_rows_fast_mode_equals_f32_rows(case, gpu_available):
    rb, _ = _knn(case, case["elem"], L.MODE_FAST)
    rf, _ = _knn(case, L.ELEM_F32, L.MODE_FAST)
    assert (rb.qstats[:, L.QS_STATUS] == 0).all()
    np.testing.assert_array_equal(rb.ids, rf.ids)
    np.testing.assert_array_equal(rb.dists.view(np.uint32), rf.dists.view(np.uint32))
    np.testing.assert_array_equal(rb.qstats[:, :8], rf.qstats[:, :8])


def test_byte_rows_sharded_equal_replica(case, gpu_available):
    rr, _ = _knn(case, case["elem"], L.MODE_FAST)
    rs, info = _knn(case, case["elem"], L.MODE_FAST, gpus=[0, 0, 0], placement="sharded", cache=0.25)
    assert info["n_gpus"] == 3 and info["elem"] == case["elem"]
    np.testing.assert_array_equal(rs.ids, rr.ids)
    np.testing.assert_array_equal(rs.dists.view(np.uint32), rr.dists.view(np.uint32))
    assert rs.stats["cache_hits"] + rs.stats["cache_misses"] > 0


def test_auto_picks_the_narrowest_lossless_rows(gpu_available):
    for gen, dim, want in [(D.sift_like, 128, L.ELEM_U8), (i8_like, 100, L.ELEM_I8), (D.deep_like, 100, L.ELEM_F32),
                           (D.sift_like, 96, L.ELEM_F32)]:  # no byte kernels compiled at 96: f32 rows
        base = gen(600, seed=3, d=dim)
        dumps, _, _ = O.build(base, 8, 32, 0, 1, seed=3)
        with shine_amd.Index.from_buffers(dumps, dim, 8, 0, elem=L.ELEM_AUTO, gpus=[0]) as idx:
            info = idx.info()
        assert info["elem"] == want, (gen.__name__, dim, info["elem"])
        # the device footprint shrinks with the rows: 1 byte per component (16-byte rows) instead of 4
        if want != L.ELEM_F32:
            with shine_amd.Index.from_buffers(dumps, dim, 8, 0, elem=L.ELEM_F32, gpus=[0]) as i32:
                assert i32.info()["device_bytes"] - info["device_bytes"] == 600 * (4 * dim - (dim + 15) // 16 * 16)


def test_byte_rows_distance_kernel(gpu_available):
    import torch
    for dim, metric, gen, elem in [(128, 0, D.sift_like, L.ELEM_U8), (100, 1, i8_like, L.ELEM_I8),
                                   (100, 0, i8_like, L.ELEM_I8)]:
        base = gen(500, seed=41, d=dim)
        q = D.deep_like(33, seed=42, d=dim) * np.float32(50.0)  # float queries: only the records are bytes
        dumps, _, _ = O.build(base, 8, 32, metric, 1, seed=2)
        uids = np.random.default_rng(dim).integers(0, 500, (33, 77)).astype(np.uint32)
        with shine_amd.Index.from_buffers(dumps, dim, 8, metric, elem=elem, gpus=[0]) as idx:
            qt = torch.from_numpy(q).cuda()
            ut = torch.from_numpy(uids.view(np.int32)).cuda()
            out = torch.empty((33, 77), dtype=torch.float32, device="cuda")
            idx.distance_device(qt.data_ptr(), 33, ut.data_ptr(), 77, out.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
        for i in range(33):
            for j in range(77):
                ref = O.distance(metric, q[i], base[uids[i, j]])
                assert np.float32(ref).view(np.uint32) == got[i, j].view(np.uint32), (dim, metric, i, j)


def test_byte_rows_mixed_query_kinds_exact_mode_is_the_oracle(gpu_available):
    """Byte queries take the integer dot-product path (v_dot4), other queries the f32 path, decided per query:
    a batch mixing both (half-integers, out-of-range values, negative values against u8 rows) is the oracle
    bitwise either way."""
    for gen, dim, metric, elem in [(D.sift_like, 128, 0, L.ELEM_U8), (D.sift_like, 128, 1, L.ELEM_U8),
                                   (i8_like, 100, 0, L.ELEM_I8), (i8_like, 100, 1, L.ELEM_I8)]:
        base = gen(3000, seed=81, d=dim)
        q = gen(120, seed=82, d=dim).copy()
        q[1::4] += np.float32(0.5)      # not integers
        q[2::4, 0] = np.float32(300.0)  # out of the byte range
        q[3::8, 5] = np.float32(-1.0)   # negative: a byte value for i8 rows only
        dumps, _, _ = O.build(base, 12, 64, metric, 1, seed=9)
        ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, dim, 12, metric).knn(q, 10, 64, threads=8)
        with shine_amd.Index.from_buffers(dumps, dim, 12, metric, elem=elem, gpus=[0]) as idx:
            r = idx.knn(q, 10, 64)
        np.testing.assert_array_equal(r.ids, ref_ids)
        np.testing.assert_array_equal(r.dists.view(np.uint32), ref_d.view(np.uint32))
        np.testing.assert_array_equal(r.qstats[:, :8], ref_qs[:, :8])


def test_byte_rows_distance_kernel_byte_queries(gpu_available):
    import torch
    for dim, metric, gen, elem in [(128, 0, D.sift_like, L.ELEM_U8), (128, 1, D.sift_like, L.ELEM_U8),
                                   (100, 1, i8_like, L.ELEM_I8), (100, 0, i8_like, L.ELEM_I8)]:
        base = gen(500, seed=43, d=dim)
        q = gen(21, seed=44, d=dim)  # byte queries: the integer path
        dumps, _, _ = O.build(base, 8, 32, metric, 1, seed=2)
        uids = np.random.default_rng(dim + metric).integers(0, 500, (21, 70)).astype(np.uint32)
        with shine_amd.Index.from_buffers(dumps, dim, 8, metric, elem=elem, gpus=[0]) as idx:
            qt = torch.from_numpy(q).cuda()
            ut = torch.from_numpy(uids.view(np.int32)).cuda()
            out = torch.empty((21, 70), dtype=torch.float32, device="cuda")
            idx.distance_device(qt.data_ptr(), 21, ut.data_ptr(), 70, out.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
        for i in range(21):
            for j in range(70):
                ref = O.distance(metric, q[i], base[uids[i, j]])
                assert np.float32(ref).view(np.uint32) == got[i, j].view(np.uint32), (dim, metric, i, j)
