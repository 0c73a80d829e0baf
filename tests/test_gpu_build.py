"""GPU batch builder (shine_gpu_build): HNSW::insert + select_heuristic on the GPU.

* the GPU-built graph is a valid index in the reference's dump layout: every list within capacity, no duplicates or
  self loops, levels drawn exactly as the CPU builder draws them, everything reachable;
* searching it through its own handle equals searching its dumps (reopened over 3 memory nodes) bitwise, and both
  equal the oracle's knn on those dumps (exact mode: ids, distances, counters);
* the build is deterministic;
* its recall matches the CPU builder's (same data, same M / efC);
* byte and fp16 rows open from the built arrays (u8 rows bitwise equal to f32 rows on byte-valued data).
"""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D

pytestmark = pytest.mark.gpu


def _gt(base, q, k, metric):
    import torch
    bt = torch.from_numpy(base).cuda().double()
    qt = torch.from_numpy(q).cuda().double()
    d = (qt * qt).sum(1)[:, None] + (bt * bt).sum(1)[None, :] - 2.0 * (qt @ bt.T) if metric == 0 else 1.0 - qt @ bt.T
    return torch.topk(d, k, largest=False).indices.cpu().numpy()


def _walk(dump, dim, M):
    """(uid, level, [lists]) of every record of one dump (memory_node.hh:15-27, node.hh:10-19)."""
    free = int(np.frombuffer(dump[:8].tobytes(), np.uint64)[0])
    off, out = 16, []
    while off < free:
        uid, level = (int(x) for x in np.frombuffer(dump[off + 8:off + 16].tobytes(), np.uint32))
        lists = []
        lo = off + 16 + 4 * dim
        for lv in range(level + 1):
            cap = 2 * M if lv == 0 else M
            cnt = int(np.frombuffer(dump[lo:lo + 4].tobytes(), np.uint32)[0])
            assert cnt <= cap
            lists.append(np.frombuffer(dump[lo + 4:lo + 4 + 8 * cnt].tobytes(), np.uint64).copy())
            lo += 4 + 8 * cap
        out.append((uid, level, lists, off))
        size = 16 + 4 * dim + 4 + 8 * 2 * M + level * (4 + 8 * M)
        off += size + (-size) % 8
    return out


@pytest.mark.parametrize("metric,gen,dim", [(0, "sift", 128), (1, "deep", 96)])
def test_gpu_build_valid_and_searches_equal_the_oracle(gpu_available, metric, gen, dim):
    n, M, efc = 30_000, 12, 96
    make = D.sift_like if gen == "sift" else D.deep_like
    base = make(n, seed=31, d=dim)
    q = make(256, seed=32, d=dim)
    with shine_amd.GpuBuild(base, M, efc, metric, seed=5, batch_fraction=0.05) as gb:
        st = gb.stats()
        assert st["num_nodes"] == n and st["search_failures"] == 0 and st["batches"] > 10
        dumps = gb.dumps(3)
        dumps_again = None
        with shine_amd.GpuBuild(base, M, efc, metric, seed=5, batch_fraction=0.05) as gb2:
            dumps_again = gb2.dumps(3)
        for a, b in zip(dumps, dumps_again):  # deterministic
            assert np.array_equal(a, b)
        with gb.open() as idx:
            direct = idx.knn(q, 10, 64)
            idx.set_search_mode(L.MODE_FAST)
            direct_fast = idx.knn(q, 10, 64)
    # layout: levels as the CPU builder draws them, lists within capacity, no duplicates / self loops
    lv_ref, _ = O.draw_levels(n, M, 5)
    recs = {}
    for s, d in enumerate(dumps):
        for uid, level, lists, off in _walk(d, dim, M):
            recs[(s, off)] = (uid, level, lists)
    assert len(recs) == n
    by_uid = {v[0]: v for v in recs.values()}
    levels = np.array([by_uid[i][1] for i in range(n)])
    top, expect = 0, np.zeros(n, np.int64)  # insert(): first record level 0, a higher draw takes top + 1
    for i in range(1, n):
        if lv_ref[i] > top:
            top += 1
            expect[i] = top
        else:
            expect[i] = lv_ref[i]
    np.testing.assert_array_equal(levels, expect)
    for uid, level, lists in recs.values():
        for lst in lists:
            targets = [recs[(int(r) >> 48, int(r) & ((1 << 48) - 1))][0] for r in lst]
            assert len(set(targets)) == len(targets) and uid not in targets
    gs = shine_amd.graph_stats(dumps, dim, M)
    assert gs["reachable_l0"] >= n - 2 and gs["max_level"] == st["max_level"]
    # the dumps reopened over 3 memory nodes search exactly like the built handle, and like the oracle
    with shine_amd.Index.from_buffers(dumps, dim, M, metric, gpus=[0]) as idx:
        re = idx.knn(q, 10, 64)
    np.testing.assert_array_equal(re.ids, direct.ids)
    np.testing.assert_array_equal(re.dists.view(np.uint32), direct.dists.view(np.uint32))
    np.testing.assert_array_equal(re.qstats[:, :5], direct.qstats[:, :5])
    ref_ids, ref_d, ref_qs = O.OracleIndex(dumps, dim, M, metric).knn(q[:64], 10, 64)
    np.testing.assert_array_equal(direct.ids[:64], ref_ids)
    np.testing.assert_array_equal(direct.dists[:64].view(np.uint32), ref_d.view(np.uint32))
    np.testing.assert_array_equal(direct.qstats[:64, :5], ref_qs[:, :5])
    clean = direct_fast.qstats[:, L.QS_TIES] == 0
    np.testing.assert_array_equal(np.sort(direct_fast.ids[clean], 1), np.sort(direct.ids[clean], 1))
    # recall against the CPU builder's index on the same data
    cpu_dumps, _ = shine_amd.build(base, M, efc, metric, 1, seed=5, threads=16)
    with shine_amd.Index.from_buffers(cpu_dumps, dim, M, metric, gpus=[0]) as idx:
        cpu = idx.knn(q, 10, 64)
    gt = _gt(base, q, 10, metric)
    r_gpu, r_cpu = D.recall_at_k(direct.ids, gt, 10), D.recall_at_k(cpu.ids, gt, 10)
    assert r_gpu >= r_cpu - 0.01, (r_gpu, r_cpu)


def test_gpu_build_from_device_rows_and_row_kinds(gpu_available):
    import torch
    n, M, efc = 8_000, 8, 64
    base = D.sift_like(n, seed=41)
    q = D.sift_like(128, seed=42)
    bt = torch.from_numpy(base).cuda()
    gb_dev = shine_amd.GpuBuild(bt.data_ptr(), M, efc, 0, seed=9, n=n, dim=128)
    gb_host = shine_amd.GpuBuild(base, M, efc, 0, seed=9)
    a, b = gb_dev.dumps(1), gb_host.dumps(1)
    assert np.array_equal(a[0], b[0])  # device rows and host rows build the same index
    with gb_dev.open(L.ELEM_F32) as f32, gb_host.open(L.ELEM_U8) as u8:
        assert u8.info()["elem"] == L.ELEM_U8
        r32, r8 = f32.knn(q, 10, 48), u8.knn(q, 10, 48)
    np.testing.assert_array_equal(r32.ids, r8.ids)
    np.testing.assert_array_equal(r32.dists.view(np.uint32), r8.dists.view(np.uint32))
    with pytest.raises(shine_amd.ShineError):  # the arrays moved into the handle
        gb_dev.open(L.ELEM_F32)
    gb_dev.close()
    gb_host.close()
    # float rows: u8 refused, fp16 rows searched with recall close to f32's
    deep = D.deep_like(n, seed=43)
    dq = D.deep_like(128, seed=44)
    with shine_amd.GpuBuild(deep, M, efc, 1, seed=9) as gb:
        with pytest.raises(shine_amd.ShineError):
            gb.open(L.ELEM_U8)
        with gb.open(L.ELEM_F16) as h16:
            r16 = h16.knn(dq, 10, 64)
    gt = _gt(deep, dq, 10, 1)
    assert D.recall_at_k(r16.ids, gt, 10) > 0.9
    del bt
    torch.cuda.synchronize()


def test_gpu_build_open_ex_equals_its_dumps(gpu_available):
    """shine_gpu_build_open_ex lays the build out as the dumps of the same memory nodes would be: sharded over two GPU
    slots (one device: every stripe its own allocation) it answers exactly as those dumps opened the same way, and as
    the replica."""
    n, M, efc = 20_000, 8, 64
    base = D.deep_like(n, seed=51)
    q = D.deep_like(200, seed=52)
    with shine_amd.GpuBuild(base, M, efc, 0, seed=3) as gb:
        dumps = gb.dumps(4)
        with gb.open_ex(4, gpus=[0, 0], placement="sharded", cache=0.1) as sh, \
                shine_amd.Index.from_buffers(dumps, 96, M, 0, gpus=[0, 0], placement="sharded", cache=0.1) as shd:
            a, b = sh.knn(q, 10, 48), shd.knn(q, 10, 48)
            assert sh.info()["id_space"] == shd.info()["id_space"]
        with gb.open() as rep:
            c = rep.knn(q, 10, 48)
    np.testing.assert_array_equal(a.ids, b.ids)
    np.testing.assert_array_equal(a.dists.view(np.uint32), b.dists.view(np.uint32))
    np.testing.assert_array_equal(a.qstats, b.qstats)
    np.testing.assert_array_equal(a.ids, c.ids)
