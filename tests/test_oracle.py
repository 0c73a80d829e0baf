"""The oracle against the committed golden fixtures, an independent Python restatement, and libstdc++'s RNG."""
import hashlib
import json
import random

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN
from pyref import PyRef, pop_heap, push_heap, _max_cmp, _min_cmp
from shine_amd import datasets as D
from shine_amd import formats as F

META = json.loads((GOLDEN / "meta.json").read_text())


@pytest.fixture(scope="module")
def cfg1():
    _, base = F.read_vectors(GOLDEN / "base.u8bin")
    _, q = F.read_vectors(GOLDEN / "query.u8bin")
    _, gt = F.read_vectors(GOLDEN / "groundtruth.bin")
    c = META["cfg1"]
    dumps, dc, ml = O.build(base, c["M"], c["efc"], 0, 1, c["seed"])
    return dict(base=base, q=q, gt=gt, dumps=dumps, dc=dc, ml=ml, c=c)


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_golden_base_is_siftsmall_shaped(cfg1):
    assert cfg1["base"].shape == (10_000, 128) and cfg1["q"].shape == (100, 128)
    assert cfg1["gt"].shape == (100, 100)
    assert np.array_equal(cfg1["base"], np.rint(cfg1["base"]))


def test_golden_dump_bytes(cfg1):
    m = META["dumps"]["l2_1"]
    assert [d.size for d in cfg1["dumps"]] == m["sizes"]
    assert [_sha(d) for d in cfg1["dumps"]] == m["sha256"]
    assert cfg1["dc"] == m["build_distcomps"] and cfg1["ml"] == m["max_level"]


def test_golden_multishard_dump_bytes(cfg1):
    c = cfg1["c"]
    dumps, _, _ = O.build(cfg1["base"], c["M"], c["efc"], 0, 3, c["seed"])
    assert [_sha(d) for d in dumps] == META["dumps"]["l2_3"]["sha256"]


def test_golden_knn(cfg1):
    c = cfg1["c"]
    exp = np.load(GOLDEN / "expected_l2.npz")
    ids, dd, qs = O.OracleIndex(cfg1["dumps"], c["dim"], c["M"], 0).knn(cfg1["q"], c["k"], c["ef"])
    np.testing.assert_array_equal(ids, exp["ids"])
    np.testing.assert_array_equal(dd.view(np.uint32), exp["dists"].view(np.uint32))
    np.testing.assert_array_equal(qs, exp["qstats"])
    assert D.recall_at_k(ids, cfg1["gt"], c["k"]) >= 0.95


def test_golden_knn_multithreaded_same(cfg1):
    c = cfg1["c"]
    I = O.OracleIndex(cfg1["dumps"], c["dim"], c["M"], 0)
    a = I.knn(cfg1["q"], c["k"], c["ef"], threads=1)
    b = I.knn(cfg1["q"], c["k"], c["ef"], threads=4)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_golden_ip():
    ip = META["ip"]
    _, b = F.read_vectors(GOLDEN / "ip_base.fbin")
    _, q = F.read_vectors(GOLDEN / "ip_query.fbin")
    dumps, _, _ = O.build(b, ip["M"], ip["efc"], 1, ip["shards"][0], ip["seed"])
    assert [_sha(d) for d in dumps] == META["dumps"]["ip_2"]["sha256"]
    exp = np.load(GOLDEN / "expected_ip.npz")
    ids, dd, qs = O.OracleIndex(dumps, ip["dim"], ip["M"], 1).knn(q, ip["k"], ip["ef"])
    np.testing.assert_array_equal(ids, exp["ids"])
    np.testing.assert_array_equal(dd.view(np.uint32), exp["dists"].view(np.uint32))
    np.testing.assert_array_equal(qs, exp["qstats"])


def test_oracle_matches_independent_python_restatement(cfg1):
    """Two restatements (C++ with libstdc++'s heaps; Python restating libstdc++'s algorithms) must agree."""
    c = cfg1["c"]
    ids, dd, qs = O.OracleIndex(cfg1["dumps"], c["dim"], c["M"], 0).knn(cfg1["q"][:12], c["k"], c["ef"])
    ref = PyRef(cfg1["dumps"], c["dim"], c["M"])
    for i in range(12):
        pids, pd, st = ref.knn(cfg1["q"][i], c["k"], c["ef"])
        assert pids == ids[i].tolist()
        assert np.array_equal(np.float32(pd), dd[i])
        assert [st["distcomps"], st["visited_upper"], st["visited_l0"], st["lists_upper"], st["lists_l0"]] == \
            qs[i, :5].tolist()


def test_python_restatement_multishard_and_ties():
    rng = np.random.default_rng(5)
    uniq = np.rint(rng.uniform(0, 3, (80, 16))).astype(np.float32)
    base = uniq[rng.integers(0, 80, 900)]
    q = np.rint(rng.uniform(0, 3, (15, 16))).astype(np.float32)
    dumps, _, _ = O.build(base, 6, 30, 0, 3, seed=4)
    ids, dd, qs = O.OracleIndex(dumps, 16, 6, 0).knn(q, 8, 20)
    ref = PyRef(dumps, 16, 6)
    for i in range(15):
        pids, pd, _ = ref.knn(q[i], 8, 20)
        assert pids == ids[i].tolist()


@pytest.mark.parametrize("is_max", [True, False])
def test_python_heaps_restate_libstdcxx(is_max):
    """The Python restatement of push_heap/pop_heap against libstdc++ (through the oracle)."""
    rng = np.random.default_rng(9)
    ops = rng.choice([0, 0, 1, 2], 2000).astype(np.int32)
    vals = rng.integers(0, 7, 2000).astype(np.float32)
    ids = np.arange(2000, dtype=np.uint32)
    d, i = O.heap_replay(is_max, ops, vals, ids, 50)
    comp = _max_cmp if is_max else _min_cmp
    h = []
    for op, v, u in zip(ops, vals, ids):
        e = (int(u), float(v))
        if op == 0:
            h.append(e)
            push_heap(h, comp)
        elif op == 1:
            if h:
                pop_heap(h, comp)
        else:
            if len(h) < 50:
                h.append(e)
                push_heap(h, comp)
            elif comp(e, h[0]):
                pop_heap(h, comp)
                h.append(e)
                push_heap(h, comp)
    assert [x[0] for x in h] == i.tolist()


def test_level_draw_is_libstdcxx_mt19937_and_canonical():
    """hnsw.hh:34-35,48: floor(-ln U * 1/ln M), U from std::uniform_real_distribution<double>(0,1) over
    std::mt19937(seed).  Python's random.Random is MT19937 too; libstdc++'s generate_canonical<double, 53>
    combines two 32-bit draws: (lo + hi * 2^32) / 2^64."""
    n, M, seed = 2000, 16, 1234
    lv, _ = O.draw_levels(n, M, seed, 1)
    mt = random.Random()
    mt.seed(0)
    st = list(mt.getstate())
    # reproduce std::mt19937(seed) state initialisation (init_genrand)
    key = [seed & 0xFFFFFFFF]
    for i in range(1, 624):
        key.append((1812433253 * (key[-1] ^ (key[-1] >> 30)) + i) & 0xFFFFFFFF)
    mt.setstate((st[0], tuple(key + [624]), st[2]))
    nf = 1.0 / np.log(float(M))
    exp = []
    for _ in range(n):
        lo, hi = mt.getrandbits(32), mt.getrandbits(32)
        u = (lo + hi * 2.0 ** 32) / 2.0 ** 64
        if u >= 1.0:
            u = np.nextafter(1.0, 0.0)
        exp.append(int(np.floor(-np.log(u) * nf)))
    assert lv.tolist() == exp
