"""Balanced k-means placement and adaptive query routing (§8 f3), host-only: csrc/placement.cc through the C ABI
(shine_kmeans, shine_router_run, shine_plan_regions) against oracle/placement_ref.py, the line-by-line restatement
of src/cache/kmeans.hh, src/cache/placement.hh:63-72 and src/router/query_router.hh:106-151, 280-387.

Parity pin: the reference ships no fixtures for this path and may not be built here, so both sides
restate the same source; agreement is bitwise on integer-valued inputs (see placement_ref's header)."""
import numpy as np
import pytest

import shine_amd
import placement_ref as P  # oracle/placement_ref.py (conftest puts oracle/ on sys.path)


def _rows(n, d, seed, hi=20):
    rng = np.random.default_rng(seed)
    centres = rng.integers(0, hi * 4, size=(5, d))
    pick = rng.integers(0, 5, size=n)
    return (centres[pick] + rng.integers(-hi, hi + 1, size=(n, d))).astype(np.float32)


def test_uniform_index_is_lemire_over_mt19937():
    """std::uniform_int_distribution<size_t>(0, n-1)(std::mt19937{1234}) (kmeans.hh:169-171): first draws for known
    n.  mt19937(1234)'s first output is 822569775; Lemire maps it to (x * n) >> 32."""
    mt = P.mt19937(1234)
    assert mt.getrandbits(32) == 822569775
    for n in [1, 2, 7, 500, 1 << 20]:
        assert P.uniform_index(P.mt19937(1234), 0, n - 1) == (822569775 * n) >> 32


@pytest.mark.parametrize("metric,d", [(0, 16), (0, 20), (1, 16)])
@pytest.mark.parametrize("k", [2, 3, 4])
def test_balanced_kmeans_matches_restatement(metric, d, k):
    rows = _rows(96, d, seed=10 * k + d + metric)
    if metric == 1:
        rows = rows / F32_ROWS_SCALE
    got = shine_amd.kmeans(rows, k, metric=metric)
    cent, mapping, sizes, it, bit = P.run_and_optimize(metric, rows, k)
    assert got["iterations"] == it and got["balance_iterations"] == bit
    np.testing.assert_array_equal(got["mapping"], mapping)
    np.testing.assert_array_equal(got["centroids"].view(np.uint32), cent.view(np.uint32))
    np.testing.assert_array_equal(got["sizes"], sizes)
    assert sorted(set(got["mapping"].tolist())) == list(range(k))  # every region gets centroids
    assert int(got["sizes"].sum()) == rows.shape[0]


F32_ROWS_SCALE = np.float32(64.0)  # IP rows scaled by a power of two: still exact in f32


@pytest.mark.parametrize("k", [2, 5])
def test_plain_kmeans_branch_matches_restatement(k):
    rows = _rows(80, 16, seed=3 + k)
    got = shine_amd.kmeans(rows, k, balanced=False)
    cent, mapping, sizes, it, _ = P.run_and_optimize(0, rows, k, balanced=False)
    assert got["iterations"] == it
    np.testing.assert_array_equal(got["centroids"].view(np.uint32), cent.view(np.uint32))
    np.testing.assert_array_equal(got["mapping"], mapping)
    np.testing.assert_array_equal(got["sizes"], sizes)


def test_balancing_evens_out_a_skewed_sample():
    """Five clusters of very different sizes into k = 4 regions: plain k-means leaves them unbalanced, the balanced
    run ends within the reference's max cluster size difference of 1 (kmeans.hh:279) on the assignment it moves."""
    rng = np.random.default_rng(5)
    parts = [rng.integers(0, 8, size=(m, 16)) + 100 * i for i, m in enumerate([120, 20, 20, 20, 20])]
    rows = np.concatenate(parts).astype(np.float32)
    plain = shine_amd.kmeans(rows, 4, balanced=False)
    bal = shine_amd.kmeans(rows, 4)
    assert plain["sizes"].max() - plain["sizes"].min() > 40
    assert bal["sizes"].max() - bal["sizes"].min() < plain["sizes"].max() - plain["sizes"].min()
    cent, _, _, _, _ = P.run_and_optimize(0, rows, 4)
    np.testing.assert_array_equal(bal["centroids"].view(np.uint32), cent.view(np.uint32))


def test_kmeans_rejects_fewer_rows_than_clusters():
    with pytest.raises(shine_amd.ShineError):
        shine_amd.kmeans(_rows(5, 16, seed=1), 3)  # odd k: 6 clusters over 5 rows
    with pytest.raises(shine_amd.ShineError):
        shine_amd.kmeans(_rows(5, 16, seed=1), 0)


def test_update_limits_examples():
    """query_router.hh:106-151 on hand-checked inputs."""
    assert P.update_limits([200, 200], [5, 0], 2) == [0, 400]
    assert P.update_limits([200, 200, 200], [0, 0, 0], 3) == [200, 200, 200]   # sum < k: no update
    assert P.update_limits([200, 200, 200], [1, 1, 0], 3) == [200, 200, 200]   # sum 2 < k = 3: no update
    assert P.update_limits([200, 200, 200], [2, 1, 0], 3) == [100, 200, 300]
    # Σp = 60: scale_i = (60 - p_i) / 120 * 3 -> 250, 200, 150
    assert P.update_limits([200] * 3, [10, 20, 30], 3) == [250, 200, 150]
    # truncation, then the round-robin top-up from region 0: scale = (7-p)/14*3 -> 257.14, 214.28, 128.57
    assert P.update_limits([200] * 3, [1, 2, 4], 3) == [258, 214, 128]


@pytest.mark.parametrize("k,adaptive", [(2, True), (3, True), (3, False), (4, True)])
def test_router_matches_restatement(k, adaptive):
    rows = _rows(160, 16, seed=20 + k)
    km = shine_amd.kmeans(rows, k)
    rng = np.random.default_rng(k)
    nq = P.LIMIT_PER_CN * k * 3 + 37  # three batch boundaries
    q = (rows[rng.integers(0, rows.shape[0], nq)] + rng.integers(-3, 4, size=(nq, 16))).astype(np.float32)
    queues = rng.integers(0, 900, size=(3, k)).astype(np.uint32)
    got, lim = shine_amd.router_run(km["centroids"], km["mapping"], k, q, queue_sizes=queues, adaptive=adaptive)
    want, wlim = P.route(0, km["centroids"], km["mapping"], k, q, queues, adaptive)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(lim, wlim)
    # every batch window respects the limits in force for it
    for b in range(0, nq, P.LIMIT_PER_CN * k):
        w = np.bincount(got[b:b + P.LIMIT_PER_CN * k], minlength=k)
        assert w.sum() == min(P.LIMIT_PER_CN * k, nq - b)
    if adaptive:
        assert int(lim.sum()) == P.LIMIT_PER_CN * k


def test_router_limits_follow_queue_sizes():
    """A node with a long queue gets a smaller share of the next batch (ADAPTIVE_ROUTING)."""
    rows = _rows(100, 16, seed=2)
    km = shine_amd.kmeans(rows, 2)
    q = np.repeat(km["centroids"][km["mapping"] == 0][:1], 1000, axis=0)  # every query prefers region 0
    _, lim = shine_amd.router_run(km["centroids"], km["mapping"], 2, q, queue_sizes=np.array([[900, 100]]))
    assert lim.tolist() == [40, 360]
    got, lim0 = shine_amd.router_run(km["centroids"], km["mapping"], 2, q, adaptive=False)
    assert lim0.tolist() == [200, 200]
    assert np.bincount(got[:400], minlength=2).tolist() == [200, 200]  # the overflow goes to the next-closest region
