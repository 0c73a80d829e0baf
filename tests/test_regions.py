"""Region planner of SHINE_PLACE_SHARDED_REGIONS (csrc/placement.cc), host-only: the GPU-node form of the
reference's Placement / Kmeans (cache/placement.hh:22-106, cache/kmeans.hh:24-377) over real dumps.  The k-means
itself is checked bitwise against its restatement in test_placement.py.  Runs without a GPU."""
import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import datasets as D


@pytest.fixture(scope="module")
def clustered():
    base = D.sift_like(6000, seed=31)
    dumps, _, _ = O.build(base, 8, 40, 0, 3, seed=4)
    return base, dumps


@pytest.mark.parametrize("k", [2, 3, 8])
def test_regions_are_balanced_and_cover_every_record(clustered, k):
    base, dumps = clustered
    cent, region, mapping = shine_amd.plan_regions(dumps, 128, 8, 0, k)
    assert cent.shape == (k if k % 2 == 0 else 2 * k, 128) and np.isfinite(cent).all()
    assert sorted(set(mapping.tolist())) == list(range(k))
    assert region.shape[0] == base.shape[0] and (region < k).all()
    sizes = np.bincount(region, minlength=k)
    assert sizes.max() <= int(np.ceil(base.shape[0] / k * 1.05))  # at most 5 % above an even split


def test_regions_follow_the_nearest_centroid(clustered):
    base, dumps = clustered
    cent, region, mapping = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    d = ((base[:, None, :] - cent[None, :, :]) ** 2).sum(-1)
    nearest = mapping[d.argmin(1)]
    # the balance cap moves only a few records away from their nearest region
    assert (nearest == region).mean() > 0.9


def test_planner_is_deterministic(clustered):
    _, dumps = clustered
    a = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    b = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])


def test_planner_samples_the_top_levels(clustered):
    """fetch_level(500) (placement.hh:78-106) then balanced k-means: the planner's centroids are shine_kmeans over
    the same sample, which is the entry point's breadth-first closure from the top level down until >= 500 nodes."""
    base, dumps = clustered
    cent, _, mapping = shine_amd.plan_regions(dumps, 128, 8, 0, 3)
    assert cent.shape[0] == 6 and sorted(set(mapping.tolist())) == [0, 1, 2]


def test_unknown_k_is_rejected(clustered):
    _, dumps = clustered
    with pytest.raises(shine_amd.ShineError):
        shine_amd.plan_regions(dumps, 128, 8, 0, 0)


# ---- Zipf query mix (f4: scripts/data/skew.py:80-172) -----------------------------------------------------------
def _skew_py_counts(n, num_queries, alpha):
    """skew.py:110-132 line by line: probabilities over the whole pool, then ceil-draws until num_queries."""
    import math
    h = sum(1.0 / (k ** alpha) for k in range(1, n + 1))
    probs = [(1.0 / (k ** alpha)) / h for k in range(1, n + 1)]
    dist, drawn = [], 0
    for idx in range(n):
        if drawn >= num_queries:
            break
        occ = math.ceil(num_queries * probs[idx])
        dist.append(occ)
        drawn += occ
    return dist, drawn


import pytest  # noqa: E402


@pytest.mark.parametrize("n,nq,alpha", [(1000, 1000, 0.0), (500, 2000, 0.5), (2000, 3000, 1.0), (300, 5000, 1.5)])
def test_zipf_counts_follow_skew_py(n, nq, alpha):
    from shine_amd import datasets as D
    counts, drawn = D.zipf_counts(n, nq, alpha)
    ref, ref_drawn = _skew_py_counts(n, nq, alpha)
    assert counts == ref and drawn == ref_drawn


def test_zipf_mix_overshoot_trims_or_raises():
    import numpy as np
    from shine_amd import datasets as D
    pool = np.arange(2000, dtype=np.float32).reshape(2000, 1)
    counts, drawn = D.zipf_counts(1000, 2500, 0.5)
    assert drawn > 2500  # the ceilings overshoot: the reference's assert (skew.py:135) would fire here
    with pytest.raises(ValueError):
        D.zipf_query_mix(pool[:1000], 2500, 0.5, strict=True)
    q, warm, src = D.zipf_query_mix(pool[:1000], 2500, 0.5, split=500, seed=4)
    assert q.shape[0] == 2000 and warm.shape[0] == 500
    bc = np.bincount(src, minlength=len(counts))
    want = np.array(counts)
    want[-1] -= drawn - 2500  # trimmed from the last count
    np.testing.assert_array_equal(bc[:len(counts)], want)
    np.testing.assert_array_equal(np.concatenate([q, warm])[:, 0], pool[src, 0])
    # alpha 0 with num_queries == pool size: every pool query exactly once, no overshoot (strict passes)
    q0, _, src0 = D.zipf_query_mix(pool, 2000, 0.0, strict=True, seed=1)
    assert sorted(src0.tolist()) == list(range(2000))
