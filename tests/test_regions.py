"""Region planner of SHINE_PLACE_SHARDED_REGIONS (csrc/placement.cc), host-only: the GPU-node form of the
reference's Placement / Kmeans (cache/placement.hh:22-72, cache/kmeans.hh:93-137).  Runs without a GPU."""
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
    cent, region = shine_amd.plan_regions(dumps, 128, 8, 0, k)
    assert cent.shape == (k, 128) and np.isfinite(cent).all()
    assert region.shape[0] == base.shape[0] and (region < k).all()
    sizes = np.bincount(region, minlength=k)
    assert sizes.max() <= int(np.ceil(base.shape[0] / k * 1.05))  # at most 5 % above an even split


def test_regions_follow_the_nearest_centroid(clustered):
    base, dumps = clustered
    cent, region = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    d = ((base[:, None, :] - cent[None, :, :]) ** 2).sum(-1)
    nearest = d.argmin(1)
    # the balance cap moves only a few records away from their nearest region
    assert (nearest == region).mean() > 0.9


def test_planner_is_deterministic(clustered):
    _, dumps = clustered
    a = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    b = shine_amd.plan_regions(dumps, 128, 8, 0, 4)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_unknown_k_is_rejected(clustered):
    _, dumps = clustered
    with pytest.raises(shine_amd.ShineError):
        shine_amd.plan_regions(dumps, 128, 8, 0, 0)
