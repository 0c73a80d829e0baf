"""Synthetic workloads shaped like the reference's datasets (no datasets can be fetched here).

* `sift_like`  — SIFT-shaped: integer-valued f32 in [0, 255], d = 128 (SURVEY §8d cfg 1/2).  A Gaussian mixture
  in a low-dimensional latent space with a power-law spectrum, projected to d and quantised.  Integer values
  make every L2 partial sum exact in f32 (< 2^24), as for real SIFT / BIGANN u8 data.
* `deep_like`  — DEEP-shaped: L2-normalised f32, d = 96 (cfg 3/4).
* `tti_like`   — Text-to-Image-shaped: f32, d = 200, inner product (cfg 5).
* `zipf_query_mix` — scripts/data/skew.py:80-172 query replay (Zipf α, warm-up split).
Model parameters come from a fixed seed, sample draws from `seed`, so base and queries share a distribution.
"""
from __future__ import annotations

import math

import numpy as np

_MODEL_SEED = 0x5EED


def _model(d, latent, centres, spectrum, cs, model_key):
    rm = np.random.default_rng([_MODEL_SEED, model_key, d, latent, centres])
    C = rm.normal(0.0, 1.0, (centres, latent)).astype(np.float32) * np.float32(cs)
    scale = (np.arange(1, latent + 1, dtype=np.float32) ** -np.float32(spectrum))
    P = rm.normal(0.0, 1.0, (d, latent)).astype(np.float32) / np.float32(math.sqrt(latent))
    return C, scale, P


def _latent_mixture(n, d, seed, latent, centres, spectrum, model_key, cs=2.5):
    C, scale, P = _model(d, latent, centres, spectrum, cs, model_key)
    rng = np.random.default_rng(seed)
    out = np.empty((n, d), dtype=np.float32)
    step = 1 << 16
    for s in range(0, n, step):
        m = min(step, n - s)
        lab = rng.integers(0, centres, m)
        z = (C[lab] + rng.normal(0.0, 1.0, (m, latent)).astype(np.float32)) * scale
        out[s:s + m] = z @ P.T
    return out


def _model_std(d, latent, centres, spectrum, model_key, cs):
    """Fixed output scale of the model (from a fixed calibration draw), so base and queries quantise alike."""
    x = _latent_mixture(1 << 15, d, 0xCA1, latent, centres, spectrum, model_key, cs)
    return float(x.std())


_SIFT = dict(latent=64, centres=1024, spectrum=0.35, model_key=1, cs=1.0)
_sift_std = {}


def sift_like(n: int, seed: int = 1, d: int = 128) -> np.ndarray:
    """SIFT-shaped: ~10 % zeros, mean ~50, values quantised to integers in [0, 255].  At 1M points with M=16 /
    efC=200 the reference's knn reaches recall@10 ~0.93 at ef=32 and ~0.98 at ef=128 with ~2,100 distance
    computations per query at ef=128 (measured with the oracle), close to real SIFT1M's behaviour."""
    if d not in _sift_std:
        _sift_std[d] = _model_std(d, _SIFT["latent"], _SIFT["centres"], _SIFT["spectrum"], _SIFT["model_key"],
                                  _SIFT["cs"])
    x = _latent_mixture(n, d, seed, _SIFT["latent"], _SIFT["centres"], _SIFT["spectrum"], _SIFT["model_key"],
                        _SIFT["cs"])
    x = np.rint(x * np.float32(40.0 / _sift_std[d]) + np.float32(50.0))
    np.clip(x, 0.0, 255.0, out=x)
    x += np.float32(0.0)  # -0.0 → +0.0, so the vectors survive a u8 round trip bit for bit
    return x.astype(np.float32)


def deep_like(n: int, seed: int = 1, d: int = 96) -> np.ndarray:
    x = _latent_mixture(n, d, seed, latent=32, centres=512, spectrum=0.5, model_key=2)
    x /= np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12)
    return x.astype(np.float32)


def tti_like(n: int, seed: int = 1, d: int = 200) -> np.ndarray:
    x = _latent_mixture(n, d, seed, latent=48, centres=512, spectrum=0.5, model_key=3)
    x /= np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12)
    return (x * np.float32(0.8)).astype(np.float32)


_KINDS = {
    # kind: (latent, centres, spectrum, model_key, cs, post)
    "sift_like": (64, 1024, 0.35, 1, 1.0, "sift"),
    "deep_like": (32, 512, 0.5, 2, 2.5, "unit"),
    "tti_like": (48, 512, 0.5, 3, 2.5, "tti"),
}


def generate_device(kind: str, n: int, seed: int = 1, d: int | None = None, device: str = "cuda", chunk: int = 1 << 22):
    """The same model as `kind` (sift_like / deep_like / tti_like: centres, spectrum and projection from the fixed model
    seed) sampled with torch on the GPU, for 10M-100M-record workloads whose numpy generation would take minutes of host
    time and tens of GB of host memory.  Draws come from torch's generator, so the rows differ from the numpy
    functions' rows of the same seed; the distribution is the same.  Returns a float32 tensor (n, d) on `device`."""
    import torch
    latent, centres, spectrum, key, cs, post = _KINDS[kind]
    d = d or {"sift_like": 128, "deep_like": 96, "tti_like": 200}[kind]
    C, scale, P = _model(d, latent, centres, spectrum, cs, key)
    Ct = torch.from_numpy(C).to(device)
    st = torch.from_numpy(scale).to(device)
    Pt = torch.from_numpy(P.T.copy()).to(device)
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    out = torch.empty((n, d), dtype=torch.float32, device=device)
    sstd = None
    if post == "sift":
        if d not in _sift_std:
            _sift_std[d] = _model_std(d, latent, centres, spectrum, key, cs)
        sstd = _sift_std[d]
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        lab = torch.randint(0, centres, (m,), generator=g, device=device)
        z = (Ct[lab] + torch.randn((m, latent), generator=g, device=device)) * st
        x = z @ Pt
        if post == "sift":
            x = torch.clamp(torch.round(x * (40.0 / sstd) + 50.0), 0.0, 255.0) + 0.0
        else:
            x = x / torch.clamp(torch.linalg.vector_norm(x, dim=1, keepdim=True), min=1e-12)
            if post == "tti":
                x = x * 0.8
        out[s:s + m] = x
        del lab, z, x
    return out


def ground_truth_device(base, queries, k: int, metric: int, qblock: int = 512, bchunk: int = 1 << 22,
                        refine: int = 32):
    """Exact top-k of every query over a GPU-resident base of any size, in float64 throughout: per (query block, base
    chunk) the `refine` best candidates are kept, then the best k of all chunks' candidates (ties by id), their
    distances recomputed directly.  (torch's f32 GEMM on this stack is not exact enough: on normalised rows its order
    of near neighbours disagreed with float64 at recall 0.875 in round 1)  metric 0 = squared L2,
    1 = 1 - <q, x>.  Returns an (nq, k) int64 numpy array."""
    import torch
    nq, n = queries.shape[0], base.shape[0]
    out = np.empty((nq, k), dtype=np.int64)
    for qs in range(0, nq, qblock):
        q = queries[qs:qs + qblock].double()
        qn = (q * q).sum(1, keepdim=True)
        cand_d, cand_i = [], []
        for bs in range(0, n, bchunk):
            b = base[bs:bs + bchunk].double()
            dot = q @ b.T
            dist = qn + (b * b).sum(1)[None, :] - 2.0 * dot if metric == 0 else 1.0 - dot
            r = min(refine, dist.shape[1])
            v, i = torch.topk(dist, r, dim=1, largest=False)
            cand_d.append(v)
            cand_i.append(i + bs)
            del dot, dist, b
        ci = torch.cat(cand_i, 1)
        cd = torch.cat(cand_d, 1)
        _, sel = torch.topk(cd, min(refine, cd.shape[1]), dim=1, largest=False)
        ci = torch.gather(ci, 1, sel)
        rows = base[ci].double()                       # (qb, refine, d)
        q64 = q[:, None, :]
        exact = ((rows - q64) ** 2).sum(2) if metric == 0 else 1.0 - (rows * q64).sum(2)
        ex = exact.cpu().numpy()
        ids = ci.cpu().numpy()
        for r in range(ex.shape[0]):
            o = np.lexsort((ids[r], ex[r]))[:k]
            out[qs + r] = ids[r][o]
    return out


def brute_force_knn(base: np.ndarray, queries: np.ndarray, k: int, metric: int = 0, chunk: int = 256):
    """Exact top-k (ties by id), distances in f64.  metric 0 = squared L2, 1 = 1 - <q, x>."""
    b = base.astype(np.float64)
    bn = (b * b).sum(1)
    ids = np.empty((queries.shape[0], k), dtype=np.uint32)
    dd = np.empty((queries.shape[0], k), dtype=np.float64)
    for s in range(0, queries.shape[0], chunk):
        q = queries[s:s + chunk].astype(np.float64)
        ip = q @ b.T
        dist = (q * q).sum(1)[:, None] + bn[None, :] - 2.0 * ip if metric == 0 else 1.0 - ip
        part = np.argpartition(dist, k - 1, axis=1)[:, :k] if k < dist.shape[1] else \
            np.tile(np.arange(dist.shape[1]), (dist.shape[0], 1))
        # widen to include ties at the k-th distance, then order by (distance, id)
        for r in range(dist.shape[0]):
            kth = dist[r, part[r]].max()
            cand = np.nonzero(dist[r] <= kth)[0]
            order = np.lexsort((cand, dist[r, cand]))[:k]
            ids[s + r] = cand[order]
            dd[s + r] = dist[r, cand[order]]
    return ids, dd


def recall_at_k(results: np.ndarray, gt: np.ndarray, k: int) -> float:
    """compute_node.cc:579-600 — Σ_q |result_q ∩ GT_q[0:k]| / (nq·k), set semantics."""
    hits = 0
    for r, g in zip(results, gt):
        hits += len(set(r[:k].tolist()) & set(g[:k].tolist()))
    return hits / (results.shape[0] * k)


def harmonic_number(n: int, alpha: float) -> float:  # skew.py:14-19
    return float(np.sum(1.0 / np.arange(1, n + 1, dtype=np.float64) ** alpha))


def zipf_counts(n: int, num_queries: int, alpha: float) -> tuple[list[int], int]:
    """skew.py:114-132: occurrences of pool query i (0-based) = ceil(num_queries * pmf(i+1)), drawn until the total
    reaches num_queries.  Returns (counts, drawn); drawn can exceed num_queries (the ceilings)."""
    h = harmonic_number(n, alpha)
    counts = []
    drawn = 0
    for idx in range(n):
        if drawn >= num_queries:
            break
        occ = math.ceil(num_queries * ((1.0 / (idx + 1) ** alpha) / h))  # pmf(k) = (1 / k^alpha) / H (skew.py:22-23)
        counts.append(occ)
        drawn += occ
    return counts, drawn


def zipf_query_mix(pool: np.ndarray, num_queries: int, alpha: float, split: int = 0, seed: int = 0,
                   strict: bool = False):
    """skew.py:114-164: query i of the pool is repeated ceil(num_queries * pmf(i+1)) times (until num_queries
    are drawn), the multiset is shuffled, and the last `split` become the warm-up set.  Returns
    (queries, warmup, pool_index_of_each_query).  The reference asserts drawn == num_queries (skew.py:135); with
    strict=True so does this (ValueError), otherwise the overshoot is trimmed from the last count, the fix the
    reference's TODO names (skew.py:136)."""
    n = pool.shape[0]
    counts, drawn = zipf_counts(n, num_queries, alpha)
    if drawn != num_queries:
        if strict:
            raise ValueError(f"drawn {drawn} != num_queries {num_queries} (skew.py:135)")
        counts[-1] -= drawn - num_queries
    src = np.repeat(np.arange(len(counts)), counts)
    perm = np.random.default_rng(seed).permutation(num_queries)
    src = src[perm]
    q = pool[src]
    nq = num_queries - split
    return q[:nq], q[nq:], src
