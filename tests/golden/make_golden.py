"""Generates the committed golden fixtures (run from the repo root: python tests/golden/make_golden.py).

Config 1 of BASELINE.json — siftsmall-shaped: 10,000 x 128 integer-valued vectors in [0, 255] (stored as
.u8bin), 100 queries, L2, M=16, efC=200, ef=64, k=10 — plus a small inner-product case (DEEP-shaped, d=96).
The reference ships no fixtures and could not be run here, so the expected outputs come from
the oracle (oracle/oracle.cc); they pin the oracle and, through tests/test_gpu_parity.py, the GPU path.
Files:
  base.u8bin / query.u8bin / groundtruth.bin   big-ann formats (src/io/read_data.hh)
  expected_l2.npz                               ids (heap order), dists, per-query counters of knn(k=10, ef=64)
  ip_base.fbin / ip_query.fbin / expected_ip.npz
  meta.json                                     parameters, dump sizes and sha256 of the oracle's dumps
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

import oracle as O  # noqa: E402
from shine_amd import datasets as D  # noqa: E402
from shine_amd import formats as F  # noqa: E402

CFG1 = dict(n=10_000, nq=100, dim=128, M=16, efc=200, ef=64, k=10, seed=1234, shards=(1, 3))
IP = dict(n=2_000, nq=50, dim=96, M=12, efc=100, ef=48, k=10, seed=77, shards=(2,))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    meta = {"cfg1": CFG1, "ip": IP, "dumps": {}}
    base = D.sift_like(CFG1["n"], seed=1)
    q = D.sift_like(CFG1["nq"], seed=2)
    F.write_vectors(HERE / "base.u8bin", base.astype(np.uint8))
    F.write_vectors(HERE / "query.u8bin", q.astype(np.uint8))
    gt, _ = D.brute_force_knn(base, q, 100)
    F.write_vectors(HERE / "groundtruth.bin", gt)
    for ns in CFG1["shards"]:
        dumps, dc, ml = O.build(base, CFG1["M"], CFG1["efc"], 0, ns, CFG1["seed"])
        meta["dumps"][f"l2_{ns}"] = {"sizes": [int(d.size) for d in dumps], "sha256": [sha(d) for d in dumps],
                                     "build_distcomps": dc, "max_level": ml}
        if ns == 1:
            ids, dd, qs = O.OracleIndex(dumps, CFG1["dim"], CFG1["M"], 0).knn(q, CFG1["k"], CFG1["ef"])
            np.savez(HERE / "expected_l2.npz", ids=ids, dists=dd, qstats=qs)
            meta["recall_l2"] = D.recall_at_k(ids, gt, CFG1["k"])

    ib = D.deep_like(IP["n"], seed=11, d=IP["dim"])
    iq = D.deep_like(IP["nq"], seed=12, d=IP["dim"])
    F.write_vectors(HERE / "ip_base.fbin", ib)
    F.write_vectors(HERE / "ip_query.fbin", iq)
    dumps, dc, ml = O.build(ib, IP["M"], IP["efc"], 1, IP["shards"][0], IP["seed"])
    meta["dumps"]["ip_2"] = {"sizes": [int(d.size) for d in dumps], "sha256": [sha(d) for d in dumps],
                             "build_distcomps": dc, "max_level": ml}
    ids, dd, qs = O.OracleIndex(dumps, IP["dim"], IP["M"], 1).knn(iq, IP["k"], IP["ef"])
    np.savez(HERE / "expected_ip.npz", ids=ids, dists=dd, qstats=qs)
    igt, _ = D.brute_force_knn(ib, iq, IP["k"], metric=1)
    meta["recall_ip"] = D.recall_at_k(ids, igt, IP["k"])
    (HERE / "meta.json").write_text(json.dumps(meta, indent=1) + "\n")
    print(json.dumps({k: v for k, v in meta.items() if k.startswith("recall")}))


if __name__ == "__main__":
    main()
