"""Diagnostics: one 1,024-query batch on the 1M SIFT-shaped index, for rocprofv3 --pmc passes (SQ instruction mix /
wait counters of the search kernel).  MODE=fast (default) or exact; EF (default 128).  Builds the phase-profile index
if missing."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "dm-hnsw-reference_amd"))
import shine_amd  # noqa: E402
from shine_amd import datasets as D  # noqa: E402

path = Path("/tmp/shine_bench_phase") / "dump" / shine_amd.dump_name(16, 200, 0, 1)
if not path.exists():
    dumps, _ = shine_amd.build(D.sift_like(1_000_000, seed=1), 16, 200, 0, 1, 1234,
                               threads=int(os.environ.get("OMP_NUM_THREADS", "16")))
    path.parent.mkdir(parents=True, exist_ok=True)
    dumps[0].tofile(path)
    if os.environ.get("BUILD_ONLY"):
        sys.exit(0)
q = D.sift_like(int(os.environ.get("NQ", "1024")), seed=2)
elem = shine_amd.ELEM_U8 if os.environ.get("ROWS") == "u8" else shine_amd.ELEM_F32  # ROWS=u8: byte rows
idx = shine_amd.Index.open([path], 128, 16, 0, elem=elem, gpus=[0])
idx.set_search_mode(shine_amd.MODE_FAST if os.environ.get("MODE", "fast") == "fast" else shine_amd.MODE_EXACT)
for _ in range(int(os.environ.get("REPS", "2"))):
    r = idx.knn(q, 10, int(os.environ.get("EF", "128")))
print("kernel_ms", r.stats["kernel_ms"], "L0 lists", r.qstats[:, 4].mean())
