"""big-ann file formats used by the reference's readers (src/io/read_data.hh:8-78, deserializer.hh:11-63).

Header `(u32 n, u32 d)` then n*d components: `.fbin` f32, `.u8bin` u8, `.i8bin` i8, `.bin` u32 (ground truth).
Byte formats are converted to f32 on read (deserializer.hh:24-44).  `client_id / num_clients` reproduce the
round-robin partial read (`id % num_clients == client_id`, read_data.hh:42-77).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

_DTYPES = {".fbin": np.float32, ".u8bin": np.uint8, ".i8bin": np.int8, ".bin": np.uint32}


def _dtype(path: Path):
    try:
        return _DTYPES[path.suffix]
    except KeyError:
        raise ValueError(f"unsupported file extension: {path.suffix}") from None  # read_data.hh:31-33


def read_header(path) -> tuple[int, int]:
    with open(path, "rb") as f:
        n, d = np.frombuffer(f.read(8), dtype=np.uint32)
    return int(n), int(d)


def read_vectors(path, client_id: int = 0, num_clients: int = 1, limit: int | None = None, as_float=True):
    """Returns (ids, vectors).  Vectors are f32 for f32/u8/i8 files when as_float (element_t = f32)."""
    path = Path(path)
    dt = _dtype(path)
    n, d = read_header(path)
    mm = np.memmap(path, dtype=dt, mode="r", offset=8, shape=(n, d))
    ids = np.arange(client_id, n, num_clients, dtype=np.uint32)
    if limit is not None:
        ids = ids[:limit]
    v = np.asarray(mm[ids])
    if as_float and dt != np.uint32:
        v = v.astype(np.float32)
    return ids, v


def write_vectors(path, vectors: np.ndarray) -> None:
    path = Path(path)
    dt = _dtype(path)
    v = np.ascontiguousarray(vectors, dtype=dt)
    with open(path, "wb") as f:
        f.write(np.array(v.shape, dtype=np.uint32).tobytes())
        f.write(v.tobytes())
