"""The C-ABI library: loads, exports what include/shine_gpu.h declares, and fails loudly (status codes, no exits).

Runs without a GPU: the dump parser runs before any HIP call, so format errors are observable here; a valid
dump on a machine without a device must come back as SHINE_ERR_HIP, never as a silent CPU fallback.
"""
import ctypes as C

import numpy as np
import pytest

import oracle as O
import shine_amd
from shine_amd import _lib as L
from shine_amd import datasets as D


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    declared = L.declared_symbols()
    assert len(declared) >= 15
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert set(L.PROTOTYPES) == set(declared)


def test_library_was_built_from_this_tree():
    """shine_build_id carries the hash of every source the library was built from: a stale libshine_gpu.so (sources
    edited after the build) fails here instead of being measured."""
    bid = L.build_id().split()
    assert bid[0] == "src" and bid[2] == "git", bid
    assert bid[1] == L.source_hash(), f"libshine_gpu.so was built from other sources ({bid[1]} != {L.source_hash()})"


def test_gpu_builder_rejects_bad_arguments():
    import ctypes as C
    h = C.c_void_p()
    lib = L.lib()
    base = (C.c_float * 16)()
    assert lib.shine_gpu_build(None, 0, 10, 16, 8, 32, 0, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG
    assert lib.shine_gpu_build(base, 0, 1, 16, 8, 32, 0, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG   # n < 2
    assert lib.shine_gpu_build(base, 0, 10, 16, 1, 32, 0, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG   # M < 2
    assert lib.shine_gpu_build(base, 0, 10, 16, 8, 600, 0, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG  # efC > 512
    assert lib.shine_gpu_build(base, 0, 10, 17, 8, 32, 0, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG   # no kernel for dim
    assert lib.shine_gpu_build(base, 0, 10, 16, 8, 32, 2, 1, 0, 0.0, 0, C.byref(h)) == L.ERR_ARG   # metric
    assert lib.shine_gpu_build(base, 0, 10, 16, 8, 32, 0, 1, 0, 1.5, 0, C.byref(h)) == L.ERR_ARG   # batch fraction
    assert lib.shine_gpu_build_dumps(None, 1) == L.ERR_ARG
    assert lib.shine_gpu_build_open(None, 0, C.byref(h)) == L.ERR_ARG


def test_header_has_no_torch_or_hip_types():
    import re
    code = re.sub(r"/\*.*?\*/", "", L.HEADER.read_text(), flags=re.S)  # declarations only, comments dropped
    for bad in ("torch", "hipStream_t", "hip_runtime", "at::", "std::", "class ", "template"):
        assert bad not in code, bad


@pytest.fixture(scope="module")
def small_dumps():
    base = D.sift_like(400, seed=1)
    dumps, _, _ = O.build(base, 8, 32, 0, 2, seed=3)
    return dumps


def _open(dumps, dim=128, M=8, metric=0):
    return shine_amd.Index.from_buffers(dumps, dim, M, metric, gpus=[0])


def test_truncated_dump_is_format_error(small_dumps):
    bad = [small_dumps[0][:-100], small_dumps[1]]
    bad[0] = bad[0].copy()
    with pytest.raises(shine_amd.ShineError) as e:
        _open(bad)
    assert e.value.code == L.ERR_FORMAT


def test_null_entry_point_is_format_error(small_dumps):
    d0 = small_dumps[0].copy()
    d0[8:16] = 0  # ep_ptr (memory_node.hh:21)
    with pytest.raises(shine_amd.ShineError) as e:
        _open([d0, small_dumps[1]])
    assert e.value.code == L.ERR_FORMAT and "entry" in str(e.value)


def test_dangling_remote_pointer_is_format_error(small_dumps):
    d0 = small_dumps[0].copy()
    # first record at offset 16; its level-0 list starts at 16 + 16 + 4*128
    off = 16 + 16 + 4 * 128
    assert int(np.frombuffer(d0[off:off + 4], np.uint32)[0]) > 0
    d0[off + 4:off + 12] = np.frombuffer(np.uint64(12345).tobytes(), np.uint8)  # not a record offset
    with pytest.raises(shine_amd.ShineError) as e:
        _open([d0, small_dumps[1]])
    assert e.value.code == L.ERR_FORMAT


def test_wrong_dim_or_M_is_rejected(small_dumps):
    with pytest.raises(shine_amd.ShineError) as e:
        _open(small_dumps, M=0)
    assert e.value.code == L.ERR_ARG
    with pytest.raises(shine_amd.ShineError):
        _open(small_dumps, dim=64)  # records no longer line up with free_ptr / levels


def test_valid_dump_without_gpu_fails_loudly(small_dumps):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: covered by tests/test_gpu_parity.py")
    with pytest.raises(shine_amd.ShineError) as e:
        _open(small_dumps)
    assert e.value.code == L.ERR_HIP


def test_unknown_placement_is_rejected_before_any_device_work(small_dumps):
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.from_buffers(small_dumps, 128, 8, 0, gpus=[0], placement=7)
    assert e.value.code == L.ERR_ARG and "placement" in str(e.value)
    with pytest.raises(ValueError):
        shine_amd.Index.from_buffers(small_dumps, 128, 8, 0, gpus=[0], placement="striped")


def test_cache_fraction_outside_unit_interval_is_rejected(small_dumps):
    for bad in (-0.1, 1.5, float("nan")):
        with pytest.raises(shine_amd.ShineError) as e:
            shine_amd.Index.from_buffers(small_dumps, 128, 8, 0, gpus=[0], placement="sharded", cache=bad)
        assert e.value.code == L.ERR_ARG and "cache" in str(e.value)


def test_missing_file_is_io_error(tmp_path):
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.open([tmp_path / "nope.dat"], 128, 8, 0)
    assert e.value.code == L.ERR_IO


def test_null_arguments_are_arg_errors():
    lib = L.lib()
    assert lib.shine_open_buffers(None, None, 1, 128, 8, 0, 0, None, 0, None) == L.ERR_ARG
    assert lib.shine_knn_batch(None, None, None, 1, 10, 10, None, None, None) == L.ERR_ARG
    assert lib.shine_knn_batch_ex(None, None, None, 1, 10, 10, None, None, None, None) == L.ERR_ARG
    assert lib.shine_set_search_mode(None, L.MODE_FAST) == L.ERR_ARG
    assert lib.shine_close(None) == L.OK
    assert lib.shine_last_error()  # a message is recorded


def test_algorithmic_bytes_formula_needs_handle():
    qs = np.zeros((2, 8), np.uint32)
    assert L.lib().shine_algorithmic_bytes(None, qs.ctypes.data_as(C.c_void_p), 2) == 0


def test_byte_rows_refuse_components_they_would_change(small_dumps):
    """SHINE_ELEM_U8 / _I8 store a record only if every component is exactly a byte value (checked before any
    device work): sift-like records exceed 127 (not i8), deep-like records are fractions (neither)."""
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.from_buffers(small_dumps, 128, 8, 0, elem=L.ELEM_I8, gpus=[0])
    assert e.value.code == L.ERR_ARG and "i8" in str(e.value)
    deep, _, _ = O.build(D.deep_like(300, seed=2, d=128), 8, 32, 0, 1, seed=3)
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.from_buffers(deep, 128, 8, 0, elem=L.ELEM_U8, gpus=[0])
    assert e.value.code == L.ERR_ARG and "u8" in str(e.value)
    with pytest.raises(shine_amd.ShineError) as e:
        shine_amd.Index.from_buffers(small_dumps, 128, 8, 0, elem=5, gpus=[0])
    assert e.value.code == L.ERR_ARG


def test_byte_row_layout_is_lane_contiguous():
    """kernels.h permuted_index_bytes: element a + 8t of the 16-aligned prefix at byte ((a>>1)*NCH + t//2)*4 +
    (t&1)*2 + (a&1), NCH = dim >> 4 (each of the 4 lanes of a vector reads dim/4 contiguous bytes); restated here
    and checked to be a permutation of the prefix with the tail in place."""
    for dim in (100, 128):
        nch = dim >> 4
        pos = []
        for i in range(dim):
            if i >= dim >> 4 << 4:
                pos.append(i)
                continue
            a, t = i & 7, i >> 3
            pos.append(((a >> 1) * nch + (t >> 1)) * 4 + (t & 1) * 2 + (a & 1))
        assert sorted(pos) == list(range(dim))
        # lane c's chunks: accumulators 2c, 2c+1 only
        for i in range(dim >> 4 << 4):
            assert pos[i] // (4 * nch) == (i & 7) >> 1
