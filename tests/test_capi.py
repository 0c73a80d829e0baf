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
    assert lib.shine_knn_batch(None, None, None, 1, 10, 10, None, None, None, None) == L.ERR_ARG
    assert lib.shine_set_search_mode(None, L.MODE_FAST) == L.ERR_ARG
    assert lib.shine_close(None) == L.OK
    assert lib.shine_last_error()  # a message is recorded


def test_algorithmic_bytes_formula_needs_handle():
    qs = np.zeros((2, 8), np.uint32)
    assert L.lib().shine_algorithmic_bytes(None, qs.ctypes.data_as(C.c_void_p), 2) == 0
