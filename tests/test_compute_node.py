"""shine_compute_node — the ComputeNode-shaped driver over the C ABI (dm-hnsw-reference_amd/csrc/compute_node.cc).

CPU part: the reference's flag checks (configuration.hh:88-113) with its messages, and the dataset readers'
semantics (read_data.hh:8-78, deserializer.hh:24-44) restated in shine_amd.formats.  GPU part: an end-to-end run
on the committed golden fixtures (--store-index, then --load-index) whose statistics JSON must equal the oracle's
answers (tests/golden/expected_l2.npz) under the reference's stat names (statistics.hh:122-143).
"""
import json
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG
from shine_amd import datasets as D
from shine_amd import formats as F

BIN = PKG / "shine_compute_node"
META = json.loads((GOLDEN / "meta.json").read_text())


def _run(args, timeout=600):
    return subprocess.run([str(BIN), *map(str, args)], capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("args,msg", [
    (["-t", "1", "--ef-search", "10", "-k", "10"], "Data path and query suffix cannot be empty"),
    (["-d", "/x", "-q", "a", "--ef-search", "10", "-k", "10"], "Parameters threads, ef-search, and k are required"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10", "-s", "-l"],
     "--store-index and --load-index cannot be used in conjunction"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10", "--cache", "--cache-ratio", "0"],
     "If --cache is set, --cache-ratio must be > 0"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10", "--routing"],
     "--routing can only be used in conjunction with --cache"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "5", "-k", "10"], "ef_search must be >= k"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10", "--bogus", "1"], "unknown option --bogus"),
    (["-d", "/x", "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10", "--rows", "u4"], "--rows must be f32 or auto"),
])
def test_flag_validation_matches_reference(args, msg):
    r = _run(args)
    assert r.returncode == 1
    assert f"[ERROR]: {msg}" in r.stderr


def test_missing_files_fail_loudly(tmp_path):
    r = _run(["-d", tmp_path, "-q", "a", "-t", "1", "--ef-search", "10", "-k", "10"])
    assert r.returncode == 1 and "base or query file missing" in r.stderr


def test_help_lists_reference_flags():
    r = _run(["--help"])
    assert r.returncode == 0
    for f in ("--data-path", "--query-suffix", "--threads", "--coroutines", "--store-index", "--load-index", "--cache",
              "--routing", "--cache-ratio", "--no-recall", "--ip-dist", "--ef-search", "--ef-construction"):
        assert f in r.stdout


# ---- dataset readers (f4: read_data.hh:8-78, deserializer.hh:24-44) ---------------------------------------------
@pytest.mark.parametrize("n,clients", [(10, 1), (10, 3), (11, 4), (3, 5)])
def test_partial_read_is_round_robin_by_id(tmp_path, n, clients):
    x = np.arange(n * 4, dtype=np.float32).reshape(n, 4)
    F.write_vectors(tmp_path / "v.fbin", x)
    seen = []
    for cid in range(clients):
        ids, v = F.read_vectors(tmp_path / "v.fbin", client_id=cid, num_clients=clients)
        # to_read = n / clients, +1 below the remainder (read_data.hh:42-49); ids ≡ cid (mod clients)
        assert len(ids) == n // clients + (1 if cid < n % clients else 0)
        assert (ids % clients == cid).all()
        np.testing.assert_array_equal(v, x[ids])
        seen.extend(ids.tolist())
    assert sorted(seen) == list(range(n))


def test_byte_formats_convert_elementwise_to_f32(tmp_path):
    i8 = np.array([[-128, -1, 0, 1, 127]], dtype=np.int8)
    u8 = np.array([[0, 1, 128, 254, 255]], dtype=np.uint8)
    F.write_vectors(tmp_path / "a.i8bin", i8)
    F.write_vectors(tmp_path / "b.u8bin", u8)
    _, a = F.read_vectors(tmp_path / "a.i8bin")
    _, b = F.read_vectors(tmp_path / "b.u8bin")
    assert a.dtype == np.float32 and b.dtype == np.float32
    np.testing.assert_array_equal(a, i8.astype(np.float32))  # static_cast<f32>(i8), deserializer.hh:40-42
    np.testing.assert_array_equal(b, u8.astype(np.float32))
    with pytest.raises(ValueError):
        F.read_vectors(tmp_path / "c.txt")  # unsupported extension (read_data.hh:31-33)


# ---- end to end on the GPU -------------------------------------------------------------------------------------
def _golden_dataset(root):
    (root / "queries").mkdir(parents=True)
    shutil.copy(GOLDEN / "base.u8bin", root / "base.u8bin")
    shutil.copy(GOLDEN / "query.u8bin", root / "queries" / "query-g.u8bin")
    shutil.copy(GOLDEN / "groundtruth.bin", root / "queries" / "groundtruth-g.bin")
    return root


@pytest.mark.gpu
def test_end_to_end_on_golden_fixtures(tmp_path, gpu_available):
    c = META["cfg1"]
    data = _golden_dataset(tmp_path / "siftsmall")
    exp = np.load(GOLDEN / "expected_l2.npz")
    _, gt = F.read_vectors(GOLDEN / "groundtruth.bin")
    want_recall = D.recall_at_k(exp["ids"], gt, c["k"])
    common = ["-d", data, "-q", "g", "-t", "1", "--ef-search", c["ef"], "-k", c["k"], "-m", c["M"],
              "--ef-construction", c["efc"], "--seed", c["seed"]]
    out = {}
    for phase in ("-s", "-l"):
        r = _run(common + [phase])
        assert r.returncode == 0, r.stderr[-2000:]
        out[phase] = s = json.loads(r.stdout)
        assert s["queries"]["processed"] == c["nq"]
        assert s["queries"]["dist_comps"] == int(exp["qstats"][:, 0].sum())  # same index, same searches
        assert s["queries"]["visited_nodes_l0"] == int(exp["qstats"][:, 2].sum())
        assert abs(s["queries"]["recall"] - want_recall) < 1e-12
        assert s["queries"]["queries_per_sec"] > 0 and s["num_vectors"] == c["n"]
        assert s["hnsw_parameters"] == {"k": c["k"], "m": c["M"], "ef_search": c["ef"], "ef_construction": c["efc"]}
        for key in ("hits_total", "misses_total", "hit_rate"):
            assert key in s["cache"]
    # --rows auto: the .u8bin base is byte-valued, so the records sit in HBM as u8 rows; same searches, same answers
    r = _run(common + ["-l", "--rows", "auto"])
    assert r.returncode == 0, r.stderr[-2000:]
    s = json.loads(r.stdout)
    assert s["gpu"]["rows"] == "u8"
    assert s["queries"]["dist_comps"] == int(exp["qstats"][:, 0].sum())
    assert abs(s["queries"]["recall"] - want_recall) < 1e-12
    # --store-index wrote the reference's dump name, byte-identical to the oracle's build (one thread)
    dump = data / "dump" / f"index_m{c['M']}_efc{c['efc']}_node1_of1.dat"
    import hashlib
    assert hashlib.sha256(dump.read_bytes()).hexdigest() == META["dumps"]["l2_1"]["sha256"][0]
    assert out["-s"]["build"]["dist_comps"] == META["dumps"]["l2_1"]["build_distcomps"]


@pytest.mark.gpu
def test_client_split_and_sharded_cache(tmp_path, gpu_available):
    """--num-clients 2 --client-id 1 answers the odd query ids only; --placement sharded over two slots with
    --cache reports cache hits (a 10K-record stripe is one 2 MiB page step, so any cache holds all of it)."""
    c = META["cfg1"]
    data = _golden_dataset(tmp_path / "siftsmall")
    shutil.copy(GOLDEN / "query.u8bin", data / "queries" / "warmup-g.u8bin")
    exp = np.load(GOLDEN / "expected_l2.npz")
    _, gt = F.read_vectors(GOLDEN / "groundtruth.bin")
    common = ["-d", data, "-q", "g", "-t", "1", "--ef-search", c["ef"], "-k", c["k"], "-m", c["M"],
              "--ef-construction", c["efc"], "--seed", c["seed"], "--memory-nodes", "3"]
    r = _run(common + ["-s", "--num-clients", "2", "--client-id", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    s = json.loads(r.stdout)
    assert s["queries"]["processed"] == c["nq"] // 2
    r = _run(common + ["-l", "--placement", "sharded", "--gpus", "0,0", "--cache", "--cache-ratio", "50"])
    assert r.returncode == 0, r.stderr[-2000:]
    s = json.loads(r.stdout)
    assert s["queries"]["processed"] == c["nq"]
    assert s["cache"]["hits_total"] > 0
    assert 0.0 < s["cache"]["hit_rate"] <= 1.0
    assert s["gpu"]["placement"] == "sharded" and s["gpu"]["n_gpus"] == 2
