"""The dynamic cache's replay pool (csrc/index_internal.h shine::TaskPool) under ThreadSanitizer on the host: every
task of every run exactly once while the pool grows, no data race reported (tests/native/task_pool_stress.cc)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not found")
def test_task_pool_runs_every_task_once_without_races(tmp_path):
    exe = tmp_path / "task_pool_stress"
    src = ROOT / "tests" / "native" / "task_pool_stress.cc"
    inc = ROOT / "dm-hnsw-reference_amd" / "csrc"
    build = subprocess.run(["g++", "-O1", "-g", "-std=c++20", "-pthread", "-fsanitize=thread", "-D__HIP_PLATFORM_AMD__",
                            "-I/opt/rocm/include", f"-I{inc}", str(src), "-o", str(exe)], capture_output=True, text=True)
    if build.returncode != 0:
        pytest.skip(f"host build of the stress test failed: {build.stderr[-500:]}")
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "pool ok" in run.stdout
    assert "ThreadSanitizer" not in run.stderr, run.stderr[-2000:]
