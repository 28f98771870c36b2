"""Runs the native C++ unit tests (csrc/bench/unit_tests.cpp, built by build_native.py into
build/native/unit_tests): JSON, shard map, joint majority, extent allocator, CRC, RS codec,
WAL torn tails, disk gate and in-memory Raft clusters with partitions. One pytest case per
native test so a failure names it."""
import subprocess
from pathlib import Path

import pytest

from rust_hadoop_generated_by_llm_amd import native  # noqa: F401  (builds the runtime if stale)

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "build" / "native" / "unit_tests"
SRC = ROOT / "csrc" / "bench" / "unit_tests.cpp"
if not EXE.exists() or EXE.stat().st_mtime < SRC.stat().st_mtime:
    import sys
    sys.path.insert(0, str(ROOT))
    import build_native

    build_native.build()


def _names():
    import re

    return re.findall(r"^TEST\((\w+)\)", SRC.read_text(), re.M)


def test_unit_test_binary_exists():
    assert EXE.exists(), "build_native.py must build build/native/unit_tests"


@pytest.mark.parametrize("name", _names())
def test_native(name):
    r = subprocess.run([str(EXE), name], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and f"ok {name}" in r.stdout, r.stdout + r.stderr
