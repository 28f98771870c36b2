import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# block journal at test scale: 32 MiB segments, not zero-filled (every store and chunkserver
# the tests start would otherwise write 512 MiB of spare segments); larger blocks take the
# per-file path, which the tests exercise as well
os.environ.setdefault("DFS_JOURNAL_SEG_MB", "32")
os.environ.setdefault("DFS_JOURNAL_ZERO_FILL", "0")
os.environ.setdefault("DFS_JOURNAL_PARTS", "4")  # 8 MiB part files at test scale


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: multi-process cluster test")


@pytest.fixture(scope="session")
def native():
    from rust_hadoop_generated_by_llm_amd import native as n

    return n.lib


@pytest.fixture(scope="session")
def has_gpu():
    from rust_hadoop_generated_by_llm_amd import native as n

    return n.gpu_count() > 0
