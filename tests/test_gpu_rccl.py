"""RCCL on MI355X hardware: RCCL refuses two ranks on one GPU, so the
1-GPU box runs the building blocks of csrc/p2p_rccl.cpp's RcclTransport on a 1-rank
communicator — nonblocking init through settle(), a grouped self ncclSend/ncclRecv whose
completion is observed through a hipEvent (as test() does), byte comparison, ncclCommAbort
while a 512 MiB transfer is in flight (close()'s path, the stream must drain), and a fresh
communicator afterwards (a pair rebuild)."""
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_loopback_init_transfer_abort_rebuild(native, has_gpu):
    if not has_gpu:
        pytest.fail("GPU test selected but no HIP device is visible")
    for n in (4, 1 << 20, 64 << 20):
        r = native.rccl_loopback_probe(0, n, 0, 30000)
        assert r["ok"] and r["bytes_ok"], (n, r)
    r = native.rccl_loopback_probe(0, 1 << 20, 512 << 20, 30000)
    print("\nrccl probe:", r)
    assert r["ok"], r
    assert r["drained_after_abort"] and r["reinit_ok"], r
