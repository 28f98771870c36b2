"""Reed-Solomon erasure coding over GF(2^8), bit-compatible with the reference's
``reed-solomon-erasure`` galois_8 codec (reference: dfs/common/src/erasure.rs:7-59).

``encode`` zero-pads the input to ``k * ceil(len/k)`` bytes and returns k data shards
followed by m parity shards; ``decode`` rebuilds missing shards from any k survivors and
returns the original bytes. With an HBM ChunkStore the GF(2^8) matrix product runs as the
CDNA4 kernel ``gf256_matmul_kernel`` (K4/K5); otherwise the native CPU table codec runs.
"""
from __future__ import annotations

import logging
import threading

from ..native import lib

log = logging.getLogger("dfs.erasure")


class ErasureError(ValueError):
    pass


# Matrix products that were meant for a GPU but ran on the host CPU instead (no slot, no GPU
# on the server, a failed launch): counted and logged, never silent.
STATS = {"gpu": 0, "cpu": 0, "cpu_fallbacks": 0}
_stats_lock = threading.Lock()


def _count(key: str) -> None:
    with _stats_lock:
        STATS[key] += 1


def shard_len(data_len: int, data_shards: int) -> int:
    if data_shards <= 0:
        raise ErasureError("data_shards must be > 0")
    return -(-data_len // data_shards)


def _matmul(matrix, inputs, length, store=None):
    if store is not None and getattr(store, "gpu", False):
        out = store.gf_matmul(matrix, inputs, length)
        if out is not None:
            _count("gpu")
            return out
        _count("cpu_fallbacks")
        log.warning("GPU erasure coding unavailable for a %dx%d x %d B product; using the CPU codec",
                    len(matrix), len(inputs), length)
    else:
        _count("cpu")
    return lib.gf_matmul_cpu(matrix, inputs, length)


def parity_matrix(k: int, m: int) -> list[list[int]]:
    return lib.rs_matrix(k, m)[k:]


def encode(data: bytes, data_shards: int, parity_shards: int, store=None) -> list[bytes]:
    if data_shards <= 0 or parity_shards <= 0:
        raise ErasureError("data_shards and parity_shards must both be > 0")
    if not data:
        raise ErasureError("data must not be empty")
    sl = shard_len(len(data), data_shards)
    padded = bytes(data) + b"\0" * (sl * data_shards - len(data))
    shards = [padded[i * sl:(i + 1) * sl] for i in range(data_shards)]
    parity = _matmul(parity_matrix(data_shards, parity_shards), shards, sl, store)
    return shards + list(parity)


def reconstruct(shards: list[bytes | None], data_shards: int, parity_shards: int, store=None) -> list[bytes]:
    """Fill every None entry; raises if fewer than k shards survive."""
    total = data_shards + parity_shards
    if len(shards) != total:
        raise ErasureError(f"expected {total} shards, got {len(shards)}")
    present = [i for i, s in enumerate(shards) if s is not None]
    if len(present) < data_shards:
        raise ErasureError("RS reconstruct error: TooFewShardsPresent")
    missing = [i for i, s in enumerate(shards) if s is None]
    if not missing:
        return list(shards)  # type: ignore[arg-type]
    sl = len(shards[present[0]])
    if any(len(shards[i]) != sl for i in present):
        raise ErasureError("RS reconstruct error: IncorrectShardSize")
    use = present[:data_shards]
    rows = lib.rs_decode_rows(data_shards, parity_shards, use, missing)
    rebuilt = _matmul(rows, [shards[i] for i in use], sl, store)
    out = list(shards)
    for i, r in zip(missing, rebuilt):
        out[i] = r
    return out  # type: ignore[return-value]


def decode(shards: list[bytes | None], data_shards: int, parity_shards: int, original_len: int,
           store=None) -> bytes:
    full = reconstruct(shards, data_shards, parity_shards, store)
    return b"".join(full[:data_shards])[:original_len]
