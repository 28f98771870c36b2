"""GPU discovery without opening a device (the benchmark ranks and launchers never initialise
HIP: only chunkservers own GPUs)."""
from __future__ import annotations

import os
from pathlib import Path


def visible_gpus() -> int:
    """GPUs this node exposes, from the KFD topology (sysfs; opens no device) narrowed by the
    usual visibility variables."""
    nodes = Path("/sys/class/kfd/kfd/topology/nodes")
    n = 0
    try:
        for d in nodes.iterdir():
            try:
                if int((d / "gpu_id").read_text().strip() or "0") != 0:
                    n += 1
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n
