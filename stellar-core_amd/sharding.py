"""Multi-GPU sharding of a signature batch.

Every signature is independent, so N GPUs verify contiguous slices
[g*n/G, (g+1)*n/G) of one global batch and the verdict bytes are gathered
back into disjoint ranges -- no data-path collective.  The same partition is
used by the C-ABI's in-process multi-device path (sv_api.cpp, one host thread
per device) and by bench.py's one-process-per-GPU runs; this module is the
process-level half (torch.distributed over gloo for the gather).
"""
from __future__ import annotations

import hashlib

import numpy as np


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous slice of rank `rank` (same formula as sv_api.cpp verify_host)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return rank * n // world, (rank + 1) * n // world


def gather_verdicts(local: np.ndarray, n: int, world: int, rank: int):
    """All-gather every rank's verdict slice (uint8) and return the full array
    (on every rank).  Uses torch.distributed (gloo); outside any timed region."""
    import torch
    import torch.distributed as dist

    lo, hi = shard_bounds(n, world, rank)
    if local.shape[0] != hi - lo:
        raise ValueError("local slice has %d rows, expected %d" % (local.shape[0], hi - lo))
    width = max(shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0] for r in range(world))
    buf = torch.zeros(width, dtype=torch.uint8)
    buf[: hi - lo] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.uint8))
    parts = [torch.zeros(width, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = np.empty(n, np.uint8)
    for r in range(world):
        a, b = shard_bounds(n, world, r)
        out[a:b] = parts[r][: b - a].numpy()
    return out


def verdict_digest(verdicts: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(verdicts, dtype=np.uint8).tobytes()).hexdigest()
