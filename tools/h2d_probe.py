#!/usr/bin/env python3
"""Developer tool: host -> device copy rate from pinned memory, by size and
by the number of streams the copy is split over (each stream's piece may go to
a DMA engine of its own).  One JSON line.
  python tools/h2d_probe.py            (HSA_ENABLE_SDMA=0 in the environment: shader copies)"""
import json
import os
import sys
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    sizes = [1 << 20, 4 << 20, 13 << 20, 32 << 20]
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    res = {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default"), "rows": []}
    for size in sizes:
        h = torch.empty(size, dtype=torch.uint8).pin_memory()
        d = torch.empty(size, dtype=torch.uint8, device=dev)
        for k in (1, 2, 4):
            piece = size // k
            best = []
            for it in range(12):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                for j in range(k):
                    with torch.cuda.stream(streams[j]):
                        d[j * piece:(j + 1) * piece].copy_(h[j * piece:(j + 1) * piece], non_blocking=True)
                for j in range(k):
                    streams[j].synchronize()
                dt = time.perf_counter() - t
                if it >= 2:
                    best.append(dt)
            med = sorted(best)[len(best) // 2]
            res["rows"].append({"bytes": size, "streams": k, "us": med * 1e6, "GBps": size / med / 1e9})
            print(size, k, "%.1f us %.1f GB/s" % (med * 1e6, size / med / 1e9), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
