#!/usr/bin/env python3
"""Host-feed probe of the in-process multi-GPU path (VERDICT r5 missing #2).

For G = 1, 2, 4, 8 slots (up to what the process sees; rehearse on one card
with SV_DEVICE_MAP=0,0,0,0,0,0,0,0), feeds G x 2^20 fixed-length signatures
(128 B each: pk 32 + sig 64 + msg 32) from pageable host arrays through
sv_host_feed_probe: the slices, each slot's staging workers, the pack into
pinned staging, and (upload) the H2D copies -- no kernels.  Prints one JSON
object: per G the feed rate in signatures/s and GB/s, best of `--reps`, and
what G GPUs verifying at `--gpu-rate` need (G x rate x 128 B).

  python tools/feed_probe.py [--reps 5] [--per-slot 1048576] [--gpu-rate 1.05e8]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--per-slot", type=int, default=1 << 20)
    ap.add_argument("--gpu-rate", type=float, default=1.05e8, help="verifies/s of one GPU (BENCH_r05: 1.055e8)")
    ap.add_argument("--max-g", type=int, default=8)
    args = ap.parse_args()
    sv = importlib.import_module("stellar-core_amd")
    slots = sv.device_count()
    out = {"slots": slots, "device_map": os.environ.get("SV_DEVICE_MAP"),
           "slot_threads_env": os.environ.get("SV_SLOT_THREADS"), "per_slot": args.per_slot,
           "bytes_per_signature": 128, "gpu_rate": args.gpu_rate, "per_G": {}}
    rng = np.random.default_rng(1)
    G = 1
    while G <= min(args.max_g, slots):
        n = G * args.per_slot
        P = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        S = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        M = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        row = {"signatures": n, "need_sigs_per_s": G * args.gpu_rate, "need_GBps": G * args.gpu_rate * 128 / 1e9}
        for upload in (False, True):
            sv.host_feed_probe(P[:65536 * G], S[:65536 * G], M[:65536 * G], 32, max_devices=G, upload=upload)
            best, st = None, None
            for _ in range(args.reps):
                r = sv.host_feed_probe(P, S, M, 32, max_devices=G, upload=upload)
                if best is None or r["seconds"] < best:
                    best, st = r["seconds"], r
            key = "pack_and_h2d" if upload else "pack_only"
            row[key] = {"seconds": best, "sigs_per_s": n / best, "GBps": n * 128 / best / 1e9,
                        "frac_of_need": (n / best) / (G * args.gpu_rate)}
            row["slots_used"] = st["slots"]
            row["threads_per_slot"] = st["threads_per_slot"]
            row["usable_cpus"] = st["usable_cpus"]
            row["gpu_numa"] = st["gpu_numa"]
            row["staging_numa"] = st["staging_numa"]
            row["pinned_cpus"] = st["pinned_cpus"]
        out["per_G"][str(G)] = row
        print("G=%d pack %.1f GB/s, pack+H2D %.1f GB/s (need %.1f)" % (
            G, row["pack_only"]["GBps"], row["pack_and_h2d"]["GBps"], row["need_GBps"]), file=sys.stderr, flush=True)
        del P, S, M
        G *= 2
    print(json.dumps(out))


if __name__ == "__main__":
    main()
