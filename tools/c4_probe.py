#!/usr/bin/env python3
"""Config 4 through the integration path alone (bench.py config4_integrated):
prints one JSON line per run with the shapes' verdict / main-thread latencies.
  python tools/c4_probe.py [runs]"""
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    import torch  # noqa: F401  (one HIP runtime, as bench.py)
    bench = importlib.import_module("bench")
    sv = importlib.import_module("stellar-core_amd")
    sodium = bench.load_libsodium()
    for _ in range(runs):
        r = bench.config4_integrated(sv, sodium)
        out = {"memo": os.environ.get("SV_KEY_MEMO", "1"), "memo_keyed": os.environ.get("SV_MEMO_KEYED", "1")}
        for k, f in r.items():
            if isinstance(f, dict):
                out[k] = {x: round(f[x], 4) for x in ("verdict_p50_ms", "verdict_p99_ms", "main_p50_ms", "main_p99_ms",
                                                      "ready_p50_ms", "achieved_per_s", "mean_batch",
                                                      "main_thread_verifysig_per_s")}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
