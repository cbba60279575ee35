"""Latency-class isolation probe (developer tool): the harness of
tests/test_gpu_isolation.py with its numbers written to a JSON file.

    python tools/lat_isolation.py --out iso.json            (shared mode on)
    SV_LAT_SHARE_MS=0 python tools/lat_isolation.py ...     (shared mode off)
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--host-n", type=int, default=1 << 22)
    ap.add_argument("--dev-n", type=int, default=1 << 24)
    args = ap.parse_args()
    import torch
    sv = importlib.import_module("stellar-core_amd")
    from isolation_load import run_isolation
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    o.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    o.oracle_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    o.oracle_ed25519_seed_keypair.argtypes = [ctypes.c_char_p] * 3
    res = run_isolation(sv, torch, o, host_n=args.host_n, dev_n=args.dev_n)
    res["SV_LAT_SHARE_MS"] = os.environ.get("SV_LAT_SHARE_MS", "1000 (default)")
    print(json.dumps(res, indent=1), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
