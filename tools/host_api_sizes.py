#!/usr/bin/env python3
"""Developer tool: host-API verify rate (pageable host arrays, fixed 32-byte
messages, device 0) at several batch sizes: one-chunk sizes (<= 2^18, staged
or read in place: SV_BULK_ZC_IN) and a multi-chunk 2^20.  Keys and signatures
are made on the GPU (sv_ed25519_sign_device), 1/16 of the rows corrupted; every
call's verdicts are checked.  Prints one JSON line.
Usage: python tools/host_api_sizes.py [iterations]"""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    sv = importlib.import_module("stellar-core_amd")
    dev = torch.device("cuda", 0)
    n_max = 1 << 20
    rng = np.random.default_rng(3)
    seeds = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n_max, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n_max, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n_max, pk.data_ptr(), sig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    P, S, M = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    S[::16, 40] ^= 0x08
    want = np.ones(n_max, np.uint8)
    want[::16] = 0
    res = {"bulk_in_place": os.environ.get("SV_BULK_ZC_IN", "1") != "0"}
    for n in (12289, 29217, 100000, 262144, 1 << 20):
        p, s, m = np.ascontiguousarray(P[:n]), np.ascontiguousarray(S[:n]), np.ascontiguousarray(M[:n])
        for _ in range(3):
            out = sv.verify_fixed(p, s, m, 32, device=0)
        ts = []
        for _ in range(iters):
            t = time.perf_counter()
            out = sv.verify_fixed(p, s, m, 32, device=0)
            ts.append(time.perf_counter() - t)
            assert np.array_equal(out, want[:n]), n
        med = float(np.median(ts))
        res[str(n)] = {"ms": med * 1e3, "verifies_per_s": n / med}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
