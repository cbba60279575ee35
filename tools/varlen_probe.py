#!/usr/bin/env python3
"""Developer tool: the same 32-byte-message batch through the fixed-length host
call and through the variable-length one (offsets i * 32, lengths 32), per call,
to price the variable-length image and kernel mode on medium batches.

  python tools/varlen_probe.py [calls] [sizes,comma,separated]"""
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
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    sizes = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (12289, 16384, 29217, 50000)
    sv = importlib.import_module("stellar-core_amd")
    dev = torch.device("cuda", 0)
    n_max = max(sizes)
    rng = np.random.default_rng(9)
    seeds = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n_max, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n_max, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n_max, pk.data_ptr(), sig.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    P, S, M = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    S[::16, 40] ^= 0x08
    want = np.ones(n_max, np.uint8)
    want[::16] = 0
    sv.set_key_cache(0)
    res = {}
    for n in sizes:
        p, s, m = np.ascontiguousarray(P[:n]), np.ascontiguousarray(S[:n]), np.ascontiguousarray(M[:n])
        flat = m.reshape(-1)
        off = np.arange(n, dtype=np.uint64) * 32
        ln = np.full(n, 32, np.uint32)
        row = {}
        for name, fn in (("fixed", lambda: sv.verify_fixed(p, s, m, 32, device=0)),
                         ("var", lambda: sv.verify_batch(p, s, flat, off, ln, device=0))):
            for _ in range(2):
                fn()
            ts = []
            ok = True
            for _ in range(calls):
                t = time.perf_counter()
                o = fn()
                ts.append(time.perf_counter() - t)
                ok = ok and bool(np.array_equal(o, want[:n]))
            row[name] = {"ms": float(np.median(ts)) * 1e3, "ok": ok}
        res[str(n)] = row
        print(n, json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
