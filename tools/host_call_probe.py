#!/usr/bin/env python3
"""Developer tool: where a medium host call's time goes.  Runs verify_fixed
(pageable numpy arrays, 32-byte messages, as tools/size_sweep.py's host_api
column) at the given sizes and prints each call's wall time with its
steady-clock start, so SV_STAGE_TRACE=1 lines and a rocprofv3 kernel trace
can be lined up against it (tools/host_call_timeline.py).

  python tools/host_call_probe.py [calls] [sizes,comma,separated]"""
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
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    sizes = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (16384, 29217, 50000, 100000)
    sv = importlib.import_module("stellar-core_amd")
    dev = torch.device("cuda", 0)
    n_max = max(sizes)
    rng = np.random.default_rng(5)
    seeds = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n_max, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n_max, 64), dtype=torch.uint8, device=dev)
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n_max, pk.data_ptr(), sig.data_ptr(),
                   torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    sig[::16, 40] ^= 0x08
    want = np.ones(n_max, np.uint8)
    want[::16] = 0
    P, S, M = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    sv.set_key_cache(0)
    out = {}
    for n in sizes:
        p, s, m = np.ascontiguousarray(P[:n]), np.ascontiguousarray(S[:n]), np.ascontiguousarray(M[:n])
        for _ in range(2):
            sv.verify_fixed(p, s, m, 32, device=0)
        rows = []
        for _ in range(calls):
            t_abs = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
            t = time.perf_counter()
            o = sv.verify_fixed(p, s, m, 32, device=0)
            dt = time.perf_counter() - t
            rows.append({"start_ns": t_abs, "ms": dt * 1e3, "ok": bool(np.array_equal(o, want[:n]))})
            print("PROBE n=%d start_ns=%d ms=%.3f" % (n, t_abs, dt * 1e3), file=sys.stderr, flush=True)
        out[str(n)] = {"median_ms": float(np.median([r["ms"] for r in rows])), "calls": rows}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
