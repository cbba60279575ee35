#!/usr/bin/env python3
"""Developer tool: the two kernel paths over medium batch
sizes, kernel-only (HIP events around the launches, device-resident input) and
per call (host API from pageable arrays), to set the auto crossover
(kQuickMax, csrc/sv_api.cpp) from measurements on the current kernels.

  throughput  one lane per signature (prep + persistent main kernel; SV_DBG_NO_QUAD)
  quad        one signature per quad of lanes (sv_quad_kernel; SV_DBG_QUAD)
  latency     the octet kernel, key cache off (the cold-key latency path: what a
              tx set's mostly distinct signers get)
  auto        the engine's own choice

32-byte messages, keys and signatures made on the GPU, 1/16 of the rows
corrupted; every call's verdicts are checked.  Prints one JSON line.
Usage: python tools/size_sweep.py [iterations] [sizes,comma,separated]"""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

SIZES = (4096, 8192, 12288, 16384, 20480, 24576, 29217, 40960, 50000, 65536, 100000, 131072, 262144)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 15
    sizes = tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else SIZES
    sv = importlib.import_module("stellar-core_amd")
    dev = torch.device("cuda", 0)
    n_max = max(sizes)
    rng = np.random.default_rng(5)
    seeds = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    msgs = torch.from_numpy(rng.integers(0, 256, (n_max, 32), dtype=np.uint8)).to(dev)
    pk = torch.empty((n_max, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n_max, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n_max, pk.data_ptr(), sig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    sig[::16, 40] ^= 0x08
    want = np.ones(n_max, np.uint8)
    want[::16] = 0
    P, S, M = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    out_d = torch.zeros(n_max, dtype=torch.uint8, device=dev)
    sv.set_key_cache(0)
    res = {"iters": iters, "sizes": list(sizes), "paths": {}}
    paths = (("throughput", sv.PATH_THROUGHPUT, sv.DBG_NO_QUAD), ("quad", sv.PATH_THROUGHPUT, sv.DBG_QUAD),
             ("latency", sv.PATH_LATENCY, 0), ("auto", sv.PATH_AUTO, 0))
    only = os.environ.get("SWEEP_PATHS")
    for name, code, dbg in paths:
        if only and name not in only.split(","):
            continue
        prev = sv.set_kernel_path(code)
        prev_dbg = sv.set_debug_flags(dbg)
        rows = {}
        for n in sizes:
            if name == "latency" and n > 131072:
                continue
            # kernel only
            for _ in range(2):
                sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out_d.data_ptr(), 0, st)
            sv.synchronize(0)
            torch.cuda.synchronize(dev)
            sv.kernel_time_reset()
            sv.timing_enable(True)
            t0 = time.perf_counter()
            for _ in range(iters):
                sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out_d.data_ptr(), 0, st)
            sv.synchronize(0)
            torch.cuda.synchronize(dev)
            wall_dev = (time.perf_counter() - t0) / iters
            sv.timing_enable(False)
            k_ms, k_la, _ = sv.kernel_time(0)
            ok_d = bool(np.array_equal(out_d[:n].cpu().numpy(), want[:n]))
            # per call through the host API
            p, s, m = np.ascontiguousarray(P[:n]), np.ascontiguousarray(S[:n]), np.ascontiguousarray(M[:n])
            for _ in range(2):
                sv.verify_fixed(p, s, m, 32, device=0)
            ts = []
            ok_h = True
            for _ in range(iters):
                t = time.perf_counter()
                o = sv.verify_fixed(p, s, m, 32, device=0)
                ts.append(time.perf_counter() - t)
                ok_h = ok_h and bool(np.array_equal(o, want[:n]))
            host_ms = float(np.median(ts)) * 1e3
            rows[str(n)] = {"kernel_ms_per_call": k_ms / iters, "device_api_wall_ms": wall_dev * 1e3,
                            "host_api_ms": host_ms, "host_api_verifies_per_s": n / (host_ms * 1e-3),
                            "kernel_launches_per_call": k_la / iters, "verdicts_ok": ok_d and ok_h}
            print(name, n, json.dumps(rows[str(n)]), file=sys.stderr, flush=True)
        res["paths"][name] = rows
        sv.set_kernel_path(prev)
        sv.set_debug_flags(prev_dbg)
    sv.set_key_cache(1024)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
