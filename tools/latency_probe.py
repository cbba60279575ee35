#!/usr/bin/env python3
"""Developer tool: batch latency per kernel path (device API, kernel time from
the engine's HIP events) for a range of batch sizes, plus the host-API p50 at
the first size.  Usage: python tools/latency_probe.py [n1 n2 ...]"""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

sv = importlib.import_module("stellar-core_amd")
dev = torch.device("cuda", 0)
sizes = [int(a) for a in sys.argv[1:]] or [1000]
nmax = max(sizes)
g = torch.Generator(device="cpu").manual_seed(3)
seeds = torch.randint(0, 256, (nmax, 32), dtype=torch.uint8, generator=g).to(dev)
msgs = torch.randint(0, 256, (nmax, 32), dtype=torch.uint8, generator=g).to(dev)
pk = torch.empty((nmax, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((nmax, 64), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), nmax, pk.data_ptr(), sig.data_ptr(), stream)
torch.cuda.synchronize()
out = torch.zeros(nmax, dtype=torch.uint8, device=dev)
paths = {"throughput": sv.PATH_THROUGHPUT, "latency": sv.PATH_LATENCY}
for n in sizes:
    row = []
    for name, code in paths.items():
        sv.set_kernel_path(code)
        sv.kernel_time_reset()
        sv.timing_enable(True)
        for it in range(20):
            sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        sv.timing_enable(False)
        ms, la, _ = sv.kernel_time(0)
        assert int(out[:n].sum().item()) == n
        row.append("%s %.3f ms" % (name, ms / max(1, la)))
    print("n=%7d  %s" % (n, "  ".join(row)), flush=True)
sv.set_kernel_path(sv.PATH_AUTO)
n = sizes[0]
pkh, sigh, msgh = pk[:n].cpu().numpy(), sig[:n].cpu().numpy(), msgs[:n].cpu().numpy()
off = np.arange(n, dtype=np.uint64) * 32
ln = np.full(n, 32, np.uint32)
ts = []
for it in range(60):
    t0 = time.perf_counter()
    sv.verify_batch(pkh, sigh, msgh.reshape(-1), off, ln, device=0)
    ts.append(time.perf_counter() - t0)
print("host API (auto path) n=%d p50 %.3f ms" % (n, 1e3 * float(np.median(ts[10:]))))
