#!/usr/bin/env python3
"""Developer tool: where the 1k-batch latency goes (host API vs kernel time),
for fixed 32-byte and SCP-sized variable-length messages."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

sv = importlib.import_module("stellar-core_amd")
dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
g = torch.Generator(device="cpu").manual_seed(3)
seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(), stream)
torch.cuda.synchronize()
out = torch.zeros(n, dtype=torch.uint8, device=dev)
for mode in ("device", "host"):
    ts = []
    sv.kernel_time_reset()
    sv.timing_enable(True)
    pkh, sigh, msgh = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    off = (np.arange(n, dtype=np.uint64) * 32)
    ln = np.full(n, 32, np.uint32)
    for it in range(60):
        t0 = time.perf_counter()
        if mode == "device":
            sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), stream=stream)
            torch.cuda.synchronize()
        else:
            v = sv.verify_batch(pkh, sigh, msgh.reshape(-1), off, ln, device=0)
        ts.append(time.perf_counter() - t0)
    sv.timing_enable(False)
    ms, la, _ = sv.kernel_time(0)
    print("%s n=%d p50 %.3f ms  kernel %.3f ms/launch" % (mode, n, 1e3 * float(np.median(ts[10:])), ms / max(1, la)))
