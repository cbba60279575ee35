#!/usr/bin/env python3
"""Developer tool: host-API latency of a 1k SCP-sized batch (128-384 B random
messages) vs the device API on the same batch; run with SV_STAGE_TRACE=1 for
the per-call pack time."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

sv = importlib.import_module("stellar-core_amd")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
rng = np.random.default_rng(3)
pk = rng.integers(0, 256, (n, 32), dtype=np.uint8)
sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
ln = rng.integers(128, 385, n).astype(np.uint32)
off = np.zeros(n, np.uint64)
off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
msg = rng.integers(0, 256, int(ln.sum()), dtype=np.uint8)
dev = torch.device("cuda", 0)
for _ in range(10):
    sv.verify_batch(pk, sig, msg, off, ln, device=0)
t = []
for _ in range(100):
    t0 = time.perf_counter()
    sv.verify_batch(pk, sig, msg, off, ln, device=0)
    t.append(time.perf_counter() - t0)
print("host API  n=%d p50 %.1f us" % (n, 1e6 * np.median(t)), flush=True)
dpk, dsig = torch.from_numpy(pk).to(dev), torch.from_numpy(sig).to(dev)
dmsg, doff = torch.from_numpy(msg).to(dev), torch.from_numpy(off.view(np.int64)).to(dev)
dln = torch.from_numpy(ln.view(np.int32)).to(dev)
out = torch.zeros(n, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
t = []
for it in range(110):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sv.verify_device(0, dpk.data_ptr(), dsig.data_ptr(), dmsg.data_ptr(), n, out.data_ptr(), stream=stream,
                     fixed_msg_len=0, d_msg_off=doff.data_ptr(), d_msg_len=dln.data_ptr())
    torch.cuda.synchronize()
    if it >= 10:
        t.append(time.perf_counter() - t0)
print("device API n=%d p50 %.1f us (launch + kernel + sync)" % (n, 1e6 * np.median(t)), flush=True)
