#!/usr/bin/env python3
"""Developer tool: host-buffer API rate vs device API rate at one batch size.

  python tools/host_api_probe.py [n]      (env SV_STAGE_CHUNK / SV_STAGE_RAMP / SV_HOST_THREADS)

Signs n signatures on the GPU, copies them to pageable host arrays and times
sv_ed25519_verify_batch_fixed (best of 5) beside sv_ed25519_verify_device on
the same data; prints one JSON line."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sv = importlib.import_module("stellar-core_amd")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(7)
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(), stream)
    torch.cuda.synchronize()
    pk_h, sig_h, msg_h = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    out = torch.zeros(n, dtype=torch.uint8, device=dev)
    for _ in range(2):
        sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), 0, stream)
    sv.synchronize(0)
    torch.cuda.synchronize()
    t_dev = []
    for _ in range(5):
        t0 = time.perf_counter()
        sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), 0, stream)
        sv.synchronize(0)
        torch.cuda.synchronize()
        t_dev.append(time.perf_counter() - t0)
    sv.verify_fixed(pk_h[:4096], sig_h[:4096], msg_h[:4096], 32, device=0)
    t_host = []
    ok = True
    for _ in range(5):
        t0 = time.perf_counter()
        v = sv.verify_fixed(pk_h, sig_h, msg_h, 32, device=0)
        t_host.append(time.perf_counter() - t0)
        ok = ok and bool(v.all())
    d, h = min(t_dev), min(t_host)
    print(json.dumps({"n": n, "device_ms": d * 1e3, "host_ms": h * 1e3, "host_over_device": d / h, "ok": ok,
                      "host_ms_all": [round(x * 1e3, 3) for x in t_host],
                      "env": {k: os.environ.get(k) for k in ("SV_STAGE_CHUNK", "SV_STAGE_RAMP", "SV_HOST_THREADS")}}),
          flush=True)


if __name__ == "__main__":
    main()
