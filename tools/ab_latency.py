#!/usr/bin/env python3
"""Developer tool: latency-path kernel time per verify-library variant
(tools/build_variants.sh) on one 1000-signature batch; verdicts of variants
that skip phases (SV_QPROF_*) are not checked."""
import ctypes
import glob
import os
import sys

import torch  # noqa: F401  (load torch's HIP runtime first)
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
paths = sys.argv[1:] or sorted(glob.glob(os.path.join(REPO, "variants", "libsv_*.so")))
n = 1000
dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(5)
seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
vp = ctypes.c_void_p
libs = {}
for p in paths:
    lib = ctypes.CDLL(p, mode=os.RTLD_LOCAL)
    lib.sv_kernel_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64)]
    assert lib.sv_init() == 0
    assert lib.sv_set_kernel_path(2) == 0
    libs[os.path.basename(p)] = lib
first = next(iter(libs.values()))
assert first.sv_ed25519_sign_device(0, vp(seeds.data_ptr()), vp(msgs.data_ptr()), ctypes.c_size_t(n),
                                    vp(pk.data_ptr()), vp(sig.data_ptr()), None) == 0
first.sv_device_synchronize(0)
# SCP-sized variable-length messages (128-384 B: 2-4 SHA-512 blocks), random
# bytes: timing only (every lane runs every phase whatever its verdict)
rng = np.random.default_rng(9)
vlen = rng.integers(128, 385, n).astype(np.uint32)
voff = np.zeros(n, np.uint64)
voff[1:] = np.cumsum(vlen[:-1], dtype=np.uint64)
vmsg = torch.from_numpy(rng.integers(0, 256, int(vlen.sum()), dtype=np.uint8)).to(dev)
voff_d = torch.from_numpy(voff.view(np.int64)).to(dev)
vlen_d = torch.from_numpy(vlen.view(np.int32)).to(dev)
res = {k: [] for k in libs}
resv = {k: [] for k in libs}
for rnd in range(5):
    for name, lib in libs.items():
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        lib.sv_timing_enable(1)
        lib.sv_kernel_time_reset()
        for _ in range(20):
            assert lib.sv_ed25519_verify_device(0, vp(pk.data_ptr()), vp(sig.data_ptr()), vp(vmsg.data_ptr()),
                                                vp(voff_d.data_ptr()), vp(vlen_d.data_ptr()), 0, ctypes.c_size_t(n),
                                                vp(out.data_ptr()), None, None) == 0
        lib.sv_device_synchronize(0)
        ms, la, sg = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.sv_kernel_time(0, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(sg))
        lib.sv_timing_enable(0)
        resv[name].append(ms.value / la.value)
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        lib.sv_timing_enable(1)
        lib.sv_kernel_time_reset()
        for _ in range(20):
            assert lib.sv_ed25519_verify_device(0, vp(pk.data_ptr()), vp(sig.data_ptr()), vp(msgs.data_ptr()), None,
                                                None, 32, ctypes.c_size_t(n), vp(out.data_ptr()), None, None) == 0
        lib.sv_device_synchronize(0)
        ms, la, sg = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.sv_kernel_time(0, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(sg))
        lib.sv_timing_enable(0)
        res[name].append(ms.value / la.value)
        if rnd == 0:
            print("%-28s valid rows %d" % (name, int(out.sum().item())), flush=True)
for name, v in res.items():
    print("%-28s median %.4f ms per 1k batch (latency path, 32 B)  %.4f ms (128-384 B)"
          % (name, float(np.median(v)), float(np.median(resv[name]))), flush=True)
