#!/usr/bin/env python3
"""Developer tool: per-phase s_memtime breakdown of the verify kernel, from a
variant built with -DSV_PHASE_PROF (tools/build_variants.sh prof "-DSV_PHASE_PROF").
Usage: python tools/phase_prof.py variants/libsv_prof.so
(split build: phases 0-4 are the prep kernel's; the main kernel is not instrumented)"""
import ctypes
import sys

import torch  # noqa: F401  (load torch's HIP runtime first)

NAMES = ["sha512 (prep: after loads)", "checks+decode A,R", "mod L + Euclid", "tables A,R", "W + digits (+ record)", "scalar mult (prep: input loads)",
         "identity check", "-"]
lib = ctypes.CDLL(sys.argv[1], mode=ctypes.RTLD_LOCAL)
assert lib.sv_init() == 0
dev = torch.device("cuda", 0)
n = 1 << 20
g = torch.Generator(device="cpu").manual_seed(5)
seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
vp = ctypes.c_void_p
assert lib.sv_ed25519_sign_device(0, vp(seeds.data_ptr()), vp(msgs.data_ptr()), ctypes.c_size_t(n),
                                  vp(pk.data_ptr()), vp(sig.data_ptr()), None) == 0
lib.sv_device_synchronize(0)
out = torch.zeros(n, dtype=torch.uint8, device=dev)
cyc = (ctypes.c_ulonglong * 8)()
for it in range(3):
    lib.sv_debug_phase_cycles(cyc, 1)
    assert lib.sv_ed25519_verify_device(0, vp(pk.data_ptr()), vp(sig.data_ptr()), vp(msgs.data_ptr()), None,
                                        None, 32, ctypes.c_size_t(n), vp(out.data_ptr()), None, None) == 0
    lib.sv_device_synchronize(0)
    lib.sv_debug_phase_cycles(cyc, 0)
assert int(out.sum().item()) == n
tot = sum(cyc)
for i in range(8):
    print("%-20s %6.2f %%  (%.0f per-wave cycles per signature group)" % (NAMES[i], 100.0 * cyc[i] / tot,
                                                                          cyc[i] / (n / 64)))
