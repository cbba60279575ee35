#!/usr/bin/env python3
"""Developer tool: GPU A/B timing of verify-library variants (built by
tools/build_variants.sh).  One 2^20 fixed-32B batch signed on the GPU (1/8 of
the rows corrupted); every variant must reproduce the baseline's verdicts;
prints kernel ms per launch (median over interleaved rounds) per variant."""
import os
os.environ.setdefault("SV_TEST_KNOBS", "1")  # (sv_set_debug_flags PREP_ONLY / FAIL)
import ctypes
import glob
import os
import sys

import torch  # noqa: F401  (load torch's HIP runtime first)
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
paths = sys.argv[1:] or sorted(glob.glob(os.path.join(REPO, "variants", "libsv_*.so")))
libs = {}
for p in paths:
    lib = ctypes.CDLL(p, mode=os.RTLD_LOCAL)
    lib.sv_kernel_time.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64)]
    assert lib.sv_init() == 0
    libs[os.path.basename(p)] = lib
    print("%-28s resident workgroups/CU: %d" % (os.path.basename(p), lib.sv_occupancy_blocks_per_cu()), flush=True)

dev = torch.device("cuda", 0)
_pr = torch.cuda.get_device_properties(0)
print("device %s CUs %d" % (_pr.name, _pr.multi_processor_count), flush=True)
n = 1 << 20
g = torch.Generator(device="cpu").manual_seed(5)
seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
first = next(iter(libs.values()))
vp = ctypes.c_void_p
assert first.sv_ed25519_sign_device(0, vp(seeds.data_ptr()), vp(msgs.data_ptr()), ctypes.c_size_t(n),
                                    vp(pk.data_ptr()), vp(sig.data_ptr()), None) == 0
first.sv_device_synchronize(0)
sig[::8, 3] ^= 1
torch.cuda.synchronize()
want = None
res = {k: [] for k in libs}
prep = {k: [] for k in libs}
SV_DBG_PREP_ONLY = 0x8  # (include/stellar_sigverify.h)


def timed(lib, out, reps=3):
    lib.sv_timing_enable(1)
    lib.sv_kernel_time_reset()
    for _ in range(reps):
        assert lib.sv_ed25519_verify_device(0, vp(pk.data_ptr()), vp(sig.data_ptr()), vp(msgs.data_ptr()), None,
                                            None, 32, ctypes.c_size_t(n), vp(out.data_ptr()), None, None) == 0
    lib.sv_device_synchronize(0)
    ms, la, sg = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.sv_kernel_time(0, ctypes.byref(ms), ctypes.byref(la), ctypes.byref(sg))
    lib.sv_timing_enable(0)
    return ms.value / la.value


ROUNDS = int(os.environ.get("AB_ROUNDS", "6"))
for rnd in range(ROUNDS):
    for name, lib in libs.items():
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        t = timed(lib, out)
        o = out.cpu().numpy()
        diag = any(t in name for t in os.environ.get("AB_NOCHECK", "").split(",") if t)
        if want is None and not diag:
            want = o
            assert o.sum() == n - n // 8, o.sum()
        if not diag and want is not None:
            assert (o == want).all(), name + " verdict mismatch"
        has_split = hasattr(lib, "sv_set_debug_flags") and lib.sv_set_debug_flags(SV_DBG_PREP_ONLY) >= 0
        tp = float("nan")
        if has_split:
            tp = timed(lib, torch.zeros(n, dtype=torch.uint8, device=dev))
            lib.sv_set_debug_flags(0)
        if rnd > 0:  # round 0 warms clocks and caches
            res[name].append(t)
            prep[name].append(tp)
        print("round %d %-28s %.3f ms  (prep %.3f)" % (rnd, name, t, tp), flush=True)
for name, v in res.items():
    mp = float(np.median(prep[name]))
    print("%-28s median %.3f ms per 2^20  (%.3e verifies/s)  prep %.3f  main %.3f" %
          (name, float(np.median(v)), n / (np.median(v) * 1e-3), mp, float(np.median(v)) - mp))
