"""Hardware multiply-add count of the throughput kernels (developer tool).

Runs a measurement build of the verify library (-DSV_MADCOUNT: every field
product adds its v_mad_u64_u32 count to a device counter once per wave, see
csrc/fe25519.h) on 2^20 GPU-signed signatures, first prep kernel only
(SV_DBG_PREP_ONLY), then prep + main, and writes the multiply-adds the SIMDs
issue per verify, per kernel, as JSON.  bench.py reads the result
(roofline.hw_mads_per_verify, mad_issue_frac) when its kernel_source_sha256
matches the product sources.

    bash tools/build_variants.sh madcount "-DSV_MADCOUNT"     (on the CPU host)
    python tools/madcount.py --out profiles/r03/madcount.json (on the GPU box)

Scope: products and squarings of the field (>99 % of the kernels' static
v_mad_u64_u32; the mod-L / Euclid scalar arithmetic is not counted).
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

os.environ.setdefault("SV_TEST_KNOBS", "1")  # (SV_DBG_PREP_ONLY)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
SV_DBG_PREP_ONLY = 0x8
LIBSODIUM_EQUIV = 174192  # SURVEY §8 d7 algorithmic mads per verify


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(REPO, "variants", "libsv_madcount.so"))
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    sv = importlib.import_module("stellar-core_amd")
    lib = ctypes.CDLL(args.lib, mode=os.RTLD_LOCAL)
    assert lib.sv_init() == 0
    vp = ctypes.c_void_p
    n = args.n
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(11)
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
    msgs = torch.randint(0, 256, (n, 32), dtype=torch.uint8, generator=g).to(dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    assert lib.sv_ed25519_sign_device(0, vp(seeds.data_ptr()), vp(msgs.data_ptr()), ctypes.c_size_t(n),
                                      vp(pk.data_ptr()), vp(sig.data_ptr()), None) == 0
    assert lib.sv_device_synchronize(0) == 0
    cnt = ctypes.c_ulonglong()

    def run(flags):
        assert lib.sv_set_debug_flags(flags) >= 0
        lib.sv_debug_madcount(ctypes.byref(cnt), 1)
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        assert lib.sv_ed25519_verify_device(0, vp(pk.data_ptr()), vp(sig.data_ptr()), vp(msgs.data_ptr()), None,
                                            None, 32, ctypes.c_size_t(n), vp(out.data_ptr()), None, None) == 0
        assert lib.sv_device_synchronize(0) == 0
        assert lib.sv_debug_madcount(ctypes.byref(cnt), 1) == 0
        lib.sv_set_debug_flags(0)
        return cnt.value, out

    prep, _ = run(SV_DBG_PREP_ONLY)
    full, out = run(0)
    assert int(out.sum().item()) == n, "every signed row verifies"
    # wave instructions x 64 lanes / signatures = lane-level mads per verify
    per = lambda c: c * 64.0 / n  # noqa: E731
    res = {
        "batch": n,
        "kernel_source_sha256": sv.kernel_source_digest(),
        "prep_mads_per_verify": per(prep),
        "main_mads_per_verify": per(full - prep),
        "hw_mads_per_verify": per(full),
        "libsodium_equivalent_mads_per_verify": LIBSODIUM_EQUIV,
        "ratio_hw_to_libsodium_equivalent": per(full) / LIBSODIUM_EQUIV,
        "method": "SV_MADCOUNT build: each field product / squaring adds its v_mad_u64_u32 count (101 / 56) "
                  "once per wave; wave instructions x 64 / signatures",
    }
    print(json.dumps(res, indent=1), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
