"""The C-ABI library builds for gfx950, loads on a CPU-only host and exports
every entry point include/*.h declares; the product path fails loudly (no CPU
fallback) when no GPU is present."""
import ctypes
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(sv_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


@pytest.fixture(scope="module")
def lib_path(sv):
    if not os.path.exists(sv.LIB_PATH):
        subprocess.run(["make", "-s", "-j4"], cwd=os.path.join(REPO, "stellar-core_amd"), check=True)
    return sv.LIB_PATH


def test_header_declares_expected_surface():
    names = _declared_functions()
    for must in ["sv_init", "sv_shutdown", "sv_device_count", "sv_last_error_string", "sv_ed25519_verify_batch",
                 "sv_ed25519_verify_batch_fixed", "sv_ed25519_verify_device", "sv_ed25519_sign_device"]:
        assert must in names


def test_library_exports_every_declared_symbol(lib_path, sv):
    lib = ctypes.CDLL(lib_path)
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert set(sv.EXPORTED_SYMBOLS) <= set(_declared_functions())


def test_host_library_exports_every_declared_symbol(sv):
    """libstellar_host.so (C++ PubKeyUtils / SignatureChecker / micro-batcher
    mirror) exports every svh_* entry point include/stellar_host.h declares."""
    if not os.path.exists(sv.HOSTLIB_PATH):
        subprocess.run(["make", "-s", "-j4"], cwd=os.path.join(REPO, "stellar-core_amd"), check=True)
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "stellar_host.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(svh_[a-z0-9_]+)\s*\(", src)) - {"svh_batch_verify_fn", "svh_keyed_verify_fn"})
    assert "svh_mb_run" in names and "svh_check_txset" in names
    lib = ctypes.CDLL(sv.HOSTLIB_PATH)
    for name in names:
        assert hasattr(lib, name), name


def test_code_object_is_gfx950_only(lib_path):
    blob = open(lib_path, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z]*(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_no_cpu_fallback_without_gpu(sv):
    """On a host without a GPU every verify entry point raises (never rejects)."""
    try:
        n = sv.device_count()
    except sv.SigVerifyError:
        n = 0
    if n > 0:
        pytest.skip("a GPU is present")
    d = np.load(os.path.join(REPO, "tests", "golden", "intree.npz"))
    with pytest.raises(sv.SigVerifyError):
        sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    with pytest.raises(sv.SigVerifyError):
        sv.verify_fixed(d["pk"][:2], d["sig"][:2], np.zeros(64, np.uint8))
    with pytest.raises(sv.SigVerifyError):
        sv.verify_batch_keyed(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    with pytest.raises(sv.SigVerifyError):
        sv.cache_keys(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"])
    with pytest.raises(sv.SigVerifyError):
        sv.sha256_batch(d["msg"], d["msg_off"], d["msg_len"])


def test_python_binding_validates_shapes(sv):
    with pytest.raises(ValueError):
        sv.verify_batch(np.zeros((2, 32), np.uint8), np.zeros((3, 64), np.uint8), np.zeros(4, np.uint8),
                        [0, 0], [1, 1])
    with pytest.raises(ValueError):
        sv.verify_batch(np.zeros((2, 32), np.uint8), np.zeros((2, 64), np.uint8), np.zeros(4, np.uint8),
                        [0, 3], [1, 2])


def test_kernel_path_setter_validates(sv):
    """sv_set_kernel_path accepts SV_PATH_AUTO/THROUGHPUT/LATENCY, returns the
    previous default, and rejects anything else (no GPU needed)."""
    prev = sv.set_kernel_path(sv.PATH_LATENCY)
    assert sv.set_kernel_path(sv.PATH_THROUGHPUT) == sv.PATH_LATENCY
    assert sv.set_kernel_path(prev) == sv.PATH_THROUGHPUT
    with pytest.raises(sv.SigVerifyError):
        sv.set_kernel_path(7)


def test_result_changing_knobs_need_opt_in(sv):
    """SV_DBG_FAIL / SV_DBG_PREP_ONLY (calls that err or write no verdicts) are
    refused in a process without SV_TEST_KNOBS=1; the path-selecting knobs are
    not.  Run in a child process: this one opted in (conftest.py)."""
    code = ("import ctypes,sys; l=ctypes.CDLL(sys.argv[1]); l.sv_set_debug_flags.argtypes=[ctypes.c_uint32];"
            "print(l.sv_set_debug_flags(4), l.sv_set_debug_flags(8), l.sv_set_debug_flags(1), l.sv_set_debug_flags(0))")
    env = {k: v for k, v in os.environ.items() if k != "SV_TEST_KNOBS"}
    env["SV_NO_TORCH"] = "1"
    out = subprocess.run([sys.executable, "-c", code, sv.LIB_PATH], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["-1", "-1", "0", "1"]
    env["SV_TEST_KNOBS"] = "1"
    out = subprocess.run([sys.executable, "-c", code, sv.LIB_PATH], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.stdout.split() == ["0", "4", "8", "1"]
