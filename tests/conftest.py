"""Shared test setup.

Markers: `gpu` = needs an MI355X (run by the driver on the GPU box with
`pytest -m gpu`); everything else runs on CPU here.

Native test infrastructure (oracle/liboracle.so, tests/native/libhostcore.so)
is built on demand with gcc if missing.  torch is imported before the engine
library is loaded so the process holds ONE HIP runtime (torch ships its own
libamdhip64 with the same soname).
"""
import ctypes
import faulthandler
import importlib
import os
import signal
import subprocess
import sys

import numpy as np
import pytest

# the engine's error-injection knob (sv_set_debug_flags SV_DBG_FAIL) is
# refused unless the process opts in (include/stellar_sigverify.h)
os.environ["SV_TEST_KNOBS"] = "1"

# SIGUSR1 dumps every thread's Python stack (diagnosing a run that does not exit)
faulthandler.register(signal.SIGUSR1, all_threads=True)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)

try:  # one HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (gfx950)")


def _make(dirpath, target):
    # make every time: the Makefiles list the headers, so an edited header
    # rebuilds the library instead of testing a stale one
    path = os.path.join(dirpath, target)
    subprocess.run(["make", "-s", target], cwd=dirpath, check=True)
    return path


@pytest.fixture(scope="session")
def oracle():
    lib = ctypes.CDLL(_make(os.path.join(REPO, "oracle"), "liboracle.so"))
    lib.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    lib.oracle_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    lib.oracle_ed25519_seed_keypair.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    return lib


@pytest.fixture(scope="session")
def hostcore():
    return ctypes.CDLL(_make(os.path.join(REPO, "tests", "native"), "libhostcore.so"))


@pytest.fixture(scope="session")
def sv():
    return importlib.import_module("stellar-core_amd")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def golden():
    return {n: load_golden(n) for n in ("intree", "valid", "msglen", "longmsg", "adversarial", "lattice_edge")}


def oracle_verdicts(oracle, d, rows=None):
    rows = range(len(d["verdict"])) if rows is None else rows
    out = []
    for i in rows:
        o, ln = int(d["msg_off"][i]), int(d["msg_len"][i])
        m = d["msg"][o:o + ln].tobytes()
        out.append(1 if oracle.oracle_ed25519_verify(d["sig"][i].tobytes(), m, ln, d["pk"][i].tobytes()) == 0 else 0)
    return np.array(out, np.uint8)
