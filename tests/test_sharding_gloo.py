"""N>1 path: world_size-2 gloo ranks shard one batch into contiguous slices
(stellar-core_amd/sharding.py, the partition bench.py and the C-ABI use),
verify their slice through the product library's CPU path
(sv_ed25519_verify_batch_cpu: the engine's own algorithm built for the host;
engine="gpu" takes sv_ed25519_verify_batch instead, which torchrun-launched
ranks use on GPU nodes -- never spawned from a test process that already
holds the GPU), gather the verdict bytes and must reproduce the libsodium
verdicts and their digest."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest

from conftest import REPO, load_golden

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, rows, q, engine="cpu"):
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ctypes
    sh = importlib.import_module("stellar-core_amd.sharding")
    lib = ctypes.CDLL(os.path.join(REPO, "stellar-core_amd", "libstellar_sigverify.so"))
    d = load_golden("adversarial")
    n = len(rows)
    lo, hi = sh.shard_bounds(n, world, rank)
    mine = rows[lo:hi]
    m = len(mine)
    pk = np.ascontiguousarray(d["pk"][mine])
    sig = np.ascontiguousarray(d["sig"][mine])
    ln = d["msg_len"][mine].astype(np.uint32)
    off = np.zeros(m, np.uint64)
    if m:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    msg = np.frombuffer(b"".join(d["msg"][int(d["msg_off"][i]):int(d["msg_off"][i]) + int(d["msg_len"][i])].tobytes()
                                 for i in mine) + b"\0", np.uint8)
    local = np.zeros(m, np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    if engine == "gpu":
        rc = lib.sv_ed25519_verify_batch(P(pk), P(sig), P(msg), P(off), P(ln), ctypes.c_size_t(m), P(local), None)
    else:
        rc = lib.sv_ed25519_verify_batch_cpu(P(pk), P(sig), P(msg), P(off), P(ln), ctypes.c_size_t(m), P(local), 1)
    assert rc == 0, rc
    full = sh.gather_verdicts(local, n, world, rank)
    if rank == 0:
        q.put((full.tolist(), sh.verdict_digest(full)))
        q.close()
        q.join_thread()  # the result is in the pipe before this process goes
    dist.destroy_process_group()
    # leave without the interpreter's exit handlers: a library destructor that
    # stalls at exit must not leave the parent (pytest) waiting on this child
    os._exit(0)


def test_shard_bounds_partition():
    sh = importlib.import_module("stellar-core_amd.sharding")
    for n in [0, 1, 7, 64, 1000, 1 << 20]:
        for world in [1, 2, 3, 8]:
            b = [sh.shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            assert max(h - lo for lo, h in b) - min(h - lo for lo, h in b) <= 1


def _run_world(world, rows, engine):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, rows, q, engine)) for r in range(world)]
    for p in procs:
        p.daemon = True  # never joined at interpreter exit
        p.start()
    try:
        full, digest = q.get(timeout=240)
        for p in procs:
            p.join(timeout=60)
        codes = [p.exitcode for p in procs]
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(5)
    assert codes == [0] * world, codes
    return full, digest


@pytest.mark.parametrize("world", [2])
def test_gloo_world2_gather_matches_single_process(world):
    d = load_golden("adversarial")
    rng = np.random.default_rng(0)
    rows = np.sort(rng.choice(len(d["verdict"]), 61, replace=False))  # odd size: ragged shards
    full, digest = _run_world(world, rows, "cpu")
    sh = importlib.import_module("stellar-core_amd.sharding")
    want = d["verdict"][rows]
    assert np.array_equal(np.array(full, np.uint8), want)
    assert digest == sh.verdict_digest(want)
