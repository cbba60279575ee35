"""Latency-class isolation under bulk load (VERDICT r2 "next" 3), shared by
tests/test_gpu_isolation.py and tools/lat_isolation.py.

One thread submits 1000-signature SCP batches (100 validator keys, warm key
cache: the comb kernel) back to back through the host API, as the overlay
thread's pre-verify does (/root/reference/src/overlay/Peer.cpp:963-970),
while the caller's thread runs a 2^22-signature host batch (a catchup-sized
verifySigBatch) and then a 2^24-signature device batch on the same GPU, as
concurrent verifySig callers do in the reference
(/root/reference/src/crypto/SecretKey.cpp:44,449,464).  Every latency batch's
verdicts must equal the oracle's; the bulk batches must accept exactly their
uncorrupted rows.  Latencies are grouped by the bulk phase they started in.
"""
import threading
import time

import numpy as np

from scp_sets import scp_set


def _pct(v, q):
    return float(np.percentile(v, q)) if len(v) else None


def _summary(lat_ms):
    return {"batches": len(lat_ms), "p50_ms": _pct(lat_ms, 50), "p99_ms": _pct(lat_ms, 99),
            "max_ms": float(max(lat_ms)) if lat_ms else None}


def _bulk_sets(sv, torch, dev, host_n, dev_n, seed):
    base = 1 << 20
    rng = np.random.default_rng(seed)
    seeds = torch.from_numpy(rng.integers(0, 256, (base, 32), dtype=np.uint8)).to(dev)
    tm = torch.from_numpy(rng.integers(0, 256, (base, 32), dtype=np.uint8)).to(dev)
    tpk = torch.empty((base, 32), dtype=torch.uint8, device=dev)
    tsig = torch.empty((base, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sv.sign_device(0, seeds.data_ptr(), tm.data_ptr(), base, tpk.data_ptr(), tsig.data_ptr(), st)
    torch.cuda.synchronize(dev)
    del seeds
    # host batch: the signed set tiled, 1 % of rows with an S byte flipped
    reps = max(1, host_n // base)
    pk_h = np.tile(tpk.cpu().numpy(), (reps, 1))[:host_n]
    sig_h = np.tile(tsig.cpu().numpy(), (reps, 1))[:host_n]
    msg_h = np.tile(tm.cpu().numpy(), (reps, 1))[:host_n]
    bad_h = np.unique(rng.integers(0, host_n, host_n // 100))
    sig_h[bad_h, 40 + (bad_h % 20)] ^= 0x04
    want_h = np.ones(host_n, np.uint8)
    want_h[bad_h] = 0
    # device batch
    reps = max(1, dev_n // base)
    pk_d = tpk.repeat(reps, 1)[:dev_n].contiguous()
    sig_d = tsig.repeat(reps, 1)[:dev_n].contiguous()
    msg_d = tm.repeat(reps, 1)[:dev_n].contiguous()
    bad_d = np.unique(rng.integers(0, dev_n, dev_n // 100))
    bad_t = torch.from_numpy(bad_d).to(dev)
    col = torch.from_numpy(32 + (bad_d % 32)).to(dev)
    sig_d[bad_t, col] ^= 0x01
    torch.cuda.synchronize(dev)
    return (pk_h, sig_h, msg_h, want_h), (pk_d, sig_d, msg_d, bad_t, dev_n - len(bad_d))


def _bulk(sv, torch, dev, hs, ds, phases):
    pk_h, sig_h, msg_h, want_h = hs
    pk_d, sig_d, msg_d, bad_t, n_ok = ds
    t0 = time.perf_counter()
    out = sv.verify_fixed(pk_h, sig_h, msg_h, 32, device=0)
    t1 = time.perf_counter()
    phases["host"] = (t0, t1)
    host_ok = bool(np.array_equal(out, want_h))
    n = pk_d.shape[0]
    verdict = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    t2 = time.perf_counter()
    sv.verify_device(0, pk_d.data_ptr(), sig_d.data_ptr(), msg_d.data_ptr(), n, verdict.data_ptr(), 0, st)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    phases["device"] = (t2, t3)
    dev_ok = (int(verdict.sum(dtype=torch.int64).item()) == n_ok and
              int(verdict[bad_t].sum(dtype=torch.int64).item()) == 0)
    return host_ok, dev_ok


def run_isolation(sv, torch, oracle, host_n=1 << 22, dev_n=1 << 24, seed=3, idle_batches=200):
    dev = torch.device("cuda", 0)
    d = scp_set(oracle, 1000, seed)
    want = d["verdict"]

    def lat_batch():
        return sv.verify_batch(d["pk"], d["sig"], d["msg"], d["msg_off"], d["msg_len"], device=0, path="latency")

    for _ in range(16):  # until the validator keys are cached
        w0 = sv.key_cache_stats(0)["warm_batches"]
        assert np.array_equal(lat_batch(), want)
        if sv.key_cache_stats(0)["warm_batches"] == w0 + 1:
            break
        sv.key_cache_wait(0)
    hs, ds = _bulk_sets(sv, torch, dev, host_n, dev_n, seed)
    res = {"host_batch": host_n, "device_batch": dev_n, "latency_batch": 1000}
    # bulk alone (no latency batch within the shared-mode window)
    time.sleep(1.2)
    alone = {}
    ok_alone = _bulk(sv, torch, dev, hs, ds, alone)
    res["bulk_alone_ms"] = {k: (b - a) * 1e3 for k, (a, b) in alone.items()}
    # latency alone
    idle = []
    for _ in range(idle_batches):
        t = time.perf_counter()
        out = lat_batch()
        idle.append((time.perf_counter() - t) * 1e3)
        assert np.array_equal(out, want)
    res["latency_idle"] = _summary(idle)
    # concurrent
    st0 = sv.key_cache_stats(0)
    stop = threading.Event()
    lats, errors = [], []

    def loop():
        while not stop.is_set():
            t = time.perf_counter()
            out = lat_batch()
            dt = time.perf_counter() - t
            # (the engine's own time for the batch, sv_lat_last_trace: the
            # wall time above also holds this thread's Python and GIL waits)
            lats.append((t, dt * 1e3, sv.lat_last_trace()["total_us"] / 1e3))
            if not np.array_equal(out, want):
                errors.append(int(np.count_nonzero(out != want)))

    th = threading.Thread(target=loop)
    th.start()
    time.sleep(0.05)
    phases = {}
    try:
        ok_loaded = _bulk(sv, torch, dev, hs, ds, phases)
    finally:
        stop.set()
        th.join()
    st1 = sv.key_cache_stats(0)
    res["bulk_loaded_ms"] = {k: (b - a) * 1e3 for k, (a, b) in phases.items()}
    for k, (a, b) in phases.items():
        res["latency_during_" + k] = _summary([dt for t, dt, _ in lats if a <= t < b])
    in_bulk = [(dt, de) for t, dt, de in lats if any(a <= t < b for a, b in phases.values())]
    res["latency_during_bulk"] = _summary([dt for dt, _ in in_bulk])
    res["engine_latency_during_bulk"] = _summary([de for _, de in in_bulk])
    res["warm_batches"] = st1["warm_batches"] - st0["warm_batches"]
    res["cold_batches"] = st1["cold_batches"] - st0["cold_batches"]
    res["shared_launches"] = st1["shared_launches"] - st0["shared_launches"]
    res["latency_verdict_errors"] = len(errors)
    res["bulk_verdicts_ok"] = bool(all(ok_alone) and all(ok_loaded))
    return res
