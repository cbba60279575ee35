#!/usr/bin/env python3
"""Developer tool: config-3 A/B of svh_check_txset pre-pass modes on the GPU.

Builds DISTINCT 5000-tx sets once (tests/txset_gen.py, GPU-signed like
bench.py's config 3), then in interleaved rounds runs every set once under
each mode (1: one engine batch; 4: two halves, pipelined) and prints one JSON
line per round: per-mode median / max ms over the sets, the phase split, and
whether every outcome equals mode 1's.  Usage:
  python tools/txset_mode_ab.py [ROUNDS] [SETS] [MODES]   (defaults 4, 6, "1,4")
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench_configs as bc  # noqa: E402
import txset_gen as tg  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    sets = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    modes = [int(m) for m in (sys.argv[3] if len(sys.argv) > 3 else "1,4").split(",")]
    env = bc.Env()
    n_tx = 5000

    def gpu_sign_fn(reqs):
        seeds = np.frombuffer(b"".join(r[0] for r in reqs), np.uint8).reshape(-1, 32)
        msgs = np.frombuffer(b"".join(r[1] for r in reqs), np.uint8).reshape(-1, 32)
        tpk, tsig, _ = env.gpu_sign(seeds, msgs)
        pk, sg = tpk.cpu().numpy(), tsig.cpu().numpy()
        return [(pk[i].tobytes(), sg[i].tobytes()) for i in range(len(reqs))]

    built = [tg.to_ctypes(tg.generate(n_tx, gpu_sign_fn, seed=9000 + k)) for k in range(sets + 1)]

    def run(cts, mode):
        T, S, G = cts
        ok = np.zeros(n_tx, np.uint8)
        used = np.zeros(n_tx, np.uint8)
        env.host.svh_cache_clear()
        t1 = time.perf_counter()
        rc = env.host.svh_check_txset(T, ctypes.c_size_t(n_tx), S, G, mode, ok.ctypes.data_as(ctypes.c_void_p),
                                      used.ctypes.data_as(ctypes.c_void_p), None)
        dt = (time.perf_counter() - t1) * 1e3
        assert rc == 0, env.host.svh_last_error_string()
        ph = (ctypes.c_double * 4)()
        env.host.svh_txset_last_phases(ph)
        return dt, list(ph), ok, used

    for m in modes:  # warm-up: pools, staging, workspaces
        run(built[0], m)
    want = [run(b, 1)[2:] for b in built[1:]]
    for r in range(rounds):
        line = {"round": r}
        for m in (modes if r % 2 == 0 else modes[::-1]):
            res = [run(b, m) for b in built[1:]]
            same = all((x[2] == w[0]).all() and (x[3] == w[1]).all() for x, w in zip(res, want))
            dts = [x[0] for x in res]
            line["mode%d" % m] = {"median_ms": float(np.median(dts)), "max_ms": float(max(dts)),
                                  "phases_median_ms": [round(float(np.median([x[1][j] for x in res])), 3)
                                                       for j in range(4)],
                                  "outcomes_equal_mode1": bool(same)}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
