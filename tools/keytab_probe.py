"""Per-key tables of the throughput path: what they buy (developer tool).

Device-API batches of 2^20 signatures with the tables off and on:
  * checkpoint shape: 65,536 keys x 16 signatures (tests/test_gpu_engine.py
    checkpoint prefetch; LedgerManagerImpl.cpp:1546-1609 replays a checkpoint's
    transactions, ~16 per account);
  * validator set: 100 keys x 10,486 signatures (config 4's key set at bulk size);
  * distinct keys (the headline's shape): the tables' overhead.
For each: kernel ms per launch (HIP events, sv_timing_enable), on = first call
(keys claimed and built) and steady state (every key built before).

    python tools/keytab_probe.py [--out file.json]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    sv = importlib.import_module("stellar-core_amd")
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    n = 1 << 20

    def dataset(keys, seed):
        rng = np.random.default_rng(seed)
        kseeds = rng.integers(0, 256, (keys, 32), dtype=np.uint8)
        seeds = torch.from_numpy(np.resize(kseeds, (n, 32))).to(dev)
        msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).to(dev)
        pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        sv.sign_device(0, seeds.data_ptr(), msgs.data_ptr(), n, pk.data_ptr(), sig.data_ptr(), st)
        torch.cuda.synchronize(dev)
        return pk, sig, msgs

    def timed(pk, sig, msgs, reps):
        out = torch.zeros(n, dtype=torch.uint8, device=dev)
        sv.kernel_time_reset()
        sv.timing_enable(True)
        for _ in range(reps):
            sv.verify_device(0, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), n, out.data_ptr(), 0, st)
        torch.cuda.synchronize(dev)
        sv.timing_enable(False)
        ms, la, _ = sv.kernel_time(0)
        assert int(out.sum().item()) == n, "every row is valid"
        return ms / max(1, la)

    rows = []
    prev = sv.set_key_tables(0)
    for name, keys in (("checkpoint_65536_keys", 65536), ("validators_100_keys", 100), ("distinct_keys", n)):
        pk, sig, msgs = dataset(keys, seed=keys)
        sv.set_key_tables(0)
        timed(pk, sig, msgs, 1)
        off = timed(pk, sig, msgs, args.reps)
        sv.set_key_tables(1, 1 << 21)  # (fresh tables: 2^21 slots hold 2^20 distinct keys)
        first = timed(pk, sig, msgs, 1)
        steady = timed(pk, sig, msgs, args.reps)
        st_ = sv.key_cache_stats(0)
        sv.set_key_tables(1, 1 << 19)
        r = {"set": name, "keys": keys, "signatures": n, "ms_tables_off": off, "ms_tables_on_first_call": first,
             "ms_tables_on_steady": steady, "speedup_steady": off / steady, "speedup_first": off / first,
             "table_keys": st_["table_keys"]}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del pk, sig, msgs
    sv.set_key_tables(prev)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
