"""Latency-class isolation (VERDICT r2 "next" 3): 1k SCP batches submitted
back to back while a 2^22-signature host batch and a 2^24-signature device
batch run on the same GPU (tests/isolation_load.py).  Every verdict exact;
bulk launches made while latency batches are live run in shared mode (a
workgroup slot per CU left free, csrc/sv_kernels.hip sv_launch_verify) and the
latency lane has its own high-priority stream, staging and mutex
(csrc/sv_api.cpp LatLane).  The 1k batches' p99 under load is recorded
(SV_ISOLATION_OUT, profiles/) and held to a loose bound, 1 ms by default
(SV_ISOLATION_P99_MS=x overrides): the round-4 runs measured 0.21-0.23 ms; a
lane copy queued behind bulk uploads again (0.6-0.86 ms before round 4) comes
close to it, the multi-ms stalls of an unisolated lane do not pass."""
import json
import os

import pytest

from isolation_load import run_isolation

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_latency_batches_under_bulk_load(sv, oracle):
    if sv.device_count() < 1:
        pytest.skip("no GPU")
    res = run_isolation(sv, torch, oracle)
    print(json.dumps(res))
    out = os.environ.get("SV_ISOLATION_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    assert res["latency_verdict_errors"] == 0
    assert res["bulk_verdicts_ok"]
    assert res["shared_launches"] > 0
    during = res["latency_during_bulk"]
    assert during["batches"] >= 100, res
    bound = float(os.environ.get("SV_ISOLATION_P99_MS", "1.0"))
    assert during["p99_ms"] <= bound, res
