import json, sys
for f in sys.argv[1:]:
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "host_api %.4e" % r["host_api"]["verifies_per_s"], "warm %.4f cold %.4f" % (
        r["latency_1k"]["p50_ms"], r["latency_1k_cold_keys"]["p50_ms"]),
        "inproc1 %.4e" % r["in_process_multi_gpu"]["per_G"]["1"]["verifies_per_s"], "value %.4e" % r["value"])
