import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        print(d.get("memo_keyed"), {k: (v["verdict_p50_ms"], v["main_p50_ms"], v["ready_p50_ms"], round(v["main_thread_verifysig_per_s"] or 0))
                                     for k, v in d.items() if isinstance(v, dict) and k in ("paced_1k_every_5ms", "flood", "trickle_4_every_200us")})
