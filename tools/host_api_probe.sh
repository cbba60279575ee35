set -e
# staging ramp depth and chunk size vs the host-API rate at 2^20 (developer tool)
mkdir -p gpurun_out/ramp
P="timeout -k 10 120 python -u tools/host_api_probe.py"
for r in 0 2 3 4 5; do SV_STAGE_RAMP=$r $P > gpurun_out/ramp/r$r.json 2>/dev/null; done
SV_STAGE_RAMP=4 SV_STAGE_CHUNK=131072 $P > gpurun_out/ramp/r4c17.json 2>/dev/null
SV_STAGE_RAMP=2 $P > gpurun_out/ramp/r2b.json 2>/dev/null
