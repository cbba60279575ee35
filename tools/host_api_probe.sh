set -e
mkdir -p gpurun_out
P="timeout -k 10 120 python -u tools/host_api_probe.py"
SV_STAGE_RAMP=0 $P > gpurun_out/probe_r0.json 2>/dev/null
SV_STAGE_RAMP=1 $P > gpurun_out/probe_r1.json 2>/dev/null
SV_STAGE_RAMP=1 SV_STAGE_CHUNK=131072 $P > gpurun_out/probe_r1c17.json 2>/dev/null
SV_STAGE_RAMP=1 SV_HOST_THREADS=15 $P > gpurun_out/probe_r1t15.json 2>/dev/null
