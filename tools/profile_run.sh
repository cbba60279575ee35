#!/bin/bash
# rocprofv3 evidence for the bench kernel (run on the GPU box):
#   kernel trace + stats, then one --pmc pass per counter group (never combined
#   with sys/runtime tracing), then tools/prof_summary.py over the directory.
# Usage: tools/profile_run.sh OUTDIR [batch]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$(realpath -m "${1:-$R/gpurun_out/prof}")
N=${2:-1048576}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 6 --warmup 1 --no-cpu --no-latency --no-host-api --no-config1 --no-config35 --batch $N"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d "$O/kt" -o kt -- python3 $B > "$O/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --output-format csv --pmc FETCH_SIZE -d "$O/fetch" -o fetch -- python3 $B > "$O/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --output-format csv --pmc WRITE_SIZE -d "$O/write" -o write -- python3 $B > "$O/write.log" 2>&1
timeout -k 10 300 rocprofv3 --output-format csv --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVES -d "$O/sq1" -o sq1 -- python3 $B > "$O/sq1.log" 2>&1
timeout -k 10 300 rocprofv3 --output-format csv --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d "$O/sq2" -o sq2 -- python3 $B > "$O/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d "$O/sq3" -o sq3 -- python3 $B > "$O/sq3.log" 2>&1
python3 "$R/tools/prof_summary.py" "$O" --batch $N > "$O/summary.json"
cat "$O/summary.json"
