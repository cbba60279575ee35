# Instruction-fetch stalls of the warm-key comb kernel: SQ wait / ifetch
# counters and SQC instruction-cache hits / misses, separate --pmc passes over
# 100 warm 1k batches (tools/ab_lat_capi.py, product library).
# Usage: bash tools/gpu/comb_icache.sh OUTDIR
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-comb_ic}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export AB_MODES=warm AB_ROUNDS=1 AB_ITERS=100
P="$R/tools/ab_lat_capi.py $R/variants/libsv_prod.so"
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES -d $O/p1 -o p1 -- python3 $P > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $O/p2 -o p2 -- python3 $P > $O/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $P > $O/kt.log 2>&1 || exit $?
