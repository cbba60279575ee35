# Round 5: config 3 (5000-tx set) with the host and staging traces.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r5j}; mkdir -p $OUT
export TMPDIR=/tmp
SV_HOST_TRACE=1 SV_STAGE_TRACE=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $OUT/config3.json 2> $OUT/config3_trace.err || exit $?
