# config-3 phase trace (SV_HOST_TRACE) on the GPU box (usage: bash tools/gpu/c3trace.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c3}; mkdir -p $OUT
export TMPDIR=/tmp
SV_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_configs.py --configs 3 > $OUT/c3.json 2> $OUT/c3.err
