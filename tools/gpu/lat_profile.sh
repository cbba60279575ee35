# Latency-path probe + rocprofv3 kernel trace (usage: bash tools/gpu/lat_profile.sh OUTDIR)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-lat1}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/lat_probe.py --sizes 1000,2048,4096,8192 --iters 50 --out $OUT/probe.json > $OUT/probe.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lat -- python tools/lat_probe.py --sizes 1000 --iters 50 > $OUT/prof.txt 2>&1
echo "rocprof rc=$?"
