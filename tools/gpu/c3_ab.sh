# Config 3 (5000-tx set pre-pass) with the latency lane's input staged
# (SV_LAT_ZC_IN=0) vs read in place (default), alternating, one process each.
# Usage: bash tools/gpu/c3_ab.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c3_ab}; mkdir -p $OUT
export TMPDIR=/tmp
C3='import sys,json; sys.path.insert(0,"tools"); import bench_configs as bc; r=bc.config3(bc.Env(),5000); print(json.dumps({k: r[k] for k in ("gpu_prepass_checker_s","gpu_prepass_checker_max_s","gpu_prepass_same_set_repeat_min_s","gpu_prepass_checker_first_call_s")}))'
for r in 1 2 3; do
  for m in 0 1; do
    SV_LAT_ZC_IN=$m timeout -k 10 120 python -u -c "$C3" > $OUT/c3_m${m}_r${r}.json 2> $OUT/c3_m${m}_r${r}.err || exit $?
  done
done
