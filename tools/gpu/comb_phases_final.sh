# Comb / octet phase timelines of the final latency kernels.
# Usage: bash tools/gpu/comb_phases_final.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-comb_phases_final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/comb_phases.py variants/libsv_diag_phases.so > $OUT/phases.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py --octet variants/libsv_diag_ophases.so > $OUT/ophases.txt 2>&1 || exit $?
