# Phase timeline of the cold-key octet kernel (tools/comb_phases.py --octet)
# and of the warm comb kernel.  Usage: bash tools/gpu/octet_phases.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-ophases}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/comb_phases.py --octet variants/libsv_diag_ophases.so > $OUT/octet_phases.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/comb_phases.py variants/libsv_diag_phases.so > $OUT/comb_phases.txt 2>&1 || exit $?
