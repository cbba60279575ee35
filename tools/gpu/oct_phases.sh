# Phase timeline of the cold-key octet kernel only (tools/comb_phases.py --octet).
# Usage: bash tools/gpu/oct_phases.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-oph}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/comb_phases.py --octet variants/libsv_diag_ophases.so > $OUT/octet_phases.txt 2>&1 || exit $?
