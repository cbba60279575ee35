#!/bin/bash
# per-variant PMC pass: cycles and VALU instruction counts of the verify kernels
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/$v -o pmc -- python3 $R/tools/ab_variants.py $R/variants/libsv_$v.so > $O/$v.log 2>&1
done
