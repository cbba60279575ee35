# Per-key tables: GPU tests, speed probe, headline A/B against the previous build
# usage: bash tools/gpu/keytab.sh OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-kt1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_keytables.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python -u tools/keytab_probe.py --out $OUT/keytab_probe.json > $OUT/keytab_probe.txt 2>&1 || exit $?
AB_ROUNDS=5 timeout -k 10 300 python -u tools/ab_variants.py variants/libsv_a_base.so variants/libsv_b_kt.so > $OUT/ab.txt 2>&1
