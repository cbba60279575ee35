# Round-4 first GPU pass: the new parity tests, then the traffic diagnostic.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4a; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_longmsg.py tests/test_gpu_engine.py -k "longmsg or long or mib or staging or remap" -x -v --timeout 240 --timeout-method thread > $OUT/pytest_new.txt 2>&1 || exit $?
bash tools/gpu/traffic_ab.sh r4a/traffic_ab
