# Evidence passes on the GPU box, one script for every round (the one-off
# per-experiment scripts of rounds 4-5 are in git history).
#   bash tools/gpu/round.sh MODE OUTDIR
# MODE
#   final  parity suite, smoke, bench N=1 and the 2-rank rehearsal of the N>1
#          line on one card: the round's authoritative set (DESIGN.md 3.6
#          names the copy under profiles/rNN/final/)
#   prof   rocprofv3 kernel trace + one PMC pass per counter group of the bench
#          kernels (tools/profile_run.sh), then the mad count when its
#          measurement build exists (tools/build_variants.sh madcount -DSV_MADCOUNT)
#   feed   host-feed probe at G = 1, 2, 4, 8 slots mapped onto this card, and
#          the bench's in-process multi-GPU leg over the same 8 slots
#   txset  config-3 host phases over distinct sets (tools/txset_host_probe.py)
#   sweep  host-call size sweep of the medium sizes (tools/size_sweep.py)
#   ab     kernel A/B of variants/libsv_*.so built by tools/build_variants.sh
#          (tools/ab_variants.py, interleaved rounds)
# Other scripts here: ab.sh (A/B then the suite), host_round.sh (integration
# layer: config-3 trace, host bench, the mirror's GPU tests), api_probe.hip
# and cumask_probe.hip (HIP API / CU-mask probes).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
MODE=${1:?mode}
OUT=gpurun_out/${2:-$MODE}; mkdir -p $OUT
export TMPDIR=/tmp
DEVMAP8=0,0,0,0,0,0,0,0
case $MODE in
final)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || exit $?
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit $?
  SECONDS=0; timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
  echo "bench wall $SECONDS s" > $OUT/bench_wall.txt
  SV_BENCH_SHARE_GPUS=1 timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 2 \
      > $OUT/bench_n2.json 2> $OUT/bench_n2.err || exit $?
  ;;
prof)
  bash tools/profile_run.sh $OUT/prof || exit $?
  if [ -f variants/libsv_madcount.so ]; then
    timeout -k 10 300 python -u tools/madcount.py --out $OUT/madcount.json > $OUT/madcount.txt 2>&1 || exit $?
  fi
  ;;
feed)
  SV_DEVICE_MAP=$DEVMAP8 timeout -k 10 300 python -u tools/feed_probe.py > $OUT/feed_devmap8.json 2> $OUT/feed_devmap8.err || exit $?
  SV_DEVICE_MAP=$DEVMAP8 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-latency --no-cpu \
      --no-config35 --no-config4i > $OUT/bench_devmap8.json 2> $OUT/bench_devmap8.err || exit $?
  ;;
txset)
  for r in 1 2 3; do
    TXSET_PROBE_DISTINCT=1 timeout -k 5 200 python -u tools/txset_host_probe.py 5000 6 1 >> $OUT/txset.txt 2>&1 || exit $?
  done
  ;;
sweep)
  SWEEP_PATHS=auto timeout -k 10 400 python -u tools/size_sweep.py 15 "16384,29217,50000,100000,131072,200000" \
      > $OUT/sweep.json 2> $OUT/sweep.err || exit $?
  ;;
ab)
  AB_ROUNDS=${AB_ROUNDS:-8} timeout -k 10 500 python -u tools/ab_variants.py variants/libsv_*.so > $OUT/ab.txt 2>&1 || exit $?
  ;;
*)
  echo "unknown mode $MODE" >&2; exit 2 ;;
esac
echo done
