set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ic
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_WAIT_ANY\|SQC_TC_INST[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt || true
cat $O/names.txt
B="$R/bench.py --steps 3 --warmup 1 --no-cpu --no-latency"
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY -d $O/p1 -o p1 -- python3 $B > $O/p1.log 2>&1
if grep -q "^SQC_ICACHE_MISSES$" $O/names.txt; then
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $O/p2 -o p2 -- python3 $B > $O/p2.log 2>&1
fi
