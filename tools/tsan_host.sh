#!/bin/bash
# Developer tool (CPU only): builds the C++ mirror (libstellar_host) with
# ThreadSanitizer into /tmp/tsan and runs the helper-pool stress of
# tests/test_host_mirror.py (300 host-hashed batches fanned out over
# sv::Pool) under it.  Prints the number of TSan warnings (expected 0).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=/tmp/tsan
mkdir -p $O
cd "$R/stellar-core_amd"
for f in hashes PubKeyUtils SignatureChecker VerifyMicroBatcher TransactionSignatures host_capi; do
  g++ -O1 -g -std=c++17 -fPIC -fsanitize=thread -c csrc/host/$f.cpp -o $O/$f.o
done
g++ -shared -fsanitize=thread -o $O/libstellar_host.so $O/*.o -L. -lstellar_sigverify \
    -Wl,-rpath,"$R/stellar-core_amd" -Wl,-rpath,/opt/rocm/lib -lpthread
python3 - "$R" > $O/stress.py <<'PY'
import re, sys
src = open(sys.argv[1] + "/tests/test_host_mirror.py").read()
print(re.search(r'_POOL_STRESS = r"""(.*?)"""', src, re.S).group(1).replace("range(8000)", "range(300)"))
PY
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" LD_PRELOAD=$(gcc -print-file-name=libtsan.so) \
    python3 $O/stress.py $O/libstellar_host.so "$R/tests/native/libhostcore.so" > $O/out.txt 2>&1 || true
echo "TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O/out.txt || true); stress: $(tail -1 $O/out.txt)"
