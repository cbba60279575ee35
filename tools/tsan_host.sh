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
# clang's ThreadSanitizer (ROCm's LLVM): GCC 11's libtsan has no
# pthread_cond_clockwait interceptor, which libstdc++'s condition_variable::
# wait_for uses, so it loses track of the mutex a timed wait releases and
# reports the next lock of it as a double lock (false positives in the
# micro-batcher's deadline waits, seen on round-3 and round-4 sources alike)
CXX=/opt/rocm/lib/llvm/bin/clang++
TSAN_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.tsan-x86_64.so | head -1)
for f in hashes PubKeyUtils SignatureChecker VerifyMicroBatcher TransactionSignatures host_capi; do
  $CXX -O1 -g -std=c++17 -fPIC -fsanitize=thread -c csrc/host/$f.cpp -o $O/$f.o
done
$CXX -shared -fsanitize=thread -shared-libsan -o $O/libstellar_host.so $O/*.o -L. -lstellar_sigverify \
    -Wl,-rpath,"$R/stellar-core_amd" -Wl,-rpath,/opt/rocm/lib -lpthread
python3 - "$R" > $O/stress.py <<'PY'
import re, sys
src = open(sys.argv[1] + "/tests/test_host_mirror.py").read()
print(re.search(r'_POOL_STRESS = r"""(.*?)"""', src, re.S).group(1).replace("range(8000)", "range(300)"))
PY
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" LD_PRELOAD=$TSAN_RT \
    python3 $O/stress.py $O/libstellar_host.so "$R/tests/native/libhostcore.so" > $O/out.txt 2>&1 || true
echo "pool stress: TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O/out.txt || true); result: $(tail -1 $O/out.txt)"
# the micro-batcher (VerifyMicroBatcher: producer shards, flush workers,
# futures and fire-and-forget posts) under a native 8-producer flood
cat > $O/mb.py <<'PY'
import ctypes, sys
import numpy as np
host = ctypes.CDLL(sys.argv[1]); stub = ctypes.CDLL(sys.argv[2])
host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
host.svh_set_test_verifier(ctypes.cast(stub.hc_stub_verify, ctypes.c_void_p))
n = 20000
rng = np.random.default_rng(2)
pk = rng.integers(0, 256, (n, 32), dtype=np.uint8); sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
msg = rng.integers(0, 256, 32 * n, dtype=np.uint8)
off = np.arange(n, dtype=np.uint64) * 32; ln = np.full(n, 32, np.uint32); out = np.zeros(n, np.uint8)
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
for ff in (0, 1):
    host.svh_cache_clear()
    rc = host.svh_mb_run_ex(P(pk), P(sig), P(msg), P(off), P(ln), ctypes.c_size_t(n), 8, 3, ctypes.c_uint32(512),
                            ctypes.c_uint32(200), ctypes.c_uint32(0), ff, P(out), None)
    assert rc == 0, rc
    assert ff or out.all()
print("ok")
PY
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" LD_PRELOAD=$TSAN_RT \
    python3 $O/mb.py $O/libstellar_host.so "$R/tests/native/libhostcore.so" > $O/out_mb.txt 2>&1 || true
echo "micro-batcher flood: TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O/out_mb.txt || true); result: $(tail -1 $O/out_mb.txt)"
# the SCP harness (svh_scp_run: 4 producers, 2 flush workers, the main
# thread) with per-envelope continuations and with the batch continuation
# (submitTagged + onBatch, round 6), on the native stub engine
cat > $O/scp.py <<'PY'
import ctypes, sys
import numpy as np
host = ctypes.CDLL(sys.argv[1]); stub = ctypes.CDLL(sys.argv[2])
host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
host.svh_set_test_verifier(ctypes.cast(stub.hc_stub_verify, ctypes.c_void_p))
class Prm(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint32) for k in ("struct_size", "producers", "burst", "interval_us", "max_batch",
                "max_delay_us", "workers", "policy", "linger_us", "idle_in_flight", "quiet_us", "max_linger_us",
                "batch_post")]
n = 20000
rng = np.random.default_rng(5)
pk = rng.integers(0, 256, (n, 32), dtype=np.uint8); sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
msg = rng.integers(0, 256, 32 * n, dtype=np.uint8)
off = np.arange(n, dtype=np.uint64) * 32; ln = np.full(n, 32, np.uint32); out = np.zeros(n, np.uint8)
res = (ctypes.c_char * 4096)()
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
for bp in (0, 1):
    host.svh_cache_clear()
    p = Prm(ctypes.sizeof(Prm), 4, 500, 2000, 8192, 2000, 2, 0, 0, 1, 0, 200, bp)
    rc = host.svh_scp_run(P(pk), P(sig), P(msg), P(off), P(ln), ctypes.c_size_t(n), ctypes.byref(p), P(out), res)
    assert rc == 0 and out.all(), (rc, bp)
print("ok")
PY
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" LD_PRELOAD=$TSAN_RT \
    python3 $O/scp.py $O/libstellar_host.so "$R/tests/native/libhostcore.so" > $O/out_scp.txt 2>&1 || true
echo "SCP harness, per-envelope and batched posts: TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O/out_scp.txt || true); result: $(tail -1 $O/out_scp.txt)"
# the tx-set pre-pass (round 3): parallel marshal, SignatureBatchPrefetch::addBatch parts and
# checkers on the pool, with the native stub engine; and the large keyed walk (threaded walk,
# pre-drawn evictions, inline resolve) with the native keyed stub
cat > $O/txset.py <<'PY'
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[3], "tests"))
import txset_gen as tg
host = ctypes.CDLL(sys.argv[1]); stub = ctypes.CDLL(sys.argv[2])
host.svh_set_test_verifier.argtypes = [ctypes.c_void_p]
host.svh_set_test_keyed_verifier.argtypes = [ctypes.c_void_p]
host.svh_set_keyed_threshold.argtypes = [ctypes.c_size_t]
rng = np.random.default_rng(3)
def sign(reqs):  # random keys and signatures: the stub engine accepts all
    return [(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 64, dtype=np.uint8).tobytes())
            for _ in reqs]
txs = tg.generate(2000, sign, seed=7)
T, S, G = tg.to_ctypes(txs)
host.svh_set_test_verifier(ctypes.cast(stub.hc_stub_verify, ctypes.c_void_p))
ok = np.zeros(len(txs), np.uint8); used = np.zeros(len(txs), np.uint8)
for pf in (1, 3, 4, 1):
    rc = host.svh_check_txset(T, ctypes.c_size_t(len(txs)), S, G, pf, ok.ctypes.data_as(ctypes.c_void_p),
                              used.ctypes.data_as(ctypes.c_void_p), None)
    assert rc == 0, rc
host.svh_set_test_verifier(None)
host.svh_set_test_keyed_verifier(ctypes.cast(stub.hc_stub_keyed, ctypes.c_void_p))
host.svh_set_keyed_threshold(1)
n = 40000
pk = rng.integers(0, 256, (n, 32), dtype=np.uint8); sig = rng.integers(0, 256, (n, 64), dtype=np.uint8)
msg = rng.integers(0, 256, 32 * n, dtype=np.uint8)
off = np.arange(n, dtype=np.uint64) * 32; ln = np.full(n, 32, np.uint32); out = np.zeros(n, np.uint8)
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
for _ in range(3):
    rc = host.svh_verify_sig_batch(P(pk), P(sig), None, P(msg), P(off), P(ln), ctypes.c_size_t(n), P(out))
    assert rc == 0, rc
print("ok")
PY
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" LD_PRELOAD=$TSAN_RT \
    python3 $O/txset.py $O/libstellar_host.so "$R/tests/native/libhostcore.so" "$R" > $O/out_txset.txt 2>&1 || true
echo "tx-set pre-pass + keyed walk: TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O/out_txset.txt || true); result: $(tail -1 $O/out_txset.txt)"
# the C-ABI's slot-table lifetime (sv_shutdown / sv_set_device_map against
# in-flight calls on stub slots): sv_api.cpp instrumented, the kernel objects
# as built
O2=/tmp/tsan_life
mkdir -p $O2
R2=$R/stellar-core_amd
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -Xarch_host -fsanitize=thread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    -c $R2/csrc/sv_api.cpp -o $O2/sv_api_tsan.o
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -Xarch_host -fsanitize=thread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    -c $R/tools/tsan_lifetime.cpp -o $O2/tsan_lifetime.o
/opt/rocm/bin/hipcc -Xarch_host -fsanitize=thread --offload-arch=gfx950 -o $O2/tsan_lifetime $O2/tsan_lifetime.o $O2/sv_api_tsan.o \
    $R2/build/sv_kernels.o $R2/build/sv_comb.o $R2/build/sv_hash.o $R2/build/sv_cpu.o -Wl,-rpath,/opt/rocm/lib -lpthread
TSAN_OPTIONS="report_signal_unsafe=0 halt_on_error=0" $O2/tsan_lifetime > $O2/out_life.txt 2>&1 || true
echo "slot lifetime (4 callers vs remap/shutdown): TSan warnings: $(grep -c 'WARNING: ThreadSanitizer' $O2/out_life.txt || true); result: $(tail -1 $O2/out_life.txt)"
