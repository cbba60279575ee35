// C-ABI implementation (include/stellar_sigverify.h): device slots, lazily
// created per-slot resources, pipelined host<->device staging and multi-GPU
// sharding.
//
// Replaces, for whole batches, the libsodium crypto_sign_verify_detached call
// made by stellar::PubKeyUtils::verifySig on a verify-cache miss
// (/root/reference/src/crypto/SecretKey.cpp:461-463).
//
// Device slots.  One slot per visible GPU by default; sv_set_device_map (or
// the SV_DEVICE_MAP environment variable, e.g. "0,0") maps several logical
// slots onto one physical GPU, which is how the multi-device code is tested
// on a one-GPU box.  Per slot: three HIP streams (H2D copies, kernels, D2H
// copies), the base-point tables (computed on the device at first use), and a
// workspace allocated on the first throughput-path launch and sized to the
// batch (the latency kernel needs none).  All work of a slot is serialised
// under its mutex because the workspace is shared by every launch on it.
//
// Host buffers.  A host-buffer batch is cut into staging chunks (2^18
// signatures by default; the first two are a quarter and a half chunk so the
// first kernel starts early); chunk c is packed into pinned slot c % 2 by the
// helper pool, copied up on the H2D stream, verified on the kernel stream,
// and its verdicts copied down on the D2H stream, so the packing and PCIe
// copies of one chunk overlap the kernels of the previous one and a batch of
// any size pins at most two chunks.  Measured at 2^20 on MI355X: 91 % of the
// device-API rate with the ramp, 84 % without (tools/host_api_probe.py).
//
// Multi-GPU: contiguous slices [g*n/G, (g+1)*n/G) over G slots, G limited so
// that every slice holds at least the minimum shard (2^16 signatures by
// default: a 1k SCP batch stays on one GPU), driven by the persistent helper
// pool; verdicts land in disjoint ranges of the caller's buffer -- no
// collective.
#include <emmintrin.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/stellar_sigverify.h"
#include "comb.h"
#include "keycache.h"
#include "keytab.h"
#include "pool.h"

extern "C" {
size_t sv_ws_bytes(unsigned grid, uint64_t cap);
size_t sv_verify_ws_bytes(int path, unsigned grid, uint64_t n);
size_t sv_btab_bytes(void);
int sv_block_threads(void);
hipError_t sv_launch_btab_init(uint32_t* d_btab, hipStream_t s);
int sv_occupancy_blocks_per_cu(void);
hipError_t sv_launch_verify(int mode, int path, unsigned grid, const void* pk, const void* sig, const void* msg,
                            const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                            void* verdict, void* bitmap, void* ws, const void* btab, uint32_t dbg, int share,
                            const sv_ktparams* kt, uint32_t* status, hipStream_t s);
int sv_share_blocks_per_cu(void);
size_t sv_key_table_entry_bytes(void);
uint64_t sv_plan_chunk_max(uint64_t n);
hipError_t sv_launch_sign(unsigned grid, const void* seed, const void* msg, uint64_t n, void* pk, void* sig,
                          void* ws, const void* btab, hipStream_t s);
hipError_t sv_launch_hash(int kind, unsigned max_blocks, const void* pk, const void* sig, const void* msg,
                          const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n, void* out,
                          hipStream_t s);
// warm-key latency path (sv_comb.hip)
size_t sv_comb_btab_bytes(void);
size_t sv_key_slot_bytes(void);
hipError_t sv_launch_comb_btab(uint32_t* d_ctab, hipStream_t s);
hipError_t sv_launch_keytab(const void* d_pks, const uint32_t* d_slots, uint32_t nkeys, uint32_t* d_ktab,
                            uint32_t* d_kstat, hipStream_t s);
int sv_comb_spw(uint64_t n, int cus);
hipError_t sv_launch_comb(int mode, int spw, const void* pk, const void* sig, const void* msg, const uint64_t* off,
                          const uint32_t* len, uint32_t fixed_len, uint64_t n, void* verdict, const uint32_t* kslot,
                          const uint32_t* ktab, const uint32_t* kstat, const uint32_t* ctab, hipStream_t s);
}

namespace {

thread_local std::string t_err;
bool test_knobs_enabled();

int fail(int code, const std::string& msg) {
  t_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(SV_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define SV_HIP(call)                                   \
  do {                                                 \
    hipError_t _e = (call);                            \
    if (_e != hipSuccess) return hip_fail(_e, #call);  \
  } while (0)

size_t env_size(const char* name, size_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  char* end = nullptr;
  const unsigned long long x = strtoull(v, &end, 0);
  return (end && *end == 0) ? (size_t)x : dflt;
}

sv::Pool& pool() {
  // The GPU box's share is 16 CPUs; the staging copies saturate well below.
  static sv::Pool p((unsigned)std::min<size_t>(
      env_size("SV_HOST_THREADS", std::min(8u, std::max(2u, std::thread::hardware_concurrency()))), 64));
  return p;
}
// The pool a pack runs on: a device slot's own workers inside a multi-slot
// call (shard), else the shared pool.
thread_local sv::Pool* t_pack_pool = nullptr;
thread_local size_t t_pack_parts = 0;  // (multi-slot calls: this slot's share of the CPUs; 0: no cap)
sv::Pool& pack_pool() { return t_pack_pool ? *t_pack_pool : pool(); }

// CPUs this process may use at once: its affinity mask, limited by a cgroup
// v2 CPU quota (the GPU box grants 16 of a 256-CPU host by quota).
size_t usable_cpus() {
  cpu_set_t set;
  size_t aff = std::max(1u, std::thread::hardware_concurrency());
  if (sched_getaffinity(0, sizeof(set), &set) == 0) aff = (size_t)std::max(1, CPU_COUNT(&set));
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    unsigned long long per = 0;
    if (fscanf(f, "%31s %llu", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
      const size_t quota = (size_t)(strtoull(q, nullptr, 10) / per);
      if (quota >= 1) aff = std::min(aff, quota);
    }
    fclose(f);
  }
  return aff;
}

// NUMA node of a GPU (-1: unknown) from its PCI address, and that node's CPUs
// this process may run on (empty: no placement).
int gpu_numa_node(int phys) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), phys) != hipSuccess) return -1;
  for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
  int node = -1;
  if (FILE* f = fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r")) {
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
  }
  return node;
}
std::vector<int> node_cpus(int node) {
  std::vector<int> out;
  if (node < 0) return out;
  cpu_set_t mine;
  if (sched_getaffinity(0, sizeof(mine), &mine) != 0) return out;
  FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
  if (!f) return out;
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[got] = 0;
  // "0-23,96-119"
  for (char* p = buf; *p;) {
    char* e = nullptr;
    const long a = strtol(p, &e, 10);
    if (e == p) break;
    long b = a;
    if (*e == '-') {
      p = e + 1;
      b = strtol(p, &e, 10);
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET((int)c, &mine)) out.push_back((int)c);
    p = e;
    while (*p == ',' || *p == '\n' || *p == ' ') ++p;
  }
  return out;
}
// NUMA node of the page holding p (-1: unknown): get_mempolicy(MPOL_F_NODE |
// MPOL_F_ADDR) by its syscall (no libnuma in the image).
int page_numa_node(const void* p) {
  if (!p) return -1;
  int node = -1;
  const long r = syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL /* MPOL_F_NODE | MPOL_F_ADDR */);
  return r == 0 ? node : -1;
}

// ------------------------------------------------------------ buffers
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return SV_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes, 1 << 16);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return fail(SV_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    cap = want;
    return SV_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host staging (hipHostMalloc).  `mapped` buffers are fine-grained
// (coherent) and read / written by kernels in place: `dp` is their device
// address.
struct HostBuf {
  void* p = nullptr;
  void* dp = nullptr;
  size_t cap = 0;
  bool mapped = false;
  int ensure(size_t bytes) {
    if (bytes <= cap) return SV_OK;
    release();
    const size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 16);
    hipError_t e =
        hipHostMalloc(&p, want, mapped ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault);
    if (e == hipSuccess && mapped) e = hipHostGetDevicePointer(&dp, p, 0);
    if (e != hipSuccess) {
      release();
      return fail(SV_ERR_ALLOC, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    cap = want;
    return SV_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    cap = 0;
  }
};

// One pinned + device staging slot of the host-buffer pipeline.
struct Stage {
  HostBuf h_in, h_out;
  DevBuf d_in, d_verdict, d_keys;
  hipEvent_t up = nullptr, done = nullptr, down = nullptr, keys_down = nullptr;
  std::vector<hipEvent_t> pev;  // keys of piece k are down (one-chunk keyed batches)
  bool busy = false;  // a chunk's D2H is pending on `down`
  size_t lo = 0, m = 0;
  const uint8_t* zv = nullptr;  // the chunk's verdicts in mapped memory (written in place), else in h_out
};

// Latency lane of a slot.  Batches that take the latency kernels (one staging
// chunk, SV_PATH_LATENCY) run here on their own high-priority stream, pinned
// staging and mutex, so an SCP batch never waits on the host side for the
// slot's bulk work (a tx set or a catchup batch holding Device::mu).  The lane
// also owns the key cache of the warm-key kernel (keycache.h, comb.h): a batch
// whose keys are all cached runs sv_comb_kernel, any other batch the octet
// kernel, after which its new keys are queued for a table build on the
// low-priority build stream.
// One latency batch in flight on the lane: its staging and streams.  The
// lane's mutex covers a batch's planning and launch; its wait and copy-out
// run outside it, so with two contexts the next batch (an SCP burst's second
// micro-batch) is planned and launched while the first one runs, instead of
// queueing behind it on the host (SV_LAT_CONTEXTS, default 2; 1 serialises).
struct LatCtx {
  hipStream_t stream = nullptr;   // verify work (highest priority)
  hipStream_t hstream = nullptr;  // a keyed batch's cache keys, beside the verify kernel (highest priority)
  hipEvent_t done = nullptr, keys_down = nullptr;
  hipEvent_t ev = nullptr;        // (a key-table build waits for the work queued here)
  hipEvent_t dev_done = nullptr;  // a device-API batch queued here is done (the caller's stream waits on it;
                                  // `done` stays the host batch's own, which must not wait for device-API work)
  HostBuf h_in, h_out;
  HostBuf z_out;   // mapped: the kernels write verdicts in place
  HostBuf z_keys;  // mapped: the hash kernel writes cache keys in place (keyed batches)
  HostBuf z_stat;  // mapped: the launch's failure word (sv_kparams::status), zeroed per batch
  DevBuf d_in, d_out, d_keys;
  DevBuf ws;  // the quad kernel's tables (cold batches above kOctetMax)
  bool busy = false;  // (under LatLane::mu) a batch holds it
};
constexpr int kLatCtxMax = 2;
struct LatLane {
  std::mutex mu;
  std::condition_variable freed;  // a context was released
  bool ready = false;
  int nctx = 1;
  LatCtx ctx[kLatCtxMax];
  hipStream_t build = nullptr;   // key-table builds (lowest priority)
  hipEvent_t ev_lat = nullptr;   // (device-API batches: the caller's stream)
  HostBuf h_build;
  DevBuf d_build;
  void* ctab = nullptr;  // tables of B (built at lane init)
  DevBuf ktab, kstat;    // tables of -A per cached key, status per slot
  size_t cap = 0;        // key-cache capacity the index / tables are sized for
  sv::KeyIndex index;
  uint64_t tick = 0, next_gen = 1;
  struct Build {
    uint64_t gen;
    hipEvent_t uploaded, done;
    std::vector<int32_t> slots;
  };
  std::deque<Build> inflight;
  // kernel-time accounting (sv_timing_enable), as Device::pending
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<uint64_t> pending_n;
  double total_ms = 0;
  uint64_t launches = 0, sigs = 0;
  std::vector<uint32_t> kslots;          // per signature of the batch being planned
  std::vector<const uint8_t*> fresh_pk;  // keys admitted by it
  std::vector<int32_t> fresh_slot;
  uint64_t warm = 0, cold = 0, built = 0, evicted = 0;
};

// Per-key tables of the throughput path (sv_kernels.hip sv_keyslot_kernel),
// one set per slot: claim words, entries, per-chunk slot and builder lists,
// the two counters and a pinned copy of them (read lazily: the claims decide
// when the claim words are cleared, never a verdict).
struct KeyTabs {
  DevBuf index, store, kslot, builders, count;
  HostBuf h_count;
  hipEvent_t copied = nullptr;  // h_count holds the counters after the last launch
  size_t slots = 0;
  uint64_t salt = 0;
  uint64_t launches = 0, clears = 0, claims = 0;
};

struct Device {
  int slot = -1;
  int phys = -1;
  bool ready = false;  // resources created lazily on first use (under mu)
  int cus = 0;
  unsigned grid = 0;  // persistent grid (workgroups)
  unsigned grid_share = 0;  // the same in shared mode (latency batches live: share_now)
  hipStream_t stream = nullptr, h2d = nullptr, d2h = nullptr;
  void* btab = nullptr;
  DevBuf ws;  // kernel workspace, grown on demand (after draining `stream`)
  hipEvent_t dep_in = nullptr, dep_out = nullptr;
  std::mutex mu;
  Stage st[2];
  HostBuf z_in;   // mapped: a one-chunk batch's image, read in place (bulk_in_place)
  HostBuf z_out;  // mapped: its verdicts, written in place (bulk_zc_out)
  DevBuf msg, off, len, keys;  // sha256 batches
  HostBuf h_sha;
  // timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<uint64_t> pending_n;
  double total_ms = 0;
  uint64_t launches = 0, sigs = 0;
  LatLane lat;
  KeyTabs kt;  // (under mu)
  std::atomic<int64_t> lat_last_ns{INT64_MIN / 2};  // steady clock of the last latency-lane batch
  std::atomic<uint64_t> shared_launches{0};          // bulk launches in shared mode
  // The slot's own staging workers for multi-slot calls (shard): its slice is
  // driven and packed here, not on the shared pool, so G slots pack on G sets
  // of threads at once.  Pinned to the GPU's NUMA node where the host tells
  // it (slot_pool).  Created on first multi-slot use, under spool_mu.
  std::mutex spool_mu;
  std::unique_ptr<sv::Pool> spool;
  int numa = -2;        // GPU's NUMA node (-1 unknown; -2 not looked up yet)
  size_t numa_cpus = 0;  // CPUs the workers are pinned to (0: not pinned)
};

std::mutex g_mu;
std::vector<Device*> g_devs;
std::vector<int> g_map;  // slot -> physical device (empty: identity)
bool g_inited = false;
std::atomic<int> g_timing{0};
std::atomic<int> g_path{SV_PATH_AUTO};   // sv_set_kernel_path
std::atomic<uint32_t> g_dbg{0};          // sv_set_debug_flags
std::atomic<size_t> g_min_shard{0};      // sv_set_min_shard (0: default)
std::atomic<uint64_t> g_rr{0};           // round-robin slot for single-slot calls

constexpr uint32_t kKernelDbgMask =
    SV_DBG_TRIVIAL_PAIR | SV_DBG_MAX_WINDOWS | SV_DBG_PREP_ONLY | SV_DBG_KEY_COLLIDE | SV_DBG_DROP_HANDOVER;

// Batches up to this size take the latency kernel under SV_PATH_AUTO
// (measured crossover on MI355X).
constexpr uint64_t kQuickMax = 12288;

size_t min_shard() {
  const size_t v = g_min_shard.load();
  return v ? v : env_size("SV_MIN_SHARD", (size_t)1 << 16);
}
size_t stage_chunk() {
  static const size_t c = std::max<size_t>(1024, env_size("SV_STAGE_CHUNK", (size_t)1 << 18));
  return c;
}
// Pipeline fill: the first R chunks of a multi-chunk batch grow geometrically
// (chunk / 2^R, ..., chunk / 2), so the first kernel starts after packing and
// copying a small chunk instead of a whole one.  SV_STAGE_RAMP = R (default
// 2: chunk/4 then chunk/2; 0: equal chunks).
size_t stage_ramp_steps() {
  static const size_t r = std::min<size_t>(env_size("SV_STAGE_RAMP", 2), 8);
  return r;
}
bool stage_ramp() { return stage_ramp_steps() != 0; }
size_t chunk_len(size_t c, size_t chunk, size_t left) {
  size_t m = chunk;
  const size_t r = stage_ramp_steps();
  if (c < r) m = std::max<size_t>(1024, chunk >> (r - c));
  return std::min(m, left);
}

int resolve_path(int requested, uint64_t n) {
  int p = requested != SV_PATH_AUTO ? requested : g_path.load();
  if (p == SV_PATH_AUTO) p = n <= kQuickMax ? SV_PATH_LATENCY : SV_PATH_THROUGHPUT;
  return p;
}

// Throughput-path launches of at most this many signatures run one signature
// per quad of lanes (sv_kernels.hip sv_quad_kernel): below about one wave per
// SIMD the one-lane kernels run at a lone wave's serial latency
// (tools/size_sweep.py).  SV_QUAD_MAX overrides (0: never).
constexpr uint64_t kQuadMax = 32768;
// Cold latency-lane batches above this size run the quad kernel (on the
// lane, at wave priority 3) instead of the octet kernel: one signature per 4
// lanes instead of 16 overtakes the octet's shorter chains from ~6k
// signatures (tools/size_sweep.py, profiles/r05/size_sweep/).
constexpr uint64_t kOctetMax = 6144;
uint64_t quad_max() {
  static const uint64_t v = env_size("SV_QUAD_MAX", kQuadMax);
  return v;
}
constexpr int kGeomQuad = 3;  // sv_launch_verify's path code of the quad geometry
// The kernel geometry of a launch of n on resolved path rp.  (A quad launch
// decodes every key itself: the per-key tables only serve the one-lane
// kernels of larger launches.)
int launch_geometry(int rp, uint64_t n) {
  if (rp != SV_PATH_THROUGHPUT) return rp;
  const uint32_t d = g_dbg.load();
  if (d & SV_DBG_NO_QUAD) return rp;
  if (d & SV_DBG_QUAD) return kGeomQuad;
  return n <= quad_max() ? kGeomQuad : rp;
}
int path_from_flags(uint32_t flags) {
  if (flags & SV_FLAG_PATH_LATENCY) return SV_PATH_LATENCY;
  if (flags & SV_FLAG_PATH_THROUGHPUT) return SV_PATH_THROUGHPUT;
  return SV_PATH_AUTO;
}

int init_device(Device& D) {
  SV_HIP(hipSetDevice(D.phys));
  hipDeviceProp_t prop;
  SV_HIP(hipGetDeviceProperties(&prop, D.phys));
  D.cus = prop.multiProcessorCount;
  SV_HIP(hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking));
  SV_HIP(hipStreamCreateWithFlags(&D.h2d, hipStreamNonBlocking));
  SV_HIP(hipStreamCreateWithFlags(&D.d2h, hipStreamNonBlocking));
  SV_HIP(hipEventCreateWithFlags(&D.dep_in, hipEventDisableTiming));
  SV_HIP(hipEventCreateWithFlags(&D.dep_out, hipEventDisableTiming));
  D.z_in.mapped = D.z_out.mapped = true;
  for (Stage& s : D.st) {
    SV_HIP(hipEventCreateWithFlags(&s.up, hipEventDisableTiming));
    SV_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    SV_HIP(hipEventCreateWithFlags(&s.down, hipEventDisableTiming));
    SV_HIP(hipEventCreateWithFlags(&s.keys_down, hipEventDisableTiming));
  }
  SV_HIP(hipMalloc(&D.btab, sv_btab_bytes()));
  SV_HIP(sv_launch_btab_init((uint32_t*)D.btab, D.stream));
  D.grid = (unsigned)(D.cus * sv_occupancy_blocks_per_cu());
  D.grid_share = (unsigned)(D.cus * std::max(1, sv_share_blocks_per_cu()));
  SV_HIP(hipStreamSynchronize(D.stream));
  return SV_OK;
}

void release_device(Device& D) {
  if (!D.ready) return;
  (void)hipSetDevice(D.phys);
  (void)hipStreamSynchronize(D.stream);
  (void)hipStreamSynchronize(D.h2d);
  (void)hipStreamSynchronize(D.d2h);
  for (auto& pr : D.pending) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  D.pending.clear();
  D.pending_n.clear();
  D.z_in.release();
  D.z_out.release();
  for (Stage& s : D.st) {
    s.h_in.release(); s.h_out.release();
    s.d_in.release(); s.d_verdict.release(); s.d_keys.release();
    if (s.up) (void)hipEventDestroy(s.up);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.down) (void)hipEventDestroy(s.down);
    if (s.keys_down) (void)hipEventDestroy(s.keys_down);
    for (hipEvent_t e : s.pev) (void)hipEventDestroy(e);
    s.pev.clear();
    s.up = s.done = s.down = s.keys_down = nullptr;
  }
  D.msg.release(); D.off.release(); D.len.release(); D.keys.release(); D.h_sha.release();
  D.ws.release();
  D.kt.index.release(); D.kt.store.release(); D.kt.kslot.release(); D.kt.builders.release();
  D.kt.count.release(); D.kt.h_count.release();
  if (D.kt.copied) (void)hipEventDestroy(D.kt.copied);
  D.kt.copied = nullptr;
  D.kt.slots = 0;
  if (D.btab) (void)hipFree(D.btab);
  if (D.dep_in) (void)hipEventDestroy(D.dep_in);
  if (D.dep_out) (void)hipEventDestroy(D.dep_out);
  if (D.stream) (void)hipStreamDestroy(D.stream);
  if (D.h2d) (void)hipStreamDestroy(D.h2d);
  if (D.d2h) (void)hipStreamDestroy(D.d2h);
  D.btab = nullptr;
  D.stream = D.h2d = D.d2h = nullptr;
  D.ready = false;
}

// Enumerates devices and builds the slot table; per-slot resources are
// created on first use so a process that drives one GPU (one rank per GPU)
// never touches the others.  Caller holds g_mu.
int init_locked() {
  if (g_inited) return g_devs.empty() ? fail(SV_ERR_NO_DEVICE, "no HIP device") : SV_OK;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  g_inited = true;
  // SV_TEST_STUB_SLOTS=k (with SV_TEST_KNOBS=1, no GPU): k slots on no device,
  // so the slot table's lifetime can be stressed on a CPU-only host (every
  // call that reaches a slot's resources fails with SV_ERR_HIP)
  const size_t stub = (e != hipSuccess || n <= 0) && test_knobs_enabled() ? env_size("SV_TEST_STUB_SLOTS", 0) : 0;
  if (stub) {
    const size_t k = g_map.empty() ? stub : g_map.size();
    for (size_t i = 0; i < k; ++i) {
      Device* D = new Device();
      D->slot = (int)i;
      D->phys = -1;
      g_devs.push_back(D);
    }
    return SV_OK;
  }
  if (e != hipSuccess || n <= 0) return fail(SV_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  std::vector<int> map = g_map;
  if (map.empty()) {
    if (const char* env = getenv("SV_DEVICE_MAP")) {
      const char* p = env;
      while (*p) {
        char* end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p) break;
        map.push_back((int)v);
        p = *end == ',' ? end + 1 : end;
      }
    }
  }
  if (map.empty())
    for (int i = 0; i < n; ++i) map.push_back(i);
  for (int v : map)
    if (v < 0 || v >= n) {
      g_inited = false;
      return fail(SV_ERR_INVALID_ARG, "device map names a device that does not exist");
    }
  for (size_t i = 0; i < map.size(); ++i) {
    Device* D = new Device();
    D->slot = (int)i;
    D->phys = map[i];
    g_devs.push_back(D);
  }
  return SV_OK;
}

int ensure_init() {
  std::lock_guard<std::mutex> g(g_mu);
  return init_locked();
}

// Caller holds D.mu.
int ready_locked(Device& D) {
  if (D.ready) return SV_OK;
  int rc = init_device(D);
  if (rc == SV_OK) D.ready = true;
  return rc;
}

// Workspace for a launch (caller holds D.mu, device set).  Growing it frees
// the old one, so the kernel stream is drained first.
int ensure_ws(Device& D, size_t bytes) {
  if (bytes <= D.ws.cap) return SV_OK;
  SV_HIP(hipStreamSynchronize(D.stream));
  return D.ws.ensure(bytes);
}

// Shared mode of the throughput kernels (sv_kernels.hip sv_launch_verify):
// taken by every bulk launch within SV_LAT_SHARE_MS (default 1000) ms of a
// latency-lane batch on the same slot, so SCP-class batches find free
// workgroup slots while a tx set or catchup batch runs.  0 disables it.
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
int64_t share_window_ns() {
  static const int64_t w = (int64_t)env_size("SV_LAT_SHARE_MS", 1000) * 1000000;
  return w;
}
size_t share_upload_bytes() {
  static const size_t b = std::max<size_t>(64, env_size("SV_SHARE_UPLOAD_KB", 2048)) * 1024;
  return b;
}
// One-chunk host batches (n <= SV_STAGE_CHUNK) read in place
// (SV_BULK_ZC_IN, default on; 0: one staged H2D copy): the kernels read the
// packed image from mapped pinned memory, so the copy no longer runs before
// the first kernel (a multi-chunk batch overlaps its copies with the previous
// chunk's kernels and stays staged).
bool bulk_in_place() {
  static const bool b = env_size("SV_BULK_ZC_IN", 1) != 0;
  return b;
}
// ... and their verdicts are written in place too (SV_BULK_ZC_OUT, default on):
// the kernels store them to mapped memory, so no copy is queued behind them.
bool bulk_zc_out() {
  static const bool b = env_size("SV_BULK_ZC_OUT", 1) != 0;
  return b;
}
// One-chunk throughput launches read in place run the prep kernel in its
// decode-first order (sv_kernels.hip sv_prep_kernel DF; SV_DECODE_FIRST=0: the
// device path's order)
bool decode_first() {
  static const bool b = env_size("SV_DECODE_FIRST", 1) != 0;
  return b;
}
bool share_now(const Device& D) {
  const int64_t w = share_window_ns();
  return w > 0 && now_ns() - D.lat_last_ns.load(std::memory_order_relaxed) < w;
}

unsigned grid_for(const Device& D, uint64_t n, bool share = false) {
  const uint64_t need = (n + sv_block_threads() - 1) / sv_block_threads();
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(share ? D.grid_share : D.grid, need));
}

// ---------------------------------------------------- per-key tables
// sv_set_key_tables: 0 off, 1 on for every throughput-path launch, 2 (auto,
// the default) on for host-buffer batches whose keys repeat (repeated_keys);
// -1: SV_KEY_TABLES.  Slots: SV_KEY_TABLE_SLOTS (default 2^19; claims stop at
// half of them, when the claim words are cleared).
std::atomic<int> g_kt_mode{-1};
std::atomic<size_t> g_kt_slots{0};
int kt_mode() {
  const int v = g_kt_mode.load();
  if (v >= 0) return v;
  return (int)std::min<size_t>(2, env_size("SV_KEY_TABLES", 2));
}
size_t kt_slots() {
  size_t v = g_kt_slots.load();
  if (v == 0) v = env_size("SV_KEY_TABLE_SLOTS", (size_t)1 << 19);
  size_t p = 1024;
  while (p < v && p < ((size_t)1 << 26)) p <<= 1;
  return p;
}

// Readies the slot's key tables for a launch of n (caller holds D.mu, device
// set) and fills *kt; false: tables unavailable (allocation failed), the
// launch runs without them.
bool kt_prepare(Device& D, uint64_t n, sv_ktparams* kt) {
  KeyTabs& T = D.kt;
  const size_t want = kt_slots();
  if (T.slots != want) {
    (void)hipStreamSynchronize(D.stream);
    T.index.release();
    T.store.release();
    T.slots = 0;
    if (T.index.ensure(want * 8) || T.store.ensure(want * sv_key_table_entry_bytes()) || T.count.ensure(16) ||
        T.h_count.ensure(16))
      return false;
    if (!T.copied && hipEventCreateWithFlags(&T.copied, hipEventDisableTiming) != hipSuccess) return false;
    if (hipMemsetAsync(T.index.p, 0, want * 8, D.stream) != hipSuccess ||
        hipMemsetAsync(T.count.p, 0, 16, D.stream) != hipSuccess)
      return false;
    std::memset(T.h_count.p, 0, 16);
    T.salt = ((uint64_t)std::random_device{}() << 32) ^ std::random_device{}() ^ (uint64_t)now_ns();
    T.slots = want;
  }
  const uint64_t cap = sv_plan_chunk_max(n);
  if (cap * 4 > T.kslot.cap || cap * 4 > T.builders.cap) {
    (void)hipStreamSynchronize(D.stream);  // (the lists of a running launch)
    if (T.kslot.ensure(cap * 4) || T.builders.ensure(cap * 4)) return false;
  }
  // the claims as of the last launch whose counters have come back
  const uint32_t limit = (uint32_t)(want / 2);
  if (hipEventQuery(T.copied) == hipSuccess) {
    T.claims = ((const uint32_t*)T.h_count.p)[1];
    if (T.claims >= limit) {
      if (hipMemsetAsync(T.index.p, 0, want * 8, D.stream) != hipSuccess ||
          hipMemsetAsync(T.count.p, 0, 16, D.stream) != hipSuccess)
        return false;
      std::memset(T.h_count.p, 0, 16);
      T.claims = 0;
      ++T.clears;
    }
  }
  kt->index = (unsigned long long*)T.index.p;
  kt->store = (sv_u4*)T.store.p;
  kt->kslot = (uint32_t*)T.kslot.p;
  kt->builders = (uint32_t*)T.builders.p;
  kt->count = (uint32_t*)T.count.p;
  kt->mask = want - 1;
  kt->limit = limit;
  kt->salt = T.salt;
  return true;
}

// Launch on D.stream (caller holds D.mu and has set the device).  tables:
// the launch may use the per-key tables (kt_mode / repeated_keys).
// kp: SV_KP_* launch hints (SV_KP_IN_PLACE: the inputs are mapped host memory)
int launch_locked(Device& D, int mode, int path, const void* pk, const void* sig, const void* msg, const uint64_t* off,
                  const uint32_t* len, uint32_t fixed_len, uint64_t n, void* verdict, void* bitmap,
                  bool tables = false, uint32_t kp = 0) {
  const int rp = resolve_path(path, n);
  const bool share = rp != SV_PATH_LATENCY && share_now(D);
  const unsigned grid = grid_for(D, n, share);
  int rc;
  sv_ktparams ktp{};
  const int geom = launch_geometry(rp, n);
  const bool kt_on = tables && geom == SV_PATH_THROUGHPUT && kt_prepare(D, n, &ktp);
  if ((rc = ensure_ws(D, sv_verify_ws_bytes(geom, grid, n)))) return rc;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool timing = g_timing.load() != 0;
  if (timing) {
    SV_HIP(hipEventCreate(&e0));
    SV_HIP(hipEventCreate(&e1));
    SV_HIP(hipEventRecord(e0, D.stream));
  }
  SV_HIP(sv_launch_verify(mode, geom, grid, pk, sig, msg, off, len, fixed_len, n, verdict, bitmap, D.ws.p, D.btab,
                          (g_dbg.load() & kKernelDbgMask) | (kt_on ? 0u : kp), share ? 1 : 0, kt_on ? &ktp : nullptr,
                          nullptr, D.stream));
  if (share) D.shared_launches.fetch_add(1, std::memory_order_relaxed);
  if (kt_on) {
    ++D.kt.launches;
    SV_HIP(hipMemcpyAsync(D.kt.h_count.p, D.kt.count.p, 8, hipMemcpyDeviceToHost, D.stream));
    SV_HIP(hipEventRecord(D.kt.copied, D.stream));
  }
  if (timing) {
    SV_HIP(hipEventRecord(e1, D.stream));
    D.pending.emplace_back(e0, e1);
    D.pending_n.push_back(n);
  }
  return SV_OK;
}

int harvest_timing_locked(Device& D) {
  for (size_t k = 0; k < D.pending.size(); ++k) {
    SV_HIP(hipEventSynchronize(D.pending[k].second));
    float ms = 0;
    SV_HIP(hipEventElapsedTime(&ms, D.pending[k].first, D.pending[k].second));
    D.total_ms += ms;
    D.launches += 1;
    D.sigs += D.pending_n[k];
    (void)hipEventDestroy(D.pending[k].first);
    (void)hipEventDestroy(D.pending[k].second);
  }
  D.pending.clear();
  D.pending_n.clear();
  return SV_OK;
}

// ------------------------------------------------------------ host inputs
// A batch in host memory: contiguous SoA arrays (pk n x 32, sig n x 64,
// messages by offset/length or fixed stride), or pointer arrays (gather).
struct HostIn {
  const uint8_t* pk = nullptr;
  const uint8_t* sig = nullptr;
  const uint8_t* msg = nullptr;
  const uint64_t* off = nullptr;
  const uint32_t* len = nullptr;
  uint32_t fixed = 0;  // != 0: message i = msg + i * fixed, or msg + off[i] when off is set (uniform lengths)
  const uint8_t* const* ppk = nullptr;  // gather form (ppk != nullptr)
  const uint8_t* const* psig = nullptr;
  const uint8_t* const* pmsg = nullptr;

  bool gather() const { return ppk != nullptr; }
  uint32_t mlen(size_t i) const { return fixed ? fixed : len[i]; }
  const uint8_t* pkp(size_t i) const { return gather() ? ppk[i] : pk + 32 * i; }
  const uint8_t* sigp(size_t i) const { return gather() ? psig[i] : sig + 64 * i; }
  const uint8_t* msgp(size_t i) const {
    if (gather()) return pmsg[i];
    return off ? msg + off[i] : msg + i * (size_t)fixed;
  }
  // the slice [lo, ...) as a batch of its own
  HostIn sub(size_t lo) const {
    HostIn s = *this;
    if (gather()) {
      s.ppk += lo;
      s.psig += lo;
      s.pmsg += lo;
      s.len += lo;
    } else {
      s.pk += 32 * lo;
      s.sig += 64 * lo;
      if (off) {
        s.off += lo;
        if (len) s.len += lo;
      } else {
        s.msg += lo * (size_t)fixed;
      }
    }
    return s;
  }
};

// Pinned image of m signatures starting at `lo`:
//   pk (32 m) | sig (64 m) | fixed: msgs (m L)   or   var: off (8 m) | len (4 m) | packed msgs
// (pk, sig and a fixed-length message block stay 16-byte aligned).
struct Image {
  size_t o_sig, o_off, o_len, o_msg, bytes;
  bool var;
};

Image image_of(const HostIn& in, size_t lo, size_t m, size_t* msg_total) {
  Image im;
  im.var = in.fixed == 0;
  size_t total = 0;
  if (!im.var) total = m * (size_t)in.fixed;
  else
    for (size_t i = 0; i < m; ++i) total += in.len[lo + i];
  im.o_sig = 32 * m;
  im.o_off = 96 * m;
  im.o_len = im.o_off + 8 * m;
  im.o_msg = im.var ? im.o_len + 4 * m : im.o_off;
  im.bytes = im.o_msg + std::max<size_t>(total, 1);
  *msg_total = total;
  return im;
}

// Packing [lo, lo + m) into h (layout `im`): the message offsets first, then
// rows [r0, r1) of the chunk, in parallel for large ranges.
// (rows [r0, r1), the first at message offset pos; returns the offset past r1)
uint64_t pack_offsets(const HostIn& in, size_t lo, size_t r0, size_t r1, uint64_t pos, const Image& im, uint8_t* h) {
  uint64_t* offs = (uint64_t*)(h + im.o_off);
  if (im.var) {
    for (size_t i = r0; i < r1; ++i) {
      offs[i] = pos;
      pos += in.len[lo + i];
    }
  }
  return pos;
}
// Bytes per helper task of a pack of at least 2 MB (SV_PACK_PART); smaller
// packs take 1 MB tasks.  With 1 MB tasks a 29k-signature batch (3.7 MB) was
// packed by 3 threads; 256 KB tasks spread it over the pool: host call 0.669-
// 0.707 -> 0.663-0.675 ms, 50k 0.88-0.92 -> 0.86-0.89 ms, while at 8k (1 MB)
// waking the pool cost 10 us (profiles/r05/host_call/pack_part/).
size_t pack_part() {
  static const size_t v = std::max<size_t>(4096, env_size("SV_PACK_PART", 1u << 18));
  return v;
}
// Pack stores bypass the CPU caches (SV_PACK_NT, default on): the pinned
// image is read by the GPU (DMA or in place), never again by the CPU, and a
// cached store first reads each destination line.  Measured on the GPU box's
// host, 128 MB copies: 16 threads 107 -> 180 GB/s, 8 threads 90 -> 127 GB/s
// (tools/nt_copy_probe.cpp, profiles/r06/feed/nt_copy_probe.txt).
bool pack_nt() {
  static const bool b = env_size("SV_PACK_NT", 1) != 0;
  return b;
}
// dst 16-byte aligned (else memcpy); the caller fences (_mm_sfence) before
// the data is handed to the device.
inline void nt_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  if (((uintptr_t)dst & 15u) != 0) {
    std::memcpy(dst, src, n);
    return;
  }
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128((const __m128i*)(src + i));
    const __m128i b = _mm_loadu_si128((const __m128i*)(src + i + 16));
    const __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32));
    const __m128i d = _mm_loadu_si128((const __m128i*)(src + i + 48));
    _mm_stream_si128((__m128i*)(dst + i), a);
    _mm_stream_si128((__m128i*)(dst + i + 16), b);
    _mm_stream_si128((__m128i*)(dst + i + 32), c);
    _mm_stream_si128((__m128i*)(dst + i + 48), d);
  }
  for (; i + 16 <= n; i += 16) _mm_stream_si128((__m128i*)(dst + i), _mm_loadu_si128((const __m128i*)(src + i)));
  if (i < n) std::memcpy(dst + i, src + i, n - i);
}
// kPart: bytes per helper task, as above when 0 (a keyed batch's pieces take
// smaller ones: the first verify launch waits for the last piece)
void pack_rows(const HostIn& in, size_t lo, size_t r0, size_t r1, const Image& im, uint8_t* h, size_t kPart = 0) {
  const uint64_t* offs = (const uint64_t*)(h + im.o_off);
  const size_t m = r1 - r0;
  const size_t est = im.bytes / std::max<size_t>(1, (im.o_sig / 32)) * m;  // (bytes of these rows, roughly)
  if (kPart == 0) kPart = est >= (2u << 20) ? pack_part() : (1u << 20);
  sv::Pool& pp = pack_pool();
  const size_t cap = t_pack_parts ? t_pack_parts : pp.size() + 1;
  const size_t parts = std::max<size_t>(1, std::min<size_t>(std::min(pp.size() + 1, cap), est / kPart));
  const bool nt = pack_nt();
  auto cp = [nt](uint8_t* d, const uint8_t* s, size_t k) {
    if (nt) nt_copy(d, s, k);
    else std::memcpy(d, s, k);
  };
  pp.run(parts, [&](size_t t) {
    const size_t a = r0 + m * t / parts, b = r0 + m * (t + 1) / parts;
    if (a == b) return;
    // (the streaming stores of this part are ordered before its completion,
    // which the pool publishes under a mutex, and so before the upload)
    struct Fence {
      bool nt;
      ~Fence() {
        if (nt) _mm_sfence();
      }
    } fence{nt};
    if (!in.gather()) {
      cp(h + 32 * a, in.pk + 32 * (lo + a), 32 * (b - a));
      cp(h + im.o_sig + 64 * a, in.sig + 64 * (lo + a), 64 * (b - a));
      if (!im.var && !in.off) {
        cp(h + im.o_msg + a * (size_t)in.fixed, in.msg + (lo + a) * (size_t)in.fixed, (b - a) * (size_t)in.fixed);
        return;
      }
      if (!im.var) {  // (uniform lengths, found by offset: packed at the fixed stride)
        for (size_t i = a; i < b; ++i) cp(h + im.o_msg + i * (size_t)in.fixed, in.msg + in.off[lo + i], in.fixed);
        return;
      }
    } else {
      for (size_t i = a; i < b; ++i) {
        cp(h + 32 * i, in.ppk[lo + i], 32);
        cp(h + im.o_sig + 64 * i, in.psig[lo + i], 64);
      }
      if (!im.var) {
        for (size_t i = a; i < b; ++i) cp(h + im.o_msg + i * (size_t)in.fixed, in.pmsg[lo + i], in.fixed);
        return;
      }
    }
    std::memcpy(h + im.o_len + 4 * a, in.len + lo + a, 4 * (b - a));
    for (size_t i = a; i < b; ++i) {
      const uint32_t l = in.len[lo + i];
      if (l) std::memcpy(h + im.o_msg + offs[i], in.msgp(lo + i), l);
    }
  });
}
void pack(const HostIn& in, size_t lo, size_t m, const Image& im, uint8_t* h) {
  pack_offsets(in, lo, 0, m, 0, im, h);
  pack_rows(in, lo, 0, m, im, h);
}
// H2D of rows [a, b) of a packed image (each section's slice); msg_total: the
// image's message bytes.
int upload_rows(const Image& im, size_t m, size_t a, size_t b, uint32_t fixed, size_t msg_total, const uint8_t* h,
                uint8_t* d, hipStream_t st) {
  SV_HIP(hipMemcpyAsync(d + 32 * a, h + 32 * a, 32 * (b - a), hipMemcpyHostToDevice, st));
  SV_HIP(hipMemcpyAsync(d + im.o_sig + 64 * a, h + im.o_sig + 64 * a, 64 * (b - a), hipMemcpyHostToDevice, st));
  size_t m0, m1;
  if (im.var) {
    SV_HIP(hipMemcpyAsync(d + im.o_off + 8 * a, h + im.o_off + 8 * a, 8 * (b - a), hipMemcpyHostToDevice, st));
    SV_HIP(hipMemcpyAsync(d + im.o_len + 4 * a, h + im.o_len + 4 * a, 4 * (b - a), hipMemcpyHostToDevice, st));
    const uint64_t* offs = (const uint64_t*)(h + im.o_off);
    m0 = offs[a];
    m1 = b < m ? offs[b] : msg_total;
  } else {
    m0 = a * (size_t)fixed;
    m1 = b * (size_t)fixed;
  }
  if (m1 > m0) SV_HIP(hipMemcpyAsync(d + im.o_msg + m0, h + im.o_msg + m0, m1 - m0, hipMemcpyHostToDevice, st));
  return SV_OK;
}

// SV_STAGE_TRACE: per-call host staging timings to stderr (developer knob)
bool stage_trace() {
  static const bool t = getenv("SV_STAGE_TRACE") != nullptr;
  return t;
}
thread_local double g_trace_pack_us = 0;
// (both traces also print steady-clock microseconds, to line a bulk call's
// stages up with the latency lane's batches)
double trace_abs_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Collects a finished chunk's results from its pinned slot.
int drain_stage(Stage& s, uint8_t* verdict, uint8_t* keys) {
  if (!s.busy) return SV_OK;
  SV_HIP(hipEventSynchronize(s.down));
  if (stage_trace()) fprintf(stderr, "SV_STAGE_TRACE down synced @%.1f\n", trace_abs_us());
  s.busy = false;
  const uint8_t* h = (const uint8_t*)s.h_out.p;
  if (verdict) std::memcpy(verdict + s.lo, s.zv ? s.zv : h, s.m);
  if (keys) std::memcpy(keys + 32 * s.lo, h + (verdict ? s.m : 0), 32 * s.m);
  return SV_OK;
}

thread_local std::chrono::steady_clock::time_point g_trace_t0;  // (SV_STAGE_TRACE: host_slice entry)

// Keys-ready notification of the keyed gather entry points: fn(ctx, ready)
// with keys [0, ready) in the caller's array, called with increasing `ready`,
// the last time with ready == n.
struct KeysCb {
  void (*fn)(void*, size_t) = nullptr;
  void* ctx = nullptr;
  explicit operator bool() const { return fn != nullptr; }
  void operator()(size_t ready) const { fn(ctx, ready); }
};
// A one-chunk keyed batch of at least kKeyPieceMin rows sends its keys up in
// pieces (key_pieces): the caller's cache walk starts on the first piece while
// later ones are packed, copied and hashed.  The first piece is kKeyPieceFirst
// rows, so the walk starts as early as it can; each later piece is twice the
// one before, at most kKeyPieceMax rows (a piece costs ~10 HIP calls on this
// thread: fewer pieces bring the last one, and the verify launch behind it,
// forward).
constexpr size_t kKeyPieceMin = 8192, kKeyPieceFirst = 2048, kKeyPieceMax = 1 << 15;
// Row bounds of the pieces of an m-row batch: b[0] = 0 < b[1] < ... < b[P] = m.
std::vector<size_t> key_pieces(size_t m) {
  if (m < kKeyPieceMin) return {0, m};
  std::vector<size_t> b{0};
  for (size_t len = kKeyPieceFirst; b.back() < m; len = std::min(2 * len, kKeyPieceMax))
    b.push_back(m - b.back() < len + len / 2 ? m : b.back() + len);  // (no runt last piece)
  return b;
}

// Runs fn(0), fn(1), ... fn(P - 1) on a thread of its own, fn(k) once piece
// k's events have been recorded (recorded(k + 1)); join() returns the first
// error.  The destructor stops and joins it (an early error return of the
// caller).
// Depth of engine entry points on this thread (LifeGuard below); > 0 also on a
// KeyNotifier thread, whose callbacks run inside the caller's entry point, so
// sv_shutdown / sv_set_device_map from a callback is refused there too.
thread_local int t_life_depth = 0;

class KeyNotifier {
 public:
  ~KeyNotifier() {
    stop_.store(true);
    if (th_.joinable()) th_.join();
  }
  void start(int dev, size_t P, std::function<int(size_t)> fn) {
    fn_ = std::move(fn);
    th_ = std::thread([this, dev, P] {
      // (the caller holds the lifetime lock until this thread is joined)
      t_life_depth = 1;
      (void)hipSetDevice(dev);
      for (size_t k = 0; k < P; ++k) {
        while (rec_.load(std::memory_order_acquire) <= k) {
          if (stop_.load()) return;
          std::this_thread::yield();
        }
        const int rc = fn_(k);
        if (rc != SV_OK) {
          rc_ = rc;
          return;
        }
      }
    });
  }
  void recorded(size_t k) { rec_.store(k, std::memory_order_release); }
  int join() {
    if (th_.joinable()) th_.join();
    return rc_;
  }

 private:
  std::thread th_;
  std::function<int(size_t)> fn_;
  std::atomic<size_t> rec_{0};
  std::atomic<bool> stop_{false};
  int rc_ = SV_OK;
};

// Do the keys of a host batch repeat?  A sample of up to 4096 evenly spaced
// rows: with s sampled of n and d repeats among them, K distinct keys give
// d ~ s^2 / 2K, so K <= n / 2 (each key signs twice on average) reads as
// d * n >= s^2 (exact when s = n: n - d <= n / 2).
bool repeated_keys(const HostIn& in, size_t n) {
  const size_t s = std::min<size_t>(n, 4096);
  if (s < 2) return false;
  constexpr size_t kSet = 8192;
  std::vector<const uint8_t*> set(kSet, nullptr);
  size_t d = 0;
  for (size_t k = 0; k < s; ++k) {
    const uint8_t* pk = in.pkp(k * n / s);
    uint64_t h;
    std::memcpy(&h, pk, 8);
    h *= 0x9E3779B97F4A7C15ull;
    for (size_t j = (size_t)(h >> 51) & (kSet - 1);; j = (j + 1) & (kSet - 1)) {
      if (!set[j]) {
        set[j] = pk;
        break;
      }
      if (std::memcmp(set[j], pk, 32) == 0) {
        ++d;
        break;
      }
    }
  }
  return s == n ? 2 * (n - d) <= n : (uint64_t)d * n >= (uint64_t)s * s;
}

// Host-buffer slice on one slot, pipelined over staging chunks: verdicts
// (verdict != null) and/or BLAKE2b cache keys (keys != null) into the
// caller's arrays.  keys_cb (optional, with keys and verdict): called once
// every key is in `keys` -- for a one-chunk batch while the verify kernels
// are still running, so the caller's cache walk overlaps them; *cb_done
// records that it ran.
int host_slice_locked(Device& D, const HostIn& in, size_t n, uint8_t* verdict, uint8_t* keys, int path,
                      const KeysCb& kcb, bool* cb_done) {
  KeyNotifier notifier;  // (joined on every return path)
  const size_t chunk = std::min(n, stage_chunk());
  int rc;
  const int ktm = kt_mode();
  // (decided at the first launch: a keyed batch's first pieces go up before it)
  int tables = -1;
  auto trace_at = [](const char* what) {
    if (stage_trace())
      fprintf(stderr, "SV_STAGE_TRACE %s at %.1f us @%.1f\n", what,
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - g_trace_t0).count(),
              trace_abs_us());
  };
  // the largest launch first, so the workspace never grows under a running kernel
  if (verdict) {
    const int rp = resolve_path(path, chunk);
    const size_t wb = std::max(sv_verify_ws_bytes(rp, grid_for(D, chunk), chunk),
                               sv_verify_ws_bytes(launch_geometry(rp, chunk), grid_for(D, chunk), chunk));
    if ((rc = ensure_ws(D, wb))) return rc;
  }
  trace_at("workspace");
  const size_t out_per = (verdict ? 1 : 0) + (keys ? 32 : 0);
  // one chunk (latency-bound batches): everything on the kernel stream, no
  // cross-stream event waits
  const bool single = n <= chunk;
  hipStream_t up_s = single ? D.stream : D.h2d, down_s = single ? D.stream : D.d2h;
  if (!single && stage_ramp()) {
    // size both slots for a full chunk up front (the ramped first chunks
    // would otherwise grow the pinned buffers twice)
    size_t mt;
    const Image im = image_of(in, 0, chunk, &mt);
    for (Stage& s : D.st)
      if ((rc = s.h_in.ensure(im.bytes)) || (rc = s.d_in.ensure(im.bytes)) || (rc = s.h_out.ensure(out_per * chunk)))
        return rc;
  }
  size_t c = 0;
  size_t m = 0;
  for (size_t lo = 0; lo < n; lo += m, ++c) {
    Stage& s = D.st[c & 1];
    // slot c & 1 was last used by chunk c - 2: its results are collected
    // (which also means its H2D, kernels and D2H are complete)
    if ((rc = drain_stage(s, verdict, keys))) return rc;
    trace_at("slot drained");
    m = single ? n : chunk_len(c, chunk, n - lo);
    size_t msg_total;
    const Image im = image_of(in, lo, m, &msg_total);
    const bool early = single && kcb && keys && verdict;
    // a one-chunk keyed batch with a keys-ready callback: pack, copy up, hash
    // and copy the keys down in pieces, so the caller's walk starts early
    const std::vector<size_t> pb = early ? key_pieces(m) : std::vector<size_t>{0, m};
    const size_t P = pb.size() - 1;
    const bool in_place = single && P == 1 && bulk_in_place();
    const bool zc_out = in_place && verdict && bulk_zc_out();
    HostBuf& hin = in_place ? D.z_in : s.h_in;
    if ((rc = hin.ensure(im.bytes)) || (!in_place && (rc = s.d_in.ensure(im.bytes))) ||
        (rc = s.h_out.ensure(out_per * m)))
      return rc;
    if (verdict && !zc_out && (rc = s.d_verdict.ensure(m))) return rc;
    if (zc_out && (rc = D.z_out.ensure(m))) return rc;
    if (keys && (rc = s.d_keys.ensure(32 * m))) return rc;
    uint8_t* d = (uint8_t*)(in_place ? D.z_in.dp : s.d_in.p);
    uint8_t* hp = (uint8_t*)hin.p;
    const uint64_t* d_off = im.var ? (const uint64_t*)(d + im.o_off) : nullptr;
    const uint32_t* d_len = im.var ? (const uint32_t*)(d + im.o_len) : nullptr;
    while (s.pev.size() < P) {
      hipEvent_t e;
      SV_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      s.pev.push_back(e);
    }
    const auto t_pack = stage_trace() ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
    trace_at("staging");
    if (P == 1) {
      pack(in, lo, m, im, hp);
      // While latency-lane batches are live (shared mode), a chunk goes up in
      // pieces of SV_SHARE_UPLOAD_KB (default 2048): a 1k batch's 370 KB copy
      // otherwise queues behind the whole 32 MB chunk copy (~0.65 ms, once per
      // chunk: profiles/r04/isolation/).
      const size_t piece = share_now(D) ? share_upload_bytes() : im.bytes;
      for (size_t o = 0; !in_place && o < im.bytes; o += piece)
        SV_HIP(hipMemcpyAsync((uint8_t*)s.d_in.p + o, (const uint8_t*)s.h_in.p + o, std::min(piece, im.bytes - o),
                              hipMemcpyHostToDevice, up_s));
      trace_at("uploads enqueued");
      if (!single) {
        SV_HIP(hipEventRecord(s.up, D.h2d));
        SV_HIP(hipStreamWaitEvent(D.stream, s.up, 0));
      }
      if (keys)
        SV_HIP(sv_launch_hash(0, D.grid * 2, d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, m, s.d_keys.p,
                              D.stream));
      if (early) {
        // keys down on the D2H stream while the verify kernels run
        SV_HIP(hipEventRecord(s.done, D.stream));
        SV_HIP(hipStreamWaitEvent(D.d2h, s.done, 0));
        SV_HIP(hipMemcpyAsync((uint8_t*)s.h_out.p + m, s.d_keys.p, 32 * m, hipMemcpyDeviceToHost, D.d2h));
        SV_HIP(hipEventRecord(s.pev[0], D.d2h));
      }
    } else {
      // The pieces' keys go to the caller from a notifier thread while this
      // thread packs and uploads the next pieces (every callback runs on that
      // one thread, in order).
      const auto t0 = g_trace_t0;
      auto us = [t0] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(); };
      // (pb and us by value: an error return leaves this scope before the
      // notifier is joined)
      notifier.start(D.phys, P, [&, m, lo, pb, us](size_t k) -> int {
        const size_t a = pb[k], b = pb[k + 1];
        SV_HIP(hipEventSynchronize(s.pev[k]));
        if (stage_trace()) fprintf(stderr, "SV_STAGE_TRACE keys piece %zu down at %.1f us\n", k, us());
        std::memcpy(keys + 32 * (lo + a), (uint8_t*)s.h_out.p + m + 32 * a, 32 * (b - a));
        kcb(lo + b);
        if (stage_trace()) fprintf(stderr, "SV_STAGE_TRACE keys piece %zu walked at %.1f us\n", k, us());
        return SV_OK;
      });
      uint64_t pos = 0;  // (each piece writes its own message offsets first)
      for (size_t k = 0; k < P; ++k) {
        const size_t a = pb[k], b = pb[k + 1];
        pos = pack_offsets(in, lo, a, b, pos, im, hp);
        if (im.var && b < m) ((uint64_t*)(hp + im.o_off))[b] = pos;  // (upload_rows reads the piece's end there)
        pack_rows(in, lo, a, b, im, hp, 1u << 16);
        if (k == 0) trace_at("piece 0 packed");
        // uploads on the copy stream: piece k + 1 goes up while piece k hashes
        // (the slot's earlier work is complete: drained above)
        if ((rc = upload_rows(im, m, a, b, in.fixed, msg_total, hp, d, D.h2d))) return rc;
        SV_HIP(hipEventRecord(s.up, D.h2d));
        SV_HIP(hipStreamWaitEvent(D.stream, s.up, 0));
        if (k == 0) trace_at("piece 0 uploading");
        SV_HIP(sv_launch_hash(0, D.grid * 2, d + 32 * a, d + im.o_sig + 64 * a,
                              d + im.o_msg + (im.var ? 0 : a * (size_t)in.fixed), d_off ? d_off + a : nullptr,
                              d_len ? d_len + a : nullptr, in.fixed, b - a, (uint8_t*)s.d_keys.p + 32 * a, D.stream));
        SV_HIP(hipEventRecord(s.done, D.stream));
        SV_HIP(hipStreamWaitEvent(D.d2h, s.done, 0));
        SV_HIP(hipMemcpyAsync((uint8_t*)s.h_out.p + m + 32 * a, (uint8_t*)s.d_keys.p + 32 * a, 32 * (b - a),
                              hipMemcpyDeviceToHost, D.d2h));
        SV_HIP(hipEventRecord(s.pev[k], D.d2h));
        notifier.recorded(k + 1);
        if (stage_trace()) fprintf(stderr, "SV_STAGE_TRACE piece %zu enqueued at %.1f us\n", k, us());
      }
    }
    if (stage_trace()) g_trace_pack_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_pack).count();
    if (verdict) {
      const int mode = im.var ? 1 : (in.fixed == 32 ? 0 : 2);
      // (only the one-lane geometry uses the tables: a quad-geometry batch
      // skips the key sample, ~4k scattered reads of the caller's keys)
      if (tables < 0)
        tables = launch_geometry(resolve_path(path, chunk), chunk) == SV_PATH_THROUGHPUT &&
                 (ktm == 1 || (ktm == 2 && repeated_keys(in, n)));
      if ((rc = launch_locked(D, mode, path, d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, m,
                              zc_out ? D.z_out.dp : s.d_verdict.p, nullptr, tables != 0,
                              in_place && decode_first() ? SV_KP_IN_PLACE : 0u)))
        return rc;
      trace_at("launched");
    }
    if (!single) {
      SV_HIP(hipEventRecord(s.done, D.stream));
      SV_HIP(hipStreamWaitEvent(D.d2h, s.done, 0));
    }
    uint8_t* ho = (uint8_t*)s.h_out.p;
    if (verdict && !zc_out) SV_HIP(hipMemcpyAsync(ho, s.d_verdict.p, m, hipMemcpyDeviceToHost, down_s));
    if (keys && !early)
      SV_HIP(hipMemcpyAsync(ho + (verdict ? m : 0), s.d_keys.p, 32 * m, hipMemcpyDeviceToHost, down_s));
    SV_HIP(hipEventRecord(s.down, down_s));
    s.busy = true;
    s.lo = lo;
    s.m = m;
    s.zv = zc_out ? (const uint8_t*)D.z_out.p : nullptr;
    if (early) {
      if (P == 1) {
        SV_HIP(hipEventSynchronize(s.pev[0]));
        std::memcpy(keys + 32 * lo, ho + m, 32 * m);
        kcb(lo + m);
      } else if ((rc = notifier.join())) {
        return rc;
      }
      *cb_done = true;
    }
  }
  for (Stage& s : D.st)
    if ((rc = drain_stage(s, verdict, keys))) return rc;
  return SV_OK;
}

int host_slice(Device& D, const HostIn& in, size_t n, uint8_t* verdict, uint8_t* keys, int path,
               const KeysCb& kcb = KeysCb(), bool* cb_done = nullptr) {
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  int rc;
  if ((rc = ready_locked(D))) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  g_trace_t0 = t0;
  g_trace_pack_us = 0;
  rc = host_slice_locked(D, in, n, verdict, keys, path, kcb, cb_done);
  if (stage_trace())
    fprintf(stderr, "SV_STAGE_TRACE n=%zu pack %.1f us total %.1f us\n", n, g_trace_pack_us,
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  if (rc != SV_OK) {
    // leave the slot reusable: nothing of this call may still be in flight
    (void)hipStreamSynchronize(D.h2d);
    (void)hipStreamSynchronize(D.stream);
    (void)hipStreamSynchronize(D.d2h);
    D.st[0].busy = D.st[1].busy = false;
  }
  return rc;
}

// Host feed of a slice without kernels (sv_host_feed_probe): host_slice's
// staging loop -- chunks of stage_chunk() with the ramp, packed into the
// slot's two pinned slots by the pack pool, and with `upload` copied up on
// the H2D stream, a slot reused once its copy is done -- and nothing else.
// staging_node: NUMA node of the first pinned slot's pages.
int feed_slice(Device& D, const HostIn& in, size_t n, int upload, int* staging_node) {
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  int rc;
  if ((rc = ready_locked(D))) return rc;
  const size_t chunk = std::min(n, stage_chunk());
  // (the slots' `busy` flags belong to host_slice's pending verdict copies:
  // the probe tracks its own uploads, and leaves nothing in flight on any
  // return -- the copy stream is drained before an error is reported)
  bool pending[2] = {false, false};
  auto drain = [&] { (void)hipStreamSynchronize(D.h2d); };
  size_t m = 0;
  for (size_t lo = 0, c = 0; lo < n; lo += m, ++c) {
    Stage& s = D.st[c & 1];
    if (pending[c & 1]) {
      const hipError_t e = hipEventSynchronize(s.up);
      pending[c & 1] = false;
      if (e != hipSuccess) {
        drain();
        return hip_fail(e, "feed probe: upload");
      }
    }
    m = n <= chunk ? n : chunk_len(c, chunk, n - lo);
    size_t msg_total;
    const Image im = image_of(in, lo, m, &msg_total);
    if ((rc = s.h_in.ensure(im.bytes)) || (upload && (rc = s.d_in.ensure(im.bytes)))) {
      drain();
      return rc;
    }
    pack(in, lo, m, im, (uint8_t*)s.h_in.p);
    if (upload) {
      hipError_t e = hipMemcpyAsync(s.d_in.p, s.h_in.p, im.bytes, hipMemcpyHostToDevice, D.h2d);
      if (e == hipSuccess) e = hipEventRecord(s.up, D.h2d);
      if (e != hipSuccess) {
        drain();
        return hip_fail(e, "feed probe: upload");
      }
      pending[c & 1] = true;
    }
  }
  SV_HIP(hipStreamSynchronize(D.h2d));
  if (staging_node) *staging_node = page_numa_node(D.st[0].h_in.p);
  return SV_OK;
}

// ------------------------------------------------------------ latency lane
std::atomic<size_t> g_key_cap{~(size_t)0};  // sv_set_key_cache (~0: SV_KEY_CACHE or the default)
size_t key_cache_cap() {
  const size_t v = g_key_cap.load();
  return v != ~(size_t)0 ? v : env_size("SV_KEY_CACHE", 1024);
}
// keys admitted for a table build per batch (a flood of fresh keys costs at
// most this many ~0.3 ms builds on the low-priority stream per batch)
constexpr size_t kMaxBuildsPerBatch = 256;

void lat_drop_builds(LatLane& L) {
  for (auto& b : L.inflight) {
    (void)hipEventDestroy(b.uploaded);
    (void)hipEventDestroy(b.done);
  }
  L.inflight.clear();
}

// Caller holds L.mu and has set the device.
// A context's quad workspace of at least `bytes`; growing it frees the old
// one, so the work queued on the context (a device-API batch) drains first.
int lat_ws(LatCtx& c, size_t bytes) {
  if (bytes > c.ws.cap) SV_HIP(hipStreamSynchronize(c.stream));  // (never free under a running kernel)
  return c.ws.ensure(bytes);
}

// Every batch queued on the lane's verify streams has completed.
void lat_sync(LatLane& L) {
  for (int k = 0; k < L.nctx; ++k) {
    if (L.ctx[k].stream) (void)hipStreamSynchronize(L.ctx[k].stream);
    if (L.ctx[k].hstream) (void)hipStreamSynchronize(L.ctx[k].hstream);
  }
}

// (no batch holds a context: the API's teardown guard has drained the calls)
void release_lat(LatLane& L) {
  if (!L.ready) return;
  lat_sync(L);
  (void)hipStreamSynchronize(L.build);
  lat_drop_builds(L);
  for (auto& pr : L.pending) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  L.pending.clear();
  L.pending_n.clear();
  for (LatCtx& c : L.ctx) {
    c.h_in.release(); c.h_out.release(); c.z_out.release(); c.z_keys.release(); c.z_stat.release();
    c.d_in.release(); c.d_out.release(); c.d_keys.release(); c.ws.release();
    if (c.done) (void)hipEventDestroy(c.done);
    if (c.keys_down) (void)hipEventDestroy(c.keys_down);
    if (c.ev) (void)hipEventDestroy(c.ev);
    if (c.dev_done) (void)hipEventDestroy(c.dev_done);
    if (c.stream) (void)hipStreamDestroy(c.stream);
    if (c.hstream) (void)hipStreamDestroy(c.hstream);
    c.done = c.keys_down = c.ev = c.dev_done = nullptr;
    c.stream = c.hstream = nullptr;
    c.busy = false;
  }
  L.h_build.release();
  L.d_build.release();
  L.ktab.release(); L.kstat.release();
  if (L.ctab) (void)hipFree(L.ctab);
  L.ctab = nullptr;
  if (L.ev_lat) (void)hipEventDestroy(L.ev_lat);
  L.ev_lat = nullptr;
  if (L.build) (void)hipStreamDestroy(L.build);
  L.build = nullptr;
  L.index.reset(0);
  L.cap = 0;
  L.ready = false;
}

// Creates the lane (caller holds D.lat.mu, device set).  Lock order: lat.mu
// before D.mu (the slot's base-point tables, which the octet kernel reads,
// are created under D.mu and immutable afterwards).
int lat_ready(Device& D) {
  LatLane& L = D.lat;
  if (L.ready) return SV_OK;
  int rc;
  {
    std::lock_guard<std::mutex> g(D.mu);
    if ((rc = ready_locked(D))) return rc;
  }
  int least = 0, greatest = 0;
  SV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  L.nctx = (int)std::min<size_t>(kLatCtxMax, std::max<size_t>(1, env_size("SV_LAT_CONTEXTS", 2)));
  L.ready = true;  // (release_lat cleans up whatever exists from here on)
  hipError_t e = hipSuccess;
  for (int k = 0; k < L.nctx && e == hipSuccess; ++k) {
    LatCtx& c = L.ctx[k];
    c.z_out.mapped = c.z_keys.mapped = c.z_stat.mapped = true;
    c.h_in.mapped = true;  // (the kernels read it in place: lat_in_place)
    e = hipStreamCreateWithPriority(&c.stream, hipStreamNonBlocking, greatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c.hstream, hipStreamNonBlocking, greatest);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c.keys_down, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c.ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c.dev_done, hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipStreamCreateWithPriority(&L.build, hipStreamNonBlocking, least);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&L.ev_lat, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&L.ctab, sv_comb_btab_bytes());
  if (e == hipSuccess) e = sv_launch_comb_btab((uint32_t*)L.ctab, L.ctx[0].stream);
  if (e == hipSuccess) e = hipStreamSynchronize(L.ctx[0].stream);
  if (e != hipSuccess) {
    release_lat(L);
    return hip_fail(e, "latency lane init");
  }
  const size_t build_bytes = kMaxBuildsPerBatch * 36;
  if ((rc = L.h_build.ensure(build_bytes)) || (rc = L.d_build.ensure(build_bytes))) {
    release_lat(L);
    return rc;
  }
  return SV_OK;
}

// Sizes the key cache to key_cache_cap() (caller holds L.mu, device set).  An
// allocation failure leaves the cache off: the octet kernel needs no tables.
void lat_cache_ready(LatLane& L) {
  const size_t cap = key_cache_cap();
  if (cap == L.cap) return;
  lat_sync(L);  // (no queued kernel reads the tables; a batch past its launch only copies out)
  (void)hipStreamSynchronize(L.build);
  lat_drop_builds(L);
  L.ktab.release();
  L.kstat.release();
  L.index.reset(0);
  L.cap = 0;
  if (cap == 0) return;
  if (L.ktab.ensure(cap * sv_key_slot_bytes()) != SV_OK || L.kstat.ensure(cap * 4) != SV_OK) {
    L.ktab.release();
    L.kstat.release();
    return;
  }
  L.index.reset(cap);
  L.cap = cap;
}

// Promotes the slots of finished builds to READY.
void lat_poll(LatLane& L) {
  while (!L.inflight.empty()) {
    LatLane::Build& b = L.inflight.front();
    const hipError_t q = hipEventQuery(b.done);
    if (q == hipErrorNotReady) break;
    for (int32_t s : b.slots) {
      if (q == hipSuccess) L.index.set_ready(s, b.gen);
      else L.index.drop(s, b.gen);
    }
    (void)hipEventDestroy(b.uploaded);
    (void)hipEventDestroy(b.done);
    L.inflight.pop_front();
  }
}

// Brackets the next launch on the lane's stream with timing events
// (sv_timing_enable); lat_timing_end after the launch.
int lat_timing_begin(hipStream_t st, hipEvent_t* e0) {
  *e0 = nullptr;
  if (!g_timing.load()) return SV_OK;
  SV_HIP(hipEventCreate(e0));
  SV_HIP(hipEventRecord(*e0, st));
  return SV_OK;
}
int lat_timing_end(LatLane& L, hipStream_t st, hipEvent_t e0, uint64_t n) {
  if (!e0) return SV_OK;
  hipEvent_t e1 = nullptr;
  SV_HIP(hipEventCreate(&e1));
  SV_HIP(hipEventRecord(e1, st));
  L.pending.emplace_back(e0, e1);
  L.pending_n.push_back(n);
  return SV_OK;
}
int lat_harvest(LatLane& L) {
  for (size_t k = 0; k < L.pending.size(); ++k) {
    SV_HIP(hipEventSynchronize(L.pending[k].second));
    float ms = 0;
    SV_HIP(hipEventElapsedTime(&ms, L.pending[k].first, L.pending[k].second));
    L.total_ms += ms;
    L.launches += 1;
    L.sigs += L.pending_n[k];
    (void)hipEventDestroy(L.pending[k].first);
    (void)hipEventDestroy(L.pending[k].second);
  }
  L.pending.clear();
  L.pending_n.clear();
  return SV_OK;
}

// Looks up every key of the batch: true iff all are READY (L.kslots holds
// their slots).  Keys admitted on this sighting are inserted as BUILDING and
// listed in fresh_pk / fresh_slot for lat_build.
bool lat_plan(LatLane& L, const HostIn& in, size_t n) {
  L.fresh_pk.clear();
  L.fresh_slot.clear();
  if (!L.cap) return false;
  const uint64_t now = ++L.tick;
  L.kslots.resize(n);
  bool warm = true;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* pk = in.pkp(i);
    int32_t s = L.index.find(pk);
    if (s >= 0) {
      L.index.touch(s, now);
      if (L.index.state(s) == sv::KeyIndex::READY) {
        L.kslots[i] = (uint32_t)s;
        continue;
      }
      warm = false;  // (its build is still running)
      continue;
    }
    warm = false;
    if (L.fresh_pk.size() < kMaxBuildsPerBatch && L.index.admit(pk)) {
      bool ev = false;
      s = L.index.insert(pk, L.next_gen, now, &ev);
      if (s >= 0) {
        L.fresh_pk.push_back(pk);
        L.fresh_slot.push_back(s);
        if (ev) ++L.evicted;
      }
    }
  }
  return warm;
}

// Queues the table build of the keys lat_plan admitted, after everything
// already on the lane's verify streams (a build may overwrite an evicted slot
// that an earlier comb kernel reads, on either context).  A failed build only
// leaves its keys uncached.
void lat_build(LatLane& L) {
  const size_t k = L.fresh_pk.size();
  if (!k) return;
  const uint64_t gen = L.next_gen++;
  LatLane::Build b;
  b.gen = gen;
  b.uploaded = b.done = nullptr;
  b.slots = L.fresh_slot;
  hipError_t e = hipSuccess;
  // the previous build's upload has left the pinned buffer before it is rewritten
  if (!L.inflight.empty()) e = hipEventSynchronize(L.inflight.back().uploaded);
  uint8_t* h = (uint8_t*)L.h_build.p;
  if (e == hipSuccess) {
    for (size_t i = 0; i < k; ++i) {
      std::memcpy(h + 32 * i, L.fresh_pk[i], 32);
      const uint32_t s = (uint32_t)L.fresh_slot[i];
      std::memcpy(h + 32 * k + 4 * i, &s, 4);
    }
    e = hipEventCreateWithFlags(&b.uploaded, hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&b.done, hipEventDisableTiming);
  for (int c = 0; c < L.nctx && e == hipSuccess; ++c) {
    e = hipEventRecord(L.ctx[c].ev, L.ctx[c].stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(L.build, L.ctx[c].ev, 0);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(L.d_build.p, h, 36 * k, hipMemcpyHostToDevice, L.build);
  if (e == hipSuccess) e = hipEventRecord(b.uploaded, L.build);
  if (e == hipSuccess)
    e = sv_launch_keytab(L.d_build.p, (const uint32_t*)((uint8_t*)L.d_build.p + 32 * k), (uint32_t)k,
                         (uint32_t*)L.ktab.p, (uint32_t*)L.kstat.p, L.build);
  if (e == hipSuccess) e = hipEventRecord(b.done, L.build);
  if (e != hipSuccess) {
    // (an upload already queued completes on its own; the slots stay uncached)
    if (b.uploaded) (void)hipEventSynchronize(b.uploaded);
    for (int32_t s : b.slots) L.index.drop(s, gen);
    if (b.uploaded) (void)hipEventDestroy(b.uploaded);
    if (b.done) (void)hipEventDestroy(b.done);
    return;
  }
  L.built += k;
  L.inflight.push_back(std::move(b));
}

// Zero-copy verdicts (SV_LAT_ZERO_COPY, default on): the kernel of a
// verdict-only latency batch writes its verdicts straight into mapped pinned
// memory, which saves the blit dispatch of a D2H copy (~6 us of a ~0.12 ms
// batch, tools/gpu/api_probe.hip).

std::atomic<int> g_lat_zc{-1};
bool lat_zero_copy() {
  int v = g_lat_zc.load();
  if (v < 0) {
    const char* e = getenv("SV_LAT_ZERO_COPY");
    v = (e && e[0] == '0') ? 0 : 1;
    g_lat_zc.store(v);
  }
  return v != 0;
}

// Input read in place (SV_LAT_ZC_IN, default on; 0: one staged H2D copy):
// the kernels read the packed image straight from mapped pinned memory.  The
// kernel runs longer (+10 us at 1k signatures, reads over the fabric) but the
// H2D dispatch is gone: p50 1000 / 4096 / 12288 warm 0.116 / 0.261 / 0.551 ->
// 0.112 / 0.253 / 0.508 ms, and a staged copy queues behind a bulk call's
// chunk upload (up to ~0.8 ms per 32 MB chunk): p99 under the 2^22 host
// batch 0.61-0.86 -> 0.22 ms (profiles/r04/isolation/).
// Cold latency batches of at most this many signatures take the three-wave
// octet kernel (SV_OCT_HI_MAX; 0: never).  Measured (profiles/r05/octet_hi/):
// p50 1k 0.241-0.245 -> 0.221-0.226 ms, 2k 0.256 -> 0.240, 4k 0.378 -> 0.375;
// at 6k the third wave's repeated doublings cost more than they save (0.50
// against 0.42-0.44 ms).
size_t oct_hi_max() {
  static const size_t v = env_size("SV_OCT_HI_MAX", 4096);
  return v;
}
// Above this many signatures (more octet workgroups than CUs) the third wave
// takes W / 4 of the windows instead of W / 6 (SV_KP_OCT_HI_WIDE): 4k p50
// 0.372 -> 0.352 ms, where 1k and 2k are 2-5 us faster with W / 6
// (profiles/r05/octet_hi/cold_r5an_flags_divisors.jsonl, cold_r5ao_flags.jsonl).
size_t oct_hi_wide_min() {
  static const size_t v = env_size("SV_OCT_HI_WIDE_MIN", 2048);
  return v;
}

bool lat_in_place() {
  static const bool b = env_size("SV_LAT_ZC_IN", 1) != 0;
  return b;
}

std::atomic<int> g_lat_trace{-1};
bool lat_trace() {
  int v = g_lat_trace.load();
  if (v < 0) {
    v = getenv("SV_LAT_TRACE") ? 1 : 0;
    g_lat_trace.store(v);
  }
  return v != 0;
}

// Host-side stages of this thread's last latency-lane batch (sv_lat_last_trace).
thread_local std::array<double, 8> t_lat_last{};

// What a launched latency batch leaves for its completion (lat_finish).
struct LatPending {
  size_t n = 0;
  bool warm = false, early = false, zc = false, zk = false, in_place = false;
  const uint8_t* vho = nullptr;  // its verdicts on the host, once `done`
  const volatile uint32_t* stat = nullptr;  // its kernel's failure word, once `done` (nullptr: none)
  uint8_t* kho = nullptr;        // its cache keys on the host, once `keys_down`
  std::chrono::steady_clock::time_point t0, t1, t_up, t_k, t_down, t_b;
};

// One latency-bound host batch on context c of the slot's latency lane,
// launched (caller holds L.mu): pinned image (+ the key slots when warm) read
// in place (or one H2D), [hash kernel, keys D2H], the comb kernel (every key
// cached) or the octet / quad kernel, one D2H; then the key-table builds it
// admitted.  lat_finish waits and copies out, without the lock.
int lat_launch_locked(Device& D, LatCtx& c, const HostIn& in, size_t n, uint8_t* verdict, uint8_t* keys,
                      const KeysCb& kcb, LatPending& pd) {
  LatLane& L = D.lat;
  int rc;
  pd.t0 = std::chrono::steady_clock::now();
  pd.n = n;
  D.lat_last_ns.store(now_ns(), std::memory_order_relaxed);
  lat_cache_ready(L);
  lat_poll(L);
  const uint32_t dbg = g_dbg.load() & kKernelDbgMask;
  // (the lattice test knobs select the octet kernel's code paths)
  const bool warm = lat_plan(L, in, n) && verdict && dbg == 0;
  pd.warm = warm;
  size_t msg_total;
  const Image im = image_of(in, 0, n, &msg_total);
  const size_t o_ks = (im.bytes + 3) & ~(size_t)3;
  const size_t in_bytes = warm ? o_ks + 4 * n : im.bytes;
  // zero-copy outputs: verdicts (and a keyed batch's cache keys) written by
  // the kernels straight into mapped pinned memory, no D2H blit
  const bool zc = verdict && lat_zero_copy();
  const bool zk = keys && lat_zero_copy();
  pd.zc = zc;
  pd.zk = zk;
  const size_t out_per = (verdict && !zc ? 1 : 0) + (keys && !zk ? 32 : 0);
  const bool in_place = lat_in_place();
  pd.in_place = in_place;
  if ((rc = c.h_in.ensure(in_bytes)) || (!in_place && (rc = c.d_in.ensure(in_bytes)))) return rc;
  if (zc && (rc = c.z_out.ensure(n))) return rc;
  if (zk && (rc = c.z_keys.ensure(32 * n))) return rc;
  if (out_per && (rc = c.h_out.ensure(out_per * n))) return rc;
  if (verdict && !zc && (rc = c.d_out.ensure(n))) return rc;
  if (keys && !zk && (rc = c.d_keys.ensure(32 * n))) return rc;
  uint8_t* h = (uint8_t*)c.h_in.p;
  pack(in, 0, n, im, h);
  if (warm) std::memcpy(h + o_ks, L.kslots.data(), 4 * n);
  pd.t1 = std::chrono::steady_clock::now();
  if (!in_place) SV_HIP(hipMemcpyAsync(c.d_in.p, h, in_bytes, hipMemcpyHostToDevice, c.stream));
  pd.t_up = std::chrono::steady_clock::now();
  uint8_t* d = (uint8_t*)(in_place ? c.h_in.dp : c.d_in.p);
  void* d_verdict = zc ? c.z_out.dp : c.d_out.p;
  void* d_keys = zk ? c.z_keys.dp : c.d_keys.p;
  const uint64_t* d_off = im.var ? (const uint64_t*)(d + im.o_off) : nullptr;
  const uint32_t* d_len = im.var ? (const uint32_t*)(d + im.o_len) : nullptr;
  uint8_t* ho = (uint8_t*)c.h_out.p;
  pd.vho = zc ? (const uint8_t*)c.z_out.p : ho;                  // verdicts on the host
  pd.kho = zk ? (uint8_t*)c.z_keys.p : ho + (verdict && !zc ? n : 0);  // keys on the host
  pd.early = kcb && keys && verdict;
  pd.t_k = pd.t_up;
  // A keyed batch's cache keys: with the image read in place, on the
  // context's second stream, beside the verify kernel (the caller's cache
  // walk then overlaps the verification); the windows are staged in LDS (kind 2).
  const bool kside = keys && in_place;
  hipStream_t ks = kside ? c.hstream : c.stream;
  if (keys) {
    SV_HIP(sv_launch_hash(in_place ? 2 : 0, D.grid * 2, d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, n,
                          d_keys, ks));
    if (!zk) SV_HIP(hipMemcpyAsync(pd.kho, c.d_keys.p, 32 * n, hipMemcpyDeviceToHost, ks));
    SV_HIP(hipEventRecord(c.keys_down, ks));
  }
  if (verdict) {
    const int mode = im.var ? 1 : (in.fixed == 32 ? 0 : 2);
    hipEvent_t e0;
    if ((rc = lat_timing_begin(c.stream, &e0))) return rc;
    // (while bulk work runs, only the 1-signature-per-wave geometry fits the
    // slot a shared-mode bulk launch leaves free on each CU)
    const bool bulk_busy = hipStreamQuery(D.stream) == hipErrorNotReady;
    if (warm)
      SV_HIP(sv_launch_comb(mode, bulk_busy ? 1 : sv_comb_spw(n, D.cus), d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, n,
                            d_verdict, (const uint32_t*)(d + o_ks), (const uint32_t*)L.ktab.p,
                            (const uint32_t*)L.kstat.p, (const uint32_t*)L.ctab, c.stream));
    else if (n > kOctetMax && !(g_dbg.load() & SV_DBG_NO_QUAD)) {
      if ((rc = lat_ws(c, sv_verify_ws_bytes(kGeomQuad, 0, n)))) return rc;
      SV_HIP(sv_launch_verify(mode, kGeomQuad, 1, d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, n, d_verdict,
                              nullptr, c.ws.p, D.btab, dbg | SV_KP_LAT, 0, nullptr, nullptr, c.stream));
    } else {
      // (a third wave per workgroup takes the chains' top windows while no
      // bulk work runs: its larger workgroup would not fit the slot a
      // shared-mode bulk launch leaves free)
      const uint32_t hi = (!bulk_busy && n <= oct_hi_max())
                              ? SV_KP_OCT_HI | (n > oct_hi_wide_min() ? SV_KP_OCT_HI_WIDE : 0u)
                              : 0u;
      // (the three-wave kernel's hand-overs are bounded waits: it reports one
      // that ran out in this word, and lat_finish turns that into an error)
      uint32_t* stat = nullptr;
      if (hi) {
        if ((rc = c.z_stat.ensure(sizeof(uint32_t)))) return rc;
        *(volatile uint32_t*)c.z_stat.p = 0;
        stat = (uint32_t*)c.z_stat.dp;
        pd.stat = (const volatile uint32_t*)c.z_stat.p;
      }
      SV_HIP(sv_launch_verify(mode, SV_PATH_LATENCY, 1, d, d + im.o_sig, d + im.o_msg, d_off, d_len, in.fixed, n,
                              d_verdict, nullptr, nullptr, D.btab, dbg | hi, 0, nullptr, stat, c.stream));
    }
    if ((rc = lat_timing_end(L, c.stream, e0, n))) return rc;
    pd.t_k = std::chrono::steady_clock::now();
    if (!zc) SV_HIP(hipMemcpyAsync(ho, c.d_out.p, n, hipMemcpyDeviceToHost, c.stream));
  }
  SV_HIP(hipEventRecord(c.done, c.stream));
  pd.t_down = std::chrono::steady_clock::now();
  lat_build(L);  // (after the verify work: a build waits for it on the device)
  pd.t_b = std::chrono::steady_clock::now();
  if (warm) ++L.warm;
  else ++L.cold;
  return SV_OK;
}

// The rest of a launched batch, without the lane's lock: the keys-ready
// callback, the wait, the copy-out.
int lat_finish(LatCtx& c, const LatPending& pd, uint8_t* verdict, uint8_t* keys, const KeysCb& kcb, bool* cb_done) {
  const size_t n = pd.n;
  if (pd.early) {
    SV_HIP(hipEventSynchronize(c.keys_down));
    std::memcpy(keys, pd.kho, 32 * n);
    kcb(n);
    *cb_done = true;
  }
  SV_HIP(hipEventSynchronize(c.done));
  if (keys && !pd.early) SV_HIP(hipEventSynchronize(c.keys_down));
  // An in-kernel failure: the kernel wrote fail-closed rejects, which are not
  // verdicts.  The batch errs (include/stellar_sigverify.h: an error is never
  // a reject), so a caller re-verifies it instead of caching false
  // (/root/reference/src/crypto/SecretKey.cpp:464-466 caches what it gets).
  if (pd.stat && *pd.stat != 0)
    return fail(SV_ERR_KERNEL, "in-kernel failure " + std::to_string(*pd.stat) +
                                   " (three-wave octet kernel: a hand-over wait ran out); verdicts discarded");
  if (verdict) std::memcpy(verdict, pd.vho, n);
  if (keys && !pd.early) std::memcpy(keys, pd.kho, 32 * n);
  const auto t2 = std::chrono::steady_clock::now();
  auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
  };
  t_lat_last = {us(pd.t0, pd.t1), us(pd.t1, pd.t_up), us(pd.t_up, pd.t_k), us(pd.t_k, pd.t_down),
                us(pd.t_down, pd.t_b), us(pd.t_b, t2), us(pd.t0, t2), pd.warm ? 1.0 : 0.0};
  if (lat_trace()) {
    fprintf(stderr,
            "SV_LAT_TRACE n=%zu %s plan+pack %.1f us | h2d call %.1f launch %.1f d2h+rec %.1f build %.1f sync %.1f"
            " | device %.1f us @%.1f%s\n",
            n, pd.warm ? "warm" : "cold", us(pd.t0, pd.t1), us(pd.t1, pd.t_up), us(pd.t_up, pd.t_k),
            us(pd.t_k, pd.t_down), us(pd.t_down, pd.t_b), us(pd.t_b, t2), us(pd.t1, t2),
            trace_abs_us() - us(pd.t0, t2), pd.in_place ? " in place" : "");
  }
  return SV_OK;
}

int lat_slice(Device& D, const HostIn& in, size_t n, uint8_t* verdict, uint8_t* keys, const KeysCb& kcb,
              bool* cb_done) {
  LatLane& L = D.lat;
  std::unique_lock<std::mutex> lk(L.mu);
  SV_HIP(hipSetDevice(D.phys));
  int rc;
  if ((rc = lat_ready(D))) return rc;
  // a free context (every one busy: wait for the first batch to finish)
  LatCtx* c = nullptr;
  L.freed.wait(lk, [&] {
    for (int k = 0; k < L.nctx; ++k)
      if (!L.ctx[k].busy) {
        c = &L.ctx[k];
        return true;
      }
    return false;
  });
  c->busy = true;
  // Releases the context however this call leaves (an error return, or an
  // exception from the keys-ready callback inside lat_finish): unless the
  // batch completed, its streams are drained first, so the next batch on the
  // context never overwrites staging a kernel still reads.  (notify_all: a
  // device-API caller waiting here takes no context, so a single wake-up
  // could land on it and leave a host batch asleep beside a free one.)
  struct Release {
    LatLane& L;
    LatCtx* c;
    std::unique_lock<std::mutex>& lk;
    bool completed = false;
    ~Release() {
      if (!completed) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->hstream);
      }
      if (!lk.owns_lock()) lk.lock();
      c->busy = false;
      L.freed.notify_all();
    }
  } release{L, c, lk};
  LatPending pd;
  if ((rc = lat_launch_locked(D, *c, in, n, verdict, keys, kcb, pd))) return rc;
  lk.unlock();
  rc = lat_finish(*c, pd, verdict, keys, kcb, cb_done);
  release.completed = rc == SV_OK;
  return rc;
}

// SHA-256 of a host slice of byte strings on one slot.
int sha_slice(Device& D, const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n, uint8_t* out) {
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  int rc;
  if ((rc = ready_locked(D))) return rc;
  size_t total = 0;
  for (size_t i = 0; i < n; ++i) total += len[i];
  const size_t o_len = 8 * n, o_msg = 12 * n, bytes = o_msg + std::max<size_t>(total, 1);
  if ((rc = D.h_sha.ensure(bytes)) || (rc = D.msg.ensure(bytes)) || (rc = D.keys.ensure(n * 32))) return rc;
  uint8_t* h = (uint8_t*)D.h_sha.p;
  uint64_t* offs = (uint64_t*)h;
  size_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    offs[i] = pos;
    if (len[i]) std::memcpy(h + o_msg + pos, data + off[i], len[i]);
    pos += len[i];
  }
  std::memcpy(h + o_len, len, 4 * n);
  SV_HIP(hipMemcpyAsync(D.msg.p, h, bytes, hipMemcpyHostToDevice, D.stream));
  uint8_t* d = (uint8_t*)D.msg.p;
  SV_HIP(sv_launch_hash(1, D.grid * 2, nullptr, nullptr, d + o_msg, (const uint64_t*)d, (const uint32_t*)(d + o_len),
                        0, n, D.keys.p, D.stream));
  SV_HIP(hipMemcpyAsync(out, D.keys.p, n * 32, hipMemcpyDeviceToHost, D.stream));
  SV_HIP(hipStreamSynchronize(D.stream));
  return SV_OK;
}

int check_opts(const sv_opts* opts) {
  if (opts && (opts->struct_size < sizeof(sv_opts) || (opts->flags & ~SV_FLAG_PATH_MASK) != 0 ||
               (opts->flags & SV_FLAG_PATH_MASK) == SV_FLAG_PATH_MASK))
    return fail(SV_ERR_INVALID_ARG, "bad sv_opts");
  return SV_OK;
}

// The slots a host-buffer batch of n runs on: one named slot, or contiguous
// slices over up to max_devices slots, each slice >= the minimum shard.
int select_devices(const sv_opts* opts, size_t n, std::vector<Device*>& out) {
  int rc;
  if ((rc = check_opts(opts))) return rc;
  const int dev = opts ? opts->device : -1;
  const uint32_t maxd = opts ? opts->max_devices : 0;
  if (dev >= 0) {
    if (dev >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
    out.push_back(g_devs[dev]);
    return SV_OK;
  }
  size_t G = g_devs.size();
  if (maxd) G = std::min<size_t>(G, maxd);
  G = std::max<size_t>(1, std::min<size_t>(G, n / std::max<size_t>(1, min_shard())));
  if (G == 1) {
    // single-slot calls rotate over the slots so concurrent callers spread out
    const size_t pool_n = maxd ? std::min<size_t>(g_devs.size(), maxd) : g_devs.size();
    out.push_back(g_devs[(size_t)(g_rr.fetch_add(1) % pool_n)]);
    return SV_OK;
  }
  for (size_t g = 0; g < G; ++g) out.push_back(g_devs[g]);
  return SV_OK;
}

// Staging workers per slot (SV_SLOT_THREADS, default the usable CPUs, at
// most 8), and the pack parts one slot of a G-slot call uses: the usable CPUs
// split over the G slots (16 CPUs: 8 slots 2 each, 2 slots 8 each), so the
// call's packers never outnumber the CPUs however many slots it spans
// (profiles/r06/feed/: 2 fixed workers per slot fed 2 slots slower than one
// slot on the shared pool).
size_t slot_threads() {
  const size_t v = env_size("SV_SLOT_THREADS", 0);
  if (v) return std::min<size_t>(v, 64);
  return std::max<size_t>(1, std::min<size_t>(8, usable_cpus()));
}
size_t slot_pack_parts(size_t G) {
  return std::max<size_t>(1, std::min(slot_threads(), usable_cpus() / std::max<size_t>(1, G)));
}
// The slot's worker pool (created on first use).  Each worker pins itself to
// the CPUs of the GPU's NUMA node that this process may use, so its packs
// write pinned staging allocated on that node (SV_SLOT_NUMA=0: no pinning).
sv::Pool& slot_pool(Device& D) {
  std::lock_guard<std::mutex> g(D.spool_mu);
  if (!D.spool) {
    if (D.numa == -2) D.numa = gpu_numa_node(D.phys);
    std::vector<int> cpus = env_size("SV_SLOT_NUMA", 1) ? node_cpus(D.numa) : std::vector<int>();
    D.numa_cpus = cpus.size();
    const int phys = D.phys;
    D.spool.reset(new sv::Pool((unsigned)slot_threads(), [cpus, phys] {
      if (!cpus.empty()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : cpus) CPU_SET(c, &set);
        (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
      }
      (void)hipSetDevice(phys);
    }));
  }
  return *D.spool;
}

// Runs fn(slot, lo, hi) for contiguous slices [g*n/G, (g+1)*n/G); the first
// failing slot's error is reported.  G > 1: each slice on its slot's own
// workers (slot_pool), which also pack it, while this thread only waits --
// not as tasks on the shared pool, where G slot tasks blocked in event waits
// would leave their packs one spare thread (VERDICT r5 missing #2).
template <class F>
int shard(const std::vector<Device*>& devs, size_t n, F fn) {
  const size_t G = devs.size();
  if (G == 1) return fn(*devs[0], (size_t)0, n);
  std::vector<int> rcs(G, SV_OK);
  std::vector<std::string> errs(G);
  std::mutex mu;
  std::condition_variable cv;
  size_t left = 0;
  std::vector<sv::Pool*> pools(G);
  for (size_t g = 0; g < G; ++g) pools[g] = &slot_pool(*devs[g]);
  for (size_t g = 0; g < G; ++g) {
    const size_t lo = g * n / G, hi = (g + 1) * n / G;
    if (hi == lo) continue;
    {
      std::lock_guard<std::mutex> lk(mu);
      ++left;
    }
    const int depth = t_life_depth;
    const size_t parts = slot_pack_parts(G);
    pools[g]->post([&, g, lo, hi, depth, parts] {
      // (inside the caller's entry point: its lifetime lock is held until the
      // join below, so the worker counts as inside the engine)
      t_life_depth = depth;
      t_pack_pool = pools[g];
      t_pack_parts = parts;
      int rc;
      try {
        rc = fn(*devs[g], lo, hi);
      } catch (...) {
        rc = fail(SV_ERR_INVALID_ARG, "exception in a device slot's worker");
      }
      t_pack_pool = nullptr;
      t_pack_parts = 0;
      t_life_depth = 0;
      std::lock_guard<std::mutex> lk(mu);
      rcs[g] = rc;
      if (rc) errs[g] = t_err;
      if (--left == 0) cv.notify_all();
    });
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return left == 0; });
  }
  for (size_t g = 0; g < G; ++g)
    if (rcs[g]) return fail(rcs[g], "device slot " + std::to_string(devs[g]->slot) + ": " + errs[g]);
  return SV_OK;
}

int check_msgs(const HostIn& in, size_t n) {
  if (in.gather()) {
    if (!in.psig || !in.len) return fail(SV_ERR_INVALID_ARG, "null pointer array");
    for (size_t i = 0; i < n; ++i)
      if (!in.ppk[i] || !in.psig[i] || (in.len[i] && (!in.pmsg || !in.pmsg[i])))
        return fail(SV_ERR_INVALID_ARG, "null item pointer");
    return SV_OK;
  }
  if (!in.pk || !in.sig) return fail(SV_ERR_INVALID_ARG, "null buffer");
  if (in.fixed == 0 && (!in.off || !in.len)) return fail(SV_ERR_INVALID_ARG, "null msg_off/msg_len");
  if (!in.msg) {
    bool any = in.fixed != 0;
    for (size_t i = 0; i < n && !any; ++i) any = in.len[i] != 0;
    if (any) return fail(SV_ERR_INVALID_ARG, "null msg");
  }
  return SV_OK;
}

// Test-only knobs are enabled by SV_TEST_KNOBS=1 in the process environment
// (tests/conftest.py, profiling tools); a production process never sets it.
bool test_knobs_enabled() {
  const char* v = getenv("SV_TEST_KNOBS");
  return v && v[0] == '1' && v[1] == 0;
}

int debug_fail() {
  if (g_dbg.load() & SV_DBG_FAIL) return fail(SV_ERR_HIP, "injected device error (sv_set_debug_flags SV_DBG_FAIL)");
  return SV_OK;
}

// A variable-length batch whose messages all have one length L > 0 (tx
// contents hashes: every pair of a tx-set pre-pass) goes to the device as a
// fixed-length batch: messages packed at stride L (found by their offsets
// or pointers), no offset / length arrays in the image, and the kernels' fixed
// modes instead of an offset read before each message (measured: 50-110 us per
// call at 29k-50k signatures, tools/varlen_probe.py).  The scan stops at the
// first other length.
HostIn uniform_form(const HostIn& in, size_t n) {
  HostIn u = in;
  if (in.fixed || n == 0 || !in.len) return u;
  const uint32_t L = in.len[0];
  if (L == 0) return u;
  for (size_t i = 1; i < n; ++i)
    if (in.len[i] != L) return u;
  u.fixed = L;
  return u;
}

int verify_host(const HostIn& in, size_t n, uint8_t* verdict, uint8_t* keys, const sv_opts* opts,
                const KeysCb& kcb = KeysCb()) {
  if (n == 0) {
    int rc = check_opts(opts);
    if (rc == SV_OK && kcb) kcb(0);
    return rc;
  }
  if (!verdict && !keys) return fail(SV_ERR_INVALID_ARG, "null buffer");
  int rc = check_msgs(in, n);
  if (rc) return rc;
  const HostIn u = uniform_form(in, n);
  if ((rc = debug_fail())) return rc;
  if ((rc = ensure_init())) return rc;
  std::vector<Device*> devs;
  if ((rc = select_devices(opts, n, devs))) return rc;
  const int path = path_from_flags(opts ? opts->flags : 0u);
  bool cb_done = false;
  if (devs.size() == 1) {
    // latency-bound batches (one latency launch) take the slot's latency lane
    // (at most kQuickMax: an explicit latency-path call of up to a staging
    // chunk would otherwise grow each lane context's pinned image and quad
    // workspace to that size for the life of the lane; a larger one runs the
    // latency kernels on the slot's bulk stream instead)
    if (resolve_path(path, n) == SV_PATH_LATENCY && n <= std::min<size_t>(stage_chunk(), kQuickMax))
      rc = lat_slice(*devs[0], u, n, verdict, keys, kcb, &cb_done);
    else
      rc = host_slice(*devs[0], u, n, verdict, keys, path, kcb, &cb_done);
  } else {
    rc = shard(devs, n, [&](Device& D, size_t lo, size_t hi) {
      return host_slice(D, u.sub(lo), hi - lo, verdict ? verdict + lo : nullptr, keys ? keys + 32 * lo : nullptr,
                        path);
    });
  }
  if (rc == SV_OK && kcb && !cb_done) kcb(n);  // (keys complete; no overlap possible)
  return rc;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Releases every slot (caller holds g_mu).  Lock order: lat.mu, then mu.
void shutdown_locked() {
  for (Device* D : g_devs) {
    std::lock_guard<std::mutex> gl(D->lat.mu);
    std::lock_guard<std::mutex> gd(D->mu);
    if (D->lat.ready) {
      (void)hipSetDevice(D->phys);
      release_lat(D->lat);
    }
    release_device(*D);
  }
  for (Device* D : g_devs) delete D;
  g_devs.clear();
  g_inited = false;
}

// Lifetime of the slot table.  Every entry point that reaches a Device holds
// g_life shared for the whole call (LifeGuard); sv_shutdown and
// sv_set_device_map take it exclusively, so no Device is deleted while a call
// (or the helper-pool work it fans out) still uses it.  The reference's cache
// controls are likewise safe against concurrent verifySig (SecretKey.cpp
// :317-330, one mutex).  A thread takes it once however deep its entry points
// nest: re-acquiring a shared lock behind a queued writer would deadlock.
// Lock order: g_life, then g_mu, then a slot's lat.mu, then its mu.
// Writer-preferring: once a teardown waits, new calls queue behind it (glibc's
// rwlock, behind std::shared_mutex, prefers readers, so callers that keep a
// slot busy back to back would starve sv_set_device_map forever).
class LifeLock {
 public:
  void lock_shared() {
    std::unique_lock<std::mutex> l(m_);
    cv_.wait(l, [&] { return !writer_ && waiting_ == 0; });
    ++readers_;
  }
  void unlock_shared() {
    std::lock_guard<std::mutex> l(m_);
    if (--readers_ == 0 && waiting_ != 0) cv_.notify_all();
  }
  void lock() {
    std::unique_lock<std::mutex> l(m_);
    ++waiting_;
    cv_.wait(l, [&] { return !writer_ && readers_ == 0; });
    --waiting_;
    writer_ = true;
  }
  void unlock() {
    std::lock_guard<std::mutex> l(m_);
    writer_ = false;
    cv_.notify_all();
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int readers_ = 0, waiting_ = 0;
  bool writer_ = false;
};
LifeLock g_life;
struct LifeGuard {
  LifeGuard() {
    if (t_life_depth++ == 0) g_life.lock_shared();
  }
  ~LifeGuard() {
    if (--t_life_depth == 0) g_life.unlock_shared();
  }
  LifeGuard(const LifeGuard&) = delete;
  LifeGuard& operator=(const LifeGuard&) = delete;
};

Device* device_arg(int device) {
  if (device < 0 || device >= (int)g_devs.size()) return nullptr;
  return g_devs[device];
}

}  // namespace

extern "C" {

int sv_init(void) { return ensure_init(); }

void sv_shutdown(void) {
  if (t_life_depth != 0) {  // (from inside an engine call, e.g. a keys-ready callback: refused)
    (void)fail(SV_ERR_INVALID_ARG, "sv_shutdown called from inside an engine call: refused");
    return;
  }
  std::unique_lock<LifeLock> life(g_life);  // waits for every in-flight call
  std::lock_guard<std::mutex> g(g_mu);
  shutdown_locked();
}

int sv_set_device_map(const int* physical, int count) {
  if (count < 0 || (count > 0 && !physical)) return fail(SV_ERR_INVALID_ARG, "bad device map");
  if (t_life_depth != 0) return fail(SV_ERR_INVALID_ARG, "sv_set_device_map called from inside an engine call");
  // teardown and the new map in ONE critical section: a concurrent first use
  // cannot re-initialise with the old map in between; in-flight calls finish
  // first (g_life)
  std::unique_lock<LifeLock> life(g_life);
  std::lock_guard<std::mutex> g(g_mu);
  shutdown_locked();
  g_map.assign(physical, physical + count);
  int rc = init_locked();
  if (rc != SV_OK) {
    for (Device* D : g_devs) delete D;
    g_devs.clear();
    g_map.clear();
    g_inited = false;
  }
  return rc;
}

int sv_device_count(void) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  return (int)g_devs.size();
}

const char* sv_last_error_string(void) { return t_err.c_str(); }

const char* sv_version(void) {
  return "stellar-core_amd sigverify r6 (gfx950; ed25519 == libsodium-1.0.18 crypto_sign_verify_detached)";
}

int sv_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                            const uint32_t* msg_len, size_t n, uint8_t* verdict, const sv_opts* opts) {
  LifeGuard life_;
  HostIn in;
  in.pk = pk;
  in.sig = sig;
  in.msg = msg;
  in.off = msg_off;
  in.len = msg_len;
  return verify_host(in, n, verdict, nullptr, opts);
}

int sv_ed25519_verify_batch_fixed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_len,
                                  size_t n, uint8_t* verdict, const sv_opts* opts) {
  LifeGuard life_;
  if (msg_len == 0) {
    // zero-length messages: route through the variable-length path
    std::vector<uint64_t> off(n, 0);
    std::vector<uint32_t> len(n, 0);
    static const uint8_t dummy = 0;
    return sv_ed25519_verify_batch(pk, sig, &dummy, off.data(), len.data(), n, verdict, opts);
  }
  HostIn in;
  in.pk = pk;
  in.sig = sig;
  in.msg = msg;
  in.fixed = msg_len;
  return verify_host(in, n, verdict, nullptr, opts);
}

int sv_host_feed_probe(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_len, size_t n,
                       uint32_t max_devices, int upload, sv_feed_stats* out) {
  LifeGuard life_;
  if (!out || out->struct_size < sizeof(sv_feed_stats)) return fail(SV_ERR_INVALID_ARG, "bad sv_feed_stats");
  if (!pk || !sig || !msg || msg_len == 0 || n == 0) return fail(SV_ERR_INVALID_ARG, "bad arguments");
  int rc;
  if ((rc = ensure_init())) return rc;
  HostIn in;
  in.pk = pk;
  in.sig = sig;
  in.msg = msg;
  in.fixed = msg_len;
  sv_opts o{sizeof(sv_opts), -1, max_devices, 0};
  std::vector<Device*> devs;
  if ((rc = select_devices(&o, n, devs))) return rc;
  const size_t G = devs.size();
  std::vector<int> nodes(G, -1);
  const auto t0 = std::chrono::steady_clock::now();
  rc = shard(devs, n, [&](Device& D, size_t lo, size_t hi) {
    size_t g = 0;
    while (devs[g] != &D) ++g;
    return feed_slice(D, in.sub(lo), hi - lo, upload, &nodes[g]);
  });
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc) return rc;
  out->seconds = sec;
  out->slots = (uint32_t)G;
  out->threads_per_slot = (uint32_t)(G > 1 ? slot_pack_parts(G) : pool().size() + 1);
  out->usable_cpus = (uint32_t)usable_cpus();
  for (size_t g = 0; g < 16; ++g) {
    out->gpu_numa[g] = g < G ? (devs[g]->numa == -2 ? gpu_numa_node(devs[g]->phys) : devs[g]->numa) : -1;
    out->staging_numa[g] = g < G ? nodes[g] : -1;
    out->pinned_cpus[g] = g < G ? (uint32_t)devs[g]->numa_cpus : 0;
  }
  return SV_OK;
}

int sv_ed25519_verify_batch_gather(const uint8_t* const* pk, const uint8_t* const* sig, const uint8_t* const* msg,
                                   const uint32_t* msg_len, size_t n, uint8_t* verdict, uint8_t* keys,
                                   const sv_opts* opts) {
  LifeGuard life_;
  if (n && (!pk || !verdict)) return fail(SV_ERR_INVALID_ARG, "null buffer");
  HostIn in;
  in.ppk = pk;
  in.psig = sig;
  in.pmsg = msg;
  in.len = msg_len;
  return verify_host(in, n, verdict, keys, opts);
}

int sv_ed25519_verify_batch_gather_cb(const uint8_t* const* pk, const uint8_t* const* sig,
                                      const uint8_t* const* msg, const uint32_t* msg_len, size_t n, uint8_t* verdict,
                                      uint8_t* keys, void (*keys_ready)(void* ctx), void* ctx, const sv_opts* opts) {
  LifeGuard life_;
  if (n && (!pk || !verdict || !keys || !keys_ready)) return fail(SV_ERR_INVALID_ARG, "null buffer");
  HostIn in;
  in.ppk = pk;
  in.psig = sig;
  in.pmsg = msg;
  in.len = msg_len;
  struct Once {
    void (*f)(void*);
    void* c;
    size_t n;
  } once{keys_ready, ctx, n};
  KeysCb kcb;
  kcb.fn = [](void* p, size_t ready) {
    const Once* o = static_cast<const Once*>(p);
    if (ready == o->n) o->f(o->c);
  };
  kcb.ctx = &once;
  return verify_host(in, n, verdict, keys, opts, kcb);
}

int sv_ed25519_verify_batch_gather_progress(const uint8_t* const* pk, const uint8_t* const* sig,
                                            const uint8_t* const* msg, const uint32_t* msg_len, size_t n,
                                            uint8_t* verdict, uint8_t* keys,
                                            void (*keys_ready)(void* ctx, size_t ready), void* ctx,
                                            const sv_opts* opts) {
  LifeGuard life_;
  if (n && (!pk || !verdict || !keys || !keys_ready)) return fail(SV_ERR_INVALID_ARG, "null buffer");
  HostIn in;
  in.ppk = pk;
  in.psig = sig;
  in.pmsg = msg;
  in.len = msg_len;
  KeysCb kcb;
  kcb.fn = keys_ready;
  kcb.ctx = ctx;
  return verify_host(in, n, verdict, keys, opts, kcb);
}

int sv_ed25519_verify_batch_keyed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                  const uint64_t* msg_off, const uint32_t* msg_len, size_t n, uint8_t* verdict,
                                  uint8_t* keys, const sv_opts* opts) {
  LifeGuard life_;
  if (!verdict || !keys) return n ? fail(SV_ERR_INVALID_ARG, "null verdict/keys") : SV_OK;
  HostIn in;
  in.pk = pk;
  in.sig = sig;
  in.msg = msg;
  in.off = msg_off;
  in.len = msg_len;
  return verify_host(in, n, verdict, keys, opts);
}

int sv_verify_cache_keys(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                         const uint32_t* msg_len, size_t n, uint8_t* keys, const sv_opts* opts) {
  LifeGuard life_;
  if (!keys) return n ? fail(SV_ERR_INVALID_ARG, "null keys") : SV_OK;
  HostIn in;
  in.pk = pk;
  in.sig = sig;
  in.msg = msg;
  in.off = msg_off;
  in.len = msg_len;
  return verify_host(in, n, nullptr, keys, opts);
}

int sv_sha256_batch(const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n, uint8_t* digests,
                    const sv_opts* opts) {
  LifeGuard life_;
  if (n == 0) return check_opts(opts);
  if (!digests) return fail(SV_ERR_INVALID_ARG, "null digests");
  HostIn in;
  in.pk = data;  // (only the message fields are checked / used)
  in.sig = data;
  in.msg = data;
  in.off = off;
  in.len = len;
  int rc = check_msgs(in, n);
  if (rc) return rc;
  if ((rc = debug_fail())) return rc;
  if ((rc = ensure_init())) return rc;
  std::vector<Device*> devs;
  if ((rc = select_devices(opts, n, devs))) return rc;
  return shard(devs, n, [&](Device& D, size_t lo, size_t hi) {
    return sha_slice(D, data, off + lo, len + lo, hi - lo, digests + 32 * lo);
  });
}

// Device-resident hashing (caller's stream ordering as in sv_ed25519_verify_device).
static int hash_device(int kind, int device, const void* d_pk, const void* d_sig, const void* d_msg,
                       const uint64_t* d_off, const uint32_t* d_len, uint32_t fixed_len, size_t n, void* d_out,
                       void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  if (n == 0) return SV_OK;
  if (!d_out || !d_msg || (kind == 0 && (!d_pk || !d_sig))) return fail(SV_ERR_INVALID_ARG, "null device buffer");
  if (fixed_len == 0 && (!d_off || !d_len)) return fail(SV_ERR_INVALID_ARG, "null msg_off/msg_len");
  if ((((uintptr_t)d_out) & 3u) || (kind == 0 && ((((uintptr_t)d_pk) & 3u) || (((uintptr_t)d_sig) & 3u))))
    return fail(SV_ERR_ALIGN, "pk/sig/out must be 4-byte aligned");
  if ((rc = debug_fail())) return rc;
  Device& D = *Dp;
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  if ((rc = ready_locked(D))) return rc;
  hipStream_t user = (hipStream_t)stream;
  SV_HIP(hipEventRecord(D.dep_in, user));
  SV_HIP(hipStreamWaitEvent(D.stream, D.dep_in, 0));
  SV_HIP(sv_launch_hash(kind, D.grid * 2, d_pk, d_sig, d_msg, d_off, d_len, fixed_len, n, d_out, D.stream));
  SV_HIP(hipEventRecord(D.dep_out, D.stream));
  SV_HIP(hipStreamWaitEvent(user, D.dep_out, 0));
  return SV_OK;
}

int sv_verify_cache_keys_device(int device, const void* d_pk, const void* d_sig, const void* d_msg,
                                const uint64_t* d_msg_off, const uint32_t* d_msg_len, uint32_t fixed_msg_len,
                                size_t n, void* d_keys, void* stream) {
  LifeGuard life_;
  return hash_device(0, device, d_pk, d_sig, d_msg, d_msg_off, d_msg_len, fixed_msg_len, n, d_keys, stream);
}

int sv_sha256_device(int device, const void* d_data, const uint64_t* d_off, const uint32_t* d_len,
                     uint32_t fixed_len, size_t n, void* d_digests, void* stream) {
  LifeGuard life_;
  return hash_device(1, device, nullptr, nullptr, d_data, d_off, d_len, fixed_len, n, d_digests, stream);
}

int sv_ed25519_verify_device(int device, const void* d_pk, const void* d_sig, const void* d_msg,
                             const uint64_t* d_msg_off, const uint32_t* d_msg_len, uint32_t fixed_msg_len,
                             size_t n, void* d_verdict, void* d_bitmap, void* stream) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  if (n == 0) return SV_OK;
  if (!d_pk || !d_sig || !d_verdict) return fail(SV_ERR_INVALID_ARG, "null device buffer");
  if (!aligned16(d_pk) || !aligned16(d_sig)) return fail(SV_ERR_ALIGN, "pk/sig must be 16-byte aligned");
  int mode;
  if (fixed_msg_len == 32 && aligned16(d_msg)) mode = 0;
  else if (fixed_msg_len != 0) mode = 2;
  else {
    if (!d_msg_off || !d_msg_len) return fail(SV_ERR_INVALID_ARG, "null msg_off/msg_len");
    mode = 1;
  }
  if (!d_msg) return fail(SV_ERR_INVALID_ARG, "null msg");
  if ((rc = debug_fail())) return rc;
  Device& D = *Dp;
  hipStream_t user = (hipStream_t)stream;
  if (resolve_path(SV_PATH_AUTO, n) == SV_PATH_LATENCY) {
    // the latency lane (octet kernel: the keys are in device memory, so the
    // host-side key cache is not consulted)
    LatLane& L = D.lat;
    std::lock_guard<std::mutex> g(L.mu);
    SV_HIP(hipSetDevice(D.phys));
    if ((rc = lat_ready(D))) return rc;
    // a context no host batch holds, else the first: this call only queues
    // work (stream order keeps it after a batch running on the same context,
    // and the workspace only grows once that context's stream has drained)
    LatCtx* c = &L.ctx[0];
    for (int k = 0; k < L.nctx; ++k)
      if (!L.ctx[k].busy) {
        c = &L.ctx[k];
        break;
      }
    D.lat_last_ns.store(now_ns(), std::memory_order_relaxed);
    SV_HIP(hipEventRecord(L.ev_lat, user));
    SV_HIP(hipStreamWaitEvent(c->stream, L.ev_lat, 0));
    hipEvent_t e0;
    const uint32_t dbg = g_dbg.load() & kKernelDbgMask;
    const bool quad = n > kOctetMax && !(g_dbg.load() & SV_DBG_NO_QUAD);
    if (quad && (rc = lat_ws(*c, sv_verify_ws_bytes(kGeomQuad, 0, n)))) return rc;
    if ((rc = lat_timing_begin(c->stream, &e0))) return rc;
    SV_HIP(sv_launch_verify(mode, quad ? kGeomQuad : SV_PATH_LATENCY, 1, d_pk, d_sig, d_msg, d_msg_off, d_msg_len,
                            fixed_msg_len, n, d_verdict, d_bitmap, quad ? c->ws.p : nullptr, D.btab,
                            quad ? (dbg | SV_KP_LAT) : dbg, 0, nullptr, nullptr, c->stream));
    if ((rc = lat_timing_end(L, c->stream, e0, n))) return rc;
    SV_HIP(hipEventRecord(c->dev_done, c->stream));
    SV_HIP(hipStreamWaitEvent(user, c->dev_done, 0));
    return SV_OK;
  }
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  if ((rc = ready_locked(D))) return rc;
  SV_HIP(hipEventRecord(D.dep_in, user));
  SV_HIP(hipStreamWaitEvent(D.stream, D.dep_in, 0));
  // (auto mode cannot look at device-resident keys: tables only when on)
  if ((rc = launch_locked(D, mode, SV_PATH_AUTO, d_pk, d_sig, d_msg, d_msg_off, d_msg_len, fixed_msg_len, n,
                          d_verdict, d_bitmap, kt_mode() == 1)))
    return rc;
  SV_HIP(hipEventRecord(D.dep_out, D.stream));
  SV_HIP(hipStreamWaitEvent(user, D.dep_out, 0));
  return SV_OK;
}

int sv_lat_last_trace(double out[8]) {
  if (!out) return SV_ERR_INVALID_ARG;
  for (int k = 0; k < 8; ++k) out[k] = t_lat_last[k];
  return SV_OK;
}

int sv_set_kernel_path(int path) {
  LifeGuard life_;
  if (path != SV_PATH_AUTO && path != SV_PATH_THROUGHPUT && path != SV_PATH_LATENCY) return SV_ERR_INVALID_ARG;
  return g_path.exchange(path);
}

int sv_set_debug_flags(uint32_t flags) {
  LifeGuard life_;
  if (flags & ~(SV_DBG_TRIVIAL_PAIR | SV_DBG_MAX_WINDOWS | SV_DBG_FAIL | SV_DBG_PREP_ONLY | SV_DBG_KEY_COLLIDE |
                SV_DBG_QUAD | SV_DBG_NO_QUAD | SV_DBG_DROP_HANDOVER))
    return SV_ERR_INVALID_ARG;
  if ((flags & SV_DBG_QUAD) && (flags & SV_DBG_NO_QUAD)) return SV_ERR_INVALID_ARG;
  // the knobs that change what a call returns (FAIL: every call errs;
  // PREP_ONLY: no verdicts; DROP_HANDOVER: cold three-wave batches reject)
  // only exist for processes that opt in
  if ((flags & (SV_DBG_FAIL | SV_DBG_PREP_ONLY | SV_DBG_DROP_HANDOVER)) && !test_knobs_enabled())
    return fail(SV_ERR_INVALID_ARG,
                "SV_DBG_FAIL / SV_DBG_PREP_ONLY / SV_DBG_DROP_HANDOVER need SV_TEST_KNOBS=1 in the environment");
  return (int)g_dbg.exchange(flags);
}

int sv_set_min_shard(size_t n) {
  LifeGuard life_;
  g_min_shard.store(n);
  return SV_OK;
}

int sv_ed25519_sign_device(int device, const void* d_seed, const void* d_msg32, size_t n, void* d_pk, void* d_sig,
                           void* stream) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  if (n == 0) return SV_OK;
  if (!d_seed || !d_msg32 || !d_pk || !d_sig) return fail(SV_ERR_INVALID_ARG, "null device buffer");
  if (!aligned16(d_seed) || !aligned16(d_msg32) || !aligned16(d_pk) || !aligned16(d_sig))
    return fail(SV_ERR_ALIGN, "buffers must be 16-byte aligned");
  Device& D = *Dp;
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.phys));
  if ((rc = ready_locked(D))) return rc;
  const unsigned grid = grid_for(D, n);
  if ((rc = ensure_ws(D, sv_ws_bytes(grid, 0)))) return rc;
  hipStream_t user = (hipStream_t)stream;
  SV_HIP(hipEventRecord(D.dep_in, user));
  SV_HIP(hipStreamWaitEvent(D.stream, D.dep_in, 0));
  SV_HIP(sv_launch_sign(grid, d_seed, d_msg32, n, d_pk, d_sig, D.ws.p, D.btab, D.stream));
  SV_HIP(hipEventRecord(D.dep_out, D.stream));
  SV_HIP(hipStreamWaitEvent(user, D.dep_out, 0));
  return SV_OK;
}

int sv_timing_enable(int enable) {
  LifeGuard life_;
  g_timing.store(enable ? 1 : 0);
  return SV_OK;
}

int sv_kernel_time(int device, double* total_ms, uint64_t* launches, uint64_t* signatures) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  Device& D = *Dp;
  std::lock_guard<std::mutex> gl(D.lat.mu);
  std::lock_guard<std::mutex> g(D.mu);
  double ms = 0;
  uint64_t la = 0, sg = 0;
  if (D.ready) {
    SV_HIP(hipSetDevice(D.phys));
    if ((rc = harvest_timing_locked(D))) return rc;
    if (D.lat.ready && (rc = lat_harvest(D.lat))) return rc;
    ms = D.total_ms + D.lat.total_ms;
    la = D.launches + D.lat.launches;
    sg = D.sigs + D.lat.sigs;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = la;
  if (signatures) *signatures = sg;
  return SV_OK;
}

int sv_kernel_time_reset(void) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  for (Device* D : g_devs) {
    std::lock_guard<std::mutex> gl(D->lat.mu);
    std::lock_guard<std::mutex> g(D->mu);
    if (!D->ready) continue;
    (void)hipSetDevice(D->phys);
    if ((rc = harvest_timing_locked(*D))) return rc;
    if (D->lat.ready && (rc = lat_harvest(D->lat))) return rc;
    D->total_ms = D->lat.total_ms = 0;
    D->launches = D->lat.launches = 0;
    D->sigs = D->lat.sigs = 0;
  }
  return SV_OK;
}

int sv_device_synchronize(int device) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  Device& D = *Dp;
  std::lock_guard<std::mutex> gl(D.lat.mu);
  std::lock_guard<std::mutex> g(D.mu);
  if (!D.ready) return SV_OK;
  SV_HIP(hipSetDevice(D.phys));
  SV_HIP(hipStreamSynchronize(D.stream));
  if (D.lat.ready) lat_sync(D.lat);
  return SV_OK;
}

int sv_set_key_tables(int mode, size_t slots) {
  LifeGuard life_;
  if (mode < -1 || mode > 2) return fail(SV_ERR_INVALID_ARG, "key-table mode must be -1, 0, 1 or 2");
  g_kt_slots.store(slots);
  return g_kt_mode.exchange(mode);
}

int sv_set_key_cache(size_t capacity) {
  LifeGuard life_;
  if (capacity > ((size_t)1 << 20)) return fail(SV_ERR_INVALID_ARG, "key cache capacity above 2^20 keys");
  std::lock_guard<std::mutex> g0(g_mu);
  g_key_cap.store(capacity);
  for (Device* D : g_devs) {
    std::lock_guard<std::mutex> g(D->lat.mu);
    if (!D->lat.ready) continue;
    (void)hipSetDevice(D->phys);
    lat_cache_ready(D->lat);  // (drains the lane, then resizes / clears)
  }
  return SV_OK;
}

int sv_key_cache_wait(int device) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  LatLane& L = Dp->lat;
  std::lock_guard<std::mutex> g(L.mu);
  if (!L.ready) return SV_OK;
  SV_HIP(hipSetDevice(Dp->phys));
  SV_HIP(hipStreamSynchronize(L.build));
  lat_poll(L);
  return SV_OK;
}

int sv_key_cache_get_stats(int device, sv_key_cache_stats* out) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp || !out) return fail(SV_ERR_INVALID_ARG, "bad argument");
  LatLane& L = Dp->lat;
  std::lock_guard<std::mutex> g(L.mu);
  if (L.ready) {
    (void)hipSetDevice(Dp->phys);
    lat_poll(L);
  }
  out->capacity = L.ready ? L.cap : key_cache_cap();
  out->keys = L.index.size();
  out->warm_batches = L.warm;
  out->cold_batches = L.cold;
  out->keys_built = L.built;
  out->evictions = L.evicted;
  out->shared_launches = Dp->shared_launches.load();
  {
    std::lock_guard<std::mutex> g2(Dp->mu);
    KeyTabs& T = Dp->kt;
    if (T.slots && T.copied && hipEventQuery(T.copied) == hipSuccess) T.claims = ((const uint32_t*)T.h_count.p)[1];
    out->table_launches = T.launches;
    out->table_keys = T.claims;
    out->table_clears = T.clears;
    out->table_slots = T.slots ? T.slots : kt_slots();
  }
  return SV_OK;
}

int sv_workspace_bytes(int device, size_t* bytes) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp || !bytes) return fail(SV_ERR_INVALID_ARG, "bad argument");
  // (lock order: the lane's mutex before the slot's)
  std::lock_guard<std::mutex> gl(Dp->lat.mu);
  std::lock_guard<std::mutex> g(Dp->mu);
  size_t b = Dp->ws.cap;
  for (const LatCtx& c : Dp->lat.ctx) b += c.ws.cap + c.d_in.cap + c.d_out.cap + c.d_keys.cap;
  *bytes = b;
  return SV_OK;
}

int sv_pinned_bytes(int device, size_t* bytes) {
  LifeGuard life_;
  int rc = ensure_init();
  if (rc) return rc;
  Device* Dp = device_arg(device);
  if (!Dp || !bytes) return fail(SV_ERR_INVALID_ARG, "bad argument");
  std::lock_guard<std::mutex> gl(Dp->lat.mu);
  std::lock_guard<std::mutex> g(Dp->mu);
  size_t b = 0;
  for (Stage& s : Dp->st) b += s.h_in.cap + s.h_out.cap;
  b += Dp->z_in.cap + Dp->z_out.cap + Dp->h_sha.cap;
  for (const LatCtx& c : Dp->lat.ctx) b += c.h_in.cap + c.h_out.cap + c.z_out.cap + c.z_keys.cap + c.z_stat.cap;
  b += Dp->lat.h_build.cap;
  *bytes = b;
  return SV_OK;
}

}  // extern "C"
