// C-ABI implementation (include/stellar_sigverify.h): device discovery,
// per-device resources, host<->device staging and multi-GPU sharding.
//
// Replaces, for whole batches, the libsodium crypto_sign_verify_detached call
// made by stellar::PubKeyUtils::verifySig on a verify-cache miss
// (/root/reference/src/crypto/SecretKey.cpp:461-463).
//
// Per device: one non-blocking HIP stream, the 129-entry base-point table
// (computed on the device at init), and the per-lane -A table workspace sized
// for the persistent grid (CUs x resident workgroups).  All work for a device
// is serialised on its stream under its mutex because the workspace is shared
// by every launch on that device.  Multi-GPU: contiguous slices
// [g*n/G, (g+1)*n/G), one host thread per device, verdicts copied back into
// disjoint ranges of the caller's buffer -- no collective.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/stellar_sigverify.h"

extern "C" {
size_t sv_ws_bytes_per_block(void);
size_t sv_ws_bytes(unsigned grid);
size_t sv_btab_bytes(void);
int sv_block_threads(void);
hipError_t sv_launch_btab_init(uint32_t* d_btab, hipStream_t s);
int sv_occupancy_blocks_per_cu(void);
hipError_t sv_launch_verify(int mode, int path, unsigned grid, const void* pk, const void* sig, const void* msg,
                            const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n,
                            void* verdict, void* bitmap, void* ws, const void* btab, hipStream_t s);
hipError_t sv_launch_sign(unsigned grid, const void* seed, const void* msg, uint64_t n, void* pk, void* sig,
                          void* ws, const void* btab, hipStream_t s);
hipError_t sv_launch_hash(int kind, unsigned max_blocks, const void* pk, const void* sig, const void* msg,
                          const uint64_t* off, const uint32_t* len, uint32_t fixed_len, uint64_t n, void* out,
                          hipStream_t s);
}

namespace {

thread_local std::string t_err;

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

// Pinned host staging (hipHostMalloc): one H2D copy per batch instead of one
// pageable copy per input array.
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return SV_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      p = nullptr;
      return fail(SV_ERR_ALLOC, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    cap = want;
    return SV_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Device {
  int id = -1;
  bool ready = false;  // resources created lazily on first use (under mu)
  int cus = 0;
  unsigned grid = 0;  // persistent grid (workgroups)
  hipStream_t stream = nullptr;
  void* btab = nullptr;
  void* ws = nullptr;
  hipEvent_t dep_in = nullptr, dep_out = nullptr;
  std::mutex mu;
  DevBuf pk, sig, msg, off, len, verdict, keys;
  DevBuf in;          // staged batch: pk | sig | [off | len] | msg
  HostBuf h_in, h_out;
  // timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<uint64_t> pending_n;
  double total_ms = 0;
  uint64_t launches = 0, sigs = 0;
};

std::mutex g_mu;
std::vector<Device*> g_devs;
bool g_inited = false;
std::atomic<int> g_timing{0};
std::atomic<int> g_path{SV_PATH_AUTO};  // sv_set_kernel_path

// Batches up to this size take the latency kernel under SV_PATH_AUTO
// (measured crossover on MI355X).
constexpr uint64_t kQuickMax = 12288;

// Kernel path for one launch: an explicit per-call request (sv_opts.flags),
// else the process default, else by batch size.
int resolve_path(int requested, uint64_t n) {
  int p = requested != SV_PATH_AUTO ? requested : g_path.load();
  if (p == SV_PATH_AUTO) p = n <= kQuickMax ? SV_PATH_LATENCY : SV_PATH_THROUGHPUT;
  return p;
}
int path_from_flags(uint32_t flags) {
  if (flags & SV_FLAG_PATH_LATENCY) return SV_PATH_LATENCY;
  if (flags & SV_FLAG_PATH_THROUGHPUT) return SV_PATH_THROUGHPUT;
  return SV_PATH_AUTO;
}

int init_device(Device& D, int id) {
  D.id = id;
  SV_HIP(hipSetDevice(id));
  hipDeviceProp_t prop;
  SV_HIP(hipGetDeviceProperties(&prop, id));
  D.cus = prop.multiProcessorCount;
  SV_HIP(hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking));
  SV_HIP(hipEventCreateWithFlags(&D.dep_in, hipEventDisableTiming));
  SV_HIP(hipEventCreateWithFlags(&D.dep_out, hipEventDisableTiming));
  SV_HIP(hipMalloc(&D.btab, sv_btab_bytes()));
  SV_HIP(sv_launch_btab_init((uint32_t*)D.btab, D.stream));
  const int per_cu = sv_occupancy_blocks_per_cu();
  D.grid = (unsigned)(D.cus * per_cu);
  const size_t ws_bytes = sv_ws_bytes(D.grid);
  hipError_t e = hipMalloc(&D.ws, ws_bytes);
  if (e != hipSuccess) return fail(SV_ERR_ALLOC, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
  SV_HIP(hipStreamSynchronize(D.stream));
  return SV_OK;
}

// Enumerates devices only; per-device resources are created on first use so a
// process that drives one GPU (one rank per GPU) never touches the others.
int ensure_init() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_inited) return g_devs.empty() ? fail(SV_ERR_NO_DEVICE, "no HIP device") : SV_OK;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  g_inited = true;
  if (e != hipSuccess || n <= 0) return fail(SV_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  for (int i = 0; i < n; ++i) {
    Device* D = new Device();
    D->id = i;
    g_devs.push_back(D);
  }
  return SV_OK;
}

// Caller holds D.mu.
int ready_locked(Device& D) {
  if (D.ready) return SV_OK;
  int rc = init_device(D, D.id);
  if (rc == SV_OK) D.ready = true;
  return rc;
}

unsigned grid_for(const Device& D, uint64_t n) {
  const uint64_t need = (n + sv_block_threads() - 1) / sv_block_threads();
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(D.grid, need));
}

// Launch on D.stream (caller holds D.mu and has set the device).
int launch_locked(Device& D, int mode, int path, const void* pk, const void* sig, const void* msg, const uint64_t* off,
                  const uint32_t* len, uint32_t fixed_len, uint64_t n, void* verdict, void* bitmap) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool timing = g_timing.load() != 0;
  if (timing) {
    SV_HIP(hipEventCreate(&e0));
    SV_HIP(hipEventCreate(&e1));
    SV_HIP(hipEventRecord(e0, D.stream));
  }
  SV_HIP(sv_launch_verify(mode, resolve_path(path, n), grid_for(D, n), pk, sig, msg, off, len, fixed_len, n, verdict,
                          bitmap, D.ws, D.btab, D.stream));
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

// Host-buffer slice on one device: stage once, then launch the verify kernel
// (verdict != null) and/or the cache-key kernel (keys != null) on the same
// stream, copy results back, sync.
int host_slice(Device& D, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
               const uint32_t* msg_len, uint32_t fixed_len, size_t n, uint8_t* verdict, uint8_t* keys, int path) {
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.id));
  int rc;
  if ((rc = ready_locked(D))) return rc;
  // one pinned staging image, one H2D copy:
  //   pk (32 n) | sig (64 n) | fixed: msg (n L)  or  var: off (8 n) | len (4 n) | packed msgs
  // (pk, sig, and a fixed-length msg block stay 16-byte aligned)
  const size_t o_sig = 32 * n, o_var = 96 * n;
  size_t total_msg = 0;
  if (fixed_len != 0) {
    total_msg = n * (size_t)fixed_len;
  } else {
    for (size_t i = 0; i < n; ++i) total_msg += msg_len[i];
  }
  const size_t o_off = o_var, o_len = o_var + 8 * n;
  const size_t o_msg = fixed_len != 0 ? o_var : o_var + 12 * n;
  const size_t bytes = o_msg + std::max<size_t>(total_msg, 1);
  if ((rc = D.in.ensure(bytes)) || (rc = D.h_in.ensure(bytes))) return rc;
  if (verdict && ((rc = D.verdict.ensure(n)) || (rc = D.h_out.ensure(n)))) return rc;
  if (keys && (rc = D.keys.ensure(n * 32))) return rc;
  uint8_t* h = (uint8_t*)D.h_in.p;
  memcpy(h, pk, n * 32);
  memcpy(h + o_sig, sig, n * 64);
  int mode;
  if (fixed_len != 0) {
    if (total_msg) memcpy(h + o_msg, msg, total_msg);
    mode = (fixed_len == 32) ? 0 : 2;
  } else {
    // pack this slice's messages contiguously (offsets may be arbitrary)
    uint64_t* offs = (uint64_t*)(h + o_off);
    size_t pos = 0;
    for (size_t i = 0; i < n; ++i) {
      offs[i] = pos;
      if (msg_len[i]) memcpy(h + o_msg + pos, msg + msg_off[i], msg_len[i]);
      pos += msg_len[i];
    }
    memcpy(h + o_len, msg_len, n * 4);
    mode = 1;
  }
  SV_HIP(hipMemcpyAsync(D.in.p, h, bytes, hipMemcpyHostToDevice, D.stream));
  uint8_t* d = (uint8_t*)D.in.p;
  const uint64_t* d_off = fixed_len ? nullptr : (const uint64_t*)(d + o_off);
  const uint32_t* d_len = fixed_len ? nullptr : (const uint32_t*)(d + o_len);
  if (keys) {
    SV_HIP(sv_launch_hash(0, D.grid * 2, d, d + o_sig, d + o_msg, d_off, d_len, fixed_len, n, D.keys.p, D.stream));
    SV_HIP(hipMemcpyAsync(keys, D.keys.p, n * 32, hipMemcpyDeviceToHost, D.stream));
  }
  if (verdict) {
    if ((rc = launch_locked(D, mode, path, d, d + o_sig, d + o_msg, d_off, d_len, fixed_len, n, D.verdict.p,
                            nullptr)))
      return rc;
    SV_HIP(hipMemcpyAsync(D.h_out.p, D.verdict.p, n, hipMemcpyDeviceToHost, D.stream));
  }
  SV_HIP(hipStreamSynchronize(D.stream));  // the staging buffers are reused by the next call
  if (verdict) memcpy(verdict, D.h_out.p, n);
  return SV_OK;
}

// SHA-256 of a host slice of byte strings on one device.
int sha_slice(Device& D, const uint8_t* data, const uint64_t* off, const uint32_t* len, uint32_t fixed_len,
              size_t n, uint8_t* out) {
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.id));
  int rc;
  if ((rc = ready_locked(D))) return rc;
  if ((rc = D.keys.ensure(n * 32))) return rc;
  std::vector<uint64_t> offs;
  std::vector<uint8_t> packed;
  if (fixed_len != 0) {
    if ((rc = D.msg.ensure((size_t)n * fixed_len))) return rc;
    SV_HIP(hipMemcpyAsync(D.msg.p, data, n * (size_t)fixed_len, hipMemcpyHostToDevice, D.stream));
  } else {
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) total += len[i];
    packed.resize(std::max<size_t>(total, 1));
    offs.resize(n);
    size_t pos = 0;
    for (size_t i = 0; i < n; ++i) {
      offs[i] = pos;
      if (len[i]) memcpy(packed.data() + pos, data + off[i], len[i]);
      pos += len[i];
    }
    if ((rc = D.msg.ensure(packed.size())) || (rc = D.off.ensure(n * 8)) || (rc = D.len.ensure(n * 4))) return rc;
    SV_HIP(hipMemcpyAsync(D.msg.p, packed.data(), packed.size(), hipMemcpyHostToDevice, D.stream));
    SV_HIP(hipMemcpyAsync(D.off.p, offs.data(), n * 8, hipMemcpyHostToDevice, D.stream));
    SV_HIP(hipMemcpyAsync(D.len.p, len, n * 4, hipMemcpyHostToDevice, D.stream));
  }
  SV_HIP(sv_launch_hash(1, D.grid * 2, nullptr, nullptr, D.msg.p, (const uint64_t*)D.off.p,
                        (const uint32_t*)D.len.p, fixed_len, n, D.keys.p, D.stream));
  SV_HIP(hipMemcpyAsync(out, D.keys.p, n * 32, hipMemcpyDeviceToHost, D.stream));
  SV_HIP(hipStreamSynchronize(D.stream));
  return SV_OK;
}

int select_devices(const sv_opts* opts, std::vector<Device*>& out) {
  int dev = -1;
  uint32_t maxd = 0;
  if (opts) {
    if (opts->struct_size < sizeof(sv_opts) || (opts->flags & ~SV_FLAG_PATH_MASK) != 0 ||
        (opts->flags & SV_FLAG_PATH_MASK) == SV_FLAG_PATH_MASK)
      return fail(SV_ERR_INVALID_ARG, "bad sv_opts");
    dev = opts->device;
    maxd = opts->max_devices;
  }
  if (dev >= 0) {
    if (dev >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
    out.push_back(g_devs[dev]);
  } else {
    for (Device* d : g_devs) {
      if (maxd && out.size() >= maxd) break;
      out.push_back(d);
    }
  }
  return SV_OK;
}

// Runs fn(device, lo, hi) for contiguous slices [g*n/G, (g+1)*n/G), one host
// thread per device; the first failing device's error is reported.
template <class F>
int shard(const std::vector<Device*>& devs, size_t n, F fn) {
  const size_t G = devs.size();
  if (G == 1) return fn(*devs[0], (size_t)0, n);
  std::vector<int> rcs(G, SV_OK);
  std::vector<std::string> errs(G);
  std::vector<std::thread> th;
  for (size_t g = 0; g < G; ++g) {
    const size_t lo = g * n / G, hi = (g + 1) * n / G;
    if (hi == lo) continue;
    th.emplace_back([&, g, lo, hi] {
      rcs[g] = fn(*devs[g], lo, hi);
      if (rcs[g]) errs[g] = t_err;
    });
  }
  for (auto& t : th) t.join();
  for (size_t g = 0; g < G; ++g)
    if (rcs[g]) return fail(rcs[g], "device " + std::to_string(devs[g]->id) + ": " + errs[g]);
  return SV_OK;
}

int check_msgs(const uint8_t* msg, const uint64_t* msg_off, const uint32_t* msg_len, uint32_t fixed_len, size_t n) {
  if (fixed_len == 0 && (!msg_off || !msg_len)) return fail(SV_ERR_INVALID_ARG, "null msg_off/msg_len");
  if (!msg) {
    bool any = false;
    if (fixed_len) any = true;
    else
      for (size_t i = 0; i < n && !any; ++i) any = msg_len[i] != 0;
    if (any) return fail(SV_ERR_INVALID_ARG, "null msg");
  }
  return SV_OK;
}

int verify_host(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                const uint32_t* msg_len, uint32_t fixed_len, size_t n, uint8_t* verdict, uint8_t* keys,
                const sv_opts* opts) {
  if (n == 0) return SV_OK;
  if (!pk || !sig || (!verdict && !keys)) return fail(SV_ERR_INVALID_ARG, "null buffer");
  int rc = check_msgs(msg, msg_off, msg_len, fixed_len, n);
  if (rc) return rc;
  if ((rc = ensure_init())) return rc;
  std::vector<Device*> devs;
  if ((rc = select_devices(opts, devs))) return rc;
  return shard(devs, n, [&](Device& D, size_t lo, size_t hi) {
    return host_slice(D, pk + 32 * lo, sig + 64 * lo, fixed_len ? msg + lo * (size_t)fixed_len : msg,
                      fixed_len ? nullptr : msg_off + lo, fixed_len ? nullptr : msg_len + lo, fixed_len, hi - lo,
                      verdict ? verdict + lo : nullptr, keys ? keys + 32 * lo : nullptr,
                      path_from_flags(opts ? opts->flags : 0u));
  });
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" {

int sv_init(void) { return ensure_init(); }

void sv_shutdown(void) {
  std::lock_guard<std::mutex> g(g_mu);
  for (Device* D : g_devs) {
    std::lock_guard<std::mutex> gd(D->mu);
    if (!D->ready) continue;
    (void)hipSetDevice(D->id);
    (void)hipStreamSynchronize(D->stream);
    for (auto& pr : D->pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    D->pk.release(); D->sig.release(); D->msg.release();
    D->off.release(); D->len.release(); D->verdict.release(); D->keys.release();
    D->in.release(); D->h_in.release(); D->h_out.release();
    if (D->ws) (void)hipFree(D->ws);
    if (D->btab) (void)hipFree(D->btab);
    if (D->dep_in) (void)hipEventDestroy(D->dep_in);
    if (D->dep_out) (void)hipEventDestroy(D->dep_out);
    if (D->stream) (void)hipStreamDestroy(D->stream);
  }
  for (Device* D : g_devs) delete D;
  g_devs.clear();
  g_inited = false;
}

int sv_device_count(void) {
  int rc = ensure_init();
  if (rc) return rc;
  return (int)g_devs.size();
}

const char* sv_last_error_string(void) { return t_err.c_str(); }

const char* sv_version(void) {
  return "stellar-core_amd sigverify r1 (gfx950; ed25519 == libsodium-1.0.18 crypto_sign_verify_detached)";
}

int sv_ed25519_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                            const uint32_t* msg_len, size_t n, uint8_t* verdict, const sv_opts* opts) {
  return verify_host(pk, sig, msg, msg_off, msg_len, 0, n, verdict, nullptr, opts);
}

int sv_ed25519_verify_batch_fixed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_len,
                                  size_t n, uint8_t* verdict, const sv_opts* opts) {
  if (msg_len == 0) {
    // zero-length messages: route through the variable-length path
    std::vector<uint64_t> off(n, 0);
    std::vector<uint32_t> len(n, 0);
    static const uint8_t dummy = 0;
    return verify_host(pk, sig, &dummy, off.data(), len.data(), 0, n, verdict, nullptr, opts);
  }
  return verify_host(pk, sig, msg, nullptr, nullptr, msg_len, n, verdict, nullptr, opts);
}

int sv_ed25519_verify_batch_keyed(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                                  const uint64_t* msg_off, const uint32_t* msg_len, size_t n, uint8_t* verdict,
                                  uint8_t* keys, const sv_opts* opts) {
  if (!verdict || !keys) return n ? fail(SV_ERR_INVALID_ARG, "null verdict/keys") : SV_OK;
  return verify_host(pk, sig, msg, msg_off, msg_len, 0, n, verdict, keys, opts);
}

int sv_verify_cache_keys(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* msg_off,
                         const uint32_t* msg_len, size_t n, uint8_t* keys, const sv_opts* opts) {
  if (!keys) return n ? fail(SV_ERR_INVALID_ARG, "null keys") : SV_OK;
  return verify_host(pk, sig, msg, msg_off, msg_len, 0, n, nullptr, keys, opts);
}

int sv_sha256_batch(const uint8_t* data, const uint64_t* off, const uint32_t* len, size_t n, uint8_t* digests,
                    const sv_opts* opts) {
  if (n == 0) return SV_OK;
  if (!digests) return fail(SV_ERR_INVALID_ARG, "null digests");
  int rc = check_msgs(data, off, len, 0, n);
  if (rc) return rc;
  if ((rc = ensure_init())) return rc;
  std::vector<Device*> devs;
  if ((rc = select_devices(opts, devs))) return rc;
  return shard(devs, n, [&](Device& D, size_t lo, size_t hi) {
    return sha_slice(D, data, off + lo, len + lo, 0, hi - lo, digests + 32 * lo);
  });
}

// Device-resident hashing (caller's stream ordering as in sv_ed25519_verify_device).
static int hash_device(int kind, int device, const void* d_pk, const void* d_sig, const void* d_msg,
                       const uint64_t* d_off, const uint32_t* d_len, uint32_t fixed_len, size_t n, void* d_out,
                       void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  if (n == 0) return SV_OK;
  if (!d_out || !d_msg || (kind == 0 && (!d_pk || !d_sig))) return fail(SV_ERR_INVALID_ARG, "null device buffer");
  if (fixed_len == 0 && (!d_off || !d_len)) return fail(SV_ERR_INVALID_ARG, "null msg_off/msg_len");
  if ((((uintptr_t)d_out) & 3u) || (kind == 0 && ((((uintptr_t)d_pk) & 3u) || (((uintptr_t)d_sig) & 3u))))
    return fail(SV_ERR_ALIGN, "pk/sig/out must be 4-byte aligned");
  Device& D = *g_devs[device];
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.id));
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
  return hash_device(0, device, d_pk, d_sig, d_msg, d_msg_off, d_msg_len, fixed_msg_len, n, d_keys, stream);
}

int sv_sha256_device(int device, const void* d_data, const uint64_t* d_off, const uint32_t* d_len,
                     uint32_t fixed_len, size_t n, void* d_digests, void* stream) {
  return hash_device(1, device, nullptr, nullptr, d_data, d_off, d_len, fixed_len, n, d_digests, stream);
}

int sv_ed25519_verify_device(int device, const void* d_pk, const void* d_sig, const void* d_msg,
                             const uint64_t* d_msg_off, const uint32_t* d_msg_len, uint32_t fixed_msg_len,
                             size_t n, void* d_verdict, void* d_bitmap, void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
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
  Device& D = *g_devs[device];
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.id));
  if ((rc = ready_locked(D))) return rc;
  hipStream_t user = (hipStream_t)stream;
  SV_HIP(hipEventRecord(D.dep_in, user));
  SV_HIP(hipStreamWaitEvent(D.stream, D.dep_in, 0));
  if ((rc = launch_locked(D, mode, SV_PATH_AUTO, d_pk, d_sig, d_msg, d_msg_off, d_msg_len, fixed_msg_len, n,
                          d_verdict, d_bitmap)))
    return rc;
  SV_HIP(hipEventRecord(D.dep_out, D.stream));
  SV_HIP(hipStreamWaitEvent(user, D.dep_out, 0));
  return SV_OK;
}

int sv_set_kernel_path(int path) {
  if (path != SV_PATH_AUTO && path != SV_PATH_THROUGHPUT && path != SV_PATH_LATENCY) return SV_ERR_INVALID_ARG;
  return g_path.exchange(path);
}

int sv_ed25519_sign_device(int device, const void* d_seed, const void* d_msg32, size_t n, void* d_pk, void* d_sig,
                           void* stream) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  if (n == 0) return SV_OK;
  if (!d_seed || !d_msg32 || !d_pk || !d_sig) return fail(SV_ERR_INVALID_ARG, "null device buffer");
  if (!aligned16(d_seed) || !aligned16(d_msg32) || !aligned16(d_pk) || !aligned16(d_sig))
    return fail(SV_ERR_ALIGN, "buffers must be 16-byte aligned");
  Device& D = *g_devs[device];
  std::lock_guard<std::mutex> g(D.mu);
  SV_HIP(hipSetDevice(D.id));
  if ((rc = ready_locked(D))) return rc;
  hipStream_t user = (hipStream_t)stream;
  SV_HIP(hipEventRecord(D.dep_in, user));
  SV_HIP(hipStreamWaitEvent(D.stream, D.dep_in, 0));
  SV_HIP(sv_launch_sign(grid_for(D, n), d_seed, d_msg32, n, d_pk, d_sig, D.ws, D.btab, D.stream));
  SV_HIP(hipEventRecord(D.dep_out, D.stream));
  SV_HIP(hipStreamWaitEvent(user, D.dep_out, 0));
  return SV_OK;
}

int sv_timing_enable(int enable) {
  g_timing.store(enable ? 1 : 0);
  return SV_OK;
}

int sv_kernel_time(int device, double* total_ms, uint64_t* launches, uint64_t* signatures) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  Device& D = *g_devs[device];
  std::lock_guard<std::mutex> g(D.mu);
  if (!D.ready) {
    if (total_ms) *total_ms = 0;
    if (launches) *launches = 0;
    if (signatures) *signatures = 0;
    return SV_OK;
  }
  SV_HIP(hipSetDevice(D.id));
  if ((rc = harvest_timing_locked(D))) return rc;
  if (total_ms) *total_ms = D.total_ms;
  if (launches) *launches = D.launches;
  if (signatures) *signatures = D.sigs;
  return SV_OK;
}

int sv_kernel_time_reset(void) {
  int rc = ensure_init();
  if (rc) return rc;
  for (Device* D : g_devs) {
    std::lock_guard<std::mutex> g(D->mu);
    if (!D->ready) continue;
    (void)hipSetDevice(D->id);
    if ((rc = harvest_timing_locked(*D))) return rc;
    D->total_ms = 0;
    D->launches = 0;
    D->sigs = 0;
  }
  return SV_OK;
}

int sv_device_synchronize(int device) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(SV_ERR_INVALID_ARG, "device index out of range");
  Device& D = *g_devs[device];
  std::lock_guard<std::mutex> g(D.mu);
  if (!D.ready) return SV_OK;
  SV_HIP(hipSetDevice(D.id));
  SV_HIP(hipStreamSynchronize(D.stream));
  return SV_OK;
}

}  // extern "C"
