// VALU issue-rate microbenchmark for gfx950 (MI355X): the roofline peak of
// the verify kernel is a measured number, and this harness is validated
// against the one rate the CDNA4 guide states (wave64 v_fma_f32: 2 cycles per
// wave-instruction on a SIMD-32 with >= 2 waves, i.e. 128 lane-ops/clk/CU).
//
// Per kernel: every lane runs ITERS x 32 instructions of one kind over 16
// independent accumulators (dependency distance 16); carry-out SGPR pairs
// rotate over 8 pairs (the verify kernel's scheme: a VALU write of the SAME
// SGPR pair by consecutive instructions serialises them).  One block of 256
// threads = one wave per SIMD; `occ` blocks per CU = occ waves per SIMD, all
// co-resident (<= 64 VGPRs).  Every wave stamps s_memtime / s_memrealtime
// around its loop; the chip rate is total lane-instructions / (latest end -
// earliest start) of the real-time stamps, divided by CUs and the in-kernel
// clock (shader cycles / real-time ticks), so launch overhead and partially
// filled tails do not enter.  The hipEvent wall rate is printed beside it.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu_rates.hip -o tools/ubench_valu_rates
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#ifndef ITERS
#define ITERS 2048
#endif

#define SV_NOUNROLL_LOOP _Pragma("unroll 1")

// carry-out SGPR pair for accumulator i (8 pairs, top of the SGPR file)
#define SP0 "s[80:81]"
#define SP1 "s[82:83]"
#define SP2 "s[84:85]"
#define SP3 "s[86:87]"
#define SP4 "s[88:89]"
#define SP5 "s[90:91]"
#define SP6 "s[92:93]"
#define SP7 "s[94:95]"
#define CLOB "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95"

struct Stamp {
  unsigned long long t0, t1, r0, r1;
};

#define KERNEL_HEAD(NAME, T)                                                          \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, Stamp* st, uint32_t seed) { \
    uint32_t a = threadIdx.x * 2654435761u + seed, b = a * 3u + 1u;                  \
    T acc[16];                                                                        \
    for (int i = 0; i < 16; ++i) acc[i] = (T)(a + 977u * i);                          \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    SV_NOUNROLL_LOOP for (int it = 0; it < ITERS; ++it) {
#define KERNEL_TAIL(T)                                                                               \
    }                                                                                                \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                                 \
    if ((threadIdx.x & 63) == 0) st[w] = Stamp{t0, t1, r0, r1};                                      \
    uint64_t s = 0;                                                                                  \
    for (int i = 0; i < 16; ++i) s ^= (uint64_t)acc[i];                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32)) + b;                      \
  }

// 32 instructions per iteration: ONE inline-asm statement of 16 instructions
// (accumulators %0..%15, inputs %16 %17), issued twice.  One statement, not
// one per instruction: the compiler's hazard recognizer pads every boundary
// between inline-asm statements that write SGPRs with an s_nop, which would
// be measured too.  Carry-out pairs rotate over 8 SGPR pairs.
#define OPS16 "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), \
              "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]), "+v"(acc[12]),            \
              "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15])
#define A16(F) F("0", SP0) F("1", SP1) F("2", SP2) F("3", SP3) F("4", SP4) F("5", SP5) F("6", SP6) F("7", SP7) \
               F("8", SP0) F("9", SP1) F("10", SP2) F("11", SP3) F("12", SP4) F("13", SP5) F("14", SP6) F("15", SP7)
#define DEF_KERNEL(NAME, T, F, INS...)                        \
  KERNEL_HEAD(NAME, T)                                        \
  asm volatile(A16(F) : OPS16 : INS : CLOB, "vcc");           \
  asm volatile(A16(F) : OPS16 : INS : CLOB, "vcc");           \
  KERNEL_TAIL(T)

#define F_MAD(i, P) "v_mad_u64_u32 %" i ", " P ", %16, %17, %" i "\n"
#define F_MADVCC(i, P) "v_mad_u64_u32 %" i ", vcc, %16, %17, %" i "\n"
#define F_ADDCO(i, P) "v_add_co_u32 %" i ", " P ", %" i ", %16\n"
#define F_ADDC(i, P) "v_addc_co_u32 %" i ", " P ", %" i ", %16, " P "\n"
#define F_MULLO(i, P) "v_mul_lo_u32 %" i ", %" i ", %16\n"
#define F_MULHI(i, P) "v_mul_hi_u32 %" i ", %" i ", %16\n"
#define F_ADD(i, P) "v_add_u32 %" i ", %" i ", %16\n"
#define F_ADD3(i, P) "v_add3_u32 %" i ", %" i ", %16, %17\n"
#define F_AND(i, P) "v_and_b32 %" i ", %" i ", %16\n"
#define F_XOR(i, P) "v_xor_b32 %" i ", %" i ", %16\n"
// VOP2 with a 32-bit literal (8-byte encoding) and with an SGPR operand
#define F_ANDLIT(i, P) "v_and_b32 %" i ", 0x3ffffff, %" i "\n"
#define F_ADDLIT(i, P) "v_add_u32 %" i ", 0x7ffffda, %" i "\n"
#define F_ANDSGPR(i, P) "v_and_b32 %" i ", %17, %" i "\n"
#define F_LSHL(i, P) "v_lshlrev_b32 %" i ", 1, %" i "\n"
#define F_LSHLV(i, P) "v_lshlrev_b32 %" i ", %17, %" i "\n"
#define F_ANDIC(i, P) "v_and_b32 %" i ", 7, %" i "\n"
#define F_ADDIC(i, P) "v_add_u32 %" i ", 1, %" i "\n"
#define F_SUB(i, P) "v_sub_u32 %" i ", %" i ", %16\n"
#define F_CNDS(i, P) "v_cndmask_b32_e64 %" i ", %" i ", %16, %18\n"
#define F_BFI(i, P) "v_bfi_b32 %" i ", %16, %" i ", %17\n"
#define F_LSHLADD(i, P) "v_lshl_add_u32 %" i ", %" i ", 1, %16\n"
#define F_ALIGNBIT(i, P) "v_alignbit_b32 %" i ", %" i ", %16, 7\n"
#define F_BFE(i, P) "v_bfe_u32 %" i ", %" i ", 3, 25\n"
#define F_CNDMASK(i, P) "v_cndmask_b32 %" i ", %" i ", %16, vcc\n"
#define F_LSHR64(i, P) "v_lshrrev_b64 %" i ", 26, %" i "\n"
#define F_LSHLADD64(i, P) "v_lshl_add_u64 %" i ", %" i ", 0, %17\n"
#define F_MOVDPP(i, P) "v_mov_b32_dpp %" i ", %" i " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define F_FMA(i, P) "v_fma_f32 %" i ", %" i ", %16, %17\n"
#define F_FMA64(i, P) "v_fma_f64 %" i ", %" i ", %16, %17\n"

DEF_KERNEL(k_mad_u64_u32, uint64_t, F_MAD, "v"(a), "v"(b))
// dependency distance 1 / 2 / 4: every mad accumulates into the result of the
// previous (1) or second / fourth previous mad -- the latency a column-major
// product (one dependent chain per column) exposes
#define A16D1(F) F("0", SP0) F("0", SP1) F("0", SP2) F("0", SP3) F("0", SP4) F("0", SP5) F("0", SP6) F("0", SP7) \
                 F("0", SP0) F("0", SP1) F("0", SP2) F("0", SP3) F("0", SP4) F("0", SP5) F("0", SP6) F("0", SP7)
#define A16D2(F) F("0", SP0) F("1", SP1) F("0", SP2) F("1", SP3) F("0", SP4) F("1", SP5) F("0", SP6) F("1", SP7) \
                 F("0", SP0) F("1", SP1) F("0", SP2) F("1", SP3) F("0", SP4) F("1", SP5) F("0", SP6) F("1", SP7)
#define A16D4(F) F("0", SP0) F("1", SP1) F("2", SP2) F("3", SP3) F("0", SP4) F("1", SP5) F("2", SP6) F("3", SP7) \
                 F("0", SP0) F("1", SP1) F("2", SP2) F("3", SP3) F("0", SP4) F("1", SP5) F("2", SP6) F("3", SP7)
#define DEF_KERNEL_D(NAME, T, AF, F, INS...)                  \
  KERNEL_HEAD(NAME, T)                                        \
  asm volatile(AF(F) : OPS16 : INS : CLOB, "vcc");            \
  asm volatile(AF(F) : OPS16 : INS : CLOB, "vcc");            \
  KERNEL_TAIL(T)
DEF_KERNEL_D(k_mad_dep1, uint64_t, A16D1, F_MAD, "v"(a), "v"(b))
DEF_KERNEL_D(k_mad_dep2, uint64_t, A16D2, F_MAD, "v"(a), "v"(b))
DEF_KERNEL_D(k_mad_dep4, uint64_t, A16D4, F_MAD, "v"(a), "v"(b))
DEF_KERNEL(k_mad_u64_u32_vcc, uint64_t, F_MADVCC, "v"(a), "v"(b))
DEF_KERNEL(k_add_co_u32, uint32_t, F_ADDCO, "v"(a), "v"(b))
DEF_KERNEL(k_addc_co_u32, uint32_t, F_ADDC, "v"(a), "v"(b))
DEF_KERNEL(k_mul_lo_u32, uint32_t, F_MULLO, "v"(a), "v"(b))
DEF_KERNEL(k_mul_hi_u32, uint32_t, F_MULHI, "v"(a), "v"(b))
DEF_KERNEL(k_add_u32, uint32_t, F_ADD, "v"(a), "v"(b))
DEF_KERNEL(k_add3_u32, uint32_t, F_ADD3, "v"(a), "v"(b))
DEF_KERNEL(k_and_b32, uint32_t, F_AND, "v"(a), "v"(b))
DEF_KERNEL(k_xor_b32, uint32_t, F_XOR, "v"(a), "v"(b))
DEF_KERNEL(k_and_lit, uint32_t, F_ANDLIT, "v"(a), "v"(b))
DEF_KERNEL(k_add_lit, uint32_t, F_ADDLIT, "v"(a), "v"(b))
DEF_KERNEL(k_and_sgpr, uint32_t, F_ANDSGPR, "v"(a), "s"(__builtin_amdgcn_readfirstlane(b)))
DEF_KERNEL(k_lshl_b32, uint32_t, F_LSHL, "v"(a), "v"(b))
DEF_KERNEL(k_lshl_v, uint32_t, F_LSHLV, "v"(a), "v"(b & 3u))
DEF_KERNEL(k_and_ic, uint32_t, F_ANDIC, "v"(a), "v"(b))
DEF_KERNEL(k_add_ic, uint32_t, F_ADDIC, "v"(a), "v"(b))
DEF_KERNEL(k_sub_u32, uint32_t, F_SUB, "v"(a), "v"(b))
DEF_KERNEL(k_bfi_b32, uint32_t, F_BFI, "v"(a), "v"(b))
// v_cndmask with a lane mask in an SGPR pair written by a v_cmp of this wave
// (F_CNDMASK above reads a vcc nothing in the kernel wrote)
DEF_KERNEL(k_cnd_sgpr, uint32_t, F_CNDS, "v"(a), "v"(b), "s"(__ballot((threadIdx.x ^ seed) & 1)))
DEF_KERNEL(k_lshl_add_u32, uint32_t, F_LSHLADD, "v"(a), "v"(b))
DEF_KERNEL(k_alignbit_b32, uint32_t, F_ALIGNBIT, "v"(a), "v"(b))
DEF_KERNEL(k_bfe_u32, uint32_t, F_BFE, "v"(a), "v"(b))
DEF_KERNEL(k_cndmask_b32, uint32_t, F_CNDMASK, "v"(a), "v"(b))
DEF_KERNEL(k_lshrrev_b64, uint64_t, F_LSHR64, "v"(a), "v"((uint64_t)b))
DEF_KERNEL(k_lshl_add_u64, uint64_t, F_LSHLADD64, "v"(a), "v"((uint64_t)b))
DEF_KERNEL(k_mov_dpp, uint32_t, F_MOVDPP, "v"(a), "v"(b))

// Mixed streams: 8 mads interleaved with 8 other instructions on separate
// accumulators -- are the other instructions' issue cycles additive to the
// mads' or hidden behind them?  (lane_ops below counts both.)
#define MIXK(NAME, OTHER)                                                                              \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, Stamp* st, uint32_t seed) {               \
    uint32_t a = threadIdx.x * 2654435761u + seed, b = a * 3u + 1u;                                    \
    uint64_t m[8];                                                                                     \
    uint32_t x[8];                                                                                     \
    for (int i = 0; i < 8; ++i) { m[i] = a + 977u * i; x[i] = b + 13u * i; }                           \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    SV_NOUNROLL_LOOP for (int it = 0; it < ITERS; ++it) {                                              \
      asm volatile(MIX8(OTHER) MIX8(OTHER)                                                             \
                   : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3]), "+v"(m[4]), "+v"(m[5]), "+v"(m[6]), \
                     "+v"(m[7]), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), \
                     "+v"(x[6]), "+v"(x[7])                                                            \
                   : "v"(a), "v"(b)                                                                    \
                   : CLOB, "vcc");                                                                     \
    }                                                                                                  \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                                   \
    if ((threadIdx.x & 63) == 0) st[w] = Stamp{t0, t1, r0, r1};                                        \
    uint64_t s = 0;                                                                                    \
    for (int i = 0; i < 8; ++i) s ^= m[i] ^ x[i];                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));                            \
  }
// pairs (mad on m[i], OTHER on x[i]) for i = 0..7: 16 instructions
#define MIXP(i, j, P, OTHER) "v_mad_u64_u32 %" i ", " P ", %16, %17, %" i "\n" OTHER(j)
#define MIX8(OTHER) MIXP("0", "8", SP0, OTHER) MIXP("1", "9", SP1, OTHER) MIXP("2", "10", SP2, OTHER) \
                    MIXP("3", "11", SP3, OTHER) MIXP("4", "12", SP4, OTHER) MIXP("5", "13", SP5, OTHER) \
                    MIXP("6", "14", SP6, OTHER) MIXP("7", "15", SP7, OTHER)
#define O_ADD(j) "v_add_u32 %" j ", %" j ", %16\n"
#define O_AND(j) "v_and_b32 %" j ", 0x3ffffff, %" j "\n"
#define O_LSHL(j) "v_lshlrev_b32 %" j ", 1, %" j "\n"
#define O_MUL(j) "v_mul_lo_u32 %" j ", %" j ", 19\n"
#define O_MAD(j) "v_mad_u32_u24 %" j ", %" j ", 19, %16\n"
#define O_NOP(j) "s_nop 0\n"
MIXK(k_mix_add, O_ADD)
MIXK(k_mix_and, O_AND)
MIXK(k_mix_lshl, O_LSHL)
MIXK(k_mix_mul, O_MUL)
MIXK(k_mix_nop, O_NOP)

// float kernels (own heads: float accumulators)
#define FKERNEL(NAME, T, F)                                                                            \
  __global__ __launch_bounds__(256) void NAME(uint32_t* out, Stamp* st, uint32_t seed) {               \
    const T fa = (T)0.999, fb = (T)1e-7;                                                               \
    T acc[16];                                                                                         \
    for (int i = 0; i < 16; ++i) acc[i] = (T)(1.0f + 1e-3f * (threadIdx.x + seed + i));                \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    for (int it = 0; it < ITERS; ++it) {                                                               \
      asm volatile(A16(F) : OPS16 : "v"(fa), "v"(fb));                                                 \
      asm volatile(A16(F) : OPS16 : "v"(fa), "v"(fb));                                                 \
    }                                                                                                  \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                                   \
    if ((threadIdx.x & 63) == 0) st[w] = Stamp{t0, t1, r0, r1};                                        \
    double s = 0;                                                                                      \
    for (int i = 0; i < 16; ++i) s += (double)acc[i];                                                  \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(int64_t)s;                                 \
  }
FKERNEL(k_fma_f32, float, F_FMA)
FKERNEL(k_fma_f64, double, F_FMA64)

typedef void (*kfn)(uint32_t*, Stamp*, uint32_t);

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("device %s CUs=%d, %d instructions per lane per kernel (ITERS=%d x 32)\n", p.gcnArchName, cus, ITERS * 32,
         ITERS);
  struct {
    const char* name;
    kfn k;
    int lane_ops;  // lane-operations per instruction (packed: 2)
  } ks[] = {{"v_fma_f32 (guide: 2 cyc/wave-inst)", k_fma_f32, 1},
            {"v_fma_f64", k_fma_f64, 1},
            {"v_mad_u64_u32 (8 rotating sdst pairs)", k_mad_u64_u32, 1},
            {"v_mad_u64_u32 (sdst vcc every inst)", k_mad_u64_u32_vcc, 1},
            {"v_mad_u64_u32 dependency distance 1", k_mad_dep1, 1},
            {"v_mad_u64_u32 dependency distance 2", k_mad_dep2, 1},
            {"v_mad_u64_u32 dependency distance 4", k_mad_dep4, 1},
            {"v_mul_lo_u32", k_mul_lo_u32, 1},
            {"v_mul_hi_u32", k_mul_hi_u32, 1},
            {"v_add_u32", k_add_u32, 1},
            {"v_add3_u32", k_add3_u32, 1},
            {"v_add_co_u32 (8 rotating sdst)", k_add_co_u32, 1},
            {"v_addc_co_u32 (8 rotating sdst)", k_addc_co_u32, 1},
            {"v_and_b32", k_and_b32, 1},
            {"v_xor_b32", k_xor_b32, 1},
            {"v_and_b32 32-bit literal", k_and_lit, 1},
            {"v_add_u32 32-bit literal", k_add_lit, 1},
            {"v_and_b32 SGPR operand", k_and_sgpr, 1},
            {"v_lshlrev_b32 inline constant", k_lshl_b32, 1},
            {"v_lshlrev_b32 VGPR shift", k_lshl_v, 1},
            {"v_and_b32 inline constant", k_and_ic, 1},
            {"v_add_u32 inline constant", k_add_ic, 1},
            {"v_sub_u32", k_sub_u32, 1},
            {"v_bfi_b32", k_bfi_b32, 1},
            {"v_cndmask_b32_e64 (ballot mask in SGPRs)", k_cnd_sgpr, 1},
            {"v_lshl_add_u32", k_lshl_add_u32, 1},
            {"v_alignbit_b32", k_alignbit_b32, 1},
            {"v_bfe_u32", k_bfe_u32, 1},
            {"v_cndmask_b32", k_cndmask_b32, 1},
            {"v_lshrrev_b64", k_lshrrev_b64, 1},
            {"v_lshl_add_u64", k_lshl_add_u64, 1},
            {"v_mov_b32_dpp quad_perm", k_mov_dpp, 1},
            {"mix: v_mad_u64_u32 + v_add_u32 (1:1)", k_mix_add, 1},
            {"mix: v_mad_u64_u32 + v_and_b32 literal (1:1)", k_mix_and, 1},
            {"mix: v_mad_u64_u32 + v_lshlrev_b32 (1:1)", k_mix_lshl, 1},
            {"mix: v_mad_u64_u32 + v_mul_lo_u32 (1:1)", k_mix_mul, 1},
            {"mix: v_mad_u64_u32 + s_nop 0 (1:1)", k_mix_nop, 1}};
  const int maxblocks = cus * 8;
  uint32_t* d_out;
  Stamp* d_st;
  hipMalloc(&d_out, sizeof(uint32_t) * maxblocks * 256);
  hipMalloc(&d_st, sizeof(Stamp) * maxblocks * 4);
  std::vector<Stamp> st(maxblocks * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("%-40s %5s %10s %12s %14s %14s\n", "instruction", "w/SIMD", "clk GHz", "cyc/inst/SIMD",
         "lane-ops/clk/CU", "wall lane-op/s");
  for (auto& k : ks) {
    for (int occ : {1, 2, 4, 8}) {
      const int blocks = cus * occ;
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d_out, d_st, 1u);  // warm (clocks up)
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d_out, d_st, 1u);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, d_out, d_st, 2u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const int waves = blocks * 4;
      hipMemcpy(st.data(), d_st, sizeof(Stamp) * waves, hipMemcpyDeviceToHost);
      unsigned long long rmin = ~0ull, rmax = 0;
      double cyc = 0, rt = 0;
      for (int w = 0; w < waves; ++w) {
        rmin = std::min(rmin, st[w].r0);
        rmax = std::max(rmax, st[w].r1);
        cyc += (double)(st[w].t1 - st[w].t0);
        rt += (double)(st[w].r1 - st[w].r0);
      }
      const double ghz = cyc / rt * 0.1;                  // s_memrealtime ticks at 100 MHz
      const double span_s = (double)(rmax - rmin) * 1e-8;  // earliest start .. latest end
      const double inst = (double)waves * 64.0 * ITERS * 32.0 * k.lane_ops;
      const double per_clk_cu = inst / (span_s * ghz * 1e9 * cus);
      // per-SIMD issue cycles per wave-instruction: span cycles / instructions per SIMD
      const double cyc_per_inst = span_s * ghz * 1e9 / ((double)occ * ITERS * 32.0);
      printf("%-40s %5d %10.3f %12.2f %14.1f %14.3e\n", k.name, occ, ghz, cyc_per_inst, per_clk_cu,
             inst / (ms * 1e-3));
    }
  }
  hipFree(d_out);
  hipFree(d_st);
  return 0;
}
