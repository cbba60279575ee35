#!/bin/bash
# Developer tool: timing-only diagnostic builds of the warm-key comb kernel
# (wrong verdicts by design), linked with the product's other objects into
# variants/libsv_diag_*.so for tools/ab_lat_capi.py.  The product sources are
# not modified: each variant compiles a patched copy of sv_comb.hip.
#   nodecode  decode wave: R's y only, no square root
#   nohash    chain waves: no SHA-512 (hram from R ^ A and S)
#   both      both of the above
#   phases    the product's arithmetic plus per-wave s_memrealtime stamps at
#             the phase boundaries, read back by sv_diag_comb_times()
#   ophases   the same stamps in the cold-key octet kernel (sv_kernels.hip),
#             read back by sv_diag_octet_times()
set -e
cd "$(dirname "$0")/.."
mkdir -p variants/build
C=stellar-core_amd/csrc
T=$(mktemp -d)
cp $C/*.h $C/sv_comb.hip $C/sv_kernels.hip $T/
python3 - "$T" <<'PY'
import sys
t = sys.argv[1]
src = open(t + "/sv_comb.hip").read()
dec_a = "      ok = ge_frombytes(Rp, R, false) && ok;"
dec_b = "      fe_frombytes(Rp.Y, R);\n      Rp.X = Rp.Y;"
hash_a = "  sv_load_and_hash_lds<MODE, LPS>(p, gi, lane % LPS, s_msg[wave - 1] + sw * (SV_MSG_CAP / 16), A, S, hram);"
hash_b = ("  {\n    uint32_t R_[8];\n    sv_unpack2(A, p.pk + 2 * gi);\n    sv_unpack2(R_, p.sig + 4 * gi);\n"
          "    sv_unpack2(S, p.sig + 4 * gi + 2);\n"
          "    for (int i = 0; i < 8; ++i) { hram[i] = R_[i] ^ A[i]; hram[8 + i] = S[i]; }\n  }")
assert dec_a in src and hash_a in src
open(t + "/comb_nodecode.hip", "w").write(src.replace(dec_a, dec_b))
open(t + "/comb_nohash.hip", "w").write(src.replace(hash_a, hash_b))
open(t + "/comb_both.hip", "w").write(src.replace(dec_a, dec_b).replace(hash_a, hash_b))
# phase stamps: wave w of workgroup b writes stamp k to sv_diag_t[b][w][k]
ph = src
hdr = ("__device__ unsigned long long sv_diag_t[1024][4][8];\n"
       "#define SV_DT(k) do { SV_FENCE(); const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); "
       "SV_FENCE(); if (__lane_id() == 0 && blockIdx.x < 1024) sv_diag_t[blockIdx.x][wave][k] = t_; } while (0)\n")
anchor = "// One signature per SPW-th of a chain wave; see the file header."
assert anchor in ph
ph = ph.replace(anchor, hdr + anchor)
reps = [
  ("  if (wave == 0) {\n", "  SV_DT(0);\n  if (wave == 0) {\n"),
  ("      s_rok[lane] = ok ? 1u : 0u;\n    }\n    __syncthreads();\n", "      s_rok[lane] = ok ? 1u : 0u;\n    }\n    SV_DT(1);\n    __syncthreads();\n    SV_DT(2);\n"),
  (hash_a, hash_a + "\n  SV_DT(1);"),
  ("  sc_digits_r256(dB, S);\n", "  sc_digits_r256(dB, S);\n  SV_DT(2);\n"),
  ("  qo_from_cached(P, entB[0], q, negB[0]);\n", "  qo_from_cached(P, entB[0], q, negB[0]);\n  SV_DT(3);\n"),
  ("    SV_UNROLL for (int t = 0; t < PA; ++t) qo_add(P, ent[t], q, eneg[t]);\n  }\n", "    SV_UNROLL for (int t = 0; t < PA; ++t) qo_add(P, ent[t], q, eneg[t]);\n  }\n  SV_DT(4);\n"),
  ("  __syncthreads();  // x_R, y_R from the decode wave\n", "  SV_DT(5);\n  __syncthreads();  // x_R, y_R from the decode wave\n  SV_DT(6);\n"),
  ("  if (active && quad == 0 && role == 0) p.verdict[g] = ok ? 1 : 0;\n}", "  if (active && quad == 0 && role == 0) p.verdict[g] = ok ? 1 : 0;\n  SV_DT(7);\n}"),
  ('extern "C" {\n', 'extern "C" {\n\nint sv_diag_comb_times(void* out, size_t bytes) {\n  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(sv_diag_t), bytes);\n}\n'),
]
for a, b in reps:
    assert ph.count(a) == 1, a
    ph = ph.replace(a, b)
open(t + "/comb_phases.hip", "w").write(ph)
# octet kernel stamps: wave w of workgroup b writes stamp k to sv_diag_o[b][w][k]
ok = open(t + "/sv_kernels.hip").read()
ohdr = ("__device__ unsigned long long sv_diag_o[2048][2][8];\n"
        "#define SV_OT(k) do { SV_FENCE(); const unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); "
        "SV_FENCE(); if (__lane_id() == 0 && blockIdx.x < 2048) sv_diag_o[blockIdx.x][threadIdx.x >> 6][k] = t_; } while (0)\n")
anchor = "template <int MODE, bool MSG>\n__global__ __launch_bounds__(SV_OCTET_BLOCK, 1) void sv_octet_kernel"
assert ok.count(anchor) == 1
ok = ok.replace(anchor, ohdr + anchor)
oreps = [
  ("  uint32_t A[8], S[8], hram[16], R[8];\n  if (dec_wave) {", "  SV_OT(0);\n  uint32_t A[8], S[8], hram[16], R[8];\n  if (dec_wave) {"),
  ("    const uint32_t dok = ge_frombytes(Pt, E, true) ? 1u : 0u;\n", "    const uint32_t dok = ge_frombytes(Pt, E, true) ? 1u : 0u;\n    SV_OT(1);\n"),
  ("      if (store) sv_store_lentry((sv_u4*)(tab + e * SV_QENT_DW), ce);\n    }\n  }\n", "      if (store) sv_store_lentry((sv_u4*)(tab + e * SV_QENT_DW), ce);\n    }\n    SV_OT(2);\n  }\n"),
  ("    __syncthreads();  // tables and s_dok written; s_bd read below\n", "    __syncthreads();  // tables and s_dok written; s_bd read below\n    SV_OT(3);\n"),
  ("    __syncthreads();  // s_pb written\n    return;", "    SV_OT(4);\n    __syncthreads();  // s_pb written\n    SV_OT(5);\n    return;"),
  ("  }\n  const int W = sv_wave_windows(sv_lat_windows(lat.bits), p.dbg);\n", "  }\n  SV_OT(2);\n  const int W = sv_wave_windows(sv_lat_windows(lat.bits), p.dbg);\n"),
  ("  __syncthreads();  // tables visible to the whole quad\n", "  SV_OT(3);\n  __syncthreads();  // tables visible to the whole quad\n  SV_OT(4);\n"),
  ("  ge_p3 P;\n  qo_expand(P, h);\n  // quad 0: P_A + P_R", "  SV_OT(5);\n  ge_p3 P;\n  qo_expand(P, h);\n  // quad 0: P_A + P_R"),
  ("    __syncthreads();  // [s]B from wave 1\n", "    __syncthreads();  // [s]B from wave 1\n    SV_OT(6);\n"),
  ('extern "C" {\n', 'extern "C" {\n\nint sv_diag_octet_times(void* out, size_t bytes) {\n  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(sv_diag_o), bytes);\n}\n'),
]
for a, b in oreps:
    assert ok.count(a) == 1, a
    ok = ok.replace(a, b)
# hash wave: stamp 1 after the hash (the decode wave's stamp 1 is its square roots)
a = "    sv_unpack2(R, p.sig + 4 * ii);\n  }\n  bool ok = true;"
assert ok.count(a) == 1
ok = ok.replace(a, "    sv_unpack2(R, p.sig + 4 * ii);\n    SV_OT(1);\n  }\n  bool ok = true;")
open(t + "/kernels_ophases.hip", "w").write(ok)
PY
for v in nodecode nohash both phases; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $T/comb_$v.hip -o variants/build/comb_$v.o &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c $T/kernels_ophases.hip -o variants/build/k_ophases.o &
wait
B=stellar-core_amd/build
for v in nodecode nohash both phases; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libsv_diag_$v.so $B/sv_kernels.o variants/build/comb_$v.o \
      $B/sv_api.o $B/sv_hash.o $B/sv_cpu.o -Wl,-rpath,/opt/rocm/lib -lpthread
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/libsv_diag_ophases.so variants/build/k_ophases.o \
    $B/sv_comb.o $B/sv_api.o $B/sv_hash.o $B/sv_cpu.o -Wl,-rpath,/opt/rocm/lib -lpthread
rm -rf $T
ls -la variants/libsv_diag_*.so
