// Per-key tables of the throughput path: layout and launch parameters shared
// by the kernels (sv_kernels.hip) and the host side (sv_api.cpp).  The design
// is described in sv_kernels.hip above sv_keyslot_kernel.
#pragma once

#include <cstdint>

struct sv_u4;  // (verify_core.h: 16-byte quad)

// (sv_kparams::dbg bit set by the host, never a user flag) the launch serves
// the latency lane: the kernel raises its waves' priority (s_setprio 3)
#define SV_KP_LAT 0x80000000u
#define SV_KP_OCT_HI 0x40000000u  // (octet launches) the three-wave variant (sv_kernels.hip sv_octet_kernel HI)
#define SV_KP_OCT_HI_WIDE 0x20000000u  // (with SV_KP_OCT_HI) the high wave takes more windows
#define SV_KP_IN_PLACE 0x10000000u  // (throughput launches) the inputs are read in place from mapped host memory

#define SV_KT_TQUADS 90  // table_A: SV_ATAB_ENTRIES x SV_LTAB_QUADS (checked in sv_kernels.hip)
#define SV_KT_QUADS (SV_KT_TQUADS + 3)                   // + pk (2 quads) + status
#define SV_KT_NONE 0xffffffffu
#define SV_KT_PROBES 16
struct sv_ktparams {
  unsigned long long* index;  // mask + 1 claim words (0: empty, else the claiming key's fingerprint)
  sv_u4* store;               // (mask + 1) x SV_KT_QUADS; null: tables off
  uint32_t* kslot;            // per chunk lane: the key's slot or SV_KT_NONE
  uint32_t* builders;         // slots claimed in this chunk
  uint32_t* count;            // [0] slots claimed in this chunk, [1] claims since the index was cleared
  uint64_t mask;
  uint32_t limit;             // no claims once count[1] reaches it
  uint64_t salt;
};
