// Layout of the comb tables of the warm-key latency path (sv_comb.hip),
// shared by the device code and the host engine (sv_api.cpp).
//
// The latency path evaluates libsodium's own equation
//
//     [S]B + [h](-A) == R_pt        (h = SHA-512(R || A || M) mod L)
//
// as a sum of precomputed points instead of a scalar multiplication:
//
//   [h](-A) = sum_j d_j * (16^j (-A))      64 signed radix-16 digits of h
//   [S]B    = sum_j e_j * (256^j B)        32 signed radix-256 digits of S
//
// so a signature costs 96 table lookups and ~9 point additions on the
// critical path (a tree over the 16 lane quads of one wave) instead of ~130
// doublings.  The tables of -A depend only on the 32 public-key bytes, so
// they are built once per key (one wave per key, ~0.3 ms) and kept in a
// bounded per-device key cache: SCP traffic is signed by a few hundred
// validator keys (BASELINE config 4: 100), which is exactly the workload the
// latency path serves.  Keys not (yet) in the cache take the octet kernel
// (sv_kernels.hip), which needs no per-key state.  Verdicts are identical:
// both evaluate libsodium's checks (1)-(8) exactly (see sv_comb.hip).
//
// Entry format (both table kinds): a point in cached form (Y+X, Y-X, Z, 2dT),
// each coordinate 10 limbs (radix 2^25.5, carried: R+) padded to 12 dwords
// so that a lane loads its coordinate with three 16-byte loads.
#pragma once

#define SV_CE_DW 48          // dwords per entry: 4 coordinates x 12
#define SV_KA_POS 64         // -A tables: positions j (weight 16^j)
#define SV_KA_ENT 9          //   entries |d| = 0..8 (signed radix-16 digits in [-8, 8])
#define SV_KEY_SLOT_DW (SV_KA_POS * SV_KA_ENT * SV_CE_DW)  // 27648 dwords = 108 KiB per key
#define SV_CB_POS 32         // B tables: positions j (weight 256^j)
#define SV_CB_ENT 129        //   entries e = 0..128 (signed digits in [-128, 127])
#define SV_CB_DW (SV_CB_POS * SV_CB_ENT * SV_CE_DW)        // 774 KiB per device

// per-slot key status (written by the key-table build kernel)
#define SV_KEY_BAD 0u  // A non-canonical, small-order or not on the curve: every signature rejects
#define SV_KEY_OK 1u

// signatures per workgroup of the comb kernel: 1 decode wave + 3 chain waves,
// each chain wave verifies SPW signatures (16 / SPW lane quads per signature)
#define SV_COMB_CHAIN_WAVES 3
