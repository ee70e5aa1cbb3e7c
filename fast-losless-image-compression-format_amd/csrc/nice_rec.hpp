// nice_rec.hpp -- the encoder's per-pixel record and the packer's code tables.
//
// One u32 per pixel, written by the classify kernels and read by the packer:
//   bits  3..13  c0: the pixel's first payload symbol, prefix implied by its range
//   bits 14..22  s1: second payload slot
//   bits 23..31  s2: third payload slot
//   bits  0..2   zero (c0 << 3 is the byte offset of an 8-byte table entry)
//
// A coded pixel emits its mode prefix, then its payload symbols, in this order
// (code.rs:191-366):
//   BACK_REF   prefix, k                c0 = C0_BR + k
//   SMALL_DIFF prefix, index            c0 = C0_SD + index
//   LUMA2      prefix, g, r, b          c0 = C0_L2 + g,          s1 = SX_L2 + r,   s2 = SX_L2 + b
//   LUMA       prefix, k, g, r, b       c0 = C0_LUMA + 64 k + g, s1 = SX_LUMA + r, s2 = SX_LUMA + b
//   RGB        prefix, r, g, b          c0 = C0_RGB + r,         s1 = SX_RGB + g,  s2 = SX_RGB + b
// (g, r, b: the biased payload values g+32, r+16, b+16 or the raw residuals.)
// So a pixel's codes are three table lookups in emission order: T0[c0] holds
// the mode prefix's code followed by c0's symbol code(s) (LUMA: k and g), T1[s1]
// and T2[s2] the others.  Slots a mode does not use point at SX_ABS + lane, and
// run members (uncoded pixels) have c0 = C0_UNC + lane: zero-length entries,
// one per lane so the classify histogram's atomics on them do not collide.
// The histogram of the three slot spaces converts to the reference's 858
// symbol bins (hfe.rs:29-45) once per block and frame.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nice_format.h"

namespace nice {

constexpr uint32_t C0_RGB = 0, C0_BR = 256, C0_SD = 261, C0_L2 = 604, C0_LUMA = 668, C0_UNC = 1372,
                   C0_N = 1436;
constexpr uint32_t SX_RGB = 0, SX_L2 = 256, SX_LUMA = 288, SX_ABS = 320, SX_N = 384;
// run digits (prefixes 5..12, code.rs:391-406) after a coded pixel, m = run - 1:
// entries 0..63 the natural digits of m, 64 + x the two digits (x & 7, x >> 3)
// of a longer run's first two, 128 no run
constexpr uint32_t RC_TWO = 64, RC_NONE = 128, RC_N = 130;

__host__ __device__ constexpr uint32_t rec2_abs(uint32_t lane) {
  return ((SX_ABS + lane) << 14) | ((SX_ABS + lane) << 23);
}
__host__ __device__ constexpr uint32_t rec2_unc(uint32_t lane) { return ((C0_UNC + lane) << 3) | rec2_abs(lane); }
__host__ __device__ constexpr uint32_t rec2_c0(uint32_t rec) { return (rec >> 3) & 0x7FFu; }
__host__ __device__ constexpr uint32_t rec2_s1(uint32_t rec) { return (rec >> 14) & 0x1FFu; }
__host__ __device__ constexpr uint32_t rec2_s2(uint32_t rec) { return rec >> 23; }
__host__ __device__ constexpr bool rec2_coded(uint32_t rec) { return rec2_c0(rec) < C0_UNC; }

// The symbols of a coded record in emission order as histogram bins: b[0] the
// mode prefix, then the payloads; returns their number (0: run member).
__host__ __device__ inline uint32_t rec2_syms(uint32_t rec, uint32_t (&b)[5]) {
  const uint32_t c0 = rec2_c0(rec), s1 = rec2_s1(rec), s2 = rec2_s2(rec);
  if (c0 >= C0_UNC) return 0;
  if (c0 < C0_BR) {
    b[0] = BIN_PREFIX + P_RGB; b[1] = c0; b[2] = s1; b[3] = s2;
    return 4;
  }
  if (c0 < C0_SD) { b[0] = BIN_PREFIX + P_BACK_REF; b[1] = BIN_BACK_REF + (c0 - C0_BR); return 2; }
  if (c0 < C0_L2) { b[0] = BIN_PREFIX + P_SMALL_DIFF; b[1] = BIN_SMALL_DIFF + (c0 - C0_SD); return 2; }
  if (c0 < C0_LUMA) {
    b[0] = BIN_PREFIX + P_LUMA2; b[1] = BIN_LUMA2_BASE + (c0 - C0_L2);
    b[2] = BIN_LUMA2_R + (s1 - SX_L2); b[3] = BIN_LUMA2_B + (s2 - SX_L2);
    return 4;
  }
  const uint32_t kg = c0 - C0_LUMA;
  b[0] = BIN_PREFIX + P_LUMA; b[1] = BIN_LUMA_REF + (kg >> 6); b[2] = BIN_LUMA_BASE + (kg & 63u);
  b[3] = BIN_LUMA_OTHER + (s1 - SX_LUMA); b[4] = BIN_LUMA_OTHER + (s2 - SX_LUMA);
  return 5;
}

// Histogram bin -> its count from the slot-space histogram h (C0_N + 2 SX_N
// words: c0 counts, s1 counts, s2 counts); the mode prefixes are derived by
// enc_tables and the run digits are counted separately (0 here).
__device__ __forceinline__ uint32_t slot_hist_bin(const uint32_t* h, int b) {
  const uint32_t* h1 = h + C0_N;
  const uint32_t* h2 = h1 + SX_N;
  if (b < 256) return h[C0_RGB + b] + h1[SX_RGB + b] + h2[SX_RGB + b];
  if (b < BIN_LUMA_BASE) return 0u;
  if (b < BIN_LUMA_OTHER) {   // g of LUMA: summed over the 11 references
    uint32_t s = 0;
    for (int k = 0; k < 11; ++k) s += h[C0_LUMA + 64 * k + (b - BIN_LUMA_BASE)];
    return s;
  }
  if (b < BIN_LUMA_REF) return h1[SX_LUMA + (b - BIN_LUMA_OTHER)] + h2[SX_LUMA + (b - BIN_LUMA_OTHER)];
  if (b < BIN_SMALL_DIFF) {   // k of LUMA: summed over g
    uint32_t s = 0;
    const uint32_t* p = h + C0_LUMA + 64 * (b - BIN_LUMA_REF);
    for (int g = 0; g < 64; ++g) s += p[g];
    return s;
  }
  if (b < BIN_LUMA2_BASE) return h[C0_SD + (b - BIN_SMALL_DIFF)];
  if (b < BIN_LUMA2_R) return h[C0_L2 + (b - BIN_LUMA2_BASE)];
  if (b < BIN_LUMA2_B) return h1[SX_L2 + (b - BIN_LUMA2_R)];
  if (b < BIN_BACK_REF) return h2[SX_L2 + (b - BIN_LUMA2_B)];
  return b - BIN_BACK_REF < 5 ? h[C0_BR + (b - BIN_BACK_REF)] : 0u;
}

// The packer's per-frame code tables (built by enc_packtab, copied to LDS):
// {code, length}, code right-aligned, length <= 32.
struct PackTab {
  uint2 t0[C0_N];
  uint2 t1[SX_N];
  uint2 t2[SX_N];
  uint2 rc[RC_N];
};
static_assert(sizeof(PackTab) % 16 == 0, "16-byte copies");

}  // namespace nice
