// nice_classify.hpp -- per-pixel mode decision of the NICE2 encoder on gfx950.
//
// Restates the body of the reference encoder's main loop (code.rs:159-414) as a
// pure function of the ORIGINAL input pixels, which is what makes the encoder
// data-parallel: the reference's `prev_position` is always pixel i-1 (run skips
// leave `position` on the last run pixel, code.rs:390,412), and every test reads
// original bytes only.
//
// Pixels are held in a "spread" form, X' = R | G<<10 | B<<20 (alpha and any
// byte past +2 are ignored, as in code.rs:197,215-217), so that one 32-bit
// integer op performs the three per-channel operations of the reference with
// 2 guard bits per field (no borrows or carries cross a field).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nice_format.h"

namespace nice {

__host__ __device__ constexpr uint32_t K3(uint32_t x) { return x | (x << 10) | (x << 20); }

__device__ __forceinline__ uint32_t spread_rgba(uint32_t v) {
  return (v & 0xFFu) | ((v & 0xFF00u) << 2) | ((v & 0xFF0000u) << 4);
}
__device__ __forceinline__ uint32_t spread_rgb(uint32_t r, uint32_t g, uint32_t b) {
  return r | (g << 10) | (b << 20);
}
// floor((U+L)/2) per channel: code.rs:220-222 (i16) and 260-266 (u16) agree.
__device__ __forceinline__ uint32_t avg3(uint32_t u, uint32_t l) {
  return ((u + l) >> 1) & K3(0xFFu);
}
__device__ __forceinline__ uint32_t fld(uint32_t v, int c) { return (v >> (10 * c)) & 0xFFu; }

// Symbols of one coded pixel, excluding run digits: the mode prefix
// (bin BIN_PREFIX + mode) followed by n payload bins.
struct PixSyms {
  uint32_t mode;
  uint32_t n;
  uint32_t b[4];
};

// Luma-style test shared by LUMA2 (code.rs:255-290) and LUMA (code.rs:296-336):
//   g = XG - RG, r = XR - RR - g, b = XB - RB - g (all u8 wrapping);
//   fires iff g+32, r+16, b+16 (mod 256) are < 64, < 32, < 32.
// xk = X' + LUMA_K; returns t with fields (r+16, g+32, b+16) in the low 8 bits
// of each 10-bit field (upper 2 bits are don't-care).
constexpr uint32_t LUMA_K = 560u | (288u << 10) | (560u << 20);
constexpr uint32_t LUMA_MASK = 0xE0u | (0xC0u << 10) | (0xE0u << 20);
__device__ __forceinline__ uint32_t luma_t(uint32_t xk, uint32_t ref) {
  const uint32_t d = xk - ref;                 // fields: R,B in [305,815], G in [33,543]
  const uint32_t g8 = (d >> 10) & 0xFFu;       // (g + 32) mod 256
  return d - (g8 | (g8 << 20));                // R,B fields: X-R-g8+560 in [50,815]
}

// Fetch functor contract: a(rows, px) returns X' of pixel i - (rows*W + px).
// FAST: caller guarantees i >= 3W+3 and W >= 3, so every reference is valid.
template <bool FAST, class Acc>
__device__ __forceinline__ void classify(uint32_t i, uint32_t W, const Acc& a, PixSyms& o) {
  const uint32_t X = a(0, 0);
  auto valid = [&](int rows, int px) -> bool {
    if (FAST) return true;
    const int64_t off = (int64_t)rows * (int64_t)W + px;  // usize wrap below 0 => never valid
    return off >= 0 && (int64_t)i >= off;
  };
  const bool has_up = FAST || i >= W;

  // Back references, code.rs:191-206. k=0 (pixel i-1) cannot match a coded pixel
  // except through offset 0 (W==1), which valid() and the compare handle.
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    if (valid(br_rows(k), br_px(k)) && a(br_rows(k), br_px(k)) == X) {
      o.mode = P_BACK_REF; o.n = 1; o.b[0] = BIN_BACK_REF + k;
      return;
    }
  }
  const uint32_t L = (FAST || i > 0) ? a(0, 1) : X;  // prev_position == position at i == 0
  uint32_t pred = L;
  uint32_t U = 0;
  if (has_up) { U = a(1, 0); pred = avg3(U, L); }

  // Small diff, code.rs:208-247: every X_c - pred_c in [-3, 3].
  if (FAST || i > 0) {
    const uint32_t d = X + K3(259u) - pred;  // fields in [4, 514]
    const bool hi_ok = (d & K3(0x3F8u)) == K3(0x100u);
    const bool lo_ok = (((d & K3(7u)) + K3(1u)) & K3(8u)) == 0;
    if (hi_ok && lo_ok) {
      o.mode = P_SMALL_DIFF; o.n = 1;
      o.b[0] = BIN_SMALL_DIFF + (d & 7u) + 7u * ((d >> 10) & 7u) + 49u * ((d >> 20) & 7u);
      return;
    }
  }
  const uint32_t xk = X + LUMA_K;
  // Luma2 against floor((U+L)/2), code.rs:252-292 (only when i >= W).
  if (has_up) {
    const uint32_t t = luma_t(xk, pred);
    if ((t & LUMA_MASK) == 0) {
      o.mode = P_LUMA2; o.n = 3;
      o.b[0] = BIN_LUMA2_BASE + ((t >> 10) & 0xFFu);
      o.b[1] = BIN_LUMA2_R + (t & 0xFFu);
      o.b[2] = BIN_LUMA2_B + ((t >> 20) & 0xFFu);
      return;
    }
  }
  // Luma against 11 relative references, first hit wins: code.rs:293-339.
  if (FAST || i > 0) {
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      if (valid(lr_rows(k), lr_px(k))) {
        const uint32_t t = luma_t(xk, a(lr_rows(k), lr_px(k)));
        if ((t & LUMA_MASK) == 0) {
          o.mode = P_LUMA; o.n = 4;
          o.b[0] = BIN_LUMA_REF + k;
          o.b[1] = BIN_LUMA_BASE + ((t >> 10) & 0xFFu);
          o.b[2] = BIN_LUMA_OTHER + (t & 0xFFu);
          o.b[3] = BIN_LUMA_OTHER + ((t >> 20) & 0xFFu);
          return;
        }
      }
    }
  }
  // Raw residual, code.rs:341-366: vs floor((U+L)/2) if i >= W, vs L if 0 < i < W,
  // vs 0 at i == 0; all mod 256.
  const uint32_t base = (FAST || i > 0) ? pred : 0u;
  const uint32_t r = X + K3(256u) - base;
  o.mode = P_RGB; o.n = 3;
  o.b[0] = fld(r, 0);
  o.b[1] = fld(r, 1);
  o.b[2] = fld(r, 2);
}

// Number of base-8 run digits emitted for a run of r >= 1 repeated pixels
// (code.rs:391-406: m = r-1, emit m%8 then m/=8 until m < 8).
__device__ __forceinline__ uint32_t run_digits(uint64_t r) {
  uint64_t m = r - 1;
  uint32_t n = 1;
  while (m >= 8) { m >>= 3; ++n; }
  return n;
}

}  // namespace nice
