// nice_bits.hpp -- device-side bit source and symbol decoding for the NICE2
// stream (bitreader.rs:78-100 + hfe.rs:173-222), plus the decoder grammar.
//
// The reference peeks max_aob bits MSB-first and looks the value up in a
// 2^max_aob table (hfe.rs:191-222).  For a valid (complete, Kraft = 1) canonical
// code that is equivalent to a 2-level lookup: a DEC_LUT_BITS-bit first level
// holding (symbol, length) for short codes, and a search over the canonical
// order for the rest.  Bytes past the end of the stream read as the last stream
// byte, which is what the reference's stale one-byte buffer produces
// (bitreader.rs:90-96).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nice_format.h"

namespace nice {

constexpr int DEC_LUT_MAX_BITS = 12;      // per stream first-level width cap
constexpr int DEC_LUT_BUDGET = 12288;     // entries over all 10 streams (24 KiB)

// Per-frame decode tables (global memory; copied to LDS by the kernels).
struct DecTables {
  // first level: (symbol << 5) | length, length == 0 => long code; stream s
  // occupies lut[lut_off[s] .. lut_off[s] + 2^lut_bits[s])
  uint16_t lut[DEC_LUT_BUDGET];
  uint16_t lut_off[N_STREAMS];
  // canonical order per stream: aligned lower bound (code << (max - len)),
  // symbol and length, in (len desc, symbol desc) order
  uint32_t lo[N_BINS];
  uint16_t sym[N_BINS];
  uint8_t len[N_BINS];
  uint8_t max_aob[N_STREAMS];
  uint8_t lut_bits[N_STREAMS];
  // 1: no long codes (every first-level entry is a code) and every pixel event
  // fits 64 bits -- dec_sync decodes an event from one 64-bit window
  uint8_t fast;
  uint8_t pad[17];
};
static_assert(sizeof(DecTables) % 16 == 0, "per-frame tables stay 16-byte aligned");

struct BitSrc {
  const uint8_t* p;
  uint64_t len;    // bytes
  __device__ __forceinline__ uint32_t byte_at(uint64_t i) const {
    if (i < len) return p[i];
    return len ? p[len - 1] : 0u;
  }
  // 32 bits starting at absolute bit position pos, MSB first.  p is 4-byte aligned.
  __device__ __forceinline__ uint32_t peek32(uint64_t pos) const {
    const uint64_t wi = pos >> 5;
    const uint32_t o = (uint32_t)(pos & 31);
    uint64_t x;
    if ((wi + 2) * 4 <= len) {
      const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
      x = ((uint64_t)__builtin_bswap32(w[wi]) << 32) | __builtin_bswap32(w[wi + 1]);
    } else {
      x = 0;
      for (int k = 0; k < 8; ++k) x = (x << 8) | byte_at(wi * 4 + k);
    }
    return (uint32_t)((x << o) >> 32);
  }
};

// Decode one symbol of stream s at *pos; returns the symbol, advances *pos.
template <class Tab>
__device__ __forceinline__ uint32_t dec_symbol(const BitSrc& src, const Tab& t, int s, uint64_t* pos) {
  const uint32_t v = src.peek32(*pos);
  const uint32_t lb = t.lut_bits[s];
  const uint32_t e = t.lut[t.lut_off[s] + (v >> (32 - lb))];
  if (e & 31u) {
    *pos += e & 31u;
    return e >> 5;
  }
  // long code: largest aligned lower bound <= peek (bounds decrease along the
  // canonical order, so find the first index whose bound is <= x)
  const uint32_t mx = t.max_aob[s];
  const uint32_t x = v >> (32 - mx);
  int lo = stream_base(s), hi = stream_base(s) + stream_size(s) - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (t.lo[mid] <= x) hi = mid;
    else lo = mid + 1;
  }
  *pos += t.len[lo];
  return t.sym[lo];
}

// Decoder grammar (code.rs:576-671): gstate 0 expects a prefix; the payload
// positions of each mode follow.
//   BR 1 | RGB 2,3,4 | LUMA 5,6,7,8 | SD 9 | LUMA2 10,11,12
__host__ __device__ constexpr int gs_stream(int g) {
  return g == 0 ? S_PREFIX : g == 1 ? S_BACK_REF : g <= 4 ? S_RGB : g == 5 ? S_LUMA_REF
       : g == 6 ? S_LUMA_BASE : g <= 8 ? S_LUMA_OTHER : g == 9 ? S_SMALL_DIFF
       : g == 10 ? S_LUMA2_BASE : g == 11 ? S_LUMA2_R : S_LUMA2_B;
}
__host__ __device__ constexpr int gs_first(int mode) {
  return mode == P_BACK_REF ? 1 : mode == P_RGB ? 2 : mode == P_LUMA ? 5 : mode == P_SMALL_DIFF ? 9 : 10;
}
__host__ __device__ constexpr bool gs_last(int g) { return g == 1 || g == 4 || g == 8 || g == 9 || g == 12; }

}  // namespace nice
