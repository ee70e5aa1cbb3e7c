// nice_encode.hip -- MI355X (gfx950) encoder for the NICE2 bitstream.
//
// Pipeline per batch of same-shape frames (all kernels take the whole batch):
//   enc_classify   tiles of TILE consecutive pixels (raster order) staged into
//                  LDS as 4 row windows (rows y, y-1, y-2, y-3, +-3 px halo);
//                  per-pixel mode decision (code.rs:159-369), per-frame symbol
//                  histogram (hfe.rs:29-45), per-tile first/last coded pixel.
//   enc_tailruns   one block per frame: the run of each tile's last coded pixel
//                  may cross tiles; resolve it with a suffix-min over tiles and
//                  add its base-8 digits (code.rs:371-407) to the histogram.
//   enc_tables     one wave per (frame, stream): code lengths by exact replay of
//                  std BinaryHeap (hfe.rs:58-87), canonical codes (hfe.rs:255-296).
//   enc_header     one block per frame: file header (code.rs:72-84) + table
//                  header (hfe.rs:97-103) bits, data start position.
//   enc_pack       tiles again: per-pixel bit lengths, block scan, decoupled
//                  look-back across tiles for the bit offset (carrying the last
//                  32 bits so every output word is written once, no zero-fill,
//                  no global atomics), MSB-first packing (bitwriter.rs:55-73) and
//                  the tail (hfe.rs:115, code.rs:421-422).
//   enc_pack_long  frames whose emitted codes exceed FAST_MAX_CODE_BITS: the
//                  same tile-parallel placement with full-length codes, then
//                  the writes that wrap the reference's u32 cache (pending +
//                  length > 32, bitwriter.rs:63-64) applied to their 32-bit
//                  windows in a second pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nice_classify.hpp"
#include "nice_format.h"
#include "nice_huffman.hpp"
#include "nice_kernels.h"
#include "nice_rec.hpp"

namespace nice {

constexpr int ENC_THREADS = 256;
constexpr int PX_PER_THREAD = ENC_TILE / ENC_THREADS;  // 4
constexpr int WIN = ENC_TILE + 6;
constexpr uint32_t NONE = 0xFFFFFFFFu;

// ---------------------------------------------------------------------------
// Tile staging: 4 windows, window k holds X' of pixels [start - kW - 3, start - kW - 3 + WIN).
// Out-of-frame positions hold 0 and are never used (classify<false> checks validity).
// ---------------------------------------------------------------------------
struct TileWin {
  uint32_t w[4][WIN];
};

__device__ __forceinline__ uint32_t load_spread(const uint8_t* __restrict__ frame, int64_t j, int C) {
  if (C == 4) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(frame + j * 4);
    return spread_rgba(v);
  }
  const uint8_t* p = frame + j * C;
  return spread_rgb(p[0], p[1], p[2]);
}

__device__ inline void stage_tile(TileWin& tw, const uint8_t* __restrict__ frame, int64_t start,
                                  int64_t lo, int64_t hi, uint32_t W, int C) {
  for (int k = 0; k < 4; ++k) {
    const int64_t base = start - (int64_t)k * W - 3;
    for (int j = threadIdx.x; j < WIN; j += ENC_THREADS) {
      const int64_t g = base + j;
      tw.w[k][j] = (g >= lo && g < hi) ? load_spread(frame, g, C) : 0u;
    }
  }
}

// Software-pipelined staging for 4-byte pixels: raw words of the next tile are
// loaded into registers while the current tile is classified, then spread
// into the LDS windows.
constexpr int STAGE_PER_THREAD = (WIN + ENC_THREADS - 1) / ENC_THREADS;   // 5
struct TilePrefetch {
  uint32_t v[4][STAGE_PER_THREAD];
};
__device__ __forceinline__ void prefetch_tile(TilePrefetch& pf, const uint8_t* __restrict__ frame,
                                              int64_t start, int64_t lo, int64_t hi, uint32_t W) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t base = start - (int64_t)k * W - 3;
#pragma unroll
    for (int i = 0; i < STAGE_PER_THREAD; ++i) {
      const int j = (int)threadIdx.x + i * ENC_THREADS;
      const int64_t g = base + j;
      pf.v[k][i] = (j < WIN && g >= lo && g < hi) ? reinterpret_cast<const uint32_t*>(frame)[g] : 0u;
    }
  }
}
__device__ __forceinline__ void commit_tile(TileWin& tw, const TilePrefetch& pf) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int i = 0; i < STAGE_PER_THREAD; ++i) {
      const int j = (int)threadIdx.x + i * ENC_THREADS;
      if (j < WIN) tw.w[k][j] = spread_rgba(pf.v[k][i]);
    }
  }
}

struct WinAcc {
  const TileWin* tw;
  int col;  // p + 3
  __device__ __forceinline__ uint32_t operator()(int rows, int px) const { return tw->w[rows][col - px]; }
};

// Next coded pixel strictly after local index p, using the tile's coded bitmask
// (ENC_TILE bits). Returns ENC_TILE if none inside the tile.
__device__ __forceinline__ int next_coded_local(const uint32_t* mask, int p) {
  int w = (p + 1) >> 5;
  const int b = (p + 1) & 31;
  if (p + 1 >= ENC_TILE) return ENC_TILE;
  uint32_t m = mask[w] & (b ? (0xFFFFFFFFu << b) : 0xFFFFFFFFu);
  while (true) {
    if (m) return (w << 5) + __builtin_ctz(m);
    ++w;
    if (w >= ENC_TILE / 32) return ENC_TILE;
    m = mask[w];
  }
}

// ---------------------------------------------------------------------------
// K1: classify + histogram + per-pixel symbol records.
//
// Record (one u32 per pixel, raster order): bits 0..2 the mode prefix
// (P_BACK_REF .. P_LUMA2) or REC_UNCODED for a run member; bits 3.. the payload,
// laid out as the classify arithmetic produces it (the spread/luma-space
// fields at 10-bit spacing, masked and shifted once):
//   BACK_REF  k (3) at 3            SMALL_DIFF  index 0..342 (9) at 3
//   LUMA2     r+16 (5) at 3, g+32 (6) at 13, b+16 (5) at 23
//   LUMA      k (4) at 3, r+16 (5) at 7, g+32 (6) at 17, b+16 (5) at 27
//   RGB       r, g, b residuals (8 each) at 3, 13, 23
// ---------------------------------------------------------------------------
constexpr uint32_t REC_UNCODED = 7u;
// the luma payload fields of Y(X) - Y(ref) (r: bits 0-4, g: 10-15, b: 20-24)
constexpr uint32_t LUMA_FIELDS = 0x1Fu | (0x3Fu << 10) | (0x1Fu << 20);

__device__ __forceinline__ uint32_t rec_from_syms(const PixSyms& s) {
  switch (s.mode) {
    case P_BACK_REF: return P_BACK_REF | ((s.b[0] - BIN_BACK_REF) << 3);
    case P_SMALL_DIFF: return P_SMALL_DIFF | ((s.b[0] - BIN_SMALL_DIFF) << 3);
    case P_LUMA2:
      return P_LUMA2 | ((s.b[0] - BIN_LUMA2_BASE) << 13) | ((s.b[1] - BIN_LUMA2_R) << 3) |
             ((s.b[2] - BIN_LUMA2_B) << 23);
    case P_LUMA:
      return P_LUMA | ((s.b[0] - BIN_LUMA_REF) << 3) | ((s.b[1] - BIN_LUMA_BASE) << 17) |
             ((s.b[2] - BIN_LUMA_OTHER) << 7) | ((s.b[3] - BIN_LUMA_OTHER) << 27);
    default: return P_RGB | (s.b[0] << 3) | (s.b[1] << 13) | (s.b[2] << 23);
  }
}

// Payload bins of a coded record (n = 1, 3 or 4), branch-free: per mode m
// (record bits 0..2), payload k is bits [shift, shift+width) of the record plus
// a histogram base, all looked up in packed constants (no per-mode control flow).
//   m:        0 BACK_REF   1 RGB        2 LUMA        3 SMALL_DIFF  4 LUMA2
//   k = 0     847+[3,3)    0+[3,8)      365+[3,4)     376+[3,9)     719+[13,6)
//   k = 1     -            0+[13,8)     269+[17,6)    -             783+[3,5)
//   k = 2     -            0+[23,8)     333+[7,5)     -             815+[23,5)
//   k = 3     -            -            333+[27,5)    -             -
constexpr unsigned long long rb_pack(int a0, int a1, int a2, int a3, int a4, int bits) {
  return (unsigned long long)a0 | ((unsigned long long)a1 << bits) | ((unsigned long long)a2 << (2 * bits)) |
         ((unsigned long long)a3 << (3 * bits)) | ((unsigned long long)a4 << (4 * bits));
}
// base (10 bits per mode), shift (5) | width << 5 (10 bits per mode)
constexpr unsigned long long RB_BASE[4] = {
    rb_pack(BIN_BACK_REF, 0, BIN_LUMA_REF, BIN_SMALL_DIFF, BIN_LUMA2_BASE, 10),
    rb_pack(0, 0, BIN_LUMA_BASE, 0, BIN_LUMA2_R, 10),
    rb_pack(0, 0, BIN_LUMA_OTHER, 0, BIN_LUMA2_B, 10),
    rb_pack(0, 0, BIN_LUMA_OTHER, 0, 0, 10)};
constexpr unsigned long long RB_FIELD[4] = {
    rb_pack(3 | 3 << 5, 3 | 8 << 5, 3 | 4 << 5, 3 | 9 << 5, 13 | 6 << 5, 10),
    rb_pack(0, 13 | 8 << 5, 17 | 6 << 5, 0, 3 | 5 << 5, 10),
    rb_pack(0, 23 | 8 << 5, 7 | 5 << 5, 0, 23 | 5 << 5, 10),
    rb_pack(0, 0, 27 | 5 << 5, 0, 0, 10)};
constexpr uint32_t RB_N = 1u | 3u << 3 | 4u << 6 | 1u << 9 | 3u << 12;   // payload count, 3 bits per mode
__device__ __forceinline__ uint32_t rb_bin(uint32_t rec, uint32_t m, int k) {
  const uint32_t base = (uint32_t)(RB_BASE[k] >> (10u * m)) & 0x3FFu;
  const uint32_t fw = (uint32_t)(RB_FIELD[k] >> (10u * m)) & 0x3FFu;
  return base + __builtin_amdgcn_ubfe(rec, fw & 31u, fw >> 5);
}
__device__ __forceinline__ uint32_t rec_bins(uint32_t rec, uint32_t& b0, uint32_t& b1, uint32_t& b2,
                                             uint32_t& b3) {
  const uint32_t m = min(rec & 7u, 4u);
  b0 = rb_bin(rec, m, 0);
  b1 = rb_bin(rec, m, 1);
  b2 = rb_bin(rec, m, 2);
  b3 = rb_bin(rec, m, 3);
  return (RB_N >> (3u * m)) & 7u;
}
// The same from an LDS table (two 16-byte reads per record, row m = record
// bits 0..2; rows 5..7 empty).  v_bfe_u32 reads only the low 5 bits of its
// offset and width operands, so word a[m].k = shift | base << 16 and word
// b[m].k = width (the payload count in bits 8..10 of b[m].x): a bin is one
// shift, one field extract and one add (packing shift and width in one word
// took two more shifts and a mask per bin).
struct RecBinTable { uint4 a[8], b[8]; };
__device__ __forceinline__ void rbt_init(RecBinTable& t, int tid) {
  if (tid < 8) {
    uint32_t wa[4], wb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t m = (uint32_t)tid;
      const uint32_t base = m < 5 ? (uint32_t)(RB_BASE[k] >> (10u * m)) & 0x3FFu : 0u;
      const uint32_t fw = m < 5 ? (uint32_t)(RB_FIELD[k] >> (10u * m)) & 0x3FFu : 0u;
      wa[k] = (fw & 31u) | base << 16;
      wb[k] = fw >> 5;
    }
    wb[0] |= (tid < 5 ? (RB_N >> (3u * tid)) & 7u : 0u) << 8;
    t.a[tid] = make_uint4(wa[0], wa[1], wa[2], wa[3]);
    t.b[tid] = make_uint4(wb[0], wb[1], wb[2], wb[3]);
  }
}
__device__ __forceinline__ uint32_t rec_bins(const RecBinTable& t, uint32_t rec, uint32_t& b0, uint32_t& b1,
                                             uint32_t& b2, uint32_t& b3) {
  const uint4 ra = t.a[rec & 7u], rb = t.b[rec & 7u];
  b0 = (ra.x >> 16) + __builtin_amdgcn_ubfe(rec, ra.x, rb.x);
  b1 = (ra.y >> 16) + __builtin_amdgcn_ubfe(rec, ra.y, rb.y);
  b2 = (ra.z >> 16) + __builtin_amdgcn_ubfe(rec, ra.z, rb.z);
  b3 = (ra.w >> 16) + __builtin_amdgcn_ubfe(rec, ra.w, rb.w);
  return rb.x >> 8;
}

// Window-classify record (layout above) -> the packer's record (nice_rec.hpp).
__device__ __forceinline__ uint32_t rec2_from_old(uint32_t rec, uint32_t lane) {
  const uint32_t m = rec & 7u;
  if (m == REC_UNCODED) return rec2_unc(lane);
  if (m == P_BACK_REF) return ((C0_BR + ((rec >> 3) & 7u)) << 3) | rec2_abs(lane);
  if (m == P_SMALL_DIFF) return ((C0_SD + ((rec >> 3) & 0x1FFu)) << 3) | rec2_abs(lane);
  if (m == P_LUMA2)
    return ((C0_L2 + ((rec >> 13) & 0x3Fu)) << 3) | ((SX_L2 + ((rec >> 3) & 0x1Fu)) << 14) |
           ((SX_L2 + ((rec >> 23) & 0x1Fu)) << 23);
  if (m == P_LUMA)
    return ((C0_LUMA + 64u * ((rec >> 3) & 15u) + ((rec >> 17) & 0x3Fu)) << 3) |
           ((SX_LUMA + ((rec >> 7) & 0x1Fu)) << 14) | ((SX_LUMA + ((rec >> 27) & 0x1Fu)) << 23);
  return (((rec >> 3) & 0xFFu) << 3) | (((rec >> 13) & 0xFFu) << 14) | (((rec >> 23) & 0xFFu) << 23);
}

// Each mode's identifying stream and symbols per pixel (code.rs:191-366):
// BACK_REF one SC_BACK_REF symbol, RGB three SC_RGB, LUMA one
// SC_LUMA_BACK_REF, SMALL_DIFF one SC_SMALL_DIFF1, LUMA2 one
// SC_LUMA_BASE_DIFF2 -- so a mode's prefix count is its stream's total
// divided by that number, and the classify pass does not count prefixes.
__device__ __forceinline__ bool mode_id_bin(int k, int b) {
  const int lo = k == P_BACK_REF ? BIN_BACK_REF : k == P_RGB ? 0 : k == P_LUMA ? BIN_LUMA_REF
               : k == P_SMALL_DIFF ? BIN_SMALL_DIFF : BIN_LUMA2_BASE;
  const int n = k == P_BACK_REF ? N_BINS - BIN_BACK_REF : k == P_RGB ? 256 : k == P_LUMA ? 11
              : k == P_SMALL_DIFF ? 343 : 64;
  return b >= lo && b < lo + n;
}
__device__ __forceinline__ uint32_t mode_id_syms(int k) { return k == P_RGB ? 3u : 1u; }

// Work item -> (frame, tile) without a 64-bit division per tile (one at the
// start; the scalar division sequence is ~100 instructions).
struct TileIter {
  uint32_t f, k, nt, lo, T;
  __device__ __forceinline__ TileIter(const EncArgs& a, uint64_t w)
      : f((uint32_t)(w / (a.tile_hi - a.tile_lo))), k((uint32_t)(w % (a.tile_hi - a.tile_lo))),
        nt(a.tile_hi - a.tile_lo), lo(a.tile_lo), T(a.tiles_per_frame) {}
  __device__ __forceinline__ void step(uint32_t n) {
    k += n;
    while (k >= nt) { k -= nt; ++f; }
  }
  __device__ __forceinline__ uint32_t tt() const { return lo + k; }
  __device__ __forceinline__ uint64_t tile() const { return (uint64_t)f * T + lo + k; }
};

// Branch-free mode decision from the LDS windows (column col = p + 3 of window
// `rows`, pixel i - (rows*W + px) at col - px): all tests are evaluated and the
// first hit in the reference order wins (code.rs:191-366).  HEAD = false: every
// reference exists (i >= 3W+3, W >= 3).  HEAD = true (W >= 3): the reference's
// validity rules as masks, as in classify_ring<true>.
template <bool HEAD>
__device__ __forceinline__ uint32_t classify_fast(const TileWin& tw, int col, uint32_t i, uint32_t W) {
  const uint32_t X = tw.w[0][col], L2 = tw.w[0][col - 2], L3 = tw.w[0][col - 3];
  uint32_t L = tw.w[0][col - 1];
  const uint32_t U = tw.w[1][col], UR1 = tw.w[1][col + 1], UR3 = tw.w[1][col + 3], UL3 = tw.w[1][col - 3];
  const uint32_t U2 = tw.w[2][col];
  const uint32_t V = tw.w[3][col], VR1 = tw.w[3][col + 1], VL1 = tw.w[3][col - 1];
  const uint32_t VL3 = tw.w[3][col - 3], VR3 = tw.w[3][col + 3];
  // back references k = 1..4 (k = 0, the pixel before, never equals a coded pixel)
  bool e1 = U == X, e2 = UR1 == X, e3 = L2 == X, e4 = U2 == X;
  const bool has_up = !HEAD || i >= W, has_left = !HEAD || i > 0;
  if constexpr (HEAD) {
    e1 = e1 && i >= W;
    e2 = e2 && i >= W - 1u;
    e3 = e3 && i >= 2u;
    e4 = e4 && i >= 2u * W;
    L = i > 0 ? L : X;
  }
  const bool br = e1 | e2 | e3 | e4;
  const uint32_t bk = e1 ? 1u : e2 ? 2u : e3 ? 3u : 4u;
  const uint32_t pred = has_up ? avg3(U, L) : L;
  // small diff
  const uint32_t d = X + K3(259u) - pred;
  const bool sd = has_left && ((d & K3(0x3F8u)) == K3(0x100u)) && ((((d & K3(7u)) + K3(1u)) & K3(8u)) == 0);
  const uint32_t sdi = (d & 7u) + 7u * ((d >> 10) & 7u) + 49u * ((d >> 20) & 7u);
  // luma2 against the average
  const uint32_t xk = X + LUMA_K;
  const uint32_t t2 = luma_t(xk, pred);
  const bool l2 = has_up && (t2 & LUMA_MASK) == 0;
  // luma against 11 references, first hit wins; skipped when no lane needs it
  uint32_t lk = 11u, lt = 0u;
  const bool need_luma = __builtin_amdgcn_ballot_w64(!br && !sd && !l2) != 0ull;
  if (need_luma) {
    const uint32_t refs[11] = {L, U, UR1, UR3, L3, VR1, V, VL1, UL3, VL3, VR3};
#pragma unroll
    for (int k = 10; k >= 0; --k) {
      const uint32_t t = luma_t(xk, refs[k]);
      bool ok = (t & LUMA_MASK) == 0;
      if constexpr (HEAD) ok = ok && i > 0 && i >= (uint32_t)lr_rows(k) * W + (uint32_t)lr_px(k);
      lk = ok ? (uint32_t)k : lk;
      lt = ok ? t : lt;
    }
  }
  const uint32_t r = X + K3(256u) - (has_left ? pred : 0u);
  const uint32_t rec_br = P_BACK_REF | (bk << 3);
  const uint32_t rec_sd = P_SMALL_DIFF | (sdi << 3);
  const uint32_t rec_l2 = P_LUMA2 | ((t2 & LUMA_FIELDS) << 3);
  const uint32_t rec_lu = P_LUMA | (lk << 3) | ((lt & LUMA_FIELDS) << 7);
  const uint32_t rec_rgb = P_RGB | ((r & K3(0xFFu)) << 3);
  return br ? rec_br : sd ? rec_sd : l2 ? rec_l2 : lk < 11u ? rec_lu : rec_rgb;
}

// TINY (W < 3): references wrap inside the window rows; the general
// classify<false> decides the first 3W+3 pixels (all of a tiny frame).
template <bool TINY>
__device__ __forceinline__ void enc_classify_body(const EncArgs& a) {
  __shared__ TileWin tw;
  __shared__ uint32_t hist[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];

  // work items: frame f, band tile tt in [tile_lo, tile_hi); t = f*T + tt
  const uint32_t nt = a.tile_hi - a.tile_lo;
  const uint64_t total_work = (uint64_t)a.n_frames * nt;
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  uint64_t w_end = w_begin + a.tiles_per_block;
  if (w_end > total_work) w_end = total_work;
  if (w_begin >= w_end) return;

  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) hist[b] = 0;
  uint32_t cur_frame = (uint32_t)(w_begin / nt);
  const int lane = threadIdx.x & 63;
  const int64_t N = (int64_t)a.W * a.H;
  const bool rgba = a.C == 4;
  TilePrefetch pf;
  if (rgba) {
    const uint32_t f0 = (uint32_t)(w_begin / nt);
    prefetch_tile(pf, a.px + (uint64_t)f0 * a.frame_stride,
                  (int64_t)(a.tile_lo + w_begin % nt) * ENC_TILE, a.px_lo, a.px_hi, a.W);
  }

  for (uint64_t w = w_begin; w < w_end; ++w) {
    const uint32_t f = (uint32_t)(w / nt);
    const uint32_t tt = a.tile_lo + (uint32_t)(w % nt);
    const uint64_t t = (uint64_t)f * a.tiles_per_frame + tt;
    if (f != cur_frame) {
      __syncthreads();
      for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) {
        if (hist[b]) atomicAdd(&a.hist[(uint64_t)cur_frame * N_BINS + b], hist[b]);
        hist[b] = 0;
      }
      cur_frame = f;
    }
    const uint8_t* frame = a.px + (uint64_t)f * a.frame_stride;
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    __syncthreads();
    if (rgba) {
      commit_tile(tw, pf);
      if (w + 1 < w_end) {   // next tile's pixels are in flight while this one is classified
        const uint32_t f1 = (uint32_t)((w + 1) / nt);
        prefetch_tile(pf, a.px + (uint64_t)f1 * a.frame_stride,
                      (int64_t)(a.tile_lo + (w + 1) % nt) * ENC_TILE, a.px_lo, a.px_hi, a.W);
      }
    } else {
      stage_tile(tw, frame, start, a.px_lo, a.px_hi, a.W, a.C);
    }
    __syncthreads();

    // coded flags -> bitmask
    uint32_t coded_bits = 0;
#pragma unroll
    for (int r = 0; r < PX_PER_THREAD; ++r) {
      const int p = r * ENC_THREADS + threadIdx.x;
      const int64_t i = start + p;
      bool coded = false;
      if (p < count) coded = (i == 0) || (tw.w[0][p + 3] != tw.w[0][p + 2]);
      const unsigned long long bal = __ballot(coded);
      if (lane == 0) {
        const int wbase = (r * ENC_THREADS + (threadIdx.x & ~63)) >> 5;
        mask[wbase] = (uint32_t)bal;
        mask[wbase + 1] = (uint32_t)(bal >> 32);
      }
      coded_bits |= (coded ? 1u : 0u) << r;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int first = -1, last = -1;
      for (int w = 0; w < ENC_TILE / 32; ++w)
        if (mask[w]) { first = w * 32 + __builtin_ctz(mask[w]); break; }
      for (int w = ENC_TILE / 32 - 1; w >= 0; --w)
        if (mask[w]) { last = w * 32 + 31 - __builtin_clz(mask[w]); break; }
      a.tile_first[t] = first < 0 ? NONE : (uint32_t)(start + first);
      a.tile_last[t] = last < 0 ? NONE : (uint32_t)(start + last);
    }
    const bool fast = (a.W >= 3) && (start >= 3 * (int64_t)a.W + 3);
    uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + start;
#pragma unroll
    for (int r = 0; r < PX_PER_THREAD; ++r) {
      const int p = r * ENC_THREADS + threadIdx.x;
      const bool coded = (coded_bits >> r) & 1u;
      uint32_t rec = REC_UNCODED;
      if (fast) {
        const uint32_t rf = classify_fast<false>(tw, p + 3, 0u, a.W);
        rec = coded ? rf : REC_UNCODED;
      } else if constexpr (TINY) {
        if (coded) {
          PixSyms s;
          WinAcc acc{&tw, p + 3};
          classify<false>((uint32_t)(start + p), a.W, acc, s);
          rec = rec_from_syms(s);
        }
      } else {   // block-uniform branch: both variants are straight-line code
        const uint32_t rf = classify_fast<true>(tw, p + 3, (uint32_t)(start + p), a.W);
        rec = coded ? rf : REC_UNCODED;
      }
      if (p < count) recs[p] = rec2_from_old(rec, (uint32_t)lane);
      if (coded) {
        uint32_t b0, b1, b2, b3;
        const uint32_t n = rec_bins(rec, b0, b1, b2, b3);
        atomicAdd(&hist[b0], 1u);
        if (n > 1) { atomicAdd(&hist[b1], 1u); atomicAdd(&hist[b2], 1u); }
        if (n > 3) atomicAdd(&hist[b3], 1u);
        const int nx = next_coded_local(mask, p);
        if (nx < count) {
          const uint64_t run = (uint64_t)(nx - p - 1);
          if (run > 0) {
            uint64_t m = run - 1;
            while (true) {
              atomicAdd(&hist[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)], 1u);
              if (m < 8) break;
              m >>= 3;
            }
          }
        }
      }
      // mode prefixes: derived by enc_tables from the payload streams (mode_id_bin)
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS)
    if (hist[b]) atomicAdd(&a.hist[(uint64_t)cur_frame * N_BINS + b], hist[b]);
}
__global__ __launch_bounds__(ENC_THREADS) void enc_classify(EncArgs a) { enc_classify_body<false>(a); }
__global__ __launch_bounds__(ENC_THREADS) void enc_classify_tiny(EncArgs a) { enc_classify_body<true>(a); }

// ---------------------------------------------------------------------------
// K1r: classify, ring-staged (RGBA frames, 3 <= W <= CLS_RING_MAX_W).
//
// Same outputs as enc_classify (records, histogram, tile first/last coded
// pixel), restructured for the instruction budget:
//  * every pixel is loaded from HBM and converted once: a block walks its tile
//    range in raster order and keeps the last CLS_RING pixels (>= 3 rows + 3 px
//    + one tile) in an LDS ring indexed by pixel & (CLS_RING - 1); the next
//    tile is loaded into registers while the current one is classified;
//  * pixels are held in "luma space", Y = (R-G) | G << 10 | (B-G) << 20 (each
//    field mod 256).  The transform is a bijection, so the equality tests of
//    back references and runs hold unchanged, and the luma test of code.rs:
//    296-336 against reference pixel R -- g = XG-RG in [-32,32), XR-RR-g and
//    XB-RB-g in [-16,16) -- becomes a range test on the field-wise difference
//    Y(X) - Y(R): one subtract, one AND, one compare per reference;
//  * the five mode-prefix counts are accumulated per thread in packed
//    registers and added to the histogram once per frame.
// ---------------------------------------------------------------------------
constexpr int CLS_THREADS = 512;
constexpr int CLS_PPT = ENC_TILE / CLS_THREADS;   // 2 pixels per thread
constexpr int CLS_RING = 16384;                   // ring words (64 KB)
// words 0..CLS_GUARD-1 of the ring mirrored past its end: a neighbour group
// (pixels b .. b+6 for b = ((s - rows*W - 3) mod CLS_RING) + tid, s the
// wave-uniform part of the pixel index) is one base address plus immediate
// offsets, never wrapping
constexpr int CLS_GUARD = CLS_THREADS + 8;
// luma test offsets in Y space: R,B fields +16, G field +32, plus 256 per field
constexpr uint32_t LUMA_KY = (256u + 16u) | ((256u + 32u) << 10) | ((256u + 16u) << 20);

// (R-G, B-G) by one packed 16-bit subtract of G from the halves G<<8|R and
// A<<8|B (borrows land in the G and A bytes, masked off), then B-G moved up by
// one 24-bit multiply-add: 7 VALU instead of 11 for the spread-and-subtract
// form (both checked equal over every RGB value on the host)
typedef unsigned short nice_u16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int nice_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t y_from_rgba(uint32_t v) {
  const uint32_t g = __builtin_amdgcn_ubfe(v, 8, 8);
  const nice_u16x2 d = __builtin_bit_cast(nice_u16x2, v) - __builtin_bit_cast(nice_u16x2, g | (g << 16));
  const uint32_t t = __builtin_bit_cast(uint32_t, d);
  return (__umul24(t & 0xFF0000u, 16u) + (t & 0xFFu)) | (g << 10);
}
__device__ __forceinline__ uint32_t rgb_from_y(uint32_t y) {
  // g | g << 20 as one 24-bit multiply-add (v_bfe + v_mad_u32_u24 + v_and)
  const uint32_t g = (y >> 10) & 0xFFu;
  return (y + __umul24(g, 0x100001u)) & K3(0xFFu);
}

struct RingAcc {   // classify<false> accessor: RGB spread of pixel i - (rows*W + px)
  const uint32_t* ring;
  uint32_t W;
  int64_t i;
  __device__ __forceinline__ uint32_t operator()(int rows, int px) const {
    const int64_t j = i - ((int64_t)rows * W + px);
    return rgb_from_y(ring[j & (CLS_RING - 1)]);
  }
};

// Branch-free mode decision from the Y ring; returns the record (same layout
// as classify_fast).  Four base addresses (rows 0..3 back, 3 pixels left), the
// rest immediate offsets: for pixel i = s + tid (s wave-uniform) base k is
// ring + ((s - c_k) mod RING) + tid, a scalar plus the thread index (the
// mirrored guard covers the overrun past the ring's end).
// HEAD = false: every reference valid (i >= 3W+3, W >= 3).  HEAD = true: the
// first tiles of a frame, with the reference's validity rules as masks instead
// of classify<false>'s early exits (code.rs:191-366; W >= 3): a reference
// counts only if i >= its offset, L is X itself at i = 0, without a row above
// the prediction is L and LUMA2 is skipped, SMALL_DIFF and LUMA need i > 0, and
// the raw residual is taken against 0 at i = 0.  (The back reference to pixel
// i-1 can never hit a coded pixel, so it is not tested.)
// The four neighbour groups of the lane's pixel: b0 = pixels i-3 .. i (row y),
// b1 = row y-1 from 3 left, b2 = pixel i-2W, b3 = row y-3 from 3 left; the
// hit's difference is read again at rbase[ltab[k] + tid].
// X: the lane's own pixel (Y space), from the caller's registers where it
// staged it (saves one ring read per pixel).
template <bool HEAD>
__device__ __forceinline__ uint32_t classify_y(const uint32_t* b0, const uint32_t* b1, const uint32_t* b2,
                                               const uint32_t* b3, const uint32_t* rbase, uint32_t tid, uint32_t W,
                                               uint32_t i, const uint32_t* ltab, uint32_t cbr, uint32_t csd,
                                               uint32_t X);
template <bool HEAD, int RING = CLS_RING>
__device__ __forceinline__ uint32_t classify_ring(const uint32_t* ring, uint32_t s, uint32_t tid, uint32_t W,
                                                  uint32_t i, const uint32_t* ltab, uint32_t cbr, uint32_t csd,
                                                  uint32_t X) {
  return classify_y<HEAD>(ring + ((s - 3u) & (RING - 1)) + tid, ring + ((s - W - 3u) & (RING - 1)) + tid,
                          ring + ((s - 2u * W) & (RING - 1)) + tid,
                          ring + ((s - 3u * W - 3u) & (RING - 1)) + tid, ring, tid, W, i, ltab, cbr, csd, X);
}
template <bool HEAD>
__device__ __forceinline__ uint32_t classify_y(const uint32_t* b0, const uint32_t* b1, const uint32_t* b2,
                                               const uint32_t* b3, const uint32_t* rbase, uint32_t tid, uint32_t W,
                                               uint32_t i, const uint32_t* ltab, uint32_t cbr, uint32_t csd,
                                               uint32_t X) {
  const uint32_t L2 = b0[1], L3 = b0[0];
  uint32_t L = b0[2];
  const uint32_t U = b1[3], UR1 = b1[4], UR3 = b1[6], UL3 = b1[0];
  const uint32_t U2 = b2[0];
  const uint32_t V = b3[3], VR1 = b3[4], VL1 = b3[2];
  const uint32_t VL3 = b3[0], VR3 = b3[6];
  // back references k = 1..4 (code.rs:191-206; Y equality == RGB equality)
  bool e1 = U == X, e2 = UR1 == X, e3 = L2 == X, e4 = U2 == X;
  const bool has_up = !HEAD || i >= W, has_left = !HEAD || i > 0;
  if constexpr (HEAD) {
    e1 = e1 && i >= W;
    e2 = e2 && i >= W - 1u;
    e3 = e3 && i >= 2u;
    e4 = e4 && i >= 2u * W;
    L = i > 0 ? L : X;
  }
  const bool br = e1 | e2 | e3 | e4;
  const uint32_t bk = e1 ? 1u : e2 ? 2u : e3 ? 3u : 4u;
  // prediction floor((U+L)/2) in RGB (L alone without a row above)
  const uint32_t xr = rgb_from_y(X);
  const uint32_t lrgb = rgb_from_y(L);
  const uint32_t pred = has_up ? avg3(rgb_from_y(U), lrgb) : lrgb;
  // small diff (code.rs:208-247)
  const uint32_t d = xr + K3(259u) - pred;
  // every field in [256, 262]: bits 3-9 0b0100000 (field in [256, 263]) and
  // bit 3 of field + 1 clear (field != 263), OR-ed so one compare covers all
  // three fields (an OR only adds bit 3, which 0x100 lacks; no carry: fields
  // <= 515)
  const bool sd = has_left && ((d & K3(0x3F8u)) | ((d + K3(1u)) & K3(8u))) == K3(0x100u);
  // the index f0 + 7 f1 + 49 f2 of the three 3-bit fields f (code.rs:243-245)
  // by one 24-bit multiply: the product's bits 20..29 hold it, the partial
  // products below stay under 2^20 (f <= 6) and the ones above start at bit 30
  const uint32_t sdi = (__umul24(d & K3(7u), 49u | (7u << 10) | (1u << 20)) >> 20) & 0x3FFu;
  // luma2 against the prediction (code.rs:252-292): t2 = Y(X) - Y(pred) with
  // the test offsets, Y(pred) = pred - pg in fields 0 and 2, written as
  // X + LUMA_KY - pred + pg (fields 17..782: no borrow or carry across fields,
  // and only each field's value mod 256 is used below)
  const uint32_t pg = (pred >> 10) & 0xFFu;
  const uint32_t xk = X + LUMA_KY;
  const uint32_t t2 = (xk - pred) + (pg | (pg << 20));
  const bool l2 = has_up && (t2 & LUMA_MASK) == 0;
  // luma against 11 references, first hit wins (code.rs:293-339)
  uint32_t lk = 11u, lt = 0u;
  // (A/B: the search made unconditional on the fast path -- more VALU per
  // pixel -- was 6 % slower at 512 frames: whole waves often skip it)
  const bool need_luma = __builtin_amdgcn_ballot_w64(!br && !sd && !l2) != 0ull;
  if (need_luma) {
    // the wave issues first until its block's next tile barrier (as in the
    // slide kernel's classify_win: the block waits on its slowest wave)
    if constexpr (!HEAD) __builtin_amdgcn_s_setprio(1);
    const uint32_t refs[11] = {L, U, UR1, UR3, L3, VR1, V, VL1, UL3, VL3, VR3};
    if constexpr (HEAD) {
#pragma unroll
      for (int k = 10; k >= 0; --k) {
        const uint32_t t = xk - refs[k];
        const bool ok = (t & LUMA_MASK) == 0 && i > 0 && i >= (uint32_t)lr_rows(k) * W + (uint32_t)lr_px(k);
        lk = ok ? (uint32_t)k : lk;
        lt = ok ? t : lt;
      }
    } else {
      // first hit = min over k of ((t_k & LUMA_MASK) | k): the mask's lowest
      // bit is 32 > 10, so a miss keys >= 32 and a hit keys k (one v_and_or
      // per reference, v_min3 trees, no compare/select chains); the hit's
      // difference is taken again from the ring through the tile's address
      // table (ltab[k] = ring index of reference k for thread 0)
      uint32_t key[11];
#pragma unroll
      for (int k = 0; k < 11; ++k) key[k] = ((xk - refs[k]) & LUMA_MASK) | (uint32_t)k;
      const uint32_t m = min(min(min(min(key[0], key[1]), key[2]), min(min(key[3], key[4]), key[5])),
                             min(min(min(key[6], key[7]), key[8]), min(key[9], key[10])));
      lk = min(m, 11u);
      lt = xk - rbase[ltab[m & 15u] + tid];
    }
  }
  const uint32_t r = has_left ? d - K3(3u) : xr + K3(256u);   // = xr + 256 - pred per field
  // the record (nice_rec.hpp): BACK_REF and SMALL_DIFF onto the lane's
  // constant (mode range + absent slots); RGB's r, g, b fields (spread, 10-bit
  // spacing) to c0, s1, s2 by doubling g (one bit further up); LUMA2 / LUMA: g
  // (luma-space field 1) to c0 with the mode range (LUMA: + 64 k), r and b to
  // s1 and s2
  const uint32_t rec_br = (bk << 3) + cbr;
  const uint32_t rec_sd = (sdi << 3) + csd;
  const uint32_t rs = r & K3(0xFFu);
  const uint32_t rec_rgb = (rs + (rs & (0xFFu << 10))) << 3;
  const uint32_t lf = l2 ? t2 : lt;
  const uint32_t lbase = l2 ? ((C0_L2 << 3) | (SX_L2 << 14) | (SX_L2 << 23))
                            : ((C0_LUMA << 3) | (SX_LUMA << 14) | (SX_LUMA << 23)) + (lk << 9);
  const uint32_t rec_lu = lbase + (__builtin_amdgcn_ubfe(lf, 10, 6) << 3) + ((lf & 0x1Fu) << 14) +
                          ((lf & (0x1Fu << 20)) << 3);
  return br ? rec_br : sd ? rec_sd : (l2 || lk < 11u) ? rec_lu : rec_rgb;
}

// slot histogram (nice_rec.hpp) add of one record: three unconditional LDS
// adds (run members and absent slots land on the lane's own zero slots)
__device__ __forceinline__ void slot_hist_add(uint32_t* hs, uint32_t rec) {
  char* hb = reinterpret_cast<char*>(hs);
  atomicAdd(reinterpret_cast<uint32_t*>(hb + ((rec >> 1) & 0x1FFCu)), 1u);
  atomicAdd(reinterpret_cast<uint32_t*>(hb + C0_N * 4 + ((rec >> 12) & 0x7FCu)), 1u);
  atomicAdd(reinterpret_cast<uint32_t*>(hb + (C0_N + SX_N) * 4 + ((rec >> 21) & 0x7FCu)), 1u);
}

// RGB frames (C = 3, 4-byte aligned frames): a tile's 3072 bytes arrive as 768
// dwords (one or two per thread), are staged in LDS and each pixel's 3 bytes
// are taken with one funnel shift of two dwords.
constexpr int RGB_TILE_DW = ENC_TILE * 3 / 4;   // 768
__device__ __forceinline__ uint32_t rgb_dword(const uint8_t* fr, uint64_t nbytes, uint64_t j) {
  if (4 * j + 4 <= nbytes) return reinterpret_cast<const uint32_t*>(fr)[j];
  uint32_t v = 0;
  for (int k = 0; k < 4; ++k)
    if (4 * j + k < nbytes) v |= (uint32_t)fr[4 * j + k] << (8 * k);
  return v;
}
// pixel j of a frame as R | G << 8 | B << 16 (what y_from_rgba reads)
template <int C>
__device__ __forceinline__ uint32_t px_word(const uint8_t* fr, int64_t j) {
  if (C == 4) return reinterpret_cast<const uint32_t*>(fr)[j];
  const uint8_t* p = fr + 3 * j;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}

// MASK_OUT: as enc_classify_pair_body's (frames: coded flags out, run digits by
// enc_rundigits).
template <int C, int RING, bool MASK_OUT = false>
__device__ __forceinline__ void enc_classify_ring_body(const EncArgs& a) {
  __shared__ uint32_t ring[RING + CLS_GUARD];
  __shared__ uint32_t stage[C == 3 ? RGB_TILE_DW + 4 : 1];
  __shared__ uint32_t hs[C0_N + 2 * SX_N];     // slot histogram (nice_rec.hpp)
  __shared__ uint32_t run_hist[8];             // run digits (prefixes 5..12)
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t ltab[2][CLS_PPT][16];   // [tile parity][q][luma reference]: ring index for thread 0
  // work items: frame f, tile tt in [tile_lo, tile_hi) (frames: all tiles; bands: the band's)
  const uint64_t total_work = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  const uint64_t w_end = min(w_begin + a.tiles_per_block, total_work);
  if (w_begin >= w_end) return;
  const int tid = threadIdx.x, lane = tid & 63;
  // the lane's record constants: BACK_REF / SMALL_DIFF ranges with absent
  // slots, and the run-member record
  const uint32_t cbr = (C0_BR << 3) | rec2_abs((uint32_t)lane), csd = (C0_SD << 3) | rec2_abs((uint32_t)lane);
  const uint32_t cunc = rec2_unc((uint32_t)lane);
  // back distance of luma reference k (code.rs:293-339), for the tile tables
  const uint32_t lback = tid < 16 * CLS_PPT && (tid & 15) < 11
                             ? (uint32_t)lr_rows(tid & 15) * a.W + (uint32_t)lr_px(tid & 15) : 0u;
  const uint32_t W = a.W;
  const int64_t N = (int64_t)W * a.H;
  for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
  if (tid < 8) run_hist[tid] = 0;
  // the frame's symbol counts into the 858 bins (hfe.rs:29-45), once per
  // block and frame
  auto flush = [&](uint32_t frame) {
    __syncthreads();
    for (int b = tid; b < N_BINS; b += CLS_THREADS) {
      uint32_t v = slot_hist_bin(hs, b);
      if (b >= BIN_PREFIX + P_RUN1 && b < BIN_PREFIX + P_RUN1 + 8) v += run_hist[b - BIN_PREFIX - P_RUN1];
      if (v) atomicAdd(&a.hist[(uint64_t)frame * N_BINS + b], v);
    }
    __syncthreads();
    for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
    if (tid < 8) run_hist[tid] = 0;
  };
  // prefill: the 3 rows + 3 pixels before the first tile
  TileIter it(a, w_begin), nx(a, w_begin);
  uint32_t cur_frame = it.f;
  {
    const int64_t start = (int64_t)it.tt() * ENC_TILE;
    const int64_t lo = max((int64_t)0, start - 3 * (int64_t)W - 3);
    const uint8_t* fr = a.px + (uint64_t)cur_frame * a.frame_stride;
    for (int64_t j = lo + tid; j < start; j += CLS_THREADS) {
      const uint32_t k = (uint32_t)j & (RING - 1), y = y_from_rgba(px_word<C>(fr, j));
      ring[k] = y;
      if (k < CLS_GUARD) ring[RING + k] = y;
    }
  }
  // the first tile's pixels
  uint32_t pf[CLS_PPT];
  auto fetch = [&](const TileIter& ti, uint32_t (&v)[CLS_PPT]) {
    const uint32_t f = ti.f;
    const int64_t start = (int64_t)ti.tt() * ENC_TILE;
    if (C == 4) {
      const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)f * a.frame_stride);
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) {
        const int64_t j = start + q * CLS_THREADS + tid;
        v[q] = j < N ? fr[j] : 0u;
      }
    } else {   // the tile's dwords tid and 512 + tid
      const uint8_t* fr = a.px + (uint64_t)f * a.frame_stride;
      const uint64_t j0 = (uint64_t)ti.tt() * RGB_TILE_DW, nbytes = (uint64_t)N * 3;
      v[0] = 4 * (j0 + tid) < nbytes ? rgb_dword(fr, nbytes, j0 + tid) : 0u;
      v[1] = tid < RGB_TILE_DW - CLS_THREADS && 4 * (j0 + CLS_THREADS + tid) < nbytes
                 ? rgb_dword(fr, nbytes, j0 + CLS_THREADS + tid) : 0u;
    }
  };
  // two tiles in flight: tile w is staged from one register set while tiles
  // w + 1 (the other set) and w + 2 (refilling this one) load -- one tile of
  // classify work did not cover the HBM latency under load.  The loop body is
  // written once and instantiated for each set, so no register copy waits on
  // a load still in flight.
  uint32_t pb[CLS_PPT];
  fetch(nx, pf);
  nx.step(1);
  if (w_begin + 1 < w_end) fetch(nx, pb);
  nx.step(1);
  auto tile = [&](const uint64_t w, uint32_t (&pf)[CLS_PPT]) {
    const uint32_t f = it.f;
    const uint32_t tt = it.tt();
    if (f != cur_frame) {
      flush(cur_frame);
      cur_frame = f;
    }
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)min((int64_t)ENC_TILE, N - start);
    // stage this tile (Y space), start loading the next
    uint32_t pxw[CLS_PPT];
    if (C == 4) {
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) pxw[q] = pf[q];
    } else {   // bytes via LDS: the previous tile's readers are past its staging barrier
      stage[tid] = pf[0];
      if (tid < RGB_TILE_DW - CLS_THREADS) stage[CLS_THREADS + tid] = pf[1];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) {
        const uint32_t b = 3u * (uint32_t)(q * CLS_THREADS + tid);
        pxw[q] = __builtin_amdgcn_alignbit(stage[(b >> 2) + 1], stage[b >> 2], (b & 3u) * 8u);
      }
    }
    uint32_t yv[CLS_PPT];   // the thread's pixels in Y space (classify's X)
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const uint32_t k = (uint32_t)(start + q * CLS_THREADS + tid) & (RING - 1), y = y_from_rgba(pxw[q]);
      yv[q] = y;
      ring[k] = y;
      if (k < CLS_GUARD) ring[RING + k] = y;
    }
    // this tile's luma reference table (double-buffered: the previous tile's
    // readers are past the staging barrier below before it is rewritten)
    if (tid < 16 * CLS_PPT)
      ltab[w & 1][tid >> 4][tid & 15] =
          ((uint32_t)(start + (tid >> 4) * CLS_THREADS) - lback) & (RING - 1);
    if (w + 2 < w_end) fetch(nx, pf);
    nx.step(1);
    __syncthreads();
    __builtin_amdgcn_s_setprio(0);   // (raised by classify_y's luma search)
    // coded flags -> tile bitmask (a pixel is coded iff i == 0 or Y(i) != Y(i-1))
    uint32_t coded_bits = 0;
    unsigned long long wbal[CLS_PPT];   // coded flags of the wave's 64 pixels per q
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const int64_t i = start + p;
      const uint32_t* bl = ring + ((uint32_t)(start + q * CLS_THREADS - 1) & (RING - 1)) + tid;
      const bool coded = p < count && (i == 0 || bl[1] != bl[0]);
      const unsigned long long bal = __ballot(coded);
      wbal[q] = bal;
      if (lane == 0) {
        const int wb = (q * CLS_THREADS + (tid & ~63)) >> 5;
        mask[wb] = (uint32_t)bal;
        mask[wb + 1] = (uint32_t)(bal >> 32);
        if constexpr (MASK_OUT) {
          uint32_t* cm = a.cmask + it.tile() * (ENC_TILE / 32);
          cm[wb] = (uint32_t)bal;
          cm[wb + 1] = (uint32_t)(bal >> 32);
        }
      }
      coded_bits |= (coded ? 1u : 0u) << q;
    }
    __syncthreads();
    if (tid < 64) {   // first / last coded pixel of the tile: one wave, no loop
      const uint32_t mw = tid < ENC_TILE / 32 ? mask[tid] : 0u;
      const unsigned long long nz = __ballot(mw != 0);
      if (tid == 0) {
        const uint64_t t = it.tile();
        uint32_t first = NONE, last = NONE;
        if (nz) {
          const int fw = __builtin_ctzll(nz), lw = 63 - __builtin_clzll(nz);
          first = (uint32_t)(start + fw * 32 + __builtin_ctz(mask[fw]));
          last = (uint32_t)(start + lw * 32 + 31 - __builtin_clz(mask[lw]));
        }
        a.tile_first[t] = first;
        a.tile_last[t] = last;
      }
    }
    const bool fast = start >= 3 * (int64_t)W + 3;
    uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + start;
    uint32_t rec[CLS_PPT];
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {   // both pixels' modes first (independent LDS reads)
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      uint32_t rf;
      if (fast)   // block-uniform: both variants are straight-line code
        rf = classify_ring<false, RING>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W, 0u, ltab[w & 1][q],
                                        cbr, csd, yv[q]);
      else
        rf = classify_ring<true, RING>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W, (uint32_t)(start + p),
                                       nullptr, cbr, csd, yv[q]);
      rec[q] = coded ? rf : cunc;
    }
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      if (p < count) recs[p] = rec[q];
      // payload symbols (the mode prefixes are derived from them by enc_tables)
      slot_hist_add(hs, rec[q]);
      // a run follows only if the next pixel is uncoded: most coded lanes stop
      // at this one bit test (lane 63's next pixel is in the next wave: full path)
      if constexpr (MASK_OUT) continue;   // enc_rundigits counts them
      const bool next_coded = lane < 63 && ((wbal[q] >> (lane + 1)) & 1ull);
      if (coded && !next_coded) {
        // next coded pixel: in this wave's 64 pixels from the ballot, else the tile mask
        const unsigned long long above = lane < 63 ? (wbal[q] >> (lane + 1)) : 0ull;
        const int nx = above ? p + 1 + (int)__builtin_ctzll(above) : next_coded_local(mask, p | 63);
        if (nx < count && nx > p + 1) {
          uint64_t mm = (uint64_t)(nx - p - 2);
          while (true) {
            atomicAdd(&run_hist[(uint32_t)(mm & 7u)], 1u);
            if (mm < 8) break;
            mm >>= 3;
          }
        }
      }
    }
  };
  for (uint64_t w = w_begin; w < w_end; w += 2) {
    tile(w, pf);
    it.step(1);
    if (w + 1 < w_end) {
      tile(w + 1, pb);
      it.step(1);
    }
  }
  flush(cur_frame);
}
// ---------------------------------------------------------------------------
// K1p: the ring classify with up to two tiles per iteration ("pairs": 4
// pixels per thread, one staging barrier and one mask barrier per 2048
// pixels).  The pair is two consecutive tiles of one frame -- one contiguous
// 2048-pixel range of the raster -- so staging, coded flags and the mode
// decision run over it as one, with the per-tile outputs (first / last coded
// pixel, in-tile run digits) per tile; a tile left alone at a frame end or at
// the end of the block's range takes a one-tile iteration.  The next
// iteration's pixels load during this one (two tiles of work ahead).  The
// ring holds 3W + 3 pixels behind the pair plus the pair and the next one:
// 3W + 3 + 4096 <= RING.
// ---------------------------------------------------------------------------
// MASK_OUT (frames): the coded flags go out to a.cmask and enc_rundigits counts
// the run digits from them; false (bands): the digits are counted here.
template <int C, int RING, bool MASK_OUT = false>
__device__ __forceinline__ void enc_classify_pair_body(const EncArgs& a) {
  constexpr int PQ = 2 * CLS_PPT;   // pixel slots per thread (4)
  __shared__ uint32_t ring[RING + CLS_GUARD];
  __shared__ uint32_t stage[C == 3 ? 2 * RGB_TILE_DW + 4 : 1];
  __shared__ uint32_t hs[C0_N + 2 * SX_N];     // slot histogram (nice_rec.hpp)
  __shared__ uint32_t run_hist[8];             // run digits (prefixes 5..12)
  __shared__ uint32_t mask[2 * ENC_TILE / 32];
  __shared__ uint32_t ltab[2][PQ][16];         // [iteration parity][q][luma reference]: ring index for thread 0
  const uint64_t total_work = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  const uint64_t w_end = min(w_begin + a.tiles_per_block, total_work);
  if (w_begin >= w_end) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t cbr = (C0_BR << 3) | rec2_abs((uint32_t)lane), csd = (C0_SD << 3) | rec2_abs((uint32_t)lane);
  const uint32_t cunc = rec2_unc((uint32_t)lane);
  const uint32_t lback = tid < 16 * PQ && (tid & 15) < 11
                             ? (uint32_t)lr_rows(tid & 15) * a.W + (uint32_t)lr_px(tid & 15) : 0u;
  const uint32_t W = a.W;
  const int64_t N = (int64_t)W * a.H;
  for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
  if (tid < 8) run_hist[tid] = 0;
  auto flush = [&](uint32_t frame) {
    __syncthreads();
    for (int b = tid; b < N_BINS; b += CLS_THREADS) {
      uint32_t v = slot_hist_bin(hs, b);
      if (b >= BIN_PREFIX + P_RUN1 && b < BIN_PREFIX + P_RUN1 + 8) v += run_hist[b - BIN_PREFIX - P_RUN1];
      if (v) atomicAdd(&a.hist[(uint64_t)frame * N_BINS + b], v);
    }
    __syncthreads();
    for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
    if (tid < 8) run_hist[tid] = 0;
  };
  TileIter it(a, w_begin);
  uint32_t cur_frame = it.f;
  {   // prefill: the 3 rows + 3 pixels before the first tile
    const int64_t start = (int64_t)it.tt() * ENC_TILE;
    const int64_t lo = max((int64_t)0, start - 3 * (int64_t)W - 3);
    const uint8_t* fr = a.px + (uint64_t)cur_frame * a.frame_stride;
    for (int64_t j = lo + tid; j < start; j += CLS_THREADS) {
      const uint32_t k = (uint32_t)j & (RING - 1), y = y_from_rgba(px_word<C>(fr, j));
      ring[k] = y;
      if (k < CLS_GUARD) ring[RING + k] = y;
    }
  }
  // tiles in the iteration starting at work item w (iterator ti): two when
  // the next one is in the same frame and in the block's range
  auto tiles_at = [&](const TileIter& ti, uint64_t w) -> int {
    return (w + 1 < w_end && ti.k + 1 < ti.nt) ? 2 : 1;
  };
  uint32_t pf[PQ];
  auto fetch = [&](const TileIter& ti, int nti) {
    const uint32_t f = ti.f;
    const int64_t start = (int64_t)ti.tt() * ENC_TILE;
    if (C == 4) {
      const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)f * a.frame_stride);
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const int64_t j = start + q * CLS_THREADS + tid;
        pf[q] = (q < 2 * nti && j < N) ? fr[j] : 0u;
      }
    } else {   // the iteration's dwords tid, 512 + tid, 1024 + tid
      const uint8_t* fr = a.px + (uint64_t)f * a.frame_stride;
      const uint64_t j0 = (uint64_t)ti.tt() * RGB_TILE_DW, nbytes = (uint64_t)N * 3;
      const uint32_t ndw = (uint32_t)nti * RGB_TILE_DW;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const uint32_t d = (uint32_t)(q * CLS_THREADS + tid);
        pf[q] = d < ndw && 4 * (j0 + d) < nbytes ? rgb_dword(fr, nbytes, j0 + d) : 0u;
      }
    }
  };
  uint64_t w = w_begin;
  int nti = tiles_at(it, w);
  fetch(it, nti);
  uint32_t par = 0;
  while (w < w_end) {
    const int cur = nti;
    const uint32_t f = it.f;
    const uint32_t tt = it.tt();
    if (f != cur_frame) {
      flush(cur_frame);
      cur_frame = f;
    }
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)min((int64_t)(cur * ENC_TILE), N - start);   // pixels of the iteration
    // stage the iteration's pixels (Y space)
    uint32_t pxw[PQ];
    if (C == 4) {
#pragma unroll
      for (int q = 0; q < PQ; ++q) pxw[q] = pf[q];
    } else {   // bytes via LDS: the previous iteration's readers are past its staging barrier
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if ((uint32_t)(q * CLS_THREADS + tid) < (uint32_t)cur * RGB_TILE_DW) stage[q * CLS_THREADS + tid] = pf[q];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const uint32_t b = 3u * (uint32_t)(q * CLS_THREADS + tid);
        pxw[q] = q < 2 * cur ? __builtin_amdgcn_alignbit(stage[(b >> 2) + 1], stage[b >> 2], (b & 3u) * 8u) : 0u;
      }
    }
    uint32_t yv[PQ];   // the thread's pixels in Y space (classify's X)
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      yv[q] = y_from_rgba(pxw[q]);
      if (q < 2 * cur) {
        const uint32_t k = (uint32_t)(start + q * CLS_THREADS + tid) & (RING - 1);
        ring[k] = yv[q];
        if (k < CLS_GUARD) ring[RING + k] = yv[q];
      }
    }
    if (tid < 16 * PQ)
      ltab[par][tid >> 4][tid & 15] = ((uint32_t)(start + (tid >> 4) * CLS_THREADS) - lback) & (RING - 1);
    // the next iteration's pixels, in flight during this one
    TileIter nx = it;
    nx.step((uint32_t)cur);
    if (w + cur < w_end) {
      nti = tiles_at(nx, w + cur);
      fetch(nx, nti);
    }
    __syncthreads();
    __builtin_amdgcn_s_setprio(0);   // (raised by classify_y's luma search)
    // coded flags -> bitmask (a pixel is coded iff i == 0 or Y(i) != Y(i-1))
    uint32_t coded_bits = 0;
    unsigned long long wbal[PQ];
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int p = q * CLS_THREADS + tid;
      const uint32_t* bl = ring + ((uint32_t)(start + q * CLS_THREADS - 1) & (RING - 1)) + tid;
      const bool coded = q < 2 * cur && p < count && ((start == 0 && p == 0) || bl[0] != yv[q]);
      const unsigned long long bal = __ballot(coded);
      wbal[q] = bal;
      if (lane == 0 && q < 2 * cur) {
        const int wb = (q * CLS_THREADS + (tid & ~63)) >> 5;
        mask[wb] = (uint32_t)bal;
        mask[wb + 1] = (uint32_t)(bal >> 32);
        if constexpr (MASK_OUT) {   // tiles tt, tt + 1 are consecutive: one 64-word range
          uint32_t* cm = a.cmask + it.tile() * (ENC_TILE / 32);
          cm[wb] = (uint32_t)bal;
          cm[wb + 1] = (uint32_t)(bal >> 32);
        }
      }
      coded_bits |= (coded ? 1u : 0u) << q;
    }
    __syncthreads();
    if (tid < 64 * cur) {   // wave j: first / last coded pixel of tile j
      const int j = tid >> 6;
      const uint32_t* mk = mask + 32 * j;
      const uint32_t mw = lane < ENC_TILE / 32 ? mk[lane] : 0u;
      const unsigned long long nz = __ballot(mw != 0);
      if (lane == 0) {
        const uint64_t t = it.tile() + (uint64_t)j;
        const int64_t sj = start + (int64_t)j * ENC_TILE;
        uint32_t first = NONE, last = NONE;
        if (nz) {
          const int fw = __builtin_ctzll(nz), lw = 63 - __builtin_clzll(nz);
          first = (uint32_t)(sj + fw * 32 + __builtin_ctz(mk[fw]));
          last = (uint32_t)(sj + lw * 32 + 31 - __builtin_clz(mk[lw]));
        }
        a.tile_first[t] = first;
        a.tile_last[t] = last;
      }
    }
    const bool fast = start >= 3 * (int64_t)W + 3;
    uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + start;
    uint32_t rec[PQ];
    if (fast && cur == 2) {
      // the steady state (block-uniform): the four slots as one straight-line
      // block, so the scheduler interleaves their LDS reads and arithmetic
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const uint32_t rf = classify_ring<false, RING>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W,
                                                       0u, ltab[par][q], cbr, csd, yv[q]);
        rec[q] = ((coded_bits >> q) & 1u) ? rf : cunc;
      }
    } else
#pragma unroll
    for (int q = 0; q < PQ; ++q) {   // every pixel's mode first (independent LDS reads)
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      uint32_t rf = cunc;
      if (q < 2 * cur) {   // block-uniform
        if (fast)
          rf = classify_ring<false, RING>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W, 0u,
                                          ltab[par][q], cbr, csd, yv[q]);
        else
          rf = classify_ring<true, RING>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W,
                                         (uint32_t)(start + p), nullptr, cbr, csd, yv[q]);
      }
      rec[q] = coded ? rf : cunc;
    }
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      if (q >= 2 * cur) continue;   // block-uniform
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      if (p < count) recs[p] = rec[q];
      slot_hist_add(hs, rec[q]);
      // a run follows only if the next pixel is uncoded; runs crossing the
      // tile's end are enc_tailruns' (lane 63's next pixel is in the next wave)
      if constexpr (MASK_OUT) continue;   // enc_rundigits counts them
      const bool next_coded = lane < 63 && ((wbal[q] >> (lane + 1)) & 1ull);
      if (coded && !next_coded) {
        const int j = q >> 1, pl = p - j * ENC_TILE;   // tile and index in it
        const int cj = min(count - j * ENC_TILE, ENC_TILE);
        const unsigned long long above = lane < 63 ? (wbal[q] >> (lane + 1)) : 0ull;
        const int nxl = above ? pl + 1 + (int)__builtin_ctzll(above) : next_coded_local(mask + 32 * j, pl | 63);
        if (nxl < cj && nxl > pl + 1) {
          uint32_t mm = (uint32_t)(nxl - pl - 2);
          while (true) {
            atomicAdd(&run_hist[mm & 7u], 1u);
            if (mm < 8) break;
            mm >>= 3;
          }
        }
      }
    }
    par ^= 1u;
    it.step((uint32_t)cur);
    w += (uint64_t)cur;
  }
  flush(cur_frame);
}

__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring(EncArgs a) { enc_classify_ring_body<4, CLS_RING>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring3(EncArgs a) { enc_classify_ring_body<3, CLS_RING>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring_m(EncArgs a) {
  enc_classify_ring_body<4, CLS_RING, true>(a);
}
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring3_m(EncArgs a) {
  enc_classify_ring_body<3, CLS_RING, true>(a);
}
// a 32K-pixel ring (128 KB, one block per CU) for rows of up to
// CLS_RING2_MAX_W pixels: RGBA widths the strip kernel does not take (W %
// 1024 != 0, e.g. 7680 for 8K UHD) and RGB frames
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring2(EncArgs a) { enc_classify_ring_body<4, 2 * CLS_RING>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring2_3(EncArgs a) { enc_classify_ring_body<3, 2 * CLS_RING>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring2_m(EncArgs a) {
  enc_classify_ring_body<4, 2 * CLS_RING, true>(a);
}
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring2_3_m(EncArgs a) {
  enc_classify_ring_body<3, 2 * CLS_RING, true>(a);
}
// pairs of tiles per iteration (16K ring: W <= CLS_PAIR_MAX_W)
// (RGBA; an RGB pair's 6 KB byte stage would push the block past 80 KB of LDS,
// one block per CU)
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_pair(EncArgs a) { enc_classify_pair_body<4, CLS_RING>(a); }
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_pair_m(EncArgs a) {
  enc_classify_pair_body<4, CLS_RING, true>(a);
}

// ---------------------------------------------------------------------------
// K1w: classify with per-lane sliding windows (round 6; RGBA frames, 3 <= W <=
// CLS_PAIR_MAX_W, pixel memory 16-byte aligned: the bench path).  The pair
// kernel gives each lane pixels 512 apart, so every pixel re-reads its 13
// neighbours from the ring one word at a time (about 15 LDS instructions and
// three Y -> RGB conversions per pixel).  Here a lane owns 4 CONSECUTIVE
// pixels of the iteration's 2048 (one 16-byte global load, one 16-byte ring
// store) and reads, per neighbour row, one aligned window covering its 4
// pixels' references (rows y-1 and y-3: pixels i-rW-3 .. i-rW+6; row y-2:
// i-2W .. i-2W+3; row y: the 3 pixels before) with ds_read_b128s -- 8 to 11
// per 4 pixels, conflict-free (consecutive lanes read consecutive 16 bytes).
// Every reference is then a register chosen at compile time: the window
// offsets depend only on W mod 4 (the template parameter), the left
// neighbours L, L2, L3 of pixels 1..3 are the lane's own pixels, and pixel
// q's RGB spread is pixel q+1's RGB(L) (one conversion saved per pixel).
// The coded flags come out of the compares as wave ballots; the per-tile
// first / last coded pixel are found from them with scalar bit scans, and the
// flags go to a.cmask in the ballot order (wave w's 8 words: ballot q's low
// and high halves), which enc_rundigits transposes.  Same records, histogram
// and tile edges as enc_classify_pair_m (code.rs:159-414).
// ---------------------------------------------------------------------------
// pixel word v (R | G << 8 | B << 16) -> its Y-space value and RGB spread (sharing G)
__device__ __forceinline__ void y_rgb_from_rgba(uint32_t v, uint32_t& y, uint32_t& xr) {
  const uint32_t g = __builtin_amdgcn_ubfe(v, 8, 8);
  const nice_u16x2 d = __builtin_bit_cast(nice_u16x2, v) - __builtin_bit_cast(nice_u16x2, g | (g << 16));
  const uint32_t t = __builtin_bit_cast(uint32_t, d);
  y = (__umul24(t & 0xFF0000u, 16u) + (t & 0xFFu)) | (g << 10);
  xr = (y + __umul24(g, 0x100001u)) & K3(0xFFu);
}

// classify_y<false> with every reference in registers: X (Y space) and its RGB
// spread xr, L and its spread lrgb; the luma hit's difference is read again from
// the ring at byte (i4 + loff4[k]) mod 4 RING (i4 = 4 i, loff4[k] = -4 offset of
// reference k).
__device__ __forceinline__ uint32_t classify_win(uint32_t X, uint32_t xr, uint32_t L, uint32_t lrgb, uint32_t L2,
                                                 uint32_t L3, uint32_t U, uint32_t UR1, uint32_t UR3, uint32_t UL3,
                                                 uint32_t U2, uint32_t V, uint32_t VR1, uint32_t VL1, uint32_t VL3,
                                                 uint32_t VR3, const uint32_t* ring, uint32_t i4, const uint32_t* loff4,
                                                 uint32_t cbr, uint32_t csd, uint32_t pq) {
  // back references k = 1..4 (code.rs:191-206)
  const bool e1 = U == X, e2 = UR1 == X, e3 = L2 == X, e4 = U2 == X;
  const bool br = e1 | e2 | e3 | e4;
  const uint32_t bk = e1 ? 1u : e2 ? 2u : e3 ? 3u : 4u;
  const uint32_t pred = avg3(rgb_from_y(U), lrgb);
  // small diff (code.rs:208-247), as in classify_y
  const uint32_t d = xr + K3(259u) - pred;
  const bool sd = ((d & K3(0x3F8u)) | ((d + K3(1u)) & K3(8u))) == K3(0x100u);
  const uint32_t sdi = (__umul24(d & K3(7u), 49u | (7u << 10) | (1u << 20)) >> 20) & 0x3FFu;
  // luma2 (code.rs:252-292)
  const uint32_t pg = (pred >> 10) & 0xFFu;
  const uint32_t xk = X + LUMA_KY;
  const uint32_t t2 = (xk - pred) + (pg | (pg << 20));
  const bool l2 = (t2 & LUMA_MASK) == 0;
  // luma, 11 references, first hit wins (code.rs:293-339): min-key search
  uint32_t lk = 11u, lt = 0u;
  if (__builtin_amdgcn_ballot_w64(!br && !sd && !l2) != 0ull) {
    // a wave that takes the luma search issues first until its block's next
    // barrier (the block waits on its slowest wave), the more so the later in
    // the lane's four pixels it needs it (pq: 1, 1, 2, 3): classify 15.22 ->
    // 14.12 ms per 512 frames (profiles/r06zp_ab_cls_prio.log,
    // r06zq_ab_cls_prio_modes.log; by the count of searches so far: 14.35)
    if (pq >= 3) __builtin_amdgcn_s_setprio(3);
    else if (pq == 2) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(1);
    const uint32_t refs[11] = {L, U, UR1, UR3, L3, VR1, V, VL1, UL3, VL3, VR3};
    uint32_t key[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) key[k] = ((xk - refs[k]) & LUMA_MASK) | (uint32_t)k;
    const uint32_t m = min(min(min(min(key[0], key[1]), key[2]), min(min(key[3], key[4]), key[5])),
                           min(min(min(key[6], key[7]), key[8]), min(key[9], key[10])));
    lk = min(m, 11u);
    // loff4[k]: -4 (offset of reference k) mod 4 RING bytes (0 at k = 11)
    lt = xk - *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(ring) +
                                                  ((i4 + loff4[lk]) & ((CLS_RING - 1) * 4)));
  }
  const uint32_t r = d - K3(3u);   // = xr + 256 - pred per field
  const uint32_t rec_br = (bk << 3) + cbr;
  const uint32_t rec_sd = (sdi << 3) + csd;
  const uint32_t rs = r & K3(0xFFu);
  const uint32_t rec_rgb = (rs + (rs & (0xFFu << 10))) << 3;
  const uint32_t lf = l2 ? t2 : lt;
  const uint32_t lbase = l2 ? ((C0_L2 << 3) | (SX_L2 << 14) | (SX_L2 << 23))
                            : ((C0_LUMA << 3) | (SX_LUMA << 14) | (SX_LUMA << 23)) + (lk << 9);
  const uint32_t rec_lu = lbase + (__builtin_amdgcn_ubfe(lf, 10, 6) << 3) + ((lf & 0x1Fu) << 14) +
                          ((lf & (0x1Fu << 20)) << 3);
  return br ? rec_br : sd ? rec_sd : (l2 || lk < 11u) ? rec_lu : rec_rgb;
}

// a lane's records past the frame's end are not stored (1..3 of its 4 remain)
__device__ __noinline__ void store_tail3(uint32_t* p, uint32_t r0, uint32_t r1, uint32_t r2, int n) {
  p[0] = r0;
  if (n > 1) p[1] = r1;
  if (n > 2) p[2] = r2;
}

template <int WM>   // W mod 4
__device__ __forceinline__ void enc_classify_slide_body(const EncArgs& a) {
  constexpr int RING = CLS_RING;
  constexpr uint32_t RM = RING - 1;
  // window geometry (words, all multiples of 4 away from the lane's first
  // pixel i0 = start + 4 tid): row r's window starts OFF_r before i0, rounded
  // up to a multiple of 4 by D_r, and spans NB_r 16-byte blocks
  constexpr uint32_t D1 = (4u - (uint32_t)(WM + 3) % 4u) % 4u;       // row y-1: i - W - 3 ..
  constexpr uint32_t D2 = (4u - (uint32_t)(2 * WM) % 4u) % 4u;       // row y-2: i - 2W ..
  constexpr uint32_t D3 = (4u - (uint32_t)(3 * WM + 3) % 4u) % 4u;   // row y-3: i - 3W - 3 ..
  constexpr int NB1 = (int)(D1 + 10u + 3u) / 4, NB2 = (int)(D2 + 4u + 3u) / 4, NB3 = (int)(D3 + 10u + 3u) / 4;
  // one block of LDS, laid out so that the histogram sits at address 0: its
  // atomics' base folds into the instruction's 16-bit offset (placed after
  // the 67 KB ring it cost one VALU add per atomic, three per pixel)
  struct SlideLds {
    uint32_t hs[C0_N + 2 * SX_N];               // slot histogram (nice_rec.hpp)
    uint32_t loff4[16];                         // luma reference k: -4 (its offset) mod 4 RING
    uint32_t wfl[2][CLS_THREADS / 64][2];       // [parity][wave]: first coded pixel, last + 1 (tile-relative)
    __attribute__((aligned(16))) uint32_t ring[RING + CLS_GUARD];
  };
  __shared__ SlideLds sl;
  uint32_t* const hs = sl.hs;
  uint32_t* const loff4 = sl.loff4;
  uint32_t* const ring = sl.ring;
  auto& wfl = sl.wfl;
  const uint64_t total_work = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  const uint64_t w_end = min(w_begin + a.tiles_per_block, total_work);
  if (w_begin >= w_end) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t cbr = (C0_BR << 3) | rec2_abs(lane), csd = (C0_SD << 3) | rec2_abs(lane);
  const uint32_t cunc = rec2_unc(lane);
  const uint32_t W = a.W;
  const int64_t N = (int64_t)W * a.H;
  const uint32_t OFF1 = W + 3u + D1, OFF2 = 2u * W + D2, OFF3 = 3u * W + 3u + D3;
  for (uint32_t b = tid; b < C0_N + 2 * SX_N; b += CLS_THREADS) hs[b] = 0;
  if (tid < 16)
    loff4[tid] = tid < 11 ? ((0u - ((uint32_t)lr_rows((int)tid) * W + (uint32_t)lr_px((int)tid))) & RM) * 4u : 0u;
  auto flush = [&](uint32_t frame) {
    __syncthreads();
    for (int b = tid; b < N_BINS; b += CLS_THREADS) {
      const uint32_t v = slot_hist_bin(hs, b);
      if (v) atomicAdd(&a.hist[(uint64_t)frame * N_BINS + b], v);
    }
    __syncthreads();
    for (uint32_t b = tid; b < C0_N + 2 * SX_N; b += CLS_THREADS) hs[b] = 0;
  };
  TileIter it(a, w_begin);
  uint32_t cur_frame = it.f;
  {   // prefill: the 3 rows + 3 pixels before the first tile
    const int64_t start = (int64_t)it.tt() * ENC_TILE;
    const int64_t lo = max((int64_t)0, start - 3 * (int64_t)W - 3);
    const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)cur_frame * a.frame_stride);
    for (int64_t j = lo + tid; j < start; j += CLS_THREADS) {
      const uint32_t k = (uint32_t)j & RM, y = y_from_rgba(fr[j]);
      ring[k] = y;
      if (k < CLS_GUARD) ring[RING + k] = y;
    }
  }
  auto tiles_at = [&](const TileIter& ti, uint64_t w) -> int {
    return (w + 1 < w_end && ti.k + 1 < ti.nt) ? 2 : 1;
  };
  uint4 pf;
  auto fetch = [&](const TileIter& ti, int nti) {
    const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)ti.f * a.frame_stride);
    const int64_t j = (int64_t)ti.tt() * ENC_TILE + 4 * (int64_t)tid;
    if (tid < 256u * (uint32_t)nti && j + 4 <= N) {
      pf = *reinterpret_cast<const uint4*>(fr + j);
    } else {
      const bool in = tid < 256u * (uint32_t)nti;
      pf.x = in && j < N ? fr[j] : 0u;
      pf.y = in && j + 1 < N ? fr[j + 1] : 0u;
      pf.z = in && j + 2 < N ? fr[j + 2] : 0u;
      pf.w = in && j + 3 < N ? fr[j + 3] : 0u;
    }
  };
  // the previous iteration's tiles: first / last coded pixel from its waves'
  // entries (after a barrier)
  uint64_t prev_tile = 0;
  int64_t prev_start = 0;
  uint32_t prev_cur = 0, prev_par = 0;
  auto combine = [&]() {
    if (tid < prev_cur) {
      uint32_t fi = NONE, la = 0;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        fi = min(fi, wfl[prev_par][4 * tid + v][0]);
        la = max(la, wfl[prev_par][4 * tid + v][1]);
      }
      const int64_t sj = prev_start + (int64_t)tid * ENC_TILE;
      a.tile_first[prev_tile + tid] = fi == NONE ? NONE : (uint32_t)(sj + fi);
      a.tile_last[prev_tile + tid] = la == 0 ? NONE : (uint32_t)(sj + la - 1);
    }
  };
  uint64_t w = w_begin;
  int nti = tiles_at(it, w);
  fetch(it, nti);
  uint32_t par = 0;
  while (w < w_end) {
    const int cur = nti;
    const uint32_t f = it.f;
    if (f != cur_frame) {
      flush(cur_frame);
      cur_frame = f;
    }
    const int64_t start = (int64_t)it.tt() * ENC_TILE;
    const int count = (int)min((int64_t)(cur * ENC_TILE), N - start);   // pixels of the iteration
    // the lane's 4 pixels in Y space and RGB spread; into the ring
    uint32_t X[4], XR[4];
    y_rgb_from_rgba(pf.x, X[0], XR[0]);
    y_rgb_from_rgba(pf.y, X[1], XR[1]);
    y_rgb_from_rgba(pf.z, X[2], XR[2]);
    y_rgb_from_rgba(pf.w, X[3], XR[3]);
    const uint32_t i0 = (uint32_t)start + 4u * tid;
    if (tid < 256u * (uint32_t)cur) {
      const uint32_t k = i0 & RM;
      *reinterpret_cast<uint4*>(ring + k) = make_uint4(X[0], X[1], X[2], X[3]);
      if (k < CLS_GUARD) *reinterpret_cast<uint4*>(ring + RING + k) = make_uint4(X[0], X[1], X[2], X[3]);
    }
    // the next iteration's pixels, in flight during this one
    TileIter nx = it;
    nx.step((uint32_t)cur);
    if (w + cur < w_end) {
      nti = tiles_at(nx, w + cur);
      fetch(nx, nti);
    }
    __syncthreads();
    __builtin_amdgcn_s_setprio(0);   // (raised by classify_win's luma search)
    if (prev_cur) combine();
    const bool fast = start >= 3 * (int64_t)W + 3;   // block-uniform
    uint32_t rec[4];
    unsigned long long bal[4];
    if (fast) {
      // the windows: base = ring index of (wave's first pixel - OFF_r) plus 4 lane
      const uint32_t sw = (uint32_t)start + 256u * wave;
      const uint32_t i4 = 4u * i0;
      const uint32_t* b0 = ring + ((sw - 4u) & RM) + 4u * lane;
      const uint32_t* b1 = ring + ((sw - OFF1) & RM) + 4u * lane;
      const uint32_t* b2 = ring + ((sw - OFF2) & RM) + 4u * lane;
      const uint32_t* b3 = ring + ((sw - OFF3) & RM) + 4u * lane;
      uint32_t w0[4], w1[4 * NB1], w2[4 * NB2], w3[4 * NB3];
      // whole 16-byte blocks (ds_read_b128: conflict-free for consecutive
      // lanes); the empty asm keeps the compiler from narrowing a block whose
      // end words are unused into ds_read2_b64 / b32 pieces, which conflict
      // two-way at this 16-byte lane stride (classify 15.95 -> 15.39 ms per
      // 512 4K frames)
      auto blk = [](const uint32_t* p, uint32_t* d) {
        nice_u32x4 v = *reinterpret_cast<const nice_u32x4*>(p);
        asm volatile("" : "+v"(v));
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      };
      blk(b0, w0);
#pragma unroll
      for (int b = 0; b < NB1; ++b) blk(b1 + 4 * b, w1 + 4 * b);
#pragma unroll
      for (int b = 0; b < NB2; ++b) blk(b2 + 4 * b, w2 + 4 * b);
#pragma unroll
      for (int b = 0; b < NB3; ++b) blk(b3 + 4 * b, w3 + 4 * b);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t L = q >= 1 ? X[q - 1] : w0[3];
        const uint32_t L2 = q >= 2 ? X[q - 2] : w0[2 + q];
        const uint32_t L3 = q >= 3 ? X[q - 3] : w0[1 + q];
        const uint32_t lrgb = q >= 1 ? XR[q - 1] : rgb_from_y(w0[3]);
        const uint32_t pq = q == 3 ? 3u : q == 2 ? 2u : 1u;   // (compile-time after unrolling)
        const uint32_t rf = classify_win(X[q], XR[q], L, lrgb, L2, L3, w1[q + 3 + D1], w1[q + 4 + D1],
                                         w1[q + 6 + D1], w1[q + D1], w2[q + D2], w3[q + 3 + D3], w3[q + 4 + D3],
                                         w3[q + 2 + D3], w3[q + D3], w3[q + 6 + D3], ring, i4 + 4u * (uint32_t)q,
                                         loff4, cbr, csd, pq);
        // (the flag after the decision: kept across it, it went through a VGPR)
        const bool coded = 4 * (int)tid + q < count && X[q] != L;
        bal[q] = __builtin_amdgcn_ballot_w64(coded);
        rec[q] = coded ? rf : cunc;
      }
    } else {
      // the frame's first rows: the reference's validity rules (classify_y<true>)
      // per pixel, neighbours one word at a time (s + tid: the pixel's index)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t i = i0 + (uint32_t)q;
        const bool coded = 4 * (int)tid + q < count && (i == 0 || X[q] != ring[(i - 1u) & RM]);
        bal[q] = __builtin_amdgcn_ballot_w64(coded);
        const uint32_t rf = classify_ring<true>(ring, (uint32_t)start + (uint32_t)q + 3u * tid, tid, W, i, nullptr,
                                                cbr, csd, X[q]);
        rec[q] = coded ? rf : cunc;
      }
    }
    // the wave's first / last coded pixel (tile-relative) and its coded flags
    // in ballot order (enc_rundigits transposes them)
    if (tid < 256u * (uint32_t)cur) {
      uint32_t fi = NONE, la = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (bal[q]) {
          fi = min(fi, 4u * (uint32_t)__builtin_ctzll(bal[q]) + (uint32_t)q);
          la = max(la, 4u * (uint32_t)(63 - __builtin_clzll(bal[q])) + (uint32_t)q + 1u);
        }
      }
      const uint32_t wo = 256u * (wave & 3u);
      if (lane == 0) {
        wfl[par][wave][0] = fi == NONE ? NONE : wo + fi;
        wfl[par][wave][1] = la == 0 ? 0u : wo + la;
      }
      const uint32_t hw = lane & 1u, qq = (lane >> 1) & 3u;
      const unsigned long long bq = qq == 0 ? bal[0] : qq == 1 ? bal[1] : qq == 2 ? bal[2] : bal[3];
      if (lane < 8u) a.cmask[(it.tile() + (wave >> 2)) * (ENC_TILE / 32) + 8u * (wave & 3u) + lane] =
          (uint32_t)(bq >> (32u * hw));
    }
    // records out (one 16-byte store; a lane with pixels past the frame's end
    // stores them one by one), histogram
    uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + (uint64_t)i0;
    if (4 * (int)tid + 3 < count)
      *reinterpret_cast<uint4*>(__builtin_assume_aligned(recs, 16)) = make_uint4(rec[0], rec[1], rec[2], rec[3]);
    else if (4 * (int)tid < count)
      store_tail3(recs, rec[0], rec[1], rec[2], count - 4 * (int)tid);
    if (tid < 256u * (uint32_t)cur) {
#pragma unroll
      // (same-address adds cost nothing extra: every lane on its own zero
      // slots instead measured slower, 14.07 -> 14.74 ms, r06zt_hist_probe.log)
      for (int q = 0; q < 4; ++q) slot_hist_add(hs, rec[q]);
    }
    prev_tile = it.tile();
    prev_start = start;
    prev_cur = (uint32_t)cur;
    prev_par = par;
    par ^= 1u;
    it.step((uint32_t)cur);
    w += (uint64_t)cur;
  }
  __syncthreads();
  combine();
  flush(cur_frame);
}
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_slide0(EncArgs a) { enc_classify_slide_body<0>(a); }
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_slide1(EncArgs a) { enc_classify_slide_body<1>(a); }
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_slide2(EncArgs a) { enc_classify_slide_body<2>(a); }
__global__ __launch_bounds__(CLS_THREADS, 2) void enc_classify_slide3(EncArgs a) { enc_classify_slide_body<3>(a); }

// ---------------------------------------------------------------------------
// K1r: run digits of the runs inside tiles (code.rs:371-407: a run between two
// coded pixels of one tile, length L >= 1, adds the base-8 digits of L - 1 to
// the run prefixes' bins; runs that cross a tile's end are enc_tailruns'),
// from the coded flags enc_classify_pair_m wrote, one 32-pixel word per lane.
// Counting them inside the classify loop cost that loop 17 % (21.2 vs 17.5 ms
// per 512 4K frames without the block), in its branches and live state.  A
// run ends at each coded pixel whose previous pixel is uncoded; its start is
// the previous coded pixel of the word, or the last coded pixel of the tile's
// earlier words (a max scan over the half-wave), or none in the tile (skipped).
// ---------------------------------------------------------------------------
// il != 0: the tiles' flags are in enc_classify_slide's ballot order (wave w
// of a tile: words 8w + 2q + h = half h of the ballot of its lanes' q-th
// pixels, pixel 256w + 4 lane + q), transposed here: standard word k holds
// byte k % 8 of each ballot q, bit m at 4m + q.
__global__ __launch_bounds__(256) void enc_rundigits(EncArgs a, int il) {
  __shared__ uint32_t bins[8];
  if (threadIdx.x < 8) bins[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t f = blockIdx.y, T = a.tiles_per_frame;
  const uint32_t lane = threadIdx.x & 63u, k = lane & 31u;
  const uint32_t wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nwv = gridDim.x * (blockDim.x >> 6);
  uint32_t cnt[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  // RD_U tile pairs per iteration, every load issued before any is used (one
  // pair per iteration waited on each load: 0.65 ms per 512 4K frames)
  constexpr uint32_t RD_U = 4;
  for (uint32_t tb0 = 2u * wv; tb0 < T; tb0 += 2u * nwv * RD_U) {
    uint32_t raw[RD_U][4];
#pragma unroll
    for (uint32_t u = 0; u < RD_U; ++u) {
      const uint32_t t = tb0 + 2u * nwv * u + (lane >> 5);   // lanes 0-31: the pair's first tile, 32-63: its second
      const uint32_t* tw = a.cmask + ((uint64_t)f * T + (t < T ? t : 0u)) * (ENC_TILE / 32);
      if (il) {
        tw += 8u * (k >> 3) + ((k >> 2) & 1u);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) raw[u][q] = t < T ? tw[2 * q] : 0u;
      } else {
        raw[u][0] = t < T ? tw[k] : 0u;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < RD_U; ++u) {
    const uint32_t t = tb0 + 2u * nwv * u + (lane >> 5);
    if (__all(t >= T)) break;   // (wave-uniform: the pairs past the frame's tiles)
    uint32_t m = 0;
    if (t < T) {
      if (il) {
        const uint32_t sh = 8u * (k & 3u);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
          uint32_t x = (raw[u][q] >> sh) & 0xFFu;   // bit m -> bit 4m
          x = (x | (x << 12)) & 0x000F000Fu;
          x = (x | (x << 6)) & 0x03030303u;
          x = (x | (x << 3)) & 0x11111111u;
          m |= x << q;
        }
        // the standard order back in place (enc_pack reads 16 flags per lane
        // from it); every source word of the tile was read by this wave's
        // loads above
        a.cmask[((uint64_t)f * T + t) * (ENC_TILE / 32) + k] = m;
      } else {
        m = raw[u][0];
      }
    }
    // last coded pixel of the tile before this word (-1: none)
    int inc = m ? (int)(32u * k + 31u - (uint32_t)__clz((int)m)) : -1;
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if ((int)k >= o) inc = max(inc, v);
    }
    int before = __shfl_up(inc, 1);
    uint32_t pm = __shfl_up(m, 1);
    if (k == 0u) { before = -1; pm = 0x80000000u; }   // (a run into the tile: not counted here)
    uint32_t tb = m & ~((m << 1) | (pm >> 31));        // coded pixels after an uncoded one
    while (tb) {
      const uint32_t b = (uint32_t)__builtin_ctz(tb);
      tb &= tb - 1u;
      const uint32_t below = m & ((1u << b) - 1u);
      const int prev = below ? (int)(32u * k + 31u - (uint32_t)__clz((int)below)) : before;
      if (prev >= 0) {
        uint32_t mm = (uint32_t)((int)(32u * k + b) - prev - 2);
        while (true) {
          const uint32_t d = mm & 7u;
#pragma unroll
          for (int j = 0; j < 8; ++j) cnt[j] += d == (uint32_t)j ? 1u : 0u;
          if (mm < 8u) break;
          mm >>= 3;
        }
      }
    }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {   // wave sums, then one LDS add per wave and bin
    uint32_t v = cnt[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0 && v) atomicAdd(&bins[j], v);
  }
  __syncthreads();
  if (threadIdx.x < 8 && bins[threadIdx.x])
    atomicAdd(&a.hist[(uint64_t)f * N_BINS + BIN_PREFIX + P_RUN1 + threadIdx.x], bins[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// K1s: classify, strip-staged (RGBA frames with W % 1024 == 0 too wide for the
// ring: W > CLS_RING_MAX_W).  The frame is cut into vertical strips of up to
// STRIP_W columns (a multiple of 1024, so each strip row is whole raster tiles
// and the tile bookkeeping is the ring kernel's); a block walks rows
// [y0, y1) of one strip keeping four row windows in LDS, each the LINEAR
// pixels [yW + x0 - 3, yW + x1 + 3) of its row: every reference of a pixel
// of the strip -- 0..3 rows up, 3 pixels either side, wrapping across row ends
// like the reference's linear offsets (code.rs:141-145) -- is inside the
// window of its row.  Same outputs as enc_classify_ring.
// ---------------------------------------------------------------------------
constexpr int STRIP_W = 2048;
constexpr int STRIP_RS = STRIP_W + 8;              // window words (+3 each side, padded)
constexpr int STRIP_LD = (STRIP_W + 6 + CLS_THREADS - 1) / CLS_THREADS;   // window loads per thread (5)

template <bool MASK_OUT>
__device__ __forceinline__ void enc_classify_strip_body(const EncArgs& a) {
  __shared__ uint32_t win[4][STRIP_RS];
  __shared__ uint32_t hs[C0_N + 2 * SX_N];
  __shared__ uint32_t run_hist[8];
  __shared__ uint32_t mask[STRIP_W / ENC_TILE][ENC_TILE / 32];
  __shared__ uint32_t ltab[STRIP_W / ENC_TILE][CLS_PPT][16];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t W = a.W, H = a.H;
  const uint32_t T = a.tiles_per_frame, tpr = W / ENC_TILE;   // tiles per row
  const uint32_t nstrips = (W + STRIP_W - 1) / STRIP_W;
  const uint32_t rows = a.tiles_per_block;                    // rows per block
  // the band's rows (frames: all)
  const uint32_t ylo = a.tile_lo / tpr, yhi = (a.tile_hi + tpr - 1) / tpr;
  const uint32_t nchunks = (yhi - ylo + rows - 1) / rows;
  uint32_t b = blockIdx.x;
  const uint32_t chunk = b % nchunks;
  b /= nchunks;
  const uint32_t s = b % nstrips, f = b / nstrips;
  if (f >= a.n_frames) return;
  const uint32_t y0 = ylo + chunk * rows, y1 = min(y0 + rows, yhi);
  const uint32_t x0 = s * STRIP_W, x1 = min(x0 + STRIP_W, W);
  const uint32_t ntr = (x1 - x0) / ENC_TILE;                  // tiles per strip row (1 or 2)
  const uint8_t* fr = a.px + (uint64_t)f * a.frame_stride;
  const int64_t N = (int64_t)W * H;
  const uint32_t cbr = (C0_BR << 3) | rec2_abs((uint32_t)lane), csd = (C0_SD << 3) | rec2_abs((uint32_t)lane);
  const uint32_t cunc = rec2_unc((uint32_t)lane);
  for (int k = tid; k < (int)(C0_N + 2 * SX_N); k += CLS_THREADS) hs[k] = 0;
  if (tid < 8) run_hist[tid] = 0;
  // row y's window: linear pixels [yW + x0 - 3, yW + x1 + 3) (0 outside the
  // frame / the caller's pixel memory), loaded into registers
  uint32_t pw[STRIP_LD];
  auto fetch_row = [&](int64_t y) {   // y = -1: the window of row -1 (its end is row 0's first pixels)
    const int64_t g0 = y * (int64_t)W + x0 - 3;
    const int64_t lo = max((int64_t)0, a.px_lo), hi = min(N, a.px_hi);
#pragma unroll
    for (int k = 0; k < STRIP_LD; ++k) {
      const int c = tid + k * CLS_THREADS;
      const int64_t g = g0 + c;
      pw[k] = (c < (int)(x1 - x0) + 6 && g >= lo && g < hi) ? reinterpret_cast<const uint32_t*>(fr)[g] : 0u;
    }
  };
  auto commit_row = [&](int64_t y) {
    uint32_t* wr = win[(uint32_t)y & 3u];
#pragma unroll
    for (int k = 0; k < STRIP_LD; ++k) {
      const int c = tid + k * CLS_THREADS;
      if (c < (int)(x1 - x0) + 6) wr[c] = y_from_rgba(pw[k]);
    }
  };
  // prefill rows y0-3 .. y0-1, from row -1 on: the window of the row above
  // row 0 ends with row 0's first pixels, which the last columns of row 0
  // reference through offsets W-1 and W-3 (code.rs:141-145; round 5 width
  // sweep: 10240 x 12 RGBA frames whose pixel W-3 only luma reference 3 predicts)
  for (int64_t y = y0 >= 3 ? (int64_t)y0 - 3 : -1; y < (int64_t)y0; ++y) {
    fetch_row(y);
    commit_row(y);
  }
  // back distance of luma reference k in (rows, pixels) for the tile tables
  const int lk_rows = tid < 16 && tid < 11 ? lr_rows(tid) : 0, lk_px = tid < 16 && tid < 11 ? lr_px(tid) : 0;
  fetch_row(y0);
  for (uint32_t y = y0; y < y1; ++y) {
    // row y's window replaces row y - 4's, which row y - 1 still references:
    // every thread is past row y - 1 first (also for ltab and mask)
    __syncthreads();
    commit_row(y);
    if (y + 1 < y1) fetch_row(y + 1);
    // luma reference tables: window index of reference k for thread 0 of
    // (tile j, q); the window of row y - r holds column x at x - x0 + 3
    if (tid < 16) {
      for (uint32_t j = 0; j < ntr; ++j)
#pragma unroll
        for (int q = 0; q < CLS_PPT; ++q)
          ltab[j][q][tid] = ((y - (uint32_t)lk_rows) & 3u) * STRIP_RS +
                            (uint32_t)((int)(j * ENC_TILE + q * CLS_THREADS) + 3 - lk_px);
    }
    __syncthreads();
    // coded flags of the row's tiles
    uint32_t coded_bits = 0;
    unsigned long long wbal[2][CLS_PPT];
    const uint32_t* wy = win[y & 3];
    for (uint32_t j = 0; j < ntr; ++j) {
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) {
        const int c = (int)(j * ENC_TILE) + q * CLS_THREADS + tid;   // column in the strip
        const int64_t i = (int64_t)y * W + x0 + c;
        const bool coded = i == 0 || wy[c + 3] != wy[c + 2];
        const unsigned long long bal = __ballot(coded);
        wbal[j][q] = bal;
        if (lane == 0) {
          const int wb = (q * CLS_THREADS + (tid & ~63)) >> 5;
          mask[j][wb] = (uint32_t)bal;
          mask[j][wb + 1] = (uint32_t)(bal >> 32);
          if constexpr (MASK_OUT) {   // (frames: every tile is the block's)
            uint32_t* cm = a.cmask + ((uint64_t)f * T + (y * W + x0) / ENC_TILE + j) * (ENC_TILE / 32);
            cm[wb] = (uint32_t)bal;
            cm[wb + 1] = (uint32_t)(bal >> 32);
          }
        }
        coded_bits |= (coded ? 1u : 0u) << (2 * j + q);
      }
    }
    __syncthreads();
    for (uint32_t j = 0; j < ntr; ++j) {
      const uint32_t tt = (y * W + x0) / ENC_TILE + j;   // raster tile
      const bool in_band = tt >= a.tile_lo && tt < a.tile_hi;   // block-uniform
      const int64_t start = (int64_t)tt * ENC_TILE;
      if (in_band && (tid >> 6) == (int)j) {   // first / last coded pixel: wave j
        const uint32_t mw = lane < ENC_TILE / 32 ? mask[j][lane] : 0u;
        const unsigned long long nz = __ballot(mw != 0);
        if (lane == 0) {
          const uint64_t t = (uint64_t)f * T + tt;
          uint32_t first = NONE, last = NONE;
          if (nz) {
            const int fw = __builtin_ctzll(nz), lw = 63 - __builtin_clzll(nz);
            first = (uint32_t)(start + fw * 32 + __builtin_ctz(mask[j][fw]));
            last = (uint32_t)(start + lw * 32 + 31 - __builtin_clz(mask[j][lw]));
          }
          a.tile_first[t] = first;
          a.tile_last[t] = last;
        }
      }
      if (!in_band) continue;
      const bool fast = start >= 3 * (int64_t)W + 3;
      uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + start;
      uint32_t rec[CLS_PPT];
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) {
        const int p = q * CLS_THREADS + tid;
        const uint32_t cs = j * ENC_TILE + q * CLS_THREADS;   // strip column of thread 0
        const bool coded = (coded_bits >> (2 * j + q)) & 1u;
        const uint32_t* b0 = win[y & 3] + cs + tid;
        const uint32_t* b1 = win[(y - 1) & 3] + cs + tid;
        const uint32_t* b2 = win[(y - 2) & 3] + cs + 3 + tid;
        const uint32_t* b3 = win[(y - 3) & 3] + cs + tid;
        uint32_t rf;
        if (fast)
          rf = classify_y<false>(b0, b1, b2, b3, &win[0][0], (uint32_t)tid, W, 0u, ltab[j][q], cbr, csd, b0[3]);
        else
          rf = classify_y<true>(b0, b1, b2, b3, &win[0][0], (uint32_t)tid, W, (uint32_t)(start + p), ltab[j][q], cbr,
                                csd, b0[3]);
        rec[q] = coded ? rf : cunc;
      }
#pragma unroll
      for (int q = 0; q < CLS_PPT; ++q) {
        const int p = q * CLS_THREADS + tid;
        const bool coded = (coded_bits >> (2 * j + q)) & 1u;
        recs[p] = rec[q];
        slot_hist_add(hs, rec[q]);
        if constexpr (MASK_OUT) continue;   // enc_rundigits counts the run digits
        const bool next_coded = lane < 63 && ((wbal[j][q] >> (lane + 1)) & 1ull);
        if (coded && !next_coded) {
          const unsigned long long above = lane < 63 ? (wbal[j][q] >> (lane + 1)) : 0ull;
          const int nx = above ? p + 1 + (int)__builtin_ctzll(above) : next_coded_local(mask[j], p | 63);
          if (nx < ENC_TILE && nx > p + 1) {
            uint32_t mm = (uint32_t)(nx - p - 2);
            while (true) {
              atomicAdd(&run_hist[mm & 7u], 1u);
              if (mm < 8) break;
              mm >>= 3;
            }
          }
        }
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < N_BINS; k += CLS_THREADS) {
    uint32_t v = slot_hist_bin(hs, k);
    if (k >= BIN_PREFIX + P_RUN1 && k < BIN_PREFIX + P_RUN1 + 8) v += run_hist[k - BIN_PREFIX - P_RUN1];
    if (v) atomicAdd(&a.hist[(uint64_t)f * N_BINS + k], v);
  }
}
// ---------------------------------------------------------------------------
// K1w: classify with per-tile row windows (rows too wide for any ring and not
// whole tiles per strip row: RGBA with W > CLS_RING2_MAX_W and W % 1024 != 0,
// RGB with W > CLS_RING2_MAX_W).  Each block walks a contiguous tile range
// like the ring kernels; for each tile it stages four LINEAR windows,
// window r = pixels [start - rW - 3, start - rW + 1027) in Y space, so every
// reference of the tile's pixels (0..3 rows back, 3 pixels either side,
// wrapping across row ends as code.rs:141-145's linear offsets do) is inside
// the window of its row offset.  Rows above are read from HBM/L2 once per
// window (4 B/px more than the ring's single read); the next tile's windows
// load into registers while this one is classified.  The mode decision is the
// ring kernels' classify_y over explicit window bases.
// ---------------------------------------------------------------------------
constexpr int TW_RS = ENC_TILE + 8;                                         // window words
constexpr int TW_LD = (ENC_TILE + 6 + CLS_THREADS - 1) / CLS_THREADS;       // loads per window per thread (3)

template <int C, bool MASK_OUT>
__device__ __forceinline__ void enc_classify_twin_body(const EncArgs& a) {
  __shared__ uint32_t win[4][TW_RS];
  __shared__ uint32_t hs[C0_N + 2 * SX_N];
  __shared__ uint32_t run_hist[8];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t ltab[CLS_PPT][16];
  const uint64_t total_work = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  const uint64_t w_end = min(w_begin + a.tiles_per_block, total_work);
  if (w_begin >= w_end) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t cbr = (C0_BR << 3) | rec2_abs((uint32_t)lane), csd = (C0_SD << 3) | rec2_abs((uint32_t)lane);
  const uint32_t cunc = rec2_unc((uint32_t)lane);
  const uint32_t W = a.W;
  const int64_t N = (int64_t)W * a.H;
  for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
  if (tid < 8) run_hist[tid] = 0;
  // luma reference k of slot q's thread 0: window lr_rows(k), column q * 512 + 3 - lr_px(k)
  if (tid < 16 * CLS_PPT) {
    const int q = tid >> 4, k = tid & 15;
    ltab[q][k] = k < 11 ? (uint32_t)(lr_rows(k) * TW_RS + q * CLS_THREADS + 3 - lr_px(k)) : 0u;
  }
  auto flush = [&](uint32_t frame) {
    __syncthreads();
    for (int b = tid; b < N_BINS; b += CLS_THREADS) {
      uint32_t v = slot_hist_bin(hs, b);
      if (b >= BIN_PREFIX + P_RUN1 && b < BIN_PREFIX + P_RUN1 + 8) v += run_hist[b - BIN_PREFIX - P_RUN1];
      if (v) atomicAdd(&a.hist[(uint64_t)frame * N_BINS + b], v);
    }
    __syncthreads();
    for (int b = tid; b < (int)(C0_N + 2 * SX_N); b += CLS_THREADS) hs[b] = 0;
    if (tid < 8) run_hist[tid] = 0;
  };
  // the tile's four windows into registers (0 outside the frame / the band's pixel memory)
  uint32_t pw[4][TW_LD];
  auto fetch = [&](const TileIter& ti) {
    const uint8_t* fr = a.px + (uint64_t)ti.f * a.frame_stride;
    const int64_t start = (int64_t)ti.tt() * ENC_TILE;
    const int64_t lo = max((int64_t)0, a.px_lo), hi = min(N, a.px_hi);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < TW_LD; ++k) {
        const int c = tid + k * CLS_THREADS;
        const int64_t g = start - (int64_t)r * W - 3 + c;
        pw[r][k] = (c < ENC_TILE + 6 && g >= lo && g < hi) ? px_word<C>(fr, g) : 0u;
      }
  };
  TileIter it(a, w_begin), nx(a, w_begin);
  uint32_t cur_frame = it.f;
  fetch(nx);
  nx.step(1);
  for (uint64_t w = w_begin; w < w_end; ++w, it.step(1)) {
    const uint32_t f = it.f;
    if (f != cur_frame) {
      flush(cur_frame);
      cur_frame = f;
    }
    const int64_t start = (int64_t)it.tt() * ENC_TILE;
    const int count = (int)min((int64_t)ENC_TILE, N - start);
    __syncthreads();   // the previous tile's readers are done with the windows
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int k = 0; k < TW_LD; ++k) {
        const int c = tid + k * CLS_THREADS;
        if (c < ENC_TILE + 6) win[r][c] = y_from_rgba(pw[r][k]);
      }
    if (w + 1 < w_end) fetch(nx);
    nx.step(1);
    __syncthreads();
    // coded flags -> tile bitmask (a pixel is coded iff i == 0 or Y(i) != Y(i-1))
    uint32_t coded_bits = 0;
    unsigned long long wbal[CLS_PPT];
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const int64_t i = start + p;
      const bool coded = p < count && (i == 0 || win[0][p + 3] != win[0][p + 2]);
      const unsigned long long bal = __ballot(coded);
      wbal[q] = bal;
      if (lane == 0) {
        const int wb = (q * CLS_THREADS + (tid & ~63)) >> 5;
        mask[wb] = (uint32_t)bal;
        mask[wb + 1] = (uint32_t)(bal >> 32);
        if constexpr (MASK_OUT) {
          uint32_t* cm = a.cmask + it.tile() * (ENC_TILE / 32);
          cm[wb] = (uint32_t)bal;
          cm[wb + 1] = (uint32_t)(bal >> 32);
        }
      }
      coded_bits |= (coded ? 1u : 0u) << q;
    }
    __syncthreads();
    if (tid < 64) {   // first / last coded pixel of the tile
      const uint32_t mw = tid < ENC_TILE / 32 ? mask[tid] : 0u;
      const unsigned long long nz = __ballot(mw != 0);
      if (tid == 0) {
        const uint64_t t = it.tile();
        uint32_t first = NONE, last = NONE;
        if (nz) {
          const int fw = __builtin_ctzll(nz), lw = 63 - __builtin_clzll(nz);
          first = (uint32_t)(start + fw * 32 + __builtin_ctz(mask[fw]));
          last = (uint32_t)(start + lw * 32 + 31 - __builtin_clz(mask[lw]));
        }
        a.tile_first[t] = first;
        a.tile_last[t] = last;
      }
    }
    const bool fast = start >= 3 * (int64_t)W + 3;
    uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + start;
    uint32_t rec[CLS_PPT];
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      const uint32_t* b0 = &win[0][p];
      const uint32_t* b1 = &win[1][p];
      const uint32_t* b2 = &win[2][p + 3];
      const uint32_t* b3 = &win[3][p];
      uint32_t rf;
      if (fast)   // block-uniform
        rf = classify_y<false>(b0, b1, b2, b3, &win[0][0], (uint32_t)tid, W, 0u, ltab[q], cbr, csd, b0[3]);
      else
        rf = classify_y<true>(b0, b1, b2, b3, &win[0][0], (uint32_t)tid, W, (uint32_t)(start + p), nullptr, cbr,
                              csd, b0[3]);
      rec[q] = coded ? rf : cunc;
    }
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      if (p < count) recs[p] = rec[q];
      slot_hist_add(hs, rec[q]);
      if constexpr (MASK_OUT) continue;   // enc_rundigits counts them
      const bool next_coded = lane < 63 && ((wbal[q] >> (lane + 1)) & 1ull);
      if (coded && !next_coded) {
        const unsigned long long above = lane < 63 ? (wbal[q] >> (lane + 1)) : 0ull;
        const int nxp = above ? p + 1 + (int)__builtin_ctzll(above) : next_coded_local(mask, p | 63);
        if (nxp < count && nxp > p + 1) {
          uint32_t mm = (uint32_t)(nxp - p - 2);
          while (true) {
            atomicAdd(&run_hist[mm & 7u], 1u);
            if (mm < 8) break;
            mm >>= 3;
          }
        }
      }
    }
  }
  flush(cur_frame);
}
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_twin(EncArgs a) { enc_classify_twin_body<4, false>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_twin_m(EncArgs a) { enc_classify_twin_body<4, true>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_twin3(EncArgs a) { enc_classify_twin_body<3, false>(a); }
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_twin3_m(EncArgs a) { enc_classify_twin_body<3, true>(a); }

__global__ __launch_bounds__(CLS_THREADS) void enc_classify_strip(EncArgs a) { enc_classify_strip_body<false>(a); }
// frames: the tiles' coded flags out, run digits by enc_rundigits
__global__ __launch_bounds__(CLS_THREADS) void enc_classify_strip_m(EncArgs a) { enc_classify_strip_body<true>(a); }

// ---------------------------------------------------------------------------
// K2: runs crossing tile ends. One block (1024 threads) per frame.
// tile_next[t] = first coded pixel after tile t (N if none).
// ---------------------------------------------------------------------------
// Aggregate of each group of ENC_GROUP_TILES tiles (grid: groups x frames).
__global__ __launch_bounds__(256) void enc_group_reduce(EncArgs a, int what) {
  __shared__ unsigned long long part[4];
  const uint32_t g = blockIdx.x, f = blockIdx.y;
  if (what == 1 && a.long_only && !(a.frame_flags[f] & FLAG_LONG)) return;   // bit totals: long path only
  const uint32_t nt = a.tile_hi - a.tile_lo;
  const uint32_t t0 = g * ENC_GROUP_TILES, t1 = min(t0 + ENC_GROUP_TILES, nt);
  const uint64_t base = (uint64_t)f * a.tiles_per_frame + a.tile_lo;
  unsigned long long v = what == 0 ? NONE : 0ull;
  for (uint32_t t = t0 + threadIdx.x; t < t1; t += 256) {
    if (what == 0) v = min(v, (unsigned long long)a.tile_first[base + t]);
    else v += a.tile_bits[base + t];
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long w = __shfl_xor(v, o);
    v = what == 0 ? min(v, w) : v + w;
  }
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long r = part[0];
    for (int k = 1; k < 4; ++k) r = what == 0 ? min(r, part[k]) : r + part[k];
    a.gacc[(uint64_t)f * a.groups + g] = r;
  }
}

constexpr int TR_THREADS = 1024;
__global__ __launch_bounds__(TR_THREADS) void enc_tailruns(EncArgs a) {
  __shared__ uint32_t chunk_min[TR_THREADS];
  __shared__ uint32_t digits[8];   // run-digit counts, added to the histogram once
  if (threadIdx.x < 8) digits[threadIdx.x] = 0;
  // block (group g, frame f): tiles [g, g + 1) x ENC_GROUP_TILES of the band
  const uint32_t g = blockIdx.x, f = blockIdx.y;
  const uint32_t T = a.tiles_per_frame;
  const uint32_t ntb = a.tile_hi - a.tile_lo;
  const uint32_t g0 = g * ENC_GROUP_TILES;
  const uint64_t base = (uint64_t)f * T + a.tile_lo + g0;
  const uint32_t nt = min(ntb - g0, ENC_GROUP_TILES);
  const uint32_t N = a.W * a.H;
  // the first coded pixel after the group: later groups, then after the band
  // (frames: none)
  uint32_t after = a.band ? (a.band_next_dev ? *a.band_next_dev : (uint32_t)a.band_next) : NONE;
  for (uint32_t k = g + 1; k < a.groups; ++k) after = min(after, (uint32_t)a.gacc[(uint64_t)f * a.groups + k]);
  const uint32_t per = (nt + TR_THREADS - 1) / TR_THREADS;
  const uint32_t c0 = threadIdx.x * per;
  const uint32_t c1 = min(c0 + per, nt);
  uint32_t m = NONE;
#pragma unroll 8
  for (uint32_t t = c0; t < c1; ++t) m = min(m, a.tile_first[base + t]);
  chunk_min[threadIdx.x] = m;
  __syncthreads();
  // inclusive suffix-min over chunks (Hillis-Steele, 10 steps)
  for (int d = 1; d < TR_THREADS; d <<= 1) {
    uint32_t v = chunk_min[threadIdx.x];
    if (threadIdx.x + d < TR_THREADS) v = min(v, chunk_min[threadIdx.x + d]);
    __syncthreads();
    chunk_min[threadIdx.x] = v;
    __syncthreads();
  }
  uint32_t nxt = min((threadIdx.x + 1 < TR_THREADS) ? chunk_min[threadIdx.x + 1] : NONE, after);
#pragma unroll 8
  for (int64_t t = (int64_t)c1 - 1; t >= (int64_t)c0; --t) {
    const uint32_t next_px = (nxt == NONE) ? N : nxt;
    a.tile_next[base + t] = next_px;
    const uint32_t last = a.tile_last[base + t];
    if (last != NONE) {
      const uint64_t run = (uint64_t)next_px - last - 1;
      if (run > 0) {
        uint64_t mm = run - 1;
        while (true) {
          atomicAdd(&digits[mm & 7u], 1u);
          if (mm < 8) break;
          mm >>= 3;
        }
      }
    }
    nxt = min(nxt, a.tile_first[base + t]);
  }
  __syncthreads();
  if (threadIdx.x < 8 && digits[threadIdx.x])
    atomicAdd(&a.hist[(uint64_t)f * N_BINS + BIN_PREFIX + P_RUN1 + threadIdx.x], digits[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// K3: code lengths + canonical codes, one 64-lane wave per (frame, stream).
// table entry: code in bits [5, 31), length in bits [0, 5) when length <= 25;
// the full u8 length is also kept for the header (len8).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void enc_tables(EncArgs a) {
  __shared__ HeapLds h;
  __shared__ uint32_t counts[MAX_ALPHABET];
  // stream-major, largest alphabets first (343, 256, 64, 64, 32 x 3, 13, 11,
  // 11 symbols): the long heap replays start in the first wave of blocks
  // instead of behind the short ones (a batch's blocks do not all fit at once)
  const uint32_t nf = gridDim.x / N_STREAMS;
  constexpr uint64_t ORDER = 5ull | 0ull << 4 | 2ull << 8 | 6ull << 12 | 3ull << 16 | 7ull << 20 | 8ull << 24 |
                             1ull << 28 | 4ull << 32 | 9ull << 36;
  const uint32_t f = blockIdx.x % nf;
  const int s = (int)((ORDER >> (4u * (blockIdx.x / nf))) & 15u);
  const int n = stream_size(s);
  const int sb = stream_base(s);
  const int lane = threadIdx.x;
  for (int i = lane; i < n; i += 64) counts[i] = a.hist[(uint64_t)f * N_BINS + sb + i];
  for (int i = lane; i < 2 * MAX_ALPHABET + 2; i += 64) h.parent[i] = -1;
  if (s == S_PREFIX) {   // the mode prefixes from their payload streams (every classify variant)
    __syncthreads();
    const uint32_t* hf = a.hist + (uint64_t)f * N_BINS;
    uint32_t c[5] = {0, 0, 0, 0, 0};
    for (int b = lane; b < N_BINS; b += 64) {
      const uint32_t v = hf[b];
#pragma unroll
      for (int k = 0; k < 5; ++k) c[k] += mode_id_bin(k, b) ? v : 0u;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      for (int o = 32; o > 0; o >>= 1) c[k] += (uint32_t)__shfl_xor((int)c[k], o);
      if (lane == k) counts[k] = c[k] / mode_id_syms(k);
    }
  }
  __syncthreads();
#ifdef NICE_PROF_TABLES
  const long long pt0 = clock64();
#endif
  huffman_merge_wave(h, counts, n);
  __syncthreads();
#ifdef NICE_PROF_TABLES
  const long long pt1 = clock64();
#endif
  // aob = 1 + number of merged ancestors (u8 wrapping, hfe.rs:79-82); the
  // lane's symbols' parent chains are walked together (independent loads)
  constexpr int SPL = (MAX_ALPHABET + 63) / 64;
  __shared__ uint32_t lvl_n[256], lvl_run[256];
  __shared__ unsigned long long lvl_cur[256];
  for (int b = lane; b < 256; b += 64) { lvl_n[b] = 0; lvl_run[b] = 0; }
  int pp[SPL];
  uint32_t ab[SPL];
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = lane + 64 * q;
    pp[q] = i < n ? h.parent[i] : -1;
    ab[q] = 1u;
  }
  while (true) {
    bool any = false;
#pragma unroll
    for (int q = 0; q < SPL; ++q) {
      if (pp[q] >= 0) {
        ++ab[q];
        pp[q] = h.parent[pp[q]];
        any = true;
      }
    }
    if (!__any(any)) break;
  }
  uint32_t my_max = 0, my_emit_max = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = lane + 64 * q;
    ab[q] &= 255u;
    if (i < n) {
      my_max = max(my_max, ab[q]);
      if (counts[i]) my_emit_max = max(my_emit_max, ab[q]);
      atomicAdd(&lvl_n[ab[q]], 1u);
    }
  }
  // canonical order (hfe.rs:264-270): lengths descending, then symbols
  // descending.  t = a symbol's place within its length = the symbols above it
  // with the same length: chunks of 64 from the top, one ballot per distinct
  // length in the chunk, running totals per length in LDS
  uint32_t t[SPL];
#pragma unroll
  for (int q = SPL - 1; q >= 0; --q) {
    const bool valid = lane + 64 * q < n;
    unsigned long long rem = __ballot(valid);
    t[q] = 0;
    while (rem) {
      const uint32_t av = (uint32_t)__builtin_amdgcn_readlane((int)ab[q], (int)__builtin_ctzll(rem));
      const bool mine = valid && ab[q] == av;
      const unsigned long long m = __ballot(mine);
      const uint32_t run = lvl_run[av];
      if (mine) t[q] = run + (uint32_t)__popcll(lane < 63 ? m >> (lane + 1) : 0ull);
      if (lane == 0) lvl_run[av] = run + (uint32_t)__popcll(m);
      rem &= ~m;
    }
  }
  // hfe.rs:271-290 (usize wrapping): the running code `cur` steps by one per
  // symbol within a length (not after a length-0 symbol: `prev > 0`) and is
  // shifted right by the length drop at each new length, so only its value at
  // each present length's first symbol is serial: one scalar pass over the
  // present lengths (ballots of the length histogram, bin a = lane a & 63 of
  // word a >> 6)
  __syncthreads();
  uint32_t ln_cnt[4];
  unsigned long long pres[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ln_cnt[r] = lvl_n[64 * r + lane];
    pres[r] = __ballot(ln_cnt[r] != 0);
  }
  {
    unsigned long long cur = 0;
    uint32_t prev = 0;
    bool first = true;
#pragma unroll
    for (int r = 3; r >= 0; --r) {
      unsigned long long pm = pres[r];
      while (pm) {
        const uint32_t l = 63u - (uint32_t)__clzll(pm);
        pm &= ~(1ull << l);
        const uint32_t av = 64u * r + l;
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)ln_cnt[r], (int)l);
        if (!first) cur = (cur >> ((prev - av) & 63u)) + 1ull;   // prev > av >= 0: the shift, then prev > 0
        first = false;
        if (lane == 0) lvl_cur[av] = cur;
        cur += av ? (unsigned long long)(c - 1u) : 0ull;
        prev = av;
      }
    }
  }
  __syncthreads();
#ifdef NICE_PROF_TABLES
  const long long pt2 = clock64();
#endif
#pragma unroll
  for (int q = 0; q < SPL; ++q) {
    const int i = lane + 64 * q;
    if (i < n) {
      const uint32_t av = ab[q];
      const unsigned long long cur = lvl_cur[av] + (av ? t[q] : 0u);
      const unsigned long long code = (1ull << (av & 63u)) - cur - 1ull;
      const uint64_t e = (uint64_t)f * N_BINS + sb + i;
      a.tbl_len8[e] = (uint8_t)av;
      a.tbl_code[e] = (uint32_t)code;
      a.tbl[e] = (av <= FAST_MAX_CODE_BITS) ? (uint32_t)((code << 5) | av) : 0u;
    }
  }
  // wave max
  for (int o = 32; o > 0; o >>= 1) {
    my_max = max(my_max, (uint32_t)__shfl_xor((int)my_max, o));
    my_emit_max = max(my_emit_max, (uint32_t)__shfl_xor((int)my_emit_max, o));
  }
  if (lane == 0) {
    a.stream_max[(uint64_t)f * N_STREAMS + s] = (uint8_t)my_max;
#ifdef NICE_PROF_TABLES
    const long long pt3 = clock64();
    if (f == 0) printf("enc_tables stream %d n %d: merge %lld depth+rank %lld canon %lld cycles; wall %lld\n", s, n,
                       pt1 - pt0, pt2 - pt1, pt3 - pt2, (long long)wall_clock64());
#endif
    if (my_emit_max > FAST_MAX_CODE_BITS) {
      atomicOr(&a.frame_flags[f], FLAG_LONG);
      atomicOr(&a.frame_flags[a.n_frames], FLAG_LONG);   // any frame of the batch
    }
  }
}

// Test hook (nice_test_code_lengths): code lengths of n_vec count vectors of
// n symbols, one wave each, through the same heap replay as enc_tables.
__global__ __launch_bounds__(64) void enc_code_lengths_test(const uint32_t* counts, int n, uint8_t* aob) {
  __shared__ HeapLds h;
  __shared__ uint32_t c[MAX_ALPHABET];
  const uint32_t v = blockIdx.x;
  for (int i = threadIdx.x; i < n; i += 64) c[i] = counts[(uint64_t)v * n + i];
  for (int i = threadIdx.x; i < 2 * MAX_ALPHABET + 2; i += 64) h.parent[i] = -1;
  __syncthreads();
  huffman_merge_wave(h, c, n);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 64) {
    uint32_t depth = 0;
    for (int p = h.parent[i]; p >= 0; p = h.parent[p]) ++depth;
    aob[(uint64_t)v * n + i] = (uint8_t)(1u + depth);
  }
}

// ---------------------------------------------------------------------------
// Exact replica of the reference Bitwriter (bitwriter.rs:17-73) for one lane,
// writing bytes to global memory.
// ---------------------------------------------------------------------------
struct DevBitwriter {
  uint8_t* out;
  uint64_t pos;   // bytes written
  uint8_t bit_offset;
  uint32_t cache;
  __device__ void write_8bits(uint8_t amount, uint8_t value) {
    bit_offset = (uint8_t)(bit_offset + amount);
    cache += ((uint32_t)value) << (((uint8_t)(32 - bit_offset)) & 31u);
    if (bit_offset >= 8) {
      out[pos++] = (uint8_t)(cache >> 24);
      bit_offset = (uint8_t)(bit_offset - 8);
      cache <<= 8;
    }
  }
  __device__ void write_24bits(uint8_t amount, uint32_t value) {
    bit_offset = (uint8_t)(bit_offset + amount);
    cache += value << (((uint8_t)(32 - bit_offset)) & 31u);
    while (bit_offset >= 8) {
      out[pos++] = (uint8_t)(cache >> 24);
      bit_offset = (uint8_t)(bit_offset - 8);
      cache <<= 8;
    }
  }
};

__device__ __forceinline__ uint8_t field_bits(uint8_t max_aob) {
  // u8::next_power_of_two().count_zeros() in release mode (hfe.rs:102)
  uint32_t np;
  if (max_aob <= 1) np = 1;
  else if (max_aob > 128) np = 0;
  else np = 1u << (32 - __builtin_clz((uint32_t)max_aob - 1u));
  return (uint8_t)(8 - __builtin_popcount(np));
}

// ---------------------------------------------------------------------------
// K4: headers. One wave per frame. Writes bytes [0, 4*floor(data_start/32)) and
// the frame's seed (data start bit, last 32 bits before it).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void enc_header(EncArgs a) {
  __shared__ uint32_t words[200];   // 6160 bits = 192.5 words in the normal layout
  const uint32_t f = blockIdx.x;
  const int lane = threadIdx.x;
  uint8_t* out = a.out + (uint64_t)f * a.out_stride;
  const uint8_t* smax = a.stream_max + (uint64_t)f * N_STREAMS;
  bool normal = true;
  for (int s = 0; s < N_STREAMS; ++s) normal &= smax[s] <= 31;
  const uint64_t N = (uint64_t)a.W * a.H;

  if (normal && N > 0) {
    // Every field sits at a fixed bit offset: assemble 32-bit MSB-first words.
    for (int w = lane; w < 200; w += 64) words[w] = 0;
    __syncthreads();
    if (lane == 0) {
      words[0] = ('n' << 24) | ('i' << 16) | ('c' << 8) | 'e';
      words[1] = a.W;
      words[2] = a.H;
    }
    __syncthreads();
    if (lane == 0) atomicOr(&words[3], (uint32_t)a.channels_out << 24);
    // field list: for stream s: 5-bit max at bit pos, then n x 7-bit lengths
    uint32_t pos = 104;
    for (int s = 0; s < N_STREAMS; ++s) {
      const int n = stream_size(s);
      if (lane == 0) {
        const uint32_t v = smax[s], p = pos;
        const uint32_t w = p >> 5, o = p & 31;
        if (o + 5 <= 32) atomicOr(&words[w], v << (32 - o - 5));
        else { atomicOr(&words[w], v >> (o + 5 - 32)); atomicOr(&words[w + 1], v << (64 - o - 5)); }
      }
      pos += 5;
      for (int i = lane; i < n; i += 64) {
        const uint32_t v = a.tbl_len8[(uint64_t)f * N_BINS + stream_base(s) + i];
        const uint32_t p = pos + 7u * i;
        const uint32_t w = p >> 5, o = p & 31;
        if (o + 7 <= 32) atomicOr(&words[w], v << (32 - o - 7));
        else { atomicOr(&words[w], v >> (o + 7 - 32)); atomicOr(&words[w + 1], v << (64 - o - 7)); }
      }
      pos += 7u * n;
    }
    __syncthreads();
    // pos == 104 + 6056 = 6160; write words [0, 193): the last one partial,
    // zero past the header (the first data tile ORs into it)
    const uint32_t nwords = (pos + 31) >> 5;
    for (int w = lane; w < (int)nwords; w += 64)
      reinterpret_cast<uint32_t*>(out)[w] = __builtin_bswap32(words[w]);
    if (lane == 0) {
      a.seed_bit[f] = pos;
      // last 32 bits before pos: bits [pos-32, pos)
      const uint32_t o = pos & 31;
      const uint32_t hi = words[(pos >> 5) - 1], lo = words[pos >> 5];
      a.seed_suf[f] = o ? ((hi << o) | (lo >> (32 - o))) : hi;
    }
    return;
  }
  if (lane != 0) return;
  // Serial exact path (spilled 5-bit fields, 8-bit fields, empty frames).
  for (int k = 0; k < 4; ++k) out[k] = "nice"[k];
  for (int k = 0; k < 4; ++k) out[4 + k] = (uint8_t)(a.W >> (24 - 8 * k));
  for (int k = 0; k < 4; ++k) out[8 + k] = (uint8_t)(a.H >> (24 - 8 * k));
  out[12] = a.channels_out;
  DevBitwriter bw{out, 13, 0, 0};
  for (int s = 0; s < N_STREAMS; ++s) {
    const uint8_t mx = smax[s];
    bw.write_8bits(5, mx);
    const uint8_t fb = field_bits(mx);
    for (int i = 0; i < stream_size(s); ++i)
      bw.write_8bits(fb, a.tbl_len8[(uint64_t)f * N_BINS + stream_base(s) + i]);
  }
  a.hdr_bytes[f] = bw.pos;
  a.hdr_cache[f] = bw.cache;
  a.hdr_bitoff[f] = bw.bit_offset;
  const uint64_t pos = bw.pos * 8 + bw.bit_offset;
  a.seed_bit[f] = pos;
  // last 32 bits before pos
  uint64_t acc = 0;
  for (int k = 4; k >= 1; --k) acc = (acc << 8) | (bw.pos >= (uint64_t)k ? out[bw.pos - k] : 0);
  uint32_t suf = (uint32_t)acc;
  if (bw.bit_offset) suf = (suf << bw.bit_offset) | (bw.cache >> (32 - bw.bit_offset));
  a.seed_suf[f] = suf;
  if (N > 0) {
    // pending bits (top bit_offset bits of the cache), then zeros to the end of
    // the word holding the data start: the first data tile ORs into it
    const uint64_t wend = ((pos >> 5) + 1) * 4;
    out[bw.pos] = bw.bit_offset ? (uint8_t)((bw.cache >> 24) & (0xFFu << (8 - bw.bit_offset))) : 0u;
    for (uint64_t q = bw.pos + 1; q < wend; ++q) out[q] = 0;
  }
  if (N == 0) {
    // no data symbols: tail only (hfe.rs:115, code.rs:421-422)
    const uint8_t P = (uint8_t)(bw.cache >> 24);
    uint64_t p = bw.pos;
    out[p++] = P;
    out[p++] = (uint8_t)(bw.cache >> 24);
    out[p++] = (uint8_t)(bw.cache >> 16);
    out[p++] = (uint8_t)(bw.cache >> 8);
    out[p++] = (uint8_t)(bw.cache);
    a.out_len[f] = p;
  }
}

// ---------------------------------------------------------------------------
// K5-K7: bit placement.
//   enc_packtab   per frame: the packer's code tables (nice_rec.hpp PackTab):
//                 each record slot -> {code, length}, T0 with the mode prefix
//                 composed in front, run digits composed per run length;
//                 FLAG_LONG for frames an entry of which exceeds 32 bits
//   enc_pack      per tile, one pass: the pixels' codes from three lookups
//                 each, a block scan of their lengths, the tile's stream
//                 offset by a decoupled look-back over the preceding tiles'
//                 status words (pack_mode 0; bands: from enc_tilescan,
//                 pack_mode 1), codes MSB-first into an LDS bit buffer
//                 (bitwriter.rs:55-73), then shifted to the offset and stored
//   enc_edges     ORs each tile's first partial word into the word the tile
//                 before it (or the header) wrote
//   enc_tail      per frame: [P, P, 0, 0, 0] after the data (hfe.rs:115,
//                 code.rs:421-422) and the stream length
// FLAG_LONG frames (a code over FAST_MAX_CODE_BITS, or a composed entry over
// 32 bits) take enc_tilebits -> enc_tilescan -> enc_pack_long instead.
// A thread owns 4 consecutive pixels and reads their records with one 16-byte
// load.
// ---------------------------------------------------------------------------
// LDS bit buffer: <= NICE_PACK_CAP_BPP bits per pixel on average over a group
// (denser groups go to enc_pack_over)
constexpr int PACK_CAP_BITS = PACK_SUB * ENC_TILE * NICE_PACK_CAP_BPP;
constexpr int PACK_MAX_WORDS = PACK_CAP_BITS / 32 + 2;
constexpr int PK_THREADS = 256;

struct TileQuad {
  uint32_t rc[4];
  uint32_t nib;        // coded flags of the 4 pixels
};

// The thread's 4 records of tile tt of frame f (run members past the frame end).
__device__ __forceinline__ void quad_fetch(const EncArgs& a, uint32_t f, uint32_t tt, int p0, uint32_t (&rc)[4]) {
  const int64_t N = (int64_t)a.W * a.H;
  const int64_t start = (int64_t)tt * ENC_TILE;
  const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
  const uint32_t* rp = a.recs + (uint64_t)f * a.rec_stride + start + p0;
  if (p0 + 3 < count) {
    const uint4 v = *reinterpret_cast<const uint4*>(rp);
    rc[0] = v.x; rc[1] = v.y; rc[2] = v.z; rc[3] = v.w;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) rc[q] = (p0 + q < count) ? rp[q] : rec2_unc(0);
  }
}

// The tile's coded mask from the records (LDS, needs a barrier before use).
__device__ __forceinline__ void quad_mask(const uint32_t (&rc)[4], int lane, int wid, uint32_t* mask,
                                          TileQuad& Q) {
#pragma unroll
  for (int q = 0; q < 4; ++q) Q.rc[q] = rc[q];
  Q.nib = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) Q.nib |= (rec2_coded(Q.rc[q]) ? 1u : 0u) << q;
  const uint32_t mw = wave_or8(Q.nib << (4 * (lane & 7)));
  if ((lane & 7) == 0) mask[wid * 8 + (lane >> 3)] = mw;
}

// Run after each of the thread's 4 pixels (0 for run members): the next coded
// pixel in the thread's quad, else in the tile (mask), else tile_next.  Pixel
// indices are < 2^30 (the boundary's frame cap): 32-bit arithmetic.
__device__ __forceinline__ void quad_runs(const uint32_t* mask, int64_t start, int count, int p0,
                                          uint32_t next_tile_px, const TileQuad& Q, uint32_t (&run)[4]) {
  const int nx_local = next_coded_local(mask, p0 + 3);
  const uint32_t s32 = (uint32_t)start + (uint32_t)p0;
  const uint32_t after = (nx_local < count) ? (uint32_t)start + (uint32_t)nx_local : next_tile_px;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t later = Q.nib >> (q + 1);
    const uint32_t nxt = later ? s32 + (uint32_t)(q + 1) + (uint32_t)__builtin_ctz(later) : after;
    run[q] = ((Q.nib >> q) & 1u) ? nxt - (s32 + (uint32_t)q) - 1u : 0u;
  }
}

__device__ __forceinline__ void load_lens(uint32_t* lens, const EncArgs& a, uint32_t f) {
  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) lens[b] = a.tbl_len8[(uint64_t)f * N_BINS + b];
}

// Bits of the thread's 4 pixels (prefix, payload, run digits) from full code
// lengths (any length).
__device__ __forceinline__ uint32_t quad_nbits(const uint32_t* lens, const uint32_t* mask, int64_t start, int count,
                                               int p0, uint32_t next_tile_px, const TileQuad& Q) {
  uint32_t run[4];
  quad_runs(mask, start, count, p0, next_tile_px, Q, run);
  uint32_t nb = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t b[5];
    const uint32_t n = rec2_syms(Q.rc[q], b);
    for (uint32_t k = 0; k < n; ++k) nb += lens[b[k]];
    if (run[q] > 0) {
      uint32_t m = run[q] - 1;
      while (true) {
        nb += lens[BIN_PREFIX + P_RUN1 + (m & 7u)];
        if (m < 8) break;
        m >>= 3;
      }
    }
  }
  return nb;
}

// Contiguous tile ranges per block (the code table is reloaded only when the
// frame changes).  Work items w in [w0, w1): frame w / nt, band tile tile_lo + w % nt.
__device__ __forceinline__ void tile_range(const EncArgs& a, uint64_t& w0, uint64_t& w1) {
  const uint64_t total = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
  w0 = (uint64_t)blockIdx.x * per;
  w1 = w0 + per < total ? w0 + per : total;
}

// frames the long-code path handles: all (bands), or those with FLAG_LONG
__device__ __forceinline__ bool long_path(const EncArgs& a, uint32_t f) {
  return (!a.long_only || (a.frame_flags[f] & FLAG_LONG)) && !(a.frame_flags[f] & FLAG_BAD);
}

__global__ __launch_bounds__(ENC_THREADS) void enc_tilebits(EncArgs a) {
  __shared__ uint32_t tbl[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t wsum[ENC_THREADS / 64];
  if (a.long_only && !(a.frame_flags[a.n_frames] & FLAG_LONG)) return;   // no long-code frame in the batch
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * threadIdx.x;
  uint32_t cur_f = 0xFFFFFFFFu;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  TileIter it(a, t0);
  for (uint64_t w = t0; w < t1; ++w, it.step(1)) {
    const uint64_t t = it.tile();
    const uint32_t f = it.f, tt = it.tt();
    if (!long_path(a, f)) continue;   // block-uniform
    uint32_t rc[4];
    quad_fetch(a, f, tt, p0, rc);
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    __syncthreads();
    if (f != cur_f) { load_lens(tbl, a, f); cur_f = f; }
    TileQuad Q;
    quad_mask(rc, lane, wid, mask, Q);
    __syncthreads();
    uint32_t x = quad_nbits(tbl, mask, start, count, p0, a.tile_next[t], Q);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) a.tile_bits[t] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  }
}

// One 1024-thread block per frame.
// block (group g, frame f): tiles [g, g + 1) x ENC_GROUP_TILES of the band,
// from the bits of the earlier groups on
__global__ __launch_bounds__(1024) void enc_tilescan(EncArgs a) {
  __shared__ unsigned long long part[1024];
  const uint32_t g = blockIdx.x, f = blockIdx.y;
  if (!long_path(a, f)) return;
  const uint32_t g0 = g * ENC_GROUP_TILES;
  const uint32_t nt = min(a.tile_hi - a.tile_lo - g0, ENC_GROUP_TILES);
  const uint64_t base = (uint64_t)f * a.tiles_per_frame + a.tile_lo + g0;
  unsigned long long before = 0;
  for (uint32_t k = 0; k < g; ++k) before += a.gacc[(uint64_t)f * a.groups + k];
  const uint32_t per = (nt + 1023) / 1024;
  const uint32_t c0 = threadIdx.x * per, c1 = min(c0 + per, nt);
  unsigned long long sum = 0;
#pragma unroll 8
  for (uint32_t t = c0; t < c1; ++t) sum += a.tile_bits[base + t];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const unsigned long long v = (int)threadIdx.x >= d ? part[threadIdx.x - d] : 0ull;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  // frames: data starts after the header, whose last word is already zero
  // padded; bands: at band_bit0, and every partial word is shared (zeroed)
  const uint64_t seed = a.band ? a.band_bit0 : a.seed_bit[f];
  const int64_t seed_word = a.band ? (int64_t)(seed >> 5) - 1 : (int64_t)(seed >> 5);
  uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out + (uint64_t)f * a.out_stride);
  unsigned long long run = seed + before + (threadIdx.x ? part[threadIdx.x - 1] : 0ull);
#pragma unroll 8
  for (uint32_t t = c0; t < c1; ++t) {
    a.tile_off[base + t] = run;
    // a word shared with the previous tile (or the header: pre-padded with zeros)
    if ((run & 31) && (int64_t)(run >> 5) > seed_word) out32[run >> 5] = 0u;
    run += a.tile_bits[base + t];
  }
  if (threadIdx.x == 1023 && g + 1 == a.groups) {
    const uint64_t end = seed + before + part[1023];
    a.data_end[f] = end;
    if ((end & 31) && (int64_t)(end >> 5) > seed_word) out32[end >> 5] = 0u;
  }
}

// The packer's tables of frame f (nice_rec.hpp).  An entry composes the codes
// of its symbols in emission order; entries whose symbols all occur in the
// frame must fit 32 bits with every code <= FAST_MAX_CODE_BITS, else the frame
// is FLAG_LONG (entries of absent symbols are never looked up).
__global__ __launch_bounds__(256) void enc_packtab(EncArgs a) {
  __shared__ uint32_t code[N_BINS];
  __shared__ uint8_t len[N_BINS], pres[N_BINS];
  __shared__ uint32_t s_long;
  const uint32_t f = blockIdx.x;
  if (a.frame_flags[f] & FLAG_LONG) return;
  const int tid = threadIdx.x;
  for (int b = tid; b < N_BINS; b += 256) {
    const uint64_t e = (uint64_t)f * N_BINS + b;
    code[b] = a.tbl_code[e];
    len[b] = a.tbl_len8[e];
    pres[b] = a.hist[e] != 0;
  }
  if (tid == 0) s_long = 0;
  __syncthreads();
  PackTab* out = reinterpret_cast<PackTab*>(a.packtab) + f;
  bool lng = false;
  // symbols b[k0 .. n) composed; presence from the payload symbols b[p0 .. n)
  auto ent = [&](const uint32_t* b, uint32_t k0, uint32_t n, uint32_t p0) -> uint2 {
    uint32_t L = 0, mx = 0;
    bool present = true;
    for (uint32_t k = k0; k < n; ++k) {
      L += len[b[k]];
      mx = max(mx, (uint32_t)len[b[k]]);
      if (k >= p0) present = present && pres[b[k]];
    }
    if (present && (L > 32u || mx > (uint32_t)FAST_MAX_CODE_BITS)) lng = true;
    if (L > 32u || mx > (uint32_t)FAST_MAX_CODE_BITS) return make_uint2(0u, 0u);
    uint64_t c = 0;
    for (uint32_t k = k0; k < n; ++k) c = (c << len[b[k]]) | code[b[k]];
    return make_uint2((uint32_t)c, L);
  };
  for (uint32_t e = tid; e < C0_N; e += 256) {
    uint32_t b[5];
    const uint32_t n = rec2_syms((e << 3) | rec2_abs(0), b);
    // T0: the prefix and c0's symbols (LUMA: k and g)
    out->t0[e] = n ? ent(b, 0, n == 5 ? 3u : 2u, 1) : make_uint2(0u, 0u);
  }
  for (uint32_t s = tid; s < SX_N; s += 256) {
    uint32_t b1 = 0, b2 = 0;
    const bool live = s < SX_ABS;
    if (s < SX_L2) { b1 = s; b2 = s; }
    else if (s < SX_LUMA) { b1 = BIN_LUMA2_R + (s - SX_L2); b2 = BIN_LUMA2_B + (s - SX_L2); }
    else { b1 = BIN_LUMA_OTHER + (s - SX_LUMA); b2 = b1; }
    out->t1[s] = live ? ent(&b1, 0, 1, 0) : make_uint2(0u, 0u);
    out->t2[s] = live ? ent(&b2, 0, 1, 0) : make_uint2(0u, 0u);
  }
  for (uint32_t m = tid; m < RC_N; m += 256) {
    uint32_t b[2];
    uint32_t n = 0;
    if (m < RC_TWO) {   // natural digits of m (code.rs:391-406)
      b[n++] = BIN_PREFIX + P_RUN1 + (m & 7u);
      if (m >= 8) b[n++] = BIN_PREFIX + P_RUN1 + (m >> 3);
    } else if (m < RC_NONE) {   // the first two digits of a run of >= 65
      b[n++] = BIN_PREFIX + P_RUN1 + ((m - RC_TWO) & 7u);
      b[n++] = BIN_PREFIX + P_RUN1 + ((m - RC_TWO) >> 3);
    }
    out->rc[m] = n ? ent(b, 0, n, 0) : make_uint2(0u, 0u);
  }
  if (lng) atomicOr(&s_long, 1u);
  __syncthreads();
  if (tid == 0 && s_long) {
    atomicOr(&a.frame_flags[f], FLAG_LONG);
    atomicOr(&a.frame_flags[a.n_frames], FLAG_LONG);
  }
}

// Tile status words of the decoupled look-back (pack_mode 0): the tile's bit
// count (ST_AGG) as soon as it is known, then its absolute end bit (ST_INCL).
constexpr unsigned long long ST_AGG = 1ull << 62, ST_INCL = 2ull << 62, ST_VAL = (1ull << 62) - 1;
__device__ __forceinline__ void st_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long st_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// One wave: publishes the tile's count, sums the counts of the tiles before
// it back to the nearest one whose end is known (or to the frame start,
// `base`), publishes its own end; returns the tile's start bit.  w: the tile's
// status index; k: the tiles before it in its frame.  Every tile waited on
// was claimed earlier by a running block, which never waits on a later one.
// agg_out: the count was published already (ST_AGG).
__device__ unsigned long long lookback(unsigned long long* st, uint32_t w, uint32_t k, unsigned long long base,
                                       uint32_t bits, int lane, bool agg_out = false) {
  if (k == 0) {
    if (lane == 0) st_store(&st[w], ST_INCL | (base + bits));
    return base;
  }
  if (lane == 0 && !agg_out) st_store(&st[w], ST_AGG | bits);
  unsigned long long excl = 0;
  uint32_t j = w - 1, rem = k;
  while (true) {
    const bool valid = (uint32_t)lane < rem;
    const unsigned long long v = valid ? st_load(&st[j - lane]) : 0ull;
    const uint32_t state = (uint32_t)(v >> 62);
    const unsigned long long inc = __ballot(valid && state == 2u);
    const unsigned long long notready = __ballot(valid && state == 0u);
    const int first = inc ? (int)__builtin_ctzll(inc) : 64;
    const unsigned long long need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if (notready & need) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    unsigned long long x = (valid && lane <= first) ? (v & ST_VAL) : 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    excl += x;
    if (inc) break;
    if (rem <= 64) { excl += base; break; }
    j -= 64;
    rem -= 64;
  }
  if (lane == 0) st_store(&st[w], ST_INCL | (excl + bits));
  return excl;
}

// Work distribution of enc_pack (wave 0 of a block; f = NONE: no work left).
// Per-frame tile counters: block b serves slot b % I (I = pack_slots <= 64):
// frames slot, slot + I, ..., each frame's tiles claimed in order, then any
// frame with tiles left (scanned 64 counters at a time).  A frame is worked
// by about G / I blocks at once, so a look-back rarely reaches past one
// 64-tile window; a tile is claimed only when its block is about to pack it
// (the next claim goes out once this tile's offset is published), so every
// tile a look-back waits on publishes its count within one tile's time.
// pre: the result of a claim on f already issued by the caller (NONE: none).
__device__ void pack_next(const EncArgs& a, uint32_t nt, uint32_t I, uint32_t slot, uint32_t& f, uint32_t& k,
                          uint32_t& seq, int lane, uint32_t pre = NONE) {
  const uint32_t F = a.n_frames;
  while (true) {
    if (f != NONE) {
      uint32_t kk = pre;
      if (pre == NONE) {
        if (lane == 0) kk = atomicAdd(&a.pack_ctr[f], 1u);
        kk = (uint32_t)__shfl((int)kk, 0);
      }
      pre = NONE;
      if (kk < nt) { k = kk; return; }
    }
    const uint32_t own = slot + seq * I;
    if (own < F) {
      ++seq;
      f = (a.frame_flags[own] & (FLAG_LONG | FLAG_BAD)) ? NONE : own;   // long frames: enc_pack_long
      continue;
    }
    f = NONE;
    for (uint32_t b0 = 0; b0 < F; b0 += 64) {
      const uint32_t g = b0 + (uint32_t)lane;
      const bool cand = g < F && !(a.frame_flags[g] & (FLAG_LONG | FLAG_BAD)) &&
                        __hip_atomic_load(&a.pack_ctr[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nt;
      const unsigned long long m = __ballot(cand);
      if (m) { f = b0 + (uint32_t)__builtin_ctzll(m); break; }
    }
    if (f == NONE) return;
  }
}

// The thread's 4 pixels of one tile: each pixel's codes (T0, T1, T2, run
// digits) composed into one value when they fit 32 bits, their bit count, the
// run digits past a long run's first two, and the thread's total.
struct QuadCodes {
  uint32_t v[4], tot[4], xm[4], ri[4], nb, tmax;
};
__device__ __forceinline__ uint2 pt_entry(const PackTab& tab, uint32_t r, int i) {
  // 8-byte entries at the record's field offsets (nice_rec.hpp: bits 3..13,
  // 14..22, 23..31)
  const char* tb = reinterpret_cast<const char*>(&tab);
  return i == 0 ? *reinterpret_cast<const uint2*>(tb + offsetof(PackTab, t0) + (r & 0x3FF8u))
       : i == 1 ? *reinterpret_cast<const uint2*>(tb + offsetof(PackTab, t1) + ((r >> 11) & 0xFF8u))
                : *reinterpret_cast<const uint2*>(tb + offsetof(PackTab, t2) + ((r >> 20) & 0xFF8u));
}
__device__ __forceinline__ void quad_codes(const PackTab& tab, const uint32_t* mask, int64_t start, int count, int p0,
                                           uint32_t next_tile_px, const TileQuad& Q, QuadCodes& C) {
  uint32_t run[4];
  quad_runs(mask, start, count, p0, next_tile_px, Q, run);
  C.nb = 0;
  C.tmax = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t r = Q.rc[q];
    const uint2 e0 = pt_entry(tab, r, 0), e1 = pt_entry(tab, r, 1), e2 = pt_entry(tab, r, 2);
    const uint32_t m = run[q] - 1u;
    C.ri[q] = run[q] == 0 ? RC_NONE : m < 64u ? m : RC_TWO + (m & 63u);
    const uint2 e3 = tab.rc[C.ri[q]];
    C.xm[q] = run[q] > 64u ? m >> 6 : 0u;
    C.tot[q] = e0.y + e1.y + e2.y + e3.y;
    // composed value, exact when tot <= 32 (shifts stay below 32 then)
    uint32_t v = e0.x;
    v = (v << (e1.y & 31u)) | e1.x;
    v = (v << (e2.y & 31u)) | e2.x;
    v = (v << (e3.y & 31u)) | e3.x;
    C.v[q] = v;
    C.tmax = max(C.tmax, C.tot[q]);
    C.nb += C.tot[q];
  }
  if (C.xm[0] | C.xm[1] | C.xm[2] | C.xm[3]) {   // run digits past a long run's first two (runs of >= 65)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      for (uint32_t xr = C.xm[q]; xr;) {
        C.nb += tab.rc[xr & 7u].y;
        if (xr < 8) break;
        xr >>= 3;
      }
    }
  }
}
// Every code of the thread's pixels, in order, through put(val, n) (n <= 32
// bits of val, 0 when n == 0): one put per pixel when every pixel of the wave
// fits 32 bits (the common case), else two (the entries read again), else one
// per entry.
template <class Put>
__device__ __forceinline__ void quad_emit(const PackTab& tab, const TileQuad& Q, const QuadCodes& C, Put&& put) {
  auto put_extra = [&](uint32_t xr) {
    while (true) {
      const uint2 d = tab.rc[xr & 7u];
      put(d.x, d.y);
      if (xr < 8) break;
      xr >>= 3;
    }
  };
  if (__all(C.tmax <= 32u)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      put(C.v[q], C.tot[q]);
      if (C.xm[q]) put_extra(C.xm[q]);
    }
  } else if (__all(C.tmax <= 64u)) {
    for (int q = 0; q < 4; ++q) {
      const uint2 e0 = pt_entry(tab, Q.rc[q], 0), e1 = pt_entry(tab, Q.rc[q], 1), e2 = pt_entry(tab, Q.rc[q], 2);
      const uint2 e3 = tab.rc[C.ri[q]];
      uint64_t v = e0.x;
      v = (v << e1.y) | e1.x;
      v = (v << e2.y) | e2.x;
      v = (v << e3.y) | e3.x;
      const bool two = C.tot[q] > 32u;
      put(two ? (uint32_t)(v >> 32) : 0u, two ? C.tot[q] - 32u : 0u);
      put((uint32_t)v, two ? 32u : C.tot[q]);
      if (C.xm[q]) put_extra(C.xm[q]);
    }
  } else {
    for (int q = 0; q < 4; ++q) {
      for (int i = 0; i < 3; ++i) {
        const uint2 e = pt_entry(tab, Q.rc[q], i);
        put(e.x, e.y);
      }
      const uint2 e3 = tab.rc[C.ri[q]];
      put(e3.x, e3.y);
      if (C.xm[q]) put_extra(C.xm[q]);
    }
  }
}

// One work item of enc_pack is PACK_SUB consecutive tiles of a frame (a
// "group"): one claim and one look-back per 4096 pixels.  Wave k of the block
// packs tile k of the group: lane L owns pixels 16L .. 16L + 15 of the tile
// (four 16-byte record loads), composes each pixel's codes into one value of
// <= 32 bits (T0, T1, T2, the first two run digits; a pixel with longer codes
// puts its entries one by one), and a wave prefix sum of the lanes' bit
// counts gives each lane's bit position in its tile.  The group's tile totals
// (one block barrier) place the tiles in the group's LDS bit buffer; each
// lane streams its pieces MSB-first through a 64-bit register window and ORs
// each completed word into the buffer once: about 6 LDS atomics per 16 pixels
// (round 3's per-4-pixel puts made two per pixel, and spent 45 % of the LDS
// cycles in bank conflicts) and two block barriers per group instead of three
// per tile.  A group of over pack_cap_bits bits (over 32 per pixel on average)
// is counted first and then OR-ed into the output directly, tile by tile.
constexpr int PW_PX = ENC_TILE / 64;   // pixels per lane: 16

struct LanePx {
  uint32_t v[PW_PX];     // composed codes (exact where the pixel's length <= 32)
  uint32_t tot4[PW_PX / 4];   // lengths (<= 128: 8 bits each, four per word)
  const uint32_t* rp;    // the lane's records (re-read for pixels over 32 bits)
  uint32_t cm;           // coded flags of the lane's pixels
  uint32_t after;        // first coded pixel after the lane (absolute)
  uint32_t s;            // the lane's first pixel (absolute)
  uint32_t nb, tmax, rmax;   // bits, longest pixel, longest run after a pixel
  __device__ __forceinline__ uint32_t tot(int q) const { return (tot4[q >> 2] >> (8 * (q & 3))) & 0xFFu; }
};

// run after pixel q of the lane (0 for run members)
__device__ __forceinline__ uint32_t lane_run(const LanePx& P, int q) {
  const uint32_t later = P.cm >> (q + 1);
  const uint32_t nxt = later ? P.s + (uint32_t)(q + 1) + (uint32_t)__builtin_ctz(later) : P.after;
  return ((P.cm >> q) & 1u) ? nxt - (P.s + (uint32_t)q) - 1u : 0u;
}
__device__ __forceinline__ uint32_t rc_index(uint32_t run) {
  const uint32_t m = run - 1u;
  return run == 0 ? RC_NONE : m < 64u ? m : RC_TWO + (m & 63u);
}

// The lane's 16 pixels of tile tt of frame f: each pixel's composed code and
// length, the lane's bit count.  Pixel indices are < 2^30 (the boundary's
// frame cap): 32-bit arithmetic.
// The lane's 16 records of tile tt of frame f (issued early: enc_pack loads the
// next group's records while it places the current one).
__device__ __forceinline__ void lane_recs(const EncArgs& a, uint32_t f, uint32_t tt, int lane, uint32_t (&rec)[PW_PX]) {
  const int64_t N = (int64_t)a.W * a.H;
  const int64_t start = (int64_t)tt * ENC_TILE;
  const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
  const int p0 = PW_PX * lane;
  const uint32_t* rp = a.recs + (uint64_t)f * a.rec_stride + start + p0;
  if (p0 + PW_PX <= count) {
#pragma unroll
    for (int q = 0; q < PW_PX / 4; ++q) {
      const uint4 r = reinterpret_cast<const uint4*>(rp)[q];
      rec[4 * q] = r.x; rec[4 * q + 1] = r.y; rec[4 * q + 2] = r.z; rec[4 * q + 3] = r.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < PW_PX; ++q) rec[q] = (p0 + q < count) ? rp[q] : rec2_unc(0);
  }
}
// cmw: the tile's coded-flag words in the standard order (enc_rundigits wrote
// them; 16 bits per lane) when the frame's classify produced them, else null
// (bands, the window kernels): then the flags come from the records.
__device__ __forceinline__ void lane_codes(const EncArgs& a, const PackTab& tab, uint32_t f, uint32_t tt,
                                           uint32_t next_tile_px, int lane, const uint32_t (&rec)[PW_PX], LanePx& P,
                                           const uint32_t* cmw) {
  const int64_t start = (int64_t)tt * ENC_TILE;
  const int p0 = PW_PX * lane;
  P.rp = a.recs + (uint64_t)f * a.rec_stride + start + p0;
  if (cmw) {   // one load instead of an extract, compare and insert per pixel
    P.cm = (cmw[lane >> 1] >> (16u * ((uint32_t)lane & 1u))) & 0xFFFFu;
  } else {
    P.cm = 0;
#pragma unroll
    for (int q = 0; q < PW_PX; ++q) P.cm |= (rec2_coded(rec[q]) ? 1u : 0u) << q;
  }
  // the first coded pixel after the lane: in the next lane with one, else after the tile
  const unsigned long long lanes = __ballot(P.cm != 0u);
  const unsigned long long later = lane < 63 ? lanes >> (lane + 1) : 0ull;
  const int nl = later ? lane + 1 + (int)__builtin_ctzll(later) : 64;
  const uint32_t first_local = P.cm ? (uint32_t)p0 + (uint32_t)__builtin_ctz(P.cm) : 0u;
  const uint32_t nf = (uint32_t)__shfl((int)first_local, nl & 63);
  P.s = (uint32_t)start + (uint32_t)p0;
  P.after = nl < 64 ? (uint32_t)start + nf : next_tile_px;
  P.nb = 0;
  P.tmax = 0;
  P.rmax = 0;
  // each pixel's run-code index, from the last pixel back: the next coded
  // pixel is carried in a register instead of a bit scan per pixel
  uint32_t rci[PW_PX];
  {
    uint32_t nx = P.after - P.s;   // lane-relative
#pragma unroll
    for (int q = PW_PX - 1; q >= 0; --q) {
      const uint32_t cqm = (uint32_t)__builtin_amdgcn_sbfe((int)P.cm, q, 1);   // coded: ~0
      const uint32_t run = (nx - (uint32_t)q - 1u) & cqm;
      rci[q] = rc_index(run);
      P.rmax = max(P.rmax, run);   // (a per-pixel flag bit cost three VALU)
      // one bit insert (the compiler turned the and-or form into a shift,
      // compare, select and and-or)
      asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(nx) : "v"(cqm), "I"(q), "v"(nx));
    }
  }
#pragma unroll
  for (int q = 0; q < PW_PX; ++q) {
    if ((q & 3) == 0) {
      P.tot4[q >> 2] = 0;
      __builtin_amdgcn_sched_barrier(0);   // four pixels' lookups in flight at a time (registers)
    }
    const uint32_t r = rec[q];
    const uint2 e0 = pt_entry(tab, r, 0), e1 = pt_entry(tab, r, 1), e2 = pt_entry(tab, r, 2);
    const uint2 e3 = tab.rc[rci[q]];
    const uint32_t t = e0.y + e1.y + e2.y + e3.y;
    uint32_t v = e0.x;   // exact when t <= 32 (shifts stay below 32 then)
    v = (v << (e1.y & 31u)) | e1.x;
    v = (v << (e2.y & 31u)) | e2.x;
    v = (v << (e3.y & 31u)) | e3.x;
    asm volatile("" : "+v"(v) : "v"(t));   // materialise the pixel's code now (no entries kept live)
    P.v[q] = v;
    P.tot4[q >> 2] |= t << (8 * (q & 3));
    P.tmax = max(P.tmax, t);
    P.nb += t;
  }
  if (P.rmax > 64u) {   // run digits past a long run's first two (runs of >= 65)
    for (int q = 0; q < PW_PX; ++q) {
      const uint32_t run = lane_run(P, q);
      if (run <= 64u) continue;
      for (uint32_t xr = (run - 1u) >> 6; xr;) {
        P.nb += tab.rc[xr & 7u].y;
        if (xr < 8) break;
        xr >>= 3;
      }
    }
  }
}

// The lane's codes MSB-first from bit `pos` of the group's LDS buffer
// (bitwriter.rs:55-73 placement): a 64-bit window of pending bits, each
// completed word OR-ed in once (the first and last are shared with the
// neighbouring lanes; the buffer is zero).
__device__ __forceinline__ void lane_emit(const PackTab& tab, const LanePx& P, uint32_t* bits, uint32_t pos) {
  unsigned long long acc = 0;
  uint32_t n = pos & 31u;
  uint32_t* wp = bits + (pos >> 5);
  auto put = [&](uint32_t val, uint32_t len) {   // len <= 32, val < 2^len
    acc = (acc << len) | val;
    n += len;
    if (n >= 32u) {
      // the completed word, acc >> (n - 32), as one funnel shift (32 <= n < 64);
      // the word pointer steps instead of an index scaled per flush
      atomicOr(wp, __builtin_amdgcn_alignbit((uint32_t)(acc >> 32), (uint32_t)acc, n));
      ++wp;
      n -= 32u;
    }
  };
  if (__all(P.tmax <= 32u && P.rmax <= 64u)) {
    // every pixel of the wave one composed value, no run past 64 pixels
#pragma unroll
    for (int q = 0; q < PW_PX; ++q) put(P.v[q], P.tot(q));
  } else {
    // entry by entry from the records again (each entry <= 32 bits: longer
    // ones make the frame FLAG_LONG), then a long run's further digits
    for (int q = 0; q < PW_PX; ++q) {
      if ((P.cm >> q) & 1u) {   // coded (P.cm has no bits past the frame's end)
        const uint32_t r = P.rp[q], run = lane_run(P, q);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const uint2 e = pt_entry(tab, r, i);
          put(e.x, e.y);
        }
        const uint2 e3 = tab.rc[rc_index(run)];
        put(e3.x, e3.y);
        if (run > 64u) {
          for (uint32_t xr = (run - 1u) >> 6;;) {
            const uint2 d = tab.rc[xr & 7u];
            put(d.x, d.y);
            if (xr < 8) break;
            xr >>= 3;
          }
        }
      }
    }
  }
  if (n) atomicOr(wp, (uint32_t)(acc << (32u - n)));
}

__global__ __launch_bounds__(PK_THREADS, PACK_BLOCKS_PER_CU) void enc_pack(EncArgs a) {
  __shared__ PackTab tab;
  __shared__ uint32_t bits[PACK_MAX_WORDS];
  __shared__ uint32_t wsum[PK_THREADS / 64];
  __shared__ uint32_t s_f, s_k;
  __shared__ unsigned long long s_off;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t nt = a.tile_hi - a.tile_lo;
  const uint32_t ng = (nt + PACK_SUB - 1) / PACK_SUB;   // groups per frame
  const uint32_t T = a.tiles_per_frame;
  const bool lookback_mode = a.pack_mode == 0;
  const uint32_t I = a.pack_slots, slot = blockIdx.x % a.pack_slots;
  uint32_t cf = NONE, ck = 0, seq = 0;   // wave 0's work cursor
#ifdef NICE_PACK_PROF
  long long pr[7] = {0, 0, 0, 0, 0, 0, 0}, pt = clock64(), pn = 0;
#define PROF_MARK(i) do { const long long c_ = clock64(); pr[i] += c_ - pt; pt = c_; } while (0)
#else
#define PROF_MARK(i) do {} while (0)
#endif
  if (wid == 0) {
    pack_next(a, ng, I, slot, cf, ck, seq, lane);
    if (lane == 0) { s_f = cf; s_k = ck; }
  }
  __syncthreads();
  uint32_t f = s_f, g = s_k;
  uint32_t cur_f = NONE, used_words = PACK_MAX_WORDS;
  uint32_t rec[PW_PX];    // the wave's tile records
  while (f != NONE) {
    const uint32_t k0 = g * PACK_SUB, nsub = min((uint32_t)PACK_SUB, nt - k0);
    const uint32_t tt0 = a.tile_lo + k0;
    const uint64_t t0 = (uint64_t)f * T + tt0;   // the group's first tile
    if (f != cur_f) {
      const uint4* src = reinterpret_cast<const uint4*>(a.packtab + (uint64_t)f * sizeof(PackTab));
      uint4* dst = reinterpret_cast<uint4*>(&tab);
      for (int i = tid; i < (int)(sizeof(PackTab) / 16); i += PK_THREADS) dst[i] = src[i];
      cur_f = f;
    }
    for (uint32_t i = tid; i < used_words; i += PK_THREADS) bits[i] = 0;
    __syncthreads();   // the frame's tables in LDS, the buffer clear
    PROF_MARK(0);
    // wave wid: tile tt0 + wid of the group
    LanePx P;
    uint32_t x = 0;
    const bool mine = (uint32_t)wid < nsub;   // wave-uniform
    if (mine) {
      lane_recs(a, f, tt0 + wid, lane, rec);
      lane_codes(a, tab, f, tt0 + wid, a.tile_next[(uint64_t)f * T + tt0 + wid], lane, rec, P,
                 a.cmask_std ? a.cmask + ((uint64_t)f * T + tt0 + wid) * (ENC_TILE / 32) : nullptr);
      x = wave_incl_scan(P.nb);
    }
    if (lane == 63) wsum[wid] = mine ? x : 0u;
    __syncthreads();
    uint32_t wbase = 0, gbits = 0;   // bits before this wave's tile, the group's bits
#pragma unroll
    for (int i = 0; i < PK_THREADS / 64; ++i) {
      const uint32_t ws = wsum[i];
      wbase += (i < wid) ? ws : 0u;
      gbits += ws;
    }
    // (waves ranked by their bits at priorities 3..0 for the puts: no
    // faster, r06zv_ab_pack_place.log)
    PROF_MARK(1);
    const bool over = gbits > a.pack_cap_bits;   // block-uniform
#ifndef NICE_PACK_LATE_AGG
    // the group's count goes out before the puts: the look-backs of the
    // groups after it wait on it (a look-back was ~40 % of a group's time)
    const bool agg_out = lookback_mode && g > 0;
    if (agg_out && tid == 0) st_store(&a.status[f * ng + g], ST_AGG | gbits);
#else
    const bool agg_out = false;
#endif
    if (!over && mine && P.nb) lane_emit(tab, P, bits, wbase + x - P.nb);
    PROF_MARK(2);
    if (wid == 0 && lookback_mode) {
      // the look-back first: the groups behind wait on its published prefix
      // (pack 8.12 -> 8.04 ms per 512 frames, profiles/r06zg_ab_prio.log)
      __builtin_amdgcn_s_setprio(3);
      const unsigned long long off = lookback(a.status, f * ng + g, g, a.band ? a.band_bit0 : a.seed_bit[f], gbits, lane,
                                              agg_out);
      if (lane == 0) s_off = off;
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    PROF_MARK(3);
    // place the group's bits at its stream offset
    const unsigned long long s0 = lookback_mode ? s_off : a.tile_off[t0], e0 = s0 + gbits;
    const uint32_t sh = (uint32_t)(s0 & 31);
    const uint64_t w0 = s0 >> 5;
    const uint32_t nw = gbits ? (uint32_t)(((e0 + 31) >> 5) - w0) : 0u;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out + (uint64_t)f * a.out_stride);
    if (!over) {
      for (uint32_t m = tid; m < nw; m += PK_THREADS) {
        const uint32_t hi = m ? bits[m - 1] : 0u;
        const uint32_t lo = bits[m];   // zero past the group's bits
        const uint32_t v = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
        if (lookback_mode) {
          // a word is stored by the group holding its first bit (zeros past
          // the group's end); this group's bits in the word holding its
          // start go to enc_edges
          if (m == 0 && sh) a.tile_bits[t0] = v;
          else out32[w0 + m] = __builtin_bswap32(v);
        } else {   // every partial word was zeroed by enc_tilescan
          const bool shared = (m == 0 && sh) || (m == nw - 1 && (e0 & 31));
          if (shared) atomicOr(&out32[w0 + m], __builtin_bswap32(v));
          else out32[w0 + m] = __builtin_bswap32(v);
        }
      }
    } else if (tid == 0) {
      // over the LDS buffer: listed for enc_pack_over (after this kernel, before enc_edges)
      const uint32_t k = atomicAdd(a.over_count, 1u);
      a.over_list[k] = make_uint2(f * ng + g, gbits);
    }
    if (lookback_mode && tid == 0) {
      a.tile_off[t0] = s0;
      if (over || !(nw && sh)) a.tile_bits[t0] = 0u;
      if (tt0 + nsub == T) a.data_end[f] = e0;
    }
    used_words = over ? 0u : nw + 1;   // an over-cap group writes nothing into the buffer
    PROF_MARK(4);
    // the next group: claimed only now, when this block can start it at once
    // (a group claimed earlier would keep the look-backs of the groups after
    // it waiting while its block finishes this one; claiming during the
    // placement, or loading the next group's records then, measured no
    // faster: r04e, r04n)
    if (wid == 0) {
      __builtin_amdgcn_s_setprio(3);   // (the block waits on the claim: pack 7.96 -> 7.90 ms, r06zo)
      pack_next(a, ng, I, slot, cf, ck, seq, lane);
      __builtin_amdgcn_s_setprio(0);
      if (lane == 0) { s_f = cf; s_k = ck; }
    }
    __syncthreads();
    f = s_f;
    g = s_k;
    PROF_MARK(5);
#ifdef NICE_PACK_PROF
    ++pn;
#endif
  }
#ifdef NICE_PACK_PROF
  if (tid == 0 && (blockIdx.x % 256) == 0)
    printf("enc_pack block %u: groups %lld cycles/group: wait+mask %lld codes+scan %lld puts %lld lookback %lld "
           "place %lld claim %lld\n", blockIdx.x, pn, pr[0] / max(pn, 1ll), pr[1] / max(pn, 1ll),
           pr[2] / max(pn, 1ll), pr[3] / max(pn, 1ll), pr[4] / max(pn, 1ll), pr[5] / max(pn, 1ll));
#endif
}

// Groups over enc_pack's LDS buffer (pack_cap_bits: over 32 bits per pixel on
// average), listed by enc_pack with their bit counts, once every group's
// offset is published: the words whose first bit is the group's are zeroed,
// then each code is OR-ed into place tile by tile (the word holding the
// group's first bit through tile_bits, for enc_edges).  Rare; kept out of
// enc_pack, whose registers it would otherwise take.
__global__ __launch_bounds__(PK_THREADS) void enc_pack_over(EncArgs a) {
  __shared__ PackTab tab;
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t wsum[PK_THREADS / 64];
  const uint32_t n_over = *a.over_count;
  if (blockIdx.x >= n_over) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t nt = a.tile_hi - a.tile_lo;
  const uint32_t ng = (nt + PACK_SUB - 1) / PACK_SUB;
  const uint32_t T = a.tiles_per_frame;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * tid;
  const bool lookback_mode = a.pack_mode == 0;
  uint32_t rc[4];
  for (uint32_t item = blockIdx.x; item < n_over; item += gridDim.x) {
    const uint2 it = a.over_list[item];
    const uint32_t f = it.x / ng, g = it.x % ng, gbits = it.y;
    const uint32_t k0 = g * PACK_SUB, nsub = min((uint32_t)PACK_SUB, nt - k0);
    const uint32_t tt0 = a.tile_lo + k0;
    const uint64_t t0 = (uint64_t)f * T + tt0;
    __syncthreads();   // the previous item's readers of tab
    {
      const uint4* src = reinterpret_cast<const uint4*>(a.packtab + (uint64_t)f * sizeof(PackTab));
      uint4* dst = reinterpret_cast<uint4*>(&tab);
      for (int i = tid; i < (int)(sizeof(PackTab) / 16); i += PK_THREADS) dst[i] = src[i];
    }
    const unsigned long long s0 = a.tile_off[t0], e0 = s0 + gbits;
    const uint32_t sh = (uint32_t)(s0 & 31);
    const uint64_t w0 = s0 >> 5;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out + (uint64_t)f * a.out_stride);
      // zero the words only this group writes (look-back: every word whose
      // first bit is the group's; bands: the interior ones, enc_tilescan
      // zeroed the partial ones), then OR each code into place, tile by tile
      const uint64_t z0 = (s0 + 31) >> 5, z1 = lookback_mode ? (e0 + 31) >> 5 : e0 >> 5;
      for (uint64_t m = z0 + tid; m < z1; m += PK_THREADS) out32[m] = 0u;
      if (lookback_mode && tid == 0) a.tile_bits[t0] = 0u;
      __threadfence();
      __syncthreads();
      auto or_word = [&](uint64_t wd, uint32_t v) {
        if (!v) return;
        if (lookback_mode && sh && wd == w0) atomicOr(&a.tile_bits[t0], v);
        else atomicOr(&out32[wd], __builtin_bswap32(v));
      };
      unsigned long long run = s0;
      for (uint32_t s = 0; s < nsub; ++s) {
        const uint32_t tt = tt0 + s;
        const int64_t start = (int64_t)tt * ENC_TILE;
        const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
        quad_fetch(a, f, tt, p0, rc);
        TileQuad Q;
        quad_mask(rc, lane, wid, mask, Q);
        __syncthreads();
        QuadCodes C;
        quad_codes(tab, mask, start, count, p0, a.tile_next[(uint64_t)f * T + tt], Q, C);
        const uint32_t x = wave_incl_scan(C.nb);
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
        uint32_t wbase = 0, sbits = 0;
#pragma unroll
        for (int i = 0; i < PK_THREADS / 64; ++i) {
          const uint32_t ws = wsum[i];
          wbase += (i < wid) ? ws : 0u;
          sbits += ws;
        }
        if (C.nb) {
          unsigned long long pp = run + wbase + x - C.nb;
          quad_emit(tab, Q, C, [&](uint32_t val, uint32_t n) {
            const uint32_t b = (uint32_t)(pp & 31u);
            const uint64_t v = (uint64_t)val << ((64u - b - n) & 63u);
            if (n) {
              or_word(pp >> 5, (uint32_t)(v >> 32));
              or_word((pp >> 5) + 1, (uint32_t)v);
            }
            pp += n;
          });
        }
        run += sbits;
        __syncthreads();
      }
  }
}

// Each group's bits in the word holding its first bit (pack_mode 0), OR-ed
// into that word once every group has stored its own words.
__global__ __launch_bounds__(256) void enc_edges(EncArgs a) {
  const uint32_t T = a.tiles_per_frame;
  const uint32_t ng = (a.tile_hi - a.tile_lo + PACK_SUB - 1) / PACK_SUB;   // groups of the frame (band)
  for (uint32_t f = blockIdx.y; f < a.n_frames; f += gridDim.y) {
    if (a.frame_flags[f] & (FLAG_LONG | FLAG_BAD)) continue;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out + (uint64_t)f * a.out_stride);
    for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < ng; g += gridDim.x * 256) {
      const uint64_t t = (uint64_t)f * T + a.tile_lo + (uint64_t)g * PACK_SUB;
      const uint32_t e = a.tile_bits[t];
      if (e) atomicOr(&out32[a.tile_off[t] >> 5], __builtin_bswap32(e));
    }
  }
}

__global__ __launch_bounds__(64) void enc_tail(EncArgs a) {
  const uint32_t f = blockIdx.x * 64 + threadIdx.x;
  if (f >= a.n_frames) return;
  if ((uint64_t)a.W * a.H == 0) return;
  uint8_t* out = a.out + (uint64_t)f * a.out_stride;
  const uint64_t e0 = a.data_end[f];
  const uint64_t B = e0 >> 3;            // the partial byte (the reference's cache >> 24)
  const uint8_t P = (e0 & 7) ? out[B] : 0u;
  out[B] = P;
  out[B + 1] = P;
  out[B + 2] = 0;
  out[B + 3] = 0;
  out[B + 4] = 0;
  a.out_len[f] = B + 5;
}

// ---------------------------------------------------------------------------
// K6: frames with codes over FAST_MAX_CODE_BITS (FLAG_LONG).
//
// A write of an n-bit code at absolute stream bit p behaves like the
// reference's write_24bits (bitwriter.rs:55-73) with bit_offset = p & 7
// (the writer flushes every whole byte, so bit_offset is always the position
// mod 8 once the table header is out):
//  * (p & 7) + n <= 32: the code lands exactly on bits [p, p + n);
//  * otherwise `32 - bit_offset` wraps (u8) and the shift is masked to 5 bits:
//    the 32-bit window at byte p >> 3 becomes window + (code << ((32 - (p & 7)
//    - n) & 31)) mod 2^32 -- carries into the pending bits of the codes before
//    it included -- and every bit after the window up to p + n is zero (the
//    flush loop shifts the cache out).
// Phase 0 places the codes of the first kind (global atomicOr after the tile
// zeroes the words only it writes; enc_tilescan zeroed the shared ones).
// Phase 1 re-derives every symbol's position and applies the wrapped writes to
// their windows, whose earlier bits phase 0 has finalised.  Wrapped windows
// are disjoint: a window ends before its code's end (p + n > window + 32),
// and the next code starts there.  In band mode a window that starts in the
// byte holding band_bit0 also covers (and may carry into) the previous band's
// last bits: at most one per band (n >= 26), so it is recorded in the band's
// two trailer words (band_fix) and applied by enc_band_fix after the bands are
// merged.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wrapped_write(uint8_t* out, uint64_t p, uint32_t v, uint32_t n) {
  const uint64_t B = p >> 3;
  const uint32_t bo = (uint32_t)(p & 7u);
  const uint32_t sh = (uint32_t)(uint8_t)(32u - (uint8_t)(bo + n)) & 31u;
  const uint32_t w = ((uint32_t)out[B] << 24) | ((uint32_t)out[B + 1] << 16) | ((uint32_t)out[B + 2] << 8) | out[B + 3];
  const uint32_t r = w + (v << sh);
  out[B] = (uint8_t)(r >> 24);
  out[B + 1] = (uint8_t)(r >> 16);
  out[B + 2] = (uint8_t)(r >> 8);
  out[B + 3] = (uint8_t)r;
}

__global__ __launch_bounds__(ENC_THREADS) void enc_pack_long(EncArgs a, int phase) {
  __shared__ uint32_t code[N_BINS];
  __shared__ uint32_t lens[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t wsum[ENC_THREADS / 64];
  if (!(a.frame_flags[a.n_frames] & FLAG_LONG)) return;   // no long-code frame in the batch
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * threadIdx.x;
  uint32_t cur_f = NONE;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  TileIter it(a, t0);
  for (uint64_t w = t0; w < t1; ++w, it.step(1)) {
    const uint32_t f = it.f, tt = it.tt();
    if ((a.frame_flags[f] & (FLAG_LONG | FLAG_BAD)) != FLAG_LONG) continue;   // block-uniform
    const uint64_t t = it.tile();
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    uint32_t rc[4];
    quad_fetch(a, f, tt, p0, rc);
    __syncthreads();
    if (f != cur_f) {
      for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) {
        code[b] = a.tbl_code[(uint64_t)f * N_BINS + b];
        lens[b] = a.tbl_len8[(uint64_t)f * N_BINS + b];
      }
      cur_f = f;
    }
    TileQuad Q;
    quad_mask(rc, lane, wid, mask, Q);
    __syncthreads();
    const uint32_t nb = quad_nbits(lens, mask, start, count, p0, a.tile_next[t], Q);
    const uint32_t x = wave_incl_scan(nb);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, tile_bits = 0;
#pragma unroll
    for (int k = 0; k < ENC_THREADS / 64; ++k) {
      const uint32_t ws = wsum[k];
      wbase += (k < wid) ? ws : 0u;
      tile_bits += ws;
    }
    const uint64_t s0 = a.tile_off[t];
    uint8_t* out = a.out + (uint64_t)f * a.out_stride;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
    if (phase == 0) {
      const uint64_t e0 = s0 + tile_bits, w0 = s0 >> 5;
      const uint32_t nw = tile_bits ? (uint32_t)(((e0 + 31) >> 5) - w0) : 0u;
      for (uint32_t m = threadIdx.x; m < nw; m += ENC_THREADS) {
        const bool shared = (m == 0 && (s0 & 31)) || (m == nw - 1 && (e0 & 31));
        if (!shared) out32[w0 + m] = 0u;
      }
      __threadfence();
      __syncthreads();
    }
    uint64_t pos = s0 + wbase + x - nb;
    auto emit = [&](uint32_t bin) {
      const uint32_t n = lens[bin], v = code[bin];
      const uint32_t bo = (uint32_t)(pos & 7u);
      if (bo + n <= 32u) {
        if (phase == 0 && n) {
          const uint32_t o = (uint32_t)(pos & 31u);
          const uint64_t y = (uint64_t)v << (64u - o - n);
          atomicOr(&out32[pos >> 5], __builtin_bswap32((uint32_t)(y >> 32)));
          if (o + n > 32u) atomicOr(&out32[(pos >> 5) + 1], __builtin_bswap32((uint32_t)y));
        }
      } else if (phase == 1) {
        if (a.band && (pos & ~7ull) < a.band_bit0) {   // window reaches the previous band: deferred
          a.band_fix[0] = BAND_FIX_WRITE | ((uint32_t)(pos - a.band_bit0) << 8) | n;
          a.band_fix[1] = v;
        } else {
          wrapped_write(out, pos, v, n);
        }
      }
      pos += n;
    };
    uint32_t run[4];
    quad_runs(mask, start, count, p0, a.tile_next[t], Q, run);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t b[5];
      const uint32_t n = rec2_syms(Q.rc[q], b);
      for (uint32_t k = 0; k < n; ++k) emit(b[k]);
      if (run[q] > 0) {
        uint32_t m = run[q] - 1;
        while (true) {
          emit(BIN_PREFIX + P_RUN1 + (m & 7u));
          if (m < 8) break;
          m >>= 3;
        }
      }
    }
  }
}

}  // namespace nice

namespace nice {

// ---------------------------------------------------------------------------
// Band assembly (one image sharded over ranks): OR the bands' word arrays into
// the stream (header words are already there, zero padded), then the tail.
// band_w0[r]: first stream word of band r; band_off[r]: its first word in the
// concatenated array; band_off[R]: total words.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_band_merge(uint32_t* out32, const uint32_t* words,
                                                      const unsigned long long* band_w0,
                                                      const unsigned long long* band_off, uint32_t R) {
  const uint32_t r = blockIdx.y;
  if (r >= R) return;
  const unsigned long long n = band_off[r + 1] - band_off[r];
  if (n < 3) return;
  const unsigned long long nd = n - 2;   // the last two words of a band are its trailer (enc_band_fix)
  const unsigned long long w0 = band_w0[r];
  const uint32_t* src = words + band_off[r];
  // 16 words per thread in flight: block b covers words [4096 b, 4096 (b + 1))
  constexpr int K = 16;
  const unsigned long long m0 = (unsigned long long)blockIdx.x * (256 * K) + threadIdx.x;
  if (m0 >= nd) return;
  uint32_t v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const unsigned long long m = m0 + 256ull * k;
    v[k] = m < nd ? src[m] : 0u;
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const unsigned long long m = m0 + 256ull * k;
    if (m >= nd) break;
    if (m == 0 || m + 1 == nd) atomicOr(&out32[w0 + m], v[k]);   // shared with a neighbour or the header
    else out32[w0 + m] = v[k];
  }
}

// The deferred wrapped writes, band by band (their windows are disjoint; each
// reads the merged bits of the band before it).  One thread: at most R writes.
__global__ void enc_band_fix(uint8_t* out, const uint32_t* words, const unsigned long long* band_bit0,
                             const unsigned long long* band_off, uint32_t R, unsigned long long* bad) {
  if (threadIdx.x != 0) return;
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t f = words[band_off[r + 1] - 2];
    if (f & BAND_FIX_BAD) *bad = 1;   // packed with a wrong band_bits (enc_band_check)
    else if (f & BAND_FIX_WRITE) wrapped_write(out, band_bit0[r] + ((f >> 8) & 0xFFu), words[band_off[r + 1] - 1], f & 0xFFu);
  }
}

}  // namespace nice

namespace nice {

// Band helpers: first/last coded pixel of the band (over tiles [tile_lo,
// tile_hi) of frame 0), and the band's total data bits.
__global__ __launch_bounds__(256) void enc_band_edges(EncArgs a, uint32_t* edges) {
  __shared__ uint32_t s_first, s_last;
  if (threadIdx.x == 0) { s_first = NONE; s_last = 0; }
  __syncthreads();
  uint32_t fi = NONE, la = 0;
  bool any = false;
  for (uint32_t t = a.tile_lo + threadIdx.x; t < a.tile_hi; t += 256) {
    fi = min(fi, a.tile_first[t]);
    if (a.tile_last[t] != NONE) { la = max(la, a.tile_last[t]); any = true; }
  }
  atomicMin(&s_first, fi);
  if (any) atomicMax(&s_last, la);
  __syncthreads();
  if (threadIdx.x == 0) {
    edges[0] = s_first;
    edges[1] = s_first == NONE ? NONE : s_last;
  }
}

// The band's data bits: its own symbol counts (bhist, 858 bins; the mode
// prefixes derived from the payload streams as enc_tables does) times the code
// lengths of the shared tables.  info = {bits, data start bit}.
// nice_band_pack_bits after nice_band_tables_dev: the band_bits argument must
// be the device count (d_info[0]); on a mismatch the band is flagged FLAG_BAD
// and the pack kernels write nothing (the flag is recomputed on every call)
__global__ void enc_band_check(EncArgs a, const unsigned long long* info, unsigned long long band_bits) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const bool bad = info[0] != band_bits;
    a.frame_flags[0] = (a.frame_flags[0] & ~FLAG_BAD) | (bad ? FLAG_BAD : 0u);
    if (bad) a.band_fix[0] = BAND_FIX_BAD;   // reported by nice_band_assemble
  }
}

__global__ __launch_bounds__(256) void enc_band_sum(EncArgs a, const uint32_t* bhist, unsigned long long* info) {
  __shared__ unsigned long long s_bits;
  __shared__ uint32_t s_mode[5];
  if (threadIdx.x == 0) s_bits = 0;
  if (threadIdx.x < 5) s_mode[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long v = 0;
  uint32_t c[5] = {0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < N_BINS; b += 256) {
    const uint32_t h = bhist[b];
#pragma unroll
    for (int k = 0; k < 5; ++k) c[k] += mode_id_bin(k, b) ? h : 0u;
    if (b >= BIN_PREFIX && b < BIN_PREFIX + 5) continue;   // mode prefixes: below
    v += (unsigned long long)h * a.tbl_len8[b];
  }
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (c[k]) atomicAdd(&s_mode[k], c[k]);
  atomicAdd(&s_bits, v);
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bits = s_bits;
    for (int k = 0; k < 5; ++k)
      bits += (unsigned long long)(s_mode[k] / mode_id_syms(k)) * a.tbl_len8[BIN_PREFIX + k];
    info[0] = bits;
    info[1] = a.seed_bit[0];
  }
}

}  // namespace nice
