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
  if (__any(!br && !sd && !l2)) {
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
      if (p < count) recs[p] = rec;
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

__device__ __forceinline__ uint32_t y_from_rgba(uint32_t v) {
  const uint32_t s = spread_rgba(v);
  const uint32_t g = (v >> 8) & 0xFFu;
  return (s + K3(256u) - (g | (g << 20))) & K3(0xFFu);
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
template <bool HEAD>
__device__ __forceinline__ uint32_t classify_ring(const uint32_t* ring, uint32_t s, uint32_t tid, uint32_t W,
                                                  uint32_t i, const uint32_t* ltab) {
  const uint32_t* b0 = ring + ((s - 3u) & (CLS_RING - 1)) + tid;
  const uint32_t* b1 = ring + ((s - W - 3u) & (CLS_RING - 1)) + tid;
  const uint32_t* b2 = ring + ((s - 2u * W) & (CLS_RING - 1)) + tid;
  const uint32_t* b3 = ring + ((s - 3u * W - 3u) & (CLS_RING - 1)) + tid;
  const uint32_t X = b0[3], L2 = b0[1], L3 = b0[0];
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
  const bool sd = has_left && ((d & K3(0x3F8u)) == K3(0x100u)) && ((((d & K3(7u)) + K3(1u)) & K3(8u)) == 0);
  const uint32_t sdi = (d & 7u) + 7u * ((d >> 10) & 7u) + 49u * ((d >> 20) & 7u);
  // luma2 against the prediction (code.rs:252-292)
  const uint32_t pg = (pred >> 10) & 0xFFu;
  const uint32_t py = (uint32_t)(__mul24((int)pg, -0x100001) + (int)(pred + K3(256u))) & K3(0xFFu);
  const uint32_t xk = X + LUMA_KY;
  const uint32_t t2 = xk - py;
  const bool l2 = has_up && (t2 & LUMA_MASK) == 0;
  // luma against 11 references, first hit wins (code.rs:293-339)
  uint32_t lk = 11u, lt = 0u;
  if (__any(!br && !sd && !l2)) {
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
      lt = xk - ring[ltab[m & 15u] + tid];
    }
  }
  const uint32_t r = xr + K3(256u) - (has_left ? pred : 0u);
  const uint32_t rec_br = P_BACK_REF | (bk << 3);
  const uint32_t rec_sd = P_SMALL_DIFF | (sdi << 3);
  // LUMA2 and LUMA keep the luma-space fields in place (LUMA: after its 4-bit reference)
  const uint32_t lf = (l2 ? t2 : lt) & LUMA_FIELDS;
  const uint32_t rec_l2 = P_LUMA2 | (lf << 3);
  const uint32_t rec_lu = P_LUMA | (lk << 3) | (lf << 7);
  const uint32_t rec_rgb = P_RGB | ((r & K3(0xFFu)) << 3);
  return br ? rec_br : sd ? rec_sd : l2 ? rec_l2 : lk < 11u ? rec_lu : rec_rgb;
}

__global__ __launch_bounds__(CLS_THREADS) void enc_classify_ring(EncArgs a) {
  __shared__ uint32_t ring[CLS_RING + CLS_GUARD];
  __shared__ uint32_t hist[N_BINS + 64];   // + a discard slot per lane (absent symbols)
  __shared__ uint32_t snap[N_BINS];        // hist after the previous tile
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ RecBinTable rbt;
  __shared__ uint32_t ltab[2][CLS_PPT][16];   // [tile parity][q][luma reference]: ring index for thread 0
  const uint32_t T = a.tiles_per_frame;
  const uint64_t total_work = (uint64_t)a.n_frames * T;
  const uint64_t w_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  const uint64_t w_end = min(w_begin + a.tiles_per_block, total_work);
  if (w_begin >= w_end) return;
  const int tid = threadIdx.x, lane = tid & 63;
  rbt_init(rbt, tid);
  // back distance of luma reference k (code.rs:293-339), for the tile tables
  const uint32_t lback = tid < 16 * CLS_PPT && (tid & 15) < 11
                             ? (uint32_t)lr_rows(tid & 15) * a.W + (uint32_t)lr_px(tid & 15) : 0u;
  const uint32_t W = a.W;
  const int64_t N = (int64_t)W * a.H;
  for (int b = tid; b < N_BINS; b += CLS_THREADS) { hist[b] = 0; snap[b] = 0; }
  auto flush = [&](uint32_t frame) {
    __syncthreads();
    for (int b = tid; b < N_BINS; b += CLS_THREADS) {
      if (hist[b]) atomicAdd(&a.hist[(uint64_t)frame * N_BINS + b], hist[b]);
      hist[b] = 0;
      snap[b] = 0;
    }
  };
  // prefill: the 3 rows + 3 pixels before the first tile
  uint32_t cur_frame = (uint32_t)(w_begin / T);
  {
    const int64_t start = (int64_t)(w_begin % T) * ENC_TILE;
    const int64_t lo = max((int64_t)0, start - 3 * (int64_t)W - 3);
    const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)cur_frame * a.frame_stride);
    for (int64_t j = lo + tid; j < start; j += CLS_THREADS) {
      const uint32_t k = (uint32_t)j & (CLS_RING - 1), y = y_from_rgba(fr[j]);
      ring[k] = y;
      if (k < CLS_GUARD) ring[CLS_RING + k] = y;
    }
  }
  // the first tile's pixels
  uint32_t pf[CLS_PPT];
  auto fetch = [&](const TileIter& ti, uint32_t (&v)[CLS_PPT]) {
    const uint32_t f = ti.f;
    const int64_t start = (int64_t)ti.tt() * ENC_TILE;
    const uint32_t* fr = reinterpret_cast<const uint32_t*>(a.px + (uint64_t)f * a.frame_stride);
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int64_t j = start + q * CLS_THREADS + tid;
      v[q] = j < N ? fr[j] : 0u;
    }
  };
  // this tile's symbol counts (histogram growth since the previous tile), for
  // enc_tilebits_hist: 858 u16 counts as u32 pairs.  Taken for tile t after
  // the staging barrier of tile t + 1 (every atomic of t is done, none of t + 1
  // has started): no barrier of its own.
  uint64_t prev_t = ~0ull;
  auto snap_tile = [&]() {
    if (prev_t != ~0ull && tid < (int)TH_WORDS) {
      uint32_t wv = 0;
      if (2 * tid < N_BINS) {
        const int b = 2 * tid;
        const uint32_t h0 = hist[b], h1 = hist[b + 1];
        wv = ((h0 - snap[b]) & 0xFFFFu) | ((h1 - snap[b + 1]) << 16);
        snap[b] = h0;
        snap[b + 1] = h1;
      }
      a.tile_hist[prev_t * TH_WORDS + tid] = wv;
    }
    prev_t = ~0ull;
  };
  TileIter it(a, w_begin), nx(a, w_begin);
  fetch(nx, pf);
  for (uint64_t w = w_begin; w < w_end; ++w, it.step(1)) {
    const uint32_t f = it.f;
    const uint32_t tt = it.tt();
    if (f != cur_frame) {
      __syncthreads();
      snap_tile();
      flush(cur_frame);
      cur_frame = f;
    }
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)min((int64_t)ENC_TILE, N - start);
    // stage this tile (Y space), start loading the next
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const uint32_t k = (uint32_t)(start + q * CLS_THREADS + tid) & (CLS_RING - 1), y = y_from_rgba(pf[q]);
      ring[k] = y;
      if (k < CLS_GUARD) ring[CLS_RING + k] = y;
    }
    // this tile's luma reference table (double-buffered: the previous tile's
    // readers are past the staging barrier below before it is rewritten)
    if (tid < 16 * CLS_PPT)
      ltab[w & 1][tid >> 4][tid & 15] =
          ((uint32_t)(start + (tid >> 4) * CLS_THREADS) - lback) & (CLS_RING - 1);
    nx.step(1);
    if (w + 1 < w_end) fetch(nx, pf);
    __syncthreads();
    snap_tile();
    // coded flags -> tile bitmask (a pixel is coded iff i == 0 or Y(i) != Y(i-1))
    uint32_t coded_bits = 0;
    unsigned long long wbal[CLS_PPT];   // coded flags of the wave's 64 pixels per q
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const int64_t i = start + p;
      const uint32_t* bl = ring + ((uint32_t)(start + q * CLS_THREADS - 1) & (CLS_RING - 1)) + tid;
      const bool coded = p < count && (i == 0 || bl[1] != bl[0]);
      const unsigned long long bal = __ballot(coded);
      wbal[q] = bal;
      if (lane == 0) {
        const int wb = (q * CLS_THREADS + (tid & ~63)) >> 5;
        mask[wb] = (uint32_t)bal;
        mask[wb + 1] = (uint32_t)(bal >> 32);
      }
      coded_bits |= (coded ? 1u : 0u) << q;
    }
    __syncthreads();
    if (tid < 64) {   // first / last coded pixel of the tile: one wave, no loop
      const uint32_t mw = tid < ENC_TILE / 32 ? mask[tid] : 0u;
      const unsigned long long nz = __ballot(mw != 0);
      if (tid == 0) {
        const uint64_t t = (uint64_t)f * T + tt;
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
        rf = classify_ring<false>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W, 0u, ltab[w & 1][q]);
      else
        rf = classify_ring<true>(ring, (uint32_t)(start + q * CLS_THREADS), (uint32_t)tid, W, (uint32_t)(start + p),
                                 nullptr);
      rec[q] = coded ? rf : REC_UNCODED;
    }
#pragma unroll
    for (int q = 0; q < CLS_PPT; ++q) {
      const int p = q * CLS_THREADS + tid;
      const bool coded = (coded_bits >> q) & 1u;
      if (p < count) recs[p] = rec[q];
      // the mode prefixes (bins BIN_PREFIX + 0..4) are not counted here: each
      // mode emits a fixed number of symbols into one stream of its own, so
      // enc_tables and enc_tilebits_hist derive them (mode_prefix_count)
      {
        // payload symbols: four unconditional LDS adds, absent ones into this
        // lane's discard slot (no divergent branches)
        uint32_t b0, b1, b2, b3;
        const uint32_t n = rec_bins(rbt, rec[q], b0, b1, b2, b3);
        const uint32_t dump = N_BINS + (uint32_t)lane;
        atomicAdd(&hist[coded ? b0 : dump], 1u);
        atomicAdd(&hist[coded && n > 1 ? b1 : dump], 1u);
        atomicAdd(&hist[coded && n > 1 ? b2 : dump], 1u);
        atomicAdd(&hist[coded && n > 3 ? b3 : dump], 1u);
      }
      // a run follows only if the next pixel is uncoded: most coded lanes stop
      // at this one bit test (lane 63's next pixel is in the next wave: full path)
      const bool next_coded = lane < 63 && ((wbal[q] >> (lane + 1)) & 1ull);
      if (coded && !next_coded) {
        // next coded pixel: in this wave's 64 pixels from the ballot, else the tile mask
        const unsigned long long above = lane < 63 ? (wbal[q] >> (lane + 1)) : 0ull;
        const int nx = above ? p + 1 + (int)__builtin_ctzll(above) : next_coded_local(mask, p | 63);
        if (nx < count && nx > p + 1) {
          uint64_t mm = (uint64_t)(nx - p - 2);
          while (true) {
            atomicAdd(&hist[BIN_PREFIX + P_RUN1 + (uint32_t)(mm & 7u)], 1u);
            if (mm < 8) break;
            mm >>= 3;
          }
        }
      }
    }
    prev_t = (uint64_t)f * T + tt;
  }
  __syncthreads();
  snap_tile();
  flush(cur_frame);
}

// ---------------------------------------------------------------------------
// K2: runs crossing tile ends. One block (1024 threads) per frame.
// tile_next[t] = first coded pixel after tile t (N if none).
// ---------------------------------------------------------------------------
// Aggregate of each group of ENC_GROUP_TILES tiles (grid: groups x frames).
__global__ __launch_bounds__(256) void enc_group_reduce(EncArgs a, int what) {
  __shared__ unsigned long long part[4];
  const uint32_t g = blockIdx.x, f = blockIdx.y;
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
  uint32_t after = a.band ? (uint32_t)a.band_next : NONE;
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
  const uint32_t f = blockIdx.x / N_STREAMS;
  const int s = blockIdx.x % N_STREAMS;
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
// K5-K7: bit placement without a serial dependency.
//   enc_tilebits  per tile: bits of its pixels (prefix, payload, run digits)
//   enc_tilescan  per frame: exclusive scan of tile bits from the data start;
//                 zeroes every output word two tiles (or a tile and the tail)
//                 share, so enc_pack can OR those and store the rest
//   enc_pack      per tile: codes MSB-first into an LDS bit buffer, then
//                 shifted to the tile's offset: interior words stored, the
//                 first/last partial words OR-ed (bitwriter.rs:55-73)
//   enc_tail      per frame: [P, P, 0, 0, 0] after the data (hfe.rs:115,
//                 code.rs:421-422) and the stream length
// A thread owns 4 consecutive pixels and reads their records with one 16-byte
// load.
// ---------------------------------------------------------------------------
constexpr int PACK_MAX_WORDS = ENC_TILE * 128 / 32 + 2;   // <= 125 bits/px with 25-bit codes

struct TileQuad {
  uint32_t rc[4];
  uint32_t nib;        // coded flags of the 4 pixels
  uint64_t run[4];     // run after each coded pixel
  uint32_t nb;         // bits of the 4 pixels
  uint32_t e[4][5];    // code table entries: prefix + up to 4 payload symbols (0: none)
};

// The thread's 4 records of tile t (REC_UNCODED past the frame end); issued one
// tile ahead so the loads overlap the previous tile's work.
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
    for (int q = 0; q < 4; ++q) rc[q] = (p0 + q < count) ? rp[q] : REC_UNCODED;
  }
}

// Builds the tile's coded mask from the records (LDS, needs a barrier before
// use) -- phase 1.
__device__ __forceinline__ void quad_mask(const uint32_t (&rc)[4], int lane, int wid, uint32_t* mask,
                                          TileQuad& Q) {
#pragma unroll
  for (int q = 0; q < 4; ++q) Q.rc[q] = rc[q];
  Q.nib = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) Q.nib |= ((Q.rc[q] & 7u) != REC_UNCODED ? 1u : 0u) << q;
  const uint32_t mw = wave_or8(Q.nib << (4 * (lane & 7)));
  if ((lane & 7) == 0) mask[wid * 8 + (lane >> 3)] = mw;
}

// Runs, code entries and bit counts -- phase 2 (after the mask barrier).
// Branch-free apart from the run digits: absent symbols get entry 0 (length 0).
__device__ __forceinline__ void quad_bits(const uint32_t* tbl, const RecBinTable& rbt, const uint32_t* mask,
                                          int64_t start, int count, int p0, uint32_t next_tile_px, TileQuad& Q) {
  const int nx_local = next_coded_local(mask, p0 + 3);
  const uint64_t after = (nx_local < count) ? (uint64_t)(start + nx_local) : (uint64_t)next_tile_px;
  Q.nb = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bool coded = (Q.nib >> q) & 1u;
    uint32_t b0, b1, b2, b3;
    const uint32_t n = rec_bins(rbt, Q.rc[q], b0, b1, b2, b3);
    const uint32_t t0 = tbl[BIN_PREFIX + min(Q.rc[q] & 7u, 4u)], t1 = tbl[b0], t2 = tbl[b1], t3 = tbl[b2],
                   t4 = tbl[b3];
    Q.e[q][0] = coded ? t0 : 0u;
    Q.e[q][1] = coded ? t1 : 0u;
    Q.e[q][2] = (coded && n > 1) ? t2 : 0u;
    Q.e[q][3] = (coded && n > 1) ? t3 : 0u;
    Q.e[q][4] = (coded && n > 3) ? t4 : 0u;
    Q.nb += (Q.e[q][0] & 31u) + (Q.e[q][1] & 31u) + (Q.e[q][2] & 31u) + (Q.e[q][3] & 31u) + (Q.e[q][4] & 31u);
    const uint32_t later = Q.nib >> (q + 1);
    const uint64_t nxt = later ? (uint64_t)(start + p0 + q + 1 + __builtin_ctz(later)) : after;
    Q.run[q] = coded ? nxt - (uint64_t)(start + p0 + q) - 1 : 0u;
    if (Q.run[q] > 0) {
      uint64_t m = Q.run[q] - 1;
      while (true) {
        Q.nb += tbl[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)] & 31u;
        if (m < 8) break;
        m >>= 3;
      }
    }
  }
}

__device__ __forceinline__ void load_tbl(uint32_t* tbl, const EncArgs& a, uint32_t f) {
  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) tbl[b] = a.tbl[(uint64_t)f * N_BINS + b];
}
__device__ __forceinline__ void load_lens(uint32_t* lens, const EncArgs& a, uint32_t f) {
  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) lens[b] = a.tbl_len8[(uint64_t)f * N_BINS + b];
}

// Bits of the thread's 4 pixels (prefix, payload, run digits) from full code
// lengths (any length: also the frames with codes over FAST_MAX_CODE_BITS).
__device__ __forceinline__ uint32_t quad_nbits(const uint32_t* lens, const RecBinTable& rbt, const uint32_t* mask,
                                               int64_t start, int count, int p0, uint32_t next_tile_px,
                                               const TileQuad& Q) {
  const int nx_local = next_coded_local(mask, p0 + 3);
  const uint64_t after = (nx_local < count) ? (uint64_t)(start + nx_local) : (uint64_t)next_tile_px;
  uint32_t nb = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (!((Q.nib >> q) & 1u)) continue;
    uint32_t b0, b1, b2, b3;
    const uint32_t n = rec_bins(rbt, Q.rc[q], b0, b1, b2, b3);
    nb += lens[BIN_PREFIX + min(Q.rc[q] & 7u, 4u)] + lens[b0];
    if (n > 1) nb += lens[b1] + lens[b2];
    if (n > 3) nb += lens[b3];
    const uint32_t later = Q.nib >> (q + 1);
    const uint64_t nxt = later ? (uint64_t)(start + p0 + q + 1 + __builtin_ctz(later)) : after;
    const uint64_t run = nxt - (uint64_t)(start + p0 + q) - 1;
    if (run > 0) {
      uint64_t m = run - 1;
      while (true) {
        nb += lens[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)];
        if (m < 8) break;
        m >>= 3;
      }
    }
  }
  return nb;
}

// Contiguous tile ranges per block (the code table is reloaded only when the
// frame changes); records are fetched one tile ahead.
// Work items w in [w0, w1): frame w / nt, band tile tile_lo + w % nt.
__device__ __forceinline__ void tile_range(const EncArgs& a, uint64_t& w0, uint64_t& w1) {
  const uint64_t total = (uint64_t)a.n_frames * (a.tile_hi - a.tile_lo);
  const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
  w0 = (uint64_t)blockIdx.x * per;
  w1 = w0 + per < total ? w0 + per : total;
}

__global__ __launch_bounds__(ENC_THREADS) void enc_tilebits(EncArgs a) {
  __shared__ uint32_t tbl[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t wsum[ENC_THREADS / 64];
  __shared__ RecBinTable rbt;
  rbt_init(rbt, threadIdx.x);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * threadIdx.x;
  uint32_t cur_f = 0xFFFFFFFFu;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  uint32_t rn[4];
  TileIter it(a, t0), nx(a, t0);
  if (t0 < t1) quad_fetch(a, nx.f, nx.tt(), p0, rn);
  for (uint64_t w = t0; w < t1; ++w, it.step(1)) {
    const uint64_t t = it.tile();
    uint32_t rc[4] = {rn[0], rn[1], rn[2], rn[3]};
    nx.step(1);
    if (w + 1 < t1) quad_fetch(a, nx.f, nx.tt(), p0, rn);
    const uint32_t f = it.f, tt = it.tt();
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    __syncthreads();
    if (f != cur_f) { load_lens(tbl, a, f); cur_f = f; }
    TileQuad Q;
    quad_mask(rc, lane, wid, mask, Q);
    __syncthreads();
    uint32_t x = quad_nbits(tbl, rbt, mask, start, count, p0, a.tile_next[t], Q);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) a.tile_bits[t] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  }
}

// Tile bits from the per-tile symbol counts of enc_classify_ring: sum of
// count x code length over the 858 bins, plus the run digits of the tile's
// last run (it ends at tile_next, in a later tile; code.rs:371-407).  One wave
// per tile, no block barriers: each wave keeps the code lengths of its current
// frame in its own LDS slice.
__global__ __launch_bounds__(256) void enc_tilebits_hist(EncArgs a) {
  __shared__ uint32_t lens_all[4][2 * TH_WORDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* lens = lens_all[wid];
  uint32_t cur_f = 0xFFFFFFFFu, prefix_len_rgb = 0;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  TileIter it(a, t0 + wid);
  for (uint64_t w = t0 + wid; w < t1; w += 4, it.step(4)) {
    const uint64_t t = it.tile();
    const uint32_t f = it.f;
    if (f != cur_f) {
      __builtin_amdgcn_wave_barrier();
      // the mode prefixes are not in the tile counts: each mode's prefix length
      // rides on the bins of its identifying stream (RGB: once per 3 symbols)
      const uint8_t* l8 = a.tbl_len8 + (uint64_t)f * N_BINS;
      uint32_t pl[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) pl[k] = l8[BIN_PREFIX + k];
      prefix_len_rgb = pl[P_RGB];
      for (int b = lane; b < (int)(2 * TH_WORDS); b += 64) {
        uint32_t v = b < N_BINS ? (uint32_t)l8[b] : 0u;
#pragma unroll
        for (int k = 0; k < 5; ++k) v += (k != P_RGB && mode_id_bin(k, b)) ? pl[k] : 0u;
        lens[b] = v;
      }
      cur_f = f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
    const uint32_t* th = a.tile_hist + t * TH_WORDS;
    uint32_t acc = 0, rgb = 0;
#pragma unroll
    for (int k0 = 0; k0 < (int)TH_WORDS; k0 += 64) {
      const int k = k0 + lane;
      if (k < (int)TH_WORDS) {
        const uint32_t v = th[k];
        acc += (v & 0xFFFFu) * lens[2 * k] + (v >> 16) * lens[2 * k + 1];
        if (2 * k < 256) rgb += (v & 0xFFFFu) + (v >> 16);   // SC_RGB symbols: 3 per RGB pixel
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rgb += __shfl_xor(rgb, o);
    if (lane == 0) {
      acc += rgb / 3u * prefix_len_rgb;
      const uint32_t last = a.tile_last[t];
      if (last != NONE) {
        const uint64_t run = (uint64_t)a.tile_next[t] - last - 1;
        if (run > 0) {
          uint64_t m = run - 1;
          while (true) {
            acc += lens[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)];
            if (m < 8) break;
            m >>= 3;
          }
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) a.tile_bits[t] = acc;
  }
}

// One 1024-thread block per frame.
// block (group g, frame f): tiles [g, g + 1) x ENC_GROUP_TILES of the band,
// from the bits of the earlier groups on
__global__ __launch_bounds__(1024) void enc_tilescan(EncArgs a) {
  __shared__ unsigned long long part[1024];
  const uint32_t g = blockIdx.x, f = blockIdx.y;
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

__global__ __launch_bounds__(ENC_THREADS, 5) void enc_pack(EncArgs a) {
  __shared__ uint32_t tbl[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t bits[PACK_MAX_WORDS];
  __shared__ uint32_t wsum[ENC_THREADS / 64];
  __shared__ RecBinTable rbt;
  rbt_init(rbt, threadIdx.x);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t T = a.tiles_per_frame;
  const uint64_t total = (uint64_t)a.n_frames * T;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * threadIdx.x;
  uint32_t cur_f = 0xFFFFFFFFu;
  uint32_t used_words = PACK_MAX_WORDS;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  (void)total;
  uint32_t rn[4];
  TileIter it(a, t0), nx(a, t0);
  if (t0 < t1) quad_fetch(a, nx.f, nx.tt(), p0, rn);
  for (uint64_t w = t0; w < t1; ++w, it.step(1)) {
    const uint64_t t = it.tile();
    uint32_t rc[4] = {rn[0], rn[1], rn[2], rn[3]};
    nx.step(1);
    if (w + 1 < t1) quad_fetch(a, nx.f, nx.tt(), p0, rn);
    const uint32_t f = it.f, tt = it.tt();
    if (a.frame_flags[f] & FLAG_LONG) continue;   // enc_pack_long's frame (block-uniform)
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < used_words; w += ENC_THREADS) bits[w] = 0;
    if (f != cur_f) { load_tbl(tbl, a, f); cur_f = f; }
    TileQuad Q;
    quad_mask(rc, lane, wid, mask, Q);
    __syncthreads();
    quad_bits(tbl, rbt, mask, start, count, p0, a.tile_next[t], Q);
    const uint32_t x = wave_incl_scan(Q.nb);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, tile_bits = 0;
#pragma unroll
    for (int w = 0; w < ENC_THREADS / 64; ++w) {
      const uint32_t ws = wsum[w];
      wbase += (w < wid) ? ws : 0u;
      tile_bits += ws;
    }
    if (Q.nb) {
      uint32_t pp = wbase + x - Q.nb;   // the lane's next bit in the tile
      // n <= 32 bits of val (0 when n == 0) at bit pp, MSB-first: one 64-bit
      // shift places them across words pp >> 5 and pp >> 5 + 1, both OR-ed
      // into LDS (words shared with neighbouring lanes).  No accumulator
      // carried from put to put, so a lane's puts are independent (measured:
      // the accumulator version's flush selects were ~14 VALU per put).
      auto put_n = [&](uint32_t val, uint32_t n) {
        const uint32_t s = pp & 31u, w = pp >> 5;
        const uint64_t v = (uint64_t)val << ((64u - s - n) & 63u);
        atomicOr(&bits[w], (uint32_t)(v >> 32));
        atomicOr(&bits[w + 1], (uint32_t)v);
        pp += n;
      };
      auto put = [&](uint32_t e) { put_n(e >> 5, e & 31u); };   // e == 0: no symbol
      // a pixel's codes composed into one value: 32 bits for every pixel of
      // the wave (the common case: one put per pixel), else 64 bits (two
      // puts), else one put per code
      uint32_t tot[4];
      uint32_t tmax = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        tot[q] = (Q.e[q][0] & 31u) + (Q.e[q][1] & 31u) + (Q.e[q][2] & 31u) + (Q.e[q][3] & 31u) + (Q.e[q][4] & 31u);
        tmax = max(tmax, tot[q]);
      }
      auto put_runs = [&](int q) {
        if (Q.run[q] > 0) {
          uint64_t m = Q.run[q] - 1;
          while (true) {
            put(tbl[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)]);
            if (m < 8) break;
            m >>= 3;
          }
        }
      };
      if (__all(tmax <= 32u)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t v = 0;
#pragma unroll
          for (int k = 0; k < 5; ++k) {
            const uint32_t e = Q.e[q][k];
            v = (v << (e & 31u)) | (e >> 5);
          }
          put_n(v, tot[q]);
          put_runs(q);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (tot[q] <= 64u) {
            uint64_t v = 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
              const uint32_t e = Q.e[q][k], n = e & 31u;
              v = (v << n) | (e >> 5);
            }
            const bool two = tot[q] > 32u;
            put_n(two ? (uint32_t)(v >> 32) : 0u, two ? tot[q] - 32u : 0u);
            put_n((uint32_t)v, two ? 32u : tot[q]);
          } else {
            put(Q.e[q][0]);
            put(Q.e[q][1]);
            put(Q.e[q][2]);
            put(Q.e[q][3]);
            put(Q.e[q][4]);
          }
          put_runs(q);
        }
      }
    }
    __syncthreads();
    // place the tile's bits at its stream offset
    const uint64_t s0 = a.tile_off[t], e0 = s0 + tile_bits;
    const uint32_t sh = (uint32_t)(s0 & 31);
    const uint64_t w0 = s0 >> 5;
    const uint32_t nw = tile_bits ? (uint32_t)(((e0 + 31) >> 5) - w0) : 0u;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(a.out + (uint64_t)f * a.out_stride);
    for (uint32_t m = threadIdx.x; m < nw; m += ENC_THREADS) {
      const uint32_t hi = m ? bits[m - 1] : 0u;
      const uint32_t lo = bits[m];   // zero past the tile's bits
      const uint32_t v = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
      const bool shared = (m == 0 && sh) || (m == nw - 1 && (e0 & 31));
      if (shared) atomicOr(&out32[w0 + m], __builtin_bswap32(v));
      else out32[w0 + m] = __builtin_bswap32(v);
    }
    used_words = nw + 1;
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
// and the next code starts there.  In band mode a window never reaches into
// the previous band: a band's first code is the prefix code of its first coded
// pixel (stream SC_PREFIXES, 13 symbols: at most 12 bits), never a long one.
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
  __shared__ RecBinTable rbt;
  if (!(a.frame_flags[a.n_frames] & FLAG_LONG)) return;   // no long-code frame in the batch
  rbt_init(rbt, threadIdx.x);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t N = (int64_t)a.W * a.H;
  const int p0 = 4 * threadIdx.x;
  uint32_t cur_f = NONE;
  uint64_t t0, t1;
  tile_range(a, t0, t1);
  TileIter it(a, t0);
  for (uint64_t w = t0; w < t1; ++w, it.step(1)) {
    const uint32_t f = it.f, tt = it.tt();
    if (!(a.frame_flags[f] & FLAG_LONG)) continue;   // block-uniform
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
    const uint32_t nb = quad_nbits(lens, rbt, mask, start, count, p0, a.tile_next[t], Q);
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
      } else if (phase == 1 && !(a.band && (pos & ~7ull) < a.band_bit0)) {
        wrapped_write(out, pos, v, n);
      }
      pos += n;
    };
    const int nx_local = next_coded_local(mask, p0 + 3);
    const uint64_t after = (nx_local < count) ? (uint64_t)(start + nx_local) : (uint64_t)a.tile_next[t];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!((Q.nib >> q) & 1u)) continue;
      uint32_t b0, b1, b2, b3;
      const uint32_t n = rec_bins(rbt, Q.rc[q], b0, b1, b2, b3);
      emit(BIN_PREFIX + min(Q.rc[q] & 7u, 4u));
      emit(b0);
      if (n > 1) { emit(b1); emit(b2); }
      if (n > 3) emit(b3);
      const uint32_t later = Q.nib >> (q + 1);
      const uint64_t nxt = later ? (uint64_t)(start + p0 + q + 1 + __builtin_ctz(later)) : after;
      const uint64_t run = nxt - (uint64_t)(start + p0 + q) - 1;
      if (run > 0) {
        uint64_t m = run - 1;
        while (true) {
          emit(BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u));
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
  const unsigned long long w0 = band_w0[r];
  for (unsigned long long m = (unsigned long long)blockIdx.x * 256 + threadIdx.x; m < n;
       m += (unsigned long long)gridDim.x * 256) {
    const uint32_t v = words[band_off[r] + m];
    if (m == 0 || m + 1 == n) atomicOr(&out32[w0 + m], v);   // shared with a neighbour or the header
    else out32[w0 + m] = v;
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

__global__ __launch_bounds__(256) void enc_band_sum(EncArgs a, unsigned long long* info) {
  __shared__ unsigned long long s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  unsigned long long v = 0;
  for (uint32_t t = a.tile_lo + threadIdx.x; t < a.tile_hi; t += 256) v += a.tile_bits[t];
  atomicAdd(&s, v);
  __syncthreads();
  if (threadIdx.x == 0) {
    info[0] = s;
    info[1] = a.seed_bit[0];
  }
}

}  // namespace nice
