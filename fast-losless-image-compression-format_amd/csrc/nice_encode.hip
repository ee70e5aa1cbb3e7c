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
//   enc_serial     exact single-lane replay of the reference writer, used only
//                  for frames whose emitted codes exceed FAST_MAX_CODE_BITS
//                  (where the reference's u32 cache arithmetic mangles bits).
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
                                  int64_t N, uint32_t W, int C) {
  for (int k = 0; k < 4; ++k) {
    const int64_t base = start - (int64_t)k * W - 3;
    for (int j = threadIdx.x; j < WIN; j += ENC_THREADS) {
      const int64_t g = base + j;
      tw.w[k][j] = (g >= 0 && g < N) ? load_spread(frame, g, C) : 0u;
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
// K1: classify + histogram.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(ENC_THREADS) void enc_classify(EncArgs a) {
  __shared__ TileWin tw;
  __shared__ uint32_t hist[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];

  const uint64_t total_tiles = (uint64_t)a.n_frames * a.tiles_per_frame;
  const uint64_t t_begin = (uint64_t)blockIdx.x * a.tiles_per_block;
  uint64_t t_end = t_begin + a.tiles_per_block;
  if (t_end > total_tiles) t_end = total_tiles;
  if (t_begin >= t_end) return;

  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) hist[b] = 0;
  uint32_t cur_frame = (uint32_t)(t_begin / a.tiles_per_frame);
  const int lane = threadIdx.x & 63;

  for (uint64_t t = t_begin; t < t_end; ++t) {
    const uint32_t f = (uint32_t)(t / a.tiles_per_frame);
    const uint32_t tt = (uint32_t)(t % a.tiles_per_frame);
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
    const int64_t N = (int64_t)a.W * a.H;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    __syncthreads();
    stage_tile(tw, frame, start, N, a.W, a.C);
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
#pragma unroll
    for (int r = 0; r < PX_PER_THREAD; ++r) {
      const int p = r * ENC_THREADS + threadIdx.x;
      const bool coded = (coded_bits >> r) & 1u;
      PixSyms s;
      s.mode = 0xFF;
      if (coded) {
        WinAcc acc{&tw, p + 3};
        if (fast) classify<true>((uint32_t)(start + p), a.W, acc, s);
        else classify<false>((uint32_t)(start + p), a.W, acc, s);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((uint32_t)k < s.n) atomicAdd(&hist[s.b[k]], 1u);
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
      // mode prefix: aggregate per wave (5 values, heavy contention otherwise)
#pragma unroll
      for (int v = 0; v < 5; ++v) {
        const unsigned long long bal = __ballot(s.mode == (uint32_t)v);
        if (lane == v && bal) atomicAdd(&hist[BIN_PREFIX + v], (uint32_t)__popcll(bal));
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS)
    if (hist[b]) atomicAdd(&a.hist[(uint64_t)cur_frame * N_BINS + b], hist[b]);
}

// ---------------------------------------------------------------------------
// K2: runs crossing tile ends. One block (1024 threads) per frame.
// tile_next[t] = first coded pixel after tile t (N if none).
// ---------------------------------------------------------------------------
constexpr int TR_THREADS = 1024;
__global__ __launch_bounds__(TR_THREADS) void enc_tailruns(EncArgs a) {
  __shared__ uint32_t chunk_min[TR_THREADS];
  const uint32_t f = blockIdx.x;
  const uint32_t T = a.tiles_per_frame;
  const uint64_t base = (uint64_t)f * T;
  const uint32_t N = a.W * a.H;
  const uint32_t per = (T + TR_THREADS - 1) / TR_THREADS;
  const uint32_t c0 = threadIdx.x * per;
  const uint32_t c1 = min(c0 + per, T);
  uint32_t m = NONE;
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
  uint32_t nxt = (threadIdx.x + 1 < TR_THREADS) ? chunk_min[threadIdx.x + 1] : NONE;
  for (int64_t t = (int64_t)c1 - 1; t >= (int64_t)c0; --t) {
    const uint32_t next_px = (nxt == NONE) ? N : nxt;
    a.tile_next[base + t] = next_px;
    const uint32_t last = a.tile_last[base + t];
    if (last != NONE) {
      const uint64_t run = (uint64_t)next_px - last - 1;
      if (run > 0) {
        uint64_t mm = run - 1;
        while (true) {
          atomicAdd(&a.hist[(uint64_t)f * N_BINS + BIN_PREFIX + P_RUN1 + (uint32_t)(mm & 7u)], 1u);
          if (mm < 8) break;
          mm >>= 3;
        }
      }
    }
    nxt = min(nxt, a.tile_first[base + t]);
  }
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
  __syncthreads();
  if (lane == 0) huffman_merge_tree(h, counts, n);
  __syncthreads();
  // aob = 1 + number of merged ancestors (u8 wrapping, hfe.rs:79-82)
  uint32_t my_max = 0, my_emit_max = 0;
  for (int i = lane; i < n; i += 64) {
    uint32_t depth = 0;
    for (int p = h.parent[i]; p >= 0; p = h.parent[p]) ++depth;
    const uint8_t aob = (uint8_t)(1u + depth);
    h.aob[i] = aob;
    my_max = max(my_max, (uint32_t)aob);
    if (counts[i]) my_emit_max = max(my_emit_max, (uint32_t)aob);
  }
  __syncthreads();
  // order = symbols sorted by (aob desc, symbol desc): rank by counting.
  for (int i = lane; i < n; i += 64) {
    const uint8_t ai = h.aob[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const uint8_t aj = h.aob[j];
      rank += (aj > ai) || (aj == ai && j > i);
    }
    h.order[rank] = (uint16_t)i;
  }
  // wave max
  for (int o = 32; o > 0; o >>= 1) {
    my_max = max(my_max, (uint32_t)__shfl_xor((int)my_max, o));
    my_emit_max = max(my_emit_max, (uint32_t)__shfl_xor((int)my_emit_max, o));
  }
  __syncthreads();
  if (lane == 0) {
    // hfe.rs:271-290 with usize wrapping arithmetic
    unsigned long long cur = 0;
    uint8_t prev = 0;
    for (int k = 0; k < n; ++k) {
      const int sym = h.order[k];
      const uint8_t aob = h.aob[sym];
      if (aob < prev) cur >>= ((uint8_t)(prev - aob)) & 63u;
      if (prev > 0) cur += 1;
      const unsigned long long code = (1ull << (aob & 63u)) - cur - 1ull;
      const uint64_t e = (uint64_t)f * N_BINS + sb + sym;
      a.tbl_len8[e] = aob;
      a.tbl_code[e] = (uint32_t)code;
      a.tbl[e] = (aob <= FAST_MAX_CODE_BITS) ? (uint32_t)((code << 5) | aob) : 0u;
      prev = aob;
    }
    a.stream_max[(uint64_t)f * N_STREAMS + s] = (uint8_t)my_max;
    if (my_emit_max > FAST_MAX_CODE_BITS) atomicOr(&a.frame_flags[f], FLAG_SERIAL);
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
  const bool serial_frame = (a.frame_flags[f] & FLAG_SERIAL) != 0;

  if (normal && !serial_frame && N > 0) {
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
    // pos == 104 + 6056 = 6160; write words [0, 192) (bytes 0..767)
    const uint32_t full = pos >> 5;
    for (int w = lane; w < (int)full; w += 64)
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
  // Serial exact path (spilled 5-bit fields, 8-bit fields, serial frames, empty frames).
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
  if (N == 0 && !serial_frame) {
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
// K5: pack with decoupled look-back.
// ---------------------------------------------------------------------------
constexpr uint64_t ST_AGG = 1ull << 62;
constexpr uint64_t ST_INC = 2ull << 62;
constexpr uint64_t LEN_MASK = (1ull << 62) - 1;
// per tile: {u64 flag, u32 suffix_agg, u32 suffix_inc}
struct TileDesc {
  unsigned long long flag;
  uint32_t suf_agg;
  uint32_t suf_inc;
};

__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_rlx(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_rlx64(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (len, last-32-bits) monoid
__device__ __forceinline__ void suf_combine(uint64_t& len, uint32_t& suf, uint64_t len2, uint32_t suf2) {
  if (len2 >= 32) suf = suf2;
  else if (len2 > 0) suf = (suf << len2) | suf2;
  len += len2;
}

constexpr int PACK_MAX_WORDS = ENC_TILE * 128 / 32 + 2;   // <= 125 bits/px with 25-bit codes

__device__ __forceinline__ void or_bits(uint32_t* buf, uint64_t pos, uint32_t v, uint32_t n) {
  // place the low n (1..32) bits of v at local bit position pos (MSB-first)
  const uint32_t w = (uint32_t)(pos >> 5), o = (uint32_t)(pos & 31);
  if (o + n <= 32) {
    atomicOr(&buf[w], v << (32 - o - n));
  } else {
    atomicOr(&buf[w], v >> (o + n - 32));
    atomicOr(&buf[w + 1], v << (64 - o - n));
  }
}

// Wave-parallel decoupled look-back for tile t (wave 0 only): lane i inspects
// predecessor t-1-i; a window without an inclusive prefix folds 64 aggregates
// and moves back 64 tiles.  Returns the exclusive (bit length, last 32 bits).
__device__ inline void look_back(const EncArgs& a, uint64_t t, uint32_t tt, uint32_t f, int lane,
                                 uint64_t* wlen, uint32_t* wsuf, uint64_t* out_len, uint32_t* out_suf) {
  TileDesc* desc = reinterpret_cast<TileDesc*>(a.tiles_desc);
  const int64_t fs = (int64_t)t - tt;           // first tile of this frame
  uint64_t acc_len = 0;                         // tiles (base+1 .. t-1), concatenated
  uint32_t acc_suf = 0;
  int64_t base = (int64_t)t - 1;
  uint32_t spins = 0;
  while (true) {
    const int64_t j = base - lane;
    uint64_t st, len;
    uint32_t suf = 0;
    if (j < fs) {                               // before the frame: the header seed
      st = ST_INC;
      len = a.seed_bit[f];
    } else {
      const unsigned long long fl = ld_rlx64(&desc[j].flag);
      st = fl & ~LEN_MASK;
      len = fl & LEN_MASK;
    }
    const unsigned long long inc = __ballot(st == ST_INC);
    const int first_inc = inc ? __builtin_ctzll(inc) : 64;
    const unsigned long long need = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1ull);
    if (__ballot(st == 0) & need) {
      if (++spins > 16) __builtin_amdgcn_s_sleep(1);
      continue;
    }
    if (lane <= first_inc) {
      if (j < fs) suf = a.seed_suf[f];
      else suf = st == ST_INC ? ld_rlx(&desc[j].suf_inc) : ld_rlx(&desc[j].suf_agg);
      wlen[lane] = len;
      wsuf[lane] = suf;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane == 0) {
      const int last = first_inc < 64 ? first_inc : 63;
      uint64_t l = 0;
      uint32_t sx = 0;
      for (int i = last; i >= 0; --i) suf_combine(l, sx, wlen[i], wsuf[i]);   // oldest first
      suf_combine(l, sx, acc_len, acc_suf);
      acc_len = l;
      acc_suf = sx;
    }
    acc_len = __shfl(acc_len, 0);
    acc_suf = __shfl(acc_suf, 0);
    if (first_inc < 64) break;
    base -= 64;
  }
  *out_len = acc_len;
  *out_suf = acc_suf;
}

// Persistent: each block takes tiles in ticket order (forward progress for the
// look-back), reloading the code table only when the frame changes.
__global__ __launch_bounds__(ENC_THREADS) void enc_pack(EncArgs a) {
  __shared__ TileWin tw;
  __shared__ uint32_t tbl[N_BINS];
  __shared__ uint32_t mask[ENC_TILE / 32];
  __shared__ uint32_t bits[PACK_MAX_WORDS];
  __shared__ uint32_t wsum[ENC_THREADS / 64];
  __shared__ uint64_t wlen[64];
  __shared__ uint32_t wsuf[64];
  __shared__ uint32_t s_tile;
  __shared__ uint64_t s_excl_len;
  __shared__ uint32_t s_excl_suf;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const uint32_t T = a.tiles_per_frame;
  const uint64_t total = (uint64_t)a.n_frames * T;
  const int64_t N = (int64_t)a.W * a.H;
  uint32_t cur_f = 0xFFFFFFFFu;
  uint32_t used_words = PACK_MAX_WORDS;        // bits[] words to clear before the next tile
  TileDesc* descs = reinterpret_cast<TileDesc*>(a.tiles_desc);

  while (true) {
    __syncthreads();
    if (threadIdx.x == 0) s_tile = atomicAdd(a.ticket, 1u);
    for (uint32_t w = threadIdx.x; w < used_words; w += ENC_THREADS) bits[w] = 0;
    __syncthreads();
    const uint64_t t = s_tile;
    if (t >= total) break;
    const uint32_t f = (uint32_t)(t / T);
    const uint32_t tt = (uint32_t)(t % T);
    if (a.frame_flags[f] & FLAG_SERIAL) { used_words = 0; continue; }   // enc_serial's frame
    const uint8_t* frame = a.px + (uint64_t)f * a.frame_stride;
    const int64_t start = (int64_t)tt * ENC_TILE;
    const int count = (int)((N - start) < ENC_TILE ? (N - start) : ENC_TILE);
    if (f != cur_f) {
      for (int b = threadIdx.x; b < N_BINS; b += ENC_THREADS) tbl[b] = a.tbl[(uint64_t)f * N_BINS + b];
      cur_f = f;
    }
    stage_tile(tw, frame, start, N, a.W, a.C);
    __syncthreads();

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

    const bool fast = (a.W >= 3) && (start >= 3 * (int64_t)a.W + 3);
    const uint32_t next_tile_px = a.tile_next[t];
    uint32_t round_base = 0;
#pragma unroll
    for (int r = 0; r < PX_PER_THREAD; ++r) {
      const int p = r * ENC_THREADS + threadIdx.x;
      PixSyms sy;
      sy.n = 0;
      sy.mode = 0;
      uint64_t run = 0;
      uint32_t nb = 0;
      if ((coded_bits >> r) & 1u) {
        WinAcc acc{&tw, p + 3};
        if (fast) classify<true>((uint32_t)(start + p), a.W, acc, sy);
        else classify<false>((uint32_t)(start + p), a.W, acc, sy);
        nb = tbl[BIN_PREFIX + sy.mode] & 31u;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((uint32_t)k < sy.n) nb += tbl[sy.b[k]] & 31u;
        const int nx = next_coded_local(mask, p);
        const uint64_t nxt = (nx < count) ? (uint64_t)(start + nx) : (uint64_t)next_tile_px;
        run = nxt - (uint64_t)(start + p) - 1;
        if (run > 0) {
          uint64_t m = run - 1;
          while (true) {
            nb += tbl[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)] & 31u;
            if (m < 8) break;
            m >>= 3;
          }
        }
      }
      // block-wide exclusive scan of this round's pixel bit lengths
      uint32_t x = nb;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y2 = __shfl_up(x, o);
        if (lane >= o) x += y2;
      }
      if (lane == 63) wsum[wid] = x;
      __syncthreads();
      uint32_t wbase = 0, rtotal = 0;
#pragma unroll
      for (int w = 0; w < ENC_THREADS / 64; ++w) {
        const uint32_t ws = wsum[w];
        wbase += (w < wid) ? ws : 0u;
        rtotal += ws;
      }
      const uint32_t excl = round_base + wbase + x - nb;
      round_base += rtotal;
      __syncthreads();
      // assemble this pixel's bits (MSB-first) into the tile buffer
      if (nb) {
        uint64_t pos = excl;
        uint32_t e = tbl[BIN_PREFIX + sy.mode];
        or_bits(bits, pos, e >> 5, e & 31u);
        pos += e & 31u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if ((uint32_t)k < sy.n) {
            e = tbl[sy.b[k]];
            or_bits(bits, pos, e >> 5, e & 31u);
            pos += e & 31u;
          }
        }
        if (run > 0) {
          uint64_t m = run - 1;
          while (true) {
            e = tbl[BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u)];
            or_bits(bits, pos, e >> 5, e & 31u);
            pos += e & 31u;
            if (m < 8) break;
            m >>= 3;
          }
        }
      }
    }
    const uint32_t tile_bits = round_base;
    __syncthreads();

    if (wid == 0) {
      // local last 32 bits
      uint32_t suf = 0;
      if (tile_bits > 0) {
        const uint32_t endw = (tile_bits - 1) >> 5;
        const uint32_t o = tile_bits & 31;
        if (o == 0) suf = bits[endw];
        else suf = ((endw ? bits[endw - 1] : 0u) << o) | (bits[endw] >> (32 - o));
        if (tile_bits < 32) suf &= (1u << tile_bits) - 1u;
      }
      TileDesc* desc = descs + t;
      uint64_t excl_len;
      uint32_t excl_suf;
      if (tt == 0) {
        excl_len = a.seed_bit[f];
        excl_suf = a.seed_suf[f];
      } else {
        if (lane == 0) {
          st_rlx(&desc->suf_agg, suf);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_rlx64(&desc->flag, ST_AGG | tile_bits);
        }
        look_back(a, t, tt, f, lane, wlen, wsuf, &excl_len, &excl_suf);
      }
      if (lane == 0) {
        uint64_t inc_len = excl_len;
        uint32_t inc_suf = excl_suf;
        suf_combine(inc_len, inc_suf, tile_bits, suf);
        st_rlx(&desc->suf_inc, inc_suf);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_rlx64(&desc->flag, ST_INC | inc_len);
        s_excl_len = excl_len;
        s_excl_suf = excl_suf;
      }
    }
    __syncthreads();
    const uint64_t s0 = s_excl_len;
    const uint32_t suf0 = s_excl_suf;
    const uint64_t e0 = s0 + tile_bits;
    const uint64_t w0 = s0 >> 5, w1 = e0 >> 5;
    const uint32_t sh = (uint32_t)(s0 & 31);
    uint8_t* out = a.out + (uint64_t)f * a.out_stride;
    uint32_t* out32 = reinterpret_cast<uint32_t*>(out);
    // word w0+m = (prev : bits[m]) >> sh, prev = bits[m-1] or the exclusive suffix
    for (uint64_t m = threadIdx.x; m < w1 - w0; m += ENC_THREADS) {
      const uint32_t hi = m ? bits[m - 1] : suf0;
      const uint32_t lo = bits[m];
      const uint32_t v = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
      out32[w0 + m] = __builtin_bswap32(v);
    }
    if (tt == T - 1 && threadIdx.x == 0) {
      // tail: partial word w1, then [P, P, 0, 0, 0] (hfe.rs:115, code.rs:421-422)
      const uint64_t m = w1 - w0;
      const uint32_t hi = m ? bits[m - 1] : suf0;
      const uint32_t lo = bits[m];
      uint32_t v = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
      const uint32_t q = (uint32_t)(e0 & 31);
      v = q ? (v & (0xFFFFFFFFu << (32 - q))) : 0u;
      const uint64_t B = e0 >> 3;              // index of the partial/cache byte
      uint64_t pp = w1 * 4;
      for (; pp < B; ++pp) out[pp] = (uint8_t)(v >> (24 - 8 * (pp - w1 * 4)));
      const uint8_t P = (e0 & 7) ? (uint8_t)(v >> (24 - 8 * (B - w1 * 4))) : 0u;
      out[B] = P;
      out[B + 1] = P;
      out[B + 2] = 0;
      out[B + 3] = 0;
      out[B + 4] = 0;
      a.out_len[f] = B + 5;
    }
    used_words = (uint32_t)(w1 - w0 + 2);
  }
}

// ---------------------------------------------------------------------------
// K6: exact serial replay for flagged frames (emitted code > 25 bits).
// ---------------------------------------------------------------------------
struct GlobalAcc {
  const uint8_t* frame;
  int C;
  uint32_t W;
  int64_t i;
  __device__ __forceinline__ uint32_t operator()(int rows, int px) const {
    const int64_t j = i - ((int64_t)rows * W + px);
    return load_spread(frame, j, C);
  }
};

__global__ __launch_bounds__(64) void enc_serial(EncArgs a) {
  const uint32_t f = blockIdx.x;
  if (!(a.frame_flags[f] & FLAG_SERIAL)) return;
  if (threadIdx.x != 0) return;
  const uint8_t* frame = a.px + (uint64_t)f * a.frame_stride;
  uint8_t* out = a.out + (uint64_t)f * a.out_stride;
  const uint64_t N = (uint64_t)a.W * a.H;
  DevBitwriter bw{out, a.hdr_bytes[f], a.hdr_bitoff[f], a.hdr_cache[f]};
  const uint64_t fb = (uint64_t)f * N_BINS;
  auto emit = [&](uint32_t bin) {
    // write_24bits(aob, code as u32) with the full u8 length and usize code
    const uint8_t aob = a.tbl_len8[fb + bin];
    bw.write_24bits(aob, a.tbl_code[fb + bin]);
  };
  uint64_t i = 0;
  while (i < N) {
    PixSyms s;
    GlobalAcc acc{frame, (int)a.C, a.W, (int64_t)i};
    classify<false>((uint32_t)i, a.W, acc, s);
    emit(BIN_PREFIX + s.mode);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((uint32_t)k < s.n) emit(s.b[k]);
    const uint32_t X = acc(0, 0);
    uint64_t j = i + 1;
    while (j < N && load_spread(frame, (int64_t)j, a.C) == X) ++j;
    const uint64_t run = j - i - 1;
    if (run > 0) {
      uint64_t m = run - 1;
      while (true) {
        emit(BIN_PREFIX + P_RUN1 + (uint32_t)(m & 7u));
        if (m < 8) break;
        m >>= 3;
      }
    }
    i = j;
  }
  out[bw.pos] = (uint8_t)(bw.cache >> 24);
  out[bw.pos + 1] = (uint8_t)(bw.cache >> 24);
  out[bw.pos + 2] = (uint8_t)(bw.cache >> 16);
  out[bw.pos + 3] = (uint8_t)(bw.cache >> 8);
  out[bw.pos + 4] = (uint8_t)(bw.cache);
  a.out_len[f] = bw.pos + 5;
}

}  // namespace nice
