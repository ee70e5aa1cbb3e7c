// nice_decode.hip -- MI355X (gfx950) decoder for the NICE2 bitstream.
//
// The reference decoder (code.rs:464-687) is one serial loop: a single
// context-switched Huffman stream (10 tables, grammar of code.rs:576-671) and a
// raster recurrence in which every pixel depends on its left neighbour (linear
// i-1, wrapping across rows) and on pixels up to 3W+3 back.  The GPU path splits
// it into:
//   dec_tables       header (code.rs:469-483), the 10 length tables
//                    (hfe.rs:173-190), canonical codes (hfe.rs:255-296) and a
//                    2-level lookup equivalent to the reference 2^max LUT.
//   dec_sync         chunk-parallel speculative parse: every CHUNK_BITS slice is
//                    decoded from a guessed entry state; exits become the next
//                    slice's entry (Jacobi iteration) until a fixpoint -- Huffman
//                    self-synchronisation makes this converge in a few passes.
//   dec_count        pixels produced per chunk (coded pixels + run lengths).
//   dec_scan         exclusive scan of those counts per frame.
//   dec_bounds       parse state at every row-segment start (pixel y*W + s*SEG).
//   dec_reconstruct  one wave per frame, rows in order, one lane per row segment:
//                    segments start from an unknown entry tracked as per-channel
//                    cyclic intervals (exact once they collapse -- the predictors
//                    average with the known row above), then unconverged prefixes
//                    are recomputed exactly in rounds once their left neighbour
//                    segment is final.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nice.h"
#include "nice_bits.hpp"
#include "nice_format.h"
#include "nice_kernels.h"

namespace nice {

// ---------------------------------------------------------------------------
// status helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ void set_status(int32_t* st, int32_t code) {
  atomicCAS(reinterpret_cast<int*>(st), 0, code);
}

// ---------------------------------------------------------------------------
// D0: tables. One block of 256 threads per frame.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dec_tables(DecArgs a) {
  __shared__ uint8_t lens[N_BINS];
  __shared__ uint8_t smax[N_STREAMS];
  __shared__ uint16_t order[N_BINS];
  __shared__ int bad;
  const uint32_t f = blockIdx.x;
  const uint8_t* s = a.streams + (uint64_t)f * a.stream_stride;
  const uint64_t len = a.stream_len[f];
  DecTables* T = reinterpret_cast<DecTables*>(a.tables) + f;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  if (len < (uint64_t)FILE_HEADER_BYTES + (TABLE_HEADER_BITS + 7) / 8) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_FORMAT);
    return;
  }
  // header: width/height must match the batch shape; channels byte 3 (reference
  // stride) or 4 (evident intent: RGBA with alpha not coded)
  const uint32_t w = ((uint32_t)s[4] << 24) | ((uint32_t)s[5] << 16) | ((uint32_t)s[6] << 8) | s[7];
  const uint32_t h = ((uint32_t)s[8] << 24) | ((uint32_t)s[9] << 16) | ((uint32_t)s[10] << 8) | s[11];
  const uint32_t ch = s[12];
  if (w != a.W || h != a.H) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_ARG);
    return;
  }
  if (ch != 3 && !(ch == 4 && !(a.flags & NICE_DEC_STRICT_REFERENCE))) {
    // code.rs:659 advances by 3 bytes while every other offset uses `channels`:
    // only channels == 3 decodes in the reference.
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_UNSUPPORTED);
    return;
  }
  BitSrc src{s, len};
  // Decoder side field widths are fixed: a 5-bit max (<= 31) always selects
  // 7-bit length fields (hfe.rs:177-178).
  for (int st = threadIdx.x; st < N_STREAMS; st += 256) {
    uint32_t pos = FILE_HEADER_BYTES * 8;
    for (int q = 0; q < st; ++q) pos += 5 + 7 * stream_size(q);
    smax[st] = (uint8_t)(src.peek32(pos) >> 27);
  }
  for (int st = 0; st < N_STREAMS; ++st) {
    uint32_t pos = FILE_HEADER_BYTES * 8;
    for (int q = 0; q < st; ++q) pos += 5 + 7 * stream_size(q);
    pos += 5;
    for (int i = threadIdx.x; i < stream_size(st); i += 256)
      lens[stream_base(st) + i] = (uint8_t)(src.peek32(pos + 7u * i) >> 25);
  }
  __syncthreads();
  // validity: every length in [1, max], max attained, Kraft sum == 1
  if (threadIdx.x < N_STREAMS) {
    const int st = threadIdx.x;
    const uint32_t mx = smax[st];
    uint64_t kraft = 0;
    uint32_t seen = 0;
    bool ok = mx >= 1 && mx <= 31;
    for (int i = 0; i < stream_size(st) && ok; ++i) {
      const uint32_t l = lens[stream_base(st) + i];
      if (l < 1 || l > mx) ok = false;
      else { kraft += 1ull << (mx - l); seen = max(seen, l); }
    }
    if (!ok || seen != mx || kraft != (1ull << mx)) atomicOr(&bad, 1);
    // strict: a max length above 24 lets the reference refill loop wrap its u8
    // bit offset and spin forever (bitreader.rs:88-97): outside its domain
    if ((a.flags & NICE_DEC_STRICT_REFERENCE) && mx > 24) atomicOr(&bad, 1);
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_UNSUPPORTED);
    return;
  }
  // canonical order per stream: rank by (len desc, symbol desc)
  for (int st = 0; st < N_STREAMS; ++st) {
    const int n = stream_size(st), b = stream_base(st);
    for (int i = threadIdx.x; i < n; i += 256) {
      const uint8_t li = lens[b + i];
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        const uint8_t lj = lens[b + j];
        rank += (lj > li) || (lj == li && j > i);
      }
      order[b + rank] = (uint16_t)i;
    }
  }
  __syncthreads();
  if (threadIdx.x < N_STREAMS) {
    const int st = threadIdx.x;
    const int n = stream_size(st), b = stream_base(st);
    const uint32_t mx = smax[st];
    const uint32_t lb = mx < (uint32_t)DEC_LUT_BITS ? mx : (uint32_t)DEC_LUT_BITS;
    T->max_aob[st] = (uint8_t)mx;
    T->lut_bits[st] = (uint8_t)lb;
    unsigned long long cur = 0;
    uint32_t prev = 0;
    for (int k = 0; k < n; ++k) {
      const int sym = order[b + k];
      const uint32_t l = lens[b + sym];
      if (l < prev) cur >>= (prev - l);
      if (prev > 0) cur += 1;
      const uint32_t code = (uint32_t)((1ull << l) - cur - 1ull);
      prev = l;
      T->lo[b + k] = code << (mx - l);
      T->sym[b + k] = (uint16_t)sym;
      T->len[b + k] = (uint8_t)l;
      // first-level entries
      if (l <= lb) {
        const uint32_t e0 = code << (lb - l), e1 = (code + 1) << (lb - l);
        for (uint32_t e = e0; e < e1; ++e) T->lut[st][e] = (uint16_t)((sym << 5) | l);
      } else {
        T->lut[st][code >> (l - lb)] = 0;   // long-code marker
      }
    }
  }
  if (threadIdx.x == 0) a.data_start[f] = FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS;
}

// Table copy into LDS (all threads of the block participate).
__device__ inline void load_tables(DecTables& dst, const DecTables* src) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(&dst);
  for (uint32_t i = threadIdx.x; i < sizeof(DecTables) / 4; i += blockDim.x) d[i] = s[i];
}

// One parse step (one symbol) of the grammar.  Updates the state and the pixel
// contribution; returns the symbol.  Run digits contribute d << 3k (+1 for the
// first digit), so per-chunk pixel counts are additive.
template <class Tab>
__device__ __forceinline__ uint32_t parse_step(const BitSrc& src, const Tab& T, ParseState& ps,
                                               uint64_t& px) {
  uint64_t pos = ps.pos;
  const uint32_t sym = dec_symbol(src, T, gs_stream((int)ps.g), &pos);
  ps.pos = pos;
  if (ps.g == 0) {
    if (sym >= (uint32_t)P_RUN1) {
      const uint32_t d = sym - P_RUN1;
      const uint32_t sh = (3u * ps.dk) & 63u;      // temp_curr_runcount u8 += 3, masked shift
      px += ((uint64_t)d << sh) + (ps.dk == 0 ? 1u : 0u);
      ps.acc += (uint64_t)d << sh;
      ps.dk += 1;
    } else {
      px += 1;
      ps.dk = 0;
      ps.acc = 0;
      ps.g = (uint32_t)gs_first((int)sym);
    }
  } else {
    ps.g = gs_last((int)ps.g) ? 0u : ps.g + 1u;
  }
  return sym;
}

__device__ __forceinline__ bool state_eq(const ParseState& x, const ParseState& y) {
  return x.pos == y.pos && x.g == y.g && x.dk == y.dk && x.acc == y.acc;
}

// chunk geometry: chunk j of frame f covers bits [D + j*CB, D + (j+1)*CB)
__device__ __forceinline__ uint32_t n_chunks(uint64_t len, uint64_t D) {
  const uint64_t bits = len * 8;
  return bits > D ? (uint32_t)((bits - D + DEC_CHUNK_BITS - 1) / DEC_CHUNK_BITS) : 0u;
}

// Initial entry guesses: every chunk starts at its first bit expecting a prefix.
__global__ __launch_bounds__(256) void dec_init_entries(DecArgs a, ParseState* e) {
  const uint32_t f = blockIdx.y;
  const uint64_t D = FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < a.max_chunks; j += gridDim.x * 256) {
    ParseState& p = e[(uint64_t)f * a.max_chunks + j];
    p.pos = D + (uint64_t)j * DEC_CHUNK_BITS;
    p.g = 0;
    p.dk = 0;
    p.acc = 0;
  }
}

// ---------------------------------------------------------------------------
// D1: sync iteration.  grid = n_frames * chunk_blocks, 256 threads, thread per
// chunk.  Reads entries from `in`, writes exits into `out` (entry of j+1).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dec_sync(DecArgs a, const ParseState* in, ParseState* out,
                                                uint32_t* changed) {
  __shared__ DecTables T;
  const uint32_t f = blockIdx.x / a.chunk_blocks;
  const uint32_t jb = blockIdx.x % a.chunk_blocks;
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D);
  if (jb * 256u >= nc) return;
  load_tables(T, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  const uint32_t j = jb * 256u + threadIdx.x;
  if (j >= nc) return;
  BitSrc src{a.streams + (uint64_t)f * a.stream_stride, len};
  const uint64_t base = (uint64_t)f * a.max_chunks;
  ParseState ps = in[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  uint64_t px = 0;
  while (ps.pos < end && ps.pos < hard) parse_step(src, T, ps, px);
  if (j + 1 < nc) {
    const ParseState old = in[base + j + 1];
    out[base + j + 1] = ps;
    if (!state_eq(old, ps)) atomicOr(changed, 1u);
  }
  if (j == 0) out[base] = in[base];
}

// ---------------------------------------------------------------------------
// D2: pixels per chunk (entries final).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dec_count(DecArgs a, const ParseState* entry) {
  __shared__ DecTables T;
  const uint32_t f = blockIdx.x / a.chunk_blocks;
  const uint32_t jb = blockIdx.x % a.chunk_blocks;
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D);
  if (jb * 256u >= nc) return;
  load_tables(T, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  const uint32_t j = jb * 256u + threadIdx.x;
  if (j >= nc) return;
  BitSrc src{a.streams + (uint64_t)f * a.stream_stride, len};
  const uint64_t base = (uint64_t)f * a.max_chunks;
  ParseState ps = entry[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  uint64_t px = 0;
  const uint64_t N = (uint64_t)a.W * a.H;
  while (ps.pos < end && ps.pos < hard && px <= N) parse_step(src, T, ps, px);
  a.chunk_px[base + j] = px;
}

// ---------------------------------------------------------------------------
// D3: exclusive scan of chunk pixel counts, one 1024-thread block per frame.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void dec_scan(DecArgs a) {
  __shared__ unsigned long long part[1024];
  const uint32_t f = blockIdx.x;
  if (a.status[f] != 0) return;
  const uint32_t nc = n_chunks(a.stream_len[f], a.data_start[f]);
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t per = (nc + 1023) / 1024;
  const uint32_t c0 = threadIdx.x * per, c1 = min(c0 + per, nc);
  unsigned long long sum = 0;
  for (uint32_t j = c0; j < c1; ++j) {
    const unsigned long long v = a.chunk_px[base + j];
    sum = (sum + v < sum) ? ~0ull : sum + v;   // saturate (garbage past the image end)
  }
  part[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    unsigned long long v = part[threadIdx.x];
    if ((int)threadIdx.x >= d) {
      const unsigned long long u = part[threadIdx.x - d];
      v = (v + u < v) ? ~0ull : v + u;
    }
    __syncthreads();
    part[threadIdx.x] = v;
    __syncthreads();
  }
  unsigned long long run = threadIdx.x ? part[threadIdx.x - 1] : 0ull;
  for (uint32_t j = c0; j < c1; ++j) {
    a.chunk_start[base + j] = run;
    const unsigned long long v = a.chunk_px[base + j];
    run = (run + v < run) ? ~0ull : run + v;
  }
  if (threadIdx.x == 1023) {
    // total must cover the image
    if (part[1023] < (unsigned long long)a.W * a.H) set_status(&a.status[f], NICE_E_FORMAT);
  }
}

// ---------------------------------------------------------------------------
// D4: parse state at row-segment starts.  bounds[y*nseg + s] = {pos, run}:
// run > 0: the segment starts with `run` copies of its left neighbour, then the
// next coded pixel's prefix is at pos; run == 0: a coded pixel's prefix at pos.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void put_bound(const DecArgs& a, uint64_t fb, uint64_t b, uint64_t pos,
                                          uint64_t run) {
  const uint64_t y = b / a.W, x = b - y * a.W;
  if (x % a.seg != 0) return;
  SegBound* B = reinterpret_cast<SegBound*>(a.bounds) + fb + y * a.nseg + x / a.seg;
  B->pos = pos;
  B->run = run;
}

__device__ inline void put_run_bounds(const DecArgs& a, uint64_t fb, uint64_t first, uint64_t endx,
                                      uint64_t pos) {
  // boundaries b in [first, endx): run remaining = endx - b
  uint64_t y = first / a.W;
  for (; y * a.W < endx; ++y) {
    const uint64_t row0 = y * a.W;
    uint64_t xlo = first > row0 ? first - row0 : 0;
    const uint64_t xhi = min((uint64_t)a.W, endx - row0);
    uint64_t s = (xlo + a.seg - 1) / a.seg;
    for (uint64_t x = s * a.seg; x < xhi; x += a.seg) {
      SegBound* B = reinterpret_cast<SegBound*>(a.bounds) + fb + y * a.nseg + x / a.seg;
      B->pos = pos;
      B->run = endx - (row0 + x);
    }
  }
}

__global__ __launch_bounds__(256) void dec_bounds(DecArgs a, const ParseState* entry) {
  __shared__ DecTables T;
  const uint32_t f = blockIdx.x / a.chunk_blocks;
  const uint32_t jb = blockIdx.x % a.chunk_blocks;
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D);
  if (jb * 256u >= nc) return;
  load_tables(T, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  const uint32_t j = jb * 256u + threadIdx.x;
  if (j >= nc) return;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint64_t N = (uint64_t)a.W * a.H;
  uint64_t q = a.chunk_start[base + j];   // pixels accounted before this chunk
  if (q > N) return;                      // past the image: tail bytes
  BitSrc src{a.streams + (uint64_t)f * a.stream_stride, len};
  ParseState ps = entry[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  const uint64_t fb = (uint64_t)f * a.H * a.nseg;
  const bool strict = (a.flags & NICE_DEC_STRICT_REFERENCE) != 0;
  // a run whose digits brought the count to N was closed by the chunk that read them
  bool closed = (q == N);
  while (ps.pos < hard) {
    if (q == N && ps.g == 0 && (ps.dk == 0 || closed)) {
      // every pixel is accounted for; the reference still reads one more prefix
      // (code.rs:660): if it is a run digit the reference copies past its buffer
      if (strict) {
        uint64_t px = 0;
        const uint32_t sym = parse_step(src, T, ps, px);
        if (sym >= (uint32_t)P_RUN1) set_status(&a.status[f], NICE_E_FORMAT);
      }
      return;
    }
    if (ps.pos >= end) return;
    const uint64_t at = ps.pos;
    const uint32_t g0 = ps.g, dk0 = ps.dk;
    const uint64_t acc0 = ps.acc;
    uint64_t px = 0;
    const uint32_t sym = parse_step(src, T, ps, px);
    if (g0 != 0) continue;                 // payload symbol
    if (sym >= (uint32_t)P_RUN1) {         // run digit
      if (q == N && dk0 == 0) {            // digit right after the last pixel
        if (strict) set_status(&a.status[f], NICE_E_FORMAT);
        return;
      }
      q += px;
      if (q > N) { set_status(&a.status[f], NICE_E_FORMAT); return; }
      if (q == N) {                         // the final run reaches the image end
        put_run_bounds(a, fb, N - (ps.acc + 1), N, ps.pos);
        closed = true;
      }
      continue;
    }
    // a pixel prefix: closes the previous pixel's run
    if (dk0 > 0 && !closed) put_run_bounds(a, fb, q - (acc0 + 1), q, at);
    closed = false;
    put_bound(a, fb, q, at, 0);
    q += 1;
  }
}

// ---------------------------------------------------------------------------
// D5: reconstruction.
// ---------------------------------------------------------------------------
struct Ival {       // cyclic interval [lo, lo+len] mod 256; len 255 = unknown
  uint32_t lo, len;
};
__device__ __forceinline__ Ival iv_exact(uint32_t v) { return Ival{v & 255u, 0u}; }
__device__ __forceinline__ Ival iv_add(Ival a, uint32_t c) { return Ival{(a.lo + c) & 255u, a.len}; }
__device__ __forceinline__ Ival iv_avg(Ival l, uint32_t u, uint32_t c) {
  uint32_t lo, hi;
  if (l.lo + l.len <= 255u) { lo = (l.lo + u) >> 1; hi = (l.lo + l.len + u) >> 1; }
  else { lo = u >> 1; hi = (255u + u) >> 1; }
  return Ival{(lo + c) & 255u, hi - lo};
}
constexpr Ival IV_UNKNOWN = {0u, 255u};

struct Px3 { Ival c[3]; };

__device__ __forceinline__ uint32_t pack_px(const Px3& p) {
  return p.c[0].lo | (p.c[1].lo << 8) | (p.c[2].lo << 16);
}
__device__ __forceinline__ bool px_exact(const Px3& p) {
  return (p.c[0].len | p.c[1].len | p.c[2].len) == 0;
}
__device__ __forceinline__ Px3 px_from(uint32_t v) {
  Px3 p;
  p.c[0] = iv_exact(v & 255u); p.c[1] = iv_exact((v >> 8) & 255u); p.c[2] = iv_exact((v >> 16) & 255u);
  return p;
}
__device__ __forceinline__ Px3 px_unknown() {
  Px3 p; p.c[0] = IV_UNKNOWN; p.c[1] = IV_UNKNOWN; p.c[2] = IV_UNKNOWN; return p;
}

struct RecLds {
  DecTables T;
  uint32_t y4tail[4];
  uint32_t fin;             // bitmask of final segments (<= 64 segments: lo/hi words)
  uint32_t fin_hi;
  int32_t err;
};

// Resolve a reference at linear offset off = k*W + d from pixel (x, y).
// Returns true with the packed value if it is known, false if unknown.
struct RowCtx {
  uint32_t* ring;           // R rows x W (packed RGB), R = 4 for W >= 3 else 8
  uint32_t* known;          // W bits for the current row
  const uint32_t* y4tail;   // last 3 pixels of row y-4 at [W-3..W-1] -> [0..2]
  uint32_t W, y, rmask;     // rmask = R - 1
  bool same_row_ok;         // far same-row reads allowed (rows in LDS, or after a barrier)
  __device__ __forceinline__ uint32_t* row(uint32_t r) const { return ring + (size_t)(r & rmask) * W; }
};

__device__ __forceinline__ int ref_lookup(const RowCtx& rc, uint32_t x, int k, int d, uint32_t* v) {
  // returns 1: value in *v; 0: unknown; -1: invalid (before the image)
  int64_t jx = (int64_t)x - d;
  int64_t jy = (int64_t)rc.y - k;
  while (jx < 0) { jx += rc.W; --jy; }
  while (jx >= (int64_t)rc.W) { jx -= rc.W; ++jy; }
  if (jy < 0) return -1;
  if (jy == (int64_t)rc.y) {
    if (!rc.same_row_ok || !((rc.known[jx >> 5] >> (jx & 31)) & 1u)) return 0;
    *v = rc.row(rc.y)[jx];
    return 1;
  }
  if (jy >= (int64_t)rc.y - (int64_t)rc.rmask) { *v = rc.row((uint32_t)jy)[jx]; return 1; }
  // row y-4 with R = 4: only the last 3 columns are reachable (offsets 3W+1, 3W+3)
  *v = rc.y4tail[jx - (rc.W - 3)];
  return 1;
}

// Decode one pixel (coded or run member) into intervals.  recent[0..2] hold
// pixels i-1, i-2, i-3.  Returns 0 on success, negative error code.
template <class Tab>
__device__ __forceinline__ int rec_pixel(const BitSrc& src, const Tab& T, const RowCtx& rc, uint32_t x,
                                         uint64_t& pos, uint64_t& run, const Px3 recent[3], Px3& out,
                                         uint64_t N, uint64_t i) {
  if (run > 0) {
    out = recent[0];
    --run;
    return 0;
  }
  uint64_t p = pos;
  const uint32_t mode = dec_symbol(src, T, S_PREFIX, &p);
  const uint32_t y = rc.y;
  const bool has_up = y > 0;
  uint32_t U = 0;
  if (has_up) U = rc.row(y - 1)[x];
  switch (mode) {
    case P_BACK_REF: {
      const uint32_t k = dec_symbol(src, T, S_BACK_REF, &p);
      if (k >= 5) return NICE_E_FORMAT;
      const int rk = br_rows((int)k), dk = br_px((int)k);
      const int64_t off = (int64_t)rk * rc.W + dk;
      if ((int64_t)i < off || off < 0) return NICE_E_FORMAT;   // code.rs:634 underflow
      if (off == 0) { out = px_from(0u); break; }   // self copy of a fresh (zeroed) pixel
      if (off <= 3) { out = recent[off - 1]; break; }
      uint32_t v;
      const int r = ref_lookup(rc, x, rk, dk, &v);
      if (r < 0) return NICE_E_FORMAT;
      out = r ? px_from(v) : px_unknown();
      break;
    }
    case P_SMALL_DIFF: {
      const uint32_t sd = dec_symbol(src, T, S_SMALL_DIFF, &p);
      const int rd = (int)(sd % 7), t1 = (int)(sd / 7);
      const int gd = t1 % 7, bd = t1 / 7;
      const int dd[3] = {rd - 3, gd - 3, bd - 3};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const uint32_t cc = (uint32_t)dd[c] & 255u;
        out.c[c] = has_up ? iv_avg(recent[0].c[c], (U >> (8 * c)) & 255u, cc) : iv_add(recent[0].c[c], cc);
      }
      break;
    }
    case P_LUMA2: {
      if (!has_up) return NICE_E_FORMAT;
      const uint32_t gs = dec_symbol(src, T, S_LUMA2_BASE, &p);
      const uint32_t rs = dec_symbol(src, T, S_LUMA2_R, &p);
      const uint32_t bs = dec_symbol(src, T, S_LUMA2_B, &p);
      const uint32_t g = (gs - 32u) & 255u;
      const uint32_t cc[3] = {(rs - 16u + g) & 255u, g, (bs - 16u + g) & 255u};
#pragma unroll
      for (int c = 0; c < 3; ++c) out.c[c] = iv_avg(recent[0].c[c], (U >> (8 * c)) & 255u, cc[c]);
      break;
    }
    case P_LUMA: {
      const uint32_t k = dec_symbol(src, T, S_LUMA_REF, &p);
      if (k >= 11) return NICE_E_FORMAT;
      const uint32_t gs = dec_symbol(src, T, S_LUMA_BASE, &p);
      const uint32_t rs = dec_symbol(src, T, S_LUMA_OTHER, &p);
      const uint32_t bs = dec_symbol(src, T, S_LUMA_OTHER, &p);
      const uint32_t g = (gs - 32u) & 255u;
      const uint32_t cc[3] = {(rs - 16u + g) & 255u, g, (bs - 16u + g) & 255u};
      const int rk = lr_rows((int)k), dk = lr_px((int)k);
      const int64_t off = (int64_t)rk * rc.W + dk;
      if ((int64_t)i < off || off < 0) return NICE_E_FORMAT;  // usize wrap/underflow, code.rs:548,624
      Px3 ref;
      if (off == 0) ref = px_from(0u);   // reads the not-yet-written pixel itself (zeroed)
      else if (off <= 3) ref = recent[off - 1];
      else {
        uint32_t v;
        const int r = ref_lookup(rc, x, rk, dk, &v);
        if (r < 0) return NICE_E_FORMAT;
        ref = r ? px_from(v) : px_unknown();
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) out.c[c] = iv_add(ref.c[c], cc[c]);
      break;
    }
    case P_RGB: {
      const uint32_t r0 = dec_symbol(src, T, S_RGB, &p);
      const uint32_t r1 = dec_symbol(src, T, S_RGB, &p);
      const uint32_t r2 = dec_symbol(src, T, S_RGB, &p);
      const uint32_t cc[3] = {r0, r1, r2};
#pragma unroll
      for (int c = 0; c < 3; ++c)
        out.c[c] = has_up ? iv_avg(recent[0].c[c], (U >> (8 * c)) & 255u, cc[c]) : iv_add(recent[0].c[c], cc[c]);
      break;
    }
    default:
      return NICE_E_FORMAT;   // a run digit where a pixel must start
  }
  // run digits following the pixel (code.rs:660-671)
  uint64_t acc = 0;
  uint32_t dk = 0;
  const uint64_t rem = N - i - 1;       // pixels after this one
  if (rem > 0) {
    while (true) {
      uint64_t p2 = p;
      const uint32_t nx = dec_symbol(src, T, S_PREFIX, &p2);
      if (nx < (uint32_t)P_RUN1) break;
      acc += (uint64_t)(nx - P_RUN1) << ((3u * dk) & 63u);
      ++dk;
      p = p2;
      if (acc + 1 >= rem) break;        // the run reaches the image end
      if (dk > 21) return NICE_E_FORMAT;
    }
    if (dk > 0) {
      run = acc + 1;
      if (run > rem) return NICE_E_FORMAT;
    }
  }
  pos = p;
  return 0;
}

__global__ __launch_bounds__(64) void dec_reconstruct(DecArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  RecLds& L = *reinterpret_cast<RecLds*>(smem);
  const uint32_t W = a.W, H = a.H;
  const uint32_t R = W >= 3 ? 4u : 8u;
  const uint32_t kw = (W + 31) / 32;
  uint32_t* known = reinterpret_cast<uint32_t*>(smem + ((sizeof(RecLds) + 15) & ~15ull));
  uint32_t* ring = a.rows_in_lds ? known + ((kw + 3) & ~3u)
                                 : a.rowbuf + (uint64_t)blockIdx.x * R * W;
  const uint32_t f = blockIdx.x;
  const int lane = threadIdx.x;
  if (a.status[f] != 0) return;
  load_tables(L.T, reinterpret_cast<const DecTables*>(a.tables) + f);
  if (lane == 0) L.err = 0;
  __syncthreads();
  const uint64_t N = (uint64_t)W * H;
  const uint32_t S = a.seg, nseg = a.nseg;
  const uint64_t len = a.stream_len[f];
  BitSrc src{a.streams + (uint64_t)f * a.stream_stride, len};
  const SegBound* bounds = reinterpret_cast<const SegBound*>(a.bounds) + (uint64_t)f * H * nseg;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint8_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 255 : 0;

  for (uint32_t y = 0; y < H; ++y) {
    RowCtx rc{ring, known, L.y4tail, W, y, R - 1, a.rows_in_lds != 0};
    // save row y-4's tail before its ring slot is reused for row y
    if (R == 4 && y >= 4 && lane < 3) L.y4tail[lane] = rc.row(y)[W - 3 + lane];
    for (uint32_t w = lane; w < kw; w += 64) known[w] = 0;
    __syncthreads();

    const bool active = (uint32_t)lane < nseg;
    const uint32_t x0 = lane * S;
    const uint32_t x1 = active ? min(x0 + S, W) : x0;
    uint64_t pos0 = 0, run0 = 0;
    if (active) { pos0 = bounds[(uint64_t)y * nseg + lane].pos; run0 = bounds[(uint64_t)y * nseg + lane].run; }
    // exact pixel at linear index j < y*W + x0 (final rows / final left segments)
    auto linear_px = [&](int64_t j) -> uint32_t {
      if (j < 0) return 0u;   // pixel 0's left neighbour is itself, not yet written (0)
      const uint64_t jy = (uint64_t)j / W, jx = (uint64_t)j - jy * W;
      return (R == 4 && jy + 4 == y) ? L.y4tail[jx - (W - 3)] : rc.row((uint32_t)jy)[jx];
    };
    Px3 recent[3];
    if (lane == 0) {
      // entry = pixels i-1, i-2, i-3 before the row start, all final
      for (int k = 0; k < 3; ++k) recent[k] = px_from(linear_px((int64_t)y * W - 1 - k));
    } else {
      recent[0] = px_unknown(); recent[1] = px_unknown(); recent[2] = px_unknown();
    }
    // speculative pass (lane 0 is exact from the start)
    int last_unknown = -1;
    int err = 0;
    if (active) {
      uint64_t pos = pos0, run = run0;
      for (uint32_t x = x0; x < x1; ++x) {
        Px3 v;
        const uint64_t i = (uint64_t)y * W + x;
        err = rec_pixel(src, L.T, rc, x, pos, run, recent, v, N, i);
        if (err) break;
        if (px_exact(v)) {
          rc.row(y)[x] = pack_px(v);
          atomicOr(&known[x >> 5], 1u << (x & 31));
        } else {
          last_unknown = (int)(x - x0);
        }
        recent[2] = recent[1]; recent[1] = recent[0]; recent[0] = v;
      }
    }
    if (err) atomicCAS(&L.err, 0, err);
    // fix-up rounds: a segment is final once it has no unknown pixel
    unsigned long long fin = __ballot(!active || last_unknown < 0);
    __syncthreads();
    rc.same_row_ok = true;
    while (fin != ~0ull && L.err == 0) {
      const bool mine = !((fin >> lane) & 1ull);
      const bool left_ok = lane == 0 || ((fin >> (lane - 1)) & 1ull);
      const bool ready = mine && left_ok;
      if (ready) {
        for (int k = 0; k < 3; ++k) recent[k] = px_from(linear_px((int64_t)y * W + x0 - 1 - k));
        uint64_t pos = pos0, run = run0;
        for (uint32_t jx = 0; jx <= (uint32_t)last_unknown; ++jx) {
          const uint32_t x = x0 + jx;
          Px3 v;
          const uint64_t i = (uint64_t)y * W + x;
          err = rec_pixel(src, L.T, rc, x, pos, run, recent, v, N, i);
          if (err) break;
          if (!px_exact(v)) { err = NICE_E_FORMAT; break; }   // exact inputs give exact outputs
          rc.row(y)[x] = pack_px(v);
          atomicOr(&known[x >> 5], 1u << (x & 31));
          recent[2] = recent[1]; recent[1] = recent[0]; recent[0] = v;
        }
        if (err) atomicCAS(&L.err, 0, err);
        last_unknown = -1;
      }
      __syncthreads();
      fin |= __ballot(ready);
    }
    __syncthreads();
    if (L.err) break;
    // emit the row in the caller's pixel format
    uint8_t* orow = outp + (uint64_t)y * W * OC;
    for (uint32_t x = lane; x < W; x += 64) {
      const uint32_t v = rc.row(y)[x];
      uint8_t* o = orow + (uint64_t)x * OC;
      o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)(v >> 16);
      if (OC == 4) o[3] = alpha;
    }
    __syncthreads();
  }
  if (lane == 0 && L.err) set_status(&a.status[f], L.err);
}

}  // namespace nice
