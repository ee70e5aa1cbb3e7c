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
  __shared__ uint8_t lbits[N_STREAMS];
  __shared__ uint16_t loff[N_STREAMS];
  if (threadIdx.x == 0) {
    // first-level widths: the full max length where possible, shrinking the
    // widest tables until all ten fit the budget (long codes take the search)
    uint32_t tot = 0;
    for (int st = 0; st < N_STREAMS; ++st) {
      lbits[st] = (uint8_t)min((uint32_t)smax[st], (uint32_t)DEC_LUT_MAX_BITS);
      tot += 1u << lbits[st];
    }
    while (tot > (uint32_t)DEC_LUT_BUDGET) {
      int w = 0;
      for (int st = 1; st < N_STREAMS; ++st) if (lbits[st] > lbits[w]) w = st;
      tot -= 1u << (lbits[w] - 1);
      lbits[w] -= 1;
    }
    uint32_t o = 0;
    for (int st = 0; st < N_STREAMS; ++st) { loff[st] = (uint16_t)o; o += 1u << lbits[st]; }
  }
  __syncthreads();
  if (threadIdx.x < N_STREAMS) {
    const int st = threadIdx.x;
    const int n = stream_size(st), b = stream_base(st);
    const uint32_t mx = smax[st];
    const uint32_t lb = lbits[st];
    uint16_t* lut = T->lut + loff[st];
    T->max_aob[st] = (uint8_t)mx;
    T->lut_bits[st] = (uint8_t)lb;
    T->lut_off[st] = loff[st];
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
        for (uint32_t e = e0; e < e1; ++e) lut[e] = (uint16_t)((sym << 5) | l);
      } else {
        lut[code >> (l - lb)] = 0;   // long-code marker
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
__device__ __forceinline__ uint32_t parse_step(LaneBits& br, const Tab& T, ParseState& ps,
                                               uint64_t& px) {
  const uint32_t sym = lane_symbol(br, T, gs_stream((int)ps.g));
  ps.pos = br.pos;
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
  const uint64_t base = (uint64_t)f * a.max_chunks;
  ParseState ps = in[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  LaneBits br;
  br.p = a.streams + (uint64_t)f * a.stream_stride;
  br.len = len;
  br.seek(ps.pos);
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  const uint64_t N = (uint64_t)a.W * a.H;
  uint64_t px = 0;
  while (ps.pos < end && ps.pos < hard && px <= N) parse_step(br, T, ps, px);
  // pixels this chunk produces from its current entry: exact once entries are final
  a.chunk_px[base + j] = px;
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
  const uint64_t base = (uint64_t)f * a.max_chunks;
  ParseState ps = entry[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  LaneBits br;
  br.p = a.streams + (uint64_t)f * a.stream_stride;
  br.len = len;
  br.seek(ps.pos);
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  uint64_t px = 0;
  const uint64_t N = (uint64_t)a.W * a.H;
  while (ps.pos < end && ps.pos < hard && px <= N) parse_step(br, T, ps, px);
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
// D4: per-pixel records.  With every chunk's entry state and first pixel index
// known, each chunk decodes its symbols again and writes one 32-bit record per
// coded pixel; run pixels keep the REC_RUN fill.  A record says how the pixel
// follows from already decoded pixels (code.rs:579-644):
//   value_c = src_c + c_c (mod 256), c = bits 0..23,
//   src = floor((L + U) / 2) (L on row 0)      kind AVG: SMALL_DIFF, LUMA2, RGB
//   src = pixel i - off(refid)                 kind REF: BACK_REF (refid 0..4),
//                                                        LUMA (refid 5..15)
// ---------------------------------------------------------------------------
constexpr uint32_t REC_RUN = 0xFFFFFFFFu;
constexpr uint32_t REC_REF = 1u << 28;
__host__ __device__ constexpr int ref_rows(int id) { return id < 5 ? br_rows(id) : lr_rows(id - 5); }
__host__ __device__ constexpr int ref_px_off(int id) { return id < 5 ? br_px(id) : lr_px(id - 5); }

__device__ __forceinline__ int make_record(const DecArgs& a, uint64_t q, uint32_t mode, uint32_t s0,
                                           uint32_t s1, uint32_t s2, uint32_t s3, uint32_t* rec) {
  const uint64_t W = a.W;
  const uint64_t y = q / W;
  switch (mode) {
    case P_BACK_REF:
    case P_LUMA: {
      const uint32_t id = mode == P_BACK_REF ? s0 : 5u + s0;
      if ((mode == P_BACK_REF && s0 >= 5) || (mode == P_LUMA && s0 >= 11)) return NICE_E_FORMAT;
      const int64_t off = (int64_t)ref_rows((int)id) * (int64_t)W + ref_px_off((int)id);
      // usize wrap (W < 3) or underflow before the image: the reference panics
      if (off < 0 || (int64_t)q < off) return NICE_E_FORMAT;
      uint32_t c = 0;
      if (mode == P_LUMA) {
        const uint32_t g = (s1 - 32u) & 255u;
        c = ((s2 - 16u + g) & 255u) | (g << 8) | (((s3 - 16u + g) & 255u) << 16);
      }
      *rec = REC_REF | (id << 24) | c;
      return 0;
    }
    case P_SMALL_DIFF: {
      const uint32_t rd = s0 % 7, t1 = s0 / 7;
      *rec = ((rd - 3u) & 255u) | ((((t1 % 7) - 3u) & 255u) << 8) | ((((t1 / 7) - 3u) & 255u) << 16);
      return 0;
    }
    case P_LUMA2: {
      if (y == 0) return NICE_E_FORMAT;   // position - channels*width underflows (code.rs:583)
      const uint32_t g = (s0 - 32u) & 255u;
      *rec = ((s1 - 16u + g) & 255u) | (g << 8) | (((s2 - 16u + g) & 255u) << 16);
      return 0;
    }
    case P_RGB:
      *rec = (s0 & 255u) | ((s1 & 255u) << 8) | ((s2 & 255u) << 16);
      return 0;
    default:
      return NICE_E_FORMAT;
  }
}

__global__ __launch_bounds__(256) void dec_emit(DecArgs a, const ParseState* entry) {
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
  ParseState ps = entry[base + j];
  if (j == 0) { ps.pos = D; ps.g = 0; ps.dk = 0; ps.acc = 0; }
  LaneBits src;
  src.p = a.streams + (uint64_t)f * a.stream_stride;
  src.len = len;
  src.seek(ps.pos);
  const uint64_t end = D + (uint64_t)(j + 1) * DEC_CHUNK_BITS;
  const uint64_t hard = len * 8 + 64;
  uint32_t* rec = a.recs + (uint64_t)f * N;
  const bool strict = (a.flags & NICE_DEC_STRICT_REFERENCE) != 0;
  // the pixel whose payload straddles our entry belongs to the previous chunk
  while (ps.g != 0 && ps.pos < hard) { uint64_t px = 0; parse_step(src, T, ps, px); }
  bool closed = (q == N);                 // a run completed exactly at N earlier
  uint32_t mode = 0, s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  uint64_t cur = 0;
  while (ps.pos < hard) {
    if (ps.g == 0) {
      if (q == N && (ps.dk == 0 || closed)) {
        // every pixel is accounted for; the reference still reads one more prefix
        // (code.rs:660): a run digit there makes it copy past its buffer
        if (strict) {
          uint64_t px = 0;
          const uint32_t sym = parse_step(src, T, ps, px);
          if (sym >= (uint32_t)P_RUN1) set_status(&a.status[f], NICE_E_FORMAT);
        }
        return;
      }
      if (ps.pos >= end) return;          // next chunk continues from here
    }
    const uint32_t g0 = ps.g, dk0 = ps.dk;
    uint64_t px = 0;
    const uint32_t sym = parse_step(src, T, ps, px);
    if (g0 == 0) {
      if (sym >= (uint32_t)P_RUN1) {      // run digit
        if (q == N && dk0 == 0) {         // a digit right after the last pixel
          if (strict) set_status(&a.status[f], NICE_E_FORMAT);
          return;
        }
        q += px;
        if (q > N) { set_status(&a.status[f], NICE_E_FORMAT); return; }
        if (q == N) closed = true;
        continue;
      }
      closed = false;
      mode = sym;
      cur = q;
      q += 1;
      continue;
    }
    switch (g0) {
      case 1: case 2: case 5: case 9: case 10: s0 = sym; break;
      case 3: case 6: case 11: s1 = sym; break;
      case 4: case 7: case 12: s2 = sym; break;
      default: s3 = sym; break;
    }
    if (ps.g == 0) {                       // payload complete
      uint32_t r;
      const int e = make_record(a, cur, mode, s0, s1, s2, s3, &r);
      if (e) { set_status(&a.status[f], e); return; }
      rec[cur] = r;
    }
  }
}

// ---------------------------------------------------------------------------
// D5: reconstruction.
// ---------------------------------------------------------------------------
// Per-channel cyclic interval [lo, lo+len] mod 256 packed as lo | len << 8;
// len 255 = unknown.  A pixel is three of them.
__device__ __forceinline__ uint32_t iv_add(uint32_t a, uint32_t c) {
  return ((a + c) & 255u) | (a & 0xFF00u);
}
__device__ __forceinline__ uint32_t iv_avg(uint32_t l, uint32_t u, uint32_t c) {
  const uint32_t llo = l & 255u, llen = l >> 8;
  uint32_t lo, hi;
  if (llo + llen <= 255u) { lo = (llo + u) >> 1; hi = (llo + llen + u) >> 1; }
  else { lo = u >> 1; hi = (255u + u) >> 1; }   // wrapped interval: hull of both halves
  return ((lo + c) & 255u) | ((hi - lo) << 8);
}
constexpr uint32_t IV_UNKNOWN = 255u << 8;

struct Px3 { uint32_t c0, c1, c2; };
__device__ __forceinline__ uint32_t pack_px(const Px3& p) {
  return (p.c0 & 255u) | ((p.c1 & 255u) << 8) | ((p.c2 & 255u) << 16);
}
__device__ __forceinline__ bool px_exact(const Px3& p) { return ((p.c0 | p.c1 | p.c2) >> 8) == 0; }
__device__ __forceinline__ Px3 px_from(uint32_t v) {
  return Px3{v & 255u, (v >> 8) & 255u, (v >> 16) & 255u};
}
__device__ __forceinline__ Px3 px_unknown() { return Px3{IV_UNKNOWN, IV_UNKNOWN, IV_UNKNOWN}; }
__device__ __forceinline__ Px3 px_add(const Px3& r, uint32_t c) {
  return Px3{iv_add(r.c0, c & 255u), iv_add(r.c1, (c >> 8) & 255u), iv_add(r.c2, (c >> 16) & 255u)};
}
__device__ __forceinline__ Px3 px_avg(const Px3& l, uint32_t U, uint32_t c) {
  return Px3{iv_avg(l.c0, U & 255u, c & 255u), iv_avg(l.c1, (U >> 8) & 255u, (c >> 8) & 255u),
             iv_avg(l.c2, (U >> 16) & 255u, (c >> 16) & 255u)};
}

struct RecLds {
  uint32_t y4tail[4];
  int32_t ref_k[16], ref_d[16];
  int64_t ref_off[16];
  int32_t err;
  uint32_t first3;    // which of pixels 0..2 of the current row are written
  uint32_t pad[2];
};

// Exact packed-RGB arithmetic (R | G<<8 | B<<16), per byte mod 256.
__device__ __forceinline__ uint32_t avg_rgb(uint32_t a, uint32_t b) {
  return (a & b) + (((a ^ b) >> 1) & 0x7F7F7Fu);          // floor((a+b)/2) per byte
}
__device__ __forceinline__ uint32_t add_rgb(uint32_t a, uint32_t c) {
  return (((a & 0x7F7F7Fu) + (c & 0x7F7F7Fu)) ^ ((a ^ c) & 0x808080u)) & 0xFFFFFFu;
}

// Row storage: R rows x W packed RGB (R = 4 for W >= 3, else 8) and the last 3
// pixels of row y-4 (offsets 3W+1, 3W+3).
struct RowCtx {
  uint32_t* ring;
  const uint32_t* y4tail;
  const uint32_t* first3;
  uint32_t W, y, rmask, x0;
  bool spec;          // speculative pass: other segments of this row may be unwritten
  __device__ __forceinline__ uint32_t* row(uint32_t r) const { return ring + (size_t)(r & rmask) * W; }
};

// Pixel at offset off = k*W + d >= 4 before (x, y): 1 known, 0 unknown.
// Same-row targets are pixels 0..2 (offsets W-1, W-3 from the last columns) or,
// with a single segment, this lane's own earlier pixels.
__device__ __forceinline__ int ref_lookup(const RowCtx& rc, uint32_t x, int k, int d, uint32_t* v) {
  int64_t jx = (int64_t)x - d;
  int64_t jy = (int64_t)rc.y - k;
  while (jx < 0) { jx += rc.W; --jy; }
  while (jx >= (int64_t)rc.W) { jx -= rc.W; ++jy; }
  if (jy == (int64_t)rc.y) {
    if (rc.spec && jx < (int64_t)rc.x0 && !(jx < 3 && ((*rc.first3 >> jx) & 1u))) return 0;
    *v = rc.row(rc.y)[jx];
    return 1;
  }
  if (jy >= (int64_t)rc.y - (int64_t)rc.rmask) { *v = rc.row((uint32_t)jy)[jx]; return 1; }
  *v = rc.y4tail[jx - (rc.W - 3)];
  return 1;
}

// Pixels [x0, x_stop) of the current row from their records; r0..r2 are the
// pixels before x0 as intervals.  While any of the last three pixels is not
// exact, cyclic-interval arithmetic tracks the possible values; once they all
// collapse the rest of the segment runs on exact packed-RGB arithmetic.
// Exact results go to the row.  Returns the last segment-local index left
// unknown (-1: none).
__device__ __forceinline__ int run_segment(const RowCtx& rc, const RecLds& L, uint32_t* first3,
                                           const uint32_t* recs, uint32_t x0, uint32_t x_stop,
                                           Px3 r0, Px3 r1, Px3 r2) {
  int last_unknown = -1;
  const uint32_t y = rc.y;
  uint32_t* row = rc.row(y);
  const uint32_t* up = y > 0 ? rc.row(y - 1) : nullptr;
  uint32_t x = x0;
  // ---- interval phase
  while (x < x_stop && !(px_exact(r0) && px_exact(r1) && px_exact(r2))) {
    const uint32_t r = recs[x];
    Px3 v;
    if (r == REC_RUN) {
      v = r0;
    } else if (!(r & REC_REF)) {
      v = y > 0 ? px_avg(r0, up[x], r) : px_add(r0, r);
    } else {
      const int id = (int)((r >> 24) & 15u);
      const int64_t off = L.ref_off[id];
      Px3 src;
      if (off == 0) src = px_from(0u);       // the pixel itself, not yet written (zeroed)
      else if (off == 1) src = r0;
      else if (off == 2) src = r1;
      else if (off == 3) src = r2;
      else {
        uint32_t u;
        src = ref_lookup(rc, x, L.ref_k[id], L.ref_d[id], &u) ? px_from(u) : px_unknown();
      }
      v = px_add(src, r);
    }
    if (px_exact(v)) row[x] = pack_px(v);
    else last_unknown = (int)(x - x0);
    r2 = r1; r1 = r0; r0 = v;
    ++x;
  }
  // ---- exact phase
  uint32_t p1 = pack_px(r0), p2 = pack_px(r1), p3 = pack_px(r2);
  for (; x < x_stop; ++x) {
    const uint32_t r = recs[x];
    uint32_t v;
    if (r == REC_RUN) {
      v = p1;
    } else if (!(r & REC_REF)) {
      v = add_rgb(y > 0 ? avg_rgb(p1, up[x]) : p1, r);
    } else {
      const int id = (int)((r >> 24) & 15u);
      const int64_t off = L.ref_off[id];
      uint32_t src;
      if (off == 0) src = 0u;
      else if (off == 1) src = p1;
      else if (off == 2) src = p2;
      else if (off == 3) src = p3;
      else if (!ref_lookup(rc, x, L.ref_k[id], L.ref_d[id], &src)) {
        // a same-row pixel another lane has not written yet: leave the rest of
        // the segment to the exact fix-up pass
        last_unknown = (int)(x_stop - 1 - x0);
        break;
      }
      v = add_rgb(src, r);
    }
    row[x] = v;
    if (x < 3) atomicOr(first3, 1u << x);
    p3 = p2; p2 = p1; p1 = v;
  }
  return last_unknown;
}

// The row ring lives in LDS when it fits (LDS_ROWS) -- the address space must
// be static: a runtime LDS-or-global pointer compiles to flat_* accesses, and
// every flat access waits for all outstanding global loads.
template <bool LDS_ROWS>
__device__ __forceinline__ void dec_reconstruct_body(const DecArgs& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  RecLds& L = *reinterpret_cast<RecLds*>(smem);
  const uint32_t W = a.W, H = a.H;
  const uint32_t R = W >= 3 ? 4u : 8u;
  const uint32_t kw = (W + 31) / 32;
  static_assert(sizeof(RecLds) <= 512, "host LDS sizing assumes RecLds <= 512 B");
  uint32_t* recbuf = reinterpret_cast<uint32_t*>(smem + 512) + ((kw + 3) & ~3u);   // row records
  uint32_t* ring;
  if constexpr (LDS_ROWS) ring = recbuf + ((W + 3) & ~3u);
  else ring = a.rowbuf + (uint64_t)blockIdx.x * R * W;
  const uint32_t f = blockIdx.x;
  const int lane = threadIdx.x;
  if (a.status[f] != 0) return;
  if (lane < 16) {
    L.ref_k[lane] = ref_rows(lane);
    L.ref_d[lane] = ref_px_off(lane);
    L.ref_off[lane] = (int64_t)ref_rows(lane) * W + ref_px_off(lane);
  }
  if (lane == 0) L.err = 0;
  __syncthreads();
  const uint64_t N = (uint64_t)W * H;
  const uint32_t S = a.seg, nseg = a.nseg;
  const uint32_t* recs = a.recs + (uint64_t)f * N;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint8_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 255 : 0;
  const bool active = (uint32_t)lane < nseg;
  const uint32_t x0 = lane * S;
  const uint32_t x1 = active ? min(x0 + S, W) : x0;
  const uint32_t seglen = x1 - x0;

  unsigned long long t_a = 0, t_b = 0, t_c = 0, t_d = 0;
  for (uint32_t y = 0; y < H; ++y) {
    const unsigned long long c0 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    RowCtx rc{ring, L.y4tail, &L.first3, W, y, R - 1, x0, true};
    if (R == 4 && y >= 4 && lane < 3) L.y4tail[lane] = rc.row(y)[W - 3 + lane];
    if (lane == 0) L.first3 = 0;
    // this row's records, coalesced
    const uint32_t* rrow = recs + (uint64_t)y * W;
    for (uint32_t x = lane; x < W; x += 64) recbuf[x] = rrow[x];
    __syncthreads();
    auto linear_px = [&](int64_t j) -> uint32_t {
      if (j < 0) return 0u;   // pixel 0's left neighbour is itself, not yet written (0)
      const uint64_t jy = (uint64_t)j / W, jx = (uint64_t)j - jy * W;
      return (R == 4 && jy + 4 == y) ? L.y4tail[jx - (W - 3)] : rc.row((uint32_t)jy)[jx];
    };
    Px3 r0, r1, r2;
    if (lane == 0) {
      r0 = px_from(linear_px((int64_t)y * W - 1));
      r1 = px_from(linear_px((int64_t)y * W - 2));
      r2 = px_from(linear_px((int64_t)y * W - 3));
    } else {
      r0 = px_unknown(); r1 = px_unknown(); r2 = px_unknown();
    }
    const unsigned long long c1 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    // speculative pass: lane 0 starts exact, the others from an unknown entry
    int last_unknown = -1;
    if (active) last_unknown = run_segment(rc, L, &L.first3, recbuf, x0, x1, r0, r1, r2);
    // fix-up rounds: an unconverged segment is recomputed exactly as soon as the
    // three pixels before it are exact (left segment converged before its last
    // three pixels, or already fixed) -- normally all in one parallel round
    unsigned long long fin = __ballot(!active || last_unknown < 0);
    unsigned long long tail_ok = __ballot(!active || last_unknown < 0 ||
                                          (seglen >= 3 && last_unknown < (int)seglen - 3));
    if (a.stats && lane == 0) {
      atomicAdd(&a.stats[0], 1ull);
      atomicAdd(&a.stats[1], (unsigned long long)__popcll(~fin));
      atomicAdd(&a.stats[2], (unsigned long long)__popcll(~tail_ok));
    }
    if (a.stats && active && last_unknown >= 0) atomicAdd(&a.stats[3], (unsigned long long)(last_unknown + 1));
    __syncthreads();
    const unsigned long long c2 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    rc.spec = false;
    while (fin != ~0ull) {
      const bool mine = !((fin >> lane) & 1ull);
      const bool left_ok = lane == 0 || (((fin | tail_ok) >> (lane - 1)) & 1ull);
      const bool ready = mine && left_ok;
      if (ready) {
        r0 = px_from(linear_px((int64_t)y * W + x0 - 1));
        r1 = px_from(linear_px((int64_t)y * W + x0 - 2));
        r2 = px_from(linear_px((int64_t)y * W + x0 - 3));
        const int lu = run_segment(rc, L, &L.first3, recbuf, x0, x0 + (uint32_t)last_unknown + 1,
                                   r0, r1, r2);
        if (lu >= 0) atomicCAS(&L.err, 0, NICE_E_FORMAT);   // exact inputs give exact outputs
        last_unknown = -1;
      }
      __syncthreads();
      fin |= __ballot(ready);
      tail_ok |= fin;
      if (a.stats && lane == 0) atomicAdd(&a.stats[4], 1ull);
    }
    __syncthreads();
    const unsigned long long c3 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    if (L.err) break;
    // emit the row in the caller's pixel format
    uint8_t* orow = outp + (uint64_t)y * W * OC;
    const uint32_t* row = rc.row(y);
    if (OC == 4) {
      uint32_t* o32 = reinterpret_cast<uint32_t*>(orow);
      for (uint32_t x = lane; x < W; x += 64) o32[x] = row[x] | ((uint32_t)alpha << 24);
    } else {
      for (uint32_t x = lane; x < W; x += 64) {
        const uint32_t v = row[x];
        uint8_t* o = orow + (uint64_t)x * 3;
        o[0] = (uint8_t)v; o[1] = (uint8_t)(v >> 8); o[2] = (uint8_t)(v >> 16);
      }
    }
    __syncthreads();
    if (a.stats) {
      const unsigned long long c4 = __builtin_amdgcn_s_memtime();
      t_a += c1 - c0; t_b += c2 - c1; t_c += c3 - c2; t_d += c4 - c3;
    }
  }
  if (a.stats && lane == 0) {
    atomicAdd(&a.stats[5], t_a); atomicAdd(&a.stats[6], t_b);
    atomicAdd(&a.stats[7], t_c); atomicAdd(&a.stats[8], t_d);
  }
  if (lane == 0 && L.err) set_status(&a.status[f], L.err);
}

__global__ __launch_bounds__(64) void dec_reconstruct(DecArgs a) {
  if (a.rows_in_lds) dec_reconstruct_body<true>(a);
  else dec_reconstruct_body<false>(a);
}

}  // namespace nice
