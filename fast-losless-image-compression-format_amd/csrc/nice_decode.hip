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
//                    Re-parses stop at the first checkpoint where they agree
//                    with the previous parse; the sync pass also counts pixels.
//   dec_scan         exclusive scan of the pixel counts per frame.
//   dec_emit         one 32-bit record per coded pixel (mode + constants).
//   dec_reconstruct  one wave per frame, rows in order, one lane per row segment:
//                    segments start from an unknown entry tracked as per-channel
//                    cyclic intervals (exact once they collapse -- the predictors
//                    average with the known row above), then unconverged prefixes
//                    are recomputed exactly in rounds once their left neighbour
//                    segment is final.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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

// chunk geometry: chunk j of frame f covers bits [D + j*CB, D + (j+1)*CB)
__device__ __forceinline__ uint32_t n_chunks(uint64_t len, uint64_t D, uint32_t cb) {
  const uint64_t bits = len * 8;
  return bits > D ? (uint32_t)((bits - D + cb - 1) / cb) : 0u;
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
  // the host sized the slice scratch from its copy of the lengths
  // (nice_decode_batch_dev_hl): a device length past that bound or the stream
  // stride fails the frame before any kernel indexes slices by it
  if (len > a.stream_stride ||
      n_chunks(len, FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS, a.chunk_bits) > a.max_chunks) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_ARG);
    return;
  }
  if (ch != 3 && !(ch == 4 && !(a.flags & NICE_DEC_STRICT_REFERENCE))) {
    // code.rs:659 advances by 3 bytes while every other offset uses `channels`:
    // only channels == 3 decodes in the reference.
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_UNSUPPORTED);
    return;
  }
#ifdef NICE_PROF_DTABLES
  long long tp[10];
  int tpn = 0;
#define DT_MARK() do { if (tpn < 10) tp[tpn++] = clock64(); } while (0)
#else
#define DT_MARK() do {} while (0)
#endif
  DT_MARK();
  // the file and table headers (770 bytes) staged in LDS as big-endian words
  // with one load per thread (the fields were ~12 dependent global reads per
  // thread: most of this kernel's time for a single frame)
  constexpr int HDR_WORDS = (FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS + 31) / 32 + 2;
  __shared__ uint32_t hw[HDR_WORDS];
  {
    const BitSrc src{s, len};
    for (int i = threadIdx.x; i < HDR_WORDS; i += 256) hw[i] = src.peek32((uint64_t)i * 32u);
  }
  __syncthreads();
  auto hpeek = [&](uint32_t pos) -> uint32_t {   // 32 bits at header bit pos, MSB first
    const uint32_t wi = pos >> 5, o = pos & 31u;
    return (uint32_t)((((unsigned long long)hw[wi] << 32 | hw[wi + 1]) << o) >> 32);
  };
  // Decoder side field widths are fixed: a 5-bit max (<= 31) always selects
  // 7-bit length fields (hfe.rs:177-178).
  for (int st = threadIdx.x; st < N_STREAMS; st += 256) {
    uint32_t pos = FILE_HEADER_BYTES * 8;
    for (int q = 0; q < st; ++q) pos += 5 + 7 * stream_size(q);
    smax[st] = (uint8_t)(hpeek(pos) >> 27);
  }
  for (int i = threadIdx.x; i < N_BINS; i += 256) {
    int st = 0;
    while (st + 1 < N_STREAMS && i >= stream_base(st + 1)) ++st;
    uint32_t pos = FILE_HEADER_BYTES * 8 + 5;
    for (int q = 0; q < st; ++q) pos += 5 + 7 * stream_size(q);
    lens[i] = (uint8_t)(hpeek(pos + 7u * (uint32_t)(i - stream_base(st))) >> 25);
  }
  __syncthreads();
  DT_MARK();
  const bool tolerant = (a.flags & NICE_DEC_TOLERANT_HEADER) && !(a.flags & NICE_DEC_STRICT_REFERENCE);
  if (tolerant) {
    // Spilled max fields (oracle tolerant_tables): a max above 31
    // keeps its low 5 bits in the field and adds max >> 5 into the p bits still
    // pending in the writer's u32 cache -- the low p bits of the previous
    // stream's last length, p = table-header bits written so far mod 8.  Undo it
    // from the last stream down; the table max becomes the longest decodable
    // (<= 31 bit) length.
    if (threadIdx.x == 0) {
      for (int st = N_STREAMS - 1; st >= 0; --st) {
        const int n = stream_size(st), b = stream_base(st);
        uint32_t mx = 0, dm = 0;
        for (int i = 0; i < n; ++i) {
          const uint32_t l = lens[b + i];
          mx = max(mx, l);
          if (l <= 31) dm = max(dm, l);
        }
        if ((mx & 31u) != smax[st] || mx > 127 || dm == 0) bad = 1;
        if (mx >= 32 && st > 0) {
          uint32_t bits = 0;
          for (int q = 0; q < st; ++q) bits += 5u + 7u * (uint32_t)stream_size(q);
          const uint32_t pm = (1u << (bits & 7u)) - 1u;
          uint8_t& last = lens[stream_base(st - 1) + stream_size(st - 1) - 1];
          last = (uint8_t)((last & ~pm) | ((last - (mx >> 5)) & pm));
        }
        smax[st] = (uint8_t)dm;
      }
    }
    __syncthreads();
    // every stream a complete prefix code over all its lengths (Kraft sum 1)
    if (threadIdx.x < N_STREAMS) {
      const int st = threadIdx.x, n = stream_size(st), b = stream_base(st);
      uint32_t mx = 0;
      bool ok = true;
      for (int i = 0; i < n; ++i) { mx = max(mx, (uint32_t)lens[b + i]); ok = ok && lens[b + i] >= 1; }
      unsigned __int128 kraft = 0;
      for (int i = 0; i < n && ok; ++i) kraft += (unsigned __int128)1 << (mx - lens[b + i]);
      if (!ok || kraft != ((unsigned __int128)1 << mx)) atomicOr(&bad, 1);
    }
  } else {
    // validity: every length in [1, max], max attained, Kraft sum == 1 -- every
    // symbol at once, per-stream sums by LDS atomics (a lane per stream looping
    // over its symbols took ~0.13 ms of a single frame's decode)
    __shared__ unsigned long long vkraft[N_STREAMS];
    __shared__ uint32_t vseen[N_STREAMS];
    if (threadIdx.x < N_STREAMS) { vkraft[threadIdx.x] = 0; vseen[threadIdx.x] = 0; }
    __syncthreads();
    for (int i = threadIdx.x; i < N_BINS; i += 256) {
      int st = 0;
#pragma unroll
      for (int q = 1; q < N_STREAMS; ++q) st += i >= stream_base(q) ? 1 : 0;
      const uint32_t mx = smax[st], l = lens[i];
      if (l < 1 || l > mx || mx > 31) atomicOr(&bad, 1);
      else {
        atomicAdd(&vkraft[st], 1ull << (mx - l));
        atomicMax(&vseen[st], l);
      }
    }
    __syncthreads();
    if (threadIdx.x < N_STREAMS) {
      const int st = threadIdx.x;
      const uint32_t mx = smax[st];
      if (mx < 1 || vseen[st] != mx || vkraft[st] != (1ull << mx)) atomicOr(&bad, 1);
      // strict: tables of 26..31 bits can make the reference's refill loop wrap
      // its u8 bit offset (bitreader.rs:88-97); dec_strict_refill finds the reads
      // where it does
    }
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_UNSUPPORTED);
    return;
  }
  DT_MARK();
  // canonical order per stream: rank by (len desc, symbol desc)
  for (int st = 0; st < N_STREAMS; ++st) {
    const int n = stream_size(st), b = stream_base(st);
    for (int i = threadIdx.x; i < n; i += 256) {
      const uint8_t li = lens[b + i];
      int rank = 0;
#pragma unroll 8
      for (int j = 0; j < n; ++j) {   // independent reads: unrolled, batched
        const uint8_t lj = lens[b + j];
        rank += (lj > li) || (lj == li && j > i);
      }
      order[b + rank] = (uint16_t)i;
    }
  }
  __syncthreads();
  DT_MARK();
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
  DT_MARK();
  // canonical codes (hfe.rs:271-290): one lane per stream, serial in LDS; the
  // lengths in rank order first (all threads), so the serial loop reads one
  // independent word per symbol instead of a dependent order -> length chain
  __shared__ uint32_t clo[N_BINS];
  __shared__ uint8_t clen[N_BINS];
  for (int i = threadIdx.x; i < N_BINS; i += 256) {
    int st = 0;
#pragma unroll
    for (int q = 1; q < N_STREAMS; ++q) st += i >= stream_base(q) ? 1 : 0;
    clen[i] = lens[stream_base(st) + order[i]];
  }
  __syncthreads();
  if (threadIdx.x < N_STREAMS) {
    const int st = threadIdx.x;
    const int n = stream_size(st), b = stream_base(st);
    const uint32_t mx = smax[st];
    T->max_aob[st] = (uint8_t)mx;
    T->lut_bits[st] = lbits[st];
    T->lut_off[st] = loff[st];
    // usize wrapping (shift amounts masked to 6 bits); in tolerant mode lengths
    // above 31 (zero-count symbols) get no decode entry (lo above every 31-bit
    // window value) and the decodable codes must fit their lengths and not
    // overlap
    unsigned long long cur = 0;
    uint32_t prev = 0;
    uint64_t prev_lo = ~0ull;
    bool ok = true;
#pragma unroll 4
    for (int k = 0; k < n; ++k) {
      const uint32_t l = clen[b + k];
      if (l < prev) cur >>= (prev - l) & 63u;
      if (prev > 0) cur += 1;
      const unsigned long long code64 = (1ull << (l & 63u)) - cur - 1ull;
      prev = l;
      if (l > mx) { clo[b + k] = 0xFFFFFFFFu; continue; }
      const uint64_t lo = (uint64_t)(uint32_t)code64 << (mx - l);
      if ((code64 >> l) != 0 || (prev_lo != ~0ull && lo + (1ull << (mx - l)) > prev_lo)) ok = false;
      prev_lo = lo;
      clo[b + k] = (uint32_t)lo;
    }
    if (!ok) atomicOr(&bad, 1);
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_UNSUPPORTED);
    return;
  }
  DT_MARK();
  for (int i = threadIdx.x; i < N_BINS; i += 256) {
    T->lo[i] = clo[i];
    T->sym[i] = order[i];
    T->len[i] = clen[i];
  }
  // first-level entries, all streams in parallel: entry e of stream st is the
  // window value x = e << (max - width); the code covering it is the first in
  // canonical order (lower bounds descending) with lo <= x -- a complete,
  // non-overlapping code (checked above) covers every x exactly once.  A code
  // longer than the width leaves the long-code marker 0.
  DT_MARK();
  const uint32_t n_lut = (uint32_t)loff[N_STREAMS - 1] + (1u << lbits[N_STREAMS - 1]);
  __shared__ int lut_hole;
  if (threadIdx.x == 0) lut_hole = 0;
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < n_lut; e += 256) {
    int st = 0;
#pragma unroll
    for (int q = 1; q < N_STREAMS; ++q) st += e >= loff[q] ? 1 : 0;   // independent reads, no search loop
    const uint32_t lb = lbits[st], mx = smax[st];
    const uint32_t x = (e - loff[st]) << (mx - lb);
    int lo = stream_base(st), hi = lo + stream_size(st) - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (clo[mid] <= x) hi = mid;
      else lo = mid + 1;
    }
    const uint32_t l = clen[lo];
    T->lut[e] = l <= lb ? (uint16_t)(((uint32_t)order[lo] << 5) | l) : (uint16_t)0;
    if (l > lb || l == 0) lut_hole = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // longest pixel event: the prefix plus the longest payload sequence (code.rs:576-644)
    const uint32_t m_pay = max(max((uint32_t)smax[S_BACK_REF], 3u * smax[S_RGB]),
                               max((uint32_t)smax[S_LUMA_REF] + smax[S_LUMA_BASE] + 2u * smax[S_LUMA_OTHER],
                                   max((uint32_t)smax[S_SMALL_DIFF],
                                       (uint32_t)smax[S_LUMA2_BASE] + smax[S_LUMA2_R] + smax[S_LUMA2_B])));
    T->fast = (!lut_hole && smax[S_PREFIX] + m_pay <= 64u) ? 1u : 0u;
    a.data_start[f] = FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS;
  }
#ifdef NICE_PROF_DTABLES
  DT_MARK();
  if (threadIdx.x == 0 && f == 0)
    printf("dec_tables cycles: stage+lens %lld valid %lld rank %lld widths %lld canon %lld copy %lld lut %lld (n=%d)\n",
           tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], tp[5] - tp[4], tp[6] - tp[5], tp[7] - tp[6], tpn);
#endif
}

// ---------------------------------------------------------------------------
// Parse machinery shared by dec_sync and dec_emit.
//
// A lane parses one slice of the data bits.  It reads them from a private ring
// of RING_W big-endian words in LDS, refilled for the whole wave at once with
// 16-byte loads (consecutive lanes load consecutive 16 bytes of one ring), so
// the stream is read from HBM in whole lines.  The first-level LUTs and the
// canonical order for long codes live in LDS.
//
// The parse advances one pixel event per step: a prefix symbol, then -- for a
// coded pixel -- the mode's fixed payload sequence (code.rs:576-644): BACK_REF
// k; RGB r g b; LUMA ref, g, r, b; SMALL_DIFF index; LUMA2 g r b.  Slices
// therefore begin and end at prefix positions: a slice's parse stops at the
// first prefix at or after its end bit, which is where the next slice starts.
// ---------------------------------------------------------------------------
#ifndef NICE_RING_W
#define NICE_RING_W 20
#endif
constexpr uint32_t RING_W = NICE_RING_W;   // words per lane ring (a multiple of 4, >= 12)
constexpr uint32_t RING_STRIDE = RING_W;   // 16-byte aligned rings
static_assert(RING_W % 4 == 0 && RING_W >= 12, "ring size");
#ifdef NICE_PARSE_WPE
#define PARSE_ATTR __attribute__((amdgpu_waves_per_eu(NICE_PARSE_WPE)))
#else
#define PARSE_ATTR
#endif
constexpr uint32_t RING_QUADS = RING_W / 4;
constexpr uint32_t PIXEL_WORDS = 5;    // one pixel event: <= 5 symbols of <= 31 bits

constexpr uint32_t PFX_STREAM = S_PREFIX;
// payload stream i of mode m (code.rs:576-644), 4 bits each at 4 * (4m + i)
constexpr unsigned long long PAY_STREAMS =
    ((unsigned long long)S_BACK_REF << 0) |
    ((unsigned long long)S_RGB << 16) | ((unsigned long long)S_RGB << 20) | ((unsigned long long)S_RGB << 24) |
    ((unsigned long long)S_LUMA_REF << 32) | ((unsigned long long)S_LUMA_BASE << 36) |
    ((unsigned long long)S_LUMA_OTHER << 40) | ((unsigned long long)S_LUMA_OTHER << 44) |
    ((unsigned long long)S_SMALL_DIFF << 48);   // mode 4 (LUMA2): pay_stream
static_assert(P_BACK_REF == 0 && P_RGB == 1 && P_LUMA == 2 && P_SMALL_DIFF == 3 && P_LUMA2 == 4 &&
                  P_RUN1 == 5, "prefix numbering");
__device__ __forceinline__ uint32_t pay_stream(uint32_t m, uint32_t i) {
  // mode 4 (LUMA2) does not fit the 64-bit table: handled here
  return m == (uint32_t)P_LUMA2 ? (uint32_t)S_LUMA2_BASE + i : (uint32_t)(PAY_STREAMS >> (4u * (4u * m + i))) & 15u;
}

struct LutLds {
  uint16_t lut[DEC_LUT_BUDGET];
  uint32_t lo[N_BINS];   // canonical order (long codes): aligned lower bounds,
  uint16_t sym[N_BINS];  // symbols and lengths
  uint8_t len[N_BINS];
  uint32_t gp[16];    // per stream: lut_off | lut_bits << 16 | max_aob << 24
  uint32_t gs[16];    // per stream: canonical-order base | alphabet size << 16
  uint4 pp[8];        // fast parse: per prefix 0..4, the fast_param of its payload streams 0..3
};

__device__ inline void load_lut(LutLds& S, const DecTables* T) {
  const uint4* s = reinterpret_cast<const uint4*>(T->lut);
  uint4* d = reinterpret_cast<uint4*>(S.lut);
  for (uint32_t i = threadIdx.x; i < sizeof(S.lut) / 16; i += blockDim.x) d[i] = s[i];
  for (uint32_t i = threadIdx.x; i < N_BINS; i += blockDim.x) {
    S.lo[i] = T->lo[i];
    S.sym[i] = T->sym[i];
    S.len[i] = T->len[i];
  }
  if (threadIdx.x < N_STREAMS) {
    const int st = (int)threadIdx.x;
    S.gp[st] = (uint32_t)T->lut_off[st] | ((uint32_t)T->lut_bits[st] << 16) | ((uint32_t)T->max_aob[st] << 24);
    S.gs[st] = (uint32_t)stream_base(st) | ((uint32_t)stream_size(st) << 16);
  }
  if (threadIdx.x < 8u) {   // payload streams of each mode (code.rs:576-644), as fast parameters
    const uint32_t m = threadIdx.x;
    uint32_t w[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t st = m < 5u ? pay_stream(m, i) : 0u;
      w[i] = (32u - T->lut_bits[st]) | ((uint32_t)T->lut_off[st] << 17);
    }
    S.pp[m] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__device__ __forceinline__ uint32_t stream_word(const uint8_t* p, uint64_t len, uint32_t w) {
  uint32_t v = 0;
  for (int k = 0; k < 4; ++k) {
    const uint64_t i = (uint64_t)w * 4 + k;
    v = (v << 8) | (i < len ? p[i] : (len ? p[len - 1] : 0u));   // stale last byte past the end
  }
  return v;
}

// Lane bit reader over its LDS ring: a left-aligned 64-bit window (next bit at
// bit 63) holding `avail` >= 32 valid bits between symbols.
struct Lane {
  unsigned long long pos;   // absolute bit position in the frame's stream
  unsigned long long win;
  uint32_t avail;
  uint32_t rp;              // next ring word to shift in
  uint32_t ws;              // fast parse: stream word held in ring word 0
};
// one more pixel event fits in the ring
__device__ __forceinline__ bool lane_ok(const Lane& L) { return L.rp + PIXEL_WORDS <= RING_W; }

__device__ __noinline__ void ring_fill_slow(uint32_t* dst, const uint8_t* p, uint64_t len, uint32_t w) {
  dst[0] = stream_word(p, len, w);
  dst[1] = stream_word(p, len, w + 1);
  dst[2] = stream_word(p, len, w + 2);
  dst[3] = stream_word(p, len, w + 3);
}
// Wave-cooperative refill: every lane's ring restarts at the word holding its
// position (rounded down to 16 bytes).  Must be reached by all 64 lanes.
// ws: the (16-byte aligned) stream word each lane's ring restarts at.
__device__ __forceinline__ void ring_fill_ws(uint32_t* wring, const uint8_t* p, uint64_t len, bool al16,
                                             uint32_t ws) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t full_words = al16 ? (len >> 2) : 0;   // words fully inside the stream
  uint4 v[RING_QUADS];
  uint32_t wq[RING_QUADS];
#pragma unroll
  for (uint32_t r = 0; r < RING_QUADS; ++r) {   // issue every load before waiting on any
    const uint32_t i = lane + 64u * r;
    const uint32_t owner = i / RING_QUADS, q = i - owner * RING_QUADS;
    wq[r] = (uint32_t)__shfl((int)ws, (int)owner) + 4u * q;   // all lanes: before any branch
    const uint64_t wl = (uint64_t)wq[r] + 4 <= full_words ? wq[r] : 0u;
    v[r] = *reinterpret_cast<const uint4*>(p + wl * 4);
  }
#pragma unroll
  for (uint32_t r = 0; r < RING_QUADS; ++r) {
    const uint32_t i = lane + 64u * r;
    const uint32_t owner = i / RING_QUADS, q = i - owner * RING_QUADS;
    uint32_t* dst = wring + owner * RING_STRIDE + 4u * q;
    if ((uint64_t)wq[r] + 4 <= full_words) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(__builtin_bswap32(v[r].x), __builtin_bswap32(v[r].y),
                                                  __builtin_bswap32(v[r].z), __builtin_bswap32(v[r].w));
    } else {
      ring_fill_slow(dst, p, len, wq[r]);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
template <bool FAST = false>
__device__ __forceinline__ void ring_fill(uint32_t* wring, const uint8_t* p, uint64_t len, bool al16,
                                          Lane& L) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t ws = (uint32_t)(L.pos >> 5) & ~3u;
  ring_fill_ws(wring, p, len, al16, ws);
  if constexpr (FAST) {
    L.ws = ws;
  } else {
    const uint32_t* my = wring + lane * RING_STRIDE;
    const uint32_t o = (uint32_t)(L.pos >> 5) - ws;
    const uint32_t sh = (uint32_t)(L.pos & 31u);
    L.win = (((unsigned long long)my[o] << 32) | my[o + 1]) << sh;
    L.avail = 64u - sh;
    L.rp = o + 2u;
  }
}

// Fast parse (DecTables::fast): the event's 64 bits are taken from the ring at
// its start and every symbol is one table lookup -- no long codes, no top-up.
__device__ __forceinline__ bool lane_ok_fast(const Lane& L) {
  return ((uint32_t)(L.pos >> 5) - L.ws) + 3u <= RING_W;
}
// Fast-path stream parameter: (32 - table width) | 2 * table offset << 16, so a
// lookup's byte address is ((v >> shift) << 17 + param) >> 16 (shifts use the
// low 5 bits of their operand).
__device__ __forceinline__ uint32_t fast_param(uint32_t gp) {
  return (32u - ((gp >> 16) & 31u)) | ((gp & 0xFFFFu) << 17);
}
__device__ __forceinline__ uint32_t fsym(unsigned long long& win, uint32_t& tot, const LutLds& S, uint32_t fp) {
  const uint32_t v = (uint32_t)(win >> 32);
  const uint32_t byte = (((v >> (fp & 31u)) << 17) + fp) >> 16;
  const uint32_t e = *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(S.lut) + byte);
  const uint32_t n = e & 31u;
  win <<= n;
  tot += n;
  return e >> 5;
}

// Long code (longer than the LUT width): search of the canonical order.
__device__ __forceinline__ uint32_t long_code(const LutLds& S, uint32_t v, uint32_t gp, uint32_t gsz) {
  const uint32_t x = v >> (32u - (gp >> 24));
  int lo = (int)(gsz & 0xFFFFu), hi = lo + (int)(gsz >> 16) - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (S.lo[mid] <= x) hi = mid;
    else lo = mid + 1;
  }
  return ((uint32_t)S.sym[lo] << 5) | (uint32_t)S.len[lo];
}

// One symbol of stream st (gp: S.gp[st], passed in for the prefix stream,
// which a lane reads at every event).
__device__ __forceinline__ uint32_t dsym_gp(Lane& L, const uint32_t* my, const LutLds& S, uint32_t st,
                                            uint32_t gp) {
  const uint32_t v = (uint32_t)(L.win >> 32);
  uint32_t e = S.lut[(gp & 0xFFFFu) + (v >> (32u - ((gp >> 16) & 31u)))];
  if ((e & 31u) == 0) e = long_code(S, v, gp, S.gs[st]);
  const uint32_t n = e & 31u;
  L.pos += n;
  L.win <<= n;
  L.avail -= n;
  // top up to >= 32 bits (branch-free; lane_ok() guarantees the word exists)
  const uint32_t w = my[min(L.rp, RING_W - 1u)];
  const bool need = L.avail < 32u;
  L.win |= need ? ((unsigned long long)w << (32u - L.avail)) : 0ull;
  L.rp += need ? 1u : 0u;
  L.avail += need ? 32u : 0u;
  return e >> 5;
}
// One pixel event at a prefix position: the prefix and, for a coded pixel, its
// payload symbols.  Returns the prefix; s0..s3 receive the payload.
// The frame's stream parameters (S.gp) held in scalar registers: a payload
// symbol's parameters are selected by the prefix instead of read from LDS, so
// its LUT lookup does not wait on a dependent LDS read.
struct StreamParams {
  uint32_t g[N_STREAMS];
  __device__ __forceinline__ void load(const LutLds& S) {
#pragma unroll
    for (int i = 0; i < N_STREAMS; ++i) g[i] = __builtin_amdgcn_readfirstlane(S.gp[i]);
  }
};
__device__ __forceinline__ uint32_t pixel_event(Lane& L, const uint32_t* my, const LutLds& S,
                                                const StreamParams& G, uint32_t& s0, uint32_t& s1, uint32_t& s2,
                                                uint32_t& s3) {
  const uint32_t pfx = dsym_gp(L, my, S, PFX_STREAM, G.g[PFX_STREAM]);
  if (pfx < (uint32_t)P_RUN1) {
    const bool rgb = pfx == (uint32_t)P_RGB, lu = pfx == (uint32_t)P_LUMA, l2 = pfx == (uint32_t)P_LUMA2;
    const uint32_t gp0 = pfx == (uint32_t)P_BACK_REF ? G.g[S_BACK_REF] : rgb ? G.g[S_RGB] : lu ? G.g[S_LUMA_REF]
                       : l2 ? G.g[S_LUMA2_BASE] : G.g[S_SMALL_DIFF];
    s0 = dsym_gp(L, my, S, pay_stream(pfx, 0), gp0);
    if (rgb || lu || l2) {
      s1 = dsym_gp(L, my, S, pay_stream(pfx, 1), rgb ? G.g[S_RGB] : lu ? G.g[S_LUMA_BASE] : G.g[S_LUMA2_R]);
      s2 = dsym_gp(L, my, S, pay_stream(pfx, 2), rgb ? G.g[S_RGB] : lu ? G.g[S_LUMA_OTHER] : G.g[S_LUMA2_B]);
      if (lu) s3 = dsym_gp(L, my, S, S_LUMA_OTHER, G.g[S_LUMA_OTHER]);
    }
  }
  return pfx;
}

// pixel_event on the fast path: one 64-bit window per event (DecTables::fast
// bounds every event by 64 bits), no per-symbol refill.
__device__ __forceinline__ uint32_t pixel_event_fast(Lane& L, const uint32_t* my, const LutLds& S,
                                                     const StreamParams& G, uint32_t& s0, uint32_t& s1,
                                                     uint32_t& s2, uint32_t& s3) {
  const uint32_t o = (uint32_t)(L.pos >> 5) - L.ws;
  const uint32_t sh = (uint32_t)L.pos & 31u;
  const uint32_t w0 = my[o], w1 = my[o + 1], w2 = my[o + 2];
  unsigned long long win = ((((unsigned long long)w0 << 32) | w1) << sh) | (((unsigned long long)w2 << sh) >> 32);
  uint32_t tot = 0;
  const uint32_t pfx = fsym(win, tot, S, G.g[PFX_STREAM]);
  if (pfx < (uint32_t)P_RUN1) {
    const bool rgb = pfx == (uint32_t)P_RGB, lu = pfx == (uint32_t)P_LUMA, l2 = pfx == (uint32_t)P_LUMA2;
    // the mode's payload parameters in one LDS read (selecting them from
    // scalar registers by prefix took a move and a select per candidate)
    const uint4 pp = S.pp[pfx];
    s0 = fsym(win, tot, S, pp.x);
    if (rgb || lu || l2) {
      s1 = fsym(win, tot, S, pp.y);
      s2 = fsym(win, tot, S, pp.z);
      if (lu) s3 = fsym(win, tot, S, pp.w);
    }
  }
  L.pos += tot;
  return pfx;
}

// pixel_event_fast at ring word o, bit sh of it (dec_sync's relative-position
// loop); returns the prefix and the event's bit count in tot.
__device__ __forceinline__ uint32_t pixel_event_fast_at(const uint32_t* my, const LutLds& S, uint32_t fp_pfx,
                                                        uint32_t o, uint32_t sh, uint32_t& s0, uint32_t& s1,
                                                        uint32_t& s2, uint32_t& s3, uint32_t& tot) {
  const uint32_t w0 = my[o], w1 = my[o + 1], w2 = my[o + 2];
  unsigned long long win = ((((unsigned long long)w0 << 32) | w1) << sh) | (((unsigned long long)w2 << sh) >> 32);
  tot = 0;
  const uint32_t pfx = fsym(win, tot, S, fp_pfx);
  if (pfx < (uint32_t)P_RUN1) {
    const bool rgb = pfx == (uint32_t)P_RGB, lu = pfx == (uint32_t)P_LUMA, l2 = pfx == (uint32_t)P_LUMA2;
    const uint4 pp = S.pp[pfx];
    s0 = fsym(win, tot, S, pp.x);
    if (rgb || lu || l2) {
      s1 = fsym(win, tot, S, pp.y);
      s2 = fsym(win, tot, S, pp.z);
      if (lu) s3 = fsym(win, tot, S, pp.w);
    }
  }
  return pfx;
}

// Pixels a prefix accounts for: 1 for a coded pixel; a run digit d contributes
// d << 3k (k = digits read before it; the reference's u8 shift counter `+= 3`
// only matters mod 64) plus the run's first pixel on its first digit
// (code.rs:660-680).  dk: digits read in the current run, kept in 1..64 once
// nonzero.  Saturates at 2^32 - 1 (only garbage parses get there).
__device__ __forceinline__ uint32_t pixel_count(uint32_t pfx, uint32_t& dk) {
  if (pfx < (uint32_t)P_RUN1) { dk = 0; return 1u; }
  const uint32_t sh = (3u * dk) & 63u;
  const uint64_t c = ((uint64_t)(pfx - P_RUN1) << sh) + (dk == 0 ? 1u : 0u);
  dk = dk >= 64u ? 1u : dk + 1u;
  return c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c;
}
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) { return a + b < a ? 0xFFFFFFFFu : a + b; }

// Packed slice entry: bit position relative to the data start (40 bits), run
// digits read so far (7).  Bits 56..63 of `last` hold the number of valid
// checkpoints.  Checkpoint: position in the slice (16), run digits (7) << 20,
// pixels since the slice entry << 32.
constexpr unsigned long long PS_MASK = (1ull << 51) - 1ull;
__device__ __forceinline__ unsigned long long ps_pack(unsigned long long rel, uint32_t dk) {
  return rel | ((unsigned long long)dk << 44);
}


// Initial entry guesses: every slice starts at its first bit, at a prefix.
__global__ __launch_bounds__(256) void dec_init_entries(DecArgs a) {
  const uint32_t f = blockIdx.y;
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < a.max_chunks; j += gridDim.x * 256) {
    const uint64_t i = (uint64_t)f * a.max_chunks + j;
    a.entry[i] = ps_pack((unsigned long long)j * a.chunk_bits, 0);
    a.last[i] = ~0ull;
  }
}

// Event layout: the slices of a frame in groups of 64 (one parse wave); a
// group's events are interleaved in 16-byte quads, quad c of the group's slice
// l at words (c * 64 + l) * 4.  The first pass keeps every active lane at the
// same event index, so each of its 16-byte stores is one contiguous 1 KB per
// wave (a per-slice layout made every store touch 64 lines: +10 % parse time).
// Frames are padded to a multiple of 64 slices.
__device__ __forceinline__ uint64_t ev_group(const DecArgs& a, uint32_t f, uint32_t j) {
  return ((uint64_t)f * ((a.max_chunks + 63u) & ~63u) + (j & ~63u)) * a.ev_cap + (j & 63u) * 4u;
}
__device__ __forceinline__ uint32_t ev_word(uint32_t y) { return (y >> 2) * 256u + (y & 3u); }

// Event word of a coded pixel: its prefix and payload symbols as read
// (SMALL_DIFF index < 343, bytes < 256; LUMA: reference < 11, so its fourth
// symbol fits bits 7..11); dec_place turns it into a record.
__device__ __forceinline__ uint32_t ev_pack(uint32_t pfx, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) {
  return pfx | (s0 << 3) | (s1 << 12) | (s2 << 20) | (pfx == (uint32_t)P_LUMA ? s3 << 7 : 0u);
}

// ---------------------------------------------------------------------------
// D1: sync iteration (Jacobi, in place).  Each lane parses its slice from the
// current entry guess and writes the exit as the next slice's entry.  Lanes
// whose entry did not change since their last parse do nothing.  A re-parse
// compares its state with the previous parse at the first prefix after every
// CK_BITS; once they agree the rest of the slice is unchanged (Huffman
// self-synchronisation), so the lane stops and only patches its pixel count.
// ---------------------------------------------------------------------------
// `prev`: the previous iteration's change flag -- when it is 0 the entries are
// at the fixpoint already and this launch does nothing (the host queues several
// iterations without waiting for each).
// `fchanged` (optional): per-frame change flags, for dec_sync_settle.
__global__ __launch_bounds__(DEC_PARSE_THREADS) PARSE_ATTR void dec_sync(DecArgs a, uint32_t* changed, const uint32_t* prev,
                                                              uint32_t* fchanged) {
  __shared__ LutLds S;
  __shared__ __attribute__((aligned(16))) uint32_t ring[DEC_PARSE_THREADS * RING_STRIDE];
  if (prev && *prev == 0) return;
  const uint32_t f = blockIdx.x / a.chunk_blocks;
  const uint32_t jb = blockIdx.x % a.chunk_blocks;
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D, a.chunk_bits);
  if (jb * DEC_PARSE_THREADS >= nc) return;
  const uint32_t j = jb * DEC_PARSE_THREADS + threadIdx.x;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  unsigned long long e = 0, last = ~0ull;
  if (j < nc) {
    e = j == 0 ? 0ull : a.entry[base + j];
    last = a.last[base + j];
  }
  const bool need = j < nc && (last == ~0ull || (last & PS_MASK) != e);
  if (!__syncthreads_or(need)) return;
  load_lut(S, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6;
  if (jb * DEC_PARSE_THREADS + wave * 64u >= nc) return;
  StreamParams SP;
  SP.load(S);
  uint32_t* wring = ring + wave * 64u * RING_STRIDE;
  const uint32_t* my = wring + (threadIdx.x & 63u) * RING_STRIDE;
  const uint8_t* p = a.streams + (uint64_t)f * a.stream_stride;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const bool check = last != ~0ull;
  const uint32_t nvalid_old = (uint32_t)(last >> 56);
  const unsigned long long begin = D + (unsigned long long)j * a.chunk_bits;
  const unsigned long long end = begin + a.chunk_bits;
  const unsigned long long hard = len * 8 + 64;
  const uint32_t N = a.W * a.H;
  unsigned long long* ck = a.ck + (uint64_t)f * a.n_ck * a.max_chunks + j;
  // first pass: keep the pixel events (16-byte stores of 4)
  const bool keep = a.ev != nullptr && !check;
  uint32_t* evp = a.ev + ev_group(a, f, j);
  uint32_t* evck = a.ev_ck + (uint64_t)f * a.n_ck * a.max_chunks + j;
  uint32_t ne = 0, ev0 = 0, ev1 = 0, ev2 = 0;
  Lane L;
  L.pos = D + (e & ((1ull << 40) - 1));
  L.rp = RING_W;   // empty: filled on the first step
  L.ws = (uint32_t)(L.pos >> 5) - RING_W;   // (fast path) empty as well
  uint32_t dk = (uint32_t)(e >> 44) & 127u;
  uint32_t px = 0, k = 0;
  unsigned long long next_ck = begin + a.ck_bits;
  unsigned long long ck_old = (check && nvalid_old > 0) ? ck[0] : ~0ull;
  bool active = need, synced = false;
  // diagnostics (builds with -DNICE_SYNC_CYCLES and NICE_DEC_STATS=1, first
  // pass): wave cycles, refill cycles / count, iterations.  Compiled out by
  // default: the checks alone cost ~2 % of the kernel.
  unsigned long long tw0 = 0, tfill = 0, nfill = 0, nit = 0, nact = 0;
#ifdef NICE_SYNC_CYCLES
  const bool tstat = a.stats != nullptr && !check;
#else
  constexpr bool tstat = false;
#endif
  if (tstat) tw0 = __builtin_amdgcn_s_memtime();
  // the event loop, instantiated for the fast and the general parse
  auto parse = [&](auto fast_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < N_STREAMS; ++i) SP.g[i] = fast_param(SP.g[i]);
    }
    for (;;) {
      // at a prefix position: slice end, checkpoint, or one more pixel event
      if (active && (L.pos >= end || L.pos >= hard || px > N)) active = false;
      if (active && L.pos >= next_ck) {
        const uint32_t cur = (uint32_t)(L.pos - begin) | (dk << 20);
        if (check && k < nvalid_old && (uint32_t)ck_old == cur) {
          synced = true;
          active = false;
        } else {
          ck[(uint64_t)k * a.max_chunks] = cur | ((unsigned long long)px << 32);
          if (keep) evck[(uint64_t)k * a.max_chunks] = ne;
          ++k;
          next_ck = k < a.n_ck ? next_ck + a.ck_bits : ~0ull;
          ck_old = (check && k < nvalid_old) ? ck[(uint64_t)k * a.max_chunks] : ~0ull;
        }
      }
      if (!__any(active)) break;
      if (__any(active && !(FAST ? lane_ok_fast(L) : lane_ok(L)))) {
        const unsigned long long tf = tstat ? __builtin_amdgcn_s_memtime() : 0;
        ring_fill<FAST>(wring, p, len, al16, L);
        if (tstat) { tfill += __builtin_amdgcn_s_memtime() - tf; ++nfill; }
      }
      if (tstat) { ++nit; nact += active ? 1u : 0u; }
      if (active) {
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        const uint32_t pfx = FAST ? pixel_event_fast(L, my, S, SP, s0, s1, s2, s3)
                                  : pixel_event(L, my, S, SP, s0, s1, s2, s3);
        const uint32_t c = pixel_count(pfx, dk);
        px = sat_add(px, c);
        if (keep) {
          const uint32_t ev = pfx < (uint32_t)P_RUN1 ? ev_pack(pfx, s0, s1, s2, s3) : EV_RUN | min(c, EV_RUN - 1u);
          // the last three events in a shift register (ev2 the newest)
          if (ne < a.ev_cap && (ne & 3u) == 3u)
            *reinterpret_cast<uint4*>(evp + ev_word(ne - 3u)) = make_uint4(ev0, ev1, ev2, ev);
          ev0 = ev1;
          ev1 = ev2;
          ev2 = ev;
          ++ne;
        }
      }
    }
  };
  const bool fast = !a.parse_slow && reinterpret_cast<const DecTables*>(a.tables)[f].fast;
  // Fast parse in 32-bit positions (round 6): r = bits past the word holding
  // the slice's first bit, so the slice end, stream end, checkpoints and ring
  // offsets are 32-bit compares and adds instead of 64-bit ones; the loop is
  // unrolled four times so a kept event goes straight into its slot of the
  // 16-byte quad (every active lane of the first pass is at the same event
  // index) instead of through a shift register; a run digit's pixel count is a
  // 32-bit shift below 2^30.  r counts from the word holding the slice's first
  // bit or, when the entry lies before the slice (the previous slice's parse
  // stopped at px > N: speculative garbage), from the entry's word; a wave
  // with a lane more than 2^30 bits away takes the general symbol-by-symbol
  // parse, which reads any tables.
  const unsigned long long B = (active && L.pos < begin ? L.pos : begin) & ~31ull;
  if (fast && __all(!active || (L.pos >= B && begin + a.chunk_bits - B < (1ull << 30)))) {
    // the prefix stream's fast parameter (the payload streams' come from S.pp;
    // a converted copy of SP here put SP in scratch for the general loop)
    const uint32_t fp_pfx = fast_param(SP.g[PFX_STREAM]);
    const uint32_t bwl = (uint32_t)(B >> 5);
    const uint32_t b31 = (uint32_t)(begin - B);   // the slice's first bit
    const uint32_t rhard = hard > B ? (uint32_t)min(hard - B, (unsigned long long)0xFFFFFFFFu) : 0u;
    const uint32_t rlim = min(b31 + a.chunk_bits, rhard);
    uint32_t r = active ? (uint32_t)(L.pos - B) : 0u;
    uint32_t wsr = 0;    // ring start word (relative)
    uint32_t rfill = 0;  // refill once r reaches this (ring empty: at once)
    uint32_t nck = b31 + a.ck_bits;   // next checkpoint (relative)
    uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;   // the current quad of kept events
    auto step = [&](auto slot_tag, auto keep_tag) -> bool {
      constexpr int SLOT = decltype(slot_tag)::value;
      constexpr bool KEEP = decltype(keep_tag)::value;
      if (active && (r >= rlim || px > N)) active = false;
      if (active && r >= nck) {
        const uint32_t cur = (r - b31) | (dk << 20);
        if (check && k < nvalid_old && (uint32_t)ck_old == cur) {
          synced = true;
          active = false;
        } else {
          ck[(uint64_t)k * a.max_chunks] = cur | ((unsigned long long)px << 32);
          if (keep) evck[(uint64_t)k * a.max_chunks] = ne;
          ++k;
          nck = k < a.n_ck ? nck + a.ck_bits : 0xFFFFFFFFu;
          ck_old = (check && k < nvalid_old) ? ck[(uint64_t)k * a.max_chunks] : ~0ull;
        }
      }
      // (the first pass tests for the wave's end once per quad: a step after
      // every lane stopped only evaluates masked conditions)
      if ((!KEEP || SLOT == 0) && !__any(active)) return false;
      if (__any(active && r >= rfill)) {   // the next event's 3 words would pass the ring's end
        const uint32_t wsa = (bwl + (r >> 5)) & ~3u;
        ring_fill_ws(wring, p, len, al16, wsa);
        wsr = wsa - bwl;
        rfill = (wsr + RING_W - 2u) << 5;
      }
      if (active) {
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, tot;
        const uint32_t pfx = pixel_event_fast_at(my, S, fp_pfx, (r >> 5) - wsr, r & 31u, s0, s1, s2, s3, tot);
        r += tot;
        uint32_t c;
        if (pfx < (uint32_t)P_RUN1) {
          dk = 0;
          c = 1u;
        } else {
          const uint32_t sh = (3u * dk) & 63u, d = pfx - (uint32_t)P_RUN1;
          if (sh < 30u) {
            c = (d << sh) + (dk == 0 ? 1u : 0u);
          } else {   // (exact, saturating: only a run of >= 2^30 pixels gets here)
            const uint64_t c64 = (uint64_t)d << sh;
            c = c64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c64;
          }
          dk = dk >= 64u ? 1u : dk + 1u;
        }
        px = sat_add(px, c);
        if (KEEP && keep) {
          const uint32_t ev = pfx < (uint32_t)P_RUN1 ? ev_pack(pfx, s0, s1, s2, s3) : EV_RUN | min(c, EV_RUN - 1u);
          if constexpr (SLOT == 0) q0 = ev;
          if constexpr (SLOT == 1) q1 = ev;
          if constexpr (SLOT == 2) q2 = ev;
          if constexpr (SLOT == 3) {
            q3 = ev;
            if (ne < a.ev_cap) *reinterpret_cast<uint4*>(evp + ev_word(ne - 3u)) = make_uint4(q0, q1, q2, q3);
          }
          ++ne;
        }
      }
      return true;
    };
    if (__any(keep && active)) {   // the first pass: unrolled by the quad
      for (;;) {
        if (!step(std::integral_constant<int, 0>{}, std::true_type{})) break;
        if (!step(std::integral_constant<int, 1>{}, std::true_type{})) break;
        if (!step(std::integral_constant<int, 2>{}, std::true_type{})) break;
        if (!step(std::integral_constant<int, 3>{}, std::true_type{})) break;
      }
    } else {   // later passes keep nothing (a smaller loop: these launches are short)
      while (step(std::integral_constant<int, 0>{}, std::false_type{})) {
      }
    }
    L.pos = B + r;
    // the tail below stores the last (ne & 3) events from ev0..ev2 (newest last)
    const uint32_t sl = ne & 3u;
    ev0 = q0;
    ev1 = sl == 3u ? q1 : q0;
    ev2 = sl == 3u ? q2 : sl == 2u ? q1 : q0;
  } else {
    parse(std::false_type{});   // (any tables; the general parse)
  }
  if (tstat) {
    const unsigned long long tw = __builtin_amdgcn_s_memtime() - tw0;
    if ((threadIdx.x & 63u) == 0) {
      atomicAdd(&a.stats[56], tw); atomicAdd(&a.stats[57], tfill); atomicAdd(&a.stats[58], nfill);
      atomicAdd(&a.stats[59], nit); atomicAdd(&a.stats[61], 1ull);
    }
    atomicAdd(&a.stats[60], nact);
  }
  if (!need) return;
  if (keep) {
    const uint32_t slot = ne & 3u, q0 = ne & ~3u;
    if (ne <= a.ev_cap) {
      uint32_t* t = evp + ev_word(q0);
      // the last `slot` events are the newest of ev0..ev2
      if (slot == 3u) { t[0] = ev0; t[1] = ev1; t[2] = ev2; }
      if (slot == 2u) { t[0] = ev1; t[1] = ev2; }
      if (slot == 1u) t[0] = ev2;
    }
    a.ev_n[base + j] = ne <= a.ev_cap ? ne : EV_OVERFLOW;
    a.agree[base + j] = 0;
  } else if (a.ev) {
    // the final parse equals the first pass from the latest meeting point on
    const uint32_t ag = synced ? k + 1u : AGREE_NONE;
    a.agree[base + j] = max(a.agree[base + j], ag);
  }
  if (a.stats && check) {   // diagnostics: where re-parses met the previous parse (16: never)
    atomicAdd(&a.stats[32 + (synced ? min(k, 15u) : 16u)], 1ull);
  }
  if (synced) {
    // from checkpoint k on this parse equals the previous one, shifted by delta pixels
    const uint32_t delta = px - (uint32_t)(ck_old >> 32);
    a.chunk_px[base + j] = a.chunk_px[base + j] + (uint64_t)(int64_t)(int32_t)delta;
    for (uint32_t kk = k; kk < nvalid_old; ++kk) {
      unsigned long long& c = ck[(uint64_t)kk * a.max_chunks];
      c = (c & 0xFFFFFFFFull) | ((unsigned long long)((uint32_t)(c >> 32) + delta) << 32);
    }
    a.last[base + j] = e | ((unsigned long long)nvalid_old << 56);
    return;
  }
  a.chunk_px[base + j] = px;
  a.last[base + j] = e | ((unsigned long long)k << 56);
  if (j + 1 < nc) {
    const unsigned long long x = ps_pack(L.pos - D, dk);
    if (a.entry[base + j + 1] != x) {
      a.entry[base + j + 1] = x;
      atomicOr(changed, 1u);
      if (fchanged) fchanged[f] = 1u;
    }
  }
}

// ---------------------------------------------------------------------------
// D1b: the fixpoint on the device, for frames whose entries still changed in the
// last queued Jacobi iteration (fchanged).  The exact entries are the serial
// chain E_0 = 0, E_{j+1} = exit(j, E_j) (code.rs:573-684 is one parse); what
// the Jacobi iterations left is used as far as it is provably on that chain:
//  * slice j is consistent when it was last parsed from its current entry
//    (last[j] == entry[j]): then entry[j+1] is exit(j, entry[j]);
//  * so a walk that arrives at slice j with the exact entry x == entry[j] of a
//    consistent slice continues at entry[j+1] without parsing, and only the
//    slices whose entry or parse is stale are parsed.
// The frame's slices are cut into contiguous ranges, one per lane of the
// block (512 lanes).  Round 0: every lane walks its range from the entry its
// first slice holds, skipping consistent slices, parsing the others and
// writing their exits as the next entries; the first range starts exact
// (E_0 = 0).  A round leaves each range internally consistent.  Then a lane
// whose start differs from its left neighbour's exit walks again from that
// exit, parsing only until it meets an entry it already holds (from there its
// range is consistent, so its exit stands); rounds repeat until no start
// changes.  Range r is exact once ranges 0..r-1 are, so this terminates; with
// self-synchronisation within a range it ends after round 1, and a stream
// that never re-synchronises costs one serial parse of its dirty slices, as
// the reference's own decode does.  (Round 5's settle had one lane walk every
// slice from slice 0: 3.3 s for a 4K frame that missed the fixpoint by one
// queued iteration.)  A dec_sync launch after this one (prev = *settled)
// re-parses the slices whose entries moved, bringing their pixel counts,
// checkpoints and meeting points up to date.
// ---------------------------------------------------------------------------
constexpr uint32_t SETTLE_THREADS = 512;
__global__ __launch_bounds__(SETTLE_THREADS) void dec_sync_settle(DecArgs a, const uint32_t* last_changed,
                                                                  const uint32_t* fchanged, uint32_t* settled) {
  __shared__ LutLds S;
  __shared__ __attribute__((aligned(16))) uint32_t ring[SETTLE_THREADS * RING_STRIDE];
  __shared__ unsigned long long xs[SETTLE_THREADS];   // each range's exit in the current round
  const uint32_t f = blockIdx.x;
  if (*last_changed == 0 || fchanged[f] == 0 || a.status[f] != 0) return;   // block-uniform
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = min(n_chunks(len, D, a.chunk_bits), a.max_chunks);
  if (nc < 2) return;
  load_lut(S, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  StreamParams SP;
  SP.load(S);
  const uint32_t t = threadIdx.x;
  uint32_t* wring = ring + (t & ~63u) * RING_STRIDE;
  const uint32_t* my = ring + t * RING_STRIDE;
  const uint8_t* p = a.streams + (uint64_t)f * a.stream_stride;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t N = a.W * a.H;
  const unsigned long long hard = len * 8 + 64;
  const uint32_t per = (nc + SETTLE_THREADS - 1) / SETTLE_THREADS;
  const uint32_t lo = min(t * per, nc), hi = min(lo + per, nc);   // nonempty ranges: lanes 0..k, contiguous
  unsigned long long start = lo == 0 ? 0ull : a.entry[base + lo];
  unsigned long long xprev = 0;   // the lane's exit of the previous round
  bool walk = lo < hi;
  const bool fast = !a.parse_slow && reinterpret_cast<const DecTables*>(a.tables)[f].fast;
  for (uint32_t round = 0;; ++round) {
    // ---- one round: the lanes with `walk` parse their range from `start`
    Lane L;
    L.pos = D;
    L.rp = RING_W;
    L.ws = (uint32_t)(D >> 5) - RING_W;
    uint32_t j = lo, dk = 0, px = 0;
    unsigned long long end = 0, xout = xprev;
    bool refill = true;
    // position the lane at slice j with entry x, after the slices it may skip;
    // false once the walk is done (xout set)
    auto advance = [&](unsigned long long x) -> bool {
      for (;;) {
        if (j >= hi) { xout = x; return false; }
        const unsigned long long cur = j == 0 ? 0ull : a.entry[base + j];
        if (round == 0) {
          const unsigned long long lj = a.last[base + j];
          if (x == cur && lj != ~0ull && (lj & PS_MASK) == cur) {   // consistent: its exit is the next entry
            x = j + 1 < nc ? a.entry[base + j + 1] : 0ull;
            ++j;
            continue;
          }
        } else if (j > lo && x == cur) {   // the rest of the range is consistent from here
          xout = xprev;
          return false;
        }
        if (j > lo) a.entry[base + j] = x;
        L.pos = D + (x & ((1ull << 40) - 1));
        dk = (uint32_t)(x >> 44) & 127u;
        px = 0;
        end = D + (unsigned long long)(j + 1) * a.chunk_bits;
        refill = true;
        return true;
      }
    };
    bool active = walk && advance(start);
    auto parse = [&](auto fast_tag) {
      constexpr bool FAST = decltype(fast_tag)::value;
      StreamParams G = SP;
      if constexpr (FAST) {
#pragma unroll
        for (int i = 0; i < N_STREAMS; ++i) G.g[i] = fast_param(G.g[i]);
      }
      for (;;) {
        // at a prefix position: the slice's end (same stop rule as dec_sync), or one more pixel event
        if (active && (L.pos >= end || L.pos >= hard || px > N)) {
          ++j;
          active = advance(ps_pack(L.pos - D, dk));
        }
        if (!__any(active)) break;
        if (__any(active && (refill || !(FAST ? lane_ok_fast(L) : lane_ok(L))))) {
          ring_fill<FAST>(wring, p, len, al16, L);
          refill = false;
        }
        if (active) {
          uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
          const uint32_t pfx = FAST ? pixel_event_fast(L, my, S, G, s0, s1, s2, s3)
                                    : pixel_event(L, my, S, G, s0, s1, s2, s3);
          px = sat_add(px, pixel_count(pfx, dk));
        }
      }
    };
    if (fast) parse(std::true_type{});
    else parse(std::false_type{});
    xs[t] = xout;
    __syncthreads();
    // ---- a range whose start is not its left neighbour's exit walks again
    const unsigned long long want = (t == 0 || lo >= hi) ? start : xs[t - 1];
    xprev = xout;
    walk = want != start;
    if (walk) {
      start = want;
      a.entry[base + lo] = want;   // lane t - 1 reads it only in round 0
    }
    if (!__syncthreads_or(walk)) break;
  }
  if (t == 0) *settled = 1u;
}

// ---------------------------------------------------------------------------
// D3: exclusive scan of chunk pixel counts, one 1024-thread block per frame.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void dec_scan(DecArgs a) {
  __shared__ unsigned long long part[1024];
  const uint32_t f = blockIdx.x;
  if (a.status[f] != 0) return;
  if (a.unsettled && a.unsettled[f]) {   // the parse is not at its fixpoint: fail, never decode from it
    if (threadIdx.x == 0) set_status(&a.status[f], NICE_E_HIP);
    return;
  }
  const uint32_t nc = n_chunks(a.stream_len[f], a.data_start[f], a.chunk_bits);
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t per = (nc + 1023) / 1024;
  const uint32_t c0 = threadIdx.x * per, c1 = min(c0 + per, nc);
  // a thread's range in batches of 8 independent loads (one at a time, a
  // single frame's ~85 chunks per thread were ~85 dependent round trips)
  constexpr uint32_t B = 8;
  unsigned long long sum = 0;
  for (uint32_t j0 = c0; j0 < c1; j0 += B) {
    unsigned long long v[B];
#pragma unroll
    for (uint32_t q = 0; q < B; ++q) v[q] = j0 + q < c1 ? a.chunk_px[base + j0 + q] : 0ull;
#pragma unroll
    for (uint32_t q = 0; q < B; ++q) sum = (sum + v[q] < sum) ? ~0ull : sum + v[q];   // saturate (garbage past the image end)
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
  for (uint32_t j0 = c0; j0 < c1; j0 += B) {
    unsigned long long v[B];
#pragma unroll
    for (uint32_t q = 0; q < B; ++q) v[q] = j0 + q < c1 ? a.chunk_px[base + j0 + q] : 0ull;
#pragma unroll
    for (uint32_t q = 0; q < B; ++q) {
      if (j0 + q < c1) a.chunk_start[base + j0 + q] = run;
      run = (run + v[q] < run) ? ~0ull : run + v[q];
    }
  }
  if (threadIdx.x == 1023) {
    // total must cover the image
    if (part[1023] < (unsigned long long)a.W * a.H) set_status(&a.status[f], NICE_E_FORMAT);
  }
}

// ---------------------------------------------------------------------------
// D3b (strict mode only): the reference's refill wrap (bitreader.rs:85-98).
// read_24bits_noclear(M) refills while its u8 bit offset exceeds 32 - M,
// subtracting 8 each time; the offset's residue mod 8 is the read position's
// (offset = P + 32 - 8 * bytes read), so the loop runs through the value P & 7
// and, when that is above 32 - M, subtracts 8 from it: the u8 wraps and the
// loop never ends.  A read therefore hangs the reference iff it refills at all
// -- P + M > 8 * bytes read so far -- and (P & 7) + M > 32 (only M >= 26).
// Bytes read are a running maximum of ceil((P_k + M_k) / 8) over the reads
// (M = the stream's max length, hfe.rs:209), starting at the 770 header bytes.
// The reads that end the decode: every event while pixels < N, then one more
// prefix (plus the zero digits of a run that reached N, which the reference's
// run loop keeps reading, code.rs:665-671).  One lane per slice re-parses the
// converged slice j - 1 (for its reads' running maximum; slices are >= 1024
// bits and only the last 31 bits of reads matter) and then checks slice j.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(DEC_PARSE_THREADS) void dec_strict_refill(DecArgs a) {
  __shared__ LutLds S;
  __shared__ __attribute__((aligned(16))) uint32_t ring[DEC_PARSE_THREADS * RING_STRIDE];
  const uint32_t f = blockIdx.x / a.chunk_blocks;
  const uint32_t jb = blockIdx.x % a.chunk_blocks;
  if (a.status[f] != 0) return;
  const DecTables* T = reinterpret_cast<const DecTables*>(a.tables) + f;
  uint32_t mx = 0;
#pragma unroll
  for (int st = 0; st < N_STREAMS; ++st) mx = max(mx, (uint32_t)T->max_aob[st]);
  if (mx <= 25u) return;   // (P & 7) + M <= 32 for every read
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D, a.chunk_bits);
  if (jb * DEC_PARSE_THREADS >= nc) return;
  load_lut(S, T);
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6;
  if (jb * DEC_PARSE_THREADS + wave * 64u >= nc) return;
  StreamParams SP;
  SP.load(S);
  const uint32_t j = jb * DEC_PARSE_THREADS + threadIdx.x;
  const uint32_t j0 = j > 0 ? j - 1u : 0u;
  uint32_t* wring = ring + wave * 64u * RING_STRIDE;
  const uint32_t* my = wring + (threadIdx.x & 63u) * RING_STRIDE;
  const uint8_t* p = a.streams + (uint64_t)f * a.stream_stride;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const unsigned long long N = (unsigned long long)a.W * a.H;
  const unsigned long long begin = D + (unsigned long long)j * a.chunk_bits;
  const unsigned long long end = begin + a.chunk_bits;
  const unsigned long long hard = len * 8 + 64;
  bool active = j < nc;
  unsigned long long e = 0, q = 0;
  if (active) {
    e = j0 == 0 ? 0ull : a.entry[base + j0];
    q = a.chunk_start[base + j0];
  }
  Lane L;
  L.pos = D + (e & ((1ull << 40) - 1));
  L.rp = RING_W;
  uint32_t dk = (uint32_t)(e >> 44) & 127u;
  bool closed = q == N;
  unsigned long long nb8 = D;   // 8 x bytes the reference has read (D = 770 bytes)
  bool hang = false;
  for (;;) {
    if (active && (L.pos >= end || L.pos >= hard || q > N)) active = false;
    if (!__any(active)) break;
    if (__any(active && !lane_ok(L))) ring_fill<false>(wring, p, len, al16, L);
    if (!active) continue;
    const bool chk = L.pos >= begin;   // an event of slice j (not of slice j - 1)
    // one read of stream st at L.pos, then the symbol
    auto rd = [&](uint32_t st) -> uint32_t {
      const uint32_t gp = SP.g[st], M = gp >> 24;
      if (L.pos + M > nb8) {
        hang = hang || (chk && (uint32_t)(L.pos & 7u) + M > 32u);
        nb8 = (L.pos + M + 7u) & ~7ull;
      }
      return dsym_gp(L, my, S, st, gp);
    };
    const bool at_n = q == N && (dk == 0 || closed);
    const uint32_t pfx = rd(PFX_STREAM);
    if (at_n) {
      // the extra prefix (code.rs:660); a zero digit continues the run loop
      if (dk != 0 && pfx == (uint32_t)P_RUN1) (void)pixel_count(pfx, dk);
      else active = false;
      continue;
    }
    if (pfx < (uint32_t)P_RUN1) {
      (void)rd(pay_stream(pfx, 0));
      if (pfx == (uint32_t)P_RGB || pfx == (uint32_t)P_LUMA || pfx == (uint32_t)P_LUMA2) {
        (void)rd(pay_stream(pfx, 1));
        (void)rd(pay_stream(pfx, 2));
        if (pfx == (uint32_t)P_LUMA) (void)rd(S_LUMA_OTHER);
      }
      q += 1;
      dk = 0;
      closed = false;
    } else {
      q += pixel_count(pfx, dk);
      closed = closed || q == N;
    }
  }
  if (hang) set_status(&a.status[f], NICE_E_UNSUPPORTED);
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
// Records of a lane are combined into aligned groups of four and stored with
// one 16-byte store when the group lies inside the lane's pixel range.
// ---------------------------------------------------------------------------
// Record (round 6): the additive constant c in the row kernels' spread form
// (R | G << 10 | B << 20: bits 0..7, 10..17, 20..27), bits 28..31 the source
// class: 0 = AVG, 1..3 = the pixel 1..3 back in raster order (a run pixel is
// class 1 with c = 0), 4..13 = a pixel in a row above, at (rows back, pixels
// back) = cls_rows / cls_px.  The record writers (dec_emit, dec_place) spread
// the constant, so the row kernels' pre-pass -- on the row chain -- only masks
// it (round 5 kept bytes and spread every pixel there: ~5 VALU per pixel).
constexpr uint32_t REC_RUN = 1u << 28;
constexpr uint32_t REC_K = 0xFFu | (0xFFu << 10) | (0xFFu << 20);   // the constant's bits
// Records written by a decode call carry its tag (1..15) in the gap bits 8..9
// (tag & 3) and 18..19 (tag >> 2); a slot without the current tag (stale, or
// cleared to 0) is a run pixel.  The record buffer is then cleared only when
// its tags wrap or its layout changes (nice_capi.hip), not prefilled with
// REC_RUN by every call.  The canonical record keeps the tag bits: readers take
// the class (rec_cls) and the constant (rec_c) only.
constexpr uint32_t REC_TAG_MASK = (3u << 8) | (3u << 18);
__device__ __forceinline__ uint32_t rec_tagbits(uint32_t tag) { return ((tag & 3u) << 8) | ((tag >> 2) << 18); }
__device__ __forceinline__ uint32_t rec_canon(uint32_t r, uint32_t tag) {
  return (r & REC_TAG_MASK) == rec_tagbits(tag) ? r : REC_RUN;
}
__device__ __forceinline__ uint32_t rec_cls(uint32_t r) { return r >> 28; }
__device__ __forceinline__ uint32_t rec_c(uint32_t r) { return r & REC_K; }
// R | G << 8 | B << 16 -> spread (the record writers)
__device__ __forceinline__ uint32_t rec_spread(uint32_t v) {
  return (v & 0xFFu) | ((v & 0xFF00u) << 2) | ((v & 0xFF0000u) << 4);
}
__host__ __device__ constexpr int cls_rows(int c) {
  return c < 4 ? 0 : c == 4 ? 1 : c == 5 ? 1 : c == 6 ? 2 : c == 7 ? 1 : c <= 10 ? 3 : c == 11 ? 1 : c <= 13 ? 3 : 0;
}
__host__ __device__ constexpr int cls_px(int c) {
  return c < 4 ? c : c == 4 ? 0 : c == 5 ? -1 : c == 6 ? 0 : c == 7 ? -3 : c == 8 ? -1 : c == 9 ? 0
       : c == 10 ? 1 : c == 11 ? 3 : c == 12 ? 3 : c == 13 ? -3 : 0;
}
// reference id (back refs 0..4, luma refs 5..15) -> class
__host__ __device__ constexpr int id_cls(int id) {
  return id == 0 ? 1 : id == 1 ? 4 : id == 2 ? 5 : id == 3 ? 2 : id == 4 ? 6
       : id == 5 ? 1 : id == 6 ? 4 : id == 7 ? 5 : id == 8 ? 7 : id == 9 ? 3 : id == 10 ? 8
       : id == 11 ? 9 : id == 12 ? 10 : id == 13 ? 11 : id == 14 ? 12 : 13;
}
__host__ __device__ constexpr bool cls_table_ok() {
  for (int id = 0; id < 16; ++id) {
    const int rows = id < 5 ? br_rows(id) : lr_rows(id - 5), px = id < 5 ? br_px(id) : lr_px(id - 5);
    if (cls_rows(id_cls(id)) != rows || cls_px(id_cls(id)) != px) return false;
  }
  return true;
}
static_assert(cls_table_ok(), "reference offsets (code.rs:141-145) map onto the record classes");
constexpr unsigned long long ID_CLS_PACK = [] {
  unsigned long long v = 0;
  for (int id = 0; id < 16; ++id) v |= (unsigned long long)id_cls(id) << (4 * id);
  return v;
}();
constexpr uint32_t CLS_ROWS_PACK = [] {
  uint32_t v = 0;
  for (int c = 0; c < 16; ++c) v |= (uint32_t)cls_rows(c) << (2 * c);
  return v;
}();
constexpr unsigned long long CLS_PX_PACK = [] {
  unsigned long long v = 0;
  for (int c = 0; c < 16; ++c) v |= (unsigned long long)(cls_px(c) + 3) << (3 * c);
  return v;
}();


// Record of a completed coded pixel (branch-free), as an event word: the
// record (bits 0..27) plus EV_L2 (LUMA2: needs the row above) and EV_BAD (an
// index the reference rejects wherever the pixel is, or an offset that wraps
// for W < 3).  The position-dependent checks are rec_bad_at's.
__device__ __forceinline__ uint32_t make_event_rec(uint64_t W, uint32_t mode, uint32_t s0, uint32_t s1,
                                                   uint32_t s2, uint32_t s3) {
  const bool isbr = mode == P_BACK_REF, islu = mode == P_LUMA;
  const bool issd = mode == P_SMALL_DIFF, isl2 = mode == P_LUMA2;
  const uint32_t id = min(isbr ? s0 : 5u + s0, 15u);
  const uint32_t cls = (uint32_t)(ID_CLS_PACK >> (4 * id)) & 15u;
  const uint64_t rows = (CLS_ROWS_PACK >> (2 * cls)) & 3u;
  const int64_t off = (int64_t)(rows * W) + (int64_t)((CLS_PX_PACK >> (3 * cls)) & 7u) - 3;
  const bool bad0 = (isbr && s0 >= 5u) || (islu && s0 >= 11u) || off < 0;
  const uint32_t gl = (s1 - 32u) & 255u;
  const uint32_t c_lu = ((s2 - 16u + gl) & 255u) | (gl << 10) | (((s3 - 16u + gl) & 255u) << 20);
  const uint32_t rd = s0 % 7u, t1 = s0 / 7u;
  const uint32_t c_sd = ((rd - 3u) & 255u) | ((((t1 % 7u) - 3u) & 255u) << 10) | ((((t1 / 7u) - 3u) & 255u) << 20);
  const uint32_t g2 = (s0 - 32u) & 255u;
  const uint32_t c_l2 = ((s1 - 16u + g2) & 255u) | (g2 << 10) | (((s2 - 16u + g2) & 255u) << 20);
  const uint32_t c_rgb = (s0 & 255u) | ((s1 & 255u) << 10) | ((s2 & 255u) << 20);
  const uint32_t r = (isbr || islu) ? ((cls << 28) | (islu ? c_lu : 0u)) : issd ? c_sd : isl2 ? c_l2 : c_rgb;
  return r | (isl2 ? EV_L2 : 0u) | ((isbr || islu) && bad0 ? EV_BAD : 0u);
}
// The reference panics on this pixel at position q: a reference before the
// image start (code.rs:141-145 offsets) or LUMA2 on the first row (code.rs:583).
__device__ __forceinline__ bool rec_bad_at(uint32_t ev, uint64_t q, uint64_t W) {
  const uint32_t cls = rec_cls(ev);
  const uint64_t rows = (CLS_ROWS_PACK >> (2 * cls)) & 3u;
  const uint64_t off = rows * W + ((CLS_PX_PACK >> (3 * cls)) & 7u) - 3u;   // >= 0 unless EV_BAD
  return (ev & EV_BAD) || ((ev & EV_L2) ? q < W : (cls != 0u && q < off));
}
__device__ __forceinline__ uint32_t make_record(uint64_t W, uint64_t q, uint32_t mode, uint32_t s0,
                                                uint32_t s1, uint32_t s2, uint32_t s3, bool& bad) {
  const uint32_t ev = make_event_rec(W, mode, s0, s1, s2, s3);
  bad = rec_bad_at(ev, q, W);
  return ev & ~(EV_L2 | EV_BAD);
}

struct RecGroup {
  unsigned long long grp;   // first pixel of the aligned group, ~0: empty (u64: no collision with pixels)
  uint32_t v0, v1, v2, v3, mask;
  __device__ __forceinline__ void flush(uint32_t* rec, unsigned long long lo, unsigned long long hi) {
    if (!mask) return;
    if (grp >= lo && grp + 4 <= hi) {
      uint4* dst = reinterpret_cast<uint4*>(__builtin_assume_aligned(rec + grp, 16));
      *dst = make_uint4(v0, v1, v2, v3);
    } else {
      if (mask & 1u) rec[grp] = v0;
      if (mask & 2u) rec[grp + 1] = v1;
      if (mask & 4u) rec[grp + 2] = v2;
      if (mask & 8u) rec[grp + 3] = v3;
    }
  }
  __device__ __forceinline__ void put(uint32_t* rec, unsigned long long lo, unsigned long long cur,
                                      uint32_t r) {
    const unsigned long long g4 = cur & ~3ull;
    if (g4 != grp) {
      flush(rec, lo, cur);    // every pixel of the old group below cur is this lane's
      grp = g4;
      v0 = v1 = v2 = v3 = REC_RUN;
      mask = 0;
    }
    const uint32_t k = (uint32_t)(cur & 3u);
    v0 = k == 0 ? r : v0;
    v1 = k == 1 ? r : v1;
    v2 = k == 2 ? r : v2;
    v3 = k == 3 ? r : v3;
    mask |= 1u << k;
  }
};

// Lanes take sub-slices of DEC_EMIT_BITS: sub-slice s of slice j starts at the
// converged parse's checkpoint (s * DEC_EMIT_BITS / a.ck_bits - 1) -- a prefix
// position with its run digits and pixel count -- so emission parallelism does
// not depend on the slice size the sync pass uses.  With the first pass's
// events kept (a.ev), the lanes take dec_heads' list instead and each stops at
// its slice's meeting point; dec_place writes the rest.
__global__ __launch_bounds__(DEC_PARSE_THREADS) PARSE_ATTR void dec_emit(DecArgs a) {
  __shared__ LutLds S;
  __shared__ __attribute__((aligned(16))) uint32_t ring[DEC_PARSE_THREADS * RING_STRIDE];
  const uint32_t f = blockIdx.x / a.emit_blocks;
  const uint32_t vb = blockIdx.x % a.emit_blocks;
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  const uint32_t nc = n_chunks(len, D, a.chunk_bits);
  const uint32_t subs = a.chunk_bits / DEC_EMIT_BITS;
  // with first-pass events kept, only the listed head sub-slices (dec_heads)
  const uint32_t nv = a.head_items ? a.head_count[f] : nc * subs;
  if (vb * DEC_PARSE_THREADS >= nv) return;
  load_lut(S, reinterpret_cast<const DecTables*>(a.tables) + f);
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6;
  if (vb * DEC_PARSE_THREADS + wave * 64u >= nv) return;
  StreamParams SP;
  SP.load(S);
  const uint32_t v = vb * DEC_PARSE_THREADS + threadIdx.x;
  const uint32_t item = !a.head_items ? v
                      : v < nv ? a.head_items[(uint64_t)f * a.max_chunks * subs + v] : 0u;
  const uint32_t j = item / subs, sub = item - j * subs;
  uint32_t* wring = ring + wave * 64u * RING_STRIDE;
  const uint32_t* my = wring + (threadIdx.x & 63u) * RING_STRIDE;
  const uint8_t* p = a.streams + (uint64_t)f * a.stream_stride;
  const bool al16 = (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t N = a.W * a.H;
  const unsigned long long begin = D + (unsigned long long)j * a.chunk_bits;
  unsigned long long q64 = 0, e = 0;
  unsigned long long end = begin + a.chunk_bits;
  bool active = v < nv;
  if (active) {
    q64 = a.chunk_start[base + j];   // pixels accounted before this slice
    const uint32_t nvalid = (uint32_t)(a.last[base + j] >> 56);
    const unsigned long long* ck = a.ck + (uint64_t)f * a.n_ck * a.max_chunks + j;
    const uint32_t step = DEC_EMIT_BITS / a.ck_bits;
    if (sub == 0) {
      e = j == 0 ? 0ull : a.entry[base + j];
    } else {
      const uint32_t c = sub * step - 1;
      if (c < nvalid) {
        const unsigned long long x = ck[(uint64_t)c * a.max_chunks];
        e = ((begin - D) + (x & 0xFFFFu)) | ((unsigned long long)((x >> 20) & 127u) << 44);
        q64 += x >> 32;
      } else {
        active = false;               // the slice's parse ended before this sub-slice
      }
    }
    const uint32_t c1 = (sub + 1) * step - 1;
    if (sub + 1 < subs && c1 < nvalid) end = begin + (ck[(uint64_t)c1 * a.max_chunks] & 0xFFFFu);
    if (q64 > N) active = false;      // past the image: tail bytes
    if (a.ev) {
      // dec_place writes the slice from where the final parse meets the first
      // pass (its events kept): this lane only parses the head before that
      const uint32_t ag = a.agree[base + j];
      if (ag != AGREE_NONE && a.ev_n[base + j] != EV_OVERFLOW && ag <= nvalid) {
        const unsigned long long stop =
            ag == 0u ? begin : begin + (ck[(uint64_t)(ag - 1u) * a.max_chunks] & 0xFFFFu);
        if (stop < end) end = stop;
        if (sub * step >= ag) active = false;   // starts at or past the meeting point
      }
    }
  }
  uint32_t q = (uint32_t)(q64 > N ? N : q64);
  const uint32_t q0 = q;
  const unsigned long long hard = len * 8 + 64;
  uint32_t* rec = a.recs + (uint64_t)f * a.rec_stride;
  const bool strict = (a.flags & NICE_DEC_STRICT_REFERENCE) != 0;
  Lane L;
  L.pos = D + (e & ((1ull << 40) - 1));
  L.rp = RING_W;
  L.ws = (uint32_t)(L.pos >> 5) - RING_W;   // (fast parse) empty as well
  uint32_t dk = (uint32_t)(e >> 44) & 127u;
  bool closed = (q == N);          // a run completed exactly at N earlier
  bool err = false;
  RecGroup G{~0ull, REC_RUN, REC_RUN, REC_RUN, REC_RUN, 0u};
  // one pixel event read at a prefix position: a record, a run's pixels, or
  // the end of the lane's work
  auto handle = [&](bool at_n, uint32_t pfx, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3) {
    if (at_n) {
      // a zero digit of the run that reached N: the reference's run loop
      // (code.rs:665-671) reads it and adds nothing
      if (dk != 0 && pfx == (uint32_t)P_RUN1) { (void)pixel_count(pfx, dk); return; }
      // the reference still reads one more prefix (code.rs:660): a run digit
      // there makes it copy past its buffer
      err = err || (strict && pfx >= (uint32_t)P_RUN1);
      active = false;
      return;
    }
    const uint32_t cur = q;
    const uint32_t c = pixel_count(pfx, dk);
    if (pfx < (uint32_t)P_RUN1) {
      bool bad;
      const uint32_t r = make_record(a.W, cur, pfx, s0, s1, s2, s3, bad);
      if (bad) { err = true; active = false; return; }
      G.put(rec, q0, cur, r | rec_tagbits(a.rec_tag));
      q = cur + 1;
      closed = false;
    } else {
      const unsigned long long qn = (unsigned long long)q + c;
      if (qn > N) { err = true; active = false; return; }
      q = (uint32_t)qn;
      closed = closed || q == N;
    }
  };
  // the general loop (and, before round 6, the fast one: as dec_sync)
  auto emit = [&](auto fast_tag) {
    constexpr bool FAST = decltype(fast_tag)::value;
    if constexpr (FAST) {
#pragma unroll
      for (int k = 0; k < N_STREAMS; ++k) SP.g[k] = fast_param(SP.g[k]);
    }
    for (;;) {
      // at a prefix position
      const bool at_n = q == N && (dk == 0 || closed);   // every pixel accounted for
      if (active && (L.pos >= end || L.pos >= hard)) active = false;
      if (!__any(active)) break;
      bool ok;
      if constexpr (FAST) ok = lane_ok_fast(L);
      else ok = lane_ok(L);
      if (__any(active && !ok)) ring_fill<FAST>(wring, p, len, al16, L);
      if (!active) continue;
      uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
      uint32_t pfx;
      if constexpr (FAST) pfx = pixel_event_fast(L, my, S, SP, s0, s1, s2, s3);
      else pfx = pixel_event(L, my, S, SP, s0, s1, s2, s3);
      handle(at_n, pfx, s0, s1, s2, s3);
    }
  };
  const bool fast = !a.parse_slow && reinterpret_cast<const DecTables*>(a.tables)[f].fast;
  // the fast parse in 32-bit positions relative to B, as dec_sync's (round 6)
  const unsigned long long B = (active && L.pos < begin ? L.pos : begin) & ~31ull;
  if (fast && __all(!active || (L.pos >= B && end - B < (1ull << 30)))) {
    const uint32_t fp_pfx = fast_param(SP.g[PFX_STREAM]);
    const uint32_t bwl = (uint32_t)(B >> 5);
    const uint32_t rhard = hard > B ? (uint32_t)min(hard - B, (unsigned long long)0xFFFFFFFFu) : 0u;
    const uint32_t rlim = active ? min((uint32_t)(end - B), rhard) : 0u;
    uint32_t r = active ? (uint32_t)(L.pos - B) : 0u;
    uint32_t wsr = 0, rfill = 0;
    for (;;) {
      const bool at_n = q == N && (dk == 0 || closed);   // every pixel accounted for
      if (active && r >= rlim) active = false;
      if (!__any(active)) break;
      if (__any(active && r >= rfill)) {
        const uint32_t wsa = (bwl + (r >> 5)) & ~3u;
        ring_fill_ws(wring, p, len, al16, wsa);
        wsr = wsa - bwl;
        rfill = (wsr + RING_W - 2u) << 5;
      }
      if (!active) continue;
      uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, tot;
      const uint32_t pfx = pixel_event_fast_at(my, S, fp_pfx, (r >> 5) - wsr, r & 31u, s0, s1, s2, s3, tot);
      r += tot;
      handle(at_n, pfx, s0, s1, s2, s3);
    }
  } else {
    emit(std::false_type{});   // (any tables; the general parse)
  }
  G.flush(rec, q0, q0);   // last group: per-record stores (the next lane may own the rest)
  if (err) set_status(&a.status[f], NICE_E_FORMAT);
}

// ---------------------------------------------------------------------------
// D4a: list the sub-slices dec_emit parses (one 1024-thread block per frame):
// each slice's head before the checkpoint where the final parse meets the
// first pass, or the whole slice when it never does (or its events
// overflowed).  Compact lists keep dec_emit's waves full of working lanes.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void dec_heads(DecArgs a) {
  __shared__ uint32_t part[1024];
  const uint32_t f = blockIdx.x;
  if (a.status[f] != 0) {
    if (threadIdx.x == 0) a.head_count[f] = 0;
    return;
  }
  const uint32_t nc = n_chunks(a.stream_len[f], a.data_start[f], a.chunk_bits);
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t subs = a.chunk_bits / DEC_EMIT_BITS, step = DEC_EMIT_BITS / a.ck_bits;
  const uint32_t per = (nc + 1023) / 1024;
  const uint32_t c0 = min(threadIdx.x * per, nc), c1 = min(c0 + per, nc);
  auto nsub = [&](uint32_t j) -> uint32_t {
    const uint32_t ag = a.agree[base + j], nvalid = (uint32_t)(a.last[base + j] >> 56);
    if (ag == AGREE_NONE || a.ev_n[base + j] == EV_OVERFLOW || ag > nvalid)
      return min(subs, 1u + nvalid / step);   // every sub-slice with a start (s * step - 1 < nvalid)
    return (ag + step - 1) / step;            // sub-slices starting before the meeting point
  };
  uint32_t cnt = 0;
  for (uint32_t j = c0; j < c1; ++j) cnt += nsub(j);
  part[threadIdx.x] = cnt;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t t = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t o = part[threadIdx.x] - cnt;
  uint32_t* items = a.head_items + base * subs;
  for (uint32_t j = c0; j < c1; ++j) {
    const uint32_t n = nsub(j);
    for (uint32_t s = 0; s < n; ++s) items[o++] = j * subs + s;
  }
  if (threadIdx.x == 1023) a.head_count[f] = part[1023];
}

// ---------------------------------------------------------------------------
// D4b: place the first pass's events past each slice's meeting point (one wave
// per slice): pixel positions by a wave prefix sum of the events' pixel
// counts, one coalesced 4-byte record store per coded pixel, runs left to the
// memset marker.  Same checks as dec_emit: the first event at q == N is the
// extra prefix the reference reads (strict: a run digit there is an error),
// a run past N or a reference the reference rejects sets NICE_E_FORMAT.
// ---------------------------------------------------------------------------
// make_record for dec_place: 32-bit arithmetic (q <= N <= 2^30, 3W < 2^32),
// the SMALL_DIFF constant from a table (sdl: 343 packed constants in LDS), the
// reference's class and offset from another (idt: 16 entries per block).
#ifdef NICE_PLACE_ARITH
constexpr uint32_t ID_CLS_LO = (uint32_t)ID_CLS_PACK, ID_CLS_HI = (uint32_t)(ID_CLS_PACK >> 32);
constexpr uint32_t CLS_PX_LO = (uint32_t)CLS_PX_PACK, CLS_PX_HI = (uint32_t)(CLS_PX_PACK >> 32);
#endif
__device__ __forceinline__ uint32_t place_record(uint32_t ev, uint32_t q, uint32_t W, const uint32_t* sdl,
                                                 const uint2* idt, bool& bad) {
  const uint32_t pfx = ev & 7u;
#ifndef NICE_PLACE_BRANCHY
  // prefix tests as bits of one mask: as == compares of one value, the
  // compiler turned the selects below into a switch of exec-masked branches
  const uint32_t pm = 1u << pfx;
  const bool isbr = (pm & (1u << P_BACK_REF)) != 0u, islu = (pm & (1u << P_LUMA)) != 0u;
  const bool issd = (pm & (1u << P_SMALL_DIFF)) != 0u, isl2 = (pm & (1u << P_LUMA2)) != 0u;
#else
  const bool isbr = pfx == (uint32_t)P_BACK_REF, islu = pfx == (uint32_t)P_LUMA;
  const bool issd = pfx == (uint32_t)P_SMALL_DIFF, isl2 = pfx == (uint32_t)P_LUMA2;
#endif
  const uint32_t s0 = (ev >> 3) & 511u, s1 = (ev >> 12) & 255u, s2 = (ev >> 20) & 255u, s3 = (ev >> 7) & 31u;
  const uint32_t s0l = s0 & 15u;   // LUMA: the reference (bits 3..6)
  const uint32_t id = min(isbr ? s0 : 5u + s0l, 15u);
#ifndef NICE_PLACE_ARITH
  // class and offset + 3 of the reference from the block's 16-entry table
  // (one 8-byte LDS read instead of two packed-constant extractions, one of
  // them across a word boundary, which compiled to a branch)
  const uint2 ct = idt[id];
  const uint32_t cls = ct.x, off3 = ct.y;
#else
  const uint32_t cls = (id < 8u ? ID_CLS_LO >> (4u * id) : ID_CLS_HI >> (4u * id - 32u)) & 15u;
  const uint32_t rows = (CLS_ROWS_PACK >> (2u * cls)) & 3u;
  const uint32_t b3 = 3u * cls;   // px + 3 at bits 3cls (48 bits over two words)
  const uint32_t pxp = (b3 < 32u ? (CLS_PX_LO >> b3) | (b3 > 29u ? CLS_PX_HI << (32u - b3) : 0u)
                                 : CLS_PX_HI >> (b3 - 32u)) & 7u;
  const uint32_t off3 = rows * W + pxp;   // offset + 3
#endif
  const bool bad_ref = (isbr && s0 >= 5u) || (islu && s0l >= 11u) || off3 < 3u || q + 3u < off3;
  const uint32_t gl = (s1 - 32u) & 255u;
  const uint32_t c_lu = ((s2 - 16u + gl) & 255u) | (gl << 10) | (((s3 - 16u + gl) & 255u) << 20);
  // (a conflict-free form by two reciprocal multiplies instead of this
  // gather measured the same: r06zr_ab_place_sdl_arith.log)
  const uint32_t c_sd = sdl[min(s0, 342u)];
  const uint32_t g2 = (s0 - 32u) & 255u;
  const uint32_t c_l2 = ((s1 - 16u + g2) & 255u) | (g2 << 10) | (((s2 - 16u + g2) & 255u) << 20);
  uint32_t c_rgb = (s0 & 255u) | (s1 << 10) | (s2 << 20);
  bad = (isbr || islu) ? bad_ref : (isl2 && q < W);
#ifndef NICE_PLACE_BRANCHY
  // the candidates opaque: otherwise the select chain compiles to a switch of
  // exec-masked branches on the prefix (about 35 scalar instructions and 8
  // branches per event, every prefix present in most waves)
  uint32_t c_br = (cls << 28) | (islu ? c_lu : 0u);
  uint32_t c_sd2 = c_sd, c_l22 = c_l2;
  asm volatile("" : "+v"(c_br), "+v"(c_sd2), "+v"(c_l22), "+v"(c_rgb));
  return (isbr || islu) ? c_br : issd ? c_sd2 : isl2 ? c_l22 : c_rgb;
#else
  return (isbr || islu) ? ((cls << 28) | (islu ? c_lu : 0u)) : issd ? c_sd : isl2 ? c_l2 : c_rgb;
#endif
}

// SMALL_DIFF index -> record constant (code.rs:230-247): index = rd + 7 gd + 49 bd
// (each difference + 3), constant = the three differences in spread form
struct alignas(16) SdlTable {
  uint32_t v[344];
};
constexpr SdlTable make_sdl_table() {
  SdlTable t{};
  for (uint32_t i = 0; i < 343u; ++i) {
    const uint32_t rd = i % 7u, t1 = i / 7u;
    t.v[i] = ((rd - 3u) & 255u) | ((((t1 % 7u) - 3u) & 255u) << 10) | ((((t1 / 7u) - 3u) & 255u) << 20);
  }
  return t;
}
__device__ __constant__ SdlTable kSdl = make_sdl_table();

__global__ __launch_bounds__(64 * DEC_PLACE_WAVES) void dec_place(DecArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t sdl[344];   // kSdl (code.rs:230-247)
  __shared__ uint2 idt[16];       // reference id -> {class, rows * W + px + 3}
  if (threadIdx.x < 16u) {
    const uint32_t id = threadIdx.x;
    const uint32_t cls = (uint32_t)(ID_CLS_PACK >> (4u * id)) & 15u;
    idt[id] = make_uint2(cls, (uint32_t)((CLS_ROWS_PACK >> (2u * cls)) & 3u) * a.W +
                                  (uint32_t)((CLS_PX_PACK >> (3u * cls)) & 7u));
  }
  // copied from a compile-time table: computing the 343 constants in every
  // block (divisions by 7 and 49) cost ~120 VALU per wave, and dec_place runs
  // one short-lived block per four slices
  if (threadIdx.x < 86u)
    reinterpret_cast<uint4*>(sdl)[threadIdx.x] = reinterpret_cast<const uint4*>(kSdl.v)[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  // grid (slices / waves, frames), XCD-aware: consecutive logical blocks are
  // dealt to one XCD (blocks b and b + 8 share one; bijective remap, guide T1),
  // so the two blocks whose slices share each 128-byte event line (8 slices'
  // 16-byte quads, interleaved per parse wave) read it through one L2
  const uint32_t nbx = gridDim.x, nwg = nbx * gridDim.y, lin = blockIdx.y * nbx + blockIdx.x;
  const uint32_t xq = nwg / 8u, xr = nwg % 8u, xcd = lin % 8u;
  const uint32_t lg = (xcd < xr ? xcd * (xq + 1u) : xr * (xq + 1u) + (xcd - xr) * xq) + lin / 8u;
  const uint32_t f = lg / nbx, j = (lg % nbx) * DEC_PLACE_WAVES + (threadIdx.x >> 6);
  if (a.status[f] != 0) return;
  const uint64_t len = a.stream_len[f];
  const uint64_t D = a.data_start[f];
  if (j >= n_chunks(len, D, a.chunk_bits)) return;
  const uint64_t base = (uint64_t)f * a.max_chunks;
  const uint32_t ag = a.agree[base + j], nev = a.ev_n[base + j];
  const uint32_t nvalid = (uint32_t)(a.last[base + j] >> 56);
  if (a.stats && lane == 0) {   // diagnostics: where the final parse met the first pass
    const uint32_t b = nev == EV_OVERFLOW ? 7u : ag == AGREE_NONE ? 6u : ag == 0u ? 0u : ag == 1u ? 1u
                     : ag <= 4u ? 2u : ag <= 16u ? 3u : ag <= 64u ? 4u : 5u;
    atomicAdd(&a.stats[50 + b], 1ull);
  }
  if (ag == AGREE_NONE || nev == EV_OVERFLOW || ag > nvalid) return;   // dec_emit parsed it all
  // (the bookkeeping loads issued together, the first checkpoint taken as
  // the meeting point before `agree` is in: no faster, r06zv_ab_pack_place.log)
  const uint64_t cki = (uint64_t)f * a.n_ck * a.max_chunks + j + (uint64_t)(ag ? ag - 1u : 0u) * a.max_chunks;
  const uint32_t i_first = ag == 0u ? 0u : a.ev_ck[cki];
  unsigned long long q = a.chunk_start[base + j] + (ag == 0u ? 0ull : (a.ck[cki] >> 32));
  const uint64_t N = (uint64_t)a.W * a.H;
  if (q > N) return;                    // tail bytes
  const uint32_t* evp = a.ev + ev_group(a, f, j);
  uint32_t* rec = a.recs + (uint64_t)f * a.rec_stride;
  const bool strict = (a.flags & NICE_DEC_STRICT_REFERENCE) != 0;
  bool err = false;
  // 256 events per step: 4 rows of 64 consecutive events (coalesced loads and
  // record stores), prefix sums per row plus the rows before
  // the next step's events, loaded one step ahead and unconditionally (lanes
  // past the slice's last event read that event again and are masked where
  // used): with every load issued, the compiler's wait at the top of a step
  // leaves the next step's four in flight (a conditional load with a zero
  // fill made it wait for all of them)
  if (i_first >= nev) return;
  const uint32_t ev_last = nev - 1u;
  uint32_t nx[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) nx[k] = evp[ev_word(min(i_first + 64u * k + lane, ev_last))];
  for (uint32_t i = i_first; i < nev; i += 256u) {
    uint32_t ev[4], r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ev[k] = nx[k];
      nx[k] = evp[ev_word(min(i + 256u + 64u * k + lane, ev_last))];
    }
    // fast path (nearly every step): every count < 2^16, so positions and
    // sums stay 32-bit (q <= N <= 2^30), and no event reaches the frame end or
    // carries a bad reference -- one uniform check, then plain stores
    {
      const uint32_t N32 = (uint32_t)N;
      uint32_t c32[4];
      bool big = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool valid = i + 64u * k + lane < nev;
        c32[k] = valid ? ((ev[k] & EV_RUN) ? (ev[k] & ~EV_RUN) : 1u) : 0u;
        big = big || c32[k] >= 65536u;
      }
      if (!__any(big)) {
        uint32_t qb[4];
        uint32_t base = (uint32_t)q;
        bool stop = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          // rows past the slice's last event (a slice's last step is mostly
          // empty): skipped by a uniform branch, not computed under a mask
          if (i + 64u * k >= nev) break;
          const bool valid = i + 64u * k + lane < nev;
          const bool run = (ev[k] & EV_RUN) != 0u;
          const uint32_t incl = wave_incl_scan(c32[k]);
          qb[k] = base + incl - c32[k];
          base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
          bool rbad = false;
          r[k] = place_record(ev[k], min(qb[k], N32), a.W, sdl, idt, rbad);
          stop = stop || (valid && (qb[k] >= N32 || (run ? qb[k] + c32[k] > N32 : rbad)));
        }
        if (!__any(stop)) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (i + 64u * k >= nev) break;
            if (i + 64u * k + lane < nev && !(ev[k] & EV_RUN)) rec[qb[k]] = r[k] | rec_tagbits(a.rec_tag);
          }
          q = base;
          continue;
        }
      }
    }
    // exact path: 64-bit positions, the first event at the frame end or in error stops
    unsigned long long c[4], qk[4], carry = 0;
    uint32_t stop_k = 4u, stop_lane = 64u;
    bool stop_at_n = false, stop_run = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = i + 64u * k + lane;
      const bool valid = x < nev;
      const bool run = (ev[k] & EV_RUN) != 0u;
      c[k] = valid ? (run ? (ev[k] & ~EV_RUN) : 1u) : 0u;
      unsigned long long incl;
      if (!__any(c[k] >= (1u << 25))) {   // 64 counts < 2^25: a 32-bit scan
        incl = wave_incl_scan((uint32_t)c[k]);
      } else {
        incl = c[k];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned long long t = __shfl_up(incl, o);
          if ((int)lane >= o) incl += t;
        }
      }
      const unsigned long long qb = q + carry + incl - c[k];   // pixels before this event
      carry += __shfl(incl, 63);
      qk[k] = qb;
      bool rbad = false;
      r[k] = place_record(ev[k], (uint32_t)min(qb, N), a.W, sdl, idt, rbad);
      // a zero-count run event is a zero digit continuing a run (the first
      // digit counts >= 1): at N the reference's run loop reads it and goes on
      const bool at_n = valid && qb == N && !(run && c[k] == 0);
      const bool bad = valid && !at_n && (run ? qb + c[k] > N : rbad);
      const unsigned long long m = __ballot(at_n || bad);
      if (stop_k == 4u && m) {
        stop_k = (uint32_t)k;
        stop_lane = (uint32_t)__builtin_ctzll(m);
        stop_at_n = __shfl(at_n ? 1 : 0, (int)stop_lane) != 0;
        stop_run = __shfl(run ? 1 : 0, (int)stop_lane) != 0;
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool keep = (uint32_t)k < stop_k || ((uint32_t)k == stop_k && lane < stop_lane);
      if (keep && i + 64u * k + lane < nev && !(ev[k] & EV_RUN)) rec[qk[k]] = r[k] | rec_tagbits(a.rec_tag);
    }
    if (stop_k < 4u) {
      if (lane == 0) err = stop_at_n ? (strict && stop_run) : true;
      break;
    }
    q += carry;
  }
  if (err) set_status(&a.status[f], NICE_E_FORMAT);
}

// ---------------------------------------------------------------------------
// D5: reconstruction.
// ---------------------------------------------------------------------------
struct RecLds {
  uint32_t y4tail[4];
  int32_t ref_k[16], ref_d[16];
  int32_t ref_off32[16];   // k*W + d per record class, clamped to [0, 4] (only 0..3 are special)
  int32_t err;
  uint32_t pad[3];
};

// Per-channel cyclic intervals [lo, lo+len] (mod 256) for the three channels
// in the "spread" layout (fields at bits 0, 10, 20 with two guard bits), so one
// 32-bit op acts on all channels.  An exact value is an interval with len 0;
// unknown is lo 0, len 255.  Rows are stored spread as well.
constexpr uint32_t SP_K = 0xFFu | (0xFFu << 10) | (0xFFu << 20);
constexpr uint32_t SP_K9 = 0x1FFu | (0x1FFu << 10) | (0x1FFu << 20);
constexpr uint32_t SP_1 = 1u | (1u << 10) | (1u << 20);
struct IvS { uint32_t lo, len; };
__device__ __forceinline__ uint32_t spread3(uint32_t v) {   // R | G<<8 | B<<16 -> spread
  return (v & 0xFFu) | ((v & 0xFF00u) << 2) | ((v & 0xFF0000u) << 4);
}
// unspread3(v) | alpha by two byte permutes of v (R), v >> 2 (G), v >> 4 (B):
// asel = 0x0D060100 (alpha byte 0xFF) or 0x0C060100 (0x00); 4 instructions
// per pixel instead of 7
__device__ __forceinline__ uint32_t unspread3_perm(uint32_t v, uint32_t asel) {
  const uint32_t rg = __builtin_amdgcn_perm(v >> 2, v, 0x0C0C0500u);
  return __builtin_amdgcn_perm(v >> 4, rg, asel);
}
__device__ __forceinline__ uint32_t unspread3(uint32_t v) {
  return (v & 0xFFu) | ((v >> 2) & 0xFF00u) | ((v >> 4) & 0xFF0000u);
}
__device__ __forceinline__ IvS ivs_exact(uint32_t sp) { return IvS{sp, 0u}; }
__device__ __forceinline__ IvS ivs_add(IvS a, uint32_t c) { return IvS{(a.lo + c) & SP_K, a.len}; }
// floor((L + U) / 2) + c over an interval L: halves it unless it wraps past
// 255, in which case the hull of both halves is [U/2, (255+U)/2] -- the
// average of the whole range [0, 255], so a wrapping field is widened to that
// before the one averaging (instead of averaging both forms and selecting).
__device__ __forceinline__ IvS ivs_avg(IvS l, uint32_t u, uint32_t c) {
  const uint32_t s = l.lo + l.len;
  const uint32_t wm = ((s >> 8) & SP_1) * 0x3FFu;        // fields whose interval wraps
  const uint32_t lo0 = l.lo & ~wm, s0 = (s & ~wm) | (SP_K & wm);
  const uint32_t lo1 = ((lo0 + u) >> 1) & SP_K;
  const uint32_t hi1 = ((s0 + u) >> 1) & SP_K9;
  return IvS{(lo1 + c) & SP_K, hi1 - lo1};
}

// Row storage: R rows x W spread pixels (R = 4 for W >= 3, else 8) and the last
// 3 pixels of row y-4 (offsets 3W+1, 3W+3).
struct RowCtx {
  uint32_t* ring;
  const uint32_t* y4tail;
  uint32_t W, y, rmask;
  __device__ __forceinline__ uint32_t* row(uint32_t r) const { return ring + (size_t)(r & rmask) * W; }
};

// Pixels [x0, x_stop) of the current row from their records; r0..r2 are the
// pixels before x0 (intervals).  Branch-free step: the averaging value and the
// reference value are both formed and one is selected.  Every value is written
// to the row (unknown ones are rewritten by the fix-up pass before anything
// reads them: the only same-row reads are of pixels 0..2, which lane 0 -- exact
// from the start -- writes at its steps 0..2, before the last segment reaches
// its last three columns; the host keeps that segment >= 6 pixels long).
// Returns the last segment-local index left unknown (-1: none).
__device__ __forceinline__ int run_segment(const RowCtx& rc, const RecLds& L, const uint32_t* recs,
                                           uint32_t x0, uint32_t x_stop, IvS r0, IvS r1, IvS r2) {
  int last_unknown = -1;
  const uint32_t y = rc.y;
  const uint32_t W = rc.W;
  uint32_t* row = rc.row(y);
  const uint32_t* up = rc.row(y - 1);       // unused on row 0
  const bool has_up = y > 0;
  for (uint32_t x = x0; x < x_stop; ++x) {
    const uint32_t r = recs[x];
    const uint32_t u = up[x];
    const bool ref = rec_cls(r) != 0;   // run pixels are class 1 (the pixel before) with c = 0
    const uint32_t c = rec_c(r);
    // reference value (kind REF): recent pixels or a pixel of the ring
    const int id = (int)rec_cls(r);
    const int off = (int)L.ref_off32[id];
    int jx = (int)x - L.ref_d[id];
    int jy = (int)y - L.ref_k[id];
    if (W >= 4) {                 // one wrap at most (|d| <= 3)
      const int wrapl = jx < 0, wrapr = jx >= (int)W;
      jx += wrapl ? (int)W : (wrapr ? -(int)W : 0);
      jy += wrapr - wrapl;
    } else {                      // tiny widths: general linear index
      const int64_t j = (int64_t)y * W + x - ((int64_t)L.ref_k[id] * W + L.ref_d[id]);
      const int64_t jj = j < 0 ? 0 : j;
      jy = (int)(jj / W);
      jx = (int)(jj - (int64_t)jy * W);
    }
    jx = min(max(jx, 0), (int)W - 1);
    const uint32_t far = (jy + 4 == (int)y && rc.rmask == 3u)
                             ? rc.y4tail[max(jx - (int)(W - 3), 0)]
                             : rc.ring[(size_t)((uint32_t)jy & rc.rmask) * W + (uint32_t)jx];
    IvS src;
    src.lo = off == 1 ? r0.lo : off == 2 ? r1.lo : off == 3 ? r2.lo : off == 0 ? 0u : far;
    src.len = off == 1 ? r0.len : off == 2 ? r1.len : off == 3 ? r2.len : 0u;
    src = ref ? src : r0;
    const IvS va = ivs_avg(r0, u, c);
    const IvS vr = ivs_add(src, c);
    const bool avg = !ref && has_up;
    const IvS v{avg ? va.lo : vr.lo, avg ? va.len : vr.len};
    row[x] = v.lo;
    last_unknown = v.len ? (int)(x - x0) : last_unknown;
    r2 = r1; r1 = r0; r0 = v;
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
  if (a.redo && a.hand_abort[f] != SPLIT_REDO) return;
  if (a.status[f] != 0) return;
  if (lane < 16) {
    L.ref_k[lane] = cls_rows(lane);
    L.ref_d[lane] = cls_px(lane);
    const int64_t off = (int64_t)cls_rows(lane) * W + cls_px(lane);
    L.ref_off32[lane] = (int32_t)(off < 0 ? 4 : off > 4 ? 4 : off);
  }
  if (lane == 0) L.err = 0;
  __syncthreads();
  const uint32_t S = a.seg, nseg = a.nseg;
  const uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint8_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 255 : 0;
  const bool active = (uint32_t)lane < nseg;
  const uint32_t x0 = lane * S;
  const uint32_t x1 = active ? ((uint32_t)lane == nseg - 1 ? W : x0 + S) : x0;
  const uint32_t seglen = x1 - x0;

  unsigned long long t_a = 0, t_b = 0, t_c = 0, t_d = 0;
  for (uint32_t y = 0; y < H; ++y) {
    const unsigned long long c0 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    RowCtx rc{ring, L.y4tail, W, y, R - 1};
    if (R == 4 && y >= 4 && lane < 3) L.y4tail[lane] = rc.row(y)[W - 3 + lane];
    // this row's records, coalesced
    const uint32_t* rrow = recs + (uint64_t)y * W;
    for (uint32_t x = lane; x < W; x += 64) recbuf[x] = rec_canon(rrow[x], a.rec_tag);
    __syncthreads();
    auto linear_px = [&](int64_t j) -> uint32_t {
      if (j < 0) return 0u;   // pixel 0's left neighbour is itself, not yet written (0)
      const uint64_t jy = (uint64_t)j / W, jx = (uint64_t)j - jy * W;
      return (R == 4 && jy + 4 == y) ? L.y4tail[jx - (W - 3)] : rc.row((uint32_t)jy)[jx];
    };
    IvS r0, r1, r2;
    if (lane == 0) {
      r0 = ivs_exact(linear_px((int64_t)y * W - 1));
      r1 = ivs_exact(linear_px((int64_t)y * W - 2));
      r2 = ivs_exact(linear_px((int64_t)y * W - 3));
    } else {
      r0 = IvS{0u, SP_K}; r1 = r0; r2 = r0;
    }
    const unsigned long long c1 = a.stats ? __builtin_amdgcn_s_memtime() : 0;
    // speculative pass: lane 0 starts exact, the others from an unknown entry
    int last_unknown = -1;
    if (active) last_unknown = run_segment(rc, L, recbuf, x0, x1, r0, r1, r2);
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
    while (fin != ~0ull) {
      const bool mine = !((fin >> lane) & 1ull);
      const bool left_ok = lane == 0 || (((fin | tail_ok) >> (lane - 1)) & 1ull);
      const bool ready = mine && left_ok;
      if (ready) {
        r0 = ivs_exact(linear_px((int64_t)y * W + x0 - 1));
        r1 = ivs_exact(linear_px((int64_t)y * W + x0 - 2));
        r2 = ivs_exact(linear_px((int64_t)y * W + x0 - 3));
        const int lu = run_segment(rc, L, recbuf, x0, x0 + (uint32_t)last_unknown + 1, r0, r1, r2);
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
      for (uint32_t x = lane; x < W; x += 64) o32[x] = unspread3(row[x]) | ((uint32_t)alpha << 24);
    } else {
      for (uint32_t x = lane; x < W; x += 64) {
        const uint32_t v = unspread3(row[x]);
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

// ---------------------------------------------------------------------------
// D5b: multi-wave reconstruction (64 <= W <= 16384).  One block per frame,
// one lane per 16-pixel row segment (up to 1024 lanes).  A lane keeps its
// segment of the row above and of the current row in registers (the segment
// loop is unrolled), so the left-to-right recurrence touches no memory:
//   pre-pass  records (prefetched one row ahead) -> per-pixel kind and
//             constant; references into rows above read a ring of the last
//             four rows (LDS when it fits, else global)
//   spec      from the exact entry (lane 0) or an unknown one (others), as
//             per-channel cyclic intervals that collapse within a few pixels
//   fix-up    rounds across the block: a lane whose left neighbour's last
//             three pixels are exact recomputes its unknown prefix exactly;
//             the others refine theirs from the neighbour's current intervals
//             (sound, so anything that collapses is final)
//   emit      pixels to the ring and the caller's raster
// ---------------------------------------------------------------------------
constexpr int ROWS_SEG = 16;
constexpr uint32_t ROWS_RING = 4;   // rows y-4 .. y-1 while row y is built

// Per-pixel word: spread constant c in the field bits, the kind as one-hot
// flags in the guard bits -- W_L1/W_L2/W_L3: c plus the pixel 1..3 back;
// W_AVG: c plus floor((left + up) / 2); W_CUR: c plus one of pixels 0..2 of the
// current row (index in bits 8..9), unknown until lane 0 has them; none: the
// constant itself (a reference into a row above, already added).
constexpr uint32_t W_L1 = 1u << 28, W_AVG = 1u << 31, W_CUR = 1u << 18;   // W_L2, W_L3: bits 29, 30
// Kind bits >> 28 per record class, 4 bits per class: class 0 is the average
// (on row 0: the pixel to the left), classes 1-3 the pixel 1-3 back, classes
// 4-13 a pixel of a row above (no bits; W_CUR is added per pixel).
constexpr unsigned long long ROWS_KIND = (W_AVG >> 28) | ((unsigned long long)(W_L1 >> 28) << 4) |
                                         ((unsigned long long)((W_L1 << 1) >> 28) << 8) |
                                         ((unsigned long long)((W_L1 << 2) >> 28) << 12);
constexpr unsigned long long ROWS_KIND_Y0 = (ROWS_KIND & ~15ull) | (W_L1 >> 28);
static_assert((W_AVG >> 28) == 8u && (W_L1 >> 28) == 1u, "kind bits 28..31");
__device__ __forceinline__ uint32_t wmask(uint32_t w, int bit) {
  return (uint32_t)__builtin_amdgcn_sbfe((int)w, bit, 1);   // 0 or ~0
}
// One pixel: kinds are selected with masks (no control flow, no SGPR masks).
// The constant is the word itself: its kind bits (18, 28..31) only reach a
// field's guard bits or bits >= 28 of the sums, which the masks after every
// add clear (no carry reaches a lower field: value bits <= 255 + 255 + 512).
// CUR = false: the caller knows no word holds W_CUR (waves without the row's
// last columns), two instructions fewer.
template <bool CUR = true>
__device__ __forceinline__ IvS rows_step(IvS l1, IvS l2, IvS l3, uint32_t u, uint32_t wp) {
  const uint32_t c = wp;
  const IvS va = ivs_avg(l1, u, c);
  const uint32_t m1 = wmask(wp, 28), m2 = wmask(wp, 29), m3 = wmask(wp, 30);
  const uint32_t ma = wmask(wp, 31);
  const uint32_t slo = (l1.lo & m1) | (l2.lo & m2) | (l3.lo & m3);
  const uint32_t slen = (l1.len & m1) | (l2.len & m2) | (l3.len & m3) | (CUR ? SP_K & wmask(wp, 18) : 0u);
  const uint32_t rlo = (slo + c) & SP_K;
  return IvS{(va.lo & ma) | (rlo & ~ma), (va.len & ma) | (slen & ~ma)};
}

// rows_chain when every input is exact (r0..r2 and the kept pixels): plain
// arithmetic, no intervals.  Only after the W_CUR words are resolved.
__device__ __forceinline__ uint32_t rows_step_exact(uint32_t l1, uint32_t l2, uint32_t l3, uint32_t u,
                                                    uint32_t wp) {
  // (l1 + u) >> 1 leaves the next field's lowest bit in each guard bit 9:
  // with c (the word: no W_CUR bit once resolved) a field sums to <= 1022, so
  // one mask at the end clears both
  const uint32_t c = wp;
  // kinds as sign-extended bit masks: and / and-or / bit-insert selects, the
  // constant added once after the average-or-copy select (instead of compare
  // and select chains: one 4K frame reconstruct 9.02 -> 8.72 ms, 64 x 1080p
  // 4.10 -> 3.95, profiles/r05zr_ab_flow_steps.log)
  const uint32_t sel = (l1 & wmask(wp, 28)) | (l2 & wmask(wp, 29)) | (l3 & wmask(wp, 30));
  const uint32_t ma = (uint32_t)((int32_t)wp >> 31);
  const uint32_t x = (((l1 + u) >> 1) & ma) | (sel & ~ma);
  return (x + c) & SP_K;
}

// Speculative pass over the whole segment; returns -1 when every pixel is
// exact, S - 4 when the last three are, else S - 1 (a bound on the last unknown).
// (Switching a wave to the plain step once all its lanes are exact -- one
// vote per pixel -- was 5 % slower: each vote's branch waits on the VALU.)
// A partial last segment's padding pixels are run records (copies of the pixel
// before, interval width included), so counting them leaves "every pixel
// exact" unchanged and spares 16 loop-invariant lane masks (SGPR spills).
template <int S>
__device__ __forceinline__ int rows_spec(IvS (&v)[S], IvS r0, IvS r1, IvS r2, const uint32_t (&w)[S],
                                         const uint32_t (&prev)[S]) {
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const IvS l1 = p >= 1 ? v[p - 1] : r0;
    const IvS l2 = p >= 2 ? v[p - 2] : (p == 1 ? r0 : r1);
    const IvS l3 = p >= 3 ? v[p - 3] : (p == 2 ? r0 : (p == 1 ? r1 : r2));
    v[p] = rows_step(l1, l2, l3, prev[p], w[p]);
  }
  // a coarse last unknown index from two OR trees instead of a compare and a
  // select per pixel: its users only ask "any unknown" and "last three exact",
  // and the fix-up chain recomputing exact pixels too is harmless (512-frame
  // reconstruct 20.03 -> 19.63 ms)
  uint32_t head = 0, tail = v[S - 1].len | v[S - 2].len | v[S - 3].len;
#pragma unroll
  for (int p = 0; p < S - 3; ++p) head |= v[p].len;
  return tail ? S - 1 : head ? S - 4 : -1;
}

// Recomputes pixels 0..lu (lanes with `go`), keeping the others (already
// exact); returns the new last unknown index.  Stops once no lane of the wave
// has work left.
template <int S>
__device__ __forceinline__ int rows_chain(IvS (&v)[S], IvS r0, IvS r1, IvS r2, const uint32_t (&w)[S],
                                          const uint32_t (&prev)[S], int lu, bool go) {
  int nlu = -1;
  const int upto = go ? lu : -1;
#pragma unroll
  for (int p = 0; p < S; ++p) {
    if (!__any(p <= upto)) break;
    const IvS l1 = p >= 1 ? v[p - 1] : r0;
    const IvS l2 = p >= 2 ? v[p - 2] : (p == 1 ? r0 : r1);
    const IvS l3 = p >= 3 ? v[p - 3] : (p == 2 ? r0 : (p == 1 ? r1 : r2));
    const IvS n = rows_step(l1, l2, l3, prev[p], w[p]);
    const bool upd = p <= upto;
    v[p].lo = upd ? n.lo : v[p].lo;
    v[p].len = upd ? n.len : v[p].len;
    nlu = (upd && n.len) ? p : nlu;
  }
  return go ? nlu : lu;
}

template <int S>
__device__ __forceinline__ int rows_chain_exact(IvS (&v)[S], IvS r0, IvS r1, IvS r2, const uint32_t (&w)[S],
                                                const uint32_t (&prev)[S], int lu, bool go) {
  const int upto = go ? lu : -1;
  // all S steps, predicated: a vote per pixel to stop early (its branch waits
  // on the VALU) made a single 4K frame 4 % slower, same at 512 frames (one
  // vote per call to skip waves with nothing to recompute, and kind masks
  // instead of the select chain, were no faster either)
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const uint32_t l1 = p >= 1 ? v[p - 1].lo : r0.lo;
    const uint32_t l2 = p >= 2 ? v[p - 2].lo : (p == 1 ? r0.lo : r1.lo);
    const uint32_t l3 = p >= 3 ? v[p - 3].lo : (p == 2 ? r0.lo : (p == 1 ? r1.lo : r2.lo));
    const uint32_t n = rows_step_exact(l1, l2, l3, prev[p], w[p]);
    const bool upd = p <= upto;
    v[p].lo = upd ? n : v[p].lo;
    v[p].len = upd ? 0u : v[p].len;
  }
  return go ? -1 : lu;
}

// Block barrier; with the ring in LDS only LDS traffic is ordered, so global
// stores (the raster) and the record prefetch stay in flight across it.
template <bool LDS_RING>
__device__ __forceinline__ void rows_barrier() {
  if constexpr (LDS_RING) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  } else {
    __syncthreads();
  }
}

// Ring row: W pixels padded one word per 16 (pixel x at x + (x >> 4)), plus 16
// spare words that take a partial last segment's padding pixels (stored
// unmasked), and halos so that no reference needs wrap logic: words -4..-2 hold
// the previous row's last three pixels (x = -3..-1), words g(W..W+2) the next
// row's first three (written when that row is emitted; the spare words of the
// previous use are overwritten by then).
constexpr uint32_t ROWS_RB = 4;   // left halo words before pixel 0
__host__ __device__ constexpr uint32_t rows_ring_stride(uint32_t W) { return W + (W >> 4) + 24; }

template <int MAXT, bool LDS_RING, int S = ROWS_SEG>
__device__ __forceinline__ void dec_rows_body(const DecArgs& a) {
  // diagnostics counters (NICE_DEC_STATS=1) only in -DNICE_ROWS_STATS builds:
  // the runtime checks alone held SGPRs and branches in the row loop
#ifdef NICE_ROWS_STATS
  unsigned long long* const stats = a.stats;
#else
  constexpr unsigned long long* stats = nullptr;
#endif
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  // per record class: rows back (bits 0-1), pixels back + 3 (bits 2-4), kind
  // bits (28-31); entries 16.. for row 0.  One LDS read per pixel instead of
  // three shifts of packed 64-bit constants.
  __shared__ uint32_t clsw[32];
  if (threadIdx.x < 32) {
    const uint32_t c = threadIdx.x & 15u;
    const unsigned long long kinds = threadIdx.x >= 16 ? ROWS_KIND_Y0 : ROWS_KIND;
    clsw[threadIdx.x] = ((CLS_ROWS_PACK >> (2 * c)) & 3u) | (uint32_t)((CLS_PX_PACK >> (3 * c)) & 7u) << 2 |
                        ((uint32_t)(kinds >> (4u * c)) & 15u) << 28;
  }
  const uint32_t nthr = blockDim.x;
  const uint32_t W = a.W, H = a.H;
  uint32_t* tails = sm;                 // nthr x {lo, len} x 3 (pixels S-1, S-2, S-3)
  uint32_t* flags = tails + nthr * 6;   // nthr: last three pixels exact
  uint32_t* head3 = flags + nthr;       // pixels 0..2 of the current row
  uint32_t* pend = head3 + 4;           // 2 round flags
  int* err = reinterpret_cast<int*>(pend + 2);
  const uint32_t f = blockIdx.x;
  // ring rows padded one word per 16 pixels: lane i's segment starts at bank
  // 17i mod 32, so the lanes' accesses to their segments are conflict free
  const uint32_t RS = rows_ring_stride(W);
  uint32_t* ring = (LDS_RING ? (sm + nthr * 7 + 8) : (a.rowbuf + (uint64_t)f * ROWS_RING * RS)) + ROWS_RB;
  // per-row class table (S == 16), double-buffered by row parity: x = kind bits
  // | pixels back + 3, y = ring offset of the referenced row's pixel 0 plus 3
  // minus pixels back, so a reference's word is 17 * lane + p + y (+ a +-1
  // padding correction for the first and last three pixels of a segment)
  __shared__ uint2 rtab[2][16];
  auto build_tab = [&](uint32_t yy) {
    if (threadIdx.x < 16) {
      const uint32_t c = threadIdx.x;
      const unsigned long long kinds = yy == 0 ? ROWS_KIND_Y0 : ROWS_KIND;
      const uint32_t rows = (CLS_ROWS_PACK >> (2 * c)) & 3u, dxp3 = (uint32_t)(CLS_PX_PACK >> (3 * c)) & 7u;
      rtab[yy & 1u][c] = make_uint2((((uint32_t)(kinds >> (4u * c)) & 15u) << 28) | dxp3,
                                    ((yy - rows) & (ROWS_RING - 1)) * RS + 3u - dxp3);
    }
  };
  if (S == 16) build_tab(0);
  if (a.redo && a.hand_abort[f] != SPLIT_REDO) return;   // block-uniform
  if (a.status[f] != 0) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t nseg = (W + S - 1) / S;
  const bool active = lane < nseg;
  const uint32_t x0 = lane * S;
  const int nvalid = active ? (int)min((uint32_t)S, W - x0) : 0;
  const uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint32_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 0xFF000000u : 0u;
  const uint32_t asel = alpha ? 0x0D060100u : 0x0C060100u;   // unspread3_perm
  const bool vec_rec = (W & 3u) == 0 && nvalid == S;
  const bool vec_out = (OC == 4 && (W & 3u) == 0 && nvalid == S) ||
                       (OC == 3 && S % 16 == 0 && (W & 15u) == 0 && nvalid == S);
  if (lane == 0) *err = 0;
  uint32_t prev[S], rn[S];
#pragma unroll
  for (int p = 0; p < S; ++p) prev[p] = 0;
  auto load_recs = [&](uint32_t y) {
    const uint32_t* rrow = recs + (uint64_t)y * W + x0;
    if (vec_rec) {
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        const uint4 t = reinterpret_cast<const uint4*>(rrow)[q];
        rn[4 * q] = t.x; rn[4 * q + 1] = t.y; rn[4 * q + 2] = t.z; rn[4 * q + 3] = t.w;
      }
    } else if (nvalid > 0) {   // a partial last segment
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = p < nvalid ? rrow[p] : REC_RUN;
    } else {                   // idle lane: no loads (its wave would run the masked path every row)
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = REC_RUN;
    }
  };
  if (H > 0) load_recs(0);
  __syncthreads();
  unsigned long long t_a = 0, t_b = 0, t_c = 0, t_d = 0, n_fix = 0;
  for (uint32_t y = 0; y < H; ++y) {
    const unsigned long long c0 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- pre-pass: records -> per-pixel words
    const uint32_t* const cwt = clsw + (y == 0 ? 16 : 0);
    uint32_t w[S];
#ifdef NICE_AB_PRE2   // A/B probe: the pre-pass twice (its cost)
    for (int rep = 0; rep < 2; ++rep) {
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
#else
    {
      constexpr uint32_t z = 0;
#endif
    if constexpr (S == 16) {
      // table form: every lane, no wrap logic (ring halos); only the last
      // lane's references to the current row (W_CUR) are patched below
      const uint2* tb = rtab[y & 1u];
      const uint32_t lb = 17u * lane;
#pragma unroll
      for (int p = 0; p < S; ++p) {
        const uint32_t r = rec_canon(rn[p] + z, a.rec_tag);
        const uint32_t cls = rec_cls(r);                     // 0..13
        const uint2 e = tb[cls];
        uint32_t ad = lb + e.y;
        if (p < 3 || p > S - 4) ad += (uint32_t)((int)(p + 3u - (e.x & 7u)) >> 4);   // padding word crossed
        const uint32_t o = ring[ad + p];
        const uint32_t c = rec_c(r);
        // (a VALU mask from a table bit instead of the compare: 4 % slower)
        w[p] = (e.x & 0xF0000000u) | (((cls >= 4u ? o : 0u) + c) & SP_K);
      }
      // references past the row end into row y itself (pixels 0..2): only
      // columns W-3 .. W-1 have them -- the last segment, and the one before
      // it when the last holds fewer than three pixels (W % 16 in {1, 2}).
      // Branch-free (per-pixel branches held exec masks in SGPRs, which
      // spilled), and only the wave holding those lanes runs it.
      if (x0 + S + 2u >= W) {
#pragma unroll
        for (int p = 0; p < S; ++p) {
          const uint32_t r = rec_canon(rn[p], a.rec_tag);   // padding: a run record (class 1)
          const uint32_t cls = rec_cls(r);
          const uint32_t tx = x0 + p + 3u - ((uint32_t)(CLS_PX_PACK >> (3u * cls)) & 7u);
          const bool cur = cls >= 4u && ((CLS_ROWS_PACK >> (2u * cls)) & 3u) == 1u && tx >= W;
          w[p] = cur ? (W_CUR | rec_c(r) | ((tx - W) << 8)) : w[p];
        }
      }
    } else {
#pragma unroll
    for (int p = 0; p < S; ++p) {
      const uint32_t x = x0 + p;
      const uint32_t r = rec_canon(rn[p] + z, a.rec_tag);
      const uint32_t cls = rec_cls(r);                       // 0..13
      const uint32_t cw = cwt[cls];                          // rows | px + 3 << 2 | kind bits
      const uint32_t rows = cw & 3u;
      const int dx = (int)((cw >> 2) & 7u) - 3;
      int tx = (int)x - dx;
      const int wl = tx < 0, wr = tx >= (int)W;
      tx += wl ? (int)W : (wr ? -(int)W : 0);
      const uint32_t back = rows + wl - wr;                  // rows above (0: current row)
      const bool up = cls >= 4;
      const bool cur = up && back == 0;
      // unconditional LDS read (a harmless in-range address for other classes)
      const uint32_t txc = (uint32_t)min(max(tx, 0), (int)W - 1);
      const uint32_t o = ring[__umul24((y - back) & (ROWS_RING - 1), RS) + txc + (txc >> 4)];
      const uint32_t c = rec_c(r);
      // kind bits from the class (branch-free: the ternary chain compiled to two
      // nested exec-masked branches per pixel)
      const uint32_t kb = (cw & 0xF0000000u) | (cur ? W_CUR : 0u);
      w[p] = kb | ((up && !cur) ? ((o + c) & SP_K) : c) | (cur ? ((uint32_t)tx << 8) : 0u);
    }
    }
    }
    // ---- entry: lane 0 exact (previous row's last pixels; 0 before pixel 0)
    IvS r0{0u, SP_K}, r1{0u, SP_K}, r2{0u, SP_K};
    if (lane == 0) {
      if (y == 0) {
        r0 = r1 = r2 = ivs_exact(0u);
      } else {
        const uint32_t* pr = ring + (size_t)((y - 1) & (ROWS_RING - 1)) * RS;
        r0 = ivs_exact(pr[(W - 1) + ((W - 1) >> 4)]);
        r1 = ivs_exact(pr[(W - 2) + ((W - 2) >> 4)]);
        r2 = ivs_exact(pr[(W - 3) + ((W - 3) >> 4)]);
      }
    }
    if (y + 1 < H) load_recs(y + 1);   // in flight during this row
    const unsigned long long c1 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- speculative pass
    IvS v[S];
    int lu = rows_spec<S>(v, r0, r1, r2, w, prev);
#ifdef NICE_AB_SPEC2   // A/B probe: the speculative pass twice (its cost)
    {
      IvS v2[S];
      const int lu2 = rows_spec<S>(v2, IvS{v[S - 1].lo & 1u, r0.len}, r1, r2, w, prev);
      lu = lu2 < -1 ? lu2 : lu;
#pragma unroll
      for (int p = 0; p < S; ++p) v[p].lo |= v2[p].len & 0x80000000u;
    }
#endif
    if (active) {
      uint32_t* t = tails + lane * 6;
      t[0] = v[S - 1].lo; t[1] = v[S - 1].len;
      t[2] = v[S - 2].lo; t[3] = v[S - 2].len;
      t[4] = v[S - 3].lo; t[5] = v[S - 3].len;
      flags[lane] = (lu < S - 3) ? 1u : 0u;
    }
    if (lane == 0) { head3[0] = v[0].lo; head3[1] = v[1].lo; head3[2] = v[2].lo; pend[0] = 0; pend[1] = 0; }
    bool fin = !active || lu < 0;
    if (stats && active && lu >= 0) {
      atomicAdd(&stats[1], 1ull);
      atomicAdd(&stats[3], (unsigned long long)(lu + 1));
      if (lu >= S - 3) atomicAdd(&stats[2], 1ull);
      // unknown tails: every tail pixel a full-width interval (a copy chain
      // from the unknown entry or a current-row reference) or some narrowed one
      const uint32_t tl0 = v[S - 1].len, tl1 = v[S - 2].len, tl2 = v[S - 3].len;
      if (tl0 | tl1 | tl2) {
        const bool copies = (tl0 == 0u || tl0 == SP_K) && (tl1 == 0u || tl1 == SP_K) && (tl2 == 0u || tl2 == SP_K);
        atomicAdd(&stats[copies ? 24 : 25], 1ull);
      }
    }
    rows_barrier<LDS_RING>();
    const unsigned long long c2 = stats ? __builtin_amdgcn_s_memtime() : 0;
    const unsigned long long nfix0 = n_fix;
#ifdef NICE_AB_ROUND   // A/B probe: one more (empty) fix-up round per row
    if (!fin) atomicOr(&pend[1], 0u);
    rows_barrier<LDS_RING>();
    if (pend[1] == 7u) lu = S;
    rows_barrier<LDS_RING>();
#endif
    // ---- fix-up rounds
    bool cur_done = false;
    for (uint32_t rd = 0;; ++rd) {
      if (!fin) atomicOr(&pend[rd & 1u], 1u);
      rows_barrier<LDS_RING>();
      if (pend[rd & 1u] == 0) break;
      ++n_fix;
      if (lane == 0) pend[(rd + 1) & 1u] = 0;
      if (!cur_done) {   // pixels 0..2 of the row are exact now (lane 0)
        if (x0 + S + 2u >= W) {   // the lanes that can hold W_CUR words (above)
          const uint32_t h0 = head3[0], h1 = head3[1], h2 = head3[2];
#pragma unroll
          for (int p = 0; p < S; ++p) {
            const uint32_t k = (w[p] >> 8) & 3u;
            const uint32_t hv = k == 0u ? h0 : k == 1u ? h1 : h2;
            w[p] = (w[p] & W_CUR) ? ((hv + (w[p] & SP_K)) & SP_K) : w[p];
          }
        }
        cur_done = true;
      }
      bool exact_in = false;
      if (!fin && lane > 0) {
        const uint32_t* t = tails + (lane - 1) * 6;
        r0 = IvS{t[0], t[1]}; r1 = IvS{t[2], t[3]}; r2 = IvS{t[4], t[5]};
        exact_in = flags[lane - 1] != 0;
      }
      rows_barrier<LDS_RING>();
      // only lanes whose left tail is exact recompute, with plain arithmetic:
      // refining from an inexact neighbour (interval chain) rarely collapses
      // anything in one round and forced its whole wave onto the interval
      // chain; the leftmost unfinished lane always has an exact left tail
      const bool go = !fin && exact_in;
#ifndef NICE_ROWS_HOIST
      // the words as opaque per round: otherwise the compiler hoists the select
      // masks of all 16 pixels out of the round loop, and their SGPR pairs
      // spill to VGPR lanes (a writelane per mask per row, a readlane per use)
#pragma unroll
      for (int p = 0; p < S; ++p) asm volatile("" : "+v"(w[p]));
#endif
      lu = rows_chain_exact<S>(v, r0, r1, r2, w, prev, lu, go);
      if (go) {
        if (lu >= 0) atomicCAS(err, 0, NICE_E_FORMAT);   // exact inputs give exact outputs
        uint32_t* t = tails + lane * 6;
        t[0] = v[S - 1].lo; t[1] = v[S - 1].len;
        t[2] = v[S - 2].lo; t[3] = v[S - 2].len;
        t[4] = v[S - 3].lo; t[5] = v[S - 3].len;
        flags[lane] = 1u;
        fin = true;
      }
    }
    if (stats && lane == 0) {
      const unsigned long long r = n_fix - nfix0;
      atomicAdd(&stats[9 + (r >= 6 ? 6 : r)], 1ull);
    }
    if (*err) break;
    const unsigned long long c3 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- emit: ring row y (its slot held row y-4, no longer referenced) and the raster
    if (active) {
      uint32_t* rr = ring + (size_t)(y & (ROWS_RING - 1)) * RS + x0 + (x0 >> 4);   // x0 = 16 * lane
      const uint64_t pix = (uint64_t)y * W + x0;
#pragma unroll
      for (int p = 0; p < S; ++p) rr[p] = v[p].lo;   // padding pixels land in the row's spare words
      if (lane == 0 && y > 0) {   // row y-1's right halo: this row's first three pixels
        uint32_t* h = ring + (size_t)((y - 1) & (ROWS_RING - 1)) * RS;
#pragma unroll
        for (int k = 0; k < 3; ++k) h[(W + k) + ((W + k) >> 4)] = v[k].lo;
      }
      // row y+1's left halo: this row's last three pixels -- from the last
      // segment and, when it holds fewer than three (W % 16 in {1, 2}), the one
      // before it (round 5 width sweep: W = 66, a row starting with a W+3
      // reference read a stale halo word)
      if (x0 + S + 2u >= W) {
        uint32_t* h = ring + (size_t)((y + 1) & (ROWS_RING - 1)) * RS;
#pragma unroll
        for (int p = 0; p < S; ++p)
          if (p < nvalid && x0 + p + 3u >= W) h[(int)(x0 + p - W) - 1] = v[p].lo;
      }
      if (vec_out && OC == 4) {
        uint4* o = reinterpret_cast<uint4*>(outp + pix * 4);
#pragma unroll
        for (int q = 0; q < S / 4; ++q)
          o[q] = make_uint4(unspread3_perm(v[4 * q].lo, asel), unspread3_perm(v[4 * q + 1].lo, asel),
                            unspread3_perm(v[4 * q + 2].lo, asel), unspread3_perm(v[4 * q + 3].lo, asel));
      } else if (vec_out) {
        if constexpr (S % 16 == 0) {
          uint32_t b[3 * S / 4];
#pragma unroll
          for (int q = 0; q < S / 4; ++q) {
            const uint32_t u0 = unspread3_perm(v[4 * q].lo, 0x0C060100u), u1 = unspread3_perm(v[4 * q + 1].lo, 0x0C060100u);
            const uint32_t u2 = unspread3_perm(v[4 * q + 2].lo, 0x0C060100u), u3 = unspread3_perm(v[4 * q + 3].lo, 0x0C060100u);
            b[3 * q] = __builtin_amdgcn_perm(u1, u0, 0x04020100u);       // R0 G0 B0 R1
            b[3 * q + 1] = __builtin_amdgcn_perm(u2, u1, 0x05040201u);   // G1 B1 R2 G2
            b[3 * q + 2] = __builtin_amdgcn_perm(u3, u2, 0x06050402u);   // B2 R3 G3 B3
          }
          uint4* o = reinterpret_cast<uint4*>(outp + pix * 3);
#pragma unroll
          for (int q = 0; q < 3 * S / 16; ++q) o[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
        }
      } else if (OC == 4) {
        uint32_t* o32 = reinterpret_cast<uint32_t*>(outp + pix * 4);
#pragma unroll
        for (int p = 0; p < S; ++p)
          if (p < nvalid) o32[p] = unspread3(v[p].lo) | alpha;
      } else {
        uint8_t* o8 = outp + pix * 3;
#pragma unroll
        for (int p = 0; p < S; ++p) {
          if (p < nvalid) {
            const uint32_t u = unspread3(v[p].lo);
            o8[3 * p] = (uint8_t)u; o8[3 * p + 1] = (uint8_t)(u >> 8); o8[3 * p + 2] = (uint8_t)(u >> 16);
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < S; ++p) { prev[p] = v[p].lo; }
    if (S == 16) build_tab(y + 1);   // the last readers of that buffer were row y-1's
    rows_barrier<LDS_RING>();
    if (stats) {
      const unsigned long long c4 = __builtin_amdgcn_s_memtime();
      t_a += c1 - c0; t_b += c2 - c1; t_c += c3 - c2; t_d += c4 - c3;
    }
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], (unsigned long long)H);
    atomicAdd(&stats[4], n_fix);
    atomicAdd(&stats[5], t_a); atomicAdd(&stats[6], t_b);
    atomicAdd(&stats[7], t_c); atomicAdd(&stats[8], t_d);
  }
  if (lane == 0 && *err) set_status(&a.status[f], *err);
}

// Ring in LDS (4 rows fit next to the block's tails) or in global memory.
__global__ __launch_bounds__(512) void dec_rows(DecArgs a) { dec_rows_body<512, true>(a); }
__global__ __launch_bounds__(1024) void dec_rows_wide(DecArgs a) { dec_rows_body<1024, false>(a); }
// 8-pixel segments (W <= 4096: up to 512 lanes): twice the lanes per frame,
// for batches too small to fill the CUs (single-frame latency)
__global__ __launch_bounds__(512) void dec_rows8(DecArgs a) { dec_rows_body<512, true, 8>(a); }

// ---------------------------------------------------------------------------
// D5d: dataflow row reconstruction for small batches (round 5; 64 <= W <=
// 4096, one frame per block, frames <= CUs).  dec_rows keeps every wave of a
// block on one row: a block barrier after the speculative pass, two per fix-up
// round, one after the emit, and the record pre-pass and the raster stores on
// the row's critical path.  At one frame per CU (single frames, config 3,
// small RGB batches) that path sets the decode time: 2160 rows of ~6.8 us for
// 4K.  Here the block's waves form K groups of WPR = ceil(segments / 64)
// waves; group g reconstructs rows g, g + K, ..., so rows overlap, and the
// waves synchronise only through LDS stamps (row + 1):
//   fin[slot][w]  wave w's segments of the row are final in the ring;
//   tst[slot][w]  the last three pixels of wave w's last segment are exact
//                 (tail[slot][w]): the next wave's first lane can fix up;
//   hst[slot]     the row's first three pixels (W_CUR references of the
//                 row's last columns, code.rs:141-145: offsets W-1, W-3 reach
//                 into the current row).
// Wave w of row y waits for row y-1's waves w-1..w+1 (the references reach
// +-3 pixels, rows 1..3 back: rows y-2, y-3 are final by induction), wave 0
// for all of row y-1 (its entry is the row's last pixels, code.rs:412-413),
// the last wave also for row y-1's wave 0 (right halos).  Then: pre-pass ring
// reads (the record decode and addresses are done before the wait), the
// speculative pass, and fix-up rounds inside the wave (lane shuffles, no
// barriers; the first lane takes the left wave's published tail), the ring
// row and halos, the stamp, and only then the raster stores and the next
// rows' record loads -- off the critical path.  A ring of 8 rows (K + 3 <= 8)
// in LDS.  Every dependency points to an earlier (row, wave) and all waves
// are resident, so the earliest unfinished one always progresses; every wait
// is bounded (0.2 s, then the frame fails with NICE_E_HIP and the other waves
// stop).
// ---------------------------------------------------------------------------
constexpr uint32_t FLOW_THREADS = 512;
constexpr uint32_t FLOW_SLOTS = 8;   // stamp slots

constexpr uint32_t FLOW_MAXW = 8;   // waves per row: W <= 8192 (round 6; 4 before)
constexpr unsigned long long FLOW_TIMEOUT = 20000000ull;   // s_memrealtime ticks (100 MHz): 0.2 s
// a timed-out wait (the workgroup preempted or time-sliced for longer than
// that) does not fail the frame: it is marked for the barrier kernel
// (dec_rows, launched after this one in redo mode) -- slower,
// never wrong
constexpr int FLOW_REDO = 1;
struct FlowCtl {
  uint32_t fin[FLOW_SLOTS][FLOW_MAXW];
  uint32_t tst[FLOW_SLOTS][FLOW_MAXW];
  uint32_t tail[FLOW_SLOTS][FLOW_MAXW][4];
  uint32_t hst[FLOW_SLOTS];
  uint32_t head[FLOW_SLOTS][4];
  uint2 rtab[FLOW_THREADS / 64][16];   // per wave: the class table of its current row
  uint32_t zero[4];                    // the "reference" word of records that have none
  int err;
  uint32_t abort;
  uint32_t pad[2];
};
static_assert(sizeof(FlowCtl) % 16 == 0, "ring after the control block, 16-byte aligned");
static_assert(sizeof(FlowCtl) == FLOW_CTL_BYTES_HOST && FLOW_THREADS == FLOW_THREADS_HOST, "host LDS sizing");
__device__ __forceinline__ uint32_t flow_peek(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// LDS-only release (the raster stores and record loads stay in flight)
__device__ __forceinline__ void flow_publish(uint32_t* p, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void flow_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
// the wave waits until stamps[i] >= want for every bit i of mask (lanes 0..3
// read one stamp each); false when the frame aborted or the wait timed out
__device__ __forceinline__ bool flow_wait(FlowCtl& C, const uint32_t* stamps, uint32_t mask, uint32_t want) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool mine = lane < FLOW_MAXW && ((mask >> lane) & 1u);
  unsigned long long t0 = 0;
  for (uint32_t n = 0;; ++n) {
    const uint32_t v = mine ? flow_peek(stamps + lane) : want;
    if (__ballot(v < want) == 0ull) break;
    if ((n & 31u) == 0u) {
      if (flow_peek(&C.abort)) return false;
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (n == 0) t0 = t;
      else if (t - t0 > FLOW_TIMEOUT) {
        atomicOr(&C.abort, 1u);
        atomicCAS(&C.err, 0, FLOW_REDO);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
  flow_acquire();
  return true;
}
// lane l gets lane l-1's value (lane 0: 0) by a DPP wave shift: one VALU move,
// no LDS round trip (ds_bpermute) on the hand-off path (one 4K frame 10.27 ->
// 10.21 ms, 64 x 1080p 4.79 -> 4.74, profiles/r05zl_ab_flow_dpp.log)
__device__ __forceinline__ uint32_t shfl_up1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
}
// The speculative pass; reports which parts of the segment stayed unknown
// (from OR trees over the interval widths instead of a compare and select per
// pixel): any pixel, any of pixels 8..15 (the fix-up chain's second half),
// any of the last three (the tail the next lane or wave starts from).  (A vote
// after pixel 7 switching the wave to the exact step when every lane's last
// three pixels were exact was neutral: 18.73 vs 18.64 ms at 512 frames,
// profiles/r05w_ab_flow_spec.log.)
struct SpecUnk { uint32_t any, hi, tail; };
template <int S, bool CUR>
__device__ __forceinline__ SpecUnk rows_spec_unk(IvS (&v)[S], IvS r0, IvS r1, IvS r2, const uint32_t (&w)[S],
                                                 const uint32_t (&prev)[S]) {
  static_assert(S == 16, "halves of eight pixels");
#pragma unroll
  for (int p = 0; p < S; ++p) {
    const IvS l1 = p >= 1 ? v[p - 1] : r0;
    const IvS l2 = p >= 2 ? v[p - 2] : (p == 1 ? r0 : r1);
    const IvS l3 = p >= 3 ? v[p - 3] : (p == 2 ? r0 : (p == 1 ? r1 : r2));
    v[p] = rows_step<CUR>(l1, l2, l3, prev[p], w[p]);
  }
  const uint32_t tail = v[13].len | v[14].len | v[15].len;
  const uint32_t hi = tail | v[8].len | v[9].len | v[10].len | v[11].len | v[12].len;
  const uint32_t lo = v[0].len | v[1].len | v[2].len | v[3].len | v[4].len | v[5].len | v[6].len | v[7].len;
  return SpecUnk{lo | hi, hi, tail};
}
// Exact recompute of pixels 0..7 and, when some lane with `hi` goes, 8..15,
// of the lanes with `go` (their entry is exact); the second half
// only when some lane of the wave still has unknown pixels there (one vote per
// round: 512 x 4K reconstruct -1 %, 1024 x 1080p -2 %, profiles/r05v_ab_chunks.log;
// votes every four pixels cost more than they saved at one frame per CU).
template <int S>
__device__ __forceinline__ void rows_chain_upto(IvS (&v)[S], IvS r0, IvS r1, IvS r2, const uint32_t (&w)[S],
                                                const uint32_t (&prev)[S], bool go, bool hi) {
  auto step = [&](int p) {
    const uint32_t l1 = p >= 1 ? v[p - 1].lo : r0.lo;
    const uint32_t l2 = p >= 2 ? v[p - 2].lo : (p == 1 ? r0.lo : r1.lo);
    const uint32_t l3 = p >= 3 ? v[p - 3].lo : (p == 2 ? r0.lo : (p == 1 ? r1.lo : r2.lo));
    const uint32_t n = rows_step_exact(l1, l2, l3, prev[p], w[p]);
    // a lane with an exact entry recomputes every pixel of the half (the ones
    // past its last unknown come out equal): one select on a lane mask per
    // pixel instead of a compare and a select (with the caller's asm pin of
    // the words, which cost a copy of each per round, removed: 512 x 4K
    // reconstruct 17.53 -> 16.86 ms, one 4K frame 9.56 -> 9.08,
    // profiles/r05zq_ab_flow_chain.log)
    v[p].lo = go ? n : v[p].lo;
  };
#pragma unroll
  for (int p = 0; p < 8; ++p) step(p);
  if (__ballot(go && hi) != 0ull) {
#pragma unroll
    for (int p = 8; p < 16; ++p) step(p);
  }
}
__global__ __launch_bounds__(FLOW_THREADS) void dec_rows_flow(DecArgs a) {
  constexpr int S = ROWS_SEG;
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  FlowCtl& C = *reinterpret_cast<FlowCtl*>(sm);
  constexpr uint32_t CTL_WORDS = sizeof(FlowCtl) / 4;
  constexpr uint32_t ZERO_IDX = offsetof(FlowCtl, zero) / 4;
  const uint32_t W = a.W, H = a.H, f = blockIdx.x;
  const uint32_t RS = rows_ring_stride(W);
  const uint32_t RB = CTL_WORDS + ROWS_RB;   // sm index of ring slot 0, pixel 0
  const uint32_t RM = a.flow_ring - 1u;      // ring rows - 1 (4 or 8 rows)
  uint32_t* const ring = sm + RB;
  for (uint32_t i = threadIdx.x; i < CTL_WORDS; i += blockDim.x) sm[i] = 0u;
  __syncthreads();
  if (a.status[f] != 0) return;   // block-uniform
  const uint32_t nseg = (W + S - 1) / S, WPR = (nseg + 63) / 64, K = a.flow_k;
  const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (wid >= K * WPR) return;   // no barrier below this point
  // tests (NICE_OPT_TEST_FLOW_ABSENT): the block's last wave never starts, as
  // if it were not resident, so the others' waits time out into the fallback
  if (a.test_absent_strip && wid == K * WPR - 1) return;
  const uint32_t g = wid / WPR, w = wid - g * WPR, lastw = WPR - 1;
  const uint32_t seg = w * 64u + lane;
  const bool active = seg < nseg;
  const uint32_t x0 = seg * S;
  const int nvalid = active ? (int)min((uint32_t)S, W - x0) : 0;
  const uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint32_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 0xFF000000u : 0u;
  const uint32_t asel = alpha ? 0x0D060100u : 0x0C060100u;   // unspread3_perm
  const bool vec_rec = (W & 3u) == 0 && nvalid == S;
  const bool vec_out = (OC == 4 && (W & 3u) == 0 && nvalid == S) ||
                       (OC == 3 && (W & 15u) == 0 && nvalid == S);
  const uint32_t full = (1u << WPR) - 1u;
  const uint32_t depmask = w == 0 ? full : ((((7u << w) >> 1) & full) | (w == lastw ? 1u : 0u));
  const bool curlane = active && x0 + S + 2u >= W;   // words that can reference row y itself (W_CUR)
  const bool wave_cur = __any(curlane);
  uint2* const rtab = C.rtab[wid];
  const uint32_t lb = 17u * seg;
  uint32_t rn[S];
  auto load_recs = [&](uint32_t y) {
    const uint32_t* rrow = recs + (uint64_t)y * W + x0;
    if (vec_rec) {
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        const uint4 t = reinterpret_cast<const uint4*>(rrow)[q];
        rn[4 * q] = t.x; rn[4 * q + 1] = t.y; rn[4 * q + 2] = t.z; rn[4 * q + 3] = t.w;
      }
    } else if (nvalid > 0) {
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = p < nvalid ? rrow[p] : REC_RUN;
    } else {
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = REC_RUN;
    }
  };
  if (g < H) load_recs(g);
  bool ok = true;
#ifdef NICE_FLOW_STATS   // cycle split per wave position (NICE_DEC_STATS=1): stats[64 + 8 w + k]
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define FLOW_T(k) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); ts[k] += t_ - tlast; tlast = t_; }
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
#else
#define FLOW_T(k)
#endif
  for (uint32_t y = g; y < H && ok; y += K) {
    const uint32_t s = y & (FLOW_SLOTS - 1u);                              // stamps
    const uint32_t rs = y & RM, rsp = (y - 1u) & RM;   // ring rows
    // ---- pre-pass, part 1 (no pixel values): the row's class table, each
    // record's constant and kind bits, and the ring index of its reference
    if (lane < 16) {
      const uint32_t c = lane;
      const unsigned long long kinds = y == 0 ? ROWS_KIND_Y0 : ROWS_KIND;
      const uint32_t rows = (CLS_ROWS_PACK >> (2 * c)) & 3u, dxp3 = (uint32_t)(CLS_PX_PACK >> (3 * c)) & 7u;
      rtab[c] = make_uint2((((uint32_t)(kinds >> (4u * c)) & 15u) << 28) | dxp3,
                           RB + ((y - rows) & RM) * RS + 3u - dxp3);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    uint32_t wk[S], ad[S];
#pragma unroll
    for (int p = 0; p < S; ++p) {
      const uint32_t r = rec_canon(rn[p], a.rec_tag);
      const uint32_t cls = rec_cls(r);   // 0..13
      const uint2 e = rtab[cls];
      uint32_t idx = lb + e.y + (uint32_t)p;
      if (p < 3 || p > S - 4) idx += (uint32_t)((int)(p + 3u - (e.x & 7u)) >> 4);   // padding word crossed
      ad[p] = cls >= 4u ? idx : ZERO_IDX;
      // kind bits | the constant (already spread by the writers): one bit-field
      // insert (e.x holds only kind bits 28..31 and dxp3 in bits 0..2, which
      // the constant's mask covers)
      uint32_t kw;
      asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(kw) : "s"(REC_K), "v"(r), "v"(e.x));
      wk[p] = kw;
    }
    // references past the row end into row y itself (pixels 0..2): only the
    // wave holding the row's last columns (a wave-uniform branch: as a lane
    // branch the compiler if-converted it into every wave's pre-pass once the
    // record constant no longer needed spreading here, +2 % reconstruct)
    if (wave_cur) {
#pragma unroll
      for (int p = 0; p < S; ++p) {
        const uint32_t r = rec_canon(rn[p], a.rec_tag);
        const uint32_t cls = rec_cls(r);
        const uint32_t tx = x0 + p + 3u - ((uint32_t)(CLS_PX_PACK >> (3u * cls)) & 7u);
        const bool cur = curlane && cls >= 4u && ((CLS_ROWS_PACK >> (2u * cls)) & 3u) == 1u && tx >= W;
        wk[p] = cur ? (W_CUR | rec_c(r) | ((tx - W) << 8)) : wk[p];
        ad[p] = cur ? ZERO_IDX : ad[p];
      }
    }
    FLOW_T(0)
    // ---- wait for the rows above
    if (y > 0 && !flow_wait(C, C.fin[(y - 1u) & (FLOW_SLOTS - 1u)], depmask, y)) { ok = false; break; }
    // wave priorities (round 6): the row's pass once the rows above are in
    // before the waves still decoding records or storing the raster, and the
    // fix-up chain -- the row's serial path -- before both (512 x 4K
    // reconstruct 15.54 -> 14.48 ms, one 4K frame 8.43 -> 7.92;
    // profiles/r06ze_ab_flow_prio.log, r06zf_ab_flow_prio2.log)
    __builtin_amdgcn_s_setprio(1);
    FLOW_T(1)
    // ---- pre-pass, part 2: reference values, the row above, the entry
    uint32_t wv[S], prev[S];
#pragma unroll
    for (int p = 0; p < S; ++p) {
      const uint32_t o = sm[ad[p]];
      wv[p] = (wk[p] & ~SP_K) | ((o + wk[p]) & SP_K);
    }
    uint32_t* const pr = ring + rsp * RS;
#pragma unroll
    for (int p = 0; p < S; ++p) prev[p] = y > 0 ? pr[lb + p] : 0u;
    IvS r0{0u, SP_K}, r1{0u, SP_K}, r2{0u, SP_K};
    if (seg == 0) {
      if (y == 0) {
        r0 = r1 = r2 = ivs_exact(0u);
      } else {
        r0 = ivs_exact(pr[(W - 1) + ((W - 1) >> 4)]);
        r1 = ivs_exact(pr[(W - 2) + ((W - 2) >> 4)]);
        r2 = ivs_exact(pr[(W - 3) + ((W - 3) >> 4)]);
      }
    }
    FLOW_T(2)
    // ---- speculative pass
    IvS v[S];
    // (a wave without the row's last columns skips the W_CUR width term:
    // 512 x 4K reconstruct -1 %, profiles/r05zt_ab_flow_curspec.log)
    const SpecUnk su = wave_cur ? rows_spec_unk<S, true>(v, r0, r1, r2, wv, prev)
                                : rows_spec_unk<S, false>(v, r0, r1, r2, wv, prev);
    bool fin = !active || su.any == 0u;
    bool tex = !active || su.tail == 0u;
    const bool unk_hi = su.hi != 0u;
    if (w == 0 && lane == 0) {   // the row's first three pixels (lane 0: exact entry)
      C.head[s][0] = v[0].lo; C.head[s][1] = v[1].lo; C.head[s][2] = v[2].lo;
      flow_publish(&C.hst[s], y + 1u);
    }
    bool tpub = w == lastw;   // the last wave's tail feeds no wave
    auto pub_tail = [&]() {
      if (!tpub && __builtin_amdgcn_readlane((int)tex, 63)) {
        if (lane == 63) {
          C.tail[s][w][0] = v[S - 1].lo; C.tail[s][w][1] = v[S - 2].lo; C.tail[s][w][2] = v[S - 3].lo;
          flow_publish(&C.tst[s][w], y + 1u);
        }
        tpub = true;
      }
    };
    pub_tail();
    FLOW_T(3)
    // ---- fix-up rounds inside the wave
    __builtin_amdgcn_s_setprio(2);
    bool cur_done = !wave_cur;
    unsigned long long t0 = 0;
    for (uint32_t n = 0;; ++n) {
      if (__ballot(!fin) == 0ull) break;
      if (!cur_done && flow_peek(&C.hst[s]) >= y + 1u) {
        flow_acquire();
        const uint32_t h0 = C.head[s][0], h1 = C.head[s][1], h2 = C.head[s][2];
        if (curlane) {
#pragma unroll
          for (int p = 0; p < S; ++p) {
            const uint32_t k = (wv[p] >> 8) & 3u;
            const uint32_t hv = k == 0u ? h0 : k == 1u ? h1 : h2;
            wv[p] = (wv[p] & W_CUR) ? ((hv + (wv[p] & SP_K)) & SP_K) : wv[p];
          }
        }
        cur_done = true;
      }
      IvS l0{shfl_up1(v[S - 1].lo), 0u}, l1{shfl_up1(v[S - 2].lo), 0u}, l2{shfl_up1(v[S - 3].lo), 0u};
      bool lex = shfl_up1(tex ? 1u : 0u) != 0u;
      if (lane == 0) {
        lex = false;
        if (w > 0 && flow_peek(&C.tst[s][w - 1]) >= y + 1u) {
          flow_acquire();
          l0.lo = C.tail[s][w - 1][0]; l1.lo = C.tail[s][w - 1][1]; l2.lo = C.tail[s][w - 1][2];
          lex = true;
        }
      }
      const bool go = !fin && lex && (cur_done || !curlane);
      if (__ballot(go) != 0ull) {
        rows_chain_upto<S>(v, l0, l1, l2, wv, prev, go, unk_hi);
        if (go) {
          fin = true;
          tex = true;
        }
        pub_tail();
#ifdef NICE_FLOW_STATS
        ts[6] += 1;
#endif
      } else {
        // nothing to do until the left wave's tail or the row head arrive
        if ((n & 31u) == 0u) {
          if (flow_peek(&C.abort)) { ok = false; break; }
          const unsigned long long t = __builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = t;
          else if (t - t0 > FLOW_TIMEOUT) {
            atomicOr(&C.abort, 1u);
            atomicCAS(&C.err, 0, FLOW_REDO);
            ok = false;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    FLOW_T(4)
    if (!ok) break;
    if (C.err) { atomicOr(&C.abort, 1u); ok = false; break; }
    // ---- the ring row, its halos, the stamp
    if (active) {
      uint32_t* rr = ring + rs * RS + lb;
#pragma unroll
      for (int p = 0; p < S; ++p) rr[p] = v[p].lo;   // padding pixels land in the row's spare words
      if (seg == 0 && y > 0) {   // row y-1's right halo: this row's first three pixels
#pragma unroll
        for (int k = 0; k < 3; ++k) pr[(W + k) + ((W + k) >> 4)] = v[k].lo;
      }
    }
    if (wave_cur) {   // row y+1's left halo (words -4..-2): this row's columns W-3..W-1, copied
      // from the ring words just written by the wave holding each of them
      // (a 4-row ring puts it over row y-3's left halo, which row y's first
      // wave reads in its pre-pass: wait for that wave's first pixels)
      if (RM < 7u && !flow_wait(C, &C.hst[s], 1u, y + 1u)) { ok = false; break; }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      const uint32_t col = W - 3u + lane;
      if (lane < 3u && (col / S) / 64u == w)
        ring[((y + 1u) & RM) * RS + lane - 4] = ring[rs * RS + col + (col >> 4)];
    }
    if (lane == 0) flow_publish(&C.fin[s][w], y + 1u);
    __builtin_amdgcn_s_setprio(0);
    FLOW_T(5)
    // ---- off the critical path: the next row's records, the raster
    if (y + K < H) load_recs(y + K);
    if (active) {
      const uint64_t pix = (uint64_t)y * W + x0;
      if (vec_out && OC == 4) {
        uint4* o = reinterpret_cast<uint4*>(outp + pix * 4);
#pragma unroll
        for (int q = 0; q < S / 4; ++q)
          o[q] = make_uint4(unspread3_perm(v[4 * q].lo, asel), unspread3_perm(v[4 * q + 1].lo, asel),
                            unspread3_perm(v[4 * q + 2].lo, asel), unspread3_perm(v[4 * q + 3].lo, asel));
      } else if (vec_out) {
        uint32_t b[3 * S / 4];
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
          const uint32_t u0 = unspread3_perm(v[4 * q].lo, 0x0C060100u), u1 = unspread3_perm(v[4 * q + 1].lo, 0x0C060100u);
          const uint32_t u2 = unspread3_perm(v[4 * q + 2].lo, 0x0C060100u), u3 = unspread3_perm(v[4 * q + 3].lo, 0x0C060100u);
          b[3 * q] = __builtin_amdgcn_perm(u1, u0, 0x04020100u);       // R0 G0 B0 R1
          b[3 * q + 1] = __builtin_amdgcn_perm(u2, u1, 0x05040201u);   // G1 B1 R2 G2
          b[3 * q + 2] = __builtin_amdgcn_perm(u3, u2, 0x06050402u);   // B2 R3 G3 B3
        }
        uint4* o = reinterpret_cast<uint4*>(outp + pix * 3);
#pragma unroll
        for (int q = 0; q < 3 * S / 16; ++q) o[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
      } else if (OC == 4) {
        uint32_t* o32 = reinterpret_cast<uint32_t*>(outp + pix * 4);
#pragma unroll
        for (int p = 0; p < S; ++p)
          if (p < nvalid) o32[p] = unspread3(v[p].lo) | alpha;
      } else {
        uint8_t* o8 = outp + pix * 3;
#pragma unroll
        for (int p = 0; p < S; ++p) {
          if (p < nvalid) {
            const uint32_t u = unspread3(v[p].lo);
            o8[3 * p] = (uint8_t)u; o8[3 * p + 1] = (uint8_t)(u >> 8); o8[3 * p + 2] = (uint8_t)(u >> 16);
          }
        }
      }
    }
  }
  if (lane == 0) {
    const int e = __hip_atomic_load(&C.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (e == FLOW_REDO && a.hand_abort) atomicCAS(&a.hand_abort[f], 0u, SPLIT_REDO);
    else if (e) set_status(&a.status[f], e == FLOW_REDO ? NICE_E_HIP : e);
  }
#ifdef NICE_FLOW_STATS
  if (lane == 0 && a.stats) {
    // ts[7]: rows processed; k = 0 record decode, 1 wait, 2 ring reads, 3 spec, 4 fix-up, 5 ring row + stamp, 6 fix-up rounds with work
    ts[7] = (H > g ? (H - g + K - 1) / K : 0);
    for (int k = 0; k < 8; ++k) atomicAdd(&a.stats[64 + 8 * w + k], ts[k]);
  }
#endif
#undef FLOW_T
}

// ---------------------------------------------------------------------------
// D5c: strip-split reconstruction for wide frames: a frame's row segments are
// cut into k strips of <= 256 lanes, one workgroup each (one per CU), all rows
// in order.  In raster order the strip-rows ("units" (y, j)) form one chain:
// a unit's left neighbour is (y, j-1), or (y-1, k-1) for j = 0 (the wrap of
// code.rs:412-413), its right neighbour (y, j+1), or (y+1, 0).  Each block
// keeps a 4-row ring of its columns plus three halo columns on each side in
// LDS; ring row r's left halo is the last three pixels of r's left neighbour
// unit, its right halo the first three of r's right neighbour unit -- so every
// reference (rows 1..3 back, +-3 pixels, code.rs:141-145) is one ring read
// with no wrap logic, and lane 0's entry (the three pixels before the strip)
// is ring row y's left halo.  Units publish their first and last three pixels
// as soon as they are exact (after the speculative pass, usually without
// their entry) as 8-byte {row + 1, value} granules (agent-scope relaxed
// atomics: sc1 stores / loads); a block waits for nothing before its
// speculative pass except the halos of rows y-2 and y-3 (published long
// before); halo words of row y-1 not yet published and the entry are unknown
// intervals in the speculative pass, resolved in the fix-up rounds, which poll
// for them.  Every dependency points to a unit earlier in raster order, so
// with every block resident (the host launches at most one block per CU for
// half the CUs) the earliest unfinished unit always progresses.  Polls give up
// after SPLIT_TIMEOUT (a frame-wide abort flag stops the other strips early
// on an error).
// ---------------------------------------------------------------------------
constexpr uint32_t SPLIT_THREADS = 256;                      // lanes (16-pixel segments) per strip
// s_memrealtime ticks (100 MHz): 0.2 s.  A wait this long means a strip's
// neighbour is not resident (other kernels hold the CUs): the frame is handed
// to the fallback launch (SPLIT_REDO), not failed
constexpr unsigned long long SPLIT_TIMEOUT = 20000000ull;
constexpr int SPLIT_QUIET = -1000, SPLIT_TIMED_OUT = -1001;   // block-local err codes
constexpr uint32_t SPLIT_GRAN = 8;                           // granules per unit: first3 at 0..2, last3 at 4..6
__host__ __device__ constexpr uint32_t split_ring_stride(uint32_t sw) { return (sw + 6) + ((sw + 6) >> 4) + 17; }
__device__ __forceinline__ uint32_t sr_idx(uint32_t lc3) { return lc3 + (lc3 >> 4); }

__device__ __forceinline__ void hand_put(unsigned long long* p, uint32_t row, uint32_t v) {
  __hip_atomic_store(p, ((unsigned long long)(row + 1u) << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long hand_get(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct SplitGeo {
  uint32_t f, j, k, W, H, sw, RS;
  unsigned long long* hand;   // frame f's granules
  // granule i of unit (y, jj)
  __device__ __forceinline__ unsigned long long* g(uint32_t y, uint32_t jj, uint32_t i) const {
    return hand + ((uint64_t)y * k + jj) * SPLIT_GRAN + i;
  }
  // source granule of halo pixel i (0..2) of ring row r (>= -1: ring row -1's
  // right halo is row 0's first pixels when j = k-1 -- pixel W-3 of row 0
  // may reference pixel 0 through offset W-3), side 0 (left) / 1 (right);
  // false when the source lies outside the image (never referenced)
  __device__ __forceinline__ bool src(int r, uint32_t side, uint32_t i, unsigned long long*& p,
                                      uint32_t& srow) const {
    if (side == 0) {
      if (j > 0) {
        if (r < 0) return false;
        p = g((uint32_t)r, j - 1, 4 + i); srow = (uint32_t)r; return true;
      }
      if (r < 1) return false;
      p = g((uint32_t)r - 1, k - 1, 4 + i); srow = (uint32_t)r - 1; return true;
    }
    if (j + 1 < k) {
      if (r < 0) return false;
      p = g((uint32_t)r, j + 1, i); srow = (uint32_t)r; return true;
    }
    if (r < -1 || r + 1 >= (int)H) return false;
    p = g((uint32_t)(r + 1), 0, i); srow = (uint32_t)(r + 1); return true;
  }
};

// A wave-0 poll in two halves, so the granule loads' latency overlaps other
// work.  The halo items of row y: t = 0..5 ring rows y-3, y-3, y-2, y-2, y-1,
// y-1 (left, right), t = 6 row y's left halo (the entry); lanes 3t..3t+2 take
// item t.  issue() loads the granules of the items in `mask` whose hv word
// does not say present; commit() copies every item whose three tags match
// into the ring and sets its hv word.  hv[slot * 2 + side]: the ring row
// (>= -1) whose halo the slot holds, + 2 (0: none).
struct HaloPoll {
  unsigned long long v;
  int r;
  uint32_t side, i, srow;   // side 2: no item on this lane
  bool ex;
  __device__ __forceinline__ void issue(const SplitGeo& G, const uint32_t* hv, uint32_t lane, uint32_t y,
                                        uint32_t mask) {
    side = 2u;
    ex = false;
    v = 0;
    const uint32_t t = lane / 3u;
    i = lane - 3u * t;
    if (t >= 7u || !((mask >> t) & 1u)) return;
    const int rr = t < 6u ? (int)y - 3 + (int)(t >> 1) : (int)y;
    const uint32_t sd = t < 6u ? (t & 1u) : 0u;
    if (rr < -1 || hv[((uint32_t)rr & 3u) * 2u + sd] == (uint32_t)(rr + 2)) return;
    r = rr;
    side = sd;
    unsigned long long* p = nullptr;
    ex = G.src(rr, sd, i, p, srow);
    if (ex) v = hand_get(p);
  }
  __device__ __forceinline__ void commit(const SplitGeo& G, uint32_t* ring, uint32_t* hv, uint32_t lane) {
    const bool ok = side < 2u && (!ex || (uint32_t)(v >> 32) == srow + 1u);
    if (ok) ring[((uint32_t)r & 3u) * G.RS + sr_idx(side ? G.sw + 3u + i : i)] = (uint32_t)v;
    const unsigned long long m = __ballot(ok);
    if (ok && i == 0u && ((m >> lane) & 7ull) == 7ull) hv[((uint32_t)r & 3u) * 2u + side] = (uint32_t)(r + 2);
    side = 2u;
  }
};
// present bits (t = 0..6) of row y's halo items
__device__ __forceinline__ uint32_t halo_have(const uint32_t* hv, uint32_t y) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t t = 0; t < 7u; ++t) {
    const int rr = t < 6u ? (int)y - 3 + (int)(t >> 1) : (int)y;
    const uint32_t sd = t < 6u ? (t & 1u) : 0u;
    if (rr < -1 || hv[((uint32_t)rr & 3u) * 2u + sd] == (uint32_t)(rr + 2)) m |= 1u << t;
  }
  return m;
}

__global__ __launch_bounds__(SPLIT_THREADS) void dec_rows_split(DecArgs a) {
  constexpr int S = ROWS_SEG;
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  __shared__ uint32_t clsw[32];
  __shared__ uint32_t hv[8];     // ring slot halo state (row + 1 per slot and side)
  __shared__ uint32_t pend[2];
  __shared__ int err;
  const uint32_t k = a.strips;
  const uint32_t f = a.split_f0 + blockIdx.x / k, j = blockIdx.x % k;
  if (a.test_absent_strip && j == k - 1) return;   // block-uniform (tests only)
  const uint32_t W = a.W, H = a.H;
  const uint32_t nseg = (W + S - 1) / S;
  const uint32_t sps = (nseg + k - 1) / k;
  const uint32_t s0 = j * sps, s1 = min(nseg, s0 + sps);
  const uint32_t c0 = s0 * S, sw = min(W, s1 * S) - c0;
  const uint32_t lane = threadIdx.x;
  const uint32_t nl = s1 - s0;
  const bool active = lane < nl;
  const uint32_t xl0 = lane * S;
  const int nvalid = active ? (int)min((uint32_t)S, sw - xl0) : 0;
  const SplitGeo G{f, j, k, W, H, sw, split_ring_stride(sw), a.hand + (uint64_t)f * H * k * SPLIT_GRAN};
  const uint32_t RS = G.RS;
  uint32_t* tails = sm;                              // SPLIT_THREADS x {lo, len} x 3
  uint32_t* flags = tails + SPLIT_THREADS * 6;       // SPLIT_THREADS
  uint32_t* ring = flags + SPLIT_THREADS + 4;        // 4 x RS
  if (threadIdx.x < 32) {
    const uint32_t c = threadIdx.x & 15u;
    const unsigned long long kinds = threadIdx.x >= 16 ? ROWS_KIND_Y0 : ROWS_KIND;
    clsw[threadIdx.x] = ((CLS_ROWS_PACK >> (2 * c)) & 3u) | (uint32_t)((CLS_PX_PACK >> (3 * c)) & 7u) << 2 |
                        ((uint32_t)(kinds >> (4u * c)) & 15u) << 28;
  }
  if (threadIdx.x < 8) hv[threadIdx.x] = 0;
  if (lane == 0) err = 0;
  if (a.status[f] != 0) return;   // block-uniform
  uint32_t* abort_f = a.hand_abort + f;
  const uint32_t* recs = a.recs + (uint64_t)f * a.rec_stride + c0;
  uint8_t* outp = a.px_out + (uint64_t)f * a.px_stride;
  const uint32_t OC = a.out_channels;
  const uint32_t alpha = (a.flags & NICE_DEC_ALPHA_FILL_FF) ? 0xFF000000u : 0u;
  const uint32_t asel = alpha ? 0x0D060100u : 0x0C060100u;   // unspread3_perm
  const bool vec_rec = ((W | c0) & 3u) == 0 && nvalid == S;
  const bool vec_out = (OC == 4 && ((W | c0) & 3u) == 0 && nvalid == S) ||
                       (OC == 3 && ((W | c0) & 15u) == 0 && nvalid == S);
  uint32_t prev[S], rn[S];
#pragma unroll
  for (int p = 0; p < S; ++p) prev[p] = 0;
  auto load_recs = [&](uint32_t y) {
    const uint32_t* rrow = recs + (uint64_t)y * W + xl0;
    if (vec_rec) {
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        const uint4 t = reinterpret_cast<const uint4*>(rrow)[q];
        rn[4 * q] = t.x; rn[4 * q + 1] = t.y; rn[4 * q + 2] = t.z; rn[4 * q + 3] = t.w;
      }
    } else if (nvalid > 0) {
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = p < nvalid ? rrow[p] : REC_RUN;
    } else {
#pragma unroll
      for (int p = 0; p < S; ++p) rn[p] = REC_RUN;
    }
  };
  if (H > 0) load_recs(0);
  __syncthreads();
  unsigned long long t_row = 0;   // when this row's waits began
  // wave 0: gives up (error) on a timeout or another strip's abort
  auto give_up = [&]() -> bool {
    if (__hip_atomic_load(abort_f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      if (lane == 0) atomicCAS(&err, 0, SPLIT_QUIET);   // another strip failed or timed out: exit quietly
      return true;
    }
    if (__builtin_amdgcn_s_memrealtime() - t_row > SPLIT_TIMEOUT) {
      if (lane == 0) atomicCAS(&err, 0, SPLIT_TIMED_OUT);
      return true;
    }
    return false;
  };
  HaloPoll HP;
  bool pending_poll = false;   // wave 0: HP holds issued loads
  // timing counters (NICE_DEC_STATS=1) only in -DNICE_ROWS_STATS builds
#ifdef NICE_ROWS_STATS
  unsigned long long* const stats = a.stats;
#else
  constexpr unsigned long long* stats = nullptr;
#endif
  unsigned long long c_entry = 0, c_right = 0;
  unsigned long long c_wait = 0, c_spec = 0, c_fix = 0, c_emit = 0, n_rounds = 0, n_polls = 0, n_noentry = 0;
  uint32_t y = 0;
  for (; y < H; ++y) {
    const unsigned long long cc0 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- halos: rows y-2 and y-3 (wait), row y-1 and the entry (try)
    t_row = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {   // slot y & 3 held row y-4: free it for row y
      hv[(y & 3u) * 2u] = 0u;
      hv[(y & 3u) * 2u + 1u] = 0u;
    }
    if (lane < 64) {
      // the loads issued at the end of the previous row, then rows y-2 and
      // y-3 (items 0..3) until present
      if (pending_poll) HP.commit(G, ring, hv, lane);
      pending_poll = false;
      while (true) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        const uint32_t miss = ~halo_have(hv, y) & 15u;
        if (!miss) break;
        if (give_up()) break;
        HP.issue(G, hv, lane, y, miss);
        HP.commit(G, ring, hv, lane);
        if (stats) ++n_polls;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (err) break;
    const uint32_t ym1 = (y - 1u) & 3u;
    bool hl1 = hv[ym1 * 2u] == y + 1u;               // row y-1's halos present (row -1 at y = 0)
    bool hr1 = hv[ym1 * 2u + 1u] == y + 1u;
    bool eok = hv[(y & 3u) * 2u] == y + 2u;          // the entry (row y's left halo)
    const unsigned long long cc1 = stats ? __builtin_amdgcn_s_memtime() : 0;
    if (stats && !eok) ++n_noentry;
    // ---- pre-pass: records -> per-pixel words; a reference into a halo of
    // row y-1 not yet present is marked W_CUR (unknown) with its halo slot
    // (index in bits 8..9, side in bit 19) and resolved in the fix-up rounds
    const uint32_t* const cwt = clsw + (y == 0 ? 16 : 0);
    uint32_t w[S];
    bool npend = false;
#pragma unroll
    for (int p = 0; p < S; ++p) {
      const uint32_t r = rec_canon(rn[p], a.rec_tag);
      const uint32_t cls = rec_cls(r);
      const uint32_t cw = cwt[cls];
      const uint32_t rows = cw & 3u;
      const uint32_t lc3 = xl0 + (uint32_t)p + 6u - ((cw >> 2) & 7u);   // local column + 3 - pixels back
      const bool up = cls >= 4;
      const bool pl = up && rows == 1u && lc3 < 3u && !hl1;
      const bool pr = up && rows == 1u && lc3 >= sw + 3u && !hr1;
      const uint32_t lcc = min(lc3, sw + 5u);
      const uint32_t o = ring[__umul24((y - rows) & 3u, RS) + sr_idx(lcc)];
      const uint32_t c = rec_c(r);
      const bool cur = pl || pr;
      const uint32_t hslot = pl ? lc3 : (lc3 - sw - 3u);
      const uint32_t kb = (cw & 0xF0000000u) | (cur ? W_CUR : 0u);
      w[p] = kb | ((up && !cur) ? ((o + c) & SP_K) : c) | (cur ? ((hslot << 8) | (pr ? (1u << 19) : 0u)) : 0u);
      npend = npend || cur;
    }
    // ---- entry: exact when present (strip 0 of row 0: zeros), else unknown
    IvS r0{0u, SP_K}, r1{0u, SP_K}, r2{0u, SP_K};
    if (lane == 0) {
      if (y == 0 && j == 0) {
        r0 = r1 = r2 = ivs_exact(0u);
      } else if (eok) {
        const uint32_t* hr = ring + (y & 3u) * RS;
        r0 = ivs_exact(hr[sr_idx(2)]); r1 = ivs_exact(hr[sr_idx(1)]); r2 = ivs_exact(hr[sr_idx(0)]);
      }
    }
    if (y + 1 < H) load_recs(y + 1);
    // ---- speculative pass
    IvS v[S];
    int lu = rows_spec<S>(v, r0, r1, r2, w, prev);
    if (active) {
      uint32_t* t = tails + lane * 6;
      t[0] = v[S - 1].lo; t[1] = v[S - 1].len;
      t[2] = v[S - 2].lo; t[3] = v[S - 2].len;
      t[4] = v[S - 3].lo; t[5] = v[S - 3].len;
      flags[lane] = (lu < S - 3) ? 1u : 0u;
    }
    if (lane == 0) { pend[0] = 0; pend[1] = 0; }
    bool fin = !active || lu < 0;
    // the unit's first / last three pixels, published once exact
    uint32_t pub = 0;
    const bool pub_lane = active && (lane == 0 || xl0 + S + 3u > sw);
    auto publish = [&]() {
      if (!pub_lane) return;
#pragma unroll
      for (int p = 0; p < S; ++p) {
        const uint32_t x = xl0 + (uint32_t)p;
        const uint32_t il = x + 3u - sw;   // 0..2 for the last three pixels
        if (x < 3u && !((pub >> x) & 1u) && v[p].len == 0u) {
          hand_put(G.g(y, j, x), y, v[p].lo);
          pub |= 1u << x;
        }
        if (x < sw && il < 3u && !((pub >> (4u + il)) & 1u) && v[p].len == 0u) {
          hand_put(G.g(y, j, 4u + il), y, v[p].lo);
          pub |= 16u << il;
        }
      }
    };
    publish();
    rows_barrier<true>();
    const unsigned long long cc2 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- fix-up rounds (polling for the entry and row y-1's missing halos)
    for (uint32_t rd = 0;; ++rd) {
      if (stats) ++n_rounds;
      if (!fin) atomicOr(&pend[rd & 1u], 1u);
      if (lane < 64) {
        // commit the loads issued last round, issue the still missing items
        // (row y-1's halos, the entry); their latency overlaps this round
        if (pending_poll) HP.commit(G, ring, hv, lane);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        const uint32_t miss = ~halo_have(hv, y) & 0x70u;
        pending_poll = miss != 0u;
        if (pending_poll) {
          HP.issue(G, hv, lane, y, miss);
          if (stats) ++n_polls;
          if (rd > 1u) __builtin_amdgcn_s_sleep(1);
        }
      }
      if (lane < 64 && (rd & 63u) == 63u) (void)give_up();   // bounds every wait (and any logic error)
      rows_barrier<true>();
      if (pend[rd & 1u] == 0 || err) break;
      if (lane == 0) pend[(rd + 1) & 1u] = 0;
      const bool nhl = hl1 || hv[ym1 * 2u] == y + 1u, nhr = hr1 || hv[ym1 * 2u + 1u] == y + 1u;
      bool resolved = false;
      if (npend && ((nhl && !hl1) || (nhr && !hr1))) {
        resolved = true;
        // halo words now present: resolve them (their chains are unknown from
        // there on and get recomputed below)
        const uint32_t* hrow = ring + ym1 * RS;
        bool still = false;
#pragma unroll
        for (int p = 0; p < S; ++p) {
          if (w[p] & W_CUR) {
            const uint32_t sd = (w[p] >> 19) & 1u, hs = (w[p] >> 8) & 3u;
            if (sd ? nhr : nhl)
              w[p] = (hrow[sr_idx(sd ? sw + 3u + hs : hs)] + (w[p] & SP_K)) & SP_K;
            else
              still = true;
          }
        }
        npend = still;
        if (!fin) { /* recompute below */ }
      }
      hl1 = nhl;
      hr1 = nhr;
      const bool neok = eok || hv[(y & 3u) * 2u] == y + 2u;
      if (stats && neok && !eok) c_entry += __builtin_amdgcn_s_memtime() - cc2;
      if (stats && nhr && !hr1) c_right += __builtin_amdgcn_s_memtime() - cc2;
      eok = neok;
      bool exact_in = false;
      bool go = !fin;
      if (!fin) {
        if (lane > 0) {
          const uint32_t* t = tails + (lane - 1) * 6;
          r0 = IvS{t[0], t[1]}; r1 = IvS{t[2], t[3]}; r2 = IvS{t[4], t[5]};
          exact_in = flags[lane - 1] != 0;
        } else if (eok) {
          const uint32_t* hr = ring + (y & 3u) * RS;
          r0 = ivs_exact(hr[sr_idx(2)]); r1 = ivs_exact(hr[sr_idx(1)]); r2 = ivs_exact(hr[sr_idx(0)]);
          exact_in = true;
        }
        exact_in = exact_in && !npend;
        // as in dec_rows: only exact left tails (or entries) are used
        go = exact_in;
      }
      (void)resolved;
      rows_barrier<true>();
      lu = rows_chain_exact<S>(v, r0, r1, r2, w, prev, lu, go);
      if (go) {
        if (lu >= 0) atomicCAS(&err, 0, NICE_E_FORMAT);
        uint32_t* t = tails + lane * 6;
        t[0] = v[S - 1].lo; t[1] = v[S - 1].len;
        t[2] = v[S - 2].lo; t[3] = v[S - 2].len;
        t[4] = v[S - 3].lo; t[5] = v[S - 3].len;
        flags[lane] = 1u;
        fin = true;
      }
      publish();
    }
    if (err) break;
    // prefetch the next row's halo items (committed at its start)
    if (lane < 64 && y + 1 < H) {
      if (pending_poll) HP.commit(G, ring, hv, lane);
      HP.issue(G, hv, lane, y + 1, 0x7Fu);
      pending_poll = true;
    }
    const unsigned long long cc3 = stats ? __builtin_amdgcn_s_memtime() : 0;
    // ---- emit: ring row y (local columns) and the raster
    if (active) {
      uint32_t* rr = ring + (y & 3u) * RS;
      const uint64_t pix = (uint64_t)y * W + c0 + xl0;
#pragma unroll
      for (int p = 0; p < S; ++p) rr[sr_idx(xl0 + (uint32_t)p + 3u)] = v[p].lo;   // padding: spare words
      if (vec_out && OC == 4) {
        uint4* o = reinterpret_cast<uint4*>(outp + pix * 4);
#pragma unroll
        for (int q = 0; q < S / 4; ++q)
          o[q] = make_uint4(unspread3_perm(v[4 * q].lo, asel), unspread3_perm(v[4 * q + 1].lo, asel),
                            unspread3_perm(v[4 * q + 2].lo, asel), unspread3_perm(v[4 * q + 3].lo, asel));
      } else if (vec_out) {
        uint32_t b[3 * S / 4];
#pragma unroll
        for (int q = 0; q < S / 4; ++q) {
          const uint32_t u0 = unspread3_perm(v[4 * q].lo, 0x0C060100u), u1 = unspread3_perm(v[4 * q + 1].lo, 0x0C060100u);
          const uint32_t u2 = unspread3_perm(v[4 * q + 2].lo, 0x0C060100u), u3 = unspread3_perm(v[4 * q + 3].lo, 0x0C060100u);
          b[3 * q] = __builtin_amdgcn_perm(u1, u0, 0x04020100u);       // R0 G0 B0 R1
          b[3 * q + 1] = __builtin_amdgcn_perm(u2, u1, 0x05040201u);   // G1 B1 R2 G2
          b[3 * q + 2] = __builtin_amdgcn_perm(u3, u2, 0x06050402u);   // B2 R3 G3 B3
        }
        uint4* o = reinterpret_cast<uint4*>(outp + pix * 3);
#pragma unroll
        for (int q = 0; q < 3 * S / 16; ++q) o[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
      } else if (OC == 4) {
        uint32_t* o32 = reinterpret_cast<uint32_t*>(outp + pix * 4);
#pragma unroll
        for (int p = 0; p < S; ++p)
          if (p < nvalid) o32[p] = unspread3(v[p].lo) | alpha;
      } else {
        uint8_t* o8 = outp + pix * 3;
#pragma unroll
        for (int p = 0; p < S; ++p) {
          if (p < nvalid) {
            const uint32_t u = unspread3(v[p].lo);
            o8[3 * p] = (uint8_t)u; o8[3 * p + 1] = (uint8_t)(u >> 8); o8[3 * p + 2] = (uint8_t)(u >> 16);
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < S; ++p) prev[p] = v[p].lo;
    rows_barrier<true>();
    if (stats) {
      const unsigned long long cc4 = __builtin_amdgcn_s_memtime();
      c_wait += cc1 - cc0; c_spec += cc2 - cc1; c_fix += cc3 - cc2; c_emit += cc4 - cc3;
    }
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], (unsigned long long)y); atomicAdd(&stats[4], n_rounds);
    atomicAdd(&stats[5], c_wait); atomicAdd(&stats[6], c_spec); atomicAdd(&stats[7], c_fix);
    atomicAdd(&stats[8], c_emit); atomicAdd(&stats[1], n_noentry); atomicAdd(&stats[2], n_polls);
    atomicAdd(&stats[3], c_entry); atomicAdd(&stats[9], c_right);
  }
  if (lane == 0 && err) {
    if (err == SPLIT_TIMED_OUT) {
      // not co-resident: the fallback launch reconstructs the frame (a real
      // error of another strip sets the status, which the fallback respects)
      atomicCAS(abort_f, 0u, SPLIT_REDO);
    } else if (err != SPLIT_QUIET) {
      __hip_atomic_store(abort_f, SPLIT_ABORT_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      set_status(&a.status[f], err);
    }
  }
}

__global__ __launch_bounds__(64) void dec_reconstruct(DecArgs a) {
  if (a.rows_in_lds) dec_reconstruct_body<true>(a);
  else dec_reconstruct_body<false>(a);
}

}  // namespace nice
