// nice_capi.hip -- host runtime behind include/nice.h: contexts, scratch arenas,
// kernel launch sequences and the host-buffer convenience entry points.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <algorithm>
#include <vector>

#include "../../include/nice.h"
#include "../../include/nice_test.h"
#include "nice_format.h"
#include "nice_bits.hpp"
#include "nice_kernels.h"
#include "nice_rec.hpp"
#include "nice_internal.h"

using namespace nice;

#define NICE_HIP(x)                          \
  do {                                       \
    if ((x) != hipSuccess) return NICE_E_HIP; \
  } while (0)

namespace {

// Device scratch arena, grown on demand (reserve() to pre-size).
struct Arena {
  void* ptr = nullptr;
  size_t cap = 0;
  uint64_t gen = 0;   // bumped by every (re)allocation: contents are unknown after it
  int grow(size_t bytes) {
    if (bytes <= cap) return NICE_OK;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    ++gen;
    if (hipMalloc(&ptr, bytes) != hipSuccess) return NICE_E_HIP;
    cap = bytes;
    return NICE_OK;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
  }
};

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Test / A/B options (include/nice_test.h; nice_test_set_option): stored as
// value + 1, 0 = unset.  Nothing in the library reads the environment.
std::atomic<int64_t> g_opt[NICE_OPT_COUNT];
inline bool opt_set(int id) { return g_opt[id].load(std::memory_order_relaxed) != 0; }
inline int64_t opt_val(int id) { return g_opt[id].load(std::memory_order_relaxed) - 1; }
inline bool opt_on(int id) { return opt_set(id) && opt_val(id) != 0; }

// Encoder scratch layout. The zero-per-launch block comes first (memset once).
struct EncLayout {
  size_t zero_bytes, total;
  size_t o_hist, o_flags, o_ctr, o_status, o_overn, o_overl;
  size_t o_first, o_last, o_next, o_tbl, o_tblcode, o_len8, o_smax, o_seedbit, o_seedsuf,
      o_hdrbytes, o_hdrcache, o_hdrbitoff, o_recs, o_tbits, o_toff, o_dend, o_packtab, o_gacc, o_bhist, o_cmask;
};

EncLayout enc_layout(uint32_t n_frames, uint32_t T, uint64_t npx) {
  EncLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes, 256); return r; };
  L.o_hist = take((size_t)n_frames * N_BINS * 4);
  L.o_flags = take((size_t)n_frames * 4 + 4);   // + one word: any frame FLAG_LONG
  L.o_ctr = take((size_t)n_frames * 4);
  L.o_status = take((size_t)n_frames * T * 8);
  L.o_overn = take(4);
  L.zero_bytes = align_up(o, 16);
  L.o_overl = take((size_t)n_frames * ((T + PACK_SUB - 1) / PACK_SUB) * 8);
  L.o_first = take((size_t)n_frames * T * 4);
  L.o_last = take((size_t)n_frames * T * 4);
  L.o_next = take((size_t)n_frames * T * 4);
  L.o_tbl = take((size_t)n_frames * N_BINS * 4);
  L.o_tblcode = take((size_t)n_frames * N_BINS * 4);
  L.o_len8 = take((size_t)n_frames * N_BINS);
  L.o_smax = take((size_t)n_frames * N_STREAMS);
  L.o_seedbit = take((size_t)n_frames * 8);
  L.o_seedsuf = take((size_t)n_frames * 4);
  L.o_hdrbytes = take((size_t)n_frames * 8);
  L.o_hdrcache = take((size_t)n_frames * 4);
  L.o_hdrbitoff = take((size_t)n_frames);
  L.o_recs = take((size_t)n_frames * ((npx + 3) & ~3ull) * 4);
  L.o_tbits = take((size_t)n_frames * T * 4);
  L.o_toff = take((size_t)n_frames * T * 8);
  L.o_dend = take((size_t)n_frames * 8);
  L.o_packtab = take((size_t)n_frames * sizeof(PackTab));
  L.o_gacc = take((size_t)n_frames * ((T + ENC_GROUP_TILES - 1) / ENC_GROUP_TILES + 1) * 8);
  L.o_bhist = take((size_t)N_BINS * 4);   // band API: the band's own histogram
  L.o_cmask = take((size_t)n_frames * T * (ENC_TILE / 32) * 4);   // 1 bit per pixel
  L.total = o;
  return L;
}

int check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return NICE_E_NODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return NICE_E_NODEV;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NICE_E_NODEV;
  return NICE_OK;
}

}  // namespace

static const char* kPhaseNames[NICE_PHASES] = {
    "enc_classify", "enc_tailruns", "enc_tables", "enc_header", "enc_tilebits", "enc_tilescan",
    "enc_pack", "enc_tail", "enc_pack_long", "dec_tables", "dec_sync", "dec_scan", "dec_emit",
    "dec_reconstruct", "dec_place", "dec_resync"};

// Optional per-phase HIP-event timing (bench / profiling).
struct PhaseTimer {
  bool on = false;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  struct Mark { int phase; hipEvent_t a, b; };
  std::vector<Mark> marks;
  hipEvent_t take() {
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[used++];
  }
  void begin(int phase, hipStream_t st) {
    if (!on) return;
    Mark m{phase, take(), take()};
    if (!m.a || !m.b) return;
    (void)hipEventRecord(m.a, st);
    marks.push_back(m);
  }
  void end(hipStream_t st) {
    if (!on || marks.empty()) return;
    (void)hipEventRecord(marks.back().b, st);
  }
  void release() {
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
    marks.clear();
    used = 0;
  }
};

struct BandState {
  bool classified = false, tabled = false;
  nice::EncArgs a{};
  uint64_t band_bits = 0, seed_bit = 0;
  // the band's own symbol counts (nice_band_runs), for its bit count
  uint32_t* bhist = nullptr;
  // nice_band_tables_dev's {band bits, data start}, copied into the context
  // (band_hdr): the pack compares the caller's band_bits with it
  const unsigned long long* d_info = nullptr;
};

struct nice_ctx {
  int device = 0;
  std::mutex mu;
  Arena enc, dec, host_px, host_out, dev_len, band, band_hdr;
  PhaseTimer timer;
  BandState bs;
  // decoder record tags (DecArgs::rec_tag): the region the last call used and its tag
  uint32_t* rec_region = nullptr;
  uint64_t rec_words = 0, rec_gen = 0;
  uint32_t rec_epoch = 0;
  int cus = 0;   // compute units of the device (enc_pack's persistent grid)
  // the last split decode's per-frame abort flags (test hook nice_test_split_redos)
  const uint32_t* split_abort = nullptr;
  uint32_t split_frames = 0;
  int last_classify = -1;   // ClsKind of the last encode / band classify (test hook nice_test_last_classify)
  // test hooks (nice_test_set_hooks; 0 = off): the last strip of every split
  // decode returns at entry; enc_pack's LDS group buffer in bits per pixel
  uint32_t test_split_absent = 0, test_pack_cap_bpp = 0;
};

extern "C" {

const char* nice_version(void) { return "nice-mi355x 0.1 (gfx950)"; }

int nice_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

size_t nice_encode_bound(uint32_t w, uint32_t h) {
  // Huffman cost <= fixed-length cost per stream: <= 28 bits per coded pixel,
  // <= 2 bits per run pixel for digits (code.rs:391-406). Table header <= 858
  // 8-bit fields + 10 5-bit fields. 32 bits/px keeps it simple and word aligned.
  return (size_t)FILE_HEADER_BYTES + 880 + (size_t)w * h * 4 + 32;
}

int nice_peek_header(const uint8_t* s, size_t len, uint32_t* w, uint32_t* h, uint8_t* ch) {
  if (!s || len < 13) return NICE_E_FORMAT;
  if (w) *w = ((uint32_t)s[4] << 24) | ((uint32_t)s[5] << 16) | ((uint32_t)s[6] << 8) | s[7];
  if (h) *h = ((uint32_t)s[8] << 24) | ((uint32_t)s[9] << 16) | ((uint32_t)s[10] << 8) | s[11];
  if (ch) *ch = s[12];
  return NICE_OK;
}

int nice_ctx_create(int device, nice_ctx** out) {
  if (!out) return NICE_E_ARG;
  int rc = check_device(device);
  if (rc) return rc;
  nice_ctx* c = new nice_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  c->cus = hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
  *out = c;
  return NICE_OK;
}

void nice_ctx_destroy(nice_ctx* ctx) {
  if (!ctx) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(ctx->device);
  ctx->enc.release();
  ctx->dec.release();
  ctx->host_px.release();
  ctx->host_out.release();
  ctx->dev_len.release();
  ctx->band.release();
  ctx->band_hdr.release();
  ctx->timer.release();
  (void)hipSetDevice(prev);
  delete ctx;
}

static uint32_t tiles_for(uint32_t w, uint32_t h) {
  const uint64_t N = (uint64_t)w * h;
  return (uint32_t)((N + ENC_TILE - 1) / ENC_TILE);
}

int nice_ctx_reserve(nice_ctx* ctx, uint32_t n_frames, uint32_t w, uint32_t h) {
  if (!ctx) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  EncLayout L = enc_layout(n_frames, tiles_for(w, h), (uint64_t)w * h);
  return ctx->enc.grow(L.total);
}

}  // extern "C"

namespace {
EncArgs enc_args(const EncLayout& L, uint8_t* base, uint32_t n_frames, uint32_t w, uint32_t h,
                 uint8_t channels, uint8_t channels_out, uint32_t T, uint64_t N) {
  EncArgs a{};
  a.n_frames = n_frames;
  a.W = w;
  a.H = h;
  a.C = channels;
  a.channels_out = channels_out;
  a.tiles_per_frame = T;
  a.hist = (uint32_t*)(base + L.o_hist);
  a.frame_flags = (uint32_t*)(base + L.o_flags);
  a.tile_first = (uint32_t*)(base + L.o_first);
  a.tile_last = (uint32_t*)(base + L.o_last);
  a.tile_next = (uint32_t*)(base + L.o_next);
  a.cmask = (uint32_t*)(base + L.o_cmask);
  a.tbl = (uint32_t*)(base + L.o_tbl);
  a.tbl_code = (uint32_t*)(base + L.o_tblcode);
  a.tbl_len8 = base + L.o_len8;
  a.stream_max = base + L.o_smax;
  a.seed_bit = (unsigned long long*)(base + L.o_seedbit);
  a.seed_suf = (uint32_t*)(base + L.o_seedsuf);
  a.hdr_bytes = (unsigned long long*)(base + L.o_hdrbytes);
  a.hdr_cache = (uint32_t*)(base + L.o_hdrcache);
  a.hdr_bitoff = base + L.o_hdrbitoff;
  a.recs = (uint32_t*)(base + L.o_recs);
  a.rec_stride = (N + 3) & ~3ull;
  a.tile_bits = (uint32_t*)(base + L.o_tbits);
  a.packtab = base + L.o_packtab;
  a.pack_ctr = (uint32_t*)(base + L.o_ctr);
  {   // frames packed at once: <= 64, dividing the frames about evenly
    const uint32_t per = (n_frames + 63) / 64;
    a.pack_slots = (n_frames + per - 1) / per;
  }
  a.status = (unsigned long long*)(base + L.o_status);
  a.pack_mode = 0;
  a.long_only = 1;
  a.tile_off = (unsigned long long*)(base + L.o_toff);
  a.data_end = (unsigned long long*)(base + L.o_dend);
  a.tile_lo = 0;
  a.tile_hi = T;
  a.groups = T ? (T + ENC_GROUP_TILES - 1) / ENC_GROUP_TILES : 1;
  a.gacc = (unsigned long long*)(base + L.o_gacc);
  a.px_lo = 0;
  a.px_hi = (int64_t)N;
  a.band = 0;
  a.over_count = (uint32_t*)(base + L.o_overn);
  a.over_list = (uint2*)(base + L.o_overl);
  a.pack_cap_bits = (uint32_t)PACK_SUB * ENC_TILE * NICE_PACK_CAP_BPP;
  return a;
}
}  // namespace

// enc_classify_strip: rows per block (about three blocks per CU over all
// frames and strips, >= 16 rows so the 3-row prefill stays small) and the grid
static uint32_t strip_rows(const nice_ctx* ctx, uint32_t n_frames, uint32_t w, uint32_t rows_total, uint32_t* blocks) {
  const uint64_t strips = (w + STRIP_W_HOST - 1) / STRIP_W_HOST;
  const uint64_t want = 3ull * (uint64_t)ctx->cus;
  uint64_t r = (rows_total * strips * n_frames + want - 1) / want;
  if (r < 16) r = 16;
  if (r > rows_total) r = rows_total ? rows_total : 1;
  *blocks = (uint32_t)(n_frames * strips * ((rows_total + r - 1) / r));
  return (uint32_t)r;
}

// The classify kernel for a frame shape (every kernel writes the same
// records, histogram and tile edges): the LDS ring (each pixel loaded once)
// wherever the rows fit it, the strip kernel for wider RGBA rows of whole
// tiles, per-tile row windows for every other wide shape, and the round-1
// window kernel for pixel memory that is not 4-byte aligned.  `aligned`: the
// pixel base (frames: and stride) is 4-byte aligned, as the ring, strip and
// tile-window loads need.
// `frames_al16` (frames, not a band; pixel base and frame stride 16-byte
// aligned): the per-lane sliding-window kernel for RGBA rows that fit the ring.
enum ClsKind { CLS_K_WINDOW, CLS_K_TINY, CLS_K_RING, CLS_K_RING2, CLS_K_STRIP, CLS_K_PAIR, CLS_K_TWIN, CLS_K_SLIDE };
static ClsKind pick_classify(uint32_t w, uint8_t channels, bool aligned, bool frames_al16 = false) {
  if (w < 3) return CLS_K_TINY;
  if (!aligned || opt_on(NICE_OPT_ENC_NO_RING)) return CLS_K_WINDOW;
  const bool no_pair = opt_on(NICE_OPT_ENC_NO_PAIR);   // A/B: one tile per iteration
  if (channels == 4 && w <= CLS_PAIR_MAX_W && frames_al16 && !no_pair && !opt_on(NICE_OPT_ENC_NO_SLIDE))
    return CLS_K_SLIDE;
  if (channels == 4 && w <= CLS_PAIR_MAX_W && !no_pair) return CLS_K_PAIR;
  if (w <= CLS_RING_MAX_W) return CLS_K_RING;
  if (channels == 4 && w % ENC_TILE == 0) return CLS_K_STRIP;
  if (w <= CLS_RING2_MAX_W) return CLS_K_RING2;
  return CLS_K_TWIN;   // per-tile row windows: any wider shape
}
// Launches it over `work` tiles (frames x band tiles); rows_total: the rows the
// strip kernel walks per frame.
static void launch_classify(nice_ctx* ctx, ClsKind k, EncArgs& a, uint64_t work, uint32_t rows_total,
                            hipStream_t st) {
  const bool ringk = k == CLS_K_RING || k == CLS_K_RING2 || k == CLS_K_PAIR || k == CLS_K_SLIDE;
  // contiguous tile chunks per block: keeps rows-above reuse in L2 and flushes
  // each block's LDS histogram once per frame; ring kernels: >= 16 tiles per
  // block (the 3-row prefill amortised), 2 blocks per CU (ring2: 1)
  uint64_t blocks = (k == CLS_K_RING || k == CLS_K_PAIR || k == CLS_K_SLIDE) ? 2ull * ctx->cus : k == CLS_K_RING2 ? (uint64_t)ctx->cus : 2048;
  uint64_t per = (work + blocks - 1) / blocks;
  if (per < (ringk ? 16u : 1u)) per = ringk ? 16 : 1;
  if (ringk && per > 16384) per = 16384;   // its 16-bit per-thread prefix counters
  blocks = (work + per - 1) / per;
  a.tiles_per_block = (uint32_t)per;
  const bool rgb = a.C == 3;
  switch (k) {
    case CLS_K_STRIP: {
      uint32_t sblocks;
      a.tiles_per_block = strip_rows(ctx, a.n_frames, a.W, rows_total, &sblocks);
      hipLaunchKernelGGL(a.cmask ? enc_classify_strip_m : enc_classify_strip, dim3(sblocks), dim3(CLS_THREADS_HOST), 0, st, a);
      break;
    }
    case CLS_K_RING:   // (frames: the _m forms, as for the pair kernel below)
      if (rgb) hipLaunchKernelGGL(a.cmask ? enc_classify_ring3_m : enc_classify_ring3, dim3((uint32_t)blocks),
                                  dim3(CLS_THREADS_HOST), 0, st, a);
      else hipLaunchKernelGGL(a.cmask ? enc_classify_ring_m : enc_classify_ring, dim3((uint32_t)blocks),
                              dim3(CLS_THREADS_HOST), 0, st, a);
      break;
    case CLS_K_PAIR:
      // frames: coded flags out, run digits by enc_rundigits (below); bands:
      // run digits in the kernel
      if (a.cmask) hipLaunchKernelGGL(enc_classify_pair_m, dim3((uint32_t)blocks), dim3(CLS_THREADS_HOST), 0, st, a);
      else hipLaunchKernelGGL(enc_classify_pair, dim3((uint32_t)blocks), dim3(CLS_THREADS_HOST), 0, st, a);
      break;
    case CLS_K_SLIDE: {   // frames only (coded flags out in ballot order)
      const dim3 g((uint32_t)blocks), b(CLS_THREADS_HOST);
      switch (a.W & 3u) {
        case 0: hipLaunchKernelGGL(enc_classify_slide0, g, b, 0, st, a); break;
        case 1: hipLaunchKernelGGL(enc_classify_slide1, g, b, 0, st, a); break;
        case 2: hipLaunchKernelGGL(enc_classify_slide2, g, b, 0, st, a); break;
        default: hipLaunchKernelGGL(enc_classify_slide3, g, b, 0, st, a); break;
      }
      break;
    }
    case CLS_K_RING2:
      if (rgb) hipLaunchKernelGGL(a.cmask ? enc_classify_ring2_3_m : enc_classify_ring2_3, dim3((uint32_t)blocks),
                                  dim3(CLS_THREADS_HOST), 0, st, a);
      else hipLaunchKernelGGL(a.cmask ? enc_classify_ring2_m : enc_classify_ring2, dim3((uint32_t)blocks),
                              dim3(CLS_THREADS_HOST), 0, st, a);
      break;
    case CLS_K_TINY:
      hipLaunchKernelGGL(enc_classify_tiny, dim3((uint32_t)blocks), dim3(256), 0, st, a);
      break;
    case CLS_K_TWIN: {
      const uint64_t tb = 2ull * ctx->cus, tper = (work + tb - 1) / tb;
      a.tiles_per_block = (uint32_t)tper;
      const dim3 g((uint32_t)((work + tper - 1) / tper));
      if (rgb) hipLaunchKernelGGL(a.cmask ? enc_classify_twin3_m : enc_classify_twin3, g, dim3(CLS_THREADS_HOST), 0, st, a);
      else hipLaunchKernelGGL(a.cmask ? enc_classify_twin_m : enc_classify_twin, g, dim3(CLS_THREADS_HOST), 0, st, a);
      break;
    }
    default:
      hipLaunchKernelGGL(enc_classify, dim3((uint32_t)blocks), dim3(256), 0, st, a);
  }
}

extern "C" {

int nice_encode_batch_dev(nice_ctx* ctx, void* stream, const uint8_t* d_px, uint64_t frame_stride,
                          uint32_t n_frames, uint32_t w, uint32_t h, uint8_t channels,
                          uint8_t channels_out, uint8_t* d_out, uint64_t out_stride,
                          uint64_t* d_out_len) {
  if (!ctx || !d_out || !d_out_len) return NICE_E_ARG;
  if (channels != 3 && channels != 4) return NICE_E_ARG;
  const uint64_t N = (uint64_t)w * h;
  if (N > (1ull << 30)) return NICE_E_ARG;
  if (n_frames == 0) return NICE_OK;
  if (N > 0 && !d_px) return NICE_E_ARG;
  if (out_stride < nice_encode_bound(w, h) || (out_stride & 3) || ((uintptr_t)d_out & 3))
    return NICE_E_ARG;
  if (channels == 4 && N > 0 && (((uintptr_t)d_px & 3) || (frame_stride & 3))) return NICE_E_ARG;
  if (N > 0 && frame_stride < N * channels) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const uint32_t T = tiles_for(w, h);
  // one frame: its stride is never applied (an odd W*H*3 RGB stride is fine)
  const bool aligned = ((uintptr_t)d_px & 3) == 0 && (n_frames == 1 || (frame_stride & 3) == 0);
  const bool al16 = ((uintptr_t)d_px & 15) == 0 && (n_frames == 1 || (frame_stride & 15) == 0);
  const ClsKind ck = pick_classify(w, channels, aligned, al16);
  if ((uint64_t)n_frames * T >= (1ull << 32)) return NICE_E_ARG;   // enc_pack's 32-bit work counter
  EncLayout L = enc_layout(n_frames, T, N);
  int rc = ctx->enc.grow(L.total);
  if (rc) return rc;
  uint8_t* base = (uint8_t*)ctx->enc.ptr;
  EncArgs a = enc_args(L, base, n_frames, w, h, channels, channels_out, T, N);
  if (ctx->test_pack_cap_bpp) a.pack_cap_bits = (uint32_t)PACK_SUB * ENC_TILE * ctx->test_pack_cap_bpp;
  a.px = d_px;
  a.frame_stride = frame_stride;
  a.out = d_out;
  a.out_stride = out_stride;
  a.out_len = (unsigned long long*)d_out_len;
  NICE_HIP(hipMemsetAsync(base, 0, L.zero_bytes, st));
  const uint64_t total_tiles = (uint64_t)n_frames * T;
  if (T > 0) {
    PhaseTimer& tm = ctx->timer;
    tm.begin(NICE_PH_ENC_CLASSIFY, st);
    launch_classify(ctx, ck, a, total_tiles, h, st);
    if (ck != CLS_K_WINDOW && ck != CLS_K_TINY)   // in-tile run digits, from the coded flags
      hipLaunchKernelGGL(enc_rundigits,
                         dim3(std::min<uint32_t>((T + 7) / 8, std::max<uint32_t>(64u, 2048u / n_frames)), n_frames),
                         dim3(256), 0, st, a, ck == CLS_K_SLIDE ? 1 : 0);   // (>= 2048 blocks in all for few, large frames)
    ctx->last_classify = (int)ck;
    a.cmask_std = (ck != CLS_K_WINDOW && ck != CLS_K_TINY) ? 1u : 0u;   // (enc_pack reads the flags)
    tm.end(st);
    tm.begin(NICE_PH_ENC_TAILRUNS, st);
    if (a.groups > 1) hipLaunchKernelGGL(enc_group_reduce, dim3(a.groups, n_frames), dim3(256), 0, st, a, 0);
    hipLaunchKernelGGL(enc_tailruns, dim3(a.groups, n_frames), dim3(1024), 0, st, a);
    tm.end(st);
  }
  ctx->timer.begin(NICE_PH_ENC_TABLES, st);
  hipLaunchKernelGGL(enc_tables, dim3(n_frames * N_STREAMS), dim3(64), 0, st, a);
  ctx->timer.end(st);
  ctx->timer.begin(NICE_PH_ENC_HEADER, st);
  hipLaunchKernelGGL(enc_header, dim3(n_frames), dim3(64), 0, st, a);
  ctx->timer.end(st);
  if (T > 0) {
    ctx->timer.begin(NICE_PH_ENC_TILEBITS, st);
    hipLaunchKernelGGL(enc_packtab, dim3(n_frames), dim3(256), 0, st, a);
    ctx->timer.end(st);
    // frames with codes over 25 bits or composed entries over 32 (FLAG_LONG;
    // the launches return at once for the others): tile bits, their scan,
    // codes that fit the cache, then the wrapped writes
    const uint32_t tblocks = (uint32_t)(total_tiles < 2048 ? total_tiles : 2048);
    ctx->timer.begin(NICE_PH_ENC_LONG, st);
    hipLaunchKernelGGL(enc_tilebits, dim3(tblocks), dim3(256), 0, st, a);
    if (a.groups > 1) hipLaunchKernelGGL(enc_group_reduce, dim3(a.groups, n_frames), dim3(256), 0, st, a, 1);
    hipLaunchKernelGGL(enc_tilescan, dim3(a.groups, n_frames), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(enc_pack_long, dim3(tblocks), dim3(256), 0, st, a, 0);
    hipLaunchKernelGGL(enc_pack_long, dim3(tblocks), dim3(256), 0, st, a, 1);
    ctx->timer.end(st);
    // every other frame: one pass, tile offsets by look-back
    const uint64_t pblocks = std::min<uint64_t>(total_tiles, (uint64_t)ctx->cus * PACK_BLOCKS_PER_CU);
    ctx->timer.begin(NICE_PH_ENC_PACK, st);
    hipLaunchKernelGGL(enc_pack, dim3((uint32_t)pblocks), dim3(256), 0, st, a);
    hipLaunchKernelGGL(enc_pack_over, dim3(PACK_OVER_BLOCKS), dim3(256), 0, st, a);
    hipLaunchKernelGGL(enc_edges, dim3(std::min<uint32_t>((T + 255) / 256, 64u), std::min<uint32_t>(n_frames, 4096u)),
                       dim3(256), 0, st, a);
    ctx->timer.end(st);
    ctx->timer.begin(NICE_PH_ENC_TAIL, st);
    hipLaunchKernelGGL(enc_tail, dim3((n_frames + 63) / 64), dim3(64), 0, st, a);
    ctx->timer.end(st);
  }
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}


// ---- decoder ---------------------------------------------------------------
namespace {
struct DecLayout {
  size_t total;
  size_t o_tables, o_dstart, o_entry, o_last, o_ck, o_cpx, o_cstart, o_recs, o_changed, o_fchanged, o_rowbuf;
  size_t o_ev, o_evck, o_evn, o_agree, o_items, o_icount;
  size_t o_hand, o_abort;
};
// Jacobi iterations queued (one change flag each; each returns at once when the
// previous one changed nothing), then the device-side settle (dec_sync_settle)
// and one more iteration behind its flag: no host round trip.  Flags: the
// queued iterations', the settle's, the last iteration's.
constexpr uint32_t kSyncQueuedMax = 16, kSyncFlags = kSyncQueuedMax + 2;
constexpr uint32_t kSettledFlag = kSyncQueuedMax, kFinalFlag = kSyncQueuedMax + 1;
// 8: a single 4K SYN-v1 frame needs 5; round 5 queued 16 to stay clear of its
// one-lane settle (3.3 s when 4 were queued), but the round-6 parallel settle
// finishes a frame a few iterations short in ~10 ms, and each early-exiting
// launch past the fixpoint costs ~5 us (one 4K frame: resync 0.234 -> 0.186
// ms for 16 -> 8, 512 frames 1.41 -> 1.36; profiles/r06zm_syncq.log)
#ifndef NICE_SYNC_QUEUED
#define NICE_SYNC_QUEUED 8
#endif
constexpr uint32_t kSyncQueued = NICE_SYNC_QUEUED;
static_assert(kSyncQueued >= 1 && kSyncQueued <= kSyncQueuedMax, "queued sync iterations");
DecLayout dec_layout(uint32_t n_frames, uint32_t max_chunks, uint32_t n_ck, uint64_t npx, size_t rowbuf,
                     uint32_t ev_cap, uint32_t subs, size_t hand = 0, bool abort_flags = false) {
  DecLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes, 256); return r; };
  L.o_tables = take((size_t)n_frames * sizeof(DecTables));
  L.o_dstart = take((size_t)n_frames * 8);
  L.o_entry = take((size_t)n_frames * max_chunks * 8);
  L.o_last = take((size_t)n_frames * max_chunks * 8);
  L.o_ck = take((size_t)n_frames * n_ck * max_chunks * 8);
  L.o_cpx = take((size_t)n_frames * max_chunks * 8);
  L.o_cstart = take((size_t)n_frames * max_chunks * 8);
  L.o_recs = take((size_t)n_frames * ((npx + 3) & ~3ull) * 4);
  L.o_changed = take(4 * kSyncFlags);
  L.o_fchanged = take((size_t)n_frames * 4);
  L.o_rowbuf = take(rowbuf);
  // first-pass pixel events (ev_cap per slice, 0: not kept)
  L.o_ev = take((size_t)n_frames * ((max_chunks + 63) & ~63u) * ev_cap * 4);
  L.o_evck = take(ev_cap ? (size_t)n_frames * n_ck * max_chunks * 4 : 0);
  L.o_evn = take(ev_cap ? (size_t)n_frames * max_chunks * 4 : 0);
  L.o_agree = take(ev_cap ? (size_t)n_frames * max_chunks * 4 : 0);
  L.o_items = take(ev_cap ? (size_t)n_frames * max_chunks * subs * 4 : 0);
  L.o_icount = take(ev_cap ? (size_t)n_frames * 4 : 0);
  L.o_hand = take(hand);
  L.o_abort = take(hand || abort_flags ? (size_t)n_frames * 4 : 0);
  L.total = o;
  return L;
}
struct RecGeom {
  uint32_t seg, nseg, R;
  size_t lds;
  bool in_lds;
};
RecGeom rec_geom(uint32_t w) {
  RecGeom g;
  uint32_t s = (w + DEC_MAX_SEGS - 1) / DEC_MAX_SEGS;
  if (s < 6) s = 6;
  g.seg = s;
  g.nseg = w ? (w + s - 1) / s : 1;
  // the last segment (which runs to W) must be >= 6 pixels: its last three
  // columns read pixels 0..2 of the same row, written by lane 0 at steps 0..2
  if (g.nseg > 1 && w - (g.nseg - 1) * s < 6) g.nseg -= 1;
  g.R = w >= 3 ? 4 : 8;
  const size_t kw = (w + 31) / 32;
  const size_t head = 512 + align_up(kw, 4) * 4 + align_up(w, 4) * 4;   // RecLds <= 512 B, records
  const size_t ring = (size_t)g.R * w * 4;
  g.in_lds = head + ring <= 150 * 1024;
  g.lds = g.in_lds ? head + ring : head;
  return g;
}
}  // namespace

// ---- context-free host-buffer entry points --------------------------------
static std::mutex g_default_mu;
static nice_ctx* g_default = nullptr;

static int default_ctx(nice_ctx** out) {
  std::lock_guard<std::mutex> g(g_default_mu);
  if (!g_default) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    int rc = nice_ctx_create(dev, &g_default);
    if (rc) return rc;
  }
  *out = g_default;
  return NICE_OK;
}

int nice_encode(const uint8_t* px, size_t px_len, uint32_t w, uint32_t h, uint8_t channels,
                uint8_t channels_out, uint8_t* out, size_t out_cap, size_t* out_len) {
  if (!out || !out_len) return NICE_E_ARG;
  if (channels != 3 && channels != 4) return NICE_E_ARG;
  const uint64_t N = (uint64_t)w * h;
  if (px_len < N * channels || (N > 0 && !px)) return NICE_E_ARG;
  nice_ctx* ctx;
  int rc = default_ctx(&ctx);
  if (rc) return rc;
  std::lock_guard<std::mutex> g(ctx->mu);
  NICE_HIP(hipSetDevice(ctx->device));
  const size_t in_bytes = align_up((size_t)N * channels, 256);
  const size_t bound = align_up(nice_encode_bound(w, h), 256);
  if ((rc = ctx->host_px.grow(in_bytes + 256))) return rc;
  if ((rc = ctx->host_out.grow(bound))) return rc;
  if ((rc = ctx->dev_len.grow(256))) return rc;
  if (N) NICE_HIP(hipMemcpy(ctx->host_px.ptr, px, (size_t)N * channels, hipMemcpyHostToDevice));
  rc = nice_encode_batch_dev(ctx, nullptr, (const uint8_t*)ctx->host_px.ptr, in_bytes, 1, w, h,
                             channels, channels_out, (uint8_t*)ctx->host_out.ptr, bound,
                             (uint64_t*)ctx->dev_len.ptr);
  if (rc) return rc;
  uint64_t n = 0;
  NICE_HIP(hipMemcpy(&n, ctx->dev_len.ptr, 8, hipMemcpyDeviceToHost));
  if (n > out_cap) {
    *out_len = n;
    return NICE_E_CAPACITY;
  }
  NICE_HIP(hipMemcpy(out, ctx->host_out.ptr, n, hipMemcpyDeviceToHost));
  *out_len = n;
  return NICE_OK;
}


int nice_decode_batch_dev(nice_ctx* ctx, void* stream, const uint8_t* d_streams,
                          uint64_t stream_stride, const uint64_t* d_stream_len, uint32_t n_frames,
                          uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px,
                          uint64_t px_stride, uint32_t flags, int32_t* d_status) {
  return nice::decode_batch_impl(ctx, stream, d_streams, stream_stride, d_stream_len, nullptr, n_frames, w, h,
                                 out_channels, d_px, px_stride, flags, d_status);
}

int nice_decode_batch_dev_hl(nice_ctx* ctx, void* stream, const uint8_t* d_streams, uint64_t stream_stride,
                             const uint64_t* d_stream_len, const uint64_t* h_stream_len, uint32_t n_frames,
                             uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px, uint64_t px_stride,
                             uint32_t flags, int32_t* d_status) {
  if (n_frames && !h_stream_len) return NICE_E_ARG;
  return nice::decode_batch_impl(ctx, stream, d_streams, stream_stride, d_stream_len, h_stream_len, n_frames, w, h,
                                 out_channels, d_px, px_stride, flags, d_status);
}

}  // extern "C"

// h_stream_len: the lengths on the host when the caller has them (saves a
// device round trip), else nullptr.
int nice::decode_batch_impl(nice_ctx* ctx, void* stream, const uint8_t* d_streams, uint64_t stream_stride,
                            const uint64_t* d_stream_len, const uint64_t* h_stream_len, uint32_t n_frames,
                            uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px, uint64_t px_stride,
                            uint32_t flags, int32_t* d_status) {
  if (!ctx || !d_streams || !d_stream_len || !d_status) return NICE_E_ARG;
  if (out_channels != 3 && out_channels != 4) return NICE_E_ARG;
  if ((stream_stride & 3) || ((uintptr_t)d_streams & 3)) return NICE_E_ARG;
  const uint64_t N = (uint64_t)w * h;
  if (N > (1ull << 30)) return NICE_E_ARG;
  if (n_frames == 0) return NICE_OK;
  if (N > 0 && (!d_px || px_stride < N * out_channels)) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  ctx->split_frames = 0;
  NICE_HIP(hipMemsetAsync(d_status, 0, (size_t)n_frames * 4, st));
  // stream lengths bound the chunk grid
  std::vector<uint64_t> lens(n_frames);
  if (h_stream_len) {
    std::copy(h_stream_len, h_stream_len + n_frames, lens.begin());
  } else {
    NICE_HIP(hipMemcpyAsync(lens.data(), d_stream_len, (size_t)n_frames * 8, hipMemcpyDeviceToHost, st));
    NICE_HIP(hipStreamSynchronize(st));
  }
  uint64_t max_len = 0;
  for (uint64_t l : lens) {
    if (l > stream_stride) return NICE_E_ARG;
    max_len = l > max_len ? l : max_len;
  }
  const uint64_t D = FILE_HEADER_BYTES * 8 + TABLE_HEADER_BITS;
  // slice size: long slices make the Jacobi re-parses (which run until the
  // slowest lane of a wave re-synchronises, ~1000 bits) cheap relative to the
  // first pass, short ones keep a small batch filling the GPU: aim for about
  // 256 CUs x 8 waves x 64 lanes x 2 slices, as a power of two in [1K, 16K]
  // (at least 2048 bits from ~48 Mbit of streams up: a 1024-bit slice holds
  // no checkpoint, so every Jacobi re-parse and dec_emit walk whole slices --
  // one 4K frame 9.75 -> 9.61 ms, 4 x 4K 10.03 -> 9.85, 8 x 1080p 5.17 ->
  // 5.11; one 1080p frame, whose 2048-bit slices leave the GPU emptier, 4.92
  // -> 4.96: kept at 1024, profiles/r06v_ab_slice_min.log)
  uint64_t total_bits = 0;
  for (uint64_t l : lens) total_bits += l * 8 > D ? l * 8 - D : 0;
  uint32_t cb = total_bits >= (48ull << 20) ? 2 * DEC_MIN_CHUNK_BITS : DEC_MIN_CHUNK_BITS;
  while (cb < DEC_MAX_CHUNK_BITS && total_bits / (2ull * cb) > 256ull * 8 * 64 * 2) cb *= 2;
  if (opt_set(NICE_OPT_DEC_SLICE_BITS)) {   // tests: force a slice size
    const uint32_t v = (uint32_t)opt_val(NICE_OPT_DEC_SLICE_BITS);
    if (v >= DEC_MIN_CHUNK_BITS && v <= DEC_MAX_CHUNK_BITS && (v & (v - 1)) == 0) cb = v;
  }
  const uint32_t max_chunks = max_len * 8 > D ? (uint32_t)((max_len * 8 - D + cb - 1) / cb) : 1;
  // checkpoints every 512 bits in slices up to 4K bits (small batches: the
  // re-parses and dec_emit's heads stop at the first meeting point, half as far
  // in: one 4K frame 9.59 -> 9.52 ms, 64 x 1080p 6.13 -> 6.07), every 1024 from
  // 8K bits up (512 x 4K: sync 12.0 -> 12.6 ms at 512, more checkpoint stores
  // than the shorter heads save; profiles/r06x_ab_ck_bits.log)
  const uint32_t ck_bits = cb <= 4096u ? DEC_CK_BITS_SMALL : DEC_CK_BITS;
  const uint32_t n_ck = cb / ck_bits - 1;
  const RecGeom g = rec_geom(w);
  // multi-wave row kernel for 64 <= W <= 16384 (one lane per 16-pixel segment),
  // single-wave kernel otherwise
  const uint32_t rows_thr = ((w + 15) / 16 + 63) / 64 * 64;
  const bool single_wave = opt_on(NICE_OPT_DEC_SINGLE_WAVE);
  const bool use_rows = w >= 64 && rows_thr <= 1024 && !single_wave;
  const size_t rows_lds = ((size_t)rows_thr * 7 + 8 + (size_t)4 * (w + (w >> 4) + 24)) * 4;   // rows_ring_stride
  const bool rows_in_lds = rows_thr <= 512 && rows_lds + 1024 <= 160 * 1024;   // + static LDS
  // 8-pixel segments (twice the lanes per frame) only on request
  // (NICE_DEC_SEG=8): they were the default where 16-pixel segments leave SIMDs
  // of a frame's CU idle (W <= 2048, frames not sharing CUs: 64 x 1080p 7.83 ->
  // 6.32 ms in round 2), but the round-3/4 row kernel with 16-pixel segments is
  // as fast or faster at every width measured (round 4, profiles/r04v, r04y:
  // 64 x 1080p reconstruct 6.58 vs 6.88 ms, W = 1280 / 1024 / 640: 6.68 / 5.77
  // / 6.22 vs 6.91 / 6.00 / 6.30 ms)
  const uint32_t rows8_thr = ((w + 7) / 8 + 63) / 64 * 64;
  const size_t rows8_lds = ((size_t)rows8_thr * 7 + 8 + (size_t)4 * (w + (w >> 4) + 24)) * 4;
  bool rows8 = false;
  if (opt_set(NICE_OPT_DEC_SEG)) rows8 = opt_val(NICE_OPT_DEC_SEG) == 8 && use_rows && rows_in_lds &&
                                                       rows8_thr <= 512 && rows8_lds <= 160 * 1024;
  // wide frames, few of them: strips of <= 256 segments on separate CUs
  // (dec_rows_split; its blocks wait on each other, so they should all be
  // resident: at most one per CU for half the CUs, frames in chunks of that
  // many strips).  When they are not (other kernels hold the CUs), a strip's
  // wait times out and the frame goes to the fallback launch (dec_rows_wide,
  // or dec_reconstruct above 16384 columns) -- slower, never wrong.
  // NICE_DEC_SPLIT=k forces k strips (tests), =0 disables
  const uint32_t nseg16 = (w + 15) / 16;
  const uint32_t split_cap = (uint32_t)std::max(ctx->cus / 2, 1);
  uint32_t strips = (nseg16 + SPLIT_THREADS_HOST - 1) / SPLIT_THREADS_HOST;
  if (opt_set(NICE_OPT_DEC_SPLIT)) strips = (uint32_t)opt_val(NICE_OPT_DEC_SPLIT);
  // <= 16384 columns: only when the whole batch fits at once (else one block
  // per frame is the better use of the CUs); wider: always, in frame chunks
  bool split = !single_wave && w >= 64 && strips >= 2 && strips <= split_cap &&
               (!use_rows || (uint64_t)n_frames * strips <= split_cap);
  // rows of up to 8192 pixels (8 waves) take the dataflow kernel on one CU
  // rather than strips on several (round 6: the strips' cross-CU hand-offs
  // cost more than the second CU gains); NICE_DEC_SPLIT forces the strips
  const uint32_t flow_wpr = ((w + 15) / 16 + 63) / 64;
  if (split && !opt_set(NICE_OPT_DEC_SPLIT) && use_rows && w <= FLOW_MAX_W_HOST && !opt_on(NICE_OPT_DEC_SEG) &&
      !(opt_set(NICE_OPT_DEC_FLOW) && opt_val(NICE_OPT_DEC_FLOW) <= 0))
    split = false;
  if (split) {
    const uint32_t sps = (nseg16 + strips - 1) / strips;
    // every strip >= 2 segments (>= 3 pixels: its first and last three) and <= 256 lanes
    if (sps > SPLIT_THREADS_HOST || nseg16 <= (strips - 1) * sps + 1) split = false;
  }
  const uint32_t split_frames = split ? std::min(n_frames, split_cap / strips) : 0;   // frames per launch
  // W <= 4096: the dataflow row kernel (no block barriers; dec_rows_flow).
  // At most one frame per CU: two row groups in flight and an 8-row ring (one
  // block per CU); larger batches: one group and a 4-row ring, so two frames
  // share each CU.  NICE_DEC_FLOW=0 takes dec_rows, =k forces k groups (A/B).
  uint32_t flow_k = 2, flow_ring = 8;
  bool flow = !split && use_rows && !rows8 && w <= FLOW_MAX_W_HOST;
  if (n_frames > (uint32_t)std::max(ctx->cus, 1)) { flow_k = 1; flow_ring = 4; }
  if (opt_set(NICE_OPT_DEC_FLOW)) {
    const int v = (int)opt_val(NICE_OPT_DEC_FLOW);
    if (v <= 0) flow = false;
    else flow_k = (uint32_t)v;
  }
  if (flow_k * flow_wpr > FLOW_THREADS_HOST / 64) flow_k = FLOW_THREADS_HOST / 64 / flow_wpr;
  if (flow_k > 4 || flow_k < 1) flow = false;   // (stamps of 8 rows)
  if (flow_k > 1) flow_ring = 8;
  size_t flow_lds = FLOW_CTL_BYTES_HOST + ((size_t)flow_ring * (w + (w >> 4) + 24) + 4) * 4;   // rows_ring_stride
  if (flow_lds > 160 * 1024 && flow_k == 1 && flow_ring == 8) {   // wide rows: a 4-row ring (one row group)
    flow_ring = 4;
    flow_lds = FLOW_CTL_BYTES_HOST + ((size_t)flow_ring * (w + (w >> 4) + 24) + 4) * 4;
  }
  if (flow_lds > 160 * 1024) flow = false;
  const size_t hand = split ? (size_t)n_frames * h * strips * SPLIT_GRAN_HOST * 8 : 0;
  // per-frame redo flags: the split kernel's, and the dataflow kernel's (a
  // wait that timed out sends the frame to the barrier kernel)
  const bool want_abort = split || flow;
  // the row ring in global memory: dec_rows_wide (also the split path's
  // fallback) or dec_reconstruct without room in LDS
  const size_t ring_rows = use_rows ? (size_t)n_frames * 4 * (w + (w >> 4) + 24) * 4
                                    : (g.in_lds ? 0 : (size_t)n_frames * g.R * w * 4);
  const size_t rowbuf = split ? ring_rows : (use_rows && rows_in_lds) ? 0 : ring_rows;
  // keep the first sync pass's pixel events (one per >= 4 bits of a slice;
  // a slice with more parses its events again in dec_emit) unless the scratch
  // does not fit, then every slice is parsed again in dec_emit
  uint32_t ev_cap = opt_on(NICE_OPT_DEC_NO_EVENTS) ? 0u : cb / 4;
  if (opt_set(NICE_OPT_DEC_EV_CAP)) {   // tests: force event overflow
    const uint32_t v = (uint32_t)opt_val(NICE_OPT_DEC_EV_CAP);
    if (ev_cap && v >= 4 && v % 4 == 0 && v < ev_cap) ev_cap = v;
  }
  const uint32_t subs = cb / DEC_EMIT_BITS;
  DecLayout L = dec_layout(n_frames, max_chunks, n_ck, N, rowbuf, ev_cap, subs, hand, want_abort);
  int rc = ctx->dec.grow(L.total);
  if (rc && ev_cap) {
    (void)hipGetLastError();   // the failed allocation
    ev_cap = 0;
    L = dec_layout(n_frames, max_chunks, n_ck, N, rowbuf, 0, subs, hand, want_abort);
    rc = ctx->dec.grow(L.total);
  }
  if (rc) return rc;
  uint8_t* base = (uint8_t*)ctx->dec.ptr;
  DecArgs a{};
  a.streams = d_streams;
  a.stream_stride = stream_stride;
  a.stream_len = (const unsigned long long*)d_stream_len;
  a.n_frames = n_frames;
  a.W = w;
  a.H = h;
  a.out_channels = out_channels;
  a.flags = flags;
  a.px_out = d_px;
  a.px_stride = px_stride;
  a.status = d_status;
  a.tables = base + L.o_tables;
  a.data_start = (unsigned long long*)(base + L.o_dstart);
  a.max_chunks = max_chunks;
  a.chunk_bits = cb;
  a.n_ck = n_ck;
  a.ck_bits = ck_bits;
  a.emit_blocks = (uint32_t)(((uint64_t)max_chunks * (cb / DEC_EMIT_BITS) + DEC_PARSE_THREADS - 1) / DEC_PARSE_THREADS);
  a.chunk_blocks = (max_chunks + DEC_PARSE_THREADS - 1) / DEC_PARSE_THREADS;
  a.chunk_px = (unsigned long long*)(base + L.o_cpx);
  a.chunk_start = (unsigned long long*)(base + L.o_cstart);
  a.entry = (unsigned long long*)(base + L.o_entry);
  a.last = (unsigned long long*)(base + L.o_last);
  a.ck = (unsigned long long*)(base + L.o_ck);
  a.recs = (uint32_t*)(base + L.o_recs);
  a.rec_stride = (N + 3) & ~3ull;
  a.seg = g.seg;
  a.nseg = g.nseg;
  a.rows_in_lds = g.in_lds ? 1u : 0u;
  a.parse_slow = opt_on(NICE_OPT_DEC_SLOW_PARSE) ? 1u : 0u;   // tests / A/B: the general parse only
  a.rowbuf = (uint32_t*)(base + L.o_rowbuf);
  uint32_t* changed = (uint32_t*)(base + L.o_changed);
  if (ev_cap) {
    a.ev = (uint32_t*)(base + L.o_ev);
    a.ev_cap = ev_cap;
    a.ev_ck = (uint32_t*)(base + L.o_evck);
    a.ev_n = (uint32_t*)(base + L.o_evn);
    a.agree = (uint32_t*)(base + L.o_agree);
    a.head_items = (uint32_t*)(base + L.o_items);
    a.head_count = (uint32_t*)(base + L.o_icount);
  }

  PhaseTimer& tm = ctx->timer;
  tm.begin(NICE_PH_DEC_TABLES, st);
  hipLaunchKernelGGL(dec_tables, dim3(n_frames), dim3(256), 0, st, a);
  tm.end(st);
  if (N == 0) {
    NICE_HIP(hipGetLastError());
    return NICE_OK;
  }
  const bool want_stats = opt_on(NICE_OPT_DEC_STATS);
  unsigned long long* dstats = nullptr;
  if (want_stats && hipMalloc(&dstats, 1024) == hipSuccess) {
    (void)hipMemsetAsync(dstats, 0, 1024, st);
    a.stats = dstats;
  }
  hipLaunchKernelGGL(dec_init_entries, dim3((max_chunks + 255) / 256 < 64 ? (max_chunks + 255) / 256 : 64, n_frames),
                     dim3(256), 0, st, a);
  const dim3 cgrid(n_frames * a.chunk_blocks);
  // Jacobi iteration of the chunk entry states to the fixpoint, all on the
  // device: queued iterations (each returns at once if the previous one changed
  // nothing), the sequential settle of frames still changing after the last
  // one, and one more iteration for the slices the settle moved
  uint32_t it_count = 0;
  uint32_t queued = std::min(kSyncQueued, max_chunks + 1);
  if (opt_set(NICE_OPT_DEC_SYNC_QUEUED)) {   // tests: fewer queued iterations
    const uint32_t v = (uint32_t)opt_val(NICE_OPT_DEC_SYNC_QUEUED);
    if (v >= 1 && v <= kSyncQueuedMax) queued = std::min(v, max_chunks + 1);
  }
  uint32_t* fchanged = (uint32_t*)(base + L.o_fchanged);
  NICE_HIP(hipMemsetAsync(changed, 0, 4 * kSyncFlags, st));
  NICE_HIP(hipMemsetAsync(fchanged, 0, (size_t)n_frames * 4, st));
  for (uint32_t it = 0; it < queued; ++it, ++it_count) {
    tm.begin(it ? NICE_PH_DEC_RESYNC : NICE_PH_DEC_SYNC, st);
    hipLaunchKernelGGL(dec_sync, cgrid, dim3(DEC_PARSE_THREADS), 0, st, a, changed + it, it ? changed + it - 1 : nullptr,
                       it + 1 == queued ? fchanged : nullptr);
    tm.end(st);
  }
  tm.begin(NICE_PH_DEC_RESYNC, st);
  hipLaunchKernelGGL(dec_sync_settle, dim3(n_frames), dim3(512), 0, st, a, changed + queued - 1, fchanged,
                     changed + kSettledFlag);
  // the last iteration, for the slices the settle moved: it must change no
  // entry; a frame where it does (a settle that disagreed with dec_sync) is
  // failed by dec_scan instead of decoded from a non-fixpoint
  NICE_HIP(hipMemsetAsync(fchanged, 0, (size_t)n_frames * 4, st));
  hipLaunchKernelGGL(dec_sync, cgrid, dim3(DEC_PARSE_THREADS), 0, st, a, changed + kFinalFlag,
                     changed + kSettledFlag, fchanged);
  tm.end(st);
  // the last sync iteration (no entry changed) already produced chunk_px
  tm.begin(NICE_PH_DEC_SCAN, st);
  a.unsettled = fchanged;
  hipLaunchKernelGGL(dec_scan, dim3(n_frames), dim3(1024), 0, st, a);
  a.unsettled = nullptr;
  // strict: the reads where the reference's refill loop would wrap (frames
  // whose tables are all <= 25 bits return at once)
  if (flags & NICE_DEC_STRICT_REFERENCE) hipLaunchKernelGGL(dec_strict_refill, cgrid, dim3(DEC_PARSE_THREADS), 0, st, a);
  tm.end(st);
  tm.begin(NICE_PH_DEC_EMIT, st);
  if (a.ev) hipLaunchKernelGGL(dec_heads, dim3(n_frames), dim3(1024), 0, st, a);
  {
    // run pixels: slots without this call's tag.  Clear (tag 0) only when the
    // region moved or resized (other data may have held it) or the tags wrap.
    const uint64_t words = (uint64_t)n_frames * a.rec_stride;
    if (a.recs != ctx->rec_region || words != ctx->rec_words || ctx->dec.gen != ctx->rec_gen ||
        ctx->rec_epoch >= 15u || opt_on(NICE_OPT_DEC_REC_CLEAR)) {
      NICE_HIP(hipMemsetAsync(a.recs, 0, words * 4, st));
      ctx->rec_region = a.recs;
      ctx->rec_words = words;
      ctx->rec_gen = ctx->dec.gen;
      ctx->rec_epoch = 0;
    }
    a.rec_tag = ++ctx->rec_epoch;
  }
  hipLaunchKernelGGL(dec_emit, dim3(n_frames * a.emit_blocks), dim3(DEC_PARSE_THREADS), 0, st, a);
  tm.end(st);
  if (a.ev) {
    tm.begin(NICE_PH_DEC_PLACE, st);
    hipLaunchKernelGGL(dec_place, dim3((max_chunks + DEC_PLACE_WAVES - 1) / DEC_PLACE_WAVES, n_frames), dim3(64 * DEC_PLACE_WAVES), 0, st, a);
    tm.end(st);
  }
  if (g.lds > 64 * 1024)
    NICE_HIP(hipFuncSetAttribute((const void*)dec_reconstruct,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds));
  tm.begin(NICE_PH_DEC_RECON, st);
  if (split) {
    a.strips = strips;
    a.hand = (unsigned long long*)(base + L.o_hand);
    a.hand_abort = (uint32_t*)(base + L.o_abort);
    NICE_HIP(hipMemsetAsync(a.hand, 0, hand, st));
    NICE_HIP(hipMemsetAsync(a.hand_abort, 0, (size_t)n_frames * 4, st));
    const uint32_t sps = (nseg16 + strips - 1) / strips;
    // tails + flags + 4, then the ring; above 80 KB so a CU holds one strip
    size_t lds = ((size_t)SPLIT_THREADS_HOST * 7 + 4 + 4 * ((size_t)sps * 16 + 6 + ((sps * 16 + 6) >> 4) + 17)) * 4;
    lds = std::max<size_t>(lds, 82 * 1024);
    NICE_HIP(hipFuncSetAttribute((const void*)dec_rows_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    a.test_absent_strip = ctx->test_split_absent;
    for (uint32_t f0 = 0; f0 < n_frames; f0 += split_frames) {
      a.split_f0 = f0;
      hipLaunchKernelGGL(dec_rows_split, dim3(std::min(split_frames, n_frames - f0) * strips),
                         dim3(SPLIT_THREADS_HOST), lds, st, a);
    }
    a.split_f0 = 0;
    a.test_absent_strip = 0;
    // fallback: frames whose strips timed out waiting for a non-resident
    // neighbour (every other block returns at once)
    DecArgs r = a;
    r.redo = 1;
    if (use_rows)
      hipLaunchKernelGGL(dec_rows_wide, dim3(n_frames), dim3(rows_thr), ((size_t)rows_thr * 7 + 8) * 4, st, r);
    else
      hipLaunchKernelGGL(dec_reconstruct, dim3(n_frames), dim3(64), g.lds, st, r);
    ctx->split_abort = a.hand_abort;
    ctx->split_frames = n_frames;
  } else if (flow) {
    if (flow_lds > 64 * 1024)
      NICE_HIP(hipFuncSetAttribute((const void*)dec_rows_flow, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)flow_lds));
    a.flow_k = flow_k;
    a.flow_ring = flow_ring;
    a.hand_abort = (uint32_t*)(base + L.o_abort);
    NICE_HIP(hipMemsetAsync(a.hand_abort, 0, (size_t)n_frames * 4, st));
    a.test_absent_strip = opt_on(NICE_OPT_TEST_FLOW_ABSENT) ? 1u : 0u;
    hipLaunchKernelGGL(dec_rows_flow, dim3(n_frames), dim3(64 * flow_k * flow_wpr), flow_lds, st, a);
    a.test_absent_strip = 0;
    // fallback: frames whose waits timed out (the workgroup was
    // preempted or time-sliced past the bound) go to the barrier kernel; its
    // blocks return at once for every other frame
    DecArgs r = a;
    r.redo = 1;
    if (rows_in_lds) {
      if (rows_lds > 64 * 1024)
        NICE_HIP(hipFuncSetAttribute((const void*)dec_rows, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)rows_lds));
      hipLaunchKernelGGL(dec_rows, dim3(n_frames), dim3(rows_thr), rows_lds, st, r);
    } else {
      hipLaunchKernelGGL(dec_rows_wide, dim3(n_frames), dim3(rows_thr), ((size_t)rows_thr * 7 + 8) * 4, st, r);
    }
    ctx->split_abort = a.hand_abort;
    ctx->split_frames = n_frames;
  } else if (use_rows && rows_in_lds && rows8) {
    if (rows8_lds > 64 * 1024)
      NICE_HIP(hipFuncSetAttribute((const void*)dec_rows8, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)rows8_lds));
    hipLaunchKernelGGL(dec_rows8, dim3(n_frames), dim3(rows8_thr), rows8_lds, st, a);
  } else if (use_rows && rows_in_lds) {
    if (rows_lds > 64 * 1024)
      NICE_HIP(hipFuncSetAttribute((const void*)dec_rows, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)rows_lds));
    hipLaunchKernelGGL(dec_rows, dim3(n_frames), dim3(rows_thr), rows_lds, st, a);
  } else if (use_rows) {
    hipLaunchKernelGGL(dec_rows_wide, dim3(n_frames), dim3(rows_thr), ((size_t)rows_thr * 7 + 8) * 4, st, a);
  } else {
    hipLaunchKernelGGL(dec_reconstruct, dim3(n_frames), dim3(64), g.lds, st, a);
  }
  tm.end(st);
  if (dstats) {
    unsigned long long h[128] = {0};
    (void)hipMemcpyAsync(h, dstats, 1024, hipMemcpyDeviceToHost, st);
    uint32_t chg[kSyncFlags] = {0};
    (void)hipMemcpyAsync(chg, changed, 4 * kSyncFlags, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    fprintf(stderr,
            "[nice dec stats] rows=%llu unconverged_segs=%llu tail_unknown_segs=%llu "
            "recomputed_px=%llu fixup_rounds=%llu sync_iters=%u seg=%u nseg=%u "
            "clk[load=%llu spec=%llu fix=%llu emit=%llu]\n",
            h[0], h[1], h[2], h[3], h[4], it_count, g.seg, g.nseg, h[5], h[6], h[7], h[8]);
    fprintf(stderr, "[nice dec stats] sync iterations that changed an entry:");
    for (uint32_t i = 0; i < kSyncFlags; ++i) fprintf(stderr, " %u", chg[i]);
    fprintf(stderr, " (queued %u, then settled, final)\n", queued);
    for (int w = 0; w < 4; ++w) {   // dec_rows_flow (-DNICE_FLOW_STATS builds): cycles per row by phase
      const unsigned long long* q = h + 64 + 8 * w;
      if (q[7])
        fprintf(stderr, "[nice flow stats] wave %d rows=%llu cyc/row: emit+decode=%.0f wait=%.0f ring=%.0f spec=%.0f "
                "fix=%.0f publish=%.0f rounds/row=%.2f\n", w, q[7], (double)q[0] / q[7], (double)q[1] / q[7],
                (double)q[2] / q[7], (double)q[3] / q[7], (double)q[4] / q[7], (double)q[5] / q[7],
                (double)q[6] / q[7]);
    }
    fprintf(stderr, "[nice dec stats] unknown segment tails: copies of an unknown %llu, narrowed %llu\n", h[24], h[25]);
    fprintf(stderr, "[nice dec stats] re-parse met previous parse at checkpoint:");
    for (int k = 0; k < 17; ++k) fprintf(stderr, " %d:%llu", k, h[32 + k]);
    fprintf(stderr, "\n");
    fprintf(stderr, "[nice dec stats] slice=%u emit waves=%llu wave_iters=%llu active_lane_iters=%llu fills=%llu\n",
            a.chunk_bits, h[20], h[16], h[17], h[18]);
    fprintf(stderr, "[nice dec stats] slices by first-pass meeting checkpoint: 0:%llu 1:%llu 2-4:%llu 5-16:%llu "
            "17-64:%llu 65+:%llu none:%llu overflow:%llu (ev_cap %u)\n",
            h[50], h[51], h[52], h[53], h[54], h[55], h[56], h[57], a.ev_cap);
    fprintf(stderr, "[nice dec stats] fix-up rounds per row: 0:%llu 1:%llu 2:%llu 3:%llu 4:%llu 5:%llu 6+:%llu\n",
            h[9], h[10], h[11], h[12], h[13], h[14], h[15]);
    if (h[61]) fprintf(stderr, "[nice dec stats] sync first pass: waves=%llu cycles/wave=%.0f refill cycles/wave=%.0f "
            "refills/wave=%.1f iterations/wave=%.1f active lane share=%.3f\n",
            h[61], h[61] ? (double)h[56] / h[61] : 0.0, h[61] ? (double)h[57] / h[61] : 0.0,
            h[61] ? (double)h[58] / h[61] : 0.0, h[61] ? (double)h[59] / h[61] : 0.0,
            h[59] ? (double)h[60] / (64.0 * h[59]) : 0.0);
    (void)hipFree(dstats);
  }
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}

extern "C" {

// ---- one image sharded over ranks ------------------------
int nice_band_classify(nice_ctx* ctx, void* stream, const uint8_t* d_px, uint64_t px0, uint64_t px_count,
                       uint32_t w, uint32_t h, uint8_t channels, uint8_t channels_out, uint32_t tile_lo,
                       uint32_t tile_hi, uint32_t* d_edges) {
  if (!ctx || !d_px || !d_edges || (channels != 3 && channels != 4)) return NICE_E_ARG;
  const uint64_t N = (uint64_t)w * h;
  const uint32_t T = tiles_for(w, h);
  if (N == 0 || N > (1ull << 30) || tile_lo >= tile_hi || tile_hi > T) return NICE_E_ARG;
  // pixel memory must hold the band and the 3 rows + 3 pixels its references reach
  const uint64_t band_px0 = (uint64_t)tile_lo * ENC_TILE;
  const uint64_t band_px1 = std::min<uint64_t>((uint64_t)tile_hi * ENC_TILE, N);
  const uint64_t need0 = band_px0 > 3ull * w + 3 ? band_px0 - 3ull * w - 3 : 0;
  if (px0 > need0 || px0 + px_count < band_px1 || px0 + px_count > N) return NICE_E_ARG;
  if (channels == 4 && ((uintptr_t)d_px & 3)) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  EncLayout L = enc_layout(1, T, band_px1 - band_px0);
  int rc = ctx->band.grow(L.total);
  if (rc) return rc;
  uint8_t* base = (uint8_t*)ctx->band.ptr;
  EncArgs a = enc_args(L, base, 1, w, h, channels, channels_out, T, N);
  if (ctx->test_pack_cap_bpp) a.pack_cap_bits = (uint32_t)PACK_SUB * ENC_TILE * ctx->test_pack_cap_bpp;
  a.cmask = nullptr;   // band tiles: the pair kernel counts its run digits itself
  // virtual bases: global pixel index g addresses d_px + (g - px0) * channels,
  // band records are stored from the band's first pixel
  a.px = d_px - (int64_t)px0 * channels;
  a.frame_stride = 0;
  a.recs = (uint32_t*)(base + L.o_recs) - band_px0;
  a.tile_lo = tile_lo;
  a.tile_hi = tile_hi;
  a.groups = (tile_hi - tile_lo + ENC_GROUP_TILES - 1) / ENC_GROUP_TILES;
  a.px_lo = (int64_t)px0;
  a.px_hi = (int64_t)(px0 + px_count);
  a.band = 1;
  // one-pass packer with look-back from band_bit0; FLAG_LONG bands take the
  // long-code path (tile bits, their scan) like frames
  a.pack_mode = 0;
  a.long_only = 1;
  NICE_HIP(hipMemsetAsync(base, 0, L.zero_bytes, st));
  // the ring / strip kernels read the band's pixels through the virtual base
  // as 32-bit words: it must be 4-byte aligned
  const ClsKind ck = pick_classify(w, channels, ((uintptr_t)a.px & 3) == 0);
  // strip kernel: the band's rows (tiles outside the band are staged, not classified)
  const uint32_t tpr = std::max<uint32_t>(w / ENC_TILE, 1u);
  const uint32_t rows_band = (tile_hi + tpr - 1) / tpr - tile_lo / tpr;
  launch_classify(ctx, ck, a, tile_hi - tile_lo, rows_band, st);
  ctx->last_classify = (int)ck;
  hipLaunchKernelGGL(enc_band_edges, dim3(1), dim3(256), 0, st, a, d_edges);
  NICE_HIP(hipGetLastError());
  ctx->bs = BandState{};
  ctx->bs.a = a;
  ctx->bs.bhist = (uint32_t*)(base + L.o_bhist);
  ctx->bs.classified = true;
  return NICE_OK;
}

static int band_runs(nice_ctx* ctx, void* stream, uint32_t band_next, const uint32_t* d_band_next,
                     uint32_t* d_hist) {
  if (!ctx || !d_hist || !ctx->bs.classified) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  EncArgs& a = ctx->bs.a;
  a.band_next = band_next;
  a.band_next_dev = d_band_next;
  if (a.groups > 1) hipLaunchKernelGGL(enc_group_reduce, dim3(a.groups, 1), dim3(256), 0, st, a, 0);
  hipLaunchKernelGGL(enc_tailruns, dim3(a.groups, 1), dim3(1024), 0, st, a);
  a.band_next_dev = nullptr;
  NICE_HIP(hipMemcpyAsync(ctx->bs.bhist, a.hist, N_BINS * 4, hipMemcpyDeviceToDevice, st));
  NICE_HIP(hipMemcpyAsync(d_hist, a.hist, N_BINS * 4, hipMemcpyDeviceToDevice, st));
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}

int nice_band_runs(nice_ctx* ctx, void* stream, uint32_t band_next, uint32_t* d_hist) {
  return band_runs(ctx, stream, band_next, nullptr, d_hist);
}

int nice_band_runs_dev(nice_ctx* ctx, void* stream, const uint32_t* d_band_next, uint32_t* d_hist) {
  if (!d_band_next) return NICE_E_ARG;
  return band_runs(ctx, stream, 0, d_band_next, d_hist);
}

// Code tables from the summed histogram, the header into the context's header
// buffer, the band's bit count and the data start into d_info (device).
static int band_tables(nice_ctx* ctx, hipStream_t st, const uint32_t* d_hist_total, unsigned long long* d_info) {
  EncArgs& a = ctx->bs.a;
  NICE_HIP(hipMemcpyAsync(a.hist, d_hist_total, N_BINS * 4, hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(enc_tables, dim3(N_STREAMS), dim3(64), 0, st, a);
  EncArgs h = a;   // the header goes to the context's header buffer
  h.out = (uint8_t*)ctx->band_hdr.ptr;
  h.out_stride = 4096;
  h.out_len = (unsigned long long*)((uint8_t*)ctx->band_hdr.ptr + 4096);
  hipLaunchKernelGGL(enc_header, dim3(1), dim3(64), 0, st, h);
  hipLaunchKernelGGL(enc_packtab, dim3(1), dim3(256), 0, st, a);
  hipLaunchKernelGGL(enc_band_sum, dim3(1), dim3(256), 0, st, a, (const uint32_t*)ctx->bs.bhist, d_info);
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}

int nice_band_tables(nice_ctx* ctx, void* stream, const uint32_t* d_hist_total, uint64_t* band_bits,
                     uint64_t* seed_bit) {
  if (!ctx || !d_hist_total || !ctx->bs.classified) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = ctx->band_hdr.grow(4096 + 64);
  if (rc) return rc;
  unsigned long long* info = (unsigned long long*)((uint8_t*)ctx->band_hdr.ptr + 4096 + 16);
  if ((rc = band_tables(ctx, st, d_hist_total, info))) return rc;
  unsigned long long hinfo[2];
  NICE_HIP(hipMemcpyAsync(hinfo, info, 16, hipMemcpyDeviceToHost, st));
  NICE_HIP(hipStreamSynchronize(st));
  ctx->bs.band_bits = hinfo[0];
  ctx->bs.seed_bit = hinfo[1];
  ctx->bs.tabled = true;
  if (band_bits) *band_bits = hinfo[0];
  if (seed_bit) *seed_bit = hinfo[1];
  return NICE_OK;
}

int nice_band_tables_dev(nice_ctx* ctx, void* stream, const uint32_t* d_hist_total, uint64_t* d_info) {
  if (!ctx || !d_hist_total || !d_info || !ctx->bs.classified) return NICE_E_ARG;
  NICE_HIP(hipSetDevice(ctx->device));
  int rc = ctx->band_hdr.grow(4096 + 64);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = band_tables(ctx, st, d_hist_total, (unsigned long long*)d_info))) return rc;
  // the context's own copy: the caller's buffer may be freed or reused before the pack
  unsigned long long* mine = (unsigned long long*)((uint8_t*)ctx->band_hdr.ptr + 4096 + 32);
  NICE_HIP(hipMemcpyAsync(mine, d_info, 16, hipMemcpyDeviceToDevice, st));
  ctx->bs.tabled = true;
  ctx->bs.band_bits = ~0ull;   // known to the caller once d_info is read (nice_band_pack_bits)
  ctx->bs.seed_bit = ~0ull;
  ctx->bs.d_info = mine;
  return NICE_OK;
}

uint32_t nice_tile_pixels(void) { return ENC_TILE; }

// the stream words the band touches, then a two-word trailer (a deferred
// wrapped write, enc_band_fix)
static uint64_t band_data_words(uint64_t band_bit0, uint64_t band_bits) {
  return band_bits ? ((band_bit0 + band_bits + 31) >> 5) - (band_bit0 >> 5) : 0;
}

uint64_t nice_band_words(uint64_t band_bit0, uint64_t band_bits) {
  return band_data_words(band_bit0, band_bits) + 2;   // every band has its trailer (status, deferred write)
}

int nice_band_pack_bits(nice_ctx* ctx, void* stream, uint64_t band_bit0, uint64_t band_bits, uint32_t* d_words,
                        uint64_t words_cap) {
  if (!ctx || !ctx->bs.tabled) return NICE_E_ARG;
  const uint64_t nw = nice_band_words(band_bit0, band_bits);
  if (nw > words_cap || (nw && !d_words)) return NICE_E_ARG;
  if (ctx->bs.seed_bit != ~0ull && band_bit0 < ctx->bs.seed_bit) return NICE_E_ARG;
  ctx->bs.band_bits = band_bits;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  EncArgs a = ctx->bs.a;
  a.band_bit0 = band_bit0;
  a.out = (uint8_t*)d_words - (int64_t)(band_bit0 >> 5) * 4;   // virtual: stream word w at d_words[w - w0]
  a.out_stride = 0;
  a.band_fix = d_words + (nw - 2);
  NICE_HIP(hipMemsetAsync(a.band_fix, 0, 8, st));
  // the bit count the caller read back must be the device's: on a mismatch the
  // pack kernels skip the band and the trailer carries BAND_FIX_BAD, which
  // nice_band_assemble reports
  if (ctx->bs.d_info)
    hipLaunchKernelGGL(enc_band_check, dim3(1), dim3(64), 0, st, a, ctx->bs.d_info, (unsigned long long)band_bits);
  if (band_bits == 0) {   // no data words: the trailer only
    NICE_HIP(hipGetLastError());
    return NICE_OK;
  }
  // the first word holds the previous band's last bits: only OR-ed into (enc_edges)
  NICE_HIP(hipMemsetAsync(d_words, 0, 4, st));
  const uint32_t nt = a.tile_hi - a.tile_lo;
  const uint32_t ng = (nt + PACK_SUB - 1) / PACK_SUB;
  NICE_HIP(hipMemsetAsync(a.status, 0, (size_t)ng * 8, st));
  NICE_HIP(hipMemsetAsync(a.pack_ctr, 0, 4, st));
  NICE_HIP(hipMemsetAsync(a.over_count, 0, 4, st));
  // FLAG_LONG (the launches return at once otherwise): tile bits, their scan from
  // band_bit0, the codes that fit the cache, then the wrapped writes
  const uint32_t tblocks = std::min<uint32_t>(nt, 2048u);
  hipLaunchKernelGGL(enc_tilebits, dim3(tblocks), dim3(256), 0, st, a);
  if (a.groups > 1) hipLaunchKernelGGL(enc_group_reduce, dim3(a.groups, 1), dim3(256), 0, st, a, 1);
  hipLaunchKernelGGL(enc_tilescan, dim3(a.groups, 1), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(enc_pack_long, dim3(tblocks), dim3(256), 0, st, a, 0);
  hipLaunchKernelGGL(enc_pack_long, dim3(tblocks), dim3(256), 0, st, a, 1);
  // every other band: one pass, group offsets by look-back from band_bit0
  hipLaunchKernelGGL(enc_pack, dim3((uint32_t)std::min<uint64_t>(nt, (uint64_t)ctx->cus * PACK_BLOCKS_PER_CU)),
                     dim3(256), 0, st, a);
  hipLaunchKernelGGL(enc_pack_over, dim3(PACK_OVER_BLOCKS), dim3(256), 0, st, a);
  hipLaunchKernelGGL(enc_edges, dim3(std::min<uint32_t>((ng + 255) / 256, 64u), 1), dim3(256), 0, st, a);
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}

int nice_band_pack(nice_ctx* ctx, void* stream, uint64_t band_bit0, uint32_t* d_words, uint64_t words_cap) {
  if (!ctx || !ctx->bs.tabled || ctx->bs.band_bits == ~0ull) return NICE_E_ARG;
  return nice_band_pack_bits(ctx, stream, band_bit0, ctx->bs.band_bits, d_words, words_cap);
}

int nice_band_assemble(nice_ctx* ctx, void* stream, const uint32_t* d_words, const uint64_t* band_bit0,
                       const uint64_t* band_bits, uint32_t n_bands, uint8_t* d_out, uint64_t out_cap,
                       uint64_t* out_len) {
  if (!ctx || !ctx->bs.tabled || !d_out || !out_len || n_bands == 0 || !band_bit0 || !band_bits)
    return NICE_E_ARG;
  // the data start: learned by nice_band_tables, else the first band's start
  const uint64_t seed = ctx->bs.seed_bit != ~0ull ? ctx->bs.seed_bit : band_bit0[0];
  // meta: band first words [R], band offsets [R + 1], data end, out_len, band first bits [R],
  // status (a band's trailer marked BAND_FIX_BAD: its pack saw a wrong band_bits)
  std::vector<unsigned long long> meta(3 * n_bands + 4);
  uint64_t off = 0, end = seed;
  for (uint32_t r = 0; r < n_bands; ++r) {
    if (band_bit0[r] != end) return NICE_E_ARG;   // bands must tile the data bits
    meta[r] = band_bit0[r] >> 5;
    meta[n_bands + r] = off;
    meta[2 * n_bands + 3 + r] = band_bit0[r];
    off += nice_band_words(band_bit0[r], band_bits[r]);
    end += band_bits[r];
  }
  meta[2 * n_bands] = off;
  meta[2 * n_bands + 1] = end;
  const uint64_t B = end >> 3;
  if (B + 5 > out_cap || (((uintptr_t)d_out) & 3)) return NICE_E_CAPACITY;
  NICE_HIP(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  int rc = ctx->dev_len.grow(meta.size() * 8 + 64);
  if (rc) return rc;
  unsigned long long* dmeta = (unsigned long long*)ctx->dev_len.ptr;
  NICE_HIP(hipMemcpyAsync(dmeta, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, st));
  // header words (the last one zero padded), then the bands, then the tail
  NICE_HIP(hipMemcpyAsync(d_out, ctx->band_hdr.ptr, ((seed + 31) >> 5) * 4, hipMemcpyDeviceToDevice, st));
  // words past the header up to the end are written by the bands (first/last OR-ed)
  const uint64_t hdr_words = (seed + 31) >> 5, end_words = (end + 31) >> 5;
  if (end_words > hdr_words)
    NICE_HIP(hipMemsetAsync(d_out + hdr_words * 4, 0, (end_words - hdr_words) * 4, st));
  {
    uint64_t most = 0;
    for (uint32_t r = 0; r < n_bands; ++r) most = std::max<uint64_t>(most, meta[n_bands + r + 1] - meta[n_bands + r]);
    hipLaunchKernelGGL(enc_band_merge, dim3((uint32_t)((most + 4095) / 4096), n_bands), dim3(256), 0, st,
                       (uint32_t*)d_out, d_words, dmeta, dmeta + n_bands, n_bands);
    hipLaunchKernelGGL(enc_band_fix, dim3(1), dim3(64), 0, st, d_out, d_words, dmeta + 2 * n_bands + 3,
                       dmeta + n_bands, n_bands, dmeta + 3 * n_bands + 3);
  }
  EncArgs a = ctx->bs.a;
  a.out = d_out;
  a.out_stride = 0;
  a.n_frames = 1;
  a.data_end = dmeta + 2 * n_bands + 1;
  a.out_len = dmeta + 2 * n_bands + 2;
  hipLaunchKernelGGL(enc_tail, dim3(1), dim3(64), 0, st, a);
  unsigned long long bad = 0;
  NICE_HIP(hipMemcpyAsync(&bad, dmeta + 3 * n_bands + 3, 8, hipMemcpyDeviceToHost, st));
  NICE_HIP(hipStreamSynchronize(st));   // `meta` lives on this stack frame
  if (bad) {   // a band was packed with a band_bits other than its own: its bits are missing
    *out_len = 0;
    return NICE_E_ARG;
  }
  *out_len = B + 5;
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}

int nice_ctx_set_timing(nice_ctx* ctx, int on) {
  if (!ctx) return NICE_E_ARG;
  ctx->timer.on = on != 0;
  ctx->timer.marks.clear();
  ctx->timer.used = 0;
  return NICE_OK;
}

int nice_ctx_read_timing(nice_ctx* ctx, double* ms, uint32_t* count) {
  if (!ctx || !ms) return NICE_E_ARG;
  for (int i = 0; i < NICE_PHASES; ++i) {
    ms[i] = 0.0;
    if (count) count[i] = 0;
  }
  for (auto& m : ctx->timer.marks) {
    if (hipEventSynchronize(m.b) != hipSuccess) return NICE_E_HIP;
    float t = 0.f;
    if (hipEventElapsedTime(&t, m.a, m.b) != hipSuccess) return NICE_E_HIP;
    ms[m.phase] += t;
    if (count) count[m.phase] += 1;
  }
  ctx->timer.marks.clear();
  ctx->timer.used = 0;
  return NICE_OK;
}

// Test hook: the device heap replay (enc_tables) on n_vec host count vectors
// of n <= MAX_ALPHABET symbols; aob receives n_vec * n code lengths.
int nice_test_code_lengths(const uint32_t* counts, int n_vec, int n, uint8_t* aob) {
  if (n_vec <= 0 || n <= 0 || n > MAX_ALPHABET || !counts || !aob) return NICE_E_ARG;
  const size_t cb = (size_t)n_vec * n * 4, ab = (size_t)n_vec * n;
  void *dc = nullptr, *da = nullptr;
  NICE_HIP(hipMalloc(&dc, cb));
  if (hipMalloc(&da, ab) != hipSuccess) { (void)hipFree(dc); return NICE_E_HIP; }
  int rc = NICE_OK;
  if (hipMemcpy(dc, counts, cb, hipMemcpyHostToDevice) != hipSuccess) rc = NICE_E_HIP;
  if (!rc) {
    hipLaunchKernelGGL(enc_code_lengths_test, dim3(n_vec), dim3(64), 0, 0, (const uint32_t*)dc, n, (uint8_t*)da);
    if (hipGetLastError() != hipSuccess || hipMemcpy(aob, da, ab, hipMemcpyDeviceToHost) != hipSuccess)
      rc = NICE_E_HIP;
  }
  (void)hipFree(dc);
  (void)hipFree(da);
  return rc;
}

// Test hooks for dec_rows_split's fallback (tests/test_split.py).
// nice_test_occupy: `blocks` blocks of `lds_bytes` dynamic LDS each (one per
// CU at > 80 KB) on `stream`; blocks < short_blocks spin short_us, the others
// long_us (bounded busy waits on the real-time counter).
__global__ void nice_occupy_kernel(uint32_t short_blocks, unsigned long long short_ticks,
                                   unsigned long long long_ticks) {
  extern __shared__ uint32_t occ_lds[];
  if (threadIdx.x == 0) occ_lds[0] = blockIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long d = blockIdx.x < short_blocks ? short_ticks : long_ticks;
  while (__builtin_amdgcn_s_memrealtime() - t0 < d) __builtin_amdgcn_s_sleep(127);
}
int nice_test_occupy(void* stream, uint32_t blocks, uint32_t short_blocks, uint32_t short_us, uint32_t long_us,
                     uint32_t lds_bytes) {
  if (blocks == 0 || lds_bytes > 160 * 1024 || long_us > 5000000 || short_us > 5000000) return NICE_E_ARG;
  NICE_HIP(hipFuncSetAttribute((const void*)nice_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds_bytes));
  hipLaunchKernelGGL(nice_occupy_kernel, dim3(blocks), dim3(64), lds_bytes, (hipStream_t)stream, short_blocks,
                     (unsigned long long)short_us * 100ull, (unsigned long long)long_us * 100ull);
  NICE_HIP(hipGetLastError());
  return NICE_OK;
}
// The classify kernel the context's last encode (or band classify) used:
// 0 window, 1 tiny, 2 ring, 3 ring2 (32K ring), 4 strip, 5 pair (two tiles per iteration),
// 6 twin (per-tile row windows), 7 slide (per-lane sliding windows).
int nice_test_last_classify(nice_ctx* ctx) { return ctx ? ctx->last_classify : -1; }

// Test hooks of one context (tests only; nothing reads the environment for them):
// split_absent != 0 makes the last strip of every split decode return at entry
// (a strip that never became resident); pack_cap_bpp in [1, NICE_PACK_CAP_BPP]
// lowers enc_pack's LDS group buffer to that many bits per pixel (0: default).
int nice_test_set_hooks(nice_ctx* ctx, uint32_t split_absent, uint32_t pack_cap_bpp) {
  if (!ctx || pack_cap_bpp > NICE_PACK_CAP_BPP) return NICE_E_ARG;
  ctx->test_split_absent = split_absent ? 1u : 0u;
  ctx->test_pack_cap_bpp = pack_cap_bpp;
  return NICE_OK;
}

// Frames of the context's last split decode that went to the fallback launch
// (synchronises the device).
int nice_test_split_redos(nice_ctx* ctx, uint32_t* split_frames, uint32_t* redos) {
  if (!ctx || !redos || !split_frames) return NICE_E_ARG;
  *redos = 0;
  *split_frames = ctx->split_frames;
  if (!ctx->split_abort || !ctx->split_frames) return NICE_OK;
  NICE_HIP(hipSetDevice(ctx->device));
  NICE_HIP(hipDeviceSynchronize());
  std::vector<uint32_t> h(ctx->split_frames);
  NICE_HIP(hipMemcpy(h.data(), ctx->split_abort, h.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t v : h) *redos += v == SPLIT_REDO ? 1u : 0u;
  return NICE_OK;
}

int nice_test_set_option(int id, int64_t value) {
  if (id < 0 || id >= NICE_OPT_COUNT) return NICE_E_ARG;
  g_opt[id].store(value < 0 ? 0 : value + 1, std::memory_order_relaxed);
  return NICE_OK;
}

void nice_test_reset_options(void) {
  for (auto& o : g_opt) o.store(0, std::memory_order_relaxed);
}

const char* nice_phase_name(int phase) {
  return (phase >= 0 && phase < NICE_PHASES) ? kPhaseNames[phase] : "";
}

int nice_decode(const uint8_t* s, size_t len, uint8_t* px_out, size_t cap, uint32_t flags,
                size_t* px_len) {
  uint32_t w, h;
  uint8_t ch;
  int rc = nice_peek_header(s, len, &w, &h, &ch);
  if (rc) return rc;
  if (ch != 3 && ch != 4) return NICE_E_UNSUPPORTED;
  if ((flags & NICE_DEC_STRICT_REFERENCE) && ch != 3) return NICE_E_UNSUPPORTED;
  const uint64_t N = (uint64_t)w * h;
  if (N > (1ull << 30)) return NICE_E_ARG;
  if (px_len) *px_len = (size_t)N * ch;
  if (cap < N * ch || (N && !px_out)) return NICE_E_CAPACITY;
  nice_ctx* ctx;
  if ((rc = default_ctx(&ctx))) return rc;
  std::lock_guard<std::mutex> g(ctx->mu);
  NICE_HIP(hipSetDevice(ctx->device));
  const size_t sbytes = align_up(len + 8, 256);
  const size_t pbytes = align_up((size_t)N * ch + 4, 256);
  if ((rc = ctx->host_out.grow(sbytes))) return rc;
  if ((rc = ctx->host_px.grow(pbytes))) return rc;
  if ((rc = ctx->dev_len.grow(256))) return rc;
  NICE_HIP(hipMemcpy(ctx->host_out.ptr, s, len, hipMemcpyHostToDevice));
  uint64_t l64 = len;
  NICE_HIP(hipMemcpy(ctx->dev_len.ptr, &l64, 8, hipMemcpyHostToDevice));
  int32_t* d_status = (int32_t*)((uint8_t*)ctx->dev_len.ptr + 64);
  rc = nice_decode_batch_dev(ctx, nullptr, (const uint8_t*)ctx->host_out.ptr, sbytes,
                             (const uint64_t*)ctx->dev_len.ptr, 1, w, h, ch,
                             (uint8_t*)ctx->host_px.ptr, pbytes, flags, d_status);
  if (rc) return rc;
  int32_t status = 0;
  NICE_HIP(hipMemcpy(&status, d_status, 4, hipMemcpyDeviceToHost));
  if (status) return status;
  if (N) NICE_HIP(hipMemcpy(px_out, ctx->host_px.ptr, (size_t)N * ch, hipMemcpyDeviceToHost));
  return NICE_OK;
}

}  // extern "C"
