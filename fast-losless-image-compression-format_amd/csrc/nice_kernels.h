// nice_kernels.h -- kernel argument blocks and launch-visible constants shared by
// the HIP kernels and the host runtime (nice_capi.hip).  Device pointers only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nice {

constexpr int ENC_TILE = 1024;          // pixels per encoder tile (raster-contiguous)
// frame emits a code longer than FAST_MAX_CODE_BITS: packed by enc_pack_long
// (the reference writer's u32 cache wraps for such codes, bitwriter.rs:63-64)
constexpr uint32_t FLAG_LONG = 1u;
// band pack: the caller's band_bits differ from the band's real bit count
// (nice_band_pack_bits after nice_band_tables_dev): the pack kernels skip the
// band instead of writing past the caller's words
constexpr uint32_t FLAG_BAD = 2u;

struct EncArgs {
  // input: n_frames frames of W*H pixels, C bytes per pixel, frame_stride bytes apart
  const uint8_t* px;
  uint64_t frame_stride;
  uint32_t n_frames, W, H, C;
  uint8_t channels_out;
  uint32_t tiles_per_frame, tiles_per_block;
  // output: frame f at out + f*out_stride, byte length in out_len[f]
  uint8_t* out;
  uint64_t out_stride;
  unsigned long long* out_len;
  // scratch (see nice_capi.hip for sizes)
  uint32_t* hist;            // n_frames * 858
  uint32_t* tile_first;      // n_frames * T
  uint32_t* tile_last;       // n_frames * T
  uint32_t* tile_next;       // n_frames * T
  uint32_t* cmask;           // n_frames * T * 32: coded-pixel flags per tile (enc_classify_pair_m); null in band mode
  uint32_t cmask_std;        // 1: cmask holds every tile's flags in the standard order by enc_pack time
  uint32_t* tbl;             // n_frames * 858: (code << 5) | len for len <= 25
  uint32_t* tbl_code;        // n_frames * 858: code as u32 (serial path)
  uint8_t* tbl_len8;         // n_frames * 858: u8 length
  uint8_t* stream_max;       // n_frames * 10
  uint32_t* frame_flags;     // n_frames
  unsigned long long* seed_bit;   // n_frames: absolute bit where symbol data starts
  uint32_t* seed_suf;        // n_frames: last 32 bits before seed_bit
  unsigned long long* hdr_bytes;  // n_frames (serial header path)
  uint32_t* hdr_cache;       // n_frames
  uint8_t* hdr_bitoff;       // n_frames
  uint32_t* recs;            // n_frames * rec_stride per-pixel symbol records
  uint64_t rec_stride;       // W*H rounded up to 4
  uint32_t* tile_bits;       // n_frames * T: data bits per tile (long path); pack_mode 0: the
                             // tile's bits in the word holding its first bit (enc_edges)
  unsigned long long* tile_off;   // n_frames * T: absolute bit offset of each tile
  uint8_t* packtab;          // n_frames * sizeof(PackTab): the packer's code tables (nice_rec.hpp)
  uint32_t* pack_ctr;        // n_frames: enc_pack's per-frame tile counters (zeroed per launch)
  uint32_t pack_slots;       // enc_pack: frames worked at once (blocks per frame = grid / slots)
  unsigned long long* status;   // n_frames * (tile_hi - tile_lo): look-back status words (zeroed per launch)
  uint32_t pack_mode;        // 0: tile offsets by look-back (frames); 1: from enc_tilescan (bands)
  uint32_t long_only;        // 1: enc_tilebits / enc_tilescan serve FLAG_LONG frames only
  unsigned long long* data_end;   // n_frames: bit position after the last data bit
  // Band mode (one image sharded over ranks): only tiles
  // [tile_lo, tile_hi) of each frame are processed; pixel memory is valid for
  // global indices [px_lo, px_hi); runs after the last coded pixel of the band
  // end at band_next; the band's data starts at bit band_bit0 and shared
  // output words above zero_floor are zeroed for OR-merging.  Frames: tile
  // range [0, T), pixels [0, N), band == 0.
  uint32_t tile_lo, tile_hi;
  int64_t px_lo, px_hi;
  uint32_t band;
  unsigned long long band_next, band_bit0;
  const uint32_t* band_next_dev;   // non-null: band_next read from device memory (nice_band_runs_dev)
  uint32_t* band_fix;        // band pack: {flag | offset << 8 | length, code} of a wrapped write before band_bit0
  // the per-frame tile scans (enc_tailruns, enc_tilescan) run as `groups`
  // blocks of ENC_GROUP_TILES tiles per frame; gacc holds each group's
  // aggregate (n_frames * groups: min first coded pixel, then bit total)
  uint32_t groups;
  unsigned long long* gacc;
  // enc_pack: bits a group may hold in its LDS buffer (PACK_SUB * ENC_TILE * 32;
  // the test hook nice_test_set_hooks lowers it to b bits per pixel, so tests
  // reach the over-cap path on ordinary frames)
  uint32_t pack_cap_bits;
  // groups over that buffer, for enc_pack_over: {frame * groups + group, bits}
  uint32_t* over_count;      // zeroed per launch
  uint2* over_list;          // n_frames * ceil((tile_hi - tile_lo) / PACK_SUB)
};
constexpr uint32_t ENC_GROUP_TILES = 8192;

__global__ void enc_classify(EncArgs a);        // W >= 3
__global__ void enc_classify_tiny(EncArgs a);   // W < 3
__global__ void enc_classify_ring(EncArgs a);    // RGBA
__global__ void enc_classify_ring3(EncArgs a);   // RGB, 4-byte aligned frames
__global__ void enc_classify_strip_m(EncArgs a);
__global__ void enc_classify_strip(EncArgs a);   // RGBA, W % 1024 == 0, W > CLS_RING_MAX_W (tiles_per_block = rows per block)
constexpr uint32_t STRIP_W_HOST = 2048;          // == STRIP_W (nice_encode.hip)
// the 16K-pixel ring holds 3W + 3 pixels of references plus two tiles (the one
// being classified and the next one being staged): 3W + 3 + 2048 <= 16384
constexpr uint32_t CLS_RING_MAX_W = 4777;
// enc_classify_ring2 / ring2_3: the same with a 32K-pixel ring: 3W + 3 + 2048 <= 32768
__global__ void enc_classify_ring2(EncArgs a);
__global__ void enc_classify_ring2_3(EncArgs a);
constexpr uint32_t CLS_RING2_MAX_W = 10239;
// enc_classify_pair: RGBA, two tiles per iteration, 16K ring: 3W + 3 + 4096 <= 16384
__global__ void enc_classify_pair(EncArgs a);
__global__ void enc_classify_pair_m(EncArgs a);
__global__ void enc_classify_ring_m(EncArgs a);
__global__ void enc_classify_ring3_m(EncArgs a);
__global__ void enc_classify_ring2_m(EncArgs a);
__global__ void enc_classify_ring2_3_m(EncArgs a);
__global__ void enc_rundigits(EncArgs a, int il);   // il: enc_classify_slide's ballot-order flags
// RGBA frames, 3 <= W <= CLS_PAIR_MAX_W, 16-byte aligned pixels: per-lane sliding
// windows, one kernel per W mod 4
__global__ void enc_classify_slide0(EncArgs a);
__global__ void enc_classify_slide1(EncArgs a);
__global__ void enc_classify_slide2(EncArgs a);
__global__ void enc_classify_slide3(EncArgs a);
// per-tile row windows (any W > CLS_RING2_MAX_W the strip kernel does not take; RGBA and RGB)
__global__ void enc_classify_twin(EncArgs a);
__global__ void enc_classify_twin_m(EncArgs a);
__global__ void enc_classify_twin3(EncArgs a);
__global__ void enc_classify_twin3_m(EncArgs a);
constexpr uint32_t CLS_PAIR_MAX_W = 4095;
// dec_sync / dec_emit block size: one LUT copy per 8 waves (LDS sets occupancy)
#ifndef NICE_PARSE_THREADS
#define NICE_PARSE_THREADS 512
#endif
constexpr uint32_t DEC_PARSE_THREADS = NICE_PARSE_THREADS;
constexpr uint32_t CLS_THREADS_HOST = 512;   // == CLS_THREADS (nice_encode.hip)   // enc_classify_ring: 3W + 3 + 2 tiles fit its 16K-pixel ring
__global__ void enc_tailruns(EncArgs a);
__global__ void enc_tables(EncArgs a);
__global__ void enc_code_lengths_test(const uint32_t* counts, int n, uint8_t* aob);
__global__ void enc_header(EncArgs a);
__global__ void enc_tilebits(EncArgs a);
__global__ void enc_tilescan(EncArgs a);
// group aggregates for the tile scans: what 0 = min of tile_first, 1 = sum of tile_bits
__global__ void enc_group_reduce(EncArgs a, int what);
__global__ void enc_packtab(EncArgs a);
__global__ void enc_pack(EncArgs a);
__global__ void enc_pack_over(EncArgs a);
constexpr uint32_t PACK_OVER_BLOCKS = 64;   // enc_pack_over's grid (blocks loop over the listed groups)
__global__ void enc_edges(EncArgs a);
#ifndef NICE_PACK_BPC
#define NICE_PACK_BPC 4
#endif
#ifndef NICE_PACK_CAP_BPP
#define NICE_PACK_CAP_BPP 32     // enc_pack's LDS group buffer: bits per pixel
#endif
constexpr uint32_t PACK_BLOCKS_PER_CU = NICE_PACK_BPC;   // enc_pack: 256 threads, ~35 KB LDS
constexpr int PACK_SUB = 4;                  // tiles per enc_pack work item (group)
__global__ void enc_tail(EncArgs a);
__global__ void enc_band_edges(EncArgs a, uint32_t* edges);
__global__ void enc_band_sum(EncArgs a, const uint32_t* bhist, unsigned long long* info);
__global__ void enc_band_check(EncArgs a, const unsigned long long* info, unsigned long long band_bits);
// band trailer word 0: a deferred wrapped write {BAND_FIX_WRITE | offset << 8 |
// length} (code in word 1), or BAND_FIX_BAD: the band was packed with a
// band_bits other than its own (nothing written)
constexpr uint32_t BAND_FIX_WRITE = 0x80000000u, BAND_FIX_BAD = 0x40000000u;
__global__ void enc_band_fix(uint8_t* out, const uint32_t* words, const unsigned long long* band_bit0,
                             const unsigned long long* band_off, uint32_t R, unsigned long long* bad);
__global__ void enc_band_merge(uint32_t* out32, const uint32_t* words, const unsigned long long* band_w0,
                               const unsigned long long* band_off, uint32_t R);
// long-code frames (FLAG_LONG): phase 0 packs every code whose write does not
// wrap the reference cache (pending + length <= 32); phase 1 applies the
// wrapped writes to their 32-bit windows once phase 0's bits are final
__global__ void enc_pack_long(EncArgs a, int phase);

}  // namespace nice

namespace nice {

// sync checkpoint spacing inside a slice (DecArgs::ck_bits, chosen per call:
// at most one emit sub-slice; 128: +30 % dec_sync -- scattered stores)
constexpr uint32_t DEC_CK_BITS = 1024;      // slices of 8K bits and more (the bench's 512 x 4K)
constexpr uint32_t DEC_CK_BITS_SMALL = 512;  // shorter slices (small batches)
constexpr uint32_t DEC_MIN_CHUNK_BITS = 1024;   // speculative-parse slice: a power of two
constexpr uint32_t DEC_MAX_CHUNK_BITS = 16384;  // chosen per call (nice_capi.hip)
constexpr uint32_t DEC_PLACE_WAVES = 4;          // dec_place: one wave per slice (2 or 8 per block: slower; several slices per wave, their bookkeeping loads batched: slower too)
constexpr uint32_t DEC_EMIT_BITS = 1024;        // record-emission sub-slice (<= the slice)
constexpr int DEC_MAX_SEGS = 64;            // one lane per row segment

struct DecArgs {
  const uint8_t* streams;
  uint64_t stream_stride;
  const unsigned long long* stream_len;
  uint32_t n_frames, W, H;
  uint32_t out_channels, flags;
  uint8_t* px_out;
  uint64_t px_stride;
  int32_t* status;
  // scratch
  void* tables;                       // n_frames DecTables
  unsigned long long* data_start;     // n_frames
  uint32_t max_chunks, chunk_blocks;  // per frame
  unsigned long long* entry;          // n_frames * max_chunks packed entry states
  unsigned long long* last;           // n_frames * max_chunks entry of the last parse
  unsigned long long* ck;             // n_frames * n_ck * max_chunks checkpoints
  uint32_t chunk_bits, n_ck;          // slice size; checkpoints per slice (chunk_bits / ck_bits - 1)
  uint32_t ck_bits;                   // checkpoint spacing (DEC_CK_BITS or DEC_CK_BITS_SMALL)
  uint32_t emit_blocks;               // per frame: ceil(max_chunks * chunk_bits / DEC_EMIT_BITS / 256)
  unsigned long long* chunk_px;       // n_frames * max_chunks
  unsigned long long* chunk_start;    // n_frames * max_chunks
  uint32_t* recs;                     // n_frames * rec_stride per-pixel records
  uint64_t rec_stride;                // W * H rounded up to 4 (16-byte aligned frames)
  uint32_t seg, nseg;
  uint32_t rows_in_lds;               // 1: row ring in LDS, 0: in rowbuf
  uint32_t rec_tag;                   // 1..15: records of this call carry it in bits 28..31
  uint32_t parse_slow;                // 1: dec_sync ignores DecTables::fast (tests)
  uint32_t* rowbuf;                   // n_frames * R * W (when not in LDS)
  unsigned long long* stats;          // optional diagnostics (NICE_DEC_STATS=1), else null
  // pixel events of the first sync pass, reused past the point where the final
  // parse meets it (dec_place); null: not kept (dec_emit parses every slice)
  uint32_t* ev;                       // n_frames * max_chunks * ev_cap events
  uint32_t ev_cap;                    // events per slice (multiple of 4)
  uint32_t* ev_ck;                    // n_frames * n_ck * max_chunks: events before checkpoint k (first pass)
  uint32_t* ev_n;                     // n_frames * max_chunks: events of the first pass, EV_OVERFLOW
  uint32_t* agree;                    // n_frames * max_chunks: final parse == first pass from checkpoint agree-1 (0: entry)
  uint32_t* head_items;               // n_frames * max_chunks * (chunk_bits / DEC_EMIT_BITS): dec_emit's sub-slices
  uint32_t* head_count;               // n_frames: sub-slices listed
  // dec_rows_split (wide frames, several workgroups per frame): strips per
  // frame, the units' published first / last pixels (n_frames * H * strips *
  // 8 granules, zeroed per call) and a per-frame abort flag
  uint32_t strips;
  unsigned long long* hand;
  uint32_t* hand_abort;
  uint32_t split_f0;                  // dec_rows_split: first frame of this launch (frames in chunks)
  // the fallback launch after dec_rows_split (dec_rows_wide / dec_reconstruct):
  // only frames whose strips could not all be resident (hand_abort ==
  // SPLIT_REDO: a wait timed out) are reconstructed, the others return at once
  uint32_t redo;
  // tests (nice_test_set_hooks): the last strip of every frame returns at
  // once, as a block that never became resident would, so the others time out
  uint32_t test_absent_strip;
  // dec_rows_flow: row groups per block (rows in flight), ring rows (4 or 8)
  uint32_t flow_k, flow_ring;
  // dec_scan: per-frame flags of the last sync iteration (an entry still moved:
  // the frame fails with NICE_E_HIP), or null
  const uint32_t* unsettled;
};
constexpr uint32_t SPLIT_ABORT_ERR = 1u, SPLIT_REDO = 2u;
// first-pass event of a run digit: EV_RUN | pixels (saturated); a coded
// pixel's record before its tag: EV_L2 (LUMA2: needs the row above) and EV_BAD
// in the record's tag bits (make_event_rec, rec_bad_at)
constexpr uint32_t EV_RUN = 1u << 31, EV_BAD = 1u << 9, EV_L2 = 1u << 8;
constexpr uint32_t EV_OVERFLOW = 0xFFFFFFFFu, AGREE_NONE = 0xFFFFu;

__global__ void dec_tables(DecArgs a);
__global__ void dec_init_entries(DecArgs a);
__global__ void dec_sync(DecArgs a, uint32_t* changed, const uint32_t* prev, uint32_t* fchanged);
__global__ void dec_sync_settle(DecArgs a, const uint32_t* last_changed, const uint32_t* fchanged, uint32_t* settled);
__global__ void dec_scan(DecArgs a);
__global__ void dec_strict_refill(DecArgs a);   // NICE_DEC_STRICT_REFERENCE only
__global__ void dec_emit(DecArgs a);
__global__ void dec_place(DecArgs a);
__global__ void dec_heads(DecArgs a);
__global__ void dec_reconstruct(DecArgs a);
__global__ void dec_rows(DecArgs a);
__global__ void dec_rows_wide(DecArgs a);
__global__ void dec_rows8(DecArgs a);
__global__ void dec_rows_flow(DecArgs a);   // small batches: rows in flight, LDS stamps (W <= 4096)
constexpr uint32_t FLOW_THREADS_HOST = 512, FLOW_CTL_BYTES_HOST = 2752;   // == FLOW_THREADS, sizeof(FlowCtl)
constexpr uint32_t FLOW_MAX_W_HOST = 8192;   // 8 waves of 16-pixel segments per row (FLOW_MAXW)
__global__ void dec_rows_split(DecArgs a);
constexpr uint32_t SPLIT_THREADS_HOST = 256;   // == SPLIT_THREADS (nice_decode.hip): lanes per strip
constexpr uint32_t SPLIT_GRAN_HOST = 8;        // == SPLIT_GRAN

// Inclusive wave64 prefix sum by DPP: shifts 1, 2, 4, 8 inside each row of 16
// lanes, then row 15 -> rows 1 and 3, row 31 -> rows 2 and 3.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return v;
}

// OR over each aligned group of 8 lanes (quad xor 1, xor 2, then the other
// quad of the group by row_half_mirror).
__device__ __forceinline__ uint32_t wave_or8(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
  return v;
}

}  // namespace nice
