/* nice.h -- C ABI of the MI355X-native NICE2 codec (libnice_hip.so).
 *
 * Drop-in boundary for the reference's codec entry points:
 *   code::encode  /root/reference/src/code.rs:59-64
 *       pub fn encode<W: io::Write>(input_bytes: &[u8], image_header: Image,
 *                                   channels_out: u8, output_writer: &mut W)
 *   code::decode  /root/reference/src/code.rs:464-468
 *       pub fn decode<R: io::Read>(image_reader: &mut R, channels_out: u8,
 *                                  output_vec: &mut Vec<u8>) -> io::Result<Image>
 *   image::Image::new  /root/reference/src/image.rs:22-43 (width, height, channels)
 *
 * Plain pointers and sizes only.  Every function returns a status code (0 = ok,
 * negative = error) and never aborts, where the reference panics/aborts
 * (Cargo.toml:16 panic = "abort").  Buffers are caller-owned.  Functions taking a
 * nice_ctx are thread-safe per context; the context-free functions use an
 * internal per-device context guarded by a mutex.
 *
 * Frame size cap: every encode/decode entry point (and the band API) refuses a
 * frame of more than 2^30 pixels (w * h > 1073741824, e.g. 32768 x 32768) with
 * NICE_E_ARG.  code::encode has no such limit (code.rs:59-64, 87); the cap keeps
 * pixel indices and Huffman counts 32-bit on the device: a stream's symbol
 * total is at most 3 per pixel (SC_RGB), i.e. < 3 * 2^30 < 2^32, which the
 * heap's 32-bit count keys and merge sums hold exactly (tests/test_tables.py
 * covers totals up to 3 * 2^30).  A 2^30-pixel RGBA frame is 4 GiB of input.
 */
#ifndef NICE_H
#define NICE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  NICE_OK = 0,
  NICE_E_ARG = -1,          /* bad argument (sizes, channels, alignment) */
  NICE_E_HIP = -2,          /* HIP runtime failure */
  NICE_E_NODEV = -3,        /* no usable gfx950 device */
  NICE_E_CAPACITY = -4,     /* output buffer too small */
  NICE_E_FORMAT = -5,       /* malformed stream: the reference would panic here */
  NICE_E_UNSUPPORTED = -6   /* stream outside the reference decoder's domain (see flags) */
};

/* nice_decode flags */
#define NICE_DEC_STRICT_REFERENCE 0x1u /* fail wherever the reference decoder would fail */
#define NICE_DEC_ALPHA_FILL_FF 0x2u    /* 4-channel output: write A = 255 */
/* Tolerant table header: repairs the length field a
 * spilled 5-bit max (> 31) corrupts in the reference writer, and decodes with
 * the <= 31-bit codes.  Streams of small or very flat images (every max > 31
 * because zero-count symbols chain deep in the Huffman merge) decode only
 * with this flag; the reference decoder cannot decode them.  Ignored with
 * NICE_DEC_STRICT_REFERENCE. */
#define NICE_DEC_TOLERANT_HEADER 0x4u

typedef struct nice_ctx nice_ctx;

/* Library / device queries. */
const char* nice_version(void);
int nice_device_count(void);

/* Upper bound of an encoded stream for a w x h image (any channels). */
size_t nice_encode_bound(uint32_t w, uint32_t h);

/* Replaces code::encode (code.rs:59-64): host pixels in, host stream out.
 * px: w*h pixels of `channels` (3 or 4) bytes; only bytes +0..+2 of each pixel
 * are coded (code.rs:197,215-217).  channels_out is written to header byte 12
 * (code.rs:84).  *out_len receives the stream length. */
int nice_encode(const uint8_t* px, size_t px_len, uint32_t w, uint32_t h, uint8_t channels,
                uint8_t channels_out, uint8_t* out, size_t out_cap, size_t* out_len);

/* Parses the 13-byte file header (code.rs:469-483). */
int nice_peek_header(const uint8_t* s, size_t len, uint32_t* w, uint32_t* h, uint8_t* ch);

/* Replaces code::decode (code.rs:464-468): host stream in, host pixels out.
 * Output pixel stride = header channels byte (3: RGB; 4: RGB + alpha byte, 255
 * with NICE_DEC_ALPHA_FILL_FF, else 0).  *px_len receives w*h*channels. */
int nice_decode(const uint8_t* s, size_t len, uint8_t* px_out, size_t cap, uint32_t flags,
                size_t* px_len);

/* ---- context API: device buffers, HIP streams (passed as void*), batches ---- */
int nice_ctx_create(int device, nice_ctx** out);
void nice_ctx_destroy(nice_ctx* ctx);
/* Pre-size scratch so later batch calls allocate nothing (graph-capturable). */
int nice_ctx_reserve(nice_ctx* ctx, uint32_t n_frames, uint32_t w, uint32_t h);

/* Encode n_frames same-shape frames resident in device memory.
 * d_px: frame f at d_px + f*frame_stride (4-byte aligned for channels == 4).
 * d_out: frame f's stream at d_out + f*out_stride (4-byte aligned, out_stride a
 * multiple of 4 and >= nice_encode_bound(w, h)); d_out_len[f] = its length.
 * Asynchronous on `stream`. */
int nice_encode_batch_dev(nice_ctx* ctx, void* stream, const uint8_t* d_px, uint64_t frame_stride,
                          uint32_t n_frames, uint32_t w, uint32_t h, uint8_t channels,
                          uint8_t channels_out, uint8_t* d_out, uint64_t out_stride,
                          uint64_t* d_out_len);

/* Decode n_frames streams resident in device memory (all w x h).
 * d_streams: stream f at d_streams + f*stream_stride, d_stream_len[f] bytes.
 * d_px: frame f written at d_px + f*px_stride with out_channels (3 or 4) bytes
 * per pixel.  d_status[f] = NICE_OK or a negative code.  Asynchronous: the
 * parse fixpoint is reached on the device; the call reads the lengths back
 * first (they size the scratch), i.e. waits for the work queued on `stream`
 * before it, never for the decode itself. */
int nice_decode_batch_dev(nice_ctx* ctx, void* stream, const uint8_t* d_streams,
                          uint64_t stream_stride, const uint64_t* d_stream_len, uint32_t n_frames,
                          uint32_t w, uint32_t h, uint8_t out_channels, uint8_t* d_px,
                          uint64_t px_stride, uint32_t flags, int32_t* d_status);
/* The same with the lengths also on the host (h_stream_len[f] == d_stream_len[f]):
 * the call only enqueues work, it never waits for the device. */
int nice_decode_batch_dev_hl(nice_ctx* ctx, void* stream, const uint8_t* d_streams,
                             uint64_t stream_stride, const uint64_t* d_stream_len,
                             const uint64_t* h_stream_len, uint32_t n_frames, uint32_t w, uint32_t h,
                             uint8_t out_channels, uint8_t* d_px, uint64_t px_stride, uint32_t flags,
                             int32_t* d_status);

/* ---- one image sharded over ranks (config 4) ----
 * The image's raster is cut into bands of whole encoder tiles (1024 pixels in
 * raster order); rank r encodes tiles [tile_lo, tile_hi).  The caller runs the
 * exchange steps between the calls (bench/tests use RCCL via torch.distributed):
 *   1. nice_band_classify   band records + d_edges = {first, last} coded pixel
 *                           (0xFFFFFFFF: none)
 *   2. all-gather edges     band_next = first coded pixel of the later bands (w*h: none)
 *      nice_band_runs       the band's symbol histogram (858 x u32) into d_hist
 *   3. all-reduce (sum)     nice_band_tables: identical code tables on every rank;
 *                           returns the band's data bits and the data start bit
 *   4. all-gather bits      band_bit0 = data start + bits of the earlier bands
 *      nice_band_pack       nice_band_words() words: the band's bits at their
 *                           stream position (first/last word partial)
 *   5. gather words         nice_band_assemble (one rank): header + bands + tail
 * The result equals nice_encode of the whole image byte for byte, codes longer
 * than 25 bits included.  nice_band_words() counts the band's stream words plus
 * a two-word trailer (every band has one, a band of 0 bits only the trailer):
 * a code longer than 25 bits that starts in the byte holding band_bit0
 * rewrites (reference writer wrap, bitwriter.rs:55-73) bits of the previous
 * band; it is recorded there and applied by nice_band_assemble.
 * Device-resident variants (no host synchronisation between the steps; the
 * exchanges can stay on device, e.g. RCCL collectives on the same stream):
 *   nice_band_runs_dev      band_next read from device memory (u32)
 *   nice_band_tables_dev    d_info[0] = the band's data bits, d_info[1] = the
 *                           data start bit (device u64 x 2, written in stream
 *                           order; the context keeps its own copy, so d_info may
 *                           be freed or reused once the call's work has run)
 *   nice_band_pack_bits     the band's bits passed in (from the gathered d_info);
 *                           band_bits must equal d_info[0] exactly (it sizes the
 *                           band's words): after nice_band_tables_dev the device
 *                           compares them and, on a mismatch, writes no band bits
 *                           (d_words never overrun) and marks the band's trailer;
 *                           nice_band_assemble then returns NICE_E_ARG
 * nice_band_assemble after nice_band_tables_dev takes band_bit0[0] as the data
 * start.
 * d_px holds pixels [px0, px0 + px_count) (global raster index), which must
 * cover the band and the 3 rows + 3 pixels before it. */
int nice_band_classify(nice_ctx* ctx, void* stream, const uint8_t* d_px, uint64_t px0, uint64_t px_count,
                       uint32_t w, uint32_t h, uint8_t channels, uint8_t channels_out, uint32_t tile_lo,
                       uint32_t tile_hi, uint32_t* d_edges);
int nice_band_runs(nice_ctx* ctx, void* stream, uint32_t band_next, uint32_t* d_hist);
int nice_band_tables(nice_ctx* ctx, void* stream, const uint32_t* d_hist_total, uint64_t* band_bits,
                     uint64_t* seed_bit);
int nice_band_runs_dev(nice_ctx* ctx, void* stream, const uint32_t* d_band_next, uint32_t* d_hist);
int nice_band_tables_dev(nice_ctx* ctx, void* stream, const uint32_t* d_hist_total, uint64_t* d_info);
uint64_t nice_band_words(uint64_t band_bit0, uint64_t band_bits);
int nice_band_pack(nice_ctx* ctx, void* stream, uint64_t band_bit0, uint32_t* d_words, uint64_t words_cap);
int nice_band_pack_bits(nice_ctx* ctx, void* stream, uint64_t band_bit0, uint64_t band_bits, uint32_t* d_words,
                        uint64_t words_cap);
int nice_band_assemble(nice_ctx* ctx, void* stream, const uint32_t* d_words, const uint64_t* band_bit0,
                       const uint64_t* band_bits, uint32_t n_bands, uint8_t* d_out, uint64_t out_cap,
                       uint64_t* out_len);
/* Encoder tile size (pixels) used by the band API. */
uint32_t nice_tile_pixels(void);

/* ---- streamed host pipeline (BASELINE config 5) ----
 * Frames in host memory flow through `depth` slots of `batch` frames; each slot
 * has its own HIP stream, scratch and device buffers, so one slot's H2D copy,
 * another's kernels and a third's D2H copy overlap.  Replaces calling
 * code::encode / code::decode (code.rs:59-64, 464-468) once per image from host
 * memory (main.rs:28-103).  Host buffers may be pinned (copies asynchronous) or
 * pageable.  Frames are w x h with `channels` bytes per pixel (fixed per pipe). */
typedef struct nice_pipe nice_pipe;
int nice_pipe_create(int device, uint32_t w, uint32_t h, uint8_t channels, uint32_t batch, uint32_t depth,
                     nice_pipe** out);
void nice_pipe_destroy(nice_pipe* p);
/* Bytes per stream slot on the device (>= nice_encode_bound(w, h)). */
uint64_t nice_pipe_stream_stride(const nice_pipe* p);
/* px[f]: frame f (w*h*channels bytes).  out[f]: stream f (out_cap bytes
 * available), out_len[f] its length.  Blocks until every stream is on the host. */
int nice_pipe_encode(nice_pipe* p, const uint8_t* const* px, uint32_t n_frames, uint8_t channels_out,
                     uint8_t* const* out, uint64_t out_cap, uint64_t* out_len);
/* streams[f], stream_len[f] -> px[f] (w*h*out_channels bytes, out_channels <=
 * the pipe's channels); status[f] per frame (flags as nice_decode).  Blocks.
 * px[f] is defined only where status[f] == NICE_OK. */
int nice_pipe_decode(nice_pipe* p, const uint8_t* const* streams, const uint64_t* stream_len, uint32_t n_frames,
                     uint8_t out_channels, uint8_t* const* px, uint32_t flags, int32_t* status);
/* Per-frame checksums computed on the device from what the pipe copies to the
 * host (end-to-end checks of streamed runs whose host buffers are reused):
 * while set, nice_pipe_encode writes enc_sums[f] = nice_checksum64 of stream f
 * and nice_pipe_decode dec_sums[f] = that of frame f's pixels (either pointer
 * may be null; each must hold n_frames entries of the calls that follow).
 * nice_checksum64 of n bytes: zero-pad to whole little-endian u32 words w_i,
 * A = sum w_i, B = sum (i + 1) w_i (mod 2^64), checksum = A + 0x9E3779B97F4A7C15 B
 * (mod 2^64). */
int nice_pipe_set_checksums(nice_pipe* p, uint64_t* enc_sums, uint64_t* dec_sums);

/* ---- command-line front end helper (host only) ----
 * Reverses the PNG scanline filters (types 0-4) of h rows of w pixels of bpp
 * bytes: raw = h x (1 filter byte + w*bpp bytes), out = h x w*bpp bytes.  The
 * reference CLI (main.rs:28-133) reads and writes PNG with the png crate. */
int nice_png_unfilter(const uint8_t* raw, uint32_t w, uint32_t h, uint32_t bpp, uint8_t* out);

/* ---- 5x5 sub-block traversal ----
 * d_pos[i] = Image::new(w, h, _).calc_pos_from(index0 + i) for i < count
 * (image.rs:45-102), computed on `device`, asynchronous on `stream`.  The
 * reference's map exactly: not a permutation when w % 5 and h % 5 are both
 * nonzero, and positions >= w*h for some shapes (w = 7, ...).  w == 0 is
 * NICE_E_ARG (the reference divides by zero).  The codec does not use it. */
int nice_subblock_positions_dev(int device, void* stream, uint32_t w, uint32_t h, uint64_t index0,
                                uint64_t count, uint64_t* d_pos);

/* ---- per-kernel timing (HIP events on the call's stream), for benchmarks ---- */
enum {
  NICE_PH_ENC_CLASSIFY = 0, NICE_PH_ENC_TAILRUNS, NICE_PH_ENC_TABLES, NICE_PH_ENC_HEADER,
  NICE_PH_ENC_TILEBITS, NICE_PH_ENC_TILESCAN, NICE_PH_ENC_PACK, NICE_PH_ENC_TAIL, NICE_PH_ENC_LONG,
  NICE_PH_DEC_TABLES, NICE_PH_DEC_SYNC, NICE_PH_DEC_SCAN, NICE_PH_DEC_EMIT, NICE_PH_DEC_RECON,
  NICE_PH_DEC_PLACE, NICE_PH_DEC_RESYNC, NICE_PHASES   /* RESYNC: sync iterations after the first */
};
int nice_ctx_set_timing(nice_ctx* ctx, int on);
/* Sums (ms) and launch counts per phase since the last read; synchronises. */
int nice_ctx_read_timing(nice_ctx* ctx, double* ms, uint32_t* count);
const char* nice_phase_name(int phase);

#ifdef __cplusplus
}
#endif
#endif /* NICE_H */
