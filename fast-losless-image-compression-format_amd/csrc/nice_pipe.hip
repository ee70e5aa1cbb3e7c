// nice_pipe.hip -- streamed host<->device pipeline (SURVEY.md §8f rank 1,
// BASELINE config 5: frames streamed from host memory, H2D / compute / D2H
// overlapped on HIP streams).
//
// Decode never blocks the host on a chunk: the decoder reaches its parse
// fixpoint on the device (decode_batch_impl: queued sync iterations, then
// dec_sync_settle).  (A blocking fixpoint check inside every chunk held back
// the next chunk's H2D copies behind the previous chunk's first kernels.)
//
// The reference codes one image per call from host memory (main.rs:28-75 reads
// a PNG, code.rs:59-64 encodes it, main.rs:77-103 decodes it back).  Here a
// caller hands over many host frames at once; they flow through `depth` slots
// of `batch` frames.  Each slot owns a HIP stream, a context (scratch arena)
// and device buffers, so slot k's H2D copy, slot k-1's kernels and slot k-2's
// D2H copy run concurrently on the copy engines and the CUs.
//
// Encode: stream lengths are only known after the kernels, so a slot's stream
// bytes are copied back one chunk later: lengths land in pinned host memory with
// the chunk, and the exact-size D2H copies of chunk c-1 are enqueued after
// chunk c has been submitted.  Decode: stream sizes are known up front, pixel
// sizes are fixed; everything is enqueued at once per chunk.
//
// Host buffers may be pinned (hipHostMalloc / torch pin_memory: copies are
// asynchronous) or pageable (HIP stages them; correct, with less overlap).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/nice.h"
#include "nice_internal.h"

#define PIPE_HIP(x)                          \
  do {                                       \
    if ((x) != hipSuccess) return NICE_E_HIP; \
  } while (0)

namespace {

struct Slot {
  nice_ctx* ctx = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;     // all work of the slot's current chunk (incl. D2H)
  hipEvent_t lens = nullptr;     // encode: lengths copied to host
  uint8_t* d_px = nullptr;       // batch x frame bytes
  uint8_t* d_str = nullptr;      // batch x stream stride
  uint64_t* d_len = nullptr;     // batch
  int32_t* d_status = nullptr;   // batch
  uint64_t* h_len = nullptr;     // pinned, batch
  int32_t* h_status = nullptr;   // pinned, batch
  unsigned long long* d_sum = nullptr;   // batch x {A, B} (nice_pipe_set_checksums)
  unsigned long long* h_sum = nullptr;   // pinned, batch x {A, B}
  int64_t chunk = -1;            // chunk in flight (-1: none)
  uint32_t n = 0;                // frames of that chunk
};

}  // namespace

struct nice_pipe {
  int device = 0;
  uint32_t w = 0, h = 0, ch = 0, batch = 0, depth = 0;
  uint64_t frame_bytes = 0, str_stride = 0;
  std::vector<Slot> slots;
  uint64_t* enc_sums = nullptr;   // caller's arrays (nice_pipe_set_checksums)
  uint64_t* dec_sums = nullptr;
};

namespace {
// nice_checksum64's two sums of n frames' bytes (frame i at base + i * stride,
// len[i] bytes or `fixed` when len is null): one 256-thread block per frame
// slice of 64 K words, 64-bit atomics into sums[2i], sums[2i + 1].
constexpr uint32_t CK_WORDS_PER_BLOCK = 65536;
__global__ __launch_bounds__(256) void pipe_checksum(const uint8_t* base, uint64_t stride, const uint64_t* len,
                                                     uint64_t fixed, unsigned long long* sums) {
  const uint32_t f = blockIdx.y;
  const uint64_t n = len ? len[f] : fixed;
  const uint64_t nw = (n + 3) / 4;
  const uint64_t w0 = (uint64_t)blockIdx.x * CK_WORDS_PER_BLOCK;
  if (w0 >= nw) return;
  const uint64_t w1 = w0 + CK_WORDS_PER_BLOCK < nw ? w0 + CK_WORDS_PER_BLOCK : nw;
  const uint8_t* fr = base + (uint64_t)f * stride;
  const bool al4 = (reinterpret_cast<uintptr_t>(fr) & 3u) == 0;   // (RGB frames of odd size: not)
  unsigned long long A = 0, B = 0;
  for (uint64_t w = w0 + threadIdx.x; w < w1; w += 256) {
    uint32_t v;
    if (al4 && 4 * w + 4 <= n) {
      v = *reinterpret_cast<const uint32_t*>(fr + 4 * w);
    } else {
      v = 0;
      for (uint32_t k = 0; k < 4u && 4 * w + k < n; ++k) v |= (uint32_t)fr[4 * w + k] << (8 * k);
    }
    A += v;
    B += (unsigned long long)(w + 1) * v;
  }
  for (int o = 32; o > 0; o >>= 1) {
    A += __shfl_xor(A, o);
    B += __shfl_xor(B, o);
  }
  if ((threadIdx.x & 63u) == 0) {
    atomicAdd(&sums[2 * f], A);
    atomicAdd(&sums[2 * f + 1], B);
  }
}

int launch_checksum(hipStream_t st, const uint8_t* base, uint64_t stride, const uint64_t* len, uint64_t max_bytes,
                    uint32_t n, unsigned long long* sums) {
  if (hipMemsetAsync(sums, 0, 16ull * n, st) != hipSuccess) return NICE_E_HIP;
  const uint32_t gx = (uint32_t)(((max_bytes + 3) / 4 + CK_WORDS_PER_BLOCK - 1) / CK_WORDS_PER_BLOCK);
  hipLaunchKernelGGL(pipe_checksum, dim3(gx ? gx : 1, n), dim3(256), 0, st, base, stride, len, max_bytes, sums);
  return hipGetLastError() == hipSuccess ? NICE_OK : NICE_E_HIP;
}

uint64_t ck_finish(const unsigned long long* s) { return s[0] + 0x9E3779B97F4A7C15ull * s[1]; }
}  // namespace

static void pipe_free(nice_pipe* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  for (Slot& s : p->slots) {
    if (s.st) (void)hipStreamSynchronize(s.st);
    if (s.ctx) nice_ctx_destroy(s.ctx);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.lens) (void)hipEventDestroy(s.lens);
    if (s.st) (void)hipStreamDestroy(s.st);
    (void)hipFree(s.d_px);
    (void)hipFree(s.d_str);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_status);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_status);
    (void)hipFree(s.d_sum);
    (void)hipHostFree(s.h_sum);
  }
  delete p;
}

extern "C" int nice_pipe_create(int device, uint32_t w, uint32_t h, uint8_t channels, uint32_t batch,
                                uint32_t depth, nice_pipe** out) {
  if (!out) return NICE_E_ARG;
  *out = nullptr;
  if ((channels != 3 && channels != 4) || batch == 0 || depth == 0 || depth > 8 || w == 0 || h == 0)
    return NICE_E_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NICE_E_NODEV;
  PIPE_HIP(hipSetDevice(device));
  nice_pipe* p = new nice_pipe();
  p->device = device;
  p->w = w;
  p->h = h;
  p->ch = channels;
  p->batch = batch;
  p->depth = depth;
  p->frame_bytes = (uint64_t)w * h * channels;
  p->str_stride = (nice_encode_bound(w, h) + 255) / 256 * 256;
  p->slots.resize(depth);
  for (Slot& s : p->slots) {
    int rc = nice_ctx_create(device, &s.ctx);
    if (rc == NICE_OK) rc = nice_ctx_reserve(s.ctx, batch, w, h);
    bool ok = rc == NICE_OK;
    ok = ok && hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&s.lens, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipMalloc(&s.d_px, p->frame_bytes * batch) == hipSuccess;
    ok = ok && hipMalloc(&s.d_str, p->str_stride * batch) == hipSuccess;
    ok = ok && hipMalloc(&s.d_len, 8ull * batch) == hipSuccess;
    ok = ok && hipMalloc(&s.d_status, 4ull * batch) == hipSuccess;
    ok = ok && hipHostMalloc(&s.h_len, 8ull * batch, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipHostMalloc(&s.h_status, 4ull * batch, hipHostMallocDefault) == hipSuccess;
    ok = ok && hipMalloc(&s.d_sum, 16ull * batch) == hipSuccess;
    ok = ok && hipHostMalloc(&s.h_sum, 16ull * batch, hipHostMallocDefault) == hipSuccess;
    if (!ok) {
      pipe_free(p);
      return rc != NICE_OK ? rc : NICE_E_HIP;
    }
  }
  *out = p;
  return NICE_OK;
}

extern "C" void nice_pipe_destroy(nice_pipe* p) { pipe_free(p); }

extern "C" uint64_t nice_pipe_stream_stride(const nice_pipe* p) { return p ? p->str_stride : 0; }

extern "C" int nice_pipe_set_checksums(nice_pipe* p, uint64_t* enc_sums, uint64_t* dec_sums) {
  if (!p) return NICE_E_ARG;
  p->enc_sums = enc_sums;
  p->dec_sums = dec_sums;
  return NICE_OK;
}

// Encode: streams of chunk `s.chunk` back to the host at their exact lengths.
static int pipe_encode_drain(nice_pipe* p, Slot& s, uint8_t* const* out, uint64_t out_cap,
                             uint64_t* out_len, int& status) {
  if (s.chunk < 0) return NICE_OK;
  PIPE_HIP(hipEventSynchronize(s.lens));
  const uint64_t f0 = (uint64_t)s.chunk * p->batch;
  for (uint32_t i = 0; i < s.n; ++i) {
    const uint64_t len = s.h_len[i];
    out_len[f0 + i] = len;
    if (p->enc_sums) p->enc_sums[f0 + i] = ck_finish(s.h_sum + 2 * i);
    if (len > out_cap) { status = NICE_E_CAPACITY; continue; }
    PIPE_HIP(hipMemcpyAsync(out[f0 + i], s.d_str + (uint64_t)i * p->str_stride, len, hipMemcpyDeviceToHost,
                            s.st));
  }
  PIPE_HIP(hipEventRecord(s.done, s.st));
  s.chunk = -1;
  return NICE_OK;
}

extern "C" int nice_pipe_encode(nice_pipe* p, const uint8_t* const* px, uint32_t n_frames, uint8_t channels_out,
                                uint8_t* const* out, uint64_t out_cap, uint64_t* out_len) {
  if (!p || (n_frames && (!px || !out || !out_len))) return NICE_E_ARG;
  PIPE_HIP(hipSetDevice(p->device));
  const uint32_t nchunks = (n_frames + p->batch - 1) / p->batch;
  int status = NICE_OK;
  int64_t prev = -1;   // slot whose streams are still to be copied back
  for (uint32_t c = 0; c < nchunks; ++c) {
    Slot& s = p->slots[c % p->depth];
    // the slot's previous chunk: normally drained one step after it was
    // submitted (only its stream copies may still run); with depth 1 drain now
    if (s.chunk >= 0) {
      const int rc = pipe_encode_drain(p, s, out, out_cap, out_len, status);
      if (rc != NICE_OK) return rc;
      prev = -1;
    }
    PIPE_HIP(hipEventSynchronize(s.done));
    const uint32_t n = std::min(p->batch, n_frames - c * p->batch);
    for (uint32_t i = 0; i < n; ++i)
      PIPE_HIP(hipMemcpyAsync(s.d_px + (uint64_t)i * p->frame_bytes, px[(uint64_t)c * p->batch + i], p->frame_bytes,
                              hipMemcpyHostToDevice, s.st));
    int rc = nice_encode_batch_dev(s.ctx, s.st, s.d_px, p->frame_bytes, n, p->w, p->h, (uint8_t)p->ch, channels_out,
                                   s.d_str, p->str_stride, s.d_len);
    if (rc != NICE_OK) return rc;
    if (p->enc_sums) {
      rc = launch_checksum(s.st, s.d_str, p->str_stride, s.d_len, p->str_stride, n, s.d_sum);
      if (rc != NICE_OK) return rc;
      PIPE_HIP(hipMemcpyAsync(s.h_sum, s.d_sum, 16ull * n, hipMemcpyDeviceToHost, s.st));
    }
    PIPE_HIP(hipMemcpyAsync(s.h_len, s.d_len, 8ull * n, hipMemcpyDeviceToHost, s.st));
    PIPE_HIP(hipEventRecord(s.lens, s.st));
    s.chunk = c;
    s.n = n;
    // copy back the previous chunk while this one computes
    if (prev >= 0) {
      rc = pipe_encode_drain(p, p->slots[prev], out, out_cap, out_len, status);
      if (rc != NICE_OK) return rc;
    }
    prev = c % p->depth;
  }
  if (prev >= 0) {
    const int rc = pipe_encode_drain(p, p->slots[prev], out, out_cap, out_len, status);
    if (rc != NICE_OK) return rc;
  }
  for (Slot& s : p->slots) PIPE_HIP(hipStreamSynchronize(s.st));
  return status;
}

extern "C" int nice_pipe_decode(nice_pipe* p, const uint8_t* const* streams, const uint64_t* stream_len,
                                uint32_t n_frames, uint8_t out_channels, uint8_t* const* px, uint32_t flags,
                                int32_t* status) {
  if (!p || (n_frames && (!streams || !stream_len || !px || !status))) return NICE_E_ARG;
  if (out_channels != 3 && out_channels != 4) return NICE_E_ARG;
  if (out_channels > p->ch) return NICE_E_ARG;   // device pixel buffers hold frame_bytes per frame
  PIPE_HIP(hipSetDevice(p->device));
  for (uint32_t f = 0; f < n_frames; ++f)
    if (stream_len[f] > p->str_stride) return NICE_E_ARG;
  const uint64_t out_bytes = (uint64_t)p->w * p->h * out_channels;
  const uint32_t nchunks = (n_frames + p->batch - 1) / p->batch;
  // statuses are read once a slot is reused or at the end (its stream done)
  auto collect = [&](Slot& s) -> int {
    if (s.chunk < 0) return NICE_OK;
    const uint64_t f0 = (uint64_t)s.chunk * p->batch;
    for (uint32_t i = 0; i < s.n; ++i) {
      status[f0 + i] = s.h_status[i];
      if (p->dec_sums) p->dec_sums[f0 + i] = ck_finish(s.h_sum + 2 * i);
    }
    s.chunk = -1;
    return NICE_OK;
  };
  for (uint32_t c = 0; c < nchunks; ++c) {
    Slot& s = p->slots[c % p->depth];
    PIPE_HIP(hipEventSynchronize(s.done));
    int rc = collect(s);
    if (rc != NICE_OK) return rc;
    const uint32_t n = std::min(p->batch, n_frames - c * p->batch);
    const uint64_t f0 = (uint64_t)c * p->batch;
    for (uint32_t i = 0; i < n; ++i) {
      s.h_len[i] = stream_len[f0 + i];
      PIPE_HIP(hipMemcpyAsync(s.d_str + (uint64_t)i * p->str_stride, streams[f0 + i], stream_len[f0 + i],
                              hipMemcpyHostToDevice, s.st));
    }
    PIPE_HIP(hipMemcpyAsync(s.d_len, s.h_len, 8ull * n, hipMemcpyHostToDevice, s.st));
    rc = nice::decode_batch_impl(s.ctx, s.st, s.d_str, p->str_stride, s.d_len, stream_len + f0, n, p->w, p->h,
                                 out_channels, s.d_px, out_bytes, flags, s.d_status);
    if (rc != NICE_OK) return rc;
    for (uint32_t i = 0; i < n; ++i)
      PIPE_HIP(hipMemcpyAsync(px[f0 + i], s.d_px + (uint64_t)i * out_bytes, out_bytes, hipMemcpyDeviceToHost, s.st));
    PIPE_HIP(hipMemcpyAsync(s.h_status, s.d_status, 4ull * n, hipMemcpyDeviceToHost, s.st));
    if (p->dec_sums) {
      rc = launch_checksum(s.st, s.d_px, out_bytes, nullptr, out_bytes, n, s.d_sum);
      if (rc != NICE_OK) return rc;
      PIPE_HIP(hipMemcpyAsync(s.h_sum, s.d_sum, 16ull * n, hipMemcpyDeviceToHost, s.st));
    }
    PIPE_HIP(hipEventRecord(s.done, s.st));
    s.chunk = c;
    s.n = n;
  }
  for (Slot& s : p->slots) {
    PIPE_HIP(hipStreamSynchronize(s.st));
    const int rc = collect(s);
    if (rc != NICE_OK) return rc;
  }
  for (uint32_t f = 0; f < n_frames; ++f)
    if (status[f] != NICE_OK) return status[f];
  return NICE_OK;
}
