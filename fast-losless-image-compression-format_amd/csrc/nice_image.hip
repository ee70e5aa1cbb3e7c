// nice_image.hip -- the 5x5 sub-block traversal of image.rs.
//
// image.rs:45-102 Image::calc_pos_from maps a traversal index to a raster
// position: the image is cut into bands of 5 rows (the last band holds
// h % 5 rows), each band into 5-wide sub-blocks (the last holds w % 5 columns);
// sub-blocks are walked left to right, the rows inside alternate direction and
// every odd sub-block is walked bottom-up.  The reference codec never calls it
// (it is exercised by its unit test image.rs:105-115 only); it is kept here so a
// caller of Image finds it.  The map is the reference's exactly, quirks
// included: it is not a permutation when both w % 5 and h % 5 are nonzero, and
// for some shapes (w = 7, ...) it returns positions >= w*h.  Release (wrapping)
// usize arithmetic; no step of it wraps for w >= 1.
//
// One thread per index; the work is 8 bytes written per index, so the kernel is
// HBM-write bound (~8 B / index) once the divisions are cheap: they are done in
// 32 bits when every operand fits (host-checked; 64-bit division is a long
// software loop), the band one through an fp64 reciprocal, the in-block ones by
// the constants 25 and 5 away from the leftover edges.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nice.h"

namespace {

constexpr uint32_t SUB_H = 5, SUB_W = 5;   // image.rs:3-4 SUBBLOCK_HEIGHT_MAX / SUBBLOCK_WIDTH_MAX

struct Shape {   // image.rs:30-42 Image::new, the fields calc_pos_from reads
  uint64_t width, image_size, width_block_size, width_minus_leftover, h_minus_left_times_w;
  uint32_t h_left, w_left;
  double rcp_wbs;   // 1 / width_block_size (32-bit path)
};

Shape make_shape(uint32_t w, uint32_t h) {
  Shape s;
  s.width = w;
  s.image_size = (uint64_t)w * h;
  s.width_block_size = (uint64_t)w * SUB_H;
  s.width_minus_leftover = w - w % SUB_W;
  s.h_minus_left_times_w = (uint64_t)(h - h % SUB_H) * w;
  s.h_left = h % SUB_H;
  s.w_left = w % SUB_W;
  s.rcp_wbs = 1.0 / (double)s.width_block_size;
  return s;
}

// q = n / d for n < 2^32: fp64 estimate (n is exact in a double, rcp = 1/d to
// 53 bits, so the estimate is off by at most one) and an integer fix-up.
__device__ __forceinline__ uint32_t div_rcp(uint32_t n, uint32_t d, double rcp) {
  uint32_t q = (uint32_t)((double)n * rcp);
  int64_t r = (int64_t)n - (int64_t)q * d;
  q = r < 0 ? q - 1 : (r >= (int64_t)d ? q + 1 : q);
  return q;
}

// T = uint32_t when index, width_block_size and the result fit in 32 bits.
// Outside the last band (h % 5 rows) and the last block column (w % 5) the
// sub-block is 5 x 5: those divisions are by constants.
template <typename T>
__device__ __forceinline__ uint64_t pos_from(const Shape& s, uint64_t index) {
  const bool inside = index < s.image_size;
  const T sh = (index >= s.h_minus_left_times_w && inside) ? (T)s.h_left : (T)SUB_H;
  const T idx = (T)index;
  const T wbs = (T)s.width_block_size;
  T offset;
  if constexpr (sizeof(T) == 4) offset = div_rcp(idx, wbs, s.rcp_wbs) * wbs;
  else offset = idx - idx % wbs;
  T rem = idx - offset;
  const T sw = (rem >= sh * (T)s.width_minus_leftover && inside) ? (T)s.w_left : (T)SUB_W;
  T blk, row;
  if (sw == SUB_W && sh == SUB_H) {
    blk = rem / (SUB_W * SUB_H);
    rem -= blk * (SUB_W * SUB_H);
    row = rem / SUB_W;
  } else {
    const T area = sw * sh;
    blk = rem / area;
    rem -= blk * area;
    row = rem / sw;
  }
  const T col = rem - row * sw;
  offset += blk * sw;
  offset += ((blk & 1) == 0 ? row : sh - row - 1) * (T)s.width;
  offset += (row & 1) == 1 ? sw - col - 1 : col;
  return (uint64_t)offset;
}

// Two indices per thread and one 16-byte store when pos is 16-byte aligned.
template <typename T, bool PAIRS>
__global__ __launch_bounds__(256) void subblock_positions(Shape s, uint64_t index0, uint64_t count,
                                                          uint64_t* __restrict__ pos) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (PAIRS) {
    for (uint64_t i = first; 2 * i < count; i += stride) {
      const uint64_t a = pos_from<T>(s, index0 + 2 * i);
      if (2 * i + 1 < count) {
        const uint64_t b = pos_from<T>(s, index0 + 2 * i + 1);
        reinterpret_cast<ulonglong2*>(pos)[i] = make_ulonglong2(a, b);
      } else {
        pos[2 * i] = a;
      }
    }
  } else {
    for (uint64_t i = first; i < count; i += stride) pos[i] = pos_from<T>(s, index0 + i);
  }
}

}  // namespace

extern "C" int nice_subblock_positions_dev(int device, void* stream, uint32_t w, uint32_t h, uint64_t index0,
                                           uint64_t count, uint64_t* d_pos) {
  if (w == 0) return NICE_E_ARG;   // image.rs:68: the reference divides by zero
  if (count == 0) return NICE_OK;
  if (!d_pos || index0 + count < index0) return NICE_E_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return NICE_E_NODEV;
  if (hipSetDevice(device) != hipSuccess) return NICE_E_HIP;
  const Shape s = make_shape(w, h);
  // the largest position is < last index + 5*w (one band below, one block right)
  const bool narrow = index0 + count + 6 * (uint64_t)w < (1ull << 32);
  const bool pairs = ((uintptr_t)d_pos & 15) == 0;
  const uint64_t threads = pairs ? (count + 1) / 2 : count;
  const uint64_t blocks64 = (threads + 255) / 256;
  const unsigned blocks = (unsigned)(blocks64 < 65536 ? blocks64 : 65536);
  hipStream_t st = (hipStream_t)stream;
  auto* k = narrow ? (pairs ? subblock_positions<uint32_t, true> : subblock_positions<uint32_t, false>)
                   : (pairs ? subblock_positions<uint64_t, true> : subblock_positions<uint64_t, false>);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, st, s, index0, count, d_pos);
  return hipGetLastError() == hipSuccess ? NICE_OK : NICE_E_HIP;
}
