// nice_format.h -- NICE2 bitstream constants shared by the HIP kernels and the
// host runtime.  Values follow the reference exactly:
//   prefix ids          code.rs:16-28
//   stream ids          code.rs:32-45
//   alphabet sizes      code.rs:91-116 (stream order)
//   reference offsets   code.rs:141-145 (encoder), code.rs:548-552 (decoder)
#pragma once
#include <stdint.h>

namespace nice {

// Prefix symbols (stream SC_PREFIXES).
constexpr int P_BACK_REF = 0;
constexpr int P_RGB = 1;
constexpr int P_LUMA = 2;
constexpr int P_SMALL_DIFF = 3;
constexpr int P_LUMA2 = 4;
constexpr int P_RUN1 = 5;  // run digit d is emitted as prefix 5 + d (code.rs:394)

// Symbol streams, in header order.
constexpr int S_RGB = 0;
constexpr int S_PREFIX = 1;
constexpr int S_LUMA_BASE = 2;
constexpr int S_LUMA_OTHER = 3;
constexpr int S_LUMA_REF = 4;
constexpr int S_SMALL_DIFF = 5;
constexpr int S_LUMA2_BASE = 6;
constexpr int S_LUMA2_R = 7;
constexpr int S_LUMA2_B = 8;
constexpr int S_BACK_REF = 9;
constexpr int N_STREAMS = 10;
constexpr int N_BINS = 858;  // sum of alphabet sizes
constexpr int MAX_ALPHABET = 343;

__host__ __device__ constexpr int stream_size(int s) {
  return s == 0 ? 256 : s == 1 ? 13 : s == 2 ? 64 : s == 3 ? 32 : s == 4 ? 11
       : s == 5 ? 343 : s == 6 ? 64 : s == 7 ? 32 : s == 8 ? 32 : 11;
}
__host__ __device__ constexpr int stream_base(int s) {
  return s == 0 ? 0 : s == 1 ? 256 : s == 2 ? 269 : s == 3 ? 333 : s == 4 ? 365
       : s == 5 ? 376 : s == 6 ? 719 : s == 7 ? 783 : s == 8 ? 815 : 847;
}

// Global histogram bin of (stream, symbol).
constexpr int BIN_PREFIX = 256;       // stream_base(S_PREFIX)
constexpr int BIN_LUMA_BASE = 269;
constexpr int BIN_LUMA_OTHER = 333;
constexpr int BIN_LUMA_REF = 365;
constexpr int BIN_SMALL_DIFF = 376;
constexpr int BIN_LUMA2_BASE = 719;
constexpr int BIN_LUMA2_R = 783;
constexpr int BIN_LUMA2_B = 815;
constexpr int BIN_BACK_REF = 847;

// File layout (code.rs:72-84): "nice", u32 BE width, u32 BE height, channels byte.
constexpr int FILE_HEADER_BYTES = 13;
// Normal table header: 10 x 5-bit max + 858 x 7-bit lengths = 6056 bits = 757 bytes
// (hfe.rs:97-103; field width 7 whenever every max length <= 128).
constexpr int TABLE_HEADER_BITS = 10 * 5 + 7 * N_BINS;
// Longest code the parallel packer handles: with <= 7 bits pending in the
// reference writer's u32 cache, any code of <= 25 bits is placed exactly
// (bitwriter.rs:63-64); longer emitted codes take the serial exact path.
constexpr int FAST_MAX_CODE_BITS = 25;

// Reference offsets expressed as (rows back, pixels back): off = k*W + d.
// Back references, code.rs:145: [1, W, W-1, 2, 2W].
__host__ __device__ constexpr int br_rows(int k) { return k == 0 ? 0 : k == 1 ? 1 : k == 2 ? 1 : k == 3 ? 0 : 2; }
__host__ __device__ constexpr int br_px(int k) { return k == 0 ? 1 : k == 1 ? 0 : k == 2 ? -1 : k == 3 ? 2 : 0; }
// Luma references, code.rs:141-142: [1, W, W-1, W-3, 3, 3W-1, 3W, 3W+1, W+3, 3W+3, 3W-3].
__host__ __device__ constexpr int lr_rows(int k) {
  return k == 0 ? 0 : k <= 3 ? 1 : k == 4 ? 0 : k <= 7 ? 3 : k == 8 ? 1 : 3;
}
__host__ __device__ constexpr int lr_px(int k) {
  return k == 0 ? 1 : k == 1 ? 0 : k == 2 ? -1 : k == 3 ? -3 : k == 4 ? 3 : k == 5 ? -1
       : k == 6 ? 0 : k == 7 ? 1 : k == 8 ? 3 : k == 9 ? 3 : -3;
}

}  // namespace nice
