// syn_gen.hip -- BENCHMARK / TEST INPUT GENERATOR (not part of the codec).
//
// NICE-SYN-v1 frames generated on the GPU, bit-identical to
// oracle/nice_oracle.c nice_oracle_gen_syn_v1: raster order, one xorshift32
// stream per frame (seed = seed0 + frame) drawn 3 times per non-flat pixel.
// xorshift32 is linear over GF(2), so the state at any pixel is M^k(seed)
// with k = 3 x (non-flat pixels before it); each thread jumps to the start of
// its 64-pixel segment with the precomputed matrices M^(2^j) and then steps
// serially.  Built into tools/libnice_syn.so; used by bench.py and the tests.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <vector>

namespace {

constexpr int SEG = 64;
constexpr int JUMPS = 48;   // k < 2^48

struct SynArgs {
  uint8_t* out;
  uint64_t frame_stride;
  uint32_t n, W, H, C, seed0;
  const uint32_t* jump;           // JUMPS x 32 columns: M^(2^j) e_b
  const unsigned long long* rowk; // H: draws before row y (3 x non-flat pixels)
};

__device__ __forceinline__ uint32_t matvec(const uint32_t* col, uint32_t v) {
  uint32_t r = 0;
#pragma unroll 8
  for (int b = 0; b < 32; ++b) r ^= (v >> b & 1u) ? col[b] : 0u;
  return r;
}

__global__ __launch_bounds__(256) void syn_v1(SynArgs a) {
  const uint32_t segs = (a.W + SEG - 1) / SEG;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t total = (uint64_t)a.n * a.H * segs;
  if (t >= total) return;
  const uint32_t seg = (uint32_t)(t % segs);
  const uint32_t y = (uint32_t)((t / segs) % a.H);
  const uint32_t f = (uint32_t)(t / ((uint64_t)segs * a.H));
  const uint32_t x0 = seg * SEG, x1 = min(x0 + SEG, a.W);
  const uint32_t by16 = y / 16;
  // draws before x0 in this row
  uint64_t k = a.rowk[y];
  for (uint32_t x = 0; x < x0; x += 16) {
    const uint32_t xe = min(x + 16, x0);
    if (((x / 16) + by16) % 7 != 0) k += 3ull * (xe - x);
  }
  uint32_t s = a.seed0 + f;
  for (int j = 0; j < JUMPS; ++j)
    if (k >> j & 1ull) s = matvec(a.jump + 32 * j, s);
  const int amp = (int)(const int[]){0, 1, 2, 3, 8, 24, 64, 256}[(8ull * y) / a.H];
  const unsigned byv = a.H > 1 ? (200u * y) / (a.H - 1) : 0;
  uint8_t* row = a.out + (uint64_t)f * a.frame_stride + ((uint64_t)y * a.W) * a.C;
  for (uint32_t x = x0; x < x1; ++x) {
    uint8_t* p = row + (uint64_t)x * a.C;
    const unsigned bx = a.W > 1 ? (200u * x) / (a.W - 1) : 0;
    const unsigned base[3] = {bx, byv, (bx + byv) / 2};
    uint8_t v[3];
    if (((x / 16) + by16) % 7 == 0) {
      v[0] = 40; v[1] = 80; v[2] = 120;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        s ^= s << 13; s ^= s >> 17; s ^= s << 5;
        int n;
        if (amp == 0) n = 0;
        else if (amp < 256) n = (int)(s % (uint32_t)amp) - amp / 2;
        else n = (int)(s & 255u);
        v[c] = (uint8_t)((int)base[c] + n);
      }
    }
    if (a.C == 4) {
      *reinterpret_cast<uint32_t*>(p) = (uint32_t)v[0] | (uint32_t)v[1] << 8 | (uint32_t)v[2] << 16 | 0xFF000000u;
    } else {
      p[0] = v[0]; p[1] = v[1]; p[2] = v[2];
    }
  }
}

uint32_t host_matvec(const uint32_t* col, uint32_t v) {
  uint32_t r = 0;
  for (int b = 0; b < 32; ++b) if (v >> b & 1u) r ^= col[b];
  return r;
}

}  // namespace

extern "C" int nice_syn_v1_dev(uint8_t* d_out, uint64_t frame_stride, uint32_t n, uint32_t W, uint32_t H,
                               uint32_t C, uint32_t seed0, void* stream) {
  if (!d_out || (C != 3 && C != 4) || (C == 4 && (((uintptr_t)d_out & 3) || (frame_stride & 3)))) return -1;
  if (frame_stride < (uint64_t)W * H * C) return -1;
  if (n == 0 || W == 0 || H == 0) return 0;
  std::vector<uint32_t> jump(JUMPS * 32);
  for (int b = 0; b < 32; ++b) {   // M e_b
    uint32_t s = 1u << b;
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    jump[b] = s;
  }
  for (int j = 1; j < JUMPS; ++j)
    for (int b = 0; b < 32; ++b) jump[32 * j + b] = host_matvec(&jump[32 * (j - 1)], jump[32 * (j - 1) + b]);
  std::vector<unsigned long long> rowk(H);
  unsigned long long k = 0;
  for (uint32_t y = 0; y < H; ++y) {
    rowk[y] = k;
    for (uint32_t x = 0; x < W; ++x) k += (((x / 16) + (y / 16)) % 7 != 0) ? 3 : 0;
  }
  hipStream_t st = (hipStream_t)stream;
  void* dj = nullptr;
  const size_t jb = jump.size() * 4, rb = rowk.size() * 8;
  if (hipMalloc(&dj, jb + rb) != hipSuccess) return -2;
  if (hipMemcpyAsync(dj, jump.data(), jb, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync((uint8_t*)dj + jb, rowk.data(), rb, hipMemcpyHostToDevice, st) != hipSuccess) {
    (void)hipFree(dj);
    return -2;
  }
  SynArgs a{d_out, frame_stride, n, W, H, C, seed0, (const uint32_t*)dj,
            (const unsigned long long*)((uint8_t*)dj + jb)};
  const uint64_t threads = (uint64_t)n * H * ((W + SEG - 1) / SEG);
  const uint64_t blocks = (threads + 255) / 256;
  hipLaunchKernelGGL(syn_v1, dim3((uint32_t)blocks), dim3(256), 0, st, a);
  int rc = hipGetLastError() == hipSuccess ? 0 : -2;
  if (hipStreamSynchronize(st) != hipSuccess) rc = -2;
  (void)hipFree(dj);
  return rc;
}
