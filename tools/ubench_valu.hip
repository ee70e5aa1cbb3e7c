// Diagnostic microbenchmark: issue cost of single VALU instructions on gfx950.
// Each lane runs 4 independent dependency chains of the instruction; 16 blocks
// of 256 threads per CU (16 waves per SIMD), so the SIMD's issue rate, not the
// dependency latency, sets the time.  Generated kernels; usage: ./ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 4096;
typedef void (*kfn)(uint32_t*, uint32_t, uint32_t);
__global__ __launch_bounds__(256) void k0(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_add_u32 %0, %4, %0\n v_add_u32 %1, %4, %1\n v_add_u32 %2, %4, %2\n v_add_u32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k1(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_sub_u32 %0, %0, %4\n v_sub_u32 %1, %1, %4\n v_sub_u32 %2, %2, %4\n v_sub_u32 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k2(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_and_b32 %0, %4, %0\n v_and_b32 %1, %4, %1\n v_and_b32 %2, %4, %2\n v_and_b32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k3(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_or_b32 %0, %4, %0\n v_or_b32 %1, %4, %1\n v_or_b32 %2, %4, %2\n v_or_b32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k4(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_xor_b32 %0, %4, %0\n v_xor_b32 %1, %4, %1\n v_xor_b32 %2, %4, %2\n v_xor_b32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k5(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_max_u32 %0, %4, %0\n v_max_u32 %1, %4, %1\n v_max_u32 %2, %4, %2\n v_max_u32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k6(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshlrev_b32 %0, %4, %0\n v_lshlrev_b32 %1, %4, %1\n v_lshlrev_b32 %2, %4, %2\n v_lshlrev_b32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k7(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshrrev_b32 %0, %4, %0\n v_lshrrev_b32 %1, %4, %1\n v_lshrrev_b32 %2, %4, %2\n v_lshrrev_b32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k8(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_bfe_u32 %0, %0, %4, 7\n v_bfe_u32 %1, %1, %4, 7\n v_bfe_u32 %2, %2, %4, 7\n v_bfe_u32 %3, %3, %4, 7" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k9(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshl_or_b32 %0, %0, 1, %4\n v_lshl_or_b32 %1, %1, 1, %4\n v_lshl_or_b32 %2, %2, 1, %4\n v_lshl_or_b32 %3, %3, 1, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k10(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshl_add_u32 %0, %0, 1, %4\n v_lshl_add_u32 %1, %1, 1, %4\n v_lshl_add_u32 %2, %2, 1, %4\n v_lshl_add_u32 %3, %3, 1, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k11(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_and_or_b32 %0, %0, %4, %5\n v_and_or_b32 %1, %1, %4, %5\n v_and_or_b32 %2, %2, %4, %5\n v_and_or_b32 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k12(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_or3_b32 %0, %0, %4, %5\n v_or3_b32 %1, %1, %4, %5\n v_or3_b32 %2, %2, %4, %5\n v_or3_b32 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k13(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_add3_u32 %0, %0, %4, %5\n v_add3_u32 %1, %1, %4, %5\n v_add3_u32 %2, %2, %4, %5\n v_add3_u32 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k14(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_alignbit_b32 %0, %0, %4, %5\n v_alignbit_b32 %1, %1, %4, %5\n v_alignbit_b32 %2, %2, %4, %5\n v_alignbit_b32 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k15(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k16(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mad_u32_u24 %0, %0, %4, %5\n v_mad_u32_u24 %1, %1, %4, %5\n v_mad_u32_u24 %2, %2, %4, %5\n v_mad_u32_u24 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k17(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mul_u32_u24 %0, %4, %0\n v_mul_u32_u24 %1, %4, %1\n v_mul_u32_u24 %2, %4, %2\n v_mul_u32_u24 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k18(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k19(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_add_f32 %0, %4, %0\n v_add_f32 %1, %4, %1\n v_add_f32 %2, %4, %2\n v_add_f32 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k20(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k21(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_add_co_u32 %0, s[8:9], %0, %4\n v_add_co_u32 %1, s[10:11], %1, %4\n v_add_co_u32 %2, s[12:13], %2, %4\n v_add_co_u32 %3, s[14:15], %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k22(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_cmp_gt_u32 s[8:9], %0, %4\n v_cmp_gt_u32 s[10:11], %1, %4\n v_cmp_gt_u32 s[12:13], %2, %4\n v_cmp_gt_u32 s[14:15], %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k23(uint32_t* out, uint32_t s, uint32_t t) {
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_mov_b32 %0, %0\n v_mov_b32 %1, %1\n v_mov_b32 %2, %2\n v_mov_b32 %3, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k24(uint32_t* out, uint32_t s, uint32_t t) {
  uint64_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %4, %1\n v_lshlrev_b64 %2, %4, %2\n v_lshlrev_b64 %3, %4, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
__global__ __launch_bounds__(256) void k25(uint32_t* out, uint32_t s, uint32_t t) {
  uint64_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
#pragma nounroll
  for (int i = 0; i < ITERS; ++i) asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n v_lshl_add_u64 %1, %1, 0, %1\n v_lshl_add_u64 %2, %2, 0, %2\n v_lshl_add_u64 %3, %3, 0, %3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "s8","s9","s10","s11","s12","s13","s14","s15");
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d);
}
static float run(kfn k, uint32_t* out, int blocks) {
  hipEvent_t t0, t1;
  (void)hipEventCreate(&t0); (void)hipEventCreate(&t1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u);
  (void)hipEventRecord(t0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u);
  (void)hipEventRecord(t1);
  (void)hipEventSynchronize(t1);
  float ms = 0; (void)hipEventElapsedTime(&ms, t0, t1);
  (void)hipEventDestroy(t0); (void)hipEventDestroy(t1);
  return ms;
}
int main() {
  const int blocks = 256 * 16;
  uint32_t* out; (void)hipMalloc(&out, blocks * 256 * 4);
  const double winst = (double)blocks * 4 * ITERS * 4;   // wave-instructions
  struct { const char* n; kfn k; } t[] = {
    {"v_add_u32", k0},
    {"v_sub_u32", k1},
    {"v_and_b32", k2},
    {"v_or_b32", k3},
    {"v_xor_b32", k4},
    {"v_max_u32", k5},
    {"v_lshlrev_b32", k6},
    {"v_lshrrev_b32", k7},
    {"v_bfe_u32", k8},
    {"v_lshl_or_b32", k9},
    {"v_lshl_add_u32", k10},
    {"v_and_or_b32", k11},
    {"v_or3_b32", k12},
    {"v_add3_u32", k13},
    {"v_alignbit_b32", k14},
    {"v_mul_lo_u32", k15},
    {"v_mad_u32_u24", k16},
    {"v_mul_u32_u24", k17},
    {"v_cndmask_e64", k18},
    {"v_add_f32", k19},
    {"v_fma_f32", k20},
    {"v_add_co_u32", k21},
    {"v_cmp_gt_u32 (sgpr)", k22},
    {"v_mov_b32", k23},
    {"v_lshlrev_b64", k24},
    {"v_lshl_add_u64", k25}};
  for (auto& x : t) {
    const float ms = run(x.k, out, blocks);
    printf("%-20s %.3f ms  %.2f cycles/wave-instr per SIMD (2.4 GHz)\n", x.n, ms, ms * 1e-3 * 2.4e9 * 1024 / winst);
  }
  (void)hipFree(out);
  return 0;
}
