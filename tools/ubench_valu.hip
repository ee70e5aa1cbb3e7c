// Diagnostic microbenchmark: issue cost of a few VALU instructions on gfx950
// (4 independent dependency chains per lane, every CU busy).  Usage: ./ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 4096;
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t s) {
  uint64_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  uint32_t e = threadIdx.x, f = e + 1, g = e + 2, h = e + 3;
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (OP == 0) {
      asm volatile("v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %4, %1\n v_lshlrev_b64 %2, %4, %2\n v_lshlrev_b64 %3, %4, %3"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s));
    } else if constexpr (OP == 1) {
      asm volatile("v_alignbit_b32 %0, %0, %4, %4\n v_alignbit_b32 %1, %1, %4, %4\n v_alignbit_b32 %2, %2, %4, %4\n v_alignbit_b32 %3, %3, %4, %4"
                   : "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(s));
    } else if constexpr (OP == 2) {
      asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                   : "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(s));
    } else if constexpr (OP == 3) {
      asm volatile("v_lshrrev_b64 %0, %4, %0\n v_lshrrev_b64 %1, %4, %1\n v_lshrrev_b64 %2, %4, %2\n v_lshrrev_b64 %3, %4, %3"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s));
    } else {
      asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n v_lshl_add_u64 %1, %1, 0, %1\n v_lshl_add_u64 %2, %2, 0, %2\n v_lshl_add_u64 %3, %3, 0, %3"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a ^ b ^ c ^ d) ^ e ^ f ^ g ^ h;
}
template <int OP>
static float run(uint32_t* out, int blocks) {
  hipEvent_t t0, t1;
  hipEventCreate(&t0); hipEventCreate(&t1);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  hipEventRecord(t0);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
  hipEventRecord(t1);
  hipEventSynchronize(t1);
  float ms = 0; hipEventElapsedTime(&ms, t0, t1);
  return ms;
}
int main() {
  const int blocks = 256 * 16;   // 16 blocks (64 waves) per CU
  uint32_t* out; hipMalloc(&out, blocks * 256 * 4);
  const double winst = (double)blocks * 4 * ITERS * 4;   // wave-instructions
  const char* names[] = {"v_lshlrev_b64", "v_alignbit_b32", "v_add_u32", "v_lshrrev_b64", "v_lshl_add_u64"};
  float ms[5] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks), run<4>(out, blocks)};
  for (int i = 0; i < 5; ++i)
    printf("%-16s %.3f ms  %.2f cycles/wave-instr per SIMD (2.4 GHz)\n", names[i], ms[i], ms[i] * 1e-3 * 2.4e9 * 1024 / winst);
  hipFree(out);
  return 0;
}
