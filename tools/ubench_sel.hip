// Diagnostic microbenchmark: v_cndmask_b32 with VCC vs SGPR masks, alone, in
// runs and mixed with adds (cycles per wave-instruction per SIMD, 16 waves/SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITERS = 4096;
typedef void (*kfn)(uint32_t*, uint32_t, uint32_t);
#define K(NAME, OPS) __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint32_t s, uint32_t t) { \
  uint32_t a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3; \
  asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(s) : "vcc"); \
  _Pragma("nounroll") for (int i = 0; i < ITERS; ++i) asm volatile(OPS : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(s), "v"(t) : "vcc", "s8","s9","s10","s11","s12","s13","s14","s15"); \
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d; }
// 8 instructions per iteration in each kernel
K(k_pair_vcc, "v_cmp_gt_u32 vcc, %0, %4\n v_cndmask_b32 %0, %0, %5, vcc\n v_cmp_gt_u32 vcc, %1, %4\n v_cndmask_b32 %1, %1, %5, vcc\n v_cmp_gt_u32 vcc, %2, %4\n v_cndmask_b32 %2, %2, %5, vcc\n v_cmp_gt_u32 vcc, %3, %4\n v_cndmask_b32 %3, %3, %5, vcc")
K(k_pair_sgpr, "v_cmp_gt_u32 s[8:9], %0, %4\n v_cndmask_b32_e64 %0, %0, %5, s[8:9]\n v_cmp_gt_u32 s[10:11], %1, %4\n v_cndmask_b32_e64 %1, %1, %5, s[10:11]\n v_cmp_gt_u32 s[12:13], %2, %4\n v_cndmask_b32_e64 %2, %2, %5, s[12:13]\n v_cmp_gt_u32 s[14:15], %3, %4\n v_cndmask_b32_e64 %3, %3, %5, s[14:15]")
K(k_cnd_vcc8, "v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %0, %0, %5, vcc\n v_cndmask_b32 %1, %1, %5, vcc\n v_cndmask_b32 %2, %2, %5, vcc\n v_cndmask_b32 %3, %3, %5, vcc")
K(k_cnd_mix, "v_cndmask_b32 %0, %0, %4, vcc\n v_add_u32 %1, %1, %4\n v_cndmask_b32 %2, %2, %4, vcc\n v_add_u32 %3, %3, %4\n v_cndmask_b32 %0, %0, %5, vcc\n v_add_u32 %1, %1, %5\n v_cndmask_b32 %2, %2, %5, vcc\n v_add_u32 %3, %3, %5")
K(k_add8, "v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n v_add_u32 %0, %0, %5\n v_add_u32 %1, %1, %5\n v_add_u32 %2, %2, %5\n v_add_u32 %3, %3, %5")
K(k_bitop3sel, "v_bitop3_b32 %0, %0, %4, %5 bitop3:0xca\n v_bitop3_b32 %1, %1, %4, %5 bitop3:0xca\n v_bitop3_b32 %2, %2, %4, %5 bitop3:0xca\n v_bitop3_b32 %3, %3, %4, %5 bitop3:0xca\n v_bitop3_b32 %0, %0, %5, %4 bitop3:0xca\n v_bitop3_b32 %1, %1, %5, %4 bitop3:0xca\n v_bitop3_b32 %2, %2, %5, %4 bitop3:0xca\n v_bitop3_b32 %3, %3, %5, %4 bitop3:0xca")
K(k_pairs, "v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n v_cndmask_b32 %0, %0, %5, vcc\n v_cndmask_b32 %1, %1, %5, vcc\n v_add_u32 %2, %2, %5\n v_add_u32 %3, %3, %5")
K(k_pairs_e64, "v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n v_cndmask_b32_e64 %0, %0, %5, s[8:9]\n v_cndmask_b32_e64 %1, %1, %5, s[8:9]\n v_add_u32 %2, %2, %5\n v_add_u32 %3, %3, %5")
K(k_cmp_pair, "v_cmp_gt_u32 vcc, %0, %4\n v_cndmask_b32 %0, %0, %5, vcc\n v_cndmask_b32 %1, %1, %5, vcc\n v_add_u32 %2, %2, %4\n v_cmp_gt_u32 vcc, %3, %4\n v_cndmask_b32 %3, %3, %5, vcc\n v_cndmask_b32 %2, %2, %5, vcc\n v_add_u32 %1, %1, %4")
K(k_cmp_pair_e64, "v_cmp_gt_u32 s[8:9], %0, %4\n v_cndmask_b32_e64 %0, %0, %5, s[8:9]\n v_cndmask_b32_e64 %1, %1, %5, s[8:9]\n v_add_u32 %2, %2, %4\n v_cmp_gt_u32 s[10:11], %3, %4\n v_cndmask_b32_e64 %3, %3, %5, s[10:11]\n v_cndmask_b32_e64 %2, %2, %5, s[10:11]\n v_add_u32 %1, %1, %4")
K(k_run3, "v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_add_u32 %3, %3, %4\n v_cndmask_b32 %0, %0, %5, vcc\n v_cndmask_b32 %1, %1, %5, vcc\n v_cndmask_b32 %2, %2, %5, vcc\n v_add_u32 %3, %3, %5")
K(k_run4, "v_cndmask_b32 %0, %0, %4, vcc\n v_cndmask_b32 %1, %1, %4, vcc\n v_cndmask_b32 %2, %2, %4, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n v_add_u32 %0, %0, %5\n v_add_u32 %1, %1, %5\n v_add_u32 %2, %2, %5\n v_add_u32 %3, %3, %5")
K(k_run4_e64, "v_cndmask_b32_e64 %0, %0, %4, s[8:9]\n v_cndmask_b32_e64 %1, %1, %4, s[8:9]\n v_cndmask_b32_e64 %2, %2, %4, s[8:9]\n v_cndmask_b32_e64 %3, %3, %4, s[8:9]\n v_add_u32 %0, %0, %5\n v_add_u32 %1, %1, %5\n v_add_u32 %2, %2, %5\n v_add_u32 %3, %3, %5")
static float run(kfn k, uint32_t* out, int blocks) {
  hipEvent_t t0, t1; (void)hipEventCreate(&t0); (void)hipEventCreate(&t1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u);
  (void)hipEventRecord(t0);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 1u, 3u);
  (void)hipEventRecord(t1); (void)hipEventSynchronize(t1);
  float ms = 0; (void)hipEventElapsedTime(&ms, t0, t1); return ms;
}
int main() {
  const int blocks = 256 * 16; uint32_t* out; (void)hipMalloc(&out, blocks * 256 * 4);
  const double winst = (double)blocks * 4 * ITERS * 8;
  struct { const char* n; kfn k; } t[] = {{"cmp_e32(vcc)+cndmask_e32", k_pair_vcc}, {"cmp_e64(sgpr)+cndmask_e64", k_pair_sgpr},
    {"cndmask_e32 x8", k_cnd_vcc8}, {"cndmask_e32/add mix", k_cnd_mix}, {"add x8", k_add8}, {"bitop3 select x8", k_bitop3sel}, {"vcc pairs + adds", k_pairs}, {"sgpr pairs + adds", k_pairs_e64}, {"cmp + vcc pair + add", k_cmp_pair}, {"cmp + sgpr pair + add", k_cmp_pair_e64}, {"vcc runs of 3 + add", k_run3}, {"vcc runs of 4 + 4 adds", k_run4}, {"sgpr runs of 4 + 4 adds", k_run4_e64}};
  for (auto& x : t) { const float ms = run(x.k, out, blocks);
    printf("%-28s %.3f ms  %.2f cycles/wave-instr (avg over the 8)\n", x.n, ms, ms * 1e-3 * 2.4e9 * 1024 / winst); }
  return 0;
}
