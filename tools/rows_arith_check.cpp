// Host check of the row kernels' spread-form arithmetic (nice_decode.hip,
// round 5): the shipped forms of the interval average (ivs_avg), the
// speculative step (rows_step) and the exact step (rows_step_exact) against
// the straightforward forms they replaced.  The shipped forms are restated
// here line for line; the check is what DESIGN.md's "instruction cuts" table
// cites.  Usage: rows_arith_check [random_cases]   (exit 0: all equal)
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace {
constexpr uint32_t SP_K = 0xFFu | (0xFFu << 10) | (0xFFu << 20);
constexpr uint32_t SP_K9 = 0x1FFu | (0x1FFu << 10) | (0x1FFu << 20);
constexpr uint32_t SP_1 = 1u | (1u << 10) | (1u << 20);
constexpr uint32_t W_L1 = 1u << 28, W_AVG = 1u << 31, W_CUR = 1u << 18;
struct IvS { uint32_t lo, len; };
uint32_t wmask(uint32_t w, int bit) { return (uint32_t)(-(int32_t)((w >> bit) & 1u)); }

// --- the forms before round 5's cuts
IvS avg_old(IvS l, uint32_t u, uint32_t c) {
  const uint32_t s = l.lo + l.len;
  const uint32_t wm = ((s >> 8) & SP_1) * 0x3FFu;
  uint32_t lo1 = ((l.lo + u) >> 1) & SP_K, hi1 = ((s + u) >> 1) & SP_K9;
  const uint32_t ulo = (u >> 1) & SP_K, uhi = ((u + SP_K) >> 1) & SP_K9;
  lo1 = (lo1 & ~wm) | (ulo & wm);
  hi1 = (hi1 & ~wm) | (uhi & wm);
  return IvS{(lo1 + c) & SP_K, hi1 - lo1};
}
IvS step_old(IvS l1, IvS l2, IvS l3, uint32_t u, uint32_t wp) {
  const uint32_t c = wp & SP_K;
  const IvS va = avg_old(l1, u, c);
  const uint32_t m1 = wmask(wp, 28), m2 = wmask(wp, 29), m3 = wmask(wp, 30), ma = wmask(wp, 31), mc = wmask(wp, 18);
  const uint32_t slo = (l1.lo & m1) | (l2.lo & m2) | (l3.lo & m3);
  const uint32_t slen = (l1.len & m1) | (l2.len & m2) | (l3.len & m3) | (SP_K & mc);
  const uint32_t rlo = (slo + c) & SP_K;
  return IvS{(va.lo & ma) | (rlo & ~ma), (va.len & ma) | (slen & ~ma)};
}
uint32_t exact_old(uint32_t l1, uint32_t l2, uint32_t l3, uint32_t u, uint32_t wp) {
  const uint32_t c = wp & SP_K;
  const uint32_t va = ((((l1 + u) >> 1) & SP_K) + c) & SP_K;
  const uint32_t sel = (wp & W_L1) ? l1 : (wp & (W_L1 << 1)) ? l2 : (wp & (W_L1 << 2)) ? l3 : 0u;
  return (wp & W_AVG) ? va : ((sel + c) & SP_K);
}

// --- the shipped forms (nice_decode.hip: ivs_avg, rows_step<CUR>, rows_step_exact)
IvS avg_new(IvS l, uint32_t u, uint32_t c) {
  const uint32_t s = l.lo + l.len;
  const uint32_t wm = ((s >> 8) & SP_1) * 0x3FFu;
  const uint32_t lo0 = l.lo & ~wm, s0 = (s & ~wm) | (SP_K & wm);
  const uint32_t lo1 = ((lo0 + u) >> 1) & SP_K, hi1 = ((s0 + u) >> 1) & SP_K9;
  return IvS{(lo1 + c) & SP_K, hi1 - lo1};
}
template <bool CUR>
IvS step_new(IvS l1, IvS l2, IvS l3, uint32_t u, uint32_t wp) {
  const uint32_t c = wp;
  const IvS va = avg_new(l1, u, c);
  const uint32_t m1 = wmask(wp, 28), m2 = wmask(wp, 29), m3 = wmask(wp, 30), ma = wmask(wp, 31);
  const uint32_t slo = (l1.lo & m1) | (l2.lo & m2) | (l3.lo & m3);
  const uint32_t slen = (l1.len & m1) | (l2.len & m2) | (l3.len & m3) | (CUR ? SP_K & wmask(wp, 18) : 0u);
  const uint32_t rlo = (slo + c) & SP_K;
  return IvS{(va.lo & ma) | (rlo & ~ma), (va.len & ma) | (slen & ~ma)};
}
uint32_t exact_new(uint32_t l1, uint32_t l2, uint32_t l3, uint32_t u, uint32_t wp) {
  const uint32_t c = wp;
  const uint32_t sel = (l1 & wmask(wp, 28)) | (l2 & wmask(wp, 29)) | (l3 & wmask(wp, 30));
  const uint32_t ma = (uint32_t)((int32_t)wp >> 31);
  const uint32_t x = (((l1 + u) >> 1) & ma) | (sel & ~ma);
  return (x + c) & SP_K;
}

uint32_t rs = 2463534242u;
uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 17; rs ^= rs << 5; return rs; }
}  // namespace

int main(int argc, char** argv) {
  const unsigned long long n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000000ull;
  unsigned long long bad_avg = 0, bad_step = 0, bad_exact = 0;
  // the average, exhaustively over one field's (lo, len, u), the others random
  for (uint32_t lo = 0; lo < 256; ++lo)
    for (uint32_t len = 0; len < 256; ++len)
      for (uint32_t u = 0; u < 256; u += 3) {
        const int f = (int)(rnd() % 3u);
        uint32_t L = rnd() & SP_K, N = rnd() & SP_K, U = rnd() & SP_K, C = rnd() & SP_K;
        L = (L & ~(0xFFu << 10 * f)) | (lo << 10 * f);
        N = (N & ~(0xFFu << 10 * f)) | (len << 10 * f);
        U = (U & ~(0xFFu << 10 * f)) | (u << 10 * f);
        const IvS a = avg_old({L, N}, U, C), b = avg_new({L, N}, U, C);
        bad_avg += (a.lo != b.lo || a.len != b.len);
      }
  // the steps over random words of every kind (W_CUR: the width must agree;
  // its lower end is never used, the interval being the whole range)
  const uint32_t kinds[6] = {W_AVG, W_L1, W_L1 << 1, W_L1 << 2, 0u, W_CUR};
  for (unsigned long long i = 0; i < n; ++i) {
    const uint32_t k = kinds[rnd() % 6u];
    const uint32_t wp = k | (rnd() & SP_K);
    const uint32_t l1 = rnd() & SP_K, l2 = rnd() & SP_K, l3 = rnd() & SP_K, u = rnd() & SP_K;
    if (k != W_CUR) bad_exact += exact_old(l1, l2, l3, u, wp) != exact_new(l1, l2, l3, u, wp);
    IvS a{l1, rnd() & SP_K}, b{l2, rnd() & SP_K}, c{l3, rnd() & SP_K};
    if (rnd() & 1u) a.len = 0;
    const IvS p = step_new<true>(a, b, c, u, wp), q = step_old(a, b, c, u, wp);
    bad_step += (p.len != q.len || (k != W_CUR && p.lo != q.lo));
    if (k != W_CUR) {   // waves without W_CUR words take the CUR = false step
      const IvS r = step_new<false>(a, b, c, u, wp);
      bad_step += (r.len != q.len || r.lo != q.lo);
    }
  }
  printf("average %llu, step %llu, exact %llu mismatches (%llu random step cases)\n", bad_avg, bad_step, bad_exact, n);
  return (bad_avg || bad_step || bad_exact) ? 1 : 0;
}
