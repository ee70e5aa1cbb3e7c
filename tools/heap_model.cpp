// Diagnostic: host model of the wave-parallel BinaryHeap replay used by
// enc_tables (nice_huffman.hpp huffman_merge_wave), lane loops written out,
// checked against the oracle's literal replay (oracle/nice_oracle.c,
// hfe.rs:58-87 + std BinaryHeap) on random count vectors with many ties.
// (The device version skips the pref-bit upkeep during the n initial pushes
// and sets every bit once before the merge loop; the bits it then holds are
// the ones this model maintains push by push.)
// Build: gcc -O2 -c oracle/nice_oracle.c -o /tmp/o.o && g++ -O2 tools/heap_model.cpp /tmp/o.o -Ioracle
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
extern "C" {
#include "nice_oracle.h"
}

struct Model {
  uint64_t key[512];   // count << 10 | node
  uint32_t pm[64];     // lane L < 63: pref bit of node L (levels 0..5)
  uint32_t P[64];      // lane L: pref bits of level-6 node 63+L (bit 0) and its children (bits 1, 2)
  int len = 0;
  static int lev(uint32_t i) { return 31 - __builtin_clz(i + 1); }
  static bool gt(uint64_t a, uint64_t b) { return (a | 1023) > (b | 1023); }   // cnt(a) > cnt(b)
  void setpref(uint32_t i, uint32_t b) {
    const int D = lev(i);
    if (D < 6) { pm[i] = b; return; }
    const uint32_t r = ((i + 1) >> (D - 6)) - 64, t = D - 6, o = (i + 1) - ((64 + r) << t);
    const uint32_t l = (1u << t) - 1 + o;
    P[r] = (P[r] & ~(1u << l)) | (b << l);
  }
  // right child is preferred when cnt(right) <= cnt(left) (std sift_down_to_bottom)
  uint32_t pref_of(uint32_t node, uint32_t c, uint64_t cval) const {
    const uint32_t s = (c & 1) ? c + 1 : c - 1;
    const uint32_t right = (c & 1) ? s : c;
    if (right >= (uint32_t)len) return 0;
    const uint64_t lv = (c & 1) ? cval : key[s], rv = (c & 1) ? key[s] : cval;
    (void)node;
    return gt(rv, lv) ? 0u : 1u;
  }
  uint64_t pop() {
    const uint64_t top = key[0];
    --len;
    const uint32_t e = len;
    if (len == 0) return top;
    const uint64_t elem = key[e];
    if (!(e & 1)) setpref((e - 1) >> 1, 0);
    // walk: M = ballot(pm); lane L matches iff its ancestors' prefs lead to it
    uint64_t M = 0;
    for (int L = 0; L < 63; ++L) M |= (uint64_t)(pm[L] & 1) << L;
    int r6 = -1;
    for (int L = 0; L < 64; ++L) {
      uint64_t A = 0, R = 0;
      for (int d = 0; d < 6; ++d) {
        const uint32_t anc = ((64u + L) >> (6 - d)) - 1, bit = ((64u + L) >> (5 - d)) & 1;
        A |= 1ull << anc;
        R |= (uint64_t)bit << anc;
      }
      if ((M & A) == R) { if (r6 >= 0) abort(); r6 = L; }
    }
    const uint32_t s = P[r6];
    const uint32_t l1 = 1 + (s & 1), l2 = 2 * l1 + 1 + ((s >> l1) & 1);
    const uint32_t x8 = ((64u + r6) << 2) - 1 + (l2 - 3);
    uint32_t p[9];
    int k = -1;
    for (int d = 0; d < 9; ++d) { p[d] = ((x8 + 1) >> (8 - d)) - 1; if (p[d] < (uint32_t)len) k = d; }
    uint64_t v[9];
    for (int d = 0; d < k; ++d) v[d] = key[p[d + 1]];
    int j = 0;
    for (int d = 0; d < k; ++d) if (!gt(v[d], elem)) j = d + 1;
    for (int d = 0; d < j; ++d) key[p[d]] = v[d];
    key[p[j]] = elem;
    uint32_t b[9];
    for (int d = 0; d < j; ++d) b[d] = pref_of(p[d], p[d + 1], d + 1 < j ? v[d + 1] : elem);
    for (int d = 0; d < j; ++d) setpref(p[d], b[d]);
    return top;
  }
  void push(uint64_t x) {
    const uint32_t e = len++;
    const int D = lev(e);
    uint32_t a[10];
    uint64_t old[10];
    for (int d = 0; d <= D; ++d) { a[d] = ((e + 1) >> (D - d)) - 1; old[d] = key[a[d]]; }
    int j = 0;
    for (int d = 0; d < D; ++d) if (!gt(old[d], x)) j = d + 1;
    key[a[j]] = x;
    for (int d = j + 1; d <= D; ++d) key[a[d]] = old[d - 1];
    uint32_t b[10];
    const int d0 = j > 0 ? j - 1 : 0;
    for (int d = d0; d < D; ++d) b[d] = pref_of(a[d], a[d + 1], d + 1 == j ? x : old[d]);
    for (int d = d0; d < D; ++d) setpref(a[d], b[d]);
  }
};

static void lengths(const uint64_t* counts, int n, uint8_t* aob) {
  Model m;
  for (int i = 0; i < 64; ++i) m.pm[i] = m.P[i] = 0;
  std::vector<int> parent(2 * n + 2, -1);
  for (int i = 0; i < n; ++i) m.push(counts[i] << 10 | (uint64_t)i);
  int next = n;
  while (m.len > 2) {
    const uint64_t a = m.pop(), b = m.pop();
    const int id = next++;
    parent[a & 1023] = id;
    parent[b & 1023] = id;
    m.push(((a >> 10) + (b >> 10)) << 10 | (uint64_t)id);
  }
  for (int i = 0; i < n; ++i) {
    int dpt = 0;
    for (int q = parent[i]; q >= 0; q = parent[q]) ++dpt;
    aob[i] = (uint8_t)(1 + dpt);
  }
}

int main() {
  std::mt19937_64 rng(7);
  const int sizes[] = {256, 13, 64, 32, 11, 343, 3, 2, 1};
  int bad = 0, total = 0;
  for (int it = 0; it < 20000; ++it) {
    const int n = sizes[it % 9];
    std::vector<uint64_t> c(n);
    const int mode = (it / 9) % 5;
    for (int i = 0; i < n; ++i) {
      const uint64_t r = rng();
      c[i] = mode == 0 ? r % 4 : mode == 1 ? r % 50 : mode == 2 ? (r % 3 == 0 ? 0 : r % 100000)
           : mode == 3 ? (r % 2 ? 5 : 7) : (r >> 20);
    }
    std::vector<uint8_t> x(n), y(n);
    lengths(c.data(), n, x.data());
    nice_oracle_code_lengths(c.data(), n, y.data());
    ++total;
    if (x != y) { if (bad < 5) printf("mismatch n=%d mode=%d\n", n, mode); ++bad; }
  }
  printf("%d / %d mismatches\n", bad, total);
  return bad != 0;
}
