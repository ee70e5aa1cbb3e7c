// nice_huffman.hpp -- device restatement of the reference entropy-table build.
//
//  * code lengths: hfe.rs:58-87 -- every symbol of the alphabet (zero counts
//    included) is pushed into a std::collections::BinaryHeap<TreeNode> whose Ord
//    is reversed on the count (hfe.rs:246-251); while more than two nodes remain,
//    two are popped and their merge pushed back; every symbol under a merged node
//    gets +1 (u8, wrapping) on an initial length of 1.  Tie-breaking is whatever
//    std's sift_up / sift_down_to_bottom produce, so the heap is replayed exactly.
//  * canonical codes: amount_of_bits_to_bcodes, hfe.rs:255-296.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nice_format.h"

namespace nice {

// Heap slots hold count << 32 | node id: one 64-bit LDS word, compared on the
// high word (a stream's total count is at most 3 symbols per pixel -- SC_RGB
// -- and the boundary caps frames at 2^30 pixels, so every sum fits 32 bits).
struct HeapLds {
  unsigned long long key[512];
  int16_t parent[2 * MAX_ALPHABET + 2];
};
static_assert(2 * MAX_ALPHABET < 1024 && MAX_ALPHABET < 256 + 128, "heap depth <= 8, internal nodes <= level 7");

// ---------------------------------------------------------------------------
// std BinaryHeap replay on one wave (hfe.rs:63-84; Rust library semantics:
// push = sift_up(0, len-1); pop = remove the last slot, then
// sift_down_to_bottom(0) -- the hole walks to a leaf, at every node taking the
// right child iff cnt(right) <= cnt(left) -- and sift_up of the old last
// element from there; sift_up moves while cnt(parent) > cnt(elem)).
//
// Instead of one lane stepping level by level through LDS, the wave keeps each
// internal node's walk direction ("pref" bit: 1 = right child) in registers:
//   * nodes 0..62 (levels 0..5): lane L holds node L's bit (pm), so the whole
//     top of the tree is one ballot M; lane L also holds the ancestor mask A and
//     required bits R of level-6 node 63+L, so the lane reached by the walk is
//     the one with (M & A) == R -- six levels in one compare;
//   * levels 6..7 (n <= 343: nothing deeper has children): lane L holds the
//     bits of node 63+L and its two children (P), read once by readlane.
// The path nodes' contents and siblings are then gathered in one LDS round
// (lane d = level d), the sift_up stop level is one ballot, the moves are
// parallel stores, and only the path nodes' pref bits are recomputed (their
// children are the only ones that changed; plus the parent of the removed
// last slot).  Bits of leaves and of slots past the end are don't-cares: the
// walk is cut at the deepest existing node.  Checked against the oracle on
// 20 000 random count vectors by tools/heap_model.cpp (the same steps as
// plain loops) before it was written here.
// ---------------------------------------------------------------------------
struct WaveHeap {
  HeapLds& h;
  uint32_t ln, lvl;              // lane, level of node ln (ln < 63)
  unsigned long long A, R;       // ancestors / required bits of level-6 node 63 + ln
  uint32_t pm, P;
  uint32_t len;                  // wave-uniform

  __device__ explicit WaveHeap(HeapLds& hh) : h(hh), ln(threadIdx.x & 63), pm(0), P(0), len(0) {
    lvl = 31u - (uint32_t)__clz((int)(ln + 1u));
    A = 0;
    R = 0;
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d) {
      const uint32_t anc = ((64u + ln) >> (6u - d)) - 1u, bit = ((64u + ln) >> (5u - d)) & 1u;
      A |= 1ull << anc;
      R |= (unsigned long long)bit << anc;
    }
  }
  __device__ static bool gt(unsigned long long a, unsigned long long b) {
    return (uint32_t)(a >> 32) > (uint32_t)(b >> 32);
  }

  // pref bits of the path nodes at levels [lo, hi): node at level d is
  // (x1 >> (D - d)) - 1 (x1 = deepest path node + 1, at level D), its new bit
  // is bit d of `bits`
  __device__ void apply(uint32_t x1, uint32_t D, uint32_t lo, uint32_t hi, unsigned long long bits) {
    const bool on = ln < 63u && lvl >= lo && lvl < hi && ((x1 >> ((D - lvl) & 31u)) - 1u) == ln;
    pm = on ? (uint32_t)(bits >> lvl) & 1u : pm;
    // levels 6 and 7 (scalar masks, no branches): lane r, bit 0 and bit l
    const uint32_t r = (x1 >> ((D - 6u) & 31u)) - 64u;
    const uint32_t l = 1u + ((x1 >> ((D - 7u) & 31u)) & 1u);
    const uint32_t m6 = (lo <= 6u && hi > 6u) ? 1u : 0u, m7 = (lo <= 7u && hi > 7u) ? (1u << l) : 0u;
    const uint32_t nb = ((uint32_t)(bits >> 6) & 1u) | ((((uint32_t)(bits >> 7)) & 1u) << l);
    P = ln == r ? (P & ~(m6 | m7)) | (nb & (m6 | m7)) : P;
  }
  __device__ void clear_pref(uint32_t q, bool go) {   // uniform node index (levels <= 7), no branches
    pm = (go && ln == q) ? 0u : pm;
    const uint32_t D = 31u - (uint32_t)__clz((int)(q + 1u));
    const uint32_t r = ((q + 1u) >> ((D - 6u) & 31u)) - 64u;
    const uint32_t l = (D == 7u) ? 1u + ((q + 1u) & 1u) : 0u;
    P = (go && q >= 63u && ln == r) ? (P & ~(1u << l)) : P;
  }

  __device__ unsigned long long pop() {
    const unsigned long long top = h.key[0];
    const uint32_t e = --len;
    if (e == 0) return top;
    const unsigned long long elem = h.key[e];
    clear_pref((e - 1u) >> 1, !(e & 1u));   // a right child is gone
    // the walk to the bottom
    const unsigned long long M = __ballot(pm != 0u);
    const uint32_t r6 = (uint32_t)__builtin_ctzll(__ballot((M & A) == R));
    const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)P, (int)r6);
    const uint32_t l1 = 1u + (s & 1u), l2 = 2u * l1 + 1u + ((s >> l1) & 1u);
    const uint32_t x1 = ((64u + r6) << 2) + (l2 - 3u);   // level-8 node + 1
    const uint32_t pd = (x1 >> (8u - min(ln, 8u))) - 1u;   // path node of level ln
    const uint32_t k = (uint32_t)__popcll(__ballot(ln <= 8u && pd < len)) - 1u;   // bottom level
    const uint32_t c = (x1 >> (7u - min(ln, 7u))) - 1u;    // its path child
    const uint32_t c2 = (x1 >> (6u - min(ln, 6u))) - 1u;   // and grandchild
    const uint32_t sib = (c & 1u) ? c + 1u : c - 1u;
    const unsigned long long v = h.key[c], v2 = h.key[c2], sv = h.key[sib];
    // sift_up of elem from the bottom: it rises past level d while cnt(v_d) > cnt(elem)
    const unsigned long long nb = __ballot(ln < k && !gt(v, elem));
    const uint32_t j = nb ? 64u - (uint32_t)__clzll(nb) : 0u;
    if (ln <= j) h.key[pd] = ln < j ? v : elem;
    const unsigned long long nc = ln + 1u < j ? v2 : elem;   // new content of c (ln < j)
    const bool codd = c & 1u;
    const uint32_t right = codd ? sib : c;
    const unsigned long long lv = codd ? nc : sv, rv = codd ? sv : nc;
    const unsigned long long bits = __ballot(right < len && !gt(rv, lv));
    apply(x1, 8u, 0u, j, bits);
    return top;
  }

  // push without the pref-bit upkeep (the initial pushes: no pop walks until
  // build_prefs has set every bit at once)
  __device__ void push_plain(unsigned long long x) {
    const uint32_t e = len++;
    if (e == 0) { h.key[0] = x; return; }
    const uint32_t x1 = e + 1u;
    const uint32_t D = 31u - (uint32_t)__clz((int)x1);
    const uint32_t ad = (x1 >> (D - min(ln, D))) - 1u;
    const uint32_t c = (x1 >> (D - min(ln + 1u, D))) - 1u;
    const unsigned long long old = h.key[ad];
    const unsigned long long nb = __ballot(ln < D && !gt(old, x));
    const uint32_t j = nb ? 64u - (uint32_t)__clzll(nb) : 0u;
    if (ln == j) h.key[ad] = x;
    if (ln >= j && ln < D) h.key[c] = old;
  }
  // every internal node's bit from the heap as it stands (one LDS round)
  __device__ void build_prefs() {
    auto pref = [&](uint32_t i) -> uint32_t {   // right child preferred (cnt(right) <= cnt(left))
      const uint32_t l = 2u * i + 1u, r = l + 1u;
      const unsigned long long lv = h.key[min(l, 511u)], rv = h.key[min(r, 511u)];
      return (r < len && !gt(rv, lv)) ? 1u : 0u;
    };
    pm = ln < 63u ? pref(ln) : 0u;
    P = pref(63u + ln) | pref(127u + 2u * ln) << 1 | pref(128u + 2u * ln) << 2;
  }

  __device__ void push(unsigned long long x) {
    const uint32_t e = len++;
    if (e == 0) { h.key[0] = x; return; }
    const uint32_t x1 = e + 1u;
    const uint32_t D = 31u - (uint32_t)__clz((int)x1);
    const uint32_t ad = (x1 >> (D - min(ln, D))) - 1u;          // path node of level ln
    const uint32_t c = (x1 >> (D - min(ln + 1u, D))) - 1u;      // its path child
    const uint32_t sib = (c & 1u) ? c + 1u : c - 1u;
    const unsigned long long old = h.key[ad], sv = h.key[sib];
    const unsigned long long nb = __ballot(ln < D && !gt(old, x));
    const uint32_t j = nb ? 64u - (uint32_t)__clzll(nb) : 0u;   // x's final level
    if (ln == j) h.key[ad] = x;
    if (ln >= j && ln < D) h.key[c] = old;                       // shifted one level down
    const uint32_t lo = j ? j - 1u : 0u;
    const unsigned long long nc = ln + 1u == j ? x : old;        // new content of c (ln >= lo)
    const bool codd = c & 1u;
    const uint32_t right = codd ? sib : c;
    const unsigned long long lv = codd ? nc : sv, rv = codd ? sv : nc;
    const unsigned long long bits = __ballot(right < len && !gt(rv, lv));
    apply(x1, D, lo, D, bits);
  }
};

// hfe.rs:63-84 on one wave.  counts[] has n entries.  Writes h.parent.
__device__ inline void huffman_merge_wave(HeapLds& h, const uint32_t* counts, int n) {
  WaveHeap q(h);
  for (int i = 0; i < n; ++i) q.push_plain(((unsigned long long)counts[i] << 32) | (unsigned long long)i);
  q.build_prefs();
  uint32_t next = (uint32_t)n;
  while (q.len > 2) {
    const unsigned long long a = q.pop(), b = q.pop();
    if (q.ln == 0) {
      h.parent[(uint32_t)a] = (int16_t)next;
      h.parent[(uint32_t)b] = (int16_t)next;
    }
    q.push((((a >> 32) + (b >> 32)) << 32) | next);
    ++next;
  }
}

}  // namespace nice
