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

// One heap slot: count in the high 32 bits would not be enough for very large
// frames, so keep the full u64 count and a node id side by side.
struct HeapLds {
  unsigned long long cnt[MAX_ALPHABET + 1];
  int16_t node[MAX_ALPHABET + 1];
  int16_t parent[2 * MAX_ALPHABET + 2];
  uint8_t aob[MAX_ALPHABET + 1];
  uint16_t order[MAX_ALPHABET + 1];     // symbols in (aob desc, symbol desc) order
};

// std BinaryHeap::sift_up(start, pos): moves up while elem.cnt < parent.cnt.
__device__ inline void heap_sift_up(HeapLds& h, int start, int pos) {
  const unsigned long long ec = h.cnt[pos];
  const int16_t en = h.node[pos];
  while (pos > start) {
    const int parent = (pos - 1) >> 1;
    const unsigned long long pc = h.cnt[parent];
    if (pc <= ec) break;
    h.cnt[pos] = pc;
    h.node[pos] = h.node[parent];
    pos = parent;
  }
  h.cnt[pos] = ec;
  h.node[pos] = en;
}

// std BinaryHeap::sift_down_to_bottom(0) followed by sift_up.
__device__ inline void heap_sift_down_to_bottom(HeapLds& h, int len) {
  const unsigned long long ec = h.cnt[0];
  const int16_t en = h.node[0];
  int pos = 0;
  int child = 1;
  while (len >= 2 && child <= len - 2) {
    const unsigned long long lc = h.cnt[child], rc = h.cnt[child + 1];
    if (rc <= lc) child += 1;
    h.cnt[pos] = h.cnt[child];
    h.node[pos] = h.node[child];
    pos = child;
    child = 2 * pos + 1;
  }
  if (child == len - 1) {
    h.cnt[pos] = h.cnt[child];
    h.node[pos] = h.node[child];
    pos = child;
  }
  h.cnt[pos] = ec;
  h.node[pos] = en;
  heap_sift_up(h, 0, pos);
}

// Serial heap replay by one lane.  counts[] has n entries.  Writes h.parent.
__device__ inline void huffman_merge_tree(HeapLds& h, const uint32_t* counts, int n) {
  int len = 0;
  for (int i = 0; i < n; ++i) {
    h.cnt[len] = counts[i];
    h.node[len] = (int16_t)i;
    ++len;
    heap_sift_up(h, 0, len - 1);
  }
  int next = n;
  while (len > 2) {
    // pop #1
    --len;
    unsigned long long ac = h.cnt[0];
    int16_t an = h.node[0];
    h.cnt[0] = h.cnt[len];
    h.node[0] = h.node[len];
    heap_sift_down_to_bottom(h, len);
    // pop #2
    --len;
    unsigned long long bc;
    int16_t bn;
    if (len > 0) {
      bc = h.cnt[0];
      bn = h.node[0];
      h.cnt[0] = h.cnt[len];
      h.node[0] = h.node[len];
      heap_sift_down_to_bottom(h, len);
    } else {
      bc = h.cnt[0];
      bn = h.node[0];
    }
    const int16_t id = (int16_t)next++;
    h.parent[an] = id;
    h.parent[bn] = id;
    h.cnt[len] = ac + bc;
    h.node[len] = id;
    ++len;
    heap_sift_up(h, 0, len - 1);
  }
}

}  // namespace nice
