// pf_desc_tag.hpp — the tag of a batch stream descriptor (pfmpe_step_multi), shared by the host and the device.
//
// The host writes every stream's descriptor (StreamDesc: the frame arguments and the stream's buffer pointers)
// into a pinned image; the staging kernel copies it to HBM.  The host also stores in the descriptor the batch
// generation (a counter of staging launches, passed to every kernel of the round as an argument) and a tag
// over all the descriptor's 8-byte words before the tag.  The staging kernel recomputes the tag over the words
// it actually read and checks the generation against its argument: a descriptor mixed with stale words, or a
// whole stale descriptor of an earlier round, is caught before any of its pointers is used.
//
// tag = XOR over words i of tag_mix(word_i, i).  tag_mix is a bijection of the word for each position (an add,
// then splitmix64's xorshift-multiply steps, each invertible), so changing any single word changes its term and
// therefore the tag, with certainty; several changed words cancel only by a 2^-64 coincidence.  The XOR lets
// the device compute the terms in any lanes and combine them in any order.
//
// Plain C++ (tests/test_desc_tag.py builds it with g++) and HIP.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PF_TAG_HD __host__ __device__ __forceinline__
#else
#define PF_TAG_HD inline
#endif

namespace pfmpe {

PF_TAG_HD uint64_t tag_mix(uint64_t w, uint32_t i) {
  uint64_t z = w + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1u);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

PF_TAG_HD uint64_t desc_tag(const uint64_t* words, int n) {
  uint64_t h = 0;
  for (int i = 0; i < n; ++i) h ^= tag_mix(words[i], (uint32_t)i);
  return h;
}

}  // namespace pfmpe
