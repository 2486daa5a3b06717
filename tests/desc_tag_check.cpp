// CPU check of the batch descriptor tag (pf_desc_tag.hpp), built by tests/test_desc_tag.py with g++:
// prints the tag of a fixed word sequence, then verifies that every single-word change (each word, several
// values) and random multi-word changes alter the tag.  Exit 0 on success.
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "../pf_monocular_pose_estimator_amd/csrc/pf_desc_tag.hpp"

int main() {
  const int n = 130;  // about one StreamDesc<float, __half> (tag words)
  std::vector<uint64_t> w(n);
  for (int i = 0; i < n; ++i) w[i] = 0x0123456789abcdefull * (uint64_t)(i + 1) ^ (uint64_t)i << 7;
  const uint64_t t0 = pfmpe::desc_tag(w.data(), n);
  std::printf("%016llx\n", (unsigned long long)t0);
  std::mt19937_64 rng(42);
  long checked = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t keep = w[i];
    const uint64_t deltas[] = {1ull, 1ull << 63, 0xffffffffull, rng(), rng(), ~0ull};
    for (uint64_t d : deltas) {
      w[i] = keep ^ d;
      if (pfmpe::desc_tag(w.data(), n) == t0) {
        std::printf("single-word change not detected at %d\n", i);
        return 1;
      }
      ++checked;
    }
    w[i] = keep;
  }
  for (int r = 0; r < 20000; ++r) {
    std::vector<uint64_t> v = w;
    const int k = 2 + (int)(rng() % 6);
    for (int j = 0; j < k; ++j) v[rng() % n] ^= rng() | 1ull;
    if (v != w && pfmpe::desc_tag(v.data(), n) == t0) {
      std::printf("multi-word change not detected (round %d)\n", r);
      return 1;
    }
    ++checked;
  }
  std::printf("ok %ld\n", checked);
  return 0;
}
