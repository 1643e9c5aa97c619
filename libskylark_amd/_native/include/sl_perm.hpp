// Host-side random permutations of sketch construction, shared by the HIP
// library (perm_host.cpp, called by the Python runtime) and the C API's
// interpreter-free path (capi/native_sketch.hpp), so both draw the same
// operator from the same counter-based stream.
//   * UST without replacement (reference sketch/UST_data.hpp:81-100 draws N
//     values and shuffles): S steps of the BACKWARD Fisher-Yates (position
//     i = N-1, N-2, ... swaps with j = U{0..i} from stream slot base + i),
//     displaced entries kept in a hash map: O(S) time and memory, any N;
//   * Fastfood (sketch/FRFT_data.hpp:91-116, nb (NB - 1) draws): backward
//     Fisher-Yates per block with unbiased bounded integers (multiply-high of
//     a 64-bit word by the range).
#pragma once

#include <stdint.h>

#include <unordered_map>

#include "sl_rng.hpp"

namespace slperm {

inline void ust_noreplace(int64_t* out, uint64_t seed, uint64_t base, int64_t N, int64_t S) {
  std::unordered_map<int64_t, int64_t> moved;
  moved.reserve((size_t)(2 * S + 16));
  auto get = [&](int64_t x) {
    auto it = moved.find(x);
    return it == moved.end() ? x : it->second;
  };
  for (int64_t l = 0; l < S; ++l) {
    const int64_t i = N - 1 - l;
    const sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)i);
    const int64_t j = sl::uniform_int(b.x, 0, i);
    const int64_t wi = get(i), wj = get(j);
    moved[i] = wj;
    moved[j] = wi;
    out[l] = wj;
  }
}

// permutations of blocks [b0, b1) of nb, each of length NB, into out[b * NB ...]
inline void fastfood_perms(int64_t* out, uint64_t seed, uint64_t base, int64_t b0, int64_t b1, int64_t NB) {
  for (int64_t i = b0; i < b1; ++i) {
    int64_t* w = out + i * NB;
    for (int64_t c = 0; c < NB; ++c) w[c] = c;
    for (int64_t l = 0; l < NB - 1; ++l) {
      const int64_t j = NB - 1 - l;
      const sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)(i * (NB - 1) + l));
      const int64_t k = (int64_t)sl::mulhi64(b.x, (uint64_t)(j + 1));
      const int64_t t = w[j];
      w[j] = w[k];
      w[k] = t;
    }
  }
}

}  // namespace slperm
