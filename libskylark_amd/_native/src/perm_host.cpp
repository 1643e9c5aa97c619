// Host-side random permutations for sketch construction (replaces O(N)
// Python loops).  Reference: UST without replacement draws N random values
// and runs Fisher-Yates (sketch/UST_data.hpp:81-100); the Fastfood data draws
// nb (NB - 1) integers for nb Fisher-Yates permutations of length NB
// (sketch/FRFT_data.hpp:91-116).  The context counter accounting is the
// reference's (N slots, resp. nb (NB - 1) slots), the samplers are ours:
//   * UST: S steps of the BACKWARD Fisher-Yates (position i = N-1, N-2, ...
//     swaps with j = U{0..i} from stream slot base + i), kept in a hash map of
//     displaced entries: O(S) time and memory, any N;
//   * Fastfood: backward Fisher-Yates per block with unbiased bounded
//     integers (multiply-high of a 64-bit word by the range, bias < range /
//     2^64 -- no modulo bias).
#include <stdint.h>

#include <thread>
#include <unordered_map>
#include <vector>

#include "sl_common.hpp"
#include "sl_rng.hpp"

SL_API int sl_ust_noreplace_host(int64_t* out, uint64_t seed, uint64_t base, int64_t N, int64_t S) {
  if (S < 0 || S > N) {
    sl_set_last_error("UST without replacement needs 0 <= S <= N");
    return SL_ERR_INVALID;
  }
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
  return SL_OK;
}

SL_API int sl_fastfood_perms_host(int64_t* out, uint64_t seed, uint64_t base, int64_t nb, int64_t NB) {
  if (nb <= 0 || NB <= 0) return SL_OK;
  auto work = [&](int64_t b0, int64_t b1) {
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
  };
  const int64_t work_items = nb * NB;
  unsigned nt = work_items > (1 << 16) ? std::thread::hardware_concurrency() : 1;
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;
  if ((int64_t)nt > nb) nt = (unsigned)nb;
  if (nt <= 1) {
    work(0, nb);
    return SL_OK;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (nb + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const int64_t lo = t * chunk, hi = lo + chunk < nb ? lo + chunk : nb;
    if (lo < hi) th.emplace_back(work, lo, hi);
  }
  for (auto& t : th) t.join();
  return SL_OK;
}
