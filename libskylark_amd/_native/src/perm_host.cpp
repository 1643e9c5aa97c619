// Host-side random permutations for sketch construction (replaces O(N)
// Python loops); the samplers themselves live in sl_perm.hpp, shared with the
// C API's interpreter-free path.
#include <stdint.h>

#include <thread>
#include <vector>

#include "sl_common.hpp"
#include "sl_perm.hpp"

SL_API int sl_ust_noreplace_host(int64_t* out, uint64_t seed, uint64_t base, int64_t N, int64_t S) {
  if (S < 0 || S > N) {
    sl_set_last_error("UST without replacement needs 0 <= S <= N");
    return SL_ERR_INVALID;
  }
  slperm::ust_noreplace(out, seed, base, N, S);
  return SL_OK;
}

SL_API int sl_fastfood_perms_host(int64_t* out, uint64_t seed, uint64_t base, int64_t nb, int64_t NB) {
  if (nb <= 0 || NB <= 0) return SL_OK;
  const int64_t work_items = nb * NB;
  unsigned nt = work_items > (1 << 16) ? std::thread::hardware_concurrency() : 1;
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;
  if ((int64_t)nt > nb) nt = (unsigned)nb;
  if (nt <= 1) {
    slperm::fastfood_perms(out, seed, base, 0, nb, NB);
    return SL_OK;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (nb + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const int64_t lo = t * chunk, hi = lo + chunk < nb ? lo + chunk : nb;
    if (lo < hi) th.emplace_back(slperm::fastfood_perms, out, seed, base, lo, hi, NB);
  }
  for (auto& t : th) t.join();
  return SL_OK;
}
