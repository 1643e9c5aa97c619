// Native (interpreter-free) C API path for the reference's core sketches:
// JLT, CT (dense transforms, sketch/dense_transform_data.hpp) and CWT, MMT,
// WZT (hash transforms, sketch/hash_transform_data.hpp) on host column-major
// double matrices ("Matrix"), plus their JSON (de)serialisation.  FJLT is a
// native object too (its device application is native_device.hpp's).
//
// Same parameters as the Python / GPU runtime, drawn from the same
// counter-based streams (sl_rng.hpp: Threefry-2x64-13, sample_d /
// uniform_int), so a sketch created here, serialised and loaded by the
// Python runtime (or the other way round) is the same operator:
//   dense : entries[i, k] = scale * dist(seed, base + k S + i),
//           base = creation counter, counter += N S
//   hash  : idx[k] = UniformInt(0, S - 1) at counter + k (counter += N),
//           values: CWT Rademacher / MMT Cauchy (counter += N), WZT
//           Exp e then Rademacher sign (counter += 2N), v = sign (1/e)^(1/p).
// Application: S x K panels of the dense operator realised on the fly (never
// the whole S x N), contiguous inner loops, row blocks over std::threads.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sl_rng.hpp"

namespace slnat {

struct Sketch {
  std::string type;
  int64_t N = 0, S = 0;
  uint64_t seed = 0, ctr0 = 0;
  double param = 0.0;        // CT: C, WZT: p
  bool dense = false;
  int dist = sl::DIST_NORMAL;
  double scale = 1.0;
  std::vector<int64_t> idx;  // hash
  std::vector<double> val;   // hash
};

inline bool supported(const char* t) {
  return !strcmp(t, "JLT") || !strcmp(t, "CT") || !strcmp(t, "CWT") || !strcmp(t, "MMT") || !strcmp(t, "WZT") ||
         !strcmp(t, "FJLT");
}

// host "Matrix" application is native for all but FJLT (its host path is the runtime's)
inline bool host_apply(const Sketch& s) { return s.type != "FJLT"; }

inline bool takes_param(const std::string& t) { return t == "CT" || t == "WZT"; }

// Derive the operator from (type, N, S, seed, counter, param); returns the
// counter after the sketch's draws.
inline uint64_t build(Sketch& s) {
  uint64_t c = s.ctr0;
  if (s.type == "FJLT") {
    // FJLT_data: N Rademacher signs (D), then S uniform frequencies; the
    // operator is realised on the device from (seed, ctr0, ctr0 + N)
    s.dense = false;
    return c + (uint64_t)(s.N + s.S);
  }
  if (s.type == "JLT" || s.type == "CT") {
    s.dense = true;
    s.dist = s.type == "JLT" ? sl::DIST_NORMAL : sl::DIST_CAUCHY;
    s.scale = s.type == "JLT" ? std::sqrt(1.0 / (double)s.S) : s.param / (double)s.S;
    return c + (uint64_t)(s.N * s.S);
  }
  s.dense = false;
  s.idx.resize((size_t)s.N);
  s.val.resize((size_t)s.N);
  for (int64_t k = 0; k < s.N; ++k) s.idx[k] = sl::uniform_int(sl::stream_block(s.seed, c + k).x, 0, s.S - 1);
  c += (uint64_t)s.N;
  if (s.type == "WZT") {
    std::vector<double> e((size_t)s.N);
    for (int64_t k = 0; k < s.N; ++k) e[k] = sl::sample_d(sl::DIST_EXPONENTIAL, s.seed, c + k, 0.0, 0.0);
    c += (uint64_t)s.N;
    for (int64_t k = 0; k < s.N; ++k) {
      const double sg = sl::sample_d(sl::DIST_RADEMACHER, s.seed, c + k, 0.0, 0.0);
      s.val[k] = sg * std::pow(1.0 / e[k], 1.0 / s.param);
    }
    c += (uint64_t)s.N;
  } else {
    const int d = s.type == "CWT" ? sl::DIST_RADEMACHER : sl::DIST_CAUCHY;
    for (int64_t k = 0; k < s.N; ++k) s.val[k] = sl::sample_d(d, s.seed, c + k, 0.0, 0.0);
    c += (uint64_t)s.N;
  }
  return c;
}

inline std::string fmt_double(double v) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.17g", v);
  std::string r(buf);
  if (r.find_first_of(".eEn") == std::string::npos) r += ".0";   // keep it a JSON float
  return r;
}

// Same schema as the Python runtime (sketch/base.py to_dict) and the reference.
inline std::string to_json(const Sketch& s) {
  std::string j = "{\"skylark_object_type\": \"sketch\", \"sketch_type\": \"" + s.type +
                  "\", \"skylark_version\": \"0.1.0\", \"N\": " + std::to_string(s.N) +
                  ", \"S\": " + std::to_string(s.S) +
                  ", \"creation_context\": {\"skylark_object_type\": \"context\", \"skylark_version\": \"0.1.0\", "
                  "\"seed\": " + std::to_string(s.seed) + ", \"counter\": " + std::to_string(s.ctr0) + "}";
  if (s.type == "CT") j += ", \"C\": " + fmt_double(s.param);
  if (s.type == "WZT") j += ", \"P\": " + fmt_double(s.param);
  return j + "}";
}

// --- minimal JSON field extraction (flat keys; the nested context keys are unique)
inline const char* find_key(const char* js, const char* key) {
  std::string pat = std::string("\"") + key + "\"";
  const char* p = strstr(js, pat.c_str());
  if (!p) return nullptr;
  p += pat.size();
  while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
  if (*p != ':') return nullptr;
  ++p;
  while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
  return p;
}

inline bool get_string(const char* js, const char* key, std::string& out) {
  const char* p = find_key(js, key);
  if (!p || *p != '"') return false;
  const char* q = strchr(p + 1, '"');
  if (!q) return false;
  out.assign(p + 1, q);
  return true;
}

inline bool get_number(const char* js, const char* key, double& out) {
  const char* p = find_key(js, key);
  if (!p) return false;
  char* end = nullptr;
  out = strtod(p, &end);
  return end != p;
}

inline bool get_u64(const char* js, const char* key, uint64_t& out) {
  const char* p = find_key(js, key);
  if (!p) return false;
  char* end = nullptr;
  out = strtoull(p, &end, 10);
  return end != p;
}

// Parse a serialised sketch of a natively supported type; false -> caller
// falls back to the Python runtime.
inline bool from_json(const char* js, Sketch& s) {
  std::string t;
  double N, S;
  if (!get_string(js, "sketch_type", t) || !supported(t.c_str())) return false;
  if (!get_number(js, "N", N) || !get_number(js, "S", S)) return false;
  if (!get_u64(js, "seed", s.seed) || !get_u64(js, "counter", s.ctr0)) return false;
  s.type = t;
  s.N = (int64_t)N;
  s.S = (int64_t)S;
  s.param = 1.0;
  if (t == "CT") {
    if (!get_number(js, "C", s.param)) s.param = 1.0;
  } else if (t == "WZT") {
    if (!get_number(js, "P", s.param) && !get_number(js, "p", s.param)) s.param = 1.0;
  }
  build(s);
  return true;
}

template <typename F>
inline void parallel_for(int64_t n, F&& f) {
  unsigned nt = std::thread::hardware_concurrency();
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;
  if (n < 2 * (int64_t)nt) nt = 1;
  if (nt == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t ch = (n + nt - 1) / nt;
  for (unsigned i = 0; i < nt; ++i) {
    const int64_t lo = i * ch, hi = lo + ch < n ? lo + ch : n;
    if (lo < hi) th.emplace_back(f, lo, hi);
  }
  for (auto& t : th) t.join();
}

// Realise the dense operator's columns [k0, k0 + kb) as a col-major S x kb panel.
inline void realise_panel(const Sketch& s, int64_t k0, int64_t kb, double* P) {
  parallel_for(kb, [&](int64_t lo, int64_t hi) {
    for (int64_t kk = lo; kk < hi; ++kk)
      for (int64_t i = 0; i < s.S; ++i)
        P[i + kk * s.S] = s.scale * sl::sample_d(s.dist, s.seed, s.ctr0 + (uint64_t)((k0 + kk) * s.S + i), 0.0, 0.0);
  });
}

// SA = S A (dim 0: A is N x n) or A S^T (dim 1: A is m x N); host col-major,
// SA overwritten.  Returns 104 on a dimension mismatch (host_apply(s) only).
inline int apply(const Sketch& s, const double* A, int64_t am, int64_t an, double* SA, int64_t sm, int64_t sn,
                 int dim) {
  if (dim == 0) {
    if (am != s.N || sm != s.S || sn != an) return 104;
    std::memset(SA, 0, sizeof(double) * (size_t)(sm * sn));
    if (s.dense) {
      const int64_t KB = 256;
      std::vector<double> P((size_t)(s.S * KB));
      for (int64_t k0 = 0; k0 < s.N; k0 += KB) {
        const int64_t kb = s.N - k0 < KB ? s.N - k0 : KB;
        realise_panel(s, k0, kb, P.data());
        parallel_for(an, [&](int64_t lo, int64_t hi) {
          for (int64_t j = lo; j < hi; ++j) {
            double* out = SA + j * s.S;
            for (int64_t kk = 0; kk < kb; ++kk) {
              const double a = A[(k0 + kk) + j * am];
              const double* p = P.data() + kk * s.S;
              for (int64_t i = 0; i < s.S; ++i) out[i] += p[i] * a;
            }
          }
        });
      }
    } else {
      parallel_for(an, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j)
          for (int64_t k = 0; k < s.N; ++k) SA[s.idx[k] + j * s.S] += s.val[k] * A[k + j * am];
      });
    }
    return 0;
  }
  if (an != s.N || sn != s.S || sm != am) return 104;
  std::memset(SA, 0, sizeof(double) * (size_t)(sm * sn));
  if (s.dense) {
    const int64_t KB = 256;
    std::vector<double> P((size_t)(s.S * KB));
    for (int64_t k0 = 0; k0 < s.N; k0 += KB) {
      const int64_t kb = s.N - k0 < KB ? s.N - k0 : KB;
      realise_panel(s, k0, kb, P.data());
      parallel_for(s.S, [&](int64_t lo, int64_t hi) {
        for (int64_t c = lo; c < hi; ++c) {
          double* out = SA + c * am;
          for (int64_t kk = 0; kk < kb; ++kk) {
            const double b = P[c + kk * s.S];
            const double* a = A + (k0 + kk) * am;
            for (int64_t i = 0; i < am; ++i) out[i] += a[i] * b;
          }
        }
      });
    }
  } else {
    // column k of A lands in column idx[k] of SA: split the work by output column
    parallel_for(s.S, [&](int64_t lo, int64_t hi) {
      for (int64_t k = 0; k < s.N; ++k) {
        const int64_t c = s.idx[k];
        if (c < lo || c >= hi) continue;
        double* out = SA + c * am;
        const double* a = A + k * am;
        const double v = s.val[k];
        for (int64_t i = 0; i < am; ++i) out[i] += v * a[i];
      }
    });
  }
  return 0;
}

}  // namespace slnat
