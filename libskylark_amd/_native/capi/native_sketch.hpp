// Native (interpreter-free) sketch objects of the C API: every sketch type of
// the runtime (sketch/*.py; reference sketch/*_data.hpp) is created,
// serialised, deserialised and applied here without CPython, drawing its
// parameters from the same counter-based streams (sl_rng.hpp:
// Threefry-2x64-13, sample_d / uniform_int) in the same order as the runtime,
// so a sketch made here and one made by the Python runtime on the same
// context (or loaded from the other's JSON) are the same operator.
//
// Kinds (how the operator is represented):
//   DENSE    entries scale * dist(seed, wbase + k S + i): JLT, CT, SJLT and
//            the W of GaussianRFT / LaplacianRFT / MaternRFT / ExpSemigroupRLT
//   QMC      W[i][j] = inscale * quantile(leaped Halton point skip + i,
//            coordinate j): GaussianQRFT, LaplacianQRFT, ExpSemigroupQRLT
//   FJLT     sqrt(N/S) * (sampled rows of the orthonormal DCT-II) * diag(D)
//   FASTFOOD per block F[0:e-s] diag(G) F[perm] diag(B) (FastGaussianRFT,
//            FastMaternRFT; Sm applied as the epilogue's per-feature scale)
//   HASH     CWT / MMT / WZT: one bucket and one value per input coordinate
//   SAMPLE   UST / NURST: output i = input samples[i]
//   PPT      TensorSketch: q CountSketches + the homogeneous term, circular
//            convolution of the q sketches
// Feature maps add an epilogue: outscale * cos(scales * x + shifts) (RFT,
// QRFT, Fastfood) or outscale * exp(-x) (RLT, QRLT).
//
// This header holds the parameters, the JSON and the host application
// (column-major double "Matrix", std::threads); the device application of the
// same objects is native_device.hpp's.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "sl_perm.hpp"
#include "sl_rng.hpp"

namespace slnat {

enum Kind { K_DENSE, K_QMC, K_FJLT, K_FASTFOOD, K_HASH, K_SAMPLE, K_PPT };
enum Epi { EPI_NONE = -1, EPI_COS = 0, EPI_EXP = 1 };
enum Quant { Q_NORMAL, Q_CAUCHY, Q_LEVY };

constexpr double kPi = 3.14159265358979323846;

struct Sketch {
  std::string type;
  int64_t N = 0, S = 0;
  uint64_t seed = 0, ctr0 = 0;
  // parameters as serialised
  double C = 1.0, P = 1.0, density = 1.0 / 3.0, sigma = 1.0, nu = 1.5, l = 1.0, beta = 1.0, c = 1.0, gamma = 1.0;
  int64_t skip = 0, q = 3, seq_d = -1, leap = -1;
  bool replace = true;
  std::vector<double> probs;   // NURST
  // derived operator
  int kind = K_DENSE;
  int dist = sl::DIST_NORMAL;
  double p0 = 0.0, scale = 1.0;   // DENSE: scale * dist(seed, wbase + k S + i, p0); QMC: inscale
  uint64_t wbase = 0;
  int quant = Q_NORMAL;
  std::vector<int64_t> primes;    // QMC: prime(j), j < N + 1
  int epi = EPI_NONE;
  double outscale = 1.0;
  std::vector<double> shifts, scales;  // epilogue (empty: none)
  std::vector<int64_t> idx;            // HASH buckets
  std::vector<double> val;             // HASH values
  std::vector<int64_t> samples;        // SAMPLE / FJLT rows
  std::vector<double> dsign;           // FJLT D
  int64_t nb = 0;                      // FASTFOOD blocks (block size N)
  std::vector<double> fB, fG;          // nb x N
  std::vector<int64_t> perms;          // nb x N
  std::vector<int64_t> pidx;           // PPT: q x N buckets
  std::vector<double> pval;            // PPT: q x N signs
  std::vector<int64_t> hidx;           // PPT: q homogeneous buckets
  std::vector<double> hval;            // PPT: q homogeneous signs
};

// ------------------------------------------------------------ type table
inline const char* const* all_types() {
  static const char* const t[] = {"JLT", "CT", "SJLT", "CWT", "MMT", "WZT", "FJLT", "UST", "NURST",
                                  "GaussianRFT", "LaplacianRFT", "MaternRFT", "GaussianQRFT", "LaplacianQRFT",
                                  "ExpSemigroupRLT", "ExpSemigroupQRLT", "FastGaussianRFT", "FastMaternRFT",
                                  "PPT", nullptr};
  return t;
}

inline bool supported(const char* t) {
  for (const char* const* p = all_types(); *p; ++p)
    if (!strcmp(*p, t)) return true;
  return false;
}

// C varargs of sl_create_sketch_transform per type ('d' double, 'i' int),
// the reference's csketch.cpp order (same table as capi.py _PARAMS)
inline const char* vararg_spec(const std::string& t) {
  if (t == "CT" || t == "WZT" || t == "GaussianRFT" || t == "LaplacianRFT" || t == "ExpSemigroupRLT" ||
      t == "FastGaussianRFT")
    return "d";
  if (t == "MaternRFT" || t == "FastMaternRFT") return "dd";
  if (t == "GaussianQRFT" || t == "LaplacianQRFT" || t == "ExpSemigroupQRLT") return "di";
  if (t == "PPT") return "idd";
  return "";
}

// store the varargs (in vararg_spec order) into the parameter fields
inline void set_params(Sketch& s, const double* d, const int64_t* iv) {
  const std::string& t = s.type;
  if (t == "CT") s.C = d[0];
  else if (t == "WZT") s.P = d[0];
  else if (t == "GaussianRFT" || t == "LaplacianRFT" || t == "FastGaussianRFT") s.sigma = d[0];
  else if (t == "ExpSemigroupRLT") s.beta = d[0];
  else if (t == "MaternRFT" || t == "FastMaternRFT") { s.nu = d[0]; s.l = d[1]; }
  else if (t == "GaussianQRFT" || t == "LaplacianQRFT") { s.sigma = d[0]; s.skip = iv[1]; }
  else if (t == "ExpSemigroupQRLT") { s.beta = d[0]; s.skip = iv[1]; }
  else if (t == "PPT") { s.q = iv[0]; s.c = d[1]; s.gamma = d[2]; }
}

// -------------------------------------------------------------- math
inline std::vector<int64_t> first_primes(int64_t n) {
  std::vector<int64_t> ps;
  if (n <= 0) return ps;
  int64_t limit = std::max<int64_t>(16, (int64_t)((double)n * (std::log((double)n + 2) + std::log(std::log((double)n + 3)) + 3)));
  while ((int64_t)ps.size() < n) {
    ps.clear();
    std::vector<char> sieve((size_t)limit + 1, 1);
    sieve[0] = sieve[1] = 0;
    for (int64_t i = 2; i * i <= limit; ++i)
      if (sieve[(size_t)i])
        for (int64_t j = i * i; j <= limit; j += i) sieve[(size_t)j] = 0;
    for (int64_t i = 2; i <= limit && (int64_t)ps.size() < n; ++i)
      if (sieve[(size_t)i]) ps.push_back(i);
    limit *= 2;
  }
  return ps;
}

// radical inverse of the (already 1-based) integer k, the runtime's
// quasirand._ri_vec evaluation order
inline double radical_inverse1(int64_t base, int64_t k) {
  double r = 0.0, m = 1.0 / (double)base;
  while (k > 0) {
    r += m * (double)(k % base);
    k /= base;
    m /= (double)base;
  }
  return r;
}

// Acklam's normal quantile (|rel err| < 1.2e-9): the initial guess of erfinv
inline double norm_quantile_guess(double p) {
  static const double a[] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                             1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
  static const double b[] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                             6.680131188771972e+01, -1.328068155288572e+01};
  static const double cc[] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                              -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
  static const double d[] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                             3.754408661907416e+00};
  if (p < 0.02425) {
    const double qq = std::sqrt(-2 * std::log(p));
    return (((((cc[0] * qq + cc[1]) * qq + cc[2]) * qq + cc[3]) * qq + cc[4]) * qq + cc[5]) /
           ((((d[0] * qq + d[1]) * qq + d[2]) * qq + d[3]) * qq + 1);
  }
  if (p > 1 - 0.02425) return -norm_quantile_guess(1 - p);
  const double qq = p - 0.5, r = qq * qq;
  return (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * qq /
         (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
}

// inverse error function to f64 accuracy: Acklam guess + Newton steps on
// erf (erfc in the tails, where 1 - |y| is exact)
inline double erfinv(double y) {
  if (y <= -1.0) return -HUGE_VAL;
  if (y >= 1.0) return HUGE_VAL;
  if (y == 0.0) return 0.0;
  const double ay = std::fabs(y), tail = 1.0 - ay;
  double x = -norm_quantile_guess(0.5 * tail) * 0.70710678118654752440;
  for (int it = 0; it < 3; ++it) {
    const double f = ay > 0.5 ? tail - std::erfc(x) : std::erf(x) - ay;
    x -= f / (1.12837916709551257390 * std::exp(-x * x));
  }
  return y < 0 ? -x : x;
}

inline double quantile(int qd, double u) {
  if (qd == Q_NORMAL) return 1.41421356237309504880 * erfinv(2 * u - 1);
  if (qd == Q_CAUCHY) return std::tan(kPi * (u - 0.5));
  const double v = erfinv(1 - u);   // erfc^{-1}(u)
  return 1.0 / (2 * v * v);
}

// QMC coordinate j of point idx (idx = skip + i)
inline double qmc_coord(const Sketch& s, int64_t idx, int64_t j) {
  return radical_inverse1(s.primes[(size_t)j], idx * s.leap + 1);
}

inline double qmc_entry(const Sketch& s, int64_t i, int64_t j) {
  double u = qmc_coord(s, s.skip + i, j);
  u = std::min(std::max(u, 1e-16), 1.0 - 1e-16);
  return s.scale * quantile(s.quant, u);
}

// ------------------------------------------------------------- build
inline double draw(const Sketch& s, int d, uint64_t slot, double a = 0.0, double b = 0.0) {
  return sl::sample_d(d, s.seed, slot, a, b);
}

inline int64_t draw_int(const Sketch& s, uint64_t slot, int64_t lo, int64_t hi) {
  return sl::uniform_int(sl::stream_block(s.seed, slot).x, lo, hi);
}

inline bool is_feature_map(const std::string& t) {
  return t.find("RFT") != std::string::npos || t.find("RLT") != std::string::npos;
}

// Derive the operator from (type, N, S, seed, counter, parameters); returns
// the counter after the sketch's draws, or 0 with err set on bad parameters.
inline uint64_t build(Sketch& s, std::string* err = nullptr) {
  auto bad = [&](const char* m) -> uint64_t {
    if (err) *err = m;
    return 0;
  };
  const std::string& t = s.type;
  const int64_t N = s.N, S = s.S;
  uint64_t c = s.ctr0;
  s.shifts.clear();
  s.scales.clear();
  s.epi = EPI_NONE;
  if (t == "JLT" || t == "CT" || t == "SJLT" || t == "GaussianRFT" || t == "LaplacianRFT" || t == "MaternRFT" ||
      t == "ExpSemigroupRLT") {
    s.kind = K_DENSE;
    s.wbase = c;
    s.p0 = 0.0;
    if (t == "JLT") { s.dist = sl::DIST_NORMAL; s.scale = std::sqrt(1.0 / (double)S); }
    else if (t == "CT") { s.dist = sl::DIST_CAUCHY; s.scale = s.C / (double)S; }
    else if (t == "SJLT") {
      if (!(s.density > 0.0 && s.density <= 1.0)) return bad("SJLT density must be in (0, 1]");
      s.dist = sl::DIST_SPARSE_SIGN; s.p0 = s.density; s.scale = std::sqrt(1.0 / (double)S);
    } else if (t == "GaussianRFT") { s.dist = sl::DIST_NORMAL; s.scale = 1.0 / s.sigma; }
    else if (t == "LaplacianRFT") { s.dist = sl::DIST_CAUCHY; s.scale = 1.0 / s.sigma; }
    else if (t == "MaternRFT") { s.dist = sl::DIST_NORMAL; s.scale = 1.0 / s.l; }
    else { s.dist = sl::DIST_LEVY; s.scale = s.beta * s.beta / 2; }
    c += (uint64_t)(N * S);
    if (t == "ExpSemigroupRLT") {
      s.epi = EPI_EXP;
      s.outscale = std::sqrt(1.0 / (double)S);
    } else if (t != "JLT" && t != "CT" && t != "SJLT") {
      s.epi = EPI_COS;
      s.outscale = std::sqrt(2.0 / (double)S);
      s.shifts.resize((size_t)S);
      for (int64_t i = 0; i < S; ++i) s.shifts[(size_t)i] = draw(s, sl::DIST_UNIFORM, c + i, 0.0, 2 * kPi);
      c += (uint64_t)S;
      if (t == "MaternRFT") {
        s.scales.resize((size_t)S);
        for (int64_t i = 0; i < S; ++i)
          s.scales[(size_t)i] = std::sqrt(2.0 * s.nu / draw(s, sl::DIST_CHISQ, c + i, 2 * s.nu));
        c += (uint64_t)S;
      }
    }
    return c;
  }
  if (t == "GaussianQRFT" || t == "LaplacianQRFT" || t == "ExpSemigroupQRLT") {
    s.kind = K_QMC;
    const bool rlt = t == "ExpSemigroupQRLT";
    const int64_t extra = rlt ? 0 : 1;
    if (s.seq_d < 0) s.seq_d = N + extra;
    s.primes = first_primes(std::max<int64_t>(N + 1, s.seq_d + 1));
    if (s.leap <= 0) s.leap = s.primes[(size_t)s.seq_d];
    s.quant = t == "GaussianQRFT" ? Q_NORMAL : t == "LaplacianQRFT" ? Q_CAUCHY : Q_LEVY;
    if (rlt) {
      s.scale = s.beta * s.beta / 2;
      s.epi = EPI_EXP;
      s.outscale = std::sqrt(1.0 / (double)S);
    } else {
      s.scale = 1.0 / s.sigma;
      s.epi = EPI_COS;
      s.outscale = std::sqrt(2.0 / (double)S);
      s.shifts.resize((size_t)S);
      for (int64_t i = 0; i < S; ++i) s.shifts[(size_t)i] = 2 * kPi * qmc_coord(s, s.skip + i, N);
    }
    return c;   // QMC features draw nothing from the stream
  }
  if (t == "FJLT") {
    s.kind = K_FJLT;
    s.dsign.resize((size_t)N);
    for (int64_t i = 0; i < N; ++i) s.dsign[(size_t)i] = draw(s, sl::DIST_RADEMACHER, c + i);
    c += (uint64_t)N;
    s.samples.resize((size_t)S);
    for (int64_t j = 0; j < S; ++j) s.samples[(size_t)j] = draw_int(s, c + j, 0, N - 1);
    c += (uint64_t)S;
    s.scale = std::sqrt((double)N / (double)S);
    return c;
  }
  if (t == "UST" || t == "NURST") {
    s.kind = K_SAMPLE;
    s.samples.resize((size_t)S);
    if (t == "NURST") {
      if ((int64_t)s.probs.size() != N) return bad("size of probability array should be exactly n");
      double tot = 0.0;
      for (double p : s.probs) {
        if (p < 0) return bad("p must be a non-negative, non-zero vector");
        tot += p;
      }
      if (!(tot > 0)) return bad("p must be a non-negative, non-zero vector");
      std::vector<double> cdf((size_t)N);
      double acc = 0.0;
      for (int64_t i = 0; i < N; ++i) {
        s.probs[(size_t)i] /= tot;
        acc += s.probs[(size_t)i];
        cdf[(size_t)i] = acc;
      }
      cdf[(size_t)N - 1] = 1.0;
      for (int64_t j = 0; j < S; ++j) {
        const double u = draw(s, sl::DIST_UNIFORM, c + j, 0.0, 1.0);
        const int64_t k = (int64_t)(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
        s.samples[(size_t)j] = std::min<int64_t>(k, N - 1);
      }
      return c + (uint64_t)S;
    }
    if (s.replace) {
      for (int64_t j = 0; j < S; ++j) s.samples[(size_t)j] = draw_int(s, c + j, 0, N - 1);
      return c + (uint64_t)S;
    }
    if (S > N) return bad("UST without replacement needs S <= N");
    slperm::ust_noreplace(s.samples.data(), s.seed, c, N, S);
    return c + (uint64_t)N;
  }
  if (t == "FastGaussianRFT" || t == "FastMaternRFT") {
    s.kind = K_FASTFOOD;
    s.nb = (S + N - 1) / N;
    const int64_t nb = s.nb, NB = N;
    s.epi = EPI_COS;
    s.outscale = std::sqrt(2.0 / (double)S);
    s.shifts.resize((size_t)S);
    for (int64_t i = 0; i < S; ++i) s.shifts[(size_t)i] = draw(s, sl::DIST_UNIFORM, c + i, 0.0, 2 * kPi);
    c += (uint64_t)S;
    s.fB.resize((size_t)(nb * NB));
    for (int64_t i = 0; i < nb * NB; ++i) s.fB[(size_t)i] = draw(s, sl::DIST_RADEMACHER, c + i);
    c += (uint64_t)(nb * NB);
    s.fG.resize((size_t)(nb * NB));
    for (int64_t i = 0; i < nb * NB; ++i) s.fG[(size_t)i] = draw(s, sl::DIST_NORMAL, c + i);
    c += (uint64_t)(nb * NB);
    s.perms.resize((size_t)(nb * NB));
    slperm::fastfood_perms(s.perms.data(), s.seed, c, 0, nb, NB);
    c += (uint64_t)(nb * (NB - 1));
    s.scales.resize((size_t)S);
    if (t == "FastGaussianRFT") {
      for (int64_t i = 0; i < S; ++i) s.scales[(size_t)i] = std::sqrt((double)N) / s.sigma;
    } else {
      for (int64_t i = 0; i < S; ++i)
        s.scales[(size_t)i] = std::sqrt(2.0 * s.nu / draw(s, sl::DIST_CHISQ, c + i, 2 * s.nu)) *
                              std::sqrt((double)N) / s.l;
      c += (uint64_t)S;
    }
    return c;
  }
  if (t == "PPT") {
    s.kind = K_PPT;
    if (s.q < 0) return bad("PPT needs q >= 0");
    s.pidx.resize((size_t)(s.q * N));
    s.pval.resize((size_t)(s.q * N));
    for (int64_t i = 0; i < s.q; ++i) {
      for (int64_t k = 0; k < N; ++k) s.pidx[(size_t)(i * N + k)] = draw_int(s, c + k, 0, S - 1);
      c += (uint64_t)N;
      for (int64_t k = 0; k < N; ++k) s.pval[(size_t)(i * N + k)] = draw(s, sl::DIST_RADEMACHER, c + k);
      c += (uint64_t)N;
    }
    s.hidx.resize((size_t)s.q);
    s.hval.resize((size_t)s.q);
    for (int64_t i = 0; i < s.q; ++i) s.hidx[(size_t)i] = draw_int(s, c + i, 0, S - 1);
    c += (uint64_t)s.q;
    for (int64_t i = 0; i < s.q; ++i) s.hval[(size_t)i] = draw(s, sl::DIST_RADEMACHER, c + i);
    c += (uint64_t)s.q;
    return c;
  }
  // hash transforms
  if (t == "WZT" && (s.P < 1.0 || s.P > 2.0)) return bad("WZT parameter p has to be in (1, 2)");
  s.kind = K_HASH;
  s.idx.resize((size_t)N);
  s.val.resize((size_t)N);
  for (int64_t k = 0; k < N; ++k) s.idx[(size_t)k] = draw_int(s, c + k, 0, S - 1);
  c += (uint64_t)N;
  if (t == "WZT") {
    std::vector<double> e((size_t)N);
    for (int64_t k = 0; k < N; ++k) e[(size_t)k] = draw(s, sl::DIST_EXPONENTIAL, c + k);
    c += (uint64_t)N;
    for (int64_t k = 0; k < N; ++k)
      s.val[(size_t)k] = draw(s, sl::DIST_RADEMACHER, c + k) * std::pow(1.0 / e[(size_t)k], 1.0 / s.P);
    c += (uint64_t)N;
  } else {
    const int d = t == "CWT" ? sl::DIST_RADEMACHER : sl::DIST_CAUCHY;
    for (int64_t k = 0; k < N; ++k) s.val[(size_t)k] = draw(s, d, c + k);
    c += (uint64_t)N;
  }
  return c;
}

// ------------------------------------------------------------------ JSON
inline std::string fmt_double(double v) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.17g", v);
  std::string r(buf);
  if (r.find_first_of(".eEn") == std::string::npos) r += ".0";   // keep it a JSON float
  return r;
}

// Same schema as the Python runtime (sketch/base.py to_dict + each type's
// _extra_params) and the reference.
inline std::string to_json(const Sketch& s) {
  const std::string& t = s.type;
  std::string j = "{\"skylark_object_type\": \"sketch\", \"sketch_type\": \"" + t +
                  "\", \"skylark_version\": \"0.1.0\", \"N\": " + std::to_string(s.N) +
                  ", \"S\": " + std::to_string(s.S) +
                  ", \"creation_context\": {\"skylark_object_type\": \"context\", \"skylark_version\": \"0.1.0\", "
                  "\"seed\": " + std::to_string(s.seed) + ", \"counter\": " + std::to_string(s.ctr0) + "}";
  auto num = [&](const char* k, double v) { j += std::string(", \"") + k + "\": " + fmt_double(v); };
  if (t == "CT") num("C", s.C);
  else if (t == "WZT") num("P", s.P);
  else if (t == "SJLT") num("density", s.density);
  else if (t == "GaussianRFT" || t == "LaplacianRFT" || t == "FastGaussianRFT") num("sigma", s.sigma);
  else if (t == "MaternRFT" || t == "FastMaternRFT") { num("nu", s.nu); num("l", s.l); }
  else if (t == "ExpSemigroupRLT") num("beta", s.beta);
  else if (t == "PPT") {
    j += ", \"q\": " + std::to_string(s.q);
    num("c", s.c);
    num("gamma", s.gamma);
  } else if (t == "UST") j += std::string(", \"replace\": ") + (s.replace ? "true" : "false");
  else if (t == "NURST") {
    j += ", \"p\": [";
    for (size_t i = 0; i < s.probs.size(); ++i) j += (i ? ", " : "") + fmt_double(s.probs[i]);
    j += "]";
  } else if (s.kind == K_QMC) {
    if (t == "ExpSemigroupQRLT") num("beta", s.beta);
    else num("sigma", s.sigma);
    j += ", \"skip\": " + std::to_string(s.skip) +
         ", \"sequence\": {\"skylark_object_type\": \"qmc_sequence\", \"skylark_version\": \"0.1.0\", "
         "\"sequence_type\": \"leaped halton\", \"d\": " + std::to_string(s.seq_d) +
         ", \"leap\": " + std::to_string(s.leap) + "}";
  }
  return j + "}";
}

// --- minimal JSON field extraction (the keys used here are unique in a
//     serialised sketch, nested ones included)
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

inline bool get_bool(const char* js, const char* key, bool& out) {
  const char* p = find_key(js, key);
  if (!p) return false;
  if (*p == '"') ++p;
  if (!strncmp(p, "true", 4) || !strncmp(p, "True", 4) || *p == '1') { out = true; return true; }
  if (!strncmp(p, "false", 5) || !strncmp(p, "False", 5) || *p == '0') { out = false; return true; }
  return false;
}

inline bool get_array(const char* js, const char* key, std::vector<double>& out) {
  const char* p = find_key(js, key);
  if (!p || *p != '[') return false;
  ++p;
  out.clear();
  while (*p) {
    while (*p == ' ' || *p == ',' || *p == '\n' || *p == '\t' || *p == '\r') ++p;
    if (*p == ']') return true;
    char* end = nullptr;
    const double v = strtod(p, &end);
    if (end == p) return false;
    out.push_back(v);
    p = end;
  }
  return false;
}

// Parse a serialised sketch; false -> not a (valid) sketch of a known type.
inline bool from_json(const char* js, Sketch& s, std::string* err = nullptr) {
  std::string t;
  double N, S, v;
  if (!get_string(js, "sketch_type", t) || !supported(t.c_str())) return false;
  if (!get_number(js, "N", N) || !get_number(js, "S", S)) return false;
  if (!get_u64(js, "seed", s.seed) || !get_u64(js, "counter", s.ctr0)) return false;
  s.type = t;
  s.N = (int64_t)N;
  s.S = (int64_t)S;
  if (s.N <= 0 || s.S <= 0) return false;
  if (get_number(js, "C", v)) s.C = v;
  if (get_number(js, "P", v) || get_number(js, "p", v)) s.P = v;
  if (get_number(js, "density", v)) s.density = v;
  if (get_number(js, "sigma", v)) s.sigma = v;
  if (get_number(js, "nu", v)) s.nu = v;
  if (get_number(js, "l", v)) s.l = v;
  if (get_number(js, "beta", v)) s.beta = v;
  if (get_number(js, "c", v)) s.c = v;
  if (get_number(js, "gamma", v)) s.gamma = v;
  if (get_number(js, "q", v)) s.q = (int64_t)v;
  if (get_number(js, "skip", v)) s.skip = (int64_t)v;
  if (get_number(js, "d", v)) s.seq_d = (int64_t)v;
  if (get_number(js, "leap", v)) s.leap = (int64_t)v;
  get_bool(js, "replace", s.replace);
  if (t == "NURST" && !get_array(js, "p", s.probs)) return false;
  std::string e;
  if (build(s, &e) == 0 && !e.empty()) {
    if (err) *err = e;
    return false;
  }
  return true;
}

// ------------------------------------------------------ host application
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

// orthonormal DCT-II entry F[p][i] of size N via a table of cos(pi a / 2N)
struct DctTable {
  int64_t N = 0;
  std::vector<double> cs;
  explicit DctTable(int64_t n) : N(n), cs((size_t)(4 * n)) {
    for (int64_t a = 0; a < 4 * n; ++a) cs[(size_t)a] = std::cos(kPi * (double)a / (2.0 * (double)n));
  }
  double operator()(int64_t p, int64_t i) const {
    const double c = p == 0 ? std::sqrt(1.0 / (double)N) : std::sqrt(2.0 / (double)N);
    return c * cs[(size_t)((p * (2 * i + 1)) % (4 * N))];
  }
};

inline bool explicit_kind(int k) { return k == K_DENSE || k == K_QMC || k == K_FJLT || k == K_FASTFOOD; }

// Columns [k0, k0 + kb) of an explicit operator (DENSE, QMC, FJLT, FASTFOOD;
// Fastfood without its Sm, which is the epilogue's scale) as a column-major
// S x kb panel.
inline void realise_cols(const Sketch& s, int64_t k0, int64_t kb, double* P, const DctTable* dct = nullptr) {
  const int64_t S = s.S;
  parallel_for(kb, [&](int64_t lo, int64_t hi) {
    std::vector<double> v;
    for (int64_t kk = lo; kk < hi; ++kk) {
      const int64_t k = k0 + kk;
      double* col = P + kk * S;
      if (s.kind == K_DENSE) {
        for (int64_t i = 0; i < S; ++i) col[i] = s.scale * draw(s, s.dist, s.wbase + (uint64_t)(k * S + i), s.p0);
      } else if (s.kind == K_QMC) {
        for (int64_t i = 0; i < S; ++i) col[i] = qmc_entry(s, i, k);
      } else if (s.kind == K_FJLT) {
        for (int64_t i = 0; i < S; ++i) col[i] = s.scale * (*dct)(s.samples[(size_t)i], k) * s.dsign[(size_t)k];
      } else {   // FASTFOOD: block b rows [b N, min((b+1) N, S)) = F[0:e-s] diag(G_b) F[perm_b] diag(B_b)
        const int64_t NB = s.N;
        v.resize((size_t)NB);
        for (int64_t b = 0; b < s.nb; ++b) {
          const int64_t r0 = b * NB, r1 = std::min(S, r0 + NB);
          for (int64_t j = 0; j < NB; ++j)
            v[(size_t)j] = s.fG[(size_t)(b * NB + j)] * (*dct)(s.perms[(size_t)(b * NB + j)], k) *
                           s.fB[(size_t)(b * NB + k)];
          for (int64_t r = r0; r < r1; ++r) {
            double acc = 0.0;
            for (int64_t j = 0; j < NB; ++j) acc += (*dct)(r - r0, j) * v[(size_t)j];
            col[r] = acc;
          }
        }
      }
    }
  });
}

// out (col-major, ld) feature epilogue; feature index = row (dim 0) or column (dim 1)
inline void epilogue_host(const Sketch& s, double* X, int64_t rows, int64_t cols, int64_t ld, int dim) {
  if (s.epi == EPI_NONE) return;
  parallel_for(cols, [&](int64_t lo, int64_t hi) {
    for (int64_t j = lo; j < hi; ++j)
      for (int64_t i = 0; i < rows; ++i) {
        double& x = X[i + j * ld];
        const int64_t f = dim == 0 ? i : j;
        if (s.epi == EPI_EXP) {
          x = s.outscale * std::exp(-x);
        } else {
          const double sc = s.scales.empty() ? 1.0 : s.scales[(size_t)f];
          x = s.outscale * std::cos(sc * x + s.shifts[(size_t)f]);
        }
      }
  });
}

// PPT of one input vector a (length N, stride inc) into out (length S, stride
// ost): u_i = sqrt(gamma) C_i a + sqrt(c) h_i e_{hidx_i}, out = IDFT(prod_i DFT(u_i))
inline void ppt_vector(const Sketch& s, const double* a, int64_t inc, double* out, int64_t ost,
                       const std::vector<double>& ct, const std::vector<double>& st) {
  const int64_t S = s.S, N = s.N, K = S / 2 + 1;
  const double sg = std::sqrt(s.gamma), sc = std::sqrt(s.c);
  if (s.q == 0) {
    for (int64_t t = 0; t < S; ++t) out[t * ost] = 0.0;
    return;
  }
  std::vector<double> u((size_t)S), pr((size_t)K, 1.0), pi((size_t)K, 0.0);
  for (int64_t i = 0; i < s.q; ++i) {
    std::fill(u.begin(), u.end(), 0.0);
    for (int64_t k = 0; k < N; ++k) u[(size_t)s.pidx[(size_t)(i * N + k)]] += sg * s.pval[(size_t)(i * N + k)] * a[k * inc];
    u[(size_t)s.hidx[(size_t)i]] += sc * s.hval[(size_t)i];
    for (int64_t f = 0; f < K; ++f) {
      double re = 0.0, im = 0.0;
      for (int64_t t = 0; t < S; ++t) {
        const size_t a2 = (size_t)((f * t) % S);
        re += u[(size_t)t] * ct[a2];
        im -= u[(size_t)t] * st[a2];
      }
      const double r0 = pr[(size_t)f], i0 = pi[(size_t)f];
      pr[(size_t)f] = r0 * re - i0 * im;
      pi[(size_t)f] = r0 * im + i0 * re;
    }
  }
  for (int64_t t = 0; t < S; ++t) {
    double acc = 0.0;
    for (int64_t f = 0; f < K; ++f) {
      const double w = (f == 0 || (S % 2 == 0 && f == S / 2)) ? 1.0 : 2.0;
      const size_t a2 = (size_t)((f * t) % S);
      acc += w * (pr[(size_t)f] * ct[a2] - pi[(size_t)f] * st[a2]);
    }
    out[t * ost] = acc / (double)S;
  }
}

// SA = S A (dim 0: A is N x n) or A S^T (dim 1: A is m x N); host col-major,
// SA overwritten.  Returns 104 on a dimension mismatch.
inline int apply(const Sketch& s, const double* A, int64_t am, int64_t an, double* SA, int64_t sm, int64_t sn,
                 int dim) {
  if (dim == 0 ? (am != s.N || sm != s.S || sn != an) : (an != s.N || sn != s.S || sm != am)) return 104;
  std::memset(SA, 0, sizeof(double) * (size_t)(sm * sn));
  const int64_t S = s.S, N = s.N;
  if (explicit_kind(s.kind)) {
    std::unique_ptr<DctTable> dct;
    if (s.kind == K_FJLT || s.kind == K_FASTFOOD) dct.reset(new DctTable(N));
    const int64_t KB = std::max<int64_t>(1, std::min<int64_t>(256, (int64_t(1) << 24) / S));
    std::vector<double> P((size_t)(S * KB));
    for (int64_t k0 = 0; k0 < N; k0 += KB) {
      const int64_t kb = std::min(KB, N - k0);
      realise_cols(s, k0, kb, P.data(), dct.get());
      if (dim == 0) {
        parallel_for(an, [&](int64_t lo, int64_t hi) {
          for (int64_t j = lo; j < hi; ++j) {
            double* out = SA + j * S;
            for (int64_t kk = 0; kk < kb; ++kk) {
              const double a = A[(k0 + kk) + j * am];
              const double* p = P.data() + kk * S;
              for (int64_t i = 0; i < S; ++i) out[i] += p[i] * a;
            }
          }
        });
      } else {
        parallel_for(S, [&](int64_t lo, int64_t hi) {
          for (int64_t c = lo; c < hi; ++c) {
            double* out = SA + c * am;
            for (int64_t kk = 0; kk < kb; ++kk) {
              const double b = P[(size_t)(c + kk * S)];
              const double* a = A + (k0 + kk) * am;
              for (int64_t i = 0; i < am; ++i) out[i] += a[i] * b;
            }
          }
        });
      }
    }
  } else if (s.kind == K_HASH) {
    if (dim == 0) {
      parallel_for(an, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j)
          for (int64_t k = 0; k < N; ++k) SA[s.idx[(size_t)k] + j * S] += s.val[(size_t)k] * A[k + j * am];
      });
    } else {
      // column k of A lands in column idx[k] of SA: split the work by output column
      parallel_for(S, [&](int64_t lo, int64_t hi) {
        for (int64_t k = 0; k < N; ++k) {
          const int64_t c = s.idx[(size_t)k];
          if (c < lo || c >= hi) continue;
          double* out = SA + c * am;
          const double* a = A + k * am;
          const double v = s.val[(size_t)k];
          for (int64_t i = 0; i < am; ++i) out[i] += v * a[i];
        }
      });
    }
  } else if (s.kind == K_SAMPLE) {
    if (dim == 0) {
      parallel_for(an, [&](int64_t lo, int64_t hi) {
        for (int64_t j = lo; j < hi; ++j)
          for (int64_t i = 0; i < S; ++i) SA[i + j * S] = A[s.samples[(size_t)i] + j * am];
      });
    } else {
      for (int64_t i = 0; i < S; ++i) std::memcpy(SA + i * am, A + s.samples[(size_t)i] * am, sizeof(double) * (size_t)am);
    }
  } else {   // PPT
    std::vector<double> ct((size_t)S), st((size_t)S);
    for (int64_t a = 0; a < S; ++a) {
      ct[(size_t)a] = std::cos(2 * kPi * (double)a / (double)S);
      st[(size_t)a] = std::sin(2 * kPi * (double)a / (double)S);
    }
    const int64_t ncol = dim == 0 ? an : am;
    parallel_for(ncol, [&](int64_t lo, int64_t hi) {
      for (int64_t j = lo; j < hi; ++j) {
        if (dim == 0) ppt_vector(s, A + j * am, 1, SA + j * S, 1, ct, st);
        else ppt_vector(s, A + j, am, SA + j, am, ct, st);
      }
    });
  }
  epilogue_host(s, SA, sm, sn, sm, dim);
  return 0;
}

}  // namespace slnat
