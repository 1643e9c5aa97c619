// Host-side sanitizer driver (ASan/UBSan/TSan on the host C++
// build; the GPU code is exercised by the gpu test tier).  Exercises every
// host entry point of the native library with adversarial-but-valid inputs:
// multi-threaded LIBSVM scan/fill (ragged lines, comments, blank lines,
// missing trailing newline), TD-PPR + local clustering on a small graph,
// the host Threefry/RNG fills and the Fisher-Yates prefix draw.
// Exit code 0 and a clean sanitizer report = pass.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
int sl_libsvm_scan(const char* buf, int64_t len, int nthreads, int64_t* stats, int64_t* ranges_out,
                   int64_t* chunk_counts, int* nchunks);
int sl_libsvm_fill(const char* buf, const int64_t* ranges, const int64_t* chunk_counts, int nchunks,
                   int64_t max_rows, double* labels, int64_t* rowptr, int64_t* cols, double* vals);
int sl_libsvm_range(const char* buf, int64_t len, int part, int parts, int64_t* start, int64_t* end);
int sl_td_ppr(int64_t n, const int64_t* rowptr, const int64_t* col, const int64_t* seeds, const double* seedvals,
              int64_t nseeds, const double* D, int N, int NX, double alpha, double C, int64_t* nodes_out,
              double* y_out, int64_t* nout);
int sl_local_cluster(int64_t n, const int64_t* rowptr, const int64_t* col, int64_t num_edges, const int64_t* seeds,
                     int64_t nseeds, const double* D, int N, int NX, double alpha, double C, int recursive,
                     int64_t* cluster_out, int64_t* ncluster, double* cond);
int sl_fill_random_host(void* out, int dtype, int dist, uint64_t seed, uint64_t base, int64_t rows, int64_t cols,
                        int64_t sr, int64_t sc, int64_t r0, int64_t c0, int64_t ir, int64_t ic, double p0,
                        double p1, double scale, int precise);
int sl_random_int_host(int64_t* out, uint64_t seed, uint64_t base, int64_t n, int64_t lo, int64_t hi);
int sl_uniform_prefix_host(int64_t* out, uint64_t seed, uint64_t base, int64_t n);
}

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                     \
    }                                                               \
  } while (0)

static int test_libsvm() {
  std::string txt;
  int64_t rows = 0, nnz = 0;
  for (int i = 0; i < 3000; ++i) {
    txt += std::to_string(i % 3) + " ";
    const int k = 1 + i % 7;
    for (int j = 0; j < k; ++j) txt += std::to_string(1 + (i * 13 + j * 7) % 97) + ":" + std::to_string(0.5 * j) + " ";
    nnz += k;
    ++rows;
    txt += (i % 11 == 0) ? "\n\n" : "\n";
  }
  txt += "1 3:1.5";  // no trailing newline
  rows += 1;
  nnz += 1;
  for (int nt : {1, 3, 8}) {
    int64_t stats[3], ranges[64], counts[64];
    int nch = 0;
    CHECK(sl_libsvm_scan(txt.data(), (int64_t)txt.size(), nt, stats, ranges, counts, &nch) == 0);
    CHECK(stats[0] == rows && stats[1] == nnz);
    std::vector<double> lab(stats[0]), val(stats[1]);
    std::vector<int64_t> rp(stats[0] + 1), col(stats[1]);
    CHECK(sl_libsvm_fill(txt.data(), ranges, counts, nch, -1, lab.data(), rp.data(), col.data(), val.data()) == 0);
    CHECK(rp[stats[0]] == stats[1]);
    for (int64_t c : col) CHECK(c >= 0 && c < 97);
    std::vector<double> lab2(10);
    std::vector<int64_t> rp2(11), col2(stats[1]);
    std::vector<double> val2(stats[1]);
    CHECK(sl_libsvm_fill(txt.data(), ranges, counts, nch, 10, lab2.data(), rp2.data(), col2.data(), val2.data()) == 0);
  }
  for (int parts : {1, 2, 5}) {
    int64_t prev = 0;
    for (int p = 0; p < parts; ++p) {
      int64_t s, e;
      CHECK(sl_libsvm_range(txt.data(), (int64_t)txt.size(), p, parts, &s, &e) == 0);
      CHECK(s == prev && e >= s);
      prev = e;
    }
    CHECK(prev == (int64_t)txt.size());
  }
  return 0;
}

static const char* g_opfile = nullptr;

static int test_graph() {
  // two triangles joined by an edge, symmetric CSR
  const int64_t n = 6;
  std::vector<std::vector<int64_t>> adj = {{1, 2}, {0, 2}, {0, 1, 3}, {2, 4, 5}, {3, 5}, {3, 4}};
  std::vector<int64_t> rp(1, 0), col;
  for (auto& a : adj) {
    col.insert(col.end(), a.begin(), a.end());
    rp.push_back((int64_t)col.size());
  }
  // collocation operator from the Python side (ml.graph._setup), or a
  // deliberately bad one that must hit the push budget and report failure
  int N = 8, NX = 4;
  double C = 1e-4;
  std::vector<double> D(N * N);
  bool real = false;
  if (g_opfile) {
    FILE* f = std::fopen(g_opfile, "rb");
    CHECK(f != nullptr);
    int32_t hdr[2];
    CHECK(std::fread(hdr, sizeof(int32_t), 2, f) == 2);
    N = hdr[0];
    NX = hdr[1];
    CHECK(std::fread(&C, sizeof(double), 1, f) == 1);
    D.resize((size_t)N * N);
    CHECK(std::fread(D.data(), sizeof(double), D.size(), f) == D.size());
    std::fclose(f);
    real = true;
  } else {
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) D[i * N + j] = (i == j) ? 1.0 : 0.5 * (i + 1);
  }
  int64_t seeds[1] = {0};
  double sv[1] = {1.0};
  std::vector<int64_t> nodes(n);
  std::vector<double> y(n * NX);
  int64_t nout = 0;
  const int rc = sl_td_ppr(n, rp.data(), col.data(), seeds, sv, 1, D.data(), N, NX, 0.85, C, nodes.data(), y.data(), &nout);
  if (!real) {  // the bad operator must stop with an error, not spin
    CHECK(rc != 0);
    return 0;
  }
  CHECK(rc == 0);
  CHECK(nout >= 1 && nout <= n);
  std::fprintf(stderr, "td_ppr ok (%lld vertices)\n", (long long)nout);
  std::vector<int64_t> cl(n);
  int64_t ncl = 0;
  double cond = 0;
  CHECK(sl_local_cluster(n, rp.data(), col.data(), (int64_t)col.size(), seeds, 1, D.data(), N, NX, 0.85, C, 1,
                         cl.data(), &ncl, &cond) == 0);
  CHECK(ncl >= 1 && ncl <= n);
  return 0;
}

static int test_rng() {
  std::vector<double> a(257 * 129);
  for (int dist : {0, 1, 2, 3, 4, 5, 6, 7, 8, 9}) {
    CHECK(sl_fill_random_host(a.data(), 1, dist, 42, 1000, 257, 129, 129, 1, 0, 0, 1, 257, dist == 6 ? 3.0 : 0.5,
                              dist == 7 ? 9.0 : 1.0, 1.0, 1) == 0);
    for (double v : a) CHECK(std::isfinite(v));
  }
  std::vector<float> f(1 << 17);
  CHECK(sl_fill_random_host(f.data(), 0, 0, 7, 0, 1 << 17, 1, 1, 1, 0, 0, 1, 0, 0, 0, 1.0, 0) == 0);  // threaded path
  std::vector<int64_t> ri(1000), pre(2 * 1000);
  CHECK(sl_random_int_host(ri.data(), 3, 5, 1000, -4, 9) == 0);
  for (int64_t v : ri) CHECK(v >= -4 && v <= 9);
  CHECK(sl_uniform_prefix_host(pre.data(), 3, 5, 1000) == 0);
  for (int i = 0; i < 1000; ++i) CHECK(pre[i] >= 0 && pre[i] <= i);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1) g_opfile = argv[1];
  std::fprintf(stderr, "libsvm\n");
  if (test_libsvm()) return 1;
  std::fprintf(stderr, "graph\n");
  if (test_graph()) return 1;
  std::fprintf(stderr, "rng\n");
  if (test_rng()) return 1;
  std::printf("sanitize_host ok\n");
  return 0;
}
