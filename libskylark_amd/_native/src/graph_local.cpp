// Local graph computations: time-dependent personalized PageRank (TD-PPR)
// and seed-based local clustering by sweep cut.
//
// Behaviour follows the reference ml/graph/local_computations.hpp:50-370
// (Avron & Horesh, "Community Detection Using Time-Dependent PageRank"):
// Chebyshev spectral collocation in time (N points on [0, gamma]) and a local
// "push" loop over a FIFO queue of vertices whose residual exceeds
// C * degree.  This is irregular, latency-bound, tiny work: it runs natively
// on the host (no GPU), on a CSR graph (vertices 0..n-1).  The N x N
// collocation operator D (row-major) is built by the caller.
//
// C ABI:
//   sl_td_ppr(...)        -> y values for every touched vertex with y != 0
//   sl_local_cluster(...) -> best-conductance cluster (optionally recursive)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "sl_common.hpp"

namespace {

struct Graph {
  int64_t n;
  const int64_t* rowptr;
  const int64_t* col;
  int64_t deg(int64_t v) const { return rowptr[v + 1] - rowptr[v]; }
};

struct PPR {
  const Graph& G;
  const double* D;  // N x N row-major
  int N, NX;
  double alpha, C;
  // vertex -> slot; slot layout: [N residual | NX y], in_queue flag
  std::unordered_map<int64_t, int64_t> slot;
  std::vector<double> ry;
  std::vector<char> inq;
  std::vector<int64_t> verts;

  PPR(const Graph& g, const double* d, int n, int nx, double a, double c) : G(g), D(d), N(n), NX(nx), alpha(a), C(c) {}

  int64_t get(int64_t v) {
    auto it = slot.find(v);
    if (it != slot.end()) return it->second;
    const int64_t s = (int64_t)verts.size();
    slot.emplace(v, s);
    verts.push_back(v);
    ry.resize(ry.size() + N + NX, 0.0);
    inq.push_back(0);
    return s;
  }
  double* at(int64_t s) { return ry.data() + s * (N + NX); }

  // Push budget: the reference loops until no residual violates its bound; a
  // malformed operator D (or a tolerance below roundoff) would then never
  // stop, so the native loop gives up after max_pops queue pops and reports
  // it (converged = false) instead of spinning.
  int64_t max_pops = 20000000;
  bool converged = true;

  void run(const int64_t* seeds, const double* vals, int64_t ns) {
    std::deque<int64_t> q;
    int64_t pops = 0;
    const int NR = N / NX;
    for (int64_t i = 0; i < ns; ++i) {
      const int64_t s = get(seeds[i]);
      double* r = at(s);
      for (int j = 0; j < N; ++j) r[j] = -alpha * vals[i];
      for (int j = 0; j < NX; ++j) r[N + j] = vals[i];
      inq[s] = 1;
      q.push_back(seeds[i]);
    }
    for (int64_t i = 0; i < ns; ++i)
      for (int64_t e = G.rowptr[seeds[i]]; e < G.rowptr[seeds[i] + 1]; ++e) get(G.col[e]);
    for (int64_t i = 0; i < ns; ++i) {
      const int64_t node = seeds[i];
      const double v = alpha * at(slot[node])[N] / (double)G.deg(node);
      for (int64_t e = G.rowptr[node]; e < G.rowptr[node + 1]; ++e) {
        const int64_t o = G.col[e];
        const int64_t so = slot[o];
        double* ro = at(so);
        const double B = C * (double)G.deg(o);
        bool viol = false;
        for (int j = 0; j < N; ++j) {
          ro[j] += v;
          viol = viol || std::fabs(ro[j]) > B;
        }
        if (!inq[so] && viol) {
          q.push_back(o);
          inq[so] = 1;
        }
      }
    }
    std::vector<double> dyp(N);
    while (!q.empty()) {
      if (++pops > max_pops) {
        converged = false;
        break;
      }
      const int64_t node = q.front();
      q.pop_front();
      const int64_t s = slot[node];
      {
        double* r = at(s);
        for (int i = 0; i < N; ++i) {
          const double* Di = D + (int64_t)i * N;
          double acc = 0;
          for (int j = 0; j < N; ++j) acc += Di[j] * r[j];
          dyp[i] = acc;
        }
        for (int i = 0; i < NX; ++i) r[N + i] += dyp[(int64_t)i * NR];
        const double v = dyp[N - 1];
        const double* u = D + (int64_t)(N - 1) * N;  // last row of D
        for (int i = 0; i < N; ++i) r[i] = v * u[i];
        inq[s] = 0;
      }
      const double c = alpha / (double)G.deg(node);
      for (int64_t e = G.rowptr[node]; e < G.rowptr[node + 1]; ++e) {
        const int64_t o = G.col[e];
        const int64_t so = get(o);  // may grow ry: re-fetch pointers after
        double* ro = at(so);
        const double B = C * (double)G.deg(o);
        bool viol = false;
        for (int i = 0; i < N - 1; ++i) {
          ro[i] += c * dyp[i];
          viol = viol || std::fabs(ro[i]) > B;
        }
        viol = viol || std::fabs(ro[N - 1]) > B;
        if (!inq[so] && viol) {
          q.push_back(o);
          inq[so] = 1;
        }
      }
    }
  }
};

// Sweep over vertices sorted by y_t / deg (descending); returns best
// conductance and prefix length.
std::pair<double, int64_t> sweep(const Graph& G, int64_t num_edges, std::vector<std::pair<double, int64_t>>& vals) {
  std::sort(vals.begin(), vals.end());
  int64_t volS = 0, cutS = 0;
  double best = 1.0;
  int64_t bestprefix = 0;
  std::unordered_set<int64_t> cur;
  cur.reserve(vals.size() * 2);
  for (size_t i = 0; i < vals.size(); ++i) {
    const int64_t node = vals[i].second;
    volS += G.deg(node);
    for (int64_t e = G.rowptr[node]; e < G.rowptr[node + 1]; ++e) {
      if (cur.count(G.col[e])) cutS--;
      else cutS++;
    }
    const double cond = (double)cutS / (double)std::min(volS, num_edges - volS);
    if (cond < best) {
      best = cond;
      bestprefix = (int64_t)i;
    }
    cur.insert(node);
  }
  return {best, bestprefix};
}

}  // namespace

// y_out must hold n*NX doubles, nodes_out n entries; *nout receives the count.
SL_API int sl_td_ppr(int64_t n, const int64_t* rowptr, const int64_t* col, const int64_t* seeds,
                     const double* seedvals, int64_t nseeds, const double* D, int N, int NX, double alpha, double C,
                     int64_t* nodes_out, double* y_out, int64_t* nout) {
  if (N <= 0 || NX <= 0 || N % NX != 0) {
    sl_set_last_error("td_ppr: N must be a positive multiple of NX");
    return SL_ERR_INVALID;
  }
  Graph G{n, rowptr, col};
  PPR p(G, D, N, NX, alpha, C);
  p.run(seeds, seedvals, nseeds);
  if (!p.converged) {
    sl_set_last_error("td_ppr: push loop did not converge (check the collocation operator / tolerance)");
    return SL_ERR_GENERIC;
  }
  int64_t k = 0;
  for (size_t s = 0; s < p.verts.size(); ++s) {
    const double* r = p.at((int64_t)s);
    if (r[N] != 0) {
      nodes_out[k] = p.verts[s];
      std::memcpy(y_out + k * NX, r + N, sizeof(double) * NX);
      ++k;
    }
  }
  *nout = k;
  return SL_OK;
}

// cluster_out must hold n entries.  Returns conductance in *cond.
SL_API int sl_local_cluster(int64_t n, const int64_t* rowptr, const int64_t* col, int64_t num_edges,
                            const int64_t* seeds, int64_t nseeds, const double* D, int N, int NX, double alpha,
                            double C, int recursive, int64_t* cluster_out, int64_t* ncluster, double* cond) {
  Graph G{n, rowptr, col};
  std::vector<int64_t> cluster(seeds, seeds + nseeds);
  double currentcond = -1;
  bool improve;
  int rounds = 0;   // the conductance strictly decreases, but bound the rounds anyway
  do {
    std::vector<double> sv(cluster.size(), 1.0 / (double)cluster.size());
    PPR p(G, D, N, NX, alpha, C);
    p.run(cluster.data(), sv.data(), (int64_t)cluster.size());
    if (!p.converged) {
      sl_set_last_error("local_cluster: push loop did not converge (check the collocation operator / tolerance)");
      return SL_ERR_GENERIC;
    }
    std::vector<int64_t> nz;
    for (size_t s = 0; s < p.verts.size(); ++s)
      if (p.at((int64_t)s)[N] != 0) nz.push_back((int64_t)s);
    improve = false;
    for (int t = 0; t < NX; ++t) {
      std::vector<std::pair<double, int64_t>> vals(nz.size());
      for (size_t i = 0; i < nz.size(); ++i) {
        const int64_t v = p.verts[nz[i]];
        vals[i] = {-p.at(nz[i])[N + t] / (double)G.deg(v), v};
      }
      auto [best, prefix] = sweep(G, num_edges, vals);
      if (currentcond == -1 || (best >= 0 && best < currentcond - 1e-6 * std::fabs(currentcond))) {
        improve = true;
        cluster.clear();
        for (int64_t i = 0; i <= prefix && i < (int64_t)vals.size(); ++i) cluster.push_back(vals[i].second);
        currentcond = best;
      }
    }
  } while (recursive && improve && ++rounds < 1000);
  std::copy(cluster.begin(), cluster.end(), cluster_out);
  *ncluster = (int64_t)cluster.size();
  *cond = currentcond;
  return SL_OK;
}
