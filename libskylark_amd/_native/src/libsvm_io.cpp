// Multi-threaded LIBSVM text parser (reference utility/io/libsvm_io.hpp:33-2006
// parses line by line on one rank and ships blocks with MPI send/recv).
//
// Here every rank memory-maps the file and parses ITS OWN byte range
// (line-aligned), and inside a rank the range is split again over host
// threads.  Two passes over the text: a scan (rows, nnz, max index per
// chunk), then a fill into CSR arrays at per-chunk offsets, so no
// reallocation or merging is needed.
//
// Line format: "<label> <idx>:<val> <idx>:<val> ...", 1-based idx, '#'
// starts a comment, blank lines are skipped.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "sl_common.hpp"

namespace {

struct ChunkStats {
  int64_t rows = 0, nnz = 0, maxidx = 0, bad = 0;  // bad: 1 + byte offset of a malformed line
};

inline const char* skip_ws(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  return p;
}

inline const char* line_end(const char* p, const char* e) {
  const void* q = memchr(p, '\n', (size_t)(e - p));
  return q ? (const char*)q : e;
}

// Number parsing bounded by the line end: the mapped file is not
// NUL-terminated, so strtod/strtoll run on a NUL-terminated copy of the token
// (at most 63 chars) and can neither read past the mapping nor skip the
// newline into the next line.
inline const char* token_end(const char* p, const char* e, char stop) {
  while (p < e && *p != ' ' && *p != '\t' && *p != '\r' && *p != '\n' && *p != stop) ++p;
  return p;
}

inline bool parse_double(const char* p, const char* te, double* out) {
  char tmp[64];
  const size_t n = (size_t)(te - p);
  if (n == 0 || n >= sizeof(tmp)) return false;
  memcpy(tmp, p, n);
  tmp[n] = 0;
  char* q;
  *out = strtod(tmp, &q);
  return q == tmp + n;
}

inline bool parse_int(const char* p, const char* te, long long* out) {
  char tmp[32];
  const size_t n = (size_t)(te - p);
  if (n == 0 || n >= sizeof(tmp)) return false;
  memcpy(tmp, p, n);
  tmp[n] = 0;
  char* q;
  *out = strtoll(tmp, &q, 10);
  return q == tmp + n;
}

// Returns 1 if the line holds a data row, 0 if it is blank / a comment, and
// -1 for a malformed entry (bad number, a missing value, index < 1).  Calls
// f(idx, val) per entry.
template <typename F>
inline int parse_line(const char* p, const char* e, double* label, F&& f) {
  p = skip_ws(p, e);
  if (p >= e || *p == '#') return 0;
  const char* te = token_end(p, e, 0);
  double lab;
  if (!parse_double(p, te, &lab)) return -1;
  if (label) *label = lab;
  p = te;
  while (true) {
    p = skip_ws(p, e);
    if (p >= e || *p == '#') break;
    const char* ie = token_end(p, e, ':');
    long long idx;
    if (ie >= e || *ie != ':' || !parse_int(p, ie, &idx) || idx < 1) return -1;
    p = ie + 1;
    const char* ve = token_end(p, e, 0);
    double v;
    if (!parse_double(p, ve, &v)) return -1;
    p = ve;
    f((int64_t)idx, v);
  }
  return 1;
}

void split(const char* buf, int64_t len, int nthreads, std::vector<std::pair<int64_t, int64_t>>& ranges) {
  ranges.clear();
  int64_t start = 0;
  for (int t = 0; t < nthreads && start < len; ++t) {
    int64_t end = (t == nthreads - 1) ? len : std::max(start, len * (t + 1) / nthreads);
    if (end < len) {
      const char* le = line_end(buf + end, buf + len);
      end = (int64_t)(le - buf) + (le < buf + len ? 1 : 0);
    }
    if (end > start) ranges.emplace_back(start, end);
    start = end;
  }
}

}  // namespace

// Byte range [*start, *end) of `len` bytes owned by part `part` of `parts`,
// adjusted to whole lines (a line belongs to the part where it starts).
SL_API int sl_libsvm_range(const char* buf, int64_t len, int part, int parts, int64_t* start, int64_t* end) {
  auto adjust = [&](int64_t pos) -> int64_t {
    if (pos <= 0) return 0;
    if (pos >= len) return len;
    if (buf[pos - 1] == '\n') return pos;
    const char* le = line_end(buf + pos, buf + len);
    return (int64_t)(le - buf) + (le < buf + len ? 1 : 0);
  };
  *start = adjust(len * part / parts);
  *end = adjust(len * (part + 1) / parts);
  return SL_OK;
}

// stats[0] = rows, stats[1] = nnz, stats[2] = max index (1-based); chunk
// boundaries are returned for the fill pass (ranges: 2*nthreads int64,
// per-chunk rows/nnz: 2*nthreads int64).
SL_API int sl_libsvm_scan(const char* buf, int64_t len, int nthreads, int64_t* stats, int64_t* ranges_out,
                          int64_t* chunk_counts, int* nchunks) {
  if (nthreads < 1) nthreads = 1;
  std::vector<std::pair<int64_t, int64_t>> ranges;
  split(buf, len, nthreads, ranges);
  std::vector<ChunkStats> cs(ranges.size());
  std::vector<std::thread> th;
  for (size_t c = 0; c < ranges.size(); ++c) {
    th.emplace_back([&, c]() {
      const char* p = buf + ranges[c].first;
      const char* e = buf + ranges[c].second;
      ChunkStats s;
      while (p < e) {
        const char* le = line_end(p, e);
        const int r = parse_line(p, le, nullptr, [&](int64_t idx, double) {
          ++s.nnz;
          if (idx > s.maxidx) s.maxidx = idx;
        });
        if (r < 0) {
          s.bad = (int64_t)(p - buf) + 1;
          break;
        }
        s.rows += r;
        p = le + 1;
      }
      cs[c] = s;
    });
  }
  for (auto& t : th) t.join();
  for (size_t c = 0; c < cs.size(); ++c) {
    if (cs[c].bad) {
      sl_set_last_error("LIBSVM: malformed entry (bad number, missing value or index < 1)");
      stats[0] = stats[1] = stats[2] = 0;
      stats[3] = cs[c].bad - 1;
      *nchunks = 0;
      return SL_ERR_INVALID;
    }
  }
  ChunkStats tot;
  for (size_t c = 0; c < cs.size(); ++c) {
    tot.rows += cs[c].rows;
    tot.nnz += cs[c].nnz;
    tot.maxidx = std::max(tot.maxidx, cs[c].maxidx);
    ranges_out[2 * c] = ranges[c].first;
    ranges_out[2 * c + 1] = ranges[c].second;
    chunk_counts[2 * c] = cs[c].rows;
    chunk_counts[2 * c + 1] = cs[c].nnz;
  }
  stats[0] = tot.rows;
  stats[1] = tot.nnz;
  stats[2] = tot.maxidx;
  *nchunks = (int)ranges.size();
  return SL_OK;
}

// Fill CSR (0-based column indices) + labels using the chunking from scan.
// max_rows >= 0 truncates the output to the first max_rows rows.
SL_API int sl_libsvm_fill(const char* buf, const int64_t* ranges, const int64_t* chunk_counts, int nchunks,
                          int64_t max_rows, double* labels, int64_t* rowptr, int64_t* cols, double* vals) {
  std::vector<int64_t> row0(nchunks + 1, 0), nnz0(nchunks + 1, 0);
  for (int c = 0; c < nchunks; ++c) {
    row0[c + 1] = row0[c] + chunk_counts[2 * c];
    nnz0[c + 1] = nnz0[c] + chunk_counts[2 * c + 1];
  }
  const int64_t total_rows = max_rows >= 0 ? std::min(max_rows, row0[nchunks]) : row0[nchunks];
  rowptr[0] = 0;
  std::vector<std::thread> th;
  for (int c = 0; c < nchunks; ++c) {
    if (row0[c] >= total_rows) break;
    th.emplace_back([&, c]() {
      const char* p = buf + ranges[2 * c];
      const char* e = buf + ranges[2 * c + 1];
      int64_t r = row0[c], k = nnz0[c];
      while (p < e && r < total_rows) {
        const char* le = line_end(p, e);
        double lab;
        if (parse_line(p, le, &lab, [&](int64_t idx, double v) {
              cols[k] = idx - 1;
              vals[k] = v;
              ++k;
            }) > 0) {
          labels[r] = lab;
          rowptr[r + 1] = k;
          ++r;
        }
        p = le + 1;
      }
    });
  }
  for (auto& t : th) t.join();
  return SL_OK;
}
