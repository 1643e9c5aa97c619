// Sampled DCT-II along the long dimension of a tall matrix -- the FJLT
// P F D A of reference sketch/FJLT_Elemental.hpp:144-171 (F the orthonormal
// DCT-II of utility/fft/fftw_futs.h:50-108, P the S sampled rows) -- as a
// four-step FFT that never forms the full spectrum.
//
// x = D A (N x m, row-major, the m columns are the batch).  Makhoul:
//   v[n] = x[2n] (n < N/2),  v[N-1-n] = x[2n+1],   X[k] = Re(W_4N^k V[k]),
// real-to-complex packing z[j] = v[2j] + i v[2j+1] (M = N/2 points):
//   V[k] = E + W_N^k O,  E = (Z[k] + conj Z[M-k]) / 2,  O = -i (Z[k] - conj Z[M-k]) / 2.
// Four-step split M = N1 N2, j = j1 + N1 j2, k = k2 + N2 k1:
//   stage 1  Y[k2][j1] = W_M^{j1 k2} FFT_N2(z[j1 + N1 j2])[k2]      (all j1)
//   stage 2  Z[k]      = sum_j1 W_N1^{j1 k1} Y[k2][j1]              (needed k only)
//   stage 3  out[s]    = scale c_k Re(W_4N^k (E + W_N^k O)),  k = sample s
//
// Stage 1: one workgroup per (j1, 16-column chunk), two per CU.  The first
// radix pass runs on the rows as they arrive and the last one stores Y
// directly (2.8-2.9 vs 3.2-3.4 ms staging both through LDS).  The 2 N2
// rows of x it needs are read as 64-B row pieces (D applied on load; every
// load of a batch in flight: clamped addresses, no per-element branches)
// into an LDS tile of N2 x 16 complex values; the length-N2 FFT runs in place
// in that tile as mixed-radix Stockham passes (radix 8/4/5/3/7/2: every
// thread reads its butterflies' inputs, barrier, writes the outputs,
// barrier) with a W_N2 table in LDS; the W_M twiddles of the workgroup's j1
// come from a second LDS table.  Y is laid out [k2][j1][column], so stage 2
// streams one contiguous N1 x m slab per k2.  Both grids are XCD-aware: an
// XCD walks (row, column chunk) with the chunk fastest, so the workgroups in
// flight on it cover whole rows of A / Y in its own L2.
// Stage 2: one workgroup per (k2, 64-column chunk); lane = column, the four
// waves split j1 and reduce through LDS; the frequencies with this k2 (a
// CSR group built on the host) accumulate in registers (packed f32 FMAs),
// twiddles from a W_N1 table in LDS indexed by (j1 k1) mod N1 (exact, no
// drift).  (Stage 2 as a length-N1 LDS FFT measured slower: 3.74 vs 2.36 ms
// at N1 = 1000, m = 1000.)
// HBM traffic: A once, Y written and read once (M x m complex = A's f32
// bytes each way); the dense m x N copy and the N/2-point spectrum of the
// rocFFT pipeline (ops/fut.py) are gone.
#include "sl_common.hpp"
#include <algorithm>

namespace {

constexpr int NT = 256;         // stage-2 / post threads
constexpr int NT1 = 256;        // stage-1 threads (4 waves)
constexpr int WC = 16;          // columns per stage-1 workgroup (8: 3.72 vs 3.58 ms)
constexpr int N2_MAX = 512;     // LDS tile N2 x WC float2 = 64 KB: two workgroups per CU

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
// workgroup barrier that waits for LDS traffic only (global loads in flight
// stay in flight across it; __syncthreads would drain them)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
// multiply by -i
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }

// forward DFT of R points in registers (W = e^{-2 pi i / R})
template <int R>
__device__ __forceinline__ void dft(float2* v);

template <>
__device__ __forceinline__ void dft<2>(float2* v) {
  const float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <>
__device__ __forceinline__ void dft<4>(float2* v) {
  const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
  const float2 s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(s02, s13);
  v[2] = csub(s02, s13);
  v[1] = cadd(d02, d13);
  v[3] = csub(d02, d13);
}
template <>
__device__ __forceinline__ void dft<8>(float2* v) {
  // two radix-4 on even / odd, twiddles W8^k, combine
  float2 e[4] = {v[0], v[2], v[4], v[6]};
  float2 o[4] = {v[1], v[3], v[5], v[7]};
  dft<4>(e);
  dft<4>(o);
  constexpr float h = 0.70710678118654752f;
  o[1] = make_float2(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));     // * (1 - i)/sqrt2
  o[2] = mul_mi(o[2]);                                                  // * -i
  o[3] = make_float2(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));    // * (-1 - i)/sqrt2
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = cadd(e[k], o[k]);
    v[k + 4] = csub(e[k], o[k]);
  }
}
template <>
__device__ __forceinline__ void dft<3>(float2* v) {
  constexpr float c1 = -0.5f, s1 = 0.86602540378443865f;
  const float2 a = v[0], b = v[1], c = v[2];
  const float2 t = cadd(b, c), d = csub(b, c);
  v[0] = cadd(a, t);
  const float2 m = make_float2(a.x + c1 * t.x, a.y + c1 * t.y);
  // -i s1 d
  const float2 r = make_float2(s1 * d.y, -s1 * d.x);
  v[1] = cadd(m, r);
  v[2] = csub(m, r);
}
template <>
__device__ __forceinline__ void dft<5>(float2* v) {
  constexpr float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;
  constexpr float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
  const float2 a = v[0];
  const float2 t1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
  const float2 t2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
  v[0] = cadd(a, cadd(t1, t2));
  const float2 m1 = make_float2(a.x + c1 * t1.x + c2 * t2.x, a.y + c1 * t1.y + c2 * t2.y);
  const float2 m2 = make_float2(a.x + c2 * t1.x + c1 * t2.x, a.y + c2 * t1.y + c1 * t2.y);
  // -i (s1 d1 + s2 d2), -i (s2 d1 - s1 d2)
  const float2 n1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
  const float2 n2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
  v[1] = cadd(m1, mul_mi(n1));
  v[4] = csub(m1, mul_mi(n1));
  v[2] = cadd(m2, mul_mi(n2));
  v[3] = csub(m2, mul_mi(n2));
}
template <>
__device__ __forceinline__ void dft<7>(float2* v) {
  // direct (7 is rare): v_k = sum_n v_n W7^{nk}
  float2 in[7];
#pragma unroll
  for (int n = 0; n < 7; ++n) in[n] = v[n];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    float2 acc = in[0];
#pragma unroll
    for (int n = 1; n < 7; ++n) {
      float sn, cs;
      sincospif(-2.0f * (float)((n * k) % 7) / 7.0f, &sn, &cs);
      acc = cadd(acc, cmul(in[n], make_float2(cs, sn)));
    }
    v[k] = acc;
  }
}

// One Stockham pass of radix R over the N2 x WC tile (in place: all reads,
// barrier, all writes, barrier).  Ns = product of the earlier radices.
template <int R, int NMAX>
__device__ __noinline__ void stockham_pass(float2* __restrict__ buf, const float2* __restrict__ tw, int N2, int Ns) {
  constexpr int QMAX = (NMAX / R * WC + NT1 - 1) / NT1;
  constexpr int JS = NT1 / WC;            // j step per q
  const int tid = threadIdx.x;
  const int nb = N2 / R * WC;
  const int stride = N2 / R;
  const int tstep = N2 / (Ns * R);
  const int col = tid & (WC - 1), j0 = tid / WC;
  // (j / Ns, j % Ns) stepped per q (j += JS) instead of two runtime integer
  // divisions per butterfly: one division per pass
  const int jq0 = j0 / Ns, jr0 = j0 - jq0 * Ns, sq = JS / Ns, sr = JS - sq * Ns;
  float2 v[QMAX][R];
  {
    int jq = jq0, jr = jr0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int b = tid + NT1 * q, j = j0 + JS * q;
      if (b < nb) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float2 x = buf[(j + r * stride) * WC + col];
          v[q][r] = r == 0 ? x : cmul(x, tw[r * jr * tstep]);
        }
        dft<R>(v[q]);
      }
      jq += sq;
      jr += sr;
      if (jr >= Ns) { jr -= Ns; ++jq; }
    }
  }
  __syncthreads();
  {
    int jq = jq0, jr = jr0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int b = tid + NT1 * q;
      if (b < nb) {
        const int d0 = jq * Ns * R + jr;
#pragma unroll
        for (int r = 0; r < R; ++r) buf[(d0 + r * Ns) * WC + col] = v[q][r];
      }
      jq += sq;
      jr += sr;
      if (jr >= Ns) { jr -= Ns; ++jq; }
    }
  }
  __syncthreads();
}

// in-place length-n FFT of the n x WC LDS tile (radix plan: 4-bit radices, low first).
// (Composite register radices 20 = 4 x 5 / 25 = 5 x 5 measured: plan 25-20
// 3.73 ms, 20-5-5 3.23, 25-4-5 3.79 against 3.24-3.45 for 4-5-5-5 -- the
// radix-25 pass needs ~250 VGPRs; not kept.)
template <int NMAX>
__device__ void fft_tile(float2* buf, const float2* tw, int n, uint64_t rplan, int npass, int p0 = 0, int Ns0 = 1) {
  int Ns = Ns0;
  for (int p = p0; p < npass; ++p) {
    const int R = (int)((rplan >> (4 * p)) & 15);
    switch (R) {
      case 8: stockham_pass<8, NMAX>(buf, tw, n, Ns); break;
      case 4: stockham_pass<4, NMAX>(buf, tw, n, Ns); break;
      case 5: stockham_pass<5, NMAX>(buf, tw, n, Ns); break;
      case 3: stockham_pass<3, NMAX>(buf, tw, n, Ns); break;
      case 7: stockham_pass<7, NMAX>(buf, tw, n, Ns); break;
      default: stockham_pass<2, NMAX>(buf, tw, n, Ns); break;
    }
    Ns *= R;
  }
}

// The last Stockham pass (Ns = N2 / R: its butterfly j writes rows k2 = j + r Ns)
// straight to Y with the W_M^{j1 k2} twiddles -- no LDS write-back, barrier
// and re-read for the output.
template <int R>
__device__ __forceinline__ void last_pass_store(const float2* __restrict__ buf, const float2* __restrict__ tw,
                                                const float2* __restrict__ tm, int N2, float2* __restrict__ Yc,
                                                int64_t ystride, bool cok) {
  constexpr int QMAX = (N2_MAX / R * WC + NT1 - 1) / NT1;
  const int tid = threadIdx.x, col = tid & (WC - 1);
  const int Ns = N2 / R, nb = Ns * WC;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int b = tid + NT1 * q;
    if (b < nb) {
      const int j = b / WC;
      float2 v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float2 x = buf[(j + r * Ns) * WC + col];
        v[r] = r == 0 ? x : cmul(x, tw[r * j]);
      }
      dft<R>(v);
      if (cok) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int k2 = j + r * Ns;
          Yc[(int64_t)k2 * ystride] = cmul(v[r], tm[k2]);
        }
      }
    }
  }
}

template <typename T>
__device__ __forceinline__ float ld_f(const T* p) {
  if constexpr (sizeof(T) == 2) return bf16_to_f(*(const bf16_t*)p);
  else return (float)*p;
}

// The tile's rows loaded straight into the first Stockham pass (Ns = 1: no
// twiddles): each thread loads the R0 rows j + r N2 / R0 of its butterflies
// (D applied, every load of the tile in flight at once), runs the radix-R0
// DFT in registers and writes the pass's output -- one LDS write + read +
// barrier fewer than staging the rows first.
template <typename T, int R0>
__device__ __forceinline__ void load_first_pass(const T* __restrict__ Ac, const double* __restrict__ d, int64_t lda,
                                                int64_t N, int N1, int N2, int j1, bool cok, float2* buf) {
  constexpr int QM = (N2_MAX / R0 * WC + NT1 - 1) / NT1;
  const int64_t M = N >> 1;
  const int tid = threadIdx.x, col = tid & (WC - 1);
  const int stride = N2 / R0, nb = stride * WC;
  float2 v[QM][R0];
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int j = min(tid + NT1 * q, nb - 1) / WC;     // clamped: unconditional loads
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int64_t j4 = 4 * ((int64_t)j1 + (int64_t)N1 * (j + r * stride));   // 2 n0
      const int64_t x0 = j4 < 2 * M ? j4 : 2 * N - j4 - 1;                   // n0 = 2j < M ?
      const int64_t x1 = j4 + 2 < 2 * M ? j4 + 2 : 2 * N - j4 - 3;           // n1 = 2j + 1 < M ?
      v[q][r] = make_float2(ld_f(Ac + x0 * lda) * (float)d[x0], ld_f(Ac + x1 * lda) * (float)d[x1]);
    }
  }
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int b = tid + NT1 * q;
    if (b < nb) {
      const int j = b / WC;
      if (!cok) {
#pragma unroll
        for (int r = 0; r < R0; ++r) v[q][r] = make_float2(0.f, 0.f);
      }
      dft<R0>(v[q]);
#pragma unroll
      for (int r = 0; r < R0; ++r) buf[(j * R0 + r) * WC + col] = v[q][r];
    }
  }
}

// radix plan: up to 12 radices, 4 bits each, packed low first
template <typename T>
__global__ void __launch_bounds__(NT1)
k_fs_stage1(const T* __restrict__ A, int64_t lda, int64_t N, int m, const double* __restrict__ d, int N1, int N2,
            uint64_t rplan, int npass, float2* __restrict__ Y, int per) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2* buf = lds;                 // N2 x WC
  float2* tw = lds + N2 * WC;        // N2: W_N2^t
  const int tid = threadIdx.x;
  // XCD-aware order (block b runs on XCD b % 8): each XCD walks a contiguous
  // range of (j1, column chunk) with the chunk fastest, so the workgroups in
  // flight on one XCD cover whole rows of A and Y in that XCD's L2
  const int nch = (m + WC - 1) / WC;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= nch * N1) return;
  const int j1 = L / nch;
  const int c0 = (L - j1 * nch) * WC;
  const int64_t M = N >> 1;
  float2* tm = tw + N2;              // N2: W_M^{(j1 k2) mod M} of this j1
  for (int t = tid; t < N2; t += NT1) {
    float s, c;
    sincospif(-2.0f * (float)t / (float)N2, &s, &c);
    tw[t] = make_float2(c, s);
    const int64_t r = (int64_t)j1 * t;   // < N1 N2 = M: no reduction needed
    sincospif(-2.0f * (float)((double)r / (double)M), &s, &c);
    tm[t] = make_float2(c, s);
  }
  // ---- rows of z[j1 + N1 j2] (D applied) -> first radix pass -> tile
  const int col = tid & (WC - 1);
  const bool cok = c0 + col < m;
  const T* Ac = A + min(c0 + col, m - 1);
  const int R0 = (int)(rplan & 15);
  switch (R0) {
    case 8: load_first_pass<T, 8>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 4: load_first_pass<T, 4>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 5: load_first_pass<T, 5>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 3: load_first_pass<T, 3>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 7: load_first_pass<T, 7>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    default: load_first_pass<T, 2>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
  }
  __syncthreads();
  // ---- the middle passes of the length-N2 FFT along the tile's rows
  fft_tile<N2_MAX>(buf, tw, N2, rplan, npass - 1, 1, R0);
  // ---- the last pass, times W_M^{j1 k2}, out to Y[k2][j1][c]
  float2* Yc = Y + (int64_t)j1 * m + c0 + col;
  const int64_t ys = (int64_t)N1 * m;
  switch ((int)((rplan >> (4 * (npass - 1))) & 15)) {
    case 8: last_pass_store<8>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 4: last_pass_store<4>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 5: last_pass_store<5>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 3: last_pass_store<3>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 7: last_pass_store<7>(buf, tw, tm, N2, Yc, ys, cok); break;
    default: last_pass_store<2>(buf, tw, tm, N2, Yc, ys, cok); break;
  }
}

// Stage 2: Zs[slot][c] = sum_j1 W_N1^{j1 k1} Y[k2][j1][c] for the (k1, slot)
// pairs of group k2 (gptr CSR over k2, gk1 / gslot entries).
// Workgroup = (k2, 64 S2_NW columns): each wave owns 64 columns (lane =
// column) and runs over ALL N1 rows, so there is no cross-wave reduction.
// The group's twiddles W_N1^{j1 k1} are laid out per row in LDS, a 64-row
// chunk at a time ([row][g], zero-padded to NG = ng rounded up to 4 and for
// rows >= N1), built one chunk ahead by the whole workgroup from the W_N1
// table; the inner loop reads them as uniform-address float4 broadcasts and
// does 2 packed FMAs per (row, frequency) -- no per-element index math.  The
// rows of Y stream through an 8-deep register ring (loads issued 8 rows
// ahead; the chunk barriers wait on LDS only, never drain the ring).
// (Before: 4 waves split j1 with 2 rows in flight and per-frequency index
// arithmetic in the loop, 2.4 ms at N1 = 1000, m = 1000.)
// (Two columns per lane -- 16-B rows, each twiddle broadcast used twice --
// needs 192 VGPRs, 2 waves per SIMD: 1.51 vs 1.28 ms; not kept.)
constexpr int S2_NW = 4;        // waves per workgroup (column slices)
constexpr int S2_JC = 64;       // rows per twiddle chunk
constexpr int S2_U = 8;         // rows in flight per wave
constexpr int S2_G = 24;        // frequencies per pass

template <int NG>
__device__ __forceinline__ void fs2_pass(const float2* __restrict__ Yc, int m, int N1, const float2* tw,
                                         float2* Tg, const int* k1s, int ng, float2* __restrict__ Zs,
                                         const int* __restrict__ slots, int c, bool cok) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int nch = (N1 + S2_JC - 1) / S2_JC;
  auto build = [&](int ch, float2* dst) {
    for (int e = tid; e < S2_JC * NG; e += nthr) {
      const int r = e / NG, g = e - r * NG;
      const int j = ch * S2_JC + r;
      float2 t = make_float2(0.f, 0.f);
      if (j < N1 && g < ng) t = tw[(int)(((int64_t)j * k1s[g]) % N1)];
      dst[e] = t;
    }
  };
  f2 acc[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) acc[g] = f2{0.f, 0.f};
  float2 y[S2_U];
#pragma unroll
  for (int u = 0; u < S2_U; ++u) y[u] = Yc[(int64_t)min(u, N1 - 1) * m];
  build(0, Tg);
  lds_barrier();
  for (int ch = 0; ch < nch; ++ch) {
    const float2* T = Tg + (ch & 1) * S2_JC * NG;
    if (ch + 1 < nch) build(ch + 1, Tg + ((ch + 1) & 1) * S2_JC * NG);
    for (int r0 = 0; r0 < S2_JC; r0 += S2_U) {
#pragma unroll
      for (int u = 0; u < S2_U; ++u) {
        const int r = r0 + u;
        const float2 yv = y[u];
        y[u] = Yc[(int64_t)min(ch * S2_JC + r + S2_U, N1 - 1) * m];
        const f2 ya = f2{yv.x, yv.y}, yb = f2{yv.y, yv.x};
        const float4* Tr = (const float4*)(T + r * NG);
#pragma unroll
        for (int g = 0; g < NG; g += 2) {
          const float4 t = Tr[g >> 1];
          acc[g] = __builtin_elementwise_fma(f2{t.x, t.x}, ya, acc[g]);
          acc[g] = __builtin_elementwise_fma(f2{-t.y, t.y}, yb, acc[g]);
          acc[g + 1] = __builtin_elementwise_fma(f2{t.z, t.z}, ya, acc[g + 1]);
          acc[g + 1] = __builtin_elementwise_fma(f2{-t.w, t.w}, yb, acc[g + 1]);
        }
      }
    }
    lds_barrier();
  }
  if (cok) {
#pragma unroll
    for (int g = 0; g < NG; ++g)
      if (g < ng) Zs[(int64_t)slots[g] * m + c] = make_float2(acc[g].x, acc[g].y);
  }
}

__global__ void __launch_bounds__(64 * S2_NW, 4)
k_fs_stage2(const float2* __restrict__ Y, int N1, int N2, int m, const int* __restrict__ gptr,
            const int* __restrict__ gk1, const int* __restrict__ gslot, float2* __restrict__ Zs, int per) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2* Tg = lds;                          // 2 x S2_JC x S2_G
  float2* tw = lds + 2 * S2_JC * S2_G;       // N1: W_N1^t
  __shared__ int k1s[S2_G];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cw = 64 * (int)(blockDim.x >> 6);
  // XCD-aware order as in stage 1: an XCD walks (k2, column chunk) with the chunk fastest
  const int nch = (m + cw - 1) / cw;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= nch * N2) return;
  const int k2 = L / nch;
  const int c = (L - k2 * nch) * cw + w * 64 + lane;
  const int g0 = gptr[k2], g1 = gptr[k2 + 1];
  if (g0 == g1) return;
  for (int t = tid; t < N1; t += blockDim.x) {
    float sn, cs;
    sincospif(-2.0f * (float)((double)t / (double)N1), &sn, &cs);
    tw[t] = make_float2(cs, sn);
  }
  const bool cok = c < m;
  const float2* Yc = Y + (int64_t)k2 * N1 * m + min(c, m - 1);   // clamped: unconditional loads
  for (int gb = g0; gb < g1; gb += S2_G) {
    const int ng = min(S2_G, g1 - gb);
    if (tid < S2_G) k1s[tid] = tid < ng ? gk1[gb + tid] : 0;
    lds_barrier();    // tw and k1s visible (and the previous pass's chunk reads done)
    const int* sl = gslot + gb;
    switch ((ng + 3) >> 2) {
      case 1: fs2_pass<4>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
      case 2: fs2_pass<8>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
      case 3: fs2_pass<12>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
      case 4: fs2_pass<16>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
      case 5: fs2_pass<20>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
      default: fs2_pass<24>(Yc, m, N1, tw, Tg, k1s, ng, Zs, sl, c, cok); break;
    }
  }
}

// Stage 3: out[s][c] (row stride ldo) = scale c_k Re(W_4N^k (E + W_N^k O)).
__global__ void __launch_bounds__(NT)
k_fs_post(const float2* __restrict__ Zs, int m, int64_t N, const int64_t* __restrict__ samples, int S,
          const int* __restrict__ sa, const int* __restrict__ sb, double scale, float* __restrict__ out,
          int64_t ldo) {
  const int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (t >= (int64_t)S * m) return;
  const int s = (int)(t / m), c = (int)(t - (int64_t)s * m);
  const int64_t k = samples[s];
  const float2 za = Zs[(int64_t)sa[s] * m + c], zb = Zs[(int64_t)sb[s] * m + c];
  // E = (Za + conj Zb) / 2, O = -i (Za - conj Zb) / 2
  const double er = 0.5 * ((double)za.x + zb.x), ei = 0.5 * ((double)za.y - zb.y);
  const double dr = 0.5 * ((double)za.x - zb.x), di = 0.5 * ((double)za.y + zb.y);
  const double orr = di, oi = -dr;
  double sn, cs;
  sincospi(-2.0 * (double)k / (double)N, &sn, &cs);          // W_N^k
  const double vr = er + cs * orr - sn * oi, vi = ei + cs * oi + sn * orr;
  sincospi(-0.5 * (double)k / (double)N, &sn, &cs);          // W_4N^k
  const double x = cs * vr - sn * vi;
  const double ck = k == 0 ? sqrt(1.0 / (double)N) : sqrt(2.0 / (double)N);
  out[(int64_t)s * ldo + c] = (float)(scale * ck * x);
}

size_t stage1_lds(int N2) { return (size_t)(N2 * WC + 2 * N2) * sizeof(float2); }
size_t stage2_lds(int N1) { return (size_t)(N1 + 2 * S2_JC * S2_G) * sizeof(float2); }

}  // namespace

SL_API int64_t sl_fs_limits(int which) {
  return which == 0 ? N2_MAX : which == 1 ? WC : S2_G;
}

// Stage 1.  A: N x m (lda, f32 or bf16), d: N f64 signs, radix plan (4-bit
// radices, low first, product N2), Y: N2 x N1 x m complex f32.
SL_API int sl_fs_stage1(const void* A, int dtype, int64_t lda, int64_t N, int m, const double* d, int N1, int N2,
                        uint64_t rplan, int npass, void* Y, void* stream) {
  if (N % 2 || (int64_t)N1 * N2 != N / 2 || N2 < 2 || N2 > N2_MAX || m < 1 || npass < 2 || npass > 16) {
    sl_set_last_error("fs_stage1: needs N even, N1 N2 = N/2, 2 <= N2 <= 512, at least two radix passes");
    return SL_ERR_INVALID;
  }
  int64_t prod = 1;
  for (int p = 0; p < npass; ++p) {
    const int R = (int)((rplan >> (4 * p)) & 15);
    if (R != 2 && R != 3 && R != 4 && R != 5 && R != 7 && R != 8) {
      sl_set_last_error("fs_stage1: radices must be 2, 3, 4, 5, 7, 8");
      return SL_ERR_INVALID;
    }
    prod *= R;
  }
  if (prod != N2) { sl_set_last_error("fs_stage1: radix plan does not multiply to N2"); return SL_ERR_INVALID; }
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = stage1_lds(N2);
  const int64_t nblk = (int64_t)((m + WC - 1) / WC) * N1;
  const int per = (int)((nblk + 7) / 8);
  const unsigned grid = (unsigned)(8 * (int64_t)per);
  if (dtype == SL_F32) {
    SL_LDS_ATTR(k_fs_stage1<float>, (int)stage1_lds(N2_MAX));
    k_fs_stage1<float><<<grid, NT1, lds, s>>>((const float*)A, lda, N, m, d, N1, N2, rplan, npass, (float2*)Y, per);
  } else if (dtype == SL_BF16) {
    SL_LDS_ATTR(k_fs_stage1<bf16_t>, (int)stage1_lds(N2_MAX));
    k_fs_stage1<bf16_t><<<grid, NT1, lds, s>>>((const bf16_t*)A, lda, N, m, d, N1, N2, rplan, npass, (float2*)Y, per);
  } else {
    sl_set_last_error("fs_stage1: f32 / bf16 input");
    return SL_ERR_UNSUPPORTED;
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Stage 2.  gptr: N2 + 1 offsets into gk1 / gslot; Zs: nslots x m complex.
SL_API int sl_fs_stage2(const void* Y, int N1, int N2, int m, const int* gptr, const int* gk1, const int* gslot,
                        void* Zs, void* stream) {
  if (N1 < 1 || N1 > 8192 || N2 < 1 || m < 1) {
    sl_set_last_error("fs_stage2: needs 1 <= N1 <= 8192");
    return SL_ERR_INVALID;
  }
  SL_LDS_ATTR(k_fs_stage2, (int)stage2_lds(8192));
  // narrow batches: fewer waves per workgroup (each wave owns 64 columns)
  const int nw = (int)std::min<int64_t>(S2_NW, (m + 63) / 64);
  const int64_t nblk = (int64_t)((m + 64 * nw - 1) / (64 * nw)) * N2;
  const int per = (int)((nblk + 7) / 8);
  k_fs_stage2<<<(unsigned)(8 * (int64_t)per), 64 * nw, stage2_lds(N1), (hipStream_t)stream>>>(
      (const float2*)Y, N1, N2, m, gptr, gk1, gslot, (float2*)Zs, per);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_fs_post(const void* Zs, int m, int64_t N, const int64_t* samples, int S, const int* sa, const int* sb,
                      double scale, float* out, int64_t ldo, void* stream) {
  if (S < 1 || m < 1) return SL_OK;
  const int64_t tot = (int64_t)S * m;
  k_fs_post<<<(unsigned)((tot + NT - 1) / NT), NT, 0, (hipStream_t)stream>>>((const float2*)Zs, m, N, samples, S, sa,
                                                                            sb, scale, out, ldo);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

