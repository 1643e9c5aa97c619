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
// The Stockham passes give each thread two adjacent columns (16-B LDS
// accesses, index and twiddle arithmetic shared: VALU instructions -5 %,
// LDS instructions -26 %).  Stage 1 reads A in 64-B row pieces, which
// bounds it (request-bound like the 64-B gather of the counter calibration);
// three persistent variants (LDS-DMA double buffer on 16-column tiles,
// 8-column tiles at two workgroups per CU, 32-column tiles with a register
// prefetch) all lost to this one-shot form or did not fit the registers,
// and so did this form on 32-column tiles (128-B pieces, one 512-thread
// workgroup per CU): 3.03 vs 2.72 ms.
// Stage 2: on the matrix cores by default (k_fs_stage2m, below: 1.16 vs
// 1.34 ms for the VALU kernel at N1 = 1000, m = 1000); the VALU kernel
// stays for odd m.  It runs one workgroup per (k2, 64-column chunk); lane =
// column; the frequencies with this k2 (a CSR group built on the host)
// accumulate in registers (packed f32 FMAs), twiddles from a W_N1 table in
// LDS indexed by (j1 k1) mod N1 (exact, no drift).  (Stage 2 as a length-N1
// LDS FFT measured slower: 3.74 vs 2.36 ms at N1 = 1000, m = 1000.)
// HBM traffic: A once, Y written and read once (M x m complex = A's f32
// bytes each way); the dense m x N copy and the N/2-point spectrum of the
// rocFFT pipeline (ops/fut.py) are gone.
#include "sl_common.hpp"
#include <algorithm>
#include <type_traits>

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
  asm volatile("" ::: "memory");
}
// multiply by -i
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }

// two complex values of adjacent columns (one thread's 16-B LDS element):
// the same butterfly on both, the index arithmetic paid once
struct c2 {
  float2 a, b;
};
__device__ __forceinline__ c2 cadd(c2 x, c2 y) { return {cadd(x.a, y.a), cadd(x.b, y.b)}; }
__device__ __forceinline__ c2 csub(c2 x, c2 y) { return {csub(x.a, y.a), csub(x.b, y.b)}; }
__device__ __forceinline__ c2 mul_mi(c2 x) { return {mul_mi(x.a), mul_mi(x.b)}; }
__device__ __forceinline__ float2 cscale(float2 x, float s) { return make_float2(s * x.x, s * x.y); }
__device__ __forceinline__ c2 cscale(c2 x, float s) { return {cscale(x.a, s), cscale(x.b, s)}; }
__device__ __forceinline__ c2 cmul(c2 x, float2 w) { return {cmul(x.a, w), cmul(x.b, w)}; }

// forward DFT of R points in registers (W = e^{-2 pi i / R}); V = float2 or c2
template <typename V>
__device__ __forceinline__ void dft2(V* v) {
  const V a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <typename V>
__device__ __forceinline__ void dft4(V* v) {
  const V s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
  const V s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(s02, s13);
  v[2] = csub(s02, s13);
  v[1] = cadd(d02, d13);
  v[3] = csub(d02, d13);
}
template <typename V>
__device__ __forceinline__ void dft8(V* v) {
  // two radix-4 on even / odd, twiddles W8^k, combine
  V e[4] = {v[0], v[2], v[4], v[6]};
  V o[4] = {v[1], v[3], v[5], v[7]};
  dft4(e);
  dft4(o);
  constexpr float h = 0.70710678118654752f;
  o[1] = cscale(cadd(o[1], mul_mi(o[1])), h);     // * (1 - i)/sqrt2
  o[2] = mul_mi(o[2]);                            // * -i
  o[3] = cscale(csub(mul_mi(o[3]), o[3]), h);     // * (-1 - i)/sqrt2
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = cadd(e[k], o[k]);
    v[k + 4] = csub(e[k], o[k]);
  }
}
template <typename V>
__device__ __forceinline__ void dft3(V* v) {
  constexpr float c1 = -0.5f, s1 = 0.86602540378443865f;
  const V a = v[0];
  const V t = cadd(v[1], v[2]), d = csub(v[1], v[2]);
  v[0] = cadd(a, t);
  const V m = cadd(a, cscale(t, c1));
  const V r = cscale(mul_mi(d), s1);    // -i s1 d
  v[1] = cadd(m, r);
  v[2] = csub(m, r);
}
template <typename V>
__device__ __forceinline__ void dft5(V* v) {
  constexpr float c1 = 0.30901699437494742f, c2v = -0.80901699437494742f;
  constexpr float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;
  const V a = v[0];
  const V t1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
  const V t2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
  v[0] = cadd(a, cadd(t1, t2));
  const V m1 = cadd(a, cadd(cscale(t1, c1), cscale(t2, c2v)));
  const V m2 = cadd(a, cadd(cscale(t1, c2v), cscale(t2, c1)));
  // -i (s1 d1 + s2 d2), -i (s2 d1 - s1 d2)
  const V n1 = mul_mi(cadd(cscale(d1, s1), cscale(d2, s2)));
  const V n2 = mul_mi(csub(cscale(d1, s2), cscale(d2, s1)));
  v[1] = cadd(m1, n1);
  v[4] = csub(m1, n1);
  v[2] = cadd(m2, n2);
  v[3] = csub(m2, n2);
}
template <typename V>
__device__ __forceinline__ void dft7(V* v) {
  // direct (7 is rare): v_k = sum_n v_n W7^{nk}, W7^e = cos(2 pi e / 7) - i sin(2 pi e / 7)
  constexpr float C[7] = {1.0f, 0.62348980185873353f, -0.22252093395631440f, -0.90096886790241913f,
                          -0.90096886790241913f, -0.22252093395631440f, 0.62348980185873353f};
  constexpr float S[7] = {0.0f, -0.78183148246802981f, -0.97492791218182361f, -0.43388373911755812f,
                          0.43388373911755812f, 0.97492791218182361f, 0.78183148246802981f};
  V in[7];
#pragma unroll
  for (int n = 0; n < 7; ++n) in[n] = v[n];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    V acc = in[0];
#pragma unroll
    for (int n = 1; n < 7; ++n) acc = cadd(acc, cmul(in[n], make_float2(C[(n * k) % 7], S[(n * k) % 7])));
    v[k] = acc;
  }
}
template <int R, typename V>
__device__ __forceinline__ void dft(V* v) {
  if constexpr (R == 2) dft2(v);
  else if constexpr (R == 3) dft3(v);
  else if constexpr (R == 4) dft4(v);
  else if constexpr (R == 5) dft5(v);
  else if constexpr (R == 7) dft7(v);
  else dft8(v);
}

// LDS element of one thread: CP = 1 one column (8 B), CP = 2 two adjacent columns (16 B)
template <int CP>
using cvec = typename std::conditional<CP == 2, c2, float2>::type;
__device__ __forceinline__ void ldv(const float2* p, float2& v) { v = *p; }
__device__ __forceinline__ void ldv(const float2* p, c2& v) {
  const float4 t = *(const float4*)p;
  v = {make_float2(t.x, t.y), make_float2(t.z, t.w)};
}
__device__ __forceinline__ void stv(float2* p, float2 v) { *p = v; }
__device__ __forceinline__ void stv(float2* p, c2 v) { *(float4*)p = make_float4(v.a.x, v.a.y, v.b.x, v.b.y); }
// the same on explicit LDS pointers (an out-of-line pass gets generic
// pointers: flat accesses otherwise); native vectors, HIP's vector structs
// do not take address-space qualified operands
typedef float f2n __attribute__((ext_vector_type(2)));
typedef float f4n __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f2n lds_f2;
typedef __attribute__((address_space(3))) f4n lds_f4;
__device__ __forceinline__ void ldv(const lds_f2* p, float2& v) {
  const f2n t = *p;
  v = make_float2(t.x, t.y);
}
__device__ __forceinline__ void ldv(const lds_f2* p, c2& v) {
  const f4n t = *(const lds_f4*)p;
  v = {make_float2(t.x, t.y), make_float2(t.z, t.w)};
}
__device__ __forceinline__ void stv(lds_f2* p, float2 v) { *p = f2n{v.x, v.y}; }
__device__ __forceinline__ void stv(lds_f2* p, c2 v) { *(lds_f4*)p = f4n{v.a.x, v.a.y, v.b.x, v.b.y}; }

// One Stockham pass of radix R over the N2 x WC tile (in place: all reads,
// barrier, all writes, barrier).  Ns = product of the earlier radices.  A
// thread owns CP adjacent columns of its butterflies (CP = 2: 16-B LDS
// accesses, the index and twiddle arithmetic shared by both columns).
template <int R, int NMAX, int NTH, int W = WC, int CP = 2>
__device__ __noinline__ void stockham_pass(float2* __restrict__ gbuf, const float2* __restrict__ gtw, int N2, int Ns) {
  lds_f2* buf = (lds_f2*)gbuf;
  const lds_f2* tw = (const lds_f2*)gtw;
  const int tid = threadIdx.x;
  using V = cvec<CP>;
  constexpr int WCP = W / CP;             // column groups
  constexpr int QMAX = (NMAX / R * WCP + NTH - 1) / NTH;
  constexpr int JS = NTH / WCP;           // j step per q
  const int nb = N2 / R * WCP;
  const int stride = N2 / R;
  const int tstep = N2 / (Ns * R);
  const int col = (tid & (WCP - 1)) * CP, j0 = tid / WCP;
  // (j / Ns, j % Ns) stepped per q (j += JS) instead of two runtime integer
  // divisions per butterfly: one division per pass
  const int jq0 = j0 / Ns, jr0 = j0 - jq0 * Ns, sq = JS / Ns, sr = JS - sq * Ns;
  V v[QMAX][R];
  {
    int jq = jq0, jr = jr0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int b = tid + NTH * q, j = j0 + JS * q;
      if (b < nb) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          V x;
          ldv(buf + (j + r * stride) * W + col, x);
          if (r > 0) {
            const f2n w = tw[r * jr * tstep];
            x = cmul(x, make_float2(w.x, w.y));
          }
          v[q][r] = x;
        }
        dft<R>(v[q]);
      }
      jq += sq;
      jr += sr;
      if (jr >= Ns) { jr -= Ns; ++jq; }
    }
  }
  lds_barrier();
  {
    int jq = jq0, jr = jr0;
#pragma unroll
    for (int q = 0; q < QMAX; ++q) {
      const int b = tid + NTH * q;
      if (b < nb) {
        const int d0 = jq * Ns * R + jr;
#pragma unroll
        for (int r = 0; r < R; ++r) stv(buf + (d0 + r * Ns) * W + col, v[q][r]);
      }
      jq += sq;
      jr += sr;
      if (jr >= Ns) { jr -= Ns; ++jq; }
    }
  }
  lds_barrier();
}

// in-place length-n FFT of the n x WC LDS tile (radix plan: 4-bit radices, low first).
// (Composite register radices 20 = 4 x 5 / 25 = 5 x 5 measured: plan 25-20
// 3.73 ms, 20-5-5 3.23, 25-4-5 3.79 against 3.24-3.45 for 4-5-5-5 -- the
// radix-25 pass needs ~250 VGPRs; not kept.)
template <int NMAX, int NTH>
__device__ __forceinline__ void fft_tile(float2* buf, const float2* tw, int n, uint64_t rplan, int npass, int p0 = 0,
                                         int Ns0 = 1) {
  int Ns = Ns0;
  for (int p = p0; p < npass; ++p) {
    const int R = (int)((rplan >> (4 * p)) & 15);
    switch (R) {
      case 8: stockham_pass<8, NMAX, NTH>(buf, tw, n, Ns); break;
      case 4: stockham_pass<4, NMAX, NTH>(buf, tw, n, Ns); break;
      case 5: stockham_pass<5, NMAX, NTH>(buf, tw, n, Ns); break;
      case 3: stockham_pass<3, NMAX, NTH>(buf, tw, n, Ns); break;
      case 7: stockham_pass<7, NMAX, NTH, WC, 1>(buf, tw, n, Ns); break;   // CP = 2 spills
      default: stockham_pass<2, NMAX, NTH>(buf, tw, n, Ns); break;
    }
    Ns *= R;
  }
}

// The last Stockham pass (Ns = N2 / R: its butterfly j writes rows k2 = j + r Ns)
// straight to Y with the W_M^{j1 k2} twiddles -- no LDS write-back, barrier
// and re-read for the output.  CP = 2: a thread's two adjacent columns as
// one 16-B store (half the store instructions and address arithmetic).
template <int R, int CP>
__device__ __forceinline__ void last_pass_store(const float2* __restrict__ buf, const float2* __restrict__ tw,
                                                const float2* __restrict__ tm, int N2, float2* __restrict__ Yc,
                                                int64_t ystride, bool cok) {
  using V = cvec<CP>;
  constexpr int WCP = WC / CP;
  constexpr int QMAX = (N2_MAX / R * WCP + NT1 - 1) / NT1;
  const int tid = threadIdx.x, col = (tid & (WCP - 1)) * CP;
  const int Ns = N2 / R, nb = Ns * WCP;
#pragma unroll
  for (int q = 0; q < QMAX; ++q) {
    const int b = tid + NT1 * q;
    if (b < nb) {
      const int j = b / WCP;
      V v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        V x;
        ldv(buf + (j + r * Ns) * WC + col, x);
        v[r] = r == 0 ? x : cmul(x, tw[r * j]);
      }
      dft<R>(v);
      if (cok) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int k2 = j + r * Ns;
          stv(Yc + (int64_t)k2 * ystride, cmul(v[r], tm[k2]));
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
// two adjacent elements (8-B f32 / 4-B bf16 aligned) as floats
template <typename T>
__device__ __forceinline__ void ld_pair(const T* p, float& a, float& b) {
  if constexpr (sizeof(T) == 2) {
    const unsigned u = *(const unsigned*)p;
    a = __uint_as_float(u << 16);
    b = __uint_as_float(u & 0xffff0000u);
  } else {
    const float2 t = *(const float2*)p;
    a = t.x;
    b = t.y;
  }
}

// The tile's rows loaded straight into the first Stockham pass (Ns = 1: no
// twiddles): each thread loads the R0 rows j + r N2 / R0 of its butterflies
// (D applied, every load of the tile in flight at once), runs the radix-R0
// DFT in registers and writes the pass's output -- one LDS write + read +
// barrier fewer than staging the rows first.  CP = 2: two adjacent columns
// per thread and load (the row index arithmetic and the D loads shared).
template <typename T, int R0, int CP>
__device__ __forceinline__ void load_first_pass(const T* __restrict__ Ac, const float* __restrict__ d, int64_t lda,
                                                int64_t N, int N1, int N2, int j1, bool cok, float2* buf) {
  using V = cvec<CP>;
  constexpr int WCP = WC / CP;
  constexpr int QM = (N2_MAX / R0 * WCP + NT1 - 1) / NT1;
  const int64_t M = N >> 1;
  const int tid = threadIdx.x, col = (tid & (WCP - 1)) * CP;
  const int stride = N2 / R0, nb = stride * WCP;
  V v[QM][R0];
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int j = min(tid + NT1 * q, nb - 1) / WCP;     // clamped: unconditional loads
#pragma unroll
    for (int r = 0; r < R0; ++r) {
      const int64_t j4 = 4 * ((int64_t)j1 + (int64_t)N1 * (j + r * stride));   // 2 n0
      const int64_t x0 = j4 < 2 * M ? j4 : 2 * N - j4 - 1;                   // n0 = 2j < M ?
      const int64_t x1 = j4 + 2 < 2 * M ? j4 + 2 : 2 * N - j4 - 3;           // n1 = 2j + 1 < M ?
      if constexpr (CP == 2) {
        float a0, a1, b0, b1;
        ld_pair(Ac + x0 * lda, a0, a1);
        ld_pair(Ac + x1 * lda, b0, b1);
        const float d0 = d[x0], d1 = d[x1];
        v[q][r] = {make_float2(a0 * d0, b0 * d1), make_float2(a1 * d0, b1 * d1)};
      } else {
        v[q][r] = make_float2(ld_f(Ac + x0 * lda) * d[x0], ld_f(Ac + x1 * lda) * d[x1]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int b = tid + NT1 * q;
    if (b < nb) {
      const int j = b / WCP;
      if (!cok) {
#pragma unroll
        for (int r = 0; r < R0; ++r) v[q][r] = V{};
      }
      dft<R0>(v[q]);
#pragma unroll
      for (int r = 0; r < R0; ++r) stv(buf + (j * R0 + r) * WC + col, v[q][r]);
    }
  }
}

// radix plan: up to 12 radices, 4 bits each, packed low first.  CP = 2 (two
// adjacent columns per thread in the first / last passes) needs m, lda even
// and the operand rows 8-B (f32) / 4-B (bf16) aligned.
template <typename T, int CP>
__global__ void __launch_bounds__(NT1, 2)
k_fs_stage1(const T* __restrict__ A, int64_t lda, int64_t N, int m, const float* __restrict__ d, int N1, int N2,
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
  const double inv_m = 1.0 / (double)M;   // one f64 division per thread, not one per entry
  for (int t = tid; t < N2; t += NT1) {
    float s, c;
    sincospif(-2.0f * (float)t / (float)N2, &s, &c);
    tw[t] = make_float2(c, s);
    const int64_t r = (int64_t)j1 * t;   // < N1 N2 = M: no reduction needed
    sincospif(-2.0f * (float)((double)r * inv_m), &s, &c);
    tm[t] = make_float2(c, s);
  }
  // ---- rows of z[j1 + N1 j2] (D applied) -> first radix pass -> tile
  const int col = (tid & (WC / CP - 1)) * CP;
  const bool cok = c0 + col < m;     // CP = 2: m even, so a pair is all in or all out
  const T* Ac = A + min(c0 + col, m - CP);
  const int R0 = (int)(rplan & 15);
  switch (R0) {
    case 8: load_first_pass<T, 8, CP>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 4: load_first_pass<T, 4, CP>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 5: load_first_pass<T, 5, CP>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 3: load_first_pass<T, 3, CP>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
    case 7: load_first_pass<T, 7, 1>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;   // CP = 2 spills
    default: load_first_pass<T, 2, CP>(Ac, d, lda, N, N1, N2, j1, cok, buf); break;
  }
  __syncthreads();
  // ---- the middle passes of the length-N2 FFT along the tile's rows
  fft_tile<N2_MAX, NT1>(buf, tw, N2, rplan, npass - 1, 1, R0);
  // ---- the last pass, times W_M^{j1 k2}, out to Y[k2][j1][c]
  float2* Yc = Y + (int64_t)j1 * m + c0 + col;
  const int64_t ys = (int64_t)N1 * m;
  switch ((int)((rplan >> (4 * (npass - 1))) & 15)) {
    case 8: last_pass_store<8, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 4: last_pass_store<4, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 5: last_pass_store<5, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 3: last_pass_store<3, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
    case 7: last_pass_store<7, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
    default: last_pass_store<2, CP>(buf, tw, tm, N2, Yc, ys, cok); break;
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

// Stage 2 on the matrix cores: the same sums as a real GEMM per k2,
//   [Re Z; Im Z] (2 ng x cols) = [[Tr, -Ti], [Ti, Tr]] (2 ng x 2 N1) [Yr; Yi] (2 N1 x cols),
// with v_mfma_f32_16x16x4_f32 (exact f32 products and sums, at the f32
// vector rate, but the twiddles now reach the wave as one 8-B LDS read per
// lane per 16 x 4 A tile instead of a uniform broadcast per (row, frequency)
// -- the VALU kernel above is bound by those broadcasts and its FMAs).  A
// 16-row M tile holds 8 frequencies (row i: frequency i / 2, real part for
// even i, imaginary for odd); per 4 rows of Y (K = 4) a wave runs two MFMAs
// per (M tile, 16-column N tile): A_re x Yr + A_im x Yi.  A lane's twiddle
// index (row k1) mod N1 advances by 4 k1 mod N1 per step (exact).  Waves are
// independent (no barriers after the W_N1 table): each streams its 4 x 64
// slices of Y through its own LDS ring of M2_PD steps by LDS-DMA (counted
// waits; a register ring of inline-asm loads is not safe across the loop's
// back edge, where hipcc may copy a destination before the data lands) and
// reads the B fragments back with ds_read_b64.  m even (16-B pieces).
constexpr int M2_NT = 4;            // 16-column N tiles per wave (64 columns)
constexpr int M2_MTMAX = 4;         // M tiles per pass (32 frequencies)
constexpr int M2_G = 8 * M2_MTMAX;  // frequencies per pass
constexpr int M2_PD = 4;            // 4-row steps in flight per wave
constexpr int M2_SLOT = 4 * 64;     // float2 per ring slot (4 rows x 64 columns)
typedef float f32x4m __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_v;

__device__ __forceinline__ void glds16(const void* g, unsigned base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(base) : "memory");
}

template <int MT>
__device__ __forceinline__ void fs2m_pass(const float2* __restrict__ Yk, int m, int N1, const lds_f2* tw,
                                          const int* k1s, int ng, float2* __restrict__ Zs,
                                          const int* __restrict__ slots, int cw0, float2* ring) {
  const int lane = threadIdx.x & 63, kr = lane >> 4, li = lane & 15;
  // this lane's A rows: frequency g = mt * 8 + li / 2, real (li even) or imaginary part
  const bool part = li & 1;
  int idx[MT], d4[MT];
  bool gok[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int g = mt * 8 + (li >> 1);
    gok[mt] = g < ng;
    const int k1 = gok[mt] ? k1s[g] : 0;
    idx[mt] = (int)(((int64_t)kr * k1) % N1);
    d4[mt] = (int)((4 * (int64_t)k1) % N1);
  }
  f32x4m acc[MT][M2_NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < M2_NT; ++nt) acc[mt][nt] = f32x4m{0.f, 0.f, 0.f, 0.f};
  const int nst = ((N1 + 3) / 4 + M2_PD - 1) / M2_PD * M2_PD;   // steps, padded (rows >= N1 masked)
  // LDS-DMA of one step: two instructions, each two rows x 64 columns (16 B = two columns per lane)
  const int pc = min(cw0 + 2 * (lane & 31), m - 2);
  const unsigned rbase = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_v*)ring);
  auto issue = [&](int slot, int step) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = min(4 * step + 2 * h + (lane >> 5), N1 - 1);
      glds16(Yk + (int64_t)row * m + pc, rbase + (slot * M2_SLOT + h * 128) * 8);
    }
  };
#pragma unroll
  for (int sl = 0; sl < M2_PD; ++sl) issue(sl, sl);
  const lds_f2* rl = (const lds_f2*)ring;
  for (int s0 = 0; s0 < nst; s0 += M2_PD) {
#pragma unroll
    for (int sl = 0; sl < M2_PD; ++sl) {
      const int step = s0 + sl;
      // this slot's rows have landed ((M2_PD - 1) later steps may still fly)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((M2_PD - 1) * 2) : "memory");
      const bool rok = 4 * step + kr < N1;
      float are[MT], aim[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f2n t = tw[idx[mt]];
        if (!(rok && gok[mt])) t = f2n{0.f, 0.f};
        are[mt] = part ? t.y : t.x;
        aim[mt] = part ? t.x : -t.y;
        idx[mt] += d4[mt];
        if (idx[mt] >= N1) idx[mt] -= N1;
      }
      f2n y[M2_NT];
#pragma unroll
      for (int nt = 0; nt < M2_NT; ++nt) y[nt] = rl[sl * M2_SLOT + kr * 64 + 16 * nt + li];
      // slot read back into registers: refill it (steps past the end re-read the last row: uniform counts)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(sl, step + M2_PD);
      // all real-part products, then all imaginary-part ones: no MFMA waits
      // on the one just before it (40-cycle dependent latency vs 32 issue)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < M2_NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(are[mt], y[nt].x, acc[mt][nt], 0, 0, 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < M2_NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim[mt], y[nt].y, acc[mt][nt], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the ring's last (unused) refills, before the next pass reuses it
  // D: lane holds rows 4 kr + r (r = 0..3) of column li: frequencies 2 kr and 2 kr + 1, (re, im) each
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int g = mt * 8 + 2 * kr + h;
      if (g < ng) {
        float2* zr = Zs + (int64_t)slots[g] * m;
#pragma unroll
        for (int nt = 0; nt < M2_NT; ++nt) {
          const int c = cw0 + 16 * nt + li;
          if (c < m) zr[c] = make_float2(acc[mt][nt][2 * h], acc[mt][nt][2 * h + 1]);
        }
      }
    }
}

__global__ void __launch_bounds__(256, 3)
k_fs_stage2m(const float2* __restrict__ Y, int N1, int N2, int m, const int* __restrict__ gptr,
             const int* __restrict__ gk1, const int* __restrict__ gslot, float2* __restrict__ Zs, int per,
             const int* __restrict__ gord) {
  extern __shared__ __attribute__((aligned(16))) float2 lds[];
  float2* ringb = lds;                          // 4 waves x M2_PD slots
  float2* tw = lds + 4 * M2_PD * M2_SLOT;       // N1: W_N1^t
  __shared__ int k1s[M2_G];
  const int tid = threadIdx.x, w = tid >> 6;
  const int cw = 64 * (int)(blockDim.x >> 6);
  const int nch = (m + cw - 1) / cw;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= nch * N2) return;
  const int gi = L / nch;             // group (largest first when gord is given)
  const int k2 = gord ? gord[gi] : gi;
  const int cw0 = (L - gi * nch) * cw + w * 64;
  const int g0 = gptr[gi], g1 = gptr[gi + 1];
  if (g0 == g1) return;
  for (int t = tid; t < N1; t += blockDim.x) {
    float sn, cs;
    sincospif(-2.0f * (float)((double)t / (double)N1), &sn, &cs);
    tw[t] = make_float2(cs, sn);
  }
  const float2* Yk = Y + (int64_t)k2 * N1 * m;
  const lds_f2* twl = (const lds_f2*)tw;
  float2* ring = ringb + w * M2_PD * M2_SLOT;
  for (int gb = g0; gb < g1; gb += M2_G) {
    const int ng = min(M2_G, g1 - gb);
    __syncthreads();   // the previous pass's k1s reads done
    if (tid < M2_G) k1s[tid] = tid < ng ? gk1[gb + tid] : 0;
    __syncthreads();   // tw and k1s visible
    if (cw0 >= m) continue;
    const int* sl = gslot + gb;
    switch ((ng + 7) >> 3) {
      case 1: fs2m_pass<1>(Yk, m, N1, twl, k1s, ng, Zs, sl, cw0, ring); break;
      case 2: fs2m_pass<2>(Yk, m, N1, twl, k1s, ng, Zs, sl, cw0, ring); break;
      case 3: fs2m_pass<3>(Yk, m, N1, twl, k1s, ng, Zs, sl, cw0, ring); break;
      default: fs2m_pass<4>(Yk, m, N1, twl, k1s, ng, Zs, sl, cw0, ring); break;
    }
  }
}

size_t stage2m_lds(int N1) { return (size_t)(4 * M2_PD * M2_SLOT + N1) * sizeof(float2); }

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

template <typename T>
int launch_stage1(const T* A, int64_t lda, int64_t N, int m, const float* d, int N1, int N2, uint64_t rplan,
                  int npass, float2* Y, hipStream_t s) {
  const int64_t ntiles = (int64_t)((m + WC - 1) / WC) * N1;
  const int per = (int)((ntiles + 7) / 8);
  const bool pair = m % 2 == 0 && m >= 2 && lda % 2 == 0 && (uintptr_t)A % (2 * sizeof(T)) == 0 &&
                    (uintptr_t)Y % 16 == 0;
  const unsigned grid = (unsigned)(8 * (int64_t)per);
  if (pair) {
    SL_LDS_ATTR((k_fs_stage1<T, 2>), (int)stage1_lds(N2_MAX));
    k_fs_stage1<T, 2><<<grid, NT1, stage1_lds(N2), s>>>(A, lda, N, m, d, N1, N2, rplan, npass, Y, per);
  } else {
    SL_LDS_ATTR((k_fs_stage1<T, 1>), (int)stage1_lds(N2_MAX));
    k_fs_stage1<T, 1><<<grid, NT1, stage1_lds(N2), s>>>(A, lda, N, m, d, N1, N2, rplan, npass, Y, per);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

int g_stage2_variant = 1;

}  // namespace

// stage-2 kernel: 1 the MFMA kernel (default), 0 the VALU kernel (A/B)
SL_API void sl_fs_set_stage2_variant(int v) { g_stage2_variant = v; }

SL_API int64_t sl_fs_limits(int which) {
  return which == 0 ? N2_MAX : which == 1 ? WC : S2_G;
}

// Stage 1.  A: N x m (lda, f32 or bf16), d: N f32 (the diagonal D), radix
// plan (4-bit radices, low first, product N2), Y: N2 x N1 x m complex f32.
SL_API int sl_fs_stage1(const void* A, int dtype, int64_t lda, int64_t N, int m, const float* d, int N1, int N2,
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
  if (dtype == SL_F32) return launch_stage1((const float*)A, lda, N, m, d, N1, N2, rplan, npass, (float2*)Y, s);
  if (dtype == SL_BF16) return launch_stage1((const bf16_t*)A, lda, N, m, d, N1, N2, rplan, npass, (float2*)Y, s);
  sl_set_last_error("fs_stage1: f32 / bf16 input");
  return SL_ERR_UNSUPPORTED;
}

// Stage 2.  gptr: N2 + 1 offsets into gk1 / gslot; Zs: nslots x m complex.
// gord (optional, MFMA kernel): group g of the CSR holds frequencies of
// k2 = gord[g] (groups sorted by size, largest first: the big groups start
// first and the grid's tail is short); null: group g is k2 = g.
SL_API int sl_fs_stage2(const void* Y, int N1, int N2, int m, const int* gptr, const int* gk1, const int* gslot,
                        void* Zs, const int* gord, void* stream) {
  if (N1 < 1 || N1 > 8192 || N2 < 1 || m < 1) {
    sl_set_last_error("fs_stage2: needs 1 <= N1 <= 8192");
    return SL_ERR_INVALID;
  }
  if (g_stage2_variant != 0 && m % 2 == 0 && m >= 2 && (uintptr_t)Y % 16 == 0) {
    SL_LDS_ATTR(k_fs_stage2m, (int)stage2m_lds(8192));
    const int nw = (int)std::min<int64_t>(4, (m + 63) / 64);
    const int64_t nblk = (int64_t)((m + 64 * nw - 1) / (64 * nw)) * N2;
    const int per = (int)((nblk + 7) / 8);
    k_fs_stage2m<<<(unsigned)(8 * (int64_t)per), 64 * nw, stage2m_lds(N1), (hipStream_t)stream>>>(
        (const float2*)Y, N1, N2, m, gptr, gk1, gslot, (float2*)Zs, per, gord);
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  if (gord) {
    sl_set_last_error("fs_stage2: a group order needs the MFMA kernel (even m)");
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

