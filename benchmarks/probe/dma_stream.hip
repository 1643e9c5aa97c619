// Probe: chip-wide LDS-DMA stream rate of the fused randSVD pass's access
// pattern (1e6 x 1000 bf16, 16-row blocks, one 512-thread workgroup per CU,
// 4-slot ring, 3 blocks in flight, one barrier per block) with no compute,
// under different source -> LDS mappings:
//   mode 0: the pass's mapping (wave w owns 128 columns of the 16 rows, 256-B
//           row pieces, swizzled chunk order)
//   mode 1: flat (the block is ONE contiguous 32000-B span: lane chunk c of
//           instruction i = i * 512 + tid, 128-B aligned whole lines)
//   mode 2: mode 1 with the nt policy
//   mode 3: mode 0 with the nt policy
//   mode 4: mode 0 + 24 LDS b128 reads per wave and block (the pass's LDS load)
//   mode 5: mode 4 + 37 MFMA 16x16x32 per wave and block (its matrix-core load)
//   mode 6: mode 5 with nt;  mode 7: mode 0 + 8 reads + 37 MFMAs
// usage: ./dma_stream [reps] [random data: 1]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_void;

template <bool NT>
__device__ __forceinline__ void glds16s(unsigned voff, const void* sbase, unsigned lds_base) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_base) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_base) : "memory");
}

__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ int swz4(int row) { return ((row << 1) & 15) ^ (((row >> 3) & 1) * 9); }

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int MODE, int LR = 0, int MF = 0>
__global__ void __launch_bounds__(512, 1) k_stream(const unsigned short* __restrict__ A, long m, int n, float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NBUF = 4, BM = 16, LPB = 4, SLOT = 32768;
  constexpr bool NT = MODE == 2 || MODE == 3;
  const bool flat = MODE == 1 || MODE == 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long nblocks = (m + BM - 1) / BM;
  const long b0 = blockIdx.x, bstep = gridDim.x;
  const long nloc = b0 < nblocks ? (nblocks - 1 - b0) / bstep + 1 : 0;
  const int bbytes = BM * n * 2;
  unsigned voff[LPB];
  unsigned ldsoff[LPB];
#pragma unroll
  for (int i = 0; i < LPB; ++i) {
    if (flat) {
      int c = i * 512 + w * 64 + lane;
      const int nch = bbytes / 16;
      voff[i] = (unsigned)((c < nch ? c : nch - 1) * 16);
      ldsoff[i] = (unsigned)((i * 512 + w * 64) * 16);
    } else {
      const int byte = i * 1024 + lane * 16;
      const int row = byte / 256;
      const int sl = (byte % 256) / 16;
      const int chunk = sl ^ swz4(row);
      int col = 128 * w + chunk * 8;
      col = col + 8 <= n ? col : n - 8;
      voff[i] = (unsigned)((row * n + col) * 2);
      ldsoff[i] = (unsigned)(w * 4096 + i * 1024);
    }
  }
  auto issue = [&](long jb) {
    const int slot = (int)(jb % NBUF);
    const long b = b0 + jb * bstep;
    const char* base = (const char*)(A + b * BM * (long)n);
#pragma unroll
    for (int i = 0; i < LPB; ++i) {
      const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(smem + slot * SLOT + ldsoff[i]));
      glds16s<NT>(voff[i], (const void*)base, dst);
    }
  };
  float acc = 0.f;
  f32x4 macc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) macc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < NBUF - 1; ++b)
    if (b < nloc) issue(b);
  for (long j = 0; j < nloc; ++j) {
    const int inflight = (j + 1 < nloc) + (j + 2 < nloc);
    wait_vm(LPB * inflight);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (j + NBUF - 1 < nloc) issue(j + NBUF - 1);
    acc += *(const float*)(smem + (int)(j % NBUF) * SLOT + (tid * 16) % 32000);
    if constexpr (LR > 0 || MF > 0) {
      // the pass's per-block LDS reads (b128 fragments of the current slot)
      // and matrix-core work (independent accumulators), no dependence on them
      const char* sl = smem + (int)(j % NBUF) * SLOT;
      bf16x8 fr[LR > 0 ? LR : 1];
#pragma unroll
      for (int q = 0; q < LR; ++q) fr[q] = *(const bf16x8*)(sl + ((q * 1024 + lane * 16 + w * 2048) & 32767));
#pragma unroll
      for (int q = 0; q < MF; ++q) macc[q & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[q % (LR > 0 ? LR : 1)], fr[(q + 1) % (LR > 0 ? LR : 1)], macc[q & 7], 0, 0, 0);
      if constexpr (MF == 0) {
#pragma unroll
        for (int q = 0; q < LR; ++q) acc += (float)fr[q][0];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) acc += macc[q][0];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 12345.f) out[tid] = acc;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const long m = 1000000;
  const int n = 1000;
  unsigned short* A;
  float* out;
  CK(hipMalloc(&A, m * n * 2));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(A, 0, m * n * 2));
  if (argc > 2 && atoi(argv[2]) == 1) {
    unsigned short* h = (unsigned short*)malloc(64 << 20);
    unsigned x = 12345;
    for (long i = 0; i < (32 << 20); ++i) { x = x * 1664525u + 1013904223u; h[i] = (unsigned short)((x >> 16) & 0xBFFF); }
    for (long off = 0; off < m * n; off += (32 << 20)) {
      const long cnt = (m * n - off) < (32 << 20) ? (m * n - off) : (32 << 20);
      CK(hipMemcpy(A + off, h, cnt * 2, hipMemcpyHostToDevice));
    }
    free(h);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int LDS = 4 * 32768;
  CK(hipFuncSetAttribute((const void*)k_stream<0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<3>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<0, 24, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<0, 24, 37>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<3, 24, 37>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  CK(hipFuncSetAttribute((const void*)k_stream<0, 8, 37>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 8; ++mode) {
      auto launch = [&]() {
        switch (mode) {
          case 0: k_stream<0><<<256, 512, LDS>>>(A, m, n, out); break;
          case 1: k_stream<1><<<256, 512, LDS>>>(A, m, n, out); break;
          case 2: k_stream<2><<<256, 512, LDS>>>(A, m, n, out); break;
          case 3: k_stream<3><<<256, 512, LDS>>>(A, m, n, out); break;
          case 4: k_stream<0, 24, 0><<<256, 512, LDS>>>(A, m, n, out); break;
          case 5: k_stream<0, 24, 37><<<256, 512, LDS>>>(A, m, n, out); break;
          case 6: k_stream<3, 24, 37><<<256, 512, LDS>>>(A, m, n, out); break;
          default: k_stream<0, 8, 37><<<256, 512, LDS>>>(A, m, n, out); break;
        }
      };
      launch();
      CK(hipDeviceSynchronize());
      float best = 1e30f, tot = 0.f;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        tot += ms;
      }
      printf("{\"round\": %d, \"mode\": %d, \"us_min\": %.1f, \"us_mean\": %.1f, \"TBps_min\": %.3f}\n", round, mode,
             best * 1e3, tot / reps * 1e3, (double)m * n * 2 / (best * 1e-3) / 1e12);
    }
  return 0;
}
