// Probe: v_permlane32_swap builtin result order and ds_read_b64_tr_b16 row
// mapping as used by the K = 32 hi/lo step 3 (tsk_kernels.hip X variant).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) short s16x4;

__global__ void k(int* out) {
  __shared__ short img[16 * 64];   // 16 rows x 64 cols, value = row * 100 + col
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * 64; i += 64) img[i] = (short)((i / 64) * 100 + (i % 64));
  __syncthreads();
  const unsigned x = 1000 + lane;
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  out[lane * 8 + 0] = r[0];
  out[lane * 8 + 1] = r[1];
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int rb = 8 * (g & 1) + 4 * (g >> 1);
  const int row = rb + q;
  const short* addr = img + row * 64 + 16 * 1 + 4 * p;   // column tile 1
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)addr);
  for (int j = 0; j < 4; ++j) out[lane * 8 + 2 + j] = v[j];
}

int main() {
  int* d;
  hipMalloc(&d, 64 * 8 * sizeof(int));
  hipMemset(d, 0, 64 * 8 * sizeof(int));
  k<<<1, 64>>>(d);
  int h[64 * 8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d: r0=%d r1=%d tr=[%d %d %d %d]\n", l, h[l * 8], h[l * 8 + 1], h[l * 8 + 2], h[l * 8 + 3],
           h[l * 8 + 4], h[l * 8 + 5]);
  }
  return bad;
}
