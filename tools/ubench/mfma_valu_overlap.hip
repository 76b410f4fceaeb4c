// Microbenchmark (measurement tool): do fp32 MFMA (v_mfma_f32_16x16x4_f32) in one wave and
// fp32 VALU FMAs in the co-resident wave of the same SIMD overlap?  512-thread workgroups,
// one per CU: waves 0-3 = one per SIMD ("A"), waves 4-7 = the partner on each SIMD ("B").
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 1: A MFMA only, 2: B VALU only, 3: A MFMA + B VALU, 4: A+B MFMA, 5: A MFMA+VALU interleaved
__global__ __launch_bounds__(512) void k(float* out, int iters) {
  const int w = threadIdx.x >> 6;
  const float a = out[threadIdx.x & 7] + 1.0f, b = out[(threadIdx.x + 3) & 7] + 0.5f;
  f4 acc[8];
  for (int m = 0; m < 8; ++m) acc[m] = f4{0, 0, 0, 0};
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = a * i;
  const bool doA = (MODE == 1 || MODE == 3 || MODE == 4 || MODE == 5) && w < 4;
  const bool doB_valu = (MODE == 2 || MODE == 3) && w >= 4;
  const bool doB_mfma = MODE == 4 && w >= 4;
  if (doA || doB_mfma) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int s = 0; s < 12; ++s)
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a + s, b, acc[m], 0, 0, 0);
          if (MODE == 5 && (m & 1)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[(s * 4 + i) & 15] = fmaf(v[(s * 4 + i) & 15], a, b);
          }
        }
    }
  }
  if (doB_valu) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 24; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = fmaf(v[i], a, b);
    }
  }
  float s = 0;
  for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  for (int i = 0; i < 16; ++i) s += v[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int MODE>
float run(float* d, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<MODE><<<256, 512>>>(d, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<MODE><<<256, 512>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  float* d; hipMalloc(&d, 4096 * 4); hipMemset(d, 0, 4096 * 4);
  const int it = 2000;
  // per wave per iter: 96 MFMA (A) = 96*32 cycles ; B: 384 v_fmac (24*16)
  float t1 = run<1>(d, it), t2 = run<2>(d, it), t3 = run<3>(d, it), t4 = run<4>(d, it), t5 = run<5>(d, it);
  const double mf = 96.0 * it * 4 * 256;   // MFMAs issued per launch by A waves
  printf("A mfma only       %.3f ms  -> %.1f cyc/MFMA at 2.4GHz\n", t1, t1 * 1e-3 * 2.4e9 / (96.0 * it));
  printf("B valu only       %.3f ms  -> %.2f cyc/VALU\n", t2, t2 * 1e-3 * 2.4e9 / (384.0 * it));
  printf("A mfma + B valu   %.3f ms  (sum %.3f, max %.3f)\n", t3, t1 + t2, t1 > t2 ? t1 : t2);
  printf("A mfma + B mfma   %.3f ms  (2x A = %.3f)\n", t4, 2 * t1);
  printf("A mfma+valu intlv %.3f ms  (A alone %.3f; 192 extra VALU per 96 MFMA)\n", t5, t1);
  printf("fp32 MFMA TF/s (A only): %.1f\n", mf * 2048.0 / (t1 * 1e-3) / 1e12);
  return 0;
}
