// Micro-benchmark + exactness check of two ways to split fp32 pairs into three bf16 parts
// (gnca_k1_split.h:split3_pair):
//   ref : cvt_pk, then unpack (shift / and) + v_sub per value per level (11 VALU per pair)
//   dot2: cvt_pk, then the residual a - bf16(a) as ONE v_dot2_f32_bf16 per value:
//         dot2({a0, b0}, {-1, 0}, a) = a - a0 (exact: the product is exact and a - a0 is
//         representable), 7 VALU per pair.
// Output: mismatching parts over a wide-exponent sample (must be 0), and ns per pair-split of
// each variant in a dependent-free loop (one wave per SIMD and 2 per SIMD).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/split_dot2.hip -o /tmp/split_dot2 && /tmp/split_dot2
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void split_ref(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){ra, rb}, bf16x2v));
  const float la = ra - __uint_as_float(m << 16), lb = rb - __uint_as_float(m & 0xffff0000u);
  p0 = h;
  p1 = m;
  p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){la, lb}, bf16x2v));
}

__device__ __forceinline__ float dot2(uint32_t x, uint32_t k, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(s16x2, x), __builtin_bit_cast(s16x2, k), c, false);
}

__device__ __forceinline__ void split_dot2(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  constexpr uint32_t KLO = 0x0000bf80u, KHI = 0xbf800000u;   // {-1, 0}, {0, -1}
  const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
  const float ra = dot2(h, KLO, a), rb = dot2(h, KHI, b);
  const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){ra, rb}, bf16x2v));
  const float la = dot2(m, KLO, ra), lb = dot2(m, KHI, rb);
  p0 = h;
  p1 = m;
  p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){la, lb}, bf16x2v));
}

template <int V>
__global__ void check(const float* x, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t p0, p1, p2;
  if (V == 0) split_ref(x[2 * i], x[2 * i + 1], p0, p1, p2);
  else split_dot2(x[2 * i], x[2 * i + 1], p0, p1, p2);
  out[3 * i] = p0;
  out[3 * i + 1] = p1;
  out[3 * i + 2] = p2;
}

// 16 independent pairs per lane, ITER rounds; the inputs are perturbed each round so nothing folds
template <int V>
__global__ void bench(const float* x, uint32_t* out, int iters) {
  float v[32];
  for (int j = 0; j < 32; ++j) v[j] = x[(threadIdx.x + 64 * j) & 1023];
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t p0, p1, p2;
      if (V == 0) split_ref(v[2 * j], v[2 * j + 1], p0, p1, p2);
      else split_dot2(v[2 * j], v[2 * j + 1], p0, p1, p2);
      acc ^= p0 ^ p1 ^ p2;
      asm volatile("" : "+v"(v[2 * j]), "+v"(v[2 * j + 1]));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int n = 1 << 20;
  std::vector<float> hx(2 * n);
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::uniform_int_distribution<int> e(-90, 90);
  for (int i = 0; i < 2 * n; ++i) {
    float v = u(rng) * std::ldexp(1.f, e(rng));
    if (i % 97 == 0) v = 0.f;
    if (i % 89 == 0) v = -0.f;
    hx[i] = v;
  }
  float* dx;
  uint32_t *d0, *d1;
  hipMalloc(&dx, sizeof(float) * 2 * n);
  hipMalloc(&d0, 12 * n);
  hipMalloc(&d1, 12 * n);
  hipMemcpy(dx, hx.data(), sizeof(float) * 2 * n, hipMemcpyHostToDevice);
  check<0><<<n / 256, 256>>>(dx, d0, n);
  check<1><<<n / 256, 256>>>(dx, d1, n);
  std::vector<uint32_t> h0(3 * n), h1(3 * n);
  hipMemcpy(h0.data(), d0, 12 * n, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), d1, 12 * n, hipMemcpyDeviceToHost);
  long bad = 0;
  for (int i = 0; i < 3 * n; ++i) bad += h0[i] != h1[i];
  // exactness of the reference split itself: a == p0 + p1 + p2 in fp64
  long inexact = 0;
  for (int i = 0; i < n; ++i)
    for (int s = 0; s < 2; ++s) {
      auto part = [&](uint32_t w) { return (double)__builtin_bit_cast(float, s ? (w & 0xffff0000u) : (w << 16)); };
      const double sum = part(h1[3 * i]) + part(h1[3 * i + 1]) + part(h1[3 * i + 2]);
      if (sum != (double)hx[2 * i + s]) ++inexact;
    }
  printf("parts differing (dot2 vs ref): %ld of %d; dot2 split inexact: %ld\n", bad, 3 * n, inexact);

  uint32_t* dout;
  hipMalloc(&dout, 4 * 1024 * 512);
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  const int iters = 2000;
  for (int wps : {1, 2}) {
    const int blocks = 256 * 4 * wps;   // one 64-thread block per wave: wps waves per SIMD
    for (int v = 0; v < 2; ++v) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(t0);
        if (v == 0) bench<0><<<blocks, 64>>>(dx, dout, iters);
        else bench<1><<<blocks, 64>>>(dx, dout, iters);
        hipEventRecord(t1);
        hipEventSynchronize(t1);
        float ms;
        hipEventElapsedTime(&ms, t0, t1);
        if (rep == 1)
          printf("%s waves/SIMD %d: %.3f ms, %.3f ns per wave pair-split per SIMD\n", v ? "dot2" : "ref ", wps, ms,
                 ms * 1e6 / ((double)iters * 16 * wps));
      }
    }
  }
  return 0;
}
