// FETCH_SIZE calibration (measurement tool): stream a 1 GiB buffer once with (a) global_load_lds
// dword (K1's staging form), (b) global_load_dwordx4 to registers (K2's form), (c) plain dword
// loads.  Run under rocprofv3 --pmc FETCH_SIZE and compare with 1 GiB.
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr size_t N = (size_t)1 << 28;  // floats = 1 GiB

__global__ __launch_bounds__(256) void dma_dword(const float* x, float* out) {
  extern __shared__ float sm[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc = 0.f;
  for (size_t base = ((size_t)blockIdx.x * 4 + w) * 64; base < N; base += (size_t)gridDim.x * 256) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(x + base + lane),
                                     (__attribute__((address_space(3))) void*)(sm + 64 * w), 4, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc += sm[64 * w + lane];
  }
  if (acc == 1234.5f) out[0] = acc;
}
__global__ __launch_bounds__(256) void vec16(const float* x, float* out) {
  float acc = 0.f;
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4; i < N; i += (size_t)gridDim.x * 1024) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}
__global__ __launch_bounds__(256) void dword(const float* x, float* out) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < N; i += (size_t)gridDim.x * 256) acc += x[i];
  if (acc == 1234.5f) out[0] = acc;
}
int main() {
  float *x, *o;
  hipMalloc(&x, N * 4); hipMalloc(&o, 64);
  hipMemset(x, 0, N * 4);
  hipDeviceSynchronize();
  dma_dword<<<2048, 256, 1024>>>(x, o);
  vec16<<<2048, 256>>>(x, o);
  dword<<<2048, 256>>>(x, o);
  hipDeviceSynchronize();
  printf("done: each kernel read %zu bytes\n", N * 4);
  return 0;
}
