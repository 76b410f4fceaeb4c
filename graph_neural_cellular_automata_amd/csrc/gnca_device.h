// gnca_device.h — device helpers shared by the forward (gnca_step.hip) and backward
// (gnca_bwd.hip) translation units of libgnca.so.
#pragma once

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include "gnca.h"

namespace gnca {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;

// Environment knobs that change kernel selection or geometry exist only in measurement builds
// (-DGNCA_AB_KNOBS, tools/ A/B scripts): in the shipped library the environment cannot change
// which product kernel runs.
#ifdef GNCA_AB_KNOBS
#define GNCA_AB_ENV(name) getenv(name)
#else
#define GNCA_AB_ENV(name) ((const char*)nullptr)
#endif

// Measurement (gnca_rollout_stamped_f32): per-workgroup wall-clock stamps from the 100 MHz
// s_memrealtime counter, st[2 * blockIdx.x + which] (0 = first instruction, 1 = after the
// workgroup's last barrier).  st == NULL (every product launch): one uniform branch, no store.
__device__ __forceinline__ void wg_stamp(uint64_t* st, int which) {
  if (st != nullptr && threadIdx.x == 0) st[2 * blockIdx.x + which] = __builtin_amdgcn_s_memrealtime();
}
#define GNCA_STAMP_END(st) do { if ((st) != nullptr) { __syncthreads(); wg_stamp((st), 1); } } while (0)

// Host: the device that owns `stream` is made current for the scope of an entry point and the
// caller's current device restored on exit, so the per-device caches (CU count, occupancy,
// helper streams and events) and every launch refer to the stream's device even when the caller
// passes a stream of a device that is not current (e.g. a cuda:1 tensor while cuda:0 is current).
struct StreamDeviceGuard {
  int prev = -1;
  explicit StreamDeviceGuard(hipStream_t stream) {
    int cur = 0;
    hipDevice_t dev = 0;
    if (stream == nullptr || hipGetDevice(&cur) != hipSuccess) return;
    if (hipStreamGetDevice(stream, &dev) != hipSuccess || (int)dev == cur) return;
    if (hipSetDevice((int)dev) == hipSuccess) prev = cur;
  }
  ~StreamDeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  StreamDeviceGuard(const StreamDeviceGuard&) = delete;
  StreamDeviceGuard& operator=(const StreamDeviceGuard&) = delete;
};

__device__ __forceinline__ int wrapi(int v, int n) {
  v %= n;
  return v < 0 ? v + n : v;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Counter-based fire RNG (the build's definition; oracle/nca_oracle.py:hash_uniform).
__device__ __forceinline__ float hash_uniform(uint64_t seed, int64_t step, uint64_t sample,
                                              uint64_t cell) {
  const uint64_t k = mix64(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(uint32_t)(step + 1));
  const uint64_t key = mix64(k ^ (sample << 32) ^ cell);
  return (float)(key >> 40) * (1.0f / 16777216.0f);
}

// The fire predicate of one cell (ncagraph.py:144-146), for every GNCA_FIRE_* mode.
__device__ __forceinline__ bool fire_at(int mode, const void* fire, float rate, uint64_t seed,
                                        int64_t step, int64_t sample_base, int b, size_t HW,
                                        size_t cell) {
  if (mode == GNCA_FIRE_RAND_F32) return reinterpret_cast<const float*>(fire)[(size_t)b * HW + cell] <= rate;
  if (mode == GNCA_FIRE_MASK_U8) return reinterpret_cast<const uint8_t*>(fire)[(size_t)b * HW + cell] != 0;
  if (mode == GNCA_FIRE_HASH) return hash_uniform(seed, step, (uint64_t)(sample_base + b), cell) <= rate;
  return true;
}

// tanh(x) = 1 - 2 / (exp(2x) + 1): v_exp + v_rcp; abs error ~2e-7 (saturates to +-1, NaN-preserving).
// K2's update tanh (and BA's recompute of the updated alpha, which must give K2's gate bits).
__device__ __forceinline__ float fast_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // exp(2x)
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

__host__ __device__ inline int r4(int v) { return (v + 3) & ~3; }

// The zero-padded shift's per (channel, row) fp64 sums of x (K0's pooled logits, BD), in ONE
// canonical order that every producer follows, so that K2's fused sums (a rollout's next step) and
// K0's own pass (single steps, a rollout's first step) give the same bits:
//  * the row's cells in vectors of V = 4 (W % 4 == 0) or 1; P_k = ((v0 + v1) + (v2 + v3)) in fp64
//    (V = 4) or v0;
//  * 32 consecutive vectors per segment, lane k of a 32-lane half-wave holding P_k (+0.0 past the
//    row's end), summed by an xor butterfly (16, 8, 4, 2, 1);
//  * the segments' sums added in order (the first one as is).
template <int V>
__device__ __forceinline__ double canon_vec_sum(const float* v) {
  if constexpr (V == 4) return ((double)v[0] + (double)v[1]) + ((double)v[2] + (double)v[3]);
  else return (double)v[0];
}

// every lane of the wave calls it (the shuffles); the 32-lane half-waves reduce independently
__device__ __forceinline__ double canon_butterfly32(double p) {
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) p += __shfl_xor(p, off);
  return p;
}

// rows r = h, h + nh, ... of the [n_rows][W] planes at x (row r at x + r * W) into rs[r]: half-wave h
// of nh, lane k = lane & 31.  U rows per half-wave in flight.  Every lane of the calling waves calls it.
template <int V, int U>
__device__ __forceinline__ void canon_row_sums(const float* x, int n_rows, int W, double* rs, int h, int nh, int k) {
  typedef float vf __attribute__((ext_vector_type(V)));
  const int nvr = W / V;
  for (int r0 = 0; r0 < n_rows; r0 += U * nh) {   // uniform over the workgroup
    double S[U];
#pragma unroll
    for (int u = 0; u < U; ++u) S[u] = 0.0;
    for (int s0 = 0; s0 < nvr; s0 += 32) {
      vf v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * nh + h, q = s0 + k;
        if (r < n_rows && q < nvr) v[u] = *reinterpret_cast<const vf*>(x + (size_t)r * W + (size_t)V * q);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * nh + h, q = s0 + k;
        float f[V];
#pragma unroll
        for (int i = 0; i < V; ++i) f[i] = v[u][i];
        const double p = canon_butterfly32((r < n_rows && q < nvr) ? canon_vec_sum<V>(f) : 0.0);
        S[u] = s0 == 0 ? p : S[u] + p;
      }
    }
    if (k == 0)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * nh + h;
        if (r < n_rows) rs[r] = S[u];
      }
  }
}
__host__ __device__ constexpr int odd4(int v) {  // round up to 4*odd: conflict-free 16-lane b128
  return ((((v + 3) & ~3) >> 2) & 1) ? ((v + 3) & ~3) : ((v + 3) & ~3) + 4;
}

// dst[idx] = f(idx) for idx < n (dst in LDS), U values per thread in flight: a plain strided loop
// waits out one global-load latency per element (~1 us at one workgroup per CU), which is what
// dominates a small-batch launch's prologue.
template <int NT, int U, class F>
__device__ __forceinline__ void lds_fill(float* dst, int n, int tid, F f) {
  for (int base = tid; base < n; base += NT * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * NT;
      v[u] = idx < n ? f(idx) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = base + u * NT;
      if (idx < n) dst[idx] = v[u];
    }
  }
}

// A compile-time-sized LDS fill split into its load half and its store half, so several fills can
// have ALL their global loads in flight before the first LDS store (one load latency for a whole
// weight set instead of one per fill batch: the prologue of a small-batch launch).
template <int NT, int N>
struct RegFill {
  static constexpr int U = (N + NT - 1) / NT;
  float v[U];
  template <class F>
  __device__ __forceinline__ void load(int tid, F f) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + u * NT;
      v[u] = idx < N ? f(idx) : 0.f;
    }
  }
  __device__ __forceinline__ void store(float* dst, int tid) const {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + u * NT;
      if (idx < N) dst[idx] = v[u];
    }
  }
  // element idx to dst[map(idx)]
  template <class M>
  __device__ __forceinline__ void store_map(float* dst, int tid, M map) const {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = tid + u * NT;
      if (idx < N) dst[map(idx)] = v[u];
    }
  }
};

// Sequential (fixed-order, bit-reproducible) sums of the pairs p[t*stride], p[t*stride+1],
// t < n, with 8 loads in flight instead of one dependent load per term.
__device__ __forceinline__ void seq_sum2(const double* p, int n, int stride, double* s0, double* s1) {
  double a = 0.0, b = 0.0;
  for (int t0 = 0; t0 < n; t0 += 8) {
    double va[8], vb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = t0 + u < n;
      va[u] = ok ? p[(size_t)(t0 + u) * stride] : 0.0;
      vb[u] = ok ? p[(size_t)(t0 + u) * stride + 1] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (t0 + u < n) {
        a += va[u];
        b += vb[u];
      }
  }
  *s0 = a;
  *s1 = b;
}

// Deterministic sums of the pairs p[stride*t], p[stride*t + 1], t < n, by one whole wave: lane l
// adds pairs l, l+64, l+128, ... in that order (4 loads in flight per lane), then a fixed xor
// butterfly combines the lanes.  The order depends only on n, so every consumer of the same
// partials (K2, the backward's BA / BS) gets the same bits.  Every lane of the wave must call
// it; all get the sums.
__device__ __forceinline__ void wave_sum2(const double* p, int n, double* s0, double* s1,
                                          int stride = 2) {
  const int lane = threadIdx.x & 63;
  double x = 0.0, y = 0.0;
  for (int t0 = lane; t0 < n; t0 += 4 * 64) {
    double a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + 64 * j;
      a[j] = t < n ? p[(size_t)stride * t] : 0.0;
      b[j] = t < n ? p[(size_t)stride * t + 1] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x += a[j];
      y += b[j];
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    x += __shfl_xor(x, off);
    y += __shfl_xor(y, off);
  }
  *s0 = __shfl(x, 0);   // lane 0's association order, on every lane
  *s1 = __shfl(y, 0);
}

// wave_sum2 for n <= 256 pairs with the pairs already in registers (lane l holds pairs l + 64 j,
// j = 0..3, zeros past n): the same additions in the same order, so the same bits.  Lets a caller
// issue the partials' loads together with its other loads.
__device__ __forceinline__ void wave_sum2_regs(const double (&a)[4], const double (&b)[4], double* s0,
                                               double* s1) {
  double x = 0.0, y = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x += a[j];
    y += b[j];
  }
  for (int off = 32; off > 0; off >>= 1) {
    x += __shfl_xor(x, off);
    y += __shfl_xor(y, off);
  }
  *s0 = __shfl(x, 0);
  *s1 = __shfl(y, 0);
}

// Where the forward keeps its intermediates in the step workspace (gnca_step.hip:make_plan);
// the backward recomputes them there.
struct FwdLayout {
  size_t ws_bytes, off_dx, off_stats, off_offw;
  size_t off_rs;   // K0's per-(channel, row) fp64 sums of x (zero-pad mode), for the backward's BD
  int tps, k;
  bool graph_on, need_k0;
};
bool fwd_layout(const gnca_step_desc* d, FwdLayout* out);

// gnca_step_phases_f32 restricted to active samples (the masked step; used by the backward)
int gnca_step_masked_phases(const gnca_step_desc* d, const gnca_weights* w, const float* x, float* x_out,
                            const void* fire, const uint8_t* active, void* ws, size_t ws_bytes,
                            void* stream, uint32_t phases);

// hipError_t of the last failed launch on this thread (gnca_last_hip_error)
extern thread_local int g_last_hip;

}  // namespace gnca
