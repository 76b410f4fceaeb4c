// gnca_aux.hip — step-adjacent batch ops of the rollout/training loop:
// the damage curriculum (reference: src/utils/damage.py:15-138), one launch for the whole batch.
//
// The reference loops over samples on the host, drawing each sample's position with a separate
// torch.randint(...).item()-style call (a device sync per sample on GPU) and applying a masked
// assignment per sample.  Here every sample's random draws arrive in device arrays and one
// elementwise kernel applies the damage to all of them.

#include "gnca_device.h"

namespace gnca {
namespace {

__global__ __launch_bounds__(kThreads) void gnca_damage(const gnca_damage_desc d, float* state,
                                                        const int32_t* pos, const float* noise) {
  const int C = d.C, H = d.H, W = d.W;
  const size_t HW = (size_t)H * W;
  const size_t cells = (size_t)d.B * HW;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < cells; e += (size_t)gridDim.x * kThreads) {
    const int b = (int)(e / HW);
    const size_t cell = e - (size_t)b * HW;
    const int i = (int)(cell / W), j = (int)(cell - (size_t)i * W);
    float* sb = state + (size_t)b * C * HW + cell;
    const int py = pos ? pos[2 * b] : 0, px = pos ? pos[2 * b + 1] : 0;
    const int sz = d.size;
    switch (d.kind) {
      case GNCA_DMG_SQUARE:        // damage.py:15-23
        if (i >= py && i < py + sz && j >= px && j < px + sz)
          for (int c = 0; c < C; ++c) sb[c * HW] = 0.f;
        break;
      case GNCA_DMG_CIRCLE: {      // damage.py:25-36 (float compare, as the reference)
        const float dy = (float)i - (float)py, dx = (float)j - (float)px;
        if (dy * dy + dx * dx <= (float)(sz * sz))
          for (int c = 0; c < C; ++c) sb[c * HW] = 0.f;
        break;
      }
      case GNCA_DMG_STRIPE_H:      // damage.py:38-50
        if (i >= py && i < py + sz)
          for (int c = 0; c < C; ++c) sb[c * HW] = 0.f;
        break;
      case GNCA_DMG_STRIPE_V:
        if (j >= px && j < px + sz)
          for (int c = 0; c < C; ++c) sb[c * HW] = 0.f;
        break;
      case GNCA_DMG_ALPHA_DROP:    // damage.py:52-65, hard: state *= (1 - drop)
      case GNCA_DMG_ALPHA_DROP_SOFT: {
        const float a = sb[3 * HW];
        const float drop = (noise[(size_t)b * HW + cell] < d.p ? 1.f : 0.f) * (a > d.alpha_thr ? 1.f : 0.f);
        if (d.kind == GNCA_DMG_ALPHA_DROP) {
          for (int c = 0; c < C; ++c) sb[c * HW] *= (1.f - drop);
        } else {
          sb[3 * HW] = a * (1.f - drop);
        }
        break;
      }
      case GNCA_DMG_SALT_PEPPER:   // damage.py:67-72
        sb[3 * HW] *= (1.f - (noise[(size_t)b * HW + cell] < d.p ? 1.f : 0.f));
        break;
      case GNCA_DMG_GAUSSIAN: {    // damage.py:82-97
        const float dy = (float)i - (float)py, dx = (float)j - (float)px;
        const float r2 = dy * dy + dx * dx;
        const float s = (float)sz * fmaxf(1e-6f, d.softness);
        const float m = expf(-(r2 / (2.f * s * s)));
        const float damp = fminf(fmaxf(1.f - m, 0.f), 1.f);
        for (int c = 0; c < C; ++c) sb[c * HW] *= damp;
        break;
      }
      case GNCA_DMG_HIDDEN_NOISE:  // damage.py:74-80
        for (int c = 4; c < C; ++c) {
          const float v = sb[c * HW] + noise[((size_t)b * (C - 4) + (c - 4)) * HW + cell] * d.sigma;
          sb[c * HW] = fminf(fmaxf(v, 0.f), 1.f);
        }
        break;
      default:
        break;
    }
  }
}

// loss_premult_rgba (train_graph_augmented_nca.py:52-61): one workgroup per sample, fixed-order
// fp64 reduction (deterministic)
__global__ __launch_bounds__(kThreads) void gnca_loss_fwd(int H, int W, const float* pred, long pbs,
                                                          const float* tgt, long tbs, float* out) {
  __shared__ double red[kThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t HW = (size_t)H * W;
  const float* p = pred + (size_t)b * pbs;
  const float* t = tgt + (size_t)b * tbs;
  double acc = 0.0;
  for (size_t e = tid; e < HW; e += kThreads) {
    const float a = p[3 * HW + e];
    float s = 0.f;
    for (int c = 0; c < 3; ++c) {
      const float r = p[c * HW + e] * a - t[c * HW + e];
      s = fmaf(r, r, s);
    }
    const float ra = a - t[3 * HW + e];
    acc += (double)fmaf(ra, ra, s);
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((tid & 63) == 0) red[tid >> 6] = acc;
  __syncthreads();
  if (tid == 0) {
    double v = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) v += red[w];
    out[b] = (float)(v / (4.0 * (double)HW));
  }
}

__global__ __launch_bounds__(kThreads) void gnca_loss_bwd(int B, int H, int W, const float* pred, long pbs,
                                                          const float* tgt, long tbs, const float* g,
                                                          float* gp, long gbs) {
  const size_t HW = (size_t)H * W, total = (size_t)B * HW;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += (size_t)gridDim.x * kThreads) {
    const size_t b = e / HW, q = e - b * HW;
    const float* p = pred + b * pbs;
    const float* t = tgt + b * tbs;
    float* o = gp + b * gbs;
    const float s = g[b] * (float)(2.0 / (4.0 * (double)HW));
    const float a = p[3 * HW + q];
    float ga = a - t[3 * HW + q];
    for (int c = 0; c < 3; ++c) {
      const float x = p[c * HW + q];
      const float r = x * a - t[c * HW + q];
      o[c * HW + q] = s * r * a;
      ga = fmaf(r, x, ga);
    }
    o[3 * HW + q] = s * ga;
  }
}

}  // namespace
}  // namespace gnca

using namespace gnca;

extern "C" int gnca_loss_premult_f32(int32_t B, int32_t H, int32_t W, const float* pred, int64_t pbs,
                                     const float* target, int64_t tbs, float* per_sample, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || !pred || !target || !per_sample) return GNCA_ERR_INVALID;
  hipLaunchKernelGGL(gnca_loss_fwd, dim3(B), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream), H, W,
                     pred, (long)pbs, target, (long)tbs, per_sample);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { g_last_hip = (int)e; return GNCA_ERR_HIP; }
  return GNCA_OK;
}

extern "C" int gnca_loss_premult_bwd_f32(int32_t B, int32_t H, int32_t W, const float* pred, int64_t pbs,
                                         const float* target, int64_t tbs, const float* g, float* grad_pred,
                                         int64_t gbs, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || !pred || !target || !g || !grad_pred) return GNCA_ERR_INVALID;
  const size_t total = (size_t)B * H * W;
  size_t blocks = (total + kThreads - 1) / kThreads;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gnca_loss_bwd, dim3((unsigned)blocks), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     B, H, W, pred, (long)pbs, target, (long)tbs, g, grad_pred, (long)gbs);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { g_last_hip = (int)e; return GNCA_ERR_HIP; }
  return GNCA_OK;
}

extern "C" int gnca_damage_f32(const gnca_damage_desc* d, float* state, const int32_t* pos,
                               const float* noise, void* stream) {
  if (!d || !state || d->B <= 0 || d->C < 4 || d->H <= 0 || d->W <= 0) return GNCA_ERR_INVALID;
  if (d->kind < GNCA_DMG_SQUARE || d->kind > GNCA_DMG_HIDDEN_NOISE) return GNCA_ERR_INVALID;
  const bool geo = d->kind == GNCA_DMG_SQUARE || d->kind == GNCA_DMG_CIRCLE || d->kind == GNCA_DMG_STRIPE_H ||
                   d->kind == GNCA_DMG_STRIPE_V || d->kind == GNCA_DMG_GAUSSIAN;
  if (geo && !pos) return GNCA_ERR_INVALID;
  if (!geo && !noise) return GNCA_ERR_INVALID;
  if (d->kind == GNCA_DMG_HIDDEN_NOISE && d->C <= 4) return GNCA_OK;
  const size_t cells = (size_t)d->B * d->H * d->W;
  size_t blocks = (cells + kThreads - 1) / kThreads;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gnca_damage, dim3((unsigned)blocks), dim3(kThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), *d, state, pos, noise);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return GNCA_ERR_HIP;
  }
  return GNCA_OK;
}
