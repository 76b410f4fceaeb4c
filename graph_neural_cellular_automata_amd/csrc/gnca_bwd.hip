// gnca_bwd.hip — MI355X (gfx950 / CDNA4) backward of the NCA step (BPTT), SURVEY.md §8f rank 1.
//
// The vector-Jacobian product of one step (reference forward: src/modules/ncagraph.py:106-168,
// src/modules/nca.py:64-105, src/modules/graph_augmentation.py:104-169; the reference gets its
// gradients from torch autograd in the trainers' loss.backward(),
// src/training/train_graph_augmented_nca.py:369).  Restated in numpy by
// oracle/nca_oracle_vjp.py (test infrastructure), which is pinned to the reference's autograd.
//
// Nothing is saved by the forward: the backward recomputes it.
//
//   F   forward K0/K1 (gnca_step.hip) into the workspace: dx (pre-GroupNorm update, masked),
//       per-tile GroupNorm partials, zero-pad offset weights.
//   BA  gnca_b_gnprep     per (sample, row band): post-update gate (3x3 halo), tanh', GroupNorm
//                         backward prep:  gx = gy*gate (the residual),  U = gamma*g_xn,
//                         fp64 partials of sum U, sum U*xhat (per sample) and of the norm
//                         weight/bias gradients (per channel).
//   BS  gnca_b_coef       per sample: mean, rstd, mean(U), mean(U*xhat).
//   BB  gnca_b_mlp<CP,HB> the MFMA kernel, persistent, one hidden slice of HB units per launch:
//                         recompute perception / gather / GEMM1 / message, then
//                           d_pre = keep * rstd*(U - mean U - xhat*mean(U xhat))   (GN backward)
//                           dh = relu'(h) * W2^T d_pre        (MFMA)
//                           dY = W1^T dh     -> HBM           (MFMA; the perception adjoint's input)
//                           dm = d_pre*gain*tanh'(m); dG = W_M^T dm -> HBM  (MFMA)
//                         and the weight gradients dW1 = dh y^T, dW2 = d_pre h^T, dW_M = dm G^T
//                         on MFMA with the cell dimension as K (per-wave LDS transposes; per-wave
//                         register accumulators for the whole launch), db1, db_M.
//   BC  gnca_b_adjoint    gx += Sobel^T dY + A_send * sum_o w_o dG(q+o)  (adjoint of the
//                         zero-padded 3x3 correlation and of the rolled / row-shifted gather).
//   zero-pad mode only (offset weights depend on x, Q, K, scaling):
//   BC2 gnca_b_dots       per (sample, offset): dL/dw_o = sum_q A(q) (<dG(q+o), x(q)> + <dm(q+o), b_M>)
//   BD  gnca_b_attn       softmax / pooled-logit backward per sample (fp64): Q, K, scaling grads,
//                         and the per-row correction of gx through the pooled means.
//   BE  gnca_b_rowcorr    gx += corr[b, row, c].
//   R   gnca_b_reduce     fixed-order sums of the per-wave / per-band / per-sample partials into
//                         the caller's gradient buffers (deterministic: no float atomics).

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "gnca_device.h"

namespace gnca {
namespace {

constexpr int NW = kThreads / 64;
__device__ float g_bzero[4];   // LDS-DMA source for off-image cells (zero-initialised)
constexpr uint32_t kMsg = 1u << 16;      // message path active (k > 0 and message_gain != 0)
constexpr uint32_t kFirst = 1u << 17;    // first hidden slice: also the message backward
constexpr uint32_t kGN = 1u << 18;       // GroupNorm on
constexpr uint32_t kDma4 = 1u << 20;     // BB: 16-byte LDS-DMA staging (W, TW and the x halo multiples of 4)
constexpr uint32_t kZeroed = 1u << 19;   // dY / dG / dmb were zero-filled before BB: no dead-cell zero stores

// Measurement-only phase timers of BB (tools/bprof.py builds with -DGNCA_PROFILE): wave 0 of each
// workgroup accumulates s_memtime deltas per phase; gnca_bprof_dump copies them out.
#ifdef GNCA_PROFILE
constexpr int kBProfPhases = 8;
__device__ unsigned long long g_bprof[1024][kBProfPhases];
#define BPROF_DECL unsigned long long prof_t = __builtin_amdgcn_s_memtime(), prof_acc[kBProfPhases] = {0};
#define BPROF_MARK(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#define BPROF_STORE do { if (threadIdx.x == 0) for (int i_ = 0; i_ < kBProfPhases; ++i_) g_bprof[blockIdx.x & 1023][i_] = prof_acc[i_]; } while (0)
#else
#define BPROF_DECL
#define BPROF_MARK(i) do {} while (0)
#define BPROF_STORE do {} while (0)
#endif

__host__ __device__ inline int s16(int v) {  // >= v, multiple of 16, == 16 mod 32 (bank spread)
  const int s = (v + 15) & ~15;
  return (s & 31) == 16 ? s : s + 16;
}

__device__ __forceinline__ double2 block_sum2(double a, double b, double* red) {
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[2 * wave] = a;
    red[2 * wave + 1] = b;
  }
  __syncthreads();
  double ta = 0.0, tb = 0.0;
  for (int w = 0; w < NW; ++w) {  // fixed order: deterministic
    ta += red[2 * w];
    tb += red[2 * w + 1];
  }
  __syncthreads();
  return make_double2(ta, tb);
}


// ------------------------------------------------------------------------------------------
// BA: gate / tanh / GroupNorm backward prep (ncagraph.py:153-166)
// ------------------------------------------------------------------------------------------
struct BAArgs {
  const float* x;
  const float* dx;
  const float* gy;
  const float* gamma;
  const float* beta;
  const double* stats;
  float* gx;
  float* U;
  double* part;   // [B * nbands][2 + 2C]: sum U, sum U*xhat, then (sum g_xn*xhat, sum g_xn) per c
  const uint8_t* active;   // masked step: inactive samples pass the gradient through
  int B, C, H, W, tps, band, nbands;
  float gain, thr, eps;
  int use_gn;
};

__global__ __launch_bounds__(kThreads) void gnca_b_gnprep(const BAArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double red[2 * NW];
  __shared__ float sh[2];
  const int tid = threadIdx.x;
  const int b = blockIdx.x / a.nbands, band = blockIdx.x - b * a.nbands;
  const int C = a.C, H = a.H, W = a.W;
  const int r0 = band * a.band, r1 = min(H, r0 + a.band);
  const int h0 = max(0, r0 - 1), h1 = min(H, r1 + 1);
  const size_t HW = (size_t)H * W;
  const bool gn = a.use_gn != 0;
  if (a.active && !a.active[b]) {   // x_out = x for this sample: gx = gy, nothing else
    const int nbc = (r1 - r0) * W;
    for (int it = tid; it < C * nbc; it += kThreads) {
      const int c = it / nbc, e = it - c * nbc;
      const size_t p = (size_t)b * C * HW + (size_t)c * HW + (size_t)r0 * W + e;
      a.gx[p] = a.gy[p];
      a.U[p] = 0.f;
    }
    if (tid < 2 + 2 * C) a.part[(size_t)blockIdx.x * (2 + 2 * C) + tid] = 0.0;
    return;
  }
  const int lane = tid & 63, wave = tid >> 6;
  const float* xb = a.x + (size_t)b * C * HW;
  const float* db = a.dx + (size_t)b * C * HW;
  const float* gb = a.gy + (size_t)b * C * HW;
  float* gxb = a.gx + (size_t)b * C * HW;
  float* ub = a.U + (size_t)b * C * HW;
  float* at = smem;                                  // updated alpha, band rows + halo
  float* post = smem + (size_t)(a.band + 2) * W;     // post-update alive mask of the band
  const int na = (h1 - h0) * W, nb = (r1 - r0) * W;
  const size_t base = (size_t)r0 * W;
  // Latency first: the alpha rows and this wave's first channel block are loaded before the
  // per-sample statistics are known (one memory latency for the prologue of a small band).
  constexpr int NA = 2;
  float ax[NA], ad[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int e = tid + u * kThreads;
    if (e < na) {
      const size_t p = 3 * HW + (size_t)h0 * W + e;
      ax[u] = xb[p];
      ad[u] = db[p];
    }
  }
  // one wave per channel (c = cb + wave + NW*j), JM channels of the wave in flight at once
  constexpr int JM = 4;
  float dv[JM][4], gv[JM][4];
  auto load_block = [&](int cb, int e0) {
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const int c = cb + wave + NW * j;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 64 * u + lane;
        const size_t p = (size_t)c * HW + base + e;
        const bool ok = c < C && e < nb;
        dv[j][u] = ok ? db[p] : 0.f;
        gv[j][u] = ok ? gb[p] : 0.f;
      }
    }
  };
  load_block(0, 0);
  if (wave == 0) {
    float mu = 0.f, rs = 1.f;
    if (gn) {
      double t1, t2;   // wave_sum2, as the forward K2: the same mean / rstd bit for bit
      wave_sum2(a.stats + (size_t)b * a.tps * 2, a.tps, &t1, &t2);
      const double n = (double)C * (double)HW;
      const double m = t1 / n;
      double var = t2 / n - m * m;
      if (var < 0.0) var = 0.0;
      mu = (float)m;
      rs = (float)(1.0 / sqrt(var + (double)a.eps));
    }
    if (lane == 0) {
      sh[0] = mu;
      sh[1] = rs;
    }
  }
  __syncthreads();
  const float mu = sh[0], rs = sh[1];
  {
    const float g3 = gn ? a.gamma[3] : 1.f, b3 = gn ? a.beta[3] : 0.f;
    auto alpha_at = [&](float xa, float d) {
      if (gn) d = (d - mu) * rs * g3 + b3;   // the forward K2's expression for alpha
      return xa + fast_tanh(d) * a.gain;   // K2's expression, bit for bit
    };
#pragma unroll
    for (int u = 0; u < NA; ++u) {
      const int e = tid + u * kThreads;
      if (e < na) at[e] = alpha_at(ax[u], ad[u]);
    }
    for (int e = tid + NA * kThreads; e < na; e += kThreads) {
      const size_t p = 3 * HW + (size_t)h0 * W + e;
      at[e] = alpha_at(xb[p], db[p]);
    }
  }
  __syncthreads();
  for (int e = tid; e < nb; e += kThreads) {
    const int i = r0 + e / W, j = e - (e / W) * W;
    float mx = -INFINITY;
    for (int ii = max(0, i - 1); ii <= min(H - 1, i + 1); ++ii) {
      const float* row = at + (size_t)(ii - h0) * W;
      mx = fmaxf(mx, row[j]);
      if (j > 0) mx = fmaxf(mx, row[j - 1]);
      if (j < W - 1) mx = fmaxf(mx, row[j + 1]);
    }
    post[e] = mx > a.thr ? 1.f : 0.f;
  }
  __syncthreads();
  double su = 0.0, sux = 0.0;
  double* outp = a.part + (size_t)blockIdx.x * (2 + 2 * C);
  for (int cb = 0; cb < C; cb += NW * JM) {
  double sg[JM], sgx[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) { sg[j] = 0.0; sgx[j] = 0.0; }
  for (int e0 = 0; e0 < nb; e0 += 4 * 64) {
    if (e0 > 0 || cb > 0) load_block(cb, e0);
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const int c = cb + wave + NW * j;
      if (c >= C) continue;
      const float gc = gn ? a.gamma[c] : 1.f, bc = gn ? a.beta[c] : 0.f;
      const float gcr = gc * rs;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + 64 * u + lane;
        if (e >= nb) continue;
        const size_t p = (size_t)c * HW + base + e;
        const float d = dv[j][u];
        const float xhat = (d - mu) * rs;
        const float xn = gn ? (c == 3 ? (d - mu) * rs * gc + bc : (d - mu) * gcr + bc) : d;
        const float t = tanhf(xn);
        float g = gv[j][u];
        if (c == 3) g *= post[e];                       // x * gate, gate on alpha only (:158-166)
        gxb[p] = g;                                     // the residual x + ... (:155)
        const float gxn = g * a.gain * (1.f - t * t);   // tanh(.)*update_gain (:154)
        const float uu = gn ? gxn * gc : gxn;
        ub[p] = uu;
        sg[j] += (double)gxn;
        sgx[j] += (double)gxn * (double)xhat;
        su += (double)uu;
        sux += (double)uu * (double)xhat;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int c = cb + wave + NW * j;
    if (c >= C) continue;
    double x1 = sg[j], x2 = sgx[j];
    for (int off = 32; off > 0; off >>= 1) {
      x1 += __shfl_xor(x1, off);
      x2 += __shfl_xor(x2, off);
    }
    if (lane == 0) {
      outp[2 + 2 * c] = x2;
      outp[3 + 2 * c] = x1;
    }
  }
  }
  const double2 r = block_sum2(su, sux, red);
  if (tid == 0) {
    outp[0] = r.x;
    outp[1] = r.y;
  }
}

// BS: per-sample GroupNorm-backward coefficients (mu, rstd, mean U, mean U*xhat)
// one wave per sample: both partial lists load in one memory latency (wave_sum2, as the forward
// K2, so mean / rstd are the forward's bit for bit)
__global__ __launch_bounds__(64) void gnca_b_coef(const double* stats, const double* part,
                                                  float* coef, int B, int C, int HW, int tps,
                                                  int nbands, float eps, int use_gn) {
  const int b = blockIdx.x;
  float mu = 0.f, rs = 1.f, mu_u = 0.f, mu_ux = 0.f;
  if (use_gn) {
    const double n = (double)C * (double)HW;
    double t1, t2, su, sux;
    wave_sum2(stats + (size_t)b * tps * 2, tps, &t1, &t2);
    wave_sum2(part + (size_t)b * nbands * (2 + 2 * C), nbands, &su, &sux, 2 + 2 * C);
    const double m = t1 / n;
    double var = t2 / n - m * m;
    if (var < 0.0) var = 0.0;
    mu = (float)m;
    rs = (float)(1.0 / sqrt(var + (double)eps));
    mu_u = (float)(su / n);
    mu_ux = (float)(sux / n);
  }
  if (threadIdx.x == 0) {
    coef[4 * b + 0] = mu;
    coef[4 * b + 1] = rs;
    coef[4 * b + 2] = mu_u;
    coef[4 * b + 3] = mu_ux;
  }
}

// ------------------------------------------------------------------------------------------
// BB: the MFMA kernel
// ------------------------------------------------------------------------------------------
struct BBLayout {
  int xs, PSTR, al, ALW, sp, kp, lst, w1f, KSP, w1t, S1T, w2t, S2T, wms, SWM, b1s, bms, percs, wts, scr;
  int ST1, ST2, ST3, SCRW, RH, RW, NI, NIA, total;
};

// lean (the large-tile instances, LL below): no W1^T image (dY's A fragments are read from the W1
// image, one float each) and the per-wave dh / h transposes staged half a slice at a time, so that a
// 24x24 tile's 32x32 staged region fits 160 KB
__host__ __device__ inline BBLayout bb_layout(int CP, int HB, int TH, int TW, int RY, int RX, int kmax,
                                              bool lean = false) {
  BBLayout L;
  L.RH = TH + 2 * RY;
  L.RW = TW + 2 * RX;
  L.NI = (L.RH * L.RW + 63) / 64;          // LDS-DMA wave instructions per channel plane
  L.PSTR = 64 * L.NI + 16;
  L.ALW = L.RW + 2;
  L.NIA = ((L.RH + 2) * L.ALW + 63) / 64;
  const int CPM = 16 * ((CP + 15) / 16);   // channel rows padded to whole 16-row MFMA tiles
  const int MT = HB / 16, MO = (CP + 15) / 16, FT = (3 * CP + 15) / 16;
  L.KSP = odd4(3 * CP / 4);   // MFMA A-fragments, one 16-byte LDS read per 4 k-steps (as K1)
  L.S1T = odd4(4 * MT);
  L.S2T = odd4(4 * MO);
  L.SWM = odd4(CPM);
  L.ST1 = s16(lean ? HB / 2 : HB);
  L.ST2 = s16(3 * CP);
  L.ST3 = s16(CP);
  L.SCRW = 16 * (L.ST1 + std::max(L.ST2, 2 * L.ST3));   // T3/T4 reuse T2's rows (after dW1)
  int o = 0;
  L.xs = o; o += CP * L.PSTR;
  L.al = o; o += 64 * L.NIA;
  L.sp = o; o += r4(L.RH * L.RW);
  L.kp = o; o += r4(TH * TW);
  L.lst = o; o += r4(TH * TW) + 8;   // compacted live-cell list + per-wave counts
  L.w1f = o; o += MT * (64 * L.KSP + (lean ? 12 : 0));   // W1 fragments (GEMM1 recompute; lean: row skew)
  L.w1t = o; o += lean ? 0 : FT * 64 * L.S1T;   // W1^T fragments (dY = W1^T dh)
  L.w2t = o; o += MT * 64 * L.S2T;   // W2^T fragments (dh = W2^T d_pre)
  L.wms = o; o += CPM * L.SWM;
  L.b1s = o; o += r4(HB);
  L.bms = o; o += CPM;
  L.percs = o; o += CP * 36;
  L.wts = o; o += r4(kmax > 0 ? kmax : 4);
  L.scr = o; o += NW * L.SCRW;
  L.total = o;
  return L;
}

struct BBArgs {
  const float* x;
  const float* U;
  const float* dx;
  const float* coef;
  const void* fire;
  const float* perc;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* wm;
  const float* bm;
  const float* offw;   // [B*k] zero-pad weights or null (uniform 1/k)
  const uint8_t* active;   // masked step: inactive samples have no update (all cells dead)
  float* dY;           // [B, 3C, H, W]
  float* dG;           // [B, C, H, W]
  float* dmb;          // [B, H, W] <dm, b_M> (zero-pad only) or null
  // [B, H, W] keep bytes (fire AND pre-alive) written by the first slice, or null: then the dead
  // cells' dY / dG / dmb are not stored at all and their readers (BC, BC2) take them as zeros
  // from the keep plane; null (A/B builds): the dead cells' zeros are stored
  uint8_t* keep;
  // masked step (torus): the active samples in order, their count at alist[B] (gnca_b_actlist), or
  // null: the persistent grid then walks only the active samples' tiles, evenly over the workgroups
  const int* alist;
  float* part;         // [gridDim.x * NW][npart]
  uint64_t seed;
  int64_t rng_step;
  int64_t sample_base;
  int B, C, H, W, hidden, h0, k, RY, RX, TH, TW, tiles_x, tps, total_tiles, fire_mode;
  int npart, o_w1, o_b1, o_w2, o_wm, o_bm;
  float fire_rate, alpha_thr, graph_alpha_thr, message_gain, uniform_w;
  uint32_t flags;
  int odl[GNCA_MAX_OFFSETS];
};

// FULL: C == CP (no padded channels), so every per-lane channel test is a compile-time constant: at
// runtime C those tests were 64-bit lane masks held across the group loop (SGPR spills)
// TH_ .. K_ (all > 0, K_ >= 0): the tile geometry and offset count at compile time (the planned
// shapes of the C = 16 graph and classic steps, kBBS below): every LDS offset and loop bound a constant
#ifndef GNCA_BB_W1SKEW
#define GNCA_BB_W1SKEW 1      // the lean instances skew the W1 image's rows by 4 (lane >> 4) floats (A/B: 0)
#endif
// LL: the lean LDS layout (bb_layout's `lean`) of the large-tile instances
template <int CP, int HB, bool FULL = false, int TH_ = 0, int TW_ = 0, int RY_ = 0, int RX_ = 0, int K_ = -1,
          bool LL = false>
__global__ __launch_bounds__(kThreads, 1) void gnca_b_mlp(const BBArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int CPQ = CP / 4, KS = 3 * CPQ, MT = HB / 16, MO = (CP + 15) / 16, FT = (3 * CP + 15) / 16;
  const int TH = TH_ ? TH_ : a.TH, TW = TW_ ? TW_ : a.TW, RY = RY_ ? RY_ : a.RY, RX = RX_ ? RX_ : a.RX;
  static_assert(!LL || (HB / 16) % 2 == 0, "lean layout: two halves of whole 16-unit tiles");
  const BBLayout L = bb_layout(CP, HB, TH, TW, RY, RX, K_ >= 0 ? K_ : a.k, LL);
  constexpr bool W1SK = LL && GNCA_BB_W1SKEW;
  const int RH = L.RH, RW = L.RW, PSTR = L.PSTR, ALW = L.ALW;
  const int KSP = L.KSP, S1T = L.S1T, S2T = L.S2T, SWM = L.SWM, ST1 = L.ST1, ST2 = L.ST2, ST3 = L.ST3;
  float* xs = smem + L.xs;
  float* al = smem + L.al;
  float* sp = smem + L.sp;
  float* fp = smem + L.kp;
  float* w1f = smem + L.w1f;
  float* w1t = smem + L.w1t;
  float* w2t = smem + L.w2t;
  float* wms = smem + L.wms;
  float* b1s = smem + L.b1s;
  float* bms = smem + L.bms;
  float* percs = smem + L.percs;
  float* wts = smem + L.wts;

  BPROF_DECL
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int C = FULL ? CP : a.C, H = a.H, W = a.W, Hd = a.hidden, h0 = a.h0, k = K_ >= 0 ? K_ : a.k;
  const bool zp = (a.flags & GNCA_ZERO_PAD_SHIFT) != 0;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const bool msg = (a.flags & kMsg) != 0;
  const bool first = (a.flags & kFirst) != 0;
  const bool msg_bwd = msg && first;
  const bool gn = (a.flags & kGN) != 0;
  const bool uniform_w = a.offw == nullptr;
  const float thr = a.alpha_thr, gthr = a.graph_alpha_thr;
  float* T1 = smem + L.scr + wave * L.SCRW;   // per-wave transpose scratch [16 cells][...]
  float* T2 = T1 + 16 * ST1;
  float* T3 = T2;                             // d_pre / dm rows, after T2 (y) has been consumed
  float* T4 = T3 + 16 * ST3;

  // ---- weights of this hidden slice -> LDS (row-major; strides chosen bank-conflict-free for
  //      both the forward (W1) and the transposed (W1^T, W2^T, W_M^T) fragment reads) ----
  auto w1at = [&](int hid, int slot) -> float {   // W1[hid][slot], slot = f*CP + c; 0 = padding
    const int f = slot / CP, c = slot - f * CP;
    return (hid < Hd && slot < 3 * CP && c < C) ? a.w1[(size_t)hid * 3 * C + f * C + c] : 0.f;
  };
  // every load of the slice's weight set in flight before the first LDS store (one memory
  // latency for the prologue: most of a small-batch launch)
  {
    constexpr int cKSP = odd4(3 * CP / 4), cS1T = odd4(4 * MT), cS2T = odd4(4 * MO);
    constexpr int cSWM = odd4(16 * MO);
    RegFill<kThreads, MT * 64 * cKSP> f1;
    RegFill<kThreads, FT * 64 * cS1T> f2;
    RegFill<kThreads, MT * 64 * cS2T> f3;
    RegFill<kThreads, 16 * MO * cSWM> f4_;
    RegFill<kThreads, HB> f5;
    RegFill<kThreads, 16 * MO> f6;
    RegFill<kThreads, CP * 36> f7;
    f1.load(tid, [&](int idx) {   // A[hid][slot], k-step s
      const int s = idx % cKSP, ml = idx / cKSP, l = ml & 63, m = ml >> 6;
      return s < KS ? w1at(h0 + 16 * m + (l & 15), 4 * s + (l >> 4)) : 0.f;
    });
    if constexpr (!LL) f2.load(tid, [&](int idx) {   // A[slot][hid], k-step (m, r)
      const int e = idx % cS1T, fl = idx / cS1T, l = fl & 63, ft = fl >> 6;
      const int m = e >> 2, r = e & 3;
      return e < 4 * MT ? w1at(h0 + 16 * m + 4 * (l >> 4) + r, 16 * ft + (l & 15)) : 0.f;
    });
    f3.load(tid, [&](int idx) {   // A[hid][c], k-step (mo, s)
      const int e = idx % cS2T, ml = idx / cS2T, l = ml & 63, m = ml >> 6;
      const int mo = e >> 2, s4 = e & 3;
      const int c = 16 * mo + 4 * (l >> 4) + s4, hid = h0 + 16 * m + (l & 15);
      return (e < 4 * MO && c < C && hid < Hd) ? a.w2[(size_t)c * Hd + hid] : 0.f;
    });
    f4_.load(tid, [&](int idx) {
      const int co = idx / cSWM, ci = idx - co * cSWM;
      return (msg && co < C && ci < C) ? a.wm[co * C + ci] : 0.f;
    });
    f5.load(tid, [&](int idx) { return h0 + idx < Hd ? a.b1[h0 + idx] : 0.f; });
    f6.load(tid, [&](int idx) { return (msg && idx < C) ? a.bm[idx] : 0.f; });
    f7.load(tid, [&](int idx) {
      const int c = idx / 36, e = idx % 36, f = e / 12, tap = e % 12;
      return (c < C && tap < 9) ? a.perc[(3 * c + f) * 9 + tap] : 0.f;
    });
    if constexpr (LL && GNCA_BB_W1SKEW) {
      // row (m, l) starts 12 m + 4 (l >> 4) floats late: dY's single-float reads of the image (LL below) then
      // hit 64 distinct banks, GEMM1's 16-byte reads stay conflict-free (the skew is constant over
      // each 16-lane quarter)
      // (row block m: 64 KSP + 12 floats)
      f1.store_map(w1f, tid, [&](int idx) { return idx + 12 * ((idx / cKSP) >> 6) + 4 * (((idx / cKSP) & 63) >> 4); });
    } else {
      f1.store(w1f, tid);
    }
    if constexpr (!LL) f2.store(w1t, tid);
    f3.store(w2t, tid);
    f4_.store(wms, tid);
    f5.store(b1s, tid);
    f6.store(bms, tid);
    f7.store(percs, tid);
    static_assert(cKSP > 0 && cS1T > 0 && cS2T > 0 && cSWM > 0, "");
  }
  __syncthreads();
  bool sobel;
  {
    int ok = 1;
    for (int idx = tid; idx < C * 27; idx += kThreads) {
      const int c = idx / 27, e = idx % 27, f = e / 9, tap = e % 9;
      const int tr = tap / 3, tc = tap % 3;
      float ref;
      if (f == 0) ref = (tap == 4) ? 1.f : 0.f;
      else if (f == 1) ref = (float)((tc == 0 ? 1 : (tc == 2 ? -1 : 0)) * (tr == 1 ? 2 : 1));
      else ref = (float)((tr == 0 ? 1 : (tr == 2 ? -1 : 0)) * (tc == 1 ? 2 : 1));
      if (percs[c * 36 + f * 12 + tap] != ref) ok = 0;
    }
    sobel = __syncthreads_and(ok) != 0;
  }
  float gainr[MO];
#pragma unroll
  for (int mo = 0; mo < MO; ++mo)
    gainr[mo] = (msg && !(hidden_only && mo == 0 && g == 0)) ? a.message_gain : 0.f;
  BPROF_MARK(0);   // weights -> LDS

  // per-wave accumulators of the whole launch (AGPR-resident)
  f4 aw1[MT][FT], aw2[MO][MT], awm[MO][MO], abm[MO];
  float ab1[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    ab1[m] = 0.f;
#pragma unroll
    for (int f = 0; f < FT; ++f) aw1[m][f] = f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int mo = 0; mo < MO; ++mo) {
    abm[mo] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < MT; ++m) aw2[mo][m] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mi = 0; mi < MO; ++mi) awm[mo][mi] = f4{0.f, 0.f, 0.f, 0.f};
  }

  const int ncell = TH * TW, ngroups = (ncell + 15) >> 4;
  const size_t HW = (size_t)H * W;
  const int HWi = H * W;
  // per-lane dY plane offsets of this lane's MFMA output rows (slot = 16ft+4g+r -> f*C+c), or -1
  int plo[FT][4];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int slot = 16 * ft + 4 * g + r, f = slot / CP, c = slot - f * CP;
      plo[ft][r] = (slot < 3 * CP && c < C) ? (f * C + c) * HWi : -1;
    }
  const bool cfull = C == CP;   // no padded channels: every output row is live
  // XCD-aware tile order (speed only), as K1: workgroups b and b+8 share an XCD under round-robin
  // dispatch, so each XCD group sweeps a contiguous tile range and neighbouring tiles' halo
  // re-reads hit that XCD's L2
  const int nxcd = gridDim.x >= 8 ? 8 : 1;
  const int xg_ = blockIdx.x % nxcd, xr_ = blockIdx.x / nxcd;
  const int per_x = (int)(gridDim.x / nxcd) + ((int)(gridDim.x % nxcd) > xg_ ? 1 : 0);
  const int ntiles = a.alist ? a.alist[a.B] * a.tps : a.total_tiles;
  const int tq = ntiles / nxcd, trm = ntiles % nxcd;
  const int t_begin = xg_ * tq + min(xg_, trm), t_end = t_begin + tq + (xg_ < trm ? 1 : 0);
  for (int vt = t_begin + xr_; vt < t_end; vt += per_x) {
    const int tile = a.alist ? a.alist[vt / a.tps] * a.tps + vt % a.tps : vt;
    const int b = tile / a.tps, tin = tile - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const float* xb = a.x + (size_t)b * C * HW;
    const float* Ub = a.U + (size_t)b * C * HW;
    const float* Db = a.dx + (size_t)b * C * HW;
    float* dYb = a.dY + (size_t)b * 3 * C * HW;
    float* dGb = a.dG + (size_t)b * C * HW;
    __syncthreads();
    BPROF_MARK(7);   // loop tail
    if (a.active && !a.active[b]) {   // masked step, inactive sample: every cell is dead
      if (first && a.keep)
        for (int n = tid; n < ncell; n += kThreads) {
          const int ti = n / TW, tj = n - (n / TW) * TW;
          if (i0 + ti < H && j0 + tj < W) a.keep[(size_t)b * HW + (i0 + ti) * W + (j0 + tj)] = 0;
        }
      else if (first && !(a.flags & kZeroed))
        for (int n = tid; n < ncell; n += kThreads) {
          const int ti = n / TW, tj = n - (n / TW) * TW;
          if (i0 + ti >= H || j0 + tj >= W) continue;
          const int ce = (i0 + ti) * W + (j0 + tj);
          for (int pl = 0; pl < 3 * C; ++pl) dYb[pl * HWi + ce] = 0.f;
          if (msg)
            for (int c = 0; c < C; ++c) dGb[c * HWi + ce] = 0.f;
          if (a.dmb) a.dmb[(size_t)b * HW + ce] = 0.f;
        }
      continue;
    }
    // ---- staging by LDS-DMA (as the forward K1): every channel plane of the (RH x RW) region
    //      and the alpha plane with one more ring, all loads in flight at once, no VGPR round
    //      trip; torus-wrapped, or a zero source outside the image in pad mode.  16-byte pieces
    //      (kDma4: the region's quads never straddle a row end or the image edge) take a quarter
    //      of the instructions of 4-byte ones, whose issue was a fifth of BB at B=1024 ----
    if (a.flags & kDma4) {
      const int QW = RW >> 2, NQ = RH * QW, NI4 = (NQ + 63) >> 6;
      for (int ii_ = wave; ii_ < NI4; ii_ += NW) {
        const int q = 64 * ii_ + lane;
        if (q < NQ) {
          const int vr = q / QW, vc = 4 * (q - (q / QW) * QW);
          int ii = i0 - RY + vr, jj = j0 - RX + vc, off = 0;
          bool ok = true;
          if (zp) {
            ok = ii >= 0 && ii < H && jj >= 0 && jj < W;
            off = ok ? ii * W + jj : 0;
          } else {
            while (ii < 0) ii += H; while (ii >= H) ii -= H;
            while (jj < 0) jj += W; while (jj >= W) jj -= W;
            off = ii * W + jj;
          }
          float* dst = xs + 256 * ii_;
          for (int c = 0; c < CP; ++c) {
            const float* src = xb + (size_t)min(c, C - 1) * HW + off;
            if ((zp && !ok) || c >= C) src = g_bzero;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(dst + c * PSTR), 16, 0, 0);
          }
        }
      }
    } else
    for (int ii_ = wave; ii_ < L.NI; ii_ += NW) {
      const int e = 64 * ii_ + lane;
      int off = 0;
      bool ok = true;
      if (e < RH * RW) {
        const int vr = e / RW, vc = e - (e / RW) * RW;
        int ii = i0 - RY + vr, jj = j0 - RX + vc;
        if (zp) {
          ok = ii >= 0 && ii < H && jj >= 0 && jj < W;
          off = ok ? ii * W + jj : 0;
        } else {
          while (ii < 0) ii += H; while (ii >= H) ii -= H;
          while (jj < 0) jj += W; while (jj >= W) jj -= W;
          off = ii * W + jj;
        }
      }
      float* dst = xs + 64 * ii_;
      for (int c = 0; c < CP; ++c) {
        const float* src = xb + (size_t)min(c, C - 1) * HW + off;
        if ((zp && !ok) || c >= C) src = g_bzero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(dst + c * PSTR), 4, 0, 0);
      }
    }
    for (int ii_ = wave; ii_ < L.NIA; ii_ += NW) {
      const int e = 64 * ii_ + lane;
      int off = 0;
      bool ok = true;
      if (e < (RH + 2) * ALW) {
        const int vr = e / ALW, vc = e - (e / ALW) * ALW;
        int ii = i0 - RY - 1 + vr, jj = j0 - RX - 1 + vc;
        if (zp) {
          ok = ii >= 0 && ii < H && jj >= 0 && jj < W;
          off = ok ? ii * W + jj : 0;
        } else {
          while (ii < 0) ii += H; while (ii >= H) ii -= H;
          while (jj < 0) jj += W; while (jj >= W) jj -= W;
          off = ii * W + jj;
        }
      }
      const float* src = (zp && !ok) ? g_bzero : xb + 3 * HW + off;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(al + 64 * ii_), 4, 0, 0);
    }
    if (msg && !uniform_w)
      for (int o = tid; o < k; o += kThreads) wts[o] = a.offw[(size_t)b * k + o];
    BPROF_MARK(1);   // DMA issue
    for (int ti = wave; ti < TH; ti += NW) {
      if (lane < TW) {
        const int i = min(i0 + ti, H - 1), j = min(j0 + lane, W - 1);
        fp[ti * TW + lane] = fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step,
                                     a.sample_base, b, HW, (size_t)i * W + j) ? 1.f : 0.f;
      }
    }
    BPROF_MARK(6);   // fire plane
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    BPROF_MARK(2);   // DMA wait
    // ---- sender plane over the region, keep = pre-alive AND fire on the tile (as K1) ----
    {
      int jq = j0 - RX + lane;
      bool inc = true;
      if (zp) inc = jq >= 0 && jq < W;
      else { while (jq < 0) jq += W; while (jq >= W) jq -= W; }
      const bool lf = jq > 0, rt = jq < W - 1;
      for (int vr = wave; vr < RH; vr += NW) {
        if (lane >= RW) continue;
        const int vc = lane;
        int iq = i0 - RY + vr;
        bool in_img = inc;
        if (zp) in_img = in_img && iq >= 0 && iq < H;
        else { while (iq < 0) iq += H; while (iq >= H) iq -= H; }
        const float* q = al + (vr + 1) * ALW + (vc + 1);
        const float NEG = -INFINITY;
        const bool up = iq > 0, dn = iq < H - 1;
        const float mu_ = fmaxf(fmaxf(lf ? q[-ALW - 1] : NEG, q[-ALW]), rt ? q[-ALW + 1] : NEG);
        const float mm_ = fmaxf(fmaxf(lf ? q[-1] : NEG, q[0]), rt ? q[1] : NEG);
        const float md_ = fmaxf(fmaxf(lf ? q[ALW - 1] : NEG, q[ALW]), rt ? q[ALW + 1] : NEG);
        const float mx = fmaxf(fmaxf(up ? mu_ : NEG, mm_), dn ? md_ : NEG);
        const int pos = vr * RW + vc;
        sp[pos] = a2a ? ((in_img && mx > gthr) ? 1.f : 0.f) : (in_img ? 1.f : 0.f);
        const int ti = vr - RY, tj = vc - RX;
        if (ti >= 0 && ti < TH && tj >= 0 && tj < TW) {
          const int n = ti * TW + tj;
          fp[n] = (in_img && mx > thr) ? fp[n] : 0.f;
        }
      }
    }
    __syncthreads();
    const float mu = a.coef[4 * b], rs = a.coef[4 * b + 1];
    const float mu_u = a.coef[4 * b + 2], mu_ux = a.coef[4 * b + 3];
    // ---- live-cell compaction (as the forward K1): a cell with keep == 0 has d_pre = 0, so its
    //      dY / dG are zero and it adds nothing to any weight gradient; only live cells are
    //      packed into MFMA groups; the first slice stores every cell's keep byte (BC and BC2 read
    //      a dead cell's dY / dG / dmb as zeros from it: 1 byte instead of 4 (3C + C + 1) bytes of
    //      zeros per dead cell) ----
    int* lst = reinterpret_cast<int*>(smem + L.lst);
    int* wcnt = lst + r4(TH * TW);
    int nlive = 0;
    for (int n0 = 0; n0 < ncell; n0 += kThreads) {
      const int n = n0 + tid;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const bool inb = n < ncell && i0 + ti < H && j0 + tj < W;
      const bool live = inb && fp[n] != 0.f;
      const uint64_t bal = __ballot(live);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wcnt[wave] = __popcll(bal);
      __syncthreads();
      int off = nlive, tot = 0;
      for (int w_ = 0; w_ < NW; ++w_) {
        off += w_ < wave ? wcnt[w_] : 0;
        tot += wcnt[w_];
      }
      if (inb && first && a.keep) a.keep[(size_t)b * HW + (i0 + ti) * W + (j0 + tj)] = live ? 1 : 0;
      if (live) {
        lst[off + pre] = n;
      } else if (inb && first && !a.keep && !(a.flags & kZeroed)) {
        const int ce = (i0 + ti) * W + (j0 + tj);
        for (int pl = 0; pl < 3 * C; ++pl) dYb[pl * HWi + ce] = 0.f;
        if (msg)
          for (int c = 0; c < C; ++c) dGb[c * HWi + ce] = 0.f;
        if (a.dmb) a.dmb[(size_t)b * HW + ce] = 0.f;
      }
      nlive += tot;
      __syncthreads();
    }
    BPROF_MARK(3);   // planes + compaction + dead-cell zero stores

    // a group's U / dx loads (the GroupNorm-backward inputs of its cells)
    auto load_ud = [&](int qq, float (&u_)[MO][4], float (&d_)[MO][4]) {
      const int idx_ = 16 * qq + c16;
      const bool valid_ = idx_ < nlive;
      const int n_ = lst[valid_ ? idx_ : 0];
      const int ti_ = n_ / TW, tj_ = n_ - (n_ / TW) * TW;
      const int celli_ = (i0 + ti_) * W + (j0 + tj_);
      const float keep_ = valid_ ? fp[n_] : 0.f;
#pragma unroll
      for (int mo = 0; mo < MO; ++mo)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * mo + 4 * g + r;
          u_[mo][r] = 0.f;
          d_[mo][r] = 0.f;
          if (keep_ != 0.f && c < C) {
#ifndef GNCA_BB_ABL_LOAD
#define GNCA_BB_ABL_LOAD 0   // timing-only builds: 1 = U / dx not loaded (wrong results)
#endif
            if (GNCA_BB_ABL_LOAD) {
              u_[mo][r] = 0.5f + 1e-3f * (float)celli_;
              d_[mo][r] = 0.25f + 1e-3f * (float)c;
            } else {
              u_[mo][r] = Ub[c * HWi + celli_];
              if (gn) d_[mo][r] = Db[c * HWi + celli_];
            }
          }
        }
    };
    // (issuing the next group's loads once this group's were consumed, into 8 more registers, measured
    //  1 % slower at B=1024: profiles/r06h_bb_pf_skew_ab.txt)
    const int ngr = (nlive + 15) >> 4;
#pragma unroll 1
    for (int q = wave; q < ngr; q += NW) {
      const int idx = 16 * q + c16;
      const bool valid = idx < nlive;
      const int n = lst[valid ? idx : 0];
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const int pidx = (RY + ti) * RW + (RX + tj);
      const int celli = (i0 + ti) * W + (j0 + tj);
      const float* xg = xs + g * PSTR;
      // issue this group's U / dx loads first: their latency hides under the recompute below
      const float keep = valid ? fp[n] : 0.f;   // invalid (padding) lanes contribute nothing
      float ul[MO][4], dl[MO][4];
      load_ud(q, ul, dl);

      // -- gather (recompute) --
      float gv[CPQ];
#pragma unroll
      for (int t = 0; t < CPQ; ++t) gv[t] = 0.f;
      float S = 0.f;
      if (msg) {
        for (int o = 0; o < k; ++o) {
          const int qb = pidx - a.odl[o];
          const float wsp = (uniform_w ? a.uniform_w : wts[o]) * sp[qb];
          S += wsp;
#pragma unroll
          for (int t = 0; t < CPQ; ++t) gv[t] = fmaf(wsp, xg[qb + 4 * t * PSTR], gv[t]);
        }
      }
      // -- perception (recompute) --
      float y[KS];
      {
        const int ic = i0 + ti, jc = j0 + tj;
        const bool up = ic > 0, dn = ic < H - 1, lf = jc > 0, rt = jc < W - 1;
#pragma unroll
        for (int t = 0; t < CPQ; ++t) {
          const float* xc = xg + 4 * t * PSTR + pidx;
          float n0 = xc[-RW - 1], n1 = xc[-RW], n2 = xc[-RW + 1];
          float n3 = xc[-1], n4 = xc[0], n5 = xc[1];
          float n6 = xc[RW - 1], n7 = xc[RW], n8 = xc[RW + 1];
          n0 = (up && lf) ? n0 : 0.f; n1 = up ? n1 : 0.f; n2 = (up && rt) ? n2 : 0.f;
          n3 = lf ? n3 : 0.f;                               n5 = rt ? n5 : 0.f;
          n6 = (dn && lf) ? n6 : 0.f; n7 = dn ? n7 : 0.f; n8 = (dn && rt) ? n8 : 0.f;
          if (sobel) {
            y[t] = n4;
            y[CPQ + t] = (fmaf(2.f, n3, n0) + n6) - (fmaf(2.f, n5, n2) + n8);
            y[2 * CPQ + t] = (fmaf(2.f, n1, n0) + n2) - (fmaf(2.f, n7, n6) + n8);
          } else {
            const int c = 4 * t + g;
            const f4* pw = reinterpret_cast<const f4*>(percs + c * 36);
#pragma unroll
            for (int f = 0; f < 3; ++f) {
              const f4 w0 = pw[3 * f], w1 = pw[3 * f + 1], w2 = pw[3 * f + 2];
              float acc = w0[0] * n0;
              acc = fmaf(w0[1], n1, acc); acc = fmaf(w0[2], n2, acc); acc = fmaf(w0[3], n3, acc);
              acc = fmaf(w1[0], n4, acc); acc = fmaf(w1[1], n5, acc); acc = fmaf(w1[2], n6, acc);
              acc = fmaf(w1[3], n7, acc); acc = fmaf(w2[0], n8, acc);
              y[f * CPQ + t] = acc;
            }
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // -- GEMM1 (recompute): hpre[hid = 16m+4g+r][cell] --
      f4 hp[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) hp[m] = *reinterpret_cast<const f4*>(b1s + 16 * m + 4 * g);
#pragma unroll
      for (int s0 = 0; s0 < KS; s0 += 4) {
        f4 w4[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
          w4[m] = *reinterpret_cast<const f4*>(w1f + (m * 64 + lane) * KSP + s0 + (W1SK ? 12 * m + 4 * (lane >> 4) : 0));
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int m = 0; m < MT; ++m)
            if (s0 + u < KS) hp[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[m][u], y[s0 + u], hp[m], 0, 0, 0);
      }
      // -- message (recompute): m[c = 16mo+4g+r][cell] = W_M G + b_M S --
      f4 mm[MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) mm[mo] = f4{0.f, 0.f, 0.f, 0.f};
      if (msg_bwd) {
#pragma unroll
        for (int s = 0; s < CPQ; ++s)
#pragma unroll
          for (int mo = 0; mo < MO; ++mo)
            mm[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(wms[(16 * mo + c16) * SWM + 4 * s + g], gv[s], mm[mo], 0, 0, 0);
#pragma unroll
        for (int mo = 0; mo < MO; ++mo)
#pragma unroll
          for (int r = 0; r < 4; ++r) mm[mo][r] = fmaf(bms[16 * mo + 4 * g + r], S, mm[mo][r]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // -- d_pre = keep * GroupNorm-backward(U) (ncagraph.py:144-153) --
      f4 dp[MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float u = ul[mo][r];
          const bool live = keep != 0.f && 16 * mo + 4 * g + r < C;
          dp[mo][r] = live ? (gn ? rs * (u - mu_u - (dl[mo][r] - mu) * rs * mu_ux) : u) : 0.f;
        }
      // -- dh = relu'(hpre) * W2^T d_pre --
      f4 dh[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        dh[m] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mo = 0; mo < MO; ++mo) {
          const f4 wv = *reinterpret_cast<const f4*>(w2t + (m * 64 + lane) * S2T + 4 * mo);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            dh[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[s4], dp[mo][s4], dh[m], 0, 0, 0);
        }
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dh[m][r] = hp[m][r] > 0.f ? dh[m][r] : 0.f;
          hp[m][r] = __builtin_elementwise_maximum(hp[m][r], 0.f);   // relu (NaN stays NaN)
        }
      __builtin_amdgcn_sched_barrier(0);
      // -- dY = W1^T dh -> HBM (slot = f*CP + c -> plane f*C + c); FT independent chains --
      {
        f4 ay[FT];
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) ay[ft] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          f4 wv[FT];
          if constexpr (LL) {
            // A[slot = 16ft + c16][hid = 16m + 4g + r] from the W1 image: W1[16m + (l & 15)][4s + (l >> 4)]
            // sits at w1f[(64m + l) KSP + s], here l = 4g + r + 16 (c16 & 3), s = 4ft + (c16 >> 2)
            const float* wl = w1f + (4 * g + 16 * (c16 & 3)) * KSP + (c16 >> 2) + m * 64 * KSP +
                              (W1SK ? 12 * m + 4 * (c16 & 3) : 0);
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
#pragma unroll
              for (int r = 0; r < 4; ++r) wv[ft][r] = wl[r * KSP + 4 * ft];
          } else {
#pragma unroll
            for (int ft = 0; ft < FT; ++ft) wv[ft] = *reinterpret_cast<const f4*>(w1t + (ft * 64 + lane) * S1T + 4 * m);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
              ay[ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[ft][r], dh[m][r], ay[ft], 0, 0, 0);
        }
#ifndef GNCA_BB_ABL_STORE
#define GNCA_BB_ABL_STORE 0   // timing-only builds: 1 = no dY / dG stores (wrong results)
#endif
// (nontemporal dY / dG stores measured slower: B=1024 backward 3.22 -> 3.46 ms, profiles/r06h_bb_ablations.txt)
        if (valid && !GNCA_BB_ABL_STORE) {
          float* q = dYb + celli;
          if (first && cfull && 16 * FT == 3 * CP) {
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
#pragma unroll
              for (int r = 0; r < 4; ++r) q[plo[ft][r]] = ay[ft][r];
          } else if (first) {
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (plo[ft][r] >= 0) q[plo[ft][r]] = ay[ft][r];
          } else {
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (plo[ft][r] >= 0) q[plo[ft][r]] += ay[ft][r];
          }
        }
      }
      // -- message backward: dm = d_pre*gain*tanh'(m), dG = W_M^T dm -> HBM --
      f4 dm[MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) dm[mo] = f4{0.f, 0.f, 0.f, 0.f};
      if (msg_bwd) {
        float dmb = 0.f;
#pragma unroll
        for (int mo = 0; mo < MO; ++mo)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t = tanhf(mm[mo][r]);
            dm[mo][r] = dp[mo][r] * gainr[mo] * (1.f - t * t);
            abm[mo][r] = fmaf(dm[mo][r], S, abm[mo][r]);
            dmb = fmaf(dm[mo][r], bms[16 * mo + 4 * g + r], dmb);
          }
#pragma unroll
        for (int mi = 0; mi < MO; ++mi) {
          f4 ag = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int mo = 0; mo < MO; ++mo)
#pragma unroll
            for (int s = 0; s < 4; ++s)
              ag = __builtin_amdgcn_mfma_f32_16x16x4f32(wms[(16 * mo + 4 * g + s) * SWM + 16 * mi + c16],
                                                        dm[mo][s], ag, 0, 0, 0);
          if (valid && !GNCA_BB_ABL_STORE) {
            float* q = dGb + (16 * mi + 4 * g) * HWi + celli;
            if (cfull && (CP & 15) == 0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) q[r * HWi] = ag[r];
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (16 * mi + 4 * g + r < C) q[r * HWi] = ag[r];
            }
          }
        }
        if (a.dmb) {
          dmb += __shfl_xor(dmb, 16);
          dmb += __shfl_xor(dmb, 32);
          if (valid && g == 0) a.dmb[(size_t)b * HW + celli] = dmb;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // -- weight gradients, the cell dimension as the MFMA K (per-wave LDS transposes) --
      // (LL: T1 holds half the slice's hidden units at a time; every accumulator sums its k-steps in
      //  the same order either way)
      constexpr int NHH = LL ? 2 : 1, MH = MT / NHH;
#pragma unroll
      for (int s = 0; s < KS; ++s) T2[c16 * ST2 + 4 * s + g] = y[s];
#pragma unroll
      for (int hh = 0; hh < NHH; ++hh) {
#pragma unroll
        for (int m = 0; m < MH; ++m) *reinterpret_cast<f4*>(T1 + c16 * ST1 + 16 * m + 4 * g) = dh[MH * hh + m];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int row = 4 * s4 + g;
          float bv[FT];
#pragma unroll
          for (int ft = 0; ft < FT; ++ft) bv[ft] = T2[row * ST2 + 16 * ft + c16];
#pragma unroll
          for (int m = 0; m < MH; ++m) {
            const float av = T1[row * ST1 + 16 * m + c16];
            ab1[MH * hh + m] += av;
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
              aw1[MH * hh + m][ft] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[ft], aw1[MH * hh + m][ft], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) *reinterpret_cast<f4*>(T3 + c16 * ST3 + 16 * mo + 4 * g) = dp[mo];
#pragma unroll
      for (int hh = 0; hh < NHH; ++hh) {
#pragma unroll
        for (int m = 0; m < MH; ++m) *reinterpret_cast<f4*>(T1 + c16 * ST1 + 16 * m + 4 * g) = hp[MH * hh + m];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int row = 4 * s4 + g;
#pragma unroll
          for (int mo = 0; mo < MO; ++mo) {
            const float av = T3[row * ST3 + 16 * mo + c16];
#pragma unroll
            for (int m = 0; m < MH; ++m)
              aw2[mo][MH * hh + m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, T1[row * ST1 + 16 * m + c16],
                                                                         aw2[mo][MH * hh + m], 0, 0, 0);
          }
        }
      }
      if (msg_bwd) {
#pragma unroll
        for (int mo = 0; mo < MO; ++mo) *reinterpret_cast<f4*>(T3 + c16 * ST3 + 16 * mo + 4 * g) = dm[mo];
#pragma unroll
        for (int t = 0; t < CPQ; ++t) T4[c16 * ST3 + 4 * t + g] = gv[t];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int row = 4 * s4 + g;
#pragma unroll
          for (int mo = 0; mo < MO; ++mo) {
            const float av = T3[row * ST3 + 16 * mo + c16];
#pragma unroll
            for (int mi = 0; mi < MO; ++mi)
              awm[mo][mi] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, T4[row * ST3 + 16 * mi + c16], awm[mo][mi], 0, 0, 0);
          }
        }
      }
    }
    BPROF_MARK(4);   // group loop
  }

  // ---- this wave's partial gradients -> its own row (reduced later in a fixed order).  (An LDS
  //      combine of the 4 waves into one row per workgroup measured slower: 131 vs 106 us per
  //      B=16 40x40 backward.) ----
  float* outp = a.part + ((size_t)blockIdx.x * NW + wave) * a.npart;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hid = h0 + 16 * m + 4 * g + r, slot = 16 * ft + c16;
        const int f = slot / CP, c = slot - f * CP;
        if (hid < Hd && slot < 3 * CP && c < C) outp[a.o_w1 + (size_t)hid * 3 * C + f * C + c] = aw1[m][ft][r];
      }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float v = ab1[m];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    const int hid = h0 + 16 * m + c16;
    if (g == 0 && hid < Hd) outp[a.o_b1 + hid] = v;
  }
#pragma unroll
  for (int mo = 0; mo < MO; ++mo)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * mo + 4 * g + r, hid = h0 + 16 * m + c16;
        if (c < C && hid < Hd) outp[a.o_w2 + (size_t)c * Hd + hid] = aw2[mo][m][r];
      }
  if (first) {
#pragma unroll
    for (int mo = 0; mo < MO; ++mo) {
#pragma unroll
      for (int mi = 0; mi < MO; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 16 * mo + 4 * g + r, ci = 16 * mi + c16;
          if (co < C && ci < C) outp[a.o_wm + co * C + ci] = awm[mo][mi][r];
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = abm[mo][r];
        for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off);
        const int co = 16 * mo + 4 * g + r;
        if (c16 == 0 && co < C) outp[a.o_bm + co] = v;
      }
    }
  }
  BPROF_MARK(5);   // partial rows -> HBM
  BPROF_STORE;
}

// The active samples of a masked step in increasing order, their count at alist[B] (one workgroup;
// ballot prefix sums, so the list does not depend on thread timing)
__global__ __launch_bounds__(kThreads) void gnca_b_actlist(const uint8_t* active, int B, int* alist) {
  __shared__ int wsum[NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int base = 0;
  for (int b0 = 0; b0 < B; b0 += kThreads) {
    const int b = b0 + tid;
    const bool on = b < B && active[b] != 0;
    const uint64_t bal = __ballot(on);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = base, tot = 0;
    for (int u = 0; u < NW; ++u) {
      off += u < w ? wsum[u] : 0;
      tot += wsum[u];
    }
    if (on) alist[off + __popcll(bal & ((1ull << lane) - 1ull))] = b;
    base += tot;
    __syncthreads();
  }
  if (tid == 0) alist[B] = base;
}

// ------------------------------------------------------------------------------------------
// BC: adjoint of the perception (zero-padded 3x3 correlation) and of the gather
// ------------------------------------------------------------------------------------------
struct BCArgs {
  const float* dY;
  const float* dG;
  const float* x;
  const float* perc;
  const float* offw;
  const uint8_t* active;
  const uint8_t* keep;   // [B, H, W] BB's keep bytes (a dead cell's dY / dG are zeros, not stored), or null
  float* gx;
  int B, C, H, W, k, TH, TW, tiles_x, tps, RY, RX;
  int cpw, ncg;   // channels per workgroup, channel groups (small problems: more workgroups)
  float graph_alpha_thr, uniform_w;
  uint32_t flags;
  int8_t offs[2 * GNCA_MAX_OFFSETS];
};

constexpr int kBCStage = 16;   // max staged elements per thread per channel

__host__ __device__ inline int bc_stage(int TH, int TW, int RY, int RX, bool msg) {
  return 3 * (TH + 2) * (TW + 2) + (msg ? (TH + 2 * RY) * (TW + 2 * RX) : 0);
}

#ifndef GNCA_BC_DMA
#define GNCA_BC_DMA 0   // 1 (A/B builds): the slots staged by 4-byte LDS-DMA (B=1024 bwd 4.19 vs 3.98-4.00 ms: slower)
#endif
#ifndef GNCA_BC_ABL
#define GNCA_BC_ABL 0   // timing-only builds: 1 = no staging loads, 2 = no stencil arithmetic (wrong results)
#endif
// One workgroup per (sample, tile); channels are pipelined through a double-buffered LDS
// stage (the next channel's dY planes and dG halo are loaded into registers while this channel
// is computed), one barrier per channel.
// KC > 0: the offset count at compile time (the planned graph steps: 8, and 16 for C5): the
// message adjoint's KC staged reads of a cell are issued together and its weights / source deltas
// sit in registers, instead of a runtime loop that waited for each read in turn (same products in
// the same order: the same bits).  KC = 0: any count.
template <int KC>
__global__ __launch_bounds__(kThreads) void gnca_b_adjoint(const BCArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  // XCD-aware order (speed only): workgroups are dispatched round-robin over the 8 XCDs, so
  // workgroup w runs on XCD w % 8; give each XCD a contiguous range of (sample, tile, channel
  // group) items, so neighbouring tiles' halo re-reads hit that XCD's L2 instead of HBM
  const int G = (int)gridDim.x, xq = G / 8, xr = G % 8;
  const int xcd = (int)blockIdx.x % 8, xj = (int)blockIdx.x / 8;
  const int wid = G >= 8 ? xcd * xq + min(xcd, xr) + xj : (int)blockIdx.x;
  const int cg = wid % a.ncg, bt = wid / a.ncg;
  const int b = bt / a.tps, tin = bt - b * a.tps;
  if (a.active && !a.active[b]) return;   // dY = dG = 0 for an inactive sample
  const int c_lo = cg * a.cpw, c_hi = min(a.C, c_lo + a.cpw);
  const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
  const int RY = a.RY, RX = a.RX, H = a.H, W = a.W, C = a.C, k = a.k;
  const int TH = a.TH, TW = a.TW, PW = TW + 2, PA = (TH + 2) * PW;
  const int i0 = ty * TH, j0 = tx * TW;
  const size_t HW = (size_t)H * W;
  const bool zp = (a.flags & GNCA_ZERO_PAD_SHIFT) != 0;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool msg = (a.flags & kMsg) != 0;
  const int GW = TW + 2 * RX;
  const int SE = bc_stage(TH, TW, RY, RX, msg);       // staged floats per channel
  float* buf0 = smem;
  float* buf1 = smem + SE;
  float* as_ = buf1 + SE;                              // [TH*TW] sender mask of the tile cells
  float* wts = as_ + TH * TW;                          // [k]
  float* pws = wts + (k > 0 ? k : 1);                  // [C*27] perception weights
  const float* xb = a.x + (size_t)b * C * HW;
  // per-thread staging plan: element e = tid + 256*i of [3 dY planes | dG halo]. Per slot:
  // the source offset from the channel's plane base (dY plane f adds f*C*HW; -1 = zero fill),
  // and bit i of gsel set when the slot reads dG. Both are hoisted out of the channel loop, so
  // a load costs one select of two wave-uniform bases plus one 64-bit add.
  const int CHW = C * (int)HW;
  // With BB's keep plane a dead source cell's slot is a zero too (its dY / dG were not stored):
  // slot i is loaded only when bit i of sld is set (the keep bytes of the slots' cells: 16 byte
  // loads once per workgroup, all in flight together).
  int soff[kBCStage];
  uint32_t gsel = 0, sld = 0;
  uint8_t kv[kBCStage];
  const uint8_t* kb = a.keep ? a.keep + (size_t)b * HW : nullptr;
#pragma unroll
  for (int i = 0; i < kBCStage; ++i) {
    const int e = tid + kThreads * i;
    soff[i] = -1;
    kv[i] = 1;
    if (e >= SE) continue;
    int cell = -1;
    if (e < 3 * PA) {
      const int f = e / PA, r = e - f * PA;
      const int ii = i0 - 1 + r / PW, jj = j0 - 1 + r % PW;
      if (ii >= 0 && ii < H && jj >= 0 && jj < W) {
        soff[i] = f * CHW + ii * W + jj;
        cell = ii * W + jj;
      }
    } else {
      const int r = e - 3 * PA;
      int ii = i0 - RY + r / GW, jj = j0 - RX + r % GW;
      bool ok = true;
      if (zp) ok = ii >= 0 && ii < H && jj >= 0 && jj < W;
      else { ii = wrapi(ii, H); jj = wrapi(jj, W); }
      gsel |= 1u << i;
      if (ok) {
        soff[i] = ii * W + jj;
        cell = ii * W + jj;
      }
    }
    if (kb && cell >= 0) kv[i] = kb[cell];
  }
#pragma unroll
  for (int i = 0; i < kBCStage; ++i) sld |= (soff[i] >= 0 && kv[i] != 0) ? 1u << i : 0u;
  float stg[kBCStage];
  auto load = [&](int c) {
    const float* pY = a.dY + ((size_t)b * 3 * C + c) * HW;
    const float* pG = a.dG + ((size_t)b * C + c) * HW;
#pragma unroll
    for (int i = 0; i < kBCStage; ++i) {
      const float* p = ((gsel >> i) & 1u) ? pG : pY;
      stg[i] = ((sld >> i) & 1u) && !(GNCA_BC_ABL & 1) ? p[soff[i]] : 0.f;
    }
  };
  auto store = [&](float* dst) {
#pragma unroll
    for (int i = 0; i < kBCStage; ++i)
      if (tid + kThreads * i < SE) dst[tid + kThreads * i] = stg[i];
  };
  // GNCA_BC_DMA: the same slots staged by LDS-DMA straight into the buffer (a zero source for the
  // slots that read zero): no VGPR round trip, the wait moves from the LDS stores to the channel's end
  const int wave = tid >> 6;
  auto dma = [&](int c, float* dst) {
    const float* pY = a.dY + ((size_t)b * 3 * C + c) * HW;
    const float* pG = a.dG + ((size_t)b * C + c) * HW;
#pragma unroll
    for (int i = 0; i < kBCStage; ++i) {
      if (kThreads * i >= SE) break;
      if (tid + kThreads * i < SE) {
        const float* p = ((gsel >> i) & 1u) ? pG : pY;
        const float* src = ((sld >> i) & 1u) ? p + soff[i] : g_bzero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(dst + kThreads * i + 64 * wave), 4, 0, 0);
      }
    }
  };
  // gx is read-modify-written; its next-channel values are prefetched with the staging loads
  // (th*tw <= 4*kThreads: at most 4 cells per thread). Per cell: offset in the channel plane
  // (-1 = none) and the tile-local index ti*TW + tj, hoisted out of the channel loop.
  int goff[4], gtij[4];   // gtij = ti << 16 | tj
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int n = tid + kThreads * u;
    const int ti = n / TW, tj = n - (n / TW) * TW;
    const int i = i0 + ti, j = j0 + tj;
    gtij[u] = (ti << 16) | tj;
    goff[u] = (n < TH * TW && i < H && j < W) ? i * W + j : -1;
  }
  float gxc[4], gxn[4];
  auto load_gx = [&](int c, float* dst) {
    const float* pg = a.gx + ((size_t)b * C + c) * HW;
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[u] = goff[u] >= 0 ? pg[goff[u]] : 0.f;
  };
  // the first channel's staging loads go out before the perception weights / sender mask, so
  // the prologue waits out one memory latency, not three
  if (GNCA_BC_DMA) dma(c_lo, buf0);
  else load(c_lo);
  load_gx(c_lo, gxc);
  lds_fill<kThreads, 2>(pws, C * 27, tid, [&](int e) { return a.perc[e]; });
  if (msg) {
    for (int o = tid; o < k; o += kThreads) wts[o] = a.offw ? a.offw[(size_t)b * k + o] : a.uniform_w;
    for (int n = tid; n < TH * TW; n += kThreads) {
      const int i = i0 + n / TW, j = j0 + n % TW;
      float v9[9];   // the 3x3 alpha neighbourhood, all nine loads in flight
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          const int ii = i + u - 1, jj = j + v - 1;
          v9[3 * u + v] = (i < H && j < W && ii >= 0 && ii < H && jj >= 0 && jj < W)
                              ? xb[3 * HW + (size_t)ii * W + jj] : -INFINITY;
        }
      float mx = v9[0];
#pragma unroll
      for (int t = 1; t < 9; ++t) mx = fmaxf(mx, v9[t]);
      as_[n] = a2a ? (mx > a.graph_alpha_thr ? 1.f : 0.f) : 1.f;
    }
  }
  if (GNCA_BC_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else store(buf0);
  // the reference's frozen identity / Sobel bank (the module's perception, always, in practice)?
  // Then the adjoint reads only the 13 taps with nonzero weights, with the weights as constants:
  // the same nonzero products in the same order as the generic loop (a zero-weight tap adds +0 to
  // a sum that is never -0), so bitwise the same gx for finite dY (with an Inf / NaN dY the generic
  // loop and the reference's autograd give NaN from 0 * Inf at a zero-weight tap; this path does not)
  int pok = 1;
  for (int e = tid; e < C * 27; e += kThreads) {
    const int f = (e % 27) / 9, tap = e % 9, tr = tap / 3, tc = tap % 3;
    const float ref = f == 0 ? (tap == 4 ? 1.f : 0.f)
                    : f == 1 ? (float)((tc == 0 ? 1 : (tc == 2 ? -1 : 0)) * (tr == 1 ? 2 : 1))
                             : (float)((tr == 0 ? 1 : (tr == 2 ? -1 : 0)) * (tc == 1 ? 2 : 1));
    if (pws[e] != ref) pok = 0;
  }
#ifdef GNCA_BC_GENERIC   // A/B builds: the generic 27-tap loop always
  const bool sobel = __syncthreads_and(pok) != 0 && false;
#else
  const bool sobel = __syncthreads_and(pok) != 0;
#endif
  // KC > 0: the message adjoint's per-offset weights and staged-source deltas, in registers
  float wk_[KC > 0 ? KC : 1];
  int dk_[KC > 0 ? KC : 1];
  if constexpr (KC > 0) {
#pragma unroll
    for (int o = 0; o < KC; ++o) {
      wk_[o] = msg ? wts[o] : 0.f;
      dk_[o] = a.offs[2 * o] * GW + (zp ? 0 : a.offs[2 * o + 1]);
    }
  }
  for (int c = c_lo; c < c_hi; ++c) {
    float* cur = ((c - c_lo) & 1) ? buf1 : buf0;
    float* nxt = ((c - c_lo) & 1) ? buf0 : buf1;
    if (c + 1 < c_hi) {
      if (GNCA_BC_DMA) dma(c + 1, nxt);
      else load(c + 1);
      load_gx(c + 1, gxn);
    }
    const float* pw = pws + c * 27;
    float* pgx = a.gx + ((size_t)b * C + c) * HW;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (goff[u] < 0) continue;
      const int n = tid + kThreads * u;
      const int ti = gtij[u] >> 16, tj = gtij[u] & 0xffff;
      // y(p) += w[u][v] x(p + (u-1, v-1))  =>  gx(q) += w[u][v] dY(q - (u-1, v-1))
      float acc = 0.f;
      if (GNCA_BC_ABL & 2) {
      } else if (sobel) {
        // tap (u, v) of plane f reads cur[f PA + (ti + 2 - u) PW + (tj + 2 - v)]
        const float* c0 = cur + (ti + 2) * PW + (tj + 2);
        auto Y = [&](int f, int u, int v) { return c0[f * PA - u * PW - v]; };
        acc = fmaf(1.f, Y(0, 1, 1), acc);
        acc = fmaf(1.f, Y(1, 0, 0), acc);
        acc = fmaf(-1.f, Y(1, 0, 2), acc);
        acc = fmaf(2.f, Y(1, 1, 0), acc);
        acc = fmaf(-2.f, Y(1, 1, 2), acc);
        acc = fmaf(1.f, Y(1, 2, 0), acc);
        acc = fmaf(-1.f, Y(1, 2, 2), acc);
        acc = fmaf(1.f, Y(2, 0, 0), acc);
        acc = fmaf(2.f, Y(2, 0, 1), acc);
        acc = fmaf(1.f, Y(2, 0, 2), acc);
        acc = fmaf(-1.f, Y(2, 2, 0), acc);
        acc = fmaf(-2.f, Y(2, 2, 1), acc);
        acc = fmaf(-1.f, Y(2, 2, 2), acc);
      } else {
#pragma unroll
        for (int f = 0; f < 3; ++f)
#pragma unroll
          for (int u = 0; u < 3; ++u)
#pragma unroll
            for (int v = 0; v < 3; ++v)
              acc = fmaf(pw[f * 9 + u * 3 + v], cur[f * PA + (ti + 2 - u) * PW + (tj + 2 - v)], acc);
      }
      if (msg && !(GNCA_BC_ABL & 2)) {
        // msg(p) = sum_o w_o A(p-o) M(p-o)  =>  gM(q) = A(q) sum_o w_o dm(q+o)  (roll / row shift)
        const float* g0 = cur + 3 * PA + (ti + RY) * GW + (tj + RX);
        float sg = 0.f;
        if constexpr (KC > 0) {
          float gv[KC];
#pragma unroll
          for (int o = 0; o < KC; ++o) gv[o] = g0[dk_[o]];
#pragma unroll
          for (int o = 0; o < KC; ++o) sg = fmaf(wk_[o], gv[o], sg);
        } else {
          for (int o = 0; o < k; ++o) {
            const int dy = a.offs[2 * o], dx = zp ? 0 : a.offs[2 * o + 1];
            sg = fmaf(wts[o], g0[dy * GW + dx], sg);
          }
        }
        acc = fmaf(as_[n], sg, acc);
      }
      pgx[goff[u]] = gxc[u] + acc;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) gxc[u] = gxn[u];
    if (GNCA_BC_DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (c + 1 < c_hi) store(nxt);
    __syncthreads();
  }
}

// BC2 (zero-pad only): per (sample, offset, row block) partial of
//   dL/dw_o = sum_q A(q) (<dG(q+o), x(q)> + <dm(q+o), b_M>)     (o = (dy, 0): the row shift)
struct BC2Args {
  const float* x;
  const float* dG;
  const float* dmb;
  const uint8_t* keep;   // BB's keep bytes (a dead cell's dG / dmb are zeros, not stored), or null
  double* dots;   // [B][k][nrb]
  int B, C, H, W, k, nrb, rows_per;
  float gthr;
  int a2a;
  int8_t offs[2 * GNCA_MAX_OFFSETS];
};

__global__ __launch_bounds__(kThreads) void gnca_b_dots(const BC2Args a) {
  __shared__ double red[2 * NW];
  const int tid = threadIdx.x;
  const int per_b = a.k * a.nrb;
  const int b = blockIdx.x / per_b, rem = blockIdx.x - b * per_b;
  const int o = rem / a.nrb, rb = rem - o * a.nrb;
  const int H = a.H, W = a.W, C = a.C;
  const size_t HW = (size_t)H * W;
  const int dy = a.offs[2 * o];
  const int r0 = rb * a.rows_per, r1 = min(H, r0 + a.rows_per);
  const float* xb = a.x + (size_t)b * C * HW;
  const float* gb = a.dG + (size_t)b * C * HW;
  double acc = 0.0;
  for (int e = tid; e < (r1 - r0) * W; e += kThreads) {
    const int i = r0 + e / W, j = e % W;
    const int it = i + dy;
    if (it < 0 || it >= H) continue;
    if (a.a2a) {
      float mx = -INFINITY;
      for (int u = max(0, i - 1); u <= min(H - 1, i + 1); ++u)
        for (int v = max(0, j - 1); v <= min(W - 1, j + 1); ++v) mx = fmaxf(mx, xb[3 * HW + (size_t)u * W + v]);
      if (!(mx > a.gthr)) continue;
    }
    const size_t q = (size_t)i * W + j, t = (size_t)it * W + j;
    // a dead target adds exactly +0 (s = 0 + sum x * 0) for finite x: skipped (an Inf / NaN x here
    // would give the reference's autograd NaN from Inf * 0; this shortcut assumes a finite state)
    if (a.keep && !a.keep[(size_t)b * HW + t]) continue;
    float s = a.dmb[(size_t)b * HW + t];
    for (int c = 0; c < C; ++c) s = fmaf(xb[c * HW + q], gb[c * HW + t], s);
    acc += (double)s;
  }
  const double2 r = block_sum2(acc, 0.0, red);
  if (tid == 0) a.dots[((size_t)b * a.k + o) * a.nrb + rb] = r.x;
}

// BD (zero-pad only): backward of the pooled-logit softmax (graph_augmentation.py:113-154), fp64.
//   logit_o = qbar . kbar_o,  qbar = W_Q xbar + b_Q,  kbar_o = (W_K S_o + b_K n_o W) / HW,
//   w = softmax(logit / (|scaling| + 1e-6)).
// Per-sample partial gradients of W_Q, b_Q, W_K, b_K, scaling, and the per-row gx correction
// (Q and K enter only through their spatial means, so their x-gradient is constant per row).
struct BDArgs {
  const float* x;
  const double* rs;   // the forward K0's row sums of x ([B][C][H], fp64), or null: computed here
  const float* wq;
  const float* bq;
  const float* wk;
  const float* bk;
  const float* scaling;
  const double* dots;   // [B][k][nrb]
  double* pq;           // [B][2*d*C + 2*d + 1]
  float* corr;          // [B][H][C]
  int B, C, H, W, d, k, nrb;
  int8_t offs[2 * GNCA_MAX_OFFSETS];
};

__global__ __launch_bounds__(kThreads) void gnca_b_attn(const BDArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = a.C, H = a.H, W = a.W, d = a.d, k = a.k;
  double* rs = reinterpret_cast<double*>(smem);   // [C][H]
  double* xbar = rs + (size_t)C * H;              // [C]
  double* qbar = xbar + C;                        // [d]
  double* So = qbar + d;                          // [k][C]
  double* kb = So + (size_t)k * C;                // [k][d]
  double* L = kb + (size_t)k * d;                 // [k]
  double* gL = L + k;                             // [k]
  double* gqp = gL + k;                           // [d]
  double* gkp = gqp + d;                          // [k][d]
  double* gks = gkp + (size_t)k * d;              // [H][d]: sum of gkp over offsets valid for row
  double* sc = gks + (size_t)H * d;               // [2]: g_scaling, HW
  float* wqs = reinterpret_cast<float*>(sc + 2);  // [d][C] W_Q, then W_K: LDS copies (the loops below read
  float* wks = wqs + (size_t)d * C;               // them per channel / per unit, a global round trip each)
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t HW = (size_t)H * W;
  const float* xb = a.x + (size_t)b * C * HW;
  for (int e = tid; e < d * C; e += kThreads) {
    wqs[e] = a.wq[e];
    wks[e] = a.wk[e];
  }
  if (a.rs)   // the forward's K0 row sums (the same x, the same bits)
    for (int e = tid; e < C * H; e += kThreads) rs[e] = a.rs[(size_t)b * C * H + e];
  else if ((W & 3) == 0)
    canon_row_sums<4, 2>(xb, C * H, W, rs, tid >> 5, kThreads / 32, tid & 31);
  else
    canon_row_sums<1, 2>(xb, C * H, W, rs, tid >> 5, kThreads / 32, tid & 31);
  __syncthreads();
  for (int c = tid; c < C; c += kThreads) {
    double s = 0.0;
    for (int r = 0; r < H; ++r) s += rs[c * H + r];
    xbar[c] = s / (double)HW;
  }
  for (int e = tid; e < k * C; e += kThreads) {
    const int o = e / C, c = e - o * C;
    const int dy = a.offs[2 * o];
    const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;
    double s = 0.0;
    for (int r = lo; r < hi; ++r) s += rs[c * H + r];
    So[e] = s;
  }
  __syncthreads();
  for (int e = tid; e < d; e += kThreads) {
    double s = (double)a.bq[e];
    for (int c = 0; c < C; ++c) s += (double)wqs[e * C + c] * xbar[c];
    qbar[e] = s;
  }
  for (int e = tid; e < k * d; e += kThreads) {
    const int o = e / d, j = e - o * d;
    const int dy = a.offs[2 * o];
    const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;
    const double n_o = (double)(hi > lo ? hi - lo : 0) * (double)W;
    double s = (double)a.bk[j] * n_o;
    for (int c = 0; c < C; ++c) s += (double)wks[j * C + c] * So[o * C + c];
    kb[e] = s / (double)HW;
  }
  __syncthreads();
  for (int o = tid; o < k; o += kThreads) {
    double s = 0.0;
    for (int j = 0; j < d; ++j) s += qbar[j] * kb[o * d + j];
    L[o] = s;
  }
  __syncthreads();
  if (tid == 0) {
    double mx = -INFINITY;
    for (int o = 0; o < k; ++o) mx = fmax(mx, L[o]);
    const double sv = (double)a.scaling[0];
    const double T = fabs(sv) + 1e-6;
    double sum = 0.0;
    for (int o = 0; o < k; ++o) sum += exp((L[o] - mx) / T);
    double G = 0.0;
    for (int o = 0; o < k; ++o) {
      double gw = 0.0;
      for (int r = 0; r < a.nrb; ++r) gw += a.dots[((size_t)b * k + o) * a.nrb + r];
      gL[o] = gw;                                   // dL/dw_o for now
      G += exp((L[o] - mx) / T) / sum * gw;
    }
    double gT = 0.0;
    for (int o = 0; o < k; ++o) {
      const double w = exp((L[o] - mx) / T) / sum;
      const double gz = w * (gL[o] - G);
      gL[o] = gz / T;
      gT -= gz * (L[o] - mx) / (T * T);
    }
    sc[0] = gT * (sv > 0.0 ? 1.0 : (sv < 0.0 ? -1.0 : 0.0));
  }
  __syncthreads();
  for (int j = tid; j < d; j += kThreads) {
    double s = 0.0;
    for (int o = 0; o < k; ++o) s += gL[o] * kb[o * d + j];
    gqp[j] = s;
  }
  for (int e = tid; e < k * d; e += kThreads) gkp[e] = gL[e / d] * qbar[e % d];
  __syncthreads();
  for (int e = tid; e < H * d; e += kThreads) {
    const int r = e / d, j = e - r * d;
    double s = 0.0;
    for (int o = 0; o < k; ++o) {
      const int dy = a.offs[2 * o];
      const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;
      if (r >= lo && r < hi) s += gkp[o * d + j];
    }
    gks[e] = s;
  }
  double* out = a.pq + (size_t)b * (2 * d * C + 2 * d + 1);
  for (int e = tid; e < d * C; e += kThreads) {
    const int j = e / C, c = e - j * C;
    out[e] = gqp[j] * xbar[c];                       // dW_Q
    double s = 0.0;
    for (int o = 0; o < k; ++o) s += gkp[o * d + j] * So[o * C + c];
    out[d * C + d + e] = s / (double)HW;             // dW_K
  }
  for (int j = tid; j < d; j += kThreads) {
    out[d * C + j] = gqp[j];                         // db_Q
    double s = 0.0;
    for (int o = 0; o < k; ++o) {
      const int dy = a.offs[2 * o];
      const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;
      s += gkp[o * d + j] * (double)(hi > lo ? hi - lo : 0) * (double)W;
    }
    out[2 * d * C + d + j] = s / (double)HW;         // db_K
  }
  if (tid == 0) out[2 * d * C + 2 * d] = sc[0];      // d scaling
  __syncthreads();
  for (int e = tid; e < H * C; e += kThreads) {
    const int r = e / C, c = e - r * C;
    double s = 0.0;
    for (int j = 0; j < d; ++j) s += (double)wqs[j * C + c] * gqp[j] + (double)wks[j * C + c] * gks[r * d + j];
    a.corr[((size_t)b * H + r) * C + c] = (float)(s / (double)HW);
  }
}

// BE: gx[b,c,i,j] += corr[b,i,c]
__global__ __launch_bounds__(kThreads) void gnca_b_rowcorr(float* gx, const float* corr, int B, int C,
                                                           int H, int W) {
  const size_t total = (size_t)B * C * H * W;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += (size_t)gridDim.x * kThreads) {
    const size_t j = e % W, t = e / W;
    const size_t i = t % H, t2 = t / H;
    const size_t c = t2 % C, b = t2 / C;
    (void)j;
    gx[e] += corr[(b * H + i) * C + c];
  }
}

// R: fixed-order sums of partial rows into the gradient outputs (deterministic).
// The output columns of up to 12 segments are numbered consecutively; segment s maps its local
// column j to part column col0[s] + j*step[s] and writes out[s][j] (skipped if out[s] is null);
// step[s] == 0 marks a segment of exact zeros (no reads).
// A 256-thread block owns 16 columns: 16 row groups sum rows r = g, g+16, ... with 4 independent
// accumulators each, then the 16 group sums are added in order.
struct RedArgs {
  const void* part;
  int f64;
  long rows, stride;
  int nseg, ncols;
  int end[12];      // exclusive end of segment s in the concatenated column space
  long col0[12];
  int step[12];
  float* out[12];
};

// 32 columns per workgroup: a half-wave reads 32 consecutive floats of a partial row (one whole
// 128-byte line; the 16-column form read 64-byte pieces of four rows per instruction), 336
// workgroups for the 10,753 columns of the C = 16 step.  Each thread keeps the 16-column form's
// arithmetic for two row groups rg = w + 8 v (rows rg + 16 i, four interleaved sums per group),
// then the first 32 threads add the 16 groups in order: the same bits as before.
__global__ __launch_bounds__(kThreads) void gnca_b_reduce(const RedArgs a) {
  __shared__ double acc[16][33];
  const int cj = threadIdx.x & 31, w = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cj;
  int s = 0;
  while (s < a.nseg - 1 && col >= a.end[s]) ++s;
  const int begin = s == 0 ? 0 : a.end[s - 1];
  const long src = a.col0[s] + (long)(col - begin) * a.step[s];
  const bool on = col < a.ncols && a.step[s] != 0;
  // U steps of 4 rows (rows r + 16 i, i < 4U): every load in flight before the adds, which keep the
  // one-step order (t0..t3 take rows r, r + 16, r + 32, r + 48 of each step), so the sums are the
  // same bits as one step at a time, in ceil(rows / 64U) memory latencies instead of rows / 64
  // (B=16 40^2: 960 rows, 15 dependent round trips per thread before)
#pragma unroll 1
  for (int v = 0; v < 2; ++v) {
    const int rg = w + 8 * v;
    double t0 = 0.0, t1 = 0.0, t2 = 0.0, t3 = 0.0;
    auto steps = [&](auto U_, const auto* p, long& r) {
      constexpr int U = decltype(U_)::value;
      for (; r + 64 * (U - 1) + 48 < a.rows; r += 64 * U) {
        double vv[4 * U];
#pragma unroll
        for (int i = 0; i < 4 * U; ++i) vv[i] = (double)p[(r + 16 * i) * a.stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          t0 += vv[4 * u]; t1 += vv[4 * u + 1]; t2 += vv[4 * u + 2]; t3 += vv[4 * u + 3];
        }
      }
    };
    if (on) {
      long r = rg;
      if (a.f64) {
        const double* p = reinterpret_cast<const double*>(a.part) + src;
        steps(std::integral_constant<int, 8>{}, p, r);
        steps(std::integral_constant<int, 2>{}, p, r);
        steps(std::integral_constant<int, 1>{}, p, r);
        for (; r < a.rows; r += 16) t0 += p[r * a.stride];
      } else {
        const float* p = reinterpret_cast<const float*>(a.part) + src;
        steps(std::integral_constant<int, 8>{}, p, r);
        steps(std::integral_constant<int, 2>{}, p, r);
        steps(std::integral_constant<int, 1>{}, p, r);
        for (; r < a.rows; r += 16) t0 += (double)p[r * a.stride];
      }
    }
    acc[rg][cj] = (t0 + t1) + (t2 + t3);
  }
  __syncthreads();
  if (w == 0 && col < a.ncols && a.out[s]) {
    double v = 0.0;
    for (int g = 0; g < 16; ++g) v += acc[g][cj];
    a.out[s][col - begin] = (float)v;
  }
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct BBVariant {
  int CP, HB;
  const void* fn;
  const void* fnf;   // the C == CP instance (16 and 32 channels), or null
};
#define GNCA_BV(cp, hb) {cp, hb, reinterpret_cast<const void*>(&gnca_b_mlp<cp, hb>), \
                         (cp == 16 || cp == 32) ? reinterpret_cast<const void*>(&gnca_b_mlp<cp, hb, true>) : nullptr}
static const BBVariant kBB[] = {
    GNCA_BV(16, 128), GNCA_BV(4, 32),  GNCA_BV(8, 32),  GNCA_BV(16, 32), GNCA_BV(4, 64),
    GNCA_BV(8, 64),   GNCA_BV(12, 64), GNCA_BV(16, 64), GNCA_BV(20, 64), GNCA_BV(24, 64),
    GNCA_BV(28, 64),  GNCA_BV(32, 64), GNCA_BV(12, 32), GNCA_BV(20, 32), GNCA_BV(24, 32),
    GNCA_BV(28, 32),  GNCA_BV(32, 32),
};
#undef GNCA_BV
// compile-time-geometry instances of the planned shapes (16 channels, hidden 128, x halo padded to 4):
// 72^2 canvases take 8x24 tiles (24x24 in the lean layout when the batch fills the chip), the
// trainer's 40^2 8x16; graph r <= 4 (the y halo padded to 4) with 8 offsets, or classic (y halo 1, no
// offsets)
struct BBSpec {
  int TH, TW, RY, RX, K;
  bool lean;
  const void* fn;
};
#define GNCA_BS(th, tw, ry, rx, k, ll) \
  {th, tw, ry, rx, k, ll, reinterpret_cast<const void*>(&gnca_b_mlp<16, 128, true, th, tw, ry, rx, k, ll>)}
static const BBSpec kBBS[] = {
    GNCA_BS(8, 24, 4, 4, 8, false), GNCA_BS(8, 16, 4, 4, 8, false), GNCA_BS(8, 24, 1, 4, 0, false),
    GNCA_BS(8, 16, 1, 4, 0, false), GNCA_BS(24, 24, 4, 4, 8, true), GNCA_BS(24, 24, 1, 4, 0, true),
};
#undef GNCA_BS

struct BwdPlan {
  FwdLayout F;
  const BBVariant* bb;
  const void* bbfn;    // the BB kernel: bb->fn
  const void* bbfn2;   // the kernel of slices after the first (bb->fn)
  bool bbf32;          // BB is gnca_b_mlp (keep bytes, 16-byte staging): always, since round 6
  bool bblean;         // BB runs a lean-layout compile-time instance (kBBS, large tiles)
  int CP, HB, nslices;
  bool graph, msg, zp, gn;
  int RY, RX;
  int RXB;   // BB's x halo (RX padded to a multiple of 4 when W is one: 16-byte staging)
  int TH, TW, tiles_x, tps, total_tiles, gridB;
  size_t ldsB;
  int band, nbands;        // BA
  size_t ldsA;
  int TH3, TW3, tiles_x3, tps3;   // BC
  size_t ldsC;
  int nrb, rows_per;       // BC2
  size_t ldsD;
  int npart, o_w1, o_b1, o_w2, o_wm, o_bm, nq;
  size_t off_fwd, off_U, off_dY, off_dG, off_dmb, off_keep, off_alist, off_pa, off_coef, off_pb, off_dots, off_pq, off_corr,
      bytes;
};

static int bwd_device_cus() {
  static std::mutex mu;
  static std::unordered_map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  cache[dev] = cus;
  return cus;
}

// lean_ok: the large lean-layout tiles may be planned.  Not for a masked step (an active-sample mask):
// its late steps have few active samples, whose work 3x larger tiles spread over fewer CUs (the B=128
// trainer iteration measured 111-113 -> 116-120 ms with them, profiles/r06g_bb_lean_ab.txt)
static bool bwd_plan(const gnca_step_desc* d, BwdPlan* P, bool lean_ok = true) {
  if (!d || !fwd_layout(d, &P->F)) return false;
  const int C = d->C, Hd = d->hidden, H = d->H, W = d->W;
  P->CP = (C + 3) & ~3;
  P->graph = (d->flags & GNCA_GRAPH) != 0;
  P->msg = P->graph && P->F.k > 0 && d->message_gain != 0.f;
  P->zp = (d->flags & GNCA_ZERO_PAD_SHIFT) != 0;
  P->gn = (d->flags & GNCA_USE_GROUPNORM) != 0;
  int ry = 1, rx = 1;
  if (P->msg)
    for (int o = 0; o < P->F.k; ++o) {
      ry = std::max(ry, std::abs((int)d->offsets[2 * o]));
      if (!P->zp) rx = std::max(rx, std::abs((int)d->offsets[2 * o + 1]));
    }
  P->RY = ry;
  P->RX = rx;
  // BB's staged x halo: padded to a multiple of 4 columns when the rows are (16-byte LDS-DMA pieces)
  const int rxb = (W % 4 == 0) ? ((rx + 3) & ~3) : rx;
  // a graph step of the compile-time BB shapes (kBBS: 16 channels, hidden 128, 8 offsets within
  // radius 4) stages a 4-row y halo whatever its drawn offsets reach (usually 4 anyway)
  if (P->msg && C == 16 && Hd == 128 && P->F.k == 8 && ry <= 4 && W % 4 == 0) ry = 4;
  P->RY = ry;
  // hidden slice (variant) and BB tile: fewest slices first (each slice recomputes the
  // perception, gather and message), then fewest padded hidden units, then the cheapest tile
  // (padded cells + staged halo) within 160 KB of LDS
  static const int ths[] = {4, 8, 16};
  static const int tws[] = {8, 16, 24, 32};
  static const char* tile_env = GNCA_AB_ENV("GNCA_BB_TILE");   // measurement knob (A/B runs only)
  int eth = 0, etw = 0;
  if (tile_env) sscanf(tile_env, "%dx%d", &eth, &etw);
  double best = 1e300;
  P->bb = nullptr;
  P->bblean = false;
  // the compile-time instance this step's shape would run on a (th, tw) tile, if any
  const bool spec_ok = C == 16 && P->CP == 16 && Hd == 128;
  auto spec_for = [&](int th, int tw) -> const BBSpec* {
    if (!spec_ok) return nullptr;
    for (const BBSpec& sp : kBBS)
      // (a graph step without the message, e.g. the trainers' message-off steps, is a classic step
      //  for BB whatever offsets were drawn: the K = 0 instance; round 6, before it took the
      //  runtime-geometry kernel)
      if (sp.TH == th && sp.TW == tw && sp.RY == ry && sp.RX == rxb && sp.K == (P->msg ? P->F.k : 0)) return &sp;
    return nullptr;
  };
  static const int ths_lean[] = {24};
  for (const BBVariant& v : kBB) {
    if (v.CP != P->CP) continue;
    const int ns = (Hd + v.HB - 1) / v.HB;
    const int padh = ns * v.HB - Hd;
    for (int pass = 0; pass < 2; ++pass)
    for (int thi = 0; thi < (pass ? 1 : 3); ++thi)
      for (int tw : tws) {
        const int th = pass ? ths_lean[thi] : ths[thi];
        if (pass && v.HB != 128) continue;
        if ((th * tw) % 64 || tw + 2 * rxb + 2 > 64) continue;   // staging rows fit one wave
        if (eth && (th != eth || tw != etw)) continue;
        // (pass 1: the large tiles, only in the lean layout of a compile-time instance)
        const BBSpec* lsp = pass ? spec_for(th, tw) : nullptr;
        if (pass && !(lean_ok && lsp && lsp->lean)) continue;
#if defined(GNCA_BB_NO_LEAN) || defined(GNCA_BB_NO_SPEC) || defined(GNCA_BB_NO_FULL)
        if (pass) continue;   // A/B builds: the plans of round 6 (8x24 at 72^2) / no compile-time instance
#endif
        const BBLayout L = bb_layout(P->CP, v.HB, th, tw, ry, rxb, P->F.k, pass == 1);
        const size_t bytes = (size_t)L.total * 4;
        if (bytes > 160 * 1024) continue;
        const long tx = (W + tw - 1) / tw, ty = (H + th - 1) / th;
        // makespan of the persistent grid (min(CUs, tiles) workgroups): rounds x per-tile cost, so
        // a batch that cannot fill the chip takes the tile that finishes in the fewest rounds
        // (B=16 40^2: 8x8 tiles = 400 tiles = 2 rounds on 256 CUs)
        const long tiles = (long)d->B * tx * ty, cus = bwd_device_cus();
        const long rounds = (tiles + cus - 1) / cus;
        const double per_tile = (double)th * tw + 0.01 * L.RH * L.RW * P->CP + 30.0;
        const double tcost = (double)std::max<long>(rounds * cus, tiles) * per_tile;
        const double cost = 1e12 * ns + 1e9 * padh + tcost;
        if (cost < best) {
          best = cost; P->bb = &v; P->TH = th; P->TW = tw; P->ldsB = bytes; P->bblean = pass == 1;
        }
      }
  }
  if (!P->bb) return false;
#ifdef GNCA_BB_NO_FULL   // A/B builds: the runtime-C instance always
  P->bbfn = P->bbfn2 = P->bb->fn;
#else
  P->bbfn = P->bbfn2 = (C == P->CP && P->bb->fnf) ? P->bb->fnf : P->bb->fn;
#ifndef GNCA_BB_NO_SPEC   // A/B builds: no compile-time-geometry instance
  if (P->bb->HB == 128)
    if (const BBSpec* sp = spec_for(P->TH, P->TW))
      if (sp->lean == P->bblean) P->bbfn = P->bbfn2 = sp->fn;
#endif
#endif
  // a lean-layout plan runs only on its compile-time instance (the runtime-geometry kernels use the
  // full layout)
  if (P->bblean && (P->bbfn != spec_for(P->TH, P->TW)->fn)) return false;
  P->bbf32 = true;
  P->RXB = rxb;
  // (a split-arithmetic BB on bf16 MFMA was built and measured slower, 4.09 vs 3.24 ms for BB at
  // B=1024 72^2: DESIGN.md Appendix A.1; removed in round 6, it is in the git history)
  if (P->bbf32) {
  P->HB = P->bb->HB;
  P->nslices = (Hd + P->HB - 1) / P->HB;
  }
  P->tiles_x = (W + P->TW - 1) / P->TW;
  P->tps = P->tiles_x * ((H + P->TH - 1) / P->TH);
  P->total_tiles = P->tps * d->B;
  P->gridB = std::min(bwd_device_cus(), P->total_tiles);
  if (P->gridB < 1) P->gridB = 1;
  // BA bands: ~8 per sample, thinner when the batch cannot give every CU two workgroups
  // (B=16 128^2 32ch: 16-row bands = 128 workgroups on 256 CUs)
  {
    const long nb_target = std::max<long>(8, (2L * bwd_device_cus() + d->B - 1) / d->B);
    long rows = (H + nb_target - 1) / nb_target;
    const long cap = (48L * 1024 / 4 / W - 2) / 2;
    if (rows > cap) rows = cap;
    if (rows < 1) rows = 1;
    P->band = (int)rows;
    P->nbands = (H + P->band - 1) / P->band;
    P->ldsA = (size_t)(2 * P->band + 2) * W * 4;
    if (P->ldsA > 64 * 1024) return false;
  }
  // BC tiles: fewest padded cells + staged halo, within the per-thread staging registers
  {
    static const int bth[] = {4, 6, 8, 12, 16, 24, 32};
    const int btw[] = {16, 24, 32, 48, 64, W};   // W: full-width rows (contiguous line fills)
    const int rxc = P->zp ? 0 : rx;
    double bestc = 1e300;
    P->TH3 = 0;
    // 128-byte lines touched by a staged row segment of n floats at an unaligned start
    auto lines = [](int n) { return (n * 4 + 127) / 128 + 1; };
    for (int th : bth)
      for (int tw : btw) {
        const int se = bc_stage(th, tw, ry, rxc, P->msg);
        if (se > kBCStage * kThreads || th * tw > 4 * kThreads) continue;
        const long tx = (W + tw - 1) / tw, ty = (H + th - 1) / th;
        // per tile: its cells plus the cache lines its staging fills (3 dY planes with a 1-ring,
        // the dG region with the gather halo), in floats
        const double fill = 32.0 * (3.0 * (th + 2) * lines(tw + 2) +
                                    (P->msg ? (double)(th + 2 * ry) * lines(tw + 2 * rxc) : 0.0));
        const double cost = (double)tx * ty * (th * tw + 0.25 * fill);
        if (cost < bestc) { bestc = cost; P->TH3 = th; P->TW3 = tw; }
      }
    if (!P->TH3) return false;
    P->tiles_x3 = (W + P->TW3 - 1) / P->TW3;
    P->tps3 = P->tiles_x3 * ((H + P->TH3 - 1) / P->TH3);
    P->ldsC = (size_t)(2 * bc_stage(P->TH3, P->TW3, ry, rxc, P->msg) + P->TH3 * P->TW3 +
                       std::max(P->F.k, 1) + 27 * C) * 4;
  }
  P->rows_per = std::max(1, (int)((4096 + W - 1) / W));
  P->nrb = (H + P->rows_per - 1) / P->rows_per;
  const int dm = std::max(d->d_model, 1), k = std::max(P->F.k, 1);
  P->ldsD = ((size_t)C * H + C + dm + (size_t)k * C + (size_t)k * dm + 2 * k + dm + (size_t)k * dm +
             (size_t)H * dm + 2) * sizeof(double) + 2 * (size_t)dm * C * sizeof(float);
  if (P->msg && P->zp && P->ldsD > 64 * 1024) return false;
  P->o_w1 = 0;
  P->o_b1 = Hd * 3 * C;
  P->o_w2 = P->o_b1 + Hd;
  P->o_wm = P->o_w2 + C * Hd;
  P->o_bm = P->o_wm + C * C;
  P->npart = P->o_bm + C;
  P->nq = 2 * dm * C + 2 * dm + 1;
  const size_t n = (size_t)d->B * C * H * W, hw = (size_t)d->B * H * W;
  size_t o = 0;
  auto carve = [&o](size_t bytes) { size_t at = o; o += (bytes + 255) & ~(size_t)255; return at; };
  P->off_fwd = carve(P->F.ws_bytes);
  P->off_U = carve(n * 4);
  P->off_dY = carve(3 * n * 4);
  P->off_dG = carve(P->msg ? n * 4 : 0);
  P->off_dmb = carve(P->msg && P->zp ? hw * 4 : 0);
  P->off_keep = carve(hw);
  P->off_alist = carve((size_t)(d->B + 1) * 4);
  P->off_pa = carve((size_t)d->B * P->nbands * (2 + 2 * C) * 8);
  P->off_coef = carve((size_t)d->B * 4 * 4);
  P->off_pb = carve((size_t)P->gridB * NW * P->npart * 4);
  const bool att = P->msg && P->zp;
  P->off_dots = carve(att ? (size_t)d->B * P->F.k * P->nrb * 8 : 0);
  P->off_pq = carve(att ? (size_t)d->B * P->nq * 8 : 0);
  P->off_corr = carve(att ? (size_t)d->B * H * C * 4 : 0);
  P->bytes = o;
  return true;
}

static int bwd_check() {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return GNCA_ERR_HIP;
  }
  return GNCA_OK;
}

struct Reducer {
  RedArgs a;
  Reducer(const void* part, bool f64, long rows, long stride) {
    memset(&a, 0, sizeof(a));
    a.part = part; a.f64 = f64 ? 1 : 0; a.rows = rows; a.stride = stride;
  }
  void add(long col0, int ncols, int step, float* out) {   // step 0: zeros
    if (ncols <= 0 || !out) return;
    a.col0[a.nseg] = col0;
    a.step[a.nseg] = step;
    a.out[a.nseg] = out;
    a.ncols += ncols;
    a.end[a.nseg] = a.ncols;
    ++a.nseg;
  }
  int launch(hipStream_t st) {
    if (a.nseg == 0 || a.ncols == 0) return GNCA_OK;
    hipLaunchKernelGGL(gnca_b_reduce, dim3((a.ncols + 31) / 32), dim3(kThreads), 0, st, a);
    return bwd_check();
  }
};

// The weight-gradient reductions depend only on BB's and BA's partial rows, not on BC: they run on a
// per-device side stream beside BC (forked from the caller's stream after BB, joined back before
// the entry point returns, so every later use of the outputs and workspace on the caller's stream
// is ordered after them).  Created once per device, never destroyed (as the rollout's sub-streams).
struct BwdSide {
  hipStream_t s;
  hipEvent_t fork, join;
  std::mutex mu;   // one backward's fork .. join enqueue at a time per device
};

static BwdSide* bwd_side() {
  static std::mutex mu;
  static std::unordered_map<int, BwdSide*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  BwdSide* bs = new BwdSide();
  if (hipStreamCreateWithFlags(&bs->s, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&bs->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&bs->join, hipEventDisableTiming) != hipSuccess)
    return nullptr;
  cache[dev] = bs;
  return bs;
}

// Fork on construction, join on destruction (every return path of the backward, errors included);
// without a side stream (or GNCA_BWD_ONE_STREAM in A/B builds) everything stays on the caller's.
// Only for large steps: the fork and join cost a small, host-bound backward more than the overlap
// gives (B=16 40^2: 0.092 -> 0.103 ms; B=128 72^2: 0.623 -> 0.608; B=1024: equal)
constexpr long kSideMinCells = 1L << 19;
struct SideFork {
  hipStream_t main, side;
  BwdSide* bs = nullptr;
  std::unique_lock<std::mutex> lk;
  bool ok = true;
  SideFork(hipStream_t st, long cells) : main(st), side(st) {
#ifndef GNCA_BWD_ONE_STREAM
    if (cells < kSideMinCells) return;
    bs = bwd_side();
    if (!bs) return;
    lk = std::unique_lock<std::mutex>(bs->mu);
    if (hipEventRecord(bs->fork, st) != hipSuccess || hipStreamWaitEvent(bs->s, bs->fork, 0) != hipSuccess) {
      ok = false;
      return;
    }
    side = bs->s;
#endif
  }
  ~SideFork() {
    if (side != main) {
      (void)hipEventRecord(bs->join, side);
      (void)hipStreamWaitEvent(main, bs->join, 0);
    }
  }
};


}  // namespace
}  // namespace gnca

using namespace gnca;

extern "C" {

#ifdef GNCA_PROFILE
int gnca_bprof_dump(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bprof), sizeof(g_bprof)) == hipSuccess ? 0 : -1;
}
#endif

size_t gnca_bwd_workspace_bytes(const gnca_step_desc* desc) {
  BwdPlan P, Q;   // enough for the full-batch plan and the masked step's
  if (!bwd_plan(desc, &P) || !bwd_plan(desc, &Q, false)) return 0;
  return std::max(P.bytes, Q.bytes);
}

int gnca_bb_variant(const gnca_step_desc* desc, char* name, int32_t n) {
  BwdPlan P;
  if (!name || n <= 0 || !bwd_plan(desc, &P)) return GNCA_ERR_INVALID;
  int th = 0, tw = 0, ry = 0, rx = 0, k = -1;
  bool full = P.bbfn == P.bb->fnf && P.bb->fnf != nullptr, lean = false;
  for (const BBSpec& sp : kBBS)
    if (sp.fn == P.bbfn) { th = sp.TH; tw = sp.TW; ry = sp.RY; rx = sp.RX; k = sp.K; lean = sp.lean; full = true; }
  snprintf(name, (size_t)n, "gnca_b_mlp<%d,%d,%d,%d,%d,%d,%d,%d,%d>", P.CP, P.HB, full ? 1 : 0, th, tw, ry, rx, k,
           lean ? 1 : 0);
  return GNCA_OK;
}

int gnca_step_bwd_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                      const void* fire, const uint8_t* active, const float* gy, float* gx,
                      const gnca_grads* grads, const void* saved, void* ws, size_t ws_bytes,
                      void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  StreamDeviceGuard dg(st);
  if (!desc || !w || !x || !gy || !gx || !grads) return GNCA_ERR_INVALID;
  if (gx == x || gx == gy) return GNCA_ERR_INVALID;
  gnca_step_desc d = *desc;
  d.flags &= ~GNCA_ATTENTION;
  BwdPlan P;
  if (!bwd_plan(&d, &P, active == nullptr)) return GNCA_ERR_INVALID;
  if (!ws || ws_bytes < P.bytes) return GNCA_ERR_WORKSPACE;
  if (P.gn && (!w->gn_weight || !w->gn_bias)) return GNCA_ERR_INVALID;
  if (P.msg && (!w->wm || !w->bm)) return GNCA_ERR_INVALID;
  if (P.msg && P.zp && (!w->wq || !w->bq || !w->wk || !w->bk || !w->scaling)) return GNCA_ERR_INVALID;
  char* wsb = reinterpret_cast<char*>(ws);
  const int B = d.B, C = d.C, H = d.H, W = d.W, Hd = d.hidden;
  const size_t HW = (size_t)H * W;
  int rc;
  // F: recompute the forward's dx / GroupNorm partials / offset weights (gx is a dummy x_out:
  // phase K2, the only writer of x_out, is not run)
  const char* fw = saved ? reinterpret_cast<const char*>(saved) : wsb + P.off_fwd;
  if (!saved) {
    // recompute dx / partials / offset weights (K2, the only writer of x_out = gx here, is not run)
    rc = active ? gnca_step_masked_phases(&d, w, x, gx, fire, active, wsb + P.off_fwd, P.F.ws_bytes,
                                          stream, GNCA_PHASE_K0 | GNCA_PHASE_K1)
                : gnca_step_phases_f32(&d, w, x, gx, fire, nullptr, wsb + P.off_fwd, P.F.ws_bytes, stream,
                                       GNCA_PHASE_K0 | GNCA_PHASE_K1);
    if (rc != GNCA_OK) return rc;
  }
  const float* dx = reinterpret_cast<const float*>(fw + P.F.off_dx);
  const double* stats = reinterpret_cast<const double*>(fw + P.F.off_stats);
  const float* offw = (P.msg && P.zp) ? reinterpret_cast<const float*>(fw + P.F.off_offw) : nullptr;
  float* U = reinterpret_cast<float*>(wsb + P.off_U);
  float* dY = reinterpret_cast<float*>(wsb + P.off_dY);
  float* dG = reinterpret_cast<float*>(wsb + P.off_dG);
  float* dmb = (P.msg && P.zp) ? reinterpret_cast<float*>(wsb + P.off_dmb) : nullptr;
  // BB's keep bytes (gnca_b_mlp; the split BB of A/B builds stores the dead cells' zeros instead)
#ifndef GNCA_BB_NO_KEEP   // A/B builds: the dead cells' zeros stored by BB (round 4's scheme)
  uint8_t* keep = P.bbf32 ? reinterpret_cast<uint8_t*>(wsb + P.off_keep) : nullptr;
#else
  uint8_t* keep = nullptr;
#endif
  double* pa = reinterpret_cast<double*>(wsb + P.off_pa);
  float* coef = reinterpret_cast<float*>(wsb + P.off_coef);
  float* pb = reinterpret_cast<float*>(wsb + P.off_pb);
  // BA
  {
    BAArgs a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.dx = dx; a.gy = gy; a.gamma = w->gn_weight; a.beta = w->gn_bias; a.stats = stats;
    a.gx = gx; a.U = U; a.part = pa; a.active = active;
    a.B = B; a.C = C; a.H = H; a.W = W; a.tps = P.F.tps; a.band = P.band; a.nbands = P.nbands;
    a.gain = d.update_gain; a.thr = d.alpha_thr; a.eps = d.gn_eps; a.use_gn = P.gn ? 1 : 0;
    hipLaunchKernelGGL(gnca_b_gnprep, dim3(B * P.nbands), dim3(kThreads), P.ldsA, st, a);
    if ((rc = bwd_check()) != GNCA_OK) return rc;
  }
  // BS
  hipLaunchKernelGGL(gnca_b_coef, dim3(B), dim3(64), 0, st, stats,
                     (const double*)pa, coef, B, C, (int)HW, P.F.tps, P.nbands, d.gn_eps, P.gn ? 1 : 0);
  if ((rc = bwd_check()) != GNCA_OK) return rc;
  // BB, one launch per hidden slice
  {
    BBArgs a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.U = U; a.dx = dx; a.coef = coef; a.fire = fire;
    a.perc = w->perception; a.w1 = w->w1; a.b1 = w->b1; a.w2 = w->w2; a.wm = w->wm; a.bm = w->bm;
    a.offw = offw; a.active = active; a.dY = dY; a.dG = dG; a.dmb = dmb; a.keep = keep; a.part = pb;
    a.seed = d.rng_seed; a.rng_step = d.rng_step; a.sample_base = d.sample_base;
    a.B = B; a.C = C; a.H = H; a.W = W; a.hidden = Hd; a.k = P.msg ? P.F.k : 0;
    a.RY = P.RY; a.RX = P.RXB; a.TH = P.TH; a.TW = P.TW; a.tiles_x = P.tiles_x; a.tps = P.tps;
    a.total_tiles = P.total_tiles; a.fire_mode = d.fire_mode;
    a.npart = P.npart; a.o_w1 = P.o_w1; a.o_b1 = P.o_b1; a.o_w2 = P.o_w2; a.o_wm = P.o_wm; a.o_bm = P.o_bm;
    a.fire_rate = d.fire_rate; a.alpha_thr = d.alpha_thr; a.graph_alpha_thr = d.graph_alpha_thr;
    a.message_gain = d.message_gain;
    a.uniform_w = P.F.k > 0 ? (float)(1.0 / (double)P.F.k) : 0.f;
    a.flags = d.flags & (GNCA_ZERO_PAD_SHIFT | GNCA_ALIVE_TO_ALIVE | GNCA_HIDDEN_ONLY);
    if (P.msg) a.flags |= kMsg;
    if (P.gn) a.flags |= kGN;
#ifdef GNCA_BB_MEMSET
    // A/B builds: the dead cells' dY / dG / <dm, b_M> zeros as one streaming fill of the three
    // buffers ahead of BB instead of BB's per-dead-cell stores.  Measured slower (B=1024 72^2 bwd
    // 4.77-4.79 vs 4.75-4.76 ms, B=16 40^2 0.100 vs 0.097 ms): the fill writes every cell, the live
    // ones twice, while the dead-cell stores overlap BB's MFMA work
    if (hipMemsetAsync(dY, 0, 3 * (size_t)B * C * HW * sizeof(float), st) != hipSuccess ||
        (P.msg && hipMemsetAsync(dG, 0, (size_t)B * C * HW * sizeof(float), st) != hipSuccess) ||
        (dmb && hipMemsetAsync(dmb, 0, (size_t)B * HW * sizeof(float), st) != hipSuccess))
      return GNCA_ERR_HIP;
    a.flags |= kZeroed;
#endif
    const int RW = P.TW + 2 * P.RXB;
    for (int o = 0; o < a.k; ++o) a.odl[o] = d.offsets[2 * o] * RW + (P.zp ? 0 : d.offsets[2 * o + 1]);
    // a masked step walks only the active samples' tiles (the static per-workgroup tile ranges of the
    // full batch left the workgroups whose ranges held more active samples the slowest).  Not in
    // zero-pad mode: BC2 reads every sample's keep bytes, which BB writes for the inactive ones
#ifndef GNCA_BB_NO_ALIST   // A/B builds: the full batch's tile ranges (round 6 before the list)
    if (active && !P.zp && keep) {
#else
    if (false) {
#endif
      int* alist = reinterpret_cast<int*>(wsb + P.off_alist);
      hipLaunchKernelGGL(gnca_b_actlist, dim3(1), dim3(kThreads), 0, st, active, B, alist);
      if ((rc = bwd_check()) != GNCA_OK) return rc;
      a.alist = alist;
    }
#ifndef GNCA_BB_NO_DMA4   // A/B builds: 4-byte staging pieces (round 4's BB)
    if (W % 4 == 0 && P.RXB % 4 == 0 && P.TW % 4 == 0 && P.bbf32) a.flags |= kDma4;
#endif
    (void)hipFuncSetAttribute(P.bbfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.ldsB);
    (void)hipFuncSetAttribute(P.bbfn2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.ldsB);
    for (int s = 0; s < P.nslices; ++s) {
      a.h0 = s * P.HB;
      a.flags = (a.flags & ~kFirst) | (s == 0 ? kFirst : 0u);
      void* args[] = {&a};
      const hipError_t e = hipLaunchKernel(s == 0 ? P.bbfn : P.bbfn2, dim3(P.gridB), dim3(kThreads), args, P.ldsB, st);
      if (e != hipSuccess) { g_last_hip = (int)e; return GNCA_ERR_HIP; }
      if ((rc = bwd_check()) != GNCA_OK) return rc;
    }
  }
  // the weight-gradient reductions (BB's and BA's partial rows) on the side stream, beside BC
  SideFork sf(st, (long)B * (long)HW);
  if (!sf.ok) return GNCA_ERR_HIP;
  const int dmod = std::max(d.d_model, 1);
  {
    Reducer r(pb, false, (long)P.gridB * NW, P.npart);
    r.add(P.o_w1, Hd * 3 * C, 1, grads->w1);
    r.add(P.o_b1, Hd, 1, grads->b1);
    r.add(P.o_w2, C * Hd, 1, grads->w2);
    if (P.graph) {
      r.add(P.o_wm, C * C, 1, grads->wm);
      r.add(P.o_bm, C, 1, grads->bm);
      if (!(P.msg && P.zp)) {   // torus (or no message): the offset weights are constants
        r.add(0, dmod * C, 0, grads->wq);
        r.add(0, dmod, 0, grads->bq);
        r.add(0, dmod * C, 0, grads->wk);
        r.add(0, dmod, 0, grads->bk);
        r.add(0, 1, 0, grads->scaling);
      }
    }
    if ((rc = r.launch(sf.side)) != GNCA_OK) return rc;
  }
  if (P.gn) {
    Reducer r(pa, true, (long)B * P.nbands, 2 + 2 * C);
    r.add(2, C, 2, grads->gn_weight);
    r.add(3, C, 2, grads->gn_bias);
    if ((rc = r.launch(sf.side)) != GNCA_OK) return rc;
  }
  // BC
  {
    BCArgs a;
    memset(&a, 0, sizeof(a));
    a.dY = dY; a.dG = dG; a.x = x; a.perc = w->perception; a.offw = offw; a.gx = gx; a.keep = keep;
    a.active = active;
    a.B = B; a.C = C; a.H = H; a.W = W; a.k = P.msg ? P.F.k : 0;
    a.TH = P.TH3; a.TW = P.TW3; a.tiles_x = P.tiles_x3; a.tps = P.tps3;
    // channel groups: enough workgroups to fill the chip when the batch is small, ~4 per CU (each
    // walks its channels one memory round trip at a time; B=16 128^2 32ch bwd: 2 per CU 1.456,
    // 4 1.382, 8 1.392, 16 1.411 ms; tools/bc_sweep.sh)
    static const char* ncg_env = GNCA_AB_ENV("GNCA_BC_WGS_PER_CU");   // measurement knob (A/B runs only)
    const long per_cu = ncg_env && atoi(ncg_env) > 0 ? atoi(ncg_env) : 4;
    const long wgs = (long)B * P.tps3, want = per_cu * bwd_device_cus();
    a.ncg = (int)std::min<long>(C, std::max<long>(1, (want + wgs - 1) / wgs));
    a.cpw = (C + a.ncg - 1) / a.ncg;
    a.ncg = (C + a.cpw - 1) / a.cpw;
    a.RY = P.RY; a.RX = P.zp ? 0 : P.RX;
    a.graph_alpha_thr = d.graph_alpha_thr;
    a.uniform_w = P.F.k > 0 ? (float)(1.0 / (double)P.F.k) : 0.f;
    a.flags = (d.flags & (GNCA_ZERO_PAD_SHIFT | GNCA_ALIVE_TO_ALIVE)) | (P.msg ? kMsg : 0u);
    for (int o = 0; o < 2 * a.k; ++o) a.offs[o] = d.offsets[o];
    hipLaunchKernelGGL(a.k == 8 ? gnca_b_adjoint<8> : a.k == 16 ? gnca_b_adjoint<16> : gnca_b_adjoint<0>,
                       dim3(B * P.tps3 * a.ncg), dim3(kThreads), P.ldsC, st, a);
    if ((rc = bwd_check()) != GNCA_OK) return rc;
  }
  if (!P.graph || !(P.msg && P.zp)) return GNCA_OK;
  double* dots = reinterpret_cast<double*>(wsb + P.off_dots);
  double* pq = reinterpret_cast<double*>(wsb + P.off_pq);
  float* corr = reinterpret_cast<float*>(wsb + P.off_corr);
  {
    BC2Args a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.dG = dG; a.dmb = dmb; a.keep = keep; a.dots = dots;
    a.B = B; a.C = C; a.H = H; a.W = W; a.k = P.F.k; a.nrb = P.nrb; a.rows_per = P.rows_per;
    a.gthr = d.graph_alpha_thr; a.a2a = (d.flags & GNCA_ALIVE_TO_ALIVE) ? 1 : 0;
    for (int o = 0; o < 2 * P.F.k; ++o) a.offs[o] = d.offsets[o];
    // (one workgroup per (sample, offset, row block); one per (sample, row block) with every offset's
    //  sums in registers measured 3x slower at B=16 40^2: 156 vs 47 us, too few workgroups)
    hipLaunchKernelGGL(gnca_b_dots, dim3(B * P.F.k * P.nrb), dim3(kThreads), 0, st, a);
    if ((rc = bwd_check()) != GNCA_OK) return rc;
  }
  {
    BDArgs a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.wq = w->wq; a.bq = w->bq; a.wk = w->wk; a.bk = w->bk; a.scaling = w->scaling;
    a.rs = reinterpret_cast<const double*>(fw + P.F.off_rs);
    a.dots = dots; a.pq = pq; a.corr = corr;
    a.B = B; a.C = C; a.H = H; a.W = W; a.d = d.d_model; a.k = P.F.k; a.nrb = P.nrb;
    for (int o = 0; o < 2 * P.F.k; ++o) a.offs[o] = d.offsets[o];
    hipLaunchKernelGGL(gnca_b_attn, dim3(B), dim3(kThreads), P.ldsD, st, a);
    if ((rc = bwd_check()) != GNCA_OK) return rc;
  }
  {
    const size_t total = (size_t)B * C * HW;
    size_t blocks = (total + kThreads - 1) / kThreads;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(gnca_b_rowcorr, dim3((unsigned)blocks), dim3(kThreads), 0, st, gx, (const float*)corr,
                       B, C, H, W);
    if ((rc = bwd_check()) != GNCA_OK) return rc;
  }
  {
    const int dq = d.d_model;
    Reducer r(pq, true, B, P.nq);
    r.add(0, dq * C, 1, grads->wq);
    r.add(dq * C, dq, 1, grads->bq);
    r.add(dq * C + dq, dq * C, 1, grads->wk);
    r.add(2 * dq * C + dq, dq, 1, grads->bk);
    r.add(2 * dq * C + 2 * dq, 1, 1, grads->scaling);
    if ((rc = r.launch(st)) != GNCA_OK) return rc;
  }
  return GNCA_OK;
}

}  // extern "C"
