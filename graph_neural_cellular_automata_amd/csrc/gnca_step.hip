// gnca_step.hip — MI355X (gfx950 / CDNA4) kernels for the NCA rollout step + the C ABI.
//
// One CA step (reference: src/modules/ncagraph.py:106-168, src/modules/nca.py:64-105,
// src/modules/graph_augmentation.py:104-169, src/modules/perception.py:21-26) runs as:
//
//   K0  gnca_k0_offset_weights   zero-pad mode only: per-sample softmax weights over the
//                                sampled offsets from per-row channel sums of x (the reference's
//                                pooled Q.K logits, graph_augmentation.py:113-153, restated
//                                exactly: Q and K enter only through their spatial means).
//                                Torus mode needs no K0: mean(roll(K)) = mean(K), so every logit
//                                is equal and the softmax weight is exactly 1/k.
//   K1  gnca_k1_update<CP,HD>    persistent, one 256-thread workgroup per (sample, tile):
//                                x tile + halo staged in LDS (torus-wrapped or zero-padded),
//                                alive / sender planes, 3x3 depthwise perception, the offset
//                                gather of ALIVE-MASKED x (the message projection is linear, so
//                                W_M is applied once after the gather), the 1x1 MLP and the C x C
//                                message projection on fp32 MFMA (v_mfma_f32_16x16x4_f32), message
//                                policy, fire and pre-alive masks -> dx, plus per-tile fp64
//                                GroupNorm partials (no atomics: deterministic).
//   K2  gnca_k2_finalize         GroupNorm (per-sample stats combined in fixed order), tanh*gain,
//                                residual, post-update alive gate on alpha (3x3 halo) -> x_out.
//
// MFMA fragment maps (v_mfma_f32_16x16x4_f32, lane l, g = l>>4, col = l&15):
//   A[16x4]: lane supplies A[l&15][g];  B[4x16]: lane supplies B[g][l&15];
//   D[16x16]: lane holds D[4g + r][l&15], r = 0..3.
// A 16-cell group maps cell -> lane&15.  GEMM1 H[hid x cell] = W1[hid x 3C] Y[3C x cell]: lane
// (cell, g) supplies feature slot 4s+g at k-step s, i.e. channels g, g+4, ... of its own cell,
// so each lane computes its own perception features.  GEMM1's accumulator rows (hidden 4g+r of
// tile m) are exactly the B operand of GEMM2 DL = W2 H at k-step (m, r) — no data movement.

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "gnca_device.h"

namespace gnca {

// Measurement-only ablation switches (tools/ablate.py builds variants with -DGNCA_ABLATE=<bits>;
// the product library is always built with 0).  Outputs are wrong in an ablated build.
#ifndef GNCA_ABLATE
#define GNCA_ABLATE 0
#endif
constexpr int kAblStage = 1;     // skip the global->LDS staging loads (LDS keeps old data)
constexpr int kAblGather = 2;    // skip the offset gather
constexpr int kAblPerceive = 4;  // skip the 3x3 perception (y = 0)
constexpr int kAblMfma = 8;      // skip GEMM1/GEMM2 MFMAs
constexpr int kAblStore = 16;    // skip the dx stores
constexpr int kAblPlanes = 32;   // skip the alive / sender planes
constexpr int kAblFire = 64;     // fire = a fixed checkerboard instead of the hash (same density)
constexpr int kAblZero = 128;    // skip the dead-cell zero stores of the compaction pass
constexpr int kAblReduce = 256;  // skip the per-tile GroupNorm partial reduction
constexpr int kAblTiles = 512;   // skip the tile loop (times launch + prologue)
constexpr int kAblFill = 1024;   // skip the weight fill (LDS keeps old data)
constexpr int kAblPrep = 2048;   // split K1: skip the preparer after the first tile (slots keep old lists)
constexpr uint32_t kMsgOnly = 1u << 16;   // internal K1 flag: write agg message, skip MLP
constexpr uint32_t kGraphOn = 1u << 17;   // internal K1 flag: gather + message projection needed

__device__ float g_zero[4];  // LDS-DMA source for off-image cells (zero-initialised)

// Measurement-only phase timers (tools/ablate.py builds with -DGNCA_PROFILE): wave 0 of each K1
// workgroup accumulates s_memtime deltas per phase; gnca_prof_dump copies them out.
#ifdef GNCA_PROFILE
constexpr int kProfPhases = 8;
__device__ unsigned long long g_prof[1024][2 * kProfPhases];   // [.][8..15]: spare (role profiles)
#define PROF_DECL unsigned long long prof_t = __builtin_amdgcn_s_memtime(), prof_acc[kProfPhases] = {0};
#define PROF_MARK(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); prof_acc[i] += t_ - prof_t; prof_t = t_; } while (0)
#define PROF_STORE do { if (threadIdx.x == 0) for (int i_ = 0; i_ < kProfPhases; ++i_) g_prof[blockIdx.x & 1023][i_] = prof_acc[i_]; } while (0)
// waves 0 and 4 (the two waves of SIMD 0): [.][0..7] and [.][8..15]
#define PROF_STORE_W04 do { if ((threadIdx.x & 255) == 0) for (int i_ = 0; i_ < kProfPhases; ++i_) g_prof[blockIdx.x & 1023][(threadIdx.x >> 8) * kProfPhases + i_] = prof_acc[i_]; } while (0)
// waves 0 and 3 (the split K1's preparer): [.][0..7] and [.][8..15]
#define PROF_STORE_W03 do { if (threadIdx.x == 0 || threadIdx.x == 192) for (int i_ = 0; i_ < kProfPhases; ++i_) g_prof[blockIdx.x & 1023][(threadIdx.x ? kProfPhases : 0) + i_] = prof_acc[i_]; } while (0)
// waves 0 and 7 (the 32-channel split K1's preparer): [.][0..7] and [.][8..15]
#define PROF_STORE_W07 do { if (threadIdx.x == 0 || threadIdx.x == 448) for (int i_ = 0; i_ < kProfPhases; ++i_) g_prof[blockIdx.x & 1023][(threadIdx.x ? kProfPhases : 0) + i_] = prof_acc[i_]; } while (0)
// the fold's own sub-phases (gnca_k1_split<..., FOLD>): waves 0 and 3, 16 buckets each (gnca_fprof_dump)
__device__ unsigned long long g_fprof[1024][32];
#define FPROF_DECL unsigned long long fp_t = __builtin_amdgcn_s_memtime(), fp_acc[16] = {0};
#define FPROF_START() do { fp_t = __builtin_amdgcn_s_memtime(); } while (0)
#define FPROF_MARK(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); fp_acc[i] += t_ - fp_t; fp_t = t_; } while (0)
#define FPROF_COUNT(i) do { fp_acc[i] += 1; } while (0)
#define FPROF_STORE do { if (threadIdx.x == 0 || threadIdx.x == 192) for (int i_ = 0; i_ < 16; ++i_) g_fprof[blockIdx.x & 1023][(threadIdx.x ? 16 : 0) + i_] = fp_acc[i_]; } while (0)
// every wave's s_memtime at up to 8 points of the split K1, relative to the wave's first instruction
// (the critical path of a one-tile launch; gnca_arr_dump): [block][wave][point]
__device__ unsigned long long g_arr[1024][16][8];
#define ARR_DECL const unsigned long long arr_t0 = __builtin_amdgcn_s_memtime();
#define ARR_MARK(k) do { if ((threadIdx.x & 63) == 0) g_arr[blockIdx.x & 1023][threadIdx.x >> 6][k] = __builtin_amdgcn_s_memtime() - arr_t0; } while (0)
#else
#define ARR_DECL
#define ARR_MARK(k) do {} while (0)
#define FPROF_DECL
#define FPROF_START() do {} while (0)
#define FPROF_MARK(i) do {} while (0)
#define FPROF_COUNT(i) do {} while (0)
#define FPROF_STORE do {} while (0)
#define PROF_STORE_W07 do {} while (0)
#define PROF_STORE_W03 do {} while (0)
#define PROF_STORE_W04 do {} while (0)
#define PROF_DECL
#define PROF_MARK(i) do {} while (0)
#define PROF_STORE do {} while (0)
#endif

// ------------------------------------------------------------------------------------------
// LDS layout of K1 (floats; every region starts on a 16-byte boundary)
// ------------------------------------------------------------------------------------------
struct K1Layout {
  int b1s, bms, percs, wts, kp_, lst, red, wmf, w1f, w2f, sp, xs, al, total;
  int RH, RW, PSTR, NI, NIA, ALW;
};

// W1 fragments stay in LDS (read as 16-byte fragments every group: LDS reads cost no VALU, and
// keeping them out of VGPRs removes spills and leaves room to keep loads in flight)
__host__ __device__ constexpr bool w1_in_regs(int, int) { return false; }

// The staged region is the tile plus an (RY, RX) halo for the gather (RH x RW per channel, NI
// LDS-DMA wave-instructions of 64 dwords, plane stride PSTR >= 64*NI and = 16 mod 32), plus one
// alpha plane with one more ring ((RH+2) x (RW+2), NIA instructions) for the 3x3 alive max-pool of
// the gather sources and the Sobel-ring cells.
// Channel-plane stride of the staged region: a multiple of the DMA chunk (64 dwords, or 256 floats
// for the 16-byte DMA of quad-aligned regions) plus 16 floats, so the planes start 16 banks apart.
__host__ __device__ constexpr int k1_pstr(int RH, int RW, int RX, int TW) {
  return ((RW % 4) == 0 && (RX % 4) == 0 && (TW % 4) == 0)
             ? 256 * ((RH * RW / 4 + 63) / 64) + 16
             : 64 * ((RH * RW + 63) / 64) + 16;
}

__host__ __device__ inline K1Layout k1_layout(int CP, int HDP, int TH, int TW, int RY, int RX,
                                              int kmax) {
  K1Layout L;
  const int CPQ = CP / 4, KS = 3 * CPQ, MT = HDP / 16, MO = (CP + 15) / 16;
  const int KSP = odd4(KS), S2 = odd4(4 * MT), SWM = odd4(CPQ);
  L.RH = TH + 2 * RY;
  L.RW = TW + 2 * RX;
  L.NI = (L.RH * L.RW + 63) / 64;
  L.PSTR = k1_pstr(L.RH, L.RW, RX, TW);
  L.ALW = L.RW + 2;
  L.NIA = ((L.RH + 2) * L.ALW + 63) / 64;
  const int kp = r4(kmax > 0 ? kmax : 4);
  int o = 0;
  L.xs = o; o += CP * L.PSTR;               // first: region reads fit the 16-bit DS offsets
  L.sp = o; o += r4(L.RH * L.RW);
  L.al = o; o += 64 * L.NIA;
  L.kp_ = o; o += r4(TH * TW);              // per-tile keep plane (fire, then fire AND alive)
  L.lst = o; o += r4(TH * TW) + 8;          // compacted live-cell list (ints) + per-wave counts
  L.b1s = o; o += r4(HDP);
  L.bms = o; o += r4(CP);
  L.percs = o; o += CP * 36;
  L.wts = o; o += kp;
  L.red = o; o += 64;                     // per-wave partials (up to 8 waves)
  L.wmf = o; o += MO * 64 * SWM;
  L.w2f = o; o += MO * 64 * S2;
  L.w1f = o; o += MT * 64 * KSP;
  L.total = o;
  return L;
}

struct K1Args {
  const float* x;
  float* out;          // dx (step) or agg message (message-only)
  double* stats;       // [B * tps * 2]: per-tile (sum, sumsq) of dx
  float* attn;         // [B,H,W] raw attention (or null)
  float* attn_mm;      // [B * tps * 2]: per-tile (min, max) of raw attention
  const float* perc;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* wm;
  const float* bm;
  const float* offw;   // [B * k] per-sample offset weights, or null -> uniform_w
  const void* fire;
  const uint8_t* active;   // [B] or null: samples with active[b] == 0 are skipped (K2 copies them)
  const uint8_t* alive;    // [B,H,W] or null: this step's pre-update masks, written by the previous
                           // step's K2 (bit 0: max-pool > alpha_thr, bit 1: > graph_alpha_thr)
  // compact update field (rollout mode, split K1 only; null = dense NCHW dx in `out`): `out` holds
  // per tile [C][TH*TW] the live cells' dx in live-cell order; rmask[tile*TH + row] = the row's
  // live-cell bits, rpre[tile*TH + row] = live cells in the tile's earlier rows
  uint64_t* rmask;
  uint32_t* rpre;
  float* dxa;          // compact mode: the alpha channel's update, [B,H,W], live cells only (K2 reads it over
                       // its band's halo rows without the row tables)
  uint64_t seed;
  int64_t rng_step;
  int64_t sample_base;
  int B, C, H, W, hidden, k, RY, RX, TH, TW, tiles_x, tps, total_tiles, fire_mode;
  float fire_rate, alpha_thr, graph_alpha_thr, message_gain, uniform_w;
  uint32_t flags;
  uint64_t* stamps;    // measurement only (null in product launches): per-workgroup wall-clock stamps
  const char* wimg;    // split K1: the weight images built once per rollout (gnca_ks_images), or null
  // The fold (rollout mode, gnca_k1_split<..., FOLD = true>): this launch also FINISHES the previous
  // step.  Each tile's staged region is x = finalize(xp, dxp) (GroupNorm with the previous step's
  // partials, tanh * gain, residual, post-update alpha gate: K2's arithmetic) instead of an LDS-DMA
  // copy of `x`; the tile's interior of that state goes to xo; the pre-update masks come from the
  // finalized alpha instead of `alive`.  The previous step's compact update field: dxp / rmaskp /
  // rprep / dxap / statsp (written by the previous K1 launch, the same layout as out / rmask / rpre
  // / dxa / stats).
  const float* xp;
  float* xo;
  const float* dxp;
  const uint64_t* rmaskp;
  const uint32_t* rprep;
  const float* dxap;
  const double* statsp;
  const float* gamma;
  const float* beta;
  float gain, eps;
  int use_gn, nst;     // nst: GroupNorm partial pairs per sample (tps x waves)
  int odl[GNCA_MAX_OFFSETS];   // gather source delta in the staged region: dy*RW + dx (pad: dy*RW)
};

// ReLU with torch.relu's NaN semantics (NaN stays NaN): IEEE maximum, one v_maximum3_f32 on gfx950
// instead of a compare + select (the GEMM1 epilogue runs it on 32 accumulators per 16-cell group,
// and every VALU instruction costs fp32 MFMA issue time on the shared datapath).  Not inline asm:
// hipcc does not insert the MFMA-result read hazard wait states around an asm statement.
__device__ __forceinline__ float relu_nan(float v) { return __builtin_elementwise_maximum(v, 0.f); }

// ------------------------------------------------------------------------------------------
// The step's finalize arithmetic (ncagraph.py:153-166: GroupNorm, tanh * update_gain, residual,
// post-update alpha gate), shared by K2 and the fold K1 (gnca_k1_split<..., FOLD>) so that both
// produce the same bits.
// ------------------------------------------------------------------------------------------
constexpr float kL2E2 = 2.8853900817779268f;   // 2 / ln 2

// per-sample mean / rstd of GroupNorm(1, C) from the fixed-order fp64 sums (t1 = sum, t2 = sum of
// squares over n = C*H*W values, the zeros of masked cells included)
__device__ __forceinline__ void fin_mu_rs(double t1, double t2, double n, float eps, float* mu, float* rs) {
  const double m = t1 / n;
  double var = t2 / n - m * m;
  if (var < 0.0) var = 0.0;
  *mu = (float)m;
  *rs = (float)(1.0 / sqrt(var + (double)eps));
}

// a non-alpha channel's folded constants: x + tanh(z) * gain = (x + gain) - 2 gain / (2^(z 2 log2 e) + 1)
// with z = GN(d) = d * gamma rs + (beta - mu gamma rs): sc = 2 log2(e) gamma rs, sh = 2 log2(e) (beta - mu gamma rs)
__device__ __forceinline__ void fin_consts(float gam, float bet, float mu, float rs, bool gn, float* sc, float* sh) {
  const float gr = gn ? gam * rs : 1.f;
  *sc = gr * kL2E2;
  *sh = (gn ? fmaf(-mu, gr, bet) : 0.f) * kL2E2;
}

// the update of one non-alpha value: (x + gain) + (-2 gain) / (2^(d sc + sh) + 1), g2 = -2 gain
#ifndef GNCA_K2_ABL
#define GNCA_K2_ABL 0   // timing-only A/B builds (wrong results): 1 = K2's main pass with a clamp for its two
                        // transcendentals, 2 = its main pass a plain copy of x (no dx loads), 4 = K2's alpha
                        // phase with a clamp for tanh (the states stay bounded, the live fraction similar)
#endif
__device__ __forceinline__ float k2_update(float x, float d, float sc, float sh, float gain, float g2) {
  if (GNCA_K2_ABL & 1) return fmaf(g2, __builtin_amdgcn_fmed3f(fmaf(d, sc, sh), 0.f, 1.f), x + gain);
  return fmaf(g2, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(fmaf(d, sc, sh)) + 1.f), x + gain);
}

// the updated alpha x~_3 = x_3 + tanh(GN(d)) * gain (as the backward's BA: the same gate bits)
__device__ __forceinline__ float fin_alpha(float xa, float d, float mu, float rs, float g3, float b3, float gain,
                                           bool gn) {
  if (gn) d = (d - mu) * rs * g3 + b3;
  return xa + fast_tanh(d) * gain;
}


}  // namespace gnca

#include "gnca_k1_split.h"
#include "gnca_k1_split32.h"


namespace gnca {

// K1.  Template geometry (TH_, TW_, RY_, RX_) and the gather width KU_ are compile-time in the
// specialised instantiations (every LDS offset becomes an instruction immediate); 0 = runtime.
// fp32 MFMA shares the SIMD's fp32 datapath with VALU on gfx950 (profiles/r01_ubench_*), so the
// body is written to minimise VALU instructions per 16-cell group.
template <int CP, int HDP, int TH_, int TW_, int RY_, int RX_, int KU_, int NT = kThreads>
__global__ __launch_bounds__(NT, 512 / NT) void gnca_k1_update(const K1Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  wg_stamp(a.stamps, 0);
  constexpr int CPQ = CP / 4, KS = 3 * CPQ, MT = HDP / 16, MO = (CP + 15) / 16;
  constexpr int KSP = ((((KS + 3) & ~3) >> 2) & 1) ? ((KS + 3) & ~3) : ((KS + 3) & ~3) + 4;
  constexpr int S2r = 4 * MT;
  constexpr int S2 = ((S2r >> 2) & 1) ? S2r : S2r + 4;
  constexpr int SWMr = (CPQ + 3) & ~3;
  constexpr int SWM = ((SWMr >> 2) & 1) ? SWMr : SWMr + 4;
  constexpr int NW = NT / 64;
  constexpr bool W1REG = w1_in_regs(CP, HDP);
  constexpr bool W2REG = false;   // W2 fragments are read from LDS right before GEMM2
  constexpr bool FIXED = TH_ > 0;
  // compile-time region geometry of the fixed instantiations
  constexpr int cRH = TH_ + 2 * RY_, cRW = TW_ + 2 * RX_;
  constexpr int cNI = (cRH * cRW + 63) / 64, cPSTR = k1_pstr(cRH, cRW, RX_, TW_);
  // 16-byte LDS-DMA (global_load_lds_dwordx4): region rows of whole, aligned float quads
  constexpr bool DMA4 = FIXED && (cRW % 4) == 0 && (RX_ % 4) == 0 && (TW_ % 4) == 0;
  constexpr int cNQ = cRH * cRW / 4, cNI4 = (cNQ + 63) / 64;
  constexpr int cALW = cRW + 2, cNIA = ((cRH + 2) * cALW + 63) / 64;
  constexpr int cGPW = (TH_ * TW_ / 16 + NW - 1) / NW;   // groups per wave per tile (fixed geometry)
  static_assert(!FIXED || (TH_ * TW_) % 16 == 0, "fixed tiles hold whole 16-cell groups");

  const int TH = FIXED ? TH_ : a.TH, TW = FIXED ? TW_ : a.TW;
  const int RY = FIXED ? RY_ : a.RY, RX = FIXED ? RX_ : a.RX;
  const K1Layout L = k1_layout(CP, HDP, TH, TW, RY, RX, a.k);
  const int RH = FIXED ? cRH : L.RH, RW = FIXED ? cRW : L.RW;
  const int NI = FIXED ? cNI : L.NI, PSTR = FIXED ? cPSTR : L.PSTR;
  const int ALW = FIXED ? cALW : L.ALW, NIA = FIXED ? cNIA : L.NIA;
  float* w1f = smem + L.w1f;
  float* w2f = smem + L.w2f;
  float* wmf = smem + L.wmf;
  float* b1s = smem + L.b1s;
  float* bms = smem + L.bms;
  float* percs = smem + L.percs;
  float* wts = smem + L.wts;
  float* fp = smem + L.kp_;      // per-tile keep plane (tile cells)
  float* red = smem + L.red;
  float* xs = smem + L.xs;
  float* al = smem + L.al;       // alpha plane with the extra ring
  float* sp = smem + L.sp;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  // fixed instantiations: C == CP, torus staging, no message-only / attention, uniform weights
  const int C = FIXED ? CP : a.C, H = a.H, W = a.W, Hd = a.hidden;
  const int k = FIXED ? KU_ : a.k, kp = (k + 3) & ~3;
  const bool msg_only = FIXED ? false : (a.flags & kMsgOnly) != 0;
  const bool graph_on = FIXED ? (KU_ > 0) : (a.flags & kGraphOn) != 0;
  const bool zp = FIXED ? false : (a.flags & GNCA_ZERO_PAD_SHIFT) != 0;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const bool want_attn = FIXED ? false : (a.flags & GNCA_ATTENTION) != 0;
  const bool uniform_w = FIXED ? true : a.offw == nullptr;
  const bool compact = !msg_only && !want_attn;   // skip cells whose update is masked to zero
  const float thr = a.alpha_thr, gthr = a.graph_alpha_thr;

  // ---- weights -> LDS in MFMA fragment order (once per persistent workgroup).  Every load of
  //      the whole weight set is issued before the first LDS store: one global-load latency for
  //      the prologue, which is most of a small-batch launch. ----
  {
    RegFill<NT, MT * 64 * KSP> fw1;
    RegFill<NT, MO * 64 * S2> fw2;
    RegFill<NT, HDP> fb1;
    RegFill<NT, CP * 36> fpc;
    RegFill<NT, MO * 64 * SWM> fwm;
    RegFill<NT, CP> fbm;
    if (!msg_only && !(GNCA_ABLATE & kAblFill)) {
      fw1.load(tid, [&](int idx) {
        const int s = idx % KSP, ml = idx / KSP, l = ml & 63, m = ml >> 6;
        const int hid = 16 * m + (l & 15), slot = 4 * s + (l >> 4);
        const int f = slot / CP, c = slot - f * CP;
        return (s < KS && hid < Hd && c < C) ? a.w1[(size_t)hid * 3 * C + f * C + c] : 0.f;
      });
      fw2.load(tid, [&](int idx) {
        const int e = idx % S2, ml = idx / S2, l = ml & 63, mo = ml >> 6;
        const int m = e >> 2, r = e & 3;
        const int co = 16 * mo + (l & 15), hid = 16 * m + 4 * (l >> 4) + r;
        return (e < S2r && co < C && hid < Hd) ? a.w2[(size_t)co * Hd + hid] : 0.f;
      });
      fb1.load(tid, [&](int idx) { return idx < Hd ? a.b1[idx] : 0.f; });
      fpc.load(tid, [&](int idx) {
        const int c = idx / 36, e = idx % 36, f = e / 12, tap = e % 12;
        return (c < C && tap < 9) ? a.perc[(3 * c + f) * 9 + tap] : 0.f;
      });
    }
    fwm.load(tid, [&](int idx) {
      const int s = idx % SWM, ml = idx / SWM, l = ml & 63, mo = ml >> 6;
      const int co = 16 * mo + (l & 15), c = 4 * s + (l >> 4);
      return (graph_on && s < CPQ && co < C && c < C) ? a.wm[co * C + c] : 0.f;
    });
    fbm.load(tid, [&](int idx) { return (graph_on && idx < C) ? a.bm[idx] : 0.f; });
    if (!msg_only && !(GNCA_ABLATE & kAblFill)) {
      fw1.store(w1f, tid);
      fw2.store(w2f, tid);
      fb1.store(b1s, tid);
      fpc.store(percs, tid);
    }
    fwm.store(wmf, tid);
    fbm.store(bms, tid);
  }
  __syncthreads();

  // perception weights == the reference's frozen identity/Sobel bank? (one uniform branch)
  bool sobel = false;
  if (!msg_only) {
    int ok = 1;
    for (int idx = tid; idx < C * 27; idx += NT) {
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
  // MFMA A-fragments resident in VGPRs when they fit (C <= 16, hidden <= 128)
  float w1r[W1REG ? MT : 1][W1REG ? KS : 1];
  float w2r[W2REG ? MO : 1][W2REG ? 4 * MT : 1];
  float wmr[MO][CPQ];
  float bmr[MO][4];
  float gainr[MO];
  if (!msg_only) {
    if constexpr (W1REG) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int s0 = 0; s0 < KS; ++s0) w1r[m][s0] = w1f[(m * 64 + lane) * KSP + s0];
    }
    if constexpr (W2REG) {
#pragma unroll
      for (int mo = 0; mo < MO; ++mo)
#pragma unroll
        for (int e = 0; e < 4 * MT; ++e) w2r[mo][e] = w2f[(mo * 64 + lane) * S2 + e];
    }
  }
#pragma unroll
  for (int mo = 0; mo < MO; ++mo) {
#pragma unroll
    for (int s = 0; s < CPQ; ++s) wmr[mo][s] = wmf[(mo * 64 + lane) * SWM + s];
#pragma unroll
    for (int r = 0; r < 4; ++r) bmr[mo][r] = bms[16 * mo + 4 * g + r];
    // hidden_only: message channels 0..3 (mo 0, lane group 0) get gain 0 (ncagraph.py:98-100)
    gainr[mo] = (graph_on && !(hidden_only && mo == 0 && g == 0)) ? a.message_gain : 0.f;
  }

  const int ncell = TH * TW, ngroups = (ncell + 15) >> 4;
  const size_t HW = (size_t)H * W;

  // XCD-aware tile order (speed only, never correctness): workgroups b and b+8 share an XCD
  // under round-robin dispatch, so XCD group x = b % 8 sweeps its own contiguous range of tiles
  // with its workgroups side by side: neighbouring tiles' halo re-reads hit that XCD's L2.
  const int nxcd = gridDim.x >= 8 ? 8 : 1;
  const int xg_ = blockIdx.x % nxcd, xr_ = blockIdx.x / nxcd;
  const int per_x = (int)(gridDim.x / nxcd) + ((int)(gridDim.x % nxcd) > xg_ ? 1 : 0);
  const int tq = a.total_tiles / nxcd, trm = a.total_tiles % nxcd;
  const int t_begin = xg_ * tq + min(xg_, trm), t_end = t_begin + tq + (xg_ < trm ? 1 : 0);
  PROF_DECL
  for (int tile = t_begin + xr_; tile < ((GNCA_ABLATE & kAblTiles) ? t_begin : t_end); tile += per_x) {
    PROF_MARK(7);   // loop back-edge / tail of the previous tile
    const int b = tile / a.tps, tin = tile - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const float* xb = a.x + (size_t)b * C * HW;
    if (a.active && !a.active[b]) {   // inactive sample (masked step): nothing to update
      if (tid < 2 * NW && !msg_only) a.stats[(size_t)tile * 2 * NW + tid] = 0.0;
      continue;
    }
    __syncthreads();  // previous tile's LDS readers are done (and the fragment staging area)

    // ---- LDS-DMA staging: the (RH x RW) region of every channel, then the alpha plane with one
    //      more ring; torus-wrapped, or a zero source outside the image in pad mode.  No VGPR
    //      round trip; every load of the tile in flight at once. ----
    if (!(GNCA_ABLATE & kAblStage)) {
      if constexpr (DMA4) {
        // channel planes by 16-byte DMA: lane quad q = 4 consecutive floats of one region row
        // (rows hold whole quads; torus wrap keeps a quad contiguous since W % 4 == 0)
#pragma unroll 1
        for (int ii_ = wave; ii_ < cNI4; ii_ += NW) {
          const int q = 64 * ii_ + lane;
          int off = 0;
          bool ok = false;
          if (q < cNQ) {
            const int e = 4 * q;
            const int vr = e / cRW, vc = e - (e / cRW) * cRW;
            int ii = i0 - RY + vr, jj = j0 - RX + vc;
            while (ii < 0) ii += H; while (ii >= H) ii -= H;
            while (jj < 0) jj += W; while (jj >= W) jj -= W;
            off = ii * W + jj;
            ok = true;
          }
          float* dst = xs + 256 * ii_;
#pragma unroll 4
          for (int c = 0; c < CP; ++c) {
            const float* src = ok ? xb + (size_t)c * HW + off : g_zero;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(dst + c * PSTR),
                                             16, 0, 0);
          }
        }
      } else {
      // channel planes: element e of the (RH x RW) region -> image (i0-RY+vr, j0-RX+vc)
#pragma unroll 1
      for (int ii_ = wave; ii_ < NI; ii_ += NW) {
        const int e = 64 * ii_ + lane;
        int off = 0;          // lanes past the region fill the plane's pad from a valid address
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
#pragma unroll 4
        for (int c = 0; c < CP; ++c) {
          const float* src = xb + (size_t)min(c, C - 1) * HW + off;
          if ((zp && !ok) || c >= C) src = g_zero;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)(dst + c * PSTR),
                                           4, 0, 0);
        }
      }
      }
      if (DMA4 && a.alive) {
        // the previous K2's alive bytes over the region (the post-update mask of step
        // t is the pre-update mask of step t+1): one dword = 4 columns (W % 4 == 0, quad-aligned
        // region), RH x RW/4 dwords instead of the (RH+2) x (RW+2) alpha plane
        const uint8_t* ab = a.alive + (size_t)b * HW;
        constexpr int QW = cRW / 4, NQA = cRH * QW, NIQ = (NQA + 63) / 64;
#pragma unroll 1
        for (int ii_ = wave; ii_ < NIQ; ii_ += NW) {
          const int e = 64 * ii_ + lane;
          int off = 0;
          if (e < NQA) {
            const int vr = e / QW, vc = 4 * (e - (e / QW) * QW);
            int ii = i0 - RY + vr, jj = j0 - RX + vc;
            ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
            jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
            off = ii * W + jj;
          }
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ab + off),
                                           (__attribute__((address_space(3))) void*)(al + 64 * ii_), 4, 0, 0);
        }
      } else {
      // alpha plane with one more ring: element e of ((RH+2) x ALW) -> (i0-RY-1+vr, j0-RX-1+vc)
#pragma unroll 1
      for (int ii_ = wave; ii_ < NIA; ii_ += NW) {
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
        const float* src = xb + 3 * HW + off;
        if (zp && !ok) src = g_zero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(al + 64 * ii_),
                                         4, 0, 0);
      }
      }
    }
    PROF_MARK(0);   // DMA issue
    // ---- per-tile side tables while the DMA is in flight: offset weights, fire plane ----
    if (graph_on && !uniform_w)
      for (int o = tid; o < kp; o += NT)
        wts[o] = o >= k ? 0.f : a.offw[(size_t)b * k + o];
#pragma unroll 1
    for (int n = tid; n < ncell; n += NT) {
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const int i = min(i0 + ti, H - 1), j = min(j0 + tj, W - 1);
      const size_t cell = (size_t)i * W + j;
      bool fire = true;
      if (a.fire_mode == GNCA_FIRE_RAND_F32)
        fire = reinterpret_cast<const float*>(a.fire)[(size_t)b * HW + cell] <= a.fire_rate;
      else if (a.fire_mode == GNCA_FIRE_MASK_U8)
        fire = reinterpret_cast<const uint8_t*>(a.fire)[(size_t)b * HW + cell] != 0;
      else if (a.fire_mode == GNCA_FIRE_HASH)
        fire = (GNCA_ABLATE & kAblFire) ? ((cell & 1) != 0)
                                        : hash_uniform(a.seed, a.rng_step, (uint64_t)(a.sample_base + b), cell) <= a.fire_rate;
      fp[n] = fire ? 1.f : 0.f;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    PROF_MARK(1);   // fire plane + DMA wait + barrier
    // ---- alive masks (max_pool 3x3 > thr, image-bounded, ncagraph.py:85-92): the sender plane
    //      (alive_to_alive ? A_graph : 1, zero where the source is off-image) over the region, and
    //      keep = pre-update alive AND fire for the tile cells ----
    if (DMA4 && a.alive) {
      const uint8_t* alb = reinterpret_cast<const uint8_t*>(al);   // region bytes, row-major
#pragma unroll 1
      for (int pos = tid; pos < ((GNCA_ABLATE & kAblPlanes) ? 0 : RH * RW); pos += NT) {
        const int vr = pos / RW, vc = pos - (pos / RW) * RW;
        const int v = alb[pos];
        sp[pos] = a2a ? (float)((v >> 1) & 1) : 1.f;
        const int ti = vr - RY, tj = vc - RX;
        if (ti >= 0 && ti < TH && tj >= 0 && tj < TW) {
          const int n = ti * TW + tj;
          fp[n] = (v & 1) ? fp[n] : 0.f;
        }
      }
    } else
#pragma unroll 1
    for (int pos = tid; pos < ((GNCA_ABLATE & kAblPlanes) ? 0 : RH * RW); pos += NT) {
      const int vr = pos / RW, vc = pos - (pos / RW) * RW;
      int iq = i0 - RY + vr, jq = j0 - RX + vc;
      bool in_img = true;
      if (zp) in_img = iq >= 0 && iq < H && jq >= 0 && jq < W;
      else {
        while (iq < 0) iq += H; while (iq >= H) iq -= H;
        while (jq < 0) jq += W; while (jq >= W) jq -= W;
      }
      const float* q = al + (vr + 1) * ALW + (vc + 1);
      const float NEG = -INFINITY;
      const bool up = iq > 0, dn = iq < H - 1, lf = jq > 0, rt = jq < W - 1;
      const float u0 = q[-ALW - 1], u1 = q[-ALW], u2 = q[-ALW + 1];
      const float m0 = q[-1], m1 = q[0], m2 = q[1];
      const float d0 = q[ALW - 1], d1 = q[ALW], d2 = q[ALW + 1];
      const float mu_ = fmaxf(fmaxf(lf ? u0 : NEG, u1), rt ? u2 : NEG);
      const float mm_ = fmaxf(fmaxf(lf ? m0 : NEG, m1), rt ? m2 : NEG);
      const float md_ = fmaxf(fmaxf(lf ? d0 : NEG, d1), rt ? d2 : NEG);
      const float mx = fmaxf(fmaxf(up ? mu_ : NEG, mm_), dn ? md_ : NEG);
      const float As = (in_img && mx > gthr) ? 1.f : 0.f;
      sp[pos] = a2a ? As : (in_img ? 1.f : 0.f);
      const int ti = vr - RY, tj = vc - RX;
      if (ti >= 0 && ti < TH && tj >= 0 && tj < TW) {
        const int n = ti * TW + tj;
        fp[n] = (in_img && mx > thr) ? fp[n] : 0.f;
      }
    }
    __syncthreads();

    float s1 = 0.f, s2 = 0.f;   // per-lane fp32 partials of this tile (<= a few dozen values)
    float amin = INFINITY, amax = -INFINITY;
    const size_t cell0 = (size_t)i0 * W + j0;

    // ---- live-cell compaction.  keep = pre-alive AND fire; a cell with keep == 0 has dx = 0
    //      exactly (the reference multiplies its update by the masks, ncagraph.py:144-150), so
    //      its MLP / message work is skipped and its zeros are stored here.  The live cells are
    //      listed in cell order (wave ballots, fixed order: deterministic) and packed 16 per MFMA
    //      group.  Off for the message-only and attention calls, which need every cell. ----
    PROF_MARK(2);   // planes + barrier
    int* lst = reinterpret_cast<int*>(smem + L.lst);
    int* wcnt = lst + r4(TH * TW);
    int nlive = 0;
    if (compact) {
      for (int n0 = 0; n0 < ncell; n0 += NT) {
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
        if (live) {
          lst[off + pre] = n;
        } else if (inb) {
          float* oz = a.out + (size_t)b * C * HW + cell0 + (size_t)ti * W + tj;
          if (!(GNCA_ABLATE & kAblZero))
            for (int c = 0; c < C; ++c) oz[(size_t)c * HW] = 0.f;
        }
        nlive += tot;
        __syncthreads();   // wcnt is rewritten by the next pass
      }
    }

    PROF_MARK(3);   // compaction
    const int qend = compact ? (nlive + 15) >> 4 : (FIXED ? cGPW * NW : ngroups);
#pragma unroll 1
    for (int q = wave; q < qend; q += NW) {
      int n = 16 * q + c16;
      bool valid = true;
      if (compact) {
        valid = n < nlive;
        n = lst[valid ? n : 0];
      }
      int ti = n / TW, tj = n - (n / TW) * TW;
      if (!FIXED && !compact) {
        valid = n < ncell && i0 + ti < H && j0 + tj < W;
        if (!valid) { ti = 0; tj = 0; }
      }
      const int pidx = (RY + ti) * RW + (RX + tj);   // cell in the staged region
      const int relcell = ti * W + tj;                       // cell - cell0 in the image
      const float* xg = xs + g * PSTR;                       // this lane's channel group

      // -- graph gather of alive-masked x (linear message: W_M applied after the sum) --
      float gv[CPQ];
#pragma unroll
      for (int t = 0; t < CPQ; ++t) gv[t] = 0.f;
      float S = 0.f;
      if (graph_on && !(GNCA_ABLATE & kAblGather)) {
        if constexpr (KU_ > 0) {
          // compile-time width, uniform weight 1/k applied once after the sum (exact for k=8)
          const float* spq = sp + pidx;
          const float* xq = xg + pidx;
#pragma unroll
          for (int o = 0; o < KU_; ++o) {
            const int d = a.odl[o];
            const float s_ = spq[-d];
            S += s_;
            const float* xo = xq - d;
#pragma unroll
            for (int t = 0; t < CPQ; ++t) gv[t] = fmaf(s_, xo[4 * t * PSTR], gv[t]);
          }
          const float wu = a.uniform_w;
#pragma unroll
          for (int t = 0; t < CPQ; ++t) gv[t] *= wu;
          S *= wu;
        } else {
          for (int o = 0; o < k; ++o) {
            const int qb = pidx - a.odl[o];
            const float wsp = (uniform_w ? a.uniform_w : wts[o]) * sp[qb];
            S += wsp;
#pragma unroll
            for (int t = 0; t < CPQ; ++t) gv[t] = fmaf(wsp, xg[qb + 4 * t * PSTR], gv[t]);
          }
        }
      }
      f4 accm[MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) accm[mo] = f4{0.f, 0.f, 0.f, 0.f};
      // phase fences: keep the scheduler from hoisting every phase's LDS loads to the top of the
      // group (that costs ~100 VGPRs and spills)
      __builtin_amdgcn_sched_barrier(0);
      if (graph_on) {
#pragma unroll
        for (int s = 0; s < CPQ; ++s)
#pragma unroll
          for (int mo = 0; mo < MO; ++mo)
            accm[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(wmr[mo][s], gv[s], accm[mo], 0, 0, 0);
      }

      // -- attention map: sum_o w_o/C * sum_c |A(q) (W_M x(q) + b_M)_c|  (graph_aug.py:160-162) --
      if (want_attn && graph_on) {
        float att = 0.f;
        for (int o = 0; o < k; ++o) {
          const int qb = pidx - a.odl[o];
          f4 tmp[MO];
#pragma unroll
          for (int mo = 0; mo < MO; ++mo) tmp[mo] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < CPQ; ++s)
#pragma unroll
            for (int mo = 0; mo < MO; ++mo)
              tmp[mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(wmr[mo][s], xg[qb + 4 * s * PSTR],
                                                             tmp[mo], 0, 0, 0);
          float part = 0.f;
#pragma unroll
          for (int mo = 0; mo < MO; ++mo)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int c = 16 * mo + 4 * g + r;
              if (c < C) part += fabsf(tmp[mo][r] + bmr[mo][r]);
            }
          part += __shfl_xor(part, 16);
          part += __shfl_xor(part, 32);
          att += (uniform_w ? a.uniform_w : wts[o]) * sp[qb] / (float)C * part;
        }
        if (valid) {
          if (g == 0) a.attn[(size_t)b * HW + cell0 + relcell] = att;
          amin = fminf(amin, att);
          amax = fmaxf(amax, att);
        }
      }

      if (msg_only) {
        // agg_message = W_M gather + b_M * sum_o w_o A(q_o)  (no policy, no masks)
#pragma unroll
        for (int mo = 0; mo < MO; ++mo)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = 16 * mo + 4 * g + r;
            if (valid && c < C)
              a.out[((size_t)b * C + c) * HW + cell0 + relcell] = fmaf(bmr[mo][r], S, accm[mo][r]);
          }
        continue;
      }

      // -- perception: 3x3 depthwise cross-correlation, zero padding (perception.py:16-25).
      //    Taps are read unconditionally (the region has a >= 1 halo); image-border groups
      //    (one uniform branch) mask the taps that fall outside the image. --
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
      // -- GEMM1: H = W1 . Y + b1 (bias as the accumulator's initial value; k-steps outer,
      //    hidden tiles inner: MT independent chains) --
      f4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = *reinterpret_cast<const f4*>(b1s + 16 * m + 4 * g);
#pragma unroll
      for (int s0 = 0; s0 < KS; s0 += 4) {
        f4 w4[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if constexpr (W1REG) w4[m] = f4{w1r[m][s0], w1r[m][s0 + 1], w1r[m][s0 + 2], w1r[m][s0 + 3]};
          else w4[m] = *reinterpret_cast<const f4*>(w1f + (m * 64 + lane) * KSP + s0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            if (s0 + u >= KS) continue;
            if (GNCA_ABLATE & kAblMfma) { asm volatile("" ::"v"(w4[m][u]), "v"(y[s0 + u])); continue; }
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[m][u], y[s0 + u], acc[m], 0, 0, 0);
          }
      }
      // -- ReLU, GEMM2: DL = W2 . H (accumulator rows are GEMM2's B operand);
      //    two accumulator chains so dependent MFMAs do not serialise --
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[m][r] = relu_nan(acc[m][r]);
      f4 acc2[2][MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) {
        acc2[0][mo] = f4{0.f, 0.f, 0.f, 0.f};
        acc2[1][mo] = f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        f4 w2v[MO];
#pragma unroll
        for (int mo = 0; mo < MO; ++mo)
          w2v[mo] = *reinterpret_cast<const f4*>(w2f + (mo * 64 + lane) * S2 + 4 * m);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int mo = 0; mo < MO; ++mo) {
            float wb;
            if constexpr (W2REG) wb = w2r[mo][4 * m + r];
            else wb = w2v[mo][r];
            if (GNCA_ABLATE & kAblMfma) { asm volatile("" ::"v"(wb), "v"(acc[m][r])); continue; }
            acc2[r & 1][mo] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb, acc[m][r], acc2[r & 1][mo], 0, 0, 0);
          }
        }
      }

      // -- epilogue: dx = (dl + tanh(m)*message_gain) * keep, keep = pre-alive AND fire --
      const float keep = valid ? fp[n] : 0.f;
      float* ob = a.out + ((size_t)b * C + 4 * g) * HW + cell0;
#pragma unroll
      for (int mo = 0; mo < MO; ++mo)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * mo + 4 * g + r;
          float v = acc2[0][mo][r] + acc2[1][mo][r];
          if (graph_on) v = fmaf(fast_tanh(fmaf(bmr[mo][r], S, accm[mo][r])), gainr[mo], v);
          v = keep != 0.f ? v : 0.f;
          if (!valid || c >= C) continue;
          if (GNCA_ABLATE & kAblStore) asm volatile("" ::"v"(v));
          else ob[(16 * mo + r) * HW + relcell] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
    }

    PROF_MARK(4);   // group loop
    // ---- per-(tile, wave) GroupNorm partials: fp64 wave shuffle, no workgroup barrier (K2 and
    //      the backward add the NW pairs of every tile in a fixed order) ----
    if (GNCA_ABLATE & kAblReduce) continue;
    if (!msg_only) {
      double d1 = s1, d2 = s2;
      for (int off = 32; off > 0; off >>= 1) {
        d1 += __shfl_xor(d1, off);
        d2 += __shfl_xor(d2, off);
      }
      if (lane == 0) {
        a.stats[((size_t)tile * NW + wave) * 2 + 0] = d1;
        a.stats[((size_t)tile * NW + wave) * 2 + 1] = d2;
      }
    }
    if (want_attn) {   // attention min / max per tile (runtime-geometry variants only)
      for (int off = 32; off > 0; off >>= 1) {
        amin = fminf(amin, __shfl_xor(amin, off));
        amax = fmaxf(amax, __shfl_xor(amax, off));
      }
      if (lane == 0) {
        red[4 * NW + wave * 2 + 0] = amin;
        red[4 * NW + wave * 2 + 1] = amax;
      }
      __syncthreads();
    }
    if (tid == 0) {
      if (want_attn) {
        float mn = INFINITY, mx = -INFINITY;
        for (int w = 0; w < NW; ++w) {
          mn = fminf(mn, red[4 * NW + w * 2]);
          mx = fmaxf(mx, red[4 * NW + w * 2 + 1]);
        }
        a.attn_mm[(size_t)tile * 2 + 0] = mn;
        a.attn_mm[(size_t)tile * 2 + 1] = mx;
      }
    }
    PROF_MARK(5);   // per-tile reduction
  }
  PROF_STORE;
  GNCA_STAMP_END(a.stamps);
}

// ------------------------------------------------------------------------------------------
// K2: GroupNorm + tanh*gain + residual + post-update alpha gate
// ------------------------------------------------------------------------------------------
struct K2Args {
  const float* x;
  const float* dx;
  float* out;
  const double* stats;   // [B * tps * 2]
  const float* gamma;
  const float* beta;
  float* attn;           // normalise in place if non-null
  const float* attn_mm;  // [B * tps * 2]
  int B, C, H, W, tps, band, nbands;
  int nst;                 // GroupNorm partial pairs per sample (tps x waves per K1 workgroup)
  uint8_t* alive_out;      // [B,H,W] or null: next step's pre-update masks (bit 0: thr, bit 1: gthr)
  float gain, thr, eps, gthr;
  int use_gn;
  const uint8_t* active;   // [B] or null: inactive samples are copied through unchanged
  int zigzag;              // sample order (below)
  // compact update field (K1Args::rmask): null = dense dx; else K1's tile geometry
  const uint64_t* rmask;
  const uint32_t* rpre;
  const float* dxa;        // [B,H,W] alpha-channel update of the live cells (K1Args::dxa)
  int TH, TW, tiles_x;
  uint64_t* stamps;        // measurement only (K1Args::stamps)
  // zero-padded-shift rollouts on the compact field: the new state's per (channel, row) fp64 sums
  // ([B][C][H], canon_row_sums' order) for the next step's K0, or null
  double* rs;
};

// K2's sample for block-row j.  zigzag: K1 sweeps 8 contiguous sample ranges (one per XCD group)
// in ascending order, so the samples it finished last are the top of each range: K2 takes them
// first (their x and dx are the most likely to still be in the Infinity Cache) and writes the
// bottom of each range last, which the next K1 reads first.
__device__ __forceinline__ int k2_sample(int j, int B, int zigzag) {
  if (!zigzag || (B & 7)) return j;
  const int per = B >> 3;
  return (j & 7) * per + (per - 1 - (j >> 3));
}

// One workgroup per (sample, band of rows).  LDS: the updated alpha x~_3 over the band + one
// halo row each side, then the post-update alive mask of the band.  The main pass streams
// (channel, cell-vector) items, V = 4 cells (16-byte loads/stores) when W % 4 == 0.  Every load
// the band needs first (GroupNorm partials, alpha rows, gamma/beta and the first KU main items)
// is issued before the first barrier: a small-batch launch waits out one memory latency, not
// one per phase.

#ifndef GNCA_K2_CU
#define GNCA_K2_CU 2
#endif
#ifndef GNCA_K2_CU_ALONE
#define GNCA_K2_CU_ALONE 2
#endif
#ifndef GNCA_K2_CU_ROWS
#define GNCA_K2_CU_ROWS 1   // the row-sum instance (ROWS below): 1 keeps it at 64 VGPRs (2: 67)
#endif
// CU: channels in flight per thread of the compact field's main pass (below)
// ROWS: the zero-padded-shift rollout's instance that also writes the new state's row sums (K2Args::rs;
// its own instance, launched with one channel in flight: the fused sums' registers would lift the
// plain one above the 64 VGPRs that let two K2 waves share a SIMD with the sub-batch pipeline's K1)
template <int V, bool COMPACT, int CU, bool ROWS>
__device__ __forceinline__ void k2_body(const K2Args& a, float* smem, float* sh_norm) {
  typedef float vf __attribute__((ext_vector_type(V)));
#ifndef GNCA_K2_KU
#define GNCA_K2_KU 2
#endif
  constexpr int KU = GNCA_K2_KU;   // main items per thread in flight (measured alone: 1: 0.184, 2: 0.178, 4: 0.187, 8: 0.207 ms)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bj = blockIdx.x / a.nbands, band = blockIdx.x - bj * a.nbands;
  const int b = k2_sample(bj, a.B, a.zigzag);
  const int C = a.C, H = a.H, W = a.W;
  const int r0 = band * a.band, r1 = min(H, r0 + a.band);
  const int h0 = max(0, r0 - 1), h1 = min(H, r1 + 1);       // alpha rows incl. halo
  const size_t HW = (size_t)H * W;
  const float* xb = a.x + (size_t)b * C * HW;
  const float* db = a.dx + (size_t)b * C * HW;
  float* ob = a.out + (size_t)b * C * HW;
  const bool gn = a.use_gn != 0;
  const size_t base = (size_t)r0 * W;
  const int nb = (r1 - r0) * W;
  const int nv = nb / V, nitems = C * nv;

  float* at = smem;                                  // [(h1-h0) x W] updated alpha
  float* post = smem + (size_t)(a.band + 2) * W;     // [(r1-r0) x W] post-update alive mask
  float* gsh = sh_norm + 4;                          // gamma[C], then beta[C] at +32
  // compact update field (K1's rollout mode): per (band row incl. halo, K1 tile column) the row's
  // live mask, live cells before it in its tile, and the tile; per column its (tile column, column
  // in tile).  dx of a cell = its packed value if live, else 0 (K1 multiplies dead cells by 0); the
  // alpha channel's dx is the [B,H,W] plane a.dxa (live cells written; dead cells masked by the row tables).
  constexpr bool compact = COMPACT;
  const int NCELL = a.TH * a.TW, txn = a.tiles_x;
  uint64_t* tab_m = reinterpret_cast<uint64_t*>(smem + (size_t)(2 * a.band + 2) * W);
  uint32_t* tab_p = reinterpret_cast<uint32_t*>(tab_m + (size_t)(a.band + 2) * txn);
  uint32_t* tab_t = tab_p + (size_t)(a.band + 2) * txn;
  uint32_t* colinfo = tab_t + (size_t)(a.band + 2) * txn;

  // (1) loads: gamma/beta, alpha rows, the first main items (the partials follow below; all in
  //     flight together)
  float gam = 1.f, bet = 0.f;
  if (gn && tid < C) { gam = a.gamma[tid]; bet = a.beta[tid]; }
  const int na = (h1 - h0) * W;
  constexpr int NA = 2;   // alpha elements per thread in flight (band + 2 rows <= 2*256 typical)
  float ax[NA], ad[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int e = tid + u * kThreads;
    if (e < na) {
      const size_t p = 3 * HW + (size_t)h0 * W + e;
      ax[u] = xb[p];
      ad[u] = compact ? a.dxa[(size_t)b * HW + (p - 3 * HW)] : db[p];
    }
  }
  if (compact) {
    const int tr = (h1 - h0) * txn;
    for (int e = tid; e < tr; e += kThreads) {
      const int ii = h0 + e / txn, tx = e - (e / txn) * txn;
      const int ti = ii - (ii / a.TH) * a.TH;
      const uint32_t t = (uint32_t)((size_t)b * a.tps + (size_t)(ii / a.TH) * txn + tx);
      tab_m[e] = a.rmask[(size_t)t * a.TH + ti];
      tab_p[e] = a.rpre[(size_t)t * a.TH + ti];
      tab_t[e] = t;
    }
    for (int j = tid; j < W; j += kThreads) colinfo[j] = ((uint32_t)(j / a.TW) << 16) | (uint32_t)(j % a.TW);
  }
  vf xv[KU], dv[KU];
  auto load_items = [&](int it0, bool lx, bool ld) {   // dense update field
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int it = it0 + u * kThreads;
      if (it < nitems) {
        const int c = it / nv, q = it - c * nv;
        if (c != 3) {
          const size_t p = (size_t)c * HW + base + (size_t)V * q;
          if (lx) xv[u] = *reinterpret_cast<const vf*>(xb + p);
          if (ld) dv[u] = *reinterpret_cast<const vf*>(db + p);
        }
      }
    }
  };
  if (!compact) load_items(tid, true, true);

  // (2) per-sample statistics (wave_sum2: fixed order, bit-reproducible)
  if (wave == 0) {
    float mu = 0.f, rs = 1.f;
    if (gn) {
      double t1, t2;
      wave_sum2(a.stats + (size_t)b * a.nst * 2, a.nst, &t1, &t2);
      fin_mu_rs(t1, t2, (double)C * (double)HW, a.eps, &mu, &rs);
    }
    if (lane == 0) {
      float amn = 0.f, amx = 0.f;
      if (a.attn) {
        amn = INFINITY; amx = -INFINITY;
        for (int t = 0; t < a.tps; ++t) {
          amn = fminf(amn, a.attn_mm[((size_t)b * a.tps + t) * 2]);
          amx = fmaxf(amx, a.attn_mm[((size_t)b * a.tps + t) * 2 + 1]);
        }
      }
      sh_norm[0] = mu; sh_norm[1] = rs; sh_norm[2] = amn; sh_norm[3] = amx;
    }
  }
  if (tid < C) { gsh[tid] = gam; gsh[32 + tid] = bet; }
  __syncthreads();
  const float mu = sh_norm[0], rs = sh_norm[1];
  const float g3 = gn ? gsh[3] : 1.f, b3 = gn ? gsh[32 + 3] : 0.f;
  // the non-alpha channels' update, folded: x + tanh(z) * gain = (x + gain) - 2 gain / (2^(z log2 e * 2) + 1)
  // with z = GN(d) = d * gamma rs + (beta - mu gamma rs); per channel k2s[c] = 2 log2(e) gamma rs,
  // k2s[32 + c] = 2 log2(e) (beta - mu gamma rs) (written here, read after the next barrier)
  float* k2s = sh_norm + 4 + 64;
  if (tid < C) fin_consts(gsh[tid], gsh[32 + tid], mu, rs, gn, &k2s[tid], &k2s[32 + tid]);
  const float g2 = -2.f * a.gain;

  // (3) updated alpha over band + halo, then the post-update alive mask (3x3 max-pool, -inf pad)
  auto alpha_at = [&](float xa, float d) {
    if (GNCA_K2_ABL & 4) return xa + __builtin_amdgcn_fmed3f(gn ? (d - mu) * rs * g3 + b3 : d, -1.f, 1.f) * a.gain;
    return fin_alpha(xa, d, mu, rs, g3, b3, a.gain, gn);
  };
  // compact field: K1 writes the alpha plane for live cells only; a dead cell's update is 0 (its
  // row's live mask, already in LDS for the band rows and the halo rows)
  auto live_at = [&](int e) {
    const int r = e / W, j = e - (e / W) * W;
    const uint32_t ci = colinfo[j];
    return ((tab_m[r * txn + (int)(ci >> 16)] >> (ci & 0xffffu)) & 1ull) != 0;
  };
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int e = tid + u * kThreads;
    if (e < na) at[e] = alpha_at(ax[u], (compact && !live_at(e)) ? 0.f : ad[u]);
  }
  for (int e = tid + NA * kThreads; e < na; e += kThreads) {
    const size_t p = 3 * HW + (size_t)h0 * W + e;
    at[e] = alpha_at(xb[p], compact ? (live_at(e) ? a.dxa[(size_t)b * HW + (p - 3 * HW)] : 0.f) : db[p]);
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
    if (a.alive_out)   // valid as next step's masks for 0 <= thr <= gthr (host checks)
      a.alive_out[(size_t)b * HW + (size_t)r0 * W + e] = (uint8_t)((mx > a.thr ? 1 : 0) | (mx > a.gthr ? 2 : 0));
  }
  __syncthreads();

  // (4) main pass: out = x + tanh(GN(dx))*gain; alpha channel = x~_3 * post
  auto store_items = [&](int it0) {
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int it = it0 + u * kThreads;
      if (it >= nitems) continue;
      const int c = it / nv, q = it - c * nv;
      const size_t p = (size_t)c * HW + base + (size_t)V * q;
      vf v;
      if (c == 3) {
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = at[(r0 - h0) * W + V * q + k] * post[V * q + k];
      } else {
        const float sc = k2s[c], sh = k2s[32 + c];
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = k2_update(xv[u][k], dv[u][k], sc, sh, a.gain, g2);
      }
      *reinterpret_cast<vf*>(ob + p) = v;
    }
  };
  typedef float vfu __attribute__((ext_vector_type(V), aligned(4)));
  if (!compact) {
    store_items(tid);
    for (int it0 = tid + KU * kThreads; it0 < nitems; it0 += KU * kThreads) {
      load_items(it0, true, true);
      store_items(it0);
    }
  } else if constexpr (ROWS) {
    // zero-padded-shift rollouts: the compact pass below with the new state's row sums fused, for
    // the next step's K0 (canon_row_sums' order: vector k of a band row on lane k of a 32-lane
    // half-wave, W / V <= 32, the host checks); the same values and stores as the plain pass
    const int nvr = W / V, nrows = r1 - r0, hw = tid >> 5, k = tid & 31;
    double* rsb = a.rs + (size_t)b * C * H + r0;
    for (int rb = 0; rb < nrows; rb += kThreads / 32) {   // uniform: every lane reaches the shuffles
      const int rr = rb + hw;
      const bool on = rr < nrows && k < nvr;
      const int e = V * (rr * nvr + k), ii = r0 + rr, j = V * k;
      const float* src = a.dx;
      int rk[V];
      size_t p0 = 0;
      if (on) {
        const uint32_t ci = colinfo[j];
        const int te = (ii - h0) * txn + (int)(ci >> 16), tj = (int)(ci & 0xffffu);
        const uint64_t m = tab_m[te];
        const uint32_t bits = (uint32_t)(m >> tj) & ((1u << V) - 1u);
        src = a.dx + (size_t)tab_t[te] * C * NCELL + tab_p[te] + (uint32_t)__popcll(m & ((1ull << tj) - 1ull));
#pragma unroll
        for (int kk = 0; kk < V; ++kk) rk[kk] = ((bits >> kk) & 1u) ? __popc(bits & ((1u << kk) - 1u)) : -1;
        p0 = base + (size_t)e;
      }
      {   // alpha: x~_3 * post (computed above)
        float f[V];
        if (on) {
          vf v;
#pragma unroll
          for (int kk = 0; kk < V; ++kk) v[kk] = f[kk] = at[(r0 - h0) * W + e + kk] * post[e + kk];
          *reinterpret_cast<vf*>(ob + 3 * HW + p0) = v;
        }
        const double S = canon_butterfly32(on ? canon_vec_sum<V>(f) : 0.0);
        if (k == 0 && rr < nrows) rsb[(size_t)3 * H + rr] = S;
      }
      for (int c0 = 0; c0 < C; c0 += CU) {
        vf xq[CU], fq[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int c = c0 + u;
          if (c >= C || c == 3 || !on) continue;
          xq[u] = *reinterpret_cast<const vf*>(xb + (size_t)c * HW + p0);
          fq[u] = *reinterpret_cast<const vfu*>(src + (size_t)c * NCELL);
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int c = c0 + u;
          if (c >= C || c == 3) continue;
          float f[V];
          if (on) {
            const float sc = k2s[c], sh = k2s[32 + c];
            vf v;
#pragma unroll
            for (int kk = 0; kk < V; ++kk) {
              float d = 0.f;
#pragma unroll
              for (int r = 0; r <= kk; ++r) d = rk[kk] == r ? fq[u][r] : d;
              v[kk] = f[kk] = k2_update(xq[u][kk], d, sc, sh, a.gain, g2);
            }
            *reinterpret_cast<vf*>(ob + (size_t)c * HW + p0) = v;
          }
          const double S = canon_butterfly32(on ? canon_vec_sum<V>(f) : 0.0);
          if (k == 0 && rr < nrows) rsb[(size_t)c * H + rr] = S;
        }
      }
    }
  } else {
    // compact: one thread per cell vector, all channels; the vector's packed-field position and
    // live ranks are found once (they are the same in every channel plane)
    for (int q = tid; q < nv; q += kThreads) {
      const int e = V * q, ii = r0 + e / W, j = e - (e / W) * W;
      const uint32_t ci = colinfo[j];
      const int te = (ii - h0) * txn + (int)(ci >> 16), tj = (int)(ci & 0xffffu);
      const uint64_t m = tab_m[te];
      const uint32_t bits = (uint32_t)(m >> tj) & ((1u << V) - 1u);
      const int cnt = __popc(bits);
      const float* src = a.dx + (size_t)tab_t[te] * C * NCELL + tab_p[te] +
                         (uint32_t)__popcll(m & ((1ull << tj) - 1ull));
      int rk[V];
#pragma unroll
      for (int k = 0; k < V; ++k) rk[k] = ((bits >> k) & 1u) ? __popc(bits & ((1u << k) - 1u)) : -1;
      const size_t p0 = base + (size_t)e;
      {   // alpha: x~_3 * post (computed above)
        vf v;
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = at[(r0 - h0) * W + e + k] * post[e + k];
        *reinterpret_cast<vf*>(ob + 3 * HW + p0) = v;
      }
      // the packed values of the vector's live cells are contiguous: one (dword-aligned) vector load
      // per channel, placed by rank with lane masks that are the same in every channel (reading up
      // to V-1 floats past the live ones stays inside the workspace: the dx field is followed by
      // the GroupNorm partials)
      typedef float vfu __attribute__((ext_vector_type(V), aligned(4)));
      // channels in flight per thread: beside the other sub-batch's K1 (the sub-batch pipeline) 2
      // (GNCA_K2_CU: 64 VGPRs, so two K2 waves fit on a SIMD beside the 190-VGPR K1; headline step
      // 0.5013 -> 0.4988 ms, c5 0.6495 -> 0.6478, interleaved A/B against 5 and 3:
      // profiles/r04_ab_k2_channels.txt); alone on the chip (one-stream rollouts such as C4's 128-sample
      // shard, the fold's last K2) also 2 (GNCA_K2_CU_ALONE, an A/B knob: round 5, interleaved, 5 vs 2 at
      // C4's shard B=128 72^2 0.0832 vs 0.0822 ms/step, c5 0.654 vs 0.653; profiles/r05f_ab_k2_alone.txt)
      for (int c0 = 0; c0 < C; c0 += CU) {
        vf xq[CU], fq[CU];
        if (GNCA_K2_ABL & 2) {   // timing only: a copy of x
#pragma unroll
          for (int u = 0; u < CU; ++u)
            if (c0 + u < C && c0 + u != 3)
              *reinterpret_cast<vf*>(ob + (size_t)(c0 + u) * HW + p0) = *reinterpret_cast<const vf*>(xb + (size_t)(c0 + u) * HW + p0);
          continue;
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int c = c0 + u;
          if (c >= C || c == 3) continue;
          xq[u] = *reinterpret_cast<const vf*>(xb + (size_t)c * HW + p0);
          fq[u] = *reinterpret_cast<const vfu*>(src + (size_t)c * NCELL);
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int c = c0 + u;
          if (c >= C || c == 3) continue;
          const float sc = k2s[c], sh = k2s[32 + c];
          vf v;
#pragma unroll
          for (int k = 0; k < V; ++k) {
            float d = 0.f;
#pragma unroll
            for (int r = 0; r <= k; ++r) d = rk[k] == r ? fq[u][r] : d;
            v[k] = k2_update(xq[u][k], d, sc, sh, a.gain, g2);
          }
          *reinterpret_cast<vf*>(ob + (size_t)c * HW + p0) = v;
        }
      }
    }
  }
  if (a.attn) {
    const float amn = sh_norm[2], amx = sh_norm[3];
    for (int e = tid; e < nb; e += kThreads) {
      float* q = a.attn + (size_t)b * HW + base + e;
      *q = (*q - amn) / (amx - amn + 1e-8f);
    }
  }
}

// one instantiation per (cell-vector width, update-field layout): each gets its own registers
// (compact: 64 VGPRs with 2 channels in flight; round 3's 5 took 75 and a cap at 64 spilled)
#ifdef GNCA_K2_MAXV   // A/B builds: a minimum of waves per SIMD (a VGPR cap), so that more K2 waves fit beside a K1
#define GNCA_K2_ATTR __attribute__((amdgpu_waves_per_eu(GNCA_K2_MAXV)))
#elif defined(GNCA_K2_NUMV)   // A/B builds: a VGPR cap of 2 x GNCA_K2_NUMV (gfx950 doubles amdgpu_num_vgpr: VGPRs + AGPRs)
#define GNCA_K2_ATTR __attribute__((amdgpu_num_vgpr(GNCA_K2_NUMV)))
#else
#define GNCA_K2_ATTR
#endif
#ifndef GNCA_K2_PRIO
#define GNCA_K2_PRIO 3
#endif
template <int V, bool COMPACT, int CU = GNCA_K2_CU, bool ROWS = false>
__global__ __launch_bounds__(kThreads) GNCA_K2_ATTR void gnca_k2_finalize(const K2Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float sh_norm[4 + 64 + 64];
  const int tid = threadIdx.x;
  wg_stamp(a.stamps, 0);
  const int bj = blockIdx.x / a.nbands, band = blockIdx.x - bj * a.nbands;
  const int b = k2_sample(bj, a.B, a.zigzag);
  if (a.active && !a.active[b]) {   // masked step: an inactive sample passes through unchanged
    const size_t HW = (size_t)a.H * a.W;
    const int r0 = band * a.band, r1 = min(a.H, r0 + a.band);
    const float* xs_ = a.x + (size_t)b * a.C * HW;
    float* os_ = a.out + (size_t)b * a.C * HW;
    const int nbc = (r1 - r0) * a.W;
    for (int it = tid; it < a.C * nbc; it += kThreads) {
      const int c = it / nbc, e = it - c * nbc;
      os_[(size_t)c * HW + (size_t)r0 * a.W + e] = xs_[(size_t)c * HW + (size_t)r0 * a.W + e];
    }
    GNCA_STAMP_END(a.stamps);
    return;
  }
  // K2's waves issue ahead of the co-resident K1's (the sub-batch pipeline, GNCA_K1_PRIO = 2): K2 is
  // memory-bound, so it issues its loads at once and then waits, and K1 has the SIMD meanwhile;
  // below K1 it was starved of issue slots and held its CU share longer (headline step 0.512 ->
  // 0.495 ms, profiles/r04_ab_k2_priority.txt)
  __builtin_amdgcn_s_setprio(GNCA_K2_PRIO);
  k2_body<V, COMPACT, CU, ROWS>(a, smem, sh_norm);
  GNCA_STAMP_END(a.stamps);
}

// This step's pre-update masks as bytes for the split K1 when no previous K2 handed them over
// (single steps, the first step of a rollout): bit 0 = maxpool3(alpha) > alpha_thr, bit 1 =
// > graph_alpha_thr (ncagraph.py:85-92: -inf padding, no wrap), the bytes K2 writes in a rollout.
template <int V>
__global__ __launch_bounds__(kThreads) void gnca_k_alive(const float* x, uint8_t* out, int B, int C, int H, int W,
                                                         float thr, float gthr) {
  // samples on blockIdx.y, V consecutive cells of a row per thread (V = 4: float4 row loads, one
  // 4-byte store); the 3x3 window clamped at the image edge (a duplicate of an in-window value: the
  // same max as the -inf border), so that every load is independent and in flight together (a row
  // loop with runtime bounds paid three dependent round trips: 24 us for 2.7 M cells)
  typedef float fv __attribute__((ext_vector_type(V)));
  const int HW = H * W, WV = W / V, nv = H * WV;
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const float* al = x + ((size_t)b * C + 3) * HW;
    uint8_t* ob = out + (size_t)b * HW;
    for (int e = blockIdx.x * kThreads + threadIdx.x; e < nv; e += gridDim.x * kThreads) {
      const int r = e / WV, c0 = V * (e - r * WV);
      const int rows[3] = {(r > 0 ? r - 1 : r) * W, r * W, (r < H - 1 ? r + 1 : r) * W};
      const int cl = c0 > 0 ? c0 - 1 : c0, cr = c0 + V < W ? c0 + V : c0 + V - 1;
      fv m;
      float ml = -INFINITY, mr = -INFINITY;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const fv v = *reinterpret_cast<const fv*>(al + rows[k] + c0);
        m = k == 0 ? v : __builtin_elementwise_max(m, v);
        ml = fmaxf(ml, al[rows[k] + cl]);
        mr = fmaxf(mr, al[rows[k] + cr]);
      }
      // column maxima m[j] of the window's 3 rows; the horizontal 3-max over columns c0-1 .. c0+V
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float left = j == 0 ? ml : m[j - 1], right = j == V - 1 ? mr : m[j + 1];
        const float mx = fmaxf(fmaxf(left, m[j]), right);
        bits |= (uint32_t)((mx > thr ? 1 : 0) | (mx > gthr ? 2 : 0)) << (8 * j);
      }
      if (V == 4) *reinterpret_cast<uint32_t*>(ob + r * W + c0) = bits;
      else ob[r * W + c0] = (uint8_t)bits;
    }
  }
}

// normalise a message-only attention map (no K2 in message mode)
__global__ __launch_bounds__(kThreads) void gnca_attn_normalize(float* attn, const float* attn_mm,
                                                                int tps, int HW) {
  const int b = blockIdx.y;
  __shared__ float mm[2];
  if (threadIdx.x == 0) {
    float mn = INFINITY, mx = -INFINITY;
    for (int t = 0; t < tps; ++t) {
      mn = fminf(mn, attn_mm[((size_t)b * tps + t) * 2]);
      mx = fmaxf(mx, attn_mm[((size_t)b * tps + t) * 2 + 1]);
    }
    mm[0] = mn; mm[1] = mx;
  }
  __syncthreads();
  for (int p = blockIdx.x * kThreads + threadIdx.x; p < HW; p += gridDim.x * kThreads) {
    float* q = attn + (size_t)b * HW + p;
    *q = (*q - mm[0]) / (mm[1] - mm[0] + 1e-8f);
  }
}

// ------------------------------------------------------------------------------------------
// K0: zero-pad offset weights.  logit_o = qbar . kbar_o with
//   qbar   = W_Q xbar + b_Q                              (mean of Q over the image)
//   kbar_o = (W_K S_o + b_K * n_o W) / (H W)             (mean of the row-shifted, zero-padded K)
// where S_o sums the per-row channel sums of x over the rows that stay inside the image and n_o
// counts them; softmax over offsets with temperature |scaling| + 1e-6.  fp64 throughout.
// ------------------------------------------------------------------------------------------
struct K0Args {
  const float* x;
  const float* wq;
  const float* bq;
  const float* wk;
  const float* bk;
  const float* scaling;
  float* offw;  // [B * k]
  const double* rs;   // [B][C][H] per-row channel sums (gnca_k0_rowsums)
  int B, C, H, W, d, k;
  int8_t offs[2 * GNCA_MAX_OFFSETS];
};

// K0's first phase: the per-(channel, row) fp64 sums of x in the canonical order (canon_row_sums), one
// workgroup per (sample, channel) so that a small batch still spreads over the chip (one workgroup per
// sample took 57 us for B=16 40^2); a rollout's later steps take them from the previous step's K2.
// Samples on grid x (up to 2^31 - 1), channels on grid y (<= 65535)
template <int V>
__global__ __launch_bounds__(kThreads) void gnca_k0_rowsums(const float* x, double* rs, int C, int H, int W) {
  const int b = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  const size_t HW = (size_t)H * W;
  canon_row_sums<V, 4>(x + ((size_t)b * C + c) * HW, H, W, rs + ((size_t)b * C + c) * H, tid >> 5, kThreads / 32,
                       tid & 31);
}

__global__ __launch_bounds__(kThreads) void gnca_k0_offset_weights(const K0Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = a.C, H = a.H, W = a.W, D = a.d, K = a.k;
  double* rs = reinterpret_cast<double*>(smem);         // [C][H] row sums
  double* xbar = rs + (size_t)C * H;                     // [C]
  double* qbar = xbar + C;                               // [d]
  double* logit = qbar + D;                              // [k]
  double* sco = logit + K;                               // [C][k] sum of a channel's rows an offset keeps
  double* kkb = sco + (size_t)C * K;                     // [k][d] pooled key of each offset
  float* wqs = reinterpret_cast<float*>(kkb + (size_t)K * D);   // [d][C] W_Q, then [d][C] W_K (LDS copies:
  float* wks = wqs + (size_t)D * C;                             //  the dot products' loops read them per c)
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t HW = (size_t)H * W;
  const float* xb = a.x + (size_t)b * C * HW;
  const int lane = tid & 63, wave = tid >> 6;
  // the projection weights and the sample's row sums (gnca_k0_rowsums, one workgroup per (sample,
  // channel) before this launch) to LDS, every load in flight
  (void)xb; (void)lane; (void)wave;
  for (int e = tid; e < D * C; e += kThreads) {
    wqs[e] = a.wq[e];
    wks[e] = a.wk[e];
  }
  for (int e = tid; e < C * H; e += kThreads) rs[e] = a.rs[(size_t)b * C * H + e];
  __syncthreads();
  // channel means; per (channel, offset) the sum of the rows the zero-padded shift keeps
  for (int c = tid; c < C; c += kThreads) {
    double s = 0.0;
    for (int r = 0; r < H; ++r) s += rs[c * H + r];
    xbar[c] = s / (double)HW;
  }
  for (int e = tid; e < C * K; e += kThreads) {
    const int c = e / K, o = e - (e / K) * K;
    const int dy = a.offs[2 * o];
    const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;  // valid source rows [lo,hi)
    double S = 0.0;
    for (int r = lo; r < hi; ++r) S += rs[c * H + r];
    sco[c * K + o] = S;
  }
  __syncthreads();
  for (int e = tid; e < D; e += kThreads) {
    double s = (double)a.bq[e];
    for (int c = 0; c < C; ++c) s += (double)wqs[e * C + c] * xbar[c];
    qbar[e] = s;
  }
  for (int i = tid; i < K * D; i += kThreads) {
    const int o = i / D, e = i - (i / D) * D;
    const int dy = a.offs[2 * o];
    const int lo = dy > 0 ? 0 : -dy, hi = dy > 0 ? H - dy : H;
    const int nrows = hi > lo ? hi - lo : 0;
    double kk = (double)a.bk[e] * (double)nrows * (double)W;
    for (int c = 0; c < C; ++c) kk += (double)wks[e * C + c] * sco[c * K + o];
    kkb[i] = kk;
  }
  __syncthreads();
  for (int o = tid; o < K; o += kThreads) {
    double L = 0.0;
    for (int e = 0; e < D; ++e) L += qbar[e] * (kkb[o * D + e] / (double)HW);
    logit[o] = L;
  }
  __syncthreads();
  if (tid == 0) {
    double mx = -INFINITY;
    for (int o = 0; o < K; ++o) mx = fmax(mx, logit[o]);
    const double T = fabs((double)a.scaling[0]) + 1e-6;
    double sum = 0.0;
    for (int o = 0; o < K; ++o) {
      logit[o] = exp((logit[o] - mx) / T);
      sum += logit[o];
    }
    for (int o = 0; o < K; ++o) a.offw[(size_t)b * K + o] = (float)(logit[o] / sum);
  }
}

// gnca_k0_offset_weights for C = 16, d = 16, k <= 8 (the module's graph defaults): one wave per sample,
// no LDS.  The LDS version (13.6 KB) never fits beside the other sub-batch stream's persistent K1
// (~6.6 KB of a CU's LDS left), so in the zero-pad rollout it waited for that K1 to retire.  Lane l
// holds channel / unit c = l & 15 and offsets p = l >> 4 and p + 4; every sum keeps the LDS
// version's order (row sums in row order, dot products in channel / unit order): the same bits.
__global__ __launch_bounds__(64) void gnca_k0_weights16(const K0Args a) {
  const int b = blockIdx.x, l = threadIdx.x, c = l & 15, p = l >> 4;
  const int H = a.H, W = a.W, K = a.k;
  const double HW = (double)H * (double)W;
  const double* rs = a.rs + ((size_t)b * 16 + c) * H;
  auto rows = [&](int o, int* lo, int* hi) {   // the source rows the zero-padded shift keeps
    const int dy = o < K ? a.offs[2 * o] : 0;
    *lo = dy > 0 ? 0 : -dy;
    *hi = dy > 0 ? H - dy : H;
  };
  int lo0, hi0, lo1, hi1;
  rows(p, &lo0, &hi0);
  rows(p + 4, &lo1, &hi1);
  // every load first (the projection rows of this lane's unit, then the row sums 24 at a time):
  // the kernel is a latency chain between a sub-batch's K2 and its K1 in the zero-pad rollout
  float wqv[16], wkv[16];
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) {
    wqv[cc] = a.wq[c * 16 + cc];
    wkv[cc] = a.wk[c * 16 + cc];
  }
  const float bqv = a.bq[c], bkv = a.bk[c];
  double tot = 0.0, s0 = 0.0, s1 = 0.0;
  constexpr int RB = 24;
  for (int rb = 0; rb < H; rb += RB) {
    double v[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) v[i] = rb + i < H ? rs[rb + i] : 0.0;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = rb + i;
      if (r < H) {
        tot += v[i];
        if (r >= lo0 && r < hi0) s0 += v[i];
        if (r >= lo1 && r < hi1) s1 += v[i];
      }
    }
  }
  const double xbar = tot / HW;
  // qbar[e] (lane e of each 16-lane group): b_Q + W_Q xbar
  double qb = (double)bqv;
  for (int cc = 0; cc < 16; ++cc) qb += (double)wqv[cc] * __shfl(xbar, cc);
  // pooled keys of this group's offsets (unit e = c): b_K * rows * W + W_K sco
  double k0 = (double)bkv * (double)(hi0 > lo0 ? hi0 - lo0 : 0) * (double)W;
  double k1 = (double)bkv * (double)(hi1 > lo1 ? hi1 - lo1 : 0) * (double)W;
  for (int cc = 0; cc < 16; ++cc) {
    const double wk = (double)wkv[cc];
    k0 += wk * __shfl(s0, 16 * p + cc);
    k1 += wk * __shfl(s1, 16 * p + cc);
  }
  // logits of offsets p and p + 4: sum over units e in order (the same expression as the LDS version)
  double L0 = 0.0, L1 = 0.0;
  for (int e = 0; e < 16; ++e) {
    const double q = __shfl(qb, 16 * p + e);
    L0 += q * (__shfl(k0, 16 * p + e) / HW);
    L1 += q * (__shfl(k1, 16 * p + e) / HW);
  }
  // softmax over the k offsets with the temperature |scaling| + 1e-6 (lane 0, in offset order)
  double lg[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) lg[o] = o < 4 ? __shfl(L0, 16 * o) : __shfl(L1, 16 * (o - 4));
  if (l == 0) {
    double mx = -INFINITY;
    for (int o = 0; o < K; ++o) mx = fmax(mx, lg[o]);
    const double T = fabs((double)a.scaling[0]) + 1e-6;
    double sum = 0.0;
    for (int o = 0; o < K; ++o) {
      lg[o] = exp((lg[o] - mx) / T);
      sum += lg[o];
    }
    for (int o = 0; o < K; ++o) a.offw[(size_t)b * K + o] = (float)(lg[o] / sum);
  }
}

// FixedSobelPerception.forward alone: y[:, f*C + c] = sum_ab w[3c+f][a][b] x(i+a-1, j+b-1).
__global__ __launch_bounds__(kThreads) void gnca_perceive(int B, int C, int H, int W,
                                                          const float* w, const float* x, float* y) {
  const size_t HW = (size_t)H * W;
  const size_t total = (size_t)B * C * HW;
  for (size_t idx = (size_t)blockIdx.x * kThreads + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * kThreads) {
    const size_t b = idx / (C * HW), rem = idx - b * C * HW;
    const int c = (int)(rem / HW);
    const size_t cell = rem - (size_t)c * HW;
    const int i = (int)(cell / W), j = (int)(cell - (size_t)i * W);
    const float* xc = x + (b * C + c) * HW;
    float nb[9];
    for (int dv = 0; dv < 3; ++dv)
      for (int du = 0; du < 3; ++du) {
        const int ii = i + dv - 1, jj = j + du - 1;
        nb[dv * 3 + du] = (ii >= 0 && ii < H && jj >= 0 && jj < W) ? xc[(size_t)ii * W + jj] : 0.f;
      }
    for (int f = 0; f < 3; ++f) {
      float acc = 0.f;
      for (int e = 0; e < 9; ++e) acc = fmaf(w[(3 * c + f) * 9 + e], nb[e], acc);
      y[(b * 3 * C + (size_t)f * C + c) * HW + cell] = acc;
    }
  }
}

// The GNCA_FIRE_HASH mask as uint8 (gnca_fire_mask_u8)
__global__ __launch_bounds__(kThreads) void gnca_fire_mask(uint8_t* mask, int B, int HW, uint64_t seed,
                                                           int64_t step, int64_t sample_base, float rate) {
  const size_t total = (size_t)B * HW;
  for (size_t e = (size_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += (size_t)gridDim.x * kThreads) {
    const size_t b = e / HW, cell = e - b * HW;
    mask[e] = hash_uniform(seed, step, (uint64_t)(sample_base + (int64_t)b), cell) <= rate ? 1 : 0;
  }
}

#ifndef GNCA_K1_PROBE   // tools/k1_probe.sh: no host code (no instance table), for register / ISA studies
// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
thread_local int g_last_hip = 0;

struct Variant {
  int CP, HDP, TH, TW, RY, RX, KU;   // TH == 0: runtime geometry (generic)
  const void* fn;
  int NT;                            // threads per workgroup
  int split;                         // 1: gnca_k1_split, 2: gnca_k1_split32 (bf16 MFMA on exact 3-way splits)
  int lds_split;                     // its LDS bytes (compile-time layout)
  const void* fold_fn[2];            // the same K1 that also finishes the previous step (rollouts) on the
                                     // [dense, compact] update field, or null
  int lds_fold;                      // the fold variant's LDS bytes
  const void* fn_zp;                 // the zero-padded-shift instance (graph split K1s), or null
};

template <int TH, int TW, int RY, int RX, int KU>
constexpr const void* ks_zp_fn() {
  if constexpr (KU > 0) return reinterpret_cast<const void*>(&gnca_k1_split<TH, TW, RY, RX, KU, 0, true>);
  else return nullptr;
}

#define GNCA_GV(cp, hd) {cp, hd, 0, 0, 0, 0, 0, reinterpret_cast<const void*>(&gnca_k1_update<cp, hd, 0, 0, 0, 0, 0>), kThreads, 0, 0, {nullptr, nullptr}, 0, nullptr}
#define GNCA_SV(th, tw, ry, rx, ku) \
  {16, 128, th, tw, ry, rx, ku, reinterpret_cast<const void*>(&gnca_k1_split<th, tw, ry, rx, ku>), GNCA_K1_SPLIT_NT, 1, \
   ks_layout<th, tw, ry, rx>().total, {nullptr, nullptr}, 0, ks_zp_fn<th, tw, ry, rx, ku>()}
// fold variants: the large-batch tile (dense: nullptr, it is only planned with the compact field) and
// the small-batch ones (both layouts)
#define GNCA_SVF(th, tw, ry, rx, ku, dense) \
  {16, 128, th, tw, ry, rx, ku, reinterpret_cast<const void*>(&gnca_k1_split<th, tw, ry, rx, ku>), GNCA_K1_SPLIT_NT, 1, \
   ks_layout<th, tw, ry, rx>().total, {dense, reinterpret_cast<const void*>(&gnca_k1_split<th, tw, ry, rx, ku, 2>)}, \
   ks_layout<th, tw, ry, rx, true>().total, ks_zp_fn<th, tw, ry, rx, ku>()}
#define GNCA_S32V(th, tw, ry, rx, ku) \
  {32, 128, th, tw, ry, rx, ku, reinterpret_cast<const void*>(&gnca_k1_split32<th, tw, ry, rx, ku>), 512, 2, \
   ks32_layout<th, tw, ry, rx>().total, {nullptr, nullptr}, 0, nullptr}
static const Variant kVariants[] = {
    // 16 channels, hidden 128, bf16 MFMA on exact 3-way splits (gnca_k1_split.h), compile-time
    // geometry: list order is the large-batch preference (24x36: the largest tiles whose halo fits
    // LDS, 1.6x halo re-read); 8x24 / 8x20 serve small batches and the trainer's 40^2 canvas
    GNCA_SVF(24, 36, 4, 4, 8, nullptr),   // + the fold variant (large-batch rollouts: one K1 launch per step)
    GNCA_SV(36, 24, 4, 4, 8),
    GNCA_SV(24, 24, 4, 4, 8),
    GNCA_SVF(8, 24, 4, 4, 8, reinterpret_cast<const void*>(&gnca_k1_split<8, 24, 4, 4, 8, 1>)),
    // classic NCA steps (and the graph model's message-off steps: the trainers' message_every) at
    // large batches: 24x36 tiles (round 6; before, the 8x24 small-batch tiles served every batch)
    GNCA_SVF(24, 36, 1, 4, 0, nullptr),   // + the compact fold (on request)
    GNCA_SVF(8, 24, 1, 4, 0, reinterpret_cast<const void*>(&gnca_k1_split<8, 24, 1, 4, 0, 1>)),   // classic NCA
                                 // (no gather; RX 4 keeps the staging rows quad-aligned)
    GNCA_SV(8, 20, 4, 4, 8),
    GNCA_SV(8, 20, 1, 4, 0),
    // 32 channels (BASELINE config 5: 128^2, r = 5, K = 16): 16x16 tiles, channel planes staged
    // in two 16-channel phases (gnca_k1_split32.h); graph and no-message steps
    GNCA_S32V(16, 16, 5, 8, 16),   // RX 8 (not 5): quad-aligned 16-byte LDS-DMA rows
    GNCA_S32V(16, 16, 1, 4, 0),
    // runtime geometry: every other shape class
    GNCA_GV(4, 32),   GNCA_GV(4, 64),   GNCA_GV(4, 128),  GNCA_GV(8, 32),   GNCA_GV(8, 64),
    GNCA_GV(8, 128),  GNCA_GV(12, 64),  GNCA_GV(12, 128), GNCA_GV(16, 32),  GNCA_GV(16, 64),
    GNCA_GV(16, 128), GNCA_GV(16, 256), GNCA_GV(20, 128), GNCA_GV(24, 128), GNCA_GV(28, 128),
    GNCA_GV(32, 64),  GNCA_GV(32, 128),
};
#undef GNCA_GV
#undef GNCA_SV
#undef GNCA_SVF
#undef GNCA_S32V

static const Variant* find_variant(int C, int Hd) {
  const int CP = (C + 3) & ~3;
  const Variant* best = nullptr;
  for (const Variant& v : kVariants)
    if (v.TH == 0 && v.CP == CP && v.HDP >= Hd && (!best || v.HDP < best->HDP)) best = &v;
  return best;
}

struct Plan {
  const Variant* var;
  const void* k1fn;   // the K1 launched: var->fn, or var->fn_zp for a zero-padded graph step
  int k, RY, RX, TH, TW, tiles_x, tiles_y, tps, total_tiles;
  int ppt;   // GroupNorm partial pairs per tile: one per K1 wave
  size_t lds1;
  bool graph_on, need_k0;
  // K2
  int band, nbands, total2;
  size_t lds2;
  int band_c, nbands_c, total2_c;   // K2 on the compact update field
  size_t lds2_c;
  // workspace carve (bytes)
  size_t off_dx, off_stats, off_mm, off_offw, off_rs, off_alive, off_rmask, off_rpre, off_dxa, off_wimg, ws_bytes;
  bool compact_ok;   // the rollout's compact update field (the bf16-split K1s, large batches)
  // the fold (rollouts of a fold-capable K1 on the compact field): K1 of step t also finishes step
  // t - 1, so the compact field (dx, row tables, alpha plane, partials) is double-buffered by the
  // parity of the global step index: set 1 at off_*2
  bool fold_ok;    // planned for rollouts by default (the dense field: small batches)
  bool fold_any;   // possible (also on the compact field, on request: GNCA_ROLLOUT_FOLD)
  size_t off_dx2, off_stats2, off_rmask2, off_rpre2, off_dxa2;
};

static int max_lds_bytes() { return 160 * 1024; }

static int device_cus();

static bool make_plan(const gnca_step_desc* d, bool msg_only, Plan* P) {
  if (!d || d->B <= 0 || d->C < 4 || d->H <= 0 || d->W <= 0 || d->hidden <= 0) return false;
  if (d->num_offsets < 0 || d->num_offsets > GNCA_MAX_OFFSETS) return false;
  const bool graph = (d->flags & GNCA_GRAPH) != 0;
  if (graph && d->d_model <= 0) return false;
  P->var = find_variant(d->C, d->hidden);
  if (!P->var) return false;
  P->k = graph ? d->num_offsets : 0;
  const bool attn = graph && (d->flags & GNCA_ATTENTION);
  P->graph_on = graph && P->k > 0 && (msg_only || attn || d->message_gain != 0.f);
  const bool zp = (d->flags & GNCA_ZERO_PAD_SHIFT) != 0;
  P->need_k0 = P->graph_on && zp;
  int ry = 1, rx = 1;
  if (P->graph_on)
    for (int o = 0; o < P->k; ++o) {
      const int dy = d->offsets[2 * o], dx = d->offsets[2 * o + 1];
      ry = ry > abs(dy) ? ry : abs(dy);
      if (!zp) rx = rx > abs(dx) ? rx : abs(dx);
    }
  P->RY = ry;
  P->RX = rx;
  const int CP = P->var->CP, HDP = P->var->HDP;
  const bool attn_on = attn && P->graph_on;
  // a compile-time-geometry instantiation (the bf16-split K1s), when the shape allows one;
  // GNCA_AB_ENV knobs exist only in -DGNCA_AB_KNOBS measurement builds (gnca_device.h):
  // GNCA_K1_TILE=<TH>x<TW> restricts the fixed variants to one tile shape
  static const char* tile_env = GNCA_AB_ENV("GNCA_K1_TILE");
  const Variant* fixed_pick = nullptr;
  long fixed_tiles = 0;
  for (const Variant& v : kVariants) {
    if (v.TH == 0 || v.CP != CP || v.HDP != HDP || d->C != CP || msg_only || attn_on) continue;
    if (tile_env) {
      int th = 0, tw = 0;
      if (sscanf(tile_env, "%dx%d", &th, &tw) == 2 && (th != v.TH || tw != v.TW)) continue;
    }
    if (d->H % v.TH || d->W % v.TW || ry > v.RY || rx > v.RX) continue;
    // (zero-padded graph steps: the variant's ZP instance, fed K0's per-sample offset weights)
    if (v.KU > 0 ? !(P->graph_on && P->k == v.KU && (!zp || v.fn_zp)) : P->graph_on) continue;
    if ((size_t)v.lds_split > (size_t)max_lds_bytes()) continue;
    // list order is the large-batch preference (big tiles amortise the per-tile work); a batch
    // too small to give every CU two workgroups' worth of tiles takes the variant with the most
    // tiles instead (measured at B=8, 72^2: 24x36 55 us/step, 8x24 43 us/step)
    const long tiles = (long)d->B * (d->H / v.TH) * (d->W / v.TW);
    const long fill = 2L * device_cus() * std::max(1, 512 / v.NT);
    if (!fixed_pick) {
      fixed_pick = &v;
      fixed_tiles = tiles;
      if (tiles >= fill) break;   // large batch: first (preferred) eligible variant
    } else if (tiles > fixed_tiles) {
      fixed_pick = &v;
      fixed_tiles = tiles;
    }
  }
  if (fixed_pick) {
    P->var = fixed_pick;
    P->RY = fixed_pick->RY;
    P->RX = fixed_pick->RX;
    ry = fixed_pick->RY;
    rx = fixed_pick->RX;
  }
  // tile choice: fewest padded cells + staged halo, LDS <= 80 KB (2 workgroups / CU) if possible
  static const int ths[] = {4, 8, 12, 16, 24};
  static const int tws[] = {8, 12, 16, 24, 32, 48, 64};
  double best = 1e300;
  int bth = 0, btw = 0;
  size_t blds = 0;
  if (P->var->TH) {
    bth = P->var->TH;
    btw = P->var->TW;
    blds = (size_t)P->var->lds_split;
  }
  for (int pass = 0; pass < 2 && !bth; ++pass) {
    const size_t cap = pass == 0 ? 80 * 1024 : (size_t)max_lds_bytes();
    for (int th : ths)
      for (int tw : tws) {
        if ((th * tw) % 16) continue;
        const K1Layout L = k1_layout(CP, HDP, th, tw, ry, rx, P->k);
        const size_t bytes = (size_t)L.total * 4;
        if (bytes > cap) continue;
        const long tx = (d->W + tw - 1) / tw, ty = (d->H + th - 1) / th;
        const double cells = (double)tx * ty * th * tw;
        const double stage = (double)tx * ty * (th + 2 * ry) * (tw + 2 * rx) * CP;
        const double cost = cells * (msg_only ? 0.1 : 1.0) + 0.004 * stage + 30.0 * tx * ty;
        if (cost < best) { best = cost; bth = th; btw = tw; blds = bytes; }
      }
  }
  P->TH = bth;
  P->TW = btw;
  P->lds1 = blds;
  P->k1fn = (zp && P->graph_on && P->var->fn_zp) ? P->var->fn_zp : P->var->fn;
  P->tiles_x = (d->W + btw - 1) / btw;
  P->tiles_y = (d->H + bth - 1) / bth;
  P->tps = P->tiles_x * P->tiles_y;
  P->total_tiles = P->tps * d->B;
  P->ppt = P->var->NT / 64;
  // K2 bands: ~6 row bands per sample (many small workgroups: no wave-quantisation tail),
  // each with its alpha rows + 2 halo rows and its post mask in LDS (<= 48 KB)
  {
    // bands of ~4 rows (measured on the B=1024 72^2 bench: 4 rows 0.177 ms, 12 rows 0.194 ms,
    // 24 rows 0.209 ms per launch; tools/k2_band_sweep.sh); thinner when the batch is too small
    // to fill the chip
    // (narrow, 16-channel canvases; wide / 32-channel ones keep ~6 bands per sample: 128^2 x 32ch
    // measured 0.164 ms at 22 rows, 0.184 ms at 4)
    const bool thin = (long)d->W * d->C <= 96L * 16;
    const long nb_target = std::max<long>(thin ? (d->H + 3) / 4 : 6, (2L * device_cus() + d->B - 1) / d->B);
    long rows = (d->H + nb_target - 1) / nb_target;
    static const char* band_env = GNCA_AB_ENV("GNCA_K2_BAND");   // measurement knob (A/B runs only)
    if (band_env && atoi(band_env) > 0) rows = atoi(band_env);
    const long cap = (48L * 1024 / 4 / d->W - 2) / 2;
    if (rows > cap) rows = cap;
    if (rows < 1) rows = 1;
    P->band = (int)rows;
    P->nbands = (d->H + P->band - 1) / P->band;
    P->total2 = P->nbands * d->B;
    P->lds2 = (size_t)(2 * P->band + 2) * d->W * 4;
    if (P->lds2 > 64 * 1024) return false;   // W too wide for one row pair
  }
  // workspace
  size_t o = 0;
  auto carve = [&o](size_t bytes) { size_t at = o; o += (bytes + 255) & ~(size_t)255; return at; };
  const size_t n = (size_t)d->B * d->C * d->H * d->W;
  P->off_dx = carve(msg_only ? 0 : n * 4);
  P->off_stats = carve((size_t)P->total_tiles * P->ppt * 2 * sizeof(double));
  P->off_mm = carve((size_t)P->total_tiles * 2 * sizeof(float));
  P->off_offw = carve((size_t)d->B * (P->k > 0 ? P->k : 1) * sizeof(float));
  P->off_rs = carve(P->need_k0 ? (size_t)d->B * d->C * d->H * sizeof(double) : 0);   // K0's row sums
  P->off_alive = carve((size_t)d->B * d->H * d->W);   // rollout: K2 -> next K1 alive bytes
  // rollout: the compact update field's per-tile-row live masks and prefixes (split K1)
  // (large batches only: a small batch's K2 needs thin bands to fill the chip, where unpacking the
  // field costs more than the dx bytes it saves; B=8 72^2: K2 10 -> 18 us)
  P->compact_ok = P->var->split > 0 && P->var->TH > 0 && !msg_only && !attn_on &&
                  (long)P->total_tiles >= 2L * device_cus() * std::max(1, 512 / P->var->NT);
  {
    // K2 bands on the compact field: ~12 rows (B=1024 72^2, tables feeding the alpha rows: 4 rows
    // 0.233, 8 0.180, 12 0.170, 24 0.170 ms; since the alpha plane is dense: 6 0.164, 8 0.158,
    // 12 0.161, 24 0.163 ms, within the box-to-box spread); wide canvases 6 rows (c5, 128^2 x 32ch,
    // step: 4 0.662, 6 0.651, 8 0.652, 12 0.660, 16 0.657, 22 0.673 ms; tools/k2_band_c5.sh).  Since
    // K2 issues ahead of the co-resident K1 (round 4), 6 rows at the headline too: step 0.4920 ->
    // 0.4865 ms over six interleaved pairs (8: 0.52, 24: 0.536; profiles/r04_k2_band_sweep.txt)
    long rows = 6;
    static const char* band_env = GNCA_AB_ENV("GNCA_K2_BAND");   // measurement knob (A/B runs only)
    if (band_env && atoi(band_env) > 0) rows = atoi(band_env);
    const long cap = (48L * 1024 / 4 / d->W - 2) / 2;
    rows = std::max(1L, std::min(rows, cap));
    P->band_c = (int)rows;
    P->nbands_c = (d->H + P->band_c - 1) / P->band_c;
    P->total2_c = P->nbands_c * d->B;
    P->lds2_c = (size_t)(2 * P->band_c + 2) * d->W * 4 + (size_t)(P->band_c + 2) * P->tiles_x * 16 +
                (size_t)d->W * 4;
    if (P->lds2_c > 64 * 1024) P->compact_ok = false;   // very wide canvases: the dense field
  }
  P->off_rmask = carve(P->compact_ok ? (size_t)P->total_tiles * P->TH * sizeof(uint64_t) : 0);
  P->off_rpre = carve(P->compact_ok ? (size_t)P->total_tiles * P->TH * sizeof(uint32_t) : 0);
  P->off_dxa = carve(P->compact_ok ? (size_t)d->B * d->H * d->W * sizeof(float) : 0);
  // the rollout's weight images of the 16-channel split K1 (built once per rollout, gnca_ks_images)
  P->off_wimg = carve(P->var->split == 1 ? (size_t)(ks_layout<24, 36, 4, 4>().total - ks_layout<24, 36, 4, 4>().w1) : 0);
  // the fold: a fold-capable K1 on the compact field, thresholds that allow the alive hand-over
  // (0 <= alpha_thr <= graph_alpha_thr), 32-bit packed-field offsets; the second set of
  // the compact field (each field + 256 B: the finalizer's quad reads may touch one float past it)
  // (the update field is compact for large batches and dense NCHW for small ones)
  // (the preparer sums a sample's partials in one wave pass: tps * waves <= 256)
  // The fold on the compact field (large batches) is not planned where the sub-batch pipeline runs:
  // measured on the headline (B=1024 72^2) it runs 0.566 ms/step against 0.504 for the
  // sub-batch pipeline (K1 + K2 on two streams), because the finalize of each tile's 1.63x halo
  // region comes after the tile's groups and waits on its loads ("The fold").  Small
  // batches (dense field) fold: one launch per step instead of two (BASELINE c2 18.6 -> 15.7 us,
  // c3 20.4 -> 18.3 us).  A rollout asks for the compact fold with GNCA_ROLLOUT_FOLD (fold_any).
  // (not with K0: the zero-padded shift's offset weights come from the step's own finalized state)
  P->fold_any = P->var->fold_fn[P->compact_ok ? 1 : 0] != nullptr && !msg_only && !attn_on && !P->need_k0 &&
               (P->graph_on ? P->k == P->var->KU : P->var->KU == 0) &&
               d->alpha_thr >= 0.f && d->graph_alpha_thr >= d->alpha_thr && n < (size_t)1 << 31 &&
               P->tps * P->ppt <= 256;
#ifdef GNCA_NO_FOLD   // A/B builds: no fold at all
  P->fold_any = false;
#endif
  // Round 6: the compact fold is the default too where a rollout runs ONE stream on the compact field
  // (a batch whose halves are below the compact field's threshold, so no sub-batch pipeline: C4's
  // 128-sample shard): there the separate K2 is not hidden beside another K1, and one K1 launch per
  // step wins (B=128 72^2: 0.0779 vs 0.0819 ms/step; B=256, two streams: 0.150 vs 0.126 without,
  // profiles/r06f_b128_ab.txt)
  const bool one_stream = P->compact_ok && P->var->TH > 0 &&
                          (long)(d->B / 2) * P->tps < 2L * device_cus() * std::max(1, 512 / P->var->NT);
#ifdef GNCA_FOLD_COMPACT_DEFAULT   // A/B builds: the compact fold planned by default too
  P->fold_ok = P->fold_any;
#else
  P->fold_ok = P->fold_any && (!P->compact_ok || one_stream);
#endif
  const bool fc = P->fold_any && P->compact_ok;
  P->off_dx2 = carve(P->fold_any ? n * 4 + 256 : 0);
  P->off_stats2 = carve(P->fold_any ? (size_t)P->total_tiles * P->ppt * 2 * sizeof(double) : 0);
  P->off_rmask2 = carve(fc ? (size_t)P->total_tiles * P->TH * sizeof(uint64_t) : 0);
  P->off_rpre2 = carve(fc ? (size_t)P->total_tiles * P->TH * sizeof(uint32_t) : 0);
  P->off_dxa2 = carve(fc ? (size_t)d->B * d->H * d->W * sizeof(float) : 0);
  P->ws_bytes = o;
  if (P->need_k0) {
    const size_t k0 = ((size_t)d->C * d->H + d->C + d->d_model + P->k) * sizeof(double);
    if (k0 > 64 * 1024) return false;
  }
  return true;
}

int gnca_step_masked_phases(const gnca_step_desc* d, const gnca_weights* w, const float* x, float* x_out,
                            const void* fire, const uint8_t* active, void* ws, size_t ws_bytes,
                            void* stream, uint32_t phases);

bool fwd_layout(const gnca_step_desc* d, FwdLayout* out) {
  Plan P;
  if (!make_plan(d, false, &P)) return false;
  out->ws_bytes = P.ws_bytes;
  out->off_dx = P.off_dx;
  out->off_stats = P.off_stats;
  out->off_offw = P.off_offw;
  out->off_rs = P.off_rs;
  out->tps = P.tps * P.ppt;   // GroupNorm partial pairs per sample
  out->k = P.k;
  out->graph_on = P.graph_on;
  out->need_k0 = P.need_k0;
  return true;
}

struct DevInfo {
  int cus = 256;
};

static int device_cus() {
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

static int occupancy(const void* fn, size_t lds, int nt = kThreads) {
  static std::mutex mu;
  static std::unordered_map<const void*, std::unordered_map<size_t, int>> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& m = cache[fn];
  auto it = m.find(lds);
  if (it != m.end()) return it->second;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, nt, lds) != hipSuccess || n <= 0) n = 1;
  if (n > 8) n = 8;
  m[lds] = n;
  return n;
}

static int check_launch() {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return GNCA_ERR_HIP;
  }
  return GNCA_OK;
}

static void fill_k1(K1Args& k1, const gnca_step_desc* d, const gnca_weights* w, const Plan& P,
                    const float* x, float* out, const void* fire, float* attn, char* ws) {
  memset(&k1, 0, sizeof(k1));
  k1.x = x;
  k1.out = out;
  k1.stats = reinterpret_cast<double*>(ws + P.off_stats);
  k1.attn = attn;
  k1.attn_mm = reinterpret_cast<float*>(ws + P.off_mm);
  k1.perc = w->perception;
  k1.w1 = w->w1;
  k1.b1 = w->b1;
  k1.w2 = w->w2;
  k1.wm = w->wm;
  k1.bm = w->bm;
  k1.offw = P.need_k0 ? reinterpret_cast<float*>(ws + P.off_offw) : nullptr;
  k1.fire = fire;
  k1.seed = d->rng_seed;
  k1.rng_step = d->rng_step;
  k1.sample_base = d->sample_base;
  k1.B = d->B; k1.C = d->C; k1.H = d->H; k1.W = d->W;
  k1.hidden = d->hidden;
  k1.k = P.graph_on ? P.k : 0;
  k1.RY = P.RY; k1.RX = P.RX; k1.TH = P.TH; k1.TW = P.TW;
  k1.tiles_x = P.tiles_x; k1.tps = P.tps; k1.total_tiles = P.total_tiles;
  k1.fire_mode = d->fire_mode;
  k1.fire_rate = d->fire_rate;
  k1.alpha_thr = d->alpha_thr;
  k1.graph_alpha_thr = d->graph_alpha_thr;
  k1.message_gain = d->message_gain;
  k1.uniform_w = P.k > 0 ? (float)(1.0 / (double)P.k) : 0.f;
  k1.flags = d->flags & (GNCA_ZERO_PAD_SHIFT | GNCA_ALIVE_TO_ALIVE | GNCA_HIDDEN_ONLY);
  if (P.graph_on) {
    k1.flags |= kGraphOn;
    if (attn && (d->flags & GNCA_ATTENTION)) k1.flags |= GNCA_ATTENTION;
  }
  const int RW = P.TW + 2 * P.RX;
  const bool zp = (d->flags & GNCA_ZERO_PAD_SHIFT) != 0;
  for (int o = 0; o < P.k; ++o)
    k1.odl[o] = d->offsets[2 * o] * RW + (zp ? 0 : d->offsets[2 * o + 1]);
}

#ifndef GNCA_K0_LDS
#define GNCA_K0_LDS 0   // A/B builds: 1 = the LDS offset-weights kernel for every shape
#endif
// rows_ready: the row sums of x are already in the workspace (the previous step's K2 wrote them)
static int launch_k0(const gnca_step_desc* d, const gnca_weights* w, const Plan& P, const float* x,
                     char* ws, hipStream_t st, bool rows_ready = false) {
  K0Args k0;
  memset(&k0, 0, sizeof(k0));
  k0.x = x; k0.wq = w->wq; k0.bq = w->bq; k0.wk = w->wk; k0.bk = w->bk; k0.scaling = w->scaling;
  k0.offw = reinterpret_cast<float*>(ws + P.off_offw);
  double* rs = reinterpret_cast<double*>(ws + P.off_rs);
  k0.rs = rs;
  k0.B = d->B; k0.C = d->C; k0.H = d->H; k0.W = d->W; k0.d = d->d_model; k0.k = P.k;
  if (!rows_ready) {
    if (d->C > 65535) return GNCA_ERR_UNSUPPORTED;   // (grid y)
    hipLaunchKernelGGL((d->W & 3) == 0 ? gnca_k0_rowsums<4> : gnca_k0_rowsums<1>, dim3(d->B, d->C), dim3(kThreads),
                       0, st, x, rs, d->C, d->H, d->W);
  }
  for (int o = 0; o < 2 * P.k; ++o) k0.offs[o] = d->offsets[o];
  const size_t lds = ((size_t)d->C * d->H + d->C + d->d_model + P.k + (size_t)d->C * P.k +
                      (size_t)P.k * d->d_model) * sizeof(double) + 2 * (size_t)d->d_model * d->C * sizeof(float);
  if (lds > 64 * 1024) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gnca_k0_offset_weights),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (d->C == 16 && d->d_model == 16 && P.k <= 8 && !GNCA_K0_LDS)
    hipLaunchKernelGGL(gnca_k0_weights16, dim3(d->B), dim3(64), 0, st, k0);
  else
    hipLaunchKernelGGL(gnca_k0_offset_weights, dim3(d->B), dim3(kThreads), lds, st, k0);
  return check_launch();
}

static int launch_k1(const K1Args& k1, const Plan& P, hipStream_t st) {
  const int occ = occupancy(P.k1fn, P.lds1, P.var->NT);
  long grid = (long)device_cus() * occ;
  // measurement knob (A/B builds only): leave CUs free of K1 workgroups (for K2 of the other sub-batch)
  static const char* free_env = GNCA_AB_ENV("GNCA_K1_FREE_CUS");
  if (free_env) grid -= atoi(free_env);
  if (grid > P.total_tiles) grid = P.total_tiles;
  if (grid < 1) grid = 1;
  void* args[] = {const_cast<K1Args*>(&k1)};
  const hipError_t e = hipLaunchKernel(P.k1fn, dim3((unsigned)grid), dim3(P.var->NT), args, P.lds1, st);
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return GNCA_ERR_HIP;
  }
  return check_launch();
}

static bool weights_ok(const gnca_step_desc* d, const gnca_weights* w, bool msg_only, const Plan& P) {
  if (!w) return false;
  if (!msg_only && (!w->perception || !w->w1 || !w->b1 || !w->w2)) return false;
  if ((d->flags & GNCA_USE_GROUPNORM) && !msg_only && (!w->gn_weight || !w->gn_bias)) return false;
  if (P.graph_on && (!w->wm || !w->bm)) return false;
  if (P.need_k0 && (!w->wq || !w->bq || !w->wk || !w->bk || !w->scaling)) return false;
  return true;
}

// The update field of one step in the workspace: set 0, or (the fold's double buffer) set 1.
struct FieldSet {
  float* dx;
  double* stats;
  uint64_t* rmask;
  uint32_t* rpre;
  float* dxa;
};
static FieldSet field_set(const Plan& P, char* wsb, int set) {
  if (set == 0)
    return {reinterpret_cast<float*>(wsb + P.off_dx), reinterpret_cast<double*>(wsb + P.off_stats),
            reinterpret_cast<uint64_t*>(wsb + P.off_rmask), reinterpret_cast<uint32_t*>(wsb + P.off_rpre),
            reinterpret_cast<float*>(wsb + P.off_dxa)};
  return {reinterpret_cast<float*>(wsb + P.off_dx2), reinterpret_cast<double*>(wsb + P.off_stats2),
          reinterpret_cast<uint64_t*>(wsb + P.off_rmask2), reinterpret_cast<uint32_t*>(wsb + P.off_rpre2),
          reinterpret_cast<float*>(wsb + P.off_dxa2)};
}

// alive_in / alive_out (rollout only): the previous step's K2 hands this step's K1 its pre-update
// masks as bytes, so K1 skips the alpha halo and the 3x3 max-pools.  set: the update
// field set (the fold rollout alternates sets 0 / 1 by step parity; everything else uses 0).
static int step_impl(const gnca_step_desc* d, const gnca_weights* w, const float* x, float* x_out,
                     const void* fire, float* attn, void* ws, size_t ws_bytes, hipStream_t st,
                     uint32_t phases = GNCA_PHASE_ALL, const uint8_t* active = nullptr,
                     bool alive_in = false, bool alive_out = false, bool compact = false,
                     uint64_t* stamps = nullptr, int stamp_cap = 0, const char* wimg = nullptr, int set = 0,
                     bool k2_co = false) {
  // k2_co: this step's K2 runs beside another sub-batch stream's K1 (the rollout's sub-batch pipeline)
  Plan P;
  if (!make_plan(d, false, &P)) {
    if (d && d->C >= 4 && d->hidden > 0 && !find_variant(d->C, d->hidden)) return GNCA_ERR_UNSUPPORTED;
    return GNCA_ERR_INVALID;
  }
  if (!x || !x_out || x == x_out || !weights_ok(d, w, false, P)) return GNCA_ERR_INVALID;
  if ((d->fire_mode == GNCA_FIRE_RAND_F32 || d->fire_mode == GNCA_FIRE_MASK_U8) && !fire)
    return GNCA_ERR_INVALID;
  if (d->fire_mode < GNCA_FIRE_NONE || d->fire_mode > GNCA_FIRE_HASH) return GNCA_ERR_INVALID;
  const bool want_attn = (d->flags & GNCA_GRAPH) && (d->flags & GNCA_ATTENTION);
  if (want_attn && !attn) return GNCA_ERR_INVALID;
  if (!ws || ws_bytes < P.ws_bytes) return GNCA_ERR_WORKSPACE;
  char* wsb = reinterpret_cast<char*>(ws);
  if (set != 0 && !P.fold_any) return GNCA_ERR_INVALID;
  const FieldSet fs = field_set(P, wsb, set);
  int rc;
  // compact update field (rollout mode): K1 packs the live cells' dx per tile, K2 unpacks them
  compact = compact && P.compact_ok && !active && !want_attn;
  // zero-padded shift in a rollout on the compact field: K2 also writes the new state's row sums, so
  // the next step's K0 skips its pass over the state (the alive-byte hand-over's condition, plus
  // rows of at most 32 cell vectors: K2's fused sums use one 32-lane half-wave per row)
  const bool rows_k2 = P.need_k0 && compact && d->W / ((d->W & 3) == 0 ? 4 : 1) <= 32;
  if ((phases & GNCA_PHASE_K0) && P.need_k0 &&
      (rc = launch_k0(d, w, P, x, wsb, st, rows_k2 && alive_in)) != GNCA_OK)
    return rc;
  // attention with no offsets (k == 0, or radius 1): the reference returns zeros unnormalised
  if (want_attn && !P.graph_on) {
    if (hipMemsetAsync(attn, 0, (size_t)d->B * d->H * d->W * sizeof(float), st) != hipSuccess)
      return GNCA_ERR_HIP;
  }
  K1Args k1;
  float* dx = fs.dx;
  fill_k1(k1, d, w, P, x, dx, fire, want_attn ? attn : nullptr, wsb);
  k1.stats = fs.stats;
  k1.active = active;
  uint8_t* alive = reinterpret_cast<uint8_t*>(wsb + P.off_alive);
  // the split K1s always read the masks as bytes (their preparer wave builds the planes from
  // them): without a hand-over from the previous K2, gnca_k_alive makes them first
  const bool bytes_k1 = P.var->split > 0;
  k1.alive = (alive_in || bytes_k1) ? alive : nullptr;
  if ((phases & GNCA_PHASE_K1) && bytes_k1 && !alive_in) {
    const bool v4 = (d->W & 3) == 0;
    const int nv = d->H * (v4 ? d->W / 4 : d->W);
    const dim3 g((unsigned)std::min((nv + kThreads - 1) / kThreads, 64), (unsigned)std::min(d->B, 65535));
    hipLaunchKernelGGL(v4 ? gnca_k_alive<4> : gnca_k_alive<1>, g, dim3(kThreads), 0, st, x, alive, d->B, d->C,
                       d->H, d->W, d->alpha_thr, d->graph_alpha_thr);
    if ((rc = check_launch()) != GNCA_OK) return rc;
  }
  uint64_t* rmask = fs.rmask;
  uint32_t* rpre = fs.rpre;
  float* dxa = fs.dxa;
  if (compact) {
    k1.rmask = rmask;
    k1.rpre = rpre;
    k1.dxa = dxa;
  }
  // measurement: K1's workgroups stamp into stamps[0 .. 2*cap), K2's into stamps[2*cap .. 4*cap)
  k1.stamps = stamps;
  k1.wimg = P.var->split == 1 ? wimg : nullptr;
  if (stamps && (long)std::min<long>((long)device_cus() * occupancy(P.k1fn, P.lds1, P.var->NT),
                                     P.total_tiles) > stamp_cap)
    return GNCA_ERR_INVALID;
  if ((phases & GNCA_PHASE_K1) && (rc = launch_k1(k1, P, st)) != GNCA_OK) return rc;
  if (!(phases & GNCA_PHASE_K2)) return GNCA_OK;
  K2Args k2;
  memset(&k2, 0, sizeof(k2));
  k2.x = x; k2.dx = dx; k2.out = x_out;
  k2.stats = fs.stats;
  k2.use_gn = (d->flags & GNCA_USE_GROUPNORM) ? 1 : 0;
  k2.gamma = w->gn_weight; k2.beta = w->gn_bias;
  k2.attn = (want_attn && P.graph_on) ? attn : nullptr;
  k2.attn_mm = reinterpret_cast<const float*>(wsb + P.off_mm);
  k2.B = d->B; k2.C = d->C; k2.H = d->H; k2.W = d->W; k2.tps = P.tps; k2.nst = P.tps * P.ppt;
  k2.band = compact ? P.band_c : P.band;
  k2.nbands = compact ? P.nbands_c : P.nbands;
  k2.gain = d->update_gain; k2.thr = d->alpha_thr; k2.eps = d->gn_eps;
  k2.gthr = d->graph_alpha_thr;
  k2.alive_out = alive_out ? alive : nullptr;
  k2.rs = (rows_k2 && alive_out) ? reinterpret_cast<double*>(wsb + P.off_rs) : nullptr;
  k2.active = active;
  // GNCA_K2_ZIGZAG=0 (measurement builds only) keeps the plain sample order; measured B=1024: 0.690
  // -> 0.679 ms/step (K2 0.182 -> 0.180 ms, the next K1 -0.5 %)
  static const char* zz_env = GNCA_AB_ENV("GNCA_K2_ZIGZAG");
  static const bool zz = zz_env == nullptr || atoi(zz_env) != 0;
  k2.zigzag = zz ? 1 : 0;
  if (compact) {
    k2.rmask = rmask;
    k2.rpre = rpre;
    k2.dxa = dxa;
    k2.TH = P.TH;
    k2.TW = P.TW;
    k2.tiles_x = P.tiles_x;
  }
  if (stamps) {
    if ((compact ? P.total2_c : P.total2) > stamp_cap) return GNCA_ERR_INVALID;
    k2.stamps = stamps + 2 * (size_t)stamp_cap;
  }
  auto k2fn = compact ? (k2.rs ? ((d->W & 3) == 0 ? gnca_k2_finalize<4, true, GNCA_K2_CU_ROWS, true>
                                                   : gnca_k2_finalize<1, true, GNCA_K2_CU_ROWS, true>)
                        : k2_co ? ((d->W & 3) == 0 ? gnca_k2_finalize<4, true> : gnca_k2_finalize<1, true>)
                              : ((d->W & 3) == 0 ? gnca_k2_finalize<4, true, GNCA_K2_CU_ALONE>
                                                 : gnca_k2_finalize<1, true, GNCA_K2_CU_ALONE>))
                      : ((d->W & 3) == 0 ? gnca_k2_finalize<4, false> : gnca_k2_finalize<1, false>);
  hipLaunchKernelGGL(k2fn, dim3(compact ? P.total2_c : P.total2), dim3(kThreads),
                     compact ? P.lds2_c : P.lds2, st, k2);
  return check_launch();
}

// One fold K1 launch of a rollout (P.fold_ok): step `d` (offsets, rng_step) on the state
// finalize(xp, field set 1 - set) — written to xo for every tile's own cells — with its update field
// into set `set`.
static int fold_k1(const gnca_step_desc* d, const gnca_weights* w, const Plan& P, const float* xp, float* xo,
                   char* wsb, int set, hipStream_t st, uint64_t* stamps, int stamp_cap, const char* wimg) {
  const FieldSet cur = field_set(P, wsb, set), prev = field_set(P, wsb, set ^ 1);
  K1Args k1;
  fill_k1(k1, d, w, P, xp, cur.dx, nullptr, nullptr, wsb);
  k1.stats = cur.stats;
  if (P.compact_ok) {   // else the dense NCHW field (small batches), dead cells' zeros included
    k1.rmask = cur.rmask;
    k1.rpre = cur.rpre;
    k1.dxa = cur.dxa;
    k1.rmaskp = prev.rmask;
    k1.rprep = prev.rpre;
    k1.dxap = prev.dxa;
  }
  k1.xp = xp;
  k1.xo = xo;
  k1.dxp = prev.dx;
  k1.statsp = prev.stats;
  k1.use_gn = (d->flags & GNCA_USE_GROUPNORM) ? 1 : 0;
  k1.gamma = w->gn_weight;
  k1.beta = w->gn_bias;
  k1.gain = d->update_gain;
  k1.eps = d->gn_eps;
  k1.nst = P.tps * P.ppt;
  k1.wimg = wimg;
  k1.stamps = stamps;
#ifdef GNCA_FOLD_PROTO_ALIVE
  k1.alive = reinterpret_cast<const uint8_t*>(wsb + P.off_alive);
#endif
  const void* fn = P.var->fold_fn[P.compact_ok ? 1 : 0];
  const size_t lds = (size_t)P.var->lds_fold;
  const int occ = occupancy(fn, lds, P.var->NT);
  long grid = std::min<long>((long)device_cus() * occ, P.total_tiles);
  if (grid < 1) grid = 1;
  if (stamps && grid > stamp_cap) return GNCA_ERR_INVALID;
  void* args[] = {&k1};
  const hipError_t e = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(P.var->NT), args, lds, st);
  if (e != hipSuccess) {
    g_last_hip = (int)e;
    return GNCA_ERR_HIP;
  }
  return check_launch();
}

int gnca_step_masked_phases(const gnca_step_desc* d, const gnca_weights* w, const float* x, float* x_out,
                            const void* fire, const uint8_t* active, void* ws, size_t ws_bytes,
                            void* stream, uint32_t phases) {
  return step_impl(d, w, x, x_out, fire, nullptr, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream),
                   phases, active);
}

}  // namespace gnca

namespace gnca {

// ---------------------------------------------------------------------------------------------
// Rollout sub-batch pipeline.  K1 (MFMA/VALU-bound, one persistent workgroup per CU) and K2
// (HBM-bound) of one step cannot overlap: K2 needs the step's GroupNorm statistics, i.e. every
// K1 tile of its sample.  Samples are independent, so a large-batch rollout runs as NSUB
// sub-batches, each stepped on its own stream (the caller's and helper streams) with its own
// workspace region: sub-batch 1's K1 follows sub-batch 0's K1 onto the CUs, and sub-batch 0's K2
// runs on the same CUs beside it (the split K1 leaves LDS, registers and wave slots for one K2
// workgroup per CU), so K2's HBM streaming hides under K1's MFMA work.  Results are bitwise those
// of the one-stream rollout (per-sample GroupNorm, fire hashed by global sample index).
// ---------------------------------------------------------------------------------------------
#ifndef GNCA_ROLLOUT_IMAGES
#define GNCA_ROLLOUT_IMAGES 1   // measurement builds: 0 = every K1 launch builds its weight images
#endif
#ifndef GNCA_ROLLOUT_SUBS
#define GNCA_ROLLOUT_SUBS 2   // measurement builds: 1 = one stream (no sub-batch pipeline)
#endif
constexpr int kRolloutSubs = GNCA_ROLLOUT_SUBS;

static void sub_desc(const gnca_step_desc* d, int sub, int nsub, gnca_step_desc* o, int* b0) {
  *o = *d;
  const int per = d->B / nsub, rem = d->B % nsub;
  *b0 = sub * per + std::min(sub, rem);
  o->B = per + (sub < rem ? 1 : 0);
  o->sample_base = d->sample_base + *b0;
}

// sub-batches of a rollout of `d`'s shape: kRolloutSubs when the planned K1 is the 16-channel
// split kernel with the compact field in every sub-batch and K1 + K2 fit one CU together
static int rollout_subs(const gnca_step_desc* d) {
  if (kRolloutSubs < 2 || !d || d->B < kRolloutSubs) return 1;
  Plan P;
#ifdef GNCA_SUBS_ANY   // A/B builds: the 32-channel K1 too (it leaves no room for a co-resident K2)
  if (!make_plan(d, false, &P) || P.var->split == 0 || !P.compact_ok || P.fold_ok) return 1;
#else
  if (!make_plan(d, false, &P) || P.var->split != 1 || !P.compact_ok || P.fold_ok) return 1;   // (fold_ok: dense)
#endif
  for (int s = 0; s < kRolloutSubs; ++s) {
    gnca_step_desc sd;
    int b0;
    sub_desc(d, s, kRolloutSubs, &sd, &b0);
    Plan Q;
    if (!make_plan(&sd, false, &Q) || Q.var != P.var || !Q.compact_ok) return 1;
#ifndef GNCA_SUBS_ANY
    if (Q.lds1 + Q.lds2_c + 512 > (size_t)max_lds_bytes()) return 1;   // K2's static LDS + margin
#endif
  }
  return kRolloutSubs;
}

static size_t sub_ws_bytes(const gnca_step_desc* d, int sub, int nsub) {
  gnca_step_desc sd;
  int b0;
  sub_desc(d, sub, nsub, &sd, &b0);
  Plan Q;
  return make_plan(&sd, false, &Q) ? (Q.ws_bytes + 255) & ~(size_t)255 : 0;
}

// per-device helper streams and fork/join events (created once, never destroyed: the library
// lives as long as the process)
struct SubStreams {
  hipStream_t s[kRolloutSubs];
  hipEvent_t fork, join[kRolloutSubs];
  std::mutex mu;   // one rollout's fork .. join enqueue at a time per device
};

static SubStreams* sub_streams() {
  static std::mutex mu;
  static std::unordered_map<int, SubStreams*> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  SubStreams* ss = new SubStreams();
  ss->s[0] = nullptr;   // sub-batch 0 runs on the caller's stream
  bool ok = hipEventCreateWithFlags(&ss->fork, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; k < kRolloutSubs && ok; ++k) {
    if (k > 0) ok = hipStreamCreateWithFlags(&ss->s[k], hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&ss->join[k], hipEventDisableTiming) == hipSuccess;
  }
  if (!ok) return nullptr;
  cache[dev] = ss;
  return ss;
}

}  // namespace gnca

using namespace gnca;

extern "C" {

int gnca_abi_version(void) { return GNCA_ABI_VERSION; }

const char* gnca_status_string(int s) {
  switch (s) {
    case GNCA_OK: return "ok";
    case GNCA_ERR_INVALID: return "invalid argument";
    case GNCA_ERR_UNSUPPORTED: return "unsupported shape class (C must be <= 32, hidden <= 256)";
    case GNCA_ERR_WORKSPACE: return "workspace too small";
    case GNCA_ERR_HIP: return "HIP launch failed";
    default: return "unknown status";
  }
}

int gnca_last_hip_error(void) { return g_last_hip; }

size_t gnca_workspace_bytes(const gnca_step_desc* desc) {
  Plan P;
  if (!make_plan(desc, false, &P)) return 0;
  Plan Q;
  size_t m = P.ws_bytes;
  if ((desc->flags & GNCA_GRAPH) && make_plan(desc, true, &Q) && Q.ws_bytes > m) m = Q.ws_bytes;
  const int nsub = rollout_subs(desc);
  if (nsub > 1) {   // a rollout of this shape carves one workspace per sub-batch
    size_t sum = 0;
    for (int k = 0; k < nsub; ++k) sum += sub_ws_bytes(desc, k, nsub);
    if (sum > m) m = sum;
  }
  return m;
}

int gnca_k1_variant(const gnca_step_desc* desc, char* name, int32_t n, int32_t* arith) {
  Plan P;
  if (!name || n <= 0 || !make_plan(desc, false, &P)) return GNCA_ERR_INVALID;
  const Variant* v = P.var;
  if (v->split)
    snprintf(name, (size_t)n, "gnca_k1_split%s<%d,%d,%d,%d,%d>", v->split == 2 ? "32" : "", v->TH, v->TW, v->RY,
             v->RX, v->KU);
  else
    snprintf(name, (size_t)n, "gnca_k1_update<%d,%d,%d,%d,%d,%d,%d,%d>", v->CP, v->HDP, v->TH, v->TW, v->RY, v->RX,
             v->KU, v->NT);
  if (arith) *arith = (v->split ? 1 : 0) | (P.compact_ok ? 2 : 0) | (rollout_subs(desc) > 1 ? 4 : 0) |
                      (P.fold_ok ? 8 : 0) | (P.fold_any ? 16 : 0);
  return GNCA_OK;
}

int gnca_step_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x, float* x_out,
                  const void* fire, float* attn, void* ws, size_t ws_bytes, void* stream) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  return step_impl(desc, w, x, x_out, fire, attn, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream));
}

int gnca_step_masked_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                         float* x_out, const void* fire, const uint8_t* active, void* ws,
                         size_t ws_bytes, void* stream) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  if (!active || (desc && (desc->flags & GNCA_ATTENTION))) return GNCA_ERR_INVALID;
  return step_impl(desc, w, x, x_out, fire, nullptr, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream),
                   GNCA_PHASE_ALL, active);
}

int gnca_step_phases_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                         float* x_out, const void* fire, float* attn, void* ws, size_t ws_bytes,
                         void* stream, uint32_t phases) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  const bool alive = (phases & GNCA_PHASE_ALIVE) && desc && desc->alpha_thr >= 0.f &&
                     desc->graph_alpha_thr >= desc->alpha_thr;
  return step_impl(desc, w, x, x_out, fire, attn, ws, ws_bytes, reinterpret_cast<hipStream_t>(stream),
                   phases, nullptr, alive, alive, (phases & GNCA_PHASE_COMPACT) != 0);
}

int gnca_message_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                     float* message, float* attn, void* ws, size_t ws_bytes, void* stream) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (!desc || !(desc->flags & GNCA_GRAPH)) return GNCA_ERR_INVALID;
  Plan P;
  if (!make_plan(desc, true, &P)) return GNCA_ERR_INVALID;
  if (!x || !message || !weights_ok(desc, w, true, P)) return GNCA_ERR_INVALID;
  const bool want_attn = (desc->flags & GNCA_ATTENTION) != 0;
  if (want_attn && !attn) return GNCA_ERR_INVALID;
  if (!ws || ws_bytes < P.ws_bytes) return GNCA_ERR_WORKSPACE;
  char* wsb = reinterpret_cast<char*>(ws);
  const size_t n = (size_t)desc->B * desc->C * desc->H * desc->W;
  if (!P.graph_on) {  // k == 0: zeros (graph_augmentation.py:141-147)
    if (hipMemsetAsync(message, 0, n * sizeof(float), st) != hipSuccess) return GNCA_ERR_HIP;
    if (want_attn &&
        hipMemsetAsync(attn, 0, (size_t)desc->B * desc->H * desc->W * sizeof(float), st) != hipSuccess)
      return GNCA_ERR_HIP;
    return GNCA_OK;
  }
  int rc;
  if (P.need_k0 && (rc = launch_k0(desc, w, P, x, wsb, st)) != GNCA_OK) return rc;
  K1Args k1;
  fill_k1(k1, desc, w, P, x, message, nullptr, want_attn ? attn : nullptr, wsb);
  k1.flags |= kMsgOnly;
  k1.fire_mode = GNCA_FIRE_NONE;
  if ((rc = launch_k1(k1, P, st)) != GNCA_OK) return rc;
  if (want_attn) {
    dim3 grid((desc->H * desc->W + kThreads - 1) / kThreads, desc->B);
    if (grid.x > 64) grid.x = 64;
    hipLaunchKernelGGL(gnca_attn_normalize, grid, dim3(kThreads), 0, st, attn,
                       reinterpret_cast<const float*>(wsb + P.off_mm), P.tps, desc->H * desc->W);
    return check_launch();
  }
  return GNCA_OK;
}

int gnca_perceive_f32(int32_t B, int32_t C, int32_t H, int32_t W, const float* weight,
                      const float* x, float* y, void* stream) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || !weight || !x || !y) return GNCA_ERR_INVALID;
  const size_t total = (size_t)B * C * H * W;
  size_t blocks = (total + kThreads - 1) / kThreads;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(gnca_perceive, dim3((unsigned)blocks), dim3(kThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), B, C, H, W, weight, x, y);
  return check_launch();
}

#ifdef GNCA_PROFILE
int gnca_prof_dump(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)) == hipSuccess ? 0 : -1;
}
int gnca_fprof_dump(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fprof), sizeof(g_fprof)) == hipSuccess ? 0 : -1;
}
int gnca_arr_dump(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_arr), sizeof(g_arr)) == hipSuccess ? 0 : -1;
}
#endif

int gnca_fire_mask_u8(const gnca_step_desc* desc, uint8_t* mask, void* stream) {
  StreamDeviceGuard dg(reinterpret_cast<hipStream_t>(stream));
  if (!desc || !mask || desc->B <= 0 || desc->H <= 0 || desc->W <= 0) return GNCA_ERR_INVALID;
  const size_t total = (size_t)desc->B * desc->H * desc->W;
  size_t blocks = (total + kThreads - 1) / kThreads;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gnca_fire_mask, dim3((unsigned)blocks), dim3(kThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), mask, desc->B, desc->H * desc->W,
                     desc->rng_seed, desc->rng_step, desc->sample_base, desc->fire_rate);
  return check_launch();
}

}  // extern "C"

static int rollout_impl(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                        const int8_t* offsets, const float* x, float* x_final, float* scratch,
                        void* ws, size_t ws_bytes, void* stream, uint64_t* stamps, int stamp_cap,
                        uint32_t flags) {
  if (!desc || steps < 0 || !x || !x_final || !scratch) return GNCA_ERR_INVALID;
  if (flags & ~(uint32_t)(GNCA_ROLLOUT_ALIVE_IN | GNCA_ROLLOUT_ALIVE_OUT | GNCA_ROLLOUT_PENDING_IN |
                          GNCA_ROLLOUT_PENDING_OUT | GNCA_ROLLOUT_FOLD))
    return GNCA_ERR_INVALID;
  if ((flags & GNCA_ROLLOUT_ALIVE_IN) && (flags & GNCA_ROLLOUT_PENDING_IN)) return GNCA_ERR_INVALID;
  if ((flags & GNCA_ROLLOUT_ALIVE_OUT) && (flags & GNCA_ROLLOUT_PENDING_OUT)) return GNCA_ERR_INVALID;
  if (desc->fire_mode != GNCA_FIRE_NONE && desc->fire_mode != GNCA_FIRE_HASH) return GNCA_ERR_INVALID;
  if (x == x_final || x == scratch || x_final == scratch) return GNCA_ERR_INVALID;
  // a zero-step piece of a rollout issued in pieces would have to order its copy after the other
  // sub-batch streams' work (and join them if it is the last piece): not a meaningful call
  if (steps == 0 && flags != 0) return GNCA_ERR_INVALID;
  const int k = desc->num_offsets;
  if ((desc->flags & GNCA_GRAPH) && k > 0 && !offsets) return GNCA_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  StreamDeviceGuard dg(st);   // helper streams, events and CU counts of the stream's device
  if (steps == 0)
    return hipMemcpyAsync(x_final, x, (size_t)desc->B * desc->C * desc->H * desc->W * sizeof(float),
                          hipMemcpyDeviceToDevice, st) == hipSuccess ? GNCA_OK : GNCA_ERR_HIP;
  gnca_step_desc dt = *desc;
  dt.flags &= ~GNCA_ATTENTION;
  // K2 -> next K1 alive masks: exact when 0 <= alpha_thr <= graph_alpha_thr (a cell with alpha
  // above either threshold keeps its alpha through the post-update gate); and only
  // when every step uses the same threshold pair (one desc for the whole rollout: yes)
  const bool hand_alive = desc->alpha_thr >= 0.f && desc->graph_alpha_thr >= desc->alpha_thr;
  if ((flags & (GNCA_ROLLOUT_ALIVE_IN | GNCA_ROLLOUT_ALIVE_OUT)) && !hand_alive) return GNCA_ERR_INVALID;
  const bool in0 = (flags & GNCA_ROLLOUT_ALIVE_IN) != 0, out_last = (flags & GNCA_ROLLOUT_ALIVE_OUT) != 0;
  const bool pend_in = (flags & GNCA_ROLLOUT_PENDING_IN) != 0, pend_out = (flags & GNCA_ROLLOUT_PENDING_OUT) != 0;
  Plan PF;
  if (!make_plan(&dt, false, &PF)) return GNCA_ERR_INVALID;
  // the fold runs the whole batch on one stream (a requested fold overrides the sub-batch pipeline,
  // whose workspace carve differs: the weight images below must use the fold's)
  const bool fold = PF.fold_ok || (PF.fold_any && (flags & GNCA_ROLLOUT_FOLD));
  const int nsub = fold ? 1 : rollout_subs(&dt);
  if ((pend_in || pend_out) && !fold) return GNCA_ERR_INVALID;
  // an ALIVE_IN / ALIVE_OUT chain must keep one plan across its pieces: the alive masks and weight
  // images sit at the plan's workspace offsets, and the sub-batch streams are forked by the first
  // piece and joined by the last.  A FOLD request that changes the plan (compact field: one-stream
  // fold instead of the sub-batch pipeline) could differ between pieces, so it is not allowed with
  // ALIVE_*; fold chains hand over with PENDING_* instead.
  if ((in0 || out_last) && (flags & GNCA_ROLLOUT_FOLD) && fold && !PF.fold_ok && rollout_subs(&dt) > 1)
    return GNCA_ERR_INVALID;
  // the 16-channel split K1's weight images, once for the whole rollout (every K1 launch then copies
  // them into LDS with LDS-DMA instead of loading, splitting and storing the fp32 weights)
  const char* wimg = nullptr;
  {
    gnca_step_desc d0 = dt;
    int b0 = 0;
    if (nsub > 1) sub_desc(&dt, 0, nsub, &d0, &b0);
    Plan P0;
    if (!make_plan(&d0, false, &P0)) return GNCA_ERR_INVALID;
    if (GNCA_ROLLOUT_IMAGES && P0.var->split == 1 && ws && ws_bytes >= P0.ws_bytes && weights_ok(&d0, w, false, P0)) {
      // a continuation piece (ALIVE_IN) reuses the images its first piece built in the same workspace
      // (rebuilding them here could overwrite them under the other sub-batch stream's K1)
      char* dst = reinterpret_cast<char*>(ws) + P0.off_wimg;
      if (!in0 && !pend_in) {
        K1Args ka;
        fill_k1(ka, &d0, w, P0, x, nullptr, nullptr, nullptr, reinterpret_cast<char*>(ws));
        hipLaunchKernelGGL(gnca_ks_images, dim3(1), dim3(512), 0, st, ka, dst);
        const int rc = check_launch();
        if (rc != GNCA_OK) return rc;
      }
      wimg = dst;
    }
  }
  if (fold) {
    // The fold: K1 of step t also finishes step t - 1 (one launch per step); the update field of
    // global step g lives in set g & 1.  State S_t = the input of step t: S_0 = x (or, PENDING_IN,
    // finalize(x, the pending field), written by the first K1); K1 of step t >= 1 writes S_t; the
    // last step is finished by K2 into x_final (or, PENDING_OUT, left pending: S_{T-1} is x_final).
    if (!weights_ok(&dt, w, false, PF)) return GNCA_ERR_INVALID;
    if (!ws || ws_bytes < PF.ws_bytes) return GNCA_ERR_WORKSPACE;
    char* wsb = reinterpret_cast<char*>(ws);
    const int T = steps;
    const int last = pend_out ? T - 1 : T;   // the state that lands in x_final
    auto buf = [&](int t) -> float* { return ((last - t) % 2 == 0) ? x_final : scratch; };
    auto state = [&](int t) -> const float* { return (t == 0 && !pend_in) ? x : buf(t); };
    for (int t = 0; t < T; ++t) {
      dt.rng_step = desc->rng_step + t;
      if ((desc->flags & GNCA_GRAPH) && k > 0) memcpy(dt.offsets, offsets + (size_t)t * 2 * k, 2 * k);
      const int set = (int)(dt.rng_step & 1);
      uint64_t* sk = stamps ? stamps + (size_t)t * 4 * stamp_cap : nullptr;
      int rc;
      if (t == 0 && !pend_in)
        rc = step_impl(&dt, w, x, x_final, nullptr, nullptr, ws, ws_bytes, st, GNCA_PHASE_K0 | GNCA_PHASE_K1,
                       nullptr, in0, false, true, sk, stamp_cap, wimg, set);
      else
        rc = fold_k1(&dt, w, PF, t == 0 ? x : state(t - 1), buf(t), wsb, set, st, sk, stamp_cap, wimg);
      if (rc != GNCA_OK) return rc;
    }
    if (pend_out) {   // the pending state S_{T-1} must be in x_final (T == 1: it is the input x)
      if (T == 1 && !pend_in &&
          hipMemcpyAsync(x_final, x, (size_t)desc->B * desc->C * desc->H * desc->W * sizeof(float),
                         hipMemcpyDeviceToDevice, st) != hipSuccess)
        return GNCA_ERR_HIP;
      return GNCA_OK;
    }
    // the last step's finish: K2 on the compact field of step T - 1
    return step_impl(&dt, w, state(T - 1), x_final, nullptr, nullptr, ws, ws_bytes, st, GNCA_PHASE_K2, nullptr,
                     false, out_last, true, stamps ? stamps + (size_t)(T - 1) * 4 * stamp_cap : nullptr, stamp_cap,
                     wimg, (int)(dt.rng_step & 1));
  }
  if (nsub == 1) {
    const float* src = x;
    for (int t = 0; t < steps; ++t) {
      float* dst = ((steps - 1 - t) % 2 == 0) ? x_final : scratch;
      dt.rng_step = desc->rng_step + t;
      if ((desc->flags & GNCA_GRAPH) && k > 0) memcpy(dt.offsets, offsets + (size_t)t * 2 * k, 2 * k);
      const int rc = step_impl(&dt, w, src, dst, nullptr, nullptr, ws, ws_bytes, st, GNCA_PHASE_ALL,
                               nullptr, hand_alive && (t > 0 || in0), hand_alive && (t + 1 < steps || out_last),
                               true, stamps ? stamps + (size_t)t * 4 * stamp_cap : nullptr, stamp_cap, wimg);
      if (rc != GNCA_OK) return rc;
      src = dst;
    }
    return GNCA_OK;
  }
  // sub-batch pipeline (above): sub-batch j on stream j with workspace region j; its launches are
  // enqueued step-major so every stream always has its next step queued
  gnca_step_desc sd[kRolloutSubs];
  size_t off[kRolloutSubs], wsz[kRolloutSubs], elem0[kRolloutSubs];
  size_t wtot = 0;
  const size_t per_sample = (size_t)desc->C * desc->H * desc->W;
  for (int j = 0; j < nsub; ++j) {
    int b0;
    sub_desc(&dt, j, nsub, &sd[j], &b0);
    elem0[j] = (size_t)b0 * per_sample;
    wsz[j] = sub_ws_bytes(&dt, j, nsub);
    off[j] = wtot;
    wtot += wsz[j];
  }
  if (!ws || ws_bytes < wtot) return GNCA_ERR_WORKSPACE;
  SubStreams* ss = sub_streams();
  if (!ss) return GNCA_ERR_HIP;
  std::lock_guard<std::mutex> lk(ss->mu);
  hipStream_t sj[kRolloutSubs];
  for (int j = 0; j < nsub; ++j) sj[j] = j == 0 ? st : ss->s[j];
  // fork (not for a continuation piece: its sub-batch streams carry on from the previous piece)
  if (!in0) {
    if (hipEventRecord(ss->fork, st) != hipSuccess) return GNCA_ERR_HIP;
    for (int j = 1; j < nsub; ++j)
      if (hipStreamWaitEvent(sj[j], ss->fork, 0) != hipSuccess) return GNCA_ERR_HIP;
  }
  char* wsb = reinterpret_cast<char*>(ws);
  int rc = GNCA_OK;
  for (int t = 0; t < steps && rc == GNCA_OK; ++t) {
    const float* src = t == 0 ? x : (((steps - t) % 2 == 0) ? x_final : scratch);
    float* dst = ((steps - 1 - t) % 2 == 0) ? x_final : scratch;
    for (int j = 0; j < nsub && rc == GNCA_OK; ++j) {
      sd[j].rng_step = desc->rng_step + t;
      if ((desc->flags & GNCA_GRAPH) && k > 0) memcpy(sd[j].offsets, offsets + (size_t)t * 2 * k, 2 * k);
      rc = step_impl(&sd[j], w, src + elem0[j], dst + elem0[j], nullptr, nullptr, wsb + off[j], wsz[j], sj[j],
                     GNCA_PHASE_ALL, nullptr, hand_alive && (t > 0 || in0),
                     hand_alive && (t + 1 < steps || out_last), true,
                     stamps ? stamps + ((size_t)t * nsub + j) * 4 * stamp_cap : nullptr, stamp_cap, wimg, 0, true);
    }
  }
  // join (also after a failed launch: the helper streams' work stays ordered before the caller's);
  // not when another piece follows (ALIVE_OUT): the last piece joins
  for (int j = 1; j < nsub && (!out_last || rc != GNCA_OK); ++j) {
    if (hipEventRecord(ss->join[j], sj[j]) != hipSuccess || hipStreamWaitEvent(st, ss->join[j], 0) != hipSuccess)
      return GNCA_ERR_HIP;
  }
  return rc;
}

extern "C" {

int gnca_rollout_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                     const int8_t* offsets, const float* x, float* x_final, float* scratch,
                     void* ws, size_t ws_bytes, void* stream) {
  return rollout_impl(desc, w, steps, offsets, x, x_final, scratch, ws, ws_bytes, stream, nullptr, 0, 0u);
}

int gnca_rollout_ex_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                        const int8_t* offsets, const float* x, float* x_final, float* scratch,
                        void* ws, size_t ws_bytes, uint32_t flags, void* stream) {
  return rollout_impl(desc, w, steps, offsets, x, x_final, scratch, ws, ws_bytes, stream, nullptr, 0, flags);
}

int gnca_rollout_stamped_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                             const int8_t* offsets, const float* x, float* x_final, float* scratch,
                             void* ws, size_t ws_bytes, uint64_t* stamps, int32_t stamp_cap,
                             void* stream) {
  if (!stamps || stamp_cap <= 0) return GNCA_ERR_INVALID;
  return rollout_impl(desc, w, steps, offsets, x, x_final, scratch, ws, ws_bytes, stream, stamps,
                      stamp_cap, 0u);
}

}  // extern "C"

#endif  // GNCA_K1_PROBE
