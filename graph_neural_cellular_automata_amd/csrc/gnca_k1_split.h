// gnca_k1_split.h — K1 of the 16-channel / hidden-128 step on bf16 MFMA with an exact 3-way
// split of every fp32 operand (included by gnca_step.hip after K1Args).
//
// Why.  gfx950 runs fp32 MFMA (v_mfma_f32_*_f32) at the fp32 VECTOR rate, 1/16 of bf16 MFMA,
// and on the same SIMD datapath as VALU (profiles/r01_ubench_mfma_valu_overlap.txt).  The f32
// K1 (gnca_k1_update) spends ~70 % of its group loop in fp32 MFMA issue.
//
// Numerics (fp32-class, not bf16).  Every fp32 operand v is split into three bf16 values
// v = v0 + v1 + v2 EXACTLY (v0 = rne_bf16(v), v1 = rne_bf16(v - v0), v2 = v - v0 - v1: 8 + 8 + 8
// significand bits hold the 24 of an fp32; for |v| > 2^-100 nothing is subnormal).  A dot
// product a.b is then sum over (i, j) of a_i . b_j, and the kernel keeps the six terms with
// i + j <= 2 (a0b0, a0b1, a1b0, a0b2, a2b0, a1b1): the dropped terms a1b2, a2b1, a2b2 are each
// <= 2^-24 |a||b|, the size of one fp32 rounding.  bf16 x bf16 products are exact in fp32 and
// the MFMA accumulates in fp32.  So each GEMM is an fp32 GEMM up to a few fp32 roundings per
// product (measured against the f64 oracle in tests/test_gpu_*.py at the same tolerances as
// the f32 kernel).  Cost: 6 bf16 products at 1/16 the cycles of one fp32 product = 0.375 of
// the fp32 MFMA time, plus the VALU that splits the activations.
//
// MFMA: v_mfma_f32_32x32x16_bf16 (32 cycles, holds VALU issue for 8 of them).  Lane l: cell
// l & 31 of a 32-cell group, channel / k half h = l >> 5.  Fragment maps
// (cdna_hip_programming.md §3): A[row l&31][k 8h+j], B[k 8h+j][col l&31], D reg r ->
// row (r&3) + 8(r>>2) + 4h, col l&31.
//   GEMM1  H[128 x 32] = W1[128 x 48] Y[48 x 32] + b1: 4 row blocks (rb) x 3 k-chunks (kc);
//          k slot (kc, h, j) = feature kc (0 id, 1 sobel-x, 2 sobel-y) of channel 8h + j, which
//          is exactly W1's column 16 kc + 8h + j, so lane (cell, h) computes the perception of
//          channels 8h..8h+7 of its own cell.  Bias: the accumulator starts at b1 (fp32, read
//          from LDS; until round 4 an extra MFMA per rb over b1's three bf16 parts, which gave
//          the same exact b1: the same bits, 4 MFMAs fewer per group).
//   GEMM2  DL[16 x 32] = W2[16 x 128] relu(H): k-chunk s = (rb, ss) takes accumulator registers
//          8ss..8ss+7 of H block rb as the B fragment, element j of half h = hidden row
//          32rb + 16ss + 8(j>>2) + 4h + (j&3) (no data movement; the A image is permuted to
//          match).  M = 32 rows hold TWO 16-channel weight planes: A = [P0; P1] gives
//          P0.H in rows 0-15 and P1.H in rows 16-31 of the SAME accumulator (one lane holds
//          both: regs r and r + 8).  Products by B plane: H0 with P0, P1, P2; H1 with P0, P1;
//          H2 with P0 -> accA += [P0;P1].H0 + [P0;P1].H1, accB += [P2;P2].H0 + [P0;P1].H2 (accB's
//          rows 16-31 are ignored), dl = accA[r] + accA[r+8] + accB[r].
//   MSG    M[16 x 32] = WM[16 x 16] G[16 x 32] (G = the gathered alive-masked x, k = channel
//          8h + j): one k-chunk, stacks [M0;M1], [M2;0], [M0;0] (0 = a zero image), all in
//          one accumulator: rows 0-15 + rows 16-31 = the six products.
// Weight images (bf16, built once per persistent workgroup): W1 36 KB, W2 12 KB, WM 1.5 KB + 0.5 KB
// of zeros; every A read is one conflict-free ds_read_b128.  The bias b1 is GEMM1's initial
// accumulator in fp32 (0.5 KB, per lane half the 16 rows of its accumulator registers).
//
// The rest of the tile pipeline is the f32 K1's (LDS-DMA staging, alive / sender / keep planes,
// live-cell compaction, fp64 GroupNorm partials per (tile, wave)), with 32-cell groups, byte
// keep plane, u16 live list and a tight channel-plane stride (DMA lanes past the region are
// masked off instead of filling a pad).  Perception zero padding at the image border uses
// per-tap LDS bases that point at a zero float (each plane's first pad float) instead of
// per-channel selects.

#pragma once

namespace gnca {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// (a, b) -> three packed bf16x2 words with a = a0 + a1 + a2, b = b0 + b1 + b2 exactly (round to
// nearest even at each level: NaN stays NaN in the leading part, v_cvt_pk_bf16_f32).
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  const uint32_t h = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
  const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
  const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){ra, rb}, bf16x2v));
  const float la = ra - __uint_as_float(m << 16), lb = rb - __uint_as_float(m & 0xffff0000u);
  p0 = h;
  p1 = m;
  p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){la, lb}, bf16x2v));
}

// 8 fp32 -> three bf16x8 fragments (k order = element order)
__device__ __forceinline__ void split3_x8(const float* v, u32x4& f0, u32x4& f1, u32x4& f2) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t a, b, c;
    split3_pair(v[2 * i], v[2 * i + 1], a, b, c);
    f0[i] = a;
    f1[i] = b;
    f2[i] = c;
  }
}

__device__ __forceinline__ f32x16 mfma_bx(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                 c, 0, 0, 0);
}

// 16 zero bytes in global memory: the LDS-DMA source of the zero-padded shift's out-of-image quads
__device__ __attribute__((aligned(16))) float gnca_zero16[4];

#ifndef GNCA_K1_PIPE_LDS
#define GNCA_K1_PIPE_LDS 1   // pipeline depth of the gather / perception reads (A/B builds: 0 = the plain loops)
#endif

// Gather of alive-masked x over the KU offsets for one lane's 8 channels (plane stride PSTR), software-
// pipelined: the 9 LDS reads of offset o + 1 are issued before the FMAs of offset o (sched_barrier
// fences keep the order), so reads are always in flight.  Left to itself the compiler emitted read /
// wait / FMA chains (a wave alone on its SIMD then pays every LDS latency: 32-channel K1, ~2/3 of
// each phase).  Same FMA order as the plain loop: bitwise the same sums.
// ZP (zero-padded shift): the per-sample offset weights wo[o] (K0's softmax) weigh each offset's sender
// byte (the uniform 1/k of the torus mode is applied once by the caller instead)
template <int KU, int PSTR, bool ZP = false>
__device__ __forceinline__ void ks_gather8(const int* odl, const float* xq, const uint8_t* spq, float (&gv)[8],
                                           float& S, const float* wo = nullptr) {
  constexpr int D = GNCA_K1_PIPE_LDS;   // offsets whose reads are in flight ahead of the FMAs
  float xv[D + 1][8];
  uint32_t sv[D + 1];
  auto ld = [&](int o) {
    const int d = odl[o];
    sv[o % (D + 1)] = spq[-d];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[o % (D + 1)][j] = xq[j * PSTR - d];
  };
#pragma unroll
  for (int o = 0; o < D && o < KU; ++o) ld(o);
#pragma unroll
  for (int o = 0; o < KU; ++o) {
    if (o + D < KU) ld(o + D);
    __builtin_amdgcn_sched_barrier(0);
    const float s_ = ZP ? wo[o] * (float)sv[o % (D + 1)] : (float)sv[o % (D + 1)];
    S += s_;
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = fmaf(s_, xv[o % (D + 1)][j], gv[j]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// The frozen Sobel bank's perception of one lane's 8 channels from the 9 tap offsets t[] (zero taps at
// the image border), pipelined as ks_gather8: channel j + 1's 9 reads in flight under channel j's
// arithmetic.  y0 = identity, y1 = Sobel-x, y2 = Sobel-y with shared diagonal differences.
template <int PSTR>
__device__ __forceinline__ void ks_sobel8(const float* xs, const int (&t)[9], float (&y0)[8], float (&y1)[8],
                                          float (&y2)[8]) {
  constexpr int D = GNCA_K1_PIPE_LDS;
  float nv[D + 1][9];
  auto ld = [&](int j) {
#pragma unroll
    for (int k = 0; k < 9; ++k) nv[j % (D + 1)][k] = xs[t[k] + j * PSTR];
  };
#pragma unroll
  for (int j = 0; j < D; ++j) ld(j);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j + D < 8) ld(j + D);
    __builtin_amdgcn_sched_barrier(0);
    const float* n = nv[j % (D + 1)];
    y0[j] = n[4];
    const float dg = n[0] - n[8], da = n[2] - n[6];
    y1[j] = fmaf(2.f, n[3] - n[5], dg - da);
    y2[j] = fmaf(2.f, n[1] - n[7], dg + da);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// channel-plane stride (floats) of the split kernel's staged region: at least one pad float
// (the zero tap of the border perception), 16 mod 32 (planes start 16 banks apart), quads
__host__ __device__ constexpr int ks_pstr(int rhw) {
  int p = rhw + 1;
  while (p % 32 != 16) ++p;
  return p;
}

struct KSLayout {
  int xs, sp, ab, lst, cnt, cb, fb, pg, fk, p0, p1, pbm, ft, w1, bias, w2, wm, wz, bml, pf, total;   // byte offsets
  int sp_slot, lst_slot, cb_slot;                                        // bytes per prepared-tile slot
};

__host__ __device__ constexpr int ks_a16(int v) { return (v + 15) & ~15; }

// The planes a tile's groups read besides the staged channel planes (the sender plane sp over the
// region and the live-cell list) come in two slots: the preparer wave fills the next tile's slot
// while the other waves still run this tile's groups (below).
template <int TH, int TW, int RY, int RX, bool FOLD = false>
__host__ __device__ constexpr KSLayout ks_layout() {
  constexpr int RH = TH + 2 * RY, RW = TW + 2 * RX, RHW = RH * RW;
  KSLayout L{};
  int o = 0;
  L.sp_slot = ks_a16(RHW);
  L.lst_slot = ks_a16(TH * TW * 2);
  L.cb_slot = ks_a16(8 * (TH * TW / 64 + 2));
  L.xs = o; o += 16 * ks_pstr(RHW) * 4;   // first: region reads fit the 16-bit DS offsets
  L.sp = o; o += 2 * L.sp_slot;           // sender plane (bytes 0/1), two slots
  L.ab = o; o += ks_a16(RHW);             // the preparer's alive bytes over the region
  L.lst = o; o += 2 * L.lst_slot;         // live-cell list (u16 cell indices), two slots
  L.cnt = o; o += 48;                     // live cells per slot; group counter; staging-reads-done counter;
                                          // fold: finalize-item counter, preparations done, group done-masks;
                                          // the first tile's fire ballots done
  L.cb = o; o += 2 * L.cb_slot;           // the preparer's 64-cell chunk keep ballots, two slots
  L.fb = o; o += 32;                      // small tiles: the first tile's fire ballots (<= 4 chunks)
  L.pg = o; o += 2 * 16 * ((TH * TW + 31) / 32);  // per-group GroupNorm partials (fp64 pairs), two slots
  // fold (gnca_k1_split<..., FOLD>): per slot the previous step's GroupNorm constants (48 floats) and
  // the region's pre-update alive row masks P0 (one u64 per region row); the preparer's sender row
  // masks P1 and its threshold-bit row masks of the pooled band (2 x (RH + 2) u64)
  // (only in the fold variant's layout: the plain K1 keeps room for a co-resident K2 workgroup)
  L.fk = o; o += FOLD ? 2 * 192 : 0;
  L.p0 = o; o += FOLD ? 2 * ks_a16(RH * 8) : 0;
  L.p1 = o; o += FOLD ? ks_a16(RH * 8) : 0;
  L.pbm = o; o += FOLD ? ks_a16(2 * (RH + 2) * 8) : 0;
  L.ft = o; o += FOLD ? 2 * ks_a16((RH + 2) * 3 * 16) : 0;   // per slot: the previous step's row tables
  L.w1 = o; o += 3 * 4 * 3 * 1024;       // [plane][rb][kc][lane] x 16 B
  L.bias = o; o += 4 * 32 * 16;          // [rb][row] x 16 B (k slots 0..2 = the three parts)
  L.w2 = o; o += 3 * 8 * 2 * 16 * 16;    // [plane][s][h][channel] x 16 B
  L.wm = o; o += 3 * 2 * 16 * 16;        // [plane][h][channel] x 16 B
  L.wz = o; o += 2 * 16 * 16;            // zeros, laid out like one WM plane
  L.bml = o; o += 2 * 8 * 4;             // message bias per (lane half h, accumulator register r)
  L.pf = o; o += 16;                     // (images built by gnca_ks_images) perception == the Sobel bank
  L.total = o;
  return L;
}

// The 16-channel split K1's weight images (bf16 parts in MFMA fragment order, layout ks_layout's
// w1 .. bml block, offsets relative to its start): W1 [part][rb][kc][lane] x 16 B, the bias, W2
// [part][s][h][channel] (the third part halved in the lean body), WM [part][h][channel] + a zero
// image, the message bias per (h, r).  Built by each K1 workgroup into LDS, or once per rollout
// into global memory (gnca_ks_images) that K1 then copies with LDS-DMA: the same bits either way.
// NT threads, every weight load of a thread in flight before its splits and stores.
template <int NT, bool GRAPH, bool TO_LDS>
__device__ __forceinline__ void ks_fill_images(const K1Args& a, char* dst, int tid);

#ifndef GNCA_K1_LEAN
#define GNCA_K1_LEAN 1   // 1: register-lean group body (one GEMM2 accumulator seeded with the message, GEMM1 row
                         // blocks double-buffered through GEMM2); 0: round 2's body; 2 (A/B builds): the lean body as
                         // a row-block software pipeline -- 250 VGPRs leave no room for a co-resident K2 wave, so
                         // the sub-batch pipeline's step is slower (0.540 vs 0.530 ms) although K1 alone is not
#endif

template <int NT, bool GRAPH, bool TO_LDS>
__device__ __forceinline__ void ks_fill_images(const K1Args& a, char* dst, int tid) {
  constexpr int C = 16, HD = 128;
  constexpr KSLayout L = ks_layout<24, 36, 4, 4>();   // the image block's offsets do not depend on the tile
  constexpr int OW1 = 0, OB = L.bias - L.w1, OW2 = L.w2 - L.w1, OWM = L.wm - L.w1, OWZ = L.wz - L.w1,
                OBM = L.bml - L.w1;
  static_assert(4 * 3 * 64 <= 2 * NT && 8 * 2 * 16 <= NT, "one pass of weight loads");
  auto st16 = [&](int off, u32x4 v) { *reinterpret_cast<u32x4*>(dst + off) = v; };
  float w1v[2][8], w2v[8], wmv[8], b1v = 0.f, bmv = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    // W1: entry e = (rb, kc, lane): W1[32rb + (lane&31)][16kc + 8(lane>>5) + 0..7]
    const int e = tid + u * NT, rb = e / 192, kc = (e / 64) % 3, l = e & 63;
    const float* src = a.w1 + (size_t)(32 * rb + (l & 31)) * 48 + 16 * kc + 8 * (l >> 5);
#pragma unroll
    for (int j = 0; j < 8; ++j) w1v[u][j] = e < 4 * 3 * 64 ? src[j] : 0.f;
  }
  {
    // W2: entry (s, h, c): W2[c][32(s>>1) + 16(s&1) + 8(j>>2) + 4h + (j&3)], j = 0..7
    const int s = (tid >> 5) & 7, hh = (tid >> 4) & 1, c = tid & 15;
    const float* src = a.w2 + (size_t)c * HD + 32 * (s >> 1) + 16 * (s & 1) + 4 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) w2v[j] = tid < 8 * 2 * 16 ? src[8 * (j >> 2) + (j & 3)] : 0.f;
    // WM: entry (h, c): WM[c][8h + 0..7]
#pragma unroll
    for (int j = 0; j < 8; ++j) wmv[j] = (GRAPH && tid < 32) ? a.wm[(tid & 15) * C + 8 * ((tid >> 4) & 1) + j] : 0.f;
  }
  if (tid < 128) b1v = a.b1[tid];
  if (GRAPH && tid < 16) bmv = a.bm[(tid & 3) + 8 * ((tid & 7) >> 2) + 4 * (tid >> 3)];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + u * NT;
    if (e < 4 * 3 * 64) {
      const int rb = e / 192, kc = (e / 64) % 3, l = e & 63;
      u32x4 f0, f1, f2;
      split3_x8(w1v[u], f0, f1, f2);
      const int img = OW1 + (rb * 3 + kc) * 1024 + l * 16;
      st16(img, f0);
      st16(img + 12288, f1);
      st16(img + 2 * 12288, f2);
    }
  }
  if (tid < 128) {   // bias: GEMM1's initial accumulator per (rb, lane half h): register r holds
                     // b1[32rb + (r&3) + 8(r>>2) + 4h] (row = tid - 32rb)
    const int rb = tid >> 5, row = tid & 31, hh = (row >> 2) & 1, r = (row & 3) + 4 * (row >> 3);
    reinterpret_cast<float*>(dst + OB)[(rb * 2 + hh) * 16 + r] = b1v;
  }
  if (tid < 8 * 2 * 16) {
    u32x4 f0, f1, f2;
    split3_x8(w2v, f0, f1, f2);
#if GNCA_K1_LEAN
    // the third part is stored halved (exact: a power-of-two scale of a bf16 value): the GEMM2
    // stack [P2/2; P2/2] adds P2.H0 / 2 to both accumulator halves, which the epilogue sums
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = __uint_as_float(f2[i] << 16) * 0.5f, hi = __uint_as_float(f2[i] & 0xffff0000u) * 0.5f;
      f2[i] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
    }
#endif
    st16(OW2 + tid * 16, f0);
    st16(OW2 + 4096 + tid * 16, f1);
    st16(OW2 + 8192 + tid * 16, f2);
  }
  if (tid < 32) {   // WM, then the zero image
    u32x4 f0, f1, f2;
    split3_x8(wmv, f0, f1, f2);
    st16(OWM + tid * 16, f0);
    st16(OWM + 512 + tid * 16, f1);
    st16(OWM + 1024 + tid * 16, f2);
    st16(OWZ + tid * 16, u32x4{0u, 0u, 0u, 0u});
  }
  // message bias of output channel c = (r&3) + 8(r>>2) + 4h at [h][r]
  if (tid < 16) reinterpret_cast<float*>(dst + OBM)[tid] = bmv;
}

// entry e (< 27) of one channel's frozen perception bank: feature e / 9 (identity, Sobel-x, Sobel-y),
// tap e % 9 (row-major 3 x 3)
__device__ __forceinline__ float ks_sobel_ref(int e) {
  const int f = e / 9, tap = e % 9, tr = tap / 3, tc = tap % 3;
  if (f == 0) return (tap == 4) ? 1.f : 0.f;
  if (f == 1) return (float)((tc == 0 ? 1 : (tc == 2 ? -1 : 0)) * (tr == 1 ? 2 : 1));
  return (float)((tr == 0 ? 1 : (tr == 2 ? -1 : 0)) * (tc == 1 ? 2 : 1));
}

// A workgroup barrier that orders LDS only (__syncthreads' fence also waits for every outstanding
// global store): where nothing in the launch reads those stores back.  LDS-DMA into LDS is waited
// for with vmcnt by its issuer.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The weight images of a rollout, once, into global memory (K1Args::wimg); one 512-thread block.
__global__ __launch_bounds__(512) void gnca_ks_images(const K1Args a, char* dst) {
  if ((a.flags & kGraphOn) != 0) ks_fill_images<512, true, false>(a, dst, threadIdx.x);
  else ks_fill_images<512, false, false>(a, dst, threadIdx.x);
  // are the perception weights the reference's frozen identity / Sobel bank?  (K1 reads the answer
  // with the images instead of reducing it per launch)
  constexpr KSLayout L = ks_layout<24, 36, 4, 4>();
  const int tid = threadIdx.x;
  int ok = 1;
  if (tid < 16 * 27) ok = a.perc[tid] == ks_sobel_ref(tid % 27) ? 1 : 0;
  const int all = __syncthreads_and(ok);
  if (tid == 0) *reinterpret_cast<int*>(dst + (L.pf - L.w1)) = all;
}

#ifndef GNCA_FOLD_ABL
#define GNCA_FOLD_ABL 0   // timing-only builds: 1 = the finalize's loads hit a few cached lines instead
#endif

#ifndef GNCA_K1_SPLIT_NT
#define GNCA_K1_SPLIT_NT 512   // threads per workgroup of the 16-channel split K1 (768: 3 waves per SIMD)
#endif

#ifndef GNCA_K1_PRIO
#define GNCA_K1_PRIO 1   // wave issue priority of K1's groups (s_setprio): below K2's (GNCA_K2_PRIO = 3) so that a
                         // co-resident K2 issues its loads first (round 4: 2 -> 1 with K2 at 3, step 0.4995 -> 0.4912 ms)
#endif

#ifndef GNCA_PREP_PRIO
#define GNCA_PREP_PRIO 2   // the preparer's issue priority while it prepares, one above the groups (K1 0.397 -> 0.384 ms; 0: unchanged)
#endif

#ifndef GNCA_K1_STAGGER
#define GNCA_K1_STAGGER 0   // A/B builds: waves 4-7 (the younger of each SIMD) sleep 64 x N cycles before their first pull of a tile
#endif

#ifndef GNCA_K1_DYNPRIO
#define GNCA_K1_DYNPRIO 0   // A/B builds: a wave raises its issue priority by this much over its group's MFMA section
#endif

#ifndef GNCA_DMA_WAVES
#define GNCA_DMA_WAVES 1   // A/B builds: waves (the first failing pulls) sharing the next tile's DMA (3: K1 0.4015-0.4044 vs 0.4008-0.4026 ms with 1)
#endif

// FOLD: 0 = the plain K1; 1 / 2 = the fold variant (this launch also finishes the previous step,
// below) on the previous step's dense / compact update field
#ifdef GNCA_K1_MAXVGPR   // A/B builds: a VGPR cap below the occupancy's (room for a co-resident K2 wave)
#define GNCA_K1_VATTR __attribute__((amdgpu_num_vgpr(GNCA_K1_MAXVGPR)))
#else
#define GNCA_K1_VATTR
#endif

#ifndef GNCA_K1_LB
#define GNCA_K1_LB GNCA_K1_SPLIT_NT   // A/B builds: launch bounds above the launched size (a VGPR cap)
#endif

// ZP: the zero-padded shift (graph_augmentation.py's zero_padded_shift): per-sample offset weights
// from K0 and no sender outside the image (the torus-wrapped staging there is multiplied by 0)
template <int TH, int TW, int RY, int RX, int KU, int FOLD = 0, bool ZP = false>
__global__ __launch_bounds__(GNCA_K1_LB, 1) GNCA_K1_VATTR void gnca_k1_split(const K1Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem_b[];
  constexpr int C = 16, HD = 128, NT = GNCA_K1_SPLIT_NT, NW = NT / 64;
  constexpr int RH = TH + 2 * RY, RW = TW + 2 * RX, RHW = RH * RW;
  constexpr int PSTR = ks_pstr(RHW);
  constexpr int NQ = RHW / 4, NI4 = (NQ + 63) / 64;
  constexpr int QW = RW / 4, NQA = RH * QW;
  constexpr int NCELL = TH * TW;
  constexpr KSLayout L = ks_layout<TH, TW, RY, RX, FOLD != 0>();
  static_assert(RW % 4 == 0 && RX % 4 == 0 && TW % 4 == 0, "16-byte staging rows");
  static_assert(RY >= 1 && RX >= 1, "perception halo");
  static_assert(L.total + 512 <= 160 * 1024, "LDS (+ the compiler's static LDS, e.g. __syncthreads_and)");
  static_assert(7 * PSTR * 4 + 4 * RHW < 65536, "channel offsets fit the DS immediate");
  static_assert(TW <= 64, "one ballot per tile row (compact update field)");
  constexpr bool GRAPH = KU > 0;
  static_assert(!ZP || (GRAPH && !FOLD), "the zero-padded shift: graph steps, no fold (K0 runs per step)");
  // The preparer is wave 3, the OLDER wave of SIMD 3 (waves w and w + 4 share SIMD w; the younger
  // one gets the leftover issue slots): it prepares the next tile first, then joins the groups.
  constexpr int PW = 3;

  float* xs = reinterpret_cast<float*>(smem_b + L.xs);
  int* cnt = reinterpret_cast<int*>(smem_b + L.cnt);
  // LDS counters, monotonic over the workgroup's tiles (no resets: every wave's last pull of a tile
  // fails exactly once, so the group counter advances by groups + NW per tile): gctr hands out
  // groups (64 per pull, one per lane), xsd counts groups past their staged-plane reads (64 each)
  int* gctr = cnt + 2;
  int* xsd = cnt + 3;
  int gbase = 0, xbase = 0;
  constexpr int NG = (TH * TW + 31) / 32;
  // fold: finalize items (64 region quads x 4 channels) handed out by fctr; pdone counts the
  // preparer's finished tiles (both monotonic over the workgroup's tiles, as gctr / xsd)
  int* fctr = cnt + 4;
  int* pdone = cnt + 5;
  int fbase = 0;
  constexpr int NQB = (NQ + 63) / 64;
  // 64-cell chunks of a tile; small tiles (the small-batch variants, where the first tile's preparation
  // is on the launch's critical path): the first tile's fire ballots come from idle waves (fdone counts
  // them), one wave per chunk
  constexpr int NCH = (NCELL + 63) / 64;
  constexpr bool SMALLT = NCH <= 4;
  // finalize items: 64 region quads x FCH channels (small tiles: 4, so that a one-tile launch's
  // items spread over the waves)
  constexpr int FCH = SMALLT ? 4 : 8, NFIT = NQB * (C / FCH);
  // the group body (GNCA_K1_LEAN): the classic small tiles take the row-block software pipeline (2),
  // which a wave alone on its SIMD needs to overlap its MFMAs with its VALU (c2 14.0 -> 13.8 us); the
  // graph ones would spill with it (c3 15.9 -> 16.4 us, profiles/r04_ab_small_lean2.txt), and its
  // 250 VGPRs would leave the large tiles no room for the sub-batch pipeline's co-resident K2
  constexpr int LEANV = (GNCA_K1_LEAN >= 1 && SMALLT && KU == 0) ? 2 : GNCA_K1_LEAN;
  // the fold reads the previous step's update field either compact (large batches) or dense NCHW
  // with the dead cells' zeros (small batches)
  constexpr bool CF = FOLD == 2;
  static_assert(!SMALLT || 4 + NCH <= NW, "one fire wave per chunk");
  int* fdone = cnt + 8;
  uint64_t* fbl = reinterpret_cast<uint64_t*>(smem_b + L.fb);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  wg_stamp(a.stamps, 0);
  FPROF_DECL
  ARR_DECL
  if constexpr (FOLD || SMALLT) {   // counters used before the prologue's barrier
    if (tid == 0) {
      if (FOLD) { *fctr = 0; *pdone = 0; cnt[6] = 0; cnt[7] = 0; cnt[9] = 0; cnt[10] = 0; }
      *fdone = 0;
    }
    __syncthreads();
  }
  if (GNCA_K1_PRIO > 0) __builtin_amdgcn_s_setprio(GNCA_K1_PRIO);
  const int h = lane >> 5, r32 = lane & 31, c16 = lane & 15;
  const int H = a.H, W = a.W;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const bool compact = a.rmask != nullptr;
  const bool hz3 = h == 0;   // this lane half holds channel 3 (register r = 3)
  const size_t HW = (size_t)H * W;

  // XCD-aware tile order (as gnca_k1_update)
  const int nxcd = gridDim.x >= 8 ? 8 : 1;
  const int xg_ = blockIdx.x % nxcd, xr_ = blockIdx.x / nxcd;
  const int per_x = (int)(gridDim.x / nxcd) + ((int)(gridDim.x % nxcd) > xg_ ? 1 : 0);
  const int tq = a.total_tiles / nxcd, trm = a.total_tiles % nxcd;
  const int t_begin = xg_ * tq + min(xg_, trm), t_end = (GNCA_ABLATE & kAblTiles) ? t_begin : t_begin + tq + (xg_ < trm ? 1 : 0);

  // the next active tile of this workgroup's sequence after `t` (inactive samples of a masked step
  // get zero GroupNorm partials and no work)
  auto next_active = [&](int t) {
    while (t < t_end && a.active && !a.active[t / a.tps]) {
      if (tid < 2 * NW) a.stats[(size_t)t * 2 * NW + tid] = 0.0;
      t += per_x;
    }
    return t;
  };

  // LDS-DMA staging of a tile's channel planes: 16-byte quads of every plane (torus-wrapped), lanes
  // past the region masked off (the plane pads stay zero).  ZP: a quad outside the image (a quad is
  // inside or outside as a whole, W % TW == 0) stages zeros from gnca_zero16, so that the gather's
  // product with its zero sender byte is an exact 0 as in _shift2d_pad (graph_augmentation.py:85-92),
  // also for a non-finite x across the opposite border (exact by construction; not observable through
  // a whole zero-pad step, whose pooled offset logits are NaN for any non-finite state)
  auto issue_dma = [&](int t, int w0, int wstep) {
    const int b = t / a.tps, tin = t - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const float* xb = a.x + (size_t)b * C * HW;
#pragma unroll 1
    for (int ii_ = w0; ii_ < ((GNCA_ABLATE & kAblStage) ? 0 : NI4); ii_ += wstep) {
      const int q = 64 * ii_ + lane;
      if (q < NQ) {
        const int e = 4 * q, vr = e / RW, vc = e - (e / RW) * RW;
        int ii = i0 - RY + vr, jj = j0 - RX + vc;
        const bool outq = ZP && (ii < 0 || ii >= H || jj < 0 || jj >= W);
        ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
        jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
        const float* src0 = outq ? gnca_zero16 : xb + ii * W + jj;
        const size_t cstr = outq ? 0 : HW;
        float* dst = xs + 256 * ii_;
#pragma unroll 4
        for (int c = 0; c < C; ++c)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src0 + (size_t)c * cstr),
                                           (__attribute__((address_space(3))) void*)(dst + c * PSTR), 16, 0, 0);
      }
    }
  };

  // ---- the fold (FOLD): the previous step's finalize, done here instead of by a K2 pass ----
  // The preparer's part for a tile of sample b at (i0, j0), slot s.  (a) Every load it needs goes out
  // at once: the finalized-alpha band's x_3 and dx_3 (the region plus one ring, RW + 8 columns,
  // quad-aligned: lane = column), the previous step's row tables of the band's <= 3 source tiles per
  // row (compact field; copied to the slot for the finalizers), and the previous step's GroupNorm
  // partials of sample b.  (b) The per-sample GroupNorm constants (K2's fixed-order sums and
  // arithmetic: fin_*).  (c) The finalized alpha x~_3 per band cell as two threshold-bit row masks
  // (ballots).  (d) Their 3x3 OR-pool with the max-pool's -inf border (no neighbour across the image
  // edge, ncagraph.py:85-92) = the region's pre-update alive masks P0 (> alpha_thr) and sender
  // masks P1 (> graph_alpha_thr): exactly the bytes K2 would have handed over.  (e) The
  // sender plane from P1.
  constexpr int PBH = RH + 2, PBW = RW + 8;
  constexpr int FTS = ks_a16(PBH * 3 * 16);   // bytes per slot of the row-table copy
  static_assert(!FOLD || PBW <= 64, "one lane per column of the pooled band");
  static_assert(!FOLD || RX + 4 <= TW, "the band spans at most 3 source tile columns");
  // mode 0: all of it; mode 2: (d) and (e) only, after prep_fold_par's rows (the first tile)
  auto prep_fold = [&](int b, int i0, int j0, int s, int mode) {
    float* fks = reinterpret_cast<float*>(smem_b + L.fk + s * 192);
    uint64_t* p0s = reinterpret_cast<uint64_t*>(smem_b + L.p0 + s * ks_a16(RH * 8));
    uint64_t* p1s = reinterpret_cast<uint64_t*>(smem_b + L.p1);
    uint64_t* pbm = reinterpret_cast<uint64_t*>(smem_b + L.pbm);
    u32x4* fts = reinterpret_cast<u32x4*>(smem_b + L.ft + s * FTS);   // [band row][k]: (m lo, m hi, pre, tile)
    uint32_t* spp = reinterpret_cast<uint32_t*>(smem_b + L.sp + s * L.sp_slot);
    const bool gn = a.use_gn != 0;
    const bool lin = lane < PBW;
    int gcol = j0 - RX - 4 + (lin ? lane : 0);
    gcol = gcol < 0 ? gcol + W : (gcol >= W ? gcol - W : gcol);
    int gc0 = j0 - RX;
    gc0 = gc0 < 0 ? gc0 + W : gc0;
    const int tx0 = gc0 / TW;                         // the source tile column of region column 0
    int kcol = gcol / TW - tx0;
    kcol = kcol < 0 ? kcol + a.tiles_x : kcol;        // this lane's source tile: entry k of a row
    const int tjS = gcol - (gcol / TW) * TW;
    const float* xpa = a.xp + ((size_t)b * C + 3) * HW;
    const float* dpa = CF ? a.dxap + (size_t)b * HW : a.dxp + ((size_t)b * C + 3) * HW;
    FPROF_START();
    if (mode == 2) {   // the band rows come from waves 0..3 (prep_fold_par)
      while (__hip_atomic_load(cnt + 10, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 4)
        __builtin_amdgcn_s_sleep(1);
    } else {
    // (a) every global load of the preparation, issued together (lanes past the band read column
    //     gcol of lane 0: valid, and masked out of the ballots)
    // (the row offset walks in a VGPR: kept per lane, the 2 x PBH row addresses would be scalar
    //  pairs and spill)
#ifdef GNCA_FOLD_PROTO_ALIVE   // timing-only prototype: the band's masks as bytes from memory (wrong results)
    uint32_t xv[PBH];
    {
      int g0 = i0 - RY - 1;
      g0 = g0 < 0 ? g0 + H : g0;
      uint32_t off = (uint32_t)(g0 * W + gcol);
      const uint8_t* alb = a.alive + (size_t)b * HW;
#pragma unroll
      for (int r = 0; r < PBH; ++r) {
        xv[r] = alb[off];
        off += (uint32_t)W;
        off = off >= (uint32_t)HW ? off - (uint32_t)HW : off;
      }
    }
#else
    float xv[PBH], dv[PBH];
    {
      int g0 = i0 - RY - 1;
      g0 = g0 < 0 ? g0 + H : g0;
      uint32_t off = (uint32_t)(g0 * W + gcol);
#pragma unroll
      for (int r = 0; r < PBH; ++r) {
        xv[r] = xpa[off];
        dv[r] = dpa[off];
        off += (uint32_t)W;
        off = off >= (uint32_t)HW ? off - (uint32_t)HW : off;   // the torus wrap of the next row
      }
    }
#endif
    constexpr int NFT = PBH * 3, NFTU = (NFT + 63) / 64;
    uint64_t fm[NFTU];
    uint32_t fp[NFTU], ft_[NFTU];
    if constexpr (CF) {
#pragma unroll
      for (int u = 0; u < NFTU; ++u) {
        const int e = min(64 * u + lane, NFT - 1);
        const int pr = e / 3, k = e - (e / 3) * 3;
        int g = i0 - RY - 1 + pr;
        g = g < 0 ? g + H : (g >= H ? g - H : g);
        const int tyS = g / TH, tiS = g - tyS * TH;
        int txk = tx0 + k;
        txk = txk >= a.tiles_x ? txk - a.tiles_x : txk;
        txk = txk >= a.tiles_x ? txk - a.tiles_x : txk;   // tiles_x may be 1
        const uint32_t tsrc = (uint32_t)(b * a.tps + tyS * a.tiles_x + txk);
        fm[u] = a.rmaskp[(size_t)tsrc * TH + tiS];
        fp[u] = a.rprep[(size_t)tsrc * TH + tiS];
        ft_[u] = tsrc;
      }
    }
    // the previous step's GroupNorm partials of sample b (nst <= 256, host-checked: wave_sum2's
    // single pass) and the affine parameters
    const double* stp = a.statsp + (size_t)b * a.nst * 2;
    double sa[4], sb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = lane + 64 * j;
      const int tc = min(t, a.nst - 1);
      const double pa = stp[2 * tc], pb = stp[2 * tc + 1];
      sa[j] = t < a.nst ? pa : 0.0;
      sb[j] = t < a.nst ? pb : 0.0;
    }
    const int lc = lane < C ? lane : 0;
    const float gam_l = a.gamma ? a.gamma[lc] : 1.f, bet_l = a.beta ? a.beta[lc] : 0.f;
    FPROF_MARK(4);
    // (b) GroupNorm constants
    float mu = 0.f, rs = 1.f;
    if (gn) {
      double t1, t2;
      wave_sum2_regs(sa, sb, &t1, &t2);
      fin_mu_rs(t1, t2, (double)C * (double)HW, a.eps, &mu, &rs);
    }
    const float g3 = gn ? __shfl(gam_l, 3) : 1.f, b3 = gn ? __shfl(bet_l, 3) : 0.f;
    if (lane < C) {
      float sc, sh;
      fin_consts(gn ? gam_l : 1.f, gn ? bet_l : 0.f, mu, rs, gn, &sc, &sh);
      fks[lane] = sc;
      fks[16 + lane] = sh;
    }
    if (lane == 0) {
      fks[32] = mu;
      fks[33] = rs;
      fks[34] = g3;
      fks[35] = b3;
    }
    if constexpr (CF) {
#pragma unroll
      for (int u = 0; u < NFTU; ++u)
        if (64 * u + lane < NFT)
          fts[64 * u + lane] = u32x4{(uint32_t)fm[u], (uint32_t)(fm[u] >> 32), fp[u], ft_[u]};
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    FPROF_MARK(5);
    // (c) the finalized alpha's threshold bits, one ballot pair per band row
    // (the compact field's live bits of this lane's column, all rows read from the slot first)
#ifdef GNCA_FOLD_PROTO_ALIVE
    (void)kcol; (void)tjS; (void)xpa; (void)dpa;
#pragma unroll
    for (int r = 0; r < PBH; ++r) {
      const uint64_t b0 = __ballot(lin && (xv[r] & 1u)), b1 = __ballot(lin && (xv[r] & 2u));
#else
    uint32_t lv[PBH];
#pragma unroll
    for (int r = 0; r < PBH; ++r) {
      lv[r] = 1u;   // dense field: every value is used (a dead cell's is 0)
      if constexpr (CF) lv[r] = (uint32_t)(*reinterpret_cast<const uint64_t*>(&fts[r * 3 + kcol]) >> tjS) & 1u;
    }
    // (every row's updated alpha first: independent chains the scheduler interleaves; then the
    //  ballots, each row's stored right away)
#pragma unroll
    for (int r = 0; r < PBH; ++r) xv[r] = fin_alpha(xv[r], lv[r] != 0 ? dv[r] : 0.f, mu, rs, g3, b3, a.gain, gn);
#pragma unroll
    for (int r = 0; r < PBH; ++r) {
      const float xa = xv[r];
      const uint64_t b0 = __ballot(lin && xa > a.alpha_thr), b1 = __ballot(lin && xa > a.graph_alpha_thr);
#endif
      if (lane == 0) {   // stored right away: no scalar pair stays live past its row
        pbm[r] = b0;
        pbm[PBH + r] = b1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    FPROF_MARK(6);
    }   // mode != 2
    // (d) bit j of nf / nl: band column j is not the image's first / last column (its left / right
    // neighbour in the band is its image neighbour, not the torus wrap)
    const uint64_t nf = __ballot(lin && gcol != 0), nl = __ballot(lin && gcol != W - 1);
    auto hz = [&](uint64_t m) { return m | ((m << 1) & nf) | ((m >> 1) & nl); };
    if (lane < RH) {
      int g = i0 - RY + lane;
      g = g < 0 ? g + H : (g >= H ? g - H : g);
      uint64_t q0 = hz(pbm[lane + 1]), q1 = hz(pbm[PBH + lane + 1]);
      if (g > 0) {
        q0 |= hz(pbm[lane]);
        q1 |= hz(pbm[PBH + lane]);
      }
      if (g < H - 1) {
        q0 |= hz(pbm[lane + 2]);
        q1 |= hz(pbm[PBH + lane + 2]);
      }
      p0s[lane] = q0;
      p1s[lane] = q1;
    }
    // what the finalizers read (the constants, P0, the row tables) is complete: they may start now,
    // beside the rest of this preparation (the sender plane, the keep mask, the live list)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(pdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    FPROF_MARK(7);
    // (e) the sender plane
    if constexpr (GRAPH) {
#pragma unroll 1
      for (int e = lane; e < NQA; e += 64) {   // 4 sender bytes per dword (band column = region column + 4)
        const int vr = e / QW, vc = 4 * (e - (e / QW) * QW);
        const uint32_t bits = (uint32_t)(p1s[vr] >> (vc + 4)) & 15u;
        spp[e] = a2a ? ((bits & 1u) | ((bits & 2u) << 7) | ((bits & 4u) << 14) | ((bits & 8u) << 21)) : 0x01010101u;
      }
    }
    FPROF_MARK(8);
  };

  // The first tile's (a) - (c) of the dense fold on waves 0..3 (one per SIMD), where a one-tile launch
  // has nothing else to do yet: each loads and finalizes the band rows r = wave mod 4 (all loads at
  // once); the preparer alone also sums the GroupNorm partials and publishes the constants (cnt[9]),
  // which the others wait for; every wave counts its rows' ballots in (cnt[10]).  Same arithmetic
  // as prep_fold: the same bits.
  constexpr int PBR = (PBH + 3) / 4;
  auto prep_fold_par = [&](int b, int i0, int j0) {
    float* fks = reinterpret_cast<float*>(smem_b + L.fk);
    uint64_t* pbm = reinterpret_cast<uint64_t*>(smem_b + L.pbm);
    const bool gn = a.use_gn != 0;
    const bool lin = lane < PBW;
    int gcol = j0 - RX - 4 + (lin ? lane : 0);
    gcol = gcol < 0 ? gcol + W : (gcol >= W ? gcol - W : gcol);
    const float* xpa = a.xp + ((size_t)b * C + 3) * HW;
    const float* dpa = a.dxp + ((size_t)b * C + 3) * HW;
    int g0 = i0 - RY - 1 + wave;
    g0 = g0 < 0 ? g0 + H : (g0 >= H ? g0 - H : g0);
    float xv[PBR], dv[PBR];
#pragma unroll
    for (int k = 0; k < PBR; ++k) {
      xv[k] = 0.f;
      dv[k] = 0.f;
      if (wave + 4 * k < PBH) {
        int g = g0 + 4 * k;
        g = g >= H ? g - H : g;
        g = g >= H ? g - H : g;   // H may be < 8
        xv[k] = xpa[g * W + gcol];
        dv[k] = dpa[g * W + gcol];
      }
    }
    if (wave == PW) {
      const double* stp = a.statsp + (size_t)b * a.nst * 2;
      double sa[4], sb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = lane + 64 * j;
        const int tc = min(t, a.nst - 1);
        const double pa = stp[2 * tc], pb = stp[2 * tc + 1];
        sa[j] = t < a.nst ? pa : 0.0;
        sb[j] = t < a.nst ? pb : 0.0;
      }
      const int lc = lane < C ? lane : 0;
      const float gam_l = a.gamma ? a.gamma[lc] : 1.f, bet_l = a.beta ? a.beta[lc] : 0.f;
      float mu = 0.f, rs = 1.f;
      if (gn) {
        double t1, t2;
        wave_sum2_regs(sa, sb, &t1, &t2);
        fin_mu_rs(t1, t2, (double)C * (double)HW, a.eps, &mu, &rs);
      }
      const float g3 = gn ? __shfl(gam_l, 3) : 1.f, b3 = gn ? __shfl(bet_l, 3) : 0.f;
      if (lane < C) {
        float sc, sh;
        fin_consts(gn ? gam_l : 1.f, gn ? bet_l : 0.f, mu, rs, gn, &sc, &sh);
        fks[lane] = sc;
        fks[16 + lane] = sh;
      }
      if (lane == 0) {
        fks[32] = mu;
        fks[33] = rs;
        fks[34] = g3;
        fks[35] = b3;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(cnt + 9, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      while (__hip_atomic_load(cnt + 9, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        __builtin_amdgcn_s_sleep(1);
    }
    const float mu = fks[32], rs = fks[33], g3 = fks[34], b3 = fks[35];
#pragma unroll
    for (int k = 0; k < PBR; ++k) {
      const int r = wave + 4 * k;
      if (r >= PBH) continue;
      const float xa = fin_alpha(xv[k], dv[k], mu, rs, g3, b3, a.gain, gn);
      const uint64_t b0 = __ballot(lin && xa > a.alpha_thr), b1 = __ballot(lin && xa > a.graph_alpha_thr);
      if (lane == 0) {
        pbm[r] = b0;
        pbm[PBH + r] = b1;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(cnt + 10, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };

  // The finalize of tile t's staged region (slot s: its constants, P0 and row tables), into the
  // staging buffer and, for the tile's own cells, into xo: x = x_prev + tanh(GN(dx_prev)) * gain
  // (alpha: the updated alpha times the post-update gate P0), K2's arithmetic value for value.
  // Items of 64 region quads x all 16 channels are pulled from fctr by every wave that gets here; an
  // item's loads (16 x_prev quads and the quad's packed dx of every channel: one memory round trip,
  // the row tables come from the slot) are issued before the wait for the staging buffer to be free
  // (every group of the current tile past its staged reads), so they overlap the other waves' last
  // groups.
  // wait_xsd: the staging buffer still holds the current tile (groups qe, live list lstc, group
  // done-mask cnt[6 + parc]): an item overwrites its rows once every group that may read them is past
  // its staged reads (the groups' cells are in row order, so the top rows free up first)
  static_assert(!FOLD || NG <= 32, "one done bit per group");
  auto finalize = [&](int t, int s, int need_prep, bool wait_xsd, int qe, const uint16_t* lstc, int parc) {
    const int b = t / a.tps, tin = t - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    FPROF_START();
    // the preparer's slot s (constants, P0, row tables) is read only after the wait below; an item's
    // loads of the previous step's x (and dense dx) go out before it
    bool prepared = false;
    auto wait_prep = [&]() {
      if (!prepared)
        while (__hip_atomic_load(pdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need_prep)
          __builtin_amdgcn_s_sleep(1);
      if (!prepared) FPROF_MARK(0);
      prepared = true;
    };
    const float* fks = reinterpret_cast<const float*>(smem_b + L.fk + s * 192);
    const uint64_t* p0s = reinterpret_cast<const uint64_t*>(smem_b + L.p0 + s * ks_a16(RH * 8));
    const u32x4* fts = reinterpret_cast<const u32x4*>(smem_b + L.ft + s * FTS);
    const bool gn = a.use_gn != 0;
    const float g2 = -2.f * a.gain;
    int gc0 = j0 - RX;
    gc0 = gc0 < 0 ? gc0 + W : gc0;
    const int tx0 = gc0 / TW;
    // lane q: the tile row of group q's first cell (the least row it reads, in region rows)
    const int grow = (wait_xsd && lane < qe) ? lstc[32 * lane] / TW : 0;
#pragma unroll 1
    for (;;) {
      const int it = (__builtin_amdgcn_readfirstlane(atomicAdd(fctr, 1)) >> 6) - fbase;
      if (it >= NFIT) break;
      const int c0 = FCH * (it % (C / FCH));
      const int q = 64 * (it / (C / FCH)) + lane;
      const bool qv = q < NQ;
      const int vr = qv ? q / QW : 0, vq = qv ? q - (q / QW) * QW : 0;
      int g = i0 - RY + vr, gc = j0 - RX + 4 * vq;
      g = g < 0 ? g + H : (g >= H ? g - H : g);
      gc = gc < 0 ? gc + W : (gc >= W ? gc - W : gc);
      const size_t cell = (size_t)g * W + gc;
      f4 xq[FCH];
#if GNCA_FOLD_ABL & 1   // timing only: no finalize loads (wrong results)
      const size_t cell_ = (size_t)(lane & 3);
#define GNCA_FCELL cell_
#else
#define GNCA_FCELL cell
#endif
#pragma unroll
      for (int u = 0; u < FCH; ++u) xq[u] = *reinterpret_cast<const f4*>(a.xp + ((size_t)b * C + c0 + u) * HW + GNCA_FCELL);
      float dv[FCH][4];
      uint32_t bits = 15u;   // dense field: every value is used (a dead cell's is 0)
      if constexpr (!CF) {
#pragma unroll
        for (int u = 0; u < FCH; ++u) {
          const f4 d4 = *reinterpret_cast<const f4*>(a.dxp + ((size_t)b * C + c0 + u) * HW + GNCA_FCELL);
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) dv[u][kk] = d4[kk];
        }
      }
      wait_prep();
      if constexpr (CF) {
        int k = gc / TW - tx0;
        k = k < 0 ? k + a.tiles_x : k;
        const u32x4 e = fts[(vr + 1) * 3 + k];
        const uint64_t m = ((uint64_t)e[1] << 32) | e[0];
        const int tjS = gc - (gc / TW) * TW;
        // the quad's live cells are consecutive in the source tile's packed field: cell k's value
        // (or, for a dead cell, the next live one's; never used) at rank r0 + (live cells before k)
        bits = (uint32_t)(m >> tjS) & 15u;
        const uint32_t r0 = e[3] * (uint32_t)(C * NCELL) + e[2] + (uint32_t)__popcll(m & ((1ull << tjS) - 1ull));
        uint32_t off[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) off[kk] = (GNCA_FOLD_ABL & 1) ? (uint32_t)(lane & 3) : r0 + (uint32_t)__popc(bits & ((1u << kk) - 1u));
#pragma unroll
        for (int u = 0; u < FCH; ++u) {
          const int c = c0 + u;
          if (c == 3) {
            const f4 d4 = *reinterpret_cast<const f4*>(a.dxap + (size_t)b * HW + GNCA_FCELL);
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) dv[u][kk] = d4[kk];
          } else {
            const float* fb = a.dxp + (size_t)c * NCELL;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) dv[u][kk] = fb[off[kk]];
          }
        }
      }
      const float mu = fks[32], rs = fks[33], g3 = fks[34], b3 = fks[35];
      if (wait_xsd) {
        const int rhi = min(RH - 1, (64 * (it / (C / FCH)) + 63) / QW);   // the item's last region row
        const uint32_t need = (uint32_t)__ballot(lane < qe && grow <= rhi);
        while ((__hip_atomic_load(cnt + 6 + parc, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) & need) != need)
          __builtin_amdgcn_s_sleep(1);
      }
      FPROF_MARK(1);
      FPROF_COUNT(3);
      const bool own = vr >= RY && vr < RY + TH && vq >= RX / 4 && vq < (RX + TW) / 4;
      const uint64_t pm = p0s[vr] >> (4 * vq + 4);
      // every channel's values in one straight block (no per-channel branch), then the stores
#pragma unroll
      for (int u = 0; u < FCH; ++u) {
        const int c = c0 + u;
        if (c == 3) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const float xa = fin_alpha(xq[u][kk], ((bits >> kk) & 1u) ? dv[u][kk] : 0.f, mu, rs, g3, b3, a.gain, gn);
            xq[u][kk] = xa * (((pm >> kk) & 1ull) ? 1.f : 0.f);
          }
        } else {
          const float sc = fks[c], sh = fks[16 + c];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            xq[u][kk] = k2_update(xq[u][kk], ((bits >> kk) & 1u) ? dv[u][kk] : 0.f, sc, sh, a.gain, g2);
        }
      }
      // lanes past the region write their quad into the (unused) alive-byte area instead: no branch
      float* const xdummy = reinterpret_cast<float*>(smem_b + L.ab) + 4 * (lane & 15);
#pragma unroll
      for (int u = 0; u < FCH; ++u) *reinterpret_cast<f4*>(qv ? xs + (c0 + u) * PSTR + 4 * q : xdummy) = xq[u];
      if (own && qv) {
        float* ob = a.xo + ((size_t)b * C + c0) * HW + cell;
#pragma unroll
        for (int u = 0; u < FCH; ++u) *reinterpret_cast<f4*>(ob + (size_t)u * HW) = xq[u];
      }
      FPROF_MARK(2);
    }
    fbase += NFIT + NW;
  };

  // The preparer (one wave, no workgroup barrier): a tile's sender plane over the region, its keep
  // mask (fire AND pre-alive) and live-cell list into slot `s`; the compact field's row tables and
  // the dead cells' zeros go to global memory.  The pre-update masks are the alive bytes (K2's
  // hand-over in a rollout, else gnca_k_alive over this step's alpha plane).
  // pf: the fire ballots of this tile are (being) written to fbl by other waves (the first small tile)
  // rows_done: the fold's band rows of this tile were prepared by waves 0..3 (prep_fold_par)
  auto prep = [&](int t, int s, bool pf, bool rows_done) {
    if (GNCA_PREP_PRIO > 0) __builtin_amdgcn_s_setprio(GNCA_PREP_PRIO);
    const int b = t / a.tps, tin = t - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    uint32_t* spp = reinterpret_cast<uint32_t*>(smem_b + L.sp + s * L.sp_slot);
    uint16_t* lstp = reinterpret_cast<uint16_t*>(smem_b + L.lst + s * L.lst_slot);
    uint32_t* abw = reinterpret_cast<uint32_t*>(smem_b + L.ab);
    const uint8_t* abq = reinterpret_cast<const uint8_t*>(smem_b + L.ab);
    uint64_t* cb = reinterpret_cast<uint64_t*>(smem_b + L.cb + s * L.cb_slot);
    // (1) the region's alive bytes, 4 columns per dword, all loads in flight together (fold: the
    //     masks from the finalized alpha, prep_fold)
    const uint64_t* p0q = reinterpret_cast<const uint64_t*>(smem_b + L.p0 + s * ks_a16(RH * 8));
    if constexpr (FOLD) {
      prep_fold(b, i0, j0, s, rows_done ? 2 : 0);
    } else {
      const uint8_t* alb = a.alive + (size_t)b * HW;
      constexpr int NU = (NQA + 63) / 64;
      uint32_t v[NU];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int e = 64 * u + lane;
        v[u] = 0u;
        if (e < NQA) {
          const int vr = e / QW, vc = 4 * (e - (e / QW) * QW);
          int ii = i0 - RY + vr, jj = j0 - RX + vc;
          // (ZP: a quad is inside the image or outside it as a whole, W % TW == 0)
          if (ZP && (ii < 0 || ii >= H || jj < 0 || jj >= W)) v[u] = 0x80000000u;   // (marker: no sender)
          ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
          jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
          if (!ZP || v[u] == 0u) v[u] = *reinterpret_cast<const uint32_t*>(alb + ii * W + jj);
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int e = 64 * u + lane;
        if (e < NQA) {
          const bool out = ZP && v[u] == 0x80000000u;
          abw[e] = out ? 0u : v[u];
          if constexpr (GRAPH)   // 4 sender bytes
            spp[e] = out ? 0u : (a2a ? (v[u] >> 1) & 0x01010101u : 0x01010101u);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (2) keep = fire AND pre-alive per 64-cell chunk; live cells listed in cell order
    int nl = 0;
    // small tiles: every chunk's alive byte read at once and the loop unrolled
    constexpr int CUNR = SMALLT ? 4 : 1;
    uint32_t cab[SMALLT ? NCH : 1];
    if constexpr (SMALLT && !FOLD) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int n = 64 * ch + lane;
        const int ti = n / TW, tj = n - (n / TW) * TW;
        cab[ch] = n < NCELL ? abq[(ti + RY) * RW + tj + RX] : 0u;
      }
    }
#pragma unroll CUNR
    for (int n0 = 0; n0 < NCELL; n0 += 64) {
      const int n = n0 + lane;
      const bool inb = n < NCELL;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const size_t cell = (size_t)(i0 + ti) * W + (j0 + tj);
      bool live = false;
      const uint32_t ab_ = FOLD ? (inb ? (uint32_t)(p0q[ti + RY] >> (tj + RX + 4)) & 1u : 0u)
                                : SMALLT ? cab[SMALLT ? (n0 >> 6) : 0] : (inb ? abq[(ti + RY) * RW + tj + RX] : 0u);
      if (SMALLT && pf) {
        if (n0 == 0)
          while (__hip_atomic_load(fdone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NCH)
            __builtin_amdgcn_s_sleep(1);
        live = inb && (ab_ & 1u) && ((fbl[n0 >> 6] >> lane) & 1ull);
      } else if (inb && (ab_ & 1u)) {
        live = (GNCA_ABLATE & kAblFire) ? ((cell & 1) != 0)
                                        : fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step,
                                                  a.sample_base, b, HW, cell);
      }
      const uint64_t bal = __ballot(live);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) cb[n0 >> 6] = bal;
      if (compact && inb && tj == 0) a.rpre[(size_t)t * TH + ti] = (uint32_t)(nl + pre);
      if (live) lstp[nl + pre] = (uint16_t)n;
      // (a dense field's dead cells get their zeros after the tile's groups: zero_item)
      nl += __popcll(bal);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (3) per-row live masks of the compact update field, from the chunk ballots
    if (compact) {
#pragma unroll 1
      for (int ti = lane; ti < TH; ti += 64) {
        const int f = ti * TW, c0 = f >> 6, sh = f & 63;
        uint64_t m = cb[c0] >> sh;
        if (sh + TW > 64) m |= cb[c0 + 1] << (64 - sh);
        if (TW < 64) m &= (1ull << TW) - 1ull;
        a.rmask[(size_t)t * TH + ti] = m;
      }
    }
    if (lane == 0) cnt[s] = nl;
    if constexpr (FOLD) FPROF_MARK(9);
    if (GNCA_PREP_PRIO > 0) __builtin_amdgcn_s_setprio(GNCA_K1_PRIO);
  };

  // A dense update field's zeros at the dead cells of the tile at outb (slot s's keep ballots): item z
  // = (64-cell chunk z / 4, channels 4 (z % 4) .. + 3), pulled after the tile's groups by the waves
  // without a group (off the preparer, whose first tile is on a small launch's critical path)
  auto zero_item = [&](int z, int s, float* outb) {
    const uint64_t* cbs = reinterpret_cast<const uint64_t*>(smem_b + L.cb + s * L.cb_slot);
    const int ch = z >> 2, c0 = 4 * (z & 3);
    const int n = 64 * ch + lane;
    const int ti = n / TW, tj = n - (n / TW) * TW;
    if (n < NCELL && !((cbs[ch] >> lane) & 1ull)) {
      float* oz = outb + (size_t)ti * W + tj + (size_t)c0 * HW;
#pragma unroll
      for (int c = 0; c < 4; ++c) oz[(size_t)c * HW] = 0.f;
    }
  };

  PROF_DECL
  int tile = next_active(t_begin + xr_);
  // Prologue (what a small batch's launch waits out): the first tile's DMA, the preparer's planes of
  // that tile, then every weight load of this thread in flight together, then the weight images'
  // splits and LDS stores (B=8 72^2 K1: 20.0 -> 19.8 us; the preparer after the weight loads 22.3 us)
  if (!FOLD && tile < t_end) issue_dma(tile, wave, NW);
  if constexpr (SMALLT) {   // the first tile's fire ballots, chunk wave - 4 (waves 4.. of SIMDs 0..)
    if (wave >= 4 && wave < 4 + NCH && tile < t_end) {
      const int b = tile / a.tps, tin = tile - b * a.tps;
      const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
      const int n = 64 * (wave - 4) + lane;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const size_t cell = (size_t)(ty * TH + ti) * W + (tx * TW + tj);
      bool f = false;
      if (n < NCELL)
        f = (GNCA_ABLATE & kAblFire) ? ((cell & 1) != 0)
                                     : fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step, a.sample_base, b,
                                               HW, cell);
      const uint64_t bal = __ballot(f);
      if (lane == 0) {
        fbl[wave - 4] = bal;
        __hip_atomic_fetch_add(fdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  PROF_MARK(0);   // (prologue) first tile's DMA issue
  ARR_MARK(0);    // first DMA + fire ballots issued
  constexpr bool PAR_ROWS = FOLD && !CF;   // the dense fold (small batches): band rows on waves 0..3
  if constexpr (PAR_ROWS) {
    if (wave < 4 && tile < t_end) {
      const int b = tile / a.tps, tin = tile - b * a.tps;
      const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
      prep_fold_par(b, ty * TH, tx * TW);
    }
  }
  if (wave == PW && tile < t_end) prep(tile, 0, SMALLT, PAR_ROWS);
  PROF_MARK(3);   // (prologue) first tile's prep
  ARR_MARK(1);
  float pcv = 0.f;
  if (!a.wimg && tid < C * 27) pcv = a.perc[tid];
  if (tid == 0) { *gctr = 0; *xsd = 0; }
  if (!(GNCA_ABLATE & kAblFill)) {
    if (a.wimg) {
      // the rollout's weight images, built once (gnca_ks_images): one LDS-DMA copy of the block (the
      // fold: by waves 4.. only, each waiting for its copies before the finalize, so that no wave
      // has to wait for its finalize's stores of x at the prologue's barrier)
      constexpr int NQI = (L.total - L.w1) / 16;
      static_assert((L.total - L.w1) % 16 == 0 && L.w1 % 16 == 0, "16-byte image block");
      const int w0 = FOLD ? 4 : 0;
      if (wave >= w0) {
#pragma unroll 1
        for (int i = wave - w0; i < (NQI + 63) / 64; i += NW - w0) {
          const int q = 64 * i + lane;
          if (q < NQI)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a.wimg + 16 * q),
                                             (__attribute__((address_space(3))) void*)(smem_b + L.w1 + 1024 * i), 16, 0, 0);
        }
        if (FOLD) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      ks_fill_images<NT, GRAPH, true>(a, smem_b + L.w1, tid);
    }
    // the perception zero tap: every channel plane's pad floats (never written by the staging)
    for (int e = tid; e < 16 * (PSTR - RHW); e += NT) xs[(e / (PSTR - RHW)) * PSTR + RHW + e % (PSTR - RHW)] = 0.f;
  }
  PROF_MARK(2);   // (prologue) weight image copy / fill issue
  if constexpr (FOLD) {   // the first tile's region: finalized by every wave (nothing to wait for)
    if (tile < t_end) finalize(tile, 0, 1, false, 0, nullptr, 0);
  }
  ARR_MARK(2);
  // the staging DMA and the images have landed (the fold with images: waited for above)
  if (!(FOLD && a.wimg)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PROF_MARK(1);   // (prologue) wait for the DMA, images and weight loads
  // perception weights == the reference's frozen identity/Sobel bank? (one uniform branch; the
  // other case reads the weights from global memory, an uncommon slow path)
  bool sobel;
  if (a.wimg) {   // the images carry the answer (gnca_ks_images)
    // the barrier after the images, DMA and prep: LDS only in the fold, whose finalize stores of x
    // need not complete here (the staging DMA and the images were waited for above)
    if (FOLD) lds_barrier();
    else __syncthreads();
    sobel = *reinterpret_cast<const int*>(smem_b + L.pf) != 0;
  } else {
    int ok = 1;
    if (tid < C * 27 && pcv != ks_sobel_ref(tid % 27)) ok = 0;
    sobel = __syncthreads_and(ok) != 0;   // also the barrier after the images, DMA and prep
  }
  ARR_MARK(3);

  // per-lane LDS offsets of the message fragments (stacks [M0;M1], [M2;0], [M0;0], read per
  // group: kept out of the registers the group loop needs) and of the message bias of this lane's 8
  // output channels c = (r&3) + 8(r>>2) + 4h; ones for the bias MFMA
  const int ent_ = (h * 16 + c16) * 16;
  const int wmA_o = L.wm + (r32 < 16 ? 0 : 512) + ent_;
  const int wmB_o = (r32 < 16 ? L.wm + 1024 : L.wz) + ent_;
  const int wmC_o = (r32 < 16 ? L.wm : L.wz) + ent_;
  const int bml_o = L.bml + h * 32;
  // GEMM1's accumulator starts at the bias (exactly the fp32 b1, as a bias MFMA over its three
  // bf16 parts gave: one ds_read_b128 x 4 instead of an MFMA per row block)
  auto bias_acc = [&](int rb) { return *reinterpret_cast<const f32x16*>(smem_b + L.bias + rb * 128 + h * 64); };
  // message gain: 0 for the RGBA channels (c < 4: h == 0, r < 4) under hidden_only
  const float mgain = GRAPH ? a.message_gain : 0.f;
  const bool hz = hidden_only && h == 0;
  // W2 A-fragment lane bases: T0 = [P0;P1], T1 = [P2;P2] (+ s * 512 per k-chunk)
  const int w2T0 = L.w2 + (r32 < 16 ? 0 : 4096) + (h * 16 + c16) * 16;
  const int w2T1 = L.w2 + 8192 + (h * 16 + c16) * 16;

  // Tile pipeline: [groups of tile t | the preparer then fills slot par^1 for tile t+1] -> barrier
  // -> LDS-DMA of tile t+1's channel planes -> wait -> barrier.  The per-tile planes and the
  // compaction run on the preparer wave beside the other waves' groups instead of between them.
  int par = 0;
  int iter = 0;
  while (tile < t_end) {
    PROF_MARK(7);
    const int nxt = next_active(tile + per_x);
    const int b = tile / a.tps, tin = tile - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const size_t cell0 = (size_t)i0 * W + j0;
    float* outb = a.out + (size_t)b * C * HW + cell0;
    const uint8_t* sp = reinterpret_cast<const uint8_t*>(smem_b + L.sp + par * L.sp_slot);
    const uint16_t* lst = reinterpret_cast<const uint16_t*>(smem_b + L.lst + par * L.lst_slot);
    const int nlive = cnt[par];

    if (wave == PW && nxt < t_end && !(GNCA_ABLATE & kAblPrep)) prep(nxt, par ^ 1, false, false);
    PROF_MARK(3);   // preparer

    // ---- 32-cell groups, pulled from an LDS counter (the faster, older wave of a SIMD takes more);
    //      each group's GroupNorm partials go to pg[q], so the sums do not depend on which wave ran it ----
    const int qend = (nlive + 31) >> 5;
    double* pg = reinterpret_cast<double*>(smem_b + L.pg) + par * 2 * NG;
    auto pull = [&]() { return (__builtin_amdgcn_readfirstlane(atomicAdd(gctr, 1)) >> 6) - gbase; };
    const bool img_top = i0 == 0, img_bot = i0 + TH == H, img_lft = j0 == 0, img_rgt = j0 + TW == W;
    // (every lane adds 1: the wave's 64 increments are one LDS instruction, so the counter moves by
    //  64 per pull and any lane's old value >> 6 is the pulled group)
    if (GNCA_K1_STAGGER > 0 && wave >= 4) __builtin_amdgcn_s_sleep(GNCA_K1_STAGGER);
    int q = pull();
#pragma unroll 1
    for (; q < qend; q = pull()) {
      float s1 = 0.f, s2 = 0.f;
      const int gi = 32 * q + r32;
      const bool valid = gi < nlive;
      const int n = lst[valid ? gi : 0];
      const int ti = n / TW, tj = n - (n / TW) * TW;
      // (GNCA_ABLATE & 8192: timing only, conflict-free stand-in addresses: lane r32 reads region
      //  cell RY*RW + RX + r32, so the 32 lanes of a half hit 32 distinct banks for every tap)
      const int pidx = (GNCA_ABLATE & 8192) ? RY * RW + RX + r32 : (RY + ti) * RW + (RX + tj);
      const int hb = 8 * h * PSTR;          // this lane's channel half
      const int relcell = ti * W + tj;

      // GEMM2's accumulator (the lean bodies: seeded with the message term)
      f32x16 acc2 = {};
      // -- gather of alive-masked x, channels 8h..8h+7 (uniform weight 1/k, applied once) --
      u32x4 g0 = {0u, 0u, 0u, 0u}, g1 = g0, g2 = g0;
      float S = 0.f;
      if constexpr (GRAPH) if (!(GNCA_ABLATE & kAblGather)) {
        float gv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = 0.f;
        const float* xq = xs + hb + pidx;
        const uint8_t* spq = sp + pidx;
        if (GNCA_K1_PIPE_LDS && !(GNCA_ABLATE & 4096)) {
          ks_gather8<KU, PSTR, ZP>(a.odl, xq, spq, gv, S, ZP ? a.offw + (size_t)b * KU : nullptr);
        } else {
#pragma unroll
          for (int o = 0; o < KU; ++o) {
            const int d = a.odl[o];
            const float s_ = ZP ? a.offw[(size_t)b * KU + o] * (float)spq[-d] : (float)spq[-d];
            S += s_;
            const float* xo = xq - d;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              // (GNCA_ABLATE & 4096: timing only, one channel's read stands in for all eight)
              float xv_ = xo[(GNCA_ABLATE & 4096) ? 0 : j * PSTR];
              if (GNCA_ABLATE & 4096) asm volatile("" : "+v"(xv_));
              gv[j] = fmaf(s_, xv_, gv[j]);
            }
          }
        }
        if constexpr (!ZP) {
          const float wu = a.uniform_w;
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] *= wu;
          S *= wu;
        }
        split3_x8(gv, g0, g1, g2);
        // materialise here (before the perception's sobel / generic branch): otherwise the
        // gather arithmetic is sunk past the branch and its loaded floats stay live longer
        asm volatile("" : "+v"(g0), "+v"(g1), "+v"(g2), "+v"(S));
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (GRAPH && LEANV == 3) {
        // the message right after the gather (its operands die before the perception's live):
        // M = WM.G, then tanh(M + bm S) * gain seeds GEMM2's accumulator (top half; bottom 0)
        f32x16 accm = {};
        if (!(GNCA_ABLATE & kAblMfma)) {
          const u32x4 wmA = *reinterpret_cast<const u32x4*>(smem_b + wmA_o);
          accm = mfma_bx(wmA, g0, accm);
          const u32x4 wmB = *reinterpret_cast<const u32x4*>(smem_b + wmB_o);
          accm = mfma_bx(wmB, g0, accm);
          accm = mfma_bx(wmA, g1, accm);
          const u32x4 wmC = *reinterpret_cast<const u32x4*>(smem_b + wmC_o);
          accm = mfma_bx(wmC, g2, accm);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float bm_ = reinterpret_cast<const float*>(smem_b + bml_o)[r];
          acc2[r] = fast_tanh(fmaf(bm_, S, accm[r] + accm[r + 8])) * ((hz && r < 4) ? 0.f : mgain);
        }
        __builtin_amdgcn_sched_barrier(0);
      }

      // -- perception of channels 8h..8h+7 (zero padding at the image border via zero taps) --
      float y0[8], y1[8], y2[8];
      {
        const int ic = i0 + ti, jc = j0 + tj;
        const bool up = !(img_top && ic == 0), dn = !(img_bot && ic == H - 1);
        const bool lf = !(img_lft && jc == 0), rt = !(img_rgt && jc == W - 1);
        const int zt = RHW + hb;    // the zero tap of this lane's first channel plane
        const int bc = pidx + hb;
        const int t0 = (up && lf) ? bc - RW - 1 : zt, t1 = up ? bc - RW : zt, t2 = (up && rt) ? bc - RW + 1 : zt;
        const int t3 = lf ? bc - 1 : zt, t5 = rt ? bc + 1 : zt;
        const int t6 = (dn && lf) ? bc + RW - 1 : zt, t7 = dn ? bc + RW : zt, t8 = (dn && rt) ? bc + RW + 1 : zt;
        if (GNCA_ABLATE & kAblPerceive) {
#pragma unroll
          for (int j = 0; j < 8; ++j) y0[j] = y1[j] = y2[j] = 0.f;
        } else if (sobel && GNCA_K1_PIPE_LDS && !(GNCA_ABLATE & 4096)) {
          const int tt[9] = {t0, t1, t2, t3, bc, t5, t6, t7, t8};
          ks_sobel8<PSTR>(xs, tt, y0, y1, y2);
        } else if (sobel) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int co = (GNCA_ABLATE & 4096) ? 0 : j * PSTR;
            float n0 = xs[t0 + co], n1 = xs[t1 + co], n2 = xs[t2 + co];
            float n3 = xs[t3 + co], n4 = xs[bc + co], n5 = xs[t5 + co];
            float n6 = xs[t6 + co], n7 = xs[t7 + co], n8 = xs[t8 + co];
            if (GNCA_ABLATE & 4096)
              asm volatile("" : "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3), "+v"(n4), "+v"(n5), "+v"(n6), "+v"(n7), "+v"(n8));
            y0[j] = n4;
            // Sobel-x / -y with shared diagonal differences: 8 VALU instead of 10
            const float dg = n0 - n8, da = n2 - n6;
            y1[j] = fmaf(2.f, n3 - n5, dg - da);
            y2[j] = fmaf(2.f, n1 - n7, dg + da);
          }
        } else {
#pragma unroll 1
          for (int j = 0; j < 8; ++j) {
            const int co = j * PSTR;
            const float nn[9] = {xs[t0 + co], xs[t1 + co], xs[t2 + co], xs[t3 + co], xs[bc + co],
                                 xs[t5 + co], xs[t6 + co], xs[t7 + co], xs[t8 + co]};
            const float* pw = a.perc + (size_t)3 * (8 * h + j) * 9;
            float acc3[3];
#pragma unroll
            for (int f = 0; f < 3; ++f) {
              float acc = pw[9 * f] * nn[0];
#pragma unroll
              for (int t = 1; t < 9; ++t) acc = fmaf(pw[9 * f + t], nn[t], acc);
              acc3[f] = acc;
            }
            y0[j] = acc3[0];
            y1[j] = acc3[1];
            y2[j] = acc3[2];
          }
        }
      }
      u32x4 yf[3][3];   // [kc][part]
      split3_x8(y0, yf[0][0], yf[0][1], yf[0][2]);
      split3_x8(y1, yf[1][0], yf[1][1], yf[1][2]);
      split3_x8(y2, yf[2][0], yf[2][1], yf[2][2]);
      // this group's reads of the staged planes are done (release: they stay before the count)
      __hip_atomic_fetch_add(xsd, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if constexpr (FOLD) __hip_atomic_fetch_or(cnt + 6 + par, 1 << q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      PROF_MARK(2);   // pull + gather + perception + splits
      if (GNCA_K1_DYNPRIO > 0) __builtin_amdgcn_s_setprio(GNCA_K1_PRIO + GNCA_K1_DYNPRIO);
      if (GNCA_ABLATE & kAblMfma) {
#pragma unroll
        for (int kc = 0; kc < 3; ++kc) asm volatile("" ::"v"(yf[kc][0]), "v"(yf[kc][1]), "v"(yf[kc][2]));
      }

#if GNCA_K1_LEAN
      if constexpr (LEANV == 3) {
      // -- GEMM1 row block rb into ONE accumulator, then its ReLU / split and its two GEMM2 k-chunks,
      //    the row blocks strictly one after another (fenced): the fewest registers live, so that
      //    three K1 waves share a SIMD (768 threads) and the other waves hide each chain's latency.
      //    Same products in the same order as the other bodies: the same bits. --
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          f32x16 ac;
          if (GNCA_ABLATE & kAblMfma) {
            ac = f32x16{};
          } else {
            ac = bias_acc(rb);
#pragma unroll
            for (int kc = 0; kc < 3; ++kc) {
              const int img = L.w1 + (rb * 3 + kc) * 1024 + lane * 16;
              const u32x4 a0 = *reinterpret_cast<const u32x4*>(smem_b + img);
              const u32x4 a1 = *reinterpret_cast<const u32x4*>(smem_b + img + 12288);
              const u32x4 a2 = *reinterpret_cast<const u32x4*>(smem_b + img + 24576);
              ac = mfma_bx(a0, yf[kc][0], ac);
              ac = mfma_bx(a0, yf[kc][1], ac);
              ac = mfma_bx(a1, yf[kc][0], ac);
              ac = mfma_bx(a0, yf[kc][2], ac);
              ac = mfma_bx(a2, yf[kc][0], ac);
              ac = mfma_bx(a1, yf[kc][1], ac);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
#pragma unroll
          for (int ss = 0; ss < 2; ++ss) {
            const int s = 2 * rb + ss;
            float hv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) hv[j] = relu_nan(ac[8 * ss + j]);
            u32x4 h0, h1, h2;
            split3_x8(hv, h0, h1, h2);
            if (GNCA_ABLATE & kAblMfma) {
              asm volatile("" ::"v"(h0), "v"(h1), "v"(h2));
              continue;
            }
            const u32x4 T0 = *reinterpret_cast<const u32x4*>(smem_b + w2T0 + s * 512);
            const u32x4 T1 = *reinterpret_cast<const u32x4*>(smem_b + w2T1 + s * 512);
            acc2 = mfma_bx(T0, h0, acc2);
            acc2 = mfma_bx(T1, h0, acc2);
            acc2 = mfma_bx(T0, h1, acc2);
            acc2 = mfma_bx(T0, h2, acc2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      } else if constexpr (LEANV >= 2) {
      // -- The group's GEMMs as a software pipeline over the row blocks: stage rb issues row block
      //    rb + 1's GEMM1 chain (bias + 18 products into acc1[(rb + 1) & 1]) two MFMAs at a time,
      //    each pair fenced together with one piece of row block rb's ReLU / split VALU, then rb's two
      //    GEMM2 k-chunks.  Left alone the scheduler issued each row block's 19 MFMAs back to back and
      //    then its ~104 split VALU with the matrix pipe idle; here the VALU sits in the MFMA shadows.
      //    The message MFMAs and GEMM1 of row block 0 carry the message tanh the same way.  Every
      //    accumulation chain keeps its order: bitwise the results of the plain body. --
      // (acc2: declared above)
      f32x16 acc1[2];
      // GEMM1 product q (0..17) of one row block: k-chunk q / 6, (A part, B part) by q % 6
      // (LEANV 4, A/B builds: each A fragment read from LDS right before its MFMA instead of a row
      //  block's nine held in registers)
      auto g1p = [&](f32x16& ac, const u32x4 (&A)[3][3], int q, int rbn) {
        const int kc = q / 6, pp = q % 6;
        const int ap = (pp == 2 || pp == 5) ? 1 : (pp == 4 ? 2 : 0);
        const int bp = (pp == 1 || pp == 5) ? 1 : (pp == 3 ? 2 : 0);
        u32x4 Af;
        if constexpr (LEANV == 4)
          Af = *reinterpret_cast<const u32x4*>(smem_b + L.w1 + (rbn * 3 + kc) * 1024 + lane * 16 + ap * 12288);
        else
          Af = A[kc][ap];
        ac = mfma_bx(Af, yf[kc][bp], ac);
      };
      auto ldA = [&](int rb, u32x4 (&A)[3][3], u32x4& bz) {
        if constexpr (LEANV == 4) return;
        bz = *reinterpret_cast<const u32x4*>(smem_b + L.bias + rb * 512 + r32 * 16);
#pragma unroll
        for (int kc = 0; kc < 3; ++kc)
#pragma unroll
          for (int pt = 0; pt < 3; ++pt)
            A[kc][pt] = *reinterpret_cast<const u32x4*>(smem_b + L.w1 + (rb * 3 + kc) * 1024 + lane * 16 + pt * 12288);
      };
      {
        u32x4 A[3][3], bz;
        ldA(0, A, bz);
        f32x16 accm = {};
        if constexpr (GRAPH) {
          const u32x4 wmA = *reinterpret_cast<const u32x4*>(smem_b + wmA_o);
          const u32x4 wmB = *reinterpret_cast<const u32x4*>(smem_b + wmB_o);
          const u32x4 wmC = *reinterpret_cast<const u32x4*>(smem_b + wmC_o);
          accm = mfma_bx(wmA, g0, accm);
          accm = mfma_bx(wmB, g0, accm);
          accm = mfma_bx(wmA, g1, accm);
          accm = mfma_bx(wmC, g2, accm);
        }
        acc1[0] = bias_acc(0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          g1p(acc1[0], A, 2 * k, 0);
          g1p(acc1[0], A, 2 * k + 1, 0);
          if constexpr (GRAPH) {
            if (k < 4) {
#pragma unroll
              for (int r = 2 * k; r < 2 * k + 2; ++r) {
                const float bm_ = reinterpret_cast<const float*>(smem_b + bml_o)[r];
                acc2[r] = fast_tanh(fmaf(bm_, S, accm[r] + accm[r + 8])) * ((hz && r < 4) ? 0.f : mgain);
              }
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        f32x16& cur = acc1[rb & 1];
        f32x16& nx = acc1[(rb + 1) & 1];
        const bool more = rb < 3;
        u32x4 A[3][3], bz;
        if (more) ldA(rb + 1, A, bz);
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int s = 2 * rb + ss;
          const u32x4 T0 = *reinterpret_cast<const u32x4*>(smem_b + w2T0 + s * 512);
          const u32x4 T1 = *reinterpret_cast<const u32x4*>(smem_b + w2T1 + s * 512);
          float hv[8];
          // step: ReLU of this k-chunk (+ the bias MFMA of the next row block, first chunk)
          if (more && ss == 0) nx = bias_acc(rb + 1);
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = relu_nan(cur[8 * ss + j]);
          __builtin_amdgcn_sched_barrier(0);
          // four steps: two GEMM1 products of the next row block + one split pair
          u32x4 h0, h1, h2;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (more) {
              g1p(nx, A, 8 * ss + 2 * k, rb + 1);
              g1p(nx, A, 8 * ss + 2 * k + 1, rb + 1);
            }
            uint32_t p0, p1, p2;
            split3_pair(hv[2 * k], hv[2 * k + 1], p0, p1, p2);
            h0[k] = p0;
            h1[k] = p1;
            h2[k] = p2;
            __builtin_amdgcn_sched_barrier(0);
          }
          // step: this k-chunk's GEMM2 products (+ the next row block's last two, second chunk)
          if (more && ss == 1) {
            g1p(nx, A, 16, rb + 1);
            g1p(nx, A, 17, rb + 1);
          }
          acc2 = mfma_bx(T0, h0, acc2);
          acc2 = mfma_bx(T1, h0, acc2);
          acc2 = mfma_bx(T0, h1, acc2);
          acc2 = mfma_bx(T0, h2, acc2);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      } else {   // LEANV == 1
      // -- message: M = WM.G (stacks [M0;M1] G0 + [M2;0] G0 + [M0;M1] G1 + [M0;0] G2), then the
      //    message term tanh(M + bm S) * gain seeds GEMM2's accumulator (top half; bottom 0) --
      // (acc2: declared above)
      if constexpr (GRAPH) {
        f32x16 accm = {};
        if (!(GNCA_ABLATE & kAblMfma)) {
          const u32x4 wmA = *reinterpret_cast<const u32x4*>(smem_b + wmA_o);
          const u32x4 wmB = *reinterpret_cast<const u32x4*>(smem_b + wmB_o);
          const u32x4 wmC = *reinterpret_cast<const u32x4*>(smem_b + wmC_o);
          accm = mfma_bx(wmA, g0, accm);
          accm = mfma_bx(wmB, g0, accm);
          accm = mfma_bx(wmA, g1, accm);
          accm = mfma_bx(wmC, g2, accm);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float bm_ = reinterpret_cast<const float*>(smem_b + bml_o)[r];
          acc2[r] = fast_tanh(fmaf(bm_, S, accm[r] + accm[r + 8])) * ((hz && r < 4) ? 0.f : mgain);
        }
      }
      __builtin_amdgcn_sched_barrier(0);

      // -- GEMM1 row block rb (H = W1.Y + b1: bias + 3 k-chunks x 6 products) into acc1[rb & 1],
      //    then its ReLU / split and its two GEMM2 k-chunks (DL += [P0;P1] H0 + [P2/2;P2/2] H0 +
      //    [P0;P1] H1 + [P0;P1] H2 into the one accumulator): two row-block accumulators live --
      f32x16 acc1[2];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        f32x16& ac = acc1[rb & 1];
        if (GNCA_ABLATE & kAblMfma) {
          ac = f32x16{};
        } else {
          ac = bias_acc(rb);
#pragma unroll
          for (int kc = 0; kc < 3; ++kc) {
            const int img = L.w1 + (rb * 3 + kc) * 1024 + lane * 16;
            const u32x4 a0 = *reinterpret_cast<const u32x4*>(smem_b + img);
            const u32x4 a1 = *reinterpret_cast<const u32x4*>(smem_b + img + 12288);
            const u32x4 a2 = *reinterpret_cast<const u32x4*>(smem_b + img + 24576);
            ac = mfma_bx(a0, yf[kc][0], ac);
            ac = mfma_bx(a0, yf[kc][1], ac);
            ac = mfma_bx(a1, yf[kc][0], ac);
            ac = mfma_bx(a0, yf[kc][2], ac);
            ac = mfma_bx(a2, yf[kc][0], ac);
            ac = mfma_bx(a1, yf[kc][1], ac);
          }
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int s = 2 * rb + ss;
          float hv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = relu_nan(ac[8 * ss + j]);
          u32x4 h0, h1, h2;
          split3_x8(hv, h0, h1, h2);
          if (GNCA_ABLATE & kAblMfma) {
            asm volatile("" ::"v"(h0), "v"(h1), "v"(h2));
            continue;
          }
          const u32x4 T0 = *reinterpret_cast<const u32x4*>(smem_b + w2T0 + s * 512);
          const u32x4 T1 = *reinterpret_cast<const u32x4*>(smem_b + w2T1 + s * 512);
          acc2 = mfma_bx(T0, h0, acc2);
          acc2 = mfma_bx(T1, h0, acc2);
          acc2 = mfma_bx(T0, h1, acc2);
          acc2 = mfma_bx(T0, h2, acc2);
        }
      }

      }   // LEANV

      // -- epilogue: dx = dl + tanh(m) * gain (already in acc2's top half) for channels
      //    c = (r&3) + 8(r>>2) + 4h; the keep mask is the live list itself --
      if (valid) {
        // dense: NCHW; compact: [tile][channel][live index]
        float* ob = compact ? a.out + (size_t)tile * C * NCELL + (size_t)(4 * h) * NCELL + gi
                            : outb + relcell + (size_t)(4 * h) * HW;
        const size_t cstr = compact ? (size_t)NCELL : HW;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float v = acc2[r] + acc2[r + 8];
          if (GNCA_ABLATE & kAblStore) asm volatile("" ::"v"(v));
          else if (compact && hz3 && r == 3) a.dxa[(size_t)b * HW + cell0 + relcell] = v;   // alpha: dense
          else ob[(size_t)((r & 3) + 8 * (r >> 2)) * cstr] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
#else
      // -- message: M = WM.G (stacks [M0;M1] G0 + [M2;0] G0 + [M0;M1] G1 + [M0;0] G2) --
      f32x16 accm = {};
      if constexpr (GRAPH) if (!(GNCA_ABLATE & kAblMfma)) {
        const u32x4 wmA = *reinterpret_cast<const u32x4*>(smem_b + wmA_o);
        const u32x4 wmB = *reinterpret_cast<const u32x4*>(smem_b + wmB_o);
        const u32x4 wmC = *reinterpret_cast<const u32x4*>(smem_b + wmC_o);
        accm = mfma_bx(wmA, g0, accm);
        accm = mfma_bx(wmB, g0, accm);
        accm = mfma_bx(wmA, g1, accm);
        accm = mfma_bx(wmC, g2, accm);
      }
      __builtin_amdgcn_sched_barrier(0);

      f32x16 accA = {}, accB = {};
      // -- GEMM1: H = W1.Y + b1, 4 row blocks x (bias + 3 k-chunks x 6 products) --
      f32x16 acc[4];
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        if (GNCA_ABLATE & kAblMfma) {
          acc[rb] = f32x16{};
          continue;
        }
        acc[rb] = bias_acc(rb);
#pragma unroll
        for (int kc = 0; kc < 3; ++kc) {
          const int img = L.w1 + (rb * 3 + kc) * 1024 + lane * 16;
          const u32x4 a0 = *reinterpret_cast<const u32x4*>(smem_b + img);
          const u32x4 a1 = *reinterpret_cast<const u32x4*>(smem_b + img + 12288);
          const u32x4 a2 = *reinterpret_cast<const u32x4*>(smem_b + img + 24576);
          acc[rb] = mfma_bx(a0, yf[kc][0], acc[rb]);
          acc[rb] = mfma_bx(a0, yf[kc][1], acc[rb]);
          acc[rb] = mfma_bx(a1, yf[kc][0], acc[rb]);
          acc[rb] = mfma_bx(a0, yf[kc][2], acc[rb]);
          acc[rb] = mfma_bx(a2, yf[kc][0], acc[rb]);
          acc[rb] = mfma_bx(a1, yf[kc][1], acc[rb]);
        }
      }

      // -- ReLU, GEMM2: DL = W2.relu(H), k-chunk s = (rb, ss) = accumulator regs 8ss..8ss+7 --
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int s = 2 * rb + ss;
          float hv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = relu_nan(acc[rb][8 * ss + j]);
          u32x4 h0, h1, h2;
          split3_x8(hv, h0, h1, h2);
          if (GNCA_ABLATE & kAblMfma) {
            asm volatile("" ::"v"(h0), "v"(h1), "v"(h2));
            continue;
          }
          const u32x4 T0 = *reinterpret_cast<const u32x4*>(smem_b + w2T0 + s * 512);
          const u32x4 T1 = *reinterpret_cast<const u32x4*>(smem_b + w2T1 + s * 512);
          accA = mfma_bx(T0, h0, accA);
          accB = mfma_bx(T1, h0, accB);
          accA = mfma_bx(T0, h1, accA);
          accB = mfma_bx(T0, h2, accB);
        }

      // -- epilogue: dx = (dl + tanh(m) * gain) * keep for channels c = (r&3) + 8(r>>2) + 4h --
      if (valid) {
        // dense: NCHW; compact: [tile][channel][live index]
        float* ob = compact ? a.out + (size_t)tile * C * NCELL + (size_t)(4 * h) * NCELL + gi
                            : outb + relcell + (size_t)(4 * h) * HW;
        const size_t cstr = compact ? (size_t)NCELL : HW;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          float v = accA[r] + accA[r + 8] + accB[r];
          if constexpr (GRAPH) {
            const float bm_ = reinterpret_cast<const float*>(smem_b + bml_o)[r];
            v = fmaf(fast_tanh(fmaf(bm_, S, accm[r] + accm[r + 8])), (hz && r < 4) ? 0.f : mgain, v);
          }
          if (GNCA_ABLATE & kAblStore) asm volatile("" ::"v"(v));
          else if (compact && hz3 && r == 3) a.dxa[(size_t)b * HW + cell0 + relcell] = v;   // alpha: dense
          else ob[(size_t)((r & 3) + 8 * (r >> 2)) * cstr] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
#endif
      if (!(GNCA_ABLATE & kAblReduce)) {
        double d1 = s1, d2 = s2;
        for (int off = 32; off > 0; off >>= 1) {
          d1 += __shfl_xor(d1, off);
          d2 += __shfl_xor(d2, off);
        }
        if (lane == 0) {
          pg[2 * q] = d1;
          pg[2 * q + 1] = d2;
        }
      }
      PROF_MARK(4);   // MFMAs + epilogue + partials
      if (GNCA_K1_DYNPRIO > 0) __builtin_amdgcn_s_setprio(GNCA_K1_PRIO);
    }

    // then the dense field's zero items (the same counter: the waves without a group take them first)
    const int nz = (compact || (GNCA_ABLATE & kAblZero)) ? 0 : 4 * NCH;
    if (iter == 0) ARR_MARK(4);
#pragma unroll 1
    for (; q < qend + nz; q = pull()) zero_item(q - qend, par, outb);
    PROF_MARK(4);   // group loop
    // The wave whose pull failed first (q == qend + nz: the counter hands out consecutive values)
    // stages the next tile as soon as every group is past its staged-plane reads, while the other
    // waves still run their last groups' MFMAs and stores.
    if constexpr (FOLD) {
      // every wave: the next tile's region finalized into the staging buffer (+ its cells into xo)
      if (nxt < t_end) finalize(nxt, par ^ 1, iter + 2, true, qend, lst, par);
    } else if (q >= qend + nz && q < qend + nz + GNCA_DMA_WAVES && nxt < t_end) {
      while ((__hip_atomic_load(xsd, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >> 6) - xbase < qend)
        __builtin_amdgcn_s_sleep(1);
      issue_dma(nxt, q - qend - nz, GNCA_DMA_WAVES);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    PROF_MARK(0);
    if (iter == 0) ARR_MARK(5);
    __syncthreads();   // groups done, next tile staged, pg complete, slot par^1 ready
    PROF_MARK(6);
    if (iter == 0) ARR_MARK(6);
    gbase += qend + nz + NW;
    xbase += qend;
    if constexpr (FOLD) if (tid == 0) cnt[6 + par] = 0;   // this tile's group done-mask, for tile + 2
    // ---- the tile's GroupNorm partials in 8 bins (bin j: groups j, j + 8, ... in order; K2 sums the
    //      bins of a sample in fixed order) ----
    if (tid < 2 * NW) {
      double s_ = 0.0;
      for (int q = tid >> 1; q < qend; q += NW) s_ += pg[2 * q + (tid & 1)];
      a.stats[(size_t)tile * 2 * NW + tid] = s_;
    }
    PROF_MARK(5);   // per-tile reduction
    tile = nxt;
    par ^= 1;
    ++iter;
  }
  PROF_STORE_W03;
  FPROF_STORE;
  ARR_MARK(7);
  GNCA_STAMP_END(a.stamps);
}

}  // namespace gnca
