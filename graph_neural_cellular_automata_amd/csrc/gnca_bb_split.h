// gnca_bb_split.h — BB of the backward (gnca_bwd.hip) for the trainers' shape class (C = 16,
// hidden = 128) on bf16 MFMA with the exact 3-way split of every fp32 operand, as the forward's K1
// (gnca_k1_split.h: v = v0 + v1 + v2 exactly, six products per fp32 product, the dropped terms each
// <= 2^-24 |a||b|).  Included by gnca_bwd.hip after BBArgs; the fp32-MFMA gnca_b_mlp keeps every
// other shape.
//
// What it computes per live cell (the reference's autograd through ncagraph.py:128-153 /
// nca.py:75-100, restated by oracle/nca_oracle_vjp.py): recompute y = P(x), G = gather(x), S,
// H = W1 y + b1, m = W_M G + b_M S; then with d = keep * GroupNorm-backward(U):
//   dh = relu'(H) * W2^T d        dm = d * gain * tanh'(m)
//   dY = W1^T dh -> HBM           dG = W_M^T dm -> HBM        (the perception / gather adjoints: BC)
//   dW1 += dh y^T, db1 += dh, dW2 += d relu(H)^T, dW_M += dm G^T, db_M += dm S
//
// MI355X layout (v_mfma_f32_32x32x16_bf16, lane l: r32 = l & 31, h = l >> 5; A[row r32][k 8h+j],
// B[k 8h+j][col r32], D reg r -> row rowof(r, h) = (r&3) + 8(r>>2) + 4h, col r32).  One 32-cell group
// per wave.  The cell index lives on the lane for the loads, perception and gather (as in K1), and
// in the REGISTERS for the hidden-side products: H^T = y^T W1^T and dh^T = d^T W2 put the hidden
// unit on the lane and the cells in the accumulator rows, so that
//   * dW2 = d . h^T takes h^T's registers as its B operand and dW1 = dh . y^T takes dh^T's as its A
//     operand (an accumulator tile as the next MFMA's operand, cdna_hip_programming.md §3: sums over
//     the accumulator's row index = the cells) with no data movement;
//   * y^T (B of dW1) and dh (B of dY = W1^T dh, which sums over the hidden units) are the two
//     tiles that change orientation, through per-wave LDS images read back with
//     ds_read_b64_tr_b16 (16-bit transposed reads, T10), each image laid out so those reads hit
//     64 distinct banks per 32-lane half;
//   * the d / dm / G tiles that the weight products need with the cells in k go through small fp32
//     LDS transposes (80-byte rows: conflict-free 16-byte writes and 4-byte column reads).
// The W1 image is ONE row-major bf16 [part][hidden][48] block: row reads give H^T's B operand,
// transposed reads give dY's A operand.  16-row M or N tiles (the 16 features 32..47, the 16
// channels of W2 / W_M / d) hold two split parts side by side, so one MFMA computes two of the six
// products.  Per 32-cell group: 72 (H^T) + 24 (dh^T) + 32 (dW2) + 80 (dW1) + 80 (dY) + 14 (message)
// MFMAs.  Weight gradients accumulate per wave over the launch (fp32 accumulators) and leave as one
// partial row per wave, summed in a fixed order by gnca_b_reduce (deterministic, as gnca_b_mlp).
#pragma once

// (included inside gnca_bwd.hip's namespace gnca { namespace { ... } })

typedef __bf16 bsbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bsbf16x2 __attribute__((ext_vector_type(2)));
typedef float bsf32x2 __attribute__((ext_vector_type(2)));
typedef float bsf32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t bsu4 __attribute__((ext_vector_type(4)));
typedef short bss4 __attribute__((ext_vector_type(4)));

// (a, b) -> three packed bf16x2 words with a = a0 + a1 + a2, b = b0 + b1 + b2 exactly (round to
// nearest even at each level; the forward's split3_pair)
__device__ __forceinline__ void bs_split_pair(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  const uint32_t hh = __builtin_bit_cast(uint32_t, __builtin_convertvector((bsf32x2){a, b}, bsbf16x2));
  const float ra = a - __uint_as_float(hh << 16), rb = b - __uint_as_float(hh & 0xffff0000u);
  const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_convertvector((bsf32x2){ra, rb}, bsbf16x2));
  const float la = ra - __uint_as_float(m << 16), lb = rb - __uint_as_float(m & 0xffff0000u);
  p0 = hh;
  p1 = m;
  p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector((bsf32x2){la, lb}, bsbf16x2));
}

// 8 fp32 -> three bf16x8 fragments (element order kept)
__device__ __forceinline__ void bs_split8(const float* v, bsu4 (&f)[3]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t p0, p1, p2;
    bs_split_pair(v[2 * i], v[2 * i + 1], p0, p1, p2);
    f[0][i] = p0;
    f[1][i] = p1;
    f[2][i] = p2;
  }
}

__device__ __forceinline__ bsf32x16 bs_mfma(bsu4 a, bsu4 b, bsf32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bsbf16x8, a), __builtin_bit_cast(bsbf16x8, b),
                                                 c, 0, 0, 0);
}

// the six products of an fp32 product on split parts: (A part, B part) with part sum <= 2
#define BS_SIX(acc, A, B)                  \
  do {                                     \
    acc = bs_mfma((A)[0], (B)[0], acc);    \
    acc = bs_mfma((A)[0], (B)[1], acc);    \
    acc = bs_mfma((A)[1], (B)[0], acc);    \
    acc = bs_mfma((A)[0], (B)[2], acc);    \
    acc = bs_mfma((A)[2], (B)[0], acc);    \
    acc = bs_mfma((A)[1], (B)[1], acc);    \
  } while (0)

// 16-bit transposed LDS read: 4 rows x 16 columns per 16-lane group (lane 4q+p: row q, columns
// 4p..4p+3 at `p`), lane i of the group gets column i, row q in element q.  EXEC must be all ones.
__device__ __forceinline__ uint2 bs_tr(const char* p) {
  const bss4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bss4*)p);
  return __builtin_bit_cast(uint2, v);
}

__host__ __device__ constexpr int bs_rowof(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// LDS of gnca_b_split: the staging part in floats (as bb_layout, 16 channels), then byte offsets
struct BSLayout {
  int xs, PSTR, al, ALW, sp, kp, lst, RH, RW, NI, NIA;   // floats
  int w1i, w2b, wmf, wmt, b1s, bml, scr, total;          // bytes
};
constexpr int kBSScr = 16384;                 // per-wave scratch bytes
constexpr int kBSHB = 64;                     // hidden units whose weight gradients one launch accumulates
constexpr int kBSW1Part = 128 * 96;           // one split part of the row-major bf16 W1 image
// per-wave scratch (bytes): Y0 [part][cell 32][32 features] (features 0..31) | P [cell][y0 | y1 of
// features 32..47] | Q [cell][y2 of features 32..47 | 0] | DH [part][hidden 32][cell 32]; the fp32
// transposes [cell][16 channels] (80-byte rows) reuse DH
constexpr int kBSY0 = 0, kBSP = 6144, kBSQ = 8192, kBSDH = 10240, kBST = 10240, kBSTrow = 80;

__host__ __device__ inline BSLayout bs_layout(int TH, int TW, int RY, int RX) {
  BSLayout L;
  L.RH = TH + 2 * RY;
  L.RW = TW + 2 * RX;
  L.NI = (L.RH * L.RW + 63) / 64;
  L.PSTR = 64 * L.NI + 16;
  L.ALW = L.RW + 2;
  L.NIA = ((L.RH + 2) * L.ALW + 63) / 64;
  int o = 0;
  L.xs = o; o += 16 * L.PSTR;
  L.al = o; o += 64 * L.NIA;
  L.sp = o; o += r4(L.RH * L.RW);
  L.kp = o; o += r4(TH * TW);
  L.lst = o; o += r4(TH * TW) + 8;
  o = (o + 3) & ~3;
  int b = 4 * o;
  L.w1i = b; b += 3 * kBSW1Part;        // row-major bf16 W1 [part][hidden][48]
  L.w2b = b; b += 3 * 4 * 64 * 16;      // dh^T's B: [part][hidden block][lane] W2[phi(h,j)][hidden]
  L.wmf = b; b += 3 * 2 * 16 * 16 + 512;   // the forward's message images [part][h][channel] + zeros
  L.wmt = b; b += 3 * 64 * 16;          // dG's A stacks [w0;w1], [w0;w2], [w2;0]
  L.b1s = b; b += 128 * 4;
  L.bml = b; b += 16 * 4;               // message bias per (h, r): b_M[rowof(r, h)]
  L.scr = b; b += NW * kBSScr;
  L.total = b;
  return L;
}

#ifndef GNCA_BS_DENSE
#define GNCA_BS_DENSE 1   // the first launch's groups over every cell of the tile (A/B builds: 0 = live cells)
#endif
#ifndef BS_ABL
#define BS_ABL 0   // timing-only builds (wrong results): 1 no dY products, 2 no dW1 products, 4 no U/dx
                   // loads, 8 no dY/dG stores, 16 no H^T/dh^T products, 32 no dW2 products, 64 no
                   // groups, 128 no dead-cell zero stores, 256 no staging DMA
#endif

template <bool MSG, bool FIRST>
__global__ __launch_bounds__(kThreads, 1) void gnca_b_split(const BBArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* smb = reinterpret_cast<char*>(smem);
  constexpr int C = 16, HD = 128;
  const int TH = a.TH, TW = a.TW, RY = a.RY, RX = a.RX;
  const BSLayout L = bs_layout(TH, TW, RY, RX);
  const int RH = L.RH, RW = L.RW, PSTR = L.PSTR, ALW = L.ALW;
  float* xs = smem + L.xs;
  float* al = smem + L.al;
  float* sp = smem + L.sp;
  float* fp = smem + L.kp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5, g16 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int H = a.H, W = a.W, k = a.k;
  const bool zp = (a.flags & GNCA_ZERO_PAD_SHIFT) != 0;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const bool gn = (a.flags & kGN) != 0;
  const bool uniform_w = a.offw == nullptr;
  const float thr = a.alpha_thr, gthr = a.graph_alpha_thr;
  // Two launches: the first (h0 = 0) runs every hidden block's H^T / dh^T for dY (stored once) and
  // the message backward (dG, dW_M, db_M), and accumulates the weight gradients of hidden units
  // 0..63; the second (h0 = 64) recomputes blocks 2, 3 for the weight gradients of units 64..127 only.
  // (The accumulators of all 128 units do not fit one wave's registers; a dY read-modify-write by
  // the second launch measured slower than recomputing two blocks.)
  const int h0 = a.h0;
  constexpr bool first = FIRST;
  const bool msgb = MSG && first;
  char* scr = smb + L.scr + wave * kBSScr;
  __shared__ float wts[GNCA_MAX_OFFSETS];
  int* lst = reinterpret_cast<int*>(smem + L.lst);   // the tile's live-cell list
  int* wcnt = lst + r4(TH * TW);                      // per-wave ballot counts of the compaction

  // ---- weight images (bf16 parts) -> LDS; every load of a thread in flight before its stores ----
  {
    // W1 row-major: thread -> (hidden tid / 2, features 24 (tid & 1) .. + 23)
    float w1v[24];
    {
      const float* src = a.w1 + (size_t)(tid >> 1) * 48 + 24 * (tid & 1);
#pragma unroll
      for (int i = 0; i < 24; ++i) w1v[i] = src[i];
    }
    // dh^T's B: entry (hidden block nb, lane l'): W2[phi(h', j)][32 nb + (l' & 31)], j = 0..7
    float w2v[8];
    {
      const int nb = tid >> 6, l2 = tid & 63, hid = 32 * nb + (l2 & 31), h2 = l2 >> 5;
#pragma unroll
      for (int j = 0; j < 8; ++j) w2v[j] = a.w2[(size_t)bs_rowof(j, h2) * HD + hid];
    }
    float wmv[8], wtv[8], b1v = 0.f, bmv = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wmv[j] = 0.f;
      wtv[j] = 0.f;
    }
    if (MSG) {
      if (tid < 32) {   // the forward's message image entry (h', c): W_M[c][8h' + j]
#pragma unroll
        for (int j = 0; j < 8; ++j) wmv[j] = a.wm[(tid & 15) * C + 8 * (tid >> 4) + j];
      }
      if (tid >= 64 && tid < 128) {   // dG's A entry, lane l' = tid - 64: W_M[phi(h', j)][ci = l' & 15]
        const int l2 = tid - 64;
#pragma unroll
        for (int j = 0; j < 8; ++j) wtv[j] = a.wm[bs_rowof(j, l2 >> 5) * C + (l2 & 15)];
      }
      if (tid >= 128 && tid < 144) bmv = a.bm[bs_rowof((tid - 128) & 7, (tid - 128) >> 3)];
    }
    if (tid < HD) b1v = a.b1[tid];
    // stores
#pragma unroll
    for (int i = 0; i < 3; ++i) {   // 8 features per 16-byte store
      bsu4 f[3];
      bs_split8(w1v + 8 * i, f);
      const int off = (tid >> 1) * 96 + (24 * (tid & 1) + 8 * i) * 2;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bsu4*>(smb + L.w1i + p * kBSW1Part + off) = f[p];
    }
    {
      bsu4 f[3];
      bs_split8(w2v, f);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bsu4*>(smb + L.w2b + p * 4096 + tid * 16) = f[p];
    }
    if (MSG && tid < 32) {
      bsu4 f[3];
      bs_split8(wmv, f);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bsu4*>(smb + L.wmf + p * 512 + tid * 16) = f[p];
      *reinterpret_cast<bsu4*>(smb + L.wmf + 1536 + tid * 16) = bsu4{0u, 0u, 0u, 0u};
    }
    if (MSG && tid >= 64 && tid < 128) {
      const int l2 = tid - 64;
      bsu4 f[3];
      bs_split8(wtv, f);
      const bool top = (l2 & 31) < 16;
      const bsu4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<bsu4*>(smb + L.wmt + l2 * 16) = top ? f[0] : f[1];          // [w0; w1]
      *reinterpret_cast<bsu4*>(smb + L.wmt + 1024 + l2 * 16) = top ? f[0] : f[2];   // [w0; w2]
      *reinterpret_cast<bsu4*>(smb + L.wmt + 2048 + l2 * 16) = top ? f[2] : z;      // [w2; 0]
    }
    if (tid < HD) reinterpret_cast<float*>(smb + L.b1s)[tid] = b1v;
    if (MSG && tid >= 128 && tid < 144) reinterpret_cast<float*>(smb + L.bml)[tid - 128] = bmv;
    // the Q image's zero half (features 48..63 of the part-2 block: never written by a group)
    const int zc = r32, sw = (zc >> 1) & 3;
    *reinterpret_cast<bsu4*>(scr + kBSQ + zc * 64 + (((2 + h) ^ sw) * 16)) = bsu4{0u, 0u, 0u, 0u};
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
      if (a.perc[(3 * c + f) * 9 + tap] != ref) ok = 0;
    }
    sobel = __syncthreads_and(ok) != 0;
  }
  const float mgain = MSG ? a.message_gain : 0.f;

  // per-wave accumulators of the whole launch
  bsf32x16 dw1a[2], dw1b[2], dw2[2], dwm;
  float ab1[2], abm[8];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    dw1a[nb] = bsf32x16{};
    dw1b[nb] = bsf32x16{};
    dw2[nb] = bsf32x16{};
    ab1[nb] = 0.f;
  }
  dwm = bsf32x16{};
#pragma unroll
  for (int j = 0; j < 8; ++j) abm[j] = 0.f;

  const int ncell = TH * TW;
  const size_t HW = (size_t)H * W;
  const int HWi = H * W;
  const int nxcd = gridDim.x >= 8 ? 8 : 1;
  const int xg_ = blockIdx.x % nxcd, xr_ = blockIdx.x / nxcd;
  const int per_x = (int)(gridDim.x / nxcd) + ((int)(gridDim.x % nxcd) > xg_ ? 1 : 0);
  const int tq = a.total_tiles / nxcd, trm = a.total_tiles % nxcd;
  const int t_begin = xg_ * tq + min(xg_, trm), t_end = t_begin + tq + (xg_ < trm ? 1 : 0);
  for (int tile = t_begin + xr_; tile < t_end; tile += per_x) {
    const int b = tile / a.tps, tin = tile - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const float* xb = a.x + (size_t)b * C * HW;
    const float* Ub = a.U + (size_t)b * C * HW;
    const float* Db = a.dx + (size_t)b * C * HW;
    float* dYb = a.dY + (size_t)b * 3 * C * HW;
    float* dGb = a.dG + (size_t)b * C * HW;
    __syncthreads();
    if (a.active && !a.active[b]) {   // masked step, inactive sample: every cell is dead
      for (int n = tid; n < ncell && first; n += kThreads) {
        const int ti = n / TW, tj = n - (n / TW) * TW;
        if (i0 + ti >= H || j0 + tj >= W) continue;
        const int ce = (i0 + ti) * W + (j0 + tj);
        for (int pl = 0; pl < 3 * C; ++pl) dYb[pl * HWi + ce] = 0.f;
        if (MSG)
          for (int c = 0; c < C; ++c) dGb[c * HWi + ce] = 0.f;
        if (a.dmb) a.dmb[(size_t)b * HW + ce] = 0.f;
      }
      continue;
    }
    // ---- staging by LDS-DMA (gnca_b_mlp's): the 16 channel planes of the region and the alpha
    //      plane with one more ring; torus-wrapped, or a zero source outside the image in pad mode ----
    for (int ii_ = wave; ii_ < ((BS_ABL & 256) ? 0 : L.NI); ii_ += NW) {
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
#pragma unroll 4
      for (int c = 0; c < C; ++c) {
        const float* src = (zp && !ok) ? g_bzero : xb + (size_t)c * HW + off;
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
    if (MSG && !uniform_w)
      for (int o = tid; o < k; o += kThreads) wts[o] = a.offw[(size_t)b * k + o];
    for (int ti = wave; ti < TH; ti += NW) {
      if (lane < TW) {
        const int i = min(i0 + ti, H - 1), j = min(j0 + lane, W - 1);
        fp[ti * TW + lane] = fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step,
                                     a.sample_base, b, HW, (size_t)i * W + j) ? 1.f : 0.f;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // ---- sender plane over the region, keep = pre-alive AND fire on the tile (gnca_b_mlp's) ----
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
        const float* qa = al + (vr + 1) * ALW + (vc + 1);
        const float NEG = -INFINITY;
        const bool up = iq > 0, dn = iq < H - 1;
        const float mu_ = fmaxf(fmaxf(lf ? qa[-ALW - 1] : NEG, qa[-ALW]), rt ? qa[-ALW + 1] : NEG);
        const float mm_ = fmaxf(fmaxf(lf ? qa[-1] : NEG, qa[0]), rt ? qa[1] : NEG);
        const float md_ = fmaxf(fmaxf(lf ? qa[ALW - 1] : NEG, qa[ALW]), rt ? qa[ALW + 1] : NEG);
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
    // ---- the tile's cells in 32-cell groups.  A dead cell (keep == 0) has d = 0: zero dY / dG and
    //      no weight-gradient term.  The first launch (DENSE) lists every cell in tile order, so a
    //      group's dY / dG / U / dx accesses are runs of consecutive cells (its dead cells compute their
    //      zeros); the second lists the live cells only (it stores nothing per cell) ----
    constexpr bool DENSE = FIRST && GNCA_BS_DENSE;
    int nlive = 0;
    for (int n0 = 0; n0 < ncell; n0 += kThreads) {
      const int n = n0 + tid;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const bool inb = n < ncell && i0 + ti < H && j0 + tj < W;
      const bool live = inb && (DENSE || fp[n] != 0.f);
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
      } else if (inb && first && !DENSE && !(BS_ABL & 128)) {
        const int ce = (i0 + ti) * W + (j0 + tj);
        for (int pl = 0; pl < 3 * C; ++pl) dYb[pl * HWi + ce] = 0.f;
        if (MSG)
          for (int c = 0; c < C; ++c) dGb[c * HWi + ce] = 0.f;
        if (a.dmb) a.dmb[(size_t)b * HW + ce] = 0.f;
      }
      nlive += tot;
      __syncthreads();
    }

    // (1) U and the forward's dx for channels rowof(j, h) of a group's cells: loaded one group AHEAD
    //     (issued before this group's dY / dG stores: the wait for them then does not wait for the
    //     stores too, vmcnt counting loads and stores in issue order)
    const int ngq = (BS_ABL & 64) ? 0 : (nlive + 31) >> 5;
    float ulN[8], dlN[8];
    auto load_ud = [&](int q) {
      const int idx = 32 * q + r32;
      const int n = lst[idx < nlive ? idx : 0];
      const bool valid = idx < nlive && fp[n] != 0.f;   // (dense lists: the dead cells' d is 0)
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const int celli = (i0 + ti) * W + (j0 + tj);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = bs_rowof(j, h);
        ulN[j] = (valid && !(BS_ABL & 4)) ? Ub[c * HWi + celli] : 0.01f * j;
        dlN[j] = (valid && gn && !(BS_ABL & 4)) ? Db[c * HWi + celli] : 0.f;
      }
    };
    if (wave < ngq) load_ud(wave);
#pragma unroll 1
    for (int q = wave; q < ngq; q += NW) {
      const int idx = 32 * q + r32;
      const bool valid = idx < nlive;
      const int n = lst[valid ? idx : 0];
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const int pidx = (RY + ti) * RW + (RX + tj);
      const int celli = (i0 + ti) * W + (j0 + tj);
      float ul[8], dl[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ul[j] = ulN[j];
        dl[j] = dlN[j];
      }
      // (2) gather (recompute), channels 8h + j (as K1: uniform weights summed, then scaled once)
      float gv[8], S = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = 0.f;
      if (msgb) {
        const float* xq = xs + 8 * h * PSTR + pidx;
#pragma unroll 2
        for (int o = 0; o < k; ++o) {
          const int qb = pidx - a.odl[o];
          const float s_ = uniform_w ? sp[qb] : wts[o] * sp[qb];
          S += s_;
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] = fmaf(s_, xq[j * PSTR - a.odl[o]], gv[j]);
        }
        if (uniform_w) {
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] *= a.uniform_w;
          S *= a.uniform_w;
        }
      }
      // (3) perception (recompute), channels 8h + j, zero padding at the image border
      float y0[8], y1[8], y2[8];
      {
        const int ic = i0 + ti, jc = j0 + tj;
        const bool up = ic > 0, dn = ic < H - 1, lf = jc > 0, rt = jc < W - 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float* xc = xs + (8 * h + j) * PSTR + pidx;
          float n0 = xc[-RW - 1], n1 = xc[-RW], n2 = xc[-RW + 1];
          float n3 = xc[-1], n4 = xc[0], n5 = xc[1];
          float n6 = xc[RW - 1], n7 = xc[RW], n8 = xc[RW + 1];
          n0 = (up && lf) ? n0 : 0.f; n1 = up ? n1 : 0.f; n2 = (up && rt) ? n2 : 0.f;
          n3 = lf ? n3 : 0.f;                               n5 = rt ? n5 : 0.f;
          n6 = (dn && lf) ? n6 : 0.f; n7 = dn ? n7 : 0.f; n8 = (dn && rt) ? n8 : 0.f;
          if (sobel) {
            y0[j] = n4;
            const float dg = n0 - n8, da = n2 - n6;
            y1[j] = fmaf(2.f, n3 - n5, dg - da);
            y2[j] = fmaf(2.f, n1 - n7, dg + da);
          } else {
            const float nn[9] = {n0, n1, n2, n3, n4, n5, n6, n7, n8};
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
      bsu4 yf[3][3];
      bs_split8(y0, yf[0]);
      bs_split8(y1, yf[1]);
      bs_split8(y2, yf[2]);
      __builtin_amdgcn_sched_barrier(0);
      // (4) y^T images for dW1's B operand: row = this lane's cell, 16-byte chunk (features 8j'..)
      //     XOR (cell >> 1) & 3 (conflict-free writes and transposed reads)
      {
        const int sw = (r32 >> 1) & 3;
        char* row0 = scr + kBSY0 + r32 * 64;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          *reinterpret_cast<bsu4*>(row0 + p * 2048 + ((h ^ sw) * 16)) = yf[0][p];         // features 8h..
          *reinterpret_cast<bsu4*>(row0 + p * 2048 + (((2 + h) ^ sw) * 16)) = yf[1][p];   // 16 + 8h..
        }
        *reinterpret_cast<bsu4*>(scr + kBSP + r32 * 64 + ((h ^ sw) * 16)) = yf[2][0];         // y0 of 32 + 8h..
        *reinterpret_cast<bsu4*>(scr + kBSP + r32 * 64 + (((2 + h) ^ sw) * 16)) = yf[2][1];   // y1
        *reinterpret_cast<bsu4*>(scr + kBSQ + r32 * 64 + ((h ^ sw) * 16)) = yf[2][2];         // y2
      }
      // (5) d = keep * GroupNorm-backward(U) (ncagraph.py:144-153)
      const bool kept = valid && fp[n] != 0.f;
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        dv[j] = kept ? (gn ? rs * (ul[j] - mu_u - (dl[j] - mu) * rs * mu_ux) : ul[j]) : 0.f;
      // (6) message (recompute) and its backward: dm = d * gain * tanh'(m); dG = W_M^T dm -> HBM
      float dmv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dmv[j] = 0.f;
      if (msgb) {
        bsu4 gf[3];
        bs_split8(gv, gf);
        const int ent = (h * 16 + (r32 & 15)) * 16;
        const bsu4 wmA = *reinterpret_cast<const bsu4*>(smb + L.wmf + (r32 < 16 ? 0 : 512) + ent);
        const bsu4 wmB = *reinterpret_cast<const bsu4*>(smb + L.wmf + (r32 < 16 ? 1024 : 1536) + ent);
        const bsu4 wmC = *reinterpret_cast<const bsu4*>(smb + L.wmf + (r32 < 16 ? 0 : 1536) + ent);
        bsf32x16 accm = {};
        accm = bs_mfma(wmA, gf[0], accm);
        accm = bs_mfma(wmB, gf[0], accm);
        accm = bs_mfma(wmA, gf[1], accm);
        accm = bs_mfma(wmC, gf[2], accm);
        const float* bml = reinterpret_cast<const float*>(smb + L.bml) + 8 * h;
        float dmb = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float m = fmaf(bml[j], S, accm[j] + accm[j + 8]);
          const float t = tanhf(m);
          const float gj = (hidden_only && h == 0 && j < 4) ? 0.f : mgain;
          dmv[j] = dv[j] * gj * (1.f - t * t);
          abm[j] = fmaf(dmv[j], S, abm[j]);
          dmb = fmaf(dmv[j], bml[j], dmb);
        }
        bsu4 dmf[3];
        bs_split8(dmv, dmf);
        const bsu4 s01 = *reinterpret_cast<const bsu4*>(smb + L.wmt + lane * 16);
        const bsu4 s02 = *reinterpret_cast<const bsu4*>(smb + L.wmt + 1024 + lane * 16);
        const bsu4 s20 = *reinterpret_cast<const bsu4*>(smb + L.wmt + 2048 + lane * 16);
        bsf32x16 ag = {};
        ag = bs_mfma(s01, dmf[0], ag);
        ag = bs_mfma(s01, dmf[1], ag);
        ag = bs_mfma(s02, dmf[2], ag);
        ag = bs_mfma(s20, dmf[0], ag);
        if (valid && !(BS_ABL & 8)) {
#pragma unroll
          for (int r = 0; r < 8; ++r) dGb[bs_rowof(r, h) * HWi + celli] = ag[r] + ag[r + 8];
        }
        if (a.dmb) {
          dmb += __shfl_xor(dmb, 32);
          if (valid && h == 0) a.dmb[(size_t)b * HW + celli] = dmb;
        }
      }
      // (6b) dW_M [co (stacked parts) x ci (stacked parts)] += dm . G^T: both with the cells in k,
      //      through the fp32 transposes (dm: channels rowof(j, h); G: channels 8h + j)
      if (msgb) {
        char* Tm = scr + kBST;
        char* Tg = scr + kBST + 32 * kBSTrow;
        *reinterpret_cast<f4*>(Tm + r32 * kBSTrow + 16 * h) = f4{dmv[0], dmv[1], dmv[2], dmv[3]};
        *reinterpret_cast<f4*>(Tm + r32 * kBSTrow + 32 + 16 * h) = f4{dmv[4], dmv[5], dmv[6], dmv[7]};
        *reinterpret_cast<f4*>(Tg + r32 * kBSTrow + 32 * h) = f4{gv[0], gv[1], gv[2], gv[3]};
        *reinterpret_cast<f4*>(Tg + r32 * kBSTrow + 32 * h + 16) = f4{gv[4], gv[5], gv[6], gv[7]};
        asm volatile("" ::: "memory");
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float mt[8], gt[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int cell = 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            mt[j] = *reinterpret_cast<const float*>(Tm + cell * kBSTrow + 4 * (r32 & 15));
            gt[j] = *reinterpret_cast<const float*>(Tg + cell * kBSTrow + 4 * (r32 & 15));
          }
          bsu4 mf[3], gf2[3];
          bs_split8(mt, mf);
          bs_split8(gt, gf2);
          const bool top = r32 < 16;
          const bsu4 z = {0u, 0u, 0u, 0u};
          const bsu4 A1 = top ? mf[0] : mf[1], B1 = top ? gf2[0] : gf2[1];   // [dm0; dm1] x [G0 | G1]
          const bsu4 A2 = top ? mf[0] : mf[2], B2 = top ? gf2[2] : z;        // [dm0; dm2] x [G2 | 0]
          const bsu4 A3 = top ? mf[2] : z, B3 = top ? gf2[0] : z;            // [dm2; 0] x [G0 | 0]
          dwm = bs_mfma(A1, B1, dwm);
          dwm = bs_mfma(A2, B2, dwm);
          dwm = bs_mfma(A3, B3, dwm);
        }
        asm volatile("" ::: "memory");
      }
      // (7) d with the cells in k (dW2's A operand, channel r32 & 15 on the lane): fp32 transpose
      //     through [cell][16 channels] rows of 80 bytes
      bsu4 sA[2], sB[2], sC[2];
      {
        char* T = scr + kBST;
        *reinterpret_cast<f4*>(T + r32 * kBSTrow + 16 * h) = f4{dv[0], dv[1], dv[2], dv[3]};        // ch 4h..
        *reinterpret_cast<f4*>(T + r32 * kBSTrow + 32 + 16 * h) = f4{dv[4], dv[5], dv[6], dv[7]};   // 8 + 4h..
        asm volatile("" ::: "memory");
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float dt[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            dt[j] = *reinterpret_cast<const float*>(T + (16 * s + 8 * (j >> 2) + 4 * h + (j & 3)) * kBSTrow +
                                                    4 * (r32 & 15));
          bsu4 f[3];
          bs_split8(dt, f);
          const bool top = r32 < 16;
          const bsu4 z = {0u, 0u, 0u, 0u};
          sA[s] = top ? f[0] : f[1];   // [d0; d1]
          sB[s] = top ? f[0] : f[2];   // [d0; d2]
          sC[s] = top ? f[2] : z;      // [d2; 0]
        }
        asm volatile("" ::: "memory");
      }
      bsu4 dfa[3];
      bs_split8(dv, dfa);
      if (q + NW < ngq) load_ud(q + NW);   // the next group's U / dx
      __builtin_amdgcn_sched_barrier(0);

      // (8) per hidden block: H^T, dh^T, relu / relu', [dW2, dW1 of this launch's blocks], [dY's two
      //     k-chunks: first launch]
      bsf32x16 dy0 = {}, dy1 = {};
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        // first launch: every block for dY, the weight gradients of blocks 0, 1; second: blocks 2, 3
        const bool dw_on = first ? nb < 2 : nb >= 2;
        const int sl = nb & 1;   // the accumulator slot of a weight-gradient block
        if (!first && nb < 2) continue;
        const float bias = reinterpret_cast<const float*>(smb + L.b1s)[32 * nb + r32];
        bsf32x16 hT;
#pragma unroll
        for (int r = 0; r < 16; ++r) hT[r] = bias;
#pragma unroll
        for (int kc = 0; kc < 3; ++kc) {
          bsu4 wb[3];
          const int off = (32 * nb + r32) * 96 + (16 * kc + 8 * h) * 2;
#pragma unroll
          for (int p = 0; p < 3; ++p) wb[p] = *reinterpret_cast<const bsu4*>(smb + L.w1i + p * kBSW1Part + off);
          if (!(BS_ABL & 16)) BS_SIX(hT, yf[kc], wb);
        }
        __builtin_amdgcn_sched_barrier(0);
        bsf32x16 dhT = {};
        {
          bsu4 wb[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) wb[p] = *reinterpret_cast<const bsu4*>(smb + L.w2b + p * 4096 + (nb * 64 + lane) * 16);
          if (!(BS_ABL & 16)) BS_SIX(dhT, dfa, wb);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dhT[r] = hT[r] > 0.f ? dhT[r] : 0.f;
          hT[r] = __builtin_elementwise_maximum(hT[r], 0.f);   // relu (NaN stays NaN)
          if (dw_on) ab1[sl] += dhT[r];
        }
        __builtin_amdgcn_sched_barrier(0);
        bsu4 hf[2][3], dhf[2][3];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float t8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) t8[j] = hT[8 * s + j];
          bs_split8(t8, hf[s]);
#pragma unroll
          for (int j = 0; j < 8; ++j) t8[j] = dhT[8 * s + j];
          bs_split8(t8, dhf[s]);
        }
        __builtin_amdgcn_sched_barrier(0);
        // dW2 [channel (stacked parts) x hidden] += d . h^T
#pragma unroll
        for (int s = 0; s < 2 * !(BS_ABL & 32) && dw_on; ++s) {
          dw2[sl] = bs_mfma(sA[s], hf[s][0], dw2[sl]);
          dw2[sl] = bs_mfma(sA[s], hf[s][1], dw2[sl]);
          dw2[sl] = bs_mfma(sB[s], hf[s][2], dw2[sl]);
          dw2[sl] = bs_mfma(sC[s], hf[s][0], dw2[sl]);
        }
        __builtin_amdgcn_sched_barrier(0);
        // dW1 [hidden x feature] += dh . y^T: B = the y^T images, transposed reads (row = cell
        // 16s + 8e + 4h + q, columns 16 (g16 & 1) + 4p of a 32-feature block)
#pragma unroll
        for (int s = 0; s < 2 * !(BS_ABL & 2) && dw_on; ++s) {
          bsu4 yb[3], pb, qb;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int cell = 16 * s + 8 * e + 4 * h + qq;
            const int sw = (cell >> 1) & 3;
            const int chunk = 2 * (g16 & 1) + (pp >> 1);
            const int ro = cell * 64 + ((chunk ^ sw) * 16) + (pp & 1) * 8;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const uint2 v = bs_tr(scr + kBSY0 + p * 2048 + ro);
              yb[p][2 * e] = v.x;
              yb[p][2 * e + 1] = v.y;
            }
            const uint2 vp = bs_tr(scr + kBSP + ro), vq = bs_tr(scr + kBSQ + ro);
            pb[2 * e] = vp.x;
            pb[2 * e + 1] = vp.y;
            qb[2 * e] = vq.x;
            qb[2 * e + 1] = vq.y;
          }
          BS_SIX(dw1a[sl], dhf[s], yb);
          dw1b[sl] = bs_mfma(dhf[s][0], pb, dw1b[sl]);
          dw1b[sl] = bs_mfma(dhf[s][1], pb, dw1b[sl]);
          dw1b[sl] = bs_mfma(dhf[s][2], pb, dw1b[sl]);
          dw1b[sl] = bs_mfma(dhf[s][0], qb, dw1b[sl]);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (!first) continue;   // dY: the first launch only
        // dh with the cells on the lane (dY's B operand): image [part][hidden][cell], 8-byte slots
        // XOR (hidden >> 1) & 7; this lane's registers 4m..4m+3 are cells 8m + 4h + 0..3
        {
          const int rsw = (r32 >> 1) & 7;
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const int slot = (2 * m + h) ^ rsw;
              *reinterpret_cast<uint2*>(scr + kBSDH + p * 2048 + r32 * 64 + slot * 8) =
                  uint2{dhf[m >> 1][p][2 * (m & 1)], dhf[m >> 1][p][2 * (m & 1) + 1]};
            }
        }
        asm volatile("" ::: "memory");
        // dY [feature x cell] += W1^T dh over hidden 32nb + 16s2 + 8h + j
#pragma unroll
        for (int s2 = 0; s2 < 2 * !(BS_ABL & 1); ++s2) {
          bsu4 db[3], wa[3], wx[3];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int hrow = 16 * s2 + 8 * h + 4 * e + qq;   // hidden within the block
            const int slot = (4 * (g16 & 1) + pp) ^ ((hrow >> 1) & 7);
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const uint2 v = bs_tr(scr + kBSDH + p * 2048 + hrow * 64 + slot * 8);
              db[p][2 * e] = v.x;
              db[p][2 * e + 1] = v.y;
            }
            // W1^T (A): rows = hidden 32nb + hrow, columns = features 16 (g16 & 1) + 4p (block 0) or
            // 32 + 4p of part (r32 < 16 ? X : Y) (block 1, stacked)
            const int wrow = (32 * nb + hrow) * 96;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const uint2 v = bs_tr(smb + L.w1i + p * kBSW1Part + wrow + (16 * (g16 & 1) + 4 * pp) * 2);
              wa[p][2 * e] = v.x;
              wa[p][2 * e + 1] = v.y;
            }
            // block 1 stacks: [w0; w1], [w0; w2], [w2; 0]: the part each lane half reads
            const bool top = r32 < 16;
            const uint2 v1 = bs_tr(smb + L.w1i + (top ? 0 : 1) * kBSW1Part + wrow + (32 + 4 * pp) * 2);
            const uint2 v2 = bs_tr(smb + L.w1i + (top ? 0 : 2) * kBSW1Part + wrow + (32 + 4 * pp) * 2);
            const uint2 v3 = bs_tr(smb + L.w1i + 2 * kBSW1Part + wrow + (32 + 4 * pp) * 2);
            wx[0][2 * e] = v1.x;
            wx[0][2 * e + 1] = v1.y;
            wx[1][2 * e] = v2.x;
            wx[1][2 * e + 1] = v2.y;
            wx[2][2 * e] = top ? v3.x : 0u;
            wx[2][2 * e + 1] = top ? v3.y : 0u;
          }
          BS_SIX(dy0, wa, db);
          dy1 = bs_mfma(wx[0], db[0], dy1);   // [w0; w1] dh0
          dy1 = bs_mfma(wx[0], db[1], dy1);   // [w0; w1] dh1
          dy1 = bs_mfma(wx[1], db[2], dy1);   // [w0; w2] dh2
          dy1 = bs_mfma(wx[2], db[0], dy1);   // [w2; 0] dh0
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
      // (9) dY -> HBM: features rowof(r, h) (block 0) and 32 + rowof(r, h) (block 1, two stacked halves)
      if (valid && first && !(BS_ABL & 8)) {
        float* qy = dYb + celli;
#pragma unroll
        for (int r = 0; r < 16; ++r) qy[(size_t)bs_rowof(r, h) * HWi] = dy0[r];
#pragma unroll
        for (int r = 0; r < 8; ++r) qy[(size_t)(32 + bs_rowof(r, h)) * HWi] = dy1[r] + dy1[r + 8];
      }
    }
  }

  // ---- this wave's partial gradients -> its own row (summed in a fixed order by gnca_b_reduce) ----
  float* outp = a.part + ((size_t)blockIdx.x * NW + wave) * a.npart;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int hid = h0 + 32 * nb + bs_rowof(r, h);
      outp[a.o_w1 + hid * 48 + r32] = dw1a[nb][r];
      const float v = dw1b[nb][r] + __shfl_xor(dw1b[nb][r], 16);
      if (r32 < 16) outp[a.o_w1 + hid * 48 + 32 + r32] = v;
    }
    const float b1t = ab1[nb] + __shfl_xor(ab1[nb], 32);
    if (h == 0) outp[a.o_b1 + h0 + 32 * nb + r32] = b1t;
#pragma unroll
    for (int r = 0; r < 8; ++r) outp[a.o_w2 + bs_rowof(r, h) * HD + h0 + 32 * nb + r32] = dw2[nb][r] + dw2[nb][r + 8];
  }
  if (!first) return;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    float v = dwm[r] + dwm[r + 8];
    v += __shfl_xor(v, 16);
    if (r32 < 16) outp[a.o_wm + bs_rowof(r, h) * C + r32] = v;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = abm[j];
    for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (r32 == 0) outp[a.o_bm + bs_rowof(j, h)] = v;
  }
}
