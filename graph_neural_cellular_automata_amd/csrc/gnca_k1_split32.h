// gnca_k1_split32.h — K1 of the 32-channel / hidden-128 step (BASELINE config 5: 128^2, r = 5,
// K = 16) on bf16 MFMA with the exact 3-way fp32 splits of gnca_k1_split.h (included after it).
//
// Why.  The fp32-MFMA two-phase K1 (gnca_k1_2ph) spends 17 K of its 52 K cycles per 16x16 tile in
// fp32 MFMA issue (1/16 of the bf16 rate, on the VALU datapath).  Here every product is six exact
// bf16 products (numerics as gnca_k1_split.h: fp32-class, dropped terms <= 2^-24 |a||b| each).
//
// Tile pipeline (as gnca_k1_2ph): 16x16 tiles, the region's channel planes staged in two
// 16-channel phases through one LDS buffer (dword LDS-DMA: RW = 26 is not quad-aligned), alive /
// sender / keep planes, live-cell compaction, one 32-cell group per wave (<= 8 groups per tile),
// every accumulator of the group kept in registers across the phase boundary.
//
// MFMA (v_mfma_f32_32x32x16_bf16; lane l: cell l & 31, half h = l >> 5; D reg r -> row
// (r&3) + 8(r>>2) + 4h):
//   GEMM1  H[128 x 32] = W1[128 x 96] Y + b1: k-chunk (f, p) = feature f of channels 16p..16p+15,
//          W1 columns 32f + 16p + 8h + j, so in phase p lane (cell, h) computes the perception of
//          channels 16p + 8h + j, its B slots.  4 row blocks x (bias + 6 chunks x 6 products).
//   GEMM2  DL[32 x 32] = W2[32 x 128] relu(H): k-chunk s = (rb, ss) is accumulator registers
//          8ss..8ss+7 of block rb (hidden 32rb + 16ss + 8(j>>2) + 4h + (j&3), the A image
//          permuted to match), 6 products each, all 32 output channels in one accumulator.
//   MSG    M[32 x 32] = WM[32 x 32] G: k-chunk p = the gathered channels of phase p.
// Weight images (bf16 parts): W1 72 KB, bias 2 KB, W2 24 KB, WM 6 KB.  LDS total ~155 KB.

#pragma once

namespace gnca {

struct KS32Layout {
  int xs, sp, al, kp, lst, wcnt, w1, bias, w2, wm, bml, total;   // byte offsets
};

template <int TH, int TW, int RY, int RX>
__host__ __device__ constexpr KS32Layout ks32_layout() {
  constexpr int RH = TH + 2 * RY, RW = TW + 2 * RX, RHW = RH * RW;
  constexpr int NI = (RHW + 63) / 64, NIA = ((RH + 2) * (RW + 2) + 63) / 64;
  KS32Layout L{};
  int o = 0;
  L.xs = o; o += 16 * ks_pstr(RHW) * 4;           // one phase's 16 channel planes
  L.sp = o; o += ks_a16(RHW * 4);
  L.al = o; o += 64 * 4 * (NIA > NI ? NIA : NI);  // alive bytes (one per dword) or the alpha ring
  L.kp = o; o += ks_a16(TH * TW);
  L.lst = o; o += ks_a16(TH * TW * 2);
  L.wcnt = o; o += 32;
  L.w1 = o; o += 4 * 3 * 2 * 3 * 1024;            // [rb][f][p][part][lane] x 16 B
  L.bias = o; o += 4 * 32 * 16;                   // [rb][row] x 16 B
  L.w2 = o; o += 8 * 3 * 1024;                    // [s][part][lane] x 16 B
  L.wm = o; o += 2 * 3 * 1024;                    // [p][part][lane] x 16 B
  L.bml = o; o += 2 * 16 * 4;                     // message bias per (h, accumulator register r)
  L.total = o;
  return L;
}

template <int TH, int TW, int RY, int RX, int KU>
__global__ __launch_bounds__(512, 1) void gnca_k1_split32(const K1Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem_b[];
  constexpr int C = 32, HD = 128, NT = 512, NW = 8;
  constexpr int RH = TH + 2 * RY, RW = TW + 2 * RX, RHW = RH * RW;
  constexpr int PSTR = ks_pstr(RHW);
  constexpr int NI = (RHW + 63) / 64;
  constexpr int ALW = RW + 2, NIA = ((RH + 2) * ALW + 63) / 64;
  constexpr int NCELL = TH * TW;
  constexpr KS32Layout L = ks32_layout<TH, TW, RY, RX>();
  static_assert(NCELL <= 32 * NW, "one 32-cell group per wave");
  static_assert(RY >= 1 && RX >= 1, "perception halo");
  static_assert(L.total <= 160 * 1024, "LDS");
  static_assert(7 * PSTR * 4 + 4 * RHW < 65536, "channel offsets fit the DS immediate");
  constexpr bool GRAPH = KU > 0;

  float* xs = reinterpret_cast<float*>(smem_b + L.xs);
  float* sp = reinterpret_cast<float*>(smem_b + L.sp);
  float* al = reinterpret_cast<float*>(smem_b + L.al);
  uint8_t* kp = reinterpret_cast<uint8_t*>(smem_b + L.kp);
  uint16_t* lst = reinterpret_cast<uint16_t*>(smem_b + L.lst);
  int* wcnt = reinterpret_cast<int*>(smem_b + L.wcnt);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int H = a.H, W = a.W;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool compact = a.rmask != nullptr;   // the rollout's compact update field (gnca_k1_split.h)
  static_assert(TW <= 64, "one ballot per tile row (compact update field)");
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const float thr = a.alpha_thr, gthr = a.graph_alpha_thr;

  // ---- weight images (bf16 parts in MFMA fragment order), once per persistent workgroup ----
  {
    // W1: entry (rb, f, p, l): W1[32rb + (l&31)][32f + 16p + 8(l>>5) + 0..7]
    for (int e = tid; e < 4 * 3 * 2 * 64; e += NT) {
      const int l = e & 63, p = (e >> 6) & 1, f = (e >> 7) % 3, rb = e / 384;
      const float* src = a.w1 + (size_t)(32 * rb + (l & 31)) * (3 * C) + 32 * f + 16 * p + 8 * (l >> 5);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[j];
      u32x4 f0, f1, f2;
      split3_x8(v, f0, f1, f2);
      const int img = L.w1 + ((rb * 3 + f) * 2 + p) * 3 * 1024 + l * 16;
      *reinterpret_cast<u32x4*>(smem_b + img) = f0;
      *reinterpret_cast<u32x4*>(smem_b + img + 1024) = f1;
      *reinterpret_cast<u32x4*>(smem_b + img + 2048) = f2;
    }
    // bias: entry (rb, row): k slots 0..2 = the parts of b1[32rb + row]
    for (int e = tid; e < 128; e += NT) {
      uint32_t p0, p1, p2;
      split3_pair(a.b1[e], 0.f, p0, p1, p2);
      u32x4 f;
      f[0] = (p0 & 0xffffu) | (p1 << 16);
      f[1] = p2 & 0xffffu;
      f[2] = 0u;
      f[3] = 0u;
      *reinterpret_cast<u32x4*>(smem_b + L.bias + e * 16) = f;
    }
    // W2: entry (s, l): W2[l&31][32(s>>1) + 16(s&1) + 8(j>>2) + 4(l>>5) + (j&3)], j = 0..7
    for (int e = tid; e < 8 * 64; e += NT) {
      const int s = e >> 6, l = e & 63;
      const float* src = a.w2 + (size_t)(l & 31) * HD + 32 * (s >> 1) + 16 * (s & 1) + 4 * (l >> 5);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[8 * (j >> 2) + (j & 3)];
      u32x4 f0, f1, f2;
      split3_x8(v, f0, f1, f2);
      const int img = L.w2 + s * 3 * 1024 + l * 16;
      *reinterpret_cast<u32x4*>(smem_b + img) = f0;
      *reinterpret_cast<u32x4*>(smem_b + img + 1024) = f1;
      *reinterpret_cast<u32x4*>(smem_b + img + 2048) = f2;
    }
    // WM: entry (p, l): WM[l&31][16p + 8(l>>5) + 0..7]
    for (int e = tid; e < 2 * 64; e += NT) {
      const int p = e >> 6, l = e & 63;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = GRAPH ? a.wm[(l & 31) * C + 16 * p + 8 * (l >> 5) + j] : 0.f;
      u32x4 f0, f1, f2;
      split3_x8(v, f0, f1, f2);
      const int img = L.wm + p * 3 * 1024 + l * 16;
      *reinterpret_cast<u32x4*>(smem_b + img) = f0;
      *reinterpret_cast<u32x4*>(smem_b + img + 1024) = f1;
      *reinterpret_cast<u32x4*>(smem_b + img + 2048) = f2;
    }
    // message bias of output channel (r&3) + 8(r>>2) + 4h at [h][r]
    if (tid < 32) {
      const int hh = tid >> 4, r = tid & 15;
      reinterpret_cast<float*>(smem_b + L.bml)[tid] = GRAPH ? a.bm[(r & 3) + 8 * (r >> 2) + 4 * hh] : 0.f;
    }
    // the perception zero tap: every channel plane's pad floats (never written by the staging)
    for (int e = tid; e < 16 * (PSTR - RHW); e += NT) xs[(e / (PSTR - RHW)) * PSTR + RHW + e % (PSTR - RHW)] = 0.f;
  }
  int ok = 1;
  for (int idx = tid; idx < C * 27; idx += NT) {
    const int e = idx % 27, f = e / 9, tap = e % 9, tr = tap / 3, tc = tap % 3;
    float ref;
    if (f == 0) ref = (tap == 4) ? 1.f : 0.f;
    else if (f == 1) ref = (float)((tc == 0 ? 1 : (tc == 2 ? -1 : 0)) * (tr == 1 ? 2 : 1));
    else ref = (float)((tr == 0 ? 1 : (tr == 2 ? -1 : 0)) * (tc == 1 ? 2 : 1));
    if (a.perc[idx] != ref) ok = 0;
  }
  const bool sobel = __syncthreads_and(ok) != 0;   // also the barrier after the image stores

  const u32x4 ones = h == 0 ? u32x4{0x3f803f80u, 0x3f80u, 0u, 0u} : u32x4{0u, 0u, 0u, 0u};
  const float mgain = GRAPH ? a.message_gain : 0.f;
  const bool hz = hidden_only && h == 0;   // channels (r&3) + 4h < 4 (r < 4) are the RGBA ones
  const size_t HW = (size_t)H * W;

  // XCD-aware tile order (as gnca_k1_update)
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
    if (a.active && !a.active[b]) {   // inactive sample (masked step)
      if (tid < 2 * NW) a.stats[(size_t)tile * 2 * NW + tid] = 0.0;
      continue;
    }
    // channel planes [16ph, 16ph + 16) of the (RH x RW) region -> xs (torus-wrapped), dword DMA
    auto stage = [&](int ph) {
#pragma unroll 1
      for (int ii_ = wave; ii_ < ((GNCA_ABLATE & kAblStage) ? 0 : NI); ii_ += NW) {
        const int e = 64 * ii_ + lane;
        if (e < RHW) {   // lanes past the region masked off: the plane pads (zero taps) stay zero
          const int vr = e / RW, vc = e - (e / RW) * RW;
          int ii = i0 - RY + vr, jj = j0 - RX + vc;
          ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
          jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
          const float* src0 = xb + (size_t)(16 * ph) * HW + ii * W + jj;
          float* dst = xs + 64 * ii_;
#pragma unroll 4
          for (int c = 0; c < 16; ++c)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src0 + (size_t)c * HW),
                                             (__attribute__((address_space(3))) void*)(dst + c * PSTR), 4, 0, 0);
        }
      }
    };
    __syncthreads();   // the previous tile's LDS readers are done
    stage(0);
    if (a.alive) {
      // the previous K2's alive bytes over the region, one byte per dword
      const uint8_t* ab = a.alive + (size_t)b * HW;
#pragma unroll 1
      for (int ii_ = wave; ii_ < NI; ii_ += NW) {
        const int e = 64 * ii_ + lane;
        int off = 0;
        if (e < RHW) {
          const int vr = e / RW, vc = e - (e / RW) * RW;
          int ii = i0 - RY + vr, jj = j0 - RX + vc;
          ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
          jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
          off = ii * W + jj;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(ab + off),
                                         (__attribute__((address_space(3))) void*)(al + 64 * ii_), 1, 0, 0);
      }
    } else {
      // alpha plane with one more ring: element e of ((RH+2) x ALW) -> (i0-RY-1+vr, j0-RX-1+vc)
#pragma unroll 1
      for (int ii_ = wave; ii_ < NIA; ii_ += NW) {
        const int e = 64 * ii_ + lane;
        int off = 0;
        if (e < (RH + 2) * ALW) {
          const int vr = e / ALW, vc = e - (e / ALW) * ALW;
          int ii = i0 - RY - 1 + vr, jj = j0 - RX - 1 + vc;
          while (ii < 0) ii += H;
          while (ii >= H) ii -= H;
          while (jj < 0) jj += W;
          while (jj >= W) jj -= W;
          off = ii * W + jj;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xb + 3 * HW + off),
                                         (__attribute__((address_space(3))) void*)(al + 64 * ii_), 4, 0, 0);
      }
    }
    // ---- fire plane while the DMA is in flight ----
#pragma unroll 1
    for (int n = tid; n < NCELL; n += NT) {
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const size_t cell = (size_t)(i0 + ti) * W + (j0 + tj);
      kp[n] = fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step, a.sample_base, b, HW, cell) ? 1 : 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- sender plane over the region, keep = pre-alive AND fire over the tile ----
    if (a.alive) {
      const int* alw = reinterpret_cast<const int*>(al);
#pragma unroll 1
      for (int pos = tid; pos < RHW; pos += NT) {
        const int vr = pos / RW, vc = pos - (pos / RW) * RW;
        const int v = alw[pos] & 0xff;
        sp[pos] = a2a ? (float)((v >> 1) & 1) : 1.f;
        const int ti = vr - RY, tj = vc - RX;
        if (ti >= 0 && ti < TH && tj >= 0 && tj < TW && !(v & 1)) kp[ti * TW + tj] = 0;
      }
    } else {
#pragma unroll 1
      for (int pos = tid; pos < RHW; pos += NT) {
        const int vr = pos / RW, vc = pos - (pos / RW) * RW;
        int iq = i0 - RY + vr, jq = j0 - RX + vc;
        while (iq < 0) iq += H;
        while (iq >= H) iq -= H;
        while (jq < 0) jq += W;
        while (jq >= W) jq -= W;
        const float* q = al + (vr + 1) * ALW + (vc + 1);
        const float NEG = -INFINITY;
        const bool up = iq > 0, dn = iq < H - 1, lf = jq > 0, rt = jq < W - 1;
        const float mu_ = fmaxf(fmaxf(lf ? q[-ALW - 1] : NEG, q[-ALW]), rt ? q[-ALW + 1] : NEG);
        const float mm_ = fmaxf(fmaxf(lf ? q[-1] : NEG, q[0]), rt ? q[1] : NEG);
        const float md_ = fmaxf(fmaxf(lf ? q[ALW - 1] : NEG, q[ALW]), rt ? q[ALW + 1] : NEG);
        const float mx = fmaxf(fmaxf(up ? mu_ : NEG, mm_), dn ? md_ : NEG);
        sp[pos] = a2a ? (mx > gthr ? 1.f : 0.f) : 1.f;
        const int ti = vr - RY, tj = vc - RX;
        if (ti >= 0 && ti < TH && tj >= 0 && tj < TW && !(mx > thr)) kp[ti * TW + tj] = 0;
      }
    }
    __syncthreads();

    // ---- live-cell compaction (cell order, wave ballots: deterministic); dead cells get dx = 0 ----
    const size_t cell0 = (size_t)i0 * W + j0;
    float* outb = a.out + (size_t)b * C * HW + cell0;
    int nlive = 0;
    {
      const int n = tid;
      const bool inb = n < NCELL;
      const bool live = inb && kp[n] != 0;
      const uint64_t bal = __ballot(live);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wcnt[wave] = __popcll(bal);
      __syncthreads();
      int off = 0;
#pragma unroll
      for (int w_ = 0; w_ < NW; ++w_) {
        off += w_ < wave ? wcnt[w_] : 0;
        nlive += wcnt[w_];
      }
      if (compact && inb && n % TW == 0) a.rpre[(size_t)tile * TH + n / TW] = (uint32_t)(off + pre);
      if (live) {
        lst[off + pre] = (uint16_t)n;
      } else if (inb && !compact) {   // (compact: K2 masks the alpha plane by the row tables)
        const int ti = n / TW, tj = n - (n / TW) * TW;
        float* oz = outb + (size_t)ti * W + tj;
#pragma unroll
        for (int c = 0; c < C; ++c) oz[(size_t)c * HW] = 0.f;
      }
      __syncthreads();
    }
    if (compact) {   // per-row live masks of the compact update field
#pragma unroll 1
      for (int ti_ = wave; ti_ < TH; ti_ += NW) {
        const uint64_t m = __ballot(lane < TW && kp[ti_ * TW + (lane < TW ? lane : 0)] != 0);
        if (lane == 0) a.rmask[(size_t)tile * TH + ti_] = m;
      }
    }

    // ---- one 32-cell group per wave; its accumulators live across the two channel phases ----
    const bool has = 32 * wave < nlive;   // wave-uniform
    const int gi = 32 * wave + r32;
    const bool valid = gi < nlive;
    const int n = has ? lst[valid ? gi : 0] : 0;
    const int ti = n / TW, tj = n - (n / TW) * TW;
    const int pidx = (RY + ti) * RW + (RX + tj);
    const int hb = 8 * h * PSTR;   // this lane's channel half within a phase
    const bool img_top = i0 == 0, img_bot = i0 + TH == H, img_lft = j0 == 0, img_rgt = j0 + TW == W;

    // each phase leaves its perception / gather operands as bf16 fragments (48 VGPRs), the GEMMs run
    // after phase 1 (fewer registers across the phase boundary than GEMM1's accumulators)
    u32x4 yfr[2][3][3], gfr[2][3];   // [phase][f][part], [phase][part]
    float S = 0.f;
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      if (ph == 1) {
        __syncthreads();   // every wave is done with phase 0's planes
        stage(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      if (!has) continue;
      // -- gather of alive-masked x, this phase's channels 16ph + 8h + j (uniform weight 1/k) --
      u32x4 g0 = {0u, 0u, 0u, 0u}, g1 = g0, g2 = g0;
      if constexpr (GRAPH) if (!(GNCA_ABLATE & kAblGather)) {
        float gv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = 0.f;
        const float* xq = xs + hb + pidx;
        const float* spq = sp + pidx;
        float Sp = 0.f;
#pragma unroll
        for (int o = 0; o < KU; ++o) {
          const int d = a.odl[o];
          const float s_ = spq[-d];
          Sp += s_;
          const float* xo = xq - d;
#pragma unroll
          for (int j = 0; j < 8; ++j) gv[j] = fmaf(s_, xo[j * PSTR], gv[j]);
          if ((o & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // <= 4 offsets' reads in flight
        }
        const float wu = a.uniform_w;
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] *= wu;
        if (ph == 0) S = Sp * wu;
        split3_x8(gv, g0, g1, g2);
        // materialise here (before the perception's sobel / generic branch): otherwise the
        // gather arithmetic is sunk past the branch and its 128 loaded floats stay live (spills)
        asm volatile("" : "+v"(g0), "+v"(g1), "+v"(g2));
      }
      gfr[ph][0] = g0;
      gfr[ph][1] = g1;
      gfr[ph][2] = g2;
      __builtin_amdgcn_sched_barrier(0);

      // -- perception of channels 16ph + 8h + j (zero padding at the image border via zero taps) --
      float y0[8], y1[8], y2[8];
      const int ic = i0 + ti, jc = j0 + tj;
      const bool up = !(img_top && ic == 0), dn = !(img_bot && ic == H - 1);
      const bool lf = !(img_lft && jc == 0), rt = !(img_rgt && jc == W - 1);
      const int zt = RHW + hb;   // the zero tap of this lane's first channel plane
      const int bc = pidx + hb;
      const int t0 = (up && lf) ? bc - RW - 1 : zt, t1 = up ? bc - RW : zt, t2 = (up && rt) ? bc - RW + 1 : zt;
      const int t3 = lf ? bc - 1 : zt, t5 = rt ? bc + 1 : zt;
      const int t6 = (dn && lf) ? bc + RW - 1 : zt, t7 = dn ? bc + RW : zt, t8 = (dn && rt) ? bc + RW + 1 : zt;
      if (GNCA_ABLATE & kAblPerceive) {
#pragma unroll
        for (int j = 0; j < 8; ++j) y0[j] = y1[j] = y2[j] = 0.f;
      } else if (sobel) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int co = j * PSTR;
          const float n0 = xs[t0 + co], n1 = xs[t1 + co], n2 = xs[t2 + co];
          const float n3 = xs[t3 + co], n4 = xs[bc + co], n5 = xs[t5 + co];
          const float n6 = xs[t6 + co], n7 = xs[t7 + co], n8 = xs[t8 + co];
          y0[j] = n4;
          y1[j] = (fmaf(2.f, n3, n0) + n6) - (fmaf(2.f, n5, n2) + n8);
          y2[j] = (fmaf(2.f, n1, n0) + n2) - (fmaf(2.f, n7, n6) + n8);
        }
      } else {
#pragma unroll 1
        for (int j = 0; j < 8; ++j) {
          const int co = j * PSTR;
          const float nn[9] = {xs[t0 + co], xs[t1 + co], xs[t2 + co], xs[t3 + co], xs[bc + co],
                               xs[t5 + co], xs[t6 + co], xs[t7 + co], xs[t8 + co]};
          const float* pw = a.perc + (size_t)3 * (16 * ph + 8 * h + j) * 9;
          float acc3[3];
#pragma unroll
          for (int f = 0; f < 3; ++f) {
            float s_ = pw[9 * f] * nn[0];
#pragma unroll
            for (int t = 1; t < 9; ++t) s_ = fmaf(pw[9 * f + t], nn[t], s_);
            acc3[f] = s_;
          }
          y0[j] = acc3[0];
          y1[j] = acc3[1];
          y2[j] = acc3[2];
        }
      }
      split3_x8(y0, yfr[ph][0][0], yfr[ph][0][1], yfr[ph][0][2]);
      split3_x8(y1, yfr[ph][1][0], yfr[ph][1][1], yfr[ph][1][2]);
      split3_x8(y2, yfr[ph][2][0], yfr[ph][2][1], yfr[ph][2][2]);
      // materialise this phase's fragments here: otherwise the compiler sinks the gather /
      // perception arithmetic to its uses after phase 1 and keeps ~200 loaded floats live across
      // the phase boundary (spills)
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        asm volatile("" : "+v"(yfr[ph][f][0]), "+v"(yfr[ph][f][1]), "+v"(yfr[ph][f][2]));
        asm volatile("" : "+v"(gfr[ph][f]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    float s1 = 0.f, s2 = 0.f;
    if (has && !(GNCA_ABLATE & kAblMfma)) {
      // -- message: chunks p = 0, 1, 6 products each --
      f32x16 accm = {};
      if constexpr (GRAPH) {
#pragma unroll
        for (int ph = 0; ph < 2; ++ph) {
          const int img = L.wm + ph * 3 * 1024 + lane * 16;
          const u32x4 m0 = *reinterpret_cast<const u32x4*>(smem_b + img);
          const u32x4 m1 = *reinterpret_cast<const u32x4*>(smem_b + img + 1024);
          const u32x4 m2 = *reinterpret_cast<const u32x4*>(smem_b + img + 2048);
          accm = mfma_bx(m0, gfr[ph][0], accm);
          accm = mfma_bx(m0, gfr[ph][1], accm);
          accm = mfma_bx(m1, gfr[ph][0], accm);
          accm = mfma_bx(m0, gfr[ph][2], accm);
          accm = mfma_bx(m2, gfr[ph][0], accm);
          accm = mfma_bx(m1, gfr[ph][1], accm);
        }
      }
      // -- per row block rb: GEMM1 (bias + 6 chunks x 6 products), ReLU / split, GEMM2 k-chunks
      //    2rb, 2rb+1 (6 products each; one accumulator for all 32 output channels) --
      f32x16 accD = {};
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        const u32x4 bz = *reinterpret_cast<const u32x4*>(smem_b + L.bias + rb * 512 + r32 * 16);
        f32x16 acc1 = mfma_bx(bz, ones, f32x16{});
#pragma unroll
        for (int ph = 0; ph < 2; ++ph)
#pragma unroll
          for (int f = 0; f < 3; ++f) {
            const int img = L.w1 + ((rb * 3 + f) * 2 + ph) * 3 * 1024 + lane * 16;
            const u32x4 a0 = *reinterpret_cast<const u32x4*>(smem_b + img);
            const u32x4 a1 = *reinterpret_cast<const u32x4*>(smem_b + img + 1024);
            const u32x4 a2 = *reinterpret_cast<const u32x4*>(smem_b + img + 2048);
            acc1 = mfma_bx(a0, yfr[ph][f][0], acc1);
            acc1 = mfma_bx(a0, yfr[ph][f][1], acc1);
            acc1 = mfma_bx(a1, yfr[ph][f][0], acc1);
            acc1 = mfma_bx(a0, yfr[ph][f][2], acc1);
            acc1 = mfma_bx(a2, yfr[ph][f][0], acc1);
            acc1 = mfma_bx(a1, yfr[ph][f][1], acc1);
          }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int s = 2 * rb + ss;
          float hv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) hv[j] = relu_nan(acc1[8 * ss + j]);
          u32x4 h0, h1, h2;
          split3_x8(hv, h0, h1, h2);
          const int img = L.w2 + s * 3 * 1024 + lane * 16;
          const u32x4 p0 = *reinterpret_cast<const u32x4*>(smem_b + img);
          const u32x4 p1 = *reinterpret_cast<const u32x4*>(smem_b + img + 1024);
          const u32x4 p2 = *reinterpret_cast<const u32x4*>(smem_b + img + 2048);
          accD = mfma_bx(p0, h0, accD);
          accD = mfma_bx(p0, h1, accD);
          accD = mfma_bx(p1, h0, accD);
          accD = mfma_bx(p0, h2, accD);
          accD = mfma_bx(p2, h0, accD);
          accD = mfma_bx(p1, h1, accD);
        }
        __builtin_amdgcn_sched_barrier(0);   // bounds the fragment prefetch (registers)
      }

      // -- epilogue: dx = (dl + tanh(m) * gain) * keep for channels c = (r&3) + 8(r>>2) + 4h --
      if (valid) {
        // dense: NCHW; compact: [tile][channel][live index]
        float* ob = compact ? a.out + (size_t)tile * C * NCELL + (size_t)(4 * h) * NCELL + gi
                            : outb + (size_t)(ti * W + tj) + (size_t)(4 * h) * HW;
        const size_t cstr = compact ? (size_t)NCELL : HW;
        const float* bmp = reinterpret_cast<const float*>(smem_b + L.bml) + 16 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = accD[r];
          if constexpr (GRAPH) v = fmaf(fast_tanh(fmaf(bmp[r], S, accm[r])), (hz && r < 4) ? 0.f : mgain, v);
          if (compact && h == 0 && r == 3) a.dxa[(size_t)b * HW + cell0 + (size_t)(ti * W + tj)] = v;   // alpha: dense
          else ob[(size_t)((r & 3) + 8 * (r >> 2)) * cstr] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
    }

    // ---- per-(tile, wave) GroupNorm partials (fp64 wave shuffle; K2 sums them in fixed order) ----
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
}

}  // namespace gnca
