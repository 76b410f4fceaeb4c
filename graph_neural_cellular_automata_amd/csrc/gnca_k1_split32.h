// gnca_k1_split32.h — K1 of the 32-channel / hidden-128 step (BASELINE config 5: 128^2, r = 5,
// K = 16) on bf16 MFMA with the exact 3-way fp32 splits of gnca_k1_split.h (included after it).
//
// Why.  Round 1's fp32-MFMA two-phase K1 (since removed) spent 17 K of its 52 K cycles per 16x16
// tile in fp32 MFMA issue (1/16 of the bf16 rate, on the VALU datapath).  Here every product is six exact
// bf16 products (numerics as gnca_k1_split.h: fp32-class, dropped terms <= 2^-24 |a||b| each).
//
// Tile pipeline: 16x16 tiles, the region's channel planes staged in two 16-channel phases through
// one LDS buffer (dword LDS-DMA: RW = 26 is not quad-aligned), one 32-cell group per wave (<= 8
// groups per tile), every accumulator of the group kept in registers across the phase boundary.
// As in gnca_k1_split.h: a preparer wave (wave 7, which has no group unless > 224 cells of the tile
// are live) builds the next tile's sender plane, keep mask, live-cell list and compact-field row
// tables into a second LDS slot while the groups run, and stages the next tile's phase-0 planes
// as soon as every group is past its phase-1 reads, under the groups' MFMAs.
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

#ifndef GNCA_S32_PREP_SPLIT
#define GNCA_S32_PREP_SPLIT 0   // A/B builds: the next tile's sender plane and its live list by two waves side by side
                                // (c5 step 0.660 vs 0.656 ms with the preparer alone: not kept)
#endif

#ifndef GNCA_S32_PREP_PRIO
#define GNCA_S32_PREP_PRIO 3
#endif

#ifndef GNCA_S32_STAGERS
#define GNCA_S32_STAGERS 1   // the next tile's phase-0 DMA split over the waves without a group (0: the preparer alone)
#endif

struct KS32Layout {
  int xs, sp, ab, lst, cnt, cb, w1, bias, w2, wm, bml, total;   // byte offsets
  int sp_slot, lst_slot;                                         // bytes per prepared-tile slot
};

// channel-plane stride of the 32-channel kernel's staged region: at least one pad float (the zero
// tap of the border perception), quads (16-byte LDS-DMA rows); no bank offset between planes (the
// two lane halves' ds_read_b32 reads are separate LDS cycles), so the 26 x 32 region fits 160 KB
__host__ __device__ constexpr int ks32_pstr(int rhw) { return (rhw + 1 + 3) & ~3; }

template <int TH, int TW, int RY, int RX>
__host__ __device__ constexpr KS32Layout ks32_layout() {
  constexpr int RH = TH + 2 * RY, RW = TW + 2 * RX, RHW = RH * RW;
  KS32Layout L{};
  int o = 0;
  L.sp_slot = ks_a16(RHW);
  L.lst_slot = ks_a16(TH * TW);   // u8 cell indices (TH * TW <= 256)
  L.xs = o; o += 16 * ks32_pstr(RHW) * 4;         // one phase's 16 channel planes
  L.sp = o; o += 2 * L.sp_slot;                   // sender plane (bytes 0/1), two slots
  L.ab = o; o += ks_a16(RHW);                     // the preparer's alive bytes over the region
  L.lst = o; o += 2 * L.lst_slot;                 // live-cell list (u8), two slots
  L.cnt = o; o += 16;                             // live cells per slot; staged-reads-done counter
  L.cb = o; o += ks_a16(8 * (TH * TW / 64 + 2));  // the preparer's 64-cell chunk ballots
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
  constexpr int PSTR = ks32_pstr(RHW);
  constexpr int NQ = RHW / 4, NI4 = (NQ + 63) / 64;   // 16-byte quads of a channel plane
  static_assert(RW % 4 == 0 && RX % 4 == 0 && TW % 4 == 0, "16-byte staging rows");
  constexpr int NCELL = TH * TW;
  constexpr KS32Layout L = ks32_layout<TH, TW, RY, RX>();
  static_assert(NCELL <= 32 * NW, "one 32-cell group per wave");
  static_assert(RY >= 1 && RX >= 1, "perception halo");
  static_assert(L.total + 512 <= 160 * 1024, "LDS (+ the compiler's static LDS, e.g. __syncthreads_and)");
  static_assert(NCELL <= 256, "u8 live-cell indices");
  static_assert(7 * PSTR * 4 + 4 * RHW < 65536, "channel offsets fit the DS immediate");
  constexpr bool GRAPH = KU > 0;
  constexpr int PW = NW - 1;   // the preparer / next-tile stager (no group unless > 224 live cells)

  wg_stamp(a.stamps, 0);
  float* xs = reinterpret_cast<float*>(smem_b + L.xs);
  int* cnt = reinterpret_cast<int*>(smem_b + L.cnt);
  int* xsd = cnt + 2;   // groups past their phase-1 reads, 64 per group (monotonic over the tiles)
  int xbase = 0;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r32 = lane & 31;
  const int H = a.H, W = a.W;
  const bool a2a = (a.flags & GNCA_ALIVE_TO_ALIVE) != 0;
  const bool compact = a.rmask != nullptr;   // the rollout's compact update field (gnca_k1_split.h)
  static_assert(TW <= 64, "one ballot per tile row (compact update field)");
  const bool hidden_only = (a.flags & GNCA_HIDDEN_ONLY) != 0;
  const size_t HW = (size_t)H * W;

  // XCD-aware tile order (as gnca_k1_update)
  const int nxcd = gridDim.x >= 8 ? 8 : 1;
  const int xg_ = blockIdx.x % nxcd, xr_ = blockIdx.x / nxcd;
  const int per_x = (int)(gridDim.x / nxcd) + ((int)(gridDim.x % nxcd) > xg_ ? 1 : 0);
  const int tq = a.total_tiles / nxcd, trm = a.total_tiles % nxcd;
  const int t_begin = xg_ * tq + min(xg_, trm), t_end = (GNCA_ABLATE & kAblTiles) ? t_begin : t_begin + tq + (xg_ < trm ? 1 : 0);
  auto next_active = [&](int t) {
    while (t < t_end && a.active && !a.active[t / a.tps]) {
      if (tid < 2 * NW) a.stats[(size_t)t * 2 * NW + tid] = 0.0;
      t += per_x;
    }
    return t;
  };

  // channel planes [16ph, 16ph + 16) of tile t's (RH x RW) region -> xs (torus-wrapped), 16-byte
  // LDS-DMA quads (RX, TW multiples of 4 and W % 4 == 0: a quad never straddles the wrap), quad
  // items w0, w0 + wstep, ... of (quad block, channel slice): with more waves than quad blocks the
  // 16 channels are sliced so every wave issues a share (8 waves, 4 blocks: 8 instructions each)
  auto stage = [&](int t, int ph, int w0, int wstep) {
    const int b = t / a.tps, tin = t - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const float* xb = a.x + (size_t)b * C * HW;
    int cs = 1;
    while (cs < 16 && wstep >= 2 * cs * NI4) cs *= 2;
    const int cn = 16 / cs;
#pragma unroll 1
    for (int it = w0; it < ((GNCA_ABLATE & kAblStage) ? 0 : NI4 * cs); it += wstep) {
      const int ii_ = it % NI4, c0 = (it / NI4) * cn;
      const int q = 64 * ii_ + lane;
      if (q < NQ) {   // lanes past the region masked off: the plane pads (zero taps) stay zero
        const int e = 4 * q, vr = e / RW, vc = e - (e / RW) * RW;
        int ii = i0 - RY + vr, jj = j0 - RX + vc;
        ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
        jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
        const float* src0 = xb + (size_t)(16 * ph + c0) * HW + ii * W + jj;
        float* dst = xs + 256 * ii_ + c0 * PSTR;
#pragma unroll 4
        for (int c = 0; c < cn; ++c)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src0 + (size_t)c * HW),
                                           (__attribute__((address_space(3))) void*)(dst + c * PSTR), 16, 0, 0);
      }
    }
  };

  // The preparer (one wave): tile t's sender plane over the region, keep = fire AND pre-alive, the
  // live-cell list into slot s, the compact field's row tables (and, dense field, the dead cells'
  // zeros).  The pre-update masks are the alive bytes (the previous K2's, or gnca_k_alive's).
  // part: 3 = everything (one wave), 1 = the region's sender plane only, 2 = the keep mask, live
  // list and row tables only (keep bits from the alive bytes in global memory): with a second wave
  // without a group the two halves run side by side
  auto prep = [&](int t, int s, int part) {
    // the preparer (the younger wave of its SIMD, beside a group wave) at the top issue priority
    // while it prepares: it is on the tile's critical path (c5 K1 0.559 -> 0.534 ms)
    if (GNCA_S32_PREP_PRIO > 0) __builtin_amdgcn_s_setprio(GNCA_S32_PREP_PRIO);
    const int b = t / a.tps, tin = t - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const size_t cell0 = (size_t)i0 * W + j0;
    uint8_t* spp = reinterpret_cast<uint8_t*>(smem_b + L.sp + s * L.sp_slot);
    uint8_t* lstp = reinterpret_cast<uint8_t*>(smem_b + L.lst + s * L.lst_slot);
    uint8_t* abq = reinterpret_cast<uint8_t*>(smem_b + L.ab);
    uint64_t* cb = reinterpret_cast<uint64_t*>(smem_b + L.cb);
    if (part & 1) {
      const uint8_t* alb = a.alive + (size_t)b * HW;
      constexpr int NU = (RHW + 63) / 64;
      constexpr int NB = NU;
#pragma unroll 1
      for (int u0 = 0; u0 < NU; u0 += NB) {
        uint32_t v[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int e = 64 * (u0 + u) + lane;
          v[u] = 0u;
          if (u0 + u < NU && e < RHW) {
            const int vr = e / RW, vc = e - (e / RW) * RW;
            int ii = i0 - RY + vr, jj = j0 - RX + vc;
            ii = ii < 0 ? ii + H : (ii >= H ? ii - H : ii);
            jj = jj < 0 ? jj + W : (jj >= W ? jj - W : jj);
            v[u] = alb[ii * W + jj];
          }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int e = 64 * (u0 + u) + lane;
          if (u0 + u < NU && e < RHW) {
            abq[e] = (uint8_t)v[u];
            if constexpr (GRAPH) spp[e] = a2a ? (uint8_t)((v[u] >> 1) & 1u) : (uint8_t)1;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!(part & 2)) {
      if (GNCA_S32_PREP_PRIO > 0) __builtin_amdgcn_s_setprio(0);
      return;
    }
    // the tile cells' alive bytes: from the region plane this wave just built, or (list half alone)
    // straight from global memory, every chunk's load in flight together
    constexpr int NCH = (NCELL + 63) / 64;
    uint32_t cab[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int n = 64 * ch + lane;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      cab[ch] = 0u;
      if (n < NCELL)
        cab[ch] = (part & 1) ? abq[(ti + RY) * RW + tj + RX]
                             : a.alive[(size_t)b * HW + (size_t)(i0 + ti) * W + (j0 + tj)];
    }
    float* outb = a.out + (size_t)b * C * HW + cell0;
    int nl = 0;
#pragma unroll
    for (int n0 = 0; n0 < NCELL; n0 += 64) {
      const int n = n0 + lane;
      const bool inb = n < NCELL;
      const int ti = n / TW, tj = n - (n / TW) * TW;
      const size_t cell = (size_t)(i0 + ti) * W + (j0 + tj);
      bool live = false;
      if (inb && (cab[n0 >> 6] & 1u))
        live = fire_at(a.fire_mode, a.fire, a.fire_rate, a.seed, a.rng_step, a.sample_base, b, HW, cell);
      const uint64_t bal = __ballot(live);
      const int pre = __popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) cb[n0 >> 6] = bal;
      if (compact && inb && tj == 0) a.rpre[(size_t)t * TH + ti] = (uint32_t)(nl + pre);
      if (live) {
        lstp[nl + pre] = (uint8_t)n;
      } else if (inb && !compact) {   // (compact: K2 masks the alpha plane by the row tables)
        float* oz = outb + (size_t)ti * W + tj;
#pragma unroll
        for (int c = 0; c < C; ++c) oz[(size_t)c * HW] = 0.f;
      }
      nl += __popcll(bal);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
    if (GNCA_S32_PREP_PRIO > 0) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: the first tile's phase-0 DMA and planes, then the weight images
  int tile = next_active(t_begin + xr_);
  if (tile < t_end) stage(tile, 0, wave, NW);
  if (wave == PW && tile < t_end) prep(tile, 0, 3);
  if (tid == 0) *xsd = 0;

  // ---- weight images (bf16 parts in MFMA fragment order), once per persistent workgroup ----
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ok = 1;
  for (int idx = tid; idx < C * 27; idx += NT) {
    const int e = idx % 27, f = e / 9, tap = e % 9, tr = tap / 3, tc = tap % 3;
    float ref;
    if (f == 0) ref = (tap == 4) ? 1.f : 0.f;
    else if (f == 1) ref = (float)((tc == 0 ? 1 : (tc == 2 ? -1 : 0)) * (tr == 1 ? 2 : 1));
    else ref = (float)((tr == 0 ? 1 : (tr == 2 ? -1 : 0)) * (tc == 1 ? 2 : 1));
    if (a.perc[idx] != ref) ok = 0;
  }
  const bool sobel = __syncthreads_and(ok) != 0;   // also the barrier after the images, DMA and prep

  const u32x4 ones = h == 0 ? u32x4{0x3f803f80u, 0x3f80u, 0u, 0u} : u32x4{0u, 0u, 0u, 0u};
  const float mgain = GRAPH ? a.message_gain : 0.f;
  const bool hz = hidden_only && h == 0;   // channels (r&3) + 4h < 4 (r < 4) are the RGBA ones

  PROF_DECL
  int par = 0;
  while (tile < t_end) {
    PROF_MARK(7);   // loop top
    const int nxt = next_active(tile + per_x);
    const int b = tile / a.tps, tin = tile - b * a.tps;
    const int ty = tin / a.tiles_x, tx = tin - ty * a.tiles_x;
    const int i0 = ty * TH, j0 = tx * TW;
    const size_t cell0 = (size_t)i0 * W + j0;
    float* outb = a.out + (size_t)b * C * HW + cell0;
    const uint8_t* sp = reinterpret_cast<const uint8_t*>(smem_b + L.sp + par * L.sp_slot);
    const uint8_t* lst = reinterpret_cast<const uint8_t*>(smem_b + L.lst + par * L.lst_slot);
    const int nlive = cnt[par];
    // the next tile's slot: wave PW - 1 builds the sender plane beside the preparer's list when it
    // has no group itself (<= 192 live cells), else the preparer does both
    if (nxt < t_end) {
      const bool two = GNCA_S32_PREP_SPLIT && 32 * (PW - 1) >= nlive;
      if (wave == PW) prep(nxt, par ^ 1, two ? 2 : 3);
      else if (two && wave == PW - 1) prep(nxt, par ^ 1, 1);
    }
    PROF_MARK(0);   // preparer

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
        PROF_MARK(1);   // phase 0: gather + perception
        __syncthreads();   // every wave is done with phase 0's planes
        stage(tile, 1, wave, NW);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        PROF_MARK(2);   // phase-1 staging (barrier, DMA, wait, barrier)
      }
      if (!has) continue;
      // -- gather of alive-masked x, this phase's channels 16ph + 8h + j (uniform weight 1/k) --
      u32x4 g0 = {0u, 0u, 0u, 0u}, g1 = g0, g2 = g0;
      if constexpr (GRAPH) if (!(GNCA_ABLATE & kAblGather)) {
        float gv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = 0.f;
        const float* xq = xs + hb + pidx;
        const uint8_t* spq = sp + pidx;
        float Sp = 0.f;
        if (GNCA_K1_PIPE_LDS) {
          ks_gather8<KU, PSTR>(a.odl, xq, spq, gv, Sp);
        } else {
#pragma unroll
          for (int o = 0; o < KU; ++o) {
            const int d = a.odl[o];
            const float s_ = (float)spq[-d];
            Sp += s_;
            const float* xo = xq - d;
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] = fmaf(s_, xo[j * PSTR], gv[j]);
            if ((o & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // <= 4 offsets' reads in flight
          }
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
      } else if (sobel && GNCA_K1_PIPE_LDS) {
        const int tt[9] = {t0, t1, t2, t3, bc, t5, t6, t7, t8};
        ks_sobel8<PSTR>(xs, tt, y0, y1, y2);
      } else if (sobel) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int co = j * PSTR;
          const float n0 = xs[t0 + co], n1 = xs[t1 + co], n2 = xs[t2 + co];
          const float n3 = xs[t3 + co], n4 = xs[bc + co], n5 = xs[t5 + co];
          const float n6 = xs[t6 + co], n7 = xs[t7 + co], n8 = xs[t8 + co];
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

    // the next tile's phase-0 planes, staged by the preparer as soon as every group is past its
    // phase-1 reads (release / acquire on the LDS counter), under the groups' MFMAs
    PROF_MARK(3);   // phase 1: gather + perception
    const int ngrp = (nlive + 31) >> 5;
    if (has) __hip_atomic_fetch_add(xsd, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    // stagers: every wave without a group (waves ngrp..7, the preparer among them), or the preparer
    // alone when all 8 waves have one; the 208 LDS-DMA instructions of a phase issued by one wave
    // take longer than the groups' MFMAs (~60-100 cycles each beside MFMAs)
#if GNCA_S32_STAGERS
    const int nst = ngrp < NW ? NW - ngrp : 1;
    const bool stager = ngrp < NW ? wave >= ngrp : wave == PW;
#else
    const int nst = 1;
    const bool stager = wave == PW;
#endif
    if (stager && nxt < t_end) {
      while ((__hip_atomic_load(xsd, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >> 6) - xbase < ngrp)
        __builtin_amdgcn_s_sleep(1);
      stage(nxt, 0, nst > 1 ? wave - ngrp : 0, nst);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    xbase += ngrp;
    PROF_MARK(4);   // next tile's phase-0 staging (stagers)

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
#if GNCA_K1_LEAN
      // the message term tanh(M + bm S) * gain seeds GEMM2's accumulator (accm dies here)
      if constexpr (GRAPH) {
        const float* bmp = reinterpret_cast<const float*>(smem_b + L.bml) + 16 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) accD[r] = fast_tanh(fmaf(bmp[r], S, accm[r])) * ((hz && r < 4) ? 0.f : mgain);
      }
      __builtin_amdgcn_sched_barrier(0);
#endif
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
#if !GNCA_K1_LEAN
          if constexpr (GRAPH) v = fmaf(fast_tanh(fmaf(bmp[r], S, accm[r])), (hz && r < 4) ? 0.f : mgain, v);
#endif
          if (compact && h == 0 && r == 3) a.dxa[(size_t)b * HW + cell0 + (size_t)(ti * W + tj)] = v;   // alpha: dense
          else ob[(size_t)((r & 3) + 8 * (r >> 2)) * cstr] = v;
          s1 += v;
          s2 = fmaf(v, v, s2);
        }
      }
    }

    PROF_MARK(5);   // MFMAs + epilogue
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
    __syncthreads();   // groups done; the next tile's phase 0 staged; slot par^1 ready
    PROF_MARK(6);   // partials + tile barrier
    tile = nxt;
    par ^= 1;
  }
  PROF_STORE_W07;
  GNCA_STAMP_END(a.stamps);
}

}  // namespace gnca
