// Pipelined implicit-GEMM convolution (bf16 in, f32 accumulate, bf16 out) for
// gfx950: conv forward and conv data-gradient of the encoder
// (models.py:198-221 Bottleneck convs, models.py:310-316 stem).
//
// Structure (cdna_hip_programming.md §5, "glds" rows):
//  * the output tile is computed transposed, out^T[channel][pixel], so that an
//    MFMA accumulator lane holds 4 consecutive channels of one pixel; with the
//    channel order inside the tile permuted (below) a lane holds 8 consecutive
//    channels across two 16-row MFMA tiles and the epilogue stores 16-B bf16
//    vectors straight from registers (no LDS staging, BN statistics from the
//    f32 accumulators);
//  * both operands are staged by LDS-DMA (buffer_load ... lds, 16 B per lane):
//    one wave instruction fills 8 rows x 128 B (8 lanes per row = one full
//    128-B line of k), the LDS image of a row is its 8 k-chunks in slot order
//    chunk ^ (row & 7) (the XOR swizzle is applied to the per-lane SOURCE
//    address; the LDS destination stays lane-linear), which makes the MFMA
//    fragment reads (16 rows x one chunk per ds_read_b128) conflict-free;
//  * an NSTAGE ring of LDS stages, one raw s_barrier per K-step, counted
//    s_waitcnt vmcnt so that NSTAGE-2 stages stay in flight across the barrier;
//  * implicit im2col: per pixel row a tap-validity mask; out-of-range (padding,
//    tails) source offsets are 0x80000000, which the buffer unit turns into
//    zeros written to LDS.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "common.h"
#include "pgemm.h"
#include "../../include/artsbir.h"

#include "pgemm_dev.h"

namespace artsbir {


// BK (0 / 1 / 2 / 3, see pg_epilogue_k) and TWO select the fused epilogue.
// PF: epilogue operands prefetched into registers before the main loop
// (epi_prefetch) instead of staged through LDS after it
// KS: k per stage.  64: LDS rows of 128 B (8 chunks, slot = chunk ^ (row & 7),
// 8 rows per DMA instruction).  32: rows of 64 B (4 chunks, slot = chunk ^
// ((row >> 2) & 2), 16 rows per DMA instruction; conflict-free for the
// ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... of
// MI355X_MICROARCH §LDS — the earlier chunk ^ ((row >> 2) & 3) put rows r and
// r+4 of one group on the same banks, 2-way) — half the bytes per stage, so
// the same LDS holds twice the stages and more of them are in flight (C % 64
// == 0 only)
// GLB (fused BN-backward only): the epilogue reads y, residual, mask and BN
// constants straight from global memory (no LDS staging, no parameter table),
// so the LDS is the stage ring alone and several workgroups share a CU: one's
// epilogue streams while another's main loop runs
// X2 (1x1 only): the BatchNorm-backward fold of artsbir_conv1x1_dgrad_fold — the
// reduction runs over two operands (k < C1 from x, the rest from x2), the
// weights and the bias are those of the tile's BN segment
template <int BPX, int BCH, int WPX, int WCH, int NSTAGE, bool MULTI, int BK, bool TWO, bool PF = false, int KS = 64,
          bool GLB = false, bool X2 = false>
__global__ void __launch_bounds__(64 * WPX * WCH, GLB ? (WPX * WCH == 8 ? 4 : 3) : 1) pgemm_kernel(PgArgs a) {
  constexpr bool BNB = BK != 0;
  static_assert(!GLB || !PF, "GLB: operands from global memory, not prefetched into registers");
  static_assert(!PF || BK != 2, "PF: the bf16 mask operand of kind 2 is not prefetched");
  static_assert(KS == 64 || (KS == 32 && !MULTI), "32-k stages: uniform taps only");
  constexpr int ROWB = 2 * KS, RPI = 1024 / ROWB, CPR = ROWB / 16;
  constexpr int NW = WPX * WCH;
  constexpr int PXB = BPX * ROWB, CHB = BCH * ROWB, STAGE = PXB + CHB;
  constexpr int IPX = BPX / (RPI * NW);
  constexpr int ICH_TOT = BCH / RPI;
  constexpr int ICH = (ICH_TOT + NW - 1) / NW;
  constexpr int WTPX = BPX / WPX, WTCH = BCH / WCH;
  constexpr int NTP = WTPX / 16, MTC = WTCH / 16;
  constexpr int LPS_HI = IPX + ICH;                            // loads per stage, waves with ICH weight loads
  constexpr int LPS_LO = IPX + ICH_TOT / NW;                   // ... waves with one fewer
  static_assert(IPX >= 1 && IPX * RPI * NW == BPX, "pixel loader");
  static_assert(MTC % 2 == 0 && WTCH % 32 == 0, "channel pairs");
  // stage ring | BN statistics accumulator | (BNB) BN constants | (BNB) mask bits
  constexpr int XTRA = (BNB && !GLB) ? pg_prm_bytes<BCH>() + BPX * (BCH / 8) : 0;
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE + pg_red_bytes<BCH>() + XTRA];
  float* red = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  int* red_cnt = reinterpret_cast<int*>(smem + NSTAGE * STAGE + 6 * BCH * 4);
  float* prm = reinterpret_cast<float*>(smem + NSTAGE * STAGE + pg_red_bytes<BCH>());
  unsigned char* sbits = reinterpret_cast<unsigned char*>(smem + NSTAGE * STAGE + pg_red_bytes<BCH>() +
                                                          pg_prm_bytes<BCH>());

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wpx = wid % WPX, wch = wid / WPX;
  const int ntc = (a.Cout + BCH - 1) / BCH;
  const long long ntp = (a.M + BPX - 1) / BPX;
  const long long lid = pg_xcd_remap(blockIdx.x, ntp * ntc);
  const long long bpx = (lid / ntc) * BPX;
  const int bch = (int)(lid % ntc) * BCH;
  const long long seg0 = a.seg_m > 0 ? bpx / a.seg_m : 0;
  if constexpr (BNB && !GLB) pg_prm_fill<BCH, 64 * NW>(a, prm, bpx, bch, seg0);  // published by the main loop's barriers
  const int HoWo = a.Ho * a.Wo;
  const long long img0 = bpx / HoWo;
  const __amdgpu_buffer_rsrc_t xr =
      pg_rsrc(reinterpret_cast<const bf16*>(a.x) + img0 * a.sN, (a.x_elems - img0 * a.sN) * 2);
  const __amdgpu_buffer_rsrc_t xr2 =
      X2 ? pg_rsrc(reinterpret_cast<const bf16*>(a.x2) + img0 * a.sN2, (a.x2_elems - img0 * a.sN2) * 2) : xr;
  const __amdgpu_buffer_rsrc_t wr =
      pg_rsrc(reinterpret_cast<const bf16*>(a.w) + (X2 ? seg0 * a.w_sstride : 0), (long long)a.Cout * a.K * 2);

  // ---- loader decode: this lane fills slot (lane & 7) of row (lane >> 3)
  // of each 8-row wave instruction, with k-chunk csrc = slot ^ (row & 7)
  const int lrow = lane / CPR, lslot = lane % CPR;
  const int csrc = KS == 64 ? (lslot ^ lrow) : (lslot ^ ((lrow >> 2) & 2));
  int rowoff[IPX];
  unsigned rmask[IPX];
  // X2: the row offsets into the second operand replace rowoff[] once, at the
  // first stage past C1 (1x1, stride 1: the pixel itself) — not held beside
  // them through the first operand's stages (the 8-wave tile's 128 VGPRs)
  auto rowoff_x2 = [&](int u) {
    const int row = (u * NW + wid) * RPI + lrow;
    const long long gm = bpx + row;
    const long long gmc = gm < a.M ? gm : bpx;
    const long long img = gmc / HoWo;
    const int rem = (int)(gmc - img * HoWo);
    const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    return (int)(((img - img0) * a.sN2 + (long long)oh * a.sH2 + (long long)ow * a.sW2) * 2);
  };
#pragma unroll
  for (int u = 0; u < IPX; ++u) {
    const int row = (u * NW + wid) * RPI + lrow;
    const long long gm = bpx + row;
    const bool valid = gm < a.M;
    const long long gmc = valid ? gm : bpx;
    const long long img = gmc / HoWo;
    const int rem = (int)(gmc - img * HoWo);
    const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    rowoff[u] = (int)(((img - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * 2);
    unsigned msk = 0;
    for (int r = 0; r < a.R; ++r)
      for (int s = 0; s < a.S; ++s) {
        const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
        msk |= (ok ? 1u : 0u) << (r * a.S + s);
      }
    rmask[u] = msk;
  }
  unsigned woff[ICH];
#pragma unroll
  for (int u = 0; u < ICH; ++u) {
    const int g = u * NW + wid;
    const int ch = bch + pg_perm(g * RPI + lrow);
    woff[u] = (g < ICH_TOT && ch < a.Cout) ? (unsigned)(ch * a.K * 2 + csrc * 16) : PG_OOB;
  }
  const bool lps_hi = (ICH - 1) * NW + wid < ICH_TOT;

  int u_ci = 0, u_s = 0, u_r = 0;  // uniform-tap walk (C % 64 == 0)
  bool on2 = false;                 // X2: rowoff[] holds the second operand's offsets
  auto issue = [&](int kt, int buf) {
    char* pxs = smem + buf * STAGE;
    char* chs = pxs + PXB;
    int rs, tapoff;
    bool kval;
    bool src2 = false;  // X2: this stage's k lie in the second operand
    if constexpr (!MULTI) {
      rs = u_r * a.S + u_s;
      int ci = u_ci;
      if constexpr (X2) {
        src2 = u_ci >= a.C1;
        if (src2) {
          ci -= a.C1;
          if (!on2) {
            on2 = true;
#pragma unroll
            for (int u = 0; u < IPX; ++u) rowoff[u] = rowoff_x2(u);
          }
        }
      }
      tapoff = (u_r * (int)a.sH + u_s * (int)a.sW + ci + csrc * 8) * 2;
      kval = true;
      u_ci += KS;
      if (u_ci == a.C) {
        u_ci = 0;
        if (++u_s == a.S) { u_s = 0; ++u_r; }
      }
    } else {
      const int cpt = a.C >> 3;  // 16-B chunks per tap: 1, 2 or 4
      const int sub = csrc / cpt;
      const int ci = (csrc - sub * cpt) * 8;
      rs = kt * (64 / a.C) + sub;
      kval = rs < a.R * a.S;
      const int r = rs / a.S, s = rs - (rs / a.S) * a.S;
      tapoff = (r * (int)a.sH + s * (int)a.sW + ci) * 2;
    }
#pragma unroll
    for (int u = 0; u < IPX; ++u) {
      const bool ok = kval && ((rmask[u] >> (rs & 31)) & 1u);
      if constexpr (X2) {
        glds16(src2 ? xr2 : xr, pxs + (u * NW + wid) * 1024, ok ? (unsigned)(rowoff[u] + tapoff) : PG_OOB);
      } else {
        glds16(xr, pxs + (u * NW + wid) * 1024, ok ? (unsigned)(rowoff[u] + tapoff) : PG_OOB);
      }
    }
    const bool wk = kt * KS + csrc * 8 < a.K;
#pragma unroll
    for (int u = 0; u < ICH; ++u) {
      if (u * NW + wid < ICH_TOT)
        glds16(wr, chs + (u * NW + wid) * 1024, (wk && woff[u] != PG_OOB) ? woff[u] + kt * ROWB : PG_OOB);
    }
  };

  f32x4 acc[MTC][NTP];
#pragma unroll
  for (int i = 0; i < MTC; ++i)
#pragma unroll
    for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
    const char* pxs = smem + buf * STAGE;
    const char* chs = pxs + PXB;
#pragma unroll
    for (int kk = 0; kk < KS / 32; ++kk) {
      const int so = (KS == 64 ? ((kk * 4 + fq) ^ (fr & 7)) : (fq ^ ((fr >> 2) & 2))) << 4;
      uint4 af[MTC], bv[NTP];
#pragma unroll
      for (int i = 0; i < MTC; ++i) af[i] = *reinterpret_cast<const uint4*>(chs + (wch * WTCH + i * 16 + fr) * ROWB + so);
#pragma unroll
      for (int j = 0; j < NTP; ++j) bv[j] = *reinterpret_cast<const uint4*>(pxs + (wpx * WTPX + j * 16 + fr) * ROWB + so);
      PG_PRIO_ON();
#pragma unroll
      for (int i = 0; i < MTC; ++i)
#pragma unroll
        for (int j = 0; j < NTP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                              *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j], 0,
                                                              0, 0);
      PG_PRIO_OFF();
    }
  };

  const bool sums = BNB || a.stats != nullptr;
  if (sums) {
    for (int i = tid; i < 6 * BCH; i += 64 * NW) red[i] = 0.f;
    if (tid == 0) *red_cnt = 0;
  }
  EpiRegs<MTC / 2, NTP> er;
  if constexpr (PF) epi_prefetch<BK, TWO, MTC, NTP, WTPX, WTCH>(a, er, bpx, bch, wpx, wch, fr, fq);
  const int nk = (a.K + KS - 1) / KS;
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    int ahead = nk - 1 - kt;
    if (ahead > NSTAGE - 2) ahead = NSTAGE - 2;
    if (lps_hi) wait_stages<LPS_HI, NSTAGE>(ahead);
    else wait_stages<LPS_LO, NSTAGE>(ahead);
    // retire this wave's LDS reads of the slot the next issue overwrites
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    compute(kt % NSTAGE);
  }

  // ---- epilogue operands into the (now free) stage ring by LDS-DMA: slot 0
  // y_0, then the residual, y_1 and the bf16 mask as far as the ring holds them
  constexpr int OPB = BPX * BCH * 2;            // bytes of one staged operand
  constexpr int NOP = (NSTAGE * STAGE) / OPB;   // operands that fit
  constexpr bool RESK = BK == 2 || BK == 3;
  constexpr bool S_RES = RESK && NOP >= 2;
  constexpr bool S_Y1 = TWO && NOP >= 2 + (S_RES ? 1 : 0);
  constexpr bool S_MK = BK == 2 && NOP >= 2 + (S_RES ? 1 : 0) + (S_Y1 ? 1 : 0);
  static_assert(!BNB || NOP >= 1, "y_0 must fit the stage ring");
  EpiStage sg{nullptr, nullptr, nullptr, nullptr, nullptr, BNB ? prm : nullptr, seg0};
  if constexpr (PF) {
    const int slot = (int)(blockIdx.x % ARTSBIR_NSLOT);
    pg_epilogue_k<BK, TWO, false, false, false, BCH, MTC, NTP, WTPX, WTCH, true>(a, acc, bpx, bch, wpx, wch, fr, fq,
                                                                                red, sg, &er);
    if (sums) stats_flush<BCH>(red, red_cnt, NW - 1, a, bch, slot, lane, bpx, BPX);
    return;
  }
  if constexpr (GLB) {
    const int slot = (int)(blockIdx.x % ARTSBIR_NSLOT);
#ifndef PG_GLB_OLD
#define PG_GLB_OLD 0
#endif
    if constexpr (PG_GLB_OLD || NW >= 8) {  // channel pairs outside (the 8-wave tile: 128 VGPRs)
      EpiStage sgg{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, seg0};
      pg_epilogue_k<BK, TWO, false, false, false, BCH, MTC, NTP, WTPX, WTCH, false, 1, true, X2, NW >= 8>(
          a, acc, bpx, bch, wpx, wch, fr, fq, red, sgg);
    } else {
      // the 8-wave 256 x 128 tile runs at 128 VGPRs (two workgroups per CU):
      // statistics reduced per (tile, pair) there, carried in registers otherwise
      // statistics carried in registers across the pixel tiles; the BN constants
      // from an LDS table where the registers allow (4 waves: 168 VGPRs), else
      // from the L1-resident parameter vectors (8 waves: 128 VGPRs)
      constexpr bool SP = true, TBL = NW < 8;
      float* tprm = reinterpret_cast<float*>(smem);  // the stage ring is free after the main loop
      if constexpr (BNB && TBL) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();  // every wave is done reading the stages
        pg_prm_fill<BCH, 64 * NW>(a, tprm, bpx, bch, seg0);
        __syncthreads();
      }
      pg_epilogue_glb<BK, TWO, BCH, MTC, NTP, WTPX, WTCH, X2, SP, TBL>(a, acc, bpx, bch, wpx, wch, fr, fq, red,
                                                                       tprm, seg0);
    }
    if (sums) stats_flush<BCH>(red, red_cnt, NW - 1, a, bch, slot, lane, bpx, BPX);
    return;
  }
  if constexpr (BNB) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done reading the stages
    const long long rows = a.M;
    int n = 0;
    sg.y0 = smem;
    stage_operand<BPX, BCH, NW>(a.bnb_y[0], rows, a.ldy, smem, bpx, bch, a, false, wid, lane);
    ++n;
    if constexpr (S_RES) {
      sg.res = smem + n * OPB;
      stage_operand<BPX, BCH, NW>(a.res, a.res_mode == 2 ? rows / 4 : rows, a.ldy, smem + n * OPB, bpx, bch, a,
                                  a.res_mode == 2, wid, lane);
      ++n;
    }
    if constexpr (S_Y1) {
      sg.y1 = smem + n * OPB;
      stage_operand<BPX, BCH, NW>(a.bnb_y[1], rows, a.ldy, smem + n * OPB, bpx, bch, a, false, wid, lane);
      ++n;
    }
    if constexpr (S_MK) {
      sg.mk = smem + n * OPB;
      stage_operand<BPX, BCH, NW>(a.bnb_mask, rows, a.ldy, smem + n * OPB, bpx, bch, a, false, wid, lane);
      ++n;
    }
    if constexpr (BK == 3) {
      sg.bits = sbits;
      stage_bits<BPX, BCH, NW>(a.bnb_mask, sbits, bpx, bch, a, wid, lane);
    }
    vm_wait<0>();
    __syncthreads();  // every wave's DMA has landed
  } else if (a.res_mode) {  // plain data gradient with a residual: stage it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    sg.res = smem;
    stage_operand<BPX, BCH, NW>(a.res, a.res_mode == 2 ? a.M / 4 : a.M, a.ldy, smem, bpx, bch, a, a.res_mode == 2,
                                wid, lane);
    vm_wait<0>();
    __syncthreads();
  }
  const int slot = (int)(blockIdx.x % ARTSBIR_NSLOT);
  pg_epilogue_k<BK, TWO, S_RES, S_Y1, S_MK, BCH, MTC, NTP, WTPX, WTCH, false, 2, false, X2>(a, acc, bpx, bch, wpx, wch,
                                                                                            fr, fq, red, sg);
  if (sums) stats_flush<BCH>(red, red_cnt, NW - 1, a, bch, slot, lane, bpx, BPX);
}

#ifndef PG_NOL
#define PG_NOL 0  // 1: normalize-on-load cost probe of a diagnostic build only (pstream_kernel)
#endif
// Cost probe (round 5, tools/gpu/r5_nol.sh) for a consumer-side BatchNorm + ReLU
// on pstream_kernel's pixel fragments: relu(s * x + b) per input channel in f32,
// repacked to bf16, with coefficients read from LDS per 32-k step.  Wrong
// results by design (the coefficients are scratch); only the time matters.
__device__ __forceinline__ unsigned pg_nol2(unsigned w, float s0, float s1, float b0, float b1) {
  const float lo = fmaxf(fmaf(__uint_as_float(w << 16), s0, b0), 0.f);
  const float hi = fmaxf(fmaf(__uint_as_float(w & 0xffff0000u), s1, b1), 0.f);
  return (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
}

// ---------------------------------------------------------------------------
// Persistent producer/consumer variant for layers with many 256-pixel tiles
// (stem, layer1-3, low K).  4 loader waves only issue LDS-DMA, so their vmcnt
// counts exactly their own loads; 8 compute waves only read LDS, run MFMAs and
// store.  One s_barrier per stage hands a landed stage to the compute waves
// and the slot they just drained back to the loaders.  The stage sequence runs
// across tile boundaries: the next tile's loads are in flight while this
// tile's epilogue stores drain, which is what the low-K layers (1-5 K-steps
// per tile) need to stream at HBM rate.
// ---------------------------------------------------------------------------
// FWDS: forward with BN statistics (carried across tiles, pg_epilogue_fwd)
// BK > 0: the fused BN-backward epilogue specialised at compile time
// (pg_epilogue_k, kinds as pgemm_kernel's, TWO targets), its operands and BN
// constants read from global memory in batches of two pixel tiles while the
// loader waves already stream the next tile's stages
// KS: k per stage as in pgemm_kernel (32: 64-B LDS rows, twice the stages in
// the same LDS, uniform taps only)
// X2: the two-operand / per-segment-weight fold of pgemm_kernel (1x1 only)
// WGK > 0: the fold (X2) with its weight-gradient operands accumulated by the
// loader waves (pstream_wg_loader, K = WGK, 64 output channels)

template <int BCH, int WPX, int WCH, int NSTAGE, bool MULTI, bool BNB, bool FWDS, int BK = 0, bool TWO = false,
          int KS = 64, bool X2 = false, int WGK = 0>
__global__ void __launch_bounds__(768) pstream_kernel(PgArgs a, int ntiles) {
  constexpr int BPX = 256, NWC = 8, NWL = 4;
  static_assert(WPX * WCH == NWC, "compute waves");
  static_assert(KS == 64 || (KS == 32 && !MULTI), "32-k stages: uniform taps only");
  constexpr int ROWB = 2 * KS, RPI = 1024 / ROWB, CPR = ROWB / 16;
  constexpr int PXB = BPX * ROWB, CHB = BCH * ROWB, STAGE = PXB + CHB;
  constexpr int LPX = BPX / (RPI * NWL);
  constexpr int LCH = BCH / (RPI * NWL);
  constexpr int LPS = LPX + LCH;
  constexpr int WTPX = BPX / WPX, WTCH = BCH / WCH;
  constexpr int NTP = WTPX / 16, MTC = WTCH / 16;
  static_assert(LCH >= 1 && MTC % 2 == 0, "shape");
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE + pg_red_bytes<BCH>()];
  float* red = reinterpret_cast<float*>(smem + NSTAGE * STAGE);
  int* red_cnt = reinterpret_cast<int*>(smem + NSTAGE * STAGE + 6 * BCH * 4);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntc = (a.Cout + BCH - 1) / BCH;
  const int G = gridDim.x;
  const int bslot = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int my_tiles = bslot < ntiles ? (ntiles - 1 - bslot) / G + 1 : 0;
  const int nk = (a.K + KS - 1) / KS;
  const int total = my_tiles * nk;
  const int HoWo = a.Ho * a.Wo;

  if (wid >= NWC) {
    // ------------------------------------------------------------ loaders
    if constexpr (WGK > 0) {
      static_assert(X2 && !MULTI && KS == 64 && !FWDS, "WGK: the fold's 64-k stages");
      pstream_wg_loader<BCH, NSTAGE, LPX, LCH, STAGE, PXB, WGK>(a, smem, wid - NWC, lane, G, bslot, nk, total);
      return;
    }
    const int lw = wid - NWC;
    const int lrow = lane / CPR, lslot = lane % CPR;
    const int csrc = KS == 64 ? (lslot ^ lrow) : (lslot ^ ((lrow >> 2) & 2));
    __amdgpu_buffer_rsrc_t wr = pg_rsrc(a.w, (long long)a.Cout * a.K * 2);
    __amdgpu_buffer_rsrc_t xr = wr, xr2 = wr;
    int rowoff[LPX], rowoff2[X2 ? LPX : 1];
    unsigned rmask[LPX];
    unsigned woff[LCH];
    int u_ci = 0, u_s = 0, u_r = 0;
    auto start_tile = [&](int i) {
      const long long t = (long long)i * G + bslot;
      const long long bpx = (t / ntc) * BPX;
      const int bch = (int)(t % ntc) * BCH;
      const long long img0 = bpx / HoWo;
      xr = pg_rsrc(reinterpret_cast<const bf16*>(a.x) + img0 * a.sN, (a.x_elems - img0 * a.sN) * 2);
      if constexpr (X2) {
        xr2 = pg_rsrc(reinterpret_cast<const bf16*>(a.x2) + img0 * a.sN2, (a.x2_elems - img0 * a.sN2) * 2);
        const long long sg = a.seg_m > 0 ? bpx / a.seg_m : 0;
        wr = pg_rsrc(reinterpret_cast<const bf16*>(a.w) + sg * a.w_sstride, (long long)a.Cout * a.K * 2);
      }
#pragma unroll
      for (int u = 0; u < LPX; ++u) {
        const int row = (u * NWL + lw) * RPI + lrow;
        const long long gm = bpx + row;
        const bool valid = gm < a.M;
        const long long gmc = valid ? gm : bpx;
        const long long img = gmc / HoWo;
        const int rem = (int)(gmc - img * HoWo);
        const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
        const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
        rowoff[u] = (int)(((img - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * 2);
        if constexpr (X2)
          rowoff2[u] = (int)(((img - img0) * a.sN2 + (long long)oh * a.sH2 + (long long)ow * a.sW2) * 2);
        unsigned msk = 0;
        for (int r = 0; r < a.R; ++r)
          for (int s = 0; s < a.S; ++s) {
            const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
            msk |= (ok ? 1u : 0u) << (r * a.S + s);
          }
        rmask[u] = msk;
      }
#pragma unroll
      for (int u = 0; u < LCH; ++u) {
        const int ch = bch + pg_perm((u * NWL + lw) * RPI + lrow);
        woff[u] = ch < a.Cout ? (unsigned)(ch * a.K * 2 + csrc * 16) : PG_OOB;
      }
      u_ci = 0; u_s = 0; u_r = 0;
    };
    auto issue = [&](int sidx) {
      const int i = sidx / nk, kt = sidx - i * nk;
      if (kt == 0) start_tile(i);
      char* pxs = smem + (sidx % NSTAGE) * STAGE;
      char* chs = pxs + PXB;
      int rs, tapoff;
      bool kval;
      bool src2 = false;
      if constexpr (!MULTI) {
        rs = u_r * a.S + u_s;
        int ci = u_ci;
        if constexpr (X2) {
          src2 = u_ci >= a.C1;
          if (src2) ci -= a.C1;
        }
        tapoff = (u_r * (int)a.sH + u_s * (int)a.sW + ci + csrc * 8) * 2;
        kval = true;
        u_ci += KS;
        if (u_ci == a.C) {
          u_ci = 0;
          if (++u_s == a.S) { u_s = 0; ++u_r; }
        }
      } else {
        const int cpt = a.C >> 3;
        const int sub = csrc / cpt;
        const int ci = (csrc - sub * cpt) * 8;
        rs = kt * (64 / a.C) + sub;
        kval = rs < a.R * a.S;
        const int r = rs / a.S, s = rs - (rs / a.S) * a.S;
        tapoff = (r * (int)a.sH + s * (int)a.sW + ci) * 2;
      }
#pragma unroll
      for (int u = 0; u < LPX; ++u) {
        const bool ok = kval && ((rmask[u] >> (rs & 31)) & 1u);
        if constexpr (X2) {
          if (src2) glds16(xr2, pxs + (u * NWL + lw) * 1024, ok ? (unsigned)(rowoff2[u] + tapoff) : PG_OOB);
          else glds16(xr, pxs + (u * NWL + lw) * 1024, ok ? (unsigned)(rowoff[u] + tapoff) : PG_OOB);
        } else {
          glds16(xr, pxs + (u * NWL + lw) * 1024, ok ? (unsigned)(rowoff[u] + tapoff) : PG_OOB);
        }
      }
      const bool wk = kt * KS + csrc * 8 < a.K;
#pragma unroll
      for (int u = 0; u < LCH; ++u)
        glds16(wr, chs + (u * NWL + lw) * 1024, (wk && woff[u] != PG_OOB) ? woff[u] + kt * ROWB : PG_OOB);
    };
    for (int s = 0; s < NSTAGE - 1; ++s)
      if (s < total) issue(s);
    if (total > 0) {
      int ahead = total - 1;
      if (ahead > NSTAGE - 2) ahead = NSTAGE - 2;
      wait_stages<LPS, NSTAGE>(ahead);
    }
    for (int s = 0; s < total; ++s) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s + NSTAGE - 1 < total) issue(s + NSTAGE - 1);
      if (s + 1 < total) {
        int ahead = total - 2 - s;
        if (ahead > NSTAGE - 2) ahead = NSTAGE - 2;
        wait_stages<LPS, NSTAGE>(ahead);
      }
    }
    return;
  }

  // -------------------------------------------------------------- compute
  const bool sums = !FWDS && (BNB || a.stats != nullptr);
  if (sums) {  // ordered before any use by the first stage barrier
    for (int i = tid; i < 6 * BCH; i += 64 * NWC) red[i] = 0.f;
    if (tid == 0) *red_cnt = 0;
  }
  const int wpx = wid % WPX, wch = wid / WPX;
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[MTC][NTP];
#pragma unroll
  for (int i = 0; i < MTC; ++i)
#pragma unroll
    for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  WaveStats<MTC / 2> ws;  // forward statistics carried across tiles (pg_epilogue_fwd)
  wstats_zero(ws);
  ws.seg = -1;
  ws.bch = -1;
  const int wslot = (int)((blockIdx.x * NWC + wid) % ARTSBIR_NSLOT);
  for (int s = 0; s < total; ++s) {
    // retire this wave's LDS reads of the slot the next issue overwrites
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    {
      const char* pxs = smem + (s % NSTAGE) * STAGE;
      const char* chs = pxs + PXB;
#pragma unroll
      for (int kk = 0; kk < KS / 32; ++kk) {
        const int so = (KS == 64 ? ((kk * 4 + fq) ^ (fr & 7)) : (fq ^ ((fr >> 2) & 2))) << 4;
        uint4 af[MTC], bv[NTP];
#pragma unroll
        for (int i = 0; i < MTC; ++i)
          af[i] = *reinterpret_cast<const uint4*>(chs + (wch * WTCH + i * 16 + fr) * ROWB + so);
#pragma unroll
        for (int j = 0; j < NTP; ++j)
          bv[j] = *reinterpret_cast<const uint4*>(pxs + (wpx * WTPX + j * 16 + fr) * ROWB + so);
#if PG_NOL
        {
          const char* cbase = reinterpret_cast<const char*>(red) + fq * 32;
          const f32x4 cs0 = *reinterpret_cast<const f32x4*>(cbase), cs1 = *reinterpret_cast<const f32x4*>(cbase + 16);
          const f32x4 cb0 = *reinterpret_cast<const f32x4*>(cbase + 128);
          const f32x4 cb1 = *reinterpret_cast<const f32x4*>(cbase + 144);
#pragma unroll
          for (int j = 0; j < NTP; ++j) {
            bv[j].x = pg_nol2(bv[j].x, cs0[0], cs0[1], cb0[0], cb0[1]);
            bv[j].y = pg_nol2(bv[j].y, cs0[2], cs0[3], cb0[2], cb0[3]);
            bv[j].z = pg_nol2(bv[j].z, cs1[0], cs1[1], cb1[0], cb1[1]);
            bv[j].w = pg_nol2(bv[j].w, cs1[2], cs1[3], cb1[2], cb1[3]);
          }
        }
#endif
        PG_PRIO_ON();
#pragma unroll
        for (int i = 0; i < MTC; ++i)
#pragma unroll
          for (int j = 0; j < NTP; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                                *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j],
                                                                0, 0, 0);
        PG_PRIO_OFF();
      }
    }
    const int ti = s / nk;
    if (s - ti * nk != nk - 1) continue;
    // ---- epilogue of tile ti
    const long long t = (long long)ti * G + bslot;
    const long long bpx = (t / ntc) * BPX;
    const int bch = (int)(t % ntc) * BCH;
    const int slot = (int)(t % ARTSBIR_NSLOT);
    if constexpr (FWDS) {
      pg_epilogue_fwd<BCH, MTC, NTP, WTPX, WTCH>(a, acc, bpx, bch, wpx, wch, fr, fq, ws, wslot);
    } else if constexpr (BK != 0) {
      const EpiStage sg{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, a.seg_m > 0 ? bpx / a.seg_m : 0};
      pg_epilogue_k<BK, TWO, false, false, false, BCH, MTC, NTP, WTPX, WTCH, false, 2, true, X2>(a, acc, bpx, bch, wpx,
                                                                                              wch, fr, fq, red, sg);
      if (sums) stats_flush<BCH>(red, red_cnt, NWC * (ti + 1) - 1, a, bch, slot, lane, bpx, BPX);
    } else {
      pg_epilogue<BNB, BCH, MTC, NTP, WTPX, WTCH, 1>(a, acc, bpx, bch, wpx, wch, fr, fq, red);
      // the flushing wave zeroes red before it reaches the next stage barrier,
      // and no wave adds for tile ti+1 before passing that barrier
      if (sums) stats_flush<BCH>(red, red_cnt, NWC * (ti + 1) - 1, a, bch, slot, lane, bpx, BPX);
    }
#pragma unroll
    for (int i = 0; i < MTC; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (FWDS) wstats_flush<MTC / 2, WTCH>(ws, a, wch, fr, fq, wslot);
}

// ---------------------------------------------------------------------------
// Direct 3x3 convolution for few channels (C in {8, 32, 64} in, Cout in
// {32, 64} out): the stem (models.py:310-317, 112x112) and the layer-1 3x3
// convolutions, forward and data gradient.  Their im2col rows are short
// (K = 72..576), so the LDS-staged im2col of pgemm spends its time gathering:
// here the pixel operand is read STRAIGHT from global memory into the MFMA B
// fragments — lane (fr, fq) of a 16-pixel tile loads 16 B (8 channels) of its
// own input pixel, so for C = 32 one wave instruction reads one contiguous
// 1 KB run of 16 pixels x 64 B (coalesced; the 9 tap re-reads hit L1/L2) —
// while the whole filter bank sits in LDS (read as A fragments, XOR-swizzled
// conflict-free).  Padding and tails come back as zeros from the buffer unit.
// Output tile = 256 consecutive pixels x all Cout channels, 4 waves x 64
// pixels; the epilogue (BN statistics, BN-backward fusion, segments) is
// pgemm's.
// ---------------------------------------------------------------------------
// LDS image of the filters: block kk (32 k = 4 chunks of 16 B) holds COUT rows
// of 64 B; row rho carries channel pg_perm(rho), chunk c at slot c ^ sw(rho).
__device__ __forceinline__ int sc_sw(int rho) { return (rho ^ (rho >> 1)) & 3; }

template <int C, int COUT, int STRIDE, bool BNB>
__global__ void __launch_bounds__(256) sconv_kernel(PgArgs a, int ntiles) {
  constexpr int K = 9 * C;
  constexpr int NKK = (K + 31) / 32;  // 32-k MFMA steps
  constexpr int CPT = C / 8;          // 16-B chunks per tap
  constexpr int MTC = COUT / 16, NTP = 4, WTPX = 64, BPX = 256, BCH = COUT;
  constexpr int PF = 2;                // k-steps of B fragments in flight ahead
  constexpr int WB = NKK * COUT * 64;  // filter image bytes
  __shared__ __attribute__((aligned(16))) char smem[WB + pg_red_bytes<BCH>()];
  float* red = reinterpret_cast<float*>(smem + WB);
  int* red_cnt = reinterpret_cast<int*>(smem + WB + 6 * BCH * 4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const bool sums = a.stats != nullptr || a.bnb != 0;
  if (sums) {
    for (int i = tid; i < 6 * BCH; i += 256) red[i] = 0.f;
    if (tid == 0) *red_cnt = 0;
  }
  // ---- filters -> LDS once per (persistent) block (zero past K)
  for (int i = tid; i < NKK * COUT * 4; i += 256) {
    const int kk = i / (COUT * 4), rem = i - kk * COUT * 4;
    const int rho = rem >> 2, c = rem & 3;
    const int k = kk * 32 + c * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k < K) v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.w) + (long long)pg_perm(rho) * K + k);
    *reinterpret_cast<uint4*>(smem + (kk * COUT + rho) * 64 + ((c ^ sc_sw(rho)) << 4)) = v;
  }
  const int HoWo = a.Ho * a.Wo;
  const int G = gridDim.x;
  int ti = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += G, ++ti) {
    // filter image visible (first tile); the previous tile's statistics flush
    // is complete before any wave adds this tile's sums
    __syncthreads();
    const long long bpx = (long long)tile * BPX;
    // ---- per pixel tile: input origin and tap validity of this lane's pixel
    const long long img0 = bpx / HoWo;
    const __amdgpu_buffer_rsrc_t xr =
        pg_rsrc(reinterpret_cast<const bf16*>(a.x) + img0 * a.sN, (a.x_elems - img0 * a.sN) * 2);
    const long long wpx0 = bpx + wid * WTPX;
    int boff[NTP];
    unsigned vmask[NTP];
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const long long px = wpx0 + j * 16 + fr;
      const bool valid = px < a.M;
      const long long pc = valid ? px : bpx;
      const long long n = pc / HoWo;
      const int rem = (int)(pc - n * HoWo);
      const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
      const int ih0 = oh * STRIDE - 1, iw0 = ow * STRIDE - 1;
      boff[j] = (int)(((n - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * 2);
      unsigned m = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r = t / 3, s = t % 3;
        const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
        m |= (ok ? 1u : 0u) << t;
      }
      vmask[j] = m;
    }
    // B fragment of k-step kk, pixel tile j: 16 B of the lane's own input pixel
    auto bload = [&](int kk, int j) -> uint4 {
      const int kc = kk * 4 + fq;  // 16-B chunk of the im2col row
      const int t = kc / CPT, cc = kc - (kc / CPT) * CPT;
      const int r = t / 3, s = t - (t / 3) * 3;
      const bool ok = kc < 9 * CPT && ((vmask[j] >> t) & 1u);
      const unsigned off = (unsigned)(boff[j] + ((r * (int)a.sH + s * (int)a.sW) * 2) + cc * 16);
      const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? (int)off : (int)PG_OOB, 0, 0);
      return make_uint4(v[0], v[1], v[2], v[3]);
    };
    f32x4 acc[MTC][NTP];
#pragma unroll
    for (int i = 0; i < MTC; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // ring of PF + 1 k-steps of B fragments (fully unrolled: static indices)
    uint4 bf[PF + 1][NTP];
#pragma unroll
    for (int q = 0; q < PF; ++q)
      if (q < NKK) {
#pragma unroll
        for (int j = 0; j < NTP; ++j) bf[q][j] = bload(q, j);
      }
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      if (kk + PF < NKK) {
#pragma unroll
        for (int j = 0; j < NTP; ++j) bf[(kk + PF) % (PF + 1)][j] = bload(kk + PF, j);
      }
      uint4 af[MTC];
#pragma unroll
      for (int i = 0; i < MTC; ++i) {
        const int rho = i * 16 + fr;
        af[i] = *reinterpret_cast<const uint4*>(smem + (kk * COUT + rho) * 64 + ((fq ^ sc_sw(rho)) << 4));
      }
#pragma unroll
      for (int i = 0; i < MTC; ++i)
#pragma unroll
        for (int j = 0; j < NTP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                              *reinterpret_cast<const bf16x8*>(&bf[kk % (PF + 1)][j]),
                                                              acc[i][j], 0, 0, 0);
    }
    const int slot = tile % ARTSBIR_NSLOT;
    pg_epilogue<BNB, BCH, MTC, NTP, WTPX, COUT, 1>(a, acc, bpx, 0, wid, 0, fr, fq, red);
    if (sums) stats_flush<BCH>(red, red_cnt, 4 * (ti + 1) - 1, a, 0, slot, lane, bpx, BPX);
  }
}

// shapes the direct small-channel kernel takes
static bool sconv_ok(const PgArgs& a) {
  if (a.R != 3 || a.S != 3 || a.pad != 1 || a.M <= 0) return false;
  if (a.Cout != 32 && a.Cout != 64) return false;
  if (!((a.stride == 1 && (a.C == 32 || a.C == 64)) || (a.stride == 2 && a.C == 8 && a.Cout == 32))) return false;
  if (a.seg_m > 0 && (a.seg_m % 64 != 0 || a.seg_m < 256 || a.M % a.seg_m != 0)) return false;
  if (a.bnb && a.stats) return false;
  const long long HoWo = (long long)a.Ho * a.Wo;
  // block-relative byte offsets in 31 bits: a 256-pixel tile spans few images
  if (((256 + HoWo - 1) / HoWo + 2) * a.sN * 2 > 0x7fffffffLL) return false;
  return (a.M + 255) / 256 <= 0x7fffffffLL / 256;
}

// persistent grid: as many blocks as fit on the 256 CUs at once — by LDS and
// by registers (the runtime's occupancy of the kernel): an LDS-only count put
// 4 blocks per CU where the 150-220-register forms hold 2-3, so the last
// blocks ran their whole tile share after the others had finished
template <int C, int COUT, int ST, bool BNB>
static int sconv_grid(int ntiles) {
  constexpr int K = 9 * C, NKK = (K + 31) / 32;
  constexpr int lds = NKK * COUT * 64 + 2 * 3 * COUT * 4 + 16;
  static const int per_cu = [] {
    int n = (160 * 1024) / lds;
    if (n > 4) n = 4;  // 4 x 256 threads: 16 waves per CU
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, sconv_kernel<C, COUT, ST, BNB>, 256, 0) == hipSuccess &&
        occ >= 1 && occ < n)
      n = occ;
    return n;
  }();
  const int g = 256 * per_cu;
  return ntiles < g ? ntiles : g;
}

template <bool BNB>
static bool sconv_dispatch(const PgArgs& a, int ntiles, hipStream_t st) {
  if (a.stride == 1 && a.C == 32 && a.Cout == 32) {
    set_last_kernel(BNB ? "sconv_kernel<32,32,bnb>" : "sconv_kernel<32,32>");
    hipLaunchKernelGGL((sconv_kernel<32, 32, 1, BNB>), dim3(sconv_grid<32, 32, 1, BNB>(ntiles)), dim3(256), 0, st, a, ntiles);
  } else if (a.stride == 1 && a.C == 32 && a.Cout == 64) {
    set_last_kernel(BNB ? "sconv_kernel<32,64,bnb>" : "sconv_kernel<32,64>");
    hipLaunchKernelGGL((sconv_kernel<32, 64, 1, BNB>), dim3(sconv_grid<32, 64, 1, BNB>(ntiles)), dim3(256), 0, st, a, ntiles);
  } else if (a.stride == 1 && a.C == 64 && a.Cout == 32) {
    set_last_kernel(BNB ? "sconv_kernel<64,32,bnb>" : "sconv_kernel<64,32>");
    hipLaunchKernelGGL((sconv_kernel<64, 32, 1, BNB>), dim3(sconv_grid<64, 32, 1, BNB>(ntiles)), dim3(256), 0, st, a, ntiles);
  } else if (a.stride == 1 && a.C == 64 && a.Cout == 64) {
    set_last_kernel(BNB ? "sconv_kernel<64,64,bnb>" : "sconv_kernel<64,64>");
    hipLaunchKernelGGL((sconv_kernel<64, 64, 1, BNB>), dim3(sconv_grid<64, 64, 1, BNB>(ntiles)), dim3(256), 0, st, a, ntiles);
  } else if (a.stride == 2 && a.C == 8 && a.Cout == 32) {
    set_last_kernel(BNB ? "sconv_kernel<8,32,s2,bnb>" : "sconv_kernel<8,32,s2>");
    hipLaunchKernelGGL((sconv_kernel<8, 32, 2, BNB>), dim3(sconv_grid<8, 32, 2, BNB>(ntiles)), dim3(256), 0, st, a, ntiles);
  } else {
    return false;
  }
  return true;
}

// candidate 20: the direct small-channel kernel; false if the shape is not one
bool sconv_launch(const PgArgs& a, hipStream_t st) {
  if (!sconv_ok(a)) return false;
  const int ntiles = (int)((a.M + 255) / 256);
  if (a.bnb) return sconv_dispatch<true>(a, ntiles, st);
  return sconv_dispatch<false>(a, ntiles, st);
}

// ---------------------------------------------------------------------------
// Halo-tiled direct 3x3 convolution (stride 1, pad 1; C in {32, 64} channels
// in, Cout in {32, 64} out): the stem conv2/conv3 (models.py:312-317, 112x112)
// and the layer-1 conv2 (models.py:200-201, 56x56), forward and data gradient
// with the fused BN-backward reduction.
//
// An output tile is TR x TC pixels of one image (all Cout channels).  Its
// input halo of (TR+2) x (TC+2) pixels is brought into LDS ONCE by LDS-DMA and
// all nine taps read it there (sconv re-reads every input pixel nine times
// through L1/L2 as fragment-shaped loads).  One loader wave streams the halo
// of the block's next tile into the second of two halo buffers while four
// compute waves run the MFMAs of the current one out of the first; the filter
// bank stays in LDS for the whole persistent block.
//
// Halo LDS image: 1-KB blocks of PB pixels x CPT 16-B channel chunks, chunk
// major inside a block (lane l of a DMA instruction fills chunk l / PB of
// pixel l % PB, so one instruction reads PB whole pixels = 1 KB of contiguous
// NHWC input).  A B fragment read (16 consecutive halo pixels of one tile row,
// one chunk per lane quad) then hits 16 distinct 16-B bank slots in every
// ds_read_b128 lane group, for every tap offset.
//
// The BN-backward operand of the epilogue (y of the BN before the ReLU) and
// the per-channel parameters are loaded into registers before the MFMAs, so
// their latency hides behind them.
// ---------------------------------------------------------------------------
#define HC_MAXSEG 4
template <int C>
__device__ __forceinline__ int hc_addr(int q, int c) {
  constexpr int PB = 64 / (C / 8);
  constexpr int PBL = PB == 16 ? 4 : 3;
  return ((q >> PBL) << 10) + c * (PB * 16) + ((q & (PB - 1)) << 4);
}

template <int C, int COUT, int TR, int TC>
struct HcGeom {
  static constexpr int NWC = 4;                    // compute waves
  static constexpr int CPT = C / 8, PB = 64 / CPT;
  static constexpr int NKK = 9 * C / 32;           // 32-k MFMA steps
  static constexpr int MTC = COUT / 16, NP = MTC / 2;
  static constexpr int TCB = TC / 16;              // 16-pixel MFMA tiles per tile row
  static constexpr int NTP = TR * TCB / NWC;       // MFMA pixel tiles per compute wave
  static constexpr int HW = TC + 2, NQ = HW * (TR + 2);
  static constexpr int NB = (NQ + PB - 1) / PB;    // 1-KB halo blocks
  static constexpr int HB = NB * 1024;
  static constexpr int WB = NKK * COUT * 64;       // filter image
  static constexpr int PRM = HC_MAXSEG * 4 * COUT * 4;  // BN-backward parameters per segment
  static constexpr int FIX = WB + PRM + pg_red_bytes<COUT>();
  // halo buffers: three (two tiles in flight behind the one being computed)
  // where that fits and keeps the workgroups per CU, else two; NB <= 31 so the
  // loader's counted vmcnt(NB) fits the 6-bit field
  static constexpr bool THREE = FIX + 3 * HB <= 160 * 1024 && (160 * 1024) / (FIX + 3 * HB) ==
                                (160 * 1024) / (FIX + 2 * HB) && NB <= 31;
  static constexpr int NBUF = THREE ? 3 : 2;
  static constexpr int LDS = WB + NBUF * HB + PRM + pg_red_bytes<COUT>();
  // waves per SIMD the registers must allow for every workgroup the LDS admits
  // to fit on a CU (5 waves each: 4 compute + the loader), at most 3 (168
  // VGPRs: below that the tiles spill).  Without it the 32 -> 32 stem tile
  // (216 VGPRs, LDS for two workgroups) ran one workgroup per CU: one compute
  // wave per SIMD.
  static constexpr int WPB = (160 * 1024) / LDS > 4 ? 4 : (160 * 1024) / LDS;
  static constexpr int WPE = (5 * WPB + 3) / 4 > 3 ? 3 : (5 * WPB + 3) / 4;
};

template <int C, int COUT, int TR, int TC, bool BNB>
__global__ void __launch_bounds__(320) __attribute__((amdgpu_waves_per_eu(HcGeom<C, COUT, TR, TC>::WPE)))
hconv_kernel(PgArgs a, int ntiles) {
  using Gm = HcGeom<C, COUT, TR, TC>;
  constexpr int NWC = Gm::NWC, PB = Gm::PB, NKK = Gm::NKK, MTC = Gm::MTC, NP = Gm::NP;
  constexpr int TCB = Gm::TCB, NTP = Gm::NTP, HW = Gm::HW, NQ = Gm::NQ, NB = Gm::NB, HB = Gm::HB;
  constexpr int WB = Gm::WB, NBUF = Gm::NBUF;
  static_assert(C % 32 == 0 && COUT % 32 == 0 && TC % 16 == 0, "tile shape");
  static_assert(NTP * NWC == TR * TCB, "pixel tiles per wave");
  static_assert(Gm::LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[Gm::LDS];
  float* prm = reinterpret_cast<float*>(smem + WB + NBUF * HB);  // [seg][istd, mean, mask scale, mask beta][COUT]
  float* red = reinterpret_cast<float*>(smem + WB + NBUF * HB + Gm::PRM);
  int* red_cnt = reinterpret_cast<int*>(smem + WB + NBUF * HB + Gm::PRM + 6 * COUT * 4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int G = gridDim.x;
  const int ntw = (a.Wo + TC - 1) / TC, nth = (a.Ho + TR - 1) / TR;
  const int HoWo = a.Ho * a.Wo;
  const bool sums = a.stats != nullptr || BNB;

  // halo of tile t -> buffer buf (loader wave)
  auto issue_halo = [&](int t, int buf) {
    const int img = t / (nth * ntw), rem = t - img * (nth * ntw);
    const int h0 = (rem / ntw) * TR, w0 = (rem - (rem / ntw) * ntw) * TC;
    const __amdgpu_buffer_rsrc_t xr =
        pg_rsrc(reinterpret_cast<const bf16*>(a.x) + (long long)img * a.sN, (a.x_elems - (long long)img * a.sN) * 2);
    char* hb = smem + WB + buf * HB;
    const int c = lane / PB, ql = lane - c * PB;
#pragma unroll 4
    for (int b = 0; b < NB; ++b) {
      const int q = b * PB + ql;
      const int hr = q / HW, hc = q - (q / HW) * HW;
      const int ih = h0 - 1 + hr, iw = w0 - 1 + hc;
      const bool ok = q < NQ && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      glds16(xr, hb + b * 1024, ok ? (unsigned)((ih * (int)a.sH + iw * (int)a.sW) * 2 + c * 16) : PG_OOB);
    }
  };

  if (wid == NWC) {
    if ((int)blockIdx.x < ntiles) issue_halo(blockIdx.x, 0);
    if (NBUF == 3 && (int)blockIdx.x + G < ntiles) issue_halo(blockIdx.x + G, 1);
  } else {
    if (sums) {
      for (int i = tid; i < 6 * COUT; i += 64 * NWC) red[i] = 0.f;
      if (tid == 0) *red_cnt = 0;
    }
    if constexpr (BNB) {
      const int nsg = a.seg_m > 0 ? (int)(a.M / a.seg_m) : 1;
      for (int i = tid; i < nsg * 4 * COUT; i += 64 * NWC) {
        const int sg = i / (4 * COUT), r = (i / COUT) & 3, ch = i % COUT;
        const float* src = r == 0 ? a.bnb_istd[0] : r == 1 ? a.bnb_mean[0]
                         : r == 2 ? a.bnb_mbn + 2 * a.Cout : a.bnb_mbn + 3 * a.Cout;
        prm[i] = src[sg * a.bnb_pstride + ch];
      }
    }
    // filters -> LDS (sconv's image: block kk holds COUT rows of 64 B)
    for (int i = tid; i < NKK * COUT * 4; i += 64 * NWC) {
      const int kk = i / (COUT * 4), rem = i - kk * COUT * 4;
      const int rho = rem >> 2, c = rem & 3;
      const uint4 v =
          *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.w) + (long long)pg_perm(rho) * a.K + kk * 32 + c * 8);
      *reinterpret_cast<uint4*>(smem + (kk * COUT + rho) * 64 + ((c ^ sc_sw(rho)) << 4)) = v;
    }
  }

  // the loader and the compute waves run separate loops with one barrier per
  // tile each (a role branch inside one loop makes the compiler merge and copy
  // the accumulators every tile)
  if (wid == NWC) {
    int k = 0;
    for (int tile = blockIdx.x; tile < ntiles; tile += G, ++k) {
      // this tile's halo has landed (with three buffers the next tile's, issued
      // after it, may still be in flight: its NB DMAs are the newest)
      if (NBUF == 3 && tile + G < ntiles) vm_wait<NB>();
      else vm_wait<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // the buffer of tile k-1, which every compute wave left before this barrier
      if (tile + (NBUF - 1) * G < ntiles) issue_halo(tile + (NBUF - 1) * G, (k + NBUF - 1) % NBUF);
    }
    vm_wait<0>();
    return;
  }
  // per MFMA pixel tile j of a tile: this lane's output pixel and its halo position
  auto tile_px = [&](int tile, long long (&px)[NTP], bool (&pv)[NTP], int (&qb)[NTP]) {
    const int img = tile / (nth * ntw), rem = tile - img * (nth * ntw);
    const int h0 = (rem / ntw) * TR, w0 = (rem - (rem / ntw) * ntw) * TC;
    const long long pimg = (long long)img * HoWo;
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const int m = wid * NTP + j, row = m / TCB, cb = m - (m / TCB) * TCB;
      const int oh = h0 + row, ow = w0 + cb * 16 + fr;
      pv[j] = oh < a.Ho && ow < a.Wo;
      px[j] = pv[j] ? pimg + oh * a.Wo + ow : pimg;
      qb[j] = row * HW + cb * 16 + fr;
    }
    return pimg;
  };
  // the BN-backward operand of a tile is loaded one tile ahead (issued after the
  // previous tile's epilogue, consumed in this tile's), so its latency runs
  // under the barrier and the MFMAs instead of in front of them
  Vec16<bf16> yp[NP][NTP];
  auto load_yp = [&](const long long (&px)[NTP]) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        yp[p][j] = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[0]) + px[j] * a.ldy + 32 * p + 8 * fq);
  };
  if constexpr (BNB) {
    if ((int)blockIdx.x < ntiles) {
      long long px0[NTP];
      bool pv0[NTP];
      int qb0[NTP];
      tile_px(blockIdx.x, px0, pv0, qb0);
      load_yp(px0);
    }
  }
  int k = 0;
  for (int tile = blockIdx.x; tile < ntiles; tile += G, ++k) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // halo k visible; buffer (k-1) % NBUF and the statistics accumulator free
    asm volatile("" ::: "memory");
    long long px[NTP];
    bool pv[NTP];
    int qb[NTP];
    const long long pimg = tile_px(tile, px, pv, qb);
    const long long wseg = a.seg_m > 0 ? pimg / a.seg_m : 0;
    // ---- MFMAs: filters (A) and halo (B) from LDS
    const char* hb = smem + WB + (k % NBUF) * HB;
    f32x4 acc[MTC][NTP];
#pragma unroll
    for (int i = 0; i < MTC; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int KPT = C / 32;  // 32-k steps per tap
    // taps fully unrolled where the registers allow (no spills), else by rows
    // (by rows also where the waves-per-SIMD bound leaves too few registers)
    constexpr int TUN = ((NTP <= 2 || (C == 32 && MTC * NTP <= 8)) && !(Gm::WPE >= 3 && NTP > 2)) ? 9 : 3;
#pragma unroll TUN
    for (int t = 0; t < 9; ++t) {
      const int toff = (t / 3) * HW + (t % 3);
      int qa[NTP];
#pragma unroll
      for (int j = 0; j < NTP; ++j) qa[j] = qb[j] + toff;
#pragma unroll
    for (int h = 0; h < KPT; ++h) {
      const int kk = t * KPT + h, c = h * 4 + fq;
      uint4 af[MTC], bv[NTP];
#pragma unroll
      for (int i = 0; i < MTC; ++i) {
        const int rho = i * 16 + fr;
        af[i] = *reinterpret_cast<const uint4*>(smem + (kk * COUT + rho) * 64 + ((fq ^ sc_sw(rho)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NTP; ++j) bv[j] = *reinterpret_cast<const uint4*>(hb + hc_addr<C>(qa[j], c));
#pragma unroll
      for (int i = 0; i < MTC; ++i)
#pragma unroll
        for (int j = 0; j < NTP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                              *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j], 0, 0, 0);
    }
    }
    // ---- epilogue: BN statistics or the fused BN-backward reduction, bf16 stores
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int ch0 = 32 * p + 8 * fq;
      float s1[8], s2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
      float xa[8], xm[8], ms[8], mh[8];
      if constexpr (BNB) {
        const float* pp = prm + wseg * 4 * COUT + ch0;
        loadf8v(pp, xa);
        loadf8v(pp + COUT, xm);
        loadf8v(pp + 2 * COUT, ms);
        loadf8v(pp + 3 * COUT, mh);
      }
#pragma unroll
      for (int j = 0; j < NTP; ++j) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][j][r]; v[4 + r] = acc[2 * p + 1][j][r]; }
        if (pv[j]) {
          if constexpr (!BNB) {  // eval-mode conv + folded BN (+ ReLU): bias and activation here
            if (a.bias) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += a.bias[ch0 + e];
            }
            if (a.relu) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
            }
          }
          if constexpr (BNB) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float yv = to_f(yp[p][j].v[e]);
              v[e] = (yv - xm[e]) * ms[e] + mh[e] > 0.f ? v[e] : 0.f;  // kind 1: target 0 is the ReLU's BN
              s1[e] += v[e];
              s2[e] += v[e] * ((yv - xm[e]) * xa[e]);
            }
          } else if (sums) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
          }
          Vec16<bf16> o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o.v[e] = from_f<bf16>(v[e]);
          st16<bf16>(reinterpret_cast<bf16*>(a.y) + px[j] * a.ldy + ch0, o);
        }
      }
      if (sums) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] = dpp_row_sum(s1[e]); s2[e] = dpp_row_sum(s2[e]); }
        if (fr == 15) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            atomicAdd(red + ch0 + e, s1[e]);
            atomicAdd(red + COUT + ch0 + e, s2[e]);
          }
        }
      }
    }
    if constexpr (BNB) {
      if (tile + G < ntiles) {
        long long pxn[NTP];
        bool pvn[NTP];
        int qbn[NTP];
        tile_px(tile + G, pxn, pvn, qbn);
        load_yp(pxn);
      }
    }
    if (sums) stats_flush<COUT>(red, red_cnt, NWC * (k + 1) - 1, a, 0, tile % ARTSBIR_NSLOT, lane, pimg, 1);
  }
}

// shapes the halo-tiled kernel takes
static bool hconv_ok(const PgArgs& a) {
  if (a.R != 3 || a.S != 3 || a.pad != 1 || a.stride != 1 || a.M <= 0) return false;
  if ((a.C != 32 && a.C != 64) || (a.Cout != 32 && a.Cout != 64) || a.K != 9 * a.C) return false;
  if (a.res_mode || (a.bnb && (a.bnb != 1 || a.bnb_nt != 1 || a.stats))) return false;
  const long long HoWo = (long long)a.Ho * a.Wo;
  if (a.Ho != a.H || a.Wo != a.W || a.M % HoWo) return false;
  // statistics segments are whole images (a tile never spans two)
  if (a.seg_m > 0 && (a.seg_m % HoWo || a.M % a.seg_m)) return false;
  if (a.bnb && a.seg_m > 0 && a.M / a.seg_m > HC_MAXSEG) return false;
  if (a.sW < a.C || a.sN * 2 > 0x7fffffffLL || (long long)a.H * a.sH * 2 > 0x7fffffffLL) return false;
  const long long nt = (a.M / HoWo) * ((a.Ho + 15) / 16) * ((a.Wo + 15) / 16) * 2;
  return nt < 0x7fffffffLL;
}

template <int C, int COUT, int TR, int TC, bool BNB>
static void hconv_go(const PgArgs& a, hipStream_t st) {
  using Gm = HcGeom<C, COUT, TR, TC>;
  const int ntiles = (int)((a.M / ((long long)a.Ho * a.Wo)) * ((a.Ho + TR - 1) / TR) * ((a.Wo + TC - 1) / TC));
  int per_cu = (160 * 1024) / Gm::LDS;
  if (per_cu > 4) per_cu = 4;
  const int g = 256 * per_cu < ntiles ? 256 * per_cu : ntiles;
  static const char* nm = nullptr;
  static char buf[64];
  if (!nm) {
    snprintf(buf, sizeof buf, "hconv_kernel<%d,%d,%dx%d%s>", C, COUT, TR, TC, BNB ? ",bnb" : "");
    nm = buf;
  }
  set_last_kernel(nm);
  hipLaunchKernelGGL((hconv_kernel<C, COUT, TR, TC, BNB>), dim3(g), dim3(320), 0, st, a, ntiles);
}

template <int C, int COUT, bool BNB>
static void hconv_tiles(const PgArgs& a, hipStream_t st) {
  // 16 x 16 tiles when the image splits evenly (stem, 112 x 112), else 8 x 16
  if (a.Ho % 16 == 0 && a.Wo % 16 == 0) hconv_go<C, COUT, 16, 16, BNB>(a, st);
  else hconv_go<C, COUT, 8, 16, BNB>(a, st);
}

template <bool BNB>
static void hconv_dispatch(const PgArgs& a, hipStream_t st) {
  if (a.C == 32 && a.Cout == 32) hconv_tiles<32, 32, BNB>(a, st);
  else if (a.C == 32) hconv_tiles<32, 64, BNB>(a, st);
  else if (a.Cout == 32) hconv_tiles<64, 32, BNB>(a, st);
  else hconv_tiles<64, 64, BNB>(a, st);
}

// candidate 21: the halo-tiled small-channel kernel
bool hconv_launch(const PgArgs& a, hipStream_t st) {
  if (!hconv_ok(a)) return false;
  if (a.bnb) hconv_dispatch<true>(a, st);
  else hconv_dispatch<false>(a, st);
  return true;
}

// ---------------------------------------------------------------------------
// launch: pick the tile shape with the best (tile utilisation x CU fill)
// ---------------------------------------------------------------------------
struct PgCfg {
  int bpx, bch, lds, threads;
  float factor;
};
static const PgCfg kCfgs[] = {
    {256, 256, 2 * 256 * 256, 512, 1.00f},          // 0: 256 x 256, 2 stages
    {256, 128, 3 * (256 + 128) * 128, 512, 0.95f},  // 1: 256 x 128, 3 stages
    {256, 64, 3 * (256 + 64) * 128, 512, 0.85f},    // 2: 256 x 64, 3 stages
    {128, 128, 2 * 256 * 128, 256, 0.80f},          // 3: 128 x 128, 2 stages, 4 waves
    {256, 32, 4 * (256 + 32) * 128, 512, 0.70f},    // 4: 256 x 32, 4 stages
    {256, 256, 4 * 512 * 64, 512, 0.0f},           // 5: 256 x 256, four 32-k stages (tuned only)
};
constexpr int kNumCfg = 6;

template <bool MULTI, int BK, bool TWO>
static void pg_launch_cfg(int c, const PgArgs& a, long long tiles, hipStream_t st) {
  const dim3 g((unsigned)tiles);
  switch (c) {
    case 0: hipLaunchKernelGGL((pgemm_kernel<256, 256, 4, 2, 2, MULTI, BK, TWO>), g, dim3(512), 0, st, a); break;
    case 1: hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, MULTI, BK, TWO>), g, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL((pgemm_kernel<256, 64, 4, 2, 3, MULTI, BK, TWO>), g, dim3(512), 0, st, a); break;
    case 3: hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 2, MULTI, BK, TWO>), g, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((pgemm_kernel<256, 32, 8, 1, 4, MULTI, BK, TWO>), g, dim3(512), 0, st, a); break;
    default:
      if constexpr (!MULTI)
        hipLaunchKernelGGL((pgemm_kernel<256, 256, 4, 2, 4, false, BK, TWO, false, 32>), g, dim3(512), 0, st, a);
      break;
  }
}

// PF variants (candidates 11 / 12 / 13 = tile shapes 1 / 2 / 3 with the
// epilogue operands prefetched into registers)
template <int BK, bool TWO>
static void pg_launch_pf(int base, const PgArgs& a, long long tiles, hipStream_t st) {
  const dim3 g((unsigned)tiles);
  switch (base) {
    case 1: hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, false, BK, TWO, true>), g, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL((pgemm_kernel<256, 64, 4, 2, 3, false, BK, TWO, true>), g, dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 2, false, BK, TWO, true>), g, dim3(256), 0, st, a); break;
  }
}

static bool pg_pf_launch(int c, const PgArgs& a, bool multi, hipStream_t st) {
  const int base = c - 10;
  if (multi || base < 1 || base > 3) return false;
  if (a.bnb == 2 || (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) || (a.bnb == 3 && !a.res_mode)) return false;
  // plain: the data gradient with a residual, or the gated GEMM (res_mode 3, column sums in stats)
  if (!a.bnb && (!a.res_mode || (a.stats && a.res_mode != 3))) return false;
  const PgCfg& g = kCfgs[base];
  const long long tiles = ((a.M + g.bpx - 1) / g.bpx) * ((a.Cout + g.bch - 1) / g.bch);
  if (tiles > 0x7fffffffLL) return false;
  if (a.bnb == 1) pg_launch_pf<1, false>(base, a, tiles, st);
  else if (a.bnb == 3 && a.bnb_nt == 2) pg_launch_pf<3, true>(base, a, tiles, st);
  else if (a.bnb == 3) pg_launch_pf<3, false>(base, a, tiles, st);
  else pg_launch_pf<0, false>(base, a, tiles, st);
  static const char* names[2][3] = {{"pgemm_kernel<256,128,pf>", "pgemm_kernel<256,64,pf>", "pgemm_kernel<128,128,pf>"},
                                    {"pgemm_kernel<256,128,bnb,pf>", "pgemm_kernel<256,64,bnb,pf>",
                                     "pgemm_kernel<128,128,bnb,pf>"}};
  set_last_kernel(names[a.bnb ? 1 : 0][base - 1]);
  return true;
}

// the fused-epilogue variant of a launch: ACT (kind 1, one target, no
// residual) or RES (kinds 2/3, residual present, one or two targets)
template <bool MULTI>
static bool pg_launch_bnb(int c, const PgArgs& a, long long tiles, hipStream_t st) {
  if (a.bnb == 1) {
    if (a.bnb_nt != 1 || a.res_mode) return false;
    pg_launch_cfg<MULTI, 1, false>(c, a, tiles, st);
    return true;
  }
  if (MULTI || !a.res_mode) return false;  // RES dgrads: 1x1 convs over >= 64 channels, residual added
  if (a.bnb == 3) {
    if (a.bnb_nt == 2) pg_launch_cfg<false, 3, true>(c, a, tiles, st);
    else pg_launch_cfg<false, 3, false>(c, a, tiles, st);
  } else {
    if (a.bnb_nt == 2) pg_launch_cfg<false, 2, true>(c, a, tiles, st);
    else pg_launch_cfg<false, 2, false>(c, a, tiles, st);
  }
  return true;
}

template <bool MULTI, bool BNB, bool FWDS>
static void pstream_launch(int bch, const PgArgs& a, int grid, int ntl, hipStream_t st) {
  if (bch == 32)
    hipLaunchKernelGGL((pstream_kernel<32, 8, 1, 4, MULTI, BNB, FWDS>), dim3(grid), dim3(768), 0, st, a, ntl);
  else if (bch == 64)
    hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, MULTI, BNB, FWDS>), dim3(grid), dim3(768), 0, st, a, ntl);
  else hipLaunchKernelGGL((pstream_kernel<128, 4, 2, 3, MULTI, BNB, FWDS>), dim3(grid), dim3(768), 0, st, a, ntl);
}

template <int BK, bool TWO>
static void pstream_launch_k(int bch, const PgArgs& a, int grid, int ntl, hipStream_t st) {
  constexpr bool ONLY64 = TWO || BK == 1;  // 128-channel blocks would spill there
  if (ONLY64 || bch == 64)
    hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, false, true, false, BK, TWO>), dim3(grid), dim3(768), 0, st, a, ntl);
  else if constexpr (!ONLY64)
    hipLaunchKernelGGL((pstream_kernel<128, 4, 2, 3, false, true, false, BK, TWO>), dim3(grid), dim3(768), 0, st, a,
                       ntl);
}

// candidate 15: the persistent streaming kernel with 32-k stages (six in the
// LDS the 64-k form holds three in; plain and forward-statistics epilogues,
// C % 64 == 0, 64- / 128-channel blocks)
static bool pstream_k32_launch(const PgArgs& a, bool multi, hipStream_t st) {
  if (multi || a.bnb || a.Cout <= 32) return false;
  const int bch = a.Cout <= 64 ? 64 : 128;
  const long long nt = ((a.M + 255) / 256) * ((a.Cout + bch - 1) / bch);
  if (nt > 0x7fffffffLL) return false;
  const int grid = (int)(nt < 256 ? nt : 256), ntl = (int)nt;
  set_last_kernel(bch == 64 ? "pstream_kernel<64,k32>" : "pstream_kernel<128,k32>");
  if (a.stats) {
    if (bch == 64)
      hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 6, false, false, true, 0, false, 32>), dim3(grid), dim3(768), 0, st, a,
                         ntl);
    else hipLaunchKernelGGL((pstream_kernel<128, 4, 2, 6, false, false, true, 0, false, 32>), dim3(grid), dim3(768), 0,
                            st, a, ntl);
  } else {
    if (bch == 64)
      hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 6, false, false, false, 0, false, 32>), dim3(grid), dim3(768), 0, st,
                         a, ntl);
    else hipLaunchKernelGGL((pstream_kernel<128, 4, 2, 6, false, false, false, 0, false, 32>), dim3(grid), dim3(768), 0,
                            st, a, ntl);
  }
  return true;
}

// candidate 14: the persistent streaming kernel with the specialised fused
// BN-backward epilogue (the kinds pg_launch_bnb takes, channel blocks 64 / 128)
static bool pstream_bnb_launch(const PgArgs& a, bool multi, hipStream_t st) {
  if (!a.bnb || multi || a.Cout < 64) return false;
  if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
  if (a.bnb != 1 && !a.res_mode) return false;
  const int bch = (a.Cout <= 64 || a.bnb == 1 || a.bnb_nt == 2) ? 64 : 128;  // see pstream_launch_k
  const long long nt = ((a.M + 255) / 256) * ((a.Cout + bch - 1) / bch);
  if (nt > 0x7fffffffLL) return false;
  const int grid = (int)(nt < 256 ? nt : 256), ntl = (int)nt;
  set_last_kernel(bch == 64 ? "pstream_kernel<64,bnbk>" : "pstream_kernel<128,bnbk>");
  if (a.bnb == 1) pstream_launch_k<1, false>(bch, a, grid, ntl, st);
  else if (a.bnb == 3 && a.bnb_nt == 2) pstream_launch_k<3, true>(bch, a, grid, ntl, st);
  else if (a.bnb == 3) pstream_launch_k<3, false>(bch, a, grid, ntl, st);
  else if (a.bnb_nt == 2) pstream_launch_k<2, true>(bch, a, grid, ntl, st);
  else pstream_launch_k<2, false>(bch, a, grid, ntl, st);
  return true;
}

static bool pg_supported(const PgArgs& a, bool& multi) {
  if (a.Cout % 32 != 0 || a.M <= 0) return false;
  if (a.C % 64 == 0) multi = false;
  else if (a.C == 8 || a.C == 16 || a.C == 32) multi = true;
  else return false;
  if (a.R * a.S > 32 || a.K % 8 != 0) return false;
  if ((long long)a.Cout * a.K * 2 > 0x7fffffffLL) return false;
  const long long HoWo = (long long)a.Ho * a.Wo;
  if (((256 + HoWo - 1) / HoWo + 2) * a.sN * 2 > 0x7fffffffLL) return false;
  if (a.M > (1LL << 40)) return false;
  // segments: every wave's pixels in one segment, a tile in at most two
  if (a.seg_m > 0 && (a.seg_m % 64 != 0 || a.seg_m < 256 || a.M % a.seg_m != 0)) return false;
  if (a.bnb && (a.stats || a.Cout % 8 != 0)) return false;
  return true;
}

// candidate 16: the fused BN-backward data gradient (or a plain one with a
// residual / gate operand) on a 128 x 128 tile (4 waves) with 32-k stages
// (3-stage ring, 48 KB) and its epilogue operands read from global memory
// (GLB): three workgroups per CU
static bool pg_glb_launch(const PgArgs& a, bool multi, hipStream_t st) {
  if (multi) return false;
  if (!a.bnb) {  // plain epilogue with a residual or gate operand (res_mode 1-3), read from global memory
    if (!a.res_mode || a.bias || a.relu) return false;
    const long long tiles = ((a.M + 127) / 128) * ((a.Cout + 127) / 128);
    if (tiles > 0x7fffffffLL) return false;
    hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 3, false, 0, false, false, 32, true>), dim3((unsigned)tiles),
                       dim3(256), 0, st, a);
    set_last_kernel("pgemm_kernel<128,128,k32,glb>");
    return true;
  }
  if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
  if (a.bnb != 1 && !a.res_mode) return false;
  const long long tiles = ((a.M + 127) / 128) * ((a.Cout + 127) / 128);
  if (tiles > 0x7fffffffLL) return false;
  const dim3 g((unsigned)tiles);
#define PG_GLB(BKV, TWOV) \
  hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 3, false, BKV, TWOV, false, 32, true>), g, dim3(256), 0, st, a)
  if (a.bnb == 1) PG_GLB(1, false);
  else if (a.bnb == 3 && a.bnb_nt == 2) PG_GLB(3, true);
  else if (a.bnb == 3) PG_GLB(3, false);
  else if (a.bnb_nt == 2) PG_GLB(2, true);
  else PG_GLB(2, false);
#undef PG_GLB
  set_last_kernel("pgemm_kernel<128,128,k32,glb,bnb>");
  return true;
}

// candidate 18: the fused BN-backward RES dgrad with the mask as bits (kind 3,
// one target) on a 256 x 128 tile of 8 waves, 32-k stages in a 3-stage ring
// (72 KB), epilogue operands from global memory: two workgroups (16 waves) per
// CU at 128 VGPRs (the other kinds spill there)
static bool pg_glb2_launch(const PgArgs& a, bool multi, hipStream_t st) {
  if (multi || a.bnb != 3 || a.bnb_nt != 1 || !a.res_mode) return false;
  const long long tiles = ((a.M + 255) / 256) * ((a.Cout + 127) / 128);
  if (tiles > 0x7fffffffLL) return false;
  hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, false, 3, false, false, 32, true>), dim3((unsigned)tiles),
                     dim3(512), 0, st, a);
  set_last_kernel("pgemm_kernel<256,128,k32,glb,bnb>");
  return true;
}

// candidate 19: the plain / statistics / bias-ReLU-residual epilogues on the
// 256 x 128 8-wave tile with a 3-stage ring of 32-k stages and operands read
// from global memory (72 KB of LDS): two workgroups per CU at 128 VGPRs
static bool pg_k32w8_launch(const PgArgs& a, bool multi, hipStream_t st) {
  if (multi || a.bnb || a.res_mode == 3) return false;
  const long long tiles = ((a.M + 255) / 256) * ((a.Cout + 127) / 128);
  if (tiles > 0x7fffffffLL) return false;
  hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, false, 0, false, false, 32, true>), dim3((unsigned)tiles),
                     dim3(512), 0, st, a);
  set_last_kernel("pgemm_kernel<256,128,k32,glb>");
  return true;
}

// The y-side fold of the block's first conv with the fused BN-backward reduction
// of the previous block's output (artsbir_conv1x1_dgrad_fold_y: residual added,
// kinds 2 / 3, one or two targets): candidates 16 (128 x 128 GLB), 18 (256 x 128
// GLB, kind 3 with one target: the 8-wave tile's 128 VGPRs) and 22 (pp256)
static bool pg_fold_res_launch(const PgArgs& a, int c, hipStream_t st) {
  if (!a.res_mode) return false;
  auto ntl = [&](int bpx, int bch) { return ((a.M + bpx - 1) / bpx) * ((a.Cout + bch - 1) / bch); };
  const bool two = a.bnb_nt == 2;
  switch (c) {
    case 16: {
      if (!pg_fold_ok(a, 128, 32) || ntl(128, 128) > 0x7fffffffLL) return false;
      const dim3 g((unsigned)ntl(128, 128));
#define PG_FGLB(BKV, TWOV) \
  hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 3, false, BKV, TWOV, false, 32, true, true>), g, dim3(256), 0, st, a)
      if (a.bnb == 3 && two) PG_FGLB(3, true);
      else if (a.bnb == 3) PG_FGLB(3, false);
      else if (two) PG_FGLB(2, true);
      else PG_FGLB(2, false);
#undef PG_FGLB
      set_last_kernel("pgemm_kernel<128,128,k32,glb,bnb,fold>");
      return true;
    }
    case 18: {
      if (a.bnb != 3 || two || !pg_fold_ok(a, 256, 32) || ntl(256, 128) > 0x7fffffffLL) return false;
      hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, false, 3, false, false, 32, true, true>),
                         dim3((unsigned)ntl(256, 128)), dim3(512), 0, st, a);
      set_last_kernel("pgemm_kernel<256,128,k32,glb,bnb,fold>");
      return true;
    }
    default:
      return false;
  }
}

// The folded BatchNorm-backward data gradient (a.x2: artsbir_conv1x1_dgrad_fold):
// the candidates instantiated with the two-operand loader — 2 (256 x 64), 16 (the
// 128 x 128 GLB tile, plain or ACT epilogue), 19 (256 x 128 GLB, plain), 10 / 14
// (the persistent streaming kernel, plain / ACT, 64- or 128-channel blocks) and 22
// (pp256, in pp256_launch); epilogue: per-segment bias (+ the kind-1 mask and
// BN-backward reduction of the BatchNorm before the conv's input)
static bool pg_fold_launch(const PgArgs& a, int c, hipStream_t st) {
  if (!a.x2 || !a.bias || a.relu || a.stats || a.res_mode == 3) return false;
  if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
  bool multi;
  if (!pg_supported(a, multi) || multi) return false;
  auto ntl = [&](int bpx, int bch) { return ((a.M + bpx - 1) / bpx) * ((a.Cout + bch - 1) / bch); };
  if (a.bnb == 2 || a.bnb == 3) return pg_fold_res_launch(a, c, st);
  const bool k1 = a.bnb == 1;
  switch (c) {
    case 2: {
      if (!pg_fold_ok(a, 256, 64) || ntl(256, 64) > 0x7fffffffLL) return false;
      const dim3 g((unsigned)ntl(256, 64));
      if (k1) hipLaunchKernelGGL((pgemm_kernel<256, 64, 4, 2, 3, false, 1, false, false, 64, false, true>), g, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((pgemm_kernel<256, 64, 4, 2, 3, false, 0, false, false, 64, false, true>), g, dim3(512), 0, st, a);
      set_last_kernel(k1 ? "pgemm_kernel<256,64,bnb,fold>" : "pgemm_kernel<256,64,fold>");
      return true;
    }
    case 16: {
      if (!pg_fold_ok(a, 128, 32) || ntl(128, 128) > 0x7fffffffLL) return false;
      const dim3 g((unsigned)ntl(128, 128));
      if (k1) hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 3, false, 1, false, false, 32, true, true>), g, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((pgemm_kernel<128, 128, 2, 2, 3, false, 0, false, false, 32, true, true>), g, dim3(256), 0, st, a);
      set_last_kernel(k1 ? "pgemm_kernel<128,128,k32,glb,bnb,fold>" : "pgemm_kernel<128,128,k32,glb,fold>");
      return true;
    }
    case 19: {
      if (k1 || !pg_fold_ok(a, 256, 32) || ntl(256, 128) > 0x7fffffffLL) return false;
      hipLaunchKernelGGL((pgemm_kernel<256, 128, 4, 2, 3, false, 0, false, false, 32, true, true>),
                         dim3((unsigned)ntl(256, 128)), dim3(512), 0, st, a);
      set_last_kernel("pgemm_kernel<256,128,k32,glb,fold>");
      return true;
    }
    case 10:
    case 14: {
      if ((c == 14) != k1 || !pg_fold_ok(a, 256, 64) || a.Cout < 64) return false;
      const int bch = (k1 || a.Cout <= 64) ? 64 : 128;  // the ACT epilogue: 64-channel blocks (pstream_launch_k)
      const long long nt = ntl(256, bch);
      if (nt > 0x7fffffffLL) return false;
      const int grid = (int)(nt < 256 ? nt : 256);
      if (k1)
        hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, false, true, false, 1, false, 64, true>), dim3(grid), dim3(768), 0,
                           st, a, (int)nt);
      else if (bch == 64)
        hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, false, false, false, 0, false, 64, true>), dim3(grid), dim3(768),
                           0, st, a, (int)nt);
      else
        hipLaunchKernelGGL((pstream_kernel<128, 4, 2, 3, false, false, false, 0, false, 64, true>), dim3(grid), dim3(768),
                           0, st, a, (int)nt);
      set_last_kernel(k1 ? "pstream_kernel<64,bnbk,fold>" : bch == 64 ? "pstream_kernel<64,fold>" : "pstream_kernel<128,fold>");
      return true;
    }
    case 17: {  // the persistent streaming kernel with 32-channel blocks (four tiles per pixel panel)
      if (!pg_fold_ok(a, 256, 64) || a.Cout < 32 || a.Cout % 32) return false;
      const long long nt = ntl(256, 32);
      if (nt > 0x7fffffffLL) return false;
      const int grid = (int)(nt < 256 ? nt : 256);
      if (k1)
        hipLaunchKernelGGL((pstream_kernel<32, 8, 1, 4, false, true, false, 1, false, 64, true>), dim3(grid), dim3(768), 0,
                           st, a, (int)nt);
      else
        hipLaunchKernelGGL((pstream_kernel<32, 8, 1, 4, false, false, false, 0, false, 64, true>), dim3(grid), dim3(768),
                           0, st, a, (int)nt);
      set_last_kernel(k1 ? "pstream_kernel<32,bnbk,fold>" : "pstream_kernel<32,fold>");
      return true;
    }
    default:
      return false;
  }
}

// The fold data gradient together with its weight-gradient operands (a.wg_p,
// a.wg_gram): the persistent streaming kernel whose loader waves accumulate
// g^T x and x^T x from the stages they stream (pstream_wg_loader).  Layers with
// 64 input channels under a 256-channel output (K = 320: layer 1's conv3 and
// downsample conv), contiguous NHWC operands, whole 256-pixel tiles.
bool pg_fold_wg_launch(const PgArgs& a, hipStream_t st) {
  if (!a.x2 || !a.wg_p || !a.wg_gram || !a.bias || a.relu || a.stats || a.res_mode) return false;
  if (a.bnb && (a.bnb != 1 || a.bnb_nt != 1)) return false;
  if (a.Cout != 64 || a.K != 320 || a.C1 != 256 || a.C != a.K) return false;
  bool multi;
  if (!pg_supported(a, multi) || multi || !pg_fold_ok(a, 256, 64)) return false;
  if (a.M % 256 || (a.seg_m > 0 && a.seg_m % 256)) return false;
  if (a.sW != a.C1 || a.sH != (long long)a.W * a.sW || a.sN != (long long)a.H * a.sH) return false;
  if (a.sW2 != a.Cout || a.sH2 != (long long)a.W * a.sW2 || a.sN2 != (long long)a.H * a.sH2) return false;
  const long long nt = a.M / 256;
  if (nt > 0x7fffffffLL) return false;
  const int grid = (int)(nt < 256 ? nt : 256);
  if (a.bnb == 1) {
    hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, false, true, false, 1, false, 64, true, 320>), dim3(grid),
                       dim3(768), 0, st, a, (int)nt);
    set_last_kernel("pstream_kernel<64,bnbk,fold,wg>");
  } else {
    hipLaunchKernelGGL((pstream_kernel<64, 4, 2, 3, false, false, false, 0, false, 64, true, 320>), dim3(grid),
                       dim3(768), 0, st, a, (int)nt);
    set_last_kernel("pstream_kernel<64,fold,wg>");
  }
  return true;
}

// candidate c: 0..4 tile shapes of pgemm_kernel, 10 the persistent streaming kernel
bool pgemm_launch_cfg(const PgArgs& a, int c, hipStream_t st) {
  if (a.x2 || a.w_sstride) return c == 22 ? pp256_launch(a, false, st) : pg_fold_launch(a, c, st);
  const bool act = a.bias != nullptr || a.relu != 0;  // bias / ReLU epilogue: pgemm_kernel and pstream only
  if (act && (a.stats || a.bnb)) return false;
  // res_mode 3 (gated data gradient, pg_epilogue_k only): the plain pgemm_kernel tiles
  if (c == 22 || c == 23) return pp256_launch(a, c == 23, st);  // pp256.hip: every epilogue it supports
  if (c == 26) return rstream_launch(a, st);                      // rstream.hip: RES-kind 1x1 dgrads
  if (a.res_mode == 3 && (c < 0 || (c >= kNumCfg && c != 16 && (c < 11 || c > 13)) || a.bnb || a.R * a.S != 1))
    return false;
  if (c == 20) return !act && sconv_launch(a, st);
  if (c == 21) return hconv_launch(a, st);  // bias / ReLU epilogue supported
  if (act && c >= 11 && c <= 13) return false;
  bool multi;
  if (!pg_supported(a, multi)) return false;
  if (c >= 11 && c <= 13) return pg_pf_launch(c, a, multi, st);
  if (c == 14) return pstream_bnb_launch(a, multi, st);
  if (c == 15) return pstream_k32_launch(a, multi, st);
  if (c == 24 || c == 25) {  // 10 / 15 with the forward-statistics epilogue's stores non-temporal
    if (!a.stats || a.bnb || a.bias || a.relu) return false;
    PgArgs b = a;
    b.nts = 1;
    if (!pgemm_launch_cfg(b, c == 24 ? 10 : 15, st)) return false;
    const std::string base = artsbir_last_kernel();
    static const char* nt_names[] = {"pstream_kernel<32,nt>", "pstream_kernel<64,nt>", "pstream_kernel<128,nt>",
                                     "pstream_kernel<64,k32,nt>", "pstream_kernel<128,k32,nt>"};
    const char* nm = base == "pstream_kernel<32>"       ? nt_names[0]
                     : base == "pstream_kernel<64>"     ? nt_names[1]
                     : base == "pstream_kernel<128>"    ? nt_names[2]
                     : base == "pstream_kernel<64,k32>" ? nt_names[3]
                                                        : nt_names[4];
    set_last_kernel(nm);
    return true;
  }
  if (c == 16) return pg_glb_launch(a, multi, st);
  if (c == 18) return pg_glb2_launch(a, multi, st);
  if (c == 19) return pg_k32w8_launch(a, multi, st);
  if (c == 10) {
    const int bch = a.Cout <= 32 ? 32 : a.Cout <= 64 ? 64 : 128;
    const long long nt = ((a.M + 255) / 256) * ((a.Cout + bch - 1) / bch);
    if (nt > 0x7fffffffLL) return false;
    const int grid = (int)(nt < 256 ? nt : 256);
    const int ntl = (int)nt;
    static const char* pnames[2][3] = {{"pstream_kernel<32>", "pstream_kernel<64>", "pstream_kernel<128>"},
                                       {"pstream_kernel<32,bnb>", "pstream_kernel<64,bnb>", "pstream_kernel<128,bnb>"}};
    set_last_kernel(pnames[a.bnb ? 1 : 0][bch == 32 ? 0 : bch == 64 ? 1 : 2]);
    if (a.bnb) {
      if (multi) pstream_launch<true, true, false>(bch, a, grid, ntl, st);
      else pstream_launch<false, true, false>(bch, a, grid, ntl, st);
    } else if (a.stats) {
      if (multi) pstream_launch<true, false, true>(bch, a, grid, ntl, st);
      else pstream_launch<false, false, true>(bch, a, grid, ntl, st);
    } else {
      if (multi) pstream_launch<true, false, false>(bch, a, grid, ntl, st);
      else pstream_launch<false, false, false>(bch, a, grid, ntl, st);
    }
    return true;
  }
  if (c < 0 || c >= kNumCfg) return false;
  if (c == 5 && multi) return false;
  const PgCfg& g = kCfgs[c];
  const long long tiles = ((a.M + g.bpx - 1) / g.bpx) * ((a.Cout + g.bch - 1) / g.bch);
  if (tiles > 0x7fffffffLL) return false;
  static const char* names[2][kNumCfg] = {
      {"pgemm_kernel<256,256>", "pgemm_kernel<256,128>", "pgemm_kernel<256,64>", "pgemm_kernel<128,128>",
       "pgemm_kernel<256,32>", "pgemm_kernel<256,256,k32>"},
      {"pgemm_kernel<256,256,bnb>", "pgemm_kernel<256,128,bnb>", "pgemm_kernel<256,64,bnb>",
       "pgemm_kernel<128,128,bnb>", "pgemm_kernel<256,32,bnb>", "pgemm_kernel<256,256,k32,bnb>"}};
  if (a.bnb) {
    if (!(multi ? pg_launch_bnb<true>(c, a, tiles, st) : pg_launch_bnb<false>(c, a, tiles, st))) return false;
  } else {
    if (multi) pg_launch_cfg<true, 0, false>(c, a, tiles, st);
    else pg_launch_cfg<false, 0, false>(c, a, tiles, st);
  }
  set_last_kernel(names[a.bnb ? 1 : 0][c]);
  return true;
}

// static choice (no tuning): streaming kernel for many tiles, else best-scored tile
int pgemm_default_cfg(const PgArgs& a) {
  if (sconv_ok(a) && !a.bias && !a.relu && a.res_mode != 3) return 20;
  bool multi;
  if (!pg_supported(a, multi)) return -1;
  const int bch = a.Cout <= 32 ? 32 : a.Cout <= 64 ? 64 : 128;
  if (((a.M + 255) / 256) * ((a.Cout + bch - 1) / bch) >= 4 * 256 && a.res_mode != 3) return 10;
  int best = -1;
  float best_score = -1.f;
  for (int c = 0; c < 5; ++c) {
    const PgCfg& g = kCfgs[c];
    const long long tiles = ((a.M + g.bpx - 1) / g.bpx) * ((a.Cout + g.bch - 1) / g.bch);
    const double util = (double)a.M * a.Cout / ((double)tiles * g.bpx * g.bch);
    const int per_cu = (160 * 1024) / g.lds;
    const long long slots = 256LL * (per_cu < 1 ? 1 : per_cu);
    const long long waves = (tiles + slots - 1) / slots;
    const double fill = (double)tiles / (double)(waves * slots);
    const float score = (float)(g.factor * util * fill);
    if (score > best_score) { best_score = score; best = c; }
  }
  return best;
}

}  // namespace artsbir
