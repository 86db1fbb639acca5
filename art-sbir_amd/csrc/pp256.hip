// Ping-pong 256 x 256 implicit-GEMM tile for gfx950 (bf16 in, f32 accumulate):
// the convolution forward / data-gradient and dense NT GEMM kernel of the
// encoder for the MFMA-bound shapes — the 3x3 convs of the Bottleneck
// (models.py:198-221), the attention-pool projections (models.py:243-271) and
// the ViT projection data gradients (models.py:400-406).
//
// Schedule (cdna_hip_programming.md §5, "The 256² 8-phase template", rebuilt
// for a 32-k stage ring):
//  * 8 waves in two groups of 4 (waves 0-3: output channels 0-127 of the tile,
//    waves 4-7: channels 128-255; each wave 128 channels x 64 pixels).  Group 1
//    starts one s_barrier late, so at every barrier one group enters its MFMA
//    cluster while the other issues its LDS fragment reads and LDS-DMA stage
//    loads: the two waves that share a SIMD alternate between the MFMA pipe and
//    the memory pipes instead of waiting out the same latency together;
//  * a K-tile is 32 k (64-B LDS rows, chunk ^ ((row >> 2) & 2) on the DMA source);
//    each K-tile is two phases of 16 MFMAs per wave: phase a reads the pixel
//    fragments and the first four channel fragments, phase b the other four;
//  * four K-tile buffers (128 KB); the stage of K-tile t+3 is issued during
//    K-tile t (pixel half in phase a, weight half in phase b), so each half is
//    rewritten two phases after its last read, and one counted s_waitcnt vmcnt
//    per K-tile (never 0 in the steady state) retires K-tile t+1 one phase
//    before its first read: up to three K-tiles (96 KB) in flight per CU;
//  * the loop carries almost no vector work besides the MFMAs (a wave64 VALU
//    instruction holds the SIMD's issue port for 4 cycles, so every one of
//    them in the K loop comes out of the MFMA budget; the first version, with
//    a tap walk and offsets in VGPRs and 46 SGPR-spill reloads per K-tile, ran
//    at 0.85 PF with no memory traffic at all): the per-row part of each LDS-DMA
//    address is a VGPR fixed for the tile (for a 3x3 conv: per tap), the K-tile's
//    part is the instruction's SGPR soffset, the LDS destination an SGPR, and
//    the loop is unrolled by the four buffers so every LDS offset is an
//    immediate.
// The epilogue is pgemm's compile-time-specialised one (pg_epilogue_k), its
// operands read from global memory (no LDS staging), so every fused form of
// pgemm_kernel (forward BN statistics per segment, residual / average-unpool,
// bias + ReLU, QuickGELU gate, fused BN-backward kinds 1-3) is available.
#include <cstdio>
#include <cstdlib>

#include "pgemm_dev.h"

namespace artsbir {

namespace {

constexpr int PP_BPX = 256, PP_BCH = 256, PP_NW = 8, PP_KS = 32, PP_ROWB = 64, PP_RPI = 16;
constexpr int PP_HALF = 256 * PP_ROWB;  // one operand of one K-tile: 16 KB
constexpr int PP_BUF = 2 * PP_HALF;     // pixels | weights
constexpr int PP_NBUF = 4;

__device__ __forceinline__ void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// LDS-DMA of 16 B per lane to LDS address lds + 16 * lane (lds wave-uniform,
// in an SGPR) from buffer offset voff (VGPR) + soff (SGPR).  Out-of-range voff
// (>= the descriptor's size, e.g. 0x80000000) reads zeros.
__device__ __forceinline__ void pp_glds(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r), "s"(soff)
      : "memory");
}

}  // namespace

// TAPS: R x S > 1 (3x3 convolutions: the row offsets of a tile change with the
// tap); otherwise every K-tile of a tile reads the same rows at a growing k.
#ifndef PP_NOL
#define PP_NOL 0  // 1: normalize-on-load cost probe of a diagnostic build only (see pp_nol2)
#endif
// Cost probe for a consumer-side BatchNorm + ReLU (+ padded-tap mask) on the
// pixel fragments: relu(s * x + b) per input channel in f32, repacked to bf16,
// with coefficients read from LDS per K-tile.  Wrong results by design (the
// coefficients are scratch); only the kernel time is of interest.
__device__ __forceinline__ unsigned pp_nol2(unsigned w, float s0, float s1, float b0, float b1, bool keep) {
  float lo = __uint_as_float(w << 16), hi = __uint_as_float(w & 0xffff0000u);
  lo = fmaxf(fmaf(lo, s0, b0), 0.f);
  hi = fmaxf(fmaf(hi, s1, b1), 0.f);
  const unsigned r = (unsigned)__builtin_bit_cast(unsigned short, (bf16)lo) |
                     ((unsigned)__builtin_bit_cast(unsigned short, (bf16)hi) << 16);
  return keep ? r : 0u;
}

// X2 (1x1 only): the folded BatchNorm-backward data gradient — the reduction
// runs over x (k < C1) and then x2; the tile's BN segment selects the weights
// and the bias (artsbir_conv1x1_dgrad_fold)
template <int BK, bool TWO, bool TAPS, bool X2 = false>
__global__ void __launch_bounds__(512, 1) pp256_kernel(PgArgs a) {
  constexpr int NW = PP_NW, BCH = PP_BCH;
  constexpr int WTPX = 64, WTCH = 128, NTP = WTPX / 16, MTC = WTCH / 16;
  constexpr int IPX = 2, ICH = 2;  // DMA instructions per wave per K-tile half
  static_assert(IPX * NW * PP_RPI == PP_BPX && ICH * NW * PP_RPI == PP_BCH, "loader");
  __shared__ __attribute__((aligned(16))) char smem[PP_NBUF * PP_BUF + pg_red_bytes<BCH>()];
  float* red = reinterpret_cast<float*>(smem + PP_NBUF * PP_BUF);
  int* red_cnt = reinterpret_cast<int*>(smem + PP_NBUF * PP_BUF + 6 * BCH * 4);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int wpx = wid & 3, wch = wid >> 2;
  const int ntc = (a.Cout + BCH - 1) / BCH;
  const long long ntp = (a.M + PP_BPX - 1) / PP_BPX;
  // the N tiles of a pixel panel share an XCD (ARTSBIR_PG_DBG bit 4: dispatch order, a measurement)
  const long long tile = (a.dbg & 4) ? (long long)blockIdx.x : pg_xcd_remap(blockIdx.x, ntp * ntc);
  const long long bpx = (tile / ntc) * PP_BPX;
  const int bch = (int)(tile % ntc) * BCH;
  const int nk = a.K / PP_KS;  // K % 32 == 0 (pp256_launch)

  // ---- loader: this lane fills slot (lane & 3) of row (lane >> 2) of each
  // 16-row DMA instruction with k-chunk csrc = slot ^ ((row >> 2) & 2) (conflict-free
  // for the ds_read_b128 lane groups of MI355X_MICROARCH §LDS)
  const int lrow = lane >> 2, lslot = lane & 3;
  const int csrc = lslot ^ ((lrow >> 2) & 2);
  const int HoWo = a.Ho * a.Wo;
  const long long img0 = bpx / HoWo;
  // the pixel descriptor starts BIAS bytes before the tile's first image, so
  // the most negative row offset of a padded tap is still >= 0 (the per-row
  // part is the VGPR offset, which alone decides out-of-range)
  const int bias = (a.pad * (int)a.sH + a.pad * (int)a.sW) * 2;
  __amdgpu_buffer_rsrc_t xr =
      pg_rsrc(reinterpret_cast<const char*>(a.x) + pg_uniform(img0 * a.sN * 2 - bias),
              (a.x_elems - img0 * a.sN) * 2 + bias);
  const long long wseg0 = X2 && a.seg_m > 0 ? bpx / a.seg_m : 0;
  const __amdgpu_buffer_rsrc_t wr =
      pg_rsrc(reinterpret_cast<const char*>(a.w) + pg_uniform(wseg0 * a.w_sstride * 2), (long long)a.Cout * a.K * 2);
  int rowoff[IPX];
  unsigned rmask[IPX], vofs[IPX], woff[ICH];
  unsigned vofs2[X2 ? IPX : 1];  // X2: row offsets into the second operand
#pragma unroll
  for (int u = 0; u < IPX; ++u) {
    const int row = (u * NW + wid) * PP_RPI + lrow;
    const long long gm = bpx + row;
    const bool valid = gm < a.M;
    const long long gmc = valid ? gm : bpx;
    const long long img = gmc / HoWo;
    const int rem = (int)(gmc - img * HoWo);
    const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    rowoff[u] = (int)(((img - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * 2) + bias + csrc * 16;
    unsigned msk = 0;
    for (int r = 0; r < a.R; ++r)
      for (int s = 0; s < a.S; ++s) {
        const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
        msk |= (ok ? 1u : 0u) << (r * a.S + s);
      }
    rmask[u] = msk;
    vofs[u] = (msk & 1u) ? (unsigned)rowoff[u] : PG_OOB;
    if constexpr (X2)
      vofs2[u] = valid ? (unsigned)(((img - img0) * a.sN2 + (long long)oh * a.sH2 + (long long)ow * a.sW2) * 2 + csrc * 16)
                       : PG_OOB;
  }
  const __amdgpu_buffer_rsrc_t xr2 =
      X2 ? pg_rsrc(reinterpret_cast<const char*>(a.x2) + pg_uniform(img0 * a.sN2 * 2), (a.x2_elems - img0 * a.sN2) * 2)
         : xr;
  unsigned c1b = X2 ? (unsigned)a.C1 * 2u : 0u;  // byte offset of k = C1 in a row of x (switched once)
#pragma unroll
  for (int u = 0; u < ICH; ++u) {
    const int ch = bch + pg_perm((u * NW + wid) * PP_RPI + lrow);
    woff[u] = ch < a.Cout ? (unsigned)(ch * a.K * 2 + csrc * 16) : PG_OOB;
  }
  // K-tile parts of the addresses (SGPRs): pixel offset within the receptive
  // field (tap walk for TAPS), weight offset; LDS destination of this wave
  const int aC = a.C, aS = a.S;
  const int stepS = (int)a.sW * 2 - aC * 2, stepR = (int)a.sH * 2 - aS * (int)a.sW * 2;
  unsigned px_soff = 0, w_soff = 0;
  int u_ci = 0, u_s = 0, u_rs = 0;
  const unsigned lds0 = (unsigned)(unsigned long long)(pg_lds_t)smem + (unsigned)wid * 1024u;
  auto issue_px = [&](int slot) {
#pragma unroll
    for (int u = 0; u < IPX; ++u) pp_glds(xr, lds0 + slot * PP_BUF + u * NW * 1024, vofs[u], px_soff);
    px_soff += PP_KS * 2;
    if constexpr (X2) {
      if (px_soff == c1b) {  // past the first operand's C1 channels: the second one from its k = 0
        xr = xr2;
        px_soff = 0;
        c1b = 0xffffffffu;  // once: the second operand may be wider than the first
#pragma unroll
        for (int u = 0; u < IPX; ++u) vofs[u] = vofs2[u];
      }
    }
    if constexpr (TAPS) {
      u_ci += PP_KS;
      if (u_ci == aC) {  // next tap: its row validity
        u_ci = 0;
        px_soff += stepS;
        ++u_rs;
        if (++u_s == aS) { u_s = 0; px_soff += stepR; }
#pragma unroll
        for (int u = 0; u < IPX; ++u) vofs[u] = ((rmask[u] >> u_rs) & 1u) ? (unsigned)rowoff[u] : PG_OOB;
      }
    }
  };
  auto issue_ch = [&](int slot) {
#pragma unroll
    for (int u = 0; u < ICH; ++u) pp_glds(wr, lds0 + slot * PP_BUF + PP_HALF + u * NW * 1024, woff[u], w_soff);
    w_soff += PP_ROWB;
  };

  const bool sums = (BK != 0) || a.stats != nullptr;
  if (sums) {
    for (int i = tid; i < 6 * BCH; i += 64 * NW) red[i] = 0.f;
    if (tid == 0) *red_cnt = 0;
  }

  f32x4 acc[MTC][NTP];
#pragma unroll
  for (int i = 0; i < MTC; ++i)
#pragma unroll
    for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0..2 in flight, K-tile 0 retired
  issue_px(0);
  issue_ch(0);
  if (nk > 1) { issue_px(1); issue_ch(1); }
  if (nk > 2) { issue_px(2); issue_ch(2); }
  if (nk > 2) vm_wait<8>();
  else if (nk > 1) vm_wait<4>();
  else vm_wait<0>();
  pp_barrier();
  if (grp == 1) pp_barrier();  // the stagger: group 1 runs one barrier behind

  const int fr = lane & 15, fq = lane >> 4;
  const int so = (fq ^ ((fr >> 2) & 2)) << 4;
  const char* bbase = smem + (wpx * WTPX + fr) * PP_ROWB + so;            // pixel fragment j: + j * 16 rows
  const char* abase = smem + PP_HALF + (wch * WTCH + fr) * PP_ROWB + so;  // channel fragment i: + i * 16 rows
  uint4 bv[NTP], af[MTC];
#if PP_NOL
  const char* cbase = reinterpret_cast<const char*>(red) + fq * 32;
  unsigned nol_m = (unsigned)lane * 0x9e3779b9u;
  asm volatile("" : "+v"(nol_m));  // opaque per-lane row-validity bits
#endif
#ifndef PP_PFN
#define PP_PFN 1  // BK 0: the next channel pair's residual / gate operands loaded ahead (pg_epilogue_k PFN)
#endif
  // (loading pair 0's operands in the last K-tiles as well, under the tail's
  // counted waits, was slower: gate GEMM 2.45 -> 2.58 ms, profiles/r6_pfn.txt)
  constexpr bool PFN = PP_PFN && BK == 0 && !X2 && !TAPS;  // (3x3 convs: no residual operand)
  // one K-tile in buffer SL (compile-time: every LDS offset an immediate)
  auto ktile = [&](int s, auto slc) {
    constexpr int SL = decltype(slc)::value;
    const char* bb = bbase + SL * PP_BUF;
    const char* ab = abase + SL * PP_BUF;
    // ---- phase a: pixel fragments + channel fragments 0..3; pixel half of K-tile s+3
#ifndef PP_ABL
#define PP_ABL 0  // timing ablations of a diagnostic build only (1: no stage loads in the loop, 2: no fragment reads)
#endif
    if (!(PP_ABL & 1) && s + 3 < nk) issue_px((SL + 3) & 3);
    if (!(PP_ABL & 2) || s < 1) {
#pragma unroll
      for (int j = 0; j < NTP; ++j) bv[j] = *reinterpret_cast<const uint4*>(bb + j * 16 * PP_ROWB);
#pragma unroll
      for (int i = 0; i < MTC / 2; ++i) af[i] = *reinterpret_cast<const uint4*>(ab + i * 16 * PP_ROWB);
    }
#if PP_NOL
    const f32x4 cs0 = *reinterpret_cast<const f32x4*>(cbase), cs1 = *reinterpret_cast<const f32x4*>(cbase + 16);
    const f32x4 cb0 = *reinterpret_cast<const f32x4*>(cbase + 128), cb1 = *reinterpret_cast<const f32x4*>(cbase + 144);
#endif
    pp_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#if PP_NOL
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const bool keep = !TAPS || ((nol_m >> (j + 4 * SL)) & 1u);
      bv[j].x = pp_nol2(bv[j].x, cs0[0], cs0[1], cb0[0], cb0[1], keep);
      bv[j].y = pp_nol2(bv[j].y, cs0[2], cs0[3], cb0[2], cb0[3], keep);
      bv[j].z = pp_nol2(bv[j].z, cs1[0], cs1[1], cb1[0], cb1[1], keep);
      bv[j].w = pp_nol2(bv[j].w, cs1[2], cs1[3], cb1[2], cb1[3], keep);
    }
#endif
    PG_PRIO_ON();
#pragma unroll
    for (int i = 0; i < MTC / 2; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                            *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j], 0, 0, 0);
    PG_PRIO_OFF();
    pp_barrier();
    // ---- phase b: channel fragments 4..7; weight half of K-tile s+3; K-tile s+1 retired
    if (s + 3 < nk) {
      if (!(PP_ABL & 1)) issue_ch((SL + 3) & 3);
      vm_wait<8>();
    } else if (s + 2 < nk) {
      vm_wait<4>();
    } else if (s + 1 < nk) {
      vm_wait<0>();
    }
    if (!(PP_ABL & 2) || s < 1) {
#pragma unroll
      for (int i = MTC / 2; i < MTC; ++i) af[i] = *reinterpret_cast<const uint4*>(ab + i * 16 * PP_ROWB);
    }
    pp_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    PG_PRIO_ON();
#pragma unroll
    for (int i = MTC / 2; i < MTC; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                            *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j], 0, 0, 0);
    PG_PRIO_OFF();
    if (!(s == nk - 1 && grp == 1)) pp_barrier();  // group 1 drops its last one: equal barrier counts
  };
  for (int s = 0; s < nk; s += 4) {
    ktile(s, std::integral_constant<int, 0>{});
    if (s + 1 < nk) ktile(s + 1, std::integral_constant<int, 1>{});
    if (s + 2 < nk) ktile(s + 2, std::integral_constant<int, 2>{});
    if (s + 3 < nk) ktile(s + 3, std::integral_constant<int, 3>{});
  }

  const long long seg0 = a.seg_m > 0 ? bpx / a.seg_m : 0;
  EpiStage sgg{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, seg0};
#ifndef PP_EJB
#define PP_EJB 4  // pixel tiles whose epilogue operands are loaded together (2: 1-4 % slower fused dgrads, tools/gpu/r4_ej.sh)
#endif
  pg_epilogue_k<BK, TWO, false, false, false, BCH, MTC, NTP, WTPX, WTCH, false, PP_EJB, true, X2, false, PFN>(
      a, acc, bpx, bch, wpx, wch, fr, fq, red, sgg);
  if (sums) stats_flush<BCH>(red, red_cnt, NW - 1, a, bch, (int)(blockIdx.x % ARTSBIR_NSLOT), lane, bpx, PP_BPX);
}

// Candidate 22: C % 32 == 0 (uniform taps), every epilogue of pgemm_launch_cfg
// except the LDS-staged BN-backward forms.
bool pp256_launch(const PgArgs& a, bool persistent, hipStream_t st) {
  if (persistent) return false;  // candidate 23 (persistent form) retired: no gain over one tile per workgroup
  if (a.C % 32 != 0 || a.Cout % 32 != 0 || a.M <= 0) return false;
  if (a.R * a.S > 32 || a.K != a.R * a.S * a.C) return false;
  if ((long long)a.Cout * a.K * 2 > 0x7fffffffLL) return false;
  const long long HoWo = (long long)a.Ho * a.Wo;
  if (((256 + HoWo - 1) / HoWo + 2) * a.sN * 2 + 2LL * (a.pad * a.sH + a.pad * a.sW) > 0x7fffffffLL) return false;
  if (a.M > (1LL << 40)) return false;
  if (a.seg_m > 0 && (a.seg_m % 64 != 0 || a.seg_m < 256 || a.M % a.seg_m != 0)) return false;
  if (a.x2 || a.w_sstride) {  // the folded BatchNorm-backward data gradient (plain, ACT or RES epilogue + bias)
    if (!a.x2 || !a.bias || !pg_fold_ok(a, PP_BPX, PP_KS) || a.relu || a.stats || a.res_mode == 3) return false;
    if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
    if ((a.bnb == 2 || a.bnb == 3) && !a.res_mode) return false;
    if (a.bnb && a.Cout % 8 != 0) return false;
    if (((256 + HoWo - 1) / HoWo + 2) * a.sN2 * 2 > 0x7fffffffLL) return false;
    const long long T = ((a.M + PP_BPX - 1) / PP_BPX) * ((a.Cout + PP_BCH - 1) / PP_BCH);
    if (T > 0x7fffffffLL) return false;
    const dim3 g((unsigned)T), b(512);
    if (a.bnb == 1) hipLaunchKernelGGL((pp256_kernel<1, false, false, true>), g, b, 0, st, a);
    else if (a.bnb == 2 && a.bnb_nt == 2) hipLaunchKernelGGL((pp256_kernel<2, true, false, true>), g, b, 0, st, a);
    else if (a.bnb == 2) hipLaunchKernelGGL((pp256_kernel<2, false, false, true>), g, b, 0, st, a);
    else if (a.bnb == 3 && a.bnb_nt == 2) hipLaunchKernelGGL((pp256_kernel<3, true, false, true>), g, b, 0, st, a);
    else if (a.bnb == 3) hipLaunchKernelGGL((pp256_kernel<3, false, false, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((pp256_kernel<0, false, false, true>), g, b, 0, st, a);
    set_last_kernel(a.bnb ? "pp256_kernel<bnb,fold>" : "pp256_kernel<fold>");
    return true;
  }
  const bool act = a.bias != nullptr || a.relu != 0;
  if (act && (a.stats || a.bnb)) return false;
  if (a.bnb && (a.stats || a.Cout % 8 != 0)) return false;
  if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
  if ((a.bnb == 2 || a.bnb == 3) && !a.res_mode) return false;
  if (a.res_mode == 3 && (a.bnb || a.R * a.S != 1)) return false;
  const long long T = ((a.M + PP_BPX - 1) / PP_BPX) * ((a.Cout + PP_BCH - 1) / PP_BCH);
  if (T > 0x7fffffffLL) return false;
  const dim3 g((unsigned)T), b(512);
#define PP_GO(BKV, TWOV)                                                              \
  do {                                                                                \
    if (a.R * a.S > 1) hipLaunchKernelGGL((pp256_kernel<BKV, TWOV, true>), g, b, 0, st, a); \
    else hipLaunchKernelGGL((pp256_kernel<BKV, TWOV, false>), g, b, 0, st, a);       \
  } while (0)
  if (a.bnb == 1) PP_GO(1, false);
  else if (a.bnb == 2 && a.bnb_nt == 2) PP_GO(2, true);
  else if (a.bnb == 2) PP_GO(2, false);
  else if (a.bnb == 3 && a.bnb_nt == 2) PP_GO(3, true);
  else if (a.bnb == 3) PP_GO(3, false);
  else PP_GO(0, false);
#undef PP_GO
  set_last_kernel(a.bnb ? "pp256_kernel<bnb>" : "pp256_kernel");
  return true;
}

}  // namespace artsbir
