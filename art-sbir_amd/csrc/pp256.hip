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
//  * persistent form (G > 0): a workgroup walks a contiguous range of output
//    tiles of its XCD (tiles that share an operand panel run at the same time
//    on one L2), and the stage stream runs across tile boundaries: the next
//    tile's first three K-tiles load while this tile's epilogue stores drain.
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

__device__ __forceinline__ void pp_barrier(bool skip = false) {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (!skip) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

// retire all but the newest 4 * n LDS-DMA instructions of this wave (n = K-tiles
// left in flight; a K-tile is 2 pixel + 2 weight instructions per wave)
__device__ __forceinline__ void pp_wait(int n) {
  if (n >= 2) vm_wait<8>();
  else if (n == 1) vm_wait<4>();
  else vm_wait<0>();
}

}  // namespace

#ifndef PP_STAMP
#define PP_STAMP 0
#endif
// PP_STAMP=1: diagnostic build (never the product library) that sums the cycles
// of each segment of a K-tile per wave (cdna_hip_programming.md §7 stamps) into
// ts[block][wave][16]; read its shares, not its run time
#if PP_STAMP
#define PP_TS(k)                                                                            \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long t_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    tsum[k] += t_ - t_last;                                                                 \
    t_last = t_;                                                                            \
  } while (0)
#else
#define PP_TS(k) \
  do {           \
  } while (0)
#endif

template <int BK, bool TWO>
__global__ void __launch_bounds__(512, 1) pp256_kernel(PgArgs a, int G
#if PP_STAMP
                                                      , unsigned long long* ts
#endif
) {
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
  const int ntp = (int)((a.M + PP_BPX - 1) / PP_BPX);
  const int T = ntp * ntc;  // < 2^31 (pp256_launch)

  // ---- the tiles of this workgroup
  int t_first, t_step, ntl;
  if (G == 0) {
    t_first = (int)pg_xcd_remap(blockIdx.x, T);
    t_step = 0;
    ntl = 1;
  } else {  // XCD x = blockIdx % 8 owns tiles [x T / 8, (x + 1) T / 8); its G / 8 workgroups interleave
    const int x = (int)(blockIdx.x & 7), l = (int)(blockIdx.x >> 3), per = G >> 3;
    const int lo = (int)((long long)x * T / 8), hi = (int)((long long)(x + 1) * T / 8);
    t_first = lo + l;
    t_step = per;
    ntl = t_first < hi ? (hi - t_first + per - 1) / per : 0;
  }
  if (ntl == 0) return;
  // loop-invariant scalars, copied once: inside the loop an a.field read is a
  // kernarg load (the asm "memory" clobbers keep it from being hoisted) with an
  // lgkmcnt wait that also drains the LDS fragment reads
  const int aC = a.C, aS = a.S;
  const int nk = (a.K + PP_KS - 1) / PP_KS;
  const int S = ntl * nk;  // K-tiles of the whole stream
  const int stepS = (int)a.sW * 2 - aC * 2;         // tap walk: channel chunk wraps, next column tap
  const int stepR = (int)a.sH * 2 - aS * (int)a.sW * 2;  // column taps wrap, next row tap

  const int HoWo = a.Ho * a.Wo;
  const __amdgpu_buffer_rsrc_t wr = pg_rsrc(a.w, (long long)a.Cout * a.K * 2);

  // ---- loader: this lane fills slot (lane & 3) of row (lane >> 2) of each
  // 16-row DMA instruction with k-chunk csrc = slot ^ ((row >> 2) & 2) (conflict-free
  // for the ds_read_b128 lane groups of MI355X_MICROARCH §LDS)
  const int lrow = lane >> 2, lslot = lane & 3;
  const int csrc = lslot ^ ((lrow >> 2) & 2);
  int rowoff[IPX];
  unsigned rmask[IPX];
  unsigned woff[ICH];
  __amdgpu_buffer_rsrc_t xr = wr;
  int l_tile = 0, l_kt = 0;  // position of the next stage to issue
  // its tap walk (C % 32 == 0: a K-tile never straddles taps): byte offset of the
  // K-tile in the receptive field, channel offset within the tap, tap index r*S+s
  int u_off = 0, u_ci = 0, u_s = 0, u_rs = 0, w_off = 0;
  auto decode = [&](int tile) {
    const long long bpx = (long long)(tile / ntc) * PP_BPX;
    const int bch = (tile % ntc) * BCH;
    const long long img0 = bpx / HoWo;
    xr = pg_rsrc(reinterpret_cast<const bf16*>(a.x) + pg_uniform(img0 * a.sN), (a.x_elems - img0 * a.sN) * 2);
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
      rowoff[u] = (int)(((img - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * 2) + csrc * 16;
      unsigned msk = 0;
      for (int r = 0; r < a.R; ++r)
        for (int s = 0; s < a.S; ++s) {
          const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
          msk |= (ok ? 1u : 0u) << (r * a.S + s);
        }
      rmask[u] = msk;
    }
#pragma unroll
    for (int u = 0; u < ICH; ++u) {
      const int ch = bch + pg_perm((u * NW + wid) * PP_RPI + lrow);
      woff[u] = ch < a.Cout ? (unsigned)(ch * a.K * 2 + csrc * 16) : PG_OOB;
    }
  };
  // pixel half of the next stage (advances the tap walk); decodes a new tile first
  auto issue_px = [&](int s) {
    if (l_kt == 0) decode(t_first + l_tile * t_step);
    char* pxs = smem + (s & 3) * PP_BUF;
    const int rs = u_rs, toff = u_off;
    u_off += PP_KS * 2;
    u_ci += PP_KS;
    if (u_ci == aC) {
      u_ci = 0;
      u_off += stepS;
      ++u_rs;
      if (++u_s == aS) { u_s = 0; u_off += stepR; }
    }
#pragma unroll
    for (int u = 0; u < IPX; ++u) {
      const bool ok = (rmask[u] >> rs) & 1u;
      glds16(xr, pxs + (u * NW + wid) * 1024, ok ? (unsigned)(rowoff[u] + toff) : PG_OOB);
    }
  };
  // weight half of the same stage (K % 32 == 0: no k tail); moves the loader to the next K-tile
  auto issue_ch = [&](int s) {
    char* chs = smem + (s & 3) * PP_BUF + PP_HALF;
#pragma unroll
    for (int u = 0; u < ICH; ++u)
      glds16(wr, chs + (u * NW + wid) * 1024, woff[u] != PG_OOB ? woff[u] + w_off : PG_OOB);
    w_off += PP_ROWB;
    if (++l_kt == nk) {
      l_kt = 0;
      ++l_tile;
      u_off = 0; u_ci = 0; u_s = 0; u_rs = 0; w_off = 0;
    }
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
  const int npro = S < 3 ? S : 3;
  for (int s = 0; s < npro; ++s) {
    issue_px(s);
    issue_ch(s);
  }
  pp_wait(npro - 1);
  pp_barrier();
  if (grp == 1) pp_barrier();  // the stagger: group 1 runs one barrier behind

  const int fr = lane & 15, fq = lane >> 4;
  const int so = (fq ^ ((fr >> 2) & 2)) << 4;
  const int brow = (wpx * WTPX + fr) * PP_ROWB + so;            // pixel fragment j: + j * 16 rows
  const int arow = PP_HALF + (wch * WTCH + fr) * PP_ROWB + so;  // channel fragment i: + i * 16 rows
  int kt = 0, n = 0;
  bool after_epi = false;
  // timing ablations (ARTSBIR_PG_DBG, wrong results): 8 no stage loads in the
  // loop, 16 no fragment reads, 32 no barriers in the loop
  const int dbg = a.dbg;
  uint4 bv[NTP], af[MTC];  // fragments (declared outside the loop: the ablations reuse stale ones)
#if PP_STAMP
  unsigned long long tsum[16] = {}, t_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_last)::"memory");
#endif
  for (int s = 0; s < S; ++s) {
    const char* buf = smem + (s & 3) * PP_BUF;
    PP_TS(0);  // loop overhead / previous tail
    // ---- phase a: pixel fragments + channel fragments 0..3
    if (s + 3 < S && !(dbg & 8)) issue_px(s + 3);
    PP_TS(1);  // pixel stage issue
    if (!(dbg & 16) || s < 2) {
#pragma unroll
      for (int j = 0; j < NTP; ++j) bv[j] = *reinterpret_cast<const uint4*>(buf + brow + j * 16 * PP_ROWB);
#pragma unroll
      for (int i = 0; i < MTC / 2; ++i) af[i] = *reinterpret_cast<const uint4*>(buf + arow + i * 16 * PP_ROWB);
    }
    PP_TS(2);  // fragment reads a (issue + latency in this build)
    pp_barrier(dbg & 32);
    PP_TS(3);  // barrier 1
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    PG_PRIO_ON();
#pragma unroll
    for (int i = 0; i < MTC / 2; ++i)
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                            *reinterpret_cast<const bf16x8*>(&bv[j]), acc[i][j], 0, 0, 0);
    PG_PRIO_OFF();
    PP_TS(4);  // MFMA issue a
    pp_barrier(dbg & 32);
    PP_TS(5);  // barrier 2
    // ---- phase b: channel fragments 4..7; K-tile s+1 retired for the next phase a
    if (s + 3 < S && !(dbg & 8)) issue_ch(s + 3);
    PP_TS(6);  // weight stage issue
    if (s + 1 < S) {
      int left = (s + 3 < S ? s + 3 : S - 1) - (s + 1);
      if (after_epi && left > 1) left = 1;  // the epilogue's stores sit between the stages: retire them too
      pp_wait(left);
    }
    after_epi = false;
    PP_TS(7);  // vmcnt wait for K-tile s+1
    if (!(dbg & 16) || s < 2) {
#pragma unroll
      for (int i = MTC / 2; i < MTC; ++i) af[i] = *reinterpret_cast<const uint4*>(buf + arow + i * 16 * PP_ROWB);
    }
    PP_TS(8);  // fragment reads b
    pp_barrier(dbg & 32);
    PP_TS(9);  // barrier 3
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
    PP_TS(10);  // MFMA issue b
    if (!(s == S - 1 && grp == 1)) pp_barrier(dbg & 32);  // group 1 drops its last one: equal barrier counts
    PP_TS(11);  // barrier 4
    if (++kt == nk) {
      kt = 0;
      const int tile = t_first + n * t_step;
      const long long bpx = (long long)(tile / ntc) * PP_BPX;
      const int bch = (tile % ntc) * BCH;
      const long long seg0 = a.seg_m > 0 ? bpx / a.seg_m : 0;
      EpiStage sgg{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, seg0};
      pg_epilogue_k<BK, TWO, false, false, false, BCH, MTC, NTP, WTPX, WTCH, false, 2, true>(a, acc, bpx, bch, wpx, wch,
                                                                                            fr, fq, red, sgg);
      if (sums) stats_flush<BCH>(red, red_cnt, (n + 1) * NW - 1, a, bch, (int)(blockIdx.x % ARTSBIR_NSLOT), lane, bpx,
                                 PP_BPX);
      ++n;
      // the compiler's own count of the epilogue's global loads: tell it they are
      // retired (vmcnt 0, the other counters at their maximum), or its waitcnt pass
      // carries them round the loop and drains vmcnt(0) before every K-tile's
      // first fragment read, i.e. the whole LDS-DMA pipeline
      __builtin_amdgcn_s_waitcnt(0x0f70);
#pragma unroll
      for (int i = 0; i < MTC; ++i)
#pragma unroll
        for (int j = 0; j < NTP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      after_epi = true;
      PP_TS(12);  // epilogue
    }
  }
#if PP_STAMP
  if (lane == 0) {
    unsigned long long* o = ts + ((long long)blockIdx.x * NW + wid) * 16;
    for (int k = 0; k < 13; ++k) o[k] = tsum[k];
    o[13] = S;
  }
#endif
}

// Candidate 22 (one tile per workgroup) / 23 (persistent, 256 workgroups):
// C % 32 == 0 (uniform taps), every epilogue of pgemm_launch_cfg except the
// LDS-staged BN-backward forms.
bool pp256_launch(const PgArgs& a, bool persistent, hipStream_t st) {
  if (a.C % 32 != 0 || a.Cout % 32 != 0 || a.M <= 0) return false;
  if (a.R * a.S > 32 || a.K != a.R * a.S * a.C) return false;
  if ((long long)a.Cout * a.K * 2 > 0x7fffffffLL) return false;
  const long long HoWo = (long long)a.Ho * a.Wo;
  if (((256 + HoWo - 1) / HoWo + 2) * a.sN * 2 > 0x7fffffffLL) return false;
  if (a.M > (1LL << 40)) return false;
  if (a.seg_m > 0 && (a.seg_m % 64 != 0 || a.seg_m < 256 || a.M % a.seg_m != 0)) return false;
  const bool act = a.bias != nullptr || a.relu != 0;
  if (act && (a.stats || a.bnb)) return false;
  if (a.bnb && (a.stats || a.Cout % 8 != 0)) return false;
  if (a.bnb == 1 && (a.bnb_nt != 1 || a.res_mode)) return false;
  if ((a.bnb == 2 || a.bnb == 3) && !a.res_mode) return false;
  if (a.res_mode == 3 && (a.bnb || a.R * a.S != 1)) return false;
  const long long T = ((a.M + PP_BPX - 1) / PP_BPX) * ((a.Cout + PP_BCH - 1) / PP_BCH);
  if (T > 0x3fffffffLL) return false;
  int G = 0;
  unsigned grid = (unsigned)T;
  if (persistent) {
    // ARTSBIR_PP_GRID (tests): a smaller persistent grid (multiple of 8), so that
    // small shapes also walk several tiles per workgroup
    const char* eg = getenv("ARTSBIR_PP_GRID");
    G = eg ? atoi(eg) : 256;
    if (G < 8 || G % 8 || G > 4096) return false;
    if (!eg && T < 2LL * G) return false;  // fewer than two tiles per workgroup: the one-tile form
    grid = (unsigned)G;
  }
  const dim3 g(grid), b(512);
#if PP_STAMP
  unsigned long long* ts = reinterpret_cast<unsigned long long*>(strtoull(getenv("ARTSBIR_PP_TS"), nullptr, 0));
  if (!a.bnb) hipLaunchKernelGGL((pp256_kernel<0, false>), g, b, 0, st, a, G, ts);
  set_last_kernel(persistent ? "pp256_kernel<persistent,stamp>" : "pp256_kernel<stamp>");
  return true;
#else
  if (a.bnb == 1) hipLaunchKernelGGL((pp256_kernel<1, false>), g, b, 0, st, a, G);
  else if (a.bnb == 2 && a.bnb_nt == 2) hipLaunchKernelGGL((pp256_kernel<2, true>), g, b, 0, st, a, G);
  else if (a.bnb == 2) hipLaunchKernelGGL((pp256_kernel<2, false>), g, b, 0, st, a, G);
  else if (a.bnb == 3 && a.bnb_nt == 2) hipLaunchKernelGGL((pp256_kernel<3, true>), g, b, 0, st, a, G);
  else if (a.bnb == 3) hipLaunchKernelGGL((pp256_kernel<3, false>), g, b, 0, st, a, G);
  else hipLaunchKernelGGL((pp256_kernel<0, false>), g, b, 0, st, a, G);
  static const char* names[2][2] = {{"pp256_kernel", "pp256_kernel<bnb>"},
                                    {"pp256_kernel<persistent>", "pp256_kernel<bnb,persistent>"}};
  set_last_kernel(names[persistent ? 1 : 0][a.bnb ? 1 : 0]);
  return true;
#endif
}

}  // namespace artsbir
