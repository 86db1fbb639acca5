// Pipelined weight-gradient GEMM (bf16 in, f32 accumulate, f32 atomics out)
// for gfx950: dW[co][k] += sum_m dY[m][co] * Xcol[m][k]  — the backward of
// every nn.Conv2d / nn.Linear weight on the encoder path
// (models.py:198-221, 310-316; attention-pool projections models.py:243-246).
//
// Both operands are reduction-major in HBM (rows m = output pixels).  They are
// staged by LDS-DMA in their natural row-major form — dY rows of co, Xcol rows
// of k (implicit im2col with per-row padding masks) — and the MFMA fragments,
// which need 8 consecutive m per lane, are read with the gfx950 transposing
// LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10): no register
// transposes.  LDS image: row-major tile rows with the 16-B chunks of row m
// XOR-swizzled by pw_f<width>(m) (conflict-free transposed reads at every tile
// width; guide T10); the XOR is applied to the per-lane LDS-DMA source address.  An NSTAGE ring with counted
// vmcnt keeps NSTAGE-2 stages in flight across the per-K-step barrier; the
// reduction over m is split over workgroups (f32 atomics into dW).
#include <cstdlib>

#include "common.h"
#include "pgemm.h"

namespace artsbir {

#define PW_OOB 0x80000000u
typedef __attribute__((address_space(3))) void* pw_lds_t;
typedef short pw_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) pw_v4s* pw_lds_v4s;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pw_rsrc(const void* base, long long bytes) {
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void pw_glds16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(pw_lds_t)lds);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(r)
      : "memory");
}

template <int N>
__device__ __forceinline__ void pw_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int LPS, int NSTAGE>
__device__ __forceinline__ void pw_wait_stages(int ahead) {
  if constexpr (NSTAGE >= 4) {
    if (ahead >= 2) { pw_vm_wait<2 * LPS>(); return; }
  }
  if constexpr (NSTAGE >= 3) {
    if (ahead >= 1) { pw_vm_wait<LPS>(); return; }
  }
  pw_vm_wait<0>();
}

// XOR swizzle of the 16-B chunks of tile row m (TW elements wide).  A
// transposing read takes, per 32-lane half, 2 adjacent chunks of rows
// {m0..m0+3, m0+8..m0+11} (m0 = 0 or 4 mod 16); the swizzle spreads those 16
// chunks over the 16 bank groups of a 256-B LDS row: conflict-free for every
// tile width (rows of 256 B and more: chunk ^ f; 128-B rows fill half a bank
// row each, 64-B rows a quarter)
template <int TW>
__device__ __forceinline__ int pw_f(int m) {
  if constexpr (TW >= 128) return ((m & 3) << 2) | ((m >> 2) & 3);
  else if constexpr (TW == 64) return (((m >> 1) & 1) << 1) | (((m >> 3) & 1) << 2);
  else return ((m >> 3) & 1) << 1;
}

// byte offset in a tile image of element (m, c) of a tile TW elements wide
template <int TW>
__device__ __forceinline__ int pw_off(int m, int c) {
  return (m * TW + (((c >> 3) ^ pw_f<TW>(m)) << 3) + (c & 7)) * 2;
}

// the tile element (m, first column) whose 16-B chunk LDS-DMA slot (pr, slot)
// of the image holds (the inverse of pw_off: XOR is an involution)
template <int TW>
__device__ __forceinline__ int pw_src(int pr, int slot) {
  const int f0 = pr * 128 + slot * 8;
  const int m = f0 / TW, ch = (f0 % TW) >> 3;
  return m * TW + ((ch ^ pw_f<TW>(m)) << 3);
}

// 4 consecutive-m x 16-column block for the transposing read: lane t = 4q + p
// of a 16-lane group supplies row m0 + q, columns c0 + 4p .. c0 + 4p + 3
template <int TW>
__device__ __forceinline__ pw_v4s pw_tr(const char* tile, int m0, int c0, int t) {
  const char* p = tile + pw_off<TW>(m0 + (t >> 2), c0 + 4 * (t & 3));
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_v4s)(pw_lds_t)p);
}

__device__ __forceinline__ long long pw_xcd_remap(long long bid, long long nwg) {
  if (nwg < 8) return bid;
  const long long q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <int BCO, int BKK, int WCO, int WKK, int NSTAGE, bool DENSE>
__global__ void __launch_bounds__(64 * WCO * WKK) pwgrad_kernel(PwArgs a) {
  constexpr int NW = WCO * WKK;
  constexpr int BM = 64;  // m rows per stage
  constexpr int AB = BM * BCO * 2, BB = BM * BKK * 2, STAGE = AB + BB;
  constexpr int IA = AB / 1024, IB = BB / 1024;  // 1-KB LDS-DMA instructions per operand per stage
  static_assert(IA % NW == 0 || NW % IA == 0, "A loader split");
  static_assert(IB % NW == 0, "B loader split");
  constexpr int LA = IA >= NW ? IA / NW : 1;     // A instructions per wave (waves >= IA issue none)
  constexpr int LB = IB / NW;
  constexpr int WTCO = BCO / WCO, WTK = BKK / WKK;
  constexpr int MT = WTCO / 16, NT = WTK / 16;
  constexpr int LPS_HI = LA + LB, LPS_LO = (IA >= NW ? LA : 0) + LB;
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntco = (a.Cout + BCO - 1) / BCO, ntk = (a.K + BKK - 1) / BKK;
  const int ntiles = ntco * ntk;
  const long long nwg = (long long)gridDim.x;
  const long long lid = pw_xcd_remap(blockIdx.x, nwg);
  const long long split = lid / ntiles;
  const int tile = (int)(lid % ntiles);
  const int co0 = (tile / ntk) * BCO, k0 = (tile % ntk) * BKK;
  const long long m_beg = split * a.m_per_split;
  long long m_end = m_beg + a.m_per_split;
  if (m_end > a.M) m_end = a.M;
  const int nk = (int)((m_end - m_beg + BM - 1) / BM);

  // dY in two parts along Cout (a.dy2): this tile's rows come from one of them
  const bool s2 = DENSE && a.dy2 != nullptr && co0 >= a.Cout1;
  const bf16* dyp = reinterpret_cast<const bf16*>(s2 ? a.dy2 : a.dy);
  const long long ldd = s2 ? a.ldd2 : a.ldd;
  const int cb = s2 ? co0 - a.Cout1 : co0;                            // first dY column of the tile
  const int colim = (DENSE && a.dy2) ? (s2 ? a.Cout - a.Cout1 : a.Cout1) : a.Cout;
  float* const dwp = s2 ? a.dw2 : a.dw;
  const __amdgpu_buffer_rsrc_t dr = pw_rsrc(dyp + m_beg * ldd, ((s2 ? a.dy2_elems : a.dy_elems) - m_beg * ldd) * 2);
  const int HoWo = a.Ho * a.Wo;
  const long long img_beg = DENSE ? 0 : m_beg / HoWo;
  const __amdgpu_buffer_rsrc_t xr =
      DENSE ? pw_rsrc(reinterpret_cast<const bf16*>(a.x) + m_beg * a.ldx, (a.x_elems - m_beg * a.ldx) * 2)
            : pw_rsrc(reinterpret_cast<const bf16*>(a.x) + img_beg * a.sN, (a.x_elems - img_beg * a.sN) * 2);

  // ---- loader decode (fixed per lane): for each instruction, the tile
  // element (m_local, c) whose 16-B chunk this lane moves
  const int lpr = lane >> 4, lslot = lane & 15;
  bool a_on[LA];
  int a_m[LA];
  unsigned a_col[LA];  // byte offset of the co columns, PW_OOB if out of range
#pragma unroll
  for (int u = 0; u < LA; ++u) {
    const int g = u * NW + wid;
    a_on[u] = g < IA;
    const int pr = g * 4 + lpr;
    const int f = pw_src<BCO>(pr, lslot);
    a_m[u] = f / BCO;
    const int co = cb + f % BCO;
    a_col[u] = co < colim ? (unsigned)(co * 2) : PW_OOB;
  }
  int b_m[LB];
  unsigned b_tap[LB];  // DENSE: byte offset of the k columns; conv: ci * 2
  int b_r[LB], b_s[LB];
  int b_p[LB];  // conv: pixel index of this instruction's row at K-step 0, relative to image img_beg
#pragma unroll
  for (int u = 0; u < LB; ++u) {
    const int g = u * NW + wid;
    const int pr = g * 4 + lpr;
    const int f = pw_src<BKK>(pr, lslot);
    b_m[u] = f / BKK;
    const int k = k0 + f % BKK;
    if (k >= a.K) {
      b_tap[u] = PW_OOB;
      b_r[u] = 0; b_s[u] = 0;
    } else if (DENSE) {
      b_tap[u] = (unsigned)(k * 2);
      b_r[u] = 0; b_s[u] = 0;
    } else {
      const int rs = k / a.C, ci = k - (k / a.C) * a.C;
      b_r[u] = rs / a.S;
      b_s[u] = rs - b_r[u] * a.S;
      b_tap[u] = (unsigned)(ci * 2);  // the tap (r, s) enters through ih, iw
    }
    b_p[u] = DENSE ? 0 : (int)(m_beg - img_beg * HoWo) + b_m[u];
  }
  const bool lps_hi = a_on[0];
  const float inv_howo = 1.0f / (float)HoWo, inv_wo = 1.0f / (float)a.Wo;

  auto issue = [&](int kt, int buf) {
    char* as = smem + buf * STAGE;
    char* bs = as + AB;
    const long long mrow0 = (long long)kt * BM;  // relative to m_beg
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      if (!a_on[u]) continue;
      const long long m = mrow0 + a_m[u];
      const bool ok = m_beg + m < m_end && a_col[u] != PW_OOB;
      pw_glds16(dr, as + (u * NW + wid) * 1024, ok ? (unsigned)(m * ldd * 2) + a_col[u] : PW_OOB);
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const long long m = mrow0 + b_m[u];
      bool ok = m_beg + m < m_end && b_tap[u] != PW_OOB;
      unsigned off;
      if (DENSE) {
        off = (unsigned)(m * a.ldx * 2) + b_tap[u];
      } else {
        // pixel -> (image, oh, ow) by float-reciprocal division (exact: p < 2^22)
        const int p = b_p[u] + kt * BM;
        int im = (int)((float)p * inv_howo);
        int rem = p - im * HoWo;
        if (rem < 0) { --im; rem += HoWo; } else if (rem >= HoWo) { ++im; rem -= HoWo; }
        int oh = (int)((float)rem * inv_wo);
        int ow = rem - oh * a.Wo;
        if (ow < 0) { --oh; ow += a.Wo; } else if (ow >= a.Wo) { ++oh; ow -= a.Wo; }
        const int ih = oh * a.stride - a.pad + b_r[u];
        const int iw = ow * a.stride - a.pad + b_s[u];
        ok = ok && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
        off = (unsigned)(((long long)im * a.sN + (long long)ih * a.sH + (long long)iw * a.sW) * 2) + b_tap[u];
      }
      pw_glds16(xr, bs + (u * NW + wid) * 1024, ok ? off : PW_OOB);
    }
  };

  const int wco = wid / WKK, wkk = wid % WKK;
  const int t = lane & 15, g = lane >> 4;
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* as = smem + buf * STAGE;
    const char* bs = as + AB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int mb = kk * 32 + 8 * g;
      if constexpr (MT * NT >= 32) {
        // big wave tiles: the B fragments stay, one A fragment at a time, and
        // the LDS addresses are recomputed per k-step (an opaque lane index
        // keeps the compiler from hoisting 64 address registers out of the loop)
        int tt = t;
        asm volatile("" : "+v"(tt));
        bf16x8 bv[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const pw_v4s lo = pw_tr<BKK>(bs, mb, wkk * WTK + 16 * j, tt);
          const pw_v4s hi = pw_tr<BKK>(bs, mb + 4, wkk * WTK + 16 * j, tt);
          bv[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const pw_v4s lo = pw_tr<BCO>(as, mb, wco * WTCO + 16 * i, tt);
          const pw_v4s hi = pw_tr<BCO>(as, mb + 4, wco * WTCO + 16 * i, tt);
          const bf16x8 af = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bv[j], acc[i][j], 0, 0, 0);
        }
        continue;
      }
      bf16x8 af[MT], bv[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const pw_v4s lo = pw_tr<BCO>(as, mb, wco * WTCO + 16 * i, t);
        const pw_v4s hi = pw_tr<BCO>(as, mb + 4, wco * WTCO + 16 * i, t);
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const pw_v4s lo = pw_tr<BKK>(bs, mb, wkk * WTK + 16 * j, t);
        const pw_v4s hi = pw_tr<BKK>(bs, mb + 4, wkk * WTK + 16 * j, t);
        bv[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bv[j], acc[i][j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    int ahead = nk - 1 - kt;
    if (ahead > NSTAGE - 2) ahead = NSTAGE - 2;
    if (lps_hi) pw_wait_stages<LPS_HI, NSTAGE>(ahead);
    else pw_wait_stages<LPS_LO, NSTAGE>(ahead);
    // retire this wave's LDS reads of the slot the next issue overwrites
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTAGE - 1 < nk) issue(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    compute(kt % NSTAGE);
  }

  if (a.dbg & 1) {  // profiling: everything but the dW atomics (the sum keeps the MFMAs alive)
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 1.2345e-30f) atomicAdd(a.dw, sum);
    return;
  }
  // acc[i][j][r]: co = co0 + wco*WTCO + 16 i + 4 g + r, k = k0 + wkk*WTK + 16 j + t
  // (relative to the tile's part of dY: cb, colim, dwp)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int k = k0 + wkk * WTK + 16 * j + t;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cb + wco * WTCO + 16 * i + 4 * g + r;
        if (co < colim && k < a.K) atomicAdd(dwp + (long long)co * a.K + k, acc[i][j][r]);
      }
    }
}

// ---------------------------------------------------------------------------
// Halo-tiled weight gradient of a 3x3 stride-1 pad-1 convolution: the stem
// conv2/conv3 (models.py:312-317) and the Bottleneck conv2 of every stage
// (models.py:200-201).  The pipelined kernel above gathers every input pixel
// nine times (implicit im2col) and re-streams dY once per 128-wide k tile;
// here a workgroup owns one (CT input-channel x OT output-channel) slice of dW
// for all nine taps, kept in registers across a persistent run of TR x 16
// output-pixel tiles: per tile the dY slice and the (TR+2) x 18 input-halo
// slice come into LDS once (LDS-DMA by one loader wave, double buffer) and all
// nine taps read the halo there.  One round of f32 atomics adds the block's
// slice into dW at the end.  Compute wave w owns the (16-channel input tile,
// tap) pairs w, w + NWC, ... for all OT output channels.  LDS images are plain
// row-major (one halo / output pixel per row); the MFMA fragments, 8
// consecutive pixels per lane, come from the transposing read
// ds_read_b64_tr_b16 (2-way bank conflicts at most for every tap offset).
// Workgroups are numbered so that the NPC channel slices of one pixel-tile
// group run on the same XCD at the same time and share dY / input through L2.
// ---------------------------------------------------------------------------
template <int CT, int OT, int TR, int NWC>
struct HwGeom {
  static constexpr int TC = 16, NPX = TR * TC, HW = TC + 2, NQ = HW * (TR + 2);
  static constexpr int SX = 2 * CT, SD = 2 * OT;         // LDS row bytes (halo pixel, dY pixel)
  static constexpr int XI = (NQ * SX + 1023) / 1024;     // 1-KB halo DMA instructions
  static constexpr int DI = NPX * SD / 1024;             // 1-KB dY tile DMA instructions
  static constexpr int XB = XI * 1024, DB = DI * 1024, STAGE = XB + DB;
  static constexpr int NJ = CT / 16, MTC = OT / 16, NPAIR = NJ * 9, PPW = (NPAIR + NWC - 1) / NWC;
};

__device__ __forceinline__ pw_v4s hw_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_v4s)(pw_lds_t)(base + off));
}

template <int CT, int OT, int TR, int NWC, bool DL>
__global__ void __launch_bounds__(64 * (NWC + (DL ? 1 : 0))) hwgrad_kernel(PwArgs a, int ntiles, int npc) {
  using Gm = HwGeom<CT, OT, TR, NWC>;
  constexpr int TC = Gm::TC, NPX = Gm::NPX, HW = Gm::HW, NQ = Gm::NQ;
  constexpr int SX = Gm::SX, SD = Gm::SD, XI = Gm::XI, DI = Gm::DI, XB = Gm::XB, STAGE = Gm::STAGE;
  constexpr int NJ = Gm::NJ, MTC = Gm::MTC, NPAIR = Gm::NPAIR, PPW = Gm::PPW;
  static_assert(2 * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (pixel-tile group, channel slice): the npc slices of a group share an XCD
  const int G = gridDim.x / npc;  // groups; gridDim.x is a multiple of 8 * npc
  const int xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
  const int grp = xcd + 8 * (loc / npc), pc = loc % npc;
  const int nci = a.C / CT;
  const int ci0 = (pc % nci) * CT, co0 = (pc / nci) * OT;
  const int ntw = (a.Wo + TC - 1) / TC, nth = (a.Ho + TR - 1) / TR;
  const int HoWo = a.Ho * a.Wo;

  // operands of tile t -> stage buf (loader wave): lane l of DMA instruction
  // g moves bytes g * 1024 + 16 l .. + 15 of the row-major image
  // DL: the loader wave issues every piece; otherwise compute wave w issues
  // pieces w, w + NWC, ... of each image
  constexpr int LS = DL ? 1 : NWC;
  const int l0 = DL ? 0 : wid;
  auto issue = [&](int t, int buf) {
    const int img = t / (nth * ntw), rem = t - img * (nth * ntw);
    const int h0 = (rem / ntw) * TR, w0 = (rem - (rem / ntw) * ntw) * TC;
    char* xs = smem + buf * STAGE;
    char* ds = xs + XB;
    const __amdgpu_buffer_rsrc_t xr =
        pw_rsrc(reinterpret_cast<const bf16*>(a.x) + (long long)img * a.sN, (a.x_elems - (long long)img * a.sN) * 2);
#pragma unroll 4
    for (int g = l0; g < XI; g += LS) {
      const int b = g * 1024 + lane * 16;
      const int q = b / SX, ci = (b - (b / SX) * SX) >> 1;
      const int hr = q / HW, hc = q - (q / HW) * HW;
      const int ih = h0 - 1 + hr, iw = w0 - 1 + hc;
      const bool ok = q < NQ && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      pw_glds16(xr, xs + g * 1024, ok ? (unsigned)((ih * (int)a.sH + iw * (int)a.sW + ci0 + ci) * 2) : PW_OOB);
    }
    const long long pimg = (long long)img * HoWo;
    const __amdgpu_buffer_rsrc_t dr =
        pw_rsrc(reinterpret_cast<const bf16*>(a.dy) + pimg * a.ldd, (a.dy_elems - pimg * a.ldd) * 2);
#pragma unroll 4
    for (int g = l0; g < DI; g += LS) {
      const int b = g * 1024 + lane * 16;
      const int m = b / SD, co = (b - (b / SD) * SD) >> 1;
      const int oh = h0 + m / TC, ow = w0 + m % TC;
      const bool ok = oh < a.Ho && ow < a.Wo;
      pw_glds16(dr, ds + g * 1024, ok ? (unsigned)(((oh * a.Wo + ow) * (int)a.ldd + co0 + co) * 2) : PW_OOB);
    }
  };

  const int t = lane & 15, g = lane >> 4;
  // lane constants of the transposing reads: row t >> 2, byte column 8 (t & 3)
  const int la = (t >> 2) * SD + 8 * (t & 3);
  const int lb = (t >> 2) * SX + 8 * (t & 3);
  // this wave's (channel tile, tap) pairs as halo byte offsets (uniform);
  // pairs past NPAIR (uneven split) repeat the last one and are dropped
  int pofs[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    int pi = wid + NWC * p;
    if (pi >= NPAIR) pi = NPAIR - 1;
    const int tap = pi / NJ;
    pofs[p] = ((tap / 3) * HW + tap % 3) * SX + 32 * (pi % NJ);
  }
  f32x4 acc[PPW][MTC];
#pragma unroll
  for (int p = 0; p < PPW; ++p)
#pragma unroll
    for (int i = 0; i < MTC; ++i) acc[p][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the two roles run separate loops with one barrier per tile each (one loop
  // with a role branch would merge the accumulators of both paths and copy
  // them every tile)
  if (DL && wid == NWC) {
    if (grp < ntiles) issue(grp, 0);
    int k = 0;
    for (int tile = grp; tile < ntiles; tile += G, ++k) {
      pw_vm_wait<0>();  // this tile's operands have landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (tile + G < ntiles) issue(tile + G, (k + 1) & 1);
    }
    pw_vm_wait<0>();
    return;
  }
  if (!DL && grp < ntiles) issue(grp, 0);
  int k = 0;
  for (int tile = grp; tile < ntiles; tile += G, ++k) {
    if constexpr (!DL) pw_vm_wait<0>();  // this wave's pieces of tile k have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile k visible; the other buffer is free
    asm volatile("" ::: "memory");
    if constexpr (!DL) {
      if (tile + G < ntiles) issue(tile + G, (k + 1) & 1);
    }
    const char* xs = smem + (k & 1) * STAGE;
    const char* ds = xs + XB;
#pragma unroll 1
    for (int ks = 0; ks < NPX / 32; ++ks) {
      // this lane's 8 pixels m = mb .. mb + 7 lie in one tile row
      const int mb = ks * 32 + 8 * g;
      const int row = mb / TC, col0 = mb - (mb / TC) * TC;
      const char* da = ds + mb * SD + la;
      bf16x8 af[MTC];
#pragma unroll
      for (int i = 0; i < MTC; ++i) {
        const pw_v4s lo = hw_tr(da, 32 * i);
        const pw_v4s hi = hw_tr(da, 4 * SD + 32 * i);
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      const char* xa = xs + (row * HW + col0) * SX + lb;
#pragma unroll
      for (int p = 0; p < PPW; ++p) {
        const pw_v4s lo = hw_tr(xa, pofs[p]);
        const pw_v4s hi = hw_tr(xa, pofs[p] + 4 * SX);
        const bf16x8 bv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int i = 0; i < MTC; ++i) acc[p][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bv, acc[p][i], 0, 0, 0);
      }
    }
  }
  // acc[p][i][r]: co = co0 + 16 i + 4 g + r, input channel ci0 + 16 j + t of tap `tap`.
  // The lane offset passes through an opaque statement here so that the
  // compiler cannot hoist all the atomic addresses above the tile loop (they
  // are loop invariant) and hold them in registers through it.
  int lo = (co0 + 4 * g) * a.K + ci0 + t;
  asm volatile("" : "+v"(lo));
  float* dwl = a.dw + lo;
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int pi = wid + NWC * p;
    if (pi >= NPAIR) continue;
    const int j = pi % NJ, tap = pi / NJ;
#pragma unroll
    for (int i = 0; i < MTC; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(dwl + (16 * i + r) * a.K + tap * a.C + 16 * j, acc[p][i][r]);
  }
}

static bool hwgrad_ok(const PwArgs& a) {
  if (a.dense || a.R != 3 || a.S != 3 || a.pad != 1 || a.stride != 1 || a.M <= 0) return false;
  const bool small = (a.C == 32 || a.C == 64) && (a.Cout == 32 || a.Cout == 64) && !(a.C == 64 && a.Cout == 64);
  const bool tiled = a.C % 64 == 0 && a.Cout % 64 == 0;
  if (!small && !tiled) return false;
  if (a.K != 9 * a.C || a.Ho != a.H || a.Wo != a.W || a.M % ((long long)a.Ho * a.Wo)) return false;
  if (a.Ho < 8 || a.Wo < 8) return false;  // tiles mostly padding: the pipelined kernel
  if (a.sW < a.C || a.ldd < a.Cout) return false;
  if (a.sN * 2 > 0x7fffffffLL || (long long)a.Ho * a.Wo * a.ldd * 2 > 0x7fffffffLL) return false;
  const long long nt = (a.M / ((long long)a.Ho * a.Wo)) * ((a.Ho + 7) / 8) * ((a.Wo + 15) / 16);
  return nt < 0x7fffffffLL;
}

template <int CT, int OT, int TR, int NWC, bool DL>
static void hwgrad_go(const PwArgs& a, hipStream_t st) {
  using Gm = HwGeom<CT, OT, TR, NWC>;
  const int ntiles = (int)((a.M / ((long long)a.Ho * a.Wo)) * ((a.Ho + TR - 1) / TR) * ((a.Wo + 15) / 16));
  const int npc = (a.C / CT) * (a.Cout / OT);
  int per_cu = (160 * 1024) / (2 * Gm::STAGE);
  if (per_cu > 2) per_cu = 2;
  // pixel-tile groups: fill the chip once, a multiple of 8 (one XCD per group)
  int groups = (g_wgrad_cus * per_cu / npc) / 8 * 8;
  if (groups < 8) groups = 8;
  const int need = (ntiles + 7) / 8 * 8;
  if (groups > need) groups = need;
  hipLaunchKernelGGL((hwgrad_kernel<CT, OT, TR, NWC, DL>), dim3(groups * npc), dim3(64 * (NWC + (DL ? 1 : 0))), 0, st,
                     a, ntiles, npc);
}

template <int CT, int OT, int NWC, bool DL = true>
static void hwgrad_tiles(const PwArgs& a, hipStream_t st) {
  if (a.Ho % 16 == 0 && a.Wo % 16 == 0) hwgrad_go<CT, OT, 16, NWC, DL>(a, st);
  else hwgrad_go<CT, OT, 8, NWC, DL>(a, st);
}

// variant 0: the kernel below per channel class; variant 1 (64-channel tiled
// shapes only): 4 compute waves of 9 (channel tile, tap) pairs each instead of
// 8 waves of 4.5 (0.72 transposing LDS reads per MFMA instead of 0.9, no
// repeated pairs; 144 accumulator registers per lane).  Variants 2 / 3: the
// same two 64-channel forms (and variant 2 for every channel class) without
// the loader wave, the compute waves issuing the LDS-DMA pieces themselves.
// A loader wave is allocated the compute waves' registers: at 192 VGPRs (two
// waves per SIMD) the 4 + 1 waves of a workgroup leave no room for a second
// workgroup on the CU, so one compute wave per SIMD hides no LDS latency;
// without it two workgroups (two compute waves per SIMD) fit.
static bool hwgrad_launch(const PwArgs& a, int variant, hipStream_t st) {
  if (!hwgrad_ok(a)) return false;
  if (variant == 3) {
    if (a.C % 64 || a.Cout % 64) return false;
    set_last_kernel("hwgrad_kernel<64,64,nl>");
    hwgrad_tiles<64, 64, 8, false>(a, st);
    return true;
  }
  if (variant == 2) {
    if (a.C == 32 && a.Cout == 32) {
      set_last_kernel("hwgrad_kernel<32,32,nl>");
      hwgrad_tiles<32, 32, 4, false>(a, st);
    } else if (a.C == 32) {
      set_last_kernel("hwgrad_kernel<32,64,nl>");
      hwgrad_tiles<32, 64, 4, false>(a, st);
    } else if (a.Cout == 32) {
      set_last_kernel("hwgrad_kernel<64,32,nl>");
      hwgrad_tiles<64, 32, 4, false>(a, st);
    } else {
      set_last_kernel("hwgrad_kernel<64,64,w4,nl>");
      hwgrad_tiles<64, 64, 4, false>(a, st);
    }
    return true;
  }
  if (variant != 0) {
    if (variant != 1 || a.C % 64 || a.Cout % 64) return false;
    set_last_kernel("hwgrad_kernel<64,64,w4>");
    hwgrad_tiles<64, 64, 4>(a, st);
    return true;
  }
  if (a.C == 32 && a.Cout == 32) {
    set_last_kernel("hwgrad_kernel<32,32>");
    hwgrad_tiles<32, 32, 4>(a, st);
  } else if (a.C == 32) {
    set_last_kernel("hwgrad_kernel<32,64>");
    hwgrad_tiles<32, 64, 4>(a, st);
  } else if (a.Cout == 32) {
    set_last_kernel("hwgrad_kernel<64,32>");
    hwgrad_tiles<64, 32, 4>(a, st);
  } else {
    // 64-channel slices of input and output channels, 8 compute waves
    set_last_kernel("hwgrad_kernel<64,64>");
    hwgrad_tiles<64, 64, 8>(a, st);
  }
  return true;
}

// ---------------------------------------------------------------------------
// tile configurations (BCO x BKK output tile, waves WCO x WKK, LDS stages)
struct PwCfg {
  int bco, bkk, threads;
};
static const PwCfg kPw[] = {
    {128, 128, 256},  // 0: 4 waves 64x64, 4 stages
    {128, 256, 512},  // 1: 8 waves 64x64, 3 stages
    {256, 128, 512},  // 2: 8 waves 64x64, 3 stages
    {64, 256, 512},   // 3: 8 waves 64x32, 3 stages
    {64, 128, 256},   // 4: 4 waves 64x32, 4 stages
    {32, 128, 256},   // 5: 4 waves 32x32, 4 stages
    {64, 512, 512},   // 6: 8 waves 64x64, 2 stages
    {256, 256, 512},  // 7: 8 waves 128x64, 2 stages (half the LDS-DMA issues per MFMA of 0-2)
    {256, 256, 512},  // 8: 8 waves 64x128, 2 stages
};
constexpr int kNumPw = 9;

template <bool DENSE>
static void pw_launch_c(int c, const PwArgs& a, long long blocks, hipStream_t st) {
  const dim3 g((unsigned)blocks);
  switch (c) {
    case 0: hipLaunchKernelGGL((pwgrad_kernel<128, 128, 2, 2, 4, DENSE>), g, dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL((pwgrad_kernel<128, 256, 2, 4, 3, DENSE>), g, dim3(512), 0, st, a); break;
    case 2: hipLaunchKernelGGL((pwgrad_kernel<256, 128, 4, 2, 3, DENSE>), g, dim3(512), 0, st, a); break;
    case 3: hipLaunchKernelGGL((pwgrad_kernel<64, 256, 1, 8, 3, DENSE>), g, dim3(512), 0, st, a); break;
    case 4: hipLaunchKernelGGL((pwgrad_kernel<64, 128, 1, 4, 4, DENSE>), g, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((pwgrad_kernel<32, 128, 1, 4, 4, DENSE>), g, dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL((pwgrad_kernel<64, 512, 1, 8, 2, DENSE>), g, dim3(512), 0, st, a); break;
    case 7: hipLaunchKernelGGL((pwgrad_kernel<256, 256, 2, 4, 2, DENSE>), g, dim3(512), 0, st, a); break;
    default: hipLaunchKernelGGL((pwgrad_kernel<256, 256, 4, 2, 2, DENSE>), g, dim3(512), 0, st, a); break;
  }
}

// split-K levels: (target workgroups, minimum K-steps per workgroup).  Fewer,
// longer splits trade CU fill for fewer f32 atomics into dW (the device-scope
// atomics of the split flushes run memory-side and cost ~30 % of a dense
// wgrad at 1536 workgroups).  The split count rounds DOWN to the target, so a
// 256 / 512 target fills whole rounds of the 256 CUs (one workgroup per CU)
// instead of leaving a tail round of a few workgroups.
static const int kSplitTarget[] = {1536, 768, 512, 256};  // for 256 CUs (scaled by g_wgrad_cus)
int g_wgrad_cus = 256;
static const int kSplitMinSteps[] = {8, 16, 24, 64};
constexpr int kNumLevels = 4;

// candidates: kNumPw tile configurations x kNumLevels split levels, then the
// halo-tiled kernel (four variants, see hwgrad_launch)
int pwgrad_num_cfgs() { return kNumPw * kNumLevels + 4; }

// split level of candidate c of the pipelined wgrad (-1: the halo kernel)
int pwgrad_level(int c) { return c >= 0 && c < kNumPw * kNumLevels ? c / kNumPw : -1; }

// candidate c = cfg + kNumPw * level of the pipelined wgrad; false (nothing
// launched) if not applicable
bool pwgrad_launch(PwArgs a, int cand, hipStream_t st) {
  if (cand >= kNumPw * kNumLevels)
    return !a.dy2 && cand < pwgrad_num_cfgs() && hwgrad_launch(a, cand - kNumPw * kNumLevels, st);
  if (cand < 0 || cand >= kNumPw * kNumLevels) return false;
  const int c = cand % kNumPw, level = cand / kNumPw;
  if (a.Cout % 8 || a.K % 8 || a.M <= 0) return false;
  if (!a.dense && (a.C % 8 || a.R * a.S > 32)) return false;
  const PwCfg& g = kPw[c];
  if (a.dy2 && (!a.dense || a.Cout1 % g.bco != 0 || !a.dw2 || a.ldd2 % 8)) return false;
  // skip shapes where most of the tile would be padding
  if (g.bco > 32 && a.Cout <= g.bco / 2) return false;
  if (g.bkk > 128 && a.K <= g.bkk / 2) return false;
  const long long ntiles = (long long)((a.Cout + g.bco - 1) / g.bco) * ((a.K + g.bkk - 1) / g.bkk);
  const long long ksteps = (a.M + 63) / 64;
  const long long target = (long long)kSplitTarget[level] * g_wgrad_cus / 256;
  long long splits = target >= ntiles ? target / ntiles : 1;
  const long long max_splits = (ksteps + kSplitMinSteps[level] - 1) / kSplitMinSteps[level];
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long long per = (ksteps + splits - 1) / splits;
  // keep workgroup-relative byte offsets below 2^31 and pixel indices below 2^22
  long long ldmax = a.dense ? (a.ldx > a.ldd ? a.ldx : a.ldd) : a.ldd;
  if (a.dy2 && a.ldd2 > ldmax) ldmax = a.ldd2;
  const long long row_bytes = ldmax * 2;
  long long cap = (0x7fffffffLL / row_bytes) / 64 - 1;
  if (!a.dense) {
    const long long HoWo = (long long)a.Ho * a.Wo;
    const long long imgs = 0x7fffffffLL / (a.sN * 2) - 2;
    if (imgs < 1 || HoWo >= (1LL << 21)) return false;
    const long long cap3 = imgs * HoWo / 64;
    if (cap3 < cap) cap = cap3;
    const long long cap4 = ((1LL << 22) - 2 * HoWo) / 64;
    if (cap4 < cap) cap = cap4;
  }
  if (cap < 1) return false;
  if (per > cap) per = cap;
  a.m_per_split = per * 64;
  splits = (ksteps + per - 1) / per;
  const long long blocks = ntiles * splits;
  if (blocks > 0x7fffffffLL) return false;
  static const char* names[] = {"pwgrad_kernel<128,128>", "pwgrad_kernel<128,256>", "pwgrad_kernel<256,128>",
                                "pwgrad_kernel<64,256>",  "pwgrad_kernel<64,128>",  "pwgrad_kernel<32,128>",
                                "pwgrad_kernel<64,512>",  "pwgrad_kernel<256,256,w2x4>",
                                "pwgrad_kernel<256,256,w4x2>"};
  set_last_kernel(names[c]);
  if (a.dense) pw_launch_c<true>(c, a, blocks, st);
  else pw_launch_c<false>(c, a, blocks, st);
  return true;
}

}  // namespace artsbir

// the weight-gradient grids (split-K targets, persistent halo groups) sized for
// n CUs: the engine's side stream restricted by a CU mask (ARTSBIR_SIDE_CUS);
// returns the previous value
extern "C" int artsbir_set_wgrad_cus(int n) {
  const int old = artsbir::g_wgrad_cus;
  if (n >= 8 && n <= 4096) artsbir::g_wgrad_cus = n;
  return old;
}
