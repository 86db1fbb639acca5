// Device-side building blocks of the pipelined implicit-GEMM kernels (pgemm.hip,
// pp256.hip): LDS-DMA loads, counted waits, XCD remap, the channel permutation
// of the weight tile, BN statistics / fused BN-backward epilogues.  Header-only
// (inline device functions and templates), shared by both translation units.
#pragma once
#include "common.h"
#include "pgemm.h"

namespace artsbir {

#define PG_OOB 0x80000000u
#ifndef PG_SNAKE
#define PG_SNAKE 1  // GLB epilogue: odd channel pairs walk the pixel tiles backwards (pg_epilogue_k)
#endif
#ifndef PG_PRIO
#define PG_PRIO 1
#endif
#if PG_PRIO
// raise wave priority around each MFMA cluster (guide T5: keeps hipcc from
// spreading the cluster across the stage barriers)
#define PG_PRIO_ON() __builtin_amdgcn_s_setprio(1)
#define PG_PRIO_OFF() __builtin_amdgcn_s_setprio(0)
#else
#define PG_PRIO_ON()
#define PG_PRIO_OFF()
#endif
typedef __attribute__((address_space(3))) void* pg_lds_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;

// a wave-uniform 64-bit value the compiler cannot prove uniform (kept in SGPRs)
__device__ __forceinline__ long long pg_uniform(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(v & 0xffffffffLL));
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
  return (long long)(((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pg_rsrc(const void* base, long long bytes) {
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// LDS-DMA of 16 B per lane to lds + 16 * lane.  Inline asm on purpose: hipcc
// does not track it, so it neither drains it with vmcnt(0) before every
// ds_read nor at barriers; completion is counted by hand (vm_wait below).
// M0 is written and restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(pg_lds_t)lds);
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

// the same with a wave-uniform byte offset added by the buffer unit (soffset):
// rows u * stride of one lane base keep ONE address VGPR live, not one per row
__device__ __forceinline__ void glds16_so(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff, unsigned soff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(pg_lds_t)lds);
  const unsigned so = __builtin_amdgcn_readfirstlane(soff);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(r), "s"(so)
      : "memory");
}

// the same with 4 B per lane (lds + 4 * lane)
__device__ __forceinline__ void glds4(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(pg_lds_t)lds);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(base), "s"(r)
      : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` stages of this wave's loads are outstanding
template <int LPS, int NSTAGE>
__device__ __forceinline__ void wait_stages(int ahead) {
  if constexpr (NSTAGE >= 6) {
    if (ahead >= 4) { vm_wait<4 * LPS>(); return; }
    if (ahead >= 3) { vm_wait<3 * LPS>(); return; }
  }
  if constexpr (NSTAGE >= 4) {
    if (ahead >= 2) { vm_wait<2 * LPS>(); return; }
  }
  if constexpr (NSTAGE >= 3) {
    if (ahead >= 1) { vm_wait<LPS>(); return; }
  }
  vm_wait<0>();
}

__device__ __forceinline__ long long pg_xcd_remap(long long bid, long long nwg) {
  if (nwg < 8) return bid;
  const long long q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// channel held by LDS weight row rho of a tile (rho = 16 i + 4 q + r  ->
// 32 (i >> 1) + 8 q + 4 (i & 1) + r): MFMA output lane q then owns 8
// consecutive channels of each 32-channel pair of 16-row tiles.
__device__ __forceinline__ int pg_perm(int rho) {
  return 32 * (rho >> 5) + 8 * ((rho >> 2) & 3) + 4 * ((rho >> 4) & 1) + (rho & 3);
}

// Sum each of 16 per-lane values (s1[0..8), s2[0..8)) over the 16 lanes of a
// DPP row (lanes with the same lane >> 4) with 4 row_shr DPP adds per value
// (VALU only, no LDS round trips); the row totals end in lane 15 of the row.
__device__ __forceinline__ float dpp_row_sum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, true));
  return x;
}

// Block-level BN statistics: every compute wave adds its reduce16 result into
// an LDS accumulator red[seg][2][BCH] (ds_add_f32); the last wave of the tile
// (LDS counter) flushes it with 2*BCH global atomics per segment into the
// replica slot and zeroes it.  Cuts global atomics by the number of waves
// sharing a channel.  Segments: when one launch covers several of the
// reference's separate forward calls (the sketch / positive / negative
// branches, train.py:28-30), each keeps its own statistics; a tile of BPX <=
// seg_m pixels touches at most two segments (red[0] = the tile's first).
//
// The same accumulator serves the fused BatchNorm-backward reduction of the
// data-gradient epilogue (a.bnb): rows 0..2 = sum g, sum g*xhat_0, sum g*xhat_1
// go to slots_0[0], slots_0[1] (and slots_1[0], slots_1[1]).
template <int BCH>
__device__ __forceinline__ void stats_flush(float* red, int* cnt, int last_count, const PgArgs& a, int bch, int slot,
                                            int lane, long long bpx, int bpx_n) {
  // LDS operations of one wave complete in order; the wait makes this wave's
  // adds land before its counter increment (no global-memory fence needed)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0, 64);
  if (old != last_count) return;
  asm volatile("" ::: "memory");
  long long seg0 = 0;
  int nsg = 1;
  if (a.seg_m > 0) {
    long long last = bpx + bpx_n - 1;
    if (last >= a.M) last = a.M - 1;
    seg0 = bpx / a.seg_m;
    nsg = (int)(last / a.seg_m - seg0) + 1;
  }
  const int nrow = (a.bnb && a.bnb_nt == 2) ? 3 : 2;
  for (int sg = 0; sg < nsg; ++sg) {
    const long long so = (seg0 + sg) * a.seg_stride + (long long)slot * 2 * a.Cout;
    float* rr = red + sg * 3 * BCH;
    for (int i = lane; i < nrow * BCH; i += 64) {
      const int m = i / BCH;
      const int ch = bch + i - m * BCH;
      const float v = rr[i];
      rr[i] = 0.f;
      if (ch >= a.Cout || (a.dbg & 1)) continue;  // dbg 1: timing experiment without the global atomics
      if (!a.bnb) {
        atomicAdd(a.stats + so + m * a.Cout + ch, v);
      } else if (m == 0) {
        atomicAdd(a.bnb_slots[0] + so + ch, v);
        if (a.bnb_nt == 2) atomicAdd(a.bnb_slots[1] + so + ch, v);
      } else {
        atomicAdd(a.bnb_slots[m - 1] + so + a.Cout + ch, v);
      }
    }
  }
}

// 8 consecutive floats by two 16-B loads
__device__ __forceinline__ void loadf8v(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ---- epilogue operands staged in LDS (after the main loop the stage ring is
// free): the tile's [BPX pixels][BCH channels] slice of y_0, the residual, y_1
// and the bf16 mask are brought in by LDS-DMA, every wave's instructions in
// flight at once (one round trip per tile instead of one per pixel batch), then
// read from LDS by the epilogue lanes.  Row r of an operand holds its BCH/8
// 16-B chunks in slot order chunk ^ (r % (BCH/8)) (swizzle applied to the DMA
// source addresses), so the epilogue's reads (16 rows x one chunk per
// ds_read_b128 phase) hit 16 distinct 16-B bank groups.
struct EpiStage {
  const char* y0;   // nullptr: read from global memory
  const char* res;
  const char* y1;
  const char* mk;
  const unsigned char* bits;  // kind 3: [BPX][BCH/8] mask bytes
  const float* prm;           // BNB: [2 segments][7][BCH] per-channel BN constants (pg_prm_fill)
  long long seg0;             // segment of the tile's first pixel
};

// BN-backward constants of the tile's channels for its (at most two) segments,
// in LDS before the main loop so the epilogue reads no global memory for them:
// rows istd_0, mean_0, istd_1, mean_1, mask mean, mask scale, mask beta
constexpr int PG_PRM_ROWS = 7;
template <int BCH>
constexpr int pg_prm_bytes() {  // padded to a whole number of 512-thread passes
  return (2 * PG_PRM_ROWS * BCH + 511) / 512 * 512 * 4;
}

template <int BCH, int NT>
__device__ __forceinline__ void pg_prm_fill(const PgArgs& a, float* prm, long long bpx, int bch, long long seg0) {
  // a fixed trip count (a divergent loop exit here pushes the kernel's later
  // uniform values into VGPRs, which the LDS-DMA asm cannot take)
  constexpr int NE = 2 * PG_PRM_ROWS * BCH;
  const long long nseg = a.seg_m > 0 ? a.M / a.seg_m : 1;
  const bool two = a.bnb_nt == 2, msk = a.bnb == 1;
  // the source rows as wave-uniform pointers (selecting among the fields of the
  // by-value argument struct per lane would move it to scratch)
  const float* rows[PG_PRM_ROWS];
  rows[0] = reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_istd[0]));
  rows[1] = reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_mean[0]));
  rows[2] = two ? reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_istd[1])) : rows[0];
  rows[3] = two ? reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_mean[1])) : rows[0];
  const float* mb = msk ? reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_mbn)) : rows[0];
  rows[4] = mb;
  rows[5] = msk ? mb + 2 * a.Cout : rows[0];
  rows[6] = msk ? mb + 3 * a.Cout : rows[0];
  static_assert(pg_prm_bytes<BCH>() / 4 % NT == 0, "whole passes");
#pragma unroll
  for (int k = 0; k < pg_prm_bytes<BCH>() / 4 / NT; ++k) {
    const int i = k * NT + (int)threadIdx.x;
    const int s = i / (PG_PRM_ROWS * BCH), r = (i / BCH) % PG_PRM_ROWS, c = i % BCH;
    long long sg = seg0 + s;
    if (sg >= nseg) sg = nseg - 1;
    const int ch = bch + c;
    const bool have = i < NE && ch < a.Cout && (r < 2 || (r < 4 && two) || (r >= 4 && msk));
    // every lane loads from a valid address (channel 0 of row 0) and selects
    const float* src = rows[0];
#pragma unroll
    for (int q = 1; q < PG_PRM_ROWS; ++q) src = r == q ? rows[q] : src;
    const float v = src[have ? sg * a.bnb_pstride + ch : 0];
    prm[i] = have ? v : 0.f;
  }
}

// DMA of the tile's block-output mask bits (kind 3): row r = BCH/8 bytes
template <int BPX, int BCH, int NW>
__device__ __forceinline__ void stage_bits(const void* bits, unsigned char* lds, long long bpx, int bch,
                                           const PgArgs& a, int wid, int lane) {
  constexpr int LPR = BCH / 32;  // dwords (lanes) per row
  constexpr int RPI = 64 / LPR;
  constexpr int NI = (BPX + RPI - 1) / RPI;
  const long long rowb = a.Cout >> 3;
  const __amdgpu_buffer_rsrc_t r = pg_rsrc(reinterpret_cast<const unsigned char*>(pg_uniform((long long)bits)) +
                                               pg_uniform(bpx) * rowb, (a.M - pg_uniform(bpx)) * rowb);
  const int w = lane % LPR;
#pragma unroll
  for (int i = wid; i < NI; i += NW) {
    const int row = i * RPI + lane / LPR;
    const long long px = bpx + row;
    const unsigned off = (row < BPX && px < a.M && bch + 32 * w < a.Cout)
                             ? (unsigned)(row * rowb + (bch >> 3) + 4 * w) : PG_OOB;
    glds4(r, reinterpret_cast<char*>(lds) + i * 256, off);
  }
}

template <int BCH>
__device__ __forceinline__ Vec16<bf16> stg_read(const char* base, int row, int chunk) {
  constexpr int CPR = BCH / 8;
  return ld16<bf16>(reinterpret_cast<const bf16*>(base + row * (BCH * 2) + ((chunk ^ (row & (CPR - 1))) << 4)));
}

// DMA of one operand slice: rows bpx .. bpx+BPX-1 (source row index src_row(px)),
// channels bch .. bch+BCH-1 of a bf16 [rows][ld] tensor; res_pool: the
// AvgPool2d(2)-backward residual, row px reads pooled row (img, oh/2, ow/2)
template <int BPX, int BCH, int NW>
__device__ __forceinline__ void stage_operand(const void* t, long long t_rows, int ld, char* lds, long long bpx,
                                              int bch, const PgArgs& a, bool res_pool, int wid, int lane) {
  constexpr int CPR = BCH / 8;
  constexpr int RPI = 64 / CPR;  // rows per DMA instruction
  constexpr int NI = BPX / RPI;
  static_assert(CPR <= 64 && 64 % CPR == 0, "stage rows");
  const int HoWo = a.Ho * a.Wo;
  auto src_row = [&](long long px) -> long long {
    if (!res_pool) return px;
    const long long img = px / HoWo;
    const int rem = (int)(px - img * HoWo);
    const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    return (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
  };
  // lowest source row of the tile (pooled rows are not monotone inside an
  // output row pair: row oh+1 maps back to pooled row oh/2), so start the
  // descriptor at column 0 of the first pixel's row
  long long r0;
  {
    const long long p0 = bpx < a.M ? bpx : a.M - 1;
    r0 = pg_uniform(res_pool ? src_row(p0 - (p0 % HoWo) % a.Wo) : p0);
  }
  const __amdgpu_buffer_rsrc_t r =
      pg_rsrc(reinterpret_cast<const bf16*>(pg_uniform((long long)t)) + r0 * ld, (t_rows - r0) * (long long)ld * 2);
  const int pos = lane % CPR;
#pragma unroll
  for (int i = wid; i < NI; i += NW) {
    const int row = i * RPI + lane / CPR;
    const int c = pos ^ (row & (CPR - 1));
    const long long px = bpx + row;
    const int ch = bch + 8 * c;
    const unsigned off = (px < a.M && ch < a.Cout) ? (unsigned)(((src_row(px) - r0) * ld + ch) * 2) : PG_OOB;
    glds16(r, lds + i * 1024, off);
  }
}

// LDS accumulator half of the wave's segment (0: the tile's first segment)
__device__ __forceinline__ int stats_rseg(const PgArgs& a, long long bpx, long long wave_px0) {
  if (a.seg_m <= 0) return 0;
  return (int)(wave_px0 / a.seg_m - bpx / a.seg_m);
}

// floats of the LDS statistics accumulator of a BCH-channel tile (+ counter)
template <int BCH>
constexpr int pg_red_bytes() {
  return 2 * 3 * BCH * 4 + 16;
}

// Epilogue of one output tile straight from the accumulators: lane (fr, fq)
// holds, per channel pair p and pixel tile j, channels ch0..ch0+7 of pixel px,
// stored as one 16-B bf16 vector.  Optional, in this order: forward BN
// statistics (sum, sum of squares of the f32 result), residual add (dgrad:
// res_mode 1 / 2), fused BN-backward reduction (dgrad, a.bnb): the result d is
// the gradient at a BN+ReLU output, g = d * relu-mask is stored instead and
// sum g, sum g*xhat_t (xhat_t = (y_t - mean_t) * istd_t) are accumulated for
// up to two BN inputs t sharing g (models.py:234 bn3 + downsample BN).  The
// per-lane sums are reduced over the 16 pixel lanes by DPP and added to the
// tile's LDS accumulator (stats_flush writes it out).
template <bool BNB, int BCH, int MTC, int NTP, int WTPX, int WTCH, int EJB = 2>
__device__ __forceinline__ void pg_epilogue(const PgArgs& a, const f32x4 (&acc)[MTC][NTP], long long bpx, int bch,
                                            int wpx, int wch, int fr, int fq, float* red,
                                            const EpiStage& sg = EpiStage{nullptr, nullptr, nullptr, nullptr}) {
  const int HoWo = a.Ho * a.Wo;
  const long long wpx0 = bpx + wpx * WTPX;
  float* rb = red + stats_rseg(a, bpx, wpx0) * 3 * BCH;
  // segment of the wave's pixels (a wave past the last pixel of a tail tile
  // stores nothing; clamp so its parameter loads stay inside the last segment)
  const long long wseg = a.seg_m > 0 ? (wpx0 < a.M ? wpx0 : a.M - 1) / a.seg_m : 0;
  const bool sums = BNB || a.stats != nullptr;
  const bool two = BNB && a.bnb_nt == 2;
#pragma unroll
  for (int p = 0; p < MTC / 2; ++p) {
    const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
    const bool chok = ch0 < a.Cout;
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; s3[e] = 0.f; }
    // every global load below is issued unconditionally from a clamped, valid
    // address (pixel / channel tails are masked at the store), so the loads of
    // a batch go out together and are waited for once, not one round trip each
    const int chc = chok ? ch0 : 0;
    // BN-backward per-channel constants: xhat_t = y * xa_t + xb_t; mask affine
    // xhat_t = (y - m_t) * xa_t (the mean subtracted first: f32-exact for |mean| >> std)
    float xa0[8], m0[8], xa1[8], m1[8], mm[8], ms[8], mh[8];
    if constexpr (BNB) {
      if (sg.prm) {  // the tile's constants in LDS (pg_prm_fill)
        const float* pp = sg.prm + (int)(wseg - sg.seg0) * PG_PRM_ROWS * BCH + (chc - bch);
        loadf8v(pp, xa0);
        loadf8v(pp + BCH, m0);
        loadf8v(pp + 2 * BCH, xa1);
        loadf8v(pp + 3 * BCH, m1);
        loadf8v(pp + 4 * BCH, mm);
        loadf8v(pp + 5 * BCH, ms);
        loadf8v(pp + 6 * BCH, mh);
      } else {
        const long long po = wseg * a.bnb_pstride + chc;
        loadf8v(a.bnb_istd[0] + po, xa0);
        loadf8v(a.bnb_mean[0] + po, m0);
        if (two) {
          loadf8v(a.bnb_istd[1] + po, xa1);
          loadf8v(a.bnb_mean[1] + po, m1);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) { xa1[e] = 0.f; m1[e] = 0.f; }
        }
        if (a.bnb == 1) {  // parameter block of the BN feeding the ReLU: mean, -, scale, beta
          loadf8v(a.bnb_mbn + po, mm);
          loadf8v(a.bnb_mbn + po + 2 * a.Cout, ms);
          loadf8v(a.bnb_mbn + po + 3 * a.Cout, mh);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) { mm[e] = 0.f; ms[e] = 0.f; mh[e] = 0.f; }
        }
      }
    }
    // pixel tiles in batches of EJ: loads of the batch first, then the math
    constexpr int EJ = NTP >= EJB ? EJB : 1;
#pragma unroll
    for (int j0 = 0; j0 < NTP; j0 += EJ) {
      Vec16<bf16> rv[EJ], y0v[EJ], mkv[EJ], y1v[EJ];
      unsigned mbits[EJ];
      float rsc[EJ];
#pragma unroll
      for (int u = 0; u < EJ; ++u) {
        const long long px = wpx0 + (j0 + u) * 16 + fr;
        const long long pc = px < a.M ? px : a.M - 1;
        const int srow = (int)(pc - bpx), schunk = chok ? (chc - bch) >> 3 : 0;  // staged-operand coordinates
        rsc[u] = a.res_mode == 2 ? 0.25f : 1.f;
        if (a.res_mode) {
          if (sg.res) {
            rv[u] = stg_read<BCH>(sg.res, srow, schunk);
          } else {
            long long ri = pc;
            if (a.res_mode == 2) {
              const long long img = pc / HoWo;
              const int rem = (int)(pc - img * HoWo);
              const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
              ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
            }
            rv[u] = ld16<bf16>(reinterpret_cast<const bf16*>(a.res) + ri * a.ldy + chc);
          }
        }
        if constexpr (BNB) {
          const long long off = pc * a.ldy + chc;
          y0v[u] = sg.y0 ? stg_read<BCH>(sg.y0, srow, schunk)
                         : ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[0]) + off);
          if (a.bnb == 2)
            mkv[u] = sg.mk ? stg_read<BCH>(sg.mk, srow, schunk)
                           : ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_mask) + off);
          if (a.bnb == 3)
            mbits[u] = sg.bits ? sg.bits[srow * (BCH / 8) + schunk]
                               : reinterpret_cast<const unsigned char*>(a.bnb_mask)[pc * (a.Cout >> 3) + (chc >> 3)];
          if (two)
            y1v[u] = sg.y1 ? stg_read<BCH>(sg.y1, srow, schunk)
                           : ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[1]) + off);
        }
      }
#pragma unroll
      for (int u = 0; u < EJ; ++u) {
        const int j = j0 + u;
        const long long px = wpx0 + j * 16 + fr;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][j][r]; v[4 + r] = acc[2 * p + 1][j][r]; }
        if (px < a.M && chok) {
          if (!BNB && a.stats) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
          }
          if (a.res_mode) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += rsc[u] * to_f(rv[u].v[e]);
          }
          if constexpr (!BNB) {
            if (a.bias) {  // (per BN segment for a folded BatchNorm backward)
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += a.bias[wseg * a.bias_sstride + ch0 + e];
            }
            if (a.relu) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
            }
          }
          if constexpr (BNB) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float yv = to_f(y0v[u].v[e]);
              const bool keep = a.bnb == 1   ? (yv - mm[e]) * ms[e] + mh[e] > 0.f
                                : a.bnb == 3 ? ((mbits[u] >> e) & 1u) != 0u
                                             : to_f(mkv[u].v[e]) > 0.f;
              v[e] = keep ? v[e] : 0.f;
              s1[e] += v[e];
              s2[e] += v[e] * ((yv - m0[e]) * xa0[e]);
            }
            if (two) {
#pragma unroll
              for (int e = 0; e < 8; ++e) s3[e] += v[e] * ((to_f(y1v[u].v[e]) - m1[e]) * xa1[e]);
            }
          }
          Vec16<bf16> o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o.v[e] = from_f<bf16>(v[e]);
          st16<bf16>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0, o);
        }
      }
    }
    if (sums) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = dpp_row_sum(s1[e]); s2[e] = dpp_row_sum(s2[e]); }
      if (two) {
#pragma unroll
        for (int e = 0; e < 8; ++e) s3[e] = dpp_row_sum(s3[e]);
      }
      if (fr == 15 && chok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          atomicAdd(rb + (ch0 - bch) + e, s1[e]);
          atomicAdd(rb + BCH + (ch0 - bch) + e, s2[e]);
        }
        if (two) {
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(rb + 2 * BCH + (ch0 - bch) + e, s3[e]);
        }
      }
    }
  }
}

// d/dx [x sigmoid(1.702 x)] (models.py:391-393), as vit.hip's quickgelu_bwd
__device__ __forceinline__ float pg_quickgelu_grad(float x) {
  const float sg = 1.f / (1.f + __expf(-1.702f * x));
  return sg + 1.702f * x * sg * (1.f - sg);
}

// ---- epilogue operands prefetched into registers (PF variants): every lane
// issues the global loads of its own epilogue operands (residual, y_0, mask
// bits, y_1 — the same addresses pg_epilogue_k reads) BEFORE the main loop, so
// their latency runs under the tile's K-steps instead of as a separate
// round trip after them.  They are older than the stage loads, so the manual
// vmcnt counting of the stages only waits for them once (at the first stage).
template <int NP, int NTP>
struct EpiRegs {
  Vec16<bf16> rv[NP][NTP], y0v[NP][NTP], y1v[NP][NTP];
  unsigned mb[NP][NTP];
};

template <int BK, bool TWO, int MTC, int NTP, int WTPX, int WTCH>
__device__ __forceinline__ void epi_prefetch(const PgArgs& a, EpiRegs<MTC / 2, NTP>& er, long long bpx, int bch,
                                             int wpx, int wch, int fr, int fq) {
  constexpr bool RESK = BK == 2 || BK == 3;
  const int HoWo = a.Ho * a.Wo;
  const long long wpx0 = bpx + wpx * WTPX;
  const bool res = RESK || (BK == 0 && a.res_mode != 0);
#pragma unroll
  for (int p = 0; p < MTC / 2; ++p) {
    const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
    const int chc = ch0 < a.Cout ? ch0 : 0;
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const long long px = wpx0 + j * 16 + fr;
      const long long pc = px < a.M ? px : a.M - 1;
      if (res) {
        long long ri = pc;
        if (a.res_mode == 2) {
          const long long img = pc / HoWo;
          const int rem = (int)(pc - img * HoWo);
          const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
          ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
        }
        er.rv[p][j] = ld16<bf16>(reinterpret_cast<const bf16*>(a.res) + ri * a.ldy + chc);
      }
      if constexpr (BK != 0) er.y0v[p][j] = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[0]) + pc * a.ldy + chc);
      if constexpr (BK == 3)
        er.mb[p][j] = reinterpret_cast<const unsigned char*>(a.bnb_mask)[pc * (a.Cout >> 3) + (chc >> 3)];
      if constexpr (TWO) er.y1v[p][j] = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[1]) + pc * a.ldy + chc);
    }
  }
}

// The epilogue of pgemm_kernel, specialised at compile time on what the launch
// fuses (the generic pg_epilogue above decides per element at run time, which
// cost ~840 scalar branches in the unrolled epilogue and most of the fused
// kernels' time).  BK: 0 plain (forward statistics / data gradient, residual at
// run time), 1 ACT (mask (y_0 - m) * s + b > 0, no residual), 2 / 3 RES (block-
// output mask as bf16 / as bits, residual always present); TWO: a second BN
// target; S_RES / S_Y1 / S_MK: that operand is staged in LDS (else read from
// global memory in batches of EJB pixel tiles); y_0 and the mask bits of BK 3
// are always staged, the BN constants always come from the LDS table.
// FB: the per-segment bias of a folded BatchNorm backward (artsbir_conv1x1_dgrad_fold)
// is added to the accumulators first, before any mask / BN-backward reduction.
// FBL: that bias loaded per use (L1-resident) instead of held in 8 VGPRs across
// the pair's pixel tiles (the 8-wave 256 x 128 tile's 128-VGPR budget)
// PFN (BK 0, global residual / gate operand, one operand batch per channel pair):
// the next pair's operand loads are issued before this pair's arithmetic and
// stores, so a wave waits out one load round trip per tile instead of one per pair
template <int BK, bool TWO, bool S_RES, bool S_Y1, bool S_MK, int BCH, int MTC, int NTP, int WTPX, int WTCH,
          bool REG = false, int EJB = 2, bool GLB = false, bool FB = false, bool FBL = false, bool PFN = false>
__device__ __forceinline__ void pg_epilogue_k(const PgArgs& a, const f32x4 (&acc)[MTC][NTP], long long bpx, int bch,
                                              int wpx, int wch, int fr, int fq, float* red, const EpiStage& sg,
                                              const EpiRegs<MTC / 2, NTP>* er = nullptr) {
  constexpr bool BNB = BK != 0;
  constexpr bool RESK = BK == 2 || BK == 3;
  const int HoWo = a.Ho * a.Wo;
  const long long wpx0 = bpx + wpx * WTPX;
  float* rb = red + stats_rseg(a, bpx, wpx0) * 3 * BCH;
  const long long wseg = a.seg_m > 0 ? (wpx0 < a.M ? wpx0 : a.M - 1) / a.seg_m : 0;
  const bool sums = BNB || a.stats != nullptr;
  const bool res = RESK || (BK == 0 && a.res_mode != 0);
  const float rsc = a.res_mode == 2 ? 0.25f : 1.f;
  static_assert(!PFN || (BK == 0 && !REG && EJB >= NTP), "PFN: plain epilogue, one batch per pair");
  // PFN: the residual / gate operand rows of pair pp (the loads of the u loop below)
  auto pfn_load = [&](int pp, Vec16<bf16> (&dst)[NTP]) {
    const int c0 = bch + wch * WTCH + 32 * pp + 8 * fq;
    const int cc = c0 < a.Cout ? c0 : 0;
#pragma unroll
    for (int u = 0; u < NTP; ++u) {
      const long long px = wpx0 + u * 16 + fr;
      const long long pc = px < a.M ? px : a.M - 1;
      long long ri = pc;
      if (a.res_mode == 2) {
        const long long img = pc / HoWo;
        const int rem = (int)(pc - img * HoWo);
        const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
        ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
      }
      dst[u] = ld16<bf16>(reinterpret_cast<const bf16*>(a.res) + ri * a.ldy + cc);
    }
  };
  Vec16<bf16> pfn_next[PFN ? NTP : 1];
  if constexpr (PFN) {
    if (res) pfn_load(0, pfn_next);
  }
#pragma unroll
  for (int p = 0; p < MTC / 2; ++p) {
    const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
    const bool chok = ch0 < a.Cout;
    const int chc = chok ? ch0 : 0;
    const int schunk = chok ? (ch0 - bch) >> 3 : 0;
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; s3[e] = 0.f; }
    float fbias[FB && !FBL ? 8 : 1];
    if constexpr (FB && !FBL) loadf8v(a.bias + wseg * a.bias_sstride + chc, fbias);
    // BN constants (LDS table): xhat_t = (y - m_t) * xa_t; ACT mask (y - mm) * ms + mh > 0
    float xa0[8], m0[8], xa1[8], m1[8], mm[8], ms[8], mh[8];
    if constexpr (BNB && GLB) {  // the same rows pg_prm_fill tabulates, straight from the (L2-resident) vectors
      const long long po = wseg * a.bnb_pstride + chc;
      loadf8v(a.bnb_istd[0] + po, xa0);
      loadf8v(a.bnb_mean[0] + po, m0);
      if constexpr (TWO) { loadf8v(a.bnb_istd[1] + po, xa1); loadf8v(a.bnb_mean[1] + po, m1); }
      if constexpr (BK == 1) {
        loadf8v(a.bnb_mbn + po, mm);
        loadf8v(a.bnb_mbn + 2 * a.Cout + po, ms);
        loadf8v(a.bnb_mbn + 3 * a.Cout + po, mh);
      }
    } else if constexpr (BNB) {
      const float* pp = sg.prm + (int)(wseg - sg.seg0) * PG_PRM_ROWS * BCH + (chc - bch);
      loadf8v(pp, xa0);
      loadf8v(pp + BCH, m0);
      if constexpr (TWO) { loadf8v(pp + 2 * BCH, xa1); loadf8v(pp + 3 * BCH, m1); }
      if constexpr (BK == 1) { loadf8v(pp + 4 * BCH, mm); loadf8v(pp + 5 * BCH, ms); loadf8v(pp + 6 * BCH, mh); }
    }
    constexpr bool GLOBAL_OPS = !REG && (GLB || (RESK && !S_RES) || (TWO && !S_Y1) || (BK == 2 && !S_MK) || BK == 0);
    constexpr int EJ = (GLOBAL_OPS && NTP >= EJB) ? EJB : 1;
#pragma unroll
    for (int jj = 0; jj < NTP; jj += EJ) {
      // GLB: odd channel pairs walk the pixel tiles backwards, so the lines whose
      // first 64-B half the previous pair read last are re-read first (still in L2)
      const int j0 = (GLB && PG_SNAKE && (p & 1)) ? NTP - EJ - jj : jj;
      Vec16<bf16> rv[EJ], y0v[EJ], mkv[EJ], y1v[EJ];
      unsigned mbits[EJ];
      if constexpr (PFN) {
        if (res) {
#pragma unroll
          for (int u = 0; u < EJ; ++u) rv[u] = pfn_next[u];
          if (p + 1 < MTC / 2) pfn_load(p + 1, pfn_next);
        }
      }
#pragma unroll
      for (int u = 0; u < EJ; ++u) {  // operands of the batch (global loads issued together)
        if constexpr (PFN) continue;  // taken above
        if constexpr (REG) {  // prefetched before the main loop (epi_prefetch)
          rv[u] = er->rv[p][j0 + u];
          y0v[u] = er->y0v[p][j0 + u];
          y1v[u] = er->y1v[p][j0 + u];
          mbits[u] = er->mb[p][j0 + u];
          continue;
        }
        const long long px = wpx0 + (j0 + u) * 16 + fr;
        const long long pc = px < a.M ? px : a.M - 1;
        const int srow = (int)(pc - bpx);
        if (RESK || BK == 0) {
          if (S_RES && RESK) {
            rv[u] = stg_read<BCH>(sg.res, srow, schunk);
          } else if (BK == 0 && sg.res) {  // plain data gradient: residual staged at run time
            rv[u] = stg_read<BCH>(sg.res, srow, schunk);
          } else if (res) {
            long long ri = pc;
            if (a.res_mode == 2) {
              const long long img = pc / HoWo;
              const int rem = (int)(pc - img * HoWo);
              const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
              ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
            }
            rv[u] = ld16<bf16>(reinterpret_cast<const bf16*>(a.res) + ri * a.ldy + chc);
          }
        }
        if constexpr (BNB) {
          if constexpr (GLB) y0v[u] = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[0]) + pc * a.ldy + chc);
          else y0v[u] = stg_read<BCH>(sg.y0, srow, schunk);
          if constexpr (BK == 2)
            mkv[u] = S_MK ? stg_read<BCH>(sg.mk, srow, schunk)
                          : ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_mask) + pc * a.ldy + chc);
          if constexpr (BK == 3) {
            if constexpr (GLB) mbits[u] = reinterpret_cast<const unsigned char*>(a.bnb_mask)[pc * (a.Cout >> 3) + (chc >> 3)];
            else mbits[u] = sg.bits[srow * (BCH / 8) + schunk];
          }
          if constexpr (TWO)
            y1v[u] = S_Y1 ? stg_read<BCH>(sg.y1, srow, schunk)
                          : ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[1]) + pc * a.ldy + chc);
        }
      }
#pragma unroll
      for (int u = 0; u < EJ; ++u) {
        const long long px = wpx0 + (j0 + u) * 16 + fr;
        const bool ok = px < a.M && chok;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][j0 + u][r]; v[4 + r] = acc[2 * p + 1][j0 + u][r]; }
        if constexpr (FB && FBL) {
          float fb[8];
          loadf8v(a.bias + wseg * a.bias_sstride + chc, fb);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += fb[e];
        } else if constexpr (FB) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += fbias[e];
        }
        if (BK == 0 && a.res_mode == 3) {  // gate: the QuickGELU backward at the pre-activation in the res slot
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= pg_quickgelu_grad(to_f(rv[u].v[e]));
        } else if (RESK || (BK == 0 && res)) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += rsc * to_f(rv[u].v[e]);
        }
        if constexpr (BK == 0 && !FB) {
          if (a.bias) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += a.bias[chc + e];
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          }
        }
        if constexpr (BNB) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float yv = to_f(y0v[u].v[e]);
            bool keep;
            if constexpr (BK == 1) keep = (yv - mm[e]) * ms[e] + mh[e] > 0.f;
            else if constexpr (BK == 3) keep = ((mbits[u] >> e) & 1u) != 0u;
            else keep = to_f(mkv[u].v[e]) > 0.f;
            v[e] = (keep && ok) ? v[e] : 0.f;  // tail rows/channels add nothing to the sums
            s1[e] += v[e];
            s2[e] += v[e] * ((yv - m0[e]) * xa0[e]);
            if constexpr (TWO) s3[e] += v[e] * ((to_f(y1v[u].v[e]) - m1[e]) * xa1[e]);
          }
        } else if (a.stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float w = ok ? v[e] : 0.f;
            s1[e] += w;
            s2[e] += w * w;
          }
        }
        if (ok) {
          Vec16<bf16> o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o.v[e] = from_f<bf16>(v[e]);
#ifndef PG_NT_STORE
// the global-operand (GLB) epilogues store their output non-temporally: the
// lines are not allocated in L2, so the residual / BN-target operand lines the
// next channel pair reads stay resident (read bytes -15 %, C2 step -0.6 to
// -0.8 ms; tools/gpu/r4_ntst.sh, r4_ntst_step.sh, profiles/r4_nt_stores.txt)
#define PG_NT_STORE 1
#endif
          if (PG_NT_STORE && GLB) {
            typedef __attribute__((ext_vector_type(4))) unsigned pg_u4;
            __builtin_nontemporal_store(*reinterpret_cast<const pg_u4*>(&o),
                                        reinterpret_cast<pg_u4*>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0));
          } else
            st16<bf16>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0, o);
        }
      }
    }
    if (sums && !(a.dbg & 2)) {  // dbg 2: timing experiment without the statistics reduction
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = dpp_row_sum(s1[e]); s2[e] = dpp_row_sum(s2[e]); }
      if constexpr (TWO) {
#pragma unroll
        for (int e = 0; e < 8; ++e) s3[e] = dpp_row_sum(s3[e]);
      }
      if (fr == 15 && chok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          atomicAdd(rb + (ch0 - bch) + e, s1[e]);
          atomicAdd(rb + BCH + (ch0 - bch) + e, s2[e]);
          if constexpr (TWO) atomicAdd(rb + 2 * BCH + (ch0 - bch) + e, s3[e]);
        }
      }
    }
  }
}

// The global-operand (GLB) form of pg_epilogue_k with the loops turned round:
// pixel tile j outside, channel pair p inside, so a lane reads the two 64-B
// halves of each 128-B residual / BN-target / mask line (pairs p = 0, 1 of the
// wave's 64 channels) one right after the other.  pg_epilogue_k walks all the
// wave's pixel tiles for pair 0 before pair 1, and at every L2 read request
// being 128 B the line is often evicted in between and fetched twice (the
// 1.3x traffic of the fused BN-backward dgrads).  The per-pair
// statistics stay in registers across the tiles (SP: both pairs) or, when the
// register budget does not hold them, are reduced per (tile, pair).  The BN
// constants come from the LDS table prm (pg_prm_fill, in the stage ring the
// main loop has left) per use.
template <int BK, bool TWO, int BCH, int MTC, int NTP, int WTPX, int WTCH, bool FB, bool SP, bool TBL>
__device__ __forceinline__ void pg_epilogue_glb(const PgArgs& a, const f32x4 (&acc)[MTC][NTP], long long bpx, int bch,
                                                int wpx, int wch, int fr, int fq, float* red, const float* prm,
                                                long long seg0) {
  constexpr bool BNB = BK != 0;
  constexpr bool RESK = BK == 2 || BK == 3;
  constexpr int NP = MTC / 2;
  const int HoWo = a.Ho * a.Wo;
  const long long wpx0 = bpx + wpx * WTPX;
  float* rb = red + stats_rseg(a, bpx, wpx0) * 3 * BCH;
  const long long wseg = a.seg_m > 0 ? (wpx0 < a.M ? wpx0 : a.M - 1) / a.seg_m : 0;
  const bool sums = (BNB || a.stats != nullptr) && !(a.dbg & 2);
  const bool res = RESK || (BK == 0 && a.res_mode != 0);
  const float rsc = a.res_mode == 2 ? 0.25f : 1.f;
  // BN constants: rows of the LDS table (TBL) or the parameter vectors; + channel
  const long long po0 = wseg * a.bnb_pstride;
  const float* tp = prm + (int)(wseg - seg0) * PG_PRM_ROWS * BCH - bch;
  const float* r_is0 = TBL ? tp : a.bnb_istd[0] + po0;
  const float* r_m0 = TBL ? tp + BCH : a.bnb_mean[0] + po0;
  float sa[SP ? NP : 1][8], sb[SP ? NP : 1][8], sc[SP && TWO ? NP : 1][8];
  if constexpr (SP) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) { sa[p][e] = 0.f; sb[p][e] = 0.f; if constexpr (TWO) sc[p][e] = 0.f; }
  }
  // reduce a pair's 16 pixel lanes (DPP) and add them into the block accumulator
  auto flush = [&](float (&s1)[8], float (&s2)[8], float (&s3)[8], int ch0, bool chok) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] = dpp_row_sum(s1[e]); s2[e] = dpp_row_sum(s2[e]); }
    if constexpr (TWO) {
#pragma unroll
      for (int e = 0; e < 8; ++e) s3[e] = dpp_row_sum(s3[e]);
    }
    if (fr == 15 && chok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(rb + (ch0 - bch) + e, s1[e]);
        atomicAdd(rb + BCH + (ch0 - bch) + e, s2[e]);
        if constexpr (TWO) atomicAdd(rb + 2 * BCH + (ch0 - bch) + e, s3[e]);
      }
    }
  };
#pragma unroll
  for (int j = 0; j < NTP; ++j) {
    const long long px = wpx0 + j * 16 + fr;
    const long long pc = px < a.M ? px : a.M - 1;
    long long ri = pc;
    if (res && a.res_mode == 2) {
      const long long img = pc / HoWo;
      const int rem = (int)(pc - img * HoWo);
      const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
      ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
      const bool chok = ch0 < a.Cout;
      const int chc = chok ? ch0 : 0;
      const bool ok = px < a.M && chok;
      // operands of (tile j, pair p): the loads of pair p + 1 follow right after
      Vec16<bf16> rv, y0v, mkv, y1v;
      unsigned mbits = 0;
      if (res) rv = ld16<bf16>(reinterpret_cast<const bf16*>(a.res) + ri * a.ldy + chc);
      if constexpr (BNB) {
        y0v = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[0]) + pc * a.ldy + chc);
        if constexpr (BK == 2) mkv = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_mask) + pc * a.ldy + chc);
        if constexpr (BK == 3) mbits = reinterpret_cast<const unsigned char*>(a.bnb_mask)[pc * (a.Cout >> 3) + (chc >> 3)];
        if constexpr (TWO) y1v = ld16<bf16>(reinterpret_cast<const bf16*>(a.bnb_y[1]) + pc * a.ldy + chc);
      }
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][j][r]; v[4 + r] = acc[2 * p + 1][j][r]; }
      if constexpr (FB) {
        float fbias[8];
        loadf8v(a.bias + wseg * a.bias_sstride + chc, fbias);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += fbias[e];
      }
      if (BK == 0 && a.res_mode == 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= pg_quickgelu_grad(to_f(rv.v[e]));
      } else if (res) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rsc * to_f(rv.v[e]);
      }
      if constexpr (BK == 0 && !FB) {
        if (a.bias) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += a.bias[chc + e];
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
      }
      float t1[8], t2[8], t3[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { t1[e] = 0.f; t2[e] = 0.f; t3[e] = 0.f; }
      if constexpr (BNB) {
        float xa0[8], m0[8];
        loadf8v(r_is0 + chc, xa0);
        loadf8v(r_m0 + chc, m0);
        float mm[BK == 1 ? 8 : 1], ms[BK == 1 ? 8 : 1], mh[BK == 1 ? 8 : 1];
        if constexpr (BK == 1) {
          loadf8v((TBL ? tp + 4 * BCH : a.bnb_mbn + po0) + chc, mm);
          loadf8v((TBL ? tp + 5 * BCH : a.bnb_mbn + 2 * a.Cout + po0) + chc, ms);
          loadf8v((TBL ? tp + 6 * BCH : a.bnb_mbn + 3 * a.Cout + po0) + chc, mh);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float yv = to_f(y0v.v[e]);
          bool keep;
          if constexpr (BK == 1) keep = (yv - mm[e]) * ms[e] + mh[e] > 0.f;
          else if constexpr (BK == 3) keep = ((mbits >> e) & 1u) != 0u;
          else keep = to_f(mkv.v[e]) > 0.f;
          v[e] = (keep && ok) ? v[e] : 0.f;  // tail rows/channels add nothing to the sums
          t1[e] = v[e];
          t2[e] = v[e] * ((yv - m0[e]) * xa0[e]);
        }
        if constexpr (TWO) {
          float xa1[8], m1[8];
          loadf8v((TBL ? tp + 2 * BCH : a.bnb_istd[1] + po0) + chc, xa1);
          loadf8v((TBL ? tp + 3 * BCH : a.bnb_mean[1] + po0) + chc, m1);
#pragma unroll
          for (int e = 0; e < 8; ++e) t3[e] = v[e] * ((to_f(y1v.v[e]) - m1[e]) * xa1[e]);
        }
      } else if (a.stats) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float w = ok ? v[e] : 0.f;
          t1[e] = w;
          t2[e] = w * w;
        }
      }
      if (ok) {
        Vec16<bf16> o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o.v[e] = from_f<bf16>(v[e]);
        typedef __attribute__((ext_vector_type(4))) unsigned pg_u4;
        __builtin_nontemporal_store(*reinterpret_cast<const pg_u4*>(&o),
                                    reinterpret_cast<pg_u4*>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0));
      }
      if (sums) {
        if constexpr (SP) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            sa[p][e] += t1[e];
            sb[p][e] += t2[e];
            if constexpr (TWO) sc[p][e] += t3[e];
          }
        } else {
          flush(t1, t2, t3, ch0, chok);
        }
      }
    }
  }
  if constexpr (SP) {
    if (sums) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
        if constexpr (TWO) {
          flush(sa[p], sb[p], sc[p], ch0, ch0 < a.Cout);
        } else {
          float unused[8];
          flush(sa[p], sb[p], unused, ch0, ch0 < a.Cout);
        }
      }
    }
  }
}

// ---- BN statistics carried across the tiles of a persistent workgroup.  A
// lane's channels (wch, p, fq) are the same in every tile of the workgroup that
// shares the tile's channel block bch, so the lane adds its pixels' y and y^2
// into registers tile after tile; only when the wave's (segment, bch) changes,
// and at the end, are the 16 pixel lanes reduced (DPP) and added to the global
// statistics slot.  Per tile that leaves 2 FMAs per output value instead of the
// DPP reduction, LDS atomics and the block flush of pg_epilogue.
template <int NP>
struct WaveStats {
  float s1[NP][8], s2[NP][8];
  int seg;  // -1: empty
  int bch;
};

template <int NP>
__device__ __forceinline__ void wstats_zero(WaveStats<NP>& w) {
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) { w.s1[p][e] = 0.f; w.s2[p][e] = 0.f; }
}

template <int NP, int WTCH>
__device__ __forceinline__ void wstats_flush(WaveStats<NP>& w, const PgArgs& a, int wch, int fr, int fq, int slot) {
  if (w.seg < 0) return;
  const long long so = (long long)w.seg * a.seg_stride + (long long)slot * 2 * a.Cout;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int ch0 = w.bch + wch * WTCH + 32 * p + 8 * fq;
#pragma unroll
    for (int e = 0; e < 8; ++e) { w.s1[p][e] = dpp_row_sum(w.s1[p][e]); w.s2[p][e] = dpp_row_sum(w.s2[p][e]); }
    if (fr == 15 && ch0 < a.Cout) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(a.stats + so + ch0 + e, w.s1[p][e]);
        atomicAdd(a.stats + so + a.Cout + ch0 + e, w.s2[p][e]);
      }
    }
  }
  wstats_zero(w);
  w.seg = -1;
}

// forward epilogue with carried statistics: store the tile, add its values to w
template <int BCH, int MTC, int NTP, int WTPX, int WTCH>
__device__ __forceinline__ void pg_epilogue_fwd(const PgArgs& a, const f32x4 (&acc)[MTC][NTP], long long bpx, int bch,
                                                int wpx, int wch, int fr, int fq, WaveStats<MTC / 2>& w, int slot) {
  const long long wpx0 = bpx + wpx * WTPX;
  if (wpx0 >= a.M) return;  // a wave past the last pixel of the tail tile
  const int seg = a.seg_m > 0 ? (int)(wpx0 / a.seg_m) : 0;
  if (seg != w.seg || bch != w.bch) {
    wstats_flush<MTC / 2, WTCH>(w, a, wch, fr, fq, slot);
    w.seg = seg;
    w.bch = bch;
  }
  // a.nts: non-temporal stores (no L2 allocation for the output lines); they
  // pay on the 28^2 .. 7^2 1x1 forwards (-10..-20 %), not at 56^2 (+8 %), so
  // the autotuner picks per shape (candidates 24 / 25, profiles/r5_fwd_stores.txt)
  constexpr int NP = MTC / 2;
  const bool nts = a.nts != 0;
#pragma unroll
  for (int it = 0; it < NP * NTP; ++it) {
    const int p = it / NTP, j = it % NTP;
    const int ch0 = bch + wch * WTCH + 32 * p + 8 * fq;
    const bool chok = ch0 < a.Cout;
    const long long px = wpx0 + j * 16 + fr;
    const bool ok = px < a.M && chok;
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][j][r]; v[4 + r] = acc[2 * p + 1][j][r]; }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float u = ok ? v[e] : 0.f;
      w.s1[p][e] += u;
      w.s2[p][e] += u * u;
    }
    if (ok) {
      Vec16<bf16> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o.v[e] = from_f<bf16>(v[e]);
      if (nts) {
        typedef __attribute__((ext_vector_type(4))) unsigned pg_u4;
        __builtin_nontemporal_store(*reinterpret_cast<const pg_u4*>(&o),
                                    reinterpret_cast<pg_u4*>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0));
      } else {
        st16<bf16>(reinterpret_cast<bf16*>(a.y) + px * a.ldy + ch0, o);
      }
    }
  }
}

// transposed 16-column fragment of a 64-k stage image (rows of 128 B, chunk
// slot = chunk ^ (row & 7)): for the MFMA operand whose reduction runs over the
// image's rows (pixels).  Lane 4q + p of 16-lane group g addresses row 8g + q
// (+4 for the second read) of the 32-row block, columns 16 c0 + 4p .. + 3
// (T10); lane (g, t) receives column 16 c0 + t of rows 8g .. 8g + 7.
typedef short pg_v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) pg_v4s_t* pg_lds_v4s_t;
__device__ __forceinline__ int pg_tr_off(int g, int q, int p, int c0, int h) {
  const int row = 8 * g + q + 4 * h;
  return row * 128 + (((2 * c0 + (p >> 1)) ^ (q + 4 * h)) << 4) + 8 * (p & 1);
}
__device__ __forceinline__ bf16x8 pg_tr_frag(const char* base, int off_lo, int off_hi) {
  const pg_v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (pg_lds_v4s_t)(const __attribute__((address_space(3))) void*)(base + off_lo));
  const pg_v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (pg_lds_v4s_t)(const __attribute__((address_space(3))) void*)(base + off_hi));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Loader waves of the fold data gradient that also accumulate its weight-gradient
// operands (the backward of models.py:219-220 conv3 -> bn3 and 227-229 downsample
// conv -> BN, folded as in fold.hip): besides streaming the stages they compute,
// from the same LDS images, Q[k][co] = sum over the tile's pixels of
// [g | x][m][k] * x[m][co] — g^T x (k < C1) and the Gram matrix x^T x — so the
// weight gradient never reads g and x again.  The layer has one 64-channel block
// (Cout == 64, K == WGK); the stage order of a tile puts the x chunk first, each
// wave keeps the transposed x fragments of its 16 channels in registers for the
// tile and Q (K x 16, f32) for as long as its tiles stay in one BN segment, then
// adds it into wg_p / wg_gram with f32 atomics.  1x1 stride 1, M a whole number
// of 256-pixel tiles (a.seg_m too), so no pixel row is ever out of range.
template <int BCH, int NSTAGE, int LPX, int LCH, int STAGE, int PXB, int WGK>
__device__ __forceinline__ void pstream_wg_loader(const PgArgs& a, char* smem, int lw, int lane, int G, int bslot,
                                                  int nk, int total) {
  static_assert(BCH == 64 && WGK % 64 == 0 && WGK > 64, "one 64-channel block, K = C1 + 64");
  constexpr int NWL = 4, NKC = WGK / 64, NQ = WGK / 16, C1 = WGK - 64;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int csrc = lslot ^ lrow;
  // DMA source offsets of this lane's row of instruction u (row = 32 u + 8 lw + lrow)
  const int r0 = 8 * lw + lrow;
  const unsigned gofs = (unsigned)(r0 * a.sW * 2 + csrc * 16), gstep = (unsigned)(32 * a.sW * 2);
  const unsigned xofs = (unsigned)(r0 * a.sW2 * 2 + csrc * 16), xstep = (unsigned)(32 * a.sW2 * 2);
  // weight rows of instruction u: pg_perm(32 u + 8 lw + lrow) = 32 u + pg_perm(8 lw + lrow)
  const unsigned woff = (unsigned)(pg_perm(8 * lw + lrow) * a.K * 2 + csrc * 16), wstep = (unsigned)(32 * a.K * 2);
  // tiles per BN segment (uniform, 32-bit: segments by scalar division)
  const int tps = __builtin_amdgcn_readfirstlane(a.seg_m > 0 ? (int)(a.seg_m / 256) : 0x7fffffff);
  __amdgpu_buffer_rsrc_t gr = pg_rsrc(a.x, 0), xr = gr, wr = gr;
  auto issue = [&](int sidx) {
    const int i = sidx / nk, kt = sidx - i * nk;
    if (kt == 0) {
      const int tile = i * G + bslot;
      const long long bpx = (long long)tile * 256;
      const int sg = tile / tps;
      gr = pg_rsrc(reinterpret_cast<const bf16*>(a.x) + bpx * a.sW, (a.M - bpx) * a.sW * 2);
      xr = pg_rsrc(reinterpret_cast<const bf16*>(a.x2) + bpx * a.sW2, (a.M - bpx) * a.sW2 * 2);
      wr = pg_rsrc(reinterpret_cast<const bf16*>(a.w) + sg * a.w_sstride, (long long)a.Cout * a.K * 2);
    }
    const int kofs = kt == 0 ? C1 : (kt - 1) * 64;  // the x chunk first
    char* pxs = smem + (sidx % NSTAGE) * STAGE;
    char* chs = pxs + PXB;
#pragma unroll
    for (int u = 0; u < LPX; ++u) {
      if (kt == 0) glds16_so(xr, pxs + (u * NWL + lw) * 1024, xofs, u * xstep);
      else glds16_so(gr, pxs + (u * NWL + lw) * 1024, gofs, u * gstep + kofs * 2);
    }
#pragma unroll
    for (int u = 0; u < LCH; ++u) glds16_so(wr, chs + (u * NWL + lw) * 1024, woff, u * wstep + kofs * 2);
  };
  // MFMA operand fragments: lane (g, t = 4q + p)
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  // column block c of a read is off(c = 0) ^ (c << 5): the chunk XOR of the
  // image touches bits 4-6 only
  const int alo = pg_tr_off(g, q, p, 0, 0), ahi = pg_tr_off(g, q, p, 0, 1);
  f32x4 qacc[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) qacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 xf[8];
  int cur_seg = -1;
  // Q rows k = 16 j + 4 g + r, column co = 16 lw + t (row stride Cout = 64)
  auto flush = [&]() {
    // uniform segment bases (SGPRs) + one 32-bit lane offset
    float* P = a.wg_p + (long long)cur_seg * C1 * 64;
    float* Gm = a.wg_gram + (long long)cur_seg * 64 * 64;
    const int lo = 4 * g * 64 + 16 * lw + t;
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      __builtin_amdgcn_sched_barrier(0);  // one 16-row block of addresses at a time
      float* dst = (16 * j < C1) ? P + (lo + 16 * j * 64) : Gm + (lo + (16 * j - C1) * 64);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        atomicAdd(dst + r * 64, qacc[j][r]);
        qacc[j][r] = 0.f;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto wgrad = [&](int s) {
    const int i = s / nk, kt = s - i * nk;
    const char* pxs = smem + (s % NSTAGE) * STAGE;
    if (kt == 0) {
      // this wave's 16 channels of the x chunk (recomputed here, not held across the loop)
      int xlo, xhi;
      asm volatile("v_xor_b32 %0, %1, %2" : "=v"(xlo) : "v"(alo), "s"(lw << 5));
      asm volatile("v_xor_b32 %0, %1, %2" : "=v"(xhi) : "v"(ahi), "s"(lw << 5));
#pragma unroll
      for (int kp = 0; kp < 8; ++kp) xf[kp] = pg_tr_frag(pxs + kp * 4096, xlo, xhi);
    }
    const int kc = kt == 0 ? NKC - 1 : kt - 1;  // the stage's 64 rows of Q
#pragma unroll
    for (int c = 0; c < NKC; ++c) {
      if (c != kc) continue;
#pragma unroll
      for (int kp = 0; kp < 8; ++kp) {
        // one 32-pixel step at a time: 4 fragments live (the register budget of
        // 3 waves per SIMD holds Q, the x fragments and no more)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
          // fragment offsets recomputed per use (asm volatile: not hoisted out of
          // the loop, where the register allocator would spill them)
          int o[4];
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o[0]) : "v"(alo), "s"(jp << 5));
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o[1]) : "v"(ahi), "s"(jp << 5));
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o[2]) : "v"(alo), "s"((jp + 1) << 5));
          asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o[3]) : "v"(ahi), "s"((jp + 1) << 5));
          const bf16x8 a0 = pg_tr_frag(pxs + kp * 4096, o[0], o[1]);
          const bf16x8 a1 = pg_tr_frag(pxs + kp * 4096, o[2], o[3]);
          qacc[4 * c + jp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, xf[kp], qacc[4 * c + jp], 0, 0, 0);
          qacc[4 * c + jp + 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, xf[kp], qacc[4 * c + jp + 1], 0, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  constexpr int LPS = LPX + LCH;
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
    if (s % nk == 0) {  // a new tile: flush Q when it starts another BN segment
      const int sg = ((s / nk) * G + bslot) / tps;
      if (sg != cur_seg) {
        if (cur_seg >= 0) {
          flush();
          vm_wait<0>();  // the atomics and the stage in flight: the counted waits below see only DMA
        }
        cur_seg = sg;
      }
    }
    if (s + NSTAGE - 1 < total) issue(s + NSTAGE - 1);
    wgrad(s);
    if (s + 1 < total) {
      int ahead = total - 2 - s;
      if (ahead > NSTAGE - 2) ahead = NSTAGE - 2;
      wait_stages<LPS, NSTAGE>(ahead);
    }
  }
  if (cur_seg >= 0) flush();
}


}  // namespace artsbir
