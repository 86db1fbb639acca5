// Streaming data gradient of a Bottleneck's first 1x1 conv with the block-input
// BatchNorm backward fused in (gfx950).  Reference: models.py:198 conv1 of
// Bottleneck, whose input gradient meets the residual branch (models.py:234
// out += identity) and the ReLU / BatchNorm of the block before it (bn3 and the
// downsample BN, models.py:220, 229), all differentiated by autograd.
//
//   dx[m][c] = sum_k dy[m][k] W[k][c] + residual,  g = dx * relu-mask,
//   slots_t += (sum g, sum g * xhat_t)  per channel and BN segment
//
// with K (the conv's 64 or 128 output channels) tiny against the C = 256 / 512
// channels of dx, so the launch is a byte stream — dy, the residual, one or two
// BN inputs y_t and the mask in, dx out — with a small GEMM in front.  The
// tiled kernels (pgemm_kernel GLB, one output tile per workgroup) issue the
// epilogue's operand loads one (pixel tile, channel pair) batch at a time after
// a 2-4-step main loop and sat at ~3.7 TB/s in the C2 step against 5.3 TB/s for
// the pure streaming passes (profiles/r6_trace_gaps.txt).  Here:
//  * a workgroup of 4 waves owns 256 channels (64 per wave) and walks a
//    contiguous range of RS_CHUNK 16-pixel blocks; its W slice stays in LDS (XOR-
//    swizzled rows, channel order permuted so a lane's MFMA outputs are 8
//    consecutive channels: pg_perm), read once;
//  * each wave issues ALL loads of a block at once — the dy B fragments straight
//    from global memory into registers first, then the residual, y_t and mask —
//    one block ahead (software pipeline over two operand sets), so a block's
//    MFMAs and epilogue run while the next block's ~8-12 KB per wave are in
//    flight (no LDS staging, no barrier in the loop);
//  * the BN-backward sums stay in registers across blocks and are reduced (DPP)
//    and flushed with global atomics only when the BN segment changes.
#include "common.h"
#include "pgemm.h"
#include "pgemm_dev.h"

namespace artsbir {

constexpr int RS_TC = 256;    // channels per workgroup (4 waves x 64)
// MFMA pixel groups of 16 per wave step: one, so that two steps' operands fit the
// registers beside the carried BN sums (two groups with the next step's loads in
// flight spilled 300-900 B per lane)
constexpr int RS_NJ = 1;
constexpr int RS_WP = 16 * RS_NJ;  // pixels per wave step
constexpr int RS_NSEG = 4;    // BN segments whose constants fit the LDS table
constexpr int RS_CHUNK = 32;  // 16-pixel blocks per workgroup

// LDS chunk slot of 16-B chunk c of W row rho (K / 8 chunks per row):
// conflict-free ds_read_b128 A fragments for 128-B (K 64) and 256-B (K 128) rows
template <int K>
__device__ __forceinline__ int rs_slot(int rho, int c) {
  return K == 64 ? (c ^ (rho & 7)) : (c ^ ((rho & 7) << 1));
}

template <int K, int BK, bool TWO>
__global__ void __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) rstream_kernel(PgArgs a, int chunk) {
  constexpr int CPR = K / 8;
  constexpr int NKS = K / 32;  // MFMA k-steps
  __shared__ __attribute__((aligned(16))) char wlds[RS_TC * K * 2];
  __shared__ __attribute__((aligned(16))) float prm[RS_NSEG][4][RS_TC];  // istd_0, mean_0, istd_1, mean_1

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int ncb = a.Cout / RS_TC;
  // the channel blocks of one pixel range run next to each other on one XCD
  // (their shared dy rows come from that XCD's L2)
  const long long lid = pg_xcd_remap(blockIdx.x, (long long)gridDim.x);
  const int cb = (int)(lid % ncb), grp = (int)(lid / ncb);
  const int bch = cb * RS_TC;
  const long long nblk = a.M / RS_WP;
  const long long b0 = (long long)grp * chunk, b1 = b0 + chunk < nblk ? b0 + chunk : nblk;
  const int nseg = a.seg_m > 0 ? (int)(a.M / a.seg_m) : 1;

  // ---- W slice (permuted rows) and the BN constants of every segment into LDS
  const bf16* wg = reinterpret_cast<const bf16*>(a.w);
  for (int i = tid; i < RS_TC * CPR; i += 256) {
    const int rho = i / CPR, c = i - (i / CPR) * CPR;
    const int ch = bch + pg_perm(rho);
    const uint4 v = *reinterpret_cast<const uint4*>(wg + (long long)ch * K + c * 8);
    *reinterpret_cast<uint4*>(wlds + (rho * CPR + rs_slot<K>(rho, c)) * 16) = v;
  }
  {
    // the source rows as wave-uniform pointers (a per-lane choice among the
    // fields of the by-value argument struct would copy it to scratch)
    const float* rows[4];
    rows[0] = reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_istd[0]));
    rows[1] = reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_mean[0]));
    rows[2] = TWO ? reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_istd[1])) : rows[0];
    rows[3] = TWO ? reinterpret_cast<const float*>(pg_uniform((long long)a.bnb_mean[1])) : rows[1];
#pragma unroll
    for (int s = 0; s < RS_NSEG; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = tid;  // 256 threads, 256 channels
        prm[s][q][c] = (s < nseg && (q < 2 || TWO)) ? rows[q][(long long)s * a.bnb_pstride + bch + c] : 0.f;
      }
  }
  __syncthreads();

  const int HoWo = a.Ho * a.Wo;
  const float rsc = a.res_mode == 2 ? 0.25f : 1.f;
  const int cw = bch + 64 * wid;  // the wave's first channel
  const int lc0 = 64 * wid + 8 * fq;  // the lane's channel offset in the block (pair p: + 32 p)
  const bf16* dyp = reinterpret_cast<const bf16*>(a.x);
  const bf16* resp = reinterpret_cast<const bf16*>(a.res);
  const bf16* y0p = reinterpret_cast<const bf16*>(a.bnb_y[0]);
  const bf16* y1p = reinterpret_cast<const bf16*>(TWO ? a.bnb_y[1] : a.bnb_y[0]);
  bf16* outp = reinterpret_cast<bf16*>(a.y);
  const long long C = a.Cout;
  // the argument fields the loop uses, as locals (the lambdas below must not
  // take the by-value kernel argument by reference: that copies it to scratch)
  float* const slots0 = a.bnb_slots[0];
  float* const slots1 = TWO ? a.bnb_slots[1] : a.bnb_slots[0];
  const void* const maskp = a.bnb_mask;
  const long long seg_m = a.seg_m, seg_stride = a.seg_stride;
  const int res_mode = a.res_mode, Ho = a.Ho, Wo = a.Wo;

  // A-fragment LDS addresses: row-tile i (0..3) of the wave, k-step s
  const char* arow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) arow[i] = wlds + (64 * wid + 16 * i + fr) * CPR * 16;
  const int rrho = fr;  // (64 wid + 16 i + fr) & 7 == fr & 7

  float s1[2][8], s2[2][8], s3[TWO ? 2 : 1][8];
  auto zero_sums = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[p][e] = 0.f;
        s2[p][e] = 0.f;
        if constexpr (TWO) s3[p][e] = 0.f;
      }
  };
  zero_sums();
  const int slot = (int)(lid % ARTSBIR_NSLOT);
  auto flush = [&](int seg) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[p][e] = dpp_row_sum(s1[p][e]);
        s2[p][e] = dpp_row_sum(s2[p][e]);
        if constexpr (TWO) s3[p][e] = dpp_row_sum(s3[p][e]);
      }
      if (fr == 15) {
        const long long so = (long long)seg * seg_stride + (long long)slot * 2 * C + cw + 32 * p + 8 * fq;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          atomicAdd(slots0 + so + e, s1[p][e]);
          atomicAdd(slots0 + so + C + e, s2[p][e]);
          if constexpr (TWO) {
            atomicAdd(slots1 + so + e, s1[p][e]);
            atomicAdd(slots1 + so + C + e, s3[p][e]);
          }
        }
      }
    }
    zero_sums();
  };

  // one block's operands (16 pixels): dy B fragments, residual, y_t, mask — two
  // sets, separate arrays (an operand struct passed by reference ended in scratch)
  // issue every load of block blk: dy fragments first (the MFMAs of the block
  // wait only for them), then the epilogue operands
  auto load = [&](long long blk, uint4 (&bq)[NKS], Vec16<bf16> (&rv)[2], Vec16<bf16> (&y0v)[2],
                  Vec16<bf16> (&y1v)[2], Vec16<bf16> (&mkv)[2], unsigned long long& mb) __attribute__((always_inline)) {
    const long long px = blk * RS_WP + fr;
#pragma unroll
    for (int s = 0; s < NKS; ++s) bq[s] = *reinterpret_cast<const uint4*>(dyp + px * (long long)K + 32 * s + 8 * fq);
    long long ri = px;
    if (res_mode == 2) {
      const long long img = px / HoWo;
      const int rem = (int)(px - img * HoWo);
      const int oh = rem / Wo, ow = rem - (rem / Wo) * Wo;
      ri = (img * (Ho / 2) + oh / 2) * (Wo / 2) + ow / 2;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = cw + 32 * p + 8 * fq;
      rv[p] = ld16<bf16>(resp + ri * C + ch);
      y0v[p] = ld16<bf16>(y0p + px * C + ch);
      if constexpr (TWO) y1v[p] = ld16<bf16>(y1p + px * C + ch);
      if constexpr (BK == 2) mkv[p] = ld16<bf16>(reinterpret_cast<const bf16*>(maskp) + px * C + ch);
    }
    if constexpr (BK == 3)  // the mask bits of the wave's 64 channels: 8 bytes
      mb = *reinterpret_cast<const unsigned long long*>(reinterpret_cast<const unsigned char*>(maskp) +
                                                        px * (C >> 3) + (cw >> 3));
  };
  auto step = [&](long long blk, const uint4 (&bq)[NKS], const Vec16<bf16> (&rv)[2], const Vec16<bf16> (&y0v)[2],
                  const Vec16<bf16> (&y1v)[2], const Vec16<bf16> (&mkv)[2], unsigned long long mb) __attribute__((always_inline)) {
    const long long px = blk * RS_WP + fr;
    const int seg = seg_m > 0 ? (int)(blk * RS_WP / seg_m) : 0;
    // ---- the GEMM: out^T[channel][pixel] on v_mfma_f32_16x16x32_bf16
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      uint4 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const uint4*>(arow[i] + rs_slot<K>(rrho, 4 * s + fq) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&af[i]),
                                                         *reinterpret_cast<const bf16x8*>(&bq[s]), acc[i], 0, 0, 0);
    }
    // ---- epilogue: residual, mask, BN-backward sums, 16-B stores
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      float is0[8], m0[8], is1[TWO ? 8 : 1], m1[TWO ? 8 : 1];
      loadf8v(&prm[seg][0][lc0 + 32 * p], is0);
      loadf8v(&prm[seg][1][lc0 + 32 * p], m0);
      if constexpr (TWO) {
        loadf8v(&prm[seg][2][lc0 + 32 * p], is1);
        loadf8v(&prm[seg][3][lc0 + 32 * p], m1);
      }
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[r] = acc[2 * p][r]; v[4 + r] = acc[2 * p + 1][r]; }
      const unsigned byte = BK == 3 ? (unsigned)(mb >> (8 * (4 * p + fq))) & 0xffu : 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] += rsc * to_f(rv[p].v[e]);
        bool keep;
        if constexpr (BK == 3) keep = ((byte >> e) & 1u) != 0u;
        else keep = to_f(mkv[p].v[e]) > 0.f;
        v[e] = keep ? v[e] : 0.f;
        s1[p][e] += v[e];
        s2[p][e] += v[e] * ((to_f(y0v[p].v[e]) - m0[e]) * is0[e]);
        if constexpr (TWO) s3[p][e] += v[e] * ((to_f(y1v[p].v[e]) - m1[e]) * is1[e]);
      }
      Vec16<bf16> ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov.v[e] = from_f<bf16>(v[e]);
      typedef __attribute__((ext_vector_type(4))) unsigned rs_u4;
      __builtin_nontemporal_store(*reinterpret_cast<const rs_u4*>(&ov),
                                  reinterpret_cast<rs_u4*>(outp + px * C + cw + 32 * p + 8 * fq));
    }
  };

  // software pipeline over the blocks: the next block's loads are in flight
  // while this one's MFMAs and epilogue run (two operand sets, unrolled by 2)
  int cur = -1;
  auto enter = [&](long long blk) __attribute__((always_inline)) {
    const int seg = seg_m > 0 ? (int)(blk * RS_WP / seg_m) : 0;
    if (seg != cur) {
      if (cur >= 0) flush(cur);
      cur = seg;
    }
  };
  uint4 bqa[NKS], bqb[NKS];
  Vec16<bf16> rva[2], rvb[2], y0a[2], y0b[2], y1a[2], y1b[2], mka[2], mkb[2];
  unsigned long long mba = 0, mbb = 0;
  if (b0 < b1) load(b0, bqa, rva, y0a, y1a, mka, mba);
  for (long long blk = b0; blk < b1; blk += 2) {
    if (blk + 1 < b1) load(blk + 1, bqb, rvb, y0b, y1b, mkb, mbb);
    enter(blk);
    step(blk, bqa, rva, y0a, y1a, mka, mba);
    if (blk + 1 >= b1) break;
    if (blk + 2 < b1) load(blk + 2, bqa, rva, y0a, y1a, mka, mba);
    enter(blk + 1);
    step(blk + 1, bqb, rvb, y0b, y1b, mkb, mbb);
  }
  if (cur >= 0) flush(cur);
}

// Candidate 26 of the data gradient: the RES kinds (2: bf16 mask, 3: mask bits)
// of a stride-1 1x1 conv with K = 64 or 128, C % 256 == 0, contiguous NHWC
// operands, whole 16-pixel blocks per BN segment, at most RS_NSEG segments
bool rstream_launch(const PgArgs& a, hipStream_t st) {
  if ((a.bnb != 2 && a.bnb != 3) || (a.bnb_nt != 1 && a.bnb_nt != 2)) return false;
  if (a.res_mode != 1 && a.res_mode != 2) return false;
  if (a.x2 || a.w_sstride || a.bias || a.relu || a.stats || a.wg_p) return false;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.Ho != a.H || a.Wo != a.W) return false;
  if ((a.K != 64 && a.K != 128) || a.C != a.K || a.Cout % RS_TC != 0 || a.ldy != a.Cout) return false;
  if (a.sW != a.C || a.sH != (long long)a.W * a.sW || a.sN != (long long)a.H * a.sH) return false;
  if (a.M <= 0 || a.M % RS_WP != 0) return false;
  if (a.seg_m > 0 && (a.seg_m % RS_WP != 0 || a.M % a.seg_m != 0 || a.M / a.seg_m > RS_NSEG)) return false;
  if (a.res_mode == 2 && (a.H % 2 || a.W % 2)) return false;
  const int ncb = a.Cout / RS_TC;
  const long long nblk = a.M / RS_WP;
  // workgroups of RS_CHUNK blocks (the dispatcher balances them over the CUs
  // the other stream leaves free; a persistent grid with fixed ranges ended
  // late behind its last-started workgroups in the step); channel blocks of one
  // chunk adjacent (one XCD)
  const long long nchunk = (nblk + RS_CHUNK - 1) / RS_CHUNK;
  if (nchunk * ncb > 0x7fffffffLL) return false;
  const dim3 g((unsigned)(nchunk * ncb)), b(256);
#define RS_GO(KV, BKV, TWOV) hipLaunchKernelGGL((rstream_kernel<KV, BKV, TWOV>), g, b, 0, st, a, RS_CHUNK)
  const bool two = a.bnb_nt == 2;
  if (a.K == 64) {
    if (a.bnb == 3) { if (two) RS_GO(64, 3, true); else RS_GO(64, 3, false); }
    else { if (two) RS_GO(64, 2, true); else RS_GO(64, 2, false); }
  } else {
    if (a.bnb == 3) { if (two) RS_GO(128, 3, true); else RS_GO(128, 3, false); }
    else { if (two) RS_GO(128, 2, true); else RS_GO(128, 2, false); }
  }
#undef RS_GO
  set_last_kernel(two ? "rstream_kernel<bnb,two>" : "rstream_kernel<bnb>");
  return true;
}

}  // namespace artsbir
