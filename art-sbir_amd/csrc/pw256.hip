// Ping-pong 256 x 256 weight-gradient tile for gfx950 (bf16 in, f32 accumulate,
// f32 atomics out): dW[co][k] += sum_m dY[m][co] * Xcol[m][k], the backward of
// the encoder's large convolution / linear weights — the Bottleneck 3x3 convs
// (models.py:200-201), the attention-pool projections (models.py:243-246) and
// the ViT block projections (models.py:396-417).
//
// The schedule is pp256.hip's, transposed: 8 waves in two groups of 4 (waves
// 0-3: output channels co 0-127 of the tile, 4-7: co 128-255; each wave 128 co x
// 64 k), group 1 one s_barrier behind, so one group's 16-MFMA cluster runs while
// the other reads its fragments and issues its LDS-DMA; K-tiles of 32 m rows in
// a 4-buffer ring with the stage of K-tile t+3 issued during K-tile t and one
// counted vmcnt per K-tile.  What differs is the operand form: both operands are
// m-major in HBM (rows m = output pixels), staged as row-major [32 m][256]
// images and read with the transposing ds_read_b64_tr_b16 (two per fragment).
// The image is guide T10's (a) layout — 8-row x 32-column subtiles of 512 B,
// chunk ^ ((row >> 2) & 3) inside a subtile — so a fragment 32 columns to the
// right is a constant 512 B away (an offset: immediate) and the two 16-lane
// groups of a half, 8 rows apart, hit different banks; the LDS-DMA source
// address of each lane is the inverse of that map.  The reduction over m is
// split over workgroups; each adds its tile into dW with f32 atomics.
#include <cstdlib>

#include "pgemm_dev.h"

namespace artsbir {

namespace {

constexpr int PW_BT = 256;              // tile width (co and k)
constexpr int PW_KS = 32;               // m rows per K-tile
constexpr int PW_HALF = PW_KS * PW_BT * 2;  // one operand of one K-tile: 16 KB
constexpr int PW_BUF = 2 * PW_HALF;
constexpr int PW_NW = 8;
constexpr unsigned PW_OOB = 0xC0000000u;  // stays out of range after adding < 2^30 of K-tile offsets

typedef short pw_v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) pw_v4s_t* pw_lds_v4s_t;

__device__ __forceinline__ void pw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void pw_glds(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r)
      : "memory");
}

// byte offset in a [32][256] image of 16-B chunk ch (0..31) of row (0..31)
__device__ __forceinline__ int pw_img(int row, int ch) {
  return (row >> 3) * 4096 + (ch >> 2) * 512 + (row & 7) * 64 + (((ch & 3) ^ ((row >> 2) & 3)) << 4);
}

// the transposed read: lane 4q+p of a 16-lane group addresses row r0+q,
// 16-bit columns 16c0 .. 16c0+15 in 4-column pieces (chunk 2c0 + p/2, + 8 B for odd p)
__device__ __forceinline__ bf16x8 pw_frag(const char* p0, const char* p1) {
  const pw_v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_v4s_t)(const __attribute__((address_space(3))) void*)p0);
  const pw_v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_v4s_t)(const __attribute__((address_space(3))) void*)p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

}  // namespace

template <bool DENSE>
__global__ void __launch_bounds__(512, 1) pw256_kernel(PwArgs a, int ntiles) {
  constexpr int NW = PW_NW;
  constexpr int MT = 8, NT = 4;  // wave tile 128 co x 64 k
  __shared__ __attribute__((aligned(16))) char smem[4 * PW_BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
  const int wco = wid >> 2, wkk = wid & 3;
  // tiles of one m-split are consecutive (one XCD: they read the same dY / X rows)
  const long long lid = pg_xcd_remap(blockIdx.x, (long long)gridDim.x);
  const long long split = lid / ntiles;
  const int tile = (int)(lid % ntiles);
  const int ntk = (a.K + PW_BT - 1) / PW_BT;
  const int co0 = (tile / ntk) * PW_BT, k0 = (tile % ntk) * PW_BT;
  const long long m_beg = split * a.m_per_split;
  long long m_end = m_beg + a.m_per_split;
  if (m_end > a.M) m_end = a.M;
  if (m_beg >= m_end) return;
  const int nk = (int)((m_end - m_beg + PW_KS - 1) / PW_KS);

  // ---- loader: instruction u (= wid, wid + 8) of a stage fills LDS bytes
  // [1024 u, 1024 u + 1024): subtile st = 2u + lane / 32, row 8 (st / 8) + (lane & 31) / 4,
  // chunk 4 (st % 8) + (slot ^ ((row >> 2) & 3))
  int lrow[2], lch[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int st = 2 * (u * NW + wid) + (lane >> 5);
    const int row = 8 * (st >> 3) + ((lane & 31) >> 2);
    lrow[u] = row;
    lch[u] = 4 * (st & 7) + ((lane & 3) ^ ((row >> 2) & 3));
  }
  // dY in two parts along Cout (a.dy2, dense): this tile's rows come from one of them
  const bool s2 = DENSE && a.dy2 != nullptr && co0 >= a.Cout1;
  const long long ldd = s2 ? a.ldd2 : a.ldd;
  const int cb = s2 ? co0 - a.Cout1 : co0;  // first dY column of the tile
  const int colim = (DENSE && a.dy2) ? (s2 ? a.Cout - a.Cout1 : a.Cout1) : a.Cout;
  float* const dwp = s2 ? a.dw2 : a.dw;
  // dY rows from m_beg; out-of-range co or rows past m_end read zeros
  const __amdgpu_buffer_rsrc_t dr = pg_rsrc(reinterpret_cast<const bf16*>(s2 ? a.dy2 : a.dy) + m_beg * ldd,
                                            (m_end - m_beg) * ldd * 2);
  unsigned aoff[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int co = cb + 8 * lch[u];
    aoff[u] = co < colim ? (unsigned)(lrow[u] * ldd * 2 + co * 2) : PW_OOB;
  }
  const unsigned a_step = (unsigned)(PW_KS * ldd * 2);
  // X: dense rows from m_beg, or the implicit im2col of the conv input
  const int HoWo = a.Ho * a.Wo;
  const long long img_beg = DENSE ? 0 : m_beg / HoWo;
  const __amdgpu_buffer_rsrc_t xr =
      DENSE ? pg_rsrc(reinterpret_cast<const bf16*>(a.x) + m_beg * a.ldx, (m_end - m_beg) * a.ldx * 2)
            : pg_rsrc(reinterpret_cast<const bf16*>(a.x) + img_beg * a.sN, (a.x_elems - img_beg * a.sN) * 2);
  unsigned boff[2];  // DENSE: offset at K-tile 0; conv: the chunk's channel offset
  int b_r[2], b_s[2], b_im[2], b_oh[2], b_ow[2];
  bool b_kok[2];
  const unsigned b_step = DENSE ? (unsigned)(PW_KS * a.ldx * 2) : 0u;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = k0 + 8 * lch[u];
    b_kok[u] = k < a.K;
    if constexpr (DENSE) {
      boff[u] = b_kok[u] ? (unsigned)(lrow[u] * a.ldx * 2 + k * 2) : PW_OOB;
      b_r[u] = b_s[u] = b_im[u] = b_oh[u] = b_ow[u] = 0;
    } else {
      const int kc = b_kok[u] ? k : 0;
      const int rs = kc / a.C, ci = kc - rs * a.C;
      b_r[u] = rs / a.S;
      b_s[u] = rs - b_r[u] * a.S;
      boff[u] = (unsigned)(ci * 2);
      const long long p = m_beg + lrow[u];
      const long long im = p / HoWo;
      const int rem = (int)(p - im * HoWo);
      b_im[u] = (int)(im - img_beg);
      b_oh[u] = rem / a.Wo;
      b_ow[u] = rem - b_oh[u] * a.Wo;
    }
  }
  // conv: the per-K-tile advance of a row by 32 pixels
  const int d_ow = PW_KS % a.Wo, d_oh = PW_KS / a.Wo;
  const unsigned lds0 = (unsigned)(unsigned long long)(pg_lds_t)smem + (unsigned)wid * 1024u;
  int l_kt = 0;  // next K-tile to issue
  auto issue_a = [&](int slot) {
#pragma unroll
    for (int u = 0; u < 2; ++u) pw_glds(dr, lds0 + slot * PW_BUF + u * NW * 1024, aoff[u] + (unsigned)l_kt * a_step);
  };
  auto issue_b = [&](int slot) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      unsigned off;
      if constexpr (DENSE) {
        off = boff[u] + (unsigned)l_kt * b_step;
      } else {
        const int ih = b_oh[u] * a.stride - a.pad + b_r[u], iw = b_ow[u] * a.stride - a.pad + b_s[u];
        const bool ok = b_kok[u] && m_beg + (long long)l_kt * PW_KS + lrow[u] < m_end && ih >= 0 && ih < a.H &&
                        iw >= 0 && iw < a.W;
        off = ok ? (unsigned)((b_im[u] * (int)a.sN + ih * (int)a.sH + iw * (int)a.sW) * 2) + boff[u] : PW_OOB;
        // next K-tile: this row moves 32 pixels on
        b_ow[u] += d_ow;
        b_oh[u] += d_oh;
        if (b_ow[u] >= a.Wo) { b_ow[u] -= a.Wo; ++b_oh[u]; }
        if (b_oh[u] >= a.Ho) { b_oh[u] -= a.Ho; ++b_im[u]; }
      }
      pw_glds(xr, lds0 + slot * PW_BUF + PW_HALF + u * NW * 1024, off);
    }
    ++l_kt;
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_a(0);
  issue_b(0);
  if (nk > 1) { issue_a(1); issue_b(1); }
  if (nk > 2) { issue_a(2); issue_b(2); }
  if (nk > 2) vm_wait<8>();
  else if (nk > 1) vm_wait<4>();
  else vm_wait<0>();
  pw_barrier();
  if (grp == 1) pw_barrier();

  // fragment addresses: lane t = 4q + p of group g reads rows 8g + q (+4 for the
  // high half), 16-column block c of the operand (chunk 2c + p/2, + 8 B if p odd)
  const int t = lane & 15, g = lane >> 4, q = t >> 2, p = t & 3;
  auto fa = [&](int row, int blk) { return pw_img(row, 2 * blk + (p >> 1)) + 8 * (p & 1); };
  // blocks 2i and 2i+1 differ in (ch & 3) (XOR with the row bits): one base per parity;
  // blocks two apart (32 columns) are 512 B apart
  const int ra = 8 * g + q;
  const int aE0 = fa(ra, 8 * wco), aE1 = fa(ra + 4, 8 * wco);          // co block 8 wco + 2i
  const int aO0 = fa(ra, 8 * wco + 1), aO1 = fa(ra + 4, 8 * wco + 1);  // co block 8 wco + 2i + 1
  const int bE0 = PW_HALF + fa(ra, 4 * wkk), bE1 = PW_HALF + fa(ra + 4, 4 * wkk);
  const int bO0 = PW_HALF + fa(ra, 4 * wkk + 1), bO1 = PW_HALF + fa(ra + 4, 4 * wkk + 1);
  bf16x8 bv[NT], af[MT];
  auto ktile = [&](int s, auto slc) {
    constexpr int SL = decltype(slc)::value;
    const char* b = smem + SL * PW_BUF;
    if (s + 3 < nk) issue_a((SL + 3) & 3);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int o = (j >> 1) * 512;
      bv[j] = (j & 1) ? pw_frag(b + bO0 + o, b + bO1 + o) : pw_frag(b + bE0 + o, b + bE1 + o);
    }
#pragma unroll
    for (int i = 0; i < MT / 2; ++i) {
      const int o = (i >> 1) * 512;
      af[i] = (i & 1) ? pw_frag(b + aO0 + o, b + aO1 + o) : pw_frag(b + aE0 + o, b + aE1 + o);
    }
    pw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    PG_PRIO_ON();
#pragma unroll
    for (int i = 0; i < MT / 2; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bv[j], acc[i][j], 0, 0, 0);
    PG_PRIO_OFF();
    pw_barrier();
    if (s + 3 < nk) {
      issue_b((SL + 3) & 3);
      vm_wait<8>();
    } else if (s + 2 < nk) {
      vm_wait<4>();
    } else if (s + 1 < nk) {
      vm_wait<0>();
    }
#pragma unroll
    for (int i = MT / 2; i < MT; ++i) {
      const int o = (i >> 1) * 512;
      af[i] = (i & 1) ? pw_frag(b + aO0 + o, b + aO1 + o) : pw_frag(b + aE0 + o, b + aE1 + o);
    }
    pw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    PG_PRIO_ON();
#pragma unroll
    for (int i = MT / 2; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bv[j], acc[i][j], 0, 0, 0);
    PG_PRIO_OFF();
    if (!(s == nk - 1 && grp == 1)) pw_barrier();
  };
  for (int s = 0; s < nk; s += 4) {
    ktile(s, std::integral_constant<int, 0>{});
    if (s + 1 < nk) ktile(s + 1, std::integral_constant<int, 1>{});
    if (s + 2 < nk) ktile(s + 2, std::integral_constant<int, 2>{});
    if (s + 3 < nk) ktile(s + 3, std::integral_constant<int, 3>{});
  }

  // acc[i][j][r]: co = co0 + 128 wco + 16 i + 4 g + r, k = k0 + 64 wkk + 16 j + t
  // (relative to the tile's part of dY: cb, colim, dwp)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int k = k0 + 64 * wkk + 16 * j + t;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cb + 128 * wco + 16 * i + 4 * g + r;
        if (co < colim && k < a.K) atomicAdd(dwp + (long long)co * a.K + k, acc[i][j][r]);
      }
    }
}

// wgrad candidate 100 + level (gemm.hip tune_wgrad): the split of the m
// reduction targets 256 << level workgroups; false (nothing launched) outside
// the kernel's range
bool pw256_launch(PwArgs a, int level, hipStream_t st) {
  if (level < 0 || level > 2) return false;
  // small Cout or K leave most of the 256 x 256 tile idle; the tuner still
  // takes it where the weight gradient is bound by its HBM reads (1x1 convs of
  // 64-channel layers), not by the MFMAs
  if (a.Cout < 64 || a.K < 64 || a.Cout % 8 || a.K % 8 || a.M <= 0) return false;
  if (a.ldd % 8 || (a.dense && a.ldx % 8)) return false;
  if (a.dy2 && (!a.dense || a.Cout1 % PW_BT != 0 || !a.dw2 || a.ldd2 % 8)) return false;
  if (!a.dense && (a.C % 8 || a.R * a.S > 32 || (long long)a.Ho * a.Wo < PW_KS)) return false;
  const int ntiles = ((a.Cout + PW_BT - 1) / PW_BT) * ((a.K + PW_BT - 1) / PW_BT);
  const long long ksteps = (a.M + PW_KS - 1) / PW_KS;
  // ARTSBIR_PW256_SPLITX=f (measurement switch): f times the workgroups, each a
  // 1/f share of the m reduction (shorter-lived workgroups beside the main stream)
  static const int splitx = getenv("ARTSBIR_PW256_SPLITX") ? atoi(getenv("ARTSBIR_PW256_SPLITX")) : 1;
  const long long target = ((long long)g_wgrad_cus << level) * (splitx > 1 ? splitx : 1);
  long long splits = target / ntiles;
  if (splits < 1) splits = 1;
  long long per = (ksteps + splits - 1) / splits;
  if (per < 16) per = 16;  // at least 16 K-tiles (512 rows) per workgroup
  // K-tile offsets (32 rows x ld) summed over a split stay below 2^30 (PW_OOB stays out of range)
  long long ldmax = a.dense ? (a.ldx > a.ldd ? a.ldx : a.ldd) : a.ldd;
  if (a.dy2 && a.ldd2 > ldmax) ldmax = a.ldd2;
  const long long row_bytes = ldmax * 2;
  long long cap = (1LL << 30) / (row_bytes * PW_KS) - 1;
  if (!a.dense) {
    const long long imgs = 0x7fffffffLL / (a.sN * 2) - 2;  // image-relative conv offsets below 2^31
    const long long HoWo = (long long)a.Ho * a.Wo;
    if (imgs < 1) return false;
    const long long cap2 = imgs * HoWo / PW_KS;
    if (cap2 < cap) cap = cap2;
  }
  if (cap < 1) return false;
  if (per > cap) per = cap;
  a.m_per_split = per * PW_KS;
  splits = (ksteps + per - 1) / per;
  const long long blocks = (long long)ntiles * splits;
  if (blocks > 0x7fffffffLL) return false;
  if (a.dense) hipLaunchKernelGGL((pw256_kernel<true>), dim3((unsigned)blocks), dim3(512), 0, st, a, ntiles);
  else hipLaunchKernelGGL((pw256_kernel<false>), dim3((unsigned)blocks), dim3(512), 0, st, a, ntiles);
  set_last_kernel(a.dense ? "pw256_kernel<dense>" : "pw256_kernel<conv>");
  return true;
}

}  // namespace artsbir
