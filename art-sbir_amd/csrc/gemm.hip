// Implicit-GEMM convolution / dense GEMM / weight-gradient GEMM on MFMA (gfx950).
//
// Replaces the torch ops on the reference hot path
//   nn.Conv2d (models.py:198,202,208,219 Bottleneck; models.py:310,313,316 stem)
//   nn.Linear / F.multi_head_attention_forward projections (models.py:243-246,253-271)
// forward, data-gradient and weight-gradient.
//
// One LDS image layout serves every operand of every kernel here:
//   tile[chunk g][row][16 bytes]   row stride 16 B, chunk stride (ROWS+1)*16 B
// where a 16-byte chunk holds EPC consecutive reduction ("k") elements of one
// row (EPC = 8 bf16 or 4 f32).  A 16-lane group reading 16 consecutive rows of
// one chunk with ds_read_b128 is conflict-free, and the +1 row pad makes the
// 8 lanes of a ds_write_b128 group that write 8 different chunks of one row
// land on 8 different 16-B bank slots.
//
// MFMA mapping (both dtypes use the 16x16 output layout col = lane&15,
// row = 4*(lane>>4) + reg):
//   bf16: v_mfma_f32_16x16x32_bf16, lane (i, q=lane>>4) feeds row i, chunk q
//         (8 k) -> one ds_read_b128 per fragment per 32-k step;
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32), lane (i,q) reads chunk q (4 k)
//         with one ds_read_b128 and issues 4 MFMAs, element e in step e.  The
//         k order inside the MFMA is a permutation applied identically to A
//         and B, so the sum is unchanged.
//
// Global loads are raw buffer loads: an out-of-range byte offset returns zero,
// which implements both the convolution zero padding and every M/N/K tail
// without a branch.  Per thread, the A rows it stages are decoded once
// (pixel offset + one validity bit per filter tap); per K-step only the tap
// (r, s, ci) changes, and when C is a multiple of the K-step it is uniform
// across the workgroup (scalar arithmetic).
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "pgemm.h"

namespace artsbir {

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#define OOB_OFFSET 0x80000000u

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

template <typename T> struct MM;
template <> struct MM<bf16> {
  static constexpr int EPC = 8;  // elements per 16-B chunk
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&a),
                                                  *reinterpret_cast<const bf16x8*>(&b), acc, 0, 0, 0);
  }
};
template <> struct MM<float> {
  static constexpr int EPC = 4;
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    const float* fa = reinterpret_cast<const float*>(&a);
    const float* fb = reinterpret_cast<const float*>(&b);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[e], fb[e], acc, 0, 0, 0);
  }
};

// affine(+relu) of one 16-B chunk of T for channels sc/sh[0..EPC)
__device__ __forceinline__ uint4 affine_chunk(uint4 v, const float* sc, const float* sh, int relu, bf16) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xffff0000u);
    lo = lo * sc[2 * i] + sh[2 * i];
    hi = hi * sc[2 * i + 1] + sh[2 * i + 1];
    if (relu) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
    bf16 blo = (bf16)lo, bhi = (bf16)hi;
    w[i] = (uint32_t)__builtin_bit_cast(unsigned short, blo) | ((uint32_t)__builtin_bit_cast(unsigned short, bhi) << 16);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint4 affine_chunk(uint4 v, const float* sc, const float* sh, int relu, float) {
  float f[4] = {__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[i] = f[i] * sc[i] + sh[i];
    if (relu) f[i] = fmaxf(f[i], 0.f);
  }
  return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
}

// bijective XCD-aware block remap: blocks that share an XCD (bid % 8) get
// consecutive logical ids, so neighbouring tiles (same A panel) share an L2.
__device__ __forceinline__ long long xcd_remap(long long bid, long long nwg) {
  if (nwg < 8) return bid;
  const long long q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// ---------------------------------------------------------------------------
// Forward / data-gradient implicit GEMM:  Y[m][n] = sum_k Xcol[m][k] * W[n][k]
//   Xcol[m=(img,oh,ow)][k=(r,s,ci)] = act(X[img][oh*st-pad+r][ow*st-pad+s][ci])
//   act = optional per-input-channel affine (+ReLU); padding stays zero.
// ---------------------------------------------------------------------------
struct ConvArgs {
  const void* x;
  long long x_elems;     // extent of x (elements) for the bounds check
  long long sN, sH, sW;  // element strides of x (channel stride 1)
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  const float* in_scale;
  const float* in_shift;
  int in_relu;
  const void* w;  // [Cout][K], K contiguous
  int Cout, K;
  long long M;
  void* y;
  long long ldy;
  int out_f32;
  int accumulate;
  const float* bias;
  float* stats;     // [NSLOT][2][Cout] (x nseg)
  const void* res;  // epilogue residual (T): mode 1 same index, mode 2 2x2 average-unpool
  int res_mode;
  int relu;         // ReLU on the stored output (after bias and residual)
  // host-side only (the launcher splits / fuses; kernels ignore them)
  int nseg;                 // BN segments (separate reference forward calls) of equal size
  const void* bnb_desc;     // artsbir_bn_bwd_desc of a fused BN-backward reduction (dgrad)
  long long bnb_pstride;    // floats between the BN parameters of consecutive segments
  // the folded BatchNorm backward of artsbir_conv1x1_dgrad_fold (PgArgs: same
  // fields); only the pipelined bf16 kernels take it
  const void* x2 = nullptr;
  long long x2_elems = 0, sN2 = 0, sH2 = 0, sW2 = 0;
  int C1 = 0;
  long long w_sstride = 0, bias_sstride = 0;
  float* wg_p = nullptr;  // the fold's weight-gradient operands in the same pass (pg_fold_wg_launch)
  float* wg_gram = nullptr;
};

template <typename T, int BM, int BN, bool UNIFORM_TAP, bool AFFINE>
__global__ void __launch_bounds__(256) conv_gemm_kernel(ConvArgs a) {
  constexpr int EPC = MM<T>::EPC;
  constexpr int ES = sizeof(T);
  constexpr int BK = 8 * EPC;  // 8 chunks per K-step (128 bytes of k per row)
  constexpr int A_BYTES = 8 * (BM + 1) * 16;
  constexpr int B_BYTES = 8 * (BN + 1) * 16;
  constexpr int ARows = BM / 32;  // rows per thread in the A loader
  constexpr int BRows = BN / 32;
  constexpr int WN = BN >= 128 ? 2 : 1;  // waves along N
  constexpr int WM = 4 / WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int MAIN_BYTES = 2 * (A_BYTES + B_BYTES);
  constexpr int EPI_LD = BN + 4;  // f32 staging row stride
  constexpr int EPI_BYTES = BM * EPI_LD * 4;
  constexpr int SMEM = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int ntn = (a.Cout + BN - 1) / BN;
  const long long ntm = (a.M + BM - 1) / BM;
  const long long lid = xcd_remap(blockIdx.x, ntm * ntn);
  const long long bm = (lid / ntn) * BM;
  const int bn = (int)(lid % ntn) * BN;

  const int HoWo = a.Ho * a.Wo;
  const long long img0 = bm / HoWo;
  const __amdgpu_buffer_rsrc_t xr =
      make_rsrc(reinterpret_cast<const T*>(a.x) + img0 * a.sN, (a.x_elems - img0 * a.sN) * ES);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (long long)a.Cout * a.K * ES);

  const int lc = tid & 7;   // chunk handled by this thread
  const int lr = tid >> 3;  // first row handled by this thread
  int rowoff[ARows];
  unsigned rmask[ARows];
#pragma unroll
  for (int i = 0; i < ARows; ++i) {
    const long long gm = bm + lr + 32 * i;
    const bool valid = gm < a.M;
    const long long gmc = valid ? gm : bm;
    const long long img = gmc / HoWo;
    const int rem = (int)(gmc - img * HoWo);
    const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    rowoff[i] = (int)(((img - img0) * a.sN + (long long)ih0 * a.sH + (long long)iw0 * a.sW) * ES);
    unsigned msk = 0;
    for (int r = 0; r < a.R; ++r)
      for (int s = 0; s < a.S; ++s) {
        const bool ok = valid && ih0 + r >= 0 && ih0 + r < a.H && iw0 + s >= 0 && iw0 + s < a.W;
        msk |= (ok ? 1u : 0u) << (r * a.S + s);
      }
    rmask[i] = msk;
  }
  int boff[BRows];
#pragma unroll
  for (int i = 0; i < BRows; ++i) {
    const int n = bn + lr + 32 * i;
    boff[i] = n < a.Cout ? n * a.K * ES + lc * 16 : (int)OOB_OFFSET;
  }

  uint4 ra[ARows], rb[BRows];

  // uniform taps: (ci, s, r) of the K-step advance incrementally (no division)
  int u_ci = 0, u_s = 0, u_r = 0;
  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK;
    int rs, ci, r, s;
    if constexpr (UNIFORM_TAP) {
      ci = u_ci; s = u_s; r = u_r;
      rs = r * a.S + s;
      u_ci += BK;
      if (u_ci == a.C) {
        u_ci = 0;
        if (++u_s == a.S) { u_s = 0; ++u_r; }
      }
    } else if (a.C < BK && BK % a.C == 0) {
      // C divides the K-step (stem: C = 8 or 32): BK/C taps per step, each
      // thread's chunk sits at a fixed (sub-tap, channel) inside the step
      const int cpt = a.C / EPC;  // chunks per tap
      const int sub = lc / cpt;
      ci = (lc - sub * cpt) * EPC;
      rs = kt * (BK / a.C) + sub;
      r = rs / a.S;
      s = rs - r * a.S;
    } else {
      const int kq = k0 + lc * EPC;  // first k of this thread's chunk
      rs = kq / a.C;
      ci = kq - rs * a.C;
      r = rs / a.S;
      s = rs - r * a.S;
    }
    const bool kval = UNIFORM_TAP ? true : (k0 + lc * EPC < a.K);
    const int tapoff = (r * (int)a.sH + s * (int)a.sW + ci) * ES + (UNIFORM_TAP ? lc * 16 : 0);
#pragma unroll
    for (int i = 0; i < ARows; ++i) {
      const bool ok = kval && ((rmask[i] >> rs) & 1u);
      ra[i] = bload(xr, ok ? (unsigned)(rowoff[i] + tapoff) : OOB_OFFSET);
    }
    const bool bok = (k0 + lc * EPC) < a.K;
#pragma unroll
    for (int i = 0; i < BRows; ++i) rb[i] = bload(wr, bok ? (unsigned)(boff[i] + k0 * ES) : OOB_OFFSET);
    if constexpr (AFFINE) {
      const int cch = UNIFORM_TAP ? ci + lc * EPC : ci;
      float sc[EPC], sh[EPC];
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        sc[e] = kval ? a.in_scale[cch + e] : 0.f;
        sh[e] = kval ? a.in_shift[cch + e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < ARows; ++i) {
        const bool ok = kval && ((rmask[i] >> rs) & 1u);
        const uint4 v = affine_chunk(ra[i], sc, sh, a.in_relu, T());
        ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < ARows; ++i) *reinterpret_cast<uint4*>(As + (lc * (BM + 1) + lr + 32 * i) * 16) = ra[i];
#pragma unroll
    for (int i = 0; i < BRows; ++i) *reinterpret_cast<uint4*>(Bs + (lc * (BN + 1) + lr + 32 * i) * 16) = rb[i];
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g = kk * 4 + fq;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + (g * (BM + 1) + wm * WTM + i * 16 + fr) * 16);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + (g * (BN + 1) + wn * WTN + j * 16 + fr) * 16);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) MM<T>::mma(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue 1: batch-norm statistics straight from the accumulators
  if (a.stats) {
    const int slot = (int)(blockIdx.x % ARTSBIR_NSLOT);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int gn = bn + wn * WTN + j * 16 + fr;
      const float bval = (a.bias && gn < a.Cout) ? a.bias[gn] : 0.f;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long gm = bm + wm * WTM + i * 16 + fq * 4 + r;
          const float v = acc[i][j][r] + bval;
          if (gm < a.M) { s1 += v; s2 += v * v; }
        }
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0 && gn < a.Cout) {
        atomicAdd(a.stats + (long long)slot * 2 * a.Cout + gn, s1);
        atomicAdd(a.stats + (long long)slot * 2 * a.Cout + a.Cout + gn, s2);
      }
    }
  }
  // ---- epilogue 2: stage the f32 tile row-major in LDS, then 16-B coalesced rows
  float* st = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        st[(wm * WTM + i * 16 + fq * 4 + r) * EPI_LD + wn * WTN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int CPR = BN / 8;  // 8-column chunks per row
  for (int u = tid; u < BM * CPR; u += 256) {
    const int row = u / CPR, cc = u - (u / CPR) * CPR;
    const long long gm = bm + row;
    const int gn = bn + cc * 8;
    if (gm >= a.M || gn >= a.Cout) continue;
    float v[8];
    *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(st + row * EPI_LD + cc * 8);
    *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(st + row * EPI_LD + cc * 8 + 4);
    const int nv = a.Cout - gn < 8 ? a.Cout - gn : 8;
    if (a.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += e < nv ? a.bias[gn + e] : 0.f;
    }
    if (a.res_mode) {
      long long ri;
      float scale = 1.f;
      if (a.res_mode == 1) {
        ri = gm;
      } else {
        const long long img = gm / HoWo;
        const int rem = (int)(gm - img * HoWo);
        const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
        ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
        scale = 0.25f;
      }
      const T* rp = reinterpret_cast<const T*>(a.res) + ri * a.ldy + gn;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += e < nv ? scale * to_f(rp[e]) : 0.f;
    }
    if (a.relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (a.out_f32) {
      float* yp = reinterpret_cast<float*>(a.y) + gm * a.ldy + gn;
      if (nv == 8 && (a.ldy % 4) == 0) {
        if (a.accumulate) {
          const float4 p0 = *reinterpret_cast<const float4*>(yp), p1 = *reinterpret_cast<const float4*>(yp + 4);
          v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
          v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
        }
        *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        for (int e = 0; e < nv; ++e) yp[e] = a.accumulate ? yp[e] + v[e] : v[e];
      }
    } else {
      T* yp = reinterpret_cast<T*>(a.y) + gm * a.ldy + gn;
      if (nv == 8 && (a.ldy % 8) == 0) {
        Vec16<T> o0;
        if constexpr (EPC == 8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o0.v[e] = from_f<T>(v[e]);
          st16<T>(yp, o0);
        } else {
          Vec16<T> o1;
#pragma unroll
          for (int e = 0; e < 4; ++e) { o0.v[e] = from_f<T>(v[e]); o1.v[e] = from_f<T>(v[e + 4]); }
          st16<T>(yp, o0);
          st16<T>(yp + 4, o1);
        }
      } else {
        for (int e = 0; e < nv; ++e) yp[e] = from_f<T>(v[e]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient:  dW[co][k] += sum_m dY[m][co] * Xcol[m][k]
// Both operands arrive reduction-major ([m][...]); each loader unit reads an
// EPC x EPC block (EPC rows m, EPC consecutive co / ci) with 16-B coalesced
// loads and transposes it in registers (v_perm_b32 for bf16) into EPC chunks
// of the common LDS image.  The reduction over m is split across workgroups
// and combined with f32 atomics into dW.  The (r, s, ci) of every Xcol unit is
// loop-invariant per thread (the K-loop runs over m), so its affine
// coefficients and tap offsets are loaded/decoded once.
// ---------------------------------------------------------------------------
struct WgradArgs {
  const void* dy;
  long long dy_elems;
  long long ldd;  // row stride of dY
  const void* x;
  long long x_elems;
  long long sN, sH, sW;
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  int dense;      // Xcol[m][k] = x[m*ldx + k] (1x1, stride 1, no pad)
  long long ldx;
  const float* in_scale;
  const float* in_shift;
  int in_relu;
  int Cout, K;
  long long M;
  long long m_per_split;  // multiple of BK
  float* dw;               // [Cout][K] f32
  // dY in two parts along Cout (PwArgs: same fields; the pipelined kernels only)
  const void* dy2 = nullptr;
  long long dy2_elems = 0, ldd2 = 0;
  int Cout1 = 0;
  float* dw2 = nullptr;
};

__device__ __forceinline__ void transpose_unit(const uint4 (&in)[8], uint4 (&out)[8], bf16) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t o0[4], o1[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t a0 = reinterpret_cast<const uint32_t*>(&in[2 * w])[p];
      const uint32_t a1 = reinterpret_cast<const uint32_t*>(&in[2 * w + 1])[p];
      o0[w] = __builtin_amdgcn_perm(a1, a0, 0x05040100u);
      o1[w] = __builtin_amdgcn_perm(a1, a0, 0x07060302u);
    }
    out[2 * p] = make_uint4(o0[0], o0[1], o0[2], o0[3]);
    out[2 * p + 1] = make_uint4(o1[0], o1[1], o1[2], o1[3]);
  }
}
__device__ __forceinline__ void transpose_unit(const uint4 (&in)[4], uint4 (&out)[4], float) {
  out[0] = make_uint4(in[0].x, in[1].x, in[2].x, in[3].x);
  out[1] = make_uint4(in[0].y, in[1].y, in[2].y, in[3].y);
  out[2] = make_uint4(in[0].z, in[1].z, in[2].z, in[3].z);
  out[3] = make_uint4(in[0].w, in[1].w, in[2].w, in[3].w);
}

template <typename T, int BM, int BN, bool AFFINE>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs a) {
  constexpr int EPC = MM<T>::EPC;
  constexpr int ES = sizeof(T);
  constexpr int BK = 8 * EPC;
  constexpr int A_BYTES = 8 * (BM + 1) * 16;
  constexpr int B_BYTES = 8 * (BN + 1) * 16;
  constexpr int AU = 8 * (BM / EPC);  // loader units per operand
  constexpr int BU = 8 * (BN / EPC);
  constexpr int UT = (AU + BU + 255) / 256;
  static_assert(AU % 64 == 0, "A units must be wave aligned");
  constexpr int WN = BM >= 128 ? 2 : 4;  // waves along N (k')
  constexpr int WM = 4 / WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (a.K + BN - 1) / BN;
  const int ntm = (a.Cout + BM - 1) / BM;
  const int tile = blockIdx.x % (ntm * ntn);
  const int split = blockIdx.x / (ntm * ntn);
  const int bm = (tile / ntn) * BM;  // co
  const int bn = (tile % ntn) * BN;  // k
  const long long m_begin = (long long)split * a.m_per_split;
  long long m_end = m_begin + a.m_per_split;
  if (m_end > a.M) m_end = a.M;
  if (m_begin >= m_end) return;
  const int nk = (int)((m_end - m_begin + BK - 1) / BK);

  const int HoWo = a.Ho * a.Wo;
  const long long img0 = a.dense ? 0 : m_begin / HoWo;
  const long long xbase = a.dense ? m_begin * a.ldx : img0 * a.sN;
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(reinterpret_cast<const T*>(a.dy) + m_begin * a.ldd,
                                               (a.dy_elems - m_begin * a.ldd) * ES);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(reinterpret_cast<const T*>(a.x) + xbase, (a.x_elems - xbase) * ES);

  // per-unit loop invariants
  int u_mc[UT], u_cc[UT];
  bool u_isA[UT], u_act[UT];
  int b_r[UT], b_s[UT], b_ci[UT];
  bool b_kval[UT];
  float b_sc[UT][AFFINE ? EPC : 1], b_sh[UT][AFFINE ? EPC : 1];
#pragma unroll
  for (int t = 0; t < UT; ++t) {
    const int uu = tid + 256 * t;
    u_act[t] = uu < AU + BU;
    u_isA[t] = uu < AU;
    const int u = u_isA[t] ? uu : uu - AU;
    u_mc[t] = u & 7;
    u_cc[t] = u >> 3;
    const int k = bn + u_cc[t] * EPC;
    b_kval[t] = !u_isA[t] && k < a.K;
    const int rs = b_kval[t] ? k / a.C : 0;
    b_ci[t] = b_kval[t] ? k - rs * a.C : 0;
    b_r[t] = rs / a.S;
    b_s[t] = rs - (rs / a.S) * a.S;
    if constexpr (AFFINE) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        b_sc[t][e] = b_kval[t] ? a.in_scale[b_ci[t] + e] : 0.f;
        b_sh[t][e] = b_kval[t] ? a.in_shift[b_ci[t] + e] : 0.f;
      }
    }
  }

  uint4 tu[UT][EPC];
  // 32-bit, block-relative pixel walk: m = m_begin + rel, pos = rem0 + rel is the
  // pixel index counted from the start of image img0 (pos < 2^24 by construction)
  const int mlen = (int)(m_end - m_begin);
  const int rem0 = a.dense ? 0 : (int)(m_begin - img0 * HoWo);
  const float inv_howo = 1.f / (float)HoWo, inv_wo = 1.f / (float)a.Wo;
  const int sN = (int)a.sN, sH = (int)a.sH, sW = (int)a.sW, ldd = (int)a.ldd, ldx = (int)a.ldx;

  auto load_tiles = [&](int kt) {
    const int m0 = kt * BK;  // relative to m_begin
#pragma unroll
    for (int t = 0; t < UT; ++t) {
      if (!u_act[t]) continue;
      const int mb = m0 + u_mc[t] * EPC;
      if (u_isA[t]) {
        const int co = bm + u_cc[t] * EPC;
        const bool cval = co < a.Cout;
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const bool ok = cval && mb + e < mlen;
          tu[t][e] = bload(dyr, ok ? (unsigned)(((mb + e) * ldd + co) * ES) : OOB_OFFSET);
        }
      } else if (a.dense) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const bool ok = b_kval[t] && mb + e < mlen;
          tu[t][e] = bload(xr, ok ? (unsigned)(((mb + e) * ldx + bn + u_cc[t] * EPC) * ES) : OOB_OFFSET);
        }
      } else {
        // decode the first m of the unit, then walk along the output row
        const int pos = rem0 + mb;
        int q = (int)((float)pos * inv_howo);
        int p = pos - q * HoWo;
        if (p < 0) { --q; p += HoWo; } else if (p >= HoWo) { ++q; p -= HoWo; }
        int oh = (int)((float)p * inv_wo);
        int ow = p - oh * a.Wo;
        if (ow < 0) { --oh; ow += a.Wo; } else if (ow >= a.Wo) { ++oh; ow -= a.Wo; }
        int ih = oh * a.stride - a.pad + b_r[t], iw = ow * a.stride - a.pad + b_s[t];
        int base = q * sN + b_ci[t];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const bool ok = b_kval[t] && mb + e < mlen && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          tu[t][e] = bload(xr, ok ? (unsigned)((base + ih * sH + iw * sW) * ES) : OOB_OFFSET);
          if constexpr (AFFINE) {
            const uint4 v = affine_chunk(tu[t][e], b_sc[t], b_sh[t], a.in_relu, T());
            tu[t][e] = ok ? v : make_uint4(0, 0, 0, 0);
          }
          ++ow;
          iw += a.stride;
          if (ow == a.Wo) {
            ow = 0;
            iw = b_s[t] - a.pad;
            ih += a.stride;
            if (++oh == a.Ho) { oh = 0; ih = b_r[t] - a.pad; base += sN; }
          }
        }
      }
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int t = 0; t < UT; ++t) {
      if (!u_act[t]) continue;
      char* base = u_isA[t] ? As + (u_mc[t] * (BM + 1) + u_cc[t] * EPC) * 16
                            : Bs + (u_mc[t] * (BN + 1) + u_cc[t] * EPC) * 16;
      uint4 o[EPC];
      transpose_unit(tu[t], o, T());
#pragma unroll
      for (int c = 0; c < EPC; ++c) *reinterpret_cast<uint4*>(base + c * 16) = o[c];
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g = kk * 4 + fq;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + (g * (BM + 1) + wm * WTM + i * 16 + fr) * 16);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + (g * (BN + 1) + wn * WTN + j * 16 + fr) * 16);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) MM<T>::mma(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int gk = bn + wn * WTN + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gco = bm + wm * WTM + i * 16 + fq * 4 + r;
        if (gco < a.Cout && gk < a.K) atomicAdd(a.dw + (long long)gco * a.K + gk, acc[i][j][r]);
      }
    }
}

}  // namespace artsbir

using namespace artsbir;

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
#include "../../include/artsbir.h"

static int check_conv(const artsbir_conv_desc* d) {
  if (d->C % 8 != 0) { set_error("conv: C=%d must be a multiple of 8", d->C); return -1; }
  if (d->Cout <= 0 || d->N <= 0) { set_error("conv: empty shape"); return -1; }
  if (d->R <= 0 || d->S <= 0 || d->stride <= 0 || d->pad < 0) { set_error("conv: bad geometry"); return -1; }
  if (d->R * d->S > 32) { set_error("conv: at most 32 filter taps"); return -1; }
  return 0;
}

static void fill_geom(const artsbir_conv_desc* d, int& Ho, int& Wo) {
  Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
  Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
}

template <typename T, int BM, int BN>
static void launch_conv_tile(const ConvArgs& a, hipStream_t st) {
  constexpr int BK = 8 * MM<T>::EPC;
  const long long tiles = ((a.M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  const bool uni = (a.C % BK) == 0;
  const bool aff = a.in_scale != nullptr;
  if (uni && aff) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, true, true>), dim3((unsigned)tiles), dim3(256), 0, st, a);
  else if (uni) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, true, false>), dim3((unsigned)tiles), dim3(256), 0, st, a);
  else if (aff) hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false, true>), dim3((unsigned)tiles), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((conv_gemm_kernel<T, BM, BN, false, false>), dim3((unsigned)tiles), dim3(256), 0, st, a);
}

template <typename T>
static void launch_conv_old(const ConvArgs& a, hipStream_t st) {
  const bool bf = sizeof(T) == 2;
  if (a.Cout <= 64) {
    set_last_kernel(bf ? "conv_gemm_kernel<bf16,128,64>" : "conv_gemm_kernel<f32,128,64>");
    launch_conv_tile<T, 128, 64>(a, st);
  } else {
    set_last_kernel(bf ? "conv_gemm_kernel<bf16,128,128>" : "conv_gemm_kernel<f32,128,128>");
    launch_conv_tile<T, 128, 128>(a, st);
  }
}

// ---------------------------------------------------------------------------
// Kernel choice per convolution shape (bf16): the register-staged kernel
// above (-2), the pipelined LDS-DMA kernel's tile shapes (0..4) or the
// persistent streaming kernel (10), pgemm.hip.  By default the first call of
// a new shape times every applicable candidate on the caller's stream (output
// written to the real buffers, BN statistics to a scratch buffer) and caches
// the fastest, like a "find" step; ARTSBIR_TUNE=0 uses the static heuristic,
// ARTSBIR_PGEMM_CFG=<c> forces candidate c (tests).
// ---------------------------------------------------------------------------
struct ConvKey {
  long long M;
  int H, W, C, Cout, R, S, stride, pad, Ho, Wo, res_mode, stats, nseg, bnb;
  bool operator<(const ConvKey& o) const {
    return std::tie(M, H, W, C, Cout, R, S, stride, pad, Ho, Wo, res_mode, stats, nseg, bnb) <
           std::tie(o.M, o.H, o.W, o.C, o.Cout, o.R, o.S, o.stride, o.pad, o.Ho, o.Wo, o.res_mode, o.stats, o.nseg,
                    o.bnb);
  }
};
static std::map<ConvKey, int> g_conv_choice;
static std::mutex g_tune_mu;
static float* g_tune_stats = nullptr;
static size_t g_tune_stats_n = 0;

// The register-staged kernel over each BN segment in turn (its statistics
// epilogue has no segment logic).
template <typename T>
static void launch_conv_old_seg(const ConvArgs& a, hipStream_t st) {
  if (a.nseg <= 1 || !a.stats) { launch_conv_old<T>(a, st); return; }
  const long long seg_m = a.M / a.nseg, seg_img = seg_m / ((long long)a.Ho * a.Wo);
  for (int s = 0; s < a.nseg; ++s) {
    ConvArgs p = a;
    p.nseg = 1;
    p.x = reinterpret_cast<const T*>(a.x) + s * seg_img * a.sN;
    p.x_elems = seg_img * a.sN;
    p.M = seg_m;
    p.y = reinterpret_cast<T*>(a.y) + s * seg_m * a.ldy;
    p.stats = a.stats + (long long)s * ARTSBIR_NSLOT * 2 * a.Cout;
    launch_conv_old<T>(p, st);
  }
}

// Fused BN-backward reduction done as a separate pass (f32 mode, or a shape the
// pipelined kernel does not take): artsbir_bn_bwd_reduce per segment, writing
// g = d * mask back over d.
static int bnb_reduce_pass(const ConvArgs& a, const artsbir_bn_bwd_desc* bd, hipStream_t st) {
  const long long seg_m = a.M / a.nseg;
  const int seg_img = (int)(seg_m / ((long long)a.Ho * a.Wo));
  const long long es = bd->dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  for (int s = 0; s < a.nseg; ++s) {
    artsbir_bn_bwd_desc d = *bd;
    d.nseg = 1;
    const long long eo = s * seg_m * a.Cout * es;  // byte offset of the segment's elements
    const long long po = s * a.bnb_pstride;
    d.pool = 0;
    d.d = reinterpret_cast<const char*>(a.y) + eo;
    d.gout = reinterpret_cast<char*>(a.y) + eo;
    if (bd->mask)  // kind 3: one mask byte per 8 channels
      d.mask = reinterpret_cast<const char*>(bd->mask) + (bd->kind == 3 ? s * seg_m * (a.Cout / 8) : eo);
    if (bd->mask_bn) d.mask_bn = bd->mask_bn + po;
    for (int t = 0; t < bd->ntarget; ++t) {
      d.y[t] = reinterpret_cast<const char*>(bd->y[t]) + eo;
      d.mean[t] = bd->mean[t] + po;
      d.istd[t] = bd->istd[t] + po;
      d.slots[t] = bd->slots[t] + (long long)s * ARTSBIR_NSLOT * 2 * a.Cout;
    }
    d.B = seg_img; d.H = a.Ho; d.W = a.Wo; d.C = a.Cout;
    const int rc = artsbir_bn_bwd_reduce(&d, st);
    if (rc) return rc;
  }
  return 0;
}

template <typename T>
static int run_old(const ConvArgs& a, hipStream_t st) {
  launch_conv_old_seg<T>(a, st);
  ARTSBIR_CHECK_LAUNCH("conv_gemm");
  if (a.bnb_desc) return bnb_reduce_pass(a, reinterpret_cast<const artsbir_bn_bwd_desc*>(a.bnb_desc), st);
  return 0;
}

static bool run_candidate(int c, const ConvArgs& a, const PgArgs& p, hipStream_t st) {
  if (c == -2) return a.res_mode != 3 && !a.x2 && run_old<bf16>(a, st) == 0;
  return pgemm_launch_cfg(p, c, st);
}

static int tune_conv(const ConvArgs& a, const PgArgs& p, hipStream_t st) {
  // statistics / BN-backward sums of the trial runs go to a scratch buffer
  const artsbir_bn_bwd_desc* bd = reinterpret_cast<const artsbir_bn_bwd_desc*>(a.bnb_desc);
  const size_t per = (size_t)a.nseg * ARTSBIR_NSLOT * 2 * a.Cout;
  const size_t need = bd ? per * bd->ntarget : (a.stats ? per : 0);
  if (need > g_tune_stats_n) {
    if (g_tune_stats) (void)hipFree(g_tune_stats);
    g_tune_stats = nullptr;
    g_tune_stats_n = 0;
    if (hipMalloc(&g_tune_stats, need * sizeof(float)) != hipSuccess) return pgemm_default_cfg(p);
    g_tune_stats_n = need;
  }
  ConvArgs at = a;
  PgArgs pt = p;
  artsbir_bn_bwd_desc bt;
  if (a.stats) { at.stats = g_tune_stats; pt.stats = g_tune_stats; }
  if (bd) {
    bt = *bd;
    for (int t = 0; t < bd->ntarget; ++t) { bt.slots[t] = g_tune_stats + t * per; pt.bnb_slots[t] = bt.slots[t]; }
    at.bnb_desc = &bt;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // time the candidates on a quiet device: work queued on other streams (the
  // caller's overlapped weight gradients) would otherwise share the chip with
  // some trials and not others and make the choice noisy
  (void)hipDeviceSynchronize();
  static const int cands[] = {-2, 0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 16, 18, 19, 20, 21, 22, 24, 25, 26};
  int best = -2;
  float best_ms = 1e30f;
  for (int c : cands) {
    if (!run_candidate(c, at, pt, st)) continue;  // also the warm-up
    float ms = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, st);
      run_candidate(c, at, pt, st);
      (void)hipEventRecord(e1, st);
      (void)hipEventSynchronize(e1);
      float t = 0.f;
      (void)hipEventElapsedTime(&t, e0, e1);
      if (t < ms) ms = t;
    }
    if (ms < best_ms) { best_ms = ms; best = c; }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

template <typename T>
static int launch_conv(const ConvArgs& a, hipStream_t st) {
  if ((long long)a.Cout * a.K * sizeof(T) > 0x7fffffffLL) { set_error("conv: weight tensor too large"); return -1; }
  if (a.nseg < 1 || a.M % a.nseg || (a.M / a.nseg) % ((long long)a.Ho * a.Wo)) {
    set_error("conv: %d BN segments do not split %lld output pixels into whole images", a.nseg, a.M);
    return -1;
  }
  const artsbir_bn_bwd_desc* bd = reinterpret_cast<const artsbir_bn_bwd_desc*>(a.bnb_desc);
  if (sizeof(T) == 2 && !a.out_f32 && !a.accumulate && !a.in_scale && !((a.bias || a.relu) && a.stats)) {
    PgArgs p{};
    p.x = a.x; p.x_elems = a.x_elems; p.sN = a.sN; p.sH = a.sH; p.sW = a.sW;
    p.H = a.H; p.W = a.W; p.C = a.C; p.R = a.R; p.S = a.S; p.stride = a.stride; p.pad = a.pad;
    p.Ho = a.Ho; p.Wo = a.Wo; p.w = a.w; p.Cout = a.Cout; p.K = a.K; p.M = a.M;
    p.y = a.y; p.ldy = a.ldy; p.stats = a.stats; p.res = a.res; p.res_mode = a.res_mode;
    p.bias = a.bias; p.relu = a.relu;
    p.x2 = a.x2; p.x2_elems = a.x2_elems; p.sN2 = a.sN2; p.sH2 = a.sH2; p.sW2 = a.sW2; p.C1 = a.C1;
    p.w_sstride = a.w_sstride; p.bias_sstride = a.bias_sstride;
    {
      static const int dbg = getenv("ARTSBIR_PG_DBG") ? atoi(getenv("ARTSBIR_PG_DBG")) : 0;
      p.dbg = dbg;
    }
    p.seg_m = a.nseg > 1 ? a.M / a.nseg : 0;
    p.seg_stride = (long long)ARTSBIR_NSLOT * 2 * a.Cout;
    if (bd) {
      p.bnb = bd->kind == 1 ? 1 : bd->kind == 3 ? 3 : 2;
      p.bnb_nt = bd->ntarget;
      for (int t = 0; t < bd->ntarget; ++t) {
        p.bnb_y[t] = bd->y[t];
        p.bnb_mean[t] = bd->mean[t];
        p.bnb_istd[t] = bd->istd[t];
        p.bnb_slots[t] = bd->slots[t];
      }
      p.bnb_mbn = bd->mask_bn; p.bnb_mask = bd->mask;
      p.bnb_pstride = a.bnb_pstride;
    }
    if (a.wg_p) {  // one kernel produces the data gradient and the weight-gradient operands
      p.wg_p = a.wg_p; p.wg_gram = a.wg_gram;
      if (!pg_fold_wg_launch(p, st)) return 1;
      ARTSBIR_CHECK_LAUNCH("pgemm");
      return 0;
    }
    int choice;
    const char* force = getenv("ARTSBIR_PGEMM_CFG");
    static const char* force_bnb = getenv("ARTSBIR_BNB_CFG");  // experiment: the fused BN-backward dgrads only
    if (force || (bd && force_bnb)) {
      choice = atoi(force ? force : force_bnb);
    } else {
      const ConvKey key{a.M, a.H, a.W, a.C, a.Cout, a.R, a.S, a.stride, a.pad, a.Ho, a.Wo, a.res_mode,
                        (a.stats ? 1 : 0) | (a.bias ? 2 : 0) | (a.relu ? 4 : 0) | (a.x2 ? 8 : 0), a.nseg,
                        bd ? p.bnb * 4 + p.bnb_nt : 0};
      std::lock_guard<std::mutex> lk(g_tune_mu);
      auto it = g_conv_choice.find(key);
      if (it != g_conv_choice.end()) {
        choice = it->second;
      } else {
        const char* tune = getenv("ARTSBIR_TUNE");
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(st, &cs);
        if ((tune && atoi(tune) == 0) || cs != hipStreamCaptureStatusNone) {
          choice = pgemm_default_cfg(p);
          if (choice < 0) choice = -2;
        } else {
          choice = tune_conv(a, p, st);
        }
        g_conv_choice[key] = choice;
      }
    }
    if ((choice != -2 && pgemm_launch_cfg(p, choice, st)) || (bd && force_bnb && pgemm_launch_cfg(p, 0, st))) {
      ARTSBIR_CHECK_LAUNCH("pgemm");
      return 0;
    }
  }
  if (a.res_mode == 3) { set_error("gemm_nt_gate: no kernel for this shape"); return -1; }
  if (a.x2 || a.wg_p) return 1;  // a two-operand fold no pipelined kernel took: the caller's fallback
  return run_old<T>(a, st);
}

extern "C" int artsbir_conv2d_fwd(const artsbir_conv_desc* d, const void* x, const void* w, void* y,
                                  long long ldy, int out_f32, int accumulate, const float* bias,
                                  const float* in_scale, const float* in_shift, int in_relu,
                                  float* stats, void* stream) {
  if (check_conv(d)) return -1;
  if (accumulate && !out_f32) { set_error("conv: accumulate requires f32 output"); return -1; }
  ConvArgs a;
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  a.x = x;
  a.sW = d->C;
  a.sH = (long long)d->W * d->C;
  a.sN = (long long)d->H * d->W * d->C;
  a.x_elems = (long long)d->N * a.sN;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.in_scale = in_scale; a.in_shift = in_shift; a.in_relu = in_relu;
  a.w = w; a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.M = (long long)d->N * Ho * Wo;
  a.y = y; a.ldy = ldy > 0 ? ldy : d->Cout;
  a.out_f32 = out_f32; a.accumulate = accumulate; a.bias = bias; a.stats = stats;
  a.res = nullptr; a.res_mode = 0; a.relu = 0;
  a.nseg = 1; a.bnb_desc = nullptr; a.bnb_pstride = 0;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

extern "C" int artsbir_conv2d_fwd_seg(const artsbir_conv_desc* d, const void* x, const void* w, void* y, int nseg,
                                      float* stats, void* stream) {
  if (check_conv(d)) return -1;
  if (nseg < 1 || d->N % nseg) { set_error("conv2d_fwd_seg: %d segments do not divide batch %d", nseg, d->N); return -1; }
  ConvArgs a;
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  a.x = x;
  a.sW = d->C;
  a.sH = (long long)d->W * d->C;
  a.sN = (long long)d->H * d->W * d->C;
  a.x_elems = (long long)d->N * a.sN;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.w = w; a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.M = (long long)d->N * Ho * Wo;
  a.y = y; a.ldy = d->Cout;
  a.out_f32 = 0; a.accumulate = 0; a.bias = nullptr; a.stats = stats;
  a.res = nullptr; a.res_mode = 0; a.relu = 0;
  a.nseg = nseg; a.bnb_desc = nullptr; a.bnb_pstride = 0;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

// eval-mode Conv2d + BatchNorm2d (folded into w and bias by artsbir_bn_fold) +
// optional residual + optional ReLU in one launch (models.py:198-236 at inference)
extern "C" int artsbir_conv2d_fwd_act(const artsbir_conv_desc* d, const void* x, const void* w, void* y,
                                      const float* bias, const void* res, int res_mode, int relu, void* stream) {
  if (check_conv(d)) return -1;
  if (res_mode != 0 && res_mode != 1) { set_error("conv2d_fwd_act: res_mode %d (0 or 1)", res_mode); return -1; }
  if (res_mode && !res) { set_error("conv2d_fwd_act: residual missing"); return -1; }
  ConvArgs a;
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  a.x = x;
  a.sW = d->C;
  a.sH = (long long)d->W * d->C;
  a.sN = (long long)d->H * d->W * d->C;
  a.x_elems = (long long)d->N * a.sN;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.w = w; a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.M = (long long)d->N * Ho * Wo;
  a.y = y; a.ldy = d->Cout;
  a.out_f32 = 0; a.accumulate = 0; a.bias = bias; a.stats = nullptr;
  a.res = res; a.res_mode = res_mode; a.relu = relu ? 1 : 0;
  a.nseg = 1; a.bnb_desc = nullptr; a.bnb_pstride = 0;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

static int dgrad_common(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx, const void* res,
                        int res_mode, const artsbir_bn_bwd_desc* bnb, int nseg, long long pstride, void* stream);

extern "C" int artsbir_conv2d_dgrad(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx,
                                    const void* res, int res_mode, void* stream) {
  return dgrad_common(d, dy, wd, dx, res, res_mode, nullptr, 1, 0, stream);
}

extern "C" int artsbir_conv2d_dgrad_bnb(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx,
                                        const void* res, int res_mode, const artsbir_bn_bwd_desc* bnb, int nseg,
                                        long long param_stride, void* stream) {
  if (!bnb) { set_error("conv2d_dgrad_bnb: no BN descriptor"); return -1; }
  if (bnb->kind != 0 && bnb->kind != 1 && bnb->kind != 3) {
    set_error("conv2d_dgrad_bnb: kind must be 0, 1 or 3");
    return -1;
  }
  if (bnb->kind == 3 && (d->dtype != ARTSBIR_DT_BF16 || d->C % 8)) {
    set_error("conv2d_dgrad_bnb: bit masks (kind 3) need bf16 and C %% 8 == 0");
    return -1;
  }
  if (bnb->kind == 1 && bnb->pool > 1) { set_error("conv2d_dgrad_bnb: pooled BN inputs are not fused"); return -1; }
  if (bnb->ntarget < 1 || bnb->ntarget > 2 || (bnb->kind == 1 && bnb->ntarget != 1)) {
    set_error("conv2d_dgrad_bnb: bad target count %d", bnb->ntarget);
    return -1;
  }
  if (bnb->kind != 1 ? !bnb->mask : !bnb->mask_bn) {
    set_error("conv2d_dgrad_bnb: missing ReLU mask");
    return -1;
  }
  if (bnb->dtype != d->dtype) { set_error("conv2d_dgrad_bnb: dtype mismatch"); return -1; }
  return dgrad_common(d, dy, wd, dx, res, res_mode, bnb, nseg, param_stride, stream);
}

static int dgrad_common(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx, const void* res,
                        int res_mode, const artsbir_bn_bwd_desc* bnb, int nseg, long long pstride, void* stream) {
  // data gradient of a stride-1 convolution: a convolution of dy [N][H][W][Cout]
  // with the flipped, transposed weights wd [Cin][R][S][Cout] and padding R-1-pad.
  if (check_conv(d)) return -1;
  if (d->stride != 1) { set_error("conv2d_dgrad: only stride 1 (got %d)", d->stride); return -1; }
  if (d->Cout % 8 || d->C % 8) { set_error("conv2d_dgrad: channels must be multiples of 8"); return -1; }
  if (res_mode < 0 || res_mode > 2 || (res_mode && !res)) { set_error("conv2d_dgrad: bad residual"); return -1; }
  if (res_mode == 2 && (d->H % 2 || d->W % 2)) { set_error("conv2d_dgrad: unpool residual needs even H, W"); return -1; }
  if (nseg < 1 || d->N % nseg) { set_error("conv2d_dgrad: %d segments do not divide batch %d", nseg, d->N); return -1; }
  ConvArgs a;
  const int pad = d->R - 1 - d->pad;
  a.x = dy;
  a.sW = d->Cout; a.sH = (long long)d->W * d->Cout; a.sN = (long long)d->H * d->W * d->Cout;
  a.x_elems = (long long)d->N * a.sN;
  a.H = d->H; a.W = d->W; a.C = d->Cout;
  a.R = d->R; a.S = d->S; a.stride = 1; a.pad = pad;
  a.Ho = d->H + 2 * pad - d->R + 1; a.Wo = d->W + 2 * pad - d->S + 1;
  if (a.Ho != d->H || a.Wo != d->W) { set_error("conv2d_dgrad: only 'same' convolutions"); return -1; }
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.w = wd; a.Cout = d->C; a.K = d->R * d->S * d->Cout;
  a.M = (long long)d->N * d->H * d->W;
  a.y = dx; a.ldy = d->C;
  a.out_f32 = 0; a.accumulate = 0; a.bias = nullptr; a.stats = nullptr;
  a.res = res; a.res_mode = res_mode; a.relu = 0;
  a.nseg = nseg; a.bnb_desc = bnb; a.bnb_pstride = pstride;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

// ---------------------------------------------------------------------------
// Data gradient of a 1x1 convolution with the BatchNorm backward of its output
// folded in (artsbir.h: artsbir_conv1x1_dgrad_fold).  The reference's chain
// conv -> BatchNorm2d (models.py:219-220 conv3 -> bn3, 227-229 downsample conv ->
// BN) is differentiated by autograd as dy = c1 (g - c2 - xhat c3) followed by
// dx = dy W; since y = x W^T the whole chain is linear in (g, x):
//   dx = g (diag(c1) W) + x (W^T diag(b') W) + e,  b' = -c1 c3 istd,
//   e = (-c1 (c2 - c3 istd mean)) W
// per BN segment, so it runs as ONE GEMM over the concatenated reduction
// [g | x] (K = Co + Ci) with per-segment weights (artsbir_bn_fold_bwd_prep) and
// bias — no dy tensor is written or read.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) fold_concat_kernel(const T* __restrict__ g, const T* __restrict__ x, T* out,
                                                          long long M, int Co, int C2) {
  constexpr int EPC = 16 / sizeof(T);
  const int cg = (Co + C2) / EPC;  // 16-B chunks per output row
  const long long n = M * cg;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long m = i / cg;
    const int c = (int)(i - m * cg) * EPC;
    const uint4 v = c < Co ? *reinterpret_cast<const uint4*>(g + m * Co + c)
                           : *reinterpret_cast<const uint4*>(x + m * C2 + (c - Co));
    *reinterpret_cast<uint4*>(out + m * (Co + C2) + c) = v;
  }
}

// One fold launch: dx [N][H][W][Ci] = [g | x2] w_s^T + bias_s (+ residual) for
// the pixels of BN segment s, g with Co channels, x2 with C2 (the conv input x,
// C2 = Ci: artsbir_conv1x1_dgrad_fold; the BN input y, C2 = Co:
// artsbir_conv1x1_dgrad_fold_y), an optional fused BN-backward reduction of the
// gradient it produces
struct FoldOp {
  const artsbir_conv_desc* d;
  const void* g;
  const void* x2;
  int C2;
  const void* w;
  const float* bias;
  void* dx;
  const void* res;
  int res_mode;
  const artsbir_bn_bwd_desc* bnb;
  int nseg;
  long long pstride;
};

static int fold_concat_gemms(const FoldOp& f, const ConvArgs& a, void* ws, hipStream_t st);

// the segment s slice of a fused BN-backward descriptor (its tensors, mask and
// BN parameters advanced by whole segments)
static artsbir_bn_bwd_desc bnb_segment(const artsbir_bn_bwd_desc* bd, int s, long long seg_m, int C, long long pstride) {
  artsbir_bn_bwd_desc d = *bd;
  const long long es = bd->dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  d.nseg = 1;
  if (bd->mask_bn) d.mask_bn = bd->mask_bn + s * pstride;
  if (bd->mask)  // kind 3: one mask byte per 8 channels; kind 0: the block output
    d.mask = reinterpret_cast<const char*>(bd->mask) + (bd->kind == 3 ? s * seg_m * (C / 8) : s * seg_m * C * es);
  for (int t = 0; t < bd->ntarget; ++t) {
    d.y[t] = reinterpret_cast<const char*>(bd->y[t]) + s * seg_m * C * es;
    d.mean[t] = bd->mean[t] + s * pstride;
    d.istd[t] = bd->istd[t] + s * pstride;
    d.slots[t] = bd->slots[t] + (long long)s * ARTSBIR_NSLOT * 2 * C;
  }
  return d;
}

static int fold_check(const FoldOp& f) {
  const artsbir_conv_desc* d = f.d;
  if (check_conv(d)) return -1;
  if (d->R != 1 || d->S != 1 || d->stride != 1 || d->pad != 0) { set_error("conv1x1_dgrad_fold: 1x1 stride-1 convolutions only"); return -1; }
  if (!f.g || !f.x2 || !f.w || !f.bias || !f.dx) { set_error("conv1x1_dgrad_fold: null operand"); return -1; }
  if (d->Cout % 8 || d->C % 8 || f.C2 % 8 || f.C2 <= 0) { set_error("conv1x1_dgrad_fold: channels must be multiples of 8"); return -1; }
  if (f.nseg < 1 || d->N % f.nseg) { set_error("conv1x1_dgrad_fold: %d segments do not divide batch %d", f.nseg, d->N); return -1; }
  if (f.res_mode < 0 || f.res_mode > 2 || (f.res_mode && !f.res)) { set_error("conv1x1_dgrad_fold: bad residual"); return -1; }
  if (f.res_mode == 2 && (d->H % 2 || d->W % 2)) { set_error("conv1x1_dgrad_fold: unpool residual needs even H, W"); return -1; }
  if (f.res_mode == 2 && (d->N / f.nseg) * d->H * d->W % 4) { set_error("conv1x1_dgrad_fold: unpool residual segments"); return -1; }
  if (const artsbir_bn_bwd_desc* b = f.bnb) {
    if (b->dtype != d->dtype || b->pool > 1) { set_error("conv1x1_dgrad_fold: bad fused BN backward"); return -1; }
    if (b->kind == 1) {
      if (b->ntarget != 1 || !b->mask_bn || f.res_mode) {
        set_error("conv1x1_dgrad_fold: a kind-1 fused BN backward takes one target and no residual");
        return -1;
      }
    } else if (b->kind == 0 || b->kind == 3) {
      if (b->ntarget < 1 || b->ntarget > 2 || !b->mask || !f.res_mode) {
        set_error("conv1x1_dgrad_fold: a kind-0/3 fused BN backward takes 1-2 targets, a mask and a residual");
        return -1;
      }
      if (b->kind == 3 && (d->dtype != ARTSBIR_DT_BF16 || d->C % 8)) { set_error("conv1x1_dgrad_fold: bit masks need bf16"); return -1; }
    } else {
      set_error("conv1x1_dgrad_fold: fused BN-backward kind %d", b->kind);
      return -1;
    }
  }
  return 0;
}

// the two-operand / per-segment-weight launch arguments of the fold
static ConvArgs fold_conv_args(const FoldOp& f) {
  const artsbir_conv_desc* d = f.d;
  const int Co = d->Cout, Ci = d->C, K = Co + f.C2;
  const long long M = (long long)d->N * d->H * d->W;
  ConvArgs a;
  a.x = f.g; a.sW = Co; a.sH = (long long)d->W * Co; a.sN = (long long)d->H * d->W * Co; a.x_elems = M * Co;
  a.x2 = f.x2; a.sW2 = f.C2; a.sH2 = (long long)d->W * f.C2; a.sN2 = (long long)d->H * d->W * f.C2; a.x2_elems = M * f.C2;
  a.C1 = Co;
  a.H = d->H; a.W = d->W; a.C = K;
  a.R = 1; a.S = 1; a.stride = 1; a.pad = 0; a.Ho = d->H; a.Wo = d->W;
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.w = f.w; a.Cout = Ci; a.K = K; a.M = M;
  a.y = f.dx; a.ldy = Ci;
  a.out_f32 = 0; a.accumulate = 0; a.bias = f.bias; a.stats = nullptr;
  a.res = f.res; a.res_mode = f.res_mode; a.relu = 0;
  a.nseg = f.nseg; a.bnb_desc = f.bnb; a.bnb_pstride = f.pstride;
  a.w_sstride = (long long)Ci * K; a.bias_sstride = Ci;
  return a;
}

// segment s's slice of a fold launch (one BN segment, its weights and bias)
static ConvArgs fold_segment(const FoldOp& f, const ConvArgs& a, int s, artsbir_bn_bwd_desc* bs) {
  const int Co = f.d->Cout, Ci = f.d->C;
  const long long seg_m = a.M / f.nseg;
  const long long es = f.d->dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  ConvArgs p = a;
  if (f.bnb) { *bs = bnb_segment(f.bnb, s, seg_m, Ci, f.pstride); p.bnb_desc = bs; }
  p.nseg = 1; p.M = seg_m;
  p.x = reinterpret_cast<const char*>(f.g) + s * seg_m * Co * es; p.x_elems = seg_m * Co;
  p.x2 = reinterpret_cast<const char*>(f.x2) + s * seg_m * f.C2 * es; p.x2_elems = seg_m * f.C2;
  p.w = reinterpret_cast<const char*>(f.w) + s * a.w_sstride * es;
  p.bias = f.bias + s * Ci;
  p.y = reinterpret_cast<char*>(f.dx) + s * seg_m * Ci * es;
  if (f.res_mode) p.res = reinterpret_cast<const char*>(f.res) + s * (f.res_mode == 2 ? seg_m / 4 : seg_m) * Ci * es;
  return p;
}

static int fold_dgrad(const FoldOp& f, hipStream_t st) {
  if (fold_check(f)) return -1;
  const artsbir_conv_desc* d = f.d;
  const int K = d->Cout + f.C2;
  const long long M = (long long)d->N * d->H * d->W;
  const bool bf = d->dtype == ARTSBIR_DT_BF16;
  const long long es = bf ? 2 : 4;
  const ConvArgs a = fold_conv_args(f);
  // one launch over every segment, else one per segment (the tiles of a
  // launch then never straddle two), on the two-operand pipelined kernels
  if (bf) {
    int rc = launch_conv<bf16>(a, st);
    if (rc <= 0) return rc;
    // no kernel took the whole batch (a tile would straddle two segments): one
    // launch per segment; segment 0 decides, a refusal there drops to the
    // concatenated form below (every segment has the same shape)
    for (int s = 0; s < f.nseg; ++s) {
      artsbir_bn_bwd_desc bs;
      const ConvArgs p = fold_segment(f, a, s, &bs);
      rc = launch_conv<bf16>(p, st);
      if (rc < 0) return rc;
      if (rc > 0) {
        if (s > 0) { set_error("conv1x1_dgrad_fold: segment %d has no kernel", s); return -1; }
        break;
      }
    }
    if (rc == 0) return 0;
  }
  // f32 (the parity mode) and shapes the pipelined kernels do not take: the two
  // operands concatenated per pixel, then one plain GEMM per segment.  The
  // concatenated operand is stream-ordered scratch (hipMallocAsync / hipFreeAsync
  // on the caller's stream): no process-wide buffer shared across devices or
  // threads, no device-synchronous hipFree in the middle of a step
  const size_t need = (size_t)(M * K * es);
  void* ws = nullptr;
  if (hipMallocAsync(&ws, need, st) != hipSuccess) {
    set_error("conv1x1_dgrad_fold: workspace of %zu bytes", need);
    return -1;
  }
  const int rc = fold_concat_gemms(f, a, ws, st);
  (void)hipFreeAsync(ws, st);
  return rc;
}

extern "C" int artsbir_conv1x1_dgrad_fold(const artsbir_conv_desc* d, const void* g, const void* x, const void* w,
                                          const float* bias, void* dx, const artsbir_bn_bwd_desc* bnb, int nseg,
                                          long long param_stride, void* stream) {
  if (bnb && bnb->kind != 1) { set_error("conv1x1_dgrad_fold: the fused BN backward must be kind 1 with one target"); return -1; }
  const FoldOp f{d, g, x, d ? d->C : 0, w, bias, dx, nullptr, 0, bnb, nseg, param_stride};
  return fold_dgrad(f, (hipStream_t)stream);
}

extern "C" int artsbir_conv1x1_dgrad_fold_y(const artsbir_conv_desc* d, const void* g, const void* y, const void* w,
                                            const float* bias, void* dx, const void* res, int res_mode,
                                            const artsbir_bn_bwd_desc* bnb, int nseg, long long param_stride,
                                            void* stream) {
  const FoldOp f{d, g, y, d ? d->Cout : 0, w, bias, dx, res, res_mode, bnb, nseg, param_stride};
  return fold_dgrad(f, (hipStream_t)stream);
}

static int fold_concat_gemms(const FoldOp& f, const ConvArgs& a, void* ws, hipStream_t st) {
  const artsbir_conv_desc* d = f.d;
  const int Co = d->Cout, K = Co + f.C2;
  const long long M = (long long)d->N * d->H * d->W, seg_m = M / f.nseg;
  const bool bf = d->dtype == ARTSBIR_DT_BF16;
  const long long es = bf ? 2 : 4;
  {
    const long long n = M * (K * es / 16);
    const unsigned grid = (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
    if (bf)
      hipLaunchKernelGGL(fold_concat_kernel<bf16>, dim3(grid), dim3(256), 0, st, reinterpret_cast<const bf16*>(f.g),
                         reinterpret_cast<const bf16*>(f.x2), reinterpret_cast<bf16*>(ws), M, Co, f.C2);
    else
      hipLaunchKernelGGL(fold_concat_kernel<float>, dim3(grid), dim3(256), 0, st, reinterpret_cast<const float*>(f.g),
                         reinterpret_cast<const float*>(f.x2), reinterpret_cast<float*>(ws), M, Co, f.C2);
    ARTSBIR_CHECK_LAUNCH("fold_concat");
  }
  for (int s = 0; s < f.nseg; ++s) {
    artsbir_bn_bwd_desc bs;
    ConvArgs p = fold_segment(f, a, s, &bs);
    p.x2 = nullptr; p.C1 = 0; p.w_sstride = 0; p.bias_sstride = 0;
    p.x = reinterpret_cast<const char*>(ws) + s * seg_m * K * es; p.x_elems = seg_m * K;
    p.sW = K; p.sH = (long long)d->W * K; p.sN = (long long)d->H * d->W * K;
    const int rc = bf ? launch_conv<bf16>(p, st) : launch_conv<float>(p, st);
    if (rc) return -1;
  }
  return 0;
}

// The fold's data gradient and, from the same pass, the operands of its weight
// gradient (artsbir.h: artsbir_conv1x1_dgrad_fold_wg): per segment s
// P[s] += g_s^T x_s ([Co][Ci]) and gram[s] += x_s^T x_s ([Ci][Ci]), f32.  One
// kernel where pg_fold_wg_launch takes the shape; otherwise the data gradient
// (artsbir_conv1x1_dgrad_fold) and one artsbir_gemm_tn2 per segment.
extern "C" int artsbir_conv1x1_dgrad_fold_wg(const artsbir_conv_desc* d, const void* g, const void* x, const void* w,
                                             const float* bias, void* dx, const artsbir_bn_bwd_desc* bnb, int nseg,
                                             long long param_stride, float* P, float* gram, void* stream) {
  if (bnb && bnb->kind != 1) { set_error("conv1x1_dgrad_fold_wg: the fused BN backward must be kind 1"); return -1; }
  const FoldOp f{d, g, x, d ? d->C : 0, w, bias, dx, nullptr, 0, bnb, nseg, param_stride};
  if (fold_check(f)) return -1;
  if (!P || !gram) { set_error("conv1x1_dgrad_fold_wg: null weight-gradient operand"); return -1; }
  const int Co = d->Cout, Ci = d->C;
  const long long M = (long long)d->N * d->H * d->W, seg_m = M / nseg;
  const long long es = d->dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  static const bool off = getenv("ARTSBIR_FOLD_WG") && atoi(getenv("ARTSBIR_FOLD_WG")) == 0;  // measurement switch
  if (d->dtype == ARTSBIR_DT_BF16 && !off) {
    ConvArgs a = fold_conv_args(f);
    a.wg_p = P; a.wg_gram = gram;
    const int rc = launch_conv<bf16>(a, (hipStream_t)stream);
    if (rc <= 0) return rc;
  }
  if (artsbir_conv1x1_dgrad_fold(d, g, x, w, bias, dx, bnb, nseg, param_stride, stream)) return -1;
  for (int s = 0; s < nseg; ++s) {
    const char* gs = reinterpret_cast<const char*>(g) + s * seg_m * Co * es;
    const char* xs = reinterpret_cast<const char*>(x) + s * seg_m * Ci * es;
    if (artsbir_gemm_tn2(d->dtype, seg_m, Co, Ci, Ci, gs, Co, xs, Ci, xs, Ci, P + (long long)s * Co * Ci,
                         gram + (long long)s * Ci * Ci, stream))
      return -1;
  }
  return 0;
}

extern "C" int artsbir_gemm_nt(int dtype, long long M, int N, int K, const void* a, long long lda,
                               const void* b, void* c, long long ldc, int out_f32, int accumulate,
                               const float* bias, float* stats, void* stream) {
  if (K % 8 != 0 || lda % 8 != 0) { set_error("gemm_nt: K=%d and lda=%lld must be multiples of 8", K, lda); return -1; }
  if (accumulate && !out_f32) { set_error("gemm_nt: accumulate requires f32 output"); return -1; }
  if (M <= 0 || N <= 0) return 0;
  if (M > 0x7fffffffLL) { set_error("gemm_nt: M too large"); return -1; }
  // dense rows as "images" of one pixel: row offsets stay relative to the tile
  ConvArgs p;
  p.x = a; p.sN = lda; p.sH = 0; p.sW = 0;
  p.x_elems = (M - 1) * lda + K;
  p.H = 1; p.W = 1; p.C = K;
  p.R = 1; p.S = 1; p.stride = 1; p.pad = 0; p.Ho = 1; p.Wo = 1;
  p.in_scale = nullptr; p.in_shift = nullptr; p.in_relu = 0;
  p.w = b; p.Cout = N; p.K = K; p.M = M;
  p.y = c; p.ldy = ldc > 0 ? ldc : N;
  p.out_f32 = out_f32; p.accumulate = accumulate; p.bias = bias; p.stats = stats;
  p.res = nullptr; p.res_mode = 0; p.relu = 0;
  p.nseg = 1; p.bnb_desc = nullptr; p.bnb_pstride = 0;
  hipStream_t st = (hipStream_t)stream;
  return dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(p, st) : launch_conv<float>(p, st);
}

// C[M][N] = (A[M][K] B[N][K]^T) * quickgelu'(X[M][N]) in bf16, with the column
// sums of C added into stats ([ARTSBIR_NSLOT][2][N] f32 slots, sum and sum of
// squares): the ViT MLP backward's c_proj data gradient, QuickGELU backward
// and c_fc bias gradient (models.py:391-393, 412-417) in one pass
extern "C" int artsbir_gemm_nt_gate(long long M, int N, int K, const void* a, long long lda, const void* b, void* c,
                                    long long ldc, const void* x, float* stats, void* stream) {
  if (K % 8 != 0 || lda % 8 != 0 || N % 8 != 0) { set_error("gemm_nt_gate: K, lda and N must be multiples of 8"); return -1; }
  if (!a || !b || !c || !x) { set_error("gemm_nt_gate: null operand"); return -1; }
  if (M <= 0 || N <= 0) return 0;
  if (M > 0x7fffffffLL) { set_error("gemm_nt_gate: M too large"); return -1; }
  ConvArgs p;
  p.x = a; p.sN = lda; p.sH = 0; p.sW = 0;
  p.x_elems = (M - 1) * lda + K;
  p.H = 1; p.W = 1; p.C = K;
  p.R = 1; p.S = 1; p.stride = 1; p.pad = 0; p.Ho = 1; p.Wo = 1;
  p.in_scale = nullptr; p.in_shift = nullptr; p.in_relu = 0;
  p.w = b; p.Cout = N; p.K = K; p.M = M;
  p.y = c; p.ldy = ldc > 0 ? ldc : N;
  p.out_f32 = 0; p.accumulate = 0; p.bias = nullptr; p.stats = stats;
  p.res = x; p.res_mode = 3; p.relu = 0;
  p.nseg = 1; p.bnb_desc = nullptr; p.bnb_pstride = 0;
  return launch_conv<bf16>(p, (hipStream_t)stream);
}

template <typename T, int BM, int BN>
static void launch_wgrad_tile(WgradArgs& a, hipStream_t st) {
  constexpr int BK = 8 * MM<T>::EPC;
  const int tiles = ((a.Cout + BM - 1) / BM) * ((a.K + BN - 1) / BN);
  // ~4 workgroups per CU in total, but >= 8 K-steps per workgroup
  long long ksteps = (a.M + BK - 1) / BK;
  long long splits = (1024 + tiles - 1) / tiles;
  long long max_splits = (ksteps + 7) / 8;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long long per = (ksteps + splits - 1) / splits;
  // keep every block-relative byte offset and pixel index in 31 / 24 bits
  const long long ld = a.dense ? (a.ldx > a.ldd ? a.ldx : a.ldd) : a.ldd;
  long long cap = (1LL << 22) / BK;
  const long long cap2 = ((1LL << 30) / ((ld + 1) * (long long)sizeof(T))) / BK;
  if (cap2 < cap) cap = cap2;
  if (!a.dense) {  // images spanned by one block's pixel range
    const long long imgs = (1LL << 30) / (a.sN * (long long)sizeof(T)) - 2;
    const long long cap3 = imgs > 0 ? imgs * a.Ho * a.Wo / BK : 1;
    if (cap3 < cap) cap = cap3;
  }
  if (cap < 1) cap = 1;
  if (per > cap) per = cap;
  a.m_per_split = per * BK;
  splits = (ksteps + per - 1) / per;
  if (a.in_scale)
    hipLaunchKernelGGL((wgrad_kernel<T, BM, BN, true>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((wgrad_kernel<T, BM, BN, false>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, a);
}

// wgrad kernel choice per shape (bf16): register-staged wgrad_kernel (-1) or
// a tile configuration c >= 0 of the pipelined LDS-DMA transposed-read kernel
// (pwgrad.hip); tuned on first use into a scratch gradient buffer (the real dW
// is accumulated into, so candidates must not touch it); ARTSBIR_TUNE=0 keeps
// the register-staged kernel, ARTSBIR_WGRAD_CFG=<c> forces a candidate.
struct WgKey {
  long long M;
  int H, W, C, Cout, R, S, stride, pad, dense, K;
  long long ldd, ldx;
  bool operator<(const WgKey& o) const {
    return std::tie(M, H, W, C, Cout, R, S, stride, pad, dense, K, ldd, ldx) <
           std::tie(o.M, o.H, o.W, o.C, o.Cout, o.R, o.S, o.stride, o.pad, o.dense, o.K, o.ldd, o.ldx);
  }
};
static std::map<WgKey, int> g_wg_choice;
static float* g_tune_dw = nullptr;
static size_t g_tune_dw_n = 0;

static PwArgs to_pw(const WgradArgs& a) {
  PwArgs p;
  p.dy = a.dy; p.dy_elems = a.dy_elems; p.ldd = a.ldd;
  p.x = a.x; p.x_elems = a.x_elems; p.sN = a.sN; p.sH = a.sH; p.sW = a.sW;
  p.H = a.H; p.W = a.W; p.C = a.C; p.R = a.R; p.S = a.S; p.stride = a.stride; p.pad = a.pad;
  p.Ho = a.Ho; p.Wo = a.Wo; p.dense = a.dense; p.ldx = a.ldx;
  p.Cout = a.Cout; p.K = a.K; p.M = a.M; p.m_per_split = 0; p.dw = a.dw;
  p.dy2 = a.dy2; p.dy2_elems = a.dy2_elems; p.ldd2 = a.ldd2; p.Cout1 = a.Cout1; p.dw2 = a.dw2;
  static const int dbg = getenv("ARTSBIR_PW_DBG") ? atoi(getenv("ARTSBIR_PW_DBG")) : 0;
  p.dbg = dbg;
  return p;
}

template <typename T>
static void launch_wgrad_old(WgradArgs& a, hipStream_t st);

// candidate -1: register-staged wgrad_kernel; c >= 0: pipelined config c
static bool run_wg_candidate(int c, WgradArgs& a, hipStream_t st) {
  if (c >= 100) return pw256_launch(to_pw(a), c - 100, st);
  if (c >= 0) return pwgrad_launch(to_pw(a), c, st);
  if (a.dy2) return false;  // the register-staged kernel reads one dY
  launch_wgrad_old<bf16>(a, st);
  return true;
}

static int tune_wgrad(const WgradArgs& a, hipStream_t st) {
  const size_t need = (size_t)a.Cout * a.K;
  if (need > g_tune_dw_n) {
    if (g_tune_dw) (void)hipFree(g_tune_dw);
    g_tune_dw = nullptr;
    g_tune_dw_n = 0;
    if (hipMalloc(&g_tune_dw, need * sizeof(float)) != hipSuccess) return -1;
    g_tune_dw_n = need;
  }
  WgradArgs at = a;
  at.dw = g_tune_dw;
  if (a.dy2) at.dw2 = g_tune_dw + (size_t)a.Cout1 * a.K;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipDeviceSynchronize();  // quiet device (see tune_conv)
  int best = -1;
  float best_ms = 1e30f;
  // ARTSBIR_WGRAD_MINLEVEL=L: only split levels >= L (fewer workgroups; the
  // weight gradients share the chip with the data-gradient stream, which the
  // standalone timing here cannot see)
  static const int minlevel = getenv("ARTSBIR_WGRAD_MINLEVEL") ? atoi(getenv("ARTSBIR_WGRAD_MINLEVEL")) : 0;
  for (int ci = -1; ci < pwgrad_num_cfgs() + 3; ++ci) {
    const int c = ci < pwgrad_num_cfgs() ? ci : 100 + ci - pwgrad_num_cfgs();  // then pw256 at 3 split levels
    if (c >= 0 && pwgrad_level(c) >= 0 && pwgrad_level(c) < minlevel) continue;
    if (!run_wg_candidate(c, at, st)) continue;
    float ms = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, st);
      run_wg_candidate(c, at, st);
      (void)hipEventRecord(e1, st);
      (void)hipEventSynchronize(e1);
      float t = 0.f;
      (void)hipEventElapsedTime(&t, e0, e1);
      if (t < ms) ms = t;
    }
    if (ms < best_ms) { best_ms = ms; best = c; }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

template <typename T>
static int launch_wgrad(WgradArgs& a, hipStream_t st) {
  if (sizeof(T) == 2 && !a.in_scale) {
    int choice;
    const char* force = getenv("ARTSBIR_WGRAD_CFG");
    if (force) {
      choice = atoi(force);
    } else {
      // (dense 2: dY in two parts, artsbir_gemm_tn2)
      const WgKey key{a.M, a.H, a.W, a.C, a.Cout, a.R, a.S, a.stride, a.pad, a.dy2 ? 2 : a.dense, a.K, a.ldd, a.ldx};
      std::lock_guard<std::mutex> lk(g_tune_mu);
      auto it = g_wg_choice.find(key);
      if (it != g_wg_choice.end()) {
        choice = it->second;
      } else {
        const char* tune = getenv("ARTSBIR_TUNE");
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        (void)hipStreamIsCapturing(st, &cs);
        choice = ((tune && atoi(tune) == 0) || cs != hipStreamCaptureStatusNone) ? -1 : tune_wgrad(a, st);
        g_wg_choice[key] = choice;
      }
    }
    if (choice >= 100 && pw256_launch(to_pw(a), choice - 100, st)) {
      ARTSBIR_CHECK_LAUNCH("pw256");
      return 0;
    }
    if (choice >= 0 && choice < 100 && pwgrad_launch(to_pw(a), choice, st)) {
      ARTSBIR_CHECK_LAUNCH("pwgrad");
      return 0;
    }
  }
  if (a.dy2) return 1;  // no pipelined kernel took the two-part dY: the caller splits it
  launch_wgrad_old<T>(a, st);
  ARTSBIR_CHECK_LAUNCH("wgrad");
  return 0;
}

template <typename T>
static void launch_wgrad_old(WgradArgs& a, hipStream_t st) {
  const bool bf = sizeof(T) == 2;
  if (a.Cout <= 64) {
    set_last_kernel(bf ? "wgrad_kernel<bf16,64,128>" : "wgrad_kernel<f32,64,128>");
    launch_wgrad_tile<T, 64, 128>(a, st);
  } else {
    set_last_kernel(bf ? "wgrad_kernel<bf16,128,128>" : "wgrad_kernel<f32,128,128>");
    launch_wgrad_tile<T, 128, 128>(a, st);
  }
}

extern "C" int artsbir_conv2d_wgrad(const artsbir_conv_desc* d, const void* dy, const void* x,
                                    const float* in_scale, const float* in_shift, int in_relu,
                                    float* dw, void* stream) {
  if (check_conv(d)) return -1;
  if (d->Cout % 8 != 0) { set_error("wgrad: Cout=%d must be a multiple of 8", d->Cout); return -1; }
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  WgradArgs a;
  a.dy = dy; a.ldd = d->Cout;
  a.M = (long long)d->N * Ho * Wo;
  a.dy_elems = a.M * d->Cout;
  a.x = x;
  a.sW = d->C; a.sH = (long long)d->W * d->C; a.sN = (long long)d->H * d->W * d->C;
  a.x_elems = (long long)d->N * a.sN;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.dense = (d->R == 1 && d->S == 1 && d->stride == 1 && d->pad == 0 && !in_scale) ? 1 : 0;
  a.ldx = d->C;
  a.in_scale = in_scale; a.in_shift = in_shift; a.in_relu = in_relu;
  a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.dw = dw;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_wgrad<bf16>(a, st) : launch_wgrad<float>(a, st);
}

// Autotuner cache as a text file: one line per tuned shape ("c" conv keys, "w"
// wgrad keys, then the choice).  bench.py saves it after a run and the profiled
// re-runs load it first, so rocprofv3 / PMC passes see only the launches of the
// steady-state step, no trial launches.
extern "C" int artsbir_tune_save(const char* path) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  FILE* f = fopen(path, "w");
  if (!f) { set_error("tune_save: cannot open %s", path); return -1; }
  for (const auto& kv : g_conv_choice) {
    const ConvKey& k = kv.first;
    fprintf(f, "c %lld %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d\n", k.M, k.H, k.W, k.C, k.Cout, k.R, k.S,
            k.stride, k.pad, k.Ho, k.Wo, k.res_mode, k.stats, k.nseg, k.bnb, kv.second);
  }
  for (const auto& kv : g_wg_choice) {
    const WgKey& k = kv.first;
    fprintf(f, "w %lld %d %d %d %d %d %d %d %d %d %d %lld %lld %d\n", k.M, k.H, k.W, k.C, k.Cout, k.R, k.S, k.stride,
            k.pad, k.dense, k.K, k.ldd, k.ldx, kv.second);
  }
  fclose(f);
  return 0;
}

// returns the number of entries loaded (existing entries are overwritten)
extern "C" int artsbir_tune_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  FILE* f = fopen(path, "r");
  if (!f) { set_error("tune_load: cannot open %s", path); return -1; }
  int n = 0;
  char tag[4];
  while (fscanf(f, "%3s", tag) == 1) {
    int choice;
    if (tag[0] == 'c') {
      ConvKey k;
      if (fscanf(f, "%lld %d %d %d %d %d %d %d %d %d %d %d %d %d %d %d", &k.M, &k.H, &k.W, &k.C, &k.Cout, &k.R, &k.S,
                 &k.stride, &k.pad, &k.Ho, &k.Wo, &k.res_mode, &k.stats, &k.nseg, &k.bnb, &choice) != 16)
        break;
      if (choice < -2 || choice == 23) continue;  // retired candidates (hipBLASLt -3, persistent pp256): re-tune
      g_conv_choice[k] = choice;
    } else if (tag[0] == 'w') {
      WgKey k;
      if (fscanf(f, "%lld %d %d %d %d %d %d %d %d %d %d %lld %lld %d", &k.M, &k.H, &k.W, &k.C, &k.Cout, &k.R, &k.S,
                 &k.stride, &k.pad, &k.dense, &k.K, &k.ldd, &k.ldx, &choice) != 14)
        break;
      if (choice < -1) continue;  // the retired hipBLASLt candidate: re-tune
      g_wg_choice[k] = choice;
    } else {
      break;
    }
    ++n;
  }
  fclose(f);
  return n;
}

// dw[n][k] += sum_m dy[m][n] x[m][k] (n < N1) and dw2[n][k] += sum_m dy2[m][n] x[m][k]
// (n < N2) in one launch where a pipelined kernel takes it (the folded BatchNorm
// backward's g^T x and x^T x, fold.hip), else as two artsbir_gemm_tn
extern "C" int artsbir_gemm_tn2(int dtype, long long M, int N1, int N2, int K, const void* dy, long long ldd,
                                const void* dy2, long long ldd2, const void* x, long long ldx, float* dw, float* dw2,
                                void* stream) {
  if (N1 % 8 || N2 % 8 || K % 8 || ldd % 8 || ldd2 % 8 || ldx % 8) {
    set_error("gemm_tn2: N1=%d N2=%d K=%d and the row strides must be multiples of 8", N1, N2, K);
    return -1;
  }
  if (M <= 0) return 0;
  if (dtype == ARTSBIR_DT_BF16) {
    WgradArgs a;
    a.dy = dy; a.ldd = ldd; a.dy_elems = (M - 1) * ldd + N1;
    a.x = x; a.x_elems = (M - 1) * ldx + K;
    a.sN = 0; a.sH = 0; a.sW = 0; a.H = 1; a.W = 1; a.C = K;
    a.R = 1; a.S = 1; a.stride = 1; a.pad = 0; a.Ho = 1; a.Wo = 1;
    a.dense = 1; a.ldx = ldx;
    a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
    a.Cout = N1 + N2; a.K = K; a.M = M; a.dw = dw;
    a.dy2 = dy2; a.ldd2 = ldd2; a.dy2_elems = (M - 1) * ldd2 + N2; a.Cout1 = N1; a.dw2 = dw2;
    const int rc = launch_wgrad<bf16>(a, (hipStream_t)stream);
    if (rc <= 0) return rc;
  }
  const int rc = artsbir_gemm_tn(dtype, M, N1, K, dy, ldd, x, ldx, dw, stream);
  return rc ? rc : artsbir_gemm_tn(dtype, M, N2, K, dy2, ldd2, x, ldx, dw2, stream);
}

extern "C" int artsbir_gemm_tn(int dtype, long long M, int N, int K, const void* dy, long long ldd,
                               const void* x, long long ldx, float* dw, void* stream) {
  // dw[N][K] += sum_m dy[m][n] * x[m][k]
  if (N % 8 != 0 || K % 8 != 0 || ldd % 8 != 0 || ldx % 8 != 0) {
    set_error("gemm_tn: N=%d K=%d ldd=%lld ldx=%lld must be multiples of 8", N, K, ldd, ldx);
    return -1;
  }
  if (M <= 0) return 0;
  WgradArgs a;
  a.dy = dy; a.ldd = ldd; a.dy_elems = (M - 1) * ldd + N;
  a.x = x; a.x_elems = (M - 1) * ldx + K;
  a.sN = 0; a.sH = 0; a.sW = 0; a.H = 1; a.W = 1; a.C = K;
  a.R = 1; a.S = 1; a.stride = 1; a.pad = 0; a.Ho = 1; a.Wo = 1;
  a.dense = 1; a.ldx = ldx;
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.Cout = N; a.K = K; a.M = M; a.dw = dw;
  hipStream_t st = (hipStream_t)stream;
  return dtype == ARTSBIR_DT_BF16 ? launch_wgrad<bf16>(a, st) : launch_wgrad<float>(a, st);
}
