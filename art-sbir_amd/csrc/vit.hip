// Transformer block pieces of models.py:382-417 (LayerNorm computed in fp32,
// QuickGELU, the multi-head self-attention core of nn.MultiheadAttention as
// ResidualAttentionBlock uses it).  The reference defines the block but builds
// no model from it (block-level parity); its projections run on
// the MFMA GEMM (artsbir_gemm_nt), these kernels are the rest.
//
// Layouts follow nn.MultiheadAttention (batch_first=False): x [L][N][E]
// row-major, qkv [L*N][3E] = x @ in_proj_weight^T + in_proj_bias (q | k | v
// columns), out [L*N][E] before out_proj.  head_dim == 64, L <= 256.  The
// bf16 attention core runs on MFMA (attn.hip); the f32 parity mode keeps the
// per-row kernels below (one lane per head dimension, four keys per lane).
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

__device__ __forceinline__ float vit_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 8 consecutive elements <-> f32 (16-B accesses for bf16, 2 x 16 B for f32)
__device__ __forceinline__ void vt_load8(const bf16* p, float (&v)[8]) {
  const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
}
__device__ __forceinline__ void vt_load8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void vt_store8(bf16* p, const float (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (bf16)v[i];
  *reinterpret_cast<bf16x8*>(p) = r;
}
__device__ __forceinline__ void vt_store8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// fp8 amax of a producer's output, fused: each block folds max |y| of what it
// wrote into pmax[blockIdx.x % ARTSBIR_PMAX] (zeroed by the caller; unsigned
// order of non-negative floats = float order), so the quantiser reduces 4096
// partials instead of re-reading the tensor (artsbir_quantize_fp8_pmax)
#define ARTSBIR_PMAX 4096
__device__ __forceinline__ void vt_block_amax(float m, unsigned* pmax) {
  __shared__ float red_amax[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) red_amax[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
    for (int i = 0; i < nw; ++i) b = fmaxf(b, red_amax[i]);
    atomicMax(pmax + (blockIdx.x & (ARTSBIR_PMAX - 1)), __float_as_uint(b));
  }
}

// LayerNorm forward with 8-column chunks per lane (C % 8 == 0; chunk lane + 64 u)
template <typename T, int NCH>
__global__ void __launch_bounds__(256) layernorm_v_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, long long rows, int C,
                                                          float eps, T* __restrict__ y, unsigned* __restrict__ pmax) {
  const int lane = threadIdx.x & 63;
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  if (row >= rows) {
    if (pmax) vt_block_amax(0.f, pmax);  // every wave reaches the block's barrier
    return;
  }
  const int nch = C >> 3;
  const T* xr = x + row * C;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int ch = lane + 64 * u;
    if (ch < nch) vt_load8(xr + ch * 8, v[u]);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[u][e];
  }
  const float mean = warp_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u)
    if (lane + 64 * u < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (v[u][e] - mean) * (v[u][e] - mean);
  const float istd = rsqrtf(warp_sum(q) / (float)C + eps);
  T* yr = y + row * C;
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int ch = lane + 64 * u;
    if (ch < nch) {
      float g[8], b[8], o[8];
      vt_load8(gamma + ch * 8, g);
      vt_load8(beta + ch * 8, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[u][e] - mean) * istd * g[e] + b[e];
      vt_store8(yr + ch * 8, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) am = fmaxf(am, fabsf((float)(T)o[e]));  // the stored (rounded) value
    }
  }
  if (pmax) vt_block_amax(am, pmax);
}

typedef __attribute__((ext_vector_type(4))) unsigned vt_u32x4;
// raw 8-element chunks of a row (bf16: one 16-B load, f32: two), converted to
// f32 only when used, so that the next row's loads can be in flight meanwhile
template <typename T>
struct VtRaw {
  uint4 v[sizeof(T) == 2 ? 1 : 2];
};
__device__ __forceinline__ void vt_raw_load(const bf16* p, VtRaw<bf16>& r) { r.v[0] = *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void vt_raw_load(const float* p, VtRaw<float>& r) {
  r.v[0] = reinterpret_cast<const uint4*>(p)[0];
  r.v[1] = reinterpret_cast<const uint4*>(p)[1];
}
__device__ __forceinline__ void vt_raw_cvt(const VtRaw<bf16>& r, float (&v)[8]) {
  const bf16x8 b = __builtin_bit_cast(bf16x8, r.v[0]);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)b[i];
}
__device__ __forceinline__ void vt_raw_cvt(const VtRaw<float>& r, float (&v)[8]) {
  v[0] = __uint_as_float(r.v[0].x); v[1] = __uint_as_float(r.v[0].y); v[2] = __uint_as_float(r.v[0].z);
  v[3] = __uint_as_float(r.v[0].w); v[4] = __uint_as_float(r.v[1].x); v[5] = __uint_as_float(r.v[1].y);
  v[6] = __uint_as_float(r.v[1].z); v[7] = __uint_as_float(r.v[1].w);
}
// x, dy (and dres) of one row, every lane's chunks loaded unconditionally
// (chunks past C repeat the last one and are masked at use): no branch around
// the loads, so the compiler counts them across the row loop
template <typename T, int NCH>
struct LnRow {
  VtRaw<T> x[NCH], g[NCH], r[NCH];
};
template <typename T, int NCH, bool RES>
__device__ __forceinline__ void ln_fetch(const T* __restrict__ x, const T* __restrict__ dy, const T* dres, long long row,
                                         int C, int lane, LnRow<T, NCH>& R) {
  const int nch = C >> 3;
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int ch = min(lane + 64 * u, nch - 1);
    vt_raw_load(x + row * C + ch * 8, R.x[u]);
    vt_raw_load(dy + row * C + ch * 8, R.g[u]);
    if (RES) vt_raw_load(dres + row * C + ch * 8, R.r[u]);
  }
}

// LayerNorm backward with 8-column chunks per lane; each block's 4 waves reduce
// their dgamma / dbeta partials in LDS and add them with one atomic per column
template <typename T, int NCH, bool SUMS, bool RES>
__device__ __forceinline__ void ln_bwd_row(const LnRow<T, NCH>& R, T* dx, long long row, int C, float eps, int lane,
                                           const float (&gm)[NCH][8], float (&pg)[NCH][8], float (&pb)[NCH][8],
                                           float (&pr)[NCH][8], float (&po)[NCH][8]) {
  const int nch = C >> 3;
  float xv[NCH][8], gv[NCH][8], res[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const bool ok = lane + 64 * u < nch;
    vt_raw_cvt(R.x[u], xv[u]);
    vt_raw_cvt(R.g[u], gv[u]);
    if (RES) vt_raw_cvt(R.r[u], res[u]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (!ok) { xv[u][e] = 0.f; gv[u][e] = 0.f; }
      if (!RES || !ok) res[u][e] = 0.f;
      s += xv[u][e];
    }
  }
  const float mean = warp_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u)
    if (lane + 64 * u < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (xv[u][e] - mean) * (xv[u][e] - mean);
  const float istd = rsqrtf(warp_sum(q) / (float)C + eps);
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int u = 0; u < NCH; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (xv[u][e] - mean) * istd;  // past C: gv = 0, so no contribution
      const float g = gv[u][e] * gm[u][e];
      a += g;
      b += g * xh;
      pg[u][e] += gv[u][e] * xh;
      pb[u][e] += gv[u][e];
      xv[u][e] = xh;
      gv[u][e] = g;
    }
  a = warp_sum(a) / (float)C;
  b = warp_sum(b) / (float)C;
  // the row's dx by buffer stores: a chunk past C goes past the descriptor's
  // end and is dropped (no branch around the stores either)
  const __amdgpu_buffer_rsrc_t orow =
      __builtin_amdgcn_make_buffer_rsrc(dx + row * C, (short)0, C * (int)sizeof(T), 0x00020000);
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int ch = lane + 64 * u;
    const unsigned off = ch < nch ? (unsigned)(ch * 8 * (int)sizeof(T)) : 0x80000000u;
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = istd * (gv[u][e] - a - xv[u][e] * b) + res[u][e];
    if constexpr (sizeof(T) == 2) {
      uint4 h;
      unsigned* hp = &h.x;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        hp[k] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)out[2 * k]) |
                ((unsigned)__builtin_bit_cast(unsigned short, (bf16)out[2 * k + 1]) << 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vt_u32x4, h), orow, off, 0, 0);
    } else {
      vt_u32x4 f0, f1;
#pragma unroll
      for (int k = 0; k < 4; ++k) { f0[k] = __float_as_uint(out[k]); f1[k] = __float_as_uint(out[4 + k]); }
      __builtin_amdgcn_raw_buffer_store_b128(f0, orow, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(f1, orow, off == 0x80000000u ? off : off + 16, 0, 0);
    }
    if constexpr (SUMS) {  // column sums of the residual gradient and of dx (bias gradients; chunks past C unused)
#pragma unroll
      for (int e = 0; e < 8; ++e) { pr[u][e] += res[u][e]; po[u][e] += out[e]; }
    }
  }
}

// LayerNorm backward with 8-column chunks per lane; each block's 4 waves reduce
// their dgamma / dbeta partials in LDS and add them with one atomic per column.
// SUMS: also the column sums of dres and of dx (the bias gradients of the
// projections around the LayerNorm, instead of two colsum passes)
template <typename T, int NCH, bool SUMS>
__global__ void __launch_bounds__(256) layernorm_bwd_v_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                              const T* __restrict__ dy, long long rows, int C, float eps,
                                                              const T* dres, T* dx, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, float* __restrict__ dres_sum,
                                                              float* __restrict__ dx_sum) {
  constexpr int NR = SUMS ? 4 : 2;
  __shared__ float red[NR][3][64 * NCH * 8];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = C >> 3;
  float pg[NCH][8], pb[NCH][8], gm[NCH][8], pr[NCH][8], po[NCH][8];
#pragma unroll
  for (int u = 0; u < NCH; ++u) {
    const int ch = lane + 64 * u;
#pragma unroll
    for (int e = 0; e < 8; ++e) { pg[u][e] = 0.f; pb[u][e] = 0.f; gm[u][e] = 0.f; pr[u][e] = 0.f; po[u][e] = 0.f; }
    if (ch < nch) vt_load8(gamma + ch * 8, gm[u]);
  }
  // rows in a stride of the grid, the next row's operands loaded before this
  // row's arithmetic and store (one wave per row, two waves per SIMD: without
  // the prefetch each row's loads wait out a full memory latency)
  const long long stride = gridDim.x * 4LL;
  long long row = blockIdx.x * 4LL + w;
  if (row < rows) {
    LnRow<T, NCH> cur, nxt;
    if (dres) ln_fetch<T, NCH, true>(x, dy, dres, row, C, lane, cur);
    else ln_fetch<T, NCH, false>(x, dy, dres, row, C, lane, cur);
    for (; row < rows; row += stride) {
      const long long rn = min(row + stride, rows - 1);  // the last row re-fetched: no branch around the loads
      if (dres) {
        ln_fetch<T, NCH, true>(x, dy, dres, rn, C, lane, nxt);
        ln_bwd_row<T, NCH, SUMS, true>(cur, dx, row, C, eps, lane, gm, pg, pb, pr, po);
      } else {
        ln_fetch<T, NCH, false>(x, dy, dres, rn, C, lane, nxt);
        ln_bwd_row<T, NCH, SUMS, false>(cur, dx, row, C, eps, lane, gm, pg, pb, pr, po);
      }
      cur = nxt;
    }
  }
  if (w > 0) {
#pragma unroll
    for (int u = 0; u < NCH; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int i = (u * 64 + lane) * 8 + e;
        red[0][w - 1][i] = pg[u][e];
        red[1][w - 1][i] = pb[u][e];
        if constexpr (SUMS) {
          red[NR - 2][w - 1][i] = pr[u][e];
          red[NR - 1][w - 1][i] = po[u][e];
        }
      }
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int ch = lane + 64 * u;
      if (ch < nch)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = (u * 64 + lane) * 8 + e;
          atomicAdd(dgamma + ch * 8 + e, pg[u][e] + red[0][0][i] + red[0][1][i] + red[0][2][i]);
          atomicAdd(dbeta + ch * 8 + e, pb[u][e] + red[1][0][i] + red[1][1][i] + red[1][2][i]);
          if constexpr (SUMS) {
            if (dres_sum)
              atomicAdd(dres_sum + ch * 8 + e, pr[u][e] + red[NR - 2][0][i] + red[NR - 2][1][i] + red[NR - 2][2][i]);
            if (dx_sum)
              atomicAdd(dx_sum + ch * 8 + e, po[u][e] + red[NR - 1][0][i] + red[NR - 1][1][i] + red[NR - 1][2][i]);
          }
        }
    }
  }
}

// LayerNorm backward for bf16 rows of C = 256 NC columns (ViT-B: 768): lane l
// owns the 4-column chunks l + 64 u, u < NC (8-B loads and stores, every lane
// busy; the 8-column form leaves half the lanes idle in its second chunk at
// C = 768 and holds 232-248 VGPRs, so one row in flight per wave: ~36 KB of
// loads in flight per CU, ~3 TB/s).  At ~150 VGPRs this one keeps PF = 2 rows
// in flight per wave at the same two waves per SIMD.  Same arithmetic as
// ln_bwd_row (row sums in another order); dgamma / dbeta (and with SUMS the
// column sums of dres and dx) reduced over the block's 4 waves in LDS, then
// one atomic per column per block
template <int NC>
struct Ln4Row {
  uint2 x[NC], g[NC], r[NC];
};
__device__ __forceinline__ void ln4_cvt(uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <int NC, bool RES>
__device__ __forceinline__ void ln4_fetch(const bf16* __restrict__ x, const bf16* __restrict__ dy, const bf16* dres,
                                          long long row, int lane, Ln4Row<NC>& R) {
  constexpr int C = 256 * NC;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const long long o = row * C + 4 * (lane + 64 * u);
    R.x[u] = *reinterpret_cast<const uint2*>(x + o);
    R.g[u] = *reinterpret_cast<const uint2*>(dy + o);
    if (RES) R.r[u] = *reinterpret_cast<const uint2*>(dres + o);
  }
}
template <int NC, bool SUMS, bool RES>
__device__ __forceinline__ void ln4_row(const Ln4Row<NC>& R, bf16* __restrict__ dx, long long row, float eps, int lane,
                                        const float (&gm)[NC][4], float (&pg)[NC][4], float (&pb)[NC][4],
                                        float (&pr)[NC][4], float (&po)[NC][4]) {
  constexpr int C = 256 * NC;
  float xv[NC][4], gv[NC][4], res[NC][4];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    ln4_cvt(R.x[u], xv[u]);
    ln4_cvt(R.g[u], gv[u]);
    if (RES) ln4_cvt(R.r[u], res[u]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!RES) res[u][e] = 0.f;
      s += xv[u][e];
    }
  }
  const float mean = warp_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < NC; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (xv[u][e] - mean) * (xv[u][e] - mean);
  const float istd = rsqrtf(warp_sum(q) / (float)C + eps);
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int u = 0; u < NC; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (xv[u][e] - mean) * istd;
      const float g = gv[u][e] * gm[u][e];
      a += g;
      b += g * xh;
      pg[u][e] += gv[u][e] * xh;
      pb[u][e] += gv[u][e];
      xv[u][e] = xh;
      gv[u][e] = g;
    }
  a = warp_sum(a) / (float)C;
  b = warp_sum(b) / (float)C;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    float out[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = istd * (gv[u][e] - a - xv[u][e] * b) + res[u][e];
    uint2 h;
    h.x = (unsigned)__builtin_bit_cast(unsigned short, (bf16)out[0]) |
          ((unsigned)__builtin_bit_cast(unsigned short, (bf16)out[1]) << 16);
    h.y = (unsigned)__builtin_bit_cast(unsigned short, (bf16)out[2]) |
          ((unsigned)__builtin_bit_cast(unsigned short, (bf16)out[3]) << 16);
    *reinterpret_cast<uint2*>(dx + row * C + 4 * (lane + 64 * u)) = h;
    if constexpr (SUMS) {
#pragma unroll
      for (int e = 0; e < 4; ++e) { pr[u][e] += res[u][e]; po[u][e] += out[e]; }
    }
  }
}
template <int NC, bool SUMS, int PF>
__global__ void __launch_bounds__(256) layernorm_bwd_c4_kernel(const bf16* __restrict__ x,
                                                               const float* __restrict__ gamma,
                                                               const bf16* __restrict__ dy, long long rows, float eps,
                                                               const bf16* dres, bf16* dx, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta, float* __restrict__ dres_sum,
                                                               float* __restrict__ dx_sum) {
  constexpr int NR = SUMS ? 4 : 2;
  constexpr int C = 256 * NC;
  __shared__ float red[NR][3][C];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float pg[NC][4], pb[NC][4], gm[NC][4], pr[NC][4], po[NC][4];
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const float4 g4 = *reinterpret_cast<const float4*>(gamma + 4 * (lane + 64 * u));
    gm[u][0] = g4.x; gm[u][1] = g4.y; gm[u][2] = g4.z; gm[u][3] = g4.w;
#pragma unroll
    for (int e = 0; e < 4; ++e) { pg[u][e] = 0.f; pb[u][e] = 0.f; pr[u][e] = 0.f; po[u][e] = 0.f; }
  }
  const long long stride = gridDim.x * 4LL;
  long long row = blockIdx.x * 4LL + w;
  if (row < rows) {
    // rows PF strides ahead in flight (past the end the last row is re-fetched:
    // no branch around the loads)
    Ln4Row<NC> cur, n1, n2;
    if (dres) {
      ln4_fetch<NC, true>(x, dy, dres, row, lane, cur);
      if (PF == 2) ln4_fetch<NC, true>(x, dy, dres, min(row + stride, rows - 1), lane, n1);
    } else {
      ln4_fetch<NC, false>(x, dy, dres, row, lane, cur);
      if (PF == 2) ln4_fetch<NC, false>(x, dy, dres, min(row + stride, rows - 1), lane, n1);
    }
    for (; row < rows; row += stride) {
      const long long rn = min(row + PF * stride, rows - 1);
      if (dres) {
        ln4_fetch<NC, true>(x, dy, dres, rn, lane, PF == 2 ? n2 : n1);
        ln4_row<NC, SUMS, true>(cur, dx, row, eps, lane, gm, pg, pb, pr, po);
      } else {
        ln4_fetch<NC, false>(x, dy, dres, rn, lane, PF == 2 ? n2 : n1);
        ln4_row<NC, SUMS, false>(cur, dx, row, eps, lane, gm, pg, pb, pr, po);
      }
      cur = n1;
      if (PF == 2) n1 = n2;
    }
  }
  if (w > 0) {
#pragma unroll
    for (int u = 0; u < NC; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * (lane + 64 * u) + e;
        red[0][w - 1][i] = pg[u][e];
        red[1][w - 1][i] = pb[u][e];
        if constexpr (SUMS) {
          red[NR - 2][w - 1][i] = pr[u][e];
          red[NR - 1][w - 1][i] = po[u][e];
        }
      }
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int u = 0; u < NC; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * (lane + 64 * u) + e;
        atomicAdd(dgamma + i, pg[u][e] + red[0][0][i] + red[0][1][i] + red[0][2][i]);
        atomicAdd(dbeta + i, pb[u][e] + red[1][0][i] + red[1][1][i] + red[1][2][i]);
        if constexpr (SUMS) {
          if (dres_sum) atomicAdd(dres_sum + i, pr[u][e] + red[NR - 2][0][i] + red[NR - 2][1][i] + red[NR - 2][2][i]);
          if (dx_sum) atomicAdd(dx_sum + i, po[u][e] + red[NR - 1][0][i] + red[NR - 1][1][i] + red[NR - 1][2][i]);
        }
      }
  }
}

// y = (x - mean) / sqrt(var + eps) * gamma + beta per row, in fp32 whatever
// the storage dtype (models.py:382-388); one wave per row
template <typename T>
__global__ void __launch_bounds__(256) layernorm_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, long long rows, int C,
                                                        float eps, T* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += to_f(xr[c]);
  const float mean = warp_sum(s) / (float)C;
  float v = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = to_f(xr[c]) - mean;
    v += d * d;
  }
  const float istd = rsqrtf(warp_sum(v) / (float)C + eps);
  T* yr = y + row * C;
  for (int c = lane; c < C; c += 64) yr[c] = from_f<T>((to_f(xr[c]) - mean) * istd * gamma[c] + beta[c]);
}

// QuickGELU (models.py:391-393): x * sigmoid(1.702 x)
template <typename T>
__global__ void quickgelu_kernel(const T* __restrict__ x, long long n, T* __restrict__ y,
                                 unsigned* __restrict__ pmax) {
  const long long n8 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) ? 0 : n / 8;
  float am = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    vt_load8(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = v[e] / (1.f + __expf(-1.702f * v[e]));
      am = fmaxf(am, fabsf((float)(T)v[e]));
    }
    vt_store8(y + i * 8, v);
  }
  for (long long i = n8 * 8 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float v = to_f(x[i]);
    const T o = from_f<T>(v / (1.f + __expf(-1.702f * v)));
    y[i] = o;
    am = fmaxf(am, fabsf(to_f(o)));
  }
  if (pmax) vt_block_amax(am, pmax);
}

// softmax(q k^T / sqrt(64) + mask) v for one (query position, batch, head)
// per wave: lane l scores keys l, l+64, l+128, l+192; the probabilities go
// through LDS; lane d accumulates output dimension d over the keys
template <typename T>
__global__ void __launch_bounds__(256) mha_fwd_kernel(const T* __restrict__ qkv, int L, int N, int heads,
                                                      const float* __restrict__ mask, T* __restrict__ out,
                                                      float* __restrict__ lse) {
  __shared__ float ps[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long item = blockIdx.x * 4LL + w;  // (i, n, h) with h fastest
  if (item >= (long long)L * N * heads) return;
  const int h = (int)(item % heads);
  const long long in = item / heads;
  const int n = (int)(in % N), i = (int)(in / N);
  const int E = heads * 64;
  const long long ld = 3LL * E;
  const T* qr = qkv + ((long long)i * N + n) * ld + h * 64;
  float q[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) q[d] = to_f(qr[d]) * 0.125f;  // 1/sqrt(head_dim), applied to q as torch does
  float s[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = lane + 64 * u;
    float acc = -INFINITY;
    if (j < L) {
      const T* kr = qkv + ((long long)j * N + n) * ld + E + h * 64;
      acc = 0.f;
#pragma unroll 8
      for (int d = 0; d < 64; ++d) acc += q[d] * to_f(kr[d]);
      if (mask) acc += mask[(long long)i * L + j];
    }
    s[u] = acc;
  }
  const float m = vit_wave_max(fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3])));
  float sum = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float p = (lane + 64 * u < L && s[u] != -INFINITY) ? __expf(s[u] - m) : 0.f;
    s[u] = p;
    sum += p;
  }
  const float tot = warp_sum(sum);
  const float inv = 1.f / tot;
  if (lse && lane == 0) lse[item] = m + __logf(tot);  // log-sum-exp of the row (backward)
#pragma unroll
  for (int u = 0; u < 4; ++u) ps[w][lane + 64 * u] = s[u] * inv;
  // the wave reads its own row of ps (LDS operations of a wave complete in order)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  float o = 0.f;
  const T* vc = qkv + (long long)n * ld + 2 * E + h * 64 + lane;
  for (int j = 0; j < L; ++j) o += ps[w][j] * to_f(vc[(long long)j * N * ld]);
  out[((long long)i * N + n) * E + h * 64 + lane] = from_f<T>(o);
}

// ------------------------------------------------------------- backward
// LayerNorm backward, one wave per row (rows strided over the grid so every
// lane keeps its columns' dgamma / dbeta partial sums in registers and adds
// them once): xhat = (x - mean) istd, g = dy gamma,
// dx = istd (g - mean(g) - xhat mean(g xhat)); dgamma += dy xhat, dbeta += dy.
template <typename T, int CPL>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(const T* __restrict__ x, const float* __restrict__ gamma,
                                                            const T* __restrict__ dy, long long rows, int C, float eps,
                                                            const T* dres, T* dx,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int lane = threadIdx.x & 63;
  float pg[CPL], pb[CPL];
#pragma unroll
  for (int u = 0; u < CPL; ++u) { pg[u] = 0.f; pb[u] = 0.f; }
  for (long long row = blockIdx.x * 4LL + (threadIdx.x >> 6); row < rows; row += gridDim.x * 4LL) {
    const T* xr = x + row * C;
    const T* gr = dy + row * C;
    float xv[CPL], gv[CPL];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      const int c = lane + 64 * u;
      xv[u] = c < C ? to_f(xr[c]) : 0.f;
      gv[u] = c < C ? to_f(gr[c]) : 0.f;
      s += xv[u];
    }
    const float mean = warp_sum(s) / (float)C;
    float v = 0.f;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      const float d = lane + 64 * u < C ? xv[u] - mean : 0.f;
      v += d * d;
    }
    const float istd = rsqrtf(warp_sum(v) / (float)C + eps);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      const int c = lane + 64 * u;
      if (c < C) {
        const float xh = (xv[u] - mean) * istd;
        const float g = gv[u] * gamma[c];
        a += g;
        b += g * xh;
        pg[u] += gv[u] * xh;
        pb[u] += gv[u];
        xv[u] = xh;
        gv[u] = g;
      }
    }
    a = warp_sum(a) / (float)C;
    b = warp_sum(b) / (float)C;
    T* o = dx + row * C;
    const T* rr = dres ? dres + row * C : nullptr;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      const int c = lane + 64 * u;
      if (c < C) o[c] = from_f<T>(istd * (gv[u] - a - xv[u] * b) + (rr ? to_f(rr[c]) : 0.f));
    }
  }
#pragma unroll
  for (int u = 0; u < CPL; ++u) {
    const int c = lane + 64 * u;
    if (c < C) {
      atomicAdd(dgamma + c, pg[u]);
      atomicAdd(dbeta + c, pb[u]);
    }
  }
}

// QuickGELU backward: d/dx [x s(1.702 x)] = s + 1.702 x s (1 - s)
template <typename T>
__global__ void quickgelu_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy, long long n,
                                     T* __restrict__ dx) {
  const long long n8 =
      ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dx)) & 15)
          ? 0
          : n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float v[8], g[8];
    vt_load8(x + i * 8, v);
    vt_load8(dy + i * 8, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = 1.f / (1.f + __expf(-1.702f * v[e]));
      v[e] = g[e] * (sg + 1.702f * v[e] * sg * (1.f - sg));
    }
    vt_store8(dx + i * 8, v);
  }
  for (long long i = n8 * 8 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float v = to_f(x[i]);
    const float sg = 1.f / (1.f + __expf(-1.702f * v));
    dx[i] = from_f<T>(to_f(dy[i]) * (sg + 1.702f * v * sg * (1.f - sg)));
  }
}

// QuickGELU backward over rows of C columns with the column sums of dx (the
// bias gradient of the projection that produced x): a thread owns 8 columns
// and walks rows; one atomic per column per block at the end
template <typename T>
__global__ void __launch_bounds__(128) quickgelu_bwd_sum_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                                long long rows, int C, T* __restrict__ dx,
                                                                float* __restrict__ dsum) {
  const int c8 = blockIdx.x * 128 + threadIdx.x;
  if (c8 * 8 >= C) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int U = 4;  // rows in flight per thread
  const long long step = gridDim.y;
  long long r = blockIdx.y;
  for (; r + (U - 1) * step < rows; r += U * step) {
    float v[U][8], g[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = (r + u * step) * C + c8 * 8;
      vt_load8(x + o, v[u]);
      vt_load8(dy + o, g[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sg = 1.f / (1.f + __expf(-1.702f * v[u][e]));
        v[u][e] = g[u][e] * (sg + 1.702f * v[u][e] * sg * (1.f - sg));
        acc[e] += v[u][e];
      }
      vt_store8(dx + (r + u * step) * C + c8 * 8, v[u]);
    }
  }
  for (; r < rows; r += step) {
    const long long o = r * C + c8 * 8;
    float v[8], g[8];
    vt_load8(x + o, v);
    vt_load8(dy + o, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = 1.f / (1.f + __expf(-1.702f * v[e]));
      v[e] = g[e] * (sg + 1.702f * v[e] * sg * (1.f - sg));
      acc[e] += v[e];
    }
    vt_store8(dx + o, v);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) atomicAdd(dsum + c8 * 8 + e, acc[e]);
}

// attention backward, query side, one wave per (query i, batch n, head h):
// D_i = dO_i . O_i; per key j (lane j, j + 64, ...): p = exp(q.k_j / 8 + mask -
// lse_i), dp = dO_i . v_j, ds = p (dp - D_i) -> LDS; lane d: dq_i[d] =
// sum_j ds_j k_j[d] / 8.  D goes out for the key-side kernel.
template <typename T>
__global__ void __launch_bounds__(256) mha_bwd_q_kernel(const T* __restrict__ qkv, const T* __restrict__ o,
                                                        const T* __restrict__ dout, const float* __restrict__ lse,
                                                        int L, int N, int heads, const float* __restrict__ mask,
                                                        T* __restrict__ dqkv, float* __restrict__ Dout) {
  __shared__ float dss[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long item = blockIdx.x * 4LL + w;
  if (item >= (long long)L * N * heads) return;
  const int h = (int)(item % heads);
  const long long in = item / heads;
  const int n = (int)(in % N), i = (int)(in / N);
  const int E = heads * 64;
  const long long ld = 3LL * E;
  const long long orow = ((long long)i * N + n) * E + h * 64;
  const float Di = warp_sum(to_f(dout[orow + lane]) * to_f(o[orow + lane]));
  if (lane == 0) Dout[item] = Di;
  const T* qr = qkv + ((long long)i * N + n) * ld + h * 64;
  float q[64], g[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) { q[d] = to_f(qr[d]) * 0.125f; g[d] = to_f(dout[orow + d]); }
  const float li = lse[item];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = lane + 64 * u;
    float ds = 0.f;
    if (j < L) {
      const T* kr = qkv + ((long long)j * N + n) * ld + E + h * 64;
      const T* vr = kr + E;
      float sc = 0.f, dp = 0.f;
#pragma unroll 8
      for (int d = 0; d < 64; ++d) { sc += q[d] * to_f(kr[d]); dp += g[d] * to_f(vr[d]); }
      if (mask) sc += mask[(long long)i * L + j];
      const float p = sc == -INFINITY ? 0.f : __expf(sc - li);
      ds = p * (dp - Di);
    }
    dss[w][j] = ds;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  float acc = 0.f;
  const T* kc = qkv + (long long)n * ld + E + h * 64 + lane;
  for (int j = 0; j < L; ++j) acc += dss[w][j] * to_f(kc[(long long)j * N * ld]);
  dqkv[((long long)i * N + n) * ld + h * 64 + lane] = from_f<T>(acc * 0.125f);
}

// attention backward, key side, one wave per (key j, batch n, head h): per
// query i (lane i, i + 64, ...): p = exp(q_i.k_j / 8 + mask - lse_i), dp =
// dO_i . v_j, ds = p (dp - D_i) -> LDS; lane d: dv_j[d] = sum_i p dO_i[d],
// dk_j[d] = sum_i ds q_i[d] / 8
template <typename T>
__global__ void __launch_bounds__(256) mha_bwd_kv_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                         const float* __restrict__ lse, const float* __restrict__ Din,
                                                         int L, int N, int heads, const float* __restrict__ mask,
                                                         T* __restrict__ dqkv) {
  __shared__ float pss[4][256], dss[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long item = blockIdx.x * 4LL + w;  // (j, n, h)
  if (item >= (long long)L * N * heads) return;
  const int h = (int)(item % heads);
  const long long jn = item / heads;
  const int n = (int)(jn % N), j = (int)(jn / N);
  const int E = heads * 64;
  const long long ld = 3LL * E;
  const T* kr = qkv + ((long long)j * N + n) * ld + E + h * 64;
  float k[64], v[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) { k[d] = to_f(kr[d]); v[d] = to_f(kr[E + d]); }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = lane + 64 * u;
    float p = 0.f, ds = 0.f;
    if (i < L) {
      const long long it = ((long long)i * N + n) * heads + h;
      const T* qr = qkv + ((long long)i * N + n) * ld + h * 64;
      const T* gr = dout + ((long long)i * N + n) * E + h * 64;
      float sc = 0.f, dp = 0.f;
#pragma unroll 8
      for (int d = 0; d < 64; ++d) { sc += (to_f(qr[d]) * 0.125f) * k[d]; dp += to_f(gr[d]) * v[d]; }
      if (mask) sc += mask[(long long)i * L + j];
      p = sc == -INFINITY ? 0.f : __expf(sc - lse[it]);
      ds = p * (dp - Din[it]);
    }
    pss[w][i] = p;
    dss[w][i] = ds;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  float dk = 0.f, dv = 0.f;
  const T* qc = qkv + (long long)n * ld + h * 64 + lane;
  const T* gc = dout + (long long)n * E + h * 64 + lane;
  for (int i = 0; i < L; ++i) {
    dk += dss[w][i] * to_f(qc[(long long)i * N * ld]);
    dv += pss[w][i] * to_f(gc[(long long)i * N * E]);
  }
  T* o = dqkv + ((long long)j * N + n) * ld + h * 64 + lane;
  o[E] = from_f<T>(dk * 0.125f);
  o[2 * E] = from_f<T>(dv);
}

// ViT patch embedding operand: image [B][3][R][R] f32 -> rows [B*P][3*16*16]
// (row b*P + p, column c*256 + kh*16 + kw: the flattened conv1 weight order)
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ img, int B, int R, int ps, T* __restrict__ out) {
  const int G = R / ps, P = G * G, K = 3 * ps * ps;
  const long long n = (long long)B * P * K;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n; t += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(t % K);
    const long long r = t / K;
    const int p = (int)(r % P), b = (int)(r / P);
    const int c = k / (ps * ps), kh = (k / ps) % ps, kw = k % ps;
    const int y = (p / G) * ps + kh, x = (p % G) * ps + kw;
    out[t] = from_f<T>(img[(((long long)b * 3 + c) * R + y) * R + x]);
  }
}

// tokens [L = P + 1][B][E]: token 0 = class embedding, token 1 + p = patch p,
// plus the positional embedding (CLIP VisionTransformer.forward)
template <typename T>
__global__ void vit_tokens_kernel(const T* __restrict__ patches, const float* __restrict__ cls,
                                  const float* __restrict__ pos, int B, int P, int E, T* __restrict__ out) {
  const long long n = (long long)(P + 1) * B * E;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n; t += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(t % E);
    const long long r = t / E;
    const int b = (int)(r % B), l = (int)(r / B);
    const float v = l == 0 ? cls[e] : to_f(patches[((long long)b * P + (l - 1)) * E + e]);
    out[t] = from_f<T>(v + pos[(long long)l * E + e]);
  }
}

// its backward: dpatches[b*P+p] = dtok[1+p][b]; dcls = sum_b dtok[0][b];
// dpos[l] = sum_b dtok[l][b] (one thread per (l, e), loop over b: fixed order)
template <typename T>
__global__ void vit_tokens_bwd_kernel(const T* __restrict__ dtok, int B, int P, int E, T* __restrict__ dpatches,
                                      float* __restrict__ dcls, float* __restrict__ dpos) {
  const long long n = (long long)(P + 1) * E;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n; t += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(t % E), l = (int)(t / E);
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      const float g = to_f(dtok[((long long)l * B + b) * E + e]);
      s += g;
      if (l > 0) dpatches[((long long)b * P + (l - 1)) * E + e] = from_f<T>(g);
    }
    dpos[t] += s;
    if (l == 0) dcls[e] += s;
  }
}

#define VIT_DISPATCH(dtype, ...)                    \
  do {                                              \
    if ((dtype) == ARTSBIR_DT_BF16) {               \
      typedef bf16 T;                               \
      __VA_ARGS__;                                  \
    } else if ((dtype) == ARTSBIR_DT_F32) {         \
      typedef float T;                              \
      __VA_ARGS__;                                  \
    } else {                                        \
      set_error("unknown dtype %d", (int)(dtype));  \
      return -1;                                    \
    }                                               \
  } while (0)

// MFMA attention for the bf16 mode (attn.hip)
bool attn_fwd_mfma(const bf16* qkv, int L, int N, int heads, const float* mask, bf16* out, float* lse,
                   unsigned* pmax, hipStream_t st);
bool attn_bwd_mfma(const bf16* qkv, const bf16* o, const bf16* dout, const float* lse, int L, int N, int heads,
                   const float* mask, bf16* dqkv, float* dscratch, hipStream_t st);

static inline unsigned vit_grid(long long n) {
  long long g = (n + 255) / 256;
  return (unsigned)(g > (1 << 20) ? (1 << 20) : g < 1 ? 1 : g);
}

}  // namespace artsbir

using namespace artsbir;

static int layernorm_fwd_impl(int dtype, const void* x, const float* gamma, const float* beta, long long rows, int C,
                              float eps, void* y, unsigned* pmax, void* stream) {
  if (rows <= 0) return 0;
  const unsigned grid = (unsigned)((rows + 3) / 4);
  const bool vec = C % 8 == 0 && C <= 1024 && !((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                                                  reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta)) & 15);
  if (vec && C <= 512)
    VIT_DISPATCH(dtype, hipLaunchKernelGGL((layernorm_v_kernel<T, 1>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, gamma, beta, rows, C, eps, (T*)y, pmax));
  else if (vec)
    VIT_DISPATCH(dtype, hipLaunchKernelGGL((layernorm_v_kernel<T, 2>), dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, gamma, beta, rows, C, eps, (T*)y, pmax));
  else if (pmax) {
    set_error("layernorm_fwd: the fused amax needs C %% 8 == 0 (<= 1024) and 16-B aligned rows");
    return -1;
  } else
    VIT_DISPATCH(dtype, hipLaunchKernelGGL(layernorm_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, gamma, beta, rows, C, eps, (T*)y));
  ARTSBIR_CHECK_LAUNCH("layernorm_fwd");
  return 0;
}

extern "C" int artsbir_layernorm_fwd(int dtype, const void* x, const float* gamma, const float* beta, long long rows,
                                     int C, float eps, void* y, void* stream) {
  return layernorm_fwd_impl(dtype, x, gamma, beta, rows, C, eps, y, nullptr, stream);
}

extern "C" int artsbir_layernorm_fwd_pmax(int dtype, const void* x, const float* gamma, const float* beta,
                                          long long rows, int C, float eps, void* y, unsigned* pmax, void* stream) {
  if (!pmax) { set_error("layernorm_fwd_pmax: pmax missing"); return -1; }
  return layernorm_fwd_impl(dtype, x, gamma, beta, rows, C, eps, y, pmax, stream);
}

extern "C" int artsbir_quickgelu_pmax(int dtype, const void* x, long long n, void* y, unsigned* pmax, void* stream) {
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(quickgelu_kernel<T>, dim3(vit_grid((n + 7) / 8)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)x, n, (T*)y, pmax));
  ARTSBIR_CHECK_LAUNCH("quickgelu");
  return 0;
}

extern "C" int artsbir_quickgelu(int dtype, const void* x, long long n, void* y, void* stream) {
  return artsbir_quickgelu_pmax(dtype, x, n, y, nullptr, stream);
}

extern "C" int artsbir_mha_fwd_lse(int dtype, const void* qkv, int L, int N, int heads, const float* mask,
                                   void* out, float* lse, void* stream);

extern "C" int artsbir_mha_fwd(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out,
                               void* stream) {
  return artsbir_mha_fwd_lse(dtype, qkv, L, N, heads, mask, out, nullptr, stream);
}

static int mha_fwd_impl(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out, float* lse,
                        unsigned* pmax, void* stream);

extern "C" int artsbir_mha_fwd_lse(int dtype, const void* qkv, int L, int N, int heads, const float* mask,
                                   void* out, float* lse, void* stream) {
  return mha_fwd_impl(dtype, qkv, L, N, heads, mask, out, lse, nullptr, stream);
}

extern "C" int artsbir_mha_fwd_lse_pmax(int dtype, const void* qkv, int L, int N, int heads, const float* mask,
                                        void* out, float* lse, unsigned* pmax, void* stream) {
  if (dtype != ARTSBIR_DT_BF16 || !pmax) { set_error("mha_fwd_lse_pmax: bf16 and a pmax buffer"); return -1; }
  return mha_fwd_impl(dtype, qkv, L, N, heads, mask, out, lse, pmax, stream);
}

static int mha_fwd_impl(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out, float* lse,
                        unsigned* pmax, void* stream) {
  if (L < 1 || L > 256) { set_error("mha_fwd: sequence length %d outside [1, 256]", L); return -1; }
  if (heads < 1 || N < 1) { set_error("mha_fwd: bad batch %d / heads %d", N, heads); return -1; }
  if (dtype == ARTSBIR_DT_BF16) {  // MFMA path (attn.hip)
    if (!attn_fwd_mfma((const bf16*)qkv, L, N, heads, mask, (bf16*)out, lse, pmax, (hipStream_t)stream)) {
      set_error("mha_fwd: batch %d x heads %d too large", N, heads);
      return -1;
    }
    ARTSBIR_CHECK_LAUNCH("mha_fwd");
    return 0;
  }
  const long long items = (long long)L * N * heads;
  const unsigned grid = (unsigned)((items + 3) / 4);
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(mha_fwd_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)qkv, L, N, heads, mask, (T*)out, lse));
  ARTSBIR_CHECK_LAUNCH("mha_fwd");
  return 0;
}

static int layernorm_bwd_impl(int dtype, const void* x, const float* gamma, const void* dy, long long rows, int C,
                              float eps, const void* dres, void* dx, float* dgamma, float* dbeta, float* dres_sum,
                              float* dx_sum, void* stream) {
  if (rows <= 0) return 0;
  if (C < 1 || C > 1024) { set_error("layernorm_bwd: C=%d outside [1, 1024]", C); return -1; }
  const bool sums = dres_sum || dx_sum;
  if (dres_sum && !dres) { set_error("layernorm_bwd: dres_sum without dres"); return -1; }
  const bool vec = C % 8 == 0 && !((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
                                    reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(dres) |
                                    reinterpret_cast<uintptr_t>(gamma)) & 15);
  if (!vec && sums) { set_error("layernorm_bwd: column sums need C %% 8 == 0 and 16-B aligned rows"); return -1; }
  if (vec) {  // 8-column chunks per lane; 512 blocks: few atomics per column
    long long gv = (rows + 3) / 4;
    const unsigned gridv = (unsigned)(gv > 512 ? 512 : gv);
    // bf16 rows of 256 / 512 / 768 / 1024 columns: the 4-column form with two
    // rows in flight per wave (ARTSBIR_LN_C4=0: the 8-column form, timing comparison)
    static const bool c4 = [] { const char* e = getenv("ARTSBIR_LN_C4"); return !e || atoi(e) != 0; }();
    if (c4 && dtype == ARTSBIR_DT_BF16 && C % 256 == 0 && C <= 1024) {
      hipStream_t st = (hipStream_t)stream;
#define LNB4(N, S) hipLaunchKernelGGL((layernorm_bwd_c4_kernel<N, S, 2>), dim3(gridv), dim3(256), 0, st, (const bf16*)x, \
                                      gamma, (const bf16*)dy, rows, eps, (const bf16*)dres, (bf16*)dx, dgamma, dbeta,     \
                                      dres_sum, dx_sum)
#define LNB4S(N) do { if (sums) LNB4(N, true); else LNB4(N, false); } while (0)
      switch (C / 256) {
        case 1: LNB4S(1); break;
        case 2: LNB4S(2); break;
        case 3: LNB4S(3); break;
        default: LNB4S(4); break;
      }
#undef LNB4S
#undef LNB4
      ARTSBIR_CHECK_LAUNCH("layernorm_bwd");
      return 0;
    }
#define LNBV(N, S) VIT_DISPATCH(dtype, hipLaunchKernelGGL((layernorm_bwd_v_kernel<T, N, S>), dim3(gridv), dim3(256), 0, \
                                                         (hipStream_t)stream, (const T*)x, gamma, (const T*)dy, rows,  \
                                                         C, eps, (const T*)dres, (T*)dx, dgamma, dbeta, dres_sum,      \
                                                         dx_sum))
    if (C <= 512) {
      if (sums) LNBV(1, true);
      else LNBV(1, false);
    } else {
      if (sums) LNBV(2, true);
      else LNBV(2, false);
    }
#undef LNBV
    ARTSBIR_CHECK_LAUNCH("layernorm_bwd");
    return 0;
  }
  long long g = (rows + 3) / 4;
  const unsigned grid = (unsigned)(g > 2048 ? 2048 : g);
  const int cpl = (C + 63) / 64;
#define LNB(N) VIT_DISPATCH(dtype, hipLaunchKernelGGL((layernorm_bwd_kernel<T, N>), dim3(grid), dim3(256), 0,        \
                                                     (hipStream_t)stream, (const T*)x, gamma, (const T*)dy, rows, C, \
                                                     eps, (const T*)dres, (T*)dx, dgamma, dbeta))
  if (cpl <= 2) LNB(2);
  else if (cpl <= 4) LNB(4);
  else if (cpl <= 8) LNB(8);
  else if (cpl <= 12) LNB(12);
  else LNB(16);
#undef LNB
  ARTSBIR_CHECK_LAUNCH("layernorm_bwd");
  return 0;
}

extern "C" int artsbir_layernorm_bwd(int dtype, const void* x, const float* gamma, const void* dy, long long rows,
                                     int C, float eps, const void* dres, void* dx, float* dgamma, float* dbeta,
                                     void* stream) {
  return layernorm_bwd_impl(dtype, x, gamma, dy, rows, C, eps, dres, dx, dgamma, dbeta, nullptr, nullptr, stream);
}

extern "C" int artsbir_layernorm_bwd_sums(int dtype, const void* x, const float* gamma, const void* dy,
                                          long long rows, int C, float eps, const void* dres, void* dx, float* dgamma,
                                          float* dbeta, float* dres_sum, float* dx_sum, void* stream) {
  return layernorm_bwd_impl(dtype, x, gamma, dy, rows, C, eps, dres, dx, dgamma, dbeta, dres_sum, dx_sum, stream);
}

extern "C" int artsbir_quickgelu_bwd(int dtype, const void* x, const void* dy, long long n, void* dx, void* stream) {
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(quickgelu_bwd_kernel<T>, dim3(vit_grid((n + 7) / 8)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)x, (const T*)dy, n, (T*)dx));
  ARTSBIR_CHECK_LAUNCH("quickgelu_bwd");
  return 0;
}

extern "C" int artsbir_quickgelu_bwd_sum(int dtype, const void* x, const void* dy, long long rows, int C, void* dx,
                                         float* dsum, void* stream) {
  if (rows <= 0) return 0;
  if (C % 8 || !dsum || ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
                           reinterpret_cast<uintptr_t>(dx)) & 15)) {
    set_error("quickgelu_bwd_sum: C %% 8 == 0, 16-B aligned rows and a sum buffer required");
    return -1;
  }
  const unsigned gx = (unsigned)((C / 8 + 127) / 128);
  long long gy = 1024 / gx;
  if (gy > rows) gy = rows;
  if (gy < 1) gy = 1;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(quickgelu_bwd_sum_kernel<T>, dim3(gx, (unsigned)gy), dim3(128), 0,
                                       (hipStream_t)stream, (const T*)x, (const T*)dy, rows, C, (T*)dx, dsum));
  ARTSBIR_CHECK_LAUNCH("quickgelu_bwd_sum");
  return 0;
}

extern "C" int artsbir_mha_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse,
                               int L, int N, int heads, const float* mask, void* dqkv, float* dscratch,
                               void* stream) {
  if (L < 1 || L > 256) { set_error("mha_bwd: sequence length %d outside [1, 256]", L); return -1; }
  if (heads < 1 || N < 1 || !lse || !dscratch) { set_error("mha_bwd: bad arguments"); return -1; }
  if (dtype == ARTSBIR_DT_BF16) {  // MFMA path (attn.hip)
    if (!attn_bwd_mfma((const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse, L, N, heads, mask, (bf16*)dqkv,
                       dscratch, (hipStream_t)stream)) {
      set_error("mha_bwd: batch %d x heads %d too large", N, heads);
      return -1;
    }
    ARTSBIR_CHECK_LAUNCH("mha_bwd");
    return 0;
  }
  const long long items = (long long)L * N * heads;
  const unsigned grid = (unsigned)((items + 3) / 4);
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(mha_bwd_q_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)qkv, (const T*)out, (const T*)dout, lse, L, N, heads, mask,
                                       (T*)dqkv, dscratch));
  ARTSBIR_CHECK_LAUNCH("mha_bwd_q");
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(mha_bwd_kv_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)qkv, (const T*)dout, lse, dscratch, L, N, heads, mask, (T*)dqkv));
  ARTSBIR_CHECK_LAUNCH("mha_bwd_kv");
  return 0;
}

extern "C" int artsbir_vit_patchify(int dtype, const float* img, int B, int R, int patch, void* out, void* stream) {
  if (patch < 1 || R % patch) { set_error("vit_patchify: resolution %d not a multiple of patch %d", R, patch); return -1; }
  const long long n = (long long)B * (R / patch) * (R / patch) * 3 * patch * patch;
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(patchify_kernel<T>, dim3(vit_grid(n)), dim3(256), 0, (hipStream_t)stream,
                                       img, B, R, patch, (T*)out));
  ARTSBIR_CHECK_LAUNCH("vit_patchify");
  return 0;
}

extern "C" int artsbir_vit_tokens(int dtype, const void* patches, const float* cls, const float* pos, int B, int P,
                                  int E, void* out, void* stream) {
  const long long n = (long long)(P + 1) * B * E;
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(vit_tokens_kernel<T>, dim3(vit_grid(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)patches, cls, pos, B, P, E, (T*)out));
  ARTSBIR_CHECK_LAUNCH("vit_tokens");
  return 0;
}

extern "C" int artsbir_vit_tokens_bwd(int dtype, const void* dtok, int B, int P, int E, void* dpatches, float* dcls,
                                      float* dpos, void* stream) {
  const long long n = (long long)(P + 1) * E;
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(vit_tokens_bwd_kernel<T>, dim3(vit_grid(n)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)dtok, B, P, E, (T*)dpatches, dcls, dpos));
  ARTSBIR_CHECK_LAUNCH("vit_tokens_bwd");
  return 0;
}
