// MFMA attention core of the ViT blocks (bf16 compute mode): softmax(q k^T / 8
// + mask) v of nn.MultiheadAttention as ResidualAttentionBlock uses it
// (/root/reference/models.py:396-417), forward and backward, for head_dim 64
// and sequences up to 256 (ViT-B/16: 197 tokens).
//
// One workgroup per (batch n, head h); wave w owns the 32-row block w of the
// sequence (nb = ceil(L / 32) waves).  The whole (L x 64) slices the block
// needs sit in LDS as swizzled images of 128-B rows (16-B chunk c of row j at
// chunk c ^ at_sw(j): conflict-free for both the row reads of the MFMA A
// operand and the 4-row transposed reads ds_read_b64_tr_b16).
//
// Orientation (v_mfma_f32_32x32x16_bf16, C/D: column = lane & 31, rows in the
// 16 registers): every score tile is computed so that the product that
// follows sums over the tile's ROW index — then its registers, rounded to
// bf16, are that product's B operand as they are (k order permuted: element j
// of lane half hh is row 16s + 8(j >> 2) + 4hh + (j & 3) of k-step s), and the
// other operand is read transposed from LDS in the same permuted order.
//   forward (wave = 32 queries):   S^T = K Q^T, online softmax over the keys
//                                  (rows), O^T += V^T P^T
//   backward, query side:          S^T, dP^T = V dO^T, dS^T = P^T (dP^T - D),
//                                  dQ^T += K^T dS^T;  D_i = dO_i . O_i
//   backward, key side (32 keys):  S = Q K^T, dP = dO V^T, dS = P (dP - D),
//                                  dV^T += dO^T P, dK^T += Q^T dS
// P is recomputed from the forward's per-row log-sum-exp; nothing of size
// L x L leaves the registers.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace artsbir {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef short at_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* at_lds_t;
typedef __attribute__((address_space(3))) at_v4s* at_lds_v4s;

constexpr int AT_MAXB = 8;                  // 32-row blocks: L <= 256
constexpr int AT_IMG = AT_MAXB * 32 * 128;  // one [256][64] bf16 image

constexpr float AT_LOG2E = 1.4426950408889634f, AT_LN2 = 0.6931471805599453f;
constexpr float AT_SC2 = 0.125f * AT_LOG2E;  // the 1 / sqrt(64) score scale, log2 domain

__device__ __forceinline__ int at_sw(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int at_off(int row, int chunk) { return row * 128 + ((chunk ^ at_sw(row)) << 4); }

// rows [0, 32 nb) of two (L x 64) head slices (row strides lda / ldb elements)
// -> swizzled images; rows >= L are zero.  nthr = 64 nb threads, 4 chunks each.
__device__ __forceinline__ void at_stage2(const bf16* __restrict__ a, long long lda, const bf16* __restrict__ b,
                                          long long ldb, int L, char* ia, char* ib, int tid, int nthr) {
  uint4 va[4], vb[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + u * nthr, row = c >> 3, ch = c & 7;
    va[u] = make_uint4(0, 0, 0, 0);
    vb[u] = make_uint4(0, 0, 0, 0);
    if (row < L) {
      va[u] = *reinterpret_cast<const uint4*>(a + row * lda + ch * 8);
      vb[u] = *reinterpret_cast<const uint4*>(b + row * ldb + ch * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = tid + u * nthr, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(ia + at_off(row, ch)) = va[u];
    *reinterpret_cast<uint4*>(ib + at_off(row, ch)) = vb[u];
  }
}

// A operand (row read): row `row`, k-step s (d = 16 s .. 16 s + 15) of lane half hh
__device__ __forceinline__ bf16x8 at_row(const char* img, int row, int s, int hh) {
  return *reinterpret_cast<const bf16x8*>(img + at_off(row, 2 * s + hh));
}

__device__ __forceinline__ at_v4s at_tr(const char* img, int row, int col) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (at_lds_v4s)(at_lds_t)(img + row * 128 + (((col >> 3) ^ at_sw(row)) << 4) + ((col & 7) << 1)));
}

// A operand read transposed (X^T of an image X): A[row c0 + (lane & 31)][k]
// with element j of lane half hh = image row m0 + 8 (j >> 2) + 4 hh + (j & 3)
// — the permuted k order of an accumulator tile used as the B operand.
// ds_read_b64_tr_b16: lane t of a 16-lane group gives the address of row
// (t >> 2), columns 4 (t & 3) .. +3 of a 4 x 16 block and receives column t.
__device__ __forceinline__ bf16x8 at_trfrag(const char* img, int m0, int c0, int lane) {
  const int t = lane & 15, hh = lane >> 5, rb = lane & 16;
  const int row = m0 + 4 * hh + (t >> 2);
  const int col = c0 + rb + 4 * (t & 3);
  const at_v4s lo = at_tr(img, row, col);
  const at_v4s hi = at_tr(img, row + 8, col);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ f32x16 at_mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 at_zero() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ bf16x8 at_ld16(const bf16* p, bool ok) {
  if (!ok) {
    bf16x8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
    return z;
  }
  return *reinterpret_cast<const bf16x8*>(p);
}

// accumulator row of register rho for lane half hh
__device__ __forceinline__ int at_crow(int rho, int hh) { return (rho & 3) + 8 * (rho >> 2) + 4 * hh; }

// rows of C^T (d = 32 dt + at_crow) of column `col` (lane) -> dst[d] with
// 16-byte stores: lane half hh holds d = 32 dt + 8 g + 4 hh + (0..3), so each
// 8-element group is split over lanes l and l + 32; v_permlane32_swap hands
// lane l the upper halves of groups 0 and 2 and lane l + 32 the lower halves of
// groups 1 and 3, and every lane stores two whole groups (four dwordx4 stores
// per call instead of eight dwordx2: the epilogue store tail is issue-bound,
// MI355X_MICROARCH's attention-epilogue row)
__device__ __forceinline__ unsigned at_pack2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, (bf16)a) |
         ((unsigned)__builtin_bit_cast(unsigned short, (bf16)b) << 16);
}
__device__ __forceinline__ void at_store_t(bf16* dst, const f32x16& c0, const f32x16& c1, float scale, int hh) {
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const f32x16& c = dt ? c1 : c0;
    unsigned x[4][2];  // group g: elements 4 hh + (0, 1) | (2, 3) of d = 32 dt + 8 g
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      x[g][0] = at_pack2(c[4 * g] * scale, c[4 * g + 1] * scale);
      x[g][1] = at_pack2(c[4 * g + 2] * scale, c[4 * g + 3] * scale);
    }
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {  // groups (0, 1) then (2, 3)
      uint4 o;
      const auto s0 = __builtin_amdgcn_permlane32_swap(x[2 * gp][0], x[2 * gp + 1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(x[2 * gp][1], x[2 * gp + 1][1], false, false);
      // lane l: group 2 gp = (own lower half, lane l + 32's upper half); lane l + 32: group 2 gp + 1
      o.x = s0[0]; o.y = s1[0]; o.z = s0[1]; o.w = s1[1];
      *reinterpret_cast<uint4*>(dst + 32 * dt + 8 * (2 * gp + hh)) = o;
    }
  }
}

template <bool MASK>
__global__ void __launch_bounds__(512) attn_fwd_kernel(const bf16* __restrict__ qkv, int L, int N, int heads,
                                                       const float* __restrict__ mask, bf16* __restrict__ out,
                                                       float* __restrict__ lse, unsigned* __restrict__ pmax) {
  __shared__ __attribute__((aligned(16))) char smem[2 * AT_IMG];
  char* kimg = smem;
  char* vimg = smem + AT_IMG;
  const int nb = (L + 31) >> 5;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = (int)(blockIdx.x % heads), n = (int)(blockIdx.x / heads);
  const int E = heads * 64;
  const long long ld = 3LL * E, rs = (long long)N * ld;
  const bf16* base = qkv + (long long)n * ld + h * 64;
  at_stage2(base + E, rs, base + 2 * E, rs, L, kimg, vimg, tid, nb * 64);
  const int r = lane & 31, hh = lane >> 5;
  const int q = 32 * w + r;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = at_ld16(base + q * rs + 16 * s + 8 * hh, q < L);
  __syncthreads();

  // softmax in the log2 domain: v = s / 8 * log2(e) in one multiply, p = 2^(v - m)
  // on v_exp_f32 directly (mask values, natural-log units, scaled alike)
  f32x16 o0 = at_zero(), o1 = at_zero();
  float m = -INFINITY, l = 0.f;
  // one key block; CHK: the last block when L % 32 != 0 (keys >= L get -inf:
  // their K rows are zero, so without it they would enter the normaliser)
  auto kblock = [&](int kb, auto chk) {
    constexpr bool CHK = decltype(chk)::value;
    f32x16 st = at_zero();
#pragma unroll
    for (int s = 0; s < 4; ++s) st = at_mfma(at_row(kimg, 32 * kb + r, s, hh), qf[s], st);
    float mx = -INFINITY;
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) {
      const int key = 32 * kb + at_crow(rho, hh);
      float v = st[rho] * AT_SC2;
      if (MASK && key < L && q < L) v += mask[(long long)q * L + key] * AT_LOG2E;
      if ((CHK || MASK) && key >= L) v = -INFINITY;
      st[rho] = v;
      mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = __builtin_amdgcn_exp2f(m - mu);
    float sum = 0.f;
    bf16x8 pf0, pf1;
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) {
      const float p = __builtin_amdgcn_exp2f(st[rho] - mu);
      sum += p;
      if (rho < 8) pf0[rho] = (bf16)p;
      else pf1[rho - 8] = (bf16)p;
    }
    sum += __shfl_xor(sum, 32, 64);
    l = l * alpha + sum;
    m = mn;
    o0 *= alpha;
    o1 *= alpha;
    o0 = at_mfma(at_trfrag(vimg, 32 * kb, 0, lane), pf0, o0);
    o0 = at_mfma(at_trfrag(vimg, 32 * kb + 16, 0, lane), pf1, o0);
    o1 = at_mfma(at_trfrag(vimg, 32 * kb, 32, lane), pf0, o1);
    o1 = at_mfma(at_trfrag(vimg, 32 * kb + 16, 32, lane), pf1, o1);
  };
  const int nfull = (L & 31) ? nb - 1 : nb;
  for (int kb = 0; kb < nfull; ++kb) kblock(kb, std::false_type{});
  if (nfull < nb) kblock(nb - 1, std::true_type{});
  float am = 0.f;
  if (q < L) {
    at_store_t(out + ((long long)q * N + n) * E + h * 64, o0, o1, 1.f / l, hh);
    if (lse && hh == 0) lse[((long long)q * N + n) * heads + h] = (m + __log2f(l)) * AT_LN2;
    if (pmax) {
      const float il = 1.f / l;
#pragma unroll
      for (int i = 0; i < 16; ++i) am = fmaxf(am, fmaxf(fabsf((float)(bf16)(o0[i] * il)), fabsf((float)(bf16)(o1[i] * il))));
    }
  }
  if (pmax) {  // fused fp8 amax of the output (see vit.hip vt_block_amax)
    __shared__ float red_amax[8];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
    if (lane == 0) red_amax[w] = am;
    __syncthreads();
    if (threadIdx.x == 0) {
      float b = 0.f;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) b = fmaxf(b, red_amax[i]);
      atomicMax(pmax + (blockIdx.x & 4095), __float_as_uint(b));
    }
  }
}

template <bool MASK>
__global__ void __launch_bounds__(512) attn_bwd_q_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ o,
                                                         const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                         int L, int N, int heads, const float* __restrict__ mask,
                                                         bf16* __restrict__ dqkv, float* __restrict__ Dout) {
  __shared__ __attribute__((aligned(16))) char smem[2 * AT_IMG];
  char* kimg = smem;
  char* vimg = smem + AT_IMG;
  const int nb = (L + 31) >> 5;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = (int)(blockIdx.x % heads), n = (int)(blockIdx.x / heads);
  const int E = heads * 64;
  const long long ld = 3LL * E, rs = (long long)N * ld, ors = (long long)N * E;
  const bf16* base = qkv + (long long)n * ld + h * 64;
  at_stage2(base + E, rs, base + 2 * E, rs, L, kimg, vimg, tid, nb * 64);
  const int r = lane & 31, hh = lane >> 5;
  const int q = 32 * w + r;
  const bool qok = q < L;
  const long long orow = (long long)q * ors + (long long)n * E + h * 64;
  bf16x8 qf[4], gf[4];
  float D = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = at_ld16(base + q * rs + 16 * s + 8 * hh, qok);
    gf[s] = at_ld16(dout + orow + 16 * s + 8 * hh, qok);
    const bf16x8 of = at_ld16(o + orow + 16 * s + 8 * hh, qok);
#pragma unroll
    for (int j = 0; j < 8; ++j) D += (float)gf[s][j] * (float)of[j];
  }
  D += __shfl_xor(D, 32, 64);
  const long long item = ((long long)q * N + n) * heads + h;
  const float lq = qok ? lse[item] : 0.f;
  __syncthreads();

  f32x16 dq0 = at_zero(), dq1 = at_zero();
  for (int kb = 0; kb < nb; ++kb) {
    f32x16 st = at_zero(), dpt = at_zero();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      st = at_mfma(at_row(kimg, 32 * kb + r, s, hh), qf[s], st);
      dpt = at_mfma(at_row(vimg, 32 * kb + r, s, hh), gf[s], dpt);
    }
    bf16x8 df0, df1;
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) {
      const int key = 32 * kb + at_crow(rho, hh);
      float v = st[rho] * 0.125f;
      if (MASK && key < L && qok) v += mask[(long long)q * L + key];
      const float p = (key < L && qok) ? __expf(v - lq) : 0.f;
      const float ds = p * (dpt[rho] - D);
      if (rho < 8) df0[rho] = (bf16)ds;
      else df1[rho - 8] = (bf16)ds;
    }
    dq0 = at_mfma(at_trfrag(kimg, 32 * kb, 0, lane), df0, dq0);
    dq0 = at_mfma(at_trfrag(kimg, 32 * kb + 16, 0, lane), df1, dq0);
    dq1 = at_mfma(at_trfrag(kimg, 32 * kb, 32, lane), df0, dq1);
    dq1 = at_mfma(at_trfrag(kimg, 32 * kb + 16, 32, lane), df1, dq1);
  }
  if (qok) {
    at_store_t(dqkv + (long long)q * rs + (long long)n * ld + h * 64, dq0, dq1, 0.125f, hh);
    if (hh == 0) Dout[item] = D;
  }
}

template <bool MASK>
__global__ void __launch_bounds__(512) attn_bwd_kv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ Din, int L, int N, int heads,
                                                          const float* __restrict__ mask, bf16* __restrict__ dqkv) {
  __shared__ __attribute__((aligned(16))) char smem[2 * AT_IMG];
  __shared__ __attribute__((aligned(16))) float ls[AT_MAXB * 32], ds_[AT_MAXB * 32];
  char* qimg = smem;
  char* gimg = smem + AT_IMG;
  const int nb = (L + 31) >> 5;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = (int)(blockIdx.x % heads), n = (int)(blockIdx.x / heads);
  const int E = heads * 64;
  const long long ld = 3LL * E, rs = (long long)N * ld, ors = (long long)N * E;
  const bf16* base = qkv + (long long)n * ld + h * 64;
  at_stage2(base, rs, dout + (long long)n * E + h * 64, ors, L, qimg, gimg, tid, nb * 64);
  for (int i = tid; i < nb * 32; i += nb * 64) {
    const long long it = ((long long)i * N + n) * heads + h;
    ls[i] = i < L ? lse[it] : 0.f;
    ds_[i] = i < L ? Din[it] : 0.f;
  }
  const int r = lane & 31, hh = lane >> 5;
  const int key = 32 * w + r;
  const bool kok = key < L;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = at_ld16(base + E + key * rs + 16 * s + 8 * hh, kok);
    vf[s] = at_ld16(base + 2 * E + key * rs + 16 * s + 8 * hh, kok);
  }
  __syncthreads();

  f32x16 dk0 = at_zero(), dk1 = at_zero(), dv0 = at_zero(), dv1 = at_zero();
  for (int qb = 0; qb < nb; ++qb) {
    f32x16 sc = at_zero(), dp = at_zero();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sc = at_mfma(at_row(qimg, 32 * qb + r, s, hh), kf[s], sc);
      dp = at_mfma(at_row(gimg, 32 * qb + r, s, hh), vf[s], dp);
    }
    bf16x8 pf0, pf1, df0, df1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int q0 = 32 * qb + 8 * g + 4 * hh;
      const float4 l4 = *reinterpret_cast<const float4*>(&ls[q0]);
      const float4 d4 = *reinterpret_cast<const float4*>(&ds_[q0]);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rho = 4 * g + e, qi = q0 + e;
        float v = sc[rho] * 0.125f;
        if (MASK && qi < L && kok) v += mask[(long long)qi * L + key];
        const float p = (qi < L && kok) ? __expf(v - lv[e]) : 0.f;
        const float d = p * (dp[rho] - dv[e]);
        if (rho < 8) { pf0[rho] = (bf16)p; df0[rho] = (bf16)d; }
        else { pf1[rho - 8] = (bf16)p; df1[rho - 8] = (bf16)d; }
      }
    }
    dv0 = at_mfma(at_trfrag(gimg, 32 * qb, 0, lane), pf0, dv0);
    dv0 = at_mfma(at_trfrag(gimg, 32 * qb + 16, 0, lane), pf1, dv0);
    dv1 = at_mfma(at_trfrag(gimg, 32 * qb, 32, lane), pf0, dv1);
    dv1 = at_mfma(at_trfrag(gimg, 32 * qb + 16, 32, lane), pf1, dv1);
    dk0 = at_mfma(at_trfrag(qimg, 32 * qb, 0, lane), df0, dk0);
    dk0 = at_mfma(at_trfrag(qimg, 32 * qb + 16, 0, lane), df1, dk0);
    dk1 = at_mfma(at_trfrag(qimg, 32 * qb, 32, lane), df0, dk1);
    dk1 = at_mfma(at_trfrag(qimg, 32 * qb + 16, 32, lane), df1, dk1);
  }
  if (kok) {
    bf16* dst = dqkv + (long long)key * rs + (long long)n * ld + h * 64;
    at_store_t(dst + E, dk0, dk1, 0.125f, hh);
    at_store_t(dst + 2 * E, dv0, dv1, 1.f, hh);
  }
}

// The backward in ONE workgroup per (batch n, head h): the four (L x 64)
// slices Q, K, V, dO are staged into LDS once (128 KB) and wave w runs the query
// side of block w (dQ) and then the key side of block w (dK, dV) on them.  The
// two-kernel form above read Q, K, V and dO twice from HBM (once per side) and
// passed D = rowsum(dO o O) through global memory: 6.2 GB per ViT-B/16 layer
// at 512 triplets (profiles/r4_c5_pmc_traffic.json) where this one needs
// 3.7 GB (Q K V dO O once, dQ dK dV once).  The q side's own operands come from
// the images (at_row of image row q is the layout at_ld16 loads).  Softmax in
// the log2 domain (one FMA and v_exp_f32 per element) and, without a mask, no
// validity tests (see the comments in the loops).
template <bool MASK>
__global__ void __launch_bounds__(512) attn_bwd_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ o,
                                                       const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                       int L, int N, int heads, const float* __restrict__ mask,
                                                       bf16* __restrict__ dqkv) {
  __shared__ __attribute__((aligned(16))) char smem[4 * AT_IMG];
  __shared__ __attribute__((aligned(16))) float ls[AT_MAXB * 32], ds_[AT_MAXB * 32];
  char* kimg = smem;
  char* vimg = smem + AT_IMG;
  char* qimg = smem + 2 * AT_IMG;
  char* gimg = smem + 3 * AT_IMG;
  const int nb = (L + 31) >> 5;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = (int)(blockIdx.x % heads), n = (int)(blockIdx.x / heads);
  const int E = heads * 64;
  const long long ld = 3LL * E, rs = (long long)N * ld, ors = (long long)N * E;
  const bf16* base = qkv + (long long)n * ld + h * 64;
  const int r = lane & 31, hh = lane >> 5;
  const int q = 32 * w + r;  // the q side's row and the key side's key
  const bool qok = q < L;
  const long long orow = (long long)q * ors + (long long)n * E + h * 64;
  // O and dO of this wave's query rows for D (issued ahead of the staging)
  bf16x8 of[4], gd[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    of[s] = at_ld16(o + orow + 16 * s + 8 * hh, qok);
    gd[s] = at_ld16(dout + orow + 16 * s + 8 * hh, qok);
  }
  const long long item = ((long long)q * N + n) * heads + h;
  const float lq = qok ? lse[item] : 0.f;
  at_stage2(base + E, rs, base + 2 * E, rs, L, kimg, vimg, tid, nb * 64);
  at_stage2(base, rs, dout + (long long)n * E + h * 64, ors, L, qimg, gimg, tid, nb * 64);
  float D = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) D += (float)gd[s][j] * (float)of[s][j];
  D += __shfl_xor(D, 32, 64);
  const float lq2 = lq * AT_LOG2E;  // log-sum-exp in the log2 domain
  if (hh == 0) {
    ls[q] = lq2;
    ds_[q] = qok ? D : 0.f;
  }
  __syncthreads();

  {  // ---- query side of block w: S^T = K Q^T, dP^T = V dO^T, dQ^T += K^T dS^T
    bf16x8 qf[4], gf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = at_row(qimg, q, s, hh);
      gf[s] = at_row(gimg, q, s, hh);
    }
    f32x16 dq0 = at_zero(), dq1 = at_zero();
    // one key block; CHK: the last block when L % 32 != 0
    auto qblock = [&](int kb, auto chk) {
      constexpr bool CHK = decltype(chk)::value;
      f32x16 st = at_zero(), dpt = at_zero();
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = at_mfma(at_row(kimg, 32 * kb + r, s, hh), qf[s], st);
        dpt = at_mfma(at_row(vimg, 32 * kb + r, s, hh), gf[s], dpt);
      }
      bf16x8 df0, df1;
#pragma unroll
      for (int rho = 0; rho < 16; ++rho) {
        // without a mask a key >= L has zero K and V rows, so its dS meets a zero
        // row of K in dQ (rows q >= L are not stored); its p = exp2(-lse2) is
        // zeroed all the same in the last block (CHK), or a row whose log-sum-exp
        // is below ~-88 would make it inf and the product with the zero K row NaN
        float p;
        const int key = 32 * kb + at_crow(rho, hh);
        if (MASK) {
          float v = st[rho] * AT_SC2;
          if (key < L && qok) v += mask[(long long)q * L + key] * AT_LOG2E;
          p = (key < L && qok) ? __builtin_amdgcn_exp2f(v - lq2) : 0.f;
        } else {
          p = __builtin_amdgcn_exp2f(fmaf(st[rho], AT_SC2, -lq2));
          if (CHK) p = key < L ? p : 0.f;
        }
        const float ds = p * (dpt[rho] - D);
        if (rho < 8) df0[rho] = (bf16)ds;
        else df1[rho - 8] = (bf16)ds;
      }
      dq0 = at_mfma(at_trfrag(kimg, 32 * kb, 0, lane), df0, dq0);
      dq0 = at_mfma(at_trfrag(kimg, 32 * kb + 16, 0, lane), df1, dq0);
      dq1 = at_mfma(at_trfrag(kimg, 32 * kb, 32, lane), df0, dq1);
      dq1 = at_mfma(at_trfrag(kimg, 32 * kb + 16, 32, lane), df1, dq1);
    };
    const int nfull = (L & 31) ? nb - 1 : nb;
    for (int kb = 0; kb < nfull; ++kb) qblock(kb, std::false_type{});
    if (nfull < nb) qblock(nfull, std::true_type{});
    if (qok) at_store_t(dqkv + (long long)q * rs + (long long)n * ld + h * 64, dq0, dq1, 0.125f, hh);
  }

  // ---- key side of block w: S = Q K^T, dP = dO V^T, dS = P (dP - D),
  // dV^T += dO^T P, dK^T += Q^T dS
  const int key = q;
  const bool kok = qok;
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = at_row(kimg, key, s, hh);
    vf[s] = at_row(vimg, key, s, hh);
  }
  f32x16 dk0 = at_zero(), dk1 = at_zero(), dv0 = at_zero(), dv1 = at_zero();
  for (int qb = 0; qb < nb; ++qb) {
    f32x16 sc = at_zero(), dp = at_zero();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      sc = at_mfma(at_row(qimg, 32 * qb + r, s, hh), kf[s], sc);
      dp = at_mfma(at_row(gimg, 32 * qb + r, s, hh), vf[s], dp);
    }
    bf16x8 pf0, pf1, df0, df1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int q0 = 32 * qb + 8 * g + 4 * hh;
      const float4 l4 = *reinterpret_cast<const float4*>(&ls[q0]);
      const float4 d4 = *reinterpret_cast<const float4*>(&ds_[q0]);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rho = 4 * g + e, qi = q0 + e;
        // no validity test without a mask: a query row >= L has zero Q and dO
        // rows and ls = ds_ = 0, so p = 1 meets dP = 0 and a zero row of dO
        float p;
        if (MASK) {
          float v = sc[rho] * AT_SC2;
          if (qi < L && kok) v += mask[(long long)qi * L + key] * AT_LOG2E;
          p = (qi < L && kok) ? __builtin_amdgcn_exp2f(v - lv[e]) : 0.f;
        } else {
          p = __builtin_amdgcn_exp2f(fmaf(sc[rho], AT_SC2, -lv[e]));
        }
        const float d = p * (dp[rho] - dv[e]);
        if (rho < 8) { pf0[rho] = (bf16)p; df0[rho] = (bf16)d; }
        else { pf1[rho - 8] = (bf16)p; df1[rho - 8] = (bf16)d; }
      }
    }
    dv0 = at_mfma(at_trfrag(gimg, 32 * qb, 0, lane), pf0, dv0);
    dv0 = at_mfma(at_trfrag(gimg, 32 * qb + 16, 0, lane), pf1, dv0);
    dv1 = at_mfma(at_trfrag(gimg, 32 * qb, 32, lane), pf0, dv1);
    dv1 = at_mfma(at_trfrag(gimg, 32 * qb + 16, 32, lane), pf1, dv1);
    dk0 = at_mfma(at_trfrag(qimg, 32 * qb, 0, lane), df0, dk0);
    dk0 = at_mfma(at_trfrag(qimg, 32 * qb + 16, 0, lane), df1, dk0);
    dk1 = at_mfma(at_trfrag(qimg, 32 * qb, 32, lane), df0, dk1);
    dk1 = at_mfma(at_trfrag(qimg, 32 * qb + 16, 32, lane), df1, dk1);
  }
  if (kok) {
    bf16* dst = dqkv + (long long)key * rs + (long long)n * ld + h * 64;
    at_store_t(dst + E, dk0, dk1, 0.125f, hh);
    at_store_t(dst + 2 * E, dv0, dv1, 1.f, hh);
  }
}

// launchers (vit.hip's entry points route bf16 here): false if not applicable
bool attn_fwd_mfma(const bf16* qkv, int L, int N, int heads, const float* mask, bf16* out, float* lse,
                   unsigned* pmax, hipStream_t st) {
  if (L < 1 || L > 32 * AT_MAXB || N < 1 || heads < 1) return false;
  const long long grid = (long long)N * heads;
  if (grid > 0x7fffffffLL) return false;
  const int nthr = ((L + 31) / 32) * 64;
  if (mask)
    hipLaunchKernelGGL(attn_fwd_kernel<true>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, L, N, heads, mask, out, lse,
                       pmax);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<false>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, L, N, heads, mask, out,
                       lse, pmax);
  return true;
}

bool attn_bwd_mfma(const bf16* qkv, const bf16* o, const bf16* dout, const float* lse, int L, int N, int heads,
                   const float* mask, bf16* dqkv, float* dscratch, hipStream_t st) {
  if (L < 1 || L > 32 * AT_MAXB || N < 1 || heads < 1) return false;
  const long long grid = (long long)N * heads;
  if (grid > 0x7fffffffLL) return false;
  const int nthr = ((L + 31) / 32) * 64;
  // ARTSBIR_ATTN_BWD2=1: the two-kernel form (timing comparison)
  static const bool two = [] { const char* e = getenv("ARTSBIR_ATTN_BWD2"); return e && atoi(e) != 0; }();
  if (!two) {
    if (mask)
      hipLaunchKernelGGL(attn_bwd_kernel<true>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, o, dout, lse, L, N, heads,
                         mask, dqkv);
    else
      hipLaunchKernelGGL(attn_bwd_kernel<false>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, o, dout, lse, L, N,
                         heads, mask, dqkv);
    return true;
  }
  if (mask) {
    hipLaunchKernelGGL(attn_bwd_q_kernel<true>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, o, dout, lse, L, N,
                       heads, mask, dqkv, dscratch);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<true>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, dout, lse, dscratch, L,
                       N, heads, mask, dqkv);
  } else {
    hipLaunchKernelGGL(attn_bwd_q_kernel<false>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, o, dout, lse, L, N,
                       heads, mask, dqkv, dscratch);
    hipLaunchKernelGGL(attn_bwd_kv_kernel<false>, dim3((unsigned)grid), dim3(nthr), 0, st, qkv, dout, lse, dscratch,
                       L, N, heads, mask, dqkv);
  }
  return true;
}

}  // namespace artsbir
