// Attention-pool core of AttentionPool2d (models.py:249-272): for each image and
// head, one query (token 0) against the HW+1 tokens — softmax(q.k/sqrt(hd)).v —
// and its backward.  The q/k/v/c projections around it run on the MFMA GEMMs
// (gemm.hip); this is the small per-head part of F.multi_head_attention_forward.
//
// Layouts: Q [B][C] f32 (bias added), KV [B*T][2C] T (K in columns [0,C), V in
// [C,2C)), P [B][heads][T] f32 (saved softmax), O [B][C] T.  head_dim == 64
// (one lane per head dimension), T <= 128 (two tokens per lane).
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const float* __restrict__ Q, const T* __restrict__ KV, int C,
                                                       int heads, int Tk, float scale, float* __restrict__ P,
                                                       T* __restrict__ O) {
  extern __shared__ float qs[];  // C floats
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < C; i += blockDim.x) qs[i] = Q[(long long)b * C + i];
  __syncthreads();
  const long long ld = 2LL * C;
  const T* kvb = KV + (long long)b * Tk * ld;
  for (int h = wid; h < heads; h += blockDim.x / 64) {
    const float* q = qs + h * 64;
    float s[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t = lane + 64 * j;
      float acc = -INFINITY;
      if (t < Tk) {
        acc = 0.f;
        const T* kr = kvb + t * ld + h * 64;
#pragma unroll
        for (int d0 = 0; d0 < 64; d0 += 8) {
          Vec16<T> v0 = ld16<T>(kr + d0);
          if constexpr (Vec16<T>::N == 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc += q[d0 + e] * to_f(v0.v[e]);
          } else {
            Vec16<T> v1 = ld16<T>(kr + d0 + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc += q[d0 + e] * to_f(v0.v[e]) + 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) acc += q[d0 + 4 + e] * to_f(v1.v[e]);
          }
        }
        acc *= scale;
      }
      s[j] = acc;
    }
    const float m = wave_max(fmaxf(s[0], s[1]));
    float p[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) p[j] = (lane + 64 * j < Tk) ? __expf(s[j] - m) : 0.f;
    const float inv = 1.f / warp_sum(p[0] + p[1]);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      p[j] *= inv;
      const int t = lane + 64 * j;
      if (t < Tk) P[((long long)b * heads + h) * Tk + t] = p[j];
    }
    // o[d] = sum_t p_t v[t][d], lane = d
    float o = 0.f;
    for (int t = 0; t < Tk; ++t) {
      const float pt = __shfl(t < 64 ? p[0] : p[1], t & 63, 64);
      o += pt * to_f(kvb[t * ld + C + h * 64 + lane]);
    }
    O[(long long)b * C + h * 64 + lane] = from_f<T>(o);
  }
}

// dO [B][C] f32 -> dQ [B][C] T (pre-scale folded), dKV [B*T][2C] T
template <typename T>
__global__ void __launch_bounds__(256) attn_bwd_kernel(const float* __restrict__ Q, const T* __restrict__ KV,
                                                       const float* __restrict__ P, const float* __restrict__ dO, int C,
                                                       int heads, int Tk, float scale, T* __restrict__ dQ,
                                                       T* __restrict__ dKV) {
  extern __shared__ float sm[];  // q[C], dO[C]
  float* qs = sm;
  float* dos = sm + C;
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    qs[i] = Q[(long long)b * C + i];
    dos[i] = dO[(long long)b * C + i];
  }
  __syncthreads();
  const long long ld = 2LL * C;
  const T* kvb = KV + (long long)b * Tk * ld;
  T* dkvb = dKV + (long long)b * Tk * ld;
  for (int h = wid; h < heads; h += blockDim.x / 64) {
    const float* g = dos + h * 64;
    // dp_t = dO . v_t ; lane = t
    float p[2], dp[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int t = lane + 64 * j;
      float acc = 0.f, pv = 0.f;
      if (t < Tk) {
        pv = P[((long long)b * heads + h) * Tk + t];
        const T* vr = kvb + t * ld + C + h * 64;
        for (int d = 0; d < 64; ++d) acc += g[d] * to_f(vr[d]);
      }
      p[j] = pv;
      dp[j] = acc;
    }
    const float sdot = warp_sum(p[0] * dp[0] + p[1] * dp[1]);
    float ds[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) ds[j] = p[j] * (dp[j] - sdot);
    // lane = d
    const float qd = qs[h * 64 + lane], gd = g[lane];
    float dq = 0.f;
    for (int t = 0; t < Tk; ++t) {
      const float dst = __shfl(t < 64 ? ds[0] : ds[1], t & 63, 64);
      const float pt = __shfl(t < 64 ? p[0] : p[1], t & 63, 64);
      dq += dst * to_f(kvb[t * ld + h * 64 + lane]);
      dkvb[t * ld + h * 64 + lane] = from_f<T>(dst * qd * scale);
      dkvb[t * ld + C + h * 64 + lane] = from_f<T>(pt * gd);
    }
    dQ[(long long)b * C + h * 64 + lane] = from_f<T>(dq * scale);
  }
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_attnpool_fwd(int dtype, const float* q, const void* kv, int B, int C, int heads, int T,
                                    float* p, void* o, void* stream) {
  if (C != heads * 64) { set_error("attnpool: head_dim must be 64 (C=%d heads=%d)", C, heads); return -1; }
  if (T < 1 || T > 128) { set_error("attnpool: tokens=%d outside [1,128]", T); return -1; }
  const float scale = 1.f / sqrtf(64.f);
  const size_t sh = (size_t)C * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(attn_fwd_kernel<bf16>, dim3(B), dim3(256), sh, st, q, (const bf16*)kv, C, heads, T, scale, p, (bf16*)o);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<float>, dim3(B), dim3(256), sh, st, q, (const float*)kv, C, heads, T, scale, p, (float*)o);
  ARTSBIR_CHECK_LAUNCH("attnpool_fwd");
  return 0;
}

extern "C" int artsbir_attnpool_bwd(int dtype, const float* q, const void* kv, const float* p, const float* dout,
                                    int B, int C, int heads, int T, void* dq, void* dkv, void* stream) {
  if (C != heads * 64) { set_error("attnpool: head_dim must be 64 (C=%d heads=%d)", C, heads); return -1; }
  if (T < 1 || T > 128) { set_error("attnpool: tokens=%d outside [1,128]", T); return -1; }
  const float scale = 1.f / sqrtf(64.f);
  const size_t sh = 2 * (size_t)C * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(attn_bwd_kernel<bf16>, dim3(B), dim3(256), sh, st, q, (const bf16*)kv, p, dout, C, heads, T, scale,
                       (bf16*)dq, (bf16*)dkv);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<float>, dim3(B), dim3(256), sh, st, q, (const float*)kv, p, dout, C, heads, T,
                       scale, (float*)dq, (float*)dkv);
  ARTSBIR_CHECK_LAUNCH("attnpool_bwd");
  return 0;
}
