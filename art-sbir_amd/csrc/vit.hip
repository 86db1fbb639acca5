// Transformer block pieces of models.py:382-417 (LayerNorm computed in fp32,
// QuickGELU, the multi-head self-attention core of nn.MultiheadAttention as
// ResidualAttentionBlock uses it).  The reference defines the block but builds
// no model from it (block-level parity); its projections run on
// the MFMA GEMM (artsbir_gemm_nt), these kernels are the rest.
//
// Layouts follow nn.MultiheadAttention (batch_first=False): x [L][N][E]
// row-major, qkv [L*N][3E] = x @ in_proj_weight^T + in_proj_bias (q | k | v
// columns), out [L*N][E] before out_proj.  head_dim == 64 (one lane per head
// dimension), L <= 256 (four keys per lane).
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

__device__ __forceinline__ float vit_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
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
__global__ void quickgelu_kernel(const T* __restrict__ x, long long n, T* __restrict__ y) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = to_f(x[i]);
    y[i] = from_f<T>(v / (1.f + __expf(-1.702f * v)));
  }
}

// softmax(q k^T / sqrt(64) + mask) v for one (query position, batch, head)
// per wave: lane l scores keys l, l+64, l+128, l+192; the probabilities go
// through LDS; lane d accumulates output dimension d over the keys
template <typename T>
__global__ void __launch_bounds__(256) mha_fwd_kernel(const T* __restrict__ qkv, int L, int N, int heads,
                                                      const float* __restrict__ mask, T* __restrict__ out) {
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
  const float inv = 1.f / warp_sum(sum);
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

static inline unsigned vit_grid(long long n) {
  long long g = (n + 255) / 256;
  return (unsigned)(g > (1 << 20) ? (1 << 20) : g < 1 ? 1 : g);
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_layernorm_fwd(int dtype, const void* x, const float* gamma, const float* beta, long long rows,
                                     int C, float eps, void* y, void* stream) {
  if (rows <= 0) return 0;
  const unsigned grid = (unsigned)((rows + 3) / 4);
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(layernorm_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)x, gamma, beta, rows, C, eps, (T*)y));
  ARTSBIR_CHECK_LAUNCH("layernorm_fwd");
  return 0;
}

extern "C" int artsbir_quickgelu(int dtype, const void* x, long long n, void* y, void* stream) {
  if (n <= 0) return 0;
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(quickgelu_kernel<T>, dim3(vit_grid(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)x, n, (T*)y));
  ARTSBIR_CHECK_LAUNCH("quickgelu");
  return 0;
}

extern "C" int artsbir_mha_fwd(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out,
                               void* stream) {
  if (L < 1 || L > 256) { set_error("mha_fwd: sequence length %d outside [1, 256]", L); return -1; }
  if (heads < 1 || N < 1) { set_error("mha_fwd: bad batch %d / heads %d", N, heads); return -1; }
  const long long items = (long long)L * N * heads;
  const unsigned grid = (unsigned)((items + 3) / 4);
  VIT_DISPATCH(dtype, hipLaunchKernelGGL(mha_fwd_kernel<T>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)qkv, L, N, heads, mask, (T*)out));
  ARTSBIR_CHECK_LAUNCH("mha_fwd");
  return 0;
}
