// fp8 (OCP e4m3fn) projection GEMM for the ViT-B/16 configuration C5 (SURVEY
// §8 f4: "ViT-B/16 768-d fp8"): per-tensor scaled e4m3 operands on the
// block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales
// (E8M0 127), which runs at the fp8 rate (2x bf16; the unscaled fp8 MFMA runs
// at the bf16 rate, cdna_hip_programming.md §3).
//
//   artsbir_quantize_fp8: q = e4m3(x / s), s = amax(|x|) / 448 (1 if amax is 0),
//                         round-to-nearest-even on the f32 value, saturating
//   artsbir_gemm_nt_fp8:  C[M][N] = sa sb sum_k A[m][k] B[n][k] (+ bias[n]) (+ C)
//
// GEMM structure: 128x128 output tile per 256-thread workgroup (4 waves, each
// 64x64 = 4x4 MFMA tiles), K-step 128 (one MFMA per tile per step), operands
// register-staged into a double-buffered LDS image of 128-B rows whose 16-B
// chunks sit at slot chunk ^ (row & 7), so the fragment reads (16 rows x one
// 32-B k-slice per lane group) spread over the banks.  MFMA operand map:
// lane l supplies row / column l & 15, k = 32 (l >> 4) .. +31 (32 bytes).
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

typedef __attribute__((ext_vector_type(8))) int i32x8;

__device__ __forceinline__ float fp8_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define FP8_DISPATCH(dtype, ...)                    \
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

template <typename T>
__global__ void __launch_bounds__(256) fp8_amax_kernel(const T* __restrict__ x, long long n,
                                                       unsigned* __restrict__ amax_bits) {
  float m = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) m = fmaxf(m, fabsf(to_f(x[i])));
  m = fp8_wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(amax_bits, __float_as_uint(b));  // non-negative floats order as their bits
  }
}

// f32 -> e4m3fn, round to nearest even on the f32 value, saturating to 448.
// (v_cvt_pk_fp8_f32 rounds 61.999996 up to 64, not to 60: not an exact RNE of
// its f32 input, so the codes would differ from torch's float8_e4m3fn cast.)
__device__ __forceinline__ unsigned char fp8_e4m3_rne(float x) {
  const unsigned u = __float_as_uint(x);
  const unsigned sign = (u >> 24) & 0x80u;
  const float a = fabsf(x);
  if (!(a == a)) return 0x7f;                       // NaN
  if (a >= 448.f) return (unsigned char)(sign | 0x7eu);
  if (a < 0.015625f) {                               // below 2^-6: subnormal steps of 2^-9
    const unsigned qv = (unsigned)rintf(a * 512.f);  // exact scaling, RNE; 8 is the smallest normal
    return (unsigned char)(sign | qv);
  }
  const unsigned ua = __float_as_uint(a);
  int e = (int)((ua >> 23) & 0xffu) - 127;
  unsigned r = (ua & 0x7fffffu) >> 20;
  const unsigned rem = ua & 0xfffffu;
  if (rem > 0x80000u || (rem == 0x80000u && (r & 1u))) ++r;
  if (r == 8u) { r = 0u; ++e; }
  unsigned code = ((unsigned)(e + 7) << 3) | r;
  if (code > 0x7eu) code = 0x7eu;
  return (unsigned char)(sign | code);
}

template <typename T>
__global__ void __launch_bounds__(256) fp8_quant_kernel(const T* __restrict__ x, long long n,
                                                        const unsigned* __restrict__ amax_bits,
                                                        unsigned char* __restrict__ q) {
  const float amax = __uint_as_float(*amax_bits);
  const float sc = amax > 0.f ? amax / 448.f : 1.f;  // x / s, correctly rounded (as the documented formula)
  for (long long i = (blockIdx.x * 256LL + threadIdx.x) * 4; i < n; i += gridDim.x * 256LL * 4) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = i + e < n ? to_f(x[i + e]) / sc : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i + e < n) q[i + e] = fp8_e4m3_rne(v[e]);
  }
}

__global__ void fp8_scale_kernel(unsigned* amax_bits) {  // amax -> the scale s, in place
  const float amax = __uint_as_float(*amax_bits);
  reinterpret_cast<float*>(amax_bits)[0] = amax > 0.f ? amax / 448.f : 1.f;
}

__device__ __forceinline__ int fp8_slot(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <typename T>
__global__ void __launch_bounds__(256) gemm_fp8_kernel(int M, int N, int K, const unsigned char* __restrict__ A,
                                                       const unsigned char* __restrict__ B,
                                                       const float* __restrict__ sa, const float* __restrict__ sb,
                                                       const float* __restrict__ bias, T* __restrict__ C,
                                                       int accumulate) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2][2][128 * 128];  // [buf][A|B]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = (N + 127) / 128;
  const int m0 = (blockIdx.x / tiles_n) * 128, n0 = (blockIdx.x % tiles_n) * 128;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const int nk = K / 128;
  uint4 ra[4], rb[4];
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7;
      const long long ka = (long long)kt * 128 + ch * 16;
      ra[i] = m0 + row < M ? *reinterpret_cast<const uint4*>(A + (long long)(m0 + row) * K + ka) : uint4{0, 0, 0, 0};
      rb[i] = n0 + row < N ? *reinterpret_cast<const uint4*>(B + (long long)(n0 + row) * K + ka) : uint4{0, 0, 0, 0};
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + 256 * i, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4*>(&lds[buf][0][fp8_slot(row, ch)]) = ra[i];
      *reinterpret_cast<uint4*>(&lds[buf][1][fp8_slot(row, ch)]) = rb[i];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, kq = lane >> 4;  // fragment row / column, k slice (32 bytes = chunks 2kq, 2kq+1)
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    i32x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm + i * 16 + fr;
      const uint4 lo = *reinterpret_cast<const uint4*>(&lds[buf][0][fp8_slot(r, 2 * kq)]);
      const uint4 hi = *reinterpret_cast<const uint4*>(&lds[buf][0][fp8_slot(r, 2 * kq + 1)]);
      af[i] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn + j * 16 + fr;
      const uint4 lo = *reinterpret_cast<const uint4*>(&lds[buf][1][fp8_slot(r, 2 * kq)]);
      const uint4 hi = *reinterpret_cast<const uint4*>(&lds[buf][1][fp8_slot(r, 2 * kq + 1)]);
      bfr[j] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f,
                                                                     0, 0x7f7f7f7f);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  const float s = sa[0] * sb[0];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + j * 16 + fr;
      if (n >= N) continue;
      const float bn = bias ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + kq * 4 + r;
        if (m >= M) continue;
        float v = acc[i][j][r] * s + bn;
        T* p = C + (long long)m * N + n;
        if (accumulate) v += to_f(*p);
        *p = from_f<T>(v);
      }
    }
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_quantize_fp8(int dtype, const void* x, long long n, unsigned char* q, float* scale,
                                    void* stream) {
  if (n <= 0 || !x || !q || !scale) { set_error("quantize_fp8: bad arguments"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(scale, 0, sizeof(float), st) != hipSuccess) { set_error("quantize_fp8: memset"); return -2; }
  long long g = (n + 1023) / 1024;
  const unsigned grid = (unsigned)(g > 2048 ? 2048 : g < 1 ? 1 : g);
  unsigned* bits = reinterpret_cast<unsigned*>(scale);
  FP8_DISPATCH(dtype, hipLaunchKernelGGL(fp8_amax_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)x, n, bits));
  FP8_DISPATCH(dtype, hipLaunchKernelGGL(fp8_quant_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)x, n, bits, q));
  hipLaunchKernelGGL(fp8_scale_kernel, dim3(1), dim3(1), 0, st, bits);
  ARTSBIR_CHECK_LAUNCH("quantize_fp8");
  return 0;
}

extern "C" int artsbir_gemm_nt_fp8(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                                   const float* sa, const float* sb, const float* bias, void* c, int out_dtype,
                                   int accumulate, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 != 0 || K <= 0) { set_error("gemm_nt_fp8: K=%d must be a positive multiple of 128", K); return -1; }
  if (!a || !b || !sa || !sb || !c) { set_error("gemm_nt_fp8: bad arguments"); return -1; }
  const long long tiles = (long long)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles > 0x7fffffffLL) { set_error("gemm_nt_fp8: too many tiles"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  FP8_DISPATCH(out_dtype, hipLaunchKernelGGL(gemm_fp8_kernel<T>, dim3((unsigned)tiles), dim3(256), 0, st, M, N, K, a,
                                           b, sa, sb, bias, (T*)c, accumulate));
  ARTSBIR_CHECK_LAUNCH("gemm_nt_fp8");
  return 0;
}
