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
#include <cstdlib>

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

__device__ __forceinline__ void fp8_load8(const bf16* p, float (&v)[8]) {
  const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
}
__device__ __forceinline__ void fp8_load8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__global__ void __launch_bounds__(256) fp8_amax_kernel(const T* __restrict__ x, long long n,
                                                       unsigned* __restrict__ amax_bits) {
  float m = 0.f;
  const long long n8 = (reinterpret_cast<uintptr_t>(x) & 15) ? 0 : n / 8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += gridDim.x * 256LL) {
    float v[8];
    fp8_load8(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  for (long long i = n8 * 8 + blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL)
    m = fmaxf(m, fabsf(to_f(x[i])));
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
// Branch-free: in the normal range the f32 mantissa is rounded to 3 bits by an
// integer add (ties to even; a carry moves into the exponent) and rebiased
// (127 - 7 = 120); below 2^-6 the code counts multiples of 2^-9.  Identical to
// the branchy per-case form for all 2^32 inputs (checked exhaustively on the CPU).
__device__ __forceinline__ unsigned fp8_e4m3_rne(float x) {
  const unsigned u = __float_as_uint(x);
  const unsigned ua = u & 0x7fffffffu;
  const unsigned n = ua + 0x7ffffu + ((ua >> 20) & 1u);
  int code = (int)(n >> 20) - (120 << 3);
  code = code > 0x7e ? 0x7e : code;
  const unsigned sub = (unsigned)rintf(__uint_as_float(ua) * 512.f);
  const unsigned c = ((u >> 24) & 0x80u) | (ua < 0x3c800000u ? sub : (unsigned)code);
  return ua > 0x7f800000u ? 0x7fu : c;  // NaN
}

// x / s correctly rounded from rs = 1 / s (correctly rounded, once per thread):
// q = x rs, then one fma-corrected step (the residual x - q s is exact in f32).
// Equal to the IEEE quotient except where that residual falls below the normal
// range (|x| near 2^-126), whose quotients all encode as a signed fp8 zero; the
// sign is x's (the correction turns -0 into +0; s > 0).
__device__ __forceinline__ float fp8_div(float x, float s, float rs) {
  const float q = x * rs;
  return copysignf(fmaf(fmaf(-q, s, x), rs, q), x);
}

// four quotients to their e4m3fn codes (byte e = value e) by the hardware
// conversion (v_cvt_pk_fp8_f32: OCP e4m3fn on gfx950, round to nearest even):
// the same codes as fp8_e4m3_rne for every |v| <= 448 (the quantiser's range,
// x / s with s = amax / 448) at two instructions per four values instead of
// about 17 VALU per value; ARTSBIR_FP8_SWCVT builds the integer rounding instead
#ifndef ARTSBIR_FP8_SWCVT
__device__ __forceinline__ unsigned fp8_pack4(float a, float b, float c, float d) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (unsigned)r;
}
#else
__device__ __forceinline__ unsigned fp8_pack4(float a, float b, float c, float d) {
  return fp8_e4m3_rne(a) | fp8_e4m3_rne(b) << 8 | fp8_e4m3_rne(c) << 16 | fp8_e4m3_rne(d) << 24;
}
#endif

template <typename T>
__global__ void __launch_bounds__(256) fp8_quant_kernel(const T* __restrict__ x, long long n,
                                                        const unsigned* __restrict__ amax_bits,
                                                        unsigned char* __restrict__ q) {
  const float amax = __uint_as_float(*amax_bits);
  const float sc = amax > 0.f ? amax / 448.f : 1.f;  // x / s, correctly rounded (as the documented formula)
  const float rs = 1.f / sc;
  const long long n8 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(q)) & 15) ? 0 : n / 8;
  const long long G = gridDim.x * 256LL;
  long long i = blockIdx.x * 256LL + threadIdx.x;
  // QU chunks per trip, every load of the trip issued before the first
  // conversion: one 16-B load in flight per lane left the pass latency-bound
  constexpr int QU = 4;
  // the codes are stored non-temporally (FP8Q_NT): the pass 0.598 -> 0.585 ms at
  // 302592 x 3072, C5 step -0.3 ms (profiles/r5_quant.txt); 16 values per lane
  // (two 16-B loads, one 16-B store) measured slower
#ifndef FP8Q_NT
#define FP8Q_NT 1
#endif
  for (; i + (QU - 1) * G < n8; i += QU * G) {
    float v[QU][8];
#pragma unroll
    for (int u = 0; u < QU; ++u) fp8_load8(x + (i + u * G) * 8, v[u]);
#pragma unroll
    for (int u = 0; u < QU; ++u) {
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = fp8_div(v[u][e], sc, rs);
      const uint2 o = make_uint2(fp8_pack4(d[0], d[1], d[2], d[3]), fp8_pack4(d[4], d[5], d[6], d[7]));
      typedef __attribute__((ext_vector_type(2))) unsigned q32x2;
      const q32x2 ov = {o.x, o.y};
      if (FP8Q_NT) __builtin_nontemporal_store(ov, reinterpret_cast<q32x2*>(q + (i + u * G) * 8));
      else *reinterpret_cast<q32x2*>(q + (i + u * G) * 8) = ov;
    }
  }
  for (; i < n8; i += G) {
    float v[8];
    fp8_load8(x + i * 8, v);
    float d[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = fp8_div(v[e], sc, rs);
    *reinterpret_cast<uint2*>(q + i * 8) =
        make_uint2(fp8_pack4(d[0], d[1], d[2], d[3]), fp8_pack4(d[4], d[5], d[6], d[7]));
  }
  for (long long i = n8 * 8 + blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL)
    q[i] = (unsigned char)fp8_pack4(fp8_div(to_f(x[i]), sc, rs), 0.f, 0.f, 0.f);
}

__global__ void fp8_scale_kernel(unsigned* amax_bits) {  // amax -> the scale s, in place
  const float amax = __uint_as_float(*amax_bits);
  reinterpret_cast<float*>(amax_bits)[0] = amax > 0.f ? amax / 448.f : 1.f;
}

__device__ __forceinline__ int fp8_slot(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// QuickGELU (models.py:391-393) as vit.hip's quickgelu_kernel computes it
__device__ __forceinline__ float f8_quickgelu(float x) { return x / (1.f + __expf(-1.702f * x)); }

// a wave's max |x| into the producer partials pmax[blockIdx & 4095] (the
// fused-amax convention of vit.hip: 4096 slots, reduced by the quantiser)
__device__ __forceinline__ void f8_amax_flush(float m, unsigned* pmax) {
  m = fp8_wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(pmax + (blockIdx.x & 4095), __float_as_uint(m));
}

template <typename T>
__global__ void __launch_bounds__(256) gemm_fp8_kernel(int M, int N, int K, const unsigned char* __restrict__ A,
                                                       const unsigned char* __restrict__ B,
                                                       const float* __restrict__ sa, const float* __restrict__ sb,
                                                       const float* __restrict__ bias, T* __restrict__ C,
                                                       int accumulate, const bf16* __restrict__ res,
                                                       bf16* __restrict__ out2, int skip_c,
                                                       unsigned* __restrict__ pmax) {
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
  float am = 0.f;
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
        if (pmax) {  // c_fc + QuickGELU: C = f, out2 = quickgelu(f), max |out2| into pmax
          const bf16 f = (bf16)v;
          *p = from_f<T>(v);
          const bf16 g = (bf16)f8_quickgelu((float)f);
          out2[(long long)m * N + n] = g;
          am = fmaxf(am, fabsf((float)g));
          continue;
        }
        if (accumulate) v += to_f(*p);
        if (res) v += (float)res[(long long)m * N + n];
        if (!skip_c) *p = from_f<T>(v);
        if (out2) out2[(long long)m * N + n] = (bf16)v;
      }
    }
  if (pmax) f8_amax_flush(am, pmax);
}

// ---------------------------------------------------------------------------
// 256 x 256 output tile per 512-thread workgroup (8 waves as 2 x 4, each
// 128 x 64 = 8 x 4 MFMA tiles), K-step 128, operands moved HBM/L2 -> LDS by
// LDS-DMA (buffer_load ... lds, no VGPR staging) into a 2-stage ring; the
// next stage is in flight while this one is consumed.  4x the arithmetic
// intensity of the 128 x 128 kernel above (its operand traffic, not the MFMA,
// bounds it).  Workgroups are numbered so that the N tiles of one A panel run
// on one XCD (the panel is read from HBM once and then from that XCD's L2).
typedef __attribute__((address_space(3))) void* f8_lds_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t f8_rsrc(const void* base, long long bytes) {
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// LDS-DMA of 16 B per lane to lds + 16 * lane (M0 saved and restored inside)
__device__ __forceinline__ void f8_glds16(__amdgpu_buffer_rsrc_t r, char* lds, unsigned voff) {
  const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)(f8_lds_t)lds);
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

__device__ __forceinline__ i32x8 f8_frag(const char* img, int row, int kq) {
  const uint4 lo = *reinterpret_cast<const uint4*>(img + fp8_slot(row, 2 * kq));
  const uint4 hi = *reinterpret_cast<const uint4*>(img + fp8_slot(row, 2 * kq + 1));
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

typedef __attribute__((ext_vector_type(4))) unsigned f8_u32x4;

// epilogue stores of the fp8 GEMM: non-temporal (not allocated in L2, which
// keeps the A panels and B slices the other column tiles re-read): the four
// projection GEMMs 3.51 -> 3.29 ms per block, C5 forward -2.3 ms per step
// (tools/gpu/r4_f8nt.sh, profiles/r4_nt_stores.txt)
#ifndef F8_NT_STORE
#define F8_NT_STORE 1
#endif
template <typename V>
__device__ __forceinline__ void f8_st(V* p, const V& v) {
  if constexpr (F8_NT_STORE) {
    typedef unsigned f8_u2 __attribute__((ext_vector_type(2)));
    typedef unsigned f8_u4 __attribute__((ext_vector_type(4)));
    if constexpr (sizeof(V) == 8) __builtin_nontemporal_store(*reinterpret_cast<const f8_u2*>(&v), reinterpret_cast<f8_u2*>(p));
    else __builtin_nontemporal_store(*reinterpret_cast<const f8_u4*>(&v), reinterpret_cast<f8_u4*>(p));
  } else {
    *p = v;
  }
}

// the epilogue of four adjacent outputs of row m (offset ro, column n):
// (+ C if accumulate) (+ res) -> C unless skip_c, and a bf16 copy to out2
template <typename T>
__device__ __forceinline__ void f8_store_row4(T* __restrict__ C, const bf16* __restrict__ res,
                                              bf16* __restrict__ out2, long long ro, int n, int N, float v[4],
                                              int accumulate, int skip_c) {
  T* p = C + ro;
  typedef __attribute__((ext_vector_type(4))) bf16 bf16x4;
  if (n + 3 < N && (N & 3) == 0) {
    if (accumulate) {
      if constexpr (sizeof(T) == 4) {
        const float4 o = *reinterpret_cast<const float4*>(p);
        v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += to_f(p[e]);
      }
    }
    if (res) {  // bf16 residual input (the block's x)
      const bf16x4 r4 = *reinterpret_cast<const bf16x4*>(res + ro);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += (float)r4[e];
    }
    if (!skip_c) {
      if constexpr (sizeof(T) == 4) {
        f8_st(reinterpret_cast<float4*>(p), make_float4(v[0], v[1], v[2], v[3]));
      } else {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
        f8_st(reinterpret_cast<bf16x4*>(p), o);
      }
    }
    if (out2) {  // a bf16 copy of the result (the next LayerNorm's input / the block output)
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
      f8_st(reinterpret_cast<bf16x4*>(out2 + ro), o);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (n + e < N) {
        float w = v[e];
        if (accumulate) w += to_f(p[e]);
        if (res) w += (float)res[ro + e];
        if (!skip_c) p[e] = from_f<T>(w);
        if (out2) out2[ro + e] = (bf16)w;
      }
  }
}

// c_fc + QuickGELU epilogue of four adjacent outputs: C = f (bf16), out2 =
// quickgelu(f) computed from the stored bf16 f (as the unfused quickgelu_kernel
// reads it), am = running max |out2|
template <typename T>
__device__ __forceinline__ void f8_gelu_row4(T* __restrict__ C, bf16* __restrict__ out2, long long ro, int n, int N,
                                             const float v[4], float& am) {
  typedef __attribute__((ext_vector_type(4))) bf16 bf16x4;
  if (sizeof(T) == 2 && n + 3 < N && (N & 3) == 0) {
    bf16x4 fo, go;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      fo[e] = (bf16)v[e];
      go[e] = (bf16)f8_quickgelu((float)fo[e]);
      am = fmaxf(am, fabsf((float)go[e]));
    }
    f8_st(reinterpret_cast<bf16x4*>(C + ro), fo);
    f8_st(reinterpret_cast<bf16x4*>(out2 + ro), go);
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (n + e >= N) continue;
    const bf16 f = (bf16)v[e];
    const bf16 g = (bf16)f8_quickgelu((float)f);
    C[ro + e] = from_f<T>((float)f);
    out2[ro + e] = g;
    am = fmaxf(am, fabsf((float)g));
  }
}

// RD: the epilogue operands read from memory.  0: none; 1: C (accumulate) or
// res, one of the two, prefetched a pass ahead into registers; 2: any
// combination, read in place.  One counter (vmcnt) tracks a wave's loads and
// stores alike, so a load issued after a store waits for that store too: RD 1
// issues pass p + 1's loads before pass p's stores, and no load waits behind
// the output traffic.
//
// BM 128 (with BN 128, tile code 2, forced only): a 128 x 128 tile of 4 waves
// (2 x 2 of 64 x 64) on a 2-stage ring of 32 KB stages, two workgroups per CU,
// so one workgroup's prologue and epilogue run beside the other's k-loop (the
// 256-row tiles are one workgroup per CU: their epilogue, 0.34 of out_proj's
// 0.58 ms, leaves the matrix pipe idle).  Slower on all four C5 shapes all the
// same (qkv 0.98 vs 0.85 ms, out_proj 0.64 vs 0.57, c_fc 1.10 vs 0.98, c_proj
// 0.91 vs 0.84; without the epilogue's traffic 2.88 vs 2.59 ms per block;
// C5 210.8 vs 205.3 ms/step, profiles/r5_fp8_tile128.txt).  Two more schedules
// of the 256 x 256 tile measured and dropped (profiles/r5_fp8_kloop.txt): 64-k
// half-stages on v_mfma_scale_f32_32x32x64 with three of four 32 KB buffers in
// flight (+4 %: the ring depth does not bound the k-loop), and the next
// stage's eight LDS-DMA pieces issued one per row tile between the MFMAs
// instead of after the barrier (-2 % standalone, C5 step unchanged)
template <typename T, int RD, int BN, int BM = 256>
__global__ void __launch_bounds__(BM == 256 ? 512 : 256, BM == 256 ? 1 : 2)
    gemm_fp8_v2_kernel(int M, int N, int K, const unsigned char* __restrict__ A,
                                                          const unsigned char* __restrict__ B,
                                                          const float* __restrict__ sa, const float* __restrict__ sb,
                                                          const float* __restrict__ bias, T* __restrict__ C,
                                                          int accumulate, const bf16* __restrict__ res,
                                                          bf16* __restrict__ out2, int skip_c,
                                                          unsigned* __restrict__ pmax) {
  // BN 256: 2 x 4 waves of 128 x 64, a 2-stage ring of 64 KB stages (one in
  // flight while the other is consumed).  BN 128: 4 x 2 waves of 64 x 64, a
  // 3-stage ring of 48 KB stages, two in flight: at ~1 us of MFMA per stage the
  // single stage in flight of the 256-wide tile leaves every k-step waiting on
  // its L2/HBM round trip
  static_assert(BM == 256 || BN == 128, "the 128-row tile is 128 wide");
  constexpr int NW = BM == 256 ? 8 : 4;             // waves
  constexpr int NST = (BN == 256 || BM == 128) ? 2 : 3;
  constexpr int MI = BN == 256 ? 8 : 4;             // 16-row MFMA tiles per wave
  constexpr int SB = BM * 128 + BN * 128;           // stage bytes: A [BM][128] | B [BN][128]
  constexpr int NPA = BM / 8 / NW;                  // A pieces (1 KB, 8 rows) per wave
  constexpr int NPB = BN / 8 / NW;                  // B pieces per wave
  constexpr int PER_STAGE = NPA + NPB;              // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NST][SB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = (N + BN - 1) / BN;
  const long long G = gridDim.x;
  long long lid = blockIdx.x;
  if (G >= 8) {  // consecutive tiles (one A panel) on one XCD
    const long long q = G / 8, r = G % 8, x = lid % 8;
    lid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + lid / 8;
  }
  const int m0 = (int)(lid / tiles_n) * BM, n0 = (int)(lid % tiles_n) * BN;
  const int wm = BN == 256 ? (wid >> 2) * 128 : (wid >> 1) * 64;
  const int wn = BN == 256 ? (wid & 3) * 64 : (wid & 1) * 64;
  const int nk = K / 128;
  const __amdgpu_buffer_rsrc_t ra = f8_rsrc(A + (long long)m0 * K, (long long)(M - m0) * K);
  const __amdgpu_buffer_rsrc_t rb = f8_rsrc(B + (long long)n0 * K, (long long)(N - n0) * K);
  // loader: wave w moves 1-KB pieces w, w + 8, ... of each operand (8 rows
  // each); lane l fills slot l & 7 of row l >> 3 with the chunk that belongs
  // there under the swizzle
  const int lrow = lane >> 3, lslot = lane & 7;
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int u = 0; u < NPA; ++u) {
      const int piece = wid + NW * u, row = piece * 8 + lrow;
      const unsigned off = (unsigned)(row * K + kt * 128 + ((lslot ^ (row & 7)) << 4));
      f8_glds16(ra, &smem[buf][piece * 1024], off);
    }
#pragma unroll
    for (int u = 0; u < NPB; ++u) {
      const int piece = wid + NW * u, row = piece * 8 + lrow;
      const unsigned off = (unsigned)(row * K + kt * 128 + ((lslot ^ (row & 7)) << 4));
      f8_glds16(rb, &smem[buf][BM * 128 + piece * 1024], off);
    }
  };
  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, kq = lane >> 4;
  issue(0, 0);
  if (NST == 3 && nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = NST == 2 ? (kt & 1) : kt % 3;
    if (NST == 3 && kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STAGE) : "memory");  // stage kt landed, kt + 1 may be in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of stage kt landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // and its reads of the stage refilled next retired
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (NST == 2) {
      if (kt + 1 < nk) issue(kt + 1, buf ^ 1);
    } else {
      if (kt + 2 < nk) issue(kt + 2, (kt + 2) % 3);  // the stage consumed at kt - 1: every wave is past it
    }
    const char* ai = &smem[buf][0];
    const char* bi = &smem[buf][BM * 128];
    i32x8 bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = f8_frag(bi, wn + 16 * j + fr, kq);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const i32x8 af = f8_frag(ai, wm + 16 * i + fr, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[j], acc[i][j], 0, 0, 0, 0x7f7f7f7f, 0,
                                                                     0x7f7f7f7f);
    }
  }
  // epilogue through LDS (the ring is free): per wave four passes of a 32 x 64
  // f32 block, then row-contiguous 16-B reads and coalesced row stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int EP = 68;  // f32 row pitch of a wave's block
  static_assert(NW * 32 * EP * 4 <= NST * SB, "epilogue blocks fit the ring");
  float* eb = reinterpret_cast<float*>(&smem[0][0]) + wid * 32 * EP;
  const float s = sa[0] * sb[0];
  const int ec = (lane & 15) * 4, er = lane >> 4;  // this lane's 4 columns, row phase
  const int n = n0 + wn + ec;
  const bool vec = n + 3 < N && (N & 3) == 0;
  float bn[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) bn[e] = (bias && n + e < N) ? bias[n + e] : 0.f;
  // RD 1: row rr of pass p's operand (C as f32x4 / bf16x4, or res as bf16x4)
  f8_u32x4 pre[2][8];
  const bool rd_c = accumulate != 0;
  auto prefetch = [&](int pass, f8_u32x4* dst) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int m = m0 + wm + 32 * pass + 4 * rr + er;
      const long long ro = (long long)m * N + n;
      dst[rr] = f8_u32x4{0u, 0u, 0u, 0u};
      if (m < M && vec) {
        if (rd_c) {
          if constexpr (sizeof(T) == 4) {
            dst[rr] = *reinterpret_cast<const f8_u32x4*>(C + ro);
          } else {
            const uint2 t = *reinterpret_cast<const uint2*>(C + ro);
            dst[rr].x = t.x; dst[rr].y = t.y;
          }
        } else {
          const uint2 t = *reinterpret_cast<const uint2*>(res + ro);
          dst[rr].x = t.x; dst[rr].y = t.y;
        }
      }
    }
  };
  float am = 0.f;
  if constexpr (RD == 1) prefetch(0, pre[0]);
#pragma unroll
  for (int pass = 0; pass < MI / 2; ++pass) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) eb[(16 * ii + 4 * kq + r) * EP + 16 * j + fr] = acc[2 * pass + ii][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if constexpr (RD == 1) {
      if (pass + 1 < MI / 2) prefetch(pass + 1, pre[(pass + 1) & 1]);
      asm volatile("" ::: "memory");  // those loads go out ahead of this pass's stores
    }
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      const int lr = 4 * rr + er;
      const int m = m0 + wm + 32 * pass + lr;
      const float4 v4 = *reinterpret_cast<const float4*>(eb + lr * EP + ec);
      float v[4] = {v4.x * s + bn[0], v4.y * s + bn[1], v4.z * s + bn[2], v4.w * s + bn[3]};
      if (m >= M) continue;
      const long long ro = (long long)m * N + n;
      if (RD == 0 && pmax) {  // c_fc + QuickGELU (T = bf16): C = f, out2 = quickgelu(f)
        f8_gelu_row4<T>(C, out2, ro, n, N, v, am);
      } else if (RD == 1 && vec) {
        const f8_u32x4 t = pre[pass & 1][rr];
        if (rd_c && sizeof(T) == 4) {
          v[0] += __uint_as_float(t.x); v[1] += __uint_as_float(t.y);
          v[2] += __uint_as_float(t.z); v[3] += __uint_as_float(t.w);
        } else {  // four bf16
          v[0] += __uint_as_float(t.x << 16); v[1] += __uint_as_float(t.x & 0xffff0000u);
          v[2] += __uint_as_float(t.y << 16); v[3] += __uint_as_float(t.y & 0xffff0000u);
        }
        f8_store_row4<T>(C, nullptr, out2, ro, n, N, v, 0, skip_c);
      } else {
        f8_store_row4<T>(C, res, out2, ro, n, N, v, accumulate, skip_c);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (RD == 0 && pmax) f8_amax_flush(am, pmax);
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_quantize_fp8(int dtype, const void* x, long long n, unsigned char* q, float* scale,
                                    void* stream) {
  if (n <= 0 || !x || !q || !scale) { set_error("quantize_fp8: bad arguments"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(scale, 0, sizeof(float), st) != hipSuccess) { set_error("quantize_fp8: memset"); return -2; }
  long long g = (n + 2047) / 2048;
  const unsigned grid = (unsigned)(g > 2048 ? 2048 : g < 1 ? 1 : g);
  unsigned* bits = reinterpret_cast<unsigned*>(scale);
  FP8_DISPATCH(dtype, hipLaunchKernelGGL(fp8_amax_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)x, n, bits));
  FP8_DISPATCH(dtype, hipLaunchKernelGGL(fp8_quant_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)x, n, bits, q));
  hipLaunchKernelGGL(fp8_scale_kernel, dim3(1), dim3(1), 0, st, bits);
  ARTSBIR_CHECK_LAUNCH("quantize_fp8");
  return 0;
}

// the quantiser of a tensor whose producer already folded max |x| into 4096
// partials (artsbir_layernorm_fwd_pmax, artsbir_quickgelu_pmax,
// artsbir_mha_fwd_lse_pmax): reduce them, then the quantisation pass only
__global__ void __launch_bounds__(1024) fp8_pmax_reduce_kernel(const unsigned* __restrict__ pmax, int n,
                                                              unsigned* __restrict__ amax_bits) {
  unsigned m = 0u;
  for (int i = threadIdx.x; i < n; i += 1024) m = max(m, pmax[i]);
  __shared__ unsigned red[16];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned b = 0u;
    for (int i = 0; i < 16; ++i) b = max(b, red[i]);
    *amax_bits = b;
  }
}

extern "C" int artsbir_quantize_fp8_pmax(int dtype, const void* x, long long n, const unsigned* pmax, int npmax,
                                         unsigned char* q, float* scale, void* stream) {
  if (n <= 0 || !x || !q || !scale || !pmax || npmax <= 0) { set_error("quantize_fp8_pmax: bad arguments"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  unsigned* bits = reinterpret_cast<unsigned*>(scale);
  hipLaunchKernelGGL(fp8_pmax_reduce_kernel, dim3(1), dim3(1024), 0, st, pmax, npmax, bits);
  long long g = (n + 2047) / 2048;
  const unsigned grid = (unsigned)(g > 2048 ? 2048 : g < 1 ? 1 : g);
  FP8_DISPATCH(dtype, hipLaunchKernelGGL(fp8_quant_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)x, n, bits, q));
  hipLaunchKernelGGL(fp8_scale_kernel, dim3(1), dim3(1), 0, st, bits);
  ARTSBIR_CHECK_LAUNCH("quantize_fp8_pmax");
  return 0;
}

extern "C" int artsbir_gemm_nt_fp8_ex(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                                      const float* sa, const float* sb, const float* bias, void* c, int out_dtype,
                                      int accumulate, const void* res, void* out2, int skip_c, void* stream);

// the LDS-DMA kernel's tile width: 256 (2-stage ring).  ARTSBIR_FP8_BN=128
// selects the 256 x 128 tile with a 3-stage ring (two stages in flight): it
// measured slower on every C5 shape (qkv 1.09 vs 0.93 ms, c_fc 1.29 vs 1.13,
// out_proj 0.62 vs 0.58, c_proj 0.94 vs 0.83 ms; profiles/r3_fp8_tile_ab.txt):
// the doubled A re-reads and LDS bytes per MAC cost more than the deeper ring
// saves, so the wait per k-step is not what bounds the 256-wide tile.  Nor is
// the ring depth (round 4): pp256.hip's ping-pong schedule rebuilt for fp8
// (32x32x64 block-scaled MFMAs on 64-k LDS rows, four buffers, three K-tiles
// in flight, epilogue from the registers by buffer stores) ran 12-29 % slower
// on all four shapes (qkv 1.06 vs 0.93, out_proj 0.76 vs 0.59, c_fc 1.34 vs
// 1.14, c_proj 0.96 vs 0.83 ms; profiles/r4_fp8_attn.txt) and was dropped
//
// tile codes: 0 the 256 x 256 tile, 1 256 x 128 (ARTSBIR_FP8_BN=128), 2 the
// 128 x 128 tile at two workgroups per CU; ARTSBIR_FP8_TILE forces one
static int fp8_tile(int M, int N, int K) {
  static const int forced = [] {
    const char* e = getenv("ARTSBIR_FP8_TILE");
    if (e) return atoi(e);
    const char* b = getenv("ARTSBIR_FP8_BN");
    return b && atoi(b) == 128 ? 1 : -1;
  }();
  (void)M; (void)N; (void)K;
  return forced >= 0 && forced <= 2 ? forced : 0;
}
template <typename T, int RD>
static void fp8_v2_launch(int tile, int M, int N, int K, const unsigned char* a, const unsigned char* b,
                          const float* sa, const float* sb, const float* bias, T* c, int accumulate, const bf16* res,
                          bf16* out2, int skip_c, unsigned* pmax, hipStream_t st) {
  if (tile == 2) {
    const unsigned g = (unsigned)((long long)((M + 127) / 128) * ((N + 127) / 128));
    hipLaunchKernelGGL((gemm_fp8_v2_kernel<T, RD, 128, 128>), dim3(g), dim3(256), 0, st, M, N, K, a, b, sa, sb, bias,
                       c, accumulate, res, out2, skip_c, pmax);
  } else if (tile == 1) {
    const unsigned g = (unsigned)((long long)((M + 255) / 256) * ((N + 127) / 128));
    hipLaunchKernelGGL((gemm_fp8_v2_kernel<T, RD, 128>), dim3(g), dim3(512), 0, st, M, N, K, a, b, sa, sb, bias, c,
                       accumulate, res, out2, skip_c, pmax);
  } else {
    const unsigned g = (unsigned)((long long)((M + 255) / 256) * ((N + 255) / 256));
    hipLaunchKernelGGL((gemm_fp8_v2_kernel<T, RD, 256>), dim3(g), dim3(512), 0, st, M, N, K, a, b, sa, sb, bias, c,
                       accumulate, res, out2, skip_c, pmax);
  }
}

extern "C" int artsbir_gemm_nt_fp8(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                                   const float* sa, const float* sb, const float* bias, void* c, int out_dtype,
                                   int accumulate, void* stream) {
  return artsbir_gemm_nt_fp8_ex(M, N, K, a, b, sa, sb, bias, c, out_dtype, accumulate, nullptr, nullptr, 0, stream);
}

// the same with a fused residual input (bf16 res[M][N] added), a second bf16
// output out2 (a rounded copy of the result) and skip_c (C only read, for
// accumulate, not written): the block's residual adds and casts of
// models.py:412-417 in the projection epilogues
extern "C" int artsbir_gemm_nt_fp8_ex(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                                      const float* sa, const float* sb, const float* bias, void* c, int out_dtype,
                                      int accumulate, const void* res, void* out2, int skip_c, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 != 0 || K <= 0) { set_error("gemm_nt_fp8: K=%d must be a positive multiple of 128", K); return -1; }
  if (!a || !b || !sa || !sb || (!c && (!skip_c || accumulate))) { set_error("gemm_nt_fp8: bad arguments"); return -1; }
  if (skip_c && !out2) { set_error("gemm_nt_fp8: skip_c without a second output"); return -1; }
  const long long tiles = (long long)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles > 0x7fffffffLL) { set_error("gemm_nt_fp8: too many tiles"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  const char* old = getenv("ARTSBIR_FP8_V1");
  if (M >= 256 && N >= 256 && !(old && atoi(old))) {  // the LDS-DMA kernel
    if ((long long)M * K > 0x7fffffffLL || (long long)N * K > 0x7fffffffLL) {
      set_error("gemm_nt_fp8: operand larger than 2 GiB");
      return -1;
    }
    static const int nostore = [] { const char* e = getenv("ARTSBIR_FP8_NOSTORE"); return e ? atoi(e) : 0; }();
    if (nostore) {  // timing experiment only: the main loop without the epilogue's memory traffic
      accumulate = 0; res = nullptr; out2 = nullptr; skip_c = 1;
    }
    const int nrd = (accumulate ? 1 : 0) + (res ? 1 : 0);
    const int tile = fp8_tile(M, N, K);
    set_last_kernel(tile == 2 ? "gemm_fp8_v2_kernel<128x128>" : "gemm_fp8_v2_kernel");
    if (nrd == 0)
      FP8_DISPATCH(out_dtype, fp8_v2_launch<T, 0>(tile, M, N, K, a, b, sa, sb, bias, (T*)c, accumulate,
                                                  (const bf16*)res, (bf16*)out2, skip_c, nullptr, st));
    else if (nrd == 1)
      FP8_DISPATCH(out_dtype, fp8_v2_launch<T, 1>(tile, M, N, K, a, b, sa, sb, bias, (T*)c, accumulate,
                                                  (const bf16*)res, (bf16*)out2, skip_c, nullptr, st));
    else
      FP8_DISPATCH(out_dtype, fp8_v2_launch<T, 2>(tile, M, N, K, a, b, sa, sb, bias, (T*)c, accumulate,
                                                  (const bf16*)res, (bf16*)out2, skip_c, nullptr, st));
  } else {
    set_last_kernel("gemm_fp8_kernel");
    FP8_DISPATCH(out_dtype, hipLaunchKernelGGL(gemm_fp8_kernel<T>, dim3((unsigned)tiles), dim3(256), 0, st, M, N, K,
                                             a, b, sa, sb, bias, (T*)c, accumulate, (const bf16*)res, (bf16*)out2,
                                             skip_c, nullptr));
  }
  ARTSBIR_CHECK_LAUNCH("gemm_nt_fp8");
  return 0;
}

// c_fc + QuickGELU of the ViT MLP (models.py:391-393, 412-417) in one fp8 GEMM:
// c = f = A B^T + bias (bf16, kept for the backward), out2 = quickgelu(f) (bf16,
// the c_proj input) and max |out2| folded into pmax[4096] for its quantiser
// (artsbir_quantize_fp8_pmax) — no separate activation pass over f
extern "C" int artsbir_gemm_nt_fp8_gelu(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                                        const float* sa, const float* sb, const float* bias, void* c, void* out2,
                                        unsigned* pmax, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K % 128 != 0 || K <= 0) { set_error("gemm_nt_fp8_gelu: K=%d must be a positive multiple of 128", K); return -1; }
  if (!a || !b || !sa || !sb || !c || !out2 || !pmax) { set_error("gemm_nt_fp8_gelu: bad arguments"); return -1; }
  const long long tiles = (long long)((M + 127) / 128) * ((N + 127) / 128);
  if (tiles > 0x7fffffffLL) { set_error("gemm_nt_fp8_gelu: too many tiles"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  if (M >= 256 && N >= 256) {
    if ((long long)M * K > 0x7fffffffLL || (long long)N * K > 0x7fffffffLL) {
      set_error("gemm_nt_fp8_gelu: operand larger than 2 GiB");
      return -1;
    }
    const int tile = fp8_tile(M, N, K);
    set_last_kernel(tile == 2 ? "gemm_fp8_v2_kernel<128x128>" : "gemm_fp8_v2_kernel");
    fp8_v2_launch<bf16, 0>(tile, M, N, K, a, b, sa, sb, bias, (bf16*)c, 0, nullptr, (bf16*)out2, 0, pmax, st);
  } else {
    set_last_kernel("gemm_fp8_kernel");
    hipLaunchKernelGGL(gemm_fp8_kernel<bf16>, dim3((unsigned)tiles), dim3(256), 0, st, M, N, K, a, b, sa, sb, bias,
                       (bf16*)c, 0, (const bf16*)nullptr, (bf16*)out2, 0, pmax);
  }
  ARTSBIR_CHECK_LAUNCH("gemm_nt_fp8_gelu");
  return 0;
}
