// The BatchNorm backward folded through the 1x1 convolution in front of it
// (gfx950).  Reference chain: models.py:219-220 (Bottleneck conv3 -> bn3) and
// models.py:227-229 (downsample AvgPool -> conv -> BN), differentiated by
// autograd through BatchNorm2d (train) and Conv2d.
//
// In training mode the BN backward maps the masked output gradient g to
//   dy = c1 (g - c2 - xhat c3),   xhat = (y - mean) istd
// (artsbir_bn_bwd_finalize: c1 = gamma istd, c2 = mean g, c3 = mean g xhat), and
// the conv then needs dx = dy W and dW = dy^T x.  With y = x W^T both are linear
// in (g, x), per BN segment s:
//   dx = g (diag(c1) W) + x (W^T diag(b') W) + e,          b' = -c1 c3 istd
//   e  = k W,                                                k = -c1 (c2 - c3 istd mean)
//   dW = diag(c1) g^T x + diag(b') W (x^T x) + k (1^T x)
// so dy never exists: the data gradient is one GEMM over [g | x]
// (artsbir_conv1x1_dgrad_fold, gemm.hip) with the weights this file prepares,
// and the weight gradient is g^T x, the Gram matrix x^T x and the column sums of
// x per segment, combined here.  That removes the BN-backward apply pass (read
// g, y; write dy) and the data gradient's read of dy from the HBM-bound main
// stream of the step.
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

// one row ci of segment s: B1[s][ci][co] = c1 W^T[ci][co], A[s][ci][co] = b' W^T[ci][co]
// (the left operand of the Gram-side GEMM), bias[s][ci] = sum_co W^T[ci][co] k[co]
template <typename T>
__global__ void __launch_bounds__(256) fold_prep_kernel(const T* __restrict__ wt, int Co, int Ci,
                                                        const float* __restrict__ coef, const float* __restrict__ prm,
                                                        long long pstride, T* __restrict__ wout, T* __restrict__ amat,
                                                        float* __restrict__ bias) {
  const int ci = blockIdx.x, s = blockIdx.y;
  const float* c1 = coef + (long long)s * 3 * Co;
  const float* c2 = c1 + Co;
  const float* c3 = c2 + Co;
  const float* mean = prm + s * pstride;
  const float* istd = mean + Co;
  const T* wr = wt + (long long)ci * Co;
  T* bo = wout + ((long long)s * Ci + ci) * (Co + Ci);
  T* ao = amat + ((long long)s * Ci + ci) * Co;
  float acc = 0.f;
  for (int c = threadIdx.x; c < Co; c += 256) {
    const float w = to_f(wr[c]);
    const float a1 = c1[c], is = istd[c];
    const float bp = -a1 * c3[c] * is;
    const float k = -a1 * (c2[c] - c3[c] * is * mean[c]);
    bo[c] = from_f<T>(a1 * w);
    ao[c] = from_f<T>(bp * w);
    acc += w * k;
  }
  __shared__ float red[4];
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) bias[(long long)s * Ci + ci] = (red[0] + red[1]) + (red[2] + red[3]);
}

// The y-side fold (artsbir_bn_fold_bwd_prep_y): the BatchNorm right after the
// conv is folded with its own input y (the conv output, kept for the BN backward)
// instead of the conv input x — dy = c1 g + b' y + k, so
//   dx = g (diag(c1) W) + y (diag(b') W) + k W
// needs no Gram-side GEMM: row ci of segment s is wout[s][ci][co] = c1 W^T[ci][co],
// wout[s][ci][Co + co] = b' W^T[ci][co], bias[s][ci] = sum_co W^T[ci][co] k[co]
template <typename T>
__global__ void __launch_bounds__(256) fold_prep_y_kernel(const T* __restrict__ wt, int Co, int Ci,
                                                          const float* __restrict__ coef, const float* __restrict__ prm,
                                                          long long pstride, T* __restrict__ wout,
                                                          float* __restrict__ bias) {
  const int ci = blockIdx.x, s = blockIdx.y;
  const float* c1 = coef + (long long)s * 3 * Co;
  const float* c2 = c1 + Co;
  const float* c3 = c2 + Co;
  const float* mean = prm + s * pstride;
  const float* istd = mean + Co;
  const T* wr = wt + (long long)ci * Co;
  T* bo = wout + ((long long)s * Ci + ci) * (2 * Co);
  float acc = 0.f;
  for (int c = threadIdx.x; c < Co; c += 256) {
    const float w = to_f(wr[c]);
    const float a1 = c1[c], is = istd[c];
    const float bp = -a1 * c3[c] * is;
    const float k = -a1 * (c2[c] - c3[c] * is * mean[c]);
    bo[c] = from_f<T>(a1 * w);
    bo[Co + c] = from_f<T>(bp * w);
    acc += w * k;
  }
  __shared__ float red[4];
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) bias[(long long)s * Ci + ci] = (red[0] + red[1]) + (red[2] + red[3]);
}

// dW[co][ci] += sum_s c1_s[co] P_s[co][ci] + b'_s[co] T[co][s Ci + ci] + k_s[co] cs_s[ci]
// with T = W [Gram_0 | Gram_1 | ...] (an f32 GEMM before it) — or, for the y-side
// fold, T_s = y_s^T x_s straight from artsbir_gemm_tn2 (t_co / t_s: the strides of
// T's rows and segments): elementwise, 4 values of one dW row per thread
__global__ void __launch_bounds__(256) fold_wgrad_combine_kernel(const float* __restrict__ P,
                                                                 const float* __restrict__ T, long long t_co,
                                                                 long long t_s, const float* __restrict__ cs,
                                                                 int cs_slots, int Co, int Ci, int nseg,
                                                                 const float* __restrict__ coef,
                                                                 const float* __restrict__ prm, long long pstride,
                                                                 float* __restrict__ dw) {
  const int cq = Ci / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)Co * cq) return;
  const int co = (int)(i / cq), ci = (int)(i - (long long)co * cq) * 4;
  float4 acc = *reinterpret_cast<const float4*>(dw + (long long)co * Ci + ci);
  for (int s = 0; s < nseg; ++s) {
    const float* c = coef + (long long)s * 3 * Co;
    const float* mp = prm + s * pstride;
    const float c1 = c[co], c2 = c[Co + co], c3 = c[2 * Co + co], mean = mp[co], istd = mp[Co + co];
    const float bp = -c1 * c3 * istd, k = -c1 * (c2 - c3 * istd * mean);
    const float4 p = *reinterpret_cast<const float4*>(P + ((long long)s * Co + co) * Ci + ci);
    const float4 t = *reinterpret_cast<const float4*>(T + co * t_co + s * t_s + ci);
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);  // the column sums' replica rows of segment s
    for (int r = 0; r < cs_slots; ++r) {
      const float4 v = *reinterpret_cast<const float4*>(cs + ((long long)s * cs_slots + r) * Ci + ci);
      q.x += v.x; q.y += v.y; q.z += v.z; q.w += v.w;
    }
    acc.x += c1 * p.x + bp * t.x + k * q.x;
    acc.y += c1 * p.y + bp * t.y + k * q.y;
    acc.z += c1 * p.z + bp * t.z + k * q.z;
    acc.w += c1 * p.w + bp * t.w + k * q.w;
  }
  *reinterpret_cast<float4*>(dw + (long long)co * Ci + ci) = acc;
}

// C[m][n] (ldc) = sum_k A[m][k] B[n][k] for the two small GEMMs of the fold
// (the x-side weights W^T diag(b') W; T = W Gram in the weight gradient), with a
// footprint that lets it share a CU with the other stream's GEMM workgroups: a
// 64 x 64 tile per 4-wave workgroup, 32-k LDS stages double-buffered in 16 KB
// (24 KB with an f32 B) — the 128-160 KB tiles of the pipelined kernels wait for
// a CU the weight gradients have left, which cost these ~20-50 us GEMMs ~150 us
// each in the step.  A bf16 [M][K]; B bf16, or f32 split into two bf16 parts
// (hi + lo, so the f32 Gram matrices keep ~16 significant bits) [N][K]; f32
// accumulation on v_mfma_f32_16x16x32_bf16; output bf16 or f32.  M, N % 64 == 0,
// K % 32 == 0.
__device__ __forceinline__ int fg_slot(int row, int chunk) { return chunk ^ ((row >> 2) & 2); }

template <bool BF32, bool OF32>
__global__ void __launch_bounds__(256) fold_gemm_kernel(const bf16* __restrict__ A, long long lda,
                                                        const void* __restrict__ Bv, long long ldb, void* C,
                                                        long long ldc, int M, int N, int K) {
  constexpr int NB = BF32 ? 2 : 1;  // B parts (hi, lo)
  __shared__ __attribute__((aligned(16))) char smem[2][(1 + NB) * 64 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntn = N / 64;
  const int m0 = (blockIdx.x / ntn) * 64, n0 = (blockIdx.x % ntn) * 64;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  const int lr = tid >> 2, lc = tid & 3;  // loader: row, 16-B chunk of a 64-B row
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 ra, rb[NB];
  auto load = [&](int k0) {
    ra = *reinterpret_cast<const uint4*>(A + (long long)(m0 + lr) * lda + k0 + lc * 8);
    if constexpr (BF32) {
      const float* bp = reinterpret_cast<const float*>(Bv) + (long long)(n0 + lr) * ldb + k0 + lc * 8;
      const float4 f0 = *reinterpret_cast<const float4*>(bp), f1 = *reinterpret_cast<const float4*>(bp + 4);
      const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      bf16 hi[8], lo[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        hi[e] = (bf16)f[e];
        lo[e] = (bf16)(f[e] - (float)hi[e]);
      }
      rb[0] = *reinterpret_cast<const uint4*>(hi);
      rb[NB - 1] = *reinterpret_cast<const uint4*>(lo);
    } else {
      rb[0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(Bv) + (long long)(n0 + lr) * ldb + k0 + lc * 8);
    }
  };
  auto store = [&](int buf) {
    char* s = smem[buf];
    const int o = lr * 64 + (fg_slot(lr, lc) << 4);
    *reinterpret_cast<uint4*>(s + o) = ra;
#pragma unroll
    for (int p = 0; p < NB; ++p) *reinterpret_cast<uint4*>(s + (1 + p) * 4096 + o) = rb[p];
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = K / 32;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * 32);
    const char* s = smem[cur];
    uint4 af[2], bfr[NB][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm + 16 * i + fr;
      af[i] = *reinterpret_cast<const uint4*>(s + r * 64 + (fg_slot(r, fq) << 4));
    }
#pragma unroll
    for (int p = 0; p < NB; ++p)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn + 16 * j + fr;
        bfr[p][j] = *reinterpret_cast<const uint4*>(s + (1 + p) * 4096 + r * 64 + (fg_slot(r, fq) << 4));
      }
#pragma unroll
    for (int p = 0; p < NB; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&bfr[p][j]),
                                                              *reinterpret_cast<const bf16x8*>(&af[i]), acc[i][j], 0,
                                                              0, 0);
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }
  // acc[i][j][r]: row m = m0 + wm + 16 i + fr, column n = n0 + wn + 16 j + 4 fq + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long long m = m0 + wm + 16 * i + fr;
      const int n = n0 + wn + 16 * j + 4 * fq;
      if constexpr (OF32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + m * ldc + n) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      } else {
        bf16 o[4] = {(bf16)acc[i][j][0], (bf16)acc[i][j][1], (bf16)acc[i][j][2], (bf16)acc[i][j][3]};
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(C) + m * ldc + n) = *reinterpret_cast<const uint2*>(o);
      }
    }
}

}  // namespace artsbir

using namespace artsbir;

// the fold's small GEMMs on fold_gemm_kernel where the shape allows, else artsbir_gemm_nt
static int fold_gemm(int dtype, bool b_f32, int M, int N, int K, const void* a, long long lda, const void* b,
                     long long ldb, void* c, long long ldc, bool out_f32, hipStream_t st) {
  const bool ok = dtype == ARTSBIR_DT_BF16 && M % 64 == 0 && N % 64 == 0 && K % 32 == 0 && lda % 8 == 0 &&
                  ldb % 8 == 0 && ldc % 4 == 0 && (long long)(M / 64) * (N / 64) < 0x7fffffffLL;
  if (!ok) {
    if (b_f32 && dtype == ARTSBIR_DT_BF16) { set_error("fold_gemm: f32 B needs 64-multiple shapes"); return -1; }
    return artsbir_gemm_nt(dtype, M, N, K, a, lda, b, c, ldc, out_f32 ? 1 : 0, 0, nullptr, nullptr, st);
  }
  const dim3 g((unsigned)((M / 64) * (N / 64)));
  const bf16* A = reinterpret_cast<const bf16*>(a);
  if (b_f32 && out_f32) hipLaunchKernelGGL((fold_gemm_kernel<true, true>), g, dim3(256), 0, st, A, lda, b, ldb, c, ldc, M, N, K);
  else if (b_f32) hipLaunchKernelGGL((fold_gemm_kernel<true, false>), g, dim3(256), 0, st, A, lda, b, ldb, c, ldc, M, N, K);
  else if (out_f32) hipLaunchKernelGGL((fold_gemm_kernel<false, true>), g, dim3(256), 0, st, A, lda, b, ldb, c, ldc, M, N, K);
  else hipLaunchKernelGGL((fold_gemm_kernel<false, false>), g, dim3(256), 0, st, A, lda, b, ldb, c, ldc, M, N, K);
  ARTSBIR_CHECK_LAUNCH("fold_gemm");
  return 0;
}

extern "C" int artsbir_bn_fold_bwd_prep(int dtype, int Co, int Ci, const void* wt, const float* coef,
                                        const float* prm, long long pstride, int nseg, void* wout, float* bias,
                                        void* amat, void* stream) {
  if (Co <= 0 || Ci <= 0 || Co % 8 || Ci % 8 || nseg < 1) {
    set_error("bn_fold_bwd_prep: bad shape Co=%d Ci=%d nseg=%d", Co, Ci, nseg);
    return -1;
  }
  if (!wt || !coef || !prm || !wout || !bias || !amat) { set_error("bn_fold_bwd_prep: null operand"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)Ci, (unsigned)nseg);
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(fold_prep_kernel<bf16>, g, dim3(256), 0, st, reinterpret_cast<const bf16*>(wt), Co, Ci, coef, prm,
                       pstride, reinterpret_cast<bf16*>(wout), reinterpret_cast<bf16*>(amat), bias);
  else
    hipLaunchKernelGGL(fold_prep_kernel<float>, g, dim3(256), 0, st, reinterpret_cast<const float*>(wt), Co, Ci, coef,
                       prm, pstride, reinterpret_cast<float*>(wout), reinterpret_cast<float*>(amat), bias);
  ARTSBIR_CHECK_LAUNCH("fold_prep");
  // the x-side weights W^T diag(b') W of every segment in one GEMM: rows s*Ci + ci
  // of A times W^T (as [N = Ci][K = Co]) into columns Co.. of wout's rows
  const size_t es = dtype == ARTSBIR_DT_BF16 ? 2 : 4;
  return fold_gemm(dtype, false, nseg * Ci, Ci, Co, amat, Co, wt, Co, reinterpret_cast<char*>(wout) + Co * es, Co + Ci,
                   false, st);
}

extern "C" int artsbir_bn_fold_wgrad_combine(int dtype, int Co, int Ci, int nseg, const float* P, const float* gram,
                                             const float* colsums, int cs_slots, const void* w, const float* coef,
                                             const float* prm, long long pstride, float* dw, float* workspace,
                                             void* stream) {
  if (Co <= 0 || Ci <= 0 || Co % 8 || Ci % 8 || nseg < 1) { set_error("bn_fold_wgrad_combine: bad shape"); return -1; }
  if (!P || !gram || !colsums || !w || !coef || !prm || !dw || !workspace) {
    set_error("bn_fold_wgrad_combine: null operand");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  // T = W [Gram_0 | ... ] (the Gram matrices are [nseg * Ci][Ci] rows, symmetric):
  // bf16 W against the f32 Gram split into two bf16 parts, f32 out; in the f32
  // mode an f32 GEMM
  float* T = workspace;
  if (dtype == ARTSBIR_DT_BF16 && (Co % 64 || Ci % 64)) {
    // shapes off the 64-tile (small test models): W in f32, one f32 GEMM
    float* wc = workspace;
    T = workspace + (long long)Co * Ci;
    if (artsbir_cast(ARTSBIR_DT_BF16, w, ARTSBIR_DT_F32, wc, (long long)Co * Ci, stream)) return -1;
    if (artsbir_gemm_nt(ARTSBIR_DT_F32, Co, nseg * Ci, Ci, wc, Ci, gram, T, (long long)nseg * Ci, 1, 0, nullptr,
                        nullptr, stream))
      return -1;
  } else if (fold_gemm(dtype, true, Co, nseg * Ci, Ci, w, Ci, gram, Ci, T, (long long)nseg * Ci, true, st)) {
    return -1;
  }
  const long long n = (long long)Co * (Ci / 4);
  hipLaunchKernelGGL(fold_wgrad_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, T,
                     (long long)nseg * Ci, (long long)Ci, colsums, cs_slots < 1 ? 1 : cs_slots, Co, Ci, nseg, coef, prm,
                     pstride, dw);
  ARTSBIR_CHECK_LAUNCH("fold_wgrad_combine");
  return 0;
}

extern "C" int artsbir_bn_fold_bwd_prep_y(int dtype, int Co, int Ci, const void* wt, const float* coef,
                                          const float* prm, long long pstride, int nseg, void* wout, float* bias,
                                          void* stream) {
  if (Co <= 0 || Ci <= 0 || Co % 8 || Ci % 8 || nseg < 1) {
    set_error("bn_fold_bwd_prep_y: bad shape Co=%d Ci=%d nseg=%d", Co, Ci, nseg);
    return -1;
  }
  if (!wt || !coef || !prm || !wout || !bias) { set_error("bn_fold_bwd_prep_y: null operand"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)Ci, (unsigned)nseg);
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(fold_prep_y_kernel<bf16>, g, dim3(256), 0, st, reinterpret_cast<const bf16*>(wt), Co, Ci, coef,
                       prm, pstride, reinterpret_cast<bf16*>(wout), bias);
  else
    hipLaunchKernelGGL(fold_prep_y_kernel<float>, g, dim3(256), 0, st, reinterpret_cast<const float*>(wt), Co, Ci,
                       coef, prm, pstride, reinterpret_cast<float*>(wout), bias);
  ARTSBIR_CHECK_LAUNCH("fold_prep_y");
  return 0;
}

extern "C" int artsbir_bn_fold_wgrad_combine_y(int Co, int Ci, int nseg, const float* P, const float* Q,
                                               const float* colsums, int cs_slots, const float* coef,
                                               const float* prm, long long pstride, float* dw, void* stream) {
  if (Co <= 0 || Ci <= 0 || Co % 8 || Ci % 8 || nseg < 1) { set_error("bn_fold_wgrad_combine_y: bad shape"); return -1; }
  if (!P || !Q || !colsums || !coef || !prm || !dw) { set_error("bn_fold_wgrad_combine_y: null operand"); return -1; }
  const long long n = (long long)Co * (Ci / 4);
  hipLaunchKernelGGL(fold_wgrad_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     P, Q, (long long)Ci, (long long)Co * Ci, colsums, cs_slots < 1 ? 1 : cs_slots, Co, Ci, nseg, coef,
                     prm, pstride, dw);
  ARTSBIR_CHECK_LAUNCH("fold_wgrad_combine_y");
  return 0;
}
