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

// dW[co][ci] += sum_s c1_s[co] P_s[co][ci] + b'_s[co] (W Gram_s)[co][ci] + k_s[co] cs_s[ci]
// one 64 x 64 tile of dW per workgroup, 4 x 4 values per thread; the W Gram_s
// product in f32 through LDS (32-k slices of diag(b'_s) W and of Gram_s)
template <typename T>
__global__ void __launch_bounds__(256) fold_wgrad_combine_kernel(const float* __restrict__ P,
                                                                 const float* __restrict__ gram,
                                                                 const float* __restrict__ cs,
                                                                 const T* __restrict__ w, int Co, int Ci, int nseg,
                                                                 const float* __restrict__ coef,
                                                                 const float* __restrict__ prm, long long pstride,
                                                                 float* __restrict__ dw) {
  __shared__ float ws[64][33];
  __shared__ __attribute__((aligned(16))) float gs[32][64];
  const int co0 = blockIdx.y * 64, ci0 = blockIdx.x * 64;
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int s = 0; s < nseg; ++s) {
    const float* c1 = coef + (long long)s * 3 * Co;
    const float* c2 = c1 + Co;
    const float* c3 = c2 + Co;
    const float* mean = prm + s * pstride;
    const float* istd = mean + Co;
    const float* gm = gram + (long long)s * Ci * Ci;
    for (int k0 = 0; k0 < Ci; k0 += 32) {
      for (int i = tid; i < 64 * 32; i += 256) {
        const int r = i >> 5, kk = i & 31;
        const int co = co0 + r, k = k0 + kk;
        float v = 0.f;
        if (co < Co && k < Ci) v = -c1[co] * c3[co] * istd[co] * to_f(w[(long long)co * Ci + k]);
        ws[r][kk] = v;
      }
      for (int i = tid; i < 32 * 64; i += 256) {
        const int kk = i >> 6, c = i & 63;
        const int k = k0 + kk, ci = ci0 + c;
        gs[kk][c] = (k < Ci && ci < Ci) ? gm[(long long)k * Ci + ci] : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int kk = 0; kk < 32; ++kk) {
        const float4 g4 = *reinterpret_cast<const float4*>(&gs[kk][tx * 4]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float a = ws[ty * 4 + i][kk];
          acc[i][0] += a * g4.x;
          acc[i][1] += a * g4.y;
          acc[i][2] += a * g4.z;
          acc[i][3] += a * g4.w;
        }
      }
      __syncthreads();
    }
    const float* ps = P + (long long)s * Co * Ci;
    const float* css = cs + (long long)s * Ci;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + ty * 4 + i;
      if (co >= Co) continue;
      const float a1 = c1[co];
      const float k = -a1 * (c2[co] - c3[co] * istd[co] * mean[co]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = ci0 + tx * 4 + j;
        if (ci < Ci) acc[i][j] += a1 * ps[(long long)co * Ci + ci] + k * css[ci];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + ty * 4 + i;
    if (co >= Co) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ci = ci0 + tx * 4 + j;
      if (ci < Ci) dw[(long long)co * Ci + ci] += acc[i][j];
    }
  }
}

}  // namespace artsbir

using namespace artsbir;

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
  return artsbir_gemm_nt(dtype, (long long)nseg * Ci, Ci, Co, amat, Co, wt,
                         reinterpret_cast<char*>(wout) + Co * es, Co + Ci, 0, 0, nullptr, nullptr, stream);
}

extern "C" int artsbir_bn_fold_wgrad_combine(int dtype, int Co, int Ci, int nseg, const float* P, const float* gram,
                                             const float* colsums, const void* w, const float* coef,
                                             const float* prm, long long pstride, float* dw, void* stream) {
  if (Co <= 0 || Ci <= 0 || nseg < 1) { set_error("bn_fold_wgrad_combine: bad shape"); return -1; }
  if (!P || !gram || !colsums || !w || !coef || !prm || !dw) {
    set_error("bn_fold_wgrad_combine: null operand");
    return -1;
  }
  const dim3 g((unsigned)((Ci + 63) / 64), (unsigned)((Co + 63) / 64));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL(fold_wgrad_combine_kernel<bf16>, g, dim3(256), 0, st, P, gram, colsums,
                       reinterpret_cast<const bf16*>(w), Co, Ci, nseg, coef, prm, pstride, dw);
  else
    hipLaunchKernelGGL(fold_wgrad_combine_kernel<float>, g, dim3(256), 0, st, P, gram, colsums,
                       reinterpret_cast<const float*>(w), Co, Ci, nseg, coef, prm, pstride, dw);
  ARTSBIR_CHECK_LAUNCH("fold_wgrad_combine");
  return 0;
}
