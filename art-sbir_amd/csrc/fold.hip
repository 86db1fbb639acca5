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

// dW[co][ci] += sum_s c1_s[co] P_s[co][ci] + b'_s[co] T[co][s Ci + ci] + k_s[co] cs_s[ci]
// with T = W [Gram_0 | Gram_1 | ...] (an f32 GEMM before it): elementwise, 4
// values of one dW row per thread
__global__ void __launch_bounds__(256) fold_wgrad_combine_kernel(const float* __restrict__ P,
                                                                 const float* __restrict__ T,
                                                                 const float* __restrict__ cs, int Co, int Ci,
                                                                 int nseg, const float* __restrict__ coef,
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
    const float4 t = *reinterpret_cast<const float4*>(T + (long long)co * nseg * Ci + (long long)s * Ci + ci);
    const float4 q = *reinterpret_cast<const float4*>(cs + (long long)s * Ci + ci);
    acc.x += c1 * p.x + bp * t.x + k * q.x;
    acc.y += c1 * p.y + bp * t.y + k * q.y;
    acc.z += c1 * p.z + bp * t.z + k * q.z;
    acc.w += c1 * p.w + bp * t.w + k * q.w;
  }
  *reinterpret_cast<float4*>(dw + (long long)co * Ci + ci) = acc;
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
                                             const float* prm, long long pstride, float* dw, float* workspace,
                                             void* stream) {
  if (Co <= 0 || Ci <= 0 || Co % 8 || Ci % 8 || nseg < 1) { set_error("bn_fold_wgrad_combine: bad shape"); return -1; }
  if (!P || !gram || !colsums || !w || !coef || !prm || !dw || !workspace) {
    set_error("bn_fold_wgrad_combine: null operand");
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  // T = W [Gram_0 | ... ] in f32 (the Gram matrices are [nseg * Ci][Ci] rows, symmetric)
  const float* wf = reinterpret_cast<const float*>(w);
  float* T = workspace;
  if (dtype == ARTSBIR_DT_BF16) {
    float* wc = workspace;
    T = workspace + (long long)Co * Ci;
    if (artsbir_cast(ARTSBIR_DT_BF16, w, ARTSBIR_DT_F32, wc, (long long)Co * Ci, stream)) return -1;
    wf = wc;
  }
  if (artsbir_gemm_nt(ARTSBIR_DT_F32, Co, nseg * Ci, Ci, wf, Ci, gram, T, (long long)nseg * Ci, 1, 0, nullptr, nullptr,
                      stream))
    return -1;
  const long long n = (long long)Co * (Ci / 4);
  hipLaunchKernelGGL(fold_wgrad_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P, T, colsums, Co,
                     Ci, nseg, coef, prm, pstride, dw);
  ARTSBIR_CHECK_LAUNCH("fold_wgrad_combine");
  return 0;
}
