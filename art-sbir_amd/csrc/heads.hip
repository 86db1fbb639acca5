// Classification heads and distance losses around the embedding.
//
//   ModifiedResNet_with_classification.classifier{,2}  models.py:370-378 (nn.Linear)
//   nn.CrossEntropyLoss (mean, ignore_index)            utils.py:57,70
//   CosineLoss: 1 - CosineSimilarity(dim=1, eps=1e-8)   utils.py:31-40
//   TripletMarginWithDistanceLoss(cosine_distance)      train.py:175, utils.py:56,69
// These are tiny ([B, D<=2048] x [C<=256]); simple f32 kernels, one wave per row.
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

// y[b][c] = x[b] . W[c] + bias[c]
__global__ void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                                  int B, int D, int C, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long long n = (long long)B * C;
  for (long long i = blockIdx.x * (long long)(blockDim.x / 64) + (threadIdx.x >> 6); i < n;
       i += (long long)gridDim.x * (blockDim.x / 64)) {
    const int b = (int)(i / C), c = (int)(i % C);
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += x[(long long)b * D + d] * W[(long long)c * D + d];
    s = warp_sum(s);
    if (lane == 0) y[i] = s + (bias ? bias[c] : 0.f);
  }
}

// dx[b][d] = sum_c dy[b][c] W[c][d];  dW[c][d] += sum_b dy[b][c] x[b][d];  db[c] += sum_b dy[b][c]
__global__ void linear_bwd_dx_kernel(const float* __restrict__ dy, const float* __restrict__ W, int B, int D, int C,
                                     float* __restrict__ dx) {
  const long long n = (long long)B * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / D), d = (int)(i % D);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += dy[(long long)b * C + c] * W[(long long)c * D + d];
    dx[i] = s;
  }
}
__global__ void linear_bwd_dw_kernel(const float* __restrict__ dy, const float* __restrict__ x, int B, int D, int C,
                                     float* __restrict__ dW, float* __restrict__ db) {
  const long long n = (long long)C * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i / D), d = (int)(i % D);
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dy[(long long)b * C + c] * x[(long long)b * D + d];
    dW[i] += s;
    if (d == 0 && db) {
      float t = 0.f;
      for (int b = 0; b < B; ++b) t += dy[(long long)b * C + c];
      db[c] += t;
    }
  }
}

// mean cross entropy with ignore_index; saves the row softmax for the backward
__global__ void ce_fwd_kernel(const float* __restrict__ logits, const long long* __restrict__ labels, int B, int C,
                              long long ignore_index, float* __restrict__ prob, float* __restrict__ loss) {
  __shared__ float part[4];
  __shared__ int cntp[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float total = 0.f;
  int cnt = 0;
  for (int r = wid; r < B; r += 4) {
    const float* x = logits + (long long)r * C;
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, x[c]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += expf(x[c] - m);
    s = warp_sum(s);
    const float lse = m + logf(s);
    for (int c = lane; c < C; c += 64) prob[(long long)r * C + c] = expf(x[c] - lse);
    const long long lab = labels[r];
    if (lab != ignore_index) {
      total += lse - x[lab];
      ++cnt;
    }
  }
  if (lane == 0) { part[wid] = total; cntp[wid] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int n = cntp[0] + cntp[1] + cntp[2] + cntp[3];
    loss[0] = (part[0] + part[1] + part[2] + part[3]) / (float)(n > 0 ? n : 1);
    loss[1] = (float)n;
  }
}

__global__ void ce_bwd_kernel(const float* __restrict__ prob, const long long* __restrict__ labels, int B, int C,
                              long long ignore_index, const float* __restrict__ gout, const float* __restrict__ loss,
                              float* __restrict__ dlogits) {
  const long long n = (long long)B * C;
  const float g = gout[0] / fmaxf(loss[1], 1.f);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / C), c = (int)(i % C);
    const long long lab = labels[r];
    dlogits[i] = lab == ignore_index ? 0.f : g * (prob[i] - (c == lab ? 1.f : 0.f));
  }
}

// cosine similarity of row pairs: cos = (x1/max(|x1|,eps)) . (x2/max(|x2|,eps)); saves the norms
__global__ void cosine_fwd_kernel(const float* __restrict__ x1, long long n1, const float* __restrict__ x2, long long n2,
                                  int D, float eps, float* __restrict__ cosv, float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const long long n = n1 > n2 ? n1 : n2;
  for (long long i = blockIdx.x * (long long)(blockDim.x / 64) + (threadIdx.x >> 6); i < n;
       i += (long long)gridDim.x * (blockDim.x / 64)) {
    const float* a = x1 + (n1 == 1 ? 0 : i) * D;
    const float* b = x2 + (n2 == 1 ? 0 : i) * D;
    float aa = 0.f, bb = 0.f, ab = 0.f;
    for (int d = lane; d < D; d += 64) {
      aa += a[d] * a[d];
      bb += b[d] * b[d];
      ab += a[d] * b[d];
    }
    aa = warp_sum(aa);
    bb = warp_sum(bb);
    ab = warp_sum(ab);
    if (lane == 0) {
      const float na = fmaxf(sqrtf(aa), eps), nb = fmaxf(sqrtf(bb), eps);
      cosv[i] = ab / (na * nb);
      norms[2 * i] = na;
      norms[2 * i + 1] = nb;
    }
  }
}

// d cos / d x1 = x2/(na nb) - cos x1/na^2 (and symmetric); gcos per row
__global__ void cosine_bwd_kernel(const float* __restrict__ x1, long long n1, const float* __restrict__ x2, long long n2,
                                  int D, const float* __restrict__ cosv, const float* __restrict__ norms,
                                  const float* __restrict__ gcos, float* __restrict__ d1, float* __restrict__ d2) {
  const long long n = n1 > n2 ? n1 : n2;
  const long long tot = n * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D;
    const int d = (int)(i % D);
    const float a = x1[(n1 == 1 ? 0 : r) * D + d], b = x2[(n2 == 1 ? 0 : r) * D + d];
    const float na = norms[2 * r], nb = norms[2 * r + 1], c = cosv[r], g = gcos[r];
    const float ga = g * (b / (na * nb) - c * a / (na * na));
    const float gb = g * (a / (na * nb) - c * b / (nb * nb));
    if (d1) {
      if (n1 == 1) atomicAdd(d1 + d, ga);
      else d1[i] = ga;
    }
    if (d2) {
      if (n2 == 1) atomicAdd(d2 + d, gb);
      else d2[i] = gb;
    }
  }
}

// triplet hinge over precomputed distances: loss = mean max(0, m + dp - dn); grads wrt dp, dn
__global__ void hinge_fwd_kernel(const float* __restrict__ dp, const float* __restrict__ dn, int B, float margin,
                                 float* __restrict__ loss) {
  __shared__ float part[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) s += fmaxf(margin + dp[i] - dn[i], 0.f);
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = part[0] / (float)B;
}
__global__ void hinge_bwd_kernel(const float* __restrict__ dp, const float* __restrict__ dn, int B, float margin,
                                 const float* __restrict__ gout, float* __restrict__ gdp, float* __restrict__ gdn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const float g = (margin + dp[i] - dn[i] >= 0.f) ? gout[0] / (float)B : 0.f;
  gdp[i] = g;
  gdn[i] = -g;
}

}  // namespace artsbir

using namespace artsbir;

static unsigned g256(long long n) {
  long long g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  return (unsigned)(g < 1 ? 1 : g);
}

extern "C" int artsbir_linear_fwd(const float* x, const float* W, const float* bias, int B, int D, int C, float* y,
                                  void* stream) {
  long long g = ((long long)B * C + 3) / 4;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0,
                     (hipStream_t)stream, x, W, bias, B, D, C, y);
  ARTSBIR_CHECK_LAUNCH("linear_fwd");
  return 0;
}

extern "C" int artsbir_linear_bwd(const float* dy, const float* x, const float* W, int B, int D, int C, float* dx,
                                  float* dW, float* db, void* stream) {
  if (dx) hipLaunchKernelGGL(linear_bwd_dx_kernel, dim3(g256((long long)B * D)), dim3(256), 0, (hipStream_t)stream, dy, W, B, D, C, dx);
  if (dW) hipLaunchKernelGGL(linear_bwd_dw_kernel, dim3(g256((long long)C * D)), dim3(256), 0, (hipStream_t)stream, dy, x, B, D, C, dW, db);
  ARTSBIR_CHECK_LAUNCH("linear_bwd");
  return 0;
}

extern "C" int artsbir_cross_entropy_fwd(const float* logits, const long long* labels, int B, int C,
                                         long long ignore_index, float* prob, float* loss2, void* stream) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, labels, B, C, ignore_index, prob, loss2);
  ARTSBIR_CHECK_LAUNCH("cross_entropy_fwd");
  return 0;
}

extern "C" int artsbir_cross_entropy_bwd(const float* prob, const long long* labels, int B, int C, long long ignore_index,
                                         const float* gout, const float* loss2, float* dlogits, void* stream) {
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(g256((long long)B * C)), dim3(256), 0, (hipStream_t)stream, prob, labels, B, C,
                     ignore_index, gout, loss2, dlogits);
  ARTSBIR_CHECK_LAUNCH("cross_entropy_bwd");
  return 0;
}

extern "C" int artsbir_cosine_fwd(const float* x1, long long n1, const float* x2, long long n2, int D, float eps,
                                  float* cosv, float* norms, void* stream) {
  if (!(n1 == n2 || n1 == 1 || n2 == 1)) { set_error("cosine: shapes %lld vs %lld", n1, n2); return -1; }
  const long long n = n1 > n2 ? n1 : n2;
  long long g = (n + 3) / 4;
  hipLaunchKernelGGL(cosine_fwd_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0,
                     (hipStream_t)stream, x1, n1, x2, n2, D, eps, cosv, norms);
  ARTSBIR_CHECK_LAUNCH("cosine_fwd");
  return 0;
}

extern "C" int artsbir_cosine_bwd(const float* x1, long long n1, const float* x2, long long n2, int D, const float* cosv,
                                  const float* norms, const float* gcos, float* d1, float* d2, void* stream) {
  const long long n = n1 > n2 ? n1 : n2;
  hipLaunchKernelGGL(cosine_bwd_kernel, dim3(g256(n * D)), dim3(256), 0, (hipStream_t)stream, x1, n1, x2, n2, D, cosv,
                     norms, gcos, d1, d2);
  ARTSBIR_CHECK_LAUNCH("cosine_bwd");
  return 0;
}

extern "C" int artsbir_hinge_fwd(const float* dp, const float* dn, int B, float margin, float* loss, void* stream) {
  hipLaunchKernelGGL(hinge_fwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, dp, dn, B, margin, loss);
  ARTSBIR_CHECK_LAUNCH("hinge_fwd");
  return 0;
}

extern "C" int artsbir_hinge_bwd(const float* dp, const float* dn, int B, float margin, const float* gout, float* gdp,
                                 float* gdn, void* stream) {
  hipLaunchKernelGGL(hinge_bwd_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, dp, dn, B, margin, gout,
                     gdp, gdn);
  ARTSBIR_CHECK_LAUNCH("hinge_bwd");
  return 0;
}

// backward of ||x1 - x2 + eps||: d/dx1 = g (x1 - x2 + eps) / d, d/dx2 = -that
namespace artsbir {
__global__ void pairwise_l2_bwd_kernel(const float* __restrict__ x1, long long n1, const float* __restrict__ x2,
                                       long long n2, int D, float eps, const float* __restrict__ dist,
                                       const float* __restrict__ gout, float* __restrict__ d1, float* __restrict__ d2) {
  const long long n = n1 > n2 ? n1 : n2;
  const long long tot = n * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < tot; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / D;
    const int d = (int)(i % D);
    const float dd = dist[r];
    const float t = dd > 0.f ? gout[r] * (x1[(n1 == 1 ? 0 : r) * D + d] - x2[(n2 == 1 ? 0 : r) * D + d] + eps) / dd : 0.f;
    if (d1) {
      if (n1 == 1) atomicAdd(d1 + d, t);
      else d1[i] = t;
    }
    if (d2) {
      if (n2 == 1) atomicAdd(d2 + d, -t);
      else d2[i] = -t;
    }
  }
}
}  // namespace artsbir

extern "C" int artsbir_pairwise_l2_bwd(const float* x1, long long n1, const float* x2, long long n2, int D, float eps,
                                       const float* dist, const float* gout, float* d1, float* d2, void* stream) {
  const long long n = n1 > n2 ? n1 : n2;
  hipLaunchKernelGGL(artsbir::pairwise_l2_bwd_kernel, dim3(g256(n * D)), dim3(256), 0, (hipStream_t)stream, x1, n1, x2,
                     n2, D, eps, dist, gout, d1, d2);
  ARTSBIR_CHECK_LAUNCH("pairwise_l2_bwd");
  return 0;
}
