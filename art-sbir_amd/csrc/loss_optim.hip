// Triplet-margin loss (train.py:169 nn.TripletMarginLoss(margin=0.2): p=2,
// eps=1e-6 added to (a-p), swap=False, reduction='mean') forward + backward,
// and the Adam step (train.py:158 torch.optim.Adam(lr, weight_decay): coupled
// L2, betas (0.9, 0.999), eps 1e-8) over every parameter tensor in one launch.
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

// one wave per triplet row, B/4 workgroups; dist[2*B] saved for the backward
// (the per-row arithmetic of the single-workgroup form this replaced: one
// workgroup walked all rows, ~0.5 ms at B = 512)
__global__ void __launch_bounds__(256) triplet_rows_kernel(const float* __restrict__ a, const float* __restrict__ p,
                                                           const float* __restrict__ n, int B, int D, float eps,
                                                           float* __restrict__ dist) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  float sp = 0.f, sn = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float av = a[(long long)r * D + d];
    const float dpv = av - p[(long long)r * D + d] + eps;
    const float dnv = av - n[(long long)r * D + d] + eps;
    sp += dpv * dpv;
    sn += dnv * dnv;
  }
  sp = warp_sum(sp);
  sn = warp_sum(sn);
  if (lane == 0) { dist[2 * r] = sqrtf(sp); dist[2 * r + 1] = sqrtf(sn); }
}

// mean of the hinge over the rows in a fixed order: four partial sums over rows
// w, w + 4, ... then their sum (the single-workgroup form's order, bit for bit)
__global__ void triplet_mean_kernel(const float* __restrict__ dist, int B, float margin, float* __restrict__ loss) {
  __shared__ float part[4];
  const int w = threadIdx.x;
  if (w < 4) {
    float total = 0.f;
    for (int r = w; r < B; r += 4) total += fmaxf(margin + dist[2 * r] - dist[2 * r + 1], 0.f);
    part[w] = total;
  }
  __syncthreads();
  if (w == 0) loss[0] = (part[0] + part[1] + part[2] + part[3]) / (float)B;
}

__global__ void triplet_bwd_kernel(const float* __restrict__ a, const float* __restrict__ p, const float* __restrict__ n,
                                   int B, int D, float margin, float eps, const float* __restrict__ dist,
                                   const float* __restrict__ gout, float* __restrict__ da, float* __restrict__ dp,
                                   float* __restrict__ dn) {
  const long long total = (long long)B * D;
  const float g = gout[0] / (float)B;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / D);
    const float dap = dist[2 * r], dan = dist[2 * r + 1];
    float ga = 0.f, gp = 0.f, gn = 0.f;
    if (margin + dap - dan >= 0.f) {  // clamp_min backward passes where input >= 0
      const float av = a[i];
      const float up = dap > 0.f ? (av - p[i] + eps) / dap : 0.f;
      const float un = dan > 0.f ? (av - n[i] + eps) / dan : 0.f;
      ga = g * (up - un);
      gp = -g * up;
      gn = g * un;
    }
    if (da) da[i] = ga;
    if (dp) dp[i] = gp;
    if (dn) dn[i] = gn;
  }
}

// Adam over a table of tensors: block -> (tensor, chunk) via a block table.
struct AdamTensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long numel;
};

__global__ void __launch_bounds__(256) adam_kernel(const AdamTensor* __restrict__ tensors,
                                                  const long long* __restrict__ block_table, long long chunk, float lr,
                                                  float beta1, float beta2, float eps, float weight_decay,
                                                  float step_size, float bc2_sqrt) {
  const long long ent = block_table[blockIdx.x];
  const int ti = (int)(ent >> 40);
  const long long start = ent & ((1LL << 40) - 1);
  const AdamTensor t = tensors[ti];
  long long end = start + chunk;
  if (end > t.numel) end = t.numel;
  for (long long i = start + threadIdx.x; i < end; i += blockDim.x) {
    const float p = t.param[i];
    float g = t.grad[i];
    if (weight_decay != 0.f) g = g + weight_decay * p;
    float m = t.exp_avg[i];
    m = m + (1.f - beta1) * (g - m);  // exp_avg.lerp_(grad, 1 - beta1), weight < 0.5 branch
    float v = t.exp_avg_sq[i];
    v = v * beta2 + (1.f - beta2) * g * g;
    t.exp_avg[i] = m;
    t.exp_avg_sq[i] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    t.param[i] = p - step_size * (m / denom);
  }
}

}  // namespace artsbir

using namespace artsbir;

extern "C" int artsbir_triplet_fwd(const float* a, const float* p, const float* n, int B, int D, float margin, float eps,
                                   float* dist, float* loss, void* stream) {
  if (B <= 0) { set_error("triplet_fwd: empty batch"); return -1; }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(triplet_rows_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, a, p, n, B, D, eps, dist);
  hipLaunchKernelGGL(triplet_mean_kernel, dim3(1), dim3(64), 0, st, dist, B, margin, loss);
  ARTSBIR_CHECK_LAUNCH("triplet_fwd");
  return 0;
}

extern "C" int artsbir_triplet_bwd(const float* a, const float* p, const float* n, int B, int D, float margin, float eps,
                                   const float* dist, const float* grad_loss, float* da, float* dp, float* dn,
                                   void* stream) {
  long long total = (long long)B * D;
  unsigned grid = (unsigned)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(triplet_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, a, p, n, B, D, margin, eps, dist,
                     grad_loss, da, dp, dn);
  ARTSBIR_CHECK_LAUNCH("triplet_bwd");
  return 0;
}

extern "C" long long artsbir_adam_table_blocks(const long long* numels, int ntensors, long long chunk) {
  long long nb = 0;
  for (int i = 0; i < ntensors; ++i) nb += (numels[i] + chunk - 1) / chunk;
  return nb;
}

extern "C" int artsbir_adam_fill_table(const long long* numels, int ntensors, long long chunk, long long* table) {
  long long k = 0;
  for (int i = 0; i < ntensors; ++i)
    for (long long s = 0; s < numels[i]; s += chunk) table[k++] = ((long long)i << 40) | s;
  return 0;
}

extern "C" int artsbir_adam_step(const void* tensors, const long long* block_table, long long nblocks, long long chunk,
                                 float lr, float beta1, float beta2, float eps, float weight_decay, long long step,
                                 void* stream) {
  if (step < 1) { set_error("adam: step must be >= 1"); return -1; }
  if (nblocks <= 0) return 0;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream,
                     (const AdamTensor*)tensors, block_table, chunk, lr, beta1, beta2, eps, weight_decay, step_size,
                     bc2_sqrt);
  ARTSBIR_CHECK_LAUNCH("adam_step");
  return 0;
}
