// Memory-bound kernels of the encoder hot path (NHWC, 8 channels per thread).
//
// Reference ops replaced (all /root/reference/models.py):
//   x.type(conv1.weight.dtype) + NCHW->NHWC                       :352
//   BatchNorm2d train/eval (batch stats finalize, running update)  :199,203,209,220,311,314,317
//   ReLU, AvgPool2d(2)/(stride), residual add + ReLU               :200-206,218,234-235,312-319
//   their autograd backward (BN backward, ReLU mask, unpool)
//   AttentionPool2d token build (mean token + positional emb)      :250-252
// plus parameter (re)packing between the reference layout and the kernel layouts.
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

template <typename T> __device__ __forceinline__ void load8(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void load8<bf16>(const bf16* p, float (&v)[8]) {
  Vec16<bf16> r = ld16<bf16>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)r.v[i];
}
template <> __device__ __forceinline__ void load8<float>(const float* p, float (&v)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <typename T> __device__ __forceinline__ void store8(T* p, const float (&v)[8]);
#ifndef ARTSBIR_NT_STORES
// 1: streaming (non-temporal) stores of the elementwise passes too — measured
// slower than plain stores on top of the GEMM epilogues' (profiles/r4_nt_stores.txt)
#define ARTSBIR_NT_STORES 0
#endif
template <> __device__ __forceinline__ void store8<bf16>(bf16* p, const float (&v)[8]) {
  Vec16<bf16> r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = (bf16)v[i];
  if constexpr (ARTSBIR_NT_STORES) {
    typedef unsigned st_u32x4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(*reinterpret_cast<const st_u32x4*>(&r), reinterpret_cast<st_u32x4*>(p));
  } else {
    st16<bf16>(p, r);
  }
}
template <> __device__ __forceinline__ void store8<float>(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void loadf8(const float* p, float (&v)[8]) { load8<float>(p, v); }

// streaming read of an operand the kernel is its last reader of (non-temporal:
// no cache allocation for lines nobody reads again); ARTSBIR_NT_LOADS=0 plain
#ifndef ARTSBIR_NT_LOADS
#define ARTSBIR_NT_LOADS 1
#endif
typedef unsigned nt_u32x4 __attribute__((ext_vector_type(4)));
template <typename T> __device__ __forceinline__ void load8_last(const T* p, float (&v)[8]) {
  if constexpr (ARTSBIR_NT_LOADS && sizeof(T) == 2) {
    const nt_u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x4*>(p));
    const bf16* b = reinterpret_cast<const bf16*>(&r);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)b[i];
  } else {
    load8<T>(p, v);
  }
}

static inline unsigned grid_for(long long n, int block = 256, long long cap = 1 << 20) {
  long long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---------------------------------------------------------------- pack input
// x [B][3][H][W] f32 (NCHW) -> out [B][H][W][8] T, channels 3..7 zero.
template <typename T>
__global__ void pack_input_kernel(const float* __restrict__ x, T* __restrict__ out, int B, int Cin, int H, int W) {
  const long long npix = (long long)B * H * W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix; i += (long long)gridDim.x * blockDim.x) {
    long long b = i / ((long long)H * W);
    long long hw = i - b * H * W;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < Cin ? x[(b * Cin + c) * H * W + hw] : 0.f;
    store8<T>(out + i * 8, v);
  }
}

// ------------------------------------------------------- bn finalize (forward)
// stats [NSLOT][2][C] (sum, sum of squares) -> mean, istd, scale = gamma*istd, beta;
// train: update running stats (momentum, unbiased var) and num_batches_tracked.
__global__ void bn_finalize_kernel(const float* __restrict__ stats, int C, double count, const float* gamma,
                                   const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                                   float eps, int train, float* mean_out, float* istd_out, float* scale, float* beta_out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && train && nbt) nbt[0] += 1;
  if (c >= C) return;
  double mean, var;
  if (train) {
    double s1 = 0, s2 = 0;
    for (int k = 0; k < ARTSBIR_NSLOT; ++k) {
      s1 += stats[(long long)k * 2 * C + c];
      s2 += stats[(long long)k * 2 * C + C + c];
    }
    mean = s1 / count;
    var = s2 / count - mean * mean;
    if (var < 0) var = 0;
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * count / (count > 1 ? count - 1 : 1));
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  float is = (float)(1.0 / sqrt(var + (double)eps));
  float sc = gamma[c] * is;
  mean_out[c] = (float)mean;
  istd_out[c] = is;
  scale[c] = sc;
  beta_out[c] = beta[c];
}

// all nseg BN segments of one layer in one launch: per channel the segments in
// order (running statistics updated once per segment, as the reference's
// consecutive forward calls do); out[s] = {mean, istd, scale, beta}[C] — the BN
// parameter block every consumer applies as (y - mean) * scale + beta
// Slot sums of a BN site: 4 lanes per channel add 8 of the ARTSBIR_NSLOT
// replica slots each (16 independent loads in flight per lane instead of a
// 32-long dependent chain per channel), the quarters combined in fixed order
// by lane shuffles; segments FIN_SEGS at a time.  grid ceil(C / 64), 256
// threads: lanes 4i..4i+3 of wave w hold the quarters of channel 16w + i.
// No LDS, so the kernel co-resides with the LDS-heavy weight-gradient
// workgroups of the side stream instead of waiting for a CU to drain (the
// backward's finalizes took ~60 us each behind them, the forward's 6 us).
constexpr int FIN_CPB = 64, FIN_Q = 4, FIN_SEGS = 4;
static_assert(ARTSBIR_NSLOT % FIN_Q == 0, "slot quarters");

__device__ __forceinline__ int fin_channel() {
  return blockIdx.x * FIN_CPB + (threadIdx.x >> 6) * 16 + ((threadIdx.x & 63) >> 2);
}

// the four quarters of this lane's channel, added in quarter order (the same
// f64 order as a sequential sum over the quarters); every lane must call it
__device__ __forceinline__ void fin_combine(double& s1, double& s2) {
  const int b = (threadIdx.x & 63) & ~3;
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int u = 0; u < FIN_Q; ++u) {
    t1 += __shfl(s1, b + u, 64);
    t2 += __shfl(s2, b + u, 64);
  }
  s1 = t1;
  s2 = t2;
}

__device__ __forceinline__ void fin_quarter(const float* __restrict__ st, long long C, int c, int q, double& s1,
                                            double& s2) {
  constexpr int KQ = ARTSBIR_NSLOT / FIN_Q;
  const float* p = st + (long long)q * KQ * 2 * C + c;
  float v1[KQ], v2[KQ];
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    v1[k] = p[(long long)k * 2 * C];
    v2[k] = p[(long long)k * 2 * C + C];
  }
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int k = 0; k < KQ; ++k) {
    s1 += v1[k];
    s2 += v2[k];
  }
}

// all nseg BN segments of one layer in one launch: per channel the segments in
// order (running statistics updated once per segment, as the reference's
// consecutive forward calls do); out[s] = {mean, istd, scale, beta}[C] — the BN
// parameter block every consumer applies as (y - mean) * scale + beta
__global__ void __launch_bounds__(256) bn_finalize_seg_kernel(const float* __restrict__ stats, int nseg,
                                                              long long seg_stride, int C, double count,
                                                              const float* gamma, const float* beta, float* rmean,
                                                              float* rvar, long long* nbt, float momentum, float eps,
                                                              int train, float* __restrict__ out) {
  const int c = fin_channel(), q = threadIdx.x & 3;
  if (blockIdx.x == 0 && threadIdx.x == 0 && train && nbt) nbt[0] += nseg;
  for (int s0 = 0; s0 < nseg; s0 += FIN_SEGS) {
    const int ns = nseg - s0 < FIN_SEGS ? nseg - s0 : FIN_SEGS;
    double r1[FIN_SEGS], r2[FIN_SEGS];
#pragma unroll
    for (int s = 0; s < FIN_SEGS; ++s) {
      r1[s] = 0.0;
      r2[s] = 0.0;
      if (train && s < ns && c < C) fin_quarter(stats + (long long)(s0 + s) * seg_stride, C, c, q, r1[s], r2[s]);
    }
    if (train) {
#pragma unroll
      for (int s = 0; s < FIN_SEGS; ++s) fin_combine(r1[s], r2[s]);
    }
    if (q == 0 && c < C) {
      for (int s = 0; s < ns; ++s) {
        double mean, var;
        if (train) {
          mean = r1[s] / count;
          var = r2[s] / count - mean * mean;
          if (var < 0) var = 0;
          if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
          if (rvar) rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * count / (count > 1 ? count - 1 : 1));
        } else {
          mean = rmean[c];
          var = rvar[c];
        }
        const float is = (float)(1.0 / sqrt(var + (double)eps));
        const float sc = gamma[c] * is;
        float* o = out + (long long)(s0 + s) * 4 * C;
        o[c] = (float)mean;
        o[C + c] = is;
        o[2 * C + c] = sc;
        o[3 * C + c] = beta[c];
      }
    }
  }
}

// --------------------------------------- deterministic BN statistics (parity)
// The conv epilogues add their per-channel sums into replica slots with f32
// atomics, whose order changes from run to run; on tiny parity batches that
// noise can move a pre-activation across zero (a ReLU flip).  In the
// deterministic mode (artsbir_set_deterministic) the engine launches the conv
// without statistics and this kernel sums the stored output y of each segment
// in a fixed order in f64: thread (rl, c) takes rows rl, rl+16, ... of channel
// c, the 16 partials are added in index order.  The f64 sums are written as
// f32 hi/lo pairs into slots 0 and 1 (other slots zero), so bn_finalize's f64
// sum over the slots sees ~48 significant bits.  grid (ceil(C/64), nseg).
template <typename T>
__global__ void __launch_bounds__(1024) bn_stats_det_kernel(const T* __restrict__ y, long long rows, int C,
                                                            float* __restrict__ stats, long long seg_stride) {
  __shared__ double red[2][16][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const T* ys = y + (long long)blockIdx.y * rows * C;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    for (long long r = rl; r < rows; r += 16) {
      const double v = (double)to_f(ys[r * C + c]);
      s1 += v;
      s2 += v * v;
    }
  }
  red[0][rl][cl] = s1;
  red[1][rl][cl] = s2;
  __syncthreads();
  if (rl != 0 || c >= C) return;
  double t1 = 0.0, t2 = 0.0;
  for (int k = 0; k < 16; ++k) { t1 += red[0][k][cl]; t2 += red[1][k][cl]; }
  float* st = stats + (long long)blockIdx.y * seg_stride;
  const float h1 = (float)t1, h2 = (float)t2;
  st[c] = h1;
  st[C + c] = h2;
  st[2 * C + c] = (float)(t1 - (double)h1);
  st[3 * C + c] = (float)(t2 - (double)h2);
  for (int k = 2; k < ARTSBIR_NSLOT; ++k) {
    st[(long long)k * 2 * C + c] = 0.f;
    st[(long long)k * 2 * C + C + c] = 0.f;
  }
}

// ------------------------------------------------ affine(+relu)(+avgpool 2x2)
// out = pool?( act(x) ), act = (x - mean) * scale + beta then ReLU, from the BN
// parameter block bn [4][C] = mean, istd, scale, beta (bn == NULL: identity, no
// relu).  Subtracting the mean first keeps the f32 result accurate when
// |mean| >> std (x*scale + (beta - mean*scale) loses |mean|/std ulps).
__device__ __forceinline__ void load_bn8(const float* bn, int C, int c0, float (&m)[8], float (&s)[8], float (&b)[8]) {
  loadf8(bn + c0, m);
  loadf8(bn + 2 * C + c0, s);
  loadf8(bn + 3 * C + c0, b);
}

// nseg segments (the triplet branches): images b of segment b / (B / nseg) use
// the parameter block bn + segment * 4 C
template <typename T>
__global__ void act_pool_kernel(const T* __restrict__ x, const float* __restrict__ bn, int relu, int pool, int B,
                                int H, int W, int C, int nseg, T* __restrict__ out) {
  const int CG = C / 8;
  const int Ho = pool ? H / pool : H, Wo = pool ? W / pool : W;
  const long long n = (long long)B * Ho * Wo * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    int cg = (int)(i % CG);
    long long pix = i / CG;
    int ow = (int)(pix % Wo);
    long long t = pix / Wo;
    int oh = (int)(t % Ho);
    long long b = t / Ho;
    float mn[8], s[8], h[8];
    if (bn) load_bn8(bn + (b / (B / nseg)) * 4 * C, C, cg * 8, mn, s, h);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int P = pool ? pool : 1;
    for (int dy = 0; dy < P; ++dy)
      for (int dx = 0; dx < P; ++dx) {
        float v[8];
        load8<T>(x + (((b * H + oh * P + dy) * W + ow * P + dx) * C + cg * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float a = bn ? (v[e] - mn[e]) * s[e] + h[e] : v[e];
          if (relu) a = fmaxf(a, 0.f);
          acc[e] += a;
        }
      }
    const float inv = 1.f / (P * P);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    store8<T>(out + pix * C + cg * 8, acc);
  }
}

// The same with each lane owning one 8-channel group for the whole launch
// (BN parameters loaded once, no per-element index division) and UN units per
// trip with every load issued before the trip's stores; segment = blockIdx.y
// (Bs images each), units = output pixels.  C / 8 <= 256.
// CS: also the column sums of the stored output per segment, into one of
// ARTSBIR_NSLOT replica rows of colsum[s][slot][C] (the folded BatchNorm
// backward's 1^T x of the next conv's input, csrc/fold.hip: no extra pass over x)
template <typename T, int P, bool CS = false>
__global__ void __launch_bounds__(256) act_pool_cg_kernel(const T* __restrict__ x, const float* __restrict__ bn,
                                                          int relu, int Bs, int H, int W, int C, int units_per_block,
                                                          T* __restrict__ out, float* __restrict__ colsum = nullptr) {
  const int s = blockIdx.y;
  const int CG = C / 8, RL = 256 / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  float csum[CS ? 8 : 1];
  if constexpr (CS) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
  if (!CS && rl >= RL) return;
  const int Ho = H / P, Wo = W / P;
  const int units = Bs * Ho * Wo;
  const T* xs = x + (long long)s * Bs * H * W * C + cg * 8;
  T* os = out + (long long)s * units * C + cg * 8;
  float mn[8], sc[8], bt[8];
  if (bn) load_bn8(bn + (long long)s * 4 * C, C, cg * 8, mn, sc, bt);
  const int u0 = blockIdx.x * units_per_block;
  const int u1 = min(u0 + units_per_block, units);
  constexpr int UN = P == 1 ? 4 : 2;
  for (int ub = u0 + rl; rl < RL && ub < u1; ub += RL * UN) {
    float v[UN][P * P][8];
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      const int u = min(ub + i * RL, u1 - 1);  // clamped tail: recomputed, stored once
      if constexpr (P == 1) {
        load8<T>(xs + (long long)u * C, v[i][0]);
      } else {
        const int ow = u % Wo, t = u / Wo;
        const int oh = t % Ho, b = t / Ho;
#pragma unroll
        for (int dy = 0; dy < P; ++dy)
#pragma unroll
          for (int dx = 0; dx < P; ++dx)
            load8<T>(xs + ((long long)(b * H + oh * P + dy) * W + ow * P + dx) * C, v[i][dy * P + dx]);
      }
    }
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      if (ub + i * RL >= u1) break;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < P * P; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float a = bn ? (v[i][q][e] - mn[e]) * sc[e] + bt[e] : v[i][q][e];
          if (relu) a = fmaxf(a, 0.f);
          acc[e] += a;
        }
      constexpr float inv = 1.f / (P * P);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= inv;
      store8<T>(os + (long long)(ub + i * RL) * C, acc);
      if constexpr (CS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += to_f(from_f<T>(acc[e]));  // the stored values
      }
    }
  }
  if constexpr (CS) {  // the RL lanes of each channel group, then one atomic per channel
    __shared__ float red[256][9];
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = rl < RL ? csum[e] : 0.f;
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int g = c >> 3, e = c & 7;
      float t = 0.f;
      for (int r = 0; r < RL; ++r) t += red[r * CG + g][e];
      atomicAdd(colsum + ((long long)s * ARTSBIR_NSLOT + blockIdx.x % ARTSBIR_NSLOT) * C + c, t);
    }
  }
}

// --------------------------------------------------------- bottleneck output
// out = relu(bn3(y3) + (yd ? bnd(yd) : idn)), bn(y) = (y - mean) * scale + beta
template <typename T>
__global__ void block_out_kernel(const T* __restrict__ y3, const float* __restrict__ bn3, const T* __restrict__ yd,
                                 const float* __restrict__ bnd, const T* __restrict__ idn, long long rows, int C,
                                 int nseg, T* __restrict__ out, unsigned char* __restrict__ bits) {
  const int CG = C / 8;
  const long long n = rows * CG;
  const long long seg_rows = rows / nseg;  // rows of segment s use the blocks + s * 4 C
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    int cg = (int)(i % CG);
    const long long row = i / CG;
    long long off = row * C + cg * 8;
    const long long po = (row / seg_rows) * 4 * C;
    float a[8], m[8], s[8], h[8], r[8];
    load8<T>(y3 + off, a);
    load_bn8(bn3 + po, C, cg * 8, m, s, h);
    if (yd) {
      float m2[8], s2[8], h2[8];
      load8<T>(yd + off, r);
      load_bn8(bnd + po, C, cg * 8, m2, s2, h2);
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = (r[e] - m2[e]) * s2[e] + h2[e];
    } else {
      load8<T>(idn + off, r);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = fmaxf((a[e] - m[e]) * s[e] + h[e] + r[e], 0.f);
    store8<T>(out + off, a);
    if (bits) {  // ReLU mask of the stored values, one bit per channel
      unsigned m = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) m |= (to_f(from_f<T>(a[e])) > 0.f ? 1u : 0u) << e;
      bits[i] = (unsigned char)m;
    }
  }
}

// block_out with each lane owning one 8-channel group (parameters loaded once),
// segment = blockIdx.y (seg_rows rows each), 2 rows per trip with all loads
// issued before the stores.  C / 8 <= 256.
// CS: also the column sums of the stored output per segment into one of
// ARTSBIR_NSLOT replica rows of colsum[s][slot][C] — the 1^T x of the next
// block's folded conv1 weight gradient (csrc/fold.hip, the y-side fold)
template <typename T, bool CS = false>
__global__ void __launch_bounds__(256) block_out_cg_kernel(const T* __restrict__ y3, const float* __restrict__ bn3,
                                                           const T* __restrict__ yd, const float* __restrict__ bnd,
                                                           const T* __restrict__ idn, int seg_rows, int C,
                                                           int rows_per_block, T* __restrict__ out,
                                                           unsigned char* __restrict__ bits,
                                                           float* __restrict__ colsum = nullptr) {
  const int s = blockIdx.y;
  const int CG = C / 8, RL = 256 / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  float csum[CS ? 8 : 1];
  if constexpr (CS) {
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
  }
  if (!CS && rl >= RL) return;
  const long long po = (long long)s * 4 * C;
  float m[8], sc[8], h[8], m2[8], s2[8], h2[8];
  load_bn8(bn3 + po, C, cg * 8, m, sc, h);
  if (yd) load_bn8(bnd + po, C, cg * 8, m2, s2, h2);
  const T* rs = yd ? yd : idn;
  const long long base = (long long)s * seg_rows;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(r0 + rows_per_block, seg_rows);
  constexpr int UN = 2;
  for (int rb = r0 + rl; rl < RL && rb < r1; rb += RL * UN) {
    float a[UN][8], r[UN][8];
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      const long long off = (base + min(rb + i * RL, r1 - 1)) * C + cg * 8;
      load8<T>(y3 + off, a[i]);
      load8<T>(rs + off, r[i]);
    }
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      if (rb + i * RL >= r1) break;
      const long long row = base + rb + i * RL;
      if (yd) {
#pragma unroll
        for (int e = 0; e < 8; ++e) r[i][e] = (r[i][e] - m2[e]) * s2[e] + h2[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) a[i][e] = fmaxf((a[i][e] - m[e]) * sc[e] + h[e] + r[i][e], 0.f);
      store8<T>(out + row * C + cg * 8, a[i]);
      if (bits) {
        unsigned mk = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) mk |= (to_f(from_f<T>(a[i][e])) > 0.f ? 1u : 0u) << e;
        bits[row * CG + cg] = (unsigned char)mk;
      }
      if constexpr (CS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) csum[e] += to_f(from_f<T>(a[i][e]));  // the stored values
      }
    }
  }
  if constexpr (CS) {  // the RL lanes of each channel group, then one atomic per channel
    __shared__ float red[256][9];
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x][e] = rl < RL ? csum[e] : 0.f;
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      const int g = c >> 3, e = c & 7;
      float t = 0.f;
      for (int r = 0; r < RL; ++r) t += red[r * CG + g][e];
      atomicAdd(colsum + ((long long)s * ARTSBIR_NSLOT + blockIdx.x % ARTSBIR_NSLOT) * C + c, t);
    }
  }
}

// units per workgroup: the same workgroup sizing as the BN-backward apply (launch_bnb): ~16384
// workgroups, at least 8 unit rows each (ARTSBIR_CG_WGS / ARTSBIR_CG_MINROWS:
// other targets, measurement knobs; round 3 used 2048 and 1)
static int cg_units_per_block(long long units, int nseg, int C) {
  static const int wgs = getenv("ARTSBIR_CG_WGS") ? atoi(getenv("ARTSBIR_CG_WGS")) : 16384;
  static const int min_rows = getenv("ARTSBIR_CG_MINROWS") ? atoi(getenv("ARTSBIR_CG_MINROWS")) : 8;
  const int RL = 256 / (C / 8);
  long long upb = (units * nseg + wgs - 1) / wgs;
  if (upb < (long long)min_rows * RL) upb = (long long)min_rows * RL;
  if (upb < RL) upb = RL;
  return (int)upb;
}

// ------------------------------------------------------------ BN backward
// Two flavours of the upstream gradient g at an element of the BN output:
//   RES: g = dout * (out > 0)                      (block output ReLU)
//   ACT: g = up(d) * (bn(y) > 0)                   (ReLU after BN; up = identity
//        or 2x2 average-unpool when the forward pooled after the ReLU)
// For up to two BN targets t (y3 and the downsample yd share g), with
//   xhat_t = (y_t - mean_t) * istd_t:
//   REDUCE: slots_t[k][0][c] += sum g, slots_t[k][1][c] += sum g*xhat_t
//   APPLY : dy_t = c1_t*(g - c2_t - xhat_t*c3_t);  optional gout = g
struct BnBwdArgs {
  int kind;   // 0 RES, 1 ACT
  int pool;   // ACT: forward pooled by `pool` after the ReLU (0/1 = none)
  const void* d;     // RES: dout ; ACT: d (pooled resolution if pool>1)
  const void* mask;  // RES: out
  const float* mbn;  // ACT: parameter block [4][C] of the BN feeding the ReLU (target 0)
  int ntarget;
  const void* y[2];
  const float* mean[2];
  const float* istd[2];
  float* slots[2];           // REDUCE
  const float* coef[2];      // APPLY: [3][C] = c1, c2, c3
  void* dy[2];               // APPLY outputs
  void* gout;                // APPLY optional
  int B, H, W, C;            // geometry of y (full resolution), per segment
  long long pstride, cstride, sstride;  // per-segment strides of mean/istd/mbn, coef, slots (floats)
};

// segment blockIdx.y of a multi-segment launch: every tensor pointer advanced
// by whole segments (B images each), the per-channel arrays by their strides
template <typename T, int POOL>
__device__ __forceinline__ void bnb_seg(BnBwdArgs& a) {
  const int s = blockIdx.y;
  if (s == 0) return;
  const long long full = (long long)a.B * a.H * a.W * a.C;
  a.d = reinterpret_cast<const T*>(a.d) + s * (full / (POOL * POOL));
  if (a.mask)
    a.mask = a.kind == 3 ? static_cast<const void*>(reinterpret_cast<const unsigned char*>(a.mask) + s * (full / 8))
                         : static_cast<const void*>(reinterpret_cast<const T*>(a.mask) + s * full);
  if (a.mbn) a.mbn += s * a.pstride;
  for (int t = 0; t < 2; ++t) {
    if (a.y[t]) a.y[t] = reinterpret_cast<const T*>(a.y[t]) + s * full;
    if (a.dy[t]) a.dy[t] = reinterpret_cast<T*>(a.dy[t]) + s * full;
    if (a.mean[t]) a.mean[t] += s * a.pstride;
    if (a.istd[t]) a.istd[t] += s * a.pstride;
    if (a.coef[t]) a.coef[t] += s * a.cstride;
    if (a.slots[t]) a.slots[t] += s * a.sstride;
  }
  if (a.gout) a.gout = reinterpret_cast<T*>(a.gout) + s * full;
}

// A "unit" is one pixel, or one 2x2 (pool x pool) quad when the forward pooled
// after the ReLU: the quad's pooled gradient d is read once and spread over its
// four pixels.  Each thread owns one 8-channel group for the whole kernel, so
// per-channel parameters are loaded once; no per-element index division.
// yk (KIND 1): the BN inputs y_0 the mask was computed from, handed back so the
// caller's target-0 pass does not load them a second time
template <typename T, int KIND, int POOL>
__device__ __forceinline__ void bnb_unit_g(const BnBwdArgs& a, int u, int cg, long long (&offs)[POOL * POOL],
                                          float (&g)[POOL * POOL][8], const float (&mm)[8], const float (&ms)[8],
                                          const float (&mh)[8], float (*yk)[8] = nullptr) {
  if constexpr (POOL == 1) {
    offs[0] = (long long)u * a.C + cg * 8;
  } else {
    const int Wp = a.W / POOL, Hp = a.H / POOL;
    const int wp = u % Wp;
    const int t = u / Wp;
    const int hp = t % Hp;
    const int b = t / Hp;
#pragma unroll
    for (int dy = 0; dy < POOL; ++dy)
#pragma unroll
      for (int dx = 0; dx < POOL; ++dx)
        offs[dy * POOL + dx] = ((long long)(b * a.H + hp * POOL + dy) * a.W + wp * POOL + dx) * a.C + cg * 8;
  }
  if constexpr (KIND == 0) {
    float m[8];
    load8<T>(reinterpret_cast<const T*>(a.d) + offs[0], g[0]);
    load8<T>(reinterpret_cast<const T*>(a.mask) + offs[0], m);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[0][e] = m[e] > 0.f ? g[0][e] : 0.f;
  } else if constexpr (KIND == 3) {
    load8<T>(reinterpret_cast<const T*>(a.d) + offs[0], g[0]);
    const unsigned m = reinterpret_cast<const unsigned char*>(a.mask)[(long long)u * (a.C / 8) + cg];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[0][e] = (m >> e) & 1u ? g[0][e] : 0.f;
  } else if constexpr (KIND == 2) {
    load8<T>(reinterpret_cast<const T*>(a.d) + offs[0], g[0]);  // g given (masked upstream)
  } else {
    float dv[8];
    load8<T>(reinterpret_cast<const T*>(a.d) + (long long)u * a.C + cg * 8, dv);
    constexpr float inv = 1.f / (POOL * POOL);
#pragma unroll
    for (int q = 0; q < POOL * POOL; ++q) {
      float y[8];
      load8<T>(reinterpret_cast<const T*>(a.y[0]) + offs[q], y);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[q][e] = ((y[e] - mm[e]) * ms[e] + mh[e]) > 0.f ? dv[e] * inv : 0.f;
      if (yk) {
#pragma unroll
        for (int e = 0; e < 8; ++e) yk[q][e] = y[e];
      }
    }
  }
}

template <typename T, int KIND, int POOL, int NT>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(BnBwdArgs a, int units_per_block) {
  bnb_seg<T, POOL>(a);
  constexpr int NQ = POOL * POOL;
  const int CG = a.C / 8;
  const int RL = 256 / CG;  // unit lanes
  const int tid = threadIdx.x;
  const int cg = tid % CG, rl = tid / CG;
  const int units = a.B * (a.H / POOL) * (a.W / POOL);
  const int u0 = blockIdx.x * units_per_block;
  const int u1 = min(u0 + units_per_block, units);
  float acc[NT][2][8];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t][q][e] = 0.f;
  if (rl < RL) {
    float mn[NT][8], is[NT][8], mm[8], ms[8], mh[8];
#pragma unroll
    for (int t = 0; t < NT; ++t) { loadf8(a.mean[t] + cg * 8, mn[t]); loadf8(a.istd[t] + cg * 8, is[t]); }
    if constexpr (KIND == 1) load_bn8(a.mbn, a.C, cg * 8, mm, ms, mh);
    for (int u = u0 + rl; u < u1; u += RL) {
      long long offs[NQ];
      float g[NQ][8], yk[NQ][8];
      bnb_unit_g<T, KIND, POOL>(a, u, cg, offs, g, mm, ms, mh, KIND == 1 ? yk : nullptr);
      if constexpr (POOL == 1) {  // g written back (in place over d allowed)
        if (a.gout) store8<T>(reinterpret_cast<T*>(a.gout) + offs[0], g[0]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          float y[8];
          if (KIND == 1 && t == 0) {  // the mask's y_0, loaded once
#pragma unroll
            for (int e = 0; e < 8; ++e) y[e] = yk[q][e];
          } else {
            load8<T>(reinterpret_cast<const T*>(a.y[t]) + offs[q], y);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            acc[t][0][e] += g[q][e];
            acc[t][1][e] += g[q][e] * ((y[e] - mn[t][e]) * is[t][e]);
          }
        }
      }
    }
  }
  // reduce over unit lanes in LDS, then one atomic per channel per block
  __shared__ float red[256 * 8];
  const int slot = blockIdx.x % ARTSBIR_NSLOT;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[tid * 8 + e] = (rl < RL) ? acc[t][q][e] : 0.f;
      __syncthreads();
      if (tid < a.C) {  // one channel per thread
        const int c = tid, cgi = c / 8, e = c % 8;
        float sum = 0.f;
        for (int l = 0; l < RL; ++l) sum += red[(l * CG + cgi) * 8 + e];
        atomicAdd(a.slots[t] + (long long)slot * 2 * a.C + q * a.C + c, sum);
      }
      if (a.C > 256) {  // C up to 2048: remaining channels
        for (int c = tid + 256; c < a.C; c += 256) {
          const int cgi = c / 8, e = c % 8;
          float sum = 0.f;
          for (int l = 0; l < RL; ++l) sum += red[(l * CG + cgi) * 8 + e];
          atomicAdd(a.slots[t] + (long long)slot * 2 * a.C + q * a.C + c, sum);
        }
      }
    }
}

// Deterministic mode (artsbir_set_deterministic): the same reduction by ONE
// workgroup in a fixed order with f64 accumulators — lane (rl, cg) walks units
// rl, rl+RL, ..., the RL partials are added in lane order — written as f32 hi/lo
// pairs to slots 0/1 (other slots zeroed).  The f32 atomics above lose ~1e-7 of
// sum |g xhat| per add, which the BN backward's cancellation (g - mean g - xhat
// mean(g xhat)) turns into percent-level errors of small channels in parity runs.
template <typename T, int KIND, int POOL>
__global__ void __launch_bounds__(256) bn_bwd_reduce_det_kernel(BnBwdArgs a) {
  bnb_seg<T, POOL>(a);
  constexpr int NQ = POOL * POOL;
  const int CG = a.C / 8;
  const int RL = 256 / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, rl = tid / CG;
  const int units = a.B * (a.H / POOL) * (a.W / POOL);
  double acc[2][2][8];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t][q][e] = 0.0;
  if (rl < RL) {
    float mn[2][8], is[2][8], mm[8], ms[8], mh[8];
    for (int t = 0; t < a.ntarget; ++t) { loadf8(a.mean[t] + cg * 8, mn[t]); loadf8(a.istd[t] + cg * 8, is[t]); }
    if constexpr (KIND == 1) load_bn8(a.mbn, a.C, cg * 8, mm, ms, mh);
    for (int u = rl; u < units; u += RL) {
      long long offs[NQ];
      float g[NQ][8];
      bnb_unit_g<T, KIND, POOL>(a, u, cg, offs, g, mm, ms, mh);
      if constexpr (POOL == 1) {
        if (a.gout) store8<T>(reinterpret_cast<T*>(a.gout) + offs[0], g[0]);
      }
      for (int t = 0; t < a.ntarget; ++t) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          float y[8];
          load8<T>(reinterpret_cast<const T*>(a.y[t]) + offs[q], y);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            acc[t][0][e] += (double)g[q][e];
            acc[t][1][e] += (double)g[q][e] * ((double)(y[e] - mn[t][e]) * (double)is[t][e]);
          }
        }
      }
    }
  }
  __shared__ double red[256 * 8];
  for (int t = 0; t < a.ntarget; ++t)
    for (int q = 0; q < 2; ++q) {
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 8; ++e) red[tid * 8 + e] = (rl < RL) ? acc[t][q][e] : 0.0;
      __syncthreads();
      for (int c = tid; c < a.C; c += 256) {
        const int cgi = c / 8, e = c % 8;
        double sum = 0.0;
        for (int l = 0; l < RL; ++l) sum += red[(l * CG + cgi) * 8 + e];
        const float hi = (float)sum;
        float* sl = a.slots[t] + q * a.C + c;
        sl[0] = hi;
        sl[2LL * a.C] = (float)(sum - (double)hi);
        for (int k = 2; k < ARTSBIR_NSLOT; ++k) sl[(long long)k * 2 * a.C] = 0.f;
      }
    }
}

// NT (targets) is a template parameter so every per-target array is indexed
// statically (a run-time target count put them in scratch memory)
template <typename T, int KIND, int POOL, int NT>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(BnBwdArgs a, int units_per_block) {
  bnb_seg<T, POOL>(a);
  constexpr int NQ = POOL * POOL;
  const int CG = a.C / 8;
  const int RL = 256 / CG;
  const int tid = threadIdx.x;
  const int cg = tid % CG, rl = tid / CG;
  if (rl >= RL) return;
  const int units = a.B * (a.H / POOL) * (a.W / POOL);
  const int u0 = blockIdx.x * units_per_block;
  const int u1 = min(u0 + units_per_block, units);
  const T* yp[NT];
  T* dyp[NT];
  float mn[NT][8], is[NT][8], c1[NT][8], c2[NT][8], c3[NT][8], mm[8], ms[8], mh[8];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    yp[t] = reinterpret_cast<const T*>(a.y[t]);
    dyp[t] = reinterpret_cast<T*>(a.dy[t]);
    loadf8(a.mean[t] + cg * 8, mn[t]);
    loadf8(a.istd[t] + cg * 8, is[t]);
    loadf8(a.coef[t] + cg * 8, c1[t]);
    loadf8(a.coef[t] + a.C + cg * 8, c2[t]);
    loadf8(a.coef[t] + 2 * a.C + cg * 8, c3[t]);
  }
  if constexpr (KIND == 1) load_bn8(a.mbn, a.C, cg * 8, mm, ms, mh);
  T* const gout = reinterpret_cast<T*>(a.gout);
  // UN units per trip, every load of the trip issued before its first store
  // (the compiler cannot prove the stores alias none of the loads), so a lane
  // keeps UN units' bytes in flight instead of one
  constexpr int UN = POOL == 1 ? (NT == 1 ? 4 : 2) : 1;
  for (int ub = u0 + rl; ub < u1; ub += RL * UN) {
    long long offs[UN][NQ];
    float g[UN][NQ][8], y[UN][NT][NQ][8];
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      const int u = min(ub + i * RL, u1 - 1);  // clamped: a tail unit recomputes the last one, stored once
      if constexpr (KIND == 2 && POOL == 1) {  // g after a fused dgrad: this is its last read
        offs[i][0] = (long long)u * a.C + cg * 8;
        load8_last<T>(reinterpret_cast<const T*>(a.d) + offs[i][0], g[i][0]);
      } else {
        bnb_unit_g<T, KIND, POOL>(a, u, cg, offs[i], g[i], mm, ms, mh, KIND == 1 ? y[i][0] : nullptr);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          if (KIND == 1 && t == 0) continue;  // the mask's y_0, loaded once in bnb_unit_g
          load8_last<T>(yp[t] + offs[i][q], y[i][t][q]);
        }
    }
#pragma unroll
    for (int i = 0; i < UN; ++i) {
      if (ub + i * RL >= u1) break;
      if (gout) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) store8<T>(gout + offs[i][q], g[i][q]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e)
            o[e] = c1[t][e] * (g[i][q][e] - c2[t][e] - (y[i][t][q][e] - mn[t][e]) * is[t][e] * c3[t][e]);
          store8<T>(dyp[t] + offs[i][q], o);
        }
    }
  }
}

// all segments of one BN backward in one launch: slots of segment s at
// + s * seg_stride, its istd at + s * istd_stride; dgamma/dbeta accumulate the
// segments in order; coef[s] = {c1, c2, c3}[C]
__global__ void __launch_bounds__(256) bn_bwd_finalize_seg_kernel(const float* __restrict__ slots, int nseg,
                                                                  long long seg_stride, int C, double count,
                                                                  const float* gamma, const float* istd,
                                                                  long long istd_stride, float* dgamma, float* dbeta,
                                                                  float* coef) {
  const int c = fin_channel(), q = threadIdx.x & 3;
  for (int s0 = 0; s0 < nseg; s0 += FIN_SEGS) {
    const int ns = nseg - s0 < FIN_SEGS ? nseg - s0 : FIN_SEGS;
    double r1[FIN_SEGS], r2[FIN_SEGS];
#pragma unroll
    for (int s = 0; s < FIN_SEGS; ++s) {
      r1[s] = 0.0;
      r2[s] = 0.0;
      if (s < ns && c < C) fin_quarter(slots + (long long)(s0 + s) * seg_stride, C, c, q, r1[s], r2[s]);
    }
#pragma unroll
    for (int s = 0; s < FIN_SEGS; ++s) fin_combine(r1[s], r2[s]);
    if (q == 0 && c < C) {
      for (int s = 0; s < ns; ++s) {
        if (dbeta) dbeta[c] += (float)r1[s];
        if (dgamma) dgamma[c] += (float)r2[s];
        float* co = coef + (long long)(s0 + s) * 3 * C;
        co[c] = gamma[c] * istd[(long long)(s0 + s) * istd_stride + c];
        co[C + c] = (float)(r1[s] / count);
        co[2 * C + c] = (float)(r2[s] / count);
      }
    }
  }
}

// slots -> dgamma, dbeta (written into the parameter-gradient buffers) and the
// apply coefficients c1 = gamma*istd, c2 = sum(g)/cnt, c3 = sum(g*xhat)/cnt
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ slots, int C, double count, const float* gamma,
                                       const float* istd, float* dgamma, float* dbeta, float* coef) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s1 = 0, s2 = 0;
  for (int k = 0; k < ARTSBIR_NSLOT; ++k) {
    s1 += slots[(long long)k * 2 * C + c];
    s2 += slots[(long long)k * 2 * C + C + c];
  }
  if (dbeta) dbeta[c] += (float)s1;   // parameter gradients accumulate
  if (dgamma) dgamma[c] += (float)s2;
  coef[c] = gamma[c] * istd[c];
  coef[C + c] = (float)(s1 / count);
  coef[2 * C + c] = (float)(s2 / count);
}

// ------------------------------------------------------------------ colsum
// out[c] += sum_{r<rows} x[r*ld + c]   (x is T or f32): a 256-thread block owns
// up to 512 columns (CPR 8-column chunks) of a strip of rows; a wave reads
// 64 / CPR rows per instruction (narrow tensors — 64 columns: 8 rows — keep every
// lane busy), 8 rows in flight per lane, then one LDS reduction and ONE atomic
// per column per block (few blocks per column: the atomics on one address
// serialise in the memory-side atomic unit)
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ x, long long rows, long long ld, long long C,
                                                     long long rows_per_block, float* __restrict__ out) {
  __shared__ float red[256][9];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long cb = (long long)blockIdx.x * 512;
  const long long cw = C - cb < 512 ? C - cb : 512;  // columns of this block
  const int cpr = (int)(cw / 8);                     // 8-column chunks per row
  const int rpw = cpr >= 64 ? 1 : 64 / cpr;          // rows per wave instruction
  const int rr = lane / cpr, cc = lane - rr * cpr;
  const bool on = rr < rpw;
  const long long c0 = cb + cc * 8;
  long long r0 = blockIdx.y * rows_per_block, r1 = r0 + rows_per_block;
  if (r1 > rows) r1 = rows;
  const long long step = 4LL * rpw;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (on) {
    long long r = r0 + w * rpw + rr;
    for (; r + 7 * step < r1; r += 8 * step) {
      float v[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u) load8<T>(x + (r + u * step) * ld + c0, v[u]);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        acc[e] += ((v[0][e] + v[1][e]) + (v[2][e] + v[3][e])) + ((v[4][e] + v[5][e]) + (v[6][e] + v[7][e]));
    }
    for (; r < r1; r += step) {
      float v[8];
      load8<T>(x + r * ld + c0, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid][e] = on ? acc[e] : 0.f;
  __syncthreads();
  // column chunk q: the threads (wave, row slot) that read it
  for (int q = tid; q < cpr * 8; q += 256) {
    const int ch = q >> 3, e = q & 7;
    float s = 0.f;
    for (int ww = 0; ww < 4; ++ww)
      for (int r = 0; r < rpw; ++r) s += red[ww * 64 + r * cpr + ch][e];
    atomicAdd(out + cb + q, s);
  }
}

// ------------------------------------------------------------ casts / packs
template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, long long n) {
  // 8 elements per 16/32-B access when both pointers are 16-B aligned
  const long long n8 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) ? 0 : n / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8<TI>(x + i * 8, v);
    store8<TO>(y + i * 8, v);
  }
  for (long long i = n8 * 8 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = from_f<TO>(to_f(x[i]));
}

// src [Co][Ci][R][S] f32 (reference layout) ->
//   mode 0: dst[co][r][s][ci'] (ci' < ci_pad, zero beyond Ci)        forward operand
//   mode 1: dst[(ci*R + r)*S + s)*ldo + co] = src[co][ci][R-1-r][S-1-s]  data-gradient operand
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ src, int Co, int Ci, int R, int S, int ci_pad, int mode,
                                   long long ldo, T* __restrict__ dst) {
  const long long n = mode == 0 ? (long long)Co * R * S * ci_pad : (long long)Ci * R * S * Co;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (mode == 0) {
      int ci = (int)(i % ci_pad);
      long long t = i / ci_pad;
      int s = (int)(t % S); t /= S;
      int r = (int)(t % R);
      int co = (int)(t / R);
      float v = ci < Ci ? src[(((long long)co * Ci + ci) * R + r) * S + s] : 0.f;
      dst[i] = from_f<T>(v);
    } else {
      int co = (int)(i % Co);
      long long t = i / Co;
      int s = (int)(t % S); t /= S;
      int r = (int)(t % R);
      int ci = (int)(t / R);
      float v = src[(((long long)co * Ci + ci) * R + (R - 1 - r)) * S + (S - 1 - s)];
      dst[(((long long)ci * R + r) * S + s) * ldo + co] = from_f<T>(v);
    }
  }
}

// all packs of a model in one launch: block b finds its descriptor by binary
// search over the blk0 prefix and packs elements [1024 (b - blk0), + 1024) of it
// (mode 1: 64 x 64 tile b - blk0 of the flipped transpose)
constexpr int PACK_EPB = 1024, PACK_T = 64;
template <typename T>
__global__ void __launch_bounds__(256) pack_weights_kernel(const artsbir_pack_desc* __restrict__ tab, int n) {
  const long long b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last entry with blk0 <= b
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].blk0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const artsbir_pack_desc d = tab[lo];
  const int Co = d.Co, Ci = d.Ci, R = d.R, S = d.S;
  if (d.mode == 1) {
    // flipped transpose as a 64 x 64 tile of the [Co][Ci*R*S] source through
    // LDS: coalesced reads along k, coalesced writes along co
    __shared__ float tile[PACK_T][PACK_T + 1];
    const int RS = R * S;
    const long long K = (long long)Ci * RS, nk = (K + PACK_T - 1) / PACK_T;
    const long long t = b - d.blk0;
    const int co0 = (int)(t / nk) * PACK_T;
    const long long k0 = (t % nk) * PACK_T;
    const int col = threadIdx.x % PACK_T;
    for (int rr = threadIdx.x / PACK_T; rr < PACK_T; rr += 256 / PACK_T) {
      const int co = co0 + rr;
      const long long k = k0 + col;
      tile[rr][col] = (co < Co && k < K) ? d.src[(long long)co * K + k] : 0.f;
    }
    __syncthreads();
    for (int rr = threadIdx.x / PACK_T; rr < PACK_T; rr += 256 / PACK_T) {
      const long long k = k0 + rr;
      const int co = co0 + col;
      if (k < K && co < Co) {
        const long long ci = k / RS;
        const int rs = (int)(k - ci * RS);
        reinterpret_cast<T*>(d.dst)[(ci * RS + (RS - 1 - rs)) * d.ldo + co] = from_f<T>(tile[col][rr]);
      }
    }
    return;
  }
  const long long cnt = d.mode == 0 ? (long long)Co * R * S * d.ci_pad : Co;
  const long long i0 = (b - d.blk0) * PACK_EPB;
  for (int u = threadIdx.x; u < PACK_EPB; u += 256) {
    const long long i = i0 + u;
    if (i >= cnt) break;
    if (d.mode == 0) {
      const int ci = (int)(i % d.ci_pad);
      long long t = i / d.ci_pad;
      const int s = (int)(t % S);
      t /= S;
      const int r = (int)(t % R);
      const int co = (int)(t / R);
      const float v = ci < Ci ? d.src[(((long long)co * Ci + ci) * R + r) * S + s] : 0.f;
      reinterpret_cast<T*>(d.dst)[i] = from_f<T>(v);
    } else {
      reinterpret_cast<float*>(d.dst)[i] = d.src[i];
    }
  }
}

// wgrad workspace [Co][R][S][Cp] f32 -> += parameter-gradient layout [Co][Ci][R][S]
__global__ void unpack_wgrad_kernel(const float* __restrict__ src, int Co, int Ci, int R, int S, int Cp,
                                    float* __restrict__ dst) {
  const long long n = (long long)Co * Ci * R * S;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    int s = (int)(i % S);
    long long t = i / S;
    int r = (int)(t % R); t /= R;
    int ci = (int)(t % Ci);
    int co = (int)(t / Ci);
    dst[i] += src[(((long long)co * R + r) * S + s) * Cp + ci];  // accumulate
  }
}

// ------------------------------------------------------- attention-pool tokens
// h [B][P][C] (P = spatial positions) -> tok [B][P+1][C]:
//   tok[b][0] = mean_p h[b][p] + pos[0];  tok[b][1+p] = h[b][p] + pos[1+p]
template <typename T>
__global__ void tokens_fwd_kernel(const T* __restrict__ h, const float* __restrict__ pos, int B, int P, int C,
                                  T* __restrict__ tok) {
  const int CG = C / 8;
  const long long n = (long long)B * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long b = i / CG;
    float sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < P; ++p) {
      float v[8], pe[8];
      load8<T>(h + (b * P + p) * C + cg * 8, v);
      loadf8(pos + (long long)(p + 1) * C + cg * 8, pe);
#pragma unroll
      for (int e = 0; e < 8; ++e) { sum[e] += v[e]; v[e] += pe[e]; }
      store8<T>(tok + (b * (P + 1) + p + 1) * C + cg * 8, v);
    }
    float pe[8];
    loadf8(pos + cg * 8, pe);
#pragma unroll
    for (int e = 0; e < 8; ++e) sum[e] = sum[e] / P + pe[e];
    store8<T>(tok + (b * (P + 1)) * C + cg * 8, sum);
  }
}

// dtok [B][P+1][C] f32 -> dh [B][P][C] T: dh[b][p] = dtok[b][1+p] + dtok[b][0] / P
template <typename T>
__global__ void tokens_bwd_kernel(const float* __restrict__ dtok, int B, int P, int C, T* __restrict__ dh) {
  const int CG = C / 8;
  const long long n = (long long)B * P * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long bp = i / CG;
    const long long b = bp / P;
    const int p = (int)(bp % P);
    float d0[8], d[8];
    loadf8(dtok + (b * (P + 1)) * C + cg * 8, d0);
    loadf8(dtok + (b * (P + 1) + p + 1) * C + cg * 8, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] += d0[e] / P;
    store8<T>(dh + bp * C + cg * 8, d);
  }
}

// the same from a compute-dtype dtok whose token-0 row lacks the query
// projection's share d0 [B][C] f32 (added here): dh[b][p] = dtok[b][1+p] +
// (dtok[b][0] + d0[b]) / P
template <typename T>
__global__ void tokens_bwd_ex_kernel(const T* __restrict__ dtok, const float* __restrict__ d0, int B, int P, int C,
                                     T* __restrict__ dh) {
  const int CG = C / 8;
  const long long n = (long long)B * P * CG;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    const long long bp = i / CG;
    const long long b = bp / P;
    const int p = (int)(bp % P);
    float t0[8], e0[8], d[8];
    load8<T>(dtok + (b * (P + 1)) * C + cg * 8, t0);
    loadf8(d0 + b * C + cg * 8, e0);
    load8<T>(dtok + (b * (P + 1) + p + 1) * C + cg * 8, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] += (t0[e] + e0[e]) / P;
    store8<T>(dh + bp * C + cg * 8, d);
  }
}

}  // namespace artsbir

using namespace artsbir;

#define DISPATCH_T(dtype, ...)                      \
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

extern "C" int artsbir_pack_input(int dtype, const float* x, int B, int Cin, int H, int W, void* out, void* stream) {
  if (Cin > 8) { set_error("pack_input: Cin=%d > 8", Cin); return -1; }
  hipStream_t st = (hipStream_t)stream;
  long long n = (long long)B * H * W;
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_input_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, x, (T*)out, B, Cin, H, W));
  ARTSBIR_CHECK_LAUNCH("pack_input");
  return 0;
}

extern "C" int artsbir_bn_finalize(const float* stats, int C, double count, const float* gamma, const float* beta,
                                   float* running_mean, float* running_var, long long* num_batches_tracked,
                                   float momentum, float eps, int train, float* mean, float* istd, float* scale,
                                   float* beta_out, void* stream) {
  if (train && !stats) { set_error("bn_finalize: train mode needs stats"); return -1; }
  if (!train && (!running_mean || !running_var)) { set_error("bn_finalize: eval mode needs running stats"); return -1; }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, stats, C, count,
                     gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, train, mean, istd,
                     scale, beta_out);
  ARTSBIR_CHECK_LAUNCH("bn_finalize");
  return 0;
}

extern "C" int artsbir_bn_finalize_seg(const float* stats, int nseg, long long seg_stride, int C, double count,
                                       const float* gamma, const float* beta, float* running_mean, float* running_var,
                                       long long* num_batches_tracked, float momentum, float eps, int train,
                                       float* out, void* stream) {
  if (nseg < 1) { set_error("bn_finalize_seg: nseg=%d", nseg); return -1; }
  if (train && !stats) { set_error("bn_finalize: train mode needs stats"); return -1; }
  if (!train && (!running_mean || !running_var)) { set_error("bn_finalize: eval mode needs running stats"); return -1; }
  hipLaunchKernelGGL(bn_finalize_seg_kernel, dim3((C + FIN_CPB - 1) / FIN_CPB), dim3(256), 0, (hipStream_t)stream, stats, nseg,
                     seg_stride, C, count, gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps,
                     train, out);
  ARTSBIR_CHECK_LAUNCH("bn_finalize_seg");
  return 0;
}

extern "C" int artsbir_bn_stats_det(int dtype, const void* y, int nseg, long long rows, int C, float* stats,
                                    long long seg_stride, void* stream) {
  if (nseg < 1 || rows < 1 || C < 1 || !y || !stats) { set_error("bn_stats_det: bad arguments"); return -1; }
  if (seg_stride < (long long)ARTSBIR_NSLOT * 2 * C) { set_error("bn_stats_det: seg_stride < NSLOT*2*C"); return -1; }
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_stats_det_kernel<T>, dim3((C + 63) / 64, nseg), dim3(1024), 0,
                                       (hipStream_t)stream, (const T*)y, rows, C, stats, seg_stride));
  ARTSBIR_CHECK_LAUNCH("bn_stats_det");
  return 0;
}

extern "C" int artsbir_act_pool_colsum(int dtype, const void* x, const float* bn, int relu, int pool, int B, int H,
                                       int W, int C, int nseg, void* out, float* colsum, void* stream) {
  if (C % 8) { set_error("act_pool: C %% 8 != 0"); return -1; }
  if (nseg < 1 || B % nseg) { set_error("act_pool: %d segments do not split %d images", nseg, B); return -1; }
  if (pool > 1 && (H % pool || W % pool)) { set_error("act_pool: H,W not divisible by pool"); return -1; }
  const int Ho = pool > 1 ? H / pool : H, Wo = pool > 1 ? W / pool : W;
  long long n = (long long)B * Ho * Wo * (C / 8);
  const long long units = (long long)(B / nseg) * Ho * Wo;
  if (C / 8 <= 256 && (pool <= 1 || pool == 2) && units * C < (1LL << 40) && units < 0x7fffffffLL) {
    const int upb = cg_units_per_block(units, nseg, C);
    const dim3 g((unsigned)((units + upb - 1) / upb), (unsigned)nseg);
#define AP_GO(PV, CSV)                                                                                        \
  DISPATCH_T(dtype, hipLaunchKernelGGL((act_pool_cg_kernel<T, PV, CSV>), g, dim3(256), 0, (hipStream_t)stream, \
                                       (const T*)x, bn, relu, B / nseg, H, W, C, upb, (T*)out, colsum))
    if (pool == 2 && colsum) AP_GO(2, true);
    else if (pool == 2) AP_GO(2, false);
    else if (colsum) AP_GO(1, true);
    else AP_GO(1, false);
#undef AP_GO
    ARTSBIR_CHECK_LAUNCH("act_pool");
    return 0;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(act_pool_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)x, bn, relu, pool > 1 ? pool : 0, B, H, W, C, nseg, (T*)out));
  ARTSBIR_CHECK_LAUNCH("act_pool");
  if (colsum) {  // the generic kernel's shapes: a column-sum pass per segment into replica row 0
    const long long seg_rows = (long long)(B / nseg) * Ho * Wo, es = dtype == ARTSBIR_DT_BF16 ? 2 : 4;
    for (int s = 0; s < nseg; ++s)
      if (artsbir_colsum(dtype, reinterpret_cast<const char*>(out) + s * seg_rows * C * es, seg_rows, C, C,
                         colsum + (long long)s * ARTSBIR_NSLOT * C, stream))
        return -1;
  }
  return 0;
}

extern "C" int artsbir_act_pool(int dtype, const void* x, const float* bn, int relu, int pool, int B, int H, int W,
                                int C, int nseg, void* out, void* stream) {
  return artsbir_act_pool_colsum(dtype, x, bn, relu, pool, B, H, W, C, nseg, out, nullptr, stream);
}

extern "C" int artsbir_block_out_colsum(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                                        const void* identity, long long rows, int C, int nseg, void* out,
                                        unsigned char* mask_bits, float* colsum, void* stream) {
  if (C % 8) { set_error("block_out: C %% 8 != 0"); return -1; }
  if (nseg < 1 || rows % nseg) { set_error("block_out: %d segments do not split %lld rows", nseg, rows); return -1; }
  if (!yd && !identity) { set_error("block_out: need downsample or identity input"); return -1; }
  if (!bn3 || (yd && !bnd)) { set_error("block_out: missing BN parameter block"); return -1; }
  long long n = rows * (C / 8);
  const long long seg_rows = rows / nseg;
  if (C / 8 <= 256 && seg_rows < 0x7fffffffLL) {
    const int rpb = cg_units_per_block(seg_rows, nseg, C);
    const dim3 g((unsigned)((seg_rows + rpb - 1) / rpb), (unsigned)nseg);
    if (colsum)
      DISPATCH_T(dtype, hipLaunchKernelGGL((block_out_cg_kernel<T, true>), g, dim3(256), 0, (hipStream_t)stream,
                                           (const T*)y3, bn3, (const T*)yd, bnd, (const T*)identity, (int)seg_rows, C,
                                           rpb, (T*)out, mask_bits, colsum));
    else
      DISPATCH_T(dtype, hipLaunchKernelGGL((block_out_cg_kernel<T, false>), g, dim3(256), 0, (hipStream_t)stream,
                                           (const T*)y3, bn3, (const T*)yd, bnd, (const T*)identity, (int)seg_rows, C,
                                           rpb, (T*)out, mask_bits, nullptr));
    ARTSBIR_CHECK_LAUNCH("block_out");
    return 0;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(block_out_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)y3, bn3, (const T*)yd, bnd, (const T*)identity, rows, C, nseg,
                                       (T*)out, mask_bits));
  ARTSBIR_CHECK_LAUNCH("block_out");
  if (colsum) {  // the generic kernel's shapes: a column-sum pass per segment into replica row 0
    const long long es = dtype == ARTSBIR_DT_BF16 ? 2 : 4;
    for (int s = 0; s < nseg; ++s)
      if (artsbir_colsum(dtype, reinterpret_cast<const char*>(out) + s * seg_rows * C * es, seg_rows, C, C,
                         colsum + (long long)s * ARTSBIR_NSLOT * C, stream))
        return -1;
  }
  return 0;
}

extern "C" int artsbir_block_out_mask(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                                      const void* identity, long long rows, int C, int nseg, void* out,
                                      unsigned char* mask_bits, void* stream) {
  return artsbir_block_out_colsum(dtype, y3, bn3, yd, bnd, identity, rows, C, nseg, out, mask_bits, nullptr, stream);
}

extern "C" int artsbir_block_out(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                                 const void* identity, long long rows, int C, int nseg, void* out, void* stream) {
  return artsbir_block_out_mask(dtype, y3, bn3, yd, bnd, identity, rows, C, nseg, out, nullptr, stream);
}

static int fill_bnb(BnBwdArgs& a, const artsbir_bn_bwd_desc* d) {
  if (d->C % 8 || 256 % (d->C / 8 > 256 ? 1 : d->C / 8) || d->C / 8 > 256) {
    set_error("bn_bwd: C=%d unsupported (need C%%8==0, C/8 dividing 256)", d->C);
    return -1;
  }
  if (d->ntarget < 1 || d->ntarget > 2) { set_error("bn_bwd: ntarget must be 1 or 2"); return -1; }
  if (d->kind == 1 && d->pool > 2) { set_error("bn_bwd: pool must be <= 2"); return -1; }
  if (d->kind == 1 && d->pool == 2 && (d->H % 2 || d->W % 2)) { set_error("bn_bwd: odd H/W with pool"); return -1; }
  if (d->kind < 0 || d->kind > 3) { set_error("bn_bwd: kind must be 0 .. 3"); return -1; }
  if (d->kind != 1 && d->pool > 1) { set_error("bn_bwd: pool only with kind 1"); return -1; }
  if ((long long)d->B * d->H * d->W >= (1LL << 31)) { set_error("bn_bwd: too many pixels"); return -1; }
  a.kind = d->kind; a.pool = d->pool; a.d = d->d; a.mask = d->mask; a.mbn = d->mask_bn;
  a.ntarget = d->ntarget;
  for (int t = 0; t < 2; ++t) {
    a.y[t] = d->y[t]; a.mean[t] = d->mean[t]; a.istd[t] = d->istd[t];
    a.slots[t] = d->slots[t]; a.coef[t] = d->coef[t]; a.dy[t] = d->dy[t];
  }
  a.gout = d->gout;
  a.B = d->B; a.H = d->H; a.W = d->W; a.C = d->C;
  a.pstride = d->pstride; a.cstride = d->cstride; a.sstride = d->sstride;
  if (d->nseg > 1 && (d->pstride < 4 * (long long)d->C || d->cstride < 3 * (long long)d->C ||
                      d->sstride < 2LL * ARTSBIR_NSLOT * d->C)) {
    set_error("bn_bwd: segment strides below one parameter block");
    return -1;
  }
  return 0;
}

static int g_deterministic = 0;  // artsbir_set_deterministic

template <typename T>
static void launch_bnb(const BnBwdArgs& a, int nseg, bool reduce, hipStream_t st) {
  const int P = (a.kind == 1 && a.pool > 1) ? a.pool : 1;
  if (reduce && g_deterministic) {
#define BNB_DET(K, PP) hipLaunchKernelGGL((bn_bwd_reduce_det_kernel<T, K, PP>), dim3(1, nseg), dim3(256), 0, st, a)
    if (a.kind == 0) BNB_DET(0, 1);
    else if (a.kind == 2) BNB_DET(2, 1);
    else if (a.kind == 3) BNB_DET(3, 1);
    else if (P == 2) BNB_DET(1, 2);
    else BNB_DET(1, 1);
#undef BNB_DET
    return;
  }
  const int units = a.B * (a.H / P) * (a.W / P);
  const int RL = 256 / (a.C / 8);
  // workgroups over all segments, each walking a contiguous range of units.
  // The reduction: ~2048 (each adds one atomic per channel).  The apply: ~16384
  // but at least 8 unit rows per workgroup, so small shapes keep whole trips
  // (tools/apply_bench.py: the large shapes stream 5.0 TB/s at 2048 workgroups
  // and 5.1-5.6 at 16384, the 7^2 ones lose half their rate with one trip
  // each).  ARTSBIR_BNB_WGS / ARTSBIR_BNB_MINROWS: other targets, measurement knobs.
  static const int wgs_apply = getenv("ARTSBIR_BNB_WGS") ? atoi(getenv("ARTSBIR_BNB_WGS")) : 16384;
  static const int min_rows = getenv("ARTSBIR_BNB_MINROWS") ? atoi(getenv("ARTSBIR_BNB_MINROWS")) : 8;
  const int wgs = reduce ? 2048 : wgs_apply;
  int upb = (units * nseg + wgs - 1) / wgs;
  if (upb < RL) upb = RL;
  if (!reduce && upb < min_rows * RL) upb = min_rows * RL;
  const unsigned grid = (unsigned)((units + upb - 1) / upb);
#define BNB_LAUNCH(K, PP)                                                                                     \
  do {                                                                                                       \
    if (reduce && a.ntarget == 2)                                                                            \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, K, PP, 2>), dim3(grid, nseg), dim3(256), 0, st, a, upb);   \
    else if (reduce) hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, K, PP, 1>), dim3(grid, nseg), dim3(256), 0, st, a, upb); \
    else if (a.ntarget == 2)                                                                                 \
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, K, PP, 2>), dim3(grid, nseg), dim3(256), 0, st, a, upb);    \
    else hipLaunchKernelGGL((bn_bwd_apply_kernel<T, K, PP, 1>), dim3(grid, nseg), dim3(256), 0, st, a, upb); \
  } while (0)
  if (a.kind == 0) BNB_LAUNCH(0, 1);
  else if (a.kind == 2) BNB_LAUNCH(2, 1);
  else if (a.kind == 3) BNB_LAUNCH(3, 1);
  else if (P == 2) BNB_LAUNCH(1, 2);
  else BNB_LAUNCH(1, 1);
#undef BNB_LAUNCH
}

extern "C" int artsbir_set_deterministic(int on) {
  const int old = g_deterministic;
  g_deterministic = on ? 1 : 0;
  return old;
}

extern "C" int artsbir_bn_bwd_reduce(const artsbir_bn_bwd_desc* d, void* stream) {
  BnBwdArgs a;
  if (fill_bnb(a, d)) return -1;
  DISPATCH_T(d->dtype, launch_bnb<T>(a, d->nseg > 1 ? d->nseg : 1, true, (hipStream_t)stream));
  ARTSBIR_CHECK_LAUNCH("bn_bwd_reduce");
  return 0;
}

extern "C" int artsbir_bn_bwd_apply(const artsbir_bn_bwd_desc* d, void* stream) {
  BnBwdArgs a;
  if (fill_bnb(a, d)) return -1;
  DISPATCH_T(d->dtype, launch_bnb<T>(a, d->nseg > 1 ? d->nseg : 1, false, (hipStream_t)stream));
  ARTSBIR_CHECK_LAUNCH("bn_bwd_apply");
  return 0;
}

extern "C" int artsbir_bn_bwd_finalize_seg(const float* slots, int nseg, long long seg_stride, int C, double count,
                                           const float* gamma, const float* istd, long long istd_stride,
                                           float* dgamma, float* dbeta, float* coef, void* stream) {
  if (nseg < 1) { set_error("bn_bwd_finalize_seg: nseg=%d", nseg); return -1; }
  hipLaunchKernelGGL(bn_bwd_finalize_seg_kernel, dim3((C + FIN_CPB - 1) / FIN_CPB), dim3(256), 0, (hipStream_t)stream, slots, nseg,
                     seg_stride, C, count, gamma, istd, istd_stride, dgamma, dbeta, coef);
  ARTSBIR_CHECK_LAUNCH("bn_bwd_finalize_seg");
  return 0;
}

extern "C" int artsbir_bn_bwd_finalize(const float* slots, int C, double count, const float* gamma, const float* istd,
                                       float* dgamma, float* dbeta, float* coef, void* stream) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, slots, C, count,
                     gamma, istd, dgamma, dbeta, coef);
  ARTSBIR_CHECK_LAUNCH("bn_bwd_finalize");
  return 0;
}

// BatchNorm2d in eval mode folded into the preceding convolution:
// scale = gamma / sqrt(var + eps); w_out[co][k] = w[co][k] * scale, bias_out[co]
// = beta - mean * scale (models.py:198-236 at inference: conv -> bn -> relu)
__global__ void bn_fold_kernel(const float* __restrict__ w, int Co, long long K, const float* __restrict__ gamma,
                               const float* __restrict__ beta, const float* __restrict__ mean,
                               const float* __restrict__ var, float eps, float* __restrict__ w_out,
                               float* __restrict__ bias_out) {
  const long long n = (long long)Co * K;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i / K);
    const float sc = gamma[co] / sqrtf(var[co] + eps);
    w_out[i] = w[i] * sc;
    if (i - (long long)co * K == 0) bias_out[co] = beta[co] - mean[co] * sc;
  }
}

extern "C" int artsbir_bn_fold(const float* w, int Co, long long K, const float* gamma, const float* beta,
                               const float* mean, const float* var, float eps, float* w_out, float* bias_out,
                               void* stream) {
  if (Co <= 0 || K <= 0) { set_error("bn_fold: bad shape"); return -1; }
  hipLaunchKernelGGL(bn_fold_kernel, dim3(grid_for((long long)Co * K)), dim3(256), 0, (hipStream_t)stream, w, Co, K,
                     gamma, beta, mean, var, eps, w_out, bias_out);
  ARTSBIR_CHECK_LAUNCH("bn_fold");
  return 0;
}

extern "C" int artsbir_colsum(int dtype, const void* x, long long rows, long long ld, long long C, float* out,
                              void* stream) {
  if (C % 8 || ld % 8) { set_error("colsum: C and ld must be multiples of 8"); return -1; }
  if (rows <= 0) return 0;
  const unsigned gx = (unsigned)((C + 511) / 512);
  // about 1024 blocks in all, at least 64 rows each
  long long gy = 1024 / gx;
  if (gy < 1) gy = 1;
  long long rpb = (rows + gy - 1) / gy;
  if (rpb < 64) rpb = 64;
  gy = (rows + rpb - 1) / rpb;
  if (gy > 65535) { rpb = (rows + 65534) / 65535; gy = (rows + rpb - 1) / rpb; }
  DISPATCH_T(dtype, hipLaunchKernelGGL(colsum_kernel<T>, dim3(gx, (unsigned)gy), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)x, rows, ld, C, rpb, out));
  ARTSBIR_CHECK_LAUNCH("colsum");
  return 0;
}

extern "C" int artsbir_cast(int src_dtype, const void* x, int dst_dtype, void* y, long long n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (src_dtype == ARTSBIR_DT_F32 && dst_dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid_for((n + 7) / 8)), dim3(256), 0, st, (const float*)x, (bf16*)y, n);
  else if (src_dtype == ARTSBIR_DT_BF16 && dst_dtype == ARTSBIR_DT_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid_for((n + 7) / 8)), dim3(256), 0, st, (const bf16*)x, (float*)y, n);
  else if (src_dtype == ARTSBIR_DT_F32 && dst_dtype == ARTSBIR_DT_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(grid_for((n + 7) / 8)), dim3(256), 0, st, (const float*)x, (float*)y, n);
  else if (src_dtype == ARTSBIR_DT_BF16 && dst_dtype == ARTSBIR_DT_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(grid_for((n + 7) / 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n);
  else { set_error("cast: bad dtypes"); return -1; }
  ARTSBIR_CHECK_LAUNCH("cast");
  return 0;
}

extern "C" int artsbir_pack_weight(int dtype, const float* src, int Co, int Ci, int R, int S, int ci_pad, int mode,
                                   long long ldo, void* dst, void* stream) {
  if (mode == 0 && ci_pad < Ci) { set_error("pack_weight: ci_pad < Ci"); return -1; }
  const long long n = mode == 0 ? (long long)Co * R * S * ci_pad : (long long)Ci * R * S * Co;
  if (ldo <= 0) ldo = Co;
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_weight_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       src, Co, Ci, R, S, ci_pad, mode, ldo, (T*)dst));
  ARTSBIR_CHECK_LAUNCH("pack_weight");
  return 0;
}

extern "C" int artsbir_pack_weights(int dtype, const artsbir_pack_desc* table, int n, long long nblocks,
                                    void* stream) {
  if (n < 1 || nblocks < 1 || !table || nblocks > 0x7fffffffLL) {
    set_error("pack_weights: n=%d nblocks=%lld", n, nblocks);
    return -1;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_weights_kernel<T>, dim3((unsigned)nblocks), dim3(256), 0,
                                       (hipStream_t)stream, table, n));
  ARTSBIR_CHECK_LAUNCH("pack_weights");
  return 0;
}

extern "C" int artsbir_unpack_wgrad(const float* src, int Co, int Ci, int R, int S, int Cp, float* dst, void* stream) {
  const long long n = (long long)Co * Ci * R * S;
  hipLaunchKernelGGL(unpack_wgrad_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src, Co, Ci, R, S, Cp, dst);
  ARTSBIR_CHECK_LAUNCH("unpack_wgrad");
  return 0;
}

extern "C" int artsbir_tokens_fwd(int dtype, const void* h, const float* pos, int B, int P, int C, void* tok,
                                  void* stream) {
  if (C % 8) { set_error("tokens_fwd: C %% 8 != 0"); return -1; }
  long long n = (long long)B * (C / 8);
  DISPATCH_T(dtype, hipLaunchKernelGGL(tokens_fwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)h, pos, B, P, C, (T*)tok));
  ARTSBIR_CHECK_LAUNCH("tokens_fwd");
  return 0;
}

extern "C" int artsbir_tokens_bwd(int dtype, const float* dtok, int B, int P, int C, void* dh, void* stream) {
  if (C % 8) { set_error("tokens_bwd: C %% 8 != 0"); return -1; }
  long long n = (long long)B * P * (C / 8);
  DISPATCH_T(dtype, hipLaunchKernelGGL(tokens_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       dtok, B, P, C, (T*)dh));
  ARTSBIR_CHECK_LAUNCH("tokens_bwd");
  return 0;
}

extern "C" int artsbir_tokens_bwd_ex(int dtype, const void* dtok, const float* d0, int B, int P, int C, void* dh,
                                     void* stream) {
  if (C % 8) { set_error("tokens_bwd_ex: C %% 8 != 0"); return -1; }
  long long n = (long long)B * P * (C / 8);
  DISPATCH_T(dtype, hipLaunchKernelGGL(tokens_bwd_ex_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)dtok, d0, B, P, C, (T*)dh));
  ARTSBIR_CHECK_LAUNCH("tokens_bwd_ex");
  return 0;
}
