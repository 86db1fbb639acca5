// Implicit-GEMM convolution / dense GEMM / weight-gradient GEMM on MFMA (gfx950).
//
// Replaces the torch ops on the reference hot path
//   nn.Conv2d (models.py:198,202,208,219 Bottleneck; models.py:310,313,316 stem)
//   nn.Linear / F.multi_head_attention_forward projections (models.py:243-246,253-271)
// forward, data-gradient and weight-gradient.
//
// One LDS image layout serves every operand of every kernel here:
//   tile[chunk g][row][16 bytes]   row stride 16 B, chunk stride (ROWS+1)*16 B
// where a 16-byte chunk holds EPC consecutive reduction ("k") elements of one
// row (EPC = 8 bf16 or 4 f32).  A 16-lane group reading 16 consecutive rows of
// one chunk with ds_read_b128 is conflict-free, and the +1 row pad makes the
// 8 lanes of a ds_write_b128 group that write 8 different chunks of one row
// land on 8 different 16-B bank slots.
//
// MFMA mapping (both dtypes use the 16x16 output layout col = lane&15,
// row = 4*(lane>>4) + reg):
//   bf16: v_mfma_f32_16x16x32_bf16, lane (i, q=lane>>4) feeds row i, chunk q
//         (8 k) -> one ds_read_b128 per fragment per 32-k step;
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32), lane (i,q) reads chunk q (4 k)
//         with one ds_read_b128 and issues 4 MFMAs, element e in step e.  The
//         k order inside the MFMA is a permutation applied identically to A
//         and B, so the sum is unchanged.
#include "common.h"

namespace artsbir {

template <typename T> struct MM;
template <> struct MM<bf16> {
  static constexpr int EPC = 8;  // elements per 16-B chunk
  typedef bf16x8 frag;
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(&a),
                                                  *reinterpret_cast<const bf16x8*>(&b), acc, 0, 0, 0);
  }
};
template <> struct MM<float> {
  static constexpr int EPC = 4;
  __device__ __forceinline__ static void mma(f32x4& acc, const uint4& a, const uint4& b) {
    const float* fa = reinterpret_cast<const float*>(&a);
    const float* fb = reinterpret_cast<const float*>(&b);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[e], fb[e], acc, 0, 0, 0);
  }
};

// ---------------------------------------------------------------------------
// Forward / data-gradient implicit GEMM:  Y[m][n] = sum_k Xcol[m][k] * W[n][k]
//   Xcol[m=(img,oh,ow)][k=(r,s,ci)] = act(X[img][oh*st-pad+r][ow*st-pad+s][ci])
//   act = optional per-input-channel affine (+ReLU); padding stays zero.
// ---------------------------------------------------------------------------
struct ConvArgs {
  const void* x;
  long long sN, sH, sW;  // element strides of x (channel stride 1)
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  const float* in_scale;
  const float* in_shift;
  int in_relu;
  const void* w;  // [Cout][K], K contiguous
  int Cout, K;
  long long M;
  void* y;
  long long ldy;
  int out_f32;
  int accumulate;
  const float* bias;
  float* stats;  // [NSLOT][2][Cout]
  const void* res;  // epilogue residual (T): mode 1 same index, mode 2 2x2 average-unpool
  int res_mode;
};

template <typename T, int BM, int BN>
__global__ void __launch_bounds__(256) conv_gemm_kernel(ConvArgs a) {
  constexpr int EPC = MM<T>::EPC;
  constexpr int BK = 8 * EPC;  // 8 chunks per K-step (128 bytes of k per row)
  constexpr int A_BYTES = 8 * (BM + 1) * 16;
  constexpr int B_BYTES = 8 * (BN + 1) * 16;
  constexpr int ARows = BM / 32;  // rows per thread in the A loader
  constexpr int BRows = BN / 32;
  constexpr int WTM = BM / 2, WTN = BN / 2;  // 2x2 waves
  constexpr int MT = WTM / 16, NT = WTN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // block -> tile; consecutive blocks walk N first so the A panel is reused from L2
  const int ntn = (a.Cout + BN - 1) / BN;
  const long long bid = blockIdx.x;
  const long long bm = (bid / ntn) * BM;
  const int bn = (int)(bid % ntn) * BN;

  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ Wt = reinterpret_cast<const T*>(a.w);

  const int lc = tid & 7;    // chunk handled by this thread
  const int lr = tid >> 3;   // first row handled by this thread
  // per-row decode of the A rows this thread loads
  long long abase[ARows];
  int aih[ARows], aiw[ARows];
  bool avalid[ARows];
  const int HoWo = a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < ARows; ++i) {
    long long gm = bm + lr + 32 * i;
    avalid[i] = gm < a.M;
    long long gmc = avalid[i] ? gm : 0;
    long long img = gmc / HoWo;
    int rem = (int)(gmc - img * HoWo);
    int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    abase[i] = img * a.sN;
    aih[i] = oh * a.stride - a.pad;
    aiw[i] = ow * a.stride - a.pad;
  }

  Vec16<T> ra[ARows], rb[BRows];

  auto load_tiles = [&](int kt) {
    const int k = kt * BK + lc * EPC;
    const bool kval = k < a.K;
    int rs = kval ? k / a.C : 0;
    int ci = k - rs * a.C;
    int r = rs / a.S, s = rs - (rs / a.S) * a.S;
    float sc[EPC], sh[EPC];
    const bool aff = a.in_scale != nullptr;
    if (aff && kval) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) { sc[e] = a.in_scale[ci + e]; sh[e] = a.in_shift[ci + e]; }
    }
#pragma unroll
    for (int i = 0; i < ARows; ++i) {
      int ih = aih[i] + r, iw = aiw[i] + s;
      bool ok = kval && avalid[i] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      if (ok) {
        ra[i] = ld16<T>(X + abase[i] + ih * a.sH + iw * a.sW + ci);
        if (aff) {
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            float v = to_f(ra[i].v[e]) * sc[e] + sh[e];
            if (a.in_relu) v = fmaxf(v, 0.f);
            ra[i].v[e] = from_f<T>(v);
          }
        }
      } else {
        ra[i] = zero16<T>();
      }
    }
#pragma unroll
    for (int i = 0; i < BRows; ++i) {
      int n = bn + lr + 32 * i;
      if (kval && n < a.Cout) rb[i] = ld16<T>(Wt + (long long)n * a.K + k);
      else rb[i] = zero16<T>();
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < ARows; ++i)
      *reinterpret_cast<uint4*>(As + (lc * (BM + 1) + lr + 32 * i) * 16) = *reinterpret_cast<uint4*>(&ra[i]);
#pragma unroll
    for (int i = 0; i < BRows; ++i)
      *reinterpret_cast<uint4*>(Bs + (lc * (BN + 1) + lr + 32 * i) * 16) = *reinterpret_cast<uint4*>(&rb[i]);
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g = kk * 4 + fq;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + (g * (BM + 1) + wm * WTM + i * 16 + fr) * 16);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + (g * (BN + 1) + wn * WTN + j * 16 + fr) * 16);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) MM<T>::mma(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // epilogue
  const int slot = (int)(bid % ARTSBIR_NSLOT);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int gn = bn + wn * WTN + j * 16 + fr;
    const bool nval = gn < a.Cout;
    const float bval = (a.bias && nval) ? a.bias[gn] : 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long gm = bm + wm * WTM + i * 16 + fq * 4 + r;
        if (nval && gm < a.M) {
          float v = acc[i][j][r] + bval;
          s1 += v;
          s2 += v * v;
          if (a.res_mode == 1) {
            v += to_f(reinterpret_cast<const T*>(a.res)[gm * a.ldy + gn]);
          } else if (a.res_mode == 2) {
            const long long img = gm / HoWo;
            const int rem = (int)(gm - img * HoWo);
            const int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
            const long long ri = (img * (a.Ho / 2) + oh / 2) * (a.Wo / 2) + ow / 2;
            v += 0.25f * to_f(reinterpret_cast<const T*>(a.res)[ri * a.ldy + gn]);
          }
          if (a.out_f32) {
            float* yp = reinterpret_cast<float*>(a.y) + gm * a.ldy + gn;
            if (a.accumulate) v += *yp;
            *yp = v;
          } else {
            reinterpret_cast<T*>(a.y)[gm * a.ldy + gn] = from_f<T>(v);
          }
        }
      }
    }
    if (a.stats) {
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0 && nval) {
        atomicAdd(a.stats + (long long)slot * 2 * a.Cout + gn, s1);
        atomicAdd(a.stats + (long long)slot * 2 * a.Cout + a.Cout + gn, s2);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient:  dW[co][k] += sum_m dY[m][co] * Xcol[m][k]
// Both operands arrive reduction-major ([m][...]); each loader unit reads an
// EPC x EPC block (EPC rows m, EPC consecutive co / ci) with 16-B coalesced
// loads and transposes it in registers (v_perm_b32 for bf16) into EPC chunks
// of the common LDS image.  The reduction over m is split across workgroups
// and combined with f32 atomics into dW.
// ---------------------------------------------------------------------------
struct WgradArgs {
  const void* dy;
  long long ldd;  // row stride of dY
  const void* x;
  long long sN, sH, sW;
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  int dense;      // Xcol[m][k] = x[m*ldx + k] (1x1, stride 1, no pad)
  long long ldx;
  const float* in_scale;
  const float* in_shift;
  int in_relu;
  int Cout, K;
  long long M;
  long long m_per_split;  // multiple of BK
  float* dw;               // [Cout][K] f32
};

__device__ __forceinline__ void transpose_unit(const Vec16<bf16> (&in)[8], Vec16<bf16> (&out)[8]) {
  const uint32_t* d[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) d[e] = reinterpret_cast<const uint32_t*>(&in[e]);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t* o0 = reinterpret_cast<uint32_t*>(&out[2 * p]);
    uint32_t* o1 = reinterpret_cast<uint32_t*>(&out[2 * p + 1]);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      o0[w] = __builtin_amdgcn_perm(d[2 * w + 1][p], d[2 * w][p], 0x05040100u);
      o1[w] = __builtin_amdgcn_perm(d[2 * w + 1][p], d[2 * w][p], 0x07060302u);
    }
  }
}
__device__ __forceinline__ void transpose_unit(const Vec16<float> (&in)[4], Vec16<float> (&out)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) out[c].v[e] = in[e].v[c];
}

template <typename T, int BM, int BN>
__global__ void __launch_bounds__(256) wgrad_kernel(WgradArgs a) {
  constexpr int EPC = MM<T>::EPC;
  constexpr int BK = 8 * EPC;
  constexpr int A_BYTES = 8 * (BM + 1) * 16;
  constexpr int B_BYTES = 8 * (BN + 1) * 16;
  constexpr int AU = 8 * (BM / EPC);  // loader units per operand
  constexpr int BU = 8 * (BN / EPC);
  constexpr int UT = (AU + BU + 255) / 256;
  static_assert(AU % 64 == 0, "A units must be wave aligned");
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = (a.K + BN - 1) / BN;
  const int ntm = (a.Cout + BM - 1) / BM;
  const int tile = blockIdx.x % (ntm * ntn);
  const int split = blockIdx.x / (ntm * ntn);
  const int bm = (tile / ntn) * BM;   // co
  const int bn = (tile % ntn) * BN;   // k
  const long long m_begin = (long long)split * a.m_per_split;
  long long m_end = m_begin + a.m_per_split;
  if (m_end > a.M) m_end = a.M;
  if (m_begin >= m_end) return;
  const int nk = (int)((m_end - m_begin + BK - 1) / BK);

  const T* __restrict__ DY = reinterpret_cast<const T*>(a.dy);
  const T* __restrict__ X = reinterpret_cast<const T*>(a.x);
  const int HoWo = a.Ho * a.Wo;

  // loader units: [0, AU) are dY^T units, [AU, AU+BU) are Xcol^T units
  Vec16<T> tu[UT][EPC];

  auto load_tiles = [&](int kt) {
    const long long m0 = m_begin + (long long)kt * BK;
#pragma unroll
    for (int t = 0; t < UT; ++t) {
      const int uu = tid + 256 * t;
      if (uu < AU) {
        const int mc = uu & 7, cc = uu >> 3;
        const int co = bm + cc * EPC;
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const long long m = m0 + mc * EPC + e;
          if (m < m_end && co < a.Cout) tu[t][e] = ld16<T>(DY + m * a.ldd + co);
          else tu[t][e] = zero16<T>();
        }
      } else if (uu < AU + BU) {
        const int u = uu - AU;
        const int mc = u & 7, cc = u >> 3;
        const int k = bn + cc * EPC;
        const bool kval = k < a.K;
        int rs = kval ? k / a.C : 0;
        int ci = k - rs * a.C;
        int r = rs / a.S, s = rs - (rs / a.S) * a.S;
        float sc[EPC], sh[EPC];
        const bool aff = a.in_scale != nullptr;
        if (aff && kval) {
#pragma unroll
          for (int e = 0; e < EPC; ++e) { sc[e] = a.in_scale[ci + e]; sh[e] = a.in_shift[ci + e]; }
        }
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const long long m = m0 + mc * EPC + e;
          bool ok = kval && m < m_end;
          long long off = 0;
          if (ok) {
            if (a.dense) {
              off = m * a.ldx + k;
            } else {
              long long img = m / HoWo;
              int rem = (int)(m - img * HoWo);
              int oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
              int ih = oh * a.stride - a.pad + r, iw = ow * a.stride - a.pad + s;
              ok = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
              off = img * a.sN + ih * a.sH + iw * a.sW + ci;
            }
          }
          if (ok) {
            tu[t][e] = ld16<T>(X + off);
            if (aff) {
#pragma unroll
              for (int q = 0; q < EPC; ++q) {
                float v = to_f(tu[t][e].v[q]) * sc[q] + sh[q];
                if (a.in_relu) v = fmaxf(v, 0.f);
                tu[t][e].v[q] = from_f<T>(v);
              }
            }
          } else {
            tu[t][e] = zero16<T>();
          }
        }
      }
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int t = 0; t < UT; ++t) {
      const int uu = tid + 256 * t;
      if (uu < AU + BU) {
        const bool isA = uu < AU;
        const int u = isA ? uu : uu - AU;
        const int mc = u & 7, cc = u >> 3;
        char* base = isA ? As + (mc * (BM + 1) + cc * EPC) * 16 : Bs + (mc * (BN + 1) + cc * EPC) * 16;
        Vec16<T> o[EPC];
        transpose_unit(tu[t], o);
#pragma unroll
        for (int c = 0; c < EPC; ++c) *reinterpret_cast<uint4*>(base + c * 16) = *reinterpret_cast<uint4*>(&o[c]);
      }
    }
  };

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int g = kk * 4 + fq;
      uint4 af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + (g * (BM + 1) + wm * WTM + i * 16 + fr) * 16);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + (g * (BN + 1) + wn * WTN + j * 16 + fr) * 16);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) MM<T>::mma(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int gk = bn + wn * WTN + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gco = bm + wm * WTM + i * 16 + fq * 4 + r;
        if (gco < a.Cout && gk < a.K) atomicAdd(a.dw + (long long)gco * a.K + gk, acc[i][j][r]);
      }
    }
}

}  // namespace artsbir

using namespace artsbir;

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
#include "../../include/artsbir.h"

static int check_conv(const artsbir_conv_desc* d) {
  if (d->C % 8 != 0) { set_error("conv: C=%d must be a multiple of 8", d->C); return -1; }
  if (d->Cout <= 0 || d->N <= 0) { set_error("conv: empty shape"); return -1; }
  if (d->R <= 0 || d->S <= 0 || d->stride <= 0 || d->pad < 0) { set_error("conv: bad geometry"); return -1; }
  return 0;
}

static void fill_geom(const artsbir_conv_desc* d, int& Ho, int& Wo) {
  Ho = (d->H + 2 * d->pad - d->R) / d->stride + 1;
  Wo = (d->W + 2 * d->pad - d->S) / d->stride + 1;
}

template <typename T>
static int launch_conv(const ConvArgs& a, hipStream_t st) {
  const bool narrow = a.Cout <= 64;
  if (narrow) {
    long long tiles = ((a.M + 127) / 128) * ((a.Cout + 63) / 64);
    hipLaunchKernelGGL((conv_gemm_kernel<T, 128, 64>), dim3((unsigned)tiles), dim3(256), 0, st, a);
  } else {
    long long tiles = ((a.M + 127) / 128) * ((a.Cout + 127) / 128);
    hipLaunchKernelGGL((conv_gemm_kernel<T, 128, 128>), dim3((unsigned)tiles), dim3(256), 0, st, a);
  }
  ARTSBIR_CHECK_LAUNCH("conv_gemm");
  return 0;
}

extern "C" int artsbir_conv2d_fwd(const artsbir_conv_desc* d, const void* x, const void* w, void* y,
                                  long long ldy, int out_f32, int accumulate, const float* bias,
                                  const float* in_scale, const float* in_shift, int in_relu,
                                  float* stats, void* stream) {
  if (check_conv(d)) return -1;
  if (accumulate && !out_f32) { set_error("conv: accumulate requires f32 output"); return -1; }
  ConvArgs a;
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  a.x = x;
  a.sW = d->C;
  a.sH = (long long)d->W * d->C;
  a.sN = (long long)d->H * d->W * d->C;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.in_scale = in_scale; a.in_shift = in_shift; a.in_relu = in_relu;
  a.w = w; a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.M = (long long)d->N * Ho * Wo;
  a.y = y; a.ldy = ldy > 0 ? ldy : d->Cout;
  a.out_f32 = out_f32; a.accumulate = accumulate; a.bias = bias; a.stats = stats;
  a.res = nullptr; a.res_mode = 0;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

extern "C" int artsbir_conv2d_dgrad(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx,
                                    const void* res, int res_mode, void* stream) {
  // data gradient of a stride-1 convolution: a convolution of dy [N][H][W][Cout]
  // with the flipped, transposed weights wd [Cin][R][S][Cout] and padding R-1-pad.
  if (d->stride != 1) { set_error("conv2d_dgrad: only stride 1 (got %d)", d->stride); return -1; }
  if (d->Cout % 8 || d->C % 8) { set_error("conv2d_dgrad: channels must be multiples of 8"); return -1; }
  if (res_mode < 0 || res_mode > 2 || (res_mode && !res)) { set_error("conv2d_dgrad: bad residual"); return -1; }
  if (res_mode == 2 && (d->H % 2 || d->W % 2)) { set_error("conv2d_dgrad: unpool residual needs even H, W"); return -1; }
  ConvArgs a;
  const int pad = d->R - 1 - d->pad;
  a.x = dy;
  a.sW = d->Cout; a.sH = (long long)d->W * d->Cout; a.sN = (long long)d->H * d->W * d->Cout;
  a.H = d->H; a.W = d->W; a.C = d->Cout;
  a.R = d->R; a.S = d->S; a.stride = 1; a.pad = pad;
  a.Ho = d->H + 2 * pad - d->R + 1; a.Wo = d->W + 2 * pad - d->S + 1;
  if (a.Ho != d->H || a.Wo != d->W) { set_error("conv2d_dgrad: only 'same' convolutions"); return -1; }
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.w = wd; a.Cout = d->C; a.K = d->R * d->S * d->Cout;
  a.M = (long long)d->N * d->H * d->W;
  a.y = dx; a.ldy = d->C;
  a.out_f32 = 0; a.accumulate = 0; a.bias = nullptr; a.stats = nullptr;
  a.res = res; a.res_mode = res_mode;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(a, st) : launch_conv<float>(a, st);
}

extern "C" int artsbir_gemm_nt(int dtype, long long M, int N, int K, const void* a, long long lda,
                               const void* b, void* c, long long ldc, int out_f32, int accumulate,
                               const float* bias, float* stats, void* stream) {
  if (K % 8 != 0 || lda % 8 != 0) { set_error("gemm_nt: K=%d and lda=%lld must be multiples of 8", K, lda); return -1; }
  if (accumulate && !out_f32) { set_error("gemm_nt: accumulate requires f32 output"); return -1; }
  if (M <= 0 || N <= 0) return 0;
  ConvArgs p;
  p.x = a; p.sN = 0; p.sH = lda; p.sW = 0;
  p.H = (int)M; p.W = 1; p.C = K;
  if (M > 0x7fffffffLL) { set_error("gemm_nt: M too large"); return -1; }
  p.R = 1; p.S = 1; p.stride = 1; p.pad = 0; p.Ho = (int)M; p.Wo = 1;
  p.in_scale = nullptr; p.in_shift = nullptr; p.in_relu = 0;
  p.w = b; p.Cout = N; p.K = K; p.M = M;
  p.y = c; p.ldy = ldc > 0 ? ldc : N;
  p.out_f32 = out_f32; p.accumulate = accumulate; p.bias = bias; p.stats = stats;
  p.res = nullptr; p.res_mode = 0;
  hipStream_t st = (hipStream_t)stream;
  return dtype == ARTSBIR_DT_BF16 ? launch_conv<bf16>(p, st) : launch_conv<float>(p, st);
}

template <typename T>
static int launch_wgrad(WgradArgs& a, hipStream_t st) {
  constexpr int BM = 128, BN = 128;
  constexpr int BK = 8 * MM<T>::EPC;
  const int tiles = ((a.Cout + BM - 1) / BM) * ((a.K + BN - 1) / BN);
  // enough workgroups to fill 256 CUs ~4 deep, but >= 8 K-steps per workgroup
  long long ksteps = (a.M + BK - 1) / BK;
  long long splits = (1024 + tiles - 1) / tiles;
  long long max_splits = (ksteps + 7) / 8;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long long per = (ksteps + splits - 1) / splits;
  a.m_per_split = per * BK;
  splits = (ksteps + per - 1) / per;
  hipLaunchKernelGGL((wgrad_kernel<T, BM, BN>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, a);
  ARTSBIR_CHECK_LAUNCH("wgrad");
  return 0;
}

extern "C" int artsbir_conv2d_wgrad(const artsbir_conv_desc* d, const void* dy, const void* x,
                                    const float* in_scale, const float* in_shift, int in_relu,
                                    float* dw, void* stream) {
  if (check_conv(d)) return -1;
  if (d->Cout % 8 != 0) { set_error("wgrad: Cout=%d must be a multiple of 8", d->Cout); return -1; }
  int Ho, Wo;
  fill_geom(d, Ho, Wo);
  WgradArgs a;
  a.dy = dy; a.ldd = d->Cout;
  a.x = x;
  a.sW = d->C; a.sH = (long long)d->W * d->C; a.sN = (long long)d->H * d->W * d->C;
  a.H = d->H; a.W = d->W; a.C = d->C;
  a.R = d->R; a.S = d->S; a.stride = d->stride; a.pad = d->pad;
  a.Ho = Ho; a.Wo = Wo;
  a.dense = (d->R == 1 && d->S == 1 && d->stride == 1 && d->pad == 0) ? 1 : 0;
  a.ldx = d->C;
  a.in_scale = in_scale; a.in_shift = in_shift; a.in_relu = in_relu;
  a.Cout = d->Cout; a.K = d->R * d->S * d->C;
  a.M = (long long)d->N * Ho * Wo;
  a.dw = dw;
  hipStream_t st = (hipStream_t)stream;
  return d->dtype == ARTSBIR_DT_BF16 ? launch_wgrad<bf16>(a, st) : launch_wgrad<float>(a, st);
}

extern "C" int artsbir_gemm_tn(int dtype, long long M, int N, int K, const void* dy, long long ldd,
                               const void* x, long long ldx, float* dw, void* stream) {
  // dw[N][K] += sum_m dy[m][n] * x[m][k]
  if (N % 8 != 0 || K % 8 != 0 || ldd % 8 != 0 || ldx % 8 != 0) {
    set_error("gemm_tn: N=%d K=%d ldd=%lld ldx=%lld must be multiples of 8", N, K, ldd, ldx);
    return -1;
  }
  if (M <= 0) return 0;
  WgradArgs a;
  a.dy = dy; a.ldd = ldd; a.x = x;
  a.sN = 0; a.sH = 0; a.sW = 0; a.H = 1; a.W = 1; a.C = K;
  a.R = 1; a.S = 1; a.stride = 1; a.pad = 0; a.Ho = 1; a.Wo = 1;
  a.dense = 1; a.ldx = ldx;
  a.in_scale = nullptr; a.in_shift = nullptr; a.in_relu = 0;
  a.Cout = N; a.K = K; a.M = M; a.dw = dw;
  hipStream_t st = (hipStream_t)stream;
  return dtype == ARTSBIR_DT_BF16 ? launch_wgrad<bf16>(a, st) : launch_wgrad<float>(a, st);
}
