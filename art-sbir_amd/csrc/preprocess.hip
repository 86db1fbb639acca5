// Image preprocessing on the GPU: the encoder's transform
// (/root/reference/models.py:289-295 — Resize(res, BICUBIC) of the shorter side,
// CenterCrop(res), convert('RGB'), ToTensor, Normalize(CLIP)) for a batch of
// decoded uint8 images, bit-identical to what torchvision computes through
// Pillow on the CPU:
//   * Resize: Pillow's separable resampling (Resample.c): per output pixel the
//     bicubic (a = -0.5) taps over the source span scaled by the downscale
//     factor, weights normalised in double, converted to 22-bit fixed point,
//     integer accumulation with rounding, clipped to uint8 — a horizontal pass
//     into a uint8 intermediate, then a vertical pass (only the rows / columns
//     the centre crop keeps are computed: every output pixel is independent);
//     an axis whose size does not change is not resampled (Pillow skips it);
//   * CenterCrop offsets, the resized size and "no resize when the shorter side
//     already has the target size" are decided by the host (preprocess.py),
//     exactly as torchvision does;
//   * ToTensor + Normalize: (v / 255 - mean) / std in f32, correctly rounded
//     division (no contraction possible), so the f32 output equals torch's.
// Grayscale ('L') sources are replicated to RGB after resampling (convert('RGB')).
// The weight arithmetic is kept free of FMA contraction: Pillow's double
// expressions are evaluated unfused on the CPU, and one ulp there can move a
// 22-bit weight by one.
#include "common.h"
#include "../../include/artsbir.h"

namespace artsbir {

#define PP_BITS 22

struct PrepDev {
  const unsigned char* src;
  int H, W, C, pitch;
  int rw, rh, left, top;
  int row0, nrows;        // source rows [row0, row0 + nrows) feed the crop
  long long tmp_off;      // byte offset of this image's [nrows][res][C] intermediate
};

#pragma clang fp contract(off)
__device__ __forceinline__ double pp_bicubic(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Resample.c precompute_coeffs for output index xx of an in_size -> out_size
// resize over the full box: span [xmin, xmin + n) and the normalisation sum
struct PpSpan {
  int xmin, n;
  double center, ss, ww;
};

__device__ __forceinline__ PpSpan pp_span(int in_size, int out_size, int xx) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  PpSpan s;
  s.center = (xx + 0.5) * scale;
  s.ss = 1.0 / filterscale;
  int xmin = (int)(s.center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(s.center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  s.xmin = xmin;
  s.n = xmax - xmin;
  double ww = 0.0;
  for (int x = 0; x < s.n; ++x) ww += pp_bicubic((x + xmin - s.center + 0.5) * s.ss);
  s.ww = ww;
  return s;
}

// normalize_coeffs_8bpc: the tap's weight in 22-bit fixed point
__device__ __forceinline__ int pp_weight(const PpSpan& s, int x) {
  double k = pp_bicubic((x + s.xmin - s.center + 0.5) * s.ss);
  if (s.ww != 0.0) k /= s.ww;
  return k < 0 ? (int)(-0.5 + k * (1 << PP_BITS)) : (int)(0.5 + k * (1 << PP_BITS));
}
#pragma clang fp contract(on)

__device__ __forceinline__ unsigned char pp_clip8(int v) {
  v >>= PP_BITS;  // arithmetic shift, as Pillow's clip8 table index
  return (unsigned char)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// horizontal pass: tmp[r][x][c] = row (row0 + r), crop column x, resampled W -> rw
__global__ void __launch_bounds__(256) pp_horizontal_kernel(const PrepDev* __restrict__ imgs, int res,
                                                            unsigned char* __restrict__ tmp) {
  const PrepDev d = imgs[blockIdx.y];
  const long long total = (long long)d.nrows * res;
  unsigned char* t = tmp + d.tmp_off;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += gridDim.x * 256LL) {
    const int r = (int)(i / res), x = (int)(i % res);
    const unsigned char* row = d.src + (long long)(d.row0 + r) * d.pitch;
    unsigned char* o = t + ((long long)r * res + x) * d.C;
    const int xo = d.left + x;
    if (d.rw == d.W) {  // this axis is not resampled
      for (int c = 0; c < d.C; ++c) o[c] = row[xo * d.C + c];
      continue;
    }
    const PpSpan s = pp_span(d.W, d.rw, xo);
    int acc[3] = {1 << (PP_BITS - 1), 1 << (PP_BITS - 1), 1 << (PP_BITS - 1)};
    for (int k = 0; k < s.n; ++k) {
      const int w = pp_weight(s, k);
      const unsigned char* p = row + (s.xmin + k) * d.C;
      for (int c = 0; c < d.C; ++c) acc[c] += (int)p[c] * w;
    }
    for (int c = 0; c < d.C; ++c) o[c] = pp_clip8(acc[c]);
  }
}

// vertical pass + RGB + ToTensor + Normalize: out[n][c][y][x] f32
__global__ void __launch_bounds__(256) pp_vertical_kernel(const PrepDev* __restrict__ imgs, int res,
                                                          const unsigned char* __restrict__ tmp, float m0, float m1,
                                                          float m2, float s0, float s1, float s2,
                                                          float* __restrict__ out) {
  const PrepDev d = imgs[blockIdx.y];
  const unsigned char* t = tmp + d.tmp_off;
  float* o = out + (long long)blockIdx.y * 3 * res * res;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  for (int i = blockIdx.x * 256 + threadIdx.x; i < res * res; i += gridDim.x * 256) {
    const int y = i / res, x = i % res;
    const int yo = d.top + y;
    unsigned char v[3];
    if (d.rh == d.H) {
      for (int c = 0; c < d.C; ++c) v[c] = t[((long long)(yo - d.row0) * res + x) * d.C + c];
    } else {
      const PpSpan s = pp_span(d.H, d.rh, yo);
      int acc[3] = {1 << (PP_BITS - 1), 1 << (PP_BITS - 1), 1 << (PP_BITS - 1)};
      for (int k = 0; k < s.n; ++k) {
        const int w = pp_weight(s, k);
        const unsigned char* p = t + ((long long)(s.xmin + k - d.row0) * res + x) * d.C;
        for (int c = 0; c < d.C; ++c) acc[c] += (int)p[c] * w;
      }
      for (int c = 0; c < d.C; ++c) v[c] = pp_clip8(acc[c]);
    }
    for (int c = 0; c < 3; ++c) {
      const float f = (float)v[d.C == 1 ? 0 : c] / 255.0f;
      o[(long long)c * res * res + i] = (f - mean[c]) / sd[c];
    }
  }
}

// host restatement of the span (the rows the crop needs), same arithmetic
static void pp_span_host(int in_size, int out_size, int xx, int& xmin, int& n) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double center = (xx + 0.5) * scale;
  xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  n = xmax - xmin;
}

static int pp_plan(int n, const artsbir_image_desc* descs, int res, PrepDev* out, long long& bytes) {
  long long off = ((long long)n * sizeof(PrepDev) + 255) / 256 * 256;
  for (int i = 0; i < n; ++i) {
    const artsbir_image_desc& s = descs[i];
    if (!s.src || s.H < 1 || s.W < 1 || (s.C != 1 && s.C != 3) || s.pitch < s.W * s.C) {
      set_error("clip_preprocess: image %d: bad source (C must be 1 or 3)", i);
      return -1;
    }
    if (s.rw < res || s.rh < res || s.left < 0 || s.top < 0 || s.left + res > s.rw || s.top + res > s.rh) {
      set_error("clip_preprocess: image %d: crop %dx%d at (%d,%d) outside the resized %dx%d", i, res, res, s.left,
                s.top, s.rw, s.rh);
      return -1;
    }
    int r0, r1;
    if (s.rh == s.H) {
      r0 = s.top;
      r1 = s.top + res;
    } else {
      int a, na, b, nb;
      pp_span_host(s.H, s.rh, s.top, a, na);
      pp_span_host(s.H, s.rh, s.top + res - 1, b, nb);
      r0 = a;
      r1 = b + nb;
      for (int y = s.top; y < s.top + res; ++y) {  // spans are monotone, but make sure
        int c, nc;
        pp_span_host(s.H, s.rh, y, c, nc);
        if (c < r0) r0 = c;
        if (c + nc > r1) r1 = c + nc;
      }
    }
    if (out) {
      PrepDev& d = out[i];
      d.src = s.src; d.H = s.H; d.W = s.W; d.C = s.C; d.pitch = s.pitch;
      d.rw = s.rw; d.rh = s.rh; d.left = s.left; d.top = s.top;
      d.row0 = r0; d.nrows = r1 - r0; d.tmp_off = off;
    }
    off += ((long long)(r1 - r0) * res * s.C + 255) / 256 * 256;
  }
  bytes = off;
  return 0;
}

}  // namespace artsbir

using namespace artsbir;

extern "C" long long artsbir_clip_preprocess_workspace(int n, const artsbir_image_desc* descs, int res) {
  if (n < 0 || res < 1) { set_error("clip_preprocess_workspace: bad arguments"); return -1; }
  long long bytes = 0;
  if (n && pp_plan(n, descs, res, nullptr, bytes)) return -1;
  return bytes;
}

extern "C" int artsbir_clip_preprocess(int n, const artsbir_image_desc* descs, int res, const float* mean3,
                                       const float* std3, float* out, void* workspace, long long ws_bytes,
                                       void* stream) {
  if (n < 0 || res < 1 || !mean3 || !std3 || (n && (!out || !workspace))) {
    set_error("clip_preprocess: bad arguments");
    return -1;
  }
  if (n == 0) return 0;
  PrepDev* plan = new PrepDev[n];
  long long bytes = 0;
  if (pp_plan(n, descs, res, plan, bytes)) { delete[] plan; return -1; }
  if (bytes > ws_bytes) {
    delete[] plan;
    set_error("clip_preprocess: workspace of %lld bytes, need %lld", ws_bytes, bytes);
    return -1;
  }
  hipStream_t st = (hipStream_t)stream;
  // pageable source: the copy is staged before hipMemcpyAsync returns
  hipError_t e = hipMemcpyAsync(workspace, plan, sizeof(PrepDev) * n, hipMemcpyHostToDevice, st);
  delete[] plan;
  if (e != hipSuccess) { set_error("clip_preprocess: descriptor upload: %s", hipGetErrorString(e)); return -2; }
  const PrepDev* dimgs = reinterpret_cast<const PrepDev*>(workspace);
  unsigned char* tmp = reinterpret_cast<unsigned char*>(workspace);
  const unsigned gx = (unsigned)((res * res + 255) / 256 < 64 ? (res * res + 255) / 256 : 64);
  hipLaunchKernelGGL(pp_horizontal_kernel, dim3(gx * 4, n), dim3(256), 0, st, dimgs, res, tmp);
  ARTSBIR_CHECK_LAUNCH("clip_preprocess horizontal");
  hipLaunchKernelGGL(pp_vertical_kernel, dim3(gx, n), dim3(256), 0, st, dimgs, res, tmp, mean3[0], mean3[1],
                     mean3[2], std3[0], std3[1], std3[2], out);
  ARTSBIR_CHECK_LAUNCH("clip_preprocess vertical");
  return 0;
}
