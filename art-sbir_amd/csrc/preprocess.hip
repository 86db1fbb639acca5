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
  long long tmp_off;      // byte offset of this image's planar [C][nrows][res] intermediate
  long long htab, vtab;   // byte offsets of the per-axis tap tables (-1: axis not resampled)
  int hn, vn;             // taps per table entry (entry = xmin, n, hn / vn weights)
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

// tap tables: for each crop output index i of a resampled axis, the Resample.c
// span (xmin, n) and its n 22-bit weights, computed ONCE per image and axis
// (Pillow's precompute_coeffs) instead of per output pixel and tap
__global__ void __launch_bounds__(256) pp_coeffs_kernel(const PrepDev* __restrict__ imgs, int res,
                                                        unsigned char* __restrict__ ws) {
  const PrepDev d = imgs[blockIdx.y];
  const int axis = blockIdx.z;
  const long long off = axis ? d.vtab : d.htab;
  if (off < 0) return;
  const int nt = axis ? d.vn : d.hn;
  int* tab = reinterpret_cast<int*>(ws + off);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < res; i += gridDim.x * 256) {
    const PpSpan sp = axis ? pp_span(d.H, d.rh, d.top + i) : pp_span(d.W, d.rw, d.left + i);
    int* e = tab + (long long)i * (2 + nt);
    e[0] = sp.xmin;
    e[1] = sp.n;
    for (int k = 0; k < nt; ++k) e[2 + k] = k < sp.n ? pp_weight(sp, k) : 0;
  }
}

// The intermediate is PLANAR: tmp[c][r][x], bytes, rows of res bytes, so both
// passes move 4 outputs per lane as one dword (res % 4 == 0; other widths
// take the 1-output-per-lane form of the same arithmetic).

// horizontal pass: tmp[c][r][x] = row (row0 + r), crop column x, channel c,
// resampled W -> rw; a lane makes 4 consecutive x of one row, every channel
// (one tap-table entry read per x serves all channels), and stores one dword
// per channel plane.  Source bytes come through the L1 / L2 (a row is re-read
// by its neighbouring lanes' overlapping spans).
__global__ void __launch_bounds__(256) pp_horizontal_kernel(const PrepDev* __restrict__ imgs, int res,
                                                            unsigned char* __restrict__ tmp,
                                                            const unsigned char* __restrict__ ws) {
  const PrepDev d = imgs[blockIdx.y];
  unsigned char* t = tmp + d.tmp_off;
  const int* tab = d.htab >= 0 ? reinterpret_cast<const int*>(ws + d.htab) : nullptr;
  const int C = d.C;
  const bool vec = (res & 3) == 0;
  const int xg = vec ? res / 4 : res;
  const int nx = vec ? 4 : 1;
  const long long plane = (long long)d.nrows * res;
  const long long total = (long long)d.nrows * xg;
  for (long long it = blockIdx.x * 256LL + threadIdx.x; it < total; it += gridDim.x * 256LL) {
    const int r = (int)(it / xg), g = (int)(it - (it / xg) * xg);
    const unsigned char* src = d.src + (long long)(d.row0 + r) * d.pitch;
    const int x0 = vec ? 4 * g : g;
    unsigned packed[3] = {0u, 0u, 0u};
    for (int j = 0; j < nx; ++j) {
      const int x = x0 + j;
      int acc[3] = {1 << (PP_BITS - 1), 1 << (PP_BITS - 1), 1 << (PP_BITS - 1)};
      if (!tab) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (c < C) acc[c] = (int)src[(d.left + x) * C + c] << PP_BITS;
      } else {
        const int* e = tab + (long long)x * (2 + d.hn);
        const int xmin = e[0], n = e[1];
        const unsigned char* p = src + xmin * C;
        if (C == 3) {
          for (int k = 0; k < n; ++k) {
            const int w = e[2 + k];
            acc[0] += (int)p[3 * k] * w;
            acc[1] += (int)p[3 * k + 1] * w;
            acc[2] += (int)p[3 * k + 2] * w;
          }
        } else {
          for (int k = 0; k < n; ++k) acc[0] += (int)p[k] * e[2 + k];
        }
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) packed[c] |= (unsigned)pp_clip8(acc[c]) << (8 * j);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c >= C) break;
      unsigned char* o = t + c * plane + (long long)r * res + x0;
      if (vec) *reinterpret_cast<unsigned*>(o) = packed[c];
      else *o = (unsigned char)packed[c];
    }
  }
}

// vertical pass + RGB + ToTensor + Normalize: out[n][c][y][x] f32 (or the
// uint8 HWC rows of the augmentation's input); a lane makes 4 consecutive x of
// one (channel, y): per tap one dword of the planar intermediate, 4 MACs
__global__ void __launch_bounds__(256) pp_vertical_kernel(const PrepDev* __restrict__ imgs, int res,
                                                          const unsigned char* __restrict__ tmp, float m0, float m1,
                                                          float m2, float s0, float s1, float s2,
                                                          float* __restrict__ out, unsigned char* __restrict__ out_u8) {
  const PrepDev d = imgs[blockIdx.y];
  const unsigned char* t = tmp + d.tmp_off;
  const int* tab = d.vtab >= 0 ? reinterpret_cast<const int*>(tmp + d.vtab) : nullptr;
  float* o = out ? out + (long long)blockIdx.y * 3 * res * res : nullptr;
  unsigned char* o8 = out_u8 ? out_u8 + (long long)blockIdx.y * 3 * res * res : nullptr;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  const bool vec = (res & 3) == 0;
  const int xg = vec ? res / 4 : res;
  const long long plane = (long long)d.nrows * res;
  const int total = 3 * res * xg;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int c = i / (res * xg), rem = i - c * (res * xg);
    const int y = rem / xg, g = rem - (rem / xg) * xg;
    const int cs = d.C == 1 ? 0 : c;  // convert('RGB') of a grayscale source: replicate
    const int nx = vec ? 4 : 1, x0 = vec ? 4 * g : g;
    const unsigned char* pl = t + cs * plane + x0;
    unsigned char v[4];
    if (!tab) {
      const unsigned char* p = pl + (long long)(d.top + y - d.row0) * res;
      for (int j = 0; j < nx; ++j) v[j] = p[j];
    } else {
      const int* e = tab + (long long)y * (2 + d.vn);
      const int ymin = e[0], n = e[1];
      int acc[4] = {1 << (PP_BITS - 1), 1 << (PP_BITS - 1), 1 << (PP_BITS - 1), 1 << (PP_BITS - 1)};
      const unsigned char* p = pl + (long long)(ymin - d.row0) * res;
      if (vec) {
        for (int k = 0; k < n; ++k) {
          const unsigned q = *reinterpret_cast<const unsigned*>(p + (long long)k * res);
          const int w = e[2 + k];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] += (int)((q >> (8 * j)) & 255u) * w;
        }
      } else {
        for (int k = 0; k < n; ++k) acc[0] += (int)p[(long long)k * res] * e[2 + k];
      }
      for (int j = 0; j < nx; ++j) v[j] = pp_clip8(acc[j]);
    }
    if (o8) {  // uint8 RGB rows (HWC)
      for (int j = 0; j < nx; ++j) o8[((long long)y * res + x0 + j) * 3 + c] = v[j];
      continue;
    }
    float f[4];
    for (int j = 0; j < nx; ++j) f[j] = ((float)v[j] / 255.0f - mean[c]) / sd[c];
    float* q = o + (long long)c * res * res + (long long)y * res + x0;
    if (vec) *reinterpret_cast<float4*>(q) = make_float4(f[0], f[1], f[2], f[3]);
    else q[0] = f[0];
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
    // taps per table entry: the widest span the crop's outputs use
    int hn = 0, vn = 0;
    if (s.rw != s.W)
      for (int x = s.left; x < s.left + res; ++x) {
        int a, na;
        pp_span_host(s.W, s.rw, x, a, na);
        if (na > hn) hn = na;
      }
    if (s.rh != s.H)
      for (int y = s.top; y < s.top + res; ++y) {
        int a, na;
        pp_span_host(s.H, s.rh, y, a, na);
        if (na > vn) vn = na;
      }
    const long long tmp_off = off;
    off += ((long long)(r1 - r0) * res * s.C + 255) / 256 * 256;
    long long htab = -1, vtab = -1;
    if (s.rw != s.W) { htab = off; off += ((long long)res * (2 + hn) * 4 + 255) / 256 * 256; }
    if (s.rh != s.H) { vtab = off; off += ((long long)res * (2 + vn) * 4 + 255) / 256 * 256; }
    if (out) {
      PrepDev& d = out[i];
      d.src = s.src; d.H = s.H; d.W = s.W; d.C = s.C; d.pitch = s.pitch;
      d.rw = s.rw; d.rh = s.rh; d.left = s.left; d.top = s.top;
      d.row0 = r0; d.nrows = r1 - r0; d.tmp_off = tmp_off;
      d.htab = htab; d.vtab = vtab; d.hn = hn; d.vn = vn;
    }
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

static int pp_run(int n, const artsbir_image_desc* descs, int res, const float* mean3, const float* std3, float* out,
                  unsigned char* out_u8, void* workspace, long long ws_bytes, void* stream);

extern "C" int artsbir_clip_preprocess(int n, const artsbir_image_desc* descs, int res, const float* mean3,
                                       const float* std3, float* out, void* workspace, long long ws_bytes,
                                       void* stream) {
  if (!out && n) { set_error("clip_preprocess: bad arguments"); return -1; }
  return pp_run(n, descs, res, mean3, std3, out, nullptr, workspace, ws_bytes, stream);
}

extern "C" int artsbir_resize_u8(int n, const artsbir_image_desc* descs, int res, unsigned char* out,
                                 void* workspace, long long ws_bytes, void* stream) {
  static const float zero3[3] = {0.f, 0.f, 0.f}, one3[3] = {1.f, 1.f, 1.f};
  if (!out && n) { set_error("resize_u8: bad arguments"); return -1; }
  return pp_run(n, descs, res, zero3, one3, nullptr, out, workspace, ws_bytes, stream);
}

static int pp_run(int n, const artsbir_image_desc* descs, int res, const float* mean3, const float* std3, float* out,
                  unsigned char* out_u8, void* workspace, long long ws_bytes, void* stream) {
  if (n < 0 || res < 1 || !mean3 || !std3 || (n && !workspace)) {
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
  const int xg = (res & 3) == 0 ? res / 4 : res;
  const unsigned gv = (unsigned)((3 * res * xg + 255) / 256 < 64 ? (3 * res * xg + 255) / 256 : 64);
  int maxrows = 1;
  for (int i = 0; i < n; ++i) maxrows = descs[i].H > maxrows ? descs[i].H : maxrows;
  const long long hwork = (long long)maxrows * xg;
  const unsigned gh = (unsigned)((hwork + 255) / 256 < 256 ? (hwork + 255) / 256 : 256);
  hipLaunchKernelGGL(pp_coeffs_kernel, dim3((unsigned)((res + 255) / 256), n, 2), dim3(256), 0, st, dimgs, res, tmp);
  ARTSBIR_CHECK_LAUNCH("clip_preprocess coefficients");
  hipLaunchKernelGGL(pp_horizontal_kernel, dim3(gh, n), dim3(256), 0, st, dimgs, res, tmp,
                     (const unsigned char*)tmp);
  ARTSBIR_CHECK_LAUNCH("clip_preprocess horizontal");
  hipLaunchKernelGGL(pp_vertical_kernel, dim3(gv, n), dim3(256), 0, st, dimgs, res, tmp, mean3[0], mean3[1],
                     mean3[2], std3[0], std3[1], std3[2], out, out_u8);
  ARTSBIR_CHECK_LAUNCH("clip_preprocess vertical");
  return 0;
}

namespace artsbir {
// ------------------------------------------------------------ augmentation
// The sketch augmentation of /root/reference/transformations.py:18-34 (and the
// V2 variant :37-56) on uint8 RGB rows of one size: Pillow's Image.transform as
// torchvision's PIL backend calls it, bit-identical —
//   kind 1  AFFINE, NEAREST, a[1] == a[3] == 0 (pure scale: RandomAffine with
//           degrees 0 and no shear) -> Pillow's ImagingScaleAffine: source
//           column / row by sequential double accumulation from the pixel
//           centre, xo += a[0] per column, yo += a[4] per row;
//   kind 2  AFFINE, NEAREST, general -> Pillow's 16.16 fixed-point affine
//           (coefficients converted by the host, integer increments);
//   kind 3  PERSPECTIVE, BILINEAR (RandomPerspective) -> Pillow's generic
//           transform: pixel centre through the projective map, bilinear of
//           the clipped neighbours in double, truncated to uint8;
//   kind 0  copy.
// Pixels mapped outside the source keep the fill colour (Image.transform with
// fillcolor).  Then artsbir_erase_normalize: ToTensor, up to 4 RandomErasing
// rectangles set to their value, Normalize.
struct WarpDev {
  const unsigned char* src;
  unsigned char* dst;
  int kind;
  int fx[6];        // kind 2: a0, a1, a2', a3, a4, a5' in 16.16
  double a[8];
  unsigned char fill[3];
};

#pragma clang fp contract(off)
__global__ void __launch_bounds__(256) warp_kernel(const WarpDev* __restrict__ ws, int H, int W) {
  const WarpDev d = ws[blockIdx.y];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < H * W; i += gridDim.x * 256) {
    const int y = i / W, x = i % W;
    unsigned char px[3] = {d.fill[0], d.fill[1], d.fill[2]};
    if (d.kind == 0) {
      for (int c = 0; c < 3; ++c) px[c] = d.src[(long long)i * 3 + c];
    } else if (d.kind == 1) {
      double xo = d.a[2] + d.a[0] * 0.5, yo = d.a[5] + d.a[4] * 0.5;
      for (int k = 0; k < x; ++k) xo += d.a[0];
      for (int k = 0; k < y; ++k) yo += d.a[4];
      const int xin = xo < 0.0 ? -1 : (int)xo, yin = yo < 0.0 ? -1 : (int)yo;
      if (xin >= 0 && xin < W && yin >= 0 && yin < H)
        for (int c = 0; c < 3; ++c) px[c] = d.src[((long long)yin * W + xin) * 3 + c];
    } else if (d.kind == 2) {
      const int xx = d.fx[2] + y * d.fx[1] + x * d.fx[0];
      const int yy = d.fx[5] + y * d.fx[4] + x * d.fx[3];
      const int xin = xx >> 16, yin = yy >> 16;
      if (xin >= 0 && xin < W && yin >= 0 && yin < H)
        for (int c = 0; c < 3; ++c) px[c] = d.src[((long long)yin * W + xin) * 3 + c];
    } else {
      const double xi = x + 0.5, yi = y + 0.5;
      const double den = d.a[6] * xi + d.a[7] * yi + 1;
      double xs = (d.a[0] * xi + d.a[1] * yi + d.a[2]) / den;
      double ys = (d.a[3] * xi + d.a[4] * yi + d.a[5]) / den;
      if (xs >= 0.0 && xs < W && ys >= 0.0 && ys < H) {
        xs -= 0.5;
        ys -= 0.5;
        const int x0 = xs < 0.0 ? (int)floor(xs) : (int)xs;
        const int y0 = ys < 0.0 ? (int)floor(ys) : (int)ys;
        const double dx = xs - x0, dy = ys - y0;
        const int yc = y0 < 0 ? 0 : y0 >= H ? H - 1 : y0;
        const int xa = x0 < 0 ? 0 : x0 >= W ? W - 1 : x0;
        const int xb = x0 + 1 < 0 ? 0 : x0 + 1 >= W ? W - 1 : x0 + 1;
        const bool y1ok = y0 + 1 >= 0 && y0 + 1 < H;
        for (int c = 0; c < 3; ++c) {
          const double a0 = d.src[((long long)yc * W + xa) * 3 + c], b0 = d.src[((long long)yc * W + xb) * 3 + c];
          const double v1 = a0 + (b0 - a0) * dx;
          double v2 = v1;
          if (y1ok) {
            const double a1 = d.src[((long long)(y0 + 1) * W + xa) * 3 + c];
            const double b1 = d.src[((long long)(y0 + 1) * W + xb) * 3 + c];
            v2 = a1 + (b1 - a1) * dx;
          }
          px[c] = (unsigned char)(v1 + (v2 - v1) * dy);
        }
      }
    }
    for (int c = 0; c < 3; ++c) d.dst[(long long)i * 3 + c] = px[c];
  }
}
#pragma clang fp contract(on)

struct EraseDev {
  const unsigned char* src;
  int nrect;
  int rect[4][4];     // i, j, h, w
  float value[4];
};

__global__ void __launch_bounds__(256) erase_normalize_kernel(const EraseDev* __restrict__ es, int H, int W, float m0,
                                                              float m1, float m2, float s0, float s1, float s2,
                                                              float* __restrict__ out) {
  const EraseDev e = es[blockIdx.y];
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  float* o = out + (long long)blockIdx.y * 3 * H * W;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < H * W; i += gridDim.x * 256) {
    const int y = i / W, x = i % W;
    int hit = -1;
    for (int r = 0; r < e.nrect; ++r)  // later rectangles overwrite earlier ones
      if (y >= e.rect[r][0] && y < e.rect[r][0] + e.rect[r][2] && x >= e.rect[r][1] && x < e.rect[r][1] + e.rect[r][3])
        hit = r;
    for (int c = 0; c < 3; ++c) {
      const float f = hit >= 0 ? e.value[hit] : (float)e.src[(long long)i * 3 + c] / 255.0f;
      o[(long long)c * H * W + i] = (f - mean[c]) / sd[c];
    }
  }
}

static int fix16(double v, int& out) {  // Pillow's FIX(): floor(v * 65536 + 0.5)
  const double t = v * 65536.0 + 0.5;
  const double f = t < 0.0 ? floor(t) : (double)(long long)t;
  if (f < -2147483648.0 || f > 2147483647.0) return -1;
  out = (int)f;
  return 0;
}
static bool check_fixed(const double* a, int x, int y) {
  return fabs(x * a[0] + y * a[1] + a[2]) < 32768.0 && fabs(x * a[3] + y * a[4] + a[5]) < 32768.0;
}
}  // namespace artsbir

extern "C" int artsbir_warp_u8(int n, const artsbir_warp_desc* descs, int H, int W, void* workspace,
                               long long ws_bytes, void* stream) {
  if (n < 0 || H < 1 || W < 1 || (n && (!descs || !workspace))) { set_error("warp_u8: bad arguments"); return -1; }
  if (n == 0) return 0;
  if ((long long)n * (long long)sizeof(WarpDev) > ws_bytes) { set_error("warp_u8: workspace too small"); return -1; }
  WarpDev* w = new WarpDev[n];
  for (int i = 0; i < n; ++i) {
    const artsbir_warp_desc& s = descs[i];
    WarpDev& d = w[i];
    d.src = s.src; d.dst = s.dst; d.kind = s.kind;
    for (int k = 0; k < 8; ++k) d.a[k] = s.coeffs[k];
    for (int c = 0; c < 3; ++c) d.fill[c] = s.fill[c];
    if (!s.src || !s.dst || s.kind < 0 || s.kind > 3) { delete[] w; set_error("warp_u8: image %d: bad descriptor", i); return -1; }
    if (s.kind == 1 && (s.coeffs[1] != 0.0 || s.coeffs[3] != 0.0)) {
      delete[] w; set_error("warp_u8: image %d: kind 1 is the pure-scale affine", i); return -1;
    }
    if (s.kind == 2) {
      const double* a = s.coeffs;
      if (!(check_fixed(a, 0, 0) && check_fixed(a, W, H) && check_fixed(a, 0, H) && check_fixed(a, W, 0))) {
        delete[] w; set_error("warp_u8: image %d: affine outside Pillow's fixed-point range", i); return -1;
      }
      if (fix16(a[0], d.fx[0]) || fix16(a[1], d.fx[1]) || fix16(a[3], d.fx[3]) || fix16(a[4], d.fx[4]) ||
          fix16(a[2] + a[1] * 0.5 + a[0] * 0.5, d.fx[2]) || fix16(a[5] + a[4] * 0.5 + a[3] * 0.5, d.fx[5])) {
        delete[] w; set_error("warp_u8: image %d: coefficient overflow", i); return -1;
      }
    }
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(workspace, w, sizeof(WarpDev) * n, hipMemcpyHostToDevice, st);
  delete[] w;
  if (e != hipSuccess) { set_error("warp_u8: descriptor upload: %s", hipGetErrorString(e)); return -2; }
  const unsigned gx = (unsigned)((H * W + 255) / 256 < 128 ? (H * W + 255) / 256 : 128);
  hipLaunchKernelGGL(warp_kernel, dim3(gx, n), dim3(256), 0, st, reinterpret_cast<const WarpDev*>(workspace), H, W);
  ARTSBIR_CHECK_LAUNCH("warp_u8");
  return 0;
}

extern "C" int artsbir_erase_normalize(int n, const artsbir_erase_desc* descs, int H, int W, const float* mean3,
                                       const float* std3, float* out, void* workspace, long long ws_bytes,
                                       void* stream) {
  if (n < 0 || H < 1 || W < 1 || !mean3 || !std3 || (n && (!descs || !out || !workspace))) {
    set_error("erase_normalize: bad arguments");
    return -1;
  }
  if (n == 0) return 0;
  if ((long long)n * (long long)sizeof(EraseDev) > ws_bytes) { set_error("erase_normalize: workspace too small"); return -1; }
  EraseDev* ed = new EraseDev[n];
  for (int i = 0; i < n; ++i) {
    const artsbir_erase_desc& s = descs[i];
    if (!s.src || s.nrect < 0 || s.nrect > 4) { delete[] ed; set_error("erase_normalize: image %d: bad descriptor", i); return -1; }
    ed[i].src = s.src;
    ed[i].nrect = s.nrect;
    for (int r = 0; r < 4; ++r) {
      for (int k = 0; k < 4; ++k) ed[i].rect[r][k] = s.rect[r][k];
      ed[i].value[r] = s.value[r];
    }
  }
  hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipMemcpyAsync(workspace, ed, sizeof(EraseDev) * n, hipMemcpyHostToDevice, st);
  delete[] ed;
  if (e != hipSuccess) { set_error("erase_normalize: descriptor upload: %s", hipGetErrorString(e)); return -2; }
  const unsigned gx = (unsigned)((H * W + 255) / 256 < 128 ? (H * W + 255) / 256 : 128);
  hipLaunchKernelGGL(erase_normalize_kernel, dim3(gx, n), dim3(256), 0, st,
                     reinterpret_cast<const EraseDev*>(workspace), H, W, mean3[0], mean3[1], mean3[2], std3[0],
                     std3[1], std3[2], out);
  ARTSBIR_CHECK_LAUNCH("erase_normalize");
  return 0;
}
