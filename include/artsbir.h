/*
 * libartsbir_hip — C-ABI of the MI355X (gfx950) hot path of Peer222/art-sbir.
 *
 * The reference (pure Python/PyTorch) has no FFI; its hot path is the set of
 * torch ops listed per entry point below.  These entry points are what a
 * ctypes/cffi binding from the reference's Python modules would bind
 * (INTEGRATION.md shows that binding).  Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller (e.g. the PyTorch
 *     caching allocator); the library allocates nothing and keeps no pointer;
 *   - activations are NHWC (channel innermost), channel counts % 8 == 0;
 *   - dtype is ARTSBIR_DT_F32 (parity mode) or ARTSBIR_DT_BF16 (throughput
 *     mode); statistics, gradients of parameters and optimizer state are f32;
 *   - `stream` is a hipStream_t; no entry point synchronises the device;
 *   - return 0 on success, <0 on error; artsbir_last_error() describes it.
 */
#ifndef ARTSBIR_H_
#define ARTSBIR_H_

#ifdef __cplusplus
extern "C" {
#endif

#define ARTSBIR_DT_F32 0
#define ARTSBIR_DT_BF16 1
#define ARTSBIR_NSLOT 32

/* geometry of one convolution (input NHWC [N][H][W][C], weights [Cout][R][S][C]) */
typedef struct artsbir_conv_desc {
  int dtype;
  int N, H, W, C;
  int Cout, R, S, stride, pad;
} artsbir_conv_desc;

/* ---- library ---------------------------------------------------------- */
const char* artsbir_last_error(void);
int artsbir_version(void);

/* ---- convolution / linear (models.py:198-221,310-319 nn.Conv2d; models.py:243-246 nn.Linear) */

/* y[m][n] (+)= sum_k act(Xcol[m][k]) * w[n][k] (+ bias[n]); m = (img,oh,ow).
 * act = optional per-input-channel x*in_scale+in_shift (then ReLU if in_relu);
 * zero padding is applied after act.  If stats != NULL the per-output-channel
 * sum and sum of squares (f32, before rounding y) are atomically added into
 * stats[slot][0][n] / stats[slot][1][n], slot in [0, ARTSBIR_NSLOT).
 * Replaces nn.Conv2d.forward (and the BatchNorm2d batch-statistics pass). */
int artsbir_conv2d_fwd(const artsbir_conv_desc* d, const void* x, const void* w, void* y,
                       long long ldy, int out_f32, int accumulate, const float* bias,
                       const float* in_scale, const float* in_shift, int in_relu,
                       float* stats, void* stream);

/* dw[co][r][s][ci] += sum_m dy[m][co] * act(Xcol[m][(r,s,ci)])   (f32 atomics).
 * Replaces the weight-gradient of nn.Conv2d.backward. */
int artsbir_conv2d_wgrad(const artsbir_conv_desc* d, const void* dy, const void* x,
                         const float* in_scale, const float* in_shift, int in_relu,
                         float* dw, void* stream);

/* dense c[m][n] (+)= sum_k a[m][k] * b[n][k] (+bias[n]); a row stride lda.
 * Replaces nn.Linear.forward / F.linear inside F.multi_head_attention_forward. */
int artsbir_gemm_nt(int dtype, long long M, int N, int K, const void* a, long long lda,
                    const void* b, void* c, long long ldc, int out_f32, int accumulate,
                    const float* bias, float* stats, void* stream);

/* dw[n][k] += sum_m dy[m][n] * x[m][k]  (f32 atomics) — nn.Linear weight gradient. */
int artsbir_gemm_tn(int dtype, long long M, int N, int K, const void* dy, long long ldd,
                    const void* x, long long ldx, float* dw, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ARTSBIR_H_ */
