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
/* Name of the GEMM kernel variant the last conv2d_fwd / conv2d_dgrad / gemm_nt /
 * conv2d_wgrad / gemm_tn call on this thread launched (for per-kernel profiling). */
const char* artsbir_last_kernel(void);
/* Autotuner choices (kernel variant per conv / wgrad shape) to and from a text
 * file, so a profiled re-run launches only the steady-state kernels (no trial
 * launches).  load returns the number of entries read, or -1. */
int artsbir_tune_save(const char* path);
int artsbir_tune_load(const char* path);
/* A HIP stream restricted to the CUs set in mask (bit i of word w = CU 32w+i;
 * hipExtStreamCreateWithCUMask) and its release.  The training step runs its
 * MFMA-bound weight gradients on such a stream beside the HBM-bound data-gradient
 * chain (engine.py).  *out receives the hipStream_t. */
int artsbir_stream_create_cu_mask(const unsigned* mask, int nwords, void** out);
int artsbir_stream_destroy(void* stream);

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

/* bf16 c[m][n] = (sum_k a[m][k] * b[n][k]) * quickgelu'(x[m][n]); stats[ARTSBIR_NSLOT][2][n]
 * += column sums of c and of c^2 (f32 atomics).  Replaces, in the ViT MLP backward
 * (models.py:391-393, 412-417), the c_proj input gradient, QuickGELU.backward and
 * the c_fc bias gradient: one GEMM pass instead of a GEMM and an elementwise pass. */
int artsbir_gemm_nt_gate(long long M, int N, int K, const void* a, long long lda, const void* b, void* c,
                         long long ldc, const void* x, float* stats, void* stream);

/* dw[n][k] += sum_m dy[m][n] * x[m][k]  (f32 atomics) — nn.Linear weight gradient. */
int artsbir_gemm_tn(int dtype, long long M, int N, int K, const void* dy, long long ldd,
                    const void* x, long long ldx, float* dw, void* stream);
/* Two weight-gradient GEMMs over one x in one launch (dense rows, bf16; f32 or a
 * shape no pipelined kernel takes: two artsbir_gemm_tn):
 * dw[n][k] += sum_m dy[m][n] x[m][k] (n < N1), dw2[n][k] += sum_m dy2[m][n] x[m][k]
 * (n < N2) — the folded BatchNorm backward's g^T x and x^T x (csrc/fold.hip). */
int artsbir_gemm_tn2(int dtype, long long M, int N1, int N2, int K, const void* dy, long long ldd, const void* dy2,
                     long long ldd2, const void* x, long long ldx, float* dw, float* dw2, void* stream);

/* data gradient of a stride-1 'same' convolution: dx[m][ci] = sum dy * flipped w
 * (wd = artsbir_pack_weight mode 1, [Cin][R][S][Cout]) (+ residual: res_mode 1 =
 * res[m][ci], 2 = 0.25*res[img][oh/2][ow/2][ci], the AvgPool2d(2) backward).
 * Replaces the input-gradient of nn.Conv2d.backward (+ the residual-branch add). */
int artsbir_conv2d_dgrad(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx,
                         const void* res, int res_mode, void* stream);

/* conv2d_fwd without bias/affine, with BatchNorm statistics kept per SEGMENT:
 * the N images are nseg equal consecutive groups, each one of the reference's
 * separate forward calls (train.py:28-30 sketch / positive / negative), so one
 * launch covers them while stats[s][slot][2][Cout] hold segment s only. */
int artsbir_conv2d_fwd_seg(const artsbir_conv_desc* d, const void* x, const void* w, void* y, int nseg,
                           float* stats, void* stream);

/* y = act(conv(x) + bias[n] (+ res[m][n])), act = ReLU if relu (res_mode 0 / 1).
 * Eval-mode Conv2d + BatchNorm2d + ReLU (+ the Bottleneck's residual add) of
 * models.py:198-236 in one launch, the BatchNorm folded into w and bias by
 * artsbir_bn_fold (inference: no batch statistics, nothing else to apply). */
int artsbir_conv2d_fwd_act(const artsbir_conv_desc* d, const void* x, const void* w, void* y, const float* bias,
                           const void* res, int res_mode, int relu, void* stream);

/* conv2d_dgrad whose output is the gradient at the output of a BatchNorm2d(+ReLU)
 * (models.py:199-210, 234-235): the BN-backward reduction is fused into it.  dx
 * receives g = dx_raw * relu-mask (bnb->kind 1: mask_bn(y[0]) > 0;
 * kind 0: mask > 0, the block output; kind 3: the block output's mask bits, bf16
 * only) and bnb->slots[t] += (sum g, sum g*xhat_t)
 * exactly as artsbir_bn_bwd_reduce; finish with artsbir_bn_bwd_finalize and
 * artsbir_bn_bwd_apply of kind 2 (g given).  bnb->pool must be 0/1.  With nseg
 * segments the per-channel BN parameters of segment s are at +s*param_stride
 * floats and its slots at +s*ARTSBIR_NSLOT*2*C. */
typedef struct artsbir_bn_bwd_desc artsbir_bn_bwd_desc;
int artsbir_conv2d_dgrad_bnb(const artsbir_conv_desc* d, const void* dy, const void* wd, void* dx,
                             const void* res, int res_mode, const artsbir_bn_bwd_desc* bnb, int nseg,
                             long long param_stride, void* stream);

/* The BatchNorm2d(train) backward folded through the 1x1 Conv2d in front of it
 * (models.py:219-220 conv3 -> bn3, models.py:227-229 downsample conv -> BN;
 * replaces artsbir_bn_bwd_apply + artsbir_conv2d_dgrad of that conv, see
 * csrc/fold.hip for the algebra).  d: the FORWARD conv (x [N][H][W][C],
 * C = Ci; Cout = Co; 1x1, stride 1).  g [N][H][W][Co]: the masked gradient at
 * the BN output; x: the conv's input; w [nseg][Ci][Co + Ci] and bias
 * [nseg][Ci] f32 from artsbir_bn_fold_bwd_prep.  dx [N][H][W][Ci] =
 * [g | x] w_s^T + bias_s for the pixels of segment s (nseg equal segments of
 * the batch).  bnb (optional, kind 1, one target): dx is the gradient at the
 * output of the BN(+ReLU) feeding x; g' = dx * mask is stored and the BN
 * reduction fused as in artsbir_conv2d_dgrad_bnb (param_stride as there). */
int artsbir_conv1x1_dgrad_fold(const artsbir_conv_desc* d, const void* g, const void* x, const void* w,
                               const float* bias, void* dx, const artsbir_bn_bwd_desc* bnb, int nseg,
                               long long param_stride, void* stream);
/* artsbir_conv1x1_dgrad_fold plus the operands of the conv's weight gradient
 * through the BN (artsbir_bn_fold_wgrad_combine), from the same read of g and x:
 * P[s][co][ci] += sum over segment s of g[m][co] x[m][ci] and
 * gram[s][k][ci] += sum x[m][k] x[m][ci] (f32, accumulated: zero them first).
 * One kernel for layer-1 shapes (Ci = 64, Co = 256, bf16), else the data
 * gradient followed by artsbir_gemm_tn2 per segment. */
int artsbir_conv1x1_dgrad_fold_wg(const artsbir_conv_desc* d, const void* g, const void* x, const void* w,
                                  const float* bias, void* dx, const artsbir_bn_bwd_desc* bnb, int nseg,
                                  long long param_stride, float* P, float* gram, void* stream);
/* Weights of artsbir_conv1x1_dgrad_fold for every BN segment s:
 * wout[s][ci][co] = c1_s[co] W[co][ci], wout[s][ci][Co + k] = sum_co W[co][ci] b'_s[co] W[co][k]
 * (b' = -c1 c3 istd), bias[s][ci] = sum_co W[co][ci] (-c1 (c2 - c3 istd mean))[co].
 * wt: the conv's data-gradient operand W^T [Ci][Co] (compute dtype); coef
 * [nseg][3][Co] from artsbir_bn_bwd_finalize_seg; prm: the BN parameter blocks
 * (mean, istd, ...) [Co] of segment s at + s*pstride; amat: workspace
 * [nseg][Ci][Co] of the compute dtype. */
int artsbir_bn_fold_bwd_prep(int dtype, int Co, int Ci, const void* wt, const float* coef, const float* prm,
                             long long pstride, int nseg, void* wout, float* bias, void* amat, void* stream);
/* The weight gradient of that conv: dw[co][ci] += sum_s c1_s[co] P_s[co][ci] +
 * b'_s[co] (W Gram_s)[co][ci] + k_s[co] colsums_s[ci], with P_s = g_s^T x_s
 * [nseg][Co][Ci], Gram_s = x_s^T x_s [nseg][Ci][Ci], colsums_s = 1^T x_s
 * [nseg][cs_slots][Ci] summed over the replica rows (f32, from artsbir_gemm_tn2 and
 * artsbir_act_pool_colsum / artsbir_colsum), w the forward weight [Co][Ci]
 * (compute dtype), k = -c1 (c2 - c3 istd mean).  workspace: f32, Co * Ci *
 * (nseg + 1) floats. */
int artsbir_bn_fold_wgrad_combine(int dtype, int Co, int Ci, int nseg, const float* P, const float* gram,
                                  const float* colsums, int cs_slots, const void* w, const float* coef,
                                  const float* prm, long long pstride, float* dw, float* workspace, void* stream);

/* The y-side fold: the BatchNorm2d(train) right after a 1x1 Conv2d folded into
 * that conv's data gradient with the BN's own input y (the conv output) instead of
 * the conv input — models.py:198-199 conv1 -> bn1 of the Bottleneck, replacing
 * artsbir_bn_bwd_apply (kind 2) + artsbir_conv2d_dgrad_bnb of conv1 (see
 * csrc/fold.hip): dy = c1 g + b' y + k, so dx = [g | y] w_s^T + bias_s (+ the
 * residual: res_mode 1 res[m][ci], 2 the 2x2 average-unpool of res) for the
 * pixels of segment s.  d: the FORWARD conv (x [N][H][W][Ci], C = Ci, Cout = Co,
 * 1x1 stride 1); g, y [N][H][W][Co]; w [nseg][Ci][2 Co] and bias [nseg][Ci] from
 * artsbir_bn_fold_bwd_prep_y.  bnb (optional): the reduction of the BN(s) at
 * the block input, fused as in artsbir_conv2d_dgrad_bnb — kind 0 / 3 (1-2
 * targets, the residual required) or kind 1 (one target, no residual). */
int artsbir_conv1x1_dgrad_fold_y(const artsbir_conv_desc* d, const void* g, const void* y, const void* w,
                                 const float* bias, void* dx, const void* res, int res_mode,
                                 const artsbir_bn_bwd_desc* bnb, int nseg, long long param_stride, void* stream);
/* Weights of artsbir_conv1x1_dgrad_fold_y for every BN segment s:
 * wout[s][ci][co] = c1_s[co] W[co][ci], wout[s][ci][Co + co] = b'_s[co] W[co][ci],
 * bias[s][ci] = sum_co W[co][ci] k_s[co]  (b' = -c1 c3 istd, k = -c1 (c2 - c3 istd mean));
 * wt, coef, prm as artsbir_bn_fold_bwd_prep. */
int artsbir_bn_fold_bwd_prep_y(int dtype, int Co, int Ci, const void* wt, const float* coef, const float* prm,
                               long long pstride, int nseg, void* wout, float* bias, void* stream);
/* Its weight gradient: dw[co][ci] += sum_s c1_s[co] P_s[co][ci] + b'_s[co] Q_s[co][ci]
 * + k_s[co] colsums_s[ci] with P_s = g_s^T x_s, Q_s = y_s^T x_s ([nseg][Co][Ci] f32,
 * artsbir_gemm_tn2) and colsums [nseg][cs_slots][Ci] of the conv input x
 * (artsbir_block_out_colsum). */
int artsbir_bn_fold_wgrad_combine_y(int Co, int Ci, int nseg, const float* P, const float* Q, const float* colsums,
                                    int cs_slots, const float* coef, const float* prm, long long pstride, float* dw,
                                    void* stream);

/* ---- layout / parameter packing ---------------------------------------- */
/* x.type(weight dtype) + NCHW -> NHWC8 (models.py:352); x [B][Cin<=8][H][W] f32. */
int artsbir_pack_input(int dtype, const float* x, int B, int Cin, int H, int W, void* out, void* stream);
/* src [Co][Ci][R][S] f32 (state_dict layout) -> mode 0: [Co][R][S][ci_pad] (forward
 * operand); mode 1: flipped [Ci][R][S] rows of stride ldo (data-gradient operand). */
int artsbir_pack_weight(int dtype, const float* src, int Co, int Ci, int R, int S, int ci_pad, int mode,
                        long long ldo, void* dst, void* stream);
/* Every artsbir_pack_weight of a model in ONE launch (the re-pack after each
 * optimizer step, train.py:70 -> the next forward): `table` is a DEVICE array of
 * n descriptors; blk0 of entry i = the sum of the blocks of entries 0..i-1,
 * nblocks the total; an entry takes ceil(elements / 1024) blocks, mode 1
 * ceil(Co / 64) * ceil(Ci * R * S / 64) (64 x 64 transpose tiles).  mode 2: f32 copy of Co elements (a bias) into the
 * f32 dst.  dtype is the packed operands' dtype. */
typedef struct {
  const float* src;
  void* dst;
  int Co, Ci, R, S, ci_pad, mode;
  long long ldo;
  long long blk0;
} artsbir_pack_desc;
int artsbir_pack_weights(int dtype, const artsbir_pack_desc* table, int n, long long nblocks, void* stream);
/* wgrad workspace [Co][R][S][Cp] f32 -> dst[Co][Ci][R][S] += (parameter-gradient layout). */
int artsbir_unpack_wgrad(const float* src, int Co, int Ci, int R, int S, int Cp, float* dst, void* stream);
int artsbir_cast(int src_dtype, const void* x, int dst_dtype, void* y, long long n, void* stream);

/* ---- batch norm / activations (models.py BatchNorm2d, ReLU, AvgPool2d) -- */
/* train: mean/var from stats slots, running stats updated (momentum, unbiased
 * var), num_batches_tracked += 1; eval: from running stats.  Outputs per-channel
 * mean, istd, scale = gamma*istd and beta: the BN PARAMETER BLOCK that every
 * consumer below applies as bn(y) = (y - mean) * scale + beta (the mean is
 * subtracted first so f32 stays accurate when |mean| >> std). */
int artsbir_bn_finalize(const float* stats, int C, double count, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, long long* num_batches_tracked,
                        float momentum, float eps, int train, float* mean, float* istd, float* scale,
                        float* beta_out, void* stream);
/* artsbir_bn_finalize for the nseg BN segments of one layer in one launch
 * (segment s: stats + s*seg_stride; running statistics updated once per segment,
 * in order; num_batches_tracked += nseg); out[s][4][C] = mean, istd, scale, beta
 * (segment s's parameter block). */
int artsbir_bn_finalize_seg(const float* stats, int nseg, long long seg_stride, int C, double count,
                            const float* gamma, const float* beta, float* running_mean, float* running_var,
                            long long* num_batches_tracked, float momentum, float eps, int train, float* out,
                            void* stream);
/* Deterministic-mode BatchNorm statistics (SURVEY §5 "deterministic-kernel mode
 * for parity runs"; replaces the batch moments nn.BatchNorm2d takes in train
 * mode, models.py:199,203,209,220,311,314,317): per segment s of y
 * [nseg*rows][C], the f64 sum and sum of squares in a fixed order, written as
 * f32 hi/lo pairs to slots 0/1 of stats + s*seg_stride ([NSLOT][2][C], other
 * slots zeroed), the layout artsbir_bn_finalize_seg reads.  Bit-identical from
 * run to run (the conv epilogues' atomics are not). */
int artsbir_bn_stats_det(int dtype, const void* y, int nseg, long long rows, int C, float* stats,
                         long long seg_stride, void* stream);
/* out = avgpool_pool( relu?(bn(x)) ), bn = a [4][C] parameter block (NULL: no affine).
 * nseg segments of B/nseg images (the triplet branches): segment s uses bn + s*4*C. */
int artsbir_act_pool(int dtype, const void* x, const float* bn, int relu, int pool, int B, int H, int W, int C,
                     int nseg, void* out, void* stream);
/* The same, also accumulating the column sums of the stored output per segment:
 * colsum[s][r][c] += sum over segment s's output pixels of out[.][c], spread over
 * replica rows r < ARTSBIR_NSLOT (the consumer sums them) — the 1^T x of the folded
 * BatchNorm backward of the conv that reads out (csrc/fold.hip). */
int artsbir_act_pool_colsum(int dtype, const void* x, const float* bn, int relu, int pool, int B, int H, int W, int C,
                            int nseg, void* out, float* colsum, void* stream);
/* Bottleneck tail (models.py:234-235): out = relu(bn3(y3) + (bn_d(yd) | identity));
 * nseg segments of rows/nseg rows, segment s with the blocks + s*4*C. */
int artsbir_block_out(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                      const void* identity, long long rows, int C, int nseg, void* out, void* stream);
/* The same, also writing the block output's ReLU mask as bits: mask_bits[row][C/8],
 * bit e of byte c = out[row][8c+e] > 0 (the backward's kind-3 mask: 1/16 of the
 * bytes of re-reading out). */
int artsbir_block_out_mask(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                           const void* identity, long long rows, int C, int nseg, void* out, unsigned char* mask_bits,
                           void* stream);
/* artsbir_block_out_mask also accumulating the column sums of the stored output
 * per segment: colsum[s][r][c] += sum over segment s's rows of out[.][c], spread
 * over replica rows r < ARTSBIR_NSLOT (mask_bits optional) — the 1^T x of the
 * next block's folded conv1 (artsbir_bn_fold_wgrad_combine_y). */
int artsbir_block_out_colsum(int dtype, const void* y3, const float* bn3, const void* yd, const float* bnd,
                             const void* identity, long long rows, int C, int nseg, void* out,
                             unsigned char* mask_bits, float* colsum, void* stream);

/* BatchNorm2d(train) backward, see elementwise.hip for the math. */
struct artsbir_bn_bwd_desc {
  int dtype;
  int kind;               /* 0: g = d*(mask>0) (block output); 1: g = up(d)*(mask_bn(y[0])>0);
                             2: g = d (already masked, artsbir_conv2d_dgrad_bnb);
                             3: as 0 with mask = mask bits of artsbir_block_out_mask (reduce, dgrad_bnb) */
  int pool;               /* kind 1: d is at 1/pool resolution (AvgPool backward) */
  const void* d;
  const void* mask;
  const float* mask_bn;   /* kind 1: parameter block [4][C] of the BN feeding the ReLU */
  int ntarget;            /* 1 or 2 BN inputs sharing g */
  const void* y[2];
  const float* mean[2];
  const float* istd[2];
  float* slots[2];        /* reduce: [NSLOT][2][C] */
  const float* coef[2];   /* apply: [3][C] from artsbir_bn_bwd_finalize */
  void* dy[2];            /* apply outputs */
  void* gout;             /* apply: optional copy of g */
  int B, H, W, C;         /* per segment */
  /* nseg > 1: one launch for nseg consecutive segments (the triplet branches):
   * tensors advance by B*H*W*C elements per segment (d by its pooled size, mask
   * bits by /8), mean/istd/mask_bn by pstride, coef by cstride, slots by sstride floats */
  int nseg;
  long long pstride, cstride, sstride;
};
int artsbir_bn_bwd_reduce(const artsbir_bn_bwd_desc* d, void* stream);
/* Deterministic mode for parity runs: artsbir_bn_bwd_reduce then sums
 * in a fixed order in f64 (one workgroup, f32 hi/lo pairs in slots 0/1) instead
 * of f32 atomics.  Pair with artsbir_bn_stats_det for the forward statistics and
 * the unfused data gradients.  Returns the previous setting. */
int artsbir_set_deterministic(int on);
/* Size the weight-gradient grids (split-K targets, persistent groups) for n CUs (default 256;
 * the engine's CU-masked side stream).  Returns the previous value. */
int artsbir_set_wgrad_cus(int n);
/* dgamma += sum g*xhat, dbeta += sum g; coef = [gamma*istd, sum g/cnt, sum g*xhat/cnt]. */
int artsbir_bn_bwd_finalize(const float* slots, int C, double count, const float* gamma, const float* istd,
                            float* dgamma, float* dbeta, float* coef, void* stream);
/* the same for nseg segments in one launch: slots + s*seg_stride, istd + s*istd_stride,
 * dgamma/dbeta accumulate the segments in order, coef[s][3][C]. */
int artsbir_bn_bwd_finalize_seg(const float* slots, int nseg, long long seg_stride, int C, double count,
                                const float* gamma, const float* istd, long long istd_stride, float* dgamma,
                                float* dbeta, float* coef, void* stream);
int artsbir_bn_bwd_apply(const artsbir_bn_bwd_desc* d, void* stream);
/* BatchNorm2d (eval) folded into the preceding conv (models.py:198-236):
 * w_out[co][k] = w[co][k] * gamma/sqrt(var+eps), bias_out[co] = beta - mean*gamma/sqrt(var+eps);
 * w f32 [Co][K] in the reference layout (K = Ci*R*S). */
int artsbir_bn_fold(const float* w, int Co, long long K, const float* gamma, const float* beta, const float* mean,
                    const float* var, float eps, float* w_out, float* bias_out, void* stream);
/* out[c] += sum_r x[r*ld + c]  (bias / positional-embedding gradients). */
int artsbir_colsum(int dtype, const void* x, long long rows, long long ld, long long C, float* out, void* stream);

/* ---- attention pool (models.py:249-272) --------------------------------- */
int artsbir_tokens_fwd(int dtype, const void* h, const float* pos, int B, int P, int C, void* tok, void* stream);
int artsbir_tokens_bwd(int dtype, const float* dtok, int B, int P, int C, void* dh, void* stream);

/* the same with dtok in the compute dtype and the query projection's share of
 * the mean token's gradient d0[B][C] (f32) given apart:
 * dh[b][p] = dtok[b][1+p] + (dtok[b][0] + d0[b]) / P */
int artsbir_tokens_bwd_ex(int dtype, const void* dtok, const float* d0, int B, int P, int C, void* dh,
                          void* stream);
int artsbir_attnpool_fwd(int dtype, const float* q, const void* kv, int B, int C, int heads, int T,
                         float* p, void* o, void* stream);
int artsbir_attnpool_bwd(int dtype, const float* q, const void* kv, const float* p, const float* dout,
                         int B, int C, int heads, int T, void* dq, void* dkv, void* stream);

/* ---- transformer block (models.py:382-417) ------------------- */
/* LayerNorm computed in fp32 whatever the storage dtype (models.py:382-388):
 * y[r] = (x[r] - mean) / sqrt(var + eps) * gamma + beta, rows of C. */
int artsbir_layernorm_fwd(int dtype, const void* x, const float* gamma, const float* beta, long long rows, int C,
                          float eps, void* y, void* stream);
/* fp8 producers: the same outputs, plus max |y| of the stored values folded
 * into pmax[4096] (unsigned bits, zeroed by the caller) for
 * artsbir_quantize_fp8_pmax (the amax pass over the tensor is skipped). */
int artsbir_layernorm_fwd_pmax(int dtype, const void* x, const float* gamma, const float* beta, long long rows, int C,
                               float eps, void* y, unsigned* pmax, void* stream);
int artsbir_quickgelu_pmax(int dtype, const void* x, long long n, void* y, unsigned* pmax, void* stream);
int artsbir_mha_fwd_lse_pmax(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out,
                             float* lse, unsigned* pmax, void* stream);
/* QuickGELU (models.py:391-393): y = x * sigmoid(1.702 x), n elements. */
int artsbir_quickgelu(int dtype, const void* x, long long n, void* y, void* stream);
/* Self-attention core of nn.MultiheadAttention (models.py:399,409-411), seq-first:
 * qkv [L*N][3E] (the in-projection output, rows (position, batch)), out [L*N][E] =
 * softmax(q k^T / sqrt(64) + mask) v per head; head_dim 64, L <= 256, mask
 * [L][L] additive f32 or NULL. */
int artsbir_mha_fwd(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out,
                    void* stream);
/* The same, also writing lse[(i*N + n)*heads + h] = the log-sum-exp of each
 * score row (what the backward needs to rebuild the probabilities). */
int artsbir_mha_fwd_lse(int dtype, const void* qkv, int L, int N, int heads, const float* mask, void* out,
                        float* lse, void* stream);

/* ---- transformer block backward (the ViT-B/16 configuration C5) --------- */
/* LayerNorm backward: dx = the LayerNorm input gradient (+ dres, the residual
 * branch's gradient, when not NULL; dx may alias dres), dgamma / dbeta
 * ACCUMULATED (f32), C <= 1024. */
int artsbir_layernorm_bwd(int dtype, const void* x, const float* gamma, const void* dy, long long rows, int C,
                          float eps, const void* dres, void* dx, float* dgamma, float* dbeta, void* stream);
/* the same plus the column sums of dres and of dx added into dres_sum / dx_sum
 * (either nullable): the bias gradients of the projections before and after
 * the LayerNorm (models.py:396-417 c_proj / out_proj) in the same pass. */
int artsbir_layernorm_bwd_sums(int dtype, const void* x, const float* gamma, const void* dy, long long rows, int C,
                               float eps, const void* dres, void* dx, float* dgamma, float* dbeta, float* dres_sum,
                               float* dx_sum, void* stream);
/* QuickGELU backward: dx = dy * (s + 1.702 x s (1 - s)), s = sigmoid(1.702 x). */
int artsbir_quickgelu_bwd(int dtype, const void* x, const void* dy, long long n, void* dx, void* stream);
/* QuickGELU backward over [rows][C] with dsum[c] += sum_r dx[r][c] (the c_fc
 * bias gradient in the same pass). */
int artsbir_quickgelu_bwd_sum(int dtype, const void* x, const void* dy, long long rows, int C, void* dx, float* dsum,
                              void* stream);
/* Attention backward: dqkv [L*N][3E] (dq | dk | dv, overwritten) from qkv, the
 * forward output out, its gradient dout and lse (artsbir_mha_fwd_lse);
 * dscratch: f32 [L*N*heads] (the per-row dout . out). */
int artsbir_mha_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse, int L, int N,
                    int heads, const float* mask, void* dqkv, float* dscratch, void* stream);

/* ---- fp8 projections (configuration C5, "ViT-B/16 768-d fp8") ----------
 * q = e4m3fn(x / s) with s = amax|x| / 448 (1 when x is all zero) written to
 * scale[0] (device f32); n elements of x (dtype f32 / bf16). */
int artsbir_quantize_fp8(int dtype, const void* x, long long n, unsigned char* q, float* scale, void* stream);
/* the same for a tensor whose producer folded max |x| into the npmax partials
 * pmax (an *_pmax entry point above): no amax pass over x. */
int artsbir_quantize_fp8_pmax(int dtype, const void* x, long long n, const unsigned* pmax, int npmax,
                              unsigned char* q, float* scale, void* stream);
/* C[M][N] = sa[0] * sb[0] * sum_k A[m][k] B[n][k] (+ bias[n]) (+ C when accumulate;
 * then out_dtype must be f32) on e4m3fn operands (block-scaled MFMA, unit
 * block scales); K % 128 == 0; sa, sb, bias device f32. */
int artsbir_gemm_nt_fp8(int M, int N, int K, const unsigned char* a, const unsigned char* b, const float* sa,
                        const float* sb, const float* bias, void* c, int out_dtype, int accumulate, void* stream);
/* the same plus a bf16 residual input res[M][N] added in the epilogue, a bf16
 * copy of the result into out2[M][N] and skip_c (c is read for accumulate but
 * not written): the ViT block's residual adds and casts (models.py:412-417)
 * fused into the projections.  res / out2 nullable. */
int artsbir_gemm_nt_fp8_ex(int M, int N, int K, const unsigned char* a, const unsigned char* b, const float* sa,
                           const float* sb, const float* bias, void* c, int out_dtype, int accumulate, const void* res,
                           void* out2, int skip_c, void* stream);

/* c = f = a b^T * sa sb + bias (bf16), out2 = quickgelu(f) (bf16, from the stored f),
 * max |out2| folded into pmax[4096] (atomicMax on the f32 bits) for
 * artsbir_quantize_fp8_pmax.  Replaces c_fc + QuickGELU of the ViT MLP
 * (models.py:391-393, 412-417) in the fp8 forward: one pass instead of two. */
int artsbir_gemm_nt_fp8_gelu(int M, int N, int K, const unsigned char* a, const unsigned char* b,
                             const float* sa, const float* sb, const float* bias, void* c, void* out2,
                             unsigned* pmax, void* stream);

/* ---- ViT-B/16 embedding (CLIP VisionTransformer: conv1 patch16, class
 * token, positional embedding) ------------------------------------------ */
/* img f32 [B][3][R][R] -> rows [B*P][3*patch*patch] in conv-weight order (the
 * patch convolution as a GEMM). */
int artsbir_vit_patchify(int dtype, const float* img, int B, int R, int patch, void* out, void* stream);
/* tokens [P+1][B][E] (sequence-first): class embedding / patch rows, + pos. */
int artsbir_vit_tokens(int dtype, const void* patches, const float* cls, const float* pos, int B, int P, int E,
                       void* out, void* stream);
/* its backward: dpatches [B*P][E] (overwritten), dcls [E] and dpos [P+1][E] ACCUMULATED. */
int artsbir_vit_tokens_bwd(int dtype, const void* dtok, int B, int P, int E, void* dpatches, float* dcls,
                           float* dpos, void* stream);

/* ---- loss and optimizer (train.py:158,169) ------------------------------ */
int artsbir_triplet_fwd(const float* a, const float* p, const float* n, int B, int D, float margin, float eps,
                        float* dist, float* loss, void* stream);
int artsbir_triplet_bwd(const float* a, const float* p, const float* n, int B, int D, float margin, float eps,
                        const float* dist, const float* grad_loss, float* da, float* dp, float* dn, void* stream);
/* Adam over a device table of {param, grad, exp_avg, exp_avg_sq, numel} records
 * (host helpers size and fill the per-block table). */
long long artsbir_adam_table_blocks(const long long* numels, int ntensors, long long chunk);
int artsbir_adam_fill_table(const long long* numels, int ntensors, long long chunk, long long* table);
int artsbir_adam_step(const void* tensors, const long long* block_table, long long nblocks, long long chunk,
                      float lr, float beta1, float beta2, float eps, float weight_decay, long long step,
                      void* stream);

/* ---- retrieval (inference.py:30-69,94-136; utils.py:42) ---------------- */
/* nn.PairwiseDistance(p=2, eps): out[i] = ||x1[i] - x2[i] + eps||_2 (f32), a one-row
 * operand broadcasts.  Replaces utils.euclidean_distance. */
int artsbir_pairwise_l2(const float* x1, long long n1, const float* x2, long long n2, int D, float eps,
                        float* out, void* stream);
/* sq[i] = ||x[i]||^2 (f32) and, if xc != NULL, the compute-dtype copy of x with
 * rows zero-padded to ldc columns (the MFMA scan needs D % 64 == 0). */
int artsbir_rows_prep(int dtype, const float* x, int n, int D, float* sq, void* xc, int ldc, void* stream);
/* exact f64 distance to the positive (rows whose positive lies in [g_base, g_base+n_g)),
 * else dpos taken as given (<0: no positive); rank band lo/hi = dpos^2 -/+ eps(rel). */
int artsbir_knn_band(const float* q, const float* g, const long long* pos, long long g_base, long long n_g,
                     const float* qsq, float gsq_max, int nq, int D, float rel, double* dpos, float* lo,
                     float* hi, void* stream);
int artsbir_knn_band_from_dpos(const double* dpos, const float* qsq, float gsq_max, int nq, float rel,
                               float* lo, float* hi, void* stream);
/* candidates per query of artsbir_knn_scan for a gallery of ng rows. */
int artsbir_knn_candidates_per_query(int ng, int tiles_per_chunk);
/* fused MFMA scan: per (query, gallery chunk) the 16 smallest approximate squared
 * distances; counts of items certainly closer than the positive; queue of
 * uncertain items (unc: [unc_cap][2] int pairs followed by one int counter). */
int artsbir_knn_scan(int dtype, const void* qc, const void* gc, const float* qsq, const float* gsq, int nq,
                     int ng, int D, int tiles_per_chunk, const float* lo, const float* hi, int* cnt, int* unc,
                     int unc_cap, float* cand_d, int* cand_i, void* stream);
/* augmented bf16 gallery rows for artsbir_knn_scan_aug: xa is [n][Dp + 8] bf16, row i
 * = x[i] zero-padded to Dp columns, then the f32 bits of ||x[i]||^2 in columns
 * Dp..Dp+1 and zeros; sq[i] = ||x[i]||^2. */
int artsbir_rows_prep_aug(const float* x, int n, int D, int Dp, float* sq, void* xa, void* stream);
/* 1 if artsbir_knn_scan_aug has a kernel for this padded width (64, 128, 256, 512). */
int artsbir_knn_scan_aug_supported(int Dp);
/* the same candidate lists / counts / uncertain queue as artsbir_knn_scan (bf16), from
 * qc [nq][Dp] bf16 and the augmented gallery ga [ng][Dp + 8]: register-resident query
 * fragments, 32-row gallery tiles by LDS-DMA, 32x32x16 MFMA (inference.py:30-69).  thr0 (may be
 * NULL) seeds each query's list threshold: only items with approximate d^2 < thr0[q] enter
 * the lists (a valid seed is >= the k-th smallest approximate d^2 of the gallery + 2 eps).
 * kbound (may be NULL): [nq] shared bound, initialised to 0xFF800000 (+inf encoded); every
 * chunk publishes its k-th smallest approximate d^2 there (atomicMin of an order-preserving
 * encoding) and reads the others' every 8 tiles, using bound + 2 eps (eps = rel |q| max|g|
 * + 1e-3) as its list threshold: items at or above it cannot reach the exact top k. */
int artsbir_knn_scan_aug(const void* qc, const void* ga, const float* qsq, float gsq_max, int nq, int ng,
                         int Dp, int tiles_per_chunk, const float* thr0, unsigned* kbound, int k, float rel,
                         const float* lo, const float* hi, int* cnt, int* unc, int unc_cap, float* cand_d,
                         int* cand_i, void* stream);
/* exact f64 top-k by (distance, index) from the candidates; flag[q] = 1 when a
 * chunk list could have dropped a true top-k item (caller re-runs exhaustively). */
int artsbir_knn_merge(const float* q, const float* g, int D, int nq, int nchunks, const float* cand_d,
                      const int* cand_i, const float* qsq, float gsq_max, float rel, long long g_base, int k,
                      long long* out_i, double* out_d, int* flag, void* stream);
/* cnt[q] += #{uncertain g : d < dpos or (d == dpos and g_base+g < pos)} (exact f64). */
int artsbir_knn_uncertain(const float* q, const float* g, int D, const int* unc, int unc_cap,
                          const double* dpos, const long long* pos, long long g_base, int* cnt, void* stream);
/* out[i] = exact f64 ||q - g_i + 1e-6|| for all i (fallback / tiny galleries). */
int artsbir_knn_exact_all(const float* q, const float* g, int D, int n, double* out, void* stream);

/* ONE-CALL exact retrieval (replaces the per-query loop of inference.py:30-69:
 * utils.euclidean_distance / utils.cosine_distance of [1,D] vs the [N,D]
 * gallery, distances.topk(N, largest=False) -> position of the positive, and
 * topk(k) for get_topk_images).  metric 0: key = ||q - g + 1e-6|| (f64 from the
 * f32 rows, nn.PairwiseDistance(p=2, eps=1e-6), utils.py:42); metric 1: key =
 * 1 - q.g / (max(|q|,1e-8) max(|g|,1e-8)) (utils.py:31-40).  Order = (key,
 * gallery index), the tie rule the reference leaves unspecified.
 *   out_idx [Q][k] global indices g_base + i (-1 past the gallery), out_dist [Q][k]
 *   keys (f64, +inf past the gallery); with positives [Q] (global index, -1 =
 *   none): out_rank [Q] = #{i : (key_i, g_base+i) < (key_pos, pos)} over THIS
 *   gallery (0-based rank, inference.py:49-56), out_dpos [Q] = key of the
 *   positive (-1 if none).  dpos_in (nullable): for a shard call, the positive's
 *   key when it lives in another shard (artsbir_positive_key + a MAX all-reduce).
 * dtype: ARTSBIR_DT_BF16 (bf16 MFMA scan) or ARTSBIR_DT_F32 (f32 MFMA scan); the
 * result is exact either way.  1 <= k <= 64, N < 2^31.  tiles_per_chunk 0 = auto
 * (bf16: up to 256 tiles of 128 rows, shortened so the scan's ceil(Q/256) x
 * chunks workgroups fill whole rounds of the current device's CUs; the same
 * choice in the workspace query and the call on one device).
 * workspace: device memory of artsbir_pairwise_l2_topk_workspace() bytes.  No
 * host synchronisation; the rare fallbacks (uncertain-queue overflow, a chunk
 * list that may have hidden a top-k item) run as device kernels. */
long long artsbir_pairwise_l2_topk_workspace(int dtype, int Q, long long N, int D, int k, int tiles_per_chunk);
int artsbir_pairwise_l2_topk(int dtype, int metric, const float* q, int Q, const float* g, long long N, int D, int k,
                             const long long* positives, const double* dpos_in, long long g_base, int tiles_per_chunk,
                             long long* out_idx, double* out_dist, long long* out_rank, double* out_dpos,
                             void* workspace, long long workspace_bytes, void* stream);
/* capacity of its uncertain-item queue (default 2^20; a small value forces the
 * exhaustive recount fallback, for tests); returns the previous capacity. */
int artsbir_knn_set_unc_cap(int cap);
/* HIP-event timing of the scan kernel inside artsbir_pairwise_l2_topk (profiling):
 * on = 1 starts collecting, 0 stops; read returns the summed scan time and count. */
int artsbir_scan_profile(int on);
int artsbir_scan_profile_read(double* total_ms, int* count);
/* Diagnostics of the bf16 scan and the exact merge (env ARTSBIR_KNN_STAT=1):
 * out4 = {wave-tiles, slow-path entries, list insertions, live candidates of
 * the one-wave merge} summed since the last reset. */
int artsbir_knn_stat_read(unsigned long long* out4, int reset);
/* per-shard top-k lists gathered from nshard ranks, dist/idx [nshard][Q][k]
 * (index -1 = empty) -> global top-k by (distance, index) (sharded C4). */
int artsbir_topk_merge(int nshard, int Q, int k, const double* dist, const long long* idx, long long* out_idx,
                       double* out_dist, void* stream);
/* out[q] = exact key (metric as above) of q's positive pos[q] if it lies in rows
 * [g_base, g_base+n) of this shard g, else -1 (feeds dpos_in after a MAX all-reduce). */
int artsbir_positive_key(int metric, const float* q, int Q, const float* g, long long n, int D, const long long* pos,
                         long long g_base, double* out, void* stream);

/* backward of artsbir_pairwise_l2 (one-row operands accumulate with atomics). */
int artsbir_pairwise_l2_bwd(const float* x1, long long n1, const float* x2, long long n2, int D, float eps,
                            const float* dist, const float* gout, float* d1, float* d2, void* stream);

/* ---- heads and composite losses (models.py:363-379, utils.py:31-75) ---- */
/* y = x W^T + bias (nn.Linear of the classification heads, f32). */
int artsbir_linear_fwd(const float* x, const float* W, const float* bias, int B, int D, int C, float* y, void* stream);
/* dx = dy W; dW += dy^T x; db += colsum(dy). */
int artsbir_linear_bwd(const float* dy, const float* x, const float* W, int B, int D, int C, float* dx, float* dW,
                       float* db, void* stream);
/* nn.CrossEntropyLoss(reduction='mean', ignore_index): loss2 = {loss, #counted}; prob saved. */
int artsbir_cross_entropy_fwd(const float* logits, const long long* labels, int B, int C, long long ignore_index,
                              float* prob, float* loss2, void* stream);
int artsbir_cross_entropy_bwd(const float* prob, const long long* labels, int B, int C, long long ignore_index,
                              const float* gout, const float* loss2, float* dlogits, void* stream);
/* nn.CosineSimilarity(dim=1, eps) of row pairs (broadcasting one-row operands). */
int artsbir_cosine_fwd(const float* x1, long long n1, const float* x2, long long n2, int D, float eps, float* cosv,
                       float* norms, void* stream);
int artsbir_cosine_bwd(const float* x1, long long n1, const float* x2, long long n2, int D, const float* cosv,
                       const float* norms, const float* gcos, float* d1, float* d2, void* stream);
/* TripletMarginWithDistanceLoss hinge: loss = mean(max(0, margin + dp - dn)). */
int artsbir_hinge_fwd(const float* dp, const float* dn, int B, float margin, float* loss, void* stream);
int artsbir_hinge_bwd(const float* dp, const float* dn, int B, float margin, const float* gout, float* gdp, float* gdn,
                      void* stream);

/* ---------------------------------------------------------- preprocessing
 * The encoder's image transform on the GPU, replacing
 * /root/reference/models.py:289-295 (torchvision Resize(res, BICUBIC) ->
 * CenterCrop(res) -> convert('RGB') -> ToTensor -> Normalize(CLIP), applied by
 * Pillow per image on the CPU).  Bit-identical to the Pillow/torch result:
 * Pillow's fixed-point separable bicubic resampling (a horizontal pass into a
 * uint8 intermediate, then vertical), only the cropped pixels computed.
 * One descriptor per decoded image (device uint8 HWC rows, C = 1 'L' or 3
 * 'RGB'); rw, rh = the resized size and left, top = the crop origin, computed
 * by the caller as torchvision does (preprocess.py); rw == W (rh == H): that
 * axis is not resampled.  out: device f32 [n][3][res][res].  workspace: device
 * bytes, at least artsbir_clip_preprocess_workspace(); mean3 / std3: host. */
typedef struct artsbir_image_desc {
  const unsigned char* src;
  int H, W, C, pitch;
  int rw, rh, left, top;
} artsbir_image_desc;
long long artsbir_clip_preprocess_workspace(int n, const artsbir_image_desc* descs, int res);
int artsbir_clip_preprocess(int n, const artsbir_image_desc* descs, int res, const float* mean3, const float* std3,
                            float* out, void* workspace, long long ws_bytes, void* stream);

/* The same resize (exact target size: rw = rh = res, left = top = 0, as the
 * sketch transforms' Resize((224, 224))) into uint8 RGB rows [n][res][res][3]
 * — the input of the augmentation below. */
int artsbir_resize_u8(int n, const artsbir_image_desc* descs, int res, unsigned char* out, void* workspace,
                      long long ws_bytes, void* stream);

/* Sketch augmentation (/root/reference/transformations.py:18-56, torchvision's
 * RandomPerspective / RandomAffine through Pillow's Image.transform, and
 * RandomErasing), bit-identical to Pillow for the same parameters (the random
 * parameters are drawn on the host, preprocess.SketchAugment).  One descriptor
 * per image, all images H x W uint8 RGB rows; src and dst must not overlap.
 * kind: 0 copy, 1 AFFINE NEAREST pure scale (coeffs[1] == coeffs[3] == 0),
 * 2 AFFINE NEAREST, 3 PERSPECTIVE BILINEAR; coeffs: Pillow's data tuple (6 or
 * 8 values, the output -> input map); fill: colour of pixels mapped outside.
 * workspace: device, >= n * 160 bytes. */
typedef struct artsbir_warp_desc {
  const unsigned char* src;
  unsigned char* dst;
  int kind;
  double coeffs[8];
  unsigned char fill[3];
} artsbir_warp_desc;
int artsbir_warp_u8(int n, const artsbir_warp_desc* descs, int H, int W, void* workspace, long long ws_bytes,
                    void* stream);

/* ToTensor + RandomErasing (up to 4 rectangles (i, j, h, w), later ones on top,
 * pixels set to value) + Normalize: out f32 [n][3][H][W].  workspace: device,
 * >= n * 96 bytes. */
typedef struct artsbir_erase_desc {
  const unsigned char* src;
  int nrect;
  int rect[4][4];
  float value[4];
} artsbir_erase_desc;
int artsbir_erase_normalize(int n, const artsbir_erase_desc* descs, int H, int W, const float* mean3,
                            const float* std3, float* out, void* workspace, long long ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ARTSBIR_H_ */
