// Pipelined LDS-DMA implicit-GEMM convolution (bf16, gfx950) — see pgemm.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace artsbir {

struct PgArgs {
  const void* x;          // bf16 NHWC input (forward) or dY (dgrad)
  long long x_elems;
  long long sN, sH, sW;   // element strides of x (channel stride 1)
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  const void* w;          // bf16 [Cout][K] packed weights, K = R*S*C
  int Cout, K;
  long long M;            // output pixels
  void* y;                // bf16 output [M][ldy]
  long long ldy;
  float* stats;           // optional [nseg][NSLOT][2][Cout] BN sums
  long long seg_m;        // > 0: output pixels per BN segment (one per separate forward call
                          //      of the reference; statistics kept apart), 0: one segment
  long long seg_stride;   // floats between the statistics of consecutive segments
  const void* res;        // optional residual (res_mode 1: same index, 2: 2x2 average-unpool)
  int res_mode;
  const float* bias;      // optional per-output-channel bias (added after the residual, before the ReLU)
  int relu;               // 1: ReLU on the stored output (eval-mode conv + folded BN + ReLU)
  int dbg;                // experiment bits (ARTSBIR_PG_DBG), 0 in production
  // fused BatchNorm-backward reduction (data gradient only, no stats): the
  // output d is the gradient at a BN(+ReLU) output; g = d * mask is stored and
  // sum g, sum g * xhat_t are added to bnb_slots[t] ([nseg][NSLOT][2][Cout])
  int bnb;                // 0 off; 1: mask (y_0 - mean) * scale + beta > 0; 2: mask bnb_mask > 0;
                          // 3: bnb_mask holds one bit per channel ([M][Cout/8] bytes)
  int bnb_nt;             // BN inputs sharing g (1 or 2)
  const void* bnb_y[2];   // bf16 [M][ldy] BN inputs (pre-BN convolution outputs)
  const float* bnb_mean[2];
  const float* bnb_istd[2];
  const float* bnb_mbn;   // bnb 1: parameter block [4][Cout] (mean, istd, scale, beta) of the BN before the ReLU
  const void* bnb_mask;   // bnb 2: the ReLU output (block output)
  float* bnb_slots[2];
  long long bnb_pstride;  // floats between the per-channel parameters of consecutive segments
  // BatchNorm backward folded into a 1x1 data gradient (artsbir_conv1x1_dgrad_fold):
  // the reduction operand is two tensors, k < C1 from x (C1 channels, strides
  // sN/sH/sW) and k >= C1 from x2 (C - C1 channels, strides sN2/sH2/sW2); the
  // weights and the bias differ per BN segment (w + seg * w_sstride elements,
  // bias + seg * bias_sstride floats) — kernels taking it never let a tile
  // straddle two segments
  const void* x2 = nullptr;  // nullptr: one operand
  long long x2_elems = 0;
  long long sN2 = 0, sH2 = 0, sW2 = 0;
  int C1 = 0;
  long long w_sstride = 0;
  long long bias_sstride = 0;
  // the fold's weight-gradient operands accumulated by the same pass (pstream
  // WGK variant): wg_p[seg][k][Cout] += sum_m x[m][k] x2[m][co] for k < C1 and
  // wg_gram[seg][k - C1][Cout] += sum_m x2[m][k - C1] x2[m][co] (f32, atomics)
  float* wg_p = nullptr;
  float* wg_gram = nullptr;
  // forward with BN statistics (pg_epilogue_fwd): store the output non-temporally
  // (candidates 24 / 25: the persistent kernels 10 / 15 with this set)
  int nts = 0;
};

// Weight gradient dW[co][k] += sum_m dY[m][co] * Xcol[m][k] (pwgrad.hip).
struct PwArgs {
  const void* dy;         // bf16 [M][ldd]
  long long dy_elems;
  long long ldd;
  const void* x;          // bf16 NHWC input (conv) or [M][ldx] rows (dense)
  long long x_elems;
  long long sN, sH, sW;
  int H, W, C;
  int R, S, stride, pad;
  int Ho, Wo;
  int dense;
  long long ldx;
  int Cout, K;
  long long M;
  long long m_per_split;  // set by the launcher
  float* dw;              // f32 [Cout][K], accumulated
  int dbg;                // profiling (ARTSBIR_PW_DBG): bit 0 skips the dW atomics
  // dY in two parts along Cout (dense only; the folded BatchNorm backward's
  // g^T x and x^T x in one launch, artsbir_gemm_tn2): rows co >= Cout1 read dy2
  // (column co - Cout1, row stride ldd2) and accumulate into dw2 + (co - Cout1) * K;
  // Cout1 is a multiple of the kernel's Cout tile
  const void* dy2 = nullptr;
  long long dy2_elems = 0, ldd2 = 0;
  int Cout1 = 0;
  float* dw2 = nullptr;
};
// candidate c (0 .. pwgrad_num_cfgs()-1) of the pipelined wgrad kernel;
// false, launching nothing, if it does not apply to the shape
bool pwgrad_launch(PwArgs a, int c, hipStream_t st);
// wgrad candidates 100 + level (pw256.hip): the ping-pong 256 x 256 weight-gradient
// tile, m-split over 256 << level workgroups; false outside its range
bool pw256_launch(PwArgs a, int level, hipStream_t st);
// CUs the weight-gradient grids are sized for (artsbir_set_wgrad_cus; 256 by default)
extern int g_wgrad_cus;
int pwgrad_num_cfgs();
int pwgrad_level(int c);

// Launch candidate `cfg` (0..4: tile shapes of the pipelined kernel, 10: the
// persistent streaming kernel).  Returns false, launching nothing, when the
// shape is outside what that kernel supports.
bool pgemm_launch_cfg(const PgArgs& a, int cfg, hipStream_t st);
// Candidates 22 / 23 (pp256.hip): the ping-pong 256 x 256 tile, one tile per
// workgroup / persistent over 256 workgroups; false when the shape or epilogue
// is outside it (C % 32 != 0, LDS-staged operands).
bool pp256_launch(const PgArgs& a, bool persistent, hipStream_t st);
// Candidate 26 (rstream.hip): the streaming 1x1 data gradient with a RES-kind
// fused BN-backward epilogue (K 64 / 128, C % 256 == 0); false outside it
bool rstream_launch(const PgArgs& a, hipStream_t st);
// whether a launch with a two-operand reduction / per-segment weights can be
// taken by a tile of BPX pixels (1x1 only, C1 a whole number of KS-k stages,
// segments a whole number of tiles)
inline bool pg_fold_ok(const PgArgs& a, int bpx, int ks) {
  if (!a.x2 && !a.w_sstride) return true;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0) return false;
  if (a.x2 && (a.C1 <= 0 || a.C1 % ks != 0 || a.C1 >= a.C || (a.C - a.C1) % 8 != 0)) return false;
  if ((a.w_sstride || a.bias_sstride) && a.seg_m > 0 && a.seg_m % bpx != 0) return false;
  return true;
}
// The fold's data gradient with its weight-gradient operands in the same pass
// (a.wg_p / a.wg_gram set): false, launching nothing, outside the shapes it takes
bool pg_fold_wg_launch(const PgArgs& a, hipStream_t st);
// Heuristic candidate for a shape (-1: unsupported).
int pgemm_default_cfg(const PgArgs& a);

}  // namespace artsbir
