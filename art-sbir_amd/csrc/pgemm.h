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
  float* stats;           // optional [NSLOT][2][Cout] BN sums
  const void* res;        // optional residual (res_mode 1: same index, 2: 2x2 average-unpool)
  int res_mode;
  int dbg;                // experiment bits (ARTSBIR_PG_DBG), 0 in production
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
};
// candidate c (0 .. pwgrad_num_cfgs()-1) of the pipelined wgrad kernel;
// false, launching nothing, if it does not apply to the shape
bool pwgrad_launch(PwArgs a, int c, hipStream_t st);
int pwgrad_num_cfgs();

// Launch candidate `cfg` (0..4: tile shapes of the pipelined kernel, 10: the
// persistent streaming kernel).  Returns false, launching nothing, when the
// shape is outside what that kernel supports.
bool pgemm_launch_cfg(const PgArgs& a, int cfg, hipStream_t st);
// Heuristic candidate for a shape (-1: unsupported).
int pgemm_default_cfg(const PgArgs& a);

}  // namespace artsbir
