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

// Launch candidate `cfg` (0..4: tile shapes of the pipelined kernel, 10: the
// persistent streaming kernel).  Returns false, launching nothing, when the
// shape is outside what that kernel supports.
bool pgemm_launch_cfg(const PgArgs& a, int cfg, hipStream_t st);
// Heuristic candidate for a shape (-1: unsupported).
int pgemm_default_cfg(const PgArgs& a);

}  // namespace artsbir
