// Plain bf16 NT GEMMs through hipBLASLt: an autotuner candidate (-3) for the
// dense projections that carry no fused epilogue (the ViT's data gradients,
// models.py:396-417 backward; the attention-pool projections models.py:243-246),
// timed against the library's own pgemm tiles per shape; the fused convolution
// epilogues (BN statistics, BN backward, residual, gate) stay on pgemm.
//
// Row-major C[M][N] = A[M][K] * B[N][K]^T is the column-major product
//   D (N x M, ld ldc) = op(B) (N x K) * op(A) (K x M)
// with B stored column-major K x N (ld K, transposed) and A column-major
// K x M (ld lda, not transposed).
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "pgemm.h"

namespace artsbir {

namespace {
struct BltPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};
using BltKey = std::tuple<long long, int, int, long long, long long, bool>;
std::mutex g_blt_mu;
hipblasLtHandle_t g_blt = nullptr;
void* g_blt_ws = nullptr;
constexpr size_t kBltWs = 64ull << 20;
std::map<BltKey, BltPlan> g_blt_plans;

bool blt_init() {
  if (g_blt) return true;
  if (hipblasLtCreate(&g_blt) != HIPBLAS_STATUS_SUCCESS) { g_blt = nullptr; return false; }
  if (hipMalloc(&g_blt_ws, kBltWs) != hipSuccess) { g_blt_ws = nullptr; return false; }
  return true;
}

BltPlan make_plan(long long M, int N, int K, long long lda, long long ldc, const float* bias) {
  BltPlan pl;
  const hipblasOperation_t tA = HIPBLAS_OP_T, tB = HIPBLAS_OP_N;
  if (hipblasLtMatmulDescCreate(&pl.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return pl;
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA));
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB));
  if (bias) {  // f32 bias per row of D = per output column of the row-major C
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep));
    hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
  }
  if (hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, (uint64_t)K, (uint64_t)N, (int64_t)K) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, (uint64_t)K, (uint64_t)M, (int64_t)lda) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lc, HIP_R_16BF, (uint64_t)N, (uint64_t)M, (int64_t)ldc) != HIPBLAS_STATUS_SUCCESS)
    return pl;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return pl;
  const uint64_t wsmax = kBltWs;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax, sizeof(wsmax));
  hipblasLtMatmulHeuristicResult_t res[1];
  int nres = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(g_blt, pl.op, pl.la, pl.lb, pl.lc, pl.lc, pref, 1, res, &nres);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || nres < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) return pl;
  pl.algo = res[0].algo;
  pl.ws = res[0].workspaceSize;
  pl.ok = pl.ws <= kBltWs;
  return pl;
}
// dW (f32, [Cout][K] row-major) += dY^T X over M rows: column-major
//   dW^T (K x Cout, ld K) = X (K x M, ld ldx) * op(dY) (M x Cout), dY stored
//   column-major Cout x M (ld ldd, transposed); beta = 1 accumulates
using BltWKey = std::tuple<long long, int, int, long long, long long>;
std::map<BltWKey, BltPlan> g_blt_wplans;

BltPlan make_wplan(long long M, int Cout, int K, long long ldx, long long ldd) {
  BltPlan pl;
  const hipblasOperation_t tA = HIPBLAS_OP_N, tB = HIPBLAS_OP_T;
  if (hipblasLtMatmulDescCreate(&pl.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return pl;
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSA, &tA, sizeof(tA));
  hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tB, sizeof(tB));
  if (hipblasLtMatrixLayoutCreate(&pl.la, HIP_R_16BF, (uint64_t)K, (uint64_t)M, (int64_t)ldx) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lb, HIP_R_16BF, (uint64_t)Cout, (uint64_t)M, (int64_t)ldd) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&pl.lc, HIP_R_32F, (uint64_t)K, (uint64_t)Cout, (int64_t)K) != HIPBLAS_STATUS_SUCCESS)
    return pl;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return pl;
  const uint64_t wsmax = kBltWs;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax, sizeof(wsmax));
  hipblasLtMatmulHeuristicResult_t res[1];
  int nres = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(g_blt, pl.op, pl.la, pl.lb, pl.lc, pl.lc, pref, 1, res, &nres);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || nres < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) return pl;
  pl.algo = res[0].algo;
  pl.ws = res[0].workspaceSize;
  pl.ok = pl.ws <= kBltWs;
  return pl;
}
}  // namespace

// weight gradient of a dense 1x1 convolution (Xcol = X) through hipBLASLt,
// accumulated into the f32 dW; false (nothing launched) when no plan exists
bool blt_wgrad_tn(const void* dy, long long ldd, const void* x, long long ldx, int Cout, int K, long long M, float* dw,
                  hipStream_t st) {
  if (M <= 0 || Cout <= 0 || K <= 0) return false;
  std::lock_guard<std::mutex> lk(g_blt_mu);
  if (!blt_init()) return false;
  const BltWKey key{M, Cout, K, ldx, ldd};
  auto it = g_blt_wplans.find(key);
  if (it == g_blt_wplans.end()) it = g_blt_wplans.emplace(key, make_wplan(M, Cout, K, ldx, ldd)).first;
  const BltPlan& pl = it->second;
  if (!pl.ok) return false;
  const float alpha = 1.f, beta = 1.f;
  const hipblasStatus_t s =
      hipblasLtMatmul(g_blt, pl.op, &alpha, x, pl.la, dy, pl.lb, &beta, dw, pl.lc, dw, pl.lc, &pl.algo, g_blt_ws, pl.ws, st);
  if (s != HIPBLAS_STATUS_SUCCESS) return false;
  set_last_kernel("hipblaslt_wgrad_tn");
  return true;
}

// the dense NT GEMM of a PgArgs (H = W = 1, 1x1 "conv" over M rows) with a plain
// bf16 output (+ an f32 bias per output column); false (nothing launched) when
// the launch fuses anything else
bool blt_gemm_nt(const PgArgs& a, hipStream_t st) {
  if (a.H != 1 || a.W != 1 || a.R != 1 || a.S != 1 || a.C != a.K || a.Ho != 1 || a.Wo != 1) return false;
  if (a.stats || a.bnb || a.res_mode || a.relu || a.M <= 0) return false;
  const long long lda = a.sN, ldc = a.ldy;
  std::lock_guard<std::mutex> lk(g_blt_mu);
  if (!blt_init()) return false;
  const BltKey key{a.M, a.Cout, a.K, lda, ldc, a.bias != nullptr};
  auto it = g_blt_plans.find(key);
  if (it == g_blt_plans.end()) it = g_blt_plans.emplace(key, make_plan(a.M, a.Cout, a.K, lda, ldc, a.bias)).first;
  const BltPlan& pl = it->second;
  if (!pl.ok) return false;
  if (a.bias)  // this call's bias vector (the cached plan was made with another one)
    hipblasLtMatmulDescSetAttribute(pl.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a.bias, sizeof(a.bias));
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(g_blt, pl.op, &alpha, a.w, pl.la, a.x, pl.lb, &beta, a.y, pl.lc, a.y, pl.lc,
                                            &pl.algo, g_blt_ws, pl.ws, st);
  if (s != HIPBLAS_STATUS_SUCCESS) return false;
  set_last_kernel("hipblaslt_gemm_nt");
  return true;
}

}  // namespace artsbir
