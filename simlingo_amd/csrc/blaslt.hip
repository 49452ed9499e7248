// Plain GEMMs through hipBLASLt (slx_gemm_lt, include/slx.h). MI355X_MICROARCH / the build rules: hand-written MFMA
// kernels for the fused hot ops, the vendor library for plain GEMMs. Three step GEMMs are plain and run faster on
// hipBLASLt's tiles than on slx_gemm_bf16's 256^2 / 128^2 grids (tools/gemm_lt_probe.py, profiles/round6_gemm_lt_ab.txt):
// the Qwen2 gate/up data gradient (6384 x 960 x 9728: 100 256^2 tiles leave 56 CUs idle) and the Qwen2 o / down
// projections with their f32 residual (C = the residual, beta = 1).
//
// Row-major D[M][N] = alpha A[M][K] B[N][K]^T + beta C is the column-major D^T[N][M] = op(B) op(A) with B viewed as a
// K x N column-major matrix (transposed) and A as K x M (not transposed); C / D keep their row stride as the
// column-major leading dimension. One plan per (device, shape, strides, types, beta != 0): the descriptors and the
// heuristic's first algorithm, created on first use under a mutex and reused.
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "../../include/slx.h"

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

using LtKey = std::tuple<int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int, int64_t>;

std::mutex g_mu;
std::map<LtKey, LtPlan> g_plans;
hipblasLtHandle_t g_handle[64] = {};

const char* lt_status(hipblasStatus_t s) {
  switch (s) {
    case HIPBLAS_STATUS_SUCCESS: return "success";
    case HIPBLAS_STATUS_NOT_INITIALIZED: return "not initialized";
    case HIPBLAS_STATUS_ALLOC_FAILED: return "alloc failed";
    case HIPBLAS_STATUS_INVALID_VALUE: return "invalid value";
    case HIPBLAS_STATUS_NOT_SUPPORTED: return "not supported";
    case HIPBLAS_STATUS_EXECUTION_FAILED: return "execution failed";
    default: return "error";
  }
}

}  // namespace

#define SLX_LT_CHECK(expr)                                                                                \
  do {                                                                                                    \
    const hipblasStatus_t st_ = (expr);                                                                   \
    if (st_ != HIPBLAS_STATUS_SUCCESS) {                                                                  \
      slx::set_error("slx_gemm_lt: %s: %s", #expr, lt_status(st_));                                       \
      return -1001;                                                                                       \
    }                                                                                                     \
  } while (0)

extern "C" int slx_gemm_lt(const slx_gemm_lt_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d && d->A && d->B && d->D, "slx_gemm_lt: A, B and D");
  SLX_CHECK_ARG(d->M >= 0 && d->N > 0 && d->K > 0, "slx_gemm_lt: M >= 0, N > 0, K > 0");
  SLX_CHECK_ARG(d->lda >= d->K && d->ldb >= d->K && d->ldd >= d->N, "slx_gemm_lt: lda, ldb >= K and ldd >= N");
  SLX_CHECK_ARG(d->beta == 0.f || (d->C && d->ldc >= d->N), "slx_gemm_lt: beta != 0 needs C with ldc >= N");
  SLX_CHECK_ARG(d->ws_bytes >= 0 && (d->ws_bytes == 0 || d->ws), "slx_gemm_lt: workspace");
  if (d->M == 0) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    slx::set_error("slx_gemm_lt: hipGetDevice");
    return -1001;
  }
  const int beta_on = d->beta != 0.f;
  const int64_t ldc = beta_on ? d->ldc : d->ldd;
  const LtKey key{dev, d->M, d->N, d->K, d->lda, d->ldb, ldc, d->ldd, d->out_f32, beta_on, d->ws_bytes};
  LtPlan* plan = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it != g_plans.end()) {
      plan = &it->second;
    } else {
      if (!g_handle[dev]) SLX_LT_CHECK(hipblasLtCreate(&g_handle[dev]));
      LtPlan p;
      const hipDataType ot = d->out_f32 ? HIP_R_32F : HIP_R_16BF;
      SLX_LT_CHECK(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
      const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
      SLX_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
      SLX_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
      // library A = our B viewed K x N (ld ldb), library B = our A viewed K x M (ld lda), C / D N x M
      SLX_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, d->K, d->N, d->ldb));
      SLX_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, d->K, d->M, d->lda));
      SLX_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lc, ot, d->N, d->M, ldc));
      SLX_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.ld, ot, d->N, d->M, d->ldd));
      hipblasLtMatmulPreference_t pref;
      SLX_LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
      const uint64_t wsb = (uint64_t)d->ws_bytes;
      SLX_LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                                         sizeof(wsb)));
      hipblasLtMatmulHeuristicResult_t res[1];
      int n = 0;
      const hipblasStatus_t hs =
          hipblasLtMatmulAlgoGetHeuristic(g_handle[dev], p.op, p.la, p.lb, p.lc, p.ld, pref, 1, res, &n);
      hipblasLtMatmulPreferenceDestroy(pref);
      if (hs != HIPBLAS_STATUS_SUCCESS || n < 1) {
        slx::set_error("slx_gemm_lt: no hipBLASLt algorithm for M=%ld N=%ld K=%ld (%s)", (long)d->M, (long)d->N,
                       (long)d->K, lt_status(hs));
        return -1001;
      }
      p.algo = res[0].algo;
      p.ws = res[0].workspaceSize;
      plan = &g_plans.emplace(key, p).first->second;
    }
  }
  const float alpha = d->alpha, beta = d->beta;
  SLX_LT_CHECK(hipblasLtMatmul(g_handle[dev], plan->op, &alpha, d->B, plan->la, d->A, plan->lb, &beta,
                               beta_on ? d->C : d->D, plan->lc, d->D, plan->ld, &plan->algo,
                               plan->ws ? d->ws : nullptr, plan->ws, (hipStream_t)stream));
  return 0;
}
