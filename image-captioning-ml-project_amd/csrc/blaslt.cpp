// Plain-GEMM route through hipBLASLt (ROCm's tuned GEMM library) for the bf16 products
// whose epilogue is at most bias / residual / alpha / beta and whose A operand is K-major:
// every forward Linear without an activation, and the dX GEMMs.  Measured on MI355X
// (tools/blas_probe.py vs tools/gemm_bench.py): 890-1110 TF/s against 600-870 TF/s for
// gemm_bf16_kernel on the config-3 shapes.  Fused epilogues (activation, dropout,
// pre-activation / act' side outputs) and the split-K weight-gradient GEMMs (M-major A,
// where the hand-written kernel is 1.3-3x faster) stay on gemm.hip.
//
// Row-major C[M,N] = A(M,K) B(N,K)^T is issued column-major as C^T = B_op . A_op^T:
// hipBLASLt "A" = our B, "B" = our A, D = C^T with ld = ldc.  Bias (fp32, per output
// column n) is the BIAS epilogue over D's rows; a residual is passed as C with beta = 1.
// One plan (descriptors + heuristic algorithm) per shape/stride/type key, built once.
// The workspace is the caller's (capk_gemm_workspace covers it); the library allocates
// nothing and the algorithm choice is fixed per shape.  CAPK_GEMM_BLASLT=0 turns the route off.
#include <hipblaslt/hipblaslt.h>
#include <stdlib.h>

#include <unordered_map>

#include "common.h"

namespace capk {

constexpr size_t LT_WS_BYTES = 32u << 20;  // workspace the caller provides (capk_gemm_workspace)
size_t lt_workspace_bytes() { return LT_WS_BYTES; }

namespace {

struct LtKey {
  int M, N, K, ak, bk, out_f32, bias, with_c;
  int64_t lda, ldb, ldc, ldcin;
  bool operator==(const LtKey& o) const {
    return M == o.M && N == o.N && K == o.K && ak == o.ak && bk == o.bk && out_f32 == o.out_f32 &&
           bias == o.bias && with_c == o.with_c && lda == o.lda && ldb == o.ldb && ldc == o.ldc && ldcin == o.ldcin;
  }
};
struct LtKeyHash {
  size_t operator()(const LtKey& k) const {
    uint64_t h = 1469598103934665603ull;
    const int64_t v[12] = {k.M, k.N, k.K, k.ak, k.bk, k.out_f32, k.bias, k.with_c, k.lda, k.ldb, k.ldc, k.ldcin};
    for (int64_t x : v) h = (h ^ (uint64_t)x) * 1099511628211ull;
    return (size_t)h;
  }
};
struct LtPlan {
  bool ok = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
};

hipblasLtHandle_t lt_handle() {
  thread_local hipblasLtHandle_t h = nullptr;
  thread_local bool tried = false;
  if (!tried) {
    tried = true;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
  }
  return h;
}

bool build_plan(hipblasLtHandle_t h, const LtKey& k, LtPlan& p) {
  const hipDataType ot = k.out_f32 ? HIP_R_32F : HIP_R_16BF;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const hipblasOperation_t opA = k.bk ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // library A = our B (N x K)
  const hipblasOperation_t opB = k.ak ? HIPBLAS_OP_N : HIPBLAS_OP_T;  // library B = our A^T (K x M)
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB));
  if (k.bias) {
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  bool ok = true;
  ok &= hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, k.bk ? k.K : k.N, k.bk ? k.N : k.K, k.ldb) == HIPBLAS_STATUS_SUCCESS;
  ok &= hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, k.ak ? k.K : k.M, k.ak ? k.M : k.K, k.lda) == HIPBLAS_STATUS_SUCCESS;
  ok &= hipblasLtMatrixLayoutCreate(&p.c, ot, k.N, k.M, k.ldcin) == HIPBLAS_STATUS_SUCCESS;
  ok &= hipblasLtMatrixLayoutCreate(&p.d, ot, k.N, k.M, k.ldc) == HIPBLAS_STATUS_SUCCESS;
  if (!ok) return false;
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  const uint64_t ws = LT_WS_BYTES;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[4];
  int n = 0;
  const hipblasStatus_t s = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.d, pref, 4, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (s != HIPBLAS_STATUS_SUCCESS) return false;
  for (int i = 0; i < n; ++i) {  // best-ranked algorithm whose workspace fits the caller's buffer
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= LT_WS_BYTES) {
      p.algo = res[i].algo;
      p.ws = res[i].workspaceSize;
      return true;
    }
  }
  return false;
}

}  // namespace

bool lt_enabled() {
  static const bool on = [] {
    const char* e = getenv("CAPK_GEMM_BLASLT");  // opt-in A/B reference only (=1)
    return e && e[0] == '1';
  }();
  return on;
}

// Returns true when the product was launched through hipBLASLt; false: not applicable or no
// algorithm (the caller then runs gemm_bf16_kernel).
bool lt_gemm(int out_f32, int M, int N, int K, const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
             int b_kmajor, void* C, int64_t ldc, float alpha, float beta, const float* bias, const void* residual,
             int64_t ldr, void* ws, size_t ws_bytes, hipStream_t st) {
  if (residual && beta != 0.f) return false;
  hipblasLtHandle_t h = lt_handle();
  if (!h) return false;
  const bool with_c = residual != nullptr || beta != 0.f;
  const LtKey key{M, N, K, a_kmajor, b_kmajor, out_f32, bias != nullptr, with_c, lda, ldb, ldc, residual ? ldr : ldc};
  thread_local std::unordered_map<LtKey, LtPlan, LtKeyHash> plans;
  auto it = plans.find(key);
  if (it == plans.end()) {
    LtPlan p;
    p.ok = build_plan(h, key, p);
    it = plans.emplace(key, p).first;
  }
  LtPlan& p = it->second;
  if (!p.ok || (p.ws && (!ws || ws_bytes < p.ws))) return false;
  if (bias) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
  const void* cin = residual ? residual : C;
  const float b = residual ? 1.f : beta;
  const hipblasStatus_t s =
      hipblasLtMatmul(h, p.desc, &alpha, B, p.a, A, p.b, &b, cin, p.c, C, p.d, &p.algo, p.ws ? ws : nullptr, p.ws, st);
  return s == HIPBLAS_STATUS_SUCCESS;
}

}  // namespace capk
