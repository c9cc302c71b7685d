// Which hipBLASLt epilogues have gfx950 solutions for ViT fc1 (bf16, M=50432 N=3072 K=768)?
// Prints the descriptor-attribute statuses and the heuristic's candidate count per variant.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <vector>

int main() {
  const int64_t M = 50432, N = 3072, K = 768;
  hipblasLtHandle_t h;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) { printf("create failed\n"); return 1; }
  void *x, *w, *b, *out, *aux, *ws;
  hipMalloc(&x, M * K * 2); hipMalloc(&w, N * K * 2); hipMalloc(&b, N * 4); hipMalloc(&out, M * N * 2);
  hipMalloc(&aux, M * N * 2); hipMalloc(&ws, 32 << 20);
  struct V { const char* name; hipblasLtEpilogue_t epi; int aux; hipDataType bt; int auxdt; };
  V vs[] = {{"BIAS bf16", HIPBLASLT_EPILOGUE_BIAS, 0, HIP_R_16BF, 0},
            {"GELU", HIPBLASLT_EPILOGUE_GELU, 0, HIP_R_16BF, 0},
            {"GELU_BIAS bf16", HIPBLASLT_EPILOGUE_GELU_BIAS, 0, HIP_R_16BF, 0},
            {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX, 1, HIP_R_16BF, 0},
            {"GELU_AUX_BIAS bf16 auxdt", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, 1, HIP_R_16BF, 1},
            {"GELU_AUX_BIAS bf16", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, 1, HIP_R_16BF, 0},
            {"GELU_AUX_BIAS f32 bias", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, 1, HIP_R_32F, 0}};
  for (auto& v : vs) {
    hipblasLtMatmulDesc_t d;
    hipblasLtMatrixLayout_t la, lb, lc;
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    int s0 = hipblasLtMatmulDescCreate(&d, HIPBLAS_COMPUTE_32F, HIP_R_32F);
    int s1 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    int s2 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K);
    hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K);
    hipblasLtMatrixLayoutCreate(&lc, HIP_R_16BF, N, M, N);
    int s3 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE, &v.epi, sizeof(v.epi));
    int s4 = 0, s5 = 0, s6 = 0, s7 = 0, s8 = 0;
    if (v.epi != HIPBLASLT_EPILOGUE_GELU && v.epi != HIPBLASLT_EPILOGUE_GELU_AUX) {
      s4 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &b, sizeof(b));
      s5 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &v.bt, sizeof(v.bt));
    }
    if (v.aux) {
      int64_t ld = N;
      s6 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux));
      s7 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
      if (v.auxdt) {
        hipDataType adt = HIP_R_16BF;
        s8 = hipblasLtMatmulDescSetAttribute(d, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &adt, sizeof(adt));
      }
    }
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    uint64_t cap = 32 << 20;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap, sizeof(cap));
    std::vector<hipblasLtMatmulHeuristicResult_t> r(8);
    int found = 0;
    int s9 = hipblasLtMatmulAlgoGetHeuristic(h, d, la, lb, lc, lc, pref, 8, r.data(), &found);
    float ms = -1.f;
    if (found > 0) {
      const float alpha = 1.f, beta = 0.f;
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      hipblasLtMatmul(h, d, &alpha, w, la, x, lb, &beta, out, lc, out, lc, &r[0].algo, ws, cap, 0);
      hipEventRecord(e0, 0);
      for (int i = 0; i < 10; ++i) hipblasLtMatmul(h, d, &alpha, w, la, x, lb, &beta, out, lc, out, lc, &r[0].algo, ws, cap, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      ms /= 10;
    }
    printf("%-26s desc %d %d %d epi %d bias %d %d aux %d %d %d heur %d found %d  us %.1f\n", v.name, s0, s1, s2, s3, s4,
           s5, s6, s7, s8, s9, found, ms * 1000);
    fflush(stdout);
  }
  return 0;
}
