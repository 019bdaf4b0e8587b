// blaslt_probe.cpp — does hipBLASLt's heuristic return an algorithm for a GEMM shape / dtype?
// Prints the candidate count (8 requested).  Run with LD_LIBRARY_PATH pointing at another
// libhipblaslt.so.1 (e.g. the one bundled with torch) to compare builds.
// Build: hipcc -O2 -std=c++17 -o tools/blaslt_probe tools/blaslt_probe.cpp -lhipblaslt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>

int probe(hipblasLtHandle_t h, int rows, int K, int n, hipDataType wt, hipblasComputeType_t ct, int req) {
    hipblasLtMatmulDesc_t md;
    hipblasLtMatmulDescCreate(&md, ct, HIP_R_32F);
    hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof opT);
    hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof opN);
    hipblasLtMatrixLayout_t la, lb, lc;
    hipblasLtMatrixLayoutCreate(&la, wt, K, rows, K);
    hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, K, n, K);
    hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, rows, n, rows);
    hipblasLtMatmulPreference_t pref;
    hipblasLtMatmulPreferenceCreate(&pref);
    size_t wss = 256ull << 20;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wss, sizeof wss);
    hipblasLtMatmulHeuristicResult_t heur[8];
    int nret = 0;
    hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, req, heur, &nret);
    printf("rows %5d K %5d n %5d wt %d ct %d req %d: status %d nret %d\n", rows, K, n, (int)wt, (int)ct, req, (int)st,
           nret);
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(md);
    return nret;
}

int main() {
    hipblasLtHandle_t h;
    hipblasLtCreate(&h);
    const int shapes[][3] = {{128, 64, 74}, {128, 64, 2}, {384, 256, 200}, {768, 256, 1024}, {6144, 4096, 1024},
                             {6144, 4096, 74}, {28672, 4096, 1024}, {4096, 14336, 1024}, {128, 64, 1024},
                             {256, 64, 128}, {512, 128, 128}};
    for (auto& s : shapes) {
        probe(h, s[0], s[1], s[2], HIP_R_8F_E4M3, HIPBLAS_COMPUTE_32F_FAST_16F, 8);
        probe(h, s[0], s[1], s[2], HIP_R_8F_E4M3, HIPBLAS_COMPUTE_32F, 8);
        probe(h, s[0], s[1], s[2], HIP_R_16F, HIPBLAS_COMPUTE_32F, 8);
    }
    return 0;
}
