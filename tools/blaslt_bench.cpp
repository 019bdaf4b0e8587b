// blaslt_bench.cpp — can hipBLASLt run the prompt-pass GEMMs (Y[t][r] = sum_k X[t][k] W[r][k],
// X f16, W f16 or fp8 e4m3, Y f32) fast on gfx950?  Times W1/W3-, W2- and qkv-shaped GEMMs
// for several token counts.
// Build: hipcc -O2 -std=c++17 -o tools/blaslt_bench tools/blaslt_bench.cpp -lhipblaslt
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <utility>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define CB(x) do { hipblasStatus_t s = (x); if (s != HIPBLAS_STATUS_SUCCESS) { printf("hipBLASLt status %d @%d\n", (int)s, __LINE__); return 1; } } while (0)

// swap: W is the B operand (D = X W^T, [rows][n] column-major = Y transposed)
int run(hipblasLtHandle_t h, int rows, int K, int n, hipDataType wt, void* W, void* X, float* Y, void* ws, size_t wss,
        float* us_out, hipblasComputeType_t ct = HIPBLAS_COMPUTE_32F, bool swap = false) {
    hipblasLtMatmulDesc_t md;
    CB(hipblasLtMatmulDescCreate(&md, ct, HIP_R_32F));
    hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    CB(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof opT));
    CB(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof opN));
    hipblasLtMatrixLayout_t la, lb, lc;
    if (!swap) {
        CB(hipblasLtMatrixLayoutCreate(&la, wt, K, rows, K));
        CB(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, K, n, K));
        CB(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, rows, n, rows));
    } else {
        CB(hipblasLtMatrixLayoutCreate(&la, HIP_R_16F, K, n, K));
        CB(hipblasLtMatrixLayoutCreate(&lb, wt, K, rows, K));
        CB(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, n, rows, n));
        std::swap(W, X);
    }
    hipblasLtMatmulPreference_t pref;
    CB(hipblasLtMatmulPreferenceCreate(&pref));
    CB(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wss, sizeof wss));
    hipblasLtMatmulHeuristicResult_t heur[8];
    int nret = 0;
    CB(hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 8, heur, &nret));
    if (nret == 0) { printf("no algorithm\n"); return 1; }
    float alpha = 1.f, beta = 0.f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int a = 0; a < nret; a++) {
        for (int i = 0; i < 3; i++)
            CB(hipblasLtMatmul(h, md, &alpha, W, la, X, lb, &beta, Y, lc, Y, lc, &heur[a].algo, ws, wss, 0));
        CK(hipEventRecord(e0, 0));
        const int it = 10;
        for (int i = 0; i < it; i++)
            CB(hipblasLtMatmul(h, md, &alpha, W, la, X, lb, &beta, Y, lc, Y, lc, &heur[a].algo, ws, wss, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms * 1000 / it < best) best = ms * 1000 / it;
    }
    *us_out = best;
    hipblasLtMatmulPreferenceDestroy(pref);
    hipblasLtMatrixLayoutDestroy(la);
    hipblasLtMatrixLayoutDestroy(lb);
    hipblasLtMatrixLayoutDestroy(lc);
    hipblasLtMatmulDescDestroy(md);
    return 0;
}

int main() {
    hipblasLtHandle_t h;
    CB(hipblasLtCreate(&h));
    const size_t wss = 256ull << 20;
    void *ws, *W, *X;
    float* Y;
    CK(hipMalloc(&ws, wss));
    CK(hipMalloc(&W, 28672ull * 14336 * 2));
    CK(hipMalloc(&X, 1024ull * 14336 * 2));
    CK(hipMalloc(&Y, 1024ull * 28672 * 4));
    CK(hipMemset(W, 0x11, 28672ull * 14336 * 2));
    CK(hipMemset(X, 0x11, 1024ull * 14336 * 2));
    struct Sh { const char* name; int rows, K; } shapes[] = {{"w13", 28672, 4096}, {"w2", 4096, 14336}, {"qkv", 6144, 4096},
                                                            {"wo", 4096, 4096}};
    struct Cfg { hipDataType wt; hipblasComputeType_t ct; bool swap; const char* name; };
    const Cfg cfgs[] = {{HIP_R_16F, HIPBLAS_COMPUTE_32F, false, "f16"},
                        {HIP_R_8F_E4M3, HIPBLAS_COMPUTE_32F_FAST_16F, false, "e4m3 A fast16"},
                        {HIP_R_8F_E4M3, HIPBLAS_COMPUTE_32F, true, "e4m3 B 32f"},
                        {HIP_R_8F_E4M3, HIPBLAS_COMPUTE_32F_FAST_16F, true, "e4m3 B fast16"},
                        {HIP_R_8F_E5M2, HIPBLAS_COMPUTE_32F, true, "e5m2 B 32f"},
                        {HIP_R_8F_E5M2, HIPBLAS_COMPUTE_32F_FAST_16F, false, "e5m2 A fast16"}};
    for (const Cfg& cf : cfgs) {
        const hipDataType wt = cf.wt;
        for (auto& s : shapes) {
            for (int n : {64, 256, 512}) {
                float us = 0;
                if (run(h, s.rows, s.K, n, wt, W, X, Y, ws, wss, &us, cf.ct, cf.swap)) {
                    printf("%s %s n=%d failed\n", cf.name, s.name, n);
                    continue;
                }
                const double fl = 2.0 * s.rows * s.K * n;
                printf("%-14s %-4s n=%4d  %8.1f us  %7.1f TFLOP/s  weights %6.2f TB/s\n", cf.name,
                       s.name, n, us, fl / us / 1e6, (double)s.rows * s.K * (wt == HIP_R_16F ? 2 : 1) / us / 1e6);
            }
        }
    }
    return 0;
}
