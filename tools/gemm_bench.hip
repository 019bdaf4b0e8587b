// gemm_bench.hip — the prompt-pass GEMM (xalm_amd/csrc/gemm16.h) on Mistral-7B shapes:
// correctness against a double-precision host sum on sampled outputs, device time per launch,
// and the same GEMM on hipBLASLt (hi + lo as 2n columns, best of its heuristic candidates) on the
// same box for reference.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/gemm_bench tools/gemm_bench.hip -lhipblaslt
// Run:   tools/gemm_bench [n_tokens ...]
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../xalm_amd/csrc/gemm16.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
#define CB(x) do { hipblasStatus_t s = (x); if (s != HIPBLAS_STATUS_SUCCESS) { printf("hipBLASLt status %d @%d\n", (int)s, __LINE__); exit(1); } } while (0)

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }
static float h2f(uint16_t u) { _Float16 h; memcpy(&h, &u, 2); return (float)h; }

static int pick_ks(int rows, int n, int K) { return xalm::mm_pick_ks(rows, K, n, (size_t)2 * 2048 * 28672); }

static float blaslt_us(hipblasLtHandle_t h, int rows, int K, int n2, void* W, void* X, float* Y, void* ws, size_t wss) {
    hipblasLtMatmulDesc_t md;
    CB(hipblasLtMatmulDescCreate(&md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
    CB(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof opT));
    CB(hipblasLtMatmulDescSetAttribute(md, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof opN));
    hipblasLtMatrixLayout_t la, lb, lc;
    CB(hipblasLtMatrixLayoutCreate(&la, HIP_R_16F, K, rows, K));
    CB(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16F, K, n2, K));
    CB(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, rows, n2, rows));
    hipblasLtMatmulPreference_t pref;
    CB(hipblasLtMatmulPreferenceCreate(&pref));
    CB(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wss, sizeof wss));
    hipblasLtMatmulHeuristicResult_t heur[8];
    int nret = 0;
    CB(hipblasLtMatmulAlgoGetHeuristic(h, md, la, lb, lc, lc, pref, 8, heur, &nret));
    float alpha = 1.f, beta = 0.f, best = 1e30f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int c = 0; c < nret; c++) {
        for (int i = 0; i < 3; i++)
            CB(hipblasLtMatmul(h, md, &alpha, W, la, X, lb, &beta, Y, lc, Y, lc, &heur[c].algo, ws, wss, 0));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < 10; i++)
            CB(hipblasLtMatmul(h, md, &alpha, W, la, X, lb, &beta, Y, lc, Y, lc, &heur[c].algo, ws, wss, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms / 10 < best) best = ms / 10;
        if (getenv("GB_BLAS_ALL")) printf("      hipBLASLt candidate %d: %8.1f us\n", c, ms * 100.f);
    }
    return best * 1e3f;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);  // a line reaches the log as soon as it is printed
    std::vector<int> ns;
    for (int i = 1; i < argc; i++) ns.push_back(atoi(argv[i]));
    if (ns.empty()) ns = {512, 1024, 2048};
    struct Shape { const char* name; int rows, K; };
    const Shape shapes[] = {{"qkv", 6144, 4096}, {"wo", 4096, 4096}, {"w13", 28672, 4096}, {"w2", 4096, 14336}};
    const size_t wmax = (size_t)28672 * 4096, nmax = 2048, kmax = 14336;
    std::mt19937 rng(1);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<uint16_t> hw(wmax), hx(2 * nmax * kmax);
    for (auto& v : hw) v = f2h(0.02f * nd(rng));
    for (size_t i = 0; i < nmax * kmax; i++) {  // hi / lo of a scaled N(0,1) row (as prefill_split_kernel)
        const float u = 16384.f * nd(rng);
        const _Float16 hi = (_Float16)u;
        hx[i] = f2h((float)hi);
        hx[nmax * kmax + i] = f2h(u - (float)hi);
    }
    uint16_t *dw, *dx;
    float* dy;
    void* ws;
    CK(hipMalloc(&dw, wmax * 2));
    CK(hipMalloc(&dx, 2 * nmax * kmax * 2));
    CK(hipMalloc(&dy, (size_t)8 * nmax * 28672 * 4));
    const size_t wss = 256ull << 20;
    CK(hipMalloc(&ws, wss));
    CK(hipMemcpy(dw, hw.data(), wmax * 2, hipMemcpyHostToDevice));
    struct Var { const char* name; void (*fn)(xalm::MmArgs); int lds; int bt; int threads = xalm::MM_THREADS; int kmul = 1; };
    const Var vars[] = {
        {"m16g", xalm::mm_f16_kernel_t<64, 2, 12, 128>, xalm::MmCfg<64, 2, 128>::LDS, 128},
        {"m16b32s3", xalm::mm_f16_kernel_t<32, 3, 12, 128>, xalm::MmCfg<32, 3, 128>::LDS, 128},
        {"m16b32o4", xalm::mm_f16_kernel_t<32, 2, 12, 128, 4>, xalm::MmCfg<32, 2, 128>::LDS, 128},
        // 4 waves: each wave 64 tokens x 128 rows (a third less LDS read per MFMA)
        {"w4b64", xalm::mm_f16_kernel_t<64, 2, 12, 128, 1, 4>, xalm::MmCfg<64, 2, 128, 4>::LDS, 128, 256},
        {"w4b32s4", xalm::mm_f16_kernel_t<32, 4, 12, 128, 1, 4>, xalm::MmCfg<32, 4, 128, 4>::LDS, 128, 256},
        {"w4b32o2", xalm::mm_f16_kernel_t<32, 2, 12, 128, 2, 4>, xalm::MmCfg<32, 2, 128, 4>::LDS, 128, 256},
        {"w4b64p", xalm::mm_f16_kernel_t<64, 2, 13, 128, 1, 4>, xalm::MmCfg<64, 2, 128, 4>::LDS, 128, 256},
        // the same with twice / four times the K slices of mm_pick_ks (more workgroups per CU)
        {"w4o2k2", xalm::mm_f16_kernel_t<32, 2, 12, 128, 2, 4>, xalm::MmCfg<32, 2, 128, 4>::LDS, 128, 256, 2},
        {"w4o2k4", xalm::mm_f16_kernel_t<32, 2, 12, 128, 2, 4>, xalm::MmCfg<32, 2, 128, 4>::LDS, 128, 256, 4},
        {"m16gk2", xalm::mm_f16_kernel_t<64, 2, 12, 128>, xalm::MmCfg<64, 2, 128>::LDS, 128, 512, 2},
        // 256-token tiles: 8 waves as 4 (tokens) x 2 (rows), each 64 tokens x 128 rows; a third less
        // L2 -> LDS traffic per MFMA than the 128-token tile
        {"b256s2", xalm::mm_f16_kernel_t<32, 2, 12, 256, 1, 8>, xalm::MmCfg<32, 2, 256>::LDS, 256},
        {"b256s3", xalm::mm_f16_kernel_t<32, 3, 12, 256, 1, 8>, xalm::MmCfg<32, 3, 256>::LDS, 256},
        {"b256s3p", xalm::mm_f16_kernel_t<32, 3, 13, 256, 1, 8>, xalm::MmCfg<32, 3, 256>::LDS, 256},
    };
    const int NV = sizeof vars / sizeof vars[0];
    for (int v = 0; v < NV; v++)
        CK(hipFuncSetAttribute((const void*)vars[v].fn, hipFuncAttributeMaxDynamicSharedMemorySize, vars[v].lds));
    hipblasLtHandle_t bl;
    CB(hipblasLtCreate(&bl));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int bad = 0;
    for (int n : ns) {
        double tot_us[16] = {}, tot_bl = 0, tot_flop = 0;
        for (const Shape& sh : shapes) {
            // Xh rows [n][K] then Xl rows [n][K] (the product's layout)
            std::vector<uint16_t> xs(2 * (size_t)n * sh.K);
            for (int t = 0; t < n; t++)
                for (int k = 0; k < sh.K; k++) {
                    xs[(size_t)t * sh.K + k] = hx[(size_t)t * kmax + k];
                    xs[((size_t)n + t) * sh.K + k] = hx[nmax * kmax + (size_t)t * kmax + k];
                }
            CK(hipMemcpy(dx, xs.data(), xs.size() * 2, hipMemcpyHostToDevice));
            xalm::MmArgs a{};
            a.w = dw; a.xh = dx; a.xl = dx + (size_t)n * sh.K; a.out = dy;
            a.rows = sh.rows; a.K = sh.K; a.n = n; a.ks = pick_ks(sh.rows, n, sh.K);
            a.n_rt = (sh.rows + xalm::MM_BR - 1) / xalm::MM_BR; a.n_tt = (n + xalm::MM_BT - 1) / xalm::MM_BT;
            int grid = a.n_rt * a.n_tt * a.ks;
            if (getenv("GB_SHAPE") && strcmp(getenv("GB_SHAPE"), sh.name)) continue;
            const float bus = getenv("GB_NOBLAS") ? 1e9f : blaslt_us(bl, sh.rows, sh.K, 2 * n, dw, dx, dy, ws, wss);
            const double flop = 2.0 * sh.rows * sh.K * (double)n;  // counted once (hi + lo = 2x MFMA work)
            tot_bl += bus;
            tot_flop += flop;
            printf("n %5d %-4s rows %5d K %5d ks %d grid %4d | hipBLASLt %8.1f us = %6.1f TF/s\n", n, sh.name, sh.rows, sh.K,
                   a.ks, grid, bus, flop / bus * 1e-6);
            for (int v = 0; v < NV; v++) {
                if (getenv("GB_VAR") && atoi(getenv("GB_VAR")) != v) continue;
                a.n_tt = (n + vars[v].bt - 1) / vars[v].bt;
                a.ks = xalm::mm_pick_ks(sh.rows, sh.K, n, (size_t)2 * 2048 * 28672, 256, vars[v].bt) * vars[v].kmul;
                if (a.ks <= 0 || sh.K % (a.ks * 64) || (size_t)a.ks * n * sh.rows > (size_t)8 * 2048 * 28672) continue;
                grid = a.n_rt * a.n_tt * a.ks;
                auto launch = [&]() {
                    hipLaunchKernelGGL(vars[v].fn, dim3(grid), dim3(vars[v].threads), vars[v].lds, 0, a);
                };
                CK(hipMemset(dy, 0, (size_t)a.ks * n * sh.rows * 4));
                launch();
                CK(hipDeviceSynchronize());
                // check sampled outputs: sum of the ks partials vs a double sum
                std::vector<float> y((size_t)a.ks * n * sh.rows);
                CK(hipMemcpy(y.data(), dy, y.size() * 4, hipMemcpyDeviceToHost));
                double maxrel = 0;
                std::mt19937 pr(n + sh.rows);
                for (int smp = 0; smp < 256; smp++) {
                    const int t = pr() % n, r = pr() % sh.rows;
                    double ref = 0, mag = 0;
                    for (int k = 0; k < sh.K; k++) {
                        const double wv = h2f(hw[(size_t)r * sh.K + k]);
                        const double xv = (double)h2f(xs[(size_t)t * sh.K + k]) + (double)h2f(xs[((size_t)n + t) * sh.K + k]);
                        ref += wv * xv;
                        mag += fabs(wv * xv);
                    }
                    double got = 0;
                    for (int s = 0; s < a.ks; s++) got += y[((size_t)s * n + t) * sh.rows + r];
                    maxrel = fmax(maxrel, fabs(got - ref) / mag);
                }
                // interleaved rounds (guide rule 24): median of 5 rounds of 10 launches
                std::vector<float> rounds;
                for (int i = 0; i < 3; i++) launch();
                for (int rr = 0; rr < 5; rr++) {
                    CK(hipEventRecord(e0, 0));
                    for (int i = 0; i < 10; i++) launch();
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    rounds.push_back(ms * 100.f);
                }
                std::sort(rounds.begin(), rounds.end());
                const double us = rounds[2];
                tot_us[v] += us;
                const bool ok = maxrel < 2e-6;
                bad += !ok;
                printf("    %-8s ks %d grid %4d %8.1f us = %6.1f TF/s (MFMA %6.1f) err %.2e %s\n", vars[v].name, a.ks, grid, us,
                       flop / us * 1e-6, 2 * flop / us * 1e-6, maxrel, ok ? "ok" : "BAD");
            }
        }
        printf("n %5d layer: hipBLASLt %8.1f us = %6.1f TF/s\n", n, tot_bl, tot_flop / tot_bl * 1e-6);
        for (int v = 0; v < NV; v++)
            printf("    %-8s %8.1f us = %6.1f TF/s\n", vars[v].name, tot_us[v], tot_flop / tot_us[v] * 1e-6);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CB(hipblasLtDestroy(bl));
    CK(hipFree(ws));
    CK(hipFree(dy));
    CK(hipFree(dx));
    CK(hipFree(dw));
    printf("done: %d bad\n", bad);
    return bad ? 1 : 0;
}
