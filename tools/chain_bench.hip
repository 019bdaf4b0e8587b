// chain_bench.hip — A/B of the decode layer's four weight matvecs (qkv, wo, w1/w3, w2 at
// Mistral-7B f16 shapes; attention left out) over 32 layers:
//   seq   : gemv_kernel launches on one stream (the graph engine's kernels)
//   chain : chain_gemv_kernel on two alternating streams (csrc/chain.h)
// Weights rotate over 4 distinct layer copies (1.75 GB) so the Infinity Cache serves nothing.
// The chain result is checked against the sequential one (same math, rms summation order
// differs).  Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/chain_bench tools/chain_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../include/xalm_synth.h"
#include "../xalm_amd/csrc/chain.h"

using namespace xalm;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(uint16_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_to_f16(xs_value(seed, i, 0.f, 0.02f));
}
__global__ void fillf(float* p, size_t n, uint64_t seed, float mean, float std) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_value(seed, i, mean, std);
}

constexpr int DIM = 4096, HID = 14336, QKV = 6144, NL = 32, NCOPY = 4;
using SeqS = GemvShape<512, 2, 4, true, 4, false>;
template <int U>
using ChS = GemvShape<512, 2, U, true, 4, false>;

struct Layer { uint16_t *qkv, *wo, *w13, *w2; };

static GemvArgs args(const void* w, int rows, int n, const float* x, float* out, const float* nw) {
    GemvArgs a{};
    a.w = w; a.row_bytes = (size_t)n * 2; a.n = n; a.rows = rows; a.x = x; a.out = out;
    a.norm_w = nw; a.norm_dtype = XH_F32; a.eps = 1e-5f; a.act = XH_ACT_SILU;
    return a;
}

template <int PRO, int EPI, class SeqS>
static int seq_launch1(GemvArgs a, hipStream_t s, unsigned long long* tr) {
    a.trace = tr;
    auto k = gemv_kernel<XH_F16, PRO, EPI, SeqS>;
    static bool once = false;
    if (!once) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); once = true; }
    const int blocks = gemv_blocks<SeqS>(a.rows, 4096 / SeqS::WAVES);
    const size_t smem = gemv_smem_bytes<XH_F16, SeqS>(a.n);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), smem, s, a);
    return blocks;
}
static int g_seq_pf = 0;
// 0 plain; 1 PF U4 (product); 2 PF U8 for n=4096 row counts <= 8192 (qkv, wo); 3 PF U8 for
// n=14336 (w2); 4 = 2 + 3; 5 PF U4 ROWS 1 for w2
template <int PRO, int EPI>
static int seq_launch(GemvArgs a, hipStream_t s, unsigned long long* tr = nullptr) {
    const int v = g_seq_pf;
    if (!v) return seq_launch1<PRO, EPI, SeqS>(a, s, tr);
    if (a.n <= 4096) {
        if ((v == 2 || v == 4) && a.rows <= 8192) return seq_launch1<PRO, EPI, GemvShape<512, 2, 8, true, 4, true, 2>>(a, s, tr);
        return seq_launch1<PRO, EPI, GemvShape<512, 2, 4, true, 4, true, 2>>(a, s, tr);
    }
    if (v == 3 || v == 4) return seq_launch1<PRO, EPI, GemvShape<512, 2, 8, true, 4, true, 8>>(a, s, tr);
    if (v == 5) return seq_launch1<PRO, EPI, GemvShape<512, 1, 4, true, 4, true, 8>>(a, s, tr);
    return seq_launch1<PRO, EPI, GemvShape<512, 2, 4, true, 4, true, 8>>(a, s, tr);
}

template <int PRO, int EPI, int U>
static int chain_launch(const GemvArgs& a, hipStream_t s, const ChainSync& sy, int max_blocks) {
    using S = ChS<U>;
    auto k = chain_gemv_kernel<XH_F16, PRO, EPI, S>;
    static bool once = false;
    if (!once) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); once = true; }
    const int blocks = gemv_blocks<S>(a.rows, max_blocks);
    const size_t smem = gemv_smem_bytes<XH_F16, S>(a.n);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(512), smem, s, a, sy);
    return blocks;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    std::vector<Layer> L(NCOPY);
    for (int c = 0; c < NCOPY; c++) {
        CK(hipMalloc(&L[c].qkv, (size_t)QKV * DIM * 2));
        CK(hipMalloc(&L[c].wo, (size_t)DIM * DIM * 2));
        CK(hipMalloc(&L[c].w13, (size_t)2 * HID * DIM * 2));
        CK(hipMalloc(&L[c].w2, (size_t)DIM * HID * 2));
        hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, L[c].qkv, (size_t)QKV * DIM, 10 + c);
        hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, L[c].wo, (size_t)DIM * DIM, 20 + c);
        hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, L[c].w13, (size_t)2 * HID * DIM, 30 + c);
        hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, L[c].w2, (size_t)DIM * HID, 40 + c);
    }
    float *x, *x0, *q, *hb, *nw;
    CK(hipMalloc(&x, DIM * 4));
    CK(hipMalloc(&x0, DIM * 4));
    CK(hipMalloc(&q, QKV * 4));
    CK(hipMalloc(&hb, HID * 4));
    CK(hipMalloc(&nw, DIM * 4));
    hipLaunchKernelGGL(fillf, dim3(16), dim3(256), 0, 0, x0, DIM, 7, 0.f, 1.f);
    hipLaunchKernelGGL(fillf, dim3(16), dim3(256), 0, 0, nw, DIM, 8, 1.f, 0.01f);
    const int NK = 4 * NL;
    unsigned* ctr;
    int* err;
    CK(hipMalloc(&ctr, (size_t)NK * CHAIN_SLOT * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    CK(hipDeviceSynchronize());

    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1, ej, es;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&es, hipEventDisableTiming));

    unsigned long long* strace = nullptr;
    std::vector<int> sblocks(NK);
    auto run_seq = [&]() {
        CK(hipMemcpyAsync(x, x0, DIM * 4, hipMemcpyDeviceToDevice, s0));
        CK(hipEventRecord(e0, s0));
        int k = 0;
        auto tr = [&]() { return strace ? strace + (size_t)k * 1024 * 4 : nullptr; };
        for (int l = 0; l < NL; l++) {
            const Layer& w = L[l % NCOPY];
            sblocks[k] = seq_launch<PRO_RMSNORM, EPI_STORE>(args(w.qkv, QKV, DIM, x, q, nw), s0, tr()); k++;
            sblocks[k] = seq_launch<PRO_PLAIN, EPI_RESID>(args(w.wo, DIM, DIM, q, x, nw), s0, tr()); k++;
            sblocks[k] = seq_launch<PRO_RMSNORM, EPI_GLU>(args(w.w13, 2 * HID, DIM, x, hb, nw), s0, tr()); k++;
            sblocks[k] = seq_launch<PRO_PLAIN, EPI_RESID>(args(w.w2, DIM, HID, hb, x, nw), s0, tr()); k++;
        }
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1000.f / NL;
    };
    unsigned long long* trace;
    const size_t TR = (size_t)NK * 512 * 4;
    CK(hipMalloc(&trace, TR * 8));
    bool tracing = false;
    std::vector<int> kblocks(NK);
    auto run_chain = [&](int variant) {
        CK(hipMemcpyAsync(x, x0, DIM * 4, hipMemcpyDeviceToDevice, s0));
        CK(hipMemsetAsync(ctr, 0, (size_t)NK * CHAIN_SLOT * 4, s0));
        CK(hipEventRecord(es, s0));
        CK(hipStreamWaitEvent(s1, es, 0));
        CK(hipEventRecord(e0, s0));
        int k = 0;
        unsigned prev_blocks = 0;
        const int mb = 256;
        auto sy = [&]() {
            ChainSync c{};
            c.wait = k ? ctr + (size_t)(k - 1) * CHAIN_SLOT : nullptr;
            c.target = prev_blocks;
            c.sig = ctr + (size_t)k * CHAIN_SLOT;
            c.err = err;
            c.trace = tracing ? trace + (size_t)k * 512 * 4 : nullptr;
            return c;
        };
        for (int l = 0; l < NL; l++) {
            const Layer& w = L[l % NCOPY];
            hipStream_t st;
#define STEP(PRO, EPI, A)                                                  \
    st = ((k & 1) && variant != 2) ? s1 : s0;                              \
    prev_blocks = variant != 1 ? chain_launch<PRO, EPI, 4>(A, st, sy(), mb) \
                               : chain_launch<PRO, EPI, 8>(A, st, sy(), mb); \
    kblocks[k] = prev_blocks;                                              \
    k++;
            STEP(PRO_RMSNORM, EPI_STORE, args(w.qkv, QKV, DIM, x, q, nw));
            STEP(PRO_PLAIN, EPI_RESID, args(w.wo, DIM, DIM, q, x, nw));
            STEP(PRO_RMSNORM, EPI_GLU, args(w.w13, 2 * HID, DIM, x, hb, nw));
            STEP(PRO_PLAIN, EPI_RESID, args(w.w2, DIM, HID, hb, x, nw));
        }
        CK(hipEventRecord(ej, s1));
        CK(hipStreamWaitEvent(s0, ej, 0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1000.f / NL;
    };

    // correctness: chain vs sequential final x
    std::vector<float> hs(DIM), hc(DIM);
    run_seq();
    CK(hipMemcpy(hs.data(), x, DIM * 4, hipMemcpyDeviceToHost));
    {
        std::vector<float> hp(DIM);
        g_seq_pf = 1;
        run_seq();
        g_seq_pf = 0;
        CK(hipMemcpy(hp.data(), x, DIM * 4, hipMemcpyDeviceToHost));
        double md = 0;
        for (int i = 0; i < DIM; i++) md = std::max(md, (double)fabsf(hs[i] - hp[i]));
        printf("check seq pf: max|dx|=%.4g\n", md);
    }
    for (int v = 0; v < 2; v++) {
        run_chain(v);
        CK(hipDeviceSynchronize());
        int ev = 0;
        CK(hipMemcpy(&ev, err, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), x, DIM * 4, hipMemcpyDeviceToHost));
        double mx = 0, md = 0;
        for (int i = 0; i < DIM; i++) { mx = std::max(mx, (double)fabsf(hs[i])); md = std::max(md, (double)fabsf(hs[i] - hc[i])); }
        printf("check variant %d: err=%d max|x|=%.4g max|dx|=%.4g rel=%.3g\n", v, ev, mx, md, md / mx);
        if (ev) return 2;
    }
    std::vector<float> ts, tsp, tc4, tc8, tc1;
    std::vector<std::vector<float>> tv(6);
    for (int r = 0; r < reps; r++) {
        ts.push_back(run_seq());
        for (int v = 1; v <= 5; v++) {
            g_seq_pf = v;
            tv[v].push_back(run_seq());
        }
        g_seq_pf = 0;
        tsp = tv[1];
    }
    // per-kernel means from a traced run of each variant
    auto kstats = [&](int v) {
        const size_t STR = (size_t)NK * 1024 * 4;
        unsigned long long* tb;
        CK(hipMalloc(&tb, STR * 8));
        CK(hipMemset(tb, 0, STR * 8));
        strace = tb;
        g_seq_pf = v;
        run_seq();
        g_seq_pf = 0;
        strace = nullptr;
        std::vector<unsigned long long> hq(STR);
        CK(hipMemcpy(hq.data(), tb, STR * 8, hipMemcpyDeviceToHost));
        CK(hipFree(tb));
        double sum[4] = {0, 0, 0, 0};
        int cnt[4] = {0, 0, 0, 0};
        for (int kk = 4; kk < NK; kk++) {  // skip layer 0
            unsigned long long smin = ~0ull, dmax = 0;
            const unsigned long long* T = hq.data() + (size_t)kk * 1024 * 4;
            for (int b = 0; b < sblocks[kk]; b++) { smin = std::min(smin, T[4 * b]); dmax = std::max(dmax, T[4 * b + 2]); }
            sum[kk % 4] += (dmax - smin) / 100.0;
            cnt[kk % 4]++;
        }
        printf("  variant %d: qkv %6.2f  wo %6.2f  w13 %6.2f  w2 %6.2f us (first start -> last done)\n", v,
               sum[0] / cnt[0], sum[1] / cnt[1], sum[2] / cnt[2], sum[3] / cnt[3]);
    };
    for (int v = 1; v <= 5; v++) kstats(v);
    // timeline of one traced chain run (u4, two streams): per kernel, block start min/max,
    // staged max, done max, signalled max (us from the first kernel's first start)
    tracing = true;
    CK(hipMemset(trace, 0, TR * 8));
    run_chain(0);
    tracing = false;
    std::vector<unsigned long long> ht(TR);
    CK(hipMemcpy(ht.data(), trace, TR * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (int b = 0; b < kblocks[0]; b++) t0 = std::min(t0, ht[4 * b]);
    const char* kn[4] = {"qkv", "wo", "w13", "w2"};
    for (int kk = 0; kk < 16; kk++) {
        unsigned long long smin = ~0ull, smax = 0, stg = 0, dmin = ~0ull, dmax = 0, sg = 0;
        const unsigned long long* T = ht.data() + (size_t)kk * 512 * 4;
        for (int b = 0; b < kblocks[kk]; b++) {
            smin = std::min(smin, T[4 * b]); smax = std::max(smax, T[4 * b]);
            stg = std::max(stg, T[4 * b + 1]); dmin = std::min(dmin, T[4 * b + 2]); dmax = std::max(dmax, T[4 * b + 2]);
            sg = std::max(sg, T[4 * b + 3]);
        }
        auto us = [&](unsigned long long t) { return (double)(t - t0) / 100.0; };
        printf("  k%-3d %-4s blocks %3d start %8.2f..%8.2f staged<=%8.2f done %8.2f..%8.2f signalled<=%8.2f\n", kk,
               kn[kk % 4], kblocks[kk], us(smin), us(smax), us(stg), us(dmin), us(dmax), us(sg));
    }
    {
        const size_t STR = (size_t)NK * 1024 * 4;
        CK(hipMalloc(&strace, STR * 8));
        CK(hipMemset(strace, 0, STR * 8));
        g_seq_pf = argc > 2 ? atoi(argv[2]) : 1;
        run_seq();
        g_seq_pf = 0;
        std::vector<unsigned long long> hq(STR);
        CK(hipMemcpy(hq.data(), strace, STR * 8, hipMemcpyDeviceToHost));
        strace = nullptr;
        unsigned long long z = ~0ull;
        for (int b = 0; b < sblocks[0]; b++) z = std::min(z, hq[4 * b]);
        const char* kn2[4] = {"qkv", "wo", "w13", "w2"};
        printf("seq timeline (us):\n");
        for (int kk = 0; kk < 12; kk++) {
            unsigned long long smin = ~0ull, smax = 0, stg = 0, stgmin = ~0ull, dmin = ~0ull, dmax = 0;
            const unsigned long long* T = hq.data() + (size_t)kk * 1024 * 4;
            for (int b = 0; b < sblocks[kk]; b++) {
                smin = std::min(smin, T[4 * b]); smax = std::max(smax, T[4 * b]);
                stg = std::max(stg, T[4 * b + 1]); stgmin = std::min(stgmin, T[4 * b + 1]);
                dmin = std::min(dmin, T[4 * b + 2]); dmax = std::max(dmax, T[4 * b + 2]);
            }
            auto us = [&](unsigned long long t) { return (double)(t - z) / 100.0; };
            printf("  k%-3d %-4s blocks %3d start %8.2f..%8.2f staged %8.2f..%8.2f done %8.2f..%8.2f\n", kk, kn2[kk % 4],
                   sblocks[kk], us(smin), us(smax), us(stgmin), us(stg), us(dmin), us(dmax));
        }
    }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    const double bytes = ((double)QKV * DIM + DIM * DIM + 2.0 * HID * DIM + (double)DIM * HID) * 2;
    printf("per layer (%.1f MB of weights):\n", bytes / 1e6);
    printf("  seq      %8.2f us  %7.1f GB/s\n", med(ts), bytes / (med(ts) * 1e-6) / 1e9);
    for (int v = 1; v <= 5; v++)
        printf("  seq v%d   %8.2f us  %7.1f GB/s\n", v, med(tv[v]), bytes / (med(tv[v]) * 1e-6) / 1e9);
    for (int r = 0; r < reps; r++) {
        tc4.push_back(run_chain(0));
        tc8.push_back(run_chain(1));
        tc1.push_back(run_chain(2));
    }
    printf("  chain u4 %8.2f us  %7.1f GB/s\n", med(tc4), bytes / (med(tc4) * 1e-6) / 1e9);
    printf("  chain u8 %8.2f us  %7.1f GB/s\n", med(tc8), bytes / (med(tc8) * 1e-6) / 1e9);
    printf("  chain 1s %8.2f us  %7.1f GB/s (one stream)\n", med(tc1), bytes / (med(tc1) * 1e-6) / 1e9);
    int ev = 0;
    CK(hipMemcpy(&ev, err, 4, hipMemcpyDeviceToHost));
    printf("err=%d\n", ev);
    return 0;
}
