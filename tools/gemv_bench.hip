// gemv_bench.hip — one-process A/B of gemv launch shapes on the Mistral-7B matrix shapes.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/gemv_bench tools/gemv_bench.hip
//   fp8 e4m3 weights: add -DGB_DT=XH_F8_E4M3 (-o tools/gemv_bench_f8)
// Each shape rotates over enough weight copies (> 1 GB) that the 256 MB Infinity Cache
// cannot serve repeats; variants are interleaved over rounds (guide §5.4 rule 24).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../include/xalm_synth.h"
#include "../xalm_amd/csrc/gemv.h"

using namespace xalm;

#ifndef GB_DT
#define GB_DT XH_F16
#endif
constexpr int DT = GB_DT;
constexpr int ESZ = DT == XH_F16 ? 2 : 1;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(uint16_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_to_f16(xs_value(seed, i, 0.f, 0.02f));
}
__global__ void fill8(uint8_t* p, size_t n, uint64_t seed) {  // e4m3 bytes, no NaN code
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint8_t)(xs_to_f16(xs_value(seed, i, 0.f, 1.f)) >> 3) & 0xF7;
}
__global__ void fillf(float* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_value(seed, i, 0.f, 1.f);
}

struct Mat { const char* name; int rows, n, pro, epi; };

template <int PRO, int EPI, class S>
void launch(const GemvArgs& a, int max_waves) {
    const size_t smem = gemv_smem_bytes<DT, S>(a.n);
    const int blocks = gemv_blocks<S>(a.rows, max_waves / S::WAVES);
    auto k = gemv_kernel<DT, PRO, EPI, S>;
    static bool once = false;
    if (!once) { CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); once = true; }
    hipLaunchKernelGGL(k, dim3(blocks), dim3(S::THREADS), smem, 0, a);
}

template <class S>
void launch_any(const Mat& m, const GemvArgs& a, int mw) {
    if (m.pro == PRO_RMSNORM && m.epi == EPI_GLU) launch<PRO_RMSNORM, EPI_GLU, S>(a, mw);
    else if (m.pro == PRO_RMSNORM) launch<PRO_RMSNORM, EPI_STORE, S>(a, mw);
    else launch<PRO_PLAIN, EPI_RESID, S>(a, mw);
}

struct Variant { std::string name; std::function<void(const Mat&, const GemvArgs&)> fn; };

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 40;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    std::vector<Mat> mats = {{"w13 28672x4096", 28672, 4096, PRO_RMSNORM, EPI_GLU},
                             {"w2 4096x14336", 4096, 14336, PRO_PLAIN, EPI_RESID},
                             {"qkv 6144x4096", 6144, 4096, PRO_RMSNORM, EPI_STORE},
                             {"wo 4096x4096", 4096, 4096, PRO_PLAIN, EPI_RESID},
                             {"cls 32000x4096", 32000, 4096, PRO_RMSNORM, EPI_STORE}};
    float *x, *out, *nw;
    CK(hipMalloc(&x, 14336 * 4));
    CK(hipMalloc(&out, 32000 * 4));
    CK(hipMalloc(&nw, 14336 * 4));
    hipLaunchKernelGGL(fillf, dim3(64), dim3(256), 0, 0, x, 14336, 7);
    hipLaunchKernelGGL(fillf, dim3(64), dim3(256), 0, 0, nw, 14336, 8);
    std::vector<std::vector<uint16_t*>> copies(mats.size());
    for (size_t i = 0; i < mats.size(); i++) {
        const size_t elems = (size_t)mats[i].rows * mats[i].n;
        const int nc = std::max<int>(2, (int)((1400ull << 20) / (elems * ESZ)) + 1);
        for (int c = 0; c < nc; c++) {
            uint16_t* p;
            CK(hipMalloc(&p, elems * ESZ));
            if (ESZ == 2) hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, p, elems, 100 + i * 10 + c);
            else hipLaunchKernelGGL(fill8, dim3(2048), dim3(256), 0, 0, (uint8_t*)p, elems, 100 + i * 10 + c);
            copies[i].push_back(p);
        }
    }
    CK(hipDeviceSynchronize());

#define V(NAME, MW, ...) {NAME, [](const Mat& m, const GemvArgs& a) { launch_any<GemvShape<__VA_ARGS__>>(m, a, MW); }}
    // PF shapes as the product picks them: x in 2 float4 per thread for n <= 4096, else 8
#define VPF(NAME, MW, T, R, U) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n <= 4096) launch_any<GemvShape<T, R, U, true, 4, true, 2>>(m, a, MW); \
        else launch_any<GemvShape<T, R, U, true, 4, true, 8>>(m, a, MW); }}
#define VPP(NAME, MW, T, R, U, MINW) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n <= 4096) launch_any<GemvShape<T, R, U, true, MINW, true, 2, 2>>(m, a, MW); \
        else launch_any<GemvShape<T, R, U, true, MINW, true, 8, 2>>(m, a, MW); }}
    // 1024-thread workgroups (one per CU: a CU's second workgroup no longer stages x behind the
    // first one's weight requests); x in 1 float4 per thread for n <= 4096, else 4
#define VPK(NAME, MW, R, U) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n <= 4096) launch_any<GemvShape<1024, R, U, true, 4, true, 1, 2>>(m, a, MW); \
        else launch_any<GemvShape<1024, R, U, true, 4, true, 4, 2>>(m, a, MW); }}
    // W2-shaped (n = 14336) launch shapes: x in 8 float4 per thread; PIPE 2 needs n % (64 E U) == 0
#define VW2(NAME, MW, R, U, P) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n > 4096) launch_any<GemvShape<512, R, U, true, 4, true, 8, P>>(m, a, MW); }}
#define VW2T(NAME, MW, T, R, U, P) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n > 4096) launch_any<GemvShape<T, R, U, true, 4, true, (14336 / 4 + T - 1) / T, P>>(m, a, MW); }}
    // per-CU balance (GB_BAL): the product's 512-thread grids give W1/W3 448 workgroups (64 CUs
    // with one, 192 with two) and qkv 192; these give every CU the same row-group count
#define VB(NAME, MW, T, MINW) {NAME, [](const Mat& m, const GemvArgs& a) { \
        if (m.n <= 4096) launch_any<GemvShape<T, 2, 4, true, MINW, true, (4096 / 4 + T - 1) / T, 2>>(m, a, MW); }}
    std::vector<Variant> vs = getenv("GB_BAL") ? std::vector<Variant>{
        VPP("t512 r2 u4 pf pipe2 (product)", 4096, 512, 2, 4, 4),
        VPP("t512 w2048 (product qkv)", 2048, 512, 2, 4, 4),
        VB("t448 w3584 (2/CU x 7 waves)", 3584, 448, 4),
        VB("t896 w3584 (1/CU x 14)", 3584, 896, 4),
        VB("t384 w3072 (2/CU x 6)", 3072, 384, 3),
        VB("t768 w3072 (1/CU x 12)", 3072, 768, 3),
        VB("t512 w4096 (2/CU x 8)", 4096, 512, 4),
        VB("t256 w4096 (4/CU x 4)", 4096, 256, 4),
        VB("t448 w1792 (1/CU x 7)", 1792, 448, 2),
    } : getenv("GB_W2") ? std::vector<Variant>{
        VW2("w2 r2 u4 (product)", 4096, 2, 4, 1),
        VW2("w2 r2 u7", 4096, 2, 7, 1),
        VW2("w2 r2 u7 pipe2", 4096, 2, 7, 2),
        VW2("w2 r1 u7 pipe2", 4096, 1, 7, 2),
        VW2("w2 r2 u2 pipe2", 4096, 2, 2, 2),
        VW2("w2 r2 u4 pipe2 (f16 only)", 4096, 2, 4, 2),
        VW2("w2 r1 u4", 4096, 1, 4, 1),
        VW2("w2 r2 u7 pipe2 w2048", 2048, 2, 7, 2),
        VW2T("w2 t256 r2 u4 w2048 (2/CU x 4)", 2048, 256, 2, 4, 1),
        VW2T("w2 t512 r1 u4 w4096", 4096, 512, 1, 4, 1),
        VW2T("w2 t256 r1 u4 w4096 (4/CU x 4)", 4096, 256, 1, 4, 1),
        VW2T("w2 t384 r1 u4 w3072 (2/CU x 6)", 3072, 384, 1, 4, 1),
        VW2T("w2 t1024 r1 u4 w4096 (1/CU)", 4096, 1024, 1, 4, 1),
        VW2T("w2 t256 r2 u4 pipe2 w2048 (f16 only)", 2048, 256, 2, 4, 2),
    } : getenv("GB_T1K") ? std::vector<Variant>{
        VPP("t512 r2 u4 pf pipe2 (product)", 4096, 512, 2, 4, 4),
        VPK("t1024 r2 u4 pipe2 w4096", 4096, 2, 4),
        VPK("t1024 r2 u4 pipe2 w3072", 3072, 2, 4),
        VPK("t1024 r1 u4 pipe2 w4096", 4096, 1, 4),
        VPK("t1024 r2 u2 pipe2 w4096", 4096, 2, 2),
        VPP("t512 r2 u4 pf pipe2 w2048", 2048, 512, 2, 4, 2),
    } : getenv("GB_PIPE") ? std::vector<Variant>{
        VPF("t512 r2 u4 pf (product)", 4096, 512, 2, 4),
        VPP("t512 r2 u4 pf pipe2", 4096, 512, 2, 4, 4),
        VPP("t512 r2 u2 pf pipe2", 4096, 512, 2, 2, 4),
        VPP("t512 r1 u4 pf pipe2", 4096, 512, 1, 4, 4),
        VPP("t512 r2 u4 pf pipe2 w2048", 2048, 512, 2, 4, 2),
        VPP("t256 r2 u4 pf pipe2", 4096, 256, 2, 4, 4),
        VPP("t512 r4 u2 pf pipe2", 4096, 512, 4, 2, 4),
    } : DT != XH_F16 ? std::vector<Variant>{
        VPF("t512 r2 u4 pf (product)", 4096, 512, 2, 4),
        VPF("t512 r4 u4 pf", 4096, 512, 4, 4),
        VPF("t512 r2 u4 pf w8192", 8192, 512, 2, 4),
        VPF("t512 r4 u2 pf", 4096, 512, 4, 2),
        V("t512 r2 u4 nt --  w4096", 4096, 512, 2, 4, true, 4, false),
        V("t512 r4 u4 nt --  w4096", 4096, 512, 4, 4, true, 4, false),
    } : std::vector<Variant>{
        V("t512 r2 u4 nt --  w4096", 4096, 512, 2, 4, true, 4, false),
        V("t512 r1 u8 nt --  w4096", 4096, 512, 1, 8, true, 4, false),
        VPF("t512 r2 u4 pf (product)", 4096, 512, 2, 4),
        V("t512 r2 u8 nt --  w4096", 4096, 512, 2, 8, true, 4, false),
        V("t256 r1 u8 nt --  w4096", 4096, 256, 1, 8, true, 4, false),
        V("t512 r1 u16 nt -- w2048 mw2", 2048, 512, 1, 16, true, 2, false),
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // results[mat][variant] = list of us
    std::vector<std::vector<std::vector<float>>> res(mats.size(), std::vector<std::vector<float>>(vs.size()));
    for (int r = 0; r < rounds; r++)
        for (size_t mi = 0; mi < mats.size(); mi++)
            for (size_t vi = 0; vi < vs.size(); vi++) {
                const Mat& m = mats[mi];
                if (getenv("GB_W2") && m.n <= 4096) continue;
                if (getenv("GB_BAL") && m.n > 4096) continue;
                if (getenv("GB_W2") && DT != XH_F16 && vs[vi].name.find("f16 only") != std::string::npos) continue;
                if (m.n > 8192 && std::string(vs[vi].name).find("t128") == 0) continue;
                GemvArgs a{};
                a.row_bytes = (size_t)m.n * ESZ; a.n = m.n; a.rows = m.rows; a.x = x; a.norm_w = nw;
                a.norm_dtype = XH_F32; a.eps = 1e-5f; a.out = out; a.act = XH_ACT_SILU;
                for (int i = 0; i < 2; i++) { a.w = copies[mi][i % copies[mi].size()]; vs[vi].fn(m, a); }
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < iters; i++) { a.w = copies[mi][i % copies[mi].size()]; vs[vi].fn(m, a); }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipGetLastError());
                res[mi][vi].push_back(ms * 1000.f / iters);
            }
    for (size_t mi = 0; mi < mats.size(); mi++) {
        const double bytes = (double)mats[mi].rows * mats[mi].n * ESZ;
        printf("%s  (%.1f MB)\n", mats[mi].name, bytes / 1e6);
        for (size_t vi = 0; vi < vs.size(); vi++) {
            auto v = res[mi][vi];
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            printf("   %-28s median %8.2f us  min %8.2f  -> %7.1f GB/s\n", vs[vi].name.c_str(), v[v.size() / 2], v[0],
                   bytes / (v[v.size() / 2] * 1e-6) / 1e9);
        }
    }
    return 0;
}
