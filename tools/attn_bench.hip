// attn_bench.hip — long-context attention variants, one process (Mistral-7B shapes: 8 KV heads,
// 4 q per KV, head_dim 128, fp16 ring).  Times the split (partials) phase alone:
//   round  : attn_block<PARTIALS>  (score pass + softmax + p.V pass, 256-row rounds)
//   merged : attn_block<SIGNAL>    (the last split of each head merges, attn_wo long contexts)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/attn_bench tools/attn_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "../include/xalm_synth.h"
#include "../xalm_amd/csrc/attention.h"

using namespace xalm;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int HD = 128, QPK = 4, NKV = 8, NH = 32, KVD = NKV * HD;

__global__ void fill16(uint16_t* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_to_f16(xs_value(seed, i, 0.f, 1.f));
}
__global__ void fillf(float* p, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = xs_value(seed, i, 0.f, 1.f);
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_round(const AttnArgs a, unsigned* done) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    attn_block<HD, QPK, THREADS, true>(a, blockIdx.x / a.nsplit, blockIdx.x % a.nsplit, smem, done);
}
// timeline of the long split (attn_block's stamps: 2 split known, 3 scores done, 6 softmax done,
// 7 p.V done, 4 reduced, 5 partial drained), one record of 8 words per workgroup
__device__ unsigned long long g_stamps[8 * 1024];
template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_stamp(const AttnArgs a, unsigned* done) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    unsigned long long* d = g_stamps + 8 * blockIdx.x;
    if (threadIdx.x == 0) d[0] = __builtin_amdgcn_s_memrealtime();
    attn_block<HD, QPK, THREADS, false, attn_min_t_partials(HD, THREADS), NoWait, AddArrive, true>(
        a, blockIdx.x / a.nsplit, blockIdx.x % a.nsplit, smem, done, d);
    __syncthreads();
    if (threadIdx.x == 0) d[1] = __builtin_amdgcn_s_memrealtime();
}
template <int THREADS>
__global__ __launch_bounds__(THREADS) void k_signal(const AttnArgs a, unsigned* done) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    attn_block<HD, QPK, THREADS, false, attn_min_t_partials(HD, THREADS), NoWait, AddArrive, true>(
        a, blockIdx.x / a.nsplit, blockIdx.x % a.nsplit, smem, done);
}

// diagnostic floor: the split's K rows then V rows (same per-thread addresses as attn_block:
// 16 lanes per 256-B row slice, ATTN_PREF rows per thread per round) with D rounds in flight,
// nothing computed but an xor (the memory side of the round loop alone)
// HM: head-major ring ([g][slot][HD], 32768 slots per head) instead of [slot][kv_dim]
template <int THREADS, int D, bool HM = false>
__global__ __launch_bounds__(THREADS) void k_stream(const AttnArgs a, unsigned* sink) {
    constexpr int LPR = HD / 8, RPP = THREADS / LPR, STEP = ATTN_PREF * RPP;
    const int g = blockIdx.x / a.nsplit, s = blockIdx.x % a.nsplit;
    const int kv_len = a.sp->kv_len;
    const int T = attn_split_len(kv_len, a.nsplit, attn_min_t_partials(HD, THREADS));
    const int t0 = s * T, t1 = min(kv_len, t0 + T);
    if (t0 >= kv_len) return;
    const int sub = threadIdx.x % LPR, rr = threadIdx.x / LPR;
    const size_t col = HM ? (size_t)g * 32768 * HD + sub * 8 : (size_t)g * HD + sub * 8;
    const size_t pitch = HM ? HD : a.kv_dim;
    uint32_t acc = 0;
    for (int pass = 0; pass < 2; pass++) {
        const uint16_t* base = pass ? a.vc : a.kc;
        u32x4 r[D][ATTN_PREF];
        int nr = (t1 - t0 + STEP - 1) / STEP;
#pragma unroll
        for (int d = 0; d < D; d++)
#pragma unroll
            for (int p = 0; p < ATTN_PREF; p++)
                r[d][p] = __builtin_nontemporal_load((const u32x4*)(base + (size_t)min(t0 + d * STEP + rr + p * RPP, t1 - 1) * pitch + col));
        for (int k = 0; k < nr; k += D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
#pragma unroll
                for (int p = 0; p < ATTN_PREF; p++) acc ^= r[d][p].x ^ r[d][p].w;
#pragma unroll
                for (int p = 0; p < ATTN_PREF; p++)
                    r[d][p] = __builtin_nontemporal_load((const u32x4*)(base + (size_t)min(t0 + (k + d + D) * STEP + rr + p * RPP, t1 - 1) * pitch + col));
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int msl = 32768;
    const int kv_len = argc > 1 ? atoi(argv[1]) : 32768;
    // slot pitch in fp16 elements (KVD + pad): how the ring's row pitch maps KV heads onto HBM channels
    const int pad = argc > 2 ? atoi(argv[2]) : 0;
    const int PITCH = KVD + pad;
    const int NC = 4;  // ring copies (4 x 128 MB) so the Infinity Cache serves nothing
    std::vector<uint16_t*> kc(NC), vc(NC);
    for (int c = 0; c < NC; c++) {
        CK(hipMalloc(&kc[c], (size_t)msl * PITCH * 2));
        CK(hipMalloc(&vc[c], (size_t)msl * PITCH * 2));
        hipLaunchKernelGGL(fill16, dim3(2048), dim3(256), 0, 0, kc[c], (size_t)msl * PITCH, 10 + c);
        hipLaunchKernelGGL(fill16, dim3(2048), dim3(256), 0, 0, vc[c], (size_t)msl * PITCH, 20 + c);
    }
    float *q, *po, *pml, *out;
    int* cnt;
    CK(hipMalloc(&out, NH * HD * 4));
    CK(hipMalloc(&cnt, 64));
    CK(hipMemset(cnt, 0, 64));
    unsigned* done;
    StepParams* sp;
    CK(hipMalloc(&q, NH * HD * 4));
    CK(hipMalloc(&po, (size_t)128 * NH * HD * 4));
    CK(hipMalloc(&pml, (size_t)128 * NH * 2 * 4));
    CK(hipMalloc(&done, 4));
    CK(hipMalloc(&sp, sizeof(StepParams)));
    hipLaunchKernelGGL(fillf, dim3(16), dim3(256), 0, 0, q, NH * HD, 3);
    StepParams h{};
    h.kv_len = kv_len; h.pos = kv_len - 1; h.kv_pos = kv_len - 1; h.max_seq_len = msl;
    CK(hipMemcpy(sp, &h, sizeof h, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](auto kern, int threads, int nsplit, size_t smem, const char* name) {
        CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        AttnArgs a{};
        a.q = q; a.kv_dim = PITCH; a.n_heads = NH; a.nsplit = nsplit; a.part_o = po; a.part_ml = pml; a.sp = sp; a.out = out; a.counters = cnt;
        std::vector<float> ts;
        for (int r = 0; r < 3; r++) {
            const int it = 20;
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < it; i++) {
                a.kc = kc[i % NC]; a.vc = vc[i % NC];
                hipLaunchKernelGGL(kern, dim3(NKV * nsplit), dim3(threads), smem, 0, a, done);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms * 1000 / it);
        }
        std::sort(ts.begin(), ts.end());
        const double bytes = 2.0 * kv_len * KVD * 2;
        printf("  %-22s nsplit %3d  %8.2f us  %7.1f GB/s\n", name, nsplit, ts[1], bytes / (ts[1] * 1e-6) / 1e9);
    };
    printf("kv_len %d (%.1f MB of K+V), slot pitch %d\n", kv_len, 2.0 * kv_len * KVD * 2 / 1e6, PITCH);
    const bool quick = argc > 3;
    for (int ns : {32, 64}) {
        const int T = attn_split_len(kv_len, ns, attn_min_t_partials(HD, 1024));
        run(k_stream<1024, 2>, 1024, ns, 0, "stream  t1024 D2");
        run(k_stream<1024, 3>, 1024, ns, 0, "stream  t1024 D3");
        run(k_stream<1024, 4>, 1024, ns, 0, "stream  t1024 D4");
        run(k_stream<1024, 2, true>, 1024, ns, 0, "stream HM t1024 D2");
        run(k_stream<1024, 3, true>, 1024, ns, 0, "stream HM t1024 D3");
        run(k_round<1024>, 1024, ns, attn_smem_bytes(HD, QPK, T, ns, 1024), "round   t1024");
    }
    {
        // timeline of one launch at 32 splits (100 MHz realtime counter: 10 ns ticks)
        const int ns = 32;
        const int T = attn_split_len(kv_len, ns, attn_min_t_partials(HD, 1024));
        run(k_stamp<1024>, 1024, ns, attn_smem_bytes(HD, QPK, T, ns, 1024), "stamped t1024");
        std::vector<unsigned long long> st(8 * NKV * ns);
        CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < NKV * ns; b++) t0 = std::min(t0, st[8 * b]);
        double acc[8] = {};
        int cnt = 0;
        for (int b = 0; b < NKV * ns; b++) {
            const unsigned long long* d = &st[8 * b];
            if (!d[3] || !d[6] || !d[7]) continue;
            acc[0] += (d[0] - t0) * 0.01; acc[1] += (d[3] - d[0]) * 0.01; acc[2] += (d[6] - d[3]) * 0.01;
            acc[3] += (d[7] - d[6]) * 0.01; acc[4] += (d[1] - d[7]) * 0.01; acc[5] += (d[1] - t0) * 0.01;
            cnt++;
        }
        printf("  timeline (us, mean of %d splits): start %.2f, K pass %.2f, softmax %.2f, p.V pass %.2f, tail %.2f, end %.2f\n",
               cnt, acc[0] / cnt, acc[1] / cnt, acc[2] / cnt, acc[3] / cnt, acc[4] / cnt, acc[5] / cnt);
    }
    for (int ns : {16, 32, 64, 128}) {
        if (quick && ns > 32) continue;
        const int T = attn_split_len(kv_len, ns, attn_min_t_partials(HD, 1024));
        run(k_round<1024>, 1024, ns, attn_smem_bytes(HD, QPK, T, ns, 1024), "round   t1024");
        run(k_signal<1024>, 1024, ns, attn_smem_bytes(HD, QPK, T, ns, 1024), "merged  t1024");
        const int T5 = attn_split_len(kv_len, ns, attn_min_t_partials(HD, 512));
        run(k_round<512>, 512, ns, attn_smem_bytes(HD, QPK, T5, ns, 512), "round   t512");
        run(k_signal<512>, 512, ns, attn_smem_bytes(HD, QPK, T5, ns, 512), "merged  t512");
    }
    return 0;
}
