// dma_bench.hip — LDS-DMA ring streaming rate on MI355X (the stream engine's weight path).
//
// One workgroup per CU; NL loader waves issue global_load_lds_dwordx4 (1 KiB per wave
// instruction) into a ring of NS slots of 16 KiB, at most DEPTH slots in flight per loader,
// publishing a slot once a counted vmcnt shows it landed; NC consumer waves wait for their
// slots, read them (16 ds_read_b128 per lane) and release them.  Each CU streams its own
// region of a large buffer.  Patterns: 0 = each slot is 16 KiB contiguous; 1 = each slot is
// 16 rows x 1 KiB at a row stride (the stream engine's tile K-step, row_bytes = 8 KiB).
// Prints GB/s over the whole buffer for each configuration.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/dma_bench tools/dma_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) int lds_i32;
__device__ __forceinline__ int vload(const int* p) { return *(volatile const lds_i32*)p; }
__device__ __forceinline__ void vstore(int* p, int v) { *(volatile lds_i32*)p = v; }

template <bool NT>
__device__ __forceinline__ void glds(const void* g, uint32_t lds) {
    unsigned keep;
    if (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
#define VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void vmcnt_le(int n) {
    switch (n) {
        VM(0) VM(16) VM(32) VM(48)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

constexpr int SLOT = 16384;
constexpr int NS = 9;

template <int NL, int NC, int DEPTH, int PAT, bool NT>
__global__ __launch_bounds__(64 * (NL + NC)) void ring_kernel(const char* buf, size_t per_cu, unsigned long long* sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* full = (int*)(smem + NS * SLOT);
    int* freew = full + 16;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 32; i += blockDim.x) full[i] = -1;
    __syncthreads();
    const int nslots = (int)(per_cu / SLOT);
    const char* base = buf + (size_t)blockIdx.x * per_cu;
    if (wid >= NC) {
        const int li = wid - NC;
        const uint32_t ring = (uint32_t)(uintptr_t)smem;
        int f0 = 0, f1 = 0, f2 = 0, nfl = 0;  // in flight (named scalars: no scratch)
        for (int s = 0; s < nslots; s++) {
            if (s % NL != li) continue;
            const int slot = s % NS;
            if (s >= NS) {
                if (vload(&freew[slot]) != s - NS) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (nfl > 0) vstore(&full[f0 % NS], f0);
                    if (nfl > 1) vstore(&full[f1 % NS], f1);
                    if (nfl > 2) vstore(&full[f2 % NS], f2);
                    nfl = 0;
                    while (vload(&freew[slot]) != s - NS) __builtin_amdgcn_s_sleep(1);
                }
            }
            if (nfl == DEPTH) {
                vmcnt_le(16 * (DEPTH - 1));
                vstore(&full[f0 % NS], f0);
                f0 = f1; f1 = f2;
                nfl--;
            }
            const uint32_t dst = ring + slot * SLOT;
            for (int p = 0; p < 16; p++) {
                const char* src;
                if (PAT == 0) {
                    src = base + (size_t)s * SLOT + p * 1024 + lane * 16;
                } else {
                    // tiles of 16 rows x 8 KiB: slot s = K-step (s % 8) of tile (s / 8)
                    const int tile = s / 8, ks = s % 8;
                    src = base + (size_t)tile * (16 * 8192) + (size_t)p * 8192 + ks * 1024 + lane * 16;
                }
                glds<NT>(src, __builtin_amdgcn_readfirstlane(dst + p * 1024));
            }
            if (nfl == 0) f0 = s; else if (nfl == 1) f1 = s; else f2 = s;
            nfl++;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (nfl > 0) vstore(&full[f0 % NS], f0);
        if (nfl > 1) vstore(&full[f1 % NS], f1);
        if (nfl > 2) vstore(&full[f2 % NS], f2);
        return;
    }
    float acc = 0.f;
    for (int s = wid; s < nslots; s += NC) {
        const int slot = s % NS;
        while (vload(&full[slot]) != s) __builtin_amdgcn_s_sleep(0);
        asm volatile("" ::: "memory");
        const float4* sp = (const float4*)(smem + slot * SLOT + lane * 16);
        float4 v[16];
#pragma unroll
        for (int p = 0; p < 16; p++) v[p] = sp[p * 64];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) vstore(&freew[slot], s);
#pragma unroll
        for (int p = 0; p < 16; p++) acc += v[p].x + v[p].y + v[p].z + v[p].w;
    }
    if (acc == 123.456f) sink[blockIdx.x] = 1;  // keep the reads
}

// the graph engine's way for comparison: every wave streams with plain nt register loads
__global__ __launch_bounds__(512) void reg_kernel(const char* buf, size_t per_cu, unsigned long long* sink) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char* base = buf + (size_t)blockIdx.x * per_cu;
    const int n = (int)(per_cu / 1024);
    float acc = 0.f;
    for (int i = wid * 4; i < n; i += 8 * 4) {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        u4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            v[u] = __builtin_nontemporal_load((const __attribute__((address_space(1))) u4*)(base + (size_t)(i + u) * 1024 + lane * 16));
#pragma unroll
        for (int u = 0; u < 4; u++) acc += __builtin_bit_cast(float, v[u].x);
    }
    if (acc == 123.456f) sink[blockIdx.x] = 1;
}

// KV-cache access patterns of long-context attention (rows of 2 KiB = 8 heads x 256 B), register
// loads, 1024-thread workgroups, one round = 4 loads of 16 B per thread.
//   HEADS=1 : workgroup (head g = b % 8, split b / 8) reads 256 B of each of its rows (today)
//   HEADS=8 : workgroup (split b) reads whole 2 KiB rows
//   PIPE    : rounds in flight (1 = load, wait, next; 2 = next round requested before the wait)
template <int HEADS, int PIPE>
__global__ __launch_bounds__(1024) void kv_kernel(const char* kv, int rows_per_wg, unsigned long long* sink) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x;
    const int lpr = 16 * HEADS;             // lanes per row
    const int rpp = 1024 / lpr;             // rows per pass
    const int g = HEADS == 1 ? blockIdx.x % 8 : 0;
    const int split = HEADS == 1 ? blockIdx.x / 8 : blockIdx.x;
    const size_t row0 = (size_t)split * rows_per_wg;
    const int sub = tid % lpr, rr = tid / lpr;
    const char* base = kv + row0 * 2048 + g * 256 + sub * 16;
    float acc = 0.f;
    const int rounds = rows_per_wg / (4 * rpp);
    u4 cur[4], nxt[4];
    auto load = [&](u4 (&v)[4], int r) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const size_t row = (size_t)r * 4 * rpp + p * rpp + rr;
            v[p] = *(const __attribute__((address_space(1))) u4*)(base + row * 2048);
        }
    };
    if (PIPE == 1) {
        for (int r = 0; r < rounds; r++) {
            load(cur, r);
#pragma unroll
            for (int p = 0; p < 4; p++) acc += __builtin_bit_cast(float, cur[p].x);
        }
    } else {
        load(cur, 0);
        for (int r = 0; r < rounds; r++) {
            if (r + 1 < rounds) load(nxt, r + 1);
#pragma unroll
            for (int p = 0; p < 4; p++) acc += __builtin_bit_cast(float, cur[p].x);
#pragma unroll
            for (int p = 0; p < 4; p++) cur[p] = nxt[p];
        }
    }
    if (acc == 123.456f) sink[blockIdx.x] = 1;
}

template <int HEADS, int PIPE>
void run_kv(const char* kv, size_t bytes, int ncu, int wg_per_cu, unsigned long long* sink) {
    const int nwg = ncu * wg_per_cu;
    const size_t rows = bytes / 2048;
    const int rows_per_wg = (int)(rows * (HEADS == 1 ? 8 : 1) / nwg);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto k = kv_kernel<HEADS, PIPE>;
    for (int it = 0; it < 2; it++) hipLaunchKernelGGL(k, dim3(nwg), dim3(1024), 0, 0, kv, rows_per_wg, sink);
    hipEventRecord(e0);
    for (int it = 0; it < 5; it++) hipLaunchKernelGGL(k, dim3(nwg), dim3(1024), 0, 0, kv, rows_per_wg, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("kv pattern heads/wg=%d rounds in flight=%d wg/cu=%d rows/wg=%5d : %7.1f GB/s (%.1f us)\n", HEADS, PIPE,
           wg_per_cu, rows_per_wg, (double)bytes * 5 / (ms * 1e-3) / 1e9, ms * 1000 / 5);
}

template <int NL, int NC, int DEPTH, int PAT, bool NT>
void run(const char* buf, size_t per_cu, int ncu, unsigned long long* sink, const char* name) {
    auto k = ring_kernel<NL, NC, DEPTH, PAT, NT>;
    const size_t smem = NS * SLOT + 256;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int it = 0; it < 2; it++) hipLaunchKernelGGL(k, dim3(ncu), dim3(64 * (NL + NC)), smem, 0, buf, per_cu, sink);
    hipEventRecord(e0);
    const int iters = 5;
    for (int it = 0; it < iters; it++) hipLaunchKernelGGL(k, dim3(ncu), dim3(64 * (NL + NC)), smem, 0, buf, per_cu, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double gbs = (double)per_cu * ncu * iters / (ms * 1e-3) / 1e9;
    printf("%-44s NL=%d NC=%d DEPTH=%d pat=%d nt=%d : %7.1f GB/s (%.1f us per launch)\n", name, NL, NC, DEPTH, PAT, NT,
           gbs, ms * 1000 / iters);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) printf("error %s\n", hipGetErrorString(err));
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t per_cu = (size_t)8 << 20;  // 8 MiB per CU = 2 GiB over 256 CUs (past the 256 MiB cache)
    char* buf = nullptr;
    unsigned long long* sink = nullptr;
    if (hipMalloc(&buf, per_cu * ncu) != hipSuccess || hipMalloc(&sink, 8 * ncu) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 0, per_cu * ncu);
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int it = 0; it < 2; it++) hipLaunchKernelGGL(reg_kernel, dim3(ncu * 2), dim3(512), 0, 0, buf, per_cu / 2, sink);
        hipEventRecord(e0);
        for (int it = 0; it < 5; it++) hipLaunchKernelGGL(reg_kernel, dim3(ncu * 2), dim3(512), 0, 0, buf, per_cu / 2, sink);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s : %7.1f GB/s\n", "register nt loads, 16 waves/CU x 4 KiB", (double)per_cu * ncu * 5 / (ms * 1e-3) / 1e9);
    }
    // one 32k-context layer: K (or V) ring = 32768 rows x 2 KiB = 64 MiB; 128 MiB = K and V
    const size_t kvb = (size_t)128 << 20;
    run_kv<1, 1>(buf, kvb, ncu, 1, sink);
    run_kv<1, 2>(buf, kvb, ncu, 1, sink);
    run_kv<1, 1>(buf, kvb, ncu, 2, sink);
    run_kv<1, 2>(buf, kvb, ncu, 2, sink);
    run_kv<8, 1>(buf, kvb, ncu, 1, sink);
    run_kv<8, 2>(buf, kvb, ncu, 1, sink);
    run_kv<8, 2>(buf, kvb, ncu, 2, sink);
    run<1, 7, 3, 1, true>(buf, per_cu, ncu, sink, "ring, strided tiles (stream engine today)");
    run<1, 7, 3, 0, true>(buf, per_cu, ncu, sink, "ring, contiguous slots");
    run<1, 7, 2, 1, true>(buf, per_cu, ncu, sink, "ring, strided, depth 2");
    run<1, 7, 3, 1, false>(buf, per_cu, ncu, sink, "ring, strided, default policy");
    run<2, 6, 3, 1, true>(buf, per_cu, ncu, sink, "ring, strided, 2 loaders");
    run<3, 5, 3, 1, true>(buf, per_cu, ncu, sink, "ring, strided, 3 loaders");
    run<4, 4, 2, 1, true>(buf, per_cu, ncu, sink, "ring, strided, 4 loaders depth 2");
    run<2, 6, 3, 0, true>(buf, per_cu, ncu, sink, "ring, contiguous, 2 loaders");
    run<3, 5, 3, 0, true>(buf, per_cu, ncu, sink, "ring, contiguous, 3 loaders");
    return 0;
}
