// stream_bench.hip — the weight-stream ceiling of a batch-1 matvec on MI355X.
//
// Reads a 234.9 MB matrix (Mistral-7B W1/W3: 28672 rows x 8 KiB) per launch, rotating over 8
// copies (1.9 GB, beyond the 256 MB Infinity Cache), in the gemv row-group pattern: a wave owns
// ROWS consecutive 8-KiB rows, lane l reads 16-B chunks l, l + 64, ... of each row, U chunks per
// row per step, two register sets (the next step is requested before the current one is used).
// Variants: destination VGPR (global_load_dwordx4, nt or default policy) or LDS (LDS-DMA
// global_load_lds_dwordx4, nt or default, one per-wave double-buffered slot, consumed by
// ds_read_b128).  The consumer only folds the bytes (no dot product): this is the rate the
// memory system gives the pattern, the ceiling for gemv_kernel<..., GLU>.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/stream_bench tools/stream_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u4* gp4;


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

// VGPR destination, gemv_rows_pipe's stream: step k = group g0 + (k / steps) * total_waves,
// chunks [(k % steps) * U, + U)
template <int THREADS, int ROWS, int U, bool NT>
__global__ __launch_bounds__(THREADS) void reg_kernel(const char* w, unsigned* sink, const int nrows, const int row_bytes) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int WAVES = THREADS / 64;
    const int total_waves = gridDim.x * WAVES;
    const int g0 = blockIdx.x * WAVES + wid;
    const int n_groups = nrows / ROWS;
    const int steps = row_bytes / (1024 * U);
    const int ROW_BYTES = row_bytes;
    if (g0 >= n_groups) return;
    const int total = ((n_groups - g0 + total_waves - 1) / total_waves) * steps;
    auto load = [&](u4 (&v)[U][ROWS], const int k) {
        const int q = k / steps;
        const char* base = w + (size_t)(g0 + q * total_waves) * ROWS * ROW_BYTES + (k - q * steps) * U * 1024 + lane * 16;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < ROWS; r++) {
                gp4 p = (gp4)(base + (size_t)r * ROW_BYTES + u * 1024);
                v[u][r] = NT ? __builtin_nontemporal_load(p) : *p;
            }
    };
    uint32_t acc = 0;
    auto use = [&](const u4 (&v)[U][ROWS]) {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < ROWS; r++) acc ^= v[u][r].x ^ v[u][r].y ^ v[u][r].z ^ v[u][r].w;
    };
    u4 a[U][ROWS], b[U][ROWS];
    load(a, 0);
    int k = 0;
    for (; k + 2 < total; k += 2) {
        load(b, k + 1);
        use(a);
        load(a, k + 2);
        use(b);
    }
    if (k + 1 < total) {
        load(b, k + 1);
        use(a);
        use(b);
    } else {
        use(a);
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

// LDS destination: each wave streams the same steps through two LDS slots of U * ROWS KiB
// (LDS-DMA), waiting with a counted vmcnt for the older slot and reading it with ds_read_b128.
template <int THREADS, int ROWS, int U, bool NT>
__global__ __launch_bounds__(THREADS) void lds_kernel(const char* w, unsigned* sink, const int nrows, const int row_bytes) {
    const int ROW_BYTES = row_bytes;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int WAVES = THREADS / 64;
    constexpr int SLOT = U * ROWS * 1024;
    const int total_waves = gridDim.x * WAVES;
    const int g0 = blockIdx.x * WAVES + wid;
    const int n_groups = nrows / ROWS;
    const int steps = row_bytes / (1024 * U);
    if (g0 >= n_groups) return;
    const int total = ((n_groups - g0 + total_waves - 1) / total_waves) * steps;
    const uint32_t my = (uint32_t)(uintptr_t)smem + wid * 2 * SLOT;
    auto load = [&](const int set, const int k) {
        const int q = k / steps;
        const char* base = w + (size_t)(g0 + q * total_waves) * ROWS * ROW_BYTES + (k - q * steps) * U * 1024 + lane * 16;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < ROWS; r++)
                glds<NT>(base + (size_t)r * ROW_BYTES + u * 1024,
                         __builtin_amdgcn_readfirstlane(my + set * SLOT + (u * ROWS + r) * 1024));
    };
    uint32_t acc = 0;
    auto use = [&](const int set) {
        const u4* sp = (const u4*)(smem + wid * 2 * SLOT + set * SLOT + lane * 16);
#pragma unroll
        for (int i = 0; i < U * ROWS; i++) {
            const u4 v = sp[i * 64];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    };
    constexpr int N = U * ROWS;
    load(0, 0);
    for (int k = 0; k < total; k++) {
        if (k + 1 < total) {
            load((k + 1) & 1, k + 1);
            if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        use(k & 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot is free before it is refilled
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__global__ void fill(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)(i * 2654435761u);
}

constexpr int COPIES = 8;
constexpr size_t BUF = 256ull << 20;  // per copy: the largest matrix rounded up

template <class F>
double time_us(F launch, const std::vector<char*>& bufs, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < COPIES; i++) launch(bufs[i % COPIES]);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) launch(bufs[i % COPIES]);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1000.0 / iters;
}

struct Row { std::string name; double bytes; double us; };

// K/V ring of one layer at 32k slots (rows of 2 KiB = 8 KV heads x 256 B), K then V, register
// loads, nt, two rounds of 4 x 16 B per thread in flight.
//   HEADS = 1: workgroup (KV head b % 8, split b / 8) reads its 256-B slice of each of its rows
//              (the decode attention's split layout)
//   HEADS = 8: workgroup (split b) reads whole 2-KiB rows (every KV head of a slot range)
template <int HEADS, int THREADS>
__global__ __launch_bounds__(THREADS) void kv_kernel(const char* kc, const char* vc, const int rows_per_wg, unsigned* sink) {
    const int tid = threadIdx.x;
    constexpr int LPR = 16 * HEADS;       // lanes per row
    constexpr int RPP = THREADS / LPR;    // rows per pass
    const int g = HEADS == 1 ? blockIdx.x % 8 : 0;
    const int split = HEADS == 1 ? blockIdx.x / 8 : blockIdx.x;
    const size_t row0 = (size_t)split * rows_per_wg;
    const int sub = tid % LPR, rr = tid / LPR;
    uint32_t acc = 0;
    const int rounds = rows_per_wg / (4 * RPP);
    for (int which = 0; which < 2; which++) {
        const char* base = (which ? vc : kc) + row0 * 2048 + g * 256 + sub * 16;
        u4 cur[4], nxt[4];
        auto load = [&](u4 (&v)[4], int r) {
#pragma unroll
            for (int p = 0; p < 4; p++)
                v[p] = __builtin_nontemporal_load((gp4)(base + ((size_t)r * 4 * RPP + p * RPP + rr) * 2048));
        };
        load(cur, 0);
        for (int r = 0; r < rounds; r++) {
            if (r + 1 < rounds) load(nxt, r + 1);
#pragma unroll
            for (int p = 0; p < 4; p++) acc ^= cur[p].x ^ cur[p].y;
#pragma unroll
            for (int p = 0; p < 4; p++) cur[p] = nxt[p];
        }
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

template <int HEADS, int THREADS>
void kv_variant(std::vector<Row>& out, const std::vector<char*>& bufs, unsigned* sink, int nwg, const char* name) {
    constexpr size_t RING = 32768ull * 2048;  // one layer's K (or V)
    const int rows_per_wg = (int)(32768ull * (HEADS == 1 ? 8 : 1) / nwg);
    auto launch = [&](char* b) {
        hipLaunchKernelGGL((kv_kernel<HEADS, THREADS>), dim3(nwg), dim3(THREADS), 0, 0, b, b + RING, rows_per_wg, sink);
    };
    out.push_back({name, 2.0 * RING, time_us(launch, bufs, 32)});
}


template <int THREADS, int ROWS, int U, bool NT, bool LDS>
void variant(std::vector<Row>& out, const std::vector<char*>& bufs, unsigned* sink, int blocks, int nrows, int row_bytes,
             const char* shape) {
    if (row_bytes % (1024 * U) != 0 || nrows % ROWS != 0) return;  // whole steps only
    size_t smem = LDS ? (size_t)(THREADS / 64) * 2 * U * ROWS * 1024 : 0;
    auto k = LDS ? (void (*)(const char*, unsigned*, int, int))lds_kernel<THREADS, ROWS, U, NT>
                 : (void (*)(const char*, unsigned*, int, int))reg_kernel<THREADS, ROWS, U, NT>;
    if (smem > 64 * 1024) CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    auto launch = [&](char* b) { hipLaunchKernelGGL(k, dim3(blocks), dim3(THREADS), smem, 0, b, sink, nrows, row_bytes); };
    char name[160];
    snprintf(name, sizeof name, "%-14s %s %4dt %d rows U%d %s %4d wg", shape, LDS ? "lds" : "reg", THREADS, ROWS, U,
             NT ? "nt " : "def", blocks);
    out.push_back({name, (double)nrows * row_bytes, time_us(launch, bufs, 48)});
}

int main(int argc, char** argv) {
    const int which = argc > 1 ? atoi(argv[1]) : 0;  // 0: W1/W3 policy sweep, 1: per-launch floors, 2: fp8 pattern sweep
    std::vector<char*> bufs(COPIES);
    for (auto& b : bufs) {
        CK(hipMalloc(&b, BUF));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)b, BUF / 4);
    }
    unsigned* sink;
    CK(hipMalloc(&sink, 1 << 20));
    CK(hipDeviceSynchronize());
    // rounds interleave the variants (box drift hits all alike); report the median per variant
    constexpr int R = 5;
    std::vector<std::vector<Row>> rounds;
    for (int r = 0; r < R; r++) {
        std::vector<Row> v;
        if (which == 0) {
            const int n = 28672, rb = 8192;
            const char* s = "w13 f16";
            variant<512, 2, 4, true, false>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 4, false, false>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 4, true, false>(v, bufs, sink, 256, n, rb, s);
            variant<512, 2, 4, true, false>(v, bufs, sink, 1024, n, rb, s);
            variant<512, 2, 8, true, false>(v, bufs, sink, 512, n, rb, s);
            variant<512, 4, 2, true, false>(v, bufs, sink, 512, n, rb, s);
            variant<256, 2, 4, true, false>(v, bufs, sink, 1024, n, rb, s);
            variant<1024, 2, 4, true, false>(v, bufs, sink, 256, n, rb, s);
            variant<512, 1, 8, true, false>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 4, true, true>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 4, false, true>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 4, true, true>(v, bufs, sink, 256, n, rb, s);
            variant<256, 2, 4, true, true>(v, bufs, sink, 512, n, rb, s);
            variant<512, 2, 2, true, true>(v, bufs, sink, 512, n, rb, s);
            variant<256, 2, 8, true, true>(v, bufs, sink, 512, n, rb, s);
        } else if (which == 3) {
            kv_variant<1, 1024>(v, bufs, sink, 256, "kv 256-B head slices  256 wg x 1024t");
            kv_variant<1, 1024>(v, bufs, sink, 512, "kv 256-B head slices  512 wg x 1024t");
            kv_variant<1, 512>(v, bufs, sink, 512, "kv 256-B head slices  512 wg x  512t");
            kv_variant<8, 1024>(v, bufs, sink, 256, "kv 2-KiB rows          256 wg x 1024t");
            kv_variant<8, 1024>(v, bufs, sink, 512, "kv 2-KiB rows          512 wg x 1024t");
            kv_variant<8, 512>(v, bufs, sink, 512, "kv 2-KiB rows          512 wg x  512t");
            kv_variant<8, 512>(v, bufs, sink, 1024, "kv 2-KiB rows         1024 wg x  512t");
        } else if (which == 2) {
            // one-byte weights: bytes per wave step and rows per wave (W1/W3 pairs need 2 rows)
            struct Sh { const char* s; int n, rb; };
            const Sh f8[] = {{"w13 f8", 28672, 4096}, {"qkv f8", 6144, 4096}};
            for (const Sh& h : f8) {
                variant<512, 2, 4, true, false>(v, bufs, sink, 448, h.n, h.rb, h.s);
                variant<512, 2, 1, true, false>(v, bufs, sink, 448, h.n, h.rb, h.s);
                variant<512, 2, 1, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<512, 2, 1, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 2, 1, true, false>(v, bufs, sink, 1024, h.n, h.rb, h.s);
                variant<256, 2, 1, true, false>(v, bufs, sink, 1024, h.n, h.rb, h.s);
                variant<1024, 2, 1, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<512, 1, 1, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 1, 2, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 1, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 2, 2, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<384, 2, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<384, 2, 1, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
            }
            const Sh f16[] = {{"w13 f16", 28672, 8192}, {"qkv f16", 6144, 8192}, {"w2 f16", 4096, 28672}};
            for (const Sh& h : f16) {
                variant<512, 2, 4, true, false>(v, bufs, sink, 448, h.n, h.rb, h.s);
                variant<512, 2, 2, true, false>(v, bufs, sink, 448, h.n, h.rb, h.s);
                variant<512, 2, 1, true, false>(v, bufs, sink, 448, h.n, h.rb, h.s);
                variant<512, 2, 2, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<512, 1, 2, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 1, 4, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<384, 2, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<1024, 1, 4, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
            }
        } else {
            // the decode launches' matrices (Mistral-7B), f16 and fp8, at 8 and 16 waves per CU
            struct Sh { const char* s; int n, rb; };
            const Sh f16[] = {{"qkv f16", 6144, 8192}, {"wo f16", 4096, 8192}, {"w13 f16", 28672, 8192},
                              {"w2 f16", 4096, 28672}, {"cls f16", 32000, 8192}};
            for (const Sh& h : f16) {
                variant<512, 2, 4, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<512, 2, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 1, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
            }
            const Sh f8[] = {{"qkv f8", 6144, 4096}, {"wo f8", 4096, 4096}, {"w13 f8", 28672, 4096}, {"w2 f8", 4096, 14336}};
            for (const Sh& h : f8) {
                variant<512, 2, 4, true, false>(v, bufs, sink, 256, h.n, h.rb, h.s);
                variant<512, 2, 4, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 1, 2, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
                variant<512, 2, 2, true, false>(v, bufs, sink, 512, h.n, h.rb, h.s);
            }
        }
        rounds.push_back(v);
    }
    printf("%d copies rotated (beyond the Infinity Cache), median of %d rounds x 48 back-to-back launches\n", COPIES, R);
    for (size_t i = 0; i < rounds[0].size(); i++) {
        std::vector<double> t;
        for (auto& v : rounds) t.push_back(v[i].us);
        std::sort(t.begin(), t.end());
        const double us = t[R / 2];
        printf("%-50s %7.1f MB %8.2f us  %6.3f TB/s  (min %.2f max %.2f)\n", rounds[0][i].name.c_str(),
               rounds[0][i].bytes / 1e6, us, rounds[0][i].bytes / (us * 1e-6) / 1e12, t[0], t[R - 1]);
    }
    return 0;
}
