// attn_col.h — attention + Wo for short KV histories with NO hand-off between workgroups.
//
// Same math as attn_split_kernel + gemv_kernel<PRO_PLAIN, EPI_RESID> (the head loop and output
// projection of Block::_block_cpu, jubruckne/Xalm src/infer.cpp:434-452), partitioned by
// COLUMNS of Wo instead of rows:
//   x + Wo . o  =  x + sum_g Wo[:, cols(g)] . o_g,   cols(g) = the QPK*HD outputs of KV head g
// Workgroup b serves KV head g = b % n_kv_heads and a block of Wo rows.  It computes o_g itself
// (the whole history of head g, one split: every workgroup of head g reads the same K/V rows,
// served by the L2 of its XCD — b % 8 is the XCD, so with 8 KV heads all workgroups of a head
// share one XCD), then multiplies its rows' slice of Wo[:, cols(g)] by o_g and stores the
// partial part[g][row] (head 0 adds the residual x[row]).  The next launch's rmsnorm prologue
// (gemv.h PRO_RMSNORM_P) sums the n_kv_heads partials in head order into x.
// Nothing waits on another workgroup, so the kernel needs no co-residency, no counters and no
// write-through stores; the Wo rows are requested at kernel start (after q and the first round
// of K/V rows, so the attention's waits do not queue behind them) and stream from HBM while the
// attention runs.  The redundant K/V reads grow with the history, so the host takes this form
// only up to AC_KV_MAX slots (ctx->col_kv_max) and the split-KV form (attn_wo.h) beyond.
#pragma once

#include "attention.h"
#include "gemv.h"

namespace xalm {

constexpr int AC_THREADS = 1024; // 16 waves, one workgroup per CU: up to 128 VGPRs per lane
constexpr int AC_WAVES = AC_THREADS / 64;
constexpr int AC_NA = 8;         // attention waves [0, AC_NA); Wo waves [AC_NA, AC_WAVES)
constexpr int AC_ATHREADS = 64 * AC_NA;
constexpr int AC_WROWS = 16;     // Wo rows per Wo wave (at >= one row per wave instruction)
constexpr int AC_KV_MAX = 256;   // history bound: K and V rows of one head in LDS at once
constexpr int AC_PMAX = 8;       // partial vectors the PRO_RMSNORM_P prologue sums (n_kv_heads)

struct AcArgs {
    const void* wo;       // [dim][q_dim]
    size_t row_bytes;     // q_dim * sizeof(element)
    int dim;              // Wo rows
    int rows_per_wave;    // AcShape::RW (host check)
    int n_kv_heads;
    const float* x;       // residual stream [dim]
    float* part;          // [n_kv_heads][dim]
    unsigned* err;        // sticky: kv_len above AC_KV_MAX (the host never selects that)
    int debug;            // experiments (results invalid): 1 attention waves skip the attention,
                          // 2 Wo waves skip their loads
};

// LDS bytes of one workgroup
template <int HD, int QPK>
constexpr size_t attn_wo_col_smem_bytes() {
    return (size_t)2 * AC_KV_MAX * HD * 2 +
           sizeof(float) * ((size_t)AC_NA * QPK * HD + ((2 * QPK + 3) & ~3) + (size_t)QPK * HD + (size_t)QPK * AC_KV_MAX);
}

// 16-B chunks per Wo row slice of one KV head, rows per wave instruction, loads per lane
template <int DT, int HD, int QPK>
struct AcShape {
    static constexpr int E = WDec<DT>::E;
    static constexpr int NO = QPK * HD;
    static constexpr int C = NO / E;
    static constexpr bool OK = NO % E == 0 && C >= 1 && C <= 64 && (64 % C) == 0 &&
                               attn_wo_col_smem_bytes<HD, QPK>() <= 160 * 1024;
    static constexpr int RPI = OK ? 64 / C : 1;
    static constexpr int NLD = RPI >= AC_WROWS ? 1 : AC_WROWS / RPI;
    static constexpr int RW = NLD * RPI;                   // rows per Wo wave (<= 64)
    static constexpr int ROWS = RW * (AC_WAVES - AC_NA);   // rows per workgroup
};

// global -> LDS, 16 B per lane at lds_byte + 16 * lane (global_load_lds_dwordx4; the compiler
// does not model the LDS write or its vmcnt: the caller waits with s_waitcnt vmcnt(0))
__device__ __forceinline__ void ac_glds(const void* gsrc, const uint32_t lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_byte)
                 : "memory");
}

// The two roles run in separate branches (wave-uniform) with the same number of workgroup
// barriers, so the attention's registers and the Wo waves' registers (the whole row slice in
// flight) are never live together, and neither role's loads sit in front of the other's in a
// wave's in-order load counter.
template <int DT, int HD, int QPK>
__global__ __launch_bounds__(AC_THREADS) void attn_wo_col_kernel(const AttnArgs a, const AcArgs c) {
    using SH = AcShape<DT, HD, QPK>;
    constexpr int E = SH::E, NO = SH::NO, C = SH::C, NLD = SH::NLD, RPI = SH::RPI, RW = SH::RW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint16_t* kvs = (uint16_t*)smem;                          // [2][AC_KV_MAX][HD] fp16: K, V rows
    float* red = (float*)(smem + 2 * AC_KV_MAX * HD * 2);     // [AC_NA][NO]
    float* ml = red + AC_NA * NO;                             // [QPK][2]
    float* ov = ml + ((2 * QPK + 3) & ~3);                    // [NO] this head's attention output
    float* sc = ov + NO;                                      // [QPK][AC_KV_MAX]

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g = blockIdx.x % c.n_kv_heads, rb = blockIdx.x / c.n_kv_heads;
    const int kv_len = a.sp->kv_len;
    const int t1 = kv_len < AC_KV_MAX ? kv_len : AC_KV_MAX;

    if (wid < AC_NA && (c.debug & 1)) {
        for (int idx = tid; idx < NO; idx += AC_ATHREADS) ov[idx] = 0.f;
        for (int k = 0; k < 5; k++) __syncthreads();
    } else if (wid < AC_NA) {
        // ================= attention of KV head g over slots [0, t1) =================
        constexpr int LPR = HD / 8;            // lanes per K/V row (16 B = 8 fp16 each)
        constexpr int RPP = AC_ATHREADS / LPR; // rows per pass
        constexpr int RPW = 64 / LPR;          // rows per wave instruction
        const int sub = tid % LPR, rr = tid / LPR;
        if (kv_len > AC_KV_MAX && tid == 0) *c.err = 1u;
        float qv[QPK][8];
#pragma unroll
        for (int h = 0; h < QPK; h++) {
            const float4* qp = (const float4*)(a.q + (size_t)(g * QPK + h) * HD + sub * 8);
            const float4 q0 = qp[0], q1 = qp[1];
            qv[h][0] = q0.x; qv[h][1] = q0.y; qv[h][2] = q0.z; qv[h][3] = q0.w;
            qv[h][4] = q1.x; qv[h][5] = q1.y; qv[h][6] = q1.z; qv[h][7] = q1.w;
        }
        // every K and V row of the history straight into LDS: one round trip for the whole
        // attention (instruction i moves rows [i*RPW, (i+1)*RPW), clamped to the history)
        {
            const uint32_t lds0 = (uint32_t)(uintptr_t)kvs;
            const int n_i = (t1 + RPW - 1) / RPW;
            const size_t col_b = ((size_t)g * HD + (lane % LPR) * 8) * 2;
            for (int i = wid; i < 2 * n_i; i += AC_NA) {
                const int which = i >= n_i, ii = which ? i - n_i : i;
                const int t = min(ii * RPW + lane / LPR, t1 - 1);
                const char* src = (const char*)(which ? a.vc : a.kc) + (size_t)t * a.kv_dim * 2 + col_b;
                ac_glds(src, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(which * AC_KV_MAX + ii * RPW) * HD * 2));
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();  // barrier 1: K, V rows in LDS

        // ---- scores (src/infer.cpp:330-340) ----
        const float scale = 1.0f / sqrtf((float)HD);  // src/infer.cpp:338
        for (int t = rr; t < t1; t += RPP) {
            float kf[8];
            WDec<XH_F16>::dec(*(const u32x4*)(kvs + (size_t)t * HD + sub * 8), kf);
#pragma unroll
            for (int h = 0; h < QPK; h++) {
                float p = 0.f;
#pragma unroll
                for (int i = 0; i < 8; i++) p = fmaf(qv[h][i], kf[i], p);
                p = group_reduce<LPR>(p);
                if (sub == 0) sc[h * AC_KV_MAX + t] = p * scale;
            }
        }
        __syncthreads();  // barrier 2

        // ---- softmax statistics per head (max-subtract + expf, src/infer.cpp:280-297) ----
        for (int h = wid; h < QPK; h += AC_NA) {
            float m = -FLT_MAX;
            for (int i = lane; i < t1; i += 64) m = fmaxf(m, sc[h * AC_KV_MAX + i]);
            m = wave_max(m);
            float l = 0.f;
            for (int i = lane; i < t1; i += 64) {
                const float e = expf(sc[h * AC_KV_MAX + i] - m);
                sc[h * AC_KV_MAX + i] = e;
                l += e;
            }
            l = wave_sum(l);
            if (lane == 0) { ml[2 * h] = m; ml[2 * h + 1] = l; }
        }
        __syncthreads();  // barrier 3

        // ---- p . V ----
        float acc[QPK][8];
#pragma unroll
        for (int h = 0; h < QPK; h++)
#pragma unroll
            for (int i = 0; i < 8; i++) acc[h][i] = 0.f;
        const uint16_t* vs = kvs + (size_t)AC_KV_MAX * HD;
        for (int t = rr; t < t1; t += RPP) {
            float vf[8];
            WDec<XH_F16>::dec(*(const u32x4*)(vs + (size_t)t * HD + sub * 8), vf);
#pragma unroll
            for (int h = 0; h < QPK; h++) {
                const float e = sc[h * AC_KV_MAX + t];
#pragma unroll
                for (int i = 0; i < 8; i++) acc[h][i] = fmaf(e, vf[i], acc[h][i]);
            }
        }
        // over the lanes sharing `sub` (stride LPR), then over the waves in a fixed order
#pragma unroll
        for (int h = 0; h < QPK; h++)
#pragma unroll
            for (int i = 0; i < 8; i++) acc[h][i] = strided_reduce<LPR>(acc[h][i]);
        if (lane < LPR) {
#pragma unroll
            for (int h = 0; h < QPK; h++)
#pragma unroll
                for (int i = 0; i < 8; i++) red[wid * NO + h * HD + sub * 8 + i] = acc[h][i];
        }
        __syncthreads();  // barrier 4
        for (int idx = tid; idx < NO; idx += AC_ATHREADS) {
            float o = 0.f;
#pragma unroll
            for (int ww = 0; ww < AC_NA; ww++) o += red[ww * NO + idx];
            ov[idx] = o / ml[2 * (idx / HD) + 1];
        }
        __syncthreads();  // barrier 5: o_g in LDS
    } else {
        // ================= Wo rows: requested at once, multiplied after barrier 5 =================
        const int chunk = lane % C;
        const int rw0 = rb * SH::ROWS + (wid - AC_NA) * RW;  // this wave's rows [rw0, rw0 + RW)
        const int row0 = rw0 + lane / C;
        u32x4 w[NLD];
        const char* wbase = (const char*)c.wo + (size_t)g * NO * (16 / E) + (size_t)chunk * 16;
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int row = min(row0 + k * RPI, c.dim - 1);
            const __attribute__((address_space(1))) u32x4* p =
                (const __attribute__((address_space(1))) u32x4*)(wbase + (size_t)row * c.row_bytes);
            w[k] = (c.debug & 2) ? u32x4{0u, 0u, 0u, 0u} : __builtin_nontemporal_load(p);
        }
        // residual: lane L adds x[rw0 + L] to the total of row rw0 + L (head 0 only)
        static_assert(RW <= 64, "one row per lane");
        const float xl = c.x[min(rw0 + lane, c.dim - 1)];
        for (int k = 0; k < 5; k++) __syncthreads();
        float of[E];
#pragma unroll
        for (int e = 0; e < E; e += 4) {
            const float4 v = *(const float4*)(ov + chunk * E + e);
            of[e] = v.x; of[e + 1] = v.y; of[e + 2] = v.z; of[e + 3] = v.w;
        }
        // row rw0 + k*RPI + j (j < RPI) is reduced over lane group j; lane k*RPI + j collects it
        float mine = 0.f;
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            float f[E];
            WDec<DT>::dec(w[k], f);
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < E; e++) s = fmaf(f[e], of[e], s);
            s = group_reduce<C>(s);
#pragma unroll
            for (int j = 0; j < RPI; j++) {
                const float v = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s), j * C));
                mine = lane == k * RPI + j ? v : mine;
            }
        }
        // x + Wo . o with the head-0 partial carrying x (src/infer.cpp:449-452): one store
        if (lane < RW && rw0 + lane < c.dim) c.part[(size_t)g * c.dim + rw0 + lane] = g == 0 ? xl + mine : mine;
    }
}

}  // namespace xalm
