// xalm_hip.hip — device context, weight upload, per-token graph and the C ABI (include/xalm_hip.h).
//
// Replaces the device branch under Xalm's `-d` switch: Model::forward -> _forward_cpu
// (jubruckne/Xalm src/model.cpp:120-122, src/infer.cpp:604-638) and the host weight/KV
// ownership of Model::from_xalm (src/model.cpp:48-118).
//
// Per token the stream runs (all launches captured once into a hipGraph and replayed; the
// token/position scalars live in device memory, StepParams). Default, fuse level 1:
//   embed_kernel (argmax_embed_kernel in the greedy graph)          x = embed[token]
//   per layer:
//     gemv<PRO_RMSNORM, EPI_QKV>    [Wq;Wk;Wv] (one fused matrix) + rmsnorm + clip + rope +
//                                   fp16 K/V ring write + sink re-rotation
//     attn_wo_kernel (attn_wo.h)    split-KV GQA attention; the last split of a KV head merges
//                                   the partials, then Wo rows (x += .) in the same launch
//     gemv<PRO_RMSNORM, EPI_GLU>    [W1;W3] rows interleaved + rmsnorm + silu(g)*u
//     gemv<PRO_PLAIN, EPI_RESID>    W2, x += .
//   gemv<PRO_RMSNORM, EPI_STORE>    final rmsnorm + lm_head -> logits   (OUTPUT_LOGITS)
//   gemv<PRO_RMSNORM, EPI_LOGITS>   ... + per-workgroup argmax candidates (greedy graph)
// fuse_level 0 launches attention and Wo separately.  Prompts go through prefill.h unless
// XH_OPT_PREFILL is 0: passes of up to PF_TOK_MM tokens whose GEMMs run on the LDS-tiled MFMA GEMM
// of gemm16.h (f16 weights, fp8 through their exact f16 image; split-f16 activations), else
// passes of 64 tokens on the register-streaming MFMA GEMMs of prefill.h.  (Round 2's one-launch engines — persistent,
// LDS-DMA stream, qkv+attention+Wo, column-form attention — measured slower and were removed;
// DESIGN.md §4.5 / §4.9 keep the measurements.)
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <hipblaslt/hipblaslt.h>  // types only: the library is dlopen'ed (blas_api)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/xalm_synth.h"
#include "attention.h"
#include "gemv.h"
#include "dt_launch.h"
#include "gemm16.h"
#include "prefill.h"
#include "standalone.h"

using namespace xalm;

namespace {

thread_local std::string g_create_error;

size_t dtype_size(int dt) {
    switch (dt) {
        case XH_F32: return 4;
        case XH_F16: case XH_BF16: return 2;
        case XH_F8_E4M3: case XH_F8_E5M2: case XH_Q8: case XH_U8: return 1;
        default: return 0;
    }
}
bool matrix_dtype_ok(int dt) {
    return dt == XH_F32 || dt == XH_F16 || dt == XH_BF16 || dt == XH_F8_E4M3 || dt == XH_F8_E5M2 || dt == XH_Q8 ||
           gq_dt(dt);
}
// bytes of one [n]-element row: in the device layout (gguf blocks: planar, gq_pitch) and in
// the .xalm file / host upload (gguf blocks: n/32 blocks of gq_block_bytes)
size_t dev_row_bytes(int dt, size_t n) { return gq_dt(dt) ? gq_pitch(dt, n) : n * dtype_size(dt); }
size_t file_row_bytes(int dt, size_t n) { return gq_dt(dt) ? n / 32 * gq_block_bytes(dt) : n * dtype_size(dt); }
int elems_per_16b(int dt) { return 16 / (int)dtype_size(dt); }
// the kernel's decode form for a matrix: fp8 with NaN/Inf codes -> the exact bit decoder
int kdt(int dt, bool special) {
    if (!special) return dt;
    return dt == XH_F8_E4M3 ? XH_F8_E4M3_EXACT : dt == XH_F8_E5M2 ? XH_F8_E5M2_EXACT : dt;
}

constexpr int ROWS = 2;  // rows per wave (even: rope pairs, gate/up pairs)
constexpr int UNROLL = 4;

struct LayerW {
    void* wqkv = nullptr; int qkv_dt = 0; unsigned qkv_have = 0;  // bit0 q, bit1 k, bit2 v
    void* w13 = nullptr; int w13_dt = 0; unsigned w13_have = 0;   // bit0 w1, bit1 w3
    void* wo = nullptr; int wo_dt = 0;
    void* w2 = nullptr; int w2_dt = 0;
    // fp8 matrices holding NaN/Inf codes (decoded with the exact bit form, no fused kernels)
    bool qkv_x = false, w13_x = false, wo_x = false, w2_x = false;
    void* attn_norm = nullptr; int an_dt = 0;
    void* ffn_norm = nullptr; int fn_dt = 0;
};

}  // namespace

struct xh_ctx {
    xh_config c{};
    int dev = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<LayerW> L;
    void* embed = nullptr; int embed_dt = 0;
    void* final_norm = nullptr; int final_norm_dt = 0;
    void* wcls = nullptr; int wcls_dt = 0; bool wcls_x = false;
    int* scan_flag = nullptr;  // device word for the fp8 special-code scan
    int q_dim = 0, kv_dim = 0, qpk = 0;
    uint16_t* kv = nullptr;  // [n_layers][2][max_seq_len][kv_dim]
    float *x = nullptr, *q = nullptr, *attn_out = nullptr, *hb = nullptr, *logits = nullptr;
    float *part_o = nullptr, *part_ml = nullptr;
    int* attn_cnt = nullptr;        // [n_kv_heads] split arrival tickets
    float *rope_freq = nullptr, *sink_cos = nullptr, *sink_sin = nullptr;
    float* rope_cs = nullptr;  // [head_dim]: this step's rotations (rope_table, gemv.h)
    StepParams* sp = nullptr;       // device
    StepParams* sp_host = nullptr;  // pinned
    int* dec_tokens = nullptr;      // device, decode loop output
    unsigned long long* cand = nullptr;  // device [ARGMAX_CANDS]: lm_head workgroups' argmax keys
    bool cand_valid = false;        // cand describes the logits on the device
    int dec_cap = 0;
    int nsplit = 1, t_max = 16;
    // fused attention + Wo launch (attn_wo.h): per-layer hand-off words [n_layers][4]
    bool fuse_attn_wo = true;
    unsigned* aw_sync = nullptr;
    // batched prefill (prefill.h), buffers allocated on first use
    bool prefill_batched = true;
    // XH_OPT_PREFILL: 1 = the LDS-tiled f16 MFMA GEMM (gemm16.h) for f16 / e4m3 / e5m2 weights (fp8
    // as an exact f16 image), f32 MFMA otherwise; 2 = split-f16 register-streaming MFMA wherever the
    // weights convert exactly; 3 = f32 MFMA only; 4 = as 1 with hipBLASLt in place of gemm16.h
    int prefill_gemm = 1;
    int pf_pass = 0;                             // tokens per pass of the current prefill
    int pf_cap = 0;                              // tokens the pass buffers hold (pf_alloc)
    bool pf_scaled = false;                      // the last pf_gemm's partials carry 1 / s_t (pf_xs)
    int mm_ok = 0;                               // 0 unchecked, 1 every pass GEMM fits gemm16.h, -1 not
    // hipBLASLt (XH_OPT_PREFILL 4, created on the first prompt that uses it): handle, workspace, plans per shape
    hipblasLtHandle_t blas = nullptr;
    void* blas_ws = nullptr;
    struct BlasPlan {
        hipblasLtMatmulDesc_t md = nullptr;
        hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
        std::vector<hipblasLtMatmulAlgo_t> cands;  // the heuristic's candidates (empty: none; [0] is used)
        bool ready = false;
    };
    int blas_ok = 0;  // 0 unprobed, 1 every GEMM shape of the model has an f16 plan, -1 not
    std::map<std::vector<int>, BlasPlan> blas_plans;
    uint16_t* pf_wdq = nullptr;                  // f16 image of one fp8 matrix for the f16 GEMMs (pf_prepare)
    size_t pf_wdq_elems = 0;
    bool pf_split_ready = false;                 // pf_norm left the next GEMM's split input
    bool pf_resid_norm = true;                   // residual + rmsnorm split in one launch (XH_OPT_PREFILL_GLU_SPLIT 0: off)
    bool pf_glu_split = true;                    // XH_OPT_PREFILL_GLU_SPLIT: fused GLU -> split input
    int pf_fa_split = 1;                         // XH_OPT_PREFILL_ATTN_SPLIT: history splits for short passes
    int pf_attn_mode = 1;                        // XH_OPT_PREFILL_ATTN: 1 shared-tile MFMA (v1 for head_dim != 128),
                                                 // 2 per-wave MFMA tiles, 0 per-token split kernel
    // T = pf_cap tokens (the pass length in use; pf_alloc)
    uint16_t* pf_xh = nullptr;                   // [2T][max K] f16 halves of a GEMM input (pf_alloc)
    uint16_t* pf_xl = nullptr;                   // [PF_TOK][max K] the split kernel's lo fragments
    float* pf_xs = nullptr;                      // [T] 1 / row scale
    int* pf_tok = nullptr;                       // [T]
    float *pf_x = nullptr, *pf_xn = nullptr;     // [T][dim]
    float *pf_q = nullptr, *pf_att = nullptr;    // [T][q_dim]
    float* pf_h = nullptr;                       // [T][hidden]
    float* pf_part = nullptr;                    // split-K partials [ks][n][rows] (pf_part_floats)
    StepParams* pf_sp = nullptr;                 // [T] per-token attention scalars
    // the per-token split attention (XH_OPT_PREFILL_ATTN 0 only, allocated on its first use):
    float *pf_po = nullptr, *pf_pml = nullptr;   // [T][nsplit][q_dim], [T][nsplit][n_heads][2]
    int* pf_cnt = nullptr;                       // [T][n_kv_heads] split tickets
    int pf_po_cap = 0;                           // tokens those hold
    // xh_perplexity: per-token logits of a pass, targets, probabilities (allocated on first use)
    float* pf_logits = nullptr;                  // [T][vocab]
    int* pf_tgt = nullptr;                       // [T]
    int* ppl_tgt = nullptr;                      // [ppl_cap] targets (per-token path)
    float* ppl_prob = nullptr;                   // [ppl_cap]
    int ppl_cap = 0;
    int t_max_aw = 16;
    bool use_graphs = true;
    hipGraphExec_t g_logits = nullptr, g_hydrate = nullptr, g_decode = nullptr;
    int max_gemv_waves = 4096;  // 16 waves per CU
    // the qkv launch: its whole matrix is one round at 16 waves per CU (every wave one group,
    // requested at once); at 8 waves per CU each wave streams two groups back to back
    // (tools/gemv_bench GB_T1K: 10.95 -> 10.12 us f16, 7.93 -> 7.34 us fp8)
    int qkv_waves = 2048;
    int n_cu = 0;
    // debug timelines (xh_debug_trace): device-clock stamps per workgroup
    unsigned long long* aw_trace = nullptr;
    size_t aw_trace_len = 0;
    bool aw_trace_on = false;   // attn_wo launches ([workgroup][8])
    bool w13_trace_on = false;  // plain W1/W3 launches ([workgroup][4]: tools/balance_trace.py)
    // the last layer's launches and the lm_head each write their own region (LT_*): the step's
    // timeline, kernel boundaries included (tools/layer_trace.py)
    bool layer_trace_on = false;
    uint16_t* kcache(int l) { return kv + (size_t)l * 2 * c.max_seq_len * kv_dim; }
    uint16_t* vcache(int l) { return kcache(l) + (size_t)c.max_seq_len * kv_dim; }
};

namespace {

int set_err(xh_ctx* ctx, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf; else g_create_error = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                     \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return set_err((ctx), XH_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                           __FILE__, __LINE__);                                                \
    } while (0)

// Host <-> device copies and fills go on ctx->stream and wait for it.  ctx->stream is
// non-blocking, so null-stream work (hipMemcpy, hipMemset, hipMemcpy2D) is not ordered with
// its kernels: a fill can land after a kernel wrote the buffer, and a pageable upload can
// return before its DMA does.
hipError_t copy_sync(xh_ctx* ctx, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, ctx->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
}
hipError_t copy2d_sync(xh_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                       size_t height) {
    const hipError_t e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyHostToDevice, ctx->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
}
hipError_t fill_sync(xh_ctx* ctx, void* dst, int value, size_t bytes) {
    const hipError_t e = hipMemsetAsync(dst, value, bytes, ctx->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(ctx->stream);
}

// The dynamic-LDS limit of a kernel above 64 KiB (up to the CU's 160 KiB), set once per (kernel,
// device): the attribute belongs to the device current at the call.
void ensure_lds(const void* fn, const int bytes = 160 * 1024) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> g(mu);
    if (done.insert({fn, dev}).second) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// ---------------------------------------------------------------------------------------
// gemv launch dispatch
// ---------------------------------------------------------------------------------------
// Shapes, chosen with tools/gemv_bench.hip and tools/chain_bench.hip on MI355X
// (profiles/r01_gemv_bench.txt, profiles/r01_chain_bench.txt): 512-thread blocks (8 waves share
// one x image), 2 rows x 4 chunks in flight per wave, non-temporal weight loads, 16 waves per
// CU.  PF shapes hold x in registers (XN float4 per thread) and request the first weight chunks
// inside the prologue (-5.7 % per decode layer); the plain shape covers every other n.
using ShapeShort = GemvShape<512, ROWS, UNROLL, true, 4, false>;
using ShapeLong = GemvShape<512, ROWS, UNROLL, true, 4, false>;
using ShapePF2 = GemvShape<512, ROWS, UNROLL, true, 4, true, 2>;  // n <= 4096
using ShapePF8 = GemvShape<512, ROWS, UNROLL, true, 4, true, 8>;  // n <= 16384 (W2 / Wo inputs)

template <int DT, int PRO, int EPI, class S>
void launch_gemv_s(const GemvArgs& a, hipStream_t s, int max_waves) {
    const size_t smem = gemv_smem_bytes<DT, S>(a.n);
    const int blocks = gemv_blocks<S>(a.rows, max_waves / S::WAVES);
    auto k = gemv_kernel<DT, PRO, EPI, S>;
    if (smem > 64 * 1024) ensure_lds((const void*)k);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(S::THREADS), smem, s, a);
}

// pipelined PF shape (gemv_rows_pipe: the next row step requested before the current one is
// multiplied, across row groups too) for the qkv and W1/W3 launches: fp8 Mistral-7B decode
// 568 -> 584 tok/s (their 4 KiB rows are one step per group, so a wave drained to zero at
// every group), f16 unchanged (383 / 383); W2, Wo and lm_head unchanged either way
using ShapePF2P = GemvShape<512, ROWS, UNROLL, true, 4, true, 2, 2>;  // n <= 4096
// qkv with 2-byte weights (QKV_T384): 384-thread workgroups, two per CU, every wave ONE row group
// at 3072 waves (tools/gemv_bench GB_BAL: 10.29 -> 9.95 us f16; fp8 rows are one step: no gain)
using ShapeQ384 = GemvShape<384, ROWS, UNROLL, true, 3, true, 3, 2>;  // n <= 4608
#ifndef QKV_T384
#define QKV_T384 1
#endif
// W2-long rows of one-byte weights (W2_T1024): one 1024-thread workgroup per CU, one row per
// wave, hb in 4 float4 per thread (tools/gemv_bench GB_W2, fp8 Mistral W2: 12.58 -> 11.99 us;
// f16 no gain)
using ShapeW2K = GemvShape<1024, 1, UNROLL, true, 4, true, 4, 1>;  // n <= 16384
#ifndef W2_T1024
#define W2_T1024 1
#endif
#ifndef GEMV_BAL_GQ_GLU
#define GEMV_BAL_GQ_GLU 1
#endif
#ifndef GEMV_BAL_FP8_QKV
#define GEMV_BAL_FP8_QKV 1
#endif


template <int DT, int PRO, int EPI>
void launch_gemv_t(const GemvArgs& a, hipStream_t s, int max_waves) {
    constexpr int E = WDec<DT>::E;
    // gguf blocks take the staged shapes below (4 rows per wave measured slower: Q8_0 442 ->
    // 303 tok/s, Q4_0 560 -> 506)
    // PF needs whole first chunks (n >= 64 E U) and x in XN float4 per thread
    const bool pf = !gq_dt(DT) && a.n % 4 == 0 && a.n >= 64 * E * UNROLL;
    if constexpr ((EPI == EPI_QKV || EPI == EPI_GLU) && !gq_dt(DT)) {
        if constexpr (EPI == EPI_QKV && E <= 8 && QKV_T384) {
            if (pf && a.n / 4 <= 3 * 384 && a.n % (64 * E * UNROLL) == 0)
                return launch_gemv_s<DT, PRO, EPI, ShapeQ384>(a, s, 3 * (max_waves / 2));
        }
        if constexpr (EPI == EPI_QKV && E >= 16 && GEMV_BAL_FP8_QKV) {
            // one-byte qkv rows: 3072 one-step groups, 512 workgroups of 6 busy waves (fp8 qkv
            // 7.3 -> 7.1 us, decode +0.5 %, profiles/r06_decode_ab.txt ab9)
            using ShapePF2PB = GemvShape<512, ROWS, UNROLL, true, 4, true, 2, 2, true>;
            if (pf && a.n / 4 <= 2 * 512 && a.n % (64 * E * UNROLL) == 0)
                return launch_gemv_s<DT, PRO, EPI, ShapePF2PB>(a, s, max_waves);
        }
        if (pf && a.n / 4 <= 2 * 512 && a.n % (64 * E * UNROLL) == 0)
            return launch_gemv_s<DT, PRO, EPI, ShapePF2P>(a, s, max_waves);
    }
    if constexpr (gq_dt(DT)) {
        // gguf blocks: the pipelined PF shapes with the block scales loaded beside the codes.
        // Q4_0 rows of a 4096-wide input are 2 chunks, so 2 chunks per step; W2-long inputs
        // (14336: 14 / 7 chunks per row) step by 2 (Q8_0) / 1 (Q4_0) chunks
        constexpr int UG = DT == XH_Q4_0 ? 2 : UNROLL;
        // W1/W3 (GEMV_BAL_GQ_GLU): balanced grid, Q4_0 15.0 -> 14.0 us (profiles/r06_decode_ab.txt ab8)
        using ShapeGQ = GemvShape<512, ROWS, UG, true, 4, true, 2, 2, EPI == EPI_GLU && GEMV_BAL_GQ_GLU>;
        if (a.n % 4 == 0 && a.n / 4 <= 2 * 512 && a.n % (64 * E * UG) == 0)
            return launch_gemv_s<DT, PRO, EPI, ShapeGQ>(a, s, max_waves);
        if constexpr (PRO == PRO_PLAIN) {
            constexpr int UL = DT == XH_Q4_0 ? 1 : 2;
            using ShapeGQL = GemvShape<512, ROWS, UL, true, 4, true, 8, 2>;
            if (a.n % 4 == 0 && a.n / 4 <= 8 * 512 && a.n % (64 * E * UL) == 0)
                return launch_gemv_s<DT, PRO, EPI, ShapeGQL>(a, s, max_waves);
        }
    }
    if (pf && a.n / 4 <= 2 * 512) launch_gemv_s<DT, PRO, EPI, ShapePF2>(a, s, max_waves);
    else if constexpr (PRO == PRO_PLAIN && EPI == EPI_RESID && E >= 16 && W2_T1024) {
        if (pf && a.n / 4 <= 4 * 1024) launch_gemv_s<DT, PRO, EPI, ShapeW2K>(a, s, max_waves);
        else launch_gemv_s<DT, PRO, EPI, ShapeLong>(a, s, max_waves);
    } else if constexpr (PRO == PRO_PLAIN) {
        if (pf && a.n / 4 <= 8 * 512) launch_gemv_s<DT, PRO, EPI, ShapePF8>(a, s, max_waves);
        else launch_gemv_s<DT, PRO, EPI, ShapeLong>(a, s, max_waves);
    } else if (gemv_smem_bytes<DT, ShapeShort>(a.n) <= 40 * 1024) {
        launch_gemv_s<DT, PRO, EPI, ShapeShort>(a, s, max_waves);
    } else {
        launch_gemv_s<DT, PRO, EPI, ShapeLong>(a, s, max_waves);
    }
}

template <int PRO, int EPI>
bool launch_gemv(int dt, const GemvArgs& a, hipStream_t s, int max_blocks) {
    switch (dt) {
        case XH_F32: launch_gemv_t<XH_F32, PRO, EPI>(a, s, max_blocks); return true;
        case XH_F16: launch_gemv_t<XH_F16, PRO, EPI>(a, s, max_blocks); return true;
        case XH_BF16: launch_gemv_t<XH_BF16, PRO, EPI>(a, s, max_blocks); return true;
        case XH_F8_E4M3: launch_gemv_t<XH_F8_E4M3, PRO, EPI>(a, s, max_blocks); return true;
        case XH_F8_E5M2: launch_gemv_t<XH_F8_E5M2, PRO, EPI>(a, s, max_blocks); return true;
        case XH_Q8: launch_gemv_t<XH_Q8, PRO, EPI>(a, s, max_blocks); return true;
        case XH_F8_E4M3_EXACT: launch_gemv_t<XH_F8_E4M3_EXACT, PRO, EPI>(a, s, max_blocks); return true;
        case XH_F8_E5M2_EXACT: launch_gemv_t<XH_F8_E5M2_EXACT, PRO, EPI>(a, s, max_blocks); return true;
        case XH_Q8_0: launch_gemv_t<XH_Q8_0, PRO, EPI>(a, s, max_blocks); return true;
        case XH_Q4_0: launch_gemv_t<XH_Q4_0, PRO, EPI>(a, s, max_blocks); return true;
        default: return false;
    }
}

// ---------------------------------------------------------------------------------------
// attention launch dispatch
// ---------------------------------------------------------------------------------------
template <int HD, int QPK>
void launch_attn_t(const AttnArgs& a, int n_kv_heads, int t_max, hipStream_t s) {
    const size_t smem = attn_smem_bytes(HD, QPK, t_max, a.nsplit);
    auto k = attn_split_kernel<HD, QPK>;
    if (smem > 64 * 1024) ensure_lds((const void*)k);
    hipLaunchKernelGGL(k, dim3(n_kv_heads, a.nsplit), dim3(ATTN_THREADS), smem, s, a);
}

template <int HD>
bool launch_attn_hd(const AttnArgs& a, int qpk, int n_kv_heads, int t_max, hipStream_t s) {
    switch (qpk) {
        case 1: launch_attn_t<HD, 1>(a, n_kv_heads, t_max, s); return true;
        case 2: launch_attn_t<HD, 2>(a, n_kv_heads, t_max, s); return true;
        case 4: launch_attn_t<HD, 4>(a, n_kv_heads, t_max, s); return true;
        case 8: launch_attn_t<HD, 8>(a, n_kv_heads, t_max, s); return true;
        default: return false;
    }
}

bool launch_attn(const AttnArgs& a, int hd, int qpk, int n_kv_heads, int t_max, hipStream_t s) {
    bool ok = false;
    switch (hd) {
        case 16: ok = launch_attn_hd<16>(a, qpk, n_kv_heads, t_max, s); break;
        case 32: ok = launch_attn_hd<32>(a, qpk, n_kv_heads, t_max, s); break;
        case 64: ok = launch_attn_hd<64>(a, qpk, n_kv_heads, t_max, s); break;
        case 128: ok = launch_attn_hd<128>(a, qpk, n_kv_heads, t_max, s); break;
        case 256: ok = launch_attn_hd<256>(a, qpk, n_kv_heads, t_max, s); break;
        default: return false;
    }
    return ok;
}

int attn_nsplit(int n_kv_heads, int max_seq_len) {
    // one split workgroup per CU at the longest context (tools/attn_bench.hip, 32k: 32 splits
    // per KV head 34.9 us vs 64 splits 39.0 us)
#ifndef ATTN_SPLIT_WGS
#define ATTN_SPLIT_WGS 256
#endif
    int ns = ATTN_SPLIT_WGS / n_kv_heads;
    if (ns > 128) ns = 128;  // the merge holds <= 2 partials per lane
#ifndef ATTN_CAP_T
#define ATTN_CAP_T ATTN_MIN_T
#endif
    const int cap = (max_seq_len + ATTN_CAP_T - 1) / ATTN_CAP_T;
    if (ns > cap) ns = cap;
    return ns < 1 ? 1 : ns;
}

// ---------------------------------------------------------------------------------------
// the per-token step, enqueued on a stream (eager or under graph capture)
// ---------------------------------------------------------------------------------------
// debug layer timeline: regions of aw_trace (words) per launch of the traced (last) layer
constexpr size_t LT_QKV = 0, LT_AW = 8192, LT_W13 = 16384, LT_W2 = 20480, LT_CLS = 24576, LT_WORDS = 28672;
bool layer_traced(const xh_ctx* ctx, int l) { return ctx->layer_trace_on && l == ctx->c.n_layers - 1; }

GemvArgs qkv_args(xh_ctx* ctx, int l) {
    const LayerW& w = ctx->L[l];
    GemvArgs a{};
    a.w = w.wqkv; a.row_bytes = dev_row_bytes(w.qkv_dt, ctx->c.dim);
    a.n = ctx->c.dim; a.rows = ctx->q_dim + 2 * ctx->kv_dim; a.x = ctx->x;
    a.norm_w = w.attn_norm; a.norm_dtype = w.an_dt; a.eps = ctx->c.norm_eps;
    a.q = ctx->q; a.kcache = ctx->kcache(l); a.vcache = ctx->vcache(l);
    a.q_dim = ctx->q_dim; a.kv_dim = ctx->kv_dim; a.head_dim = ctx->c.head_dim;
    a.rope_freq = ctx->rope_freq; a.rope_cs = ctx->rope_cs; a.sink_cos = ctx->sink_cos; a.sink_sin = ctx->sink_sin;
    a.qkv_clip = ctx->c.qkv_clip; a.sp = ctx->sp;
    if (layer_traced(ctx, l)) a.trace = ctx->aw_trace + LT_QKV;
    return a;
}
GemvArgs wo_args(xh_ctx* ctx, int l) {
    const LayerW& w = ctx->L[l];
    GemvArgs a{};
    a.w = w.wo; a.row_bytes = dev_row_bytes(w.wo_dt, ctx->q_dim);
    a.n = ctx->q_dim; a.rows = ctx->c.dim; a.x = ctx->attn_out; a.out = ctx->x; a.sp = ctx->sp;
    return a;
}
GemvArgs w13_args(xh_ctx* ctx, int l) {
    const LayerW& w = ctx->L[l];
    GemvArgs a{};
    a.w = w.w13; a.row_bytes = dev_row_bytes(w.w13_dt, ctx->c.dim);
    a.n = ctx->c.dim; a.rows = 2 * ctx->c.hidden_dim; a.x = ctx->x;
    a.norm_w = w.ffn_norm; a.norm_dtype = w.fn_dt; a.eps = ctx->c.norm_eps;
    a.out = ctx->hb; a.act = ctx->c.act; a.sp = ctx->sp;
    if (ctx->w13_trace_on) a.trace = ctx->aw_trace;
    if (layer_traced(ctx, l)) a.trace = ctx->aw_trace + LT_W13;
    return a;
}
GemvArgs w2_args(xh_ctx* ctx, int l) {
    const LayerW& w = ctx->L[l];
    GemvArgs a{};
    a.w = w.w2; a.row_bytes = dev_row_bytes(w.w2_dt, ctx->c.hidden_dim);
    a.n = ctx->c.hidden_dim; a.rows = ctx->c.dim; a.x = ctx->hb; a.out = ctx->x; a.sp = ctx->sp;
    if (layer_traced(ctx, l)) a.trace = ctx->aw_trace + LT_W2;
    return a;
}
GemvArgs cls_args(xh_ctx* ctx) {
    GemvArgs a{};
    a.w = ctx->wcls; a.row_bytes = dev_row_bytes(ctx->wcls_dt, ctx->c.dim);
    a.n = ctx->c.dim; a.rows = ctx->c.vocab_size; a.x = ctx->x;
    a.norm_w = ctx->final_norm; a.norm_dtype = ctx->final_norm_dt; a.eps = ctx->c.norm_eps;
    a.out = ctx->logits; a.sp = ctx->sp; a.cand = ctx->cand;
    if (ctx->layer_trace_on) a.trace = ctx->aw_trace + LT_CLS;
    return a;
}
AttnArgs attn_args(xh_ctx* ctx, int l) {
    AttnArgs a{};
    a.q = ctx->q; a.kc = ctx->kcache(l); a.vc = ctx->vcache(l); a.kv_dim = ctx->kv_dim;
    a.n_heads = ctx->c.n_heads; a.nsplit = ctx->nsplit; a.out = ctx->attn_out;
    a.part_o = ctx->part_o; a.part_ml = ctx->part_ml; a.counters = ctx->attn_cnt; a.sp = ctx->sp;
    return a;
}

__global__ void argmax_advance_kernel(const float* logits, int vocab, StepParams* sp, int* tokens, int cap) {
    // Sampler::sample_argmax (src/sampler.cpp:19-30): max starts at FLT_MIN, strict '>',
    // so the first index of the maximum wins and all-tiny logits give token 0.
    __shared__ float bv[1024];
    __shared__ int bi[1024];
    const int tid = threadIdx.x;
    float best = FLT_MIN;
    int idx = 0;
    for (int i = tid; i < vocab; i += blockDim.x)
        if (logits[i] > best) { best = logits[i]; idx = i; }
    bv[tid] = best;
    bi[tid] = idx;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (tid < o) {
            const float v2 = bv[tid + o];
            const int i2 = bi[tid + o];
            if (v2 > bv[tid] || (v2 == bv[tid] && i2 < bi[tid])) { bv[tid] = v2; bi[tid] = i2; }
        }
        __syncthreads();
    }
    if (tid == 0) {
        const int tok = bi[0];
        if (sp->step < cap) tokens[sp->step] = tok;
        sp->step += 1;
        sp->token = tok;
        step_positions(sp, sp->pos_next);
        sp->pos_next += 1;
    }
}

// wave cap of layer l's qkv launch: ctx->qkv_waves for the pipelined shape; gguf blocks take the
// unpipelined staged shape, every wave one group at 16 waves per CU
int qkv_launch_waves(const xh_ctx* ctx, int l) {
    return gq_dt(ctx->L[l].qkv_dt) ? ctx->max_gemv_waves : ctx->qkv_waves;
}

bool use_attn_wo(const xh_ctx* ctx, int l) {
    const int dt = ctx->L[l].wo_dt;
    if (ctx->L[l].wo_x) return false;  // exact fp8 decode: the separate launches
    return ctx->fuse_attn_wo && aw_instantiated(ctx->c.head_dim, ctx->qpk) &&
           (dt == XH_F32 || dt == XH_F16 || dt == XH_BF16 || dt == XH_F8_E4M3 || dt == XH_F8_E5M2 || dt == XH_Q8);
}

int launch_attn_wo(xh_ctx* ctx, int l, hipStream_t s) {
    const AttnArgs aa = attn_args(ctx, l);
    const GemvArgs ga = wo_args(ctx, l);
    unsigned* sync = ctx->aw_sync + (size_t)AW_SYNC_WORDS * l;
    const int hd = ctx->c.head_dim, qpk = ctx->qpk, nkv = ctx->c.n_kv_heads, tm = ctx->t_max_aw;
    const int mw = ctx->max_gemv_waves;
    unsigned long long* tr = ctx->aw_trace_on ? ctx->aw_trace : layer_traced(ctx, l) ? ctx->aw_trace + LT_AW : nullptr;
    switch (ctx->L[l].wo_dt) {
        case XH_F32: return aw_launch_dt1(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        case XH_F16: return aw_launch_dt2(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        case XH_BF16: return aw_launch_dt3(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        case XH_F8_E4M3: return aw_launch_dt6(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        case XH_F8_E5M2: return aw_launch_dt7(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        case XH_Q8: return aw_launch_dt9(aa, ga, hd, qpk, nkv, tm, sync, mw, s, tr);
        default: return XH_E_INVALID;
    }
}

// a fused hand-off that timed out leaves its sticky flag: report it (after the stream sync)
int check_aw(xh_ctx* ctx) {
    if (!ctx->fuse_attn_wo) return 0;
    std::vector<unsigned> h((size_t)ctx->c.n_layers * AW_SYNC_WORDS);
    HIP_TRY(ctx, copy_sync(ctx, h.data(), ctx->aw_sync, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    for (int l = 0; l < ctx->c.n_layers; l++)
        if (h[(size_t)AW_SYNC_WORDS * l + 2]) {
            // reported once: the sticky words are cleared so the context can be reset and reused
            HIP_TRY(ctx, fill_sync(ctx, ctx->aw_sync, 0, h.size() * sizeof(unsigned)));
            return set_err(ctx, XH_E_HIP, "layer %d: attention -> Wo hand-off timed out", l);
        }
    return 0;
}

// greedy: the token is the argmax of the previous step's logits (argmax_embed_kernel)
int enqueue_step(xh_ctx* ctx, hipStream_t s, bool with_logits, bool greedy = false) {
    const xh_config& c = ctx->c;
    const int mb = ctx->max_gemv_waves;
    if (greedy)
        hipLaunchKernelGGL(argmax_embed_kernel, dim3(1), dim3(ARGMAX_CANDS), 0, s, (const unsigned long long*)ctx->cand,
                           ctx->sp, ctx->dec_tokens, ctx->dec_cap, (const void*)ctx->embed, ctx->embed_dt, c.dim,
                           ctx->x, (const float*)ctx->rope_freq, ctx->rope_cs, c.head_dim / 2);
    else
        hipLaunchKernelGGL(embed_kernel, dim3((c.dim + 255) / 256), dim3(256), 0, s, (const void*)ctx->embed,
                           ctx->embed_dt, c.dim, ctx->x, (const StepParams*)ctx->sp, (const float*)ctx->rope_freq,
                           ctx->rope_cs, c.head_dim / 2);
    for (int l = 0; l < c.n_layers; l++) {
        const LayerW& w = ctx->L[l];
        if (!launch_gemv<PRO_RMSNORM, EPI_QKV>(kdt(w.qkv_dt, w.qkv_x), qkv_args(ctx, l), s, qkv_launch_waves(ctx, l)))
            return set_err(ctx, XH_E_INVALID, "layer %d: unsupported qkv dtype %d", l, w.qkv_dt);
        GemvArgs a13 = w13_args(ctx, l);
        if (use_attn_wo(ctx, l)) {
            const int rc = launch_attn_wo(ctx, l, s);
            if (rc) return set_err(ctx, rc, "layer %d: fused attention + Wo launch failed", l);
            // W1/W3 right behind it zeroes its hand-off words for the next step
            a13.aw_reset = ctx->aw_sync + (size_t)AW_SYNC_WORDS * l;
        } else {
            if (!launch_attn(attn_args(ctx, l), c.head_dim, ctx->qpk, c.n_kv_heads, ctx->t_max, s))
                return set_err(ctx, XH_E_INVALID, "unsupported head_dim %d / q-per-kv %d", c.head_dim, ctx->qpk);
            if (!launch_gemv<PRO_PLAIN, EPI_RESID>(kdt(w.wo_dt, w.wo_x), wo_args(ctx, l), s, mb))
                return set_err(ctx, XH_E_INVALID, "layer %d: unsupported wo dtype", l);
        }
        if (!launch_gemv<PRO_RMSNORM, EPI_GLU>(kdt(w.w13_dt, w.w13_x), a13, s, mb))
            return set_err(ctx, XH_E_INVALID, "layer %d: unsupported w1/w3 dtype", l);
        if (!launch_gemv<PRO_PLAIN, EPI_RESID>(kdt(w.w2_dt, w.w2_x), w2_args(ctx, l), s, mb))
            return set_err(ctx, XH_E_INVALID, "layer %d: unsupported w2 dtype", l);
    }
    if (with_logits) {
        if (!launch_gemv<PRO_RMSNORM, EPI_LOGITS>(kdt(ctx->wcls_dt, ctx->wcls_x), cls_args(ctx), s, mb))
            return set_err(ctx, XH_E_INVALID, "unsupported wcls dtype");
    }
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int check_ready(xh_ctx* ctx) {
    if (!ctx->embed) return set_err(ctx, XH_E_STATE, "embed.weight not uploaded");
    if (!ctx->final_norm) return set_err(ctx, XH_E_STATE, "output.norm.weight not uploaded");
    if (!ctx->wcls) {
        if (ctx->c.tie_word_embeddings) { ctx->wcls = ctx->embed; ctx->wcls_dt = ctx->embed_dt; }
        else return set_err(ctx, XH_E_STATE, "output.weight not uploaded");
    }
    for (int l = 0; l < ctx->c.n_layers; l++) {
        const LayerW& w = ctx->L[l];
        if (w.qkv_have != 7 || w.w13_have != 3 || !w.wo || !w.w2 || !w.attn_norm || !w.ffn_norm)
            return set_err(ctx, XH_E_STATE, "layer %d: weights incomplete", l);
    }
    return 0;
}

void drop_graphs(xh_ctx* ctx) {
    if (ctx->g_logits) hipGraphExecDestroy(ctx->g_logits);
    if (ctx->g_hydrate) hipGraphExecDestroy(ctx->g_hydrate);
    if (ctx->g_decode) hipGraphExecDestroy(ctx->g_decode);
    ctx->g_logits = ctx->g_hydrate = ctx->g_decode = nullptr;
}

int capture(xh_ctx* ctx, int kind, hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    HIP_TRY(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_step(ctx, ctx->stream, kind != 1, kind == 2);
    hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    if (rc) { if (g) hipGraphDestroy(g); return rc; }
    if (e != hipSuccess) return set_err(ctx, XH_E_HIP, "graph capture failed: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    hipGraphDestroy(g);
    if (e != hipSuccess) return set_err(ctx, XH_E_HIP, "graph instantiate failed: %s", hipGetErrorString(e));
    return 0;
}

// an eager step that failed part-way: the attention + Wo hand-off words may hold arrivals that
// the layer's W1/W3 launch never zeroed
int eager_step(xh_ctx* ctx, bool with_logits, bool greedy) {
    const int rc = enqueue_step(ctx, ctx->stream, with_logits, greedy);
    if (rc) hipMemsetAsync(ctx->aw_sync, 0, (size_t)ctx->c.n_layers * AW_SYNC_WORDS * 4, ctx->stream);
    return rc;
}

// the step at host_step_params' position
int run_step(xh_ctx* ctx, bool with_logits) {
    if (with_logits) ctx->cand_valid = true;  // the lm_head launch writes candidates
    if (!ctx->use_graphs) return eager_step(ctx, with_logits, false);
    hipGraphExec_t* ge = with_logits ? &ctx->g_logits : &ctx->g_hydrate;
    if (!*ge) {
        int rc = capture(ctx, with_logits ? 0 : 1, ge);
        if (rc) return rc;
    }
    HIP_TRY(ctx, hipGraphLaunch(*ge, ctx->stream));
    return 0;
}

int host_step_params(xh_ctx* ctx, int token, int pos) {
    StepParams* h = ctx->sp_host;
    const int msl = ctx->c.max_seq_len;
    h->token = token;
    h->pos = pos;
    h->kv_sink = pos >= msl ? 2 : 0;
    h->kv_pos = h->kv_sink + (pos - h->kv_sink) % (msl - h->kv_sink);
    h->kv_len = pos >= msl ? msl : pos + 1;
    h->step = 0;
    h->pos_next = pos + 1;
    h->max_seq_len = msl;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->sp, h, sizeof(StepParams), hipMemcpyHostToDevice, ctx->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------
// batched prefill (prefill.h)
// ---------------------------------------------------------------------------------------
template <class T>
int dmalloc(xh_ctx* ctx, T** p, size_t n);
constexpr int PF_WAVE_TARGET = 1024;  // 1 wave per SIMD (RT=2: 2048 -16 %, 512 -38 %; fewer, longer K slices)
constexpr int PF_RT = 2;                // 32-row tiles per GEMM wave (1: -11 %, 4: -9 %)
constexpr int PF_RT16 = 4;              // 32-row tiles per split-f16 GEMM wave
constexpr size_t PF_PART_ROWS = 32 * PF_RT16 * PF_WAVE_TARGET;  // >= ks * rows (ks * ceil(rows/(32 RT)) <= target)

constexpr int PF_CLS_CHUNK = (int)(PF_PART_ROWS / 4);  // lm_head rows per GEMM (ks <= 4 fits the partials)
constexpr size_t PF_BLAS_WS = 256ull << 20;            // hipBLASLt workspace

// partials buffer: the register-streaming MFMA kernels' K slices of 64 tokens, or up to 2 T
// token rows of partials over the widest matrix (gemm16.h K slices: ks * n <= 2 T; hipBLASLt: the
// hi and lo halves)
size_t pf_part_floats(const xh_ctx* ctx, const int T) {
    const xh_config& c = ctx->c;
    const int rows = std::max({ctx->q_dim + 2 * ctx->kv_dim, 2 * c.hidden_dim, c.dim, std::min(c.vocab_size, PF_CLS_CHUNK)});
    return std::max(PF_PART_ROWS * PF_TOK, (size_t)2 * T * rows);
}

void pf_free(xh_ctx* ctx) {
    for (void* p : {(void*)ctx->pf_tok, (void*)ctx->pf_x, (void*)ctx->pf_xn, (void*)ctx->pf_q, (void*)ctx->pf_att,
                    (void*)ctx->pf_h, (void*)ctx->pf_part, (void*)ctx->pf_sp, (void*)ctx->pf_xh, (void*)ctx->pf_xl,
                    (void*)ctx->pf_xs, (void*)ctx->pf_logits, (void*)ctx->pf_tgt, (void*)ctx->pf_po,
                    (void*)ctx->pf_pml, (void*)ctx->pf_cnt})
        hipFree(p);
    ctx->pf_tok = nullptr; ctx->pf_x = ctx->pf_xn = ctx->pf_q = ctx->pf_att = ctx->pf_h = ctx->pf_part = nullptr;
    ctx->pf_sp = nullptr; ctx->pf_xh = ctx->pf_xl = nullptr; ctx->pf_xs = nullptr; ctx->pf_logits = nullptr;
    ctx->pf_tgt = nullptr; ctx->pf_po = ctx->pf_pml = nullptr; ctx->pf_cnt = nullptr;
    ctx->pf_cap = ctx->pf_po_cap = 0;
}

// pass buffers for T tokens (kept while later passes fit; a longer pass length reallocates)
int pf_alloc(xh_ctx* ctx, const int T) {
    if (ctx->pf_cap >= T) return 0;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    pf_free(ctx);
    const xh_config& c = ctx->c;
    const size_t t = (size_t)T;
    int rc;
    if ((rc = dmalloc(ctx, &ctx->pf_tok, t)) || (rc = dmalloc(ctx, &ctx->pf_x, t * c.dim)) ||
        (rc = dmalloc(ctx, &ctx->pf_xn, t * c.dim)) || (rc = dmalloc(ctx, &ctx->pf_q, t * ctx->q_dim)) ||
        (rc = dmalloc(ctx, &ctx->pf_att, t * ctx->q_dim)) || (rc = dmalloc(ctx, &ctx->pf_h, t * c.hidden_dim)) ||
        (rc = dmalloc(ctx, &ctx->pf_part, pf_part_floats(ctx, T))) || (rc = dmalloc(ctx, &ctx->pf_sp, t)))
        return rc;
    // pf_xh: the split-kernel fragments of <= 64 tokens, or hi rows then lo rows of a row-major
    // pass input (gemm16.h / hipBLASLt); pf_xl: the split kernel's lo fragments
    const size_t kmax = std::max({(size_t)c.dim, (size_t)c.hidden_dim, (size_t)ctx->q_dim});
    if ((rc = dmalloc(ctx, &ctx->pf_xh, 2 * std::max(t, (size_t)PF_TOK) * kmax)) ||
        (rc = dmalloc(ctx, &ctx->pf_xl, PF_TOK * kmax)) || (rc = dmalloc(ctx, &ctx->pf_xs, std::max(t, (size_t)PF_TOK))))
        return rc;
    ctx->pf_cap = T;
    return 0;
}

// the per-token split attention's partials (XH_OPT_PREFILL_ATTN 0), sized for the pass
int pf_alloc_split_attn(xh_ctx* ctx) {
    if (ctx->pf_po_cap >= ctx->pf_cap) return 0;
    hipFree(ctx->pf_po); hipFree(ctx->pf_pml); hipFree(ctx->pf_cnt);
    ctx->pf_po = ctx->pf_pml = nullptr; ctx->pf_cnt = nullptr; ctx->pf_po_cap = 0;
    const size_t t = (size_t)ctx->pf_cap;
    int rc;
    if ((rc = dmalloc(ctx, &ctx->pf_po, t * ctx->nsplit * ctx->q_dim)) ||
        (rc = dmalloc(ctx, &ctx->pf_pml, t * ctx->nsplit * ctx->c.n_heads * 2)) ||
        (rc = dmalloc(ctx, &ctx->pf_cnt, t * ctx->c.n_kv_heads)))
        return rc;
    ctx->pf_po_cap = ctx->pf_cap;
    return 0;
}

// hipBLASLt serves only XH_OPT_PREFILL 4 (the vendor GEMM in place of gemm16.h).  Its entry
// points are resolved on first use with dlopen / dlsym, so libxalm_hip.so has no link
// dependency on it (a process that already loaded a copy, e.g. torch's, gets that copy by
// soname); without it, mode 4 fails with an error and everything else is unaffected.
struct BlasApi {
#define XH_BLAS_FN(name) decltype(&hipblasLt##name) name = nullptr;
    XH_BLAS_FN(Create) XH_BLAS_FN(Destroy) XH_BLAS_FN(MatmulDescCreate) XH_BLAS_FN(MatmulDescDestroy)
    XH_BLAS_FN(MatmulDescSetAttribute) XH_BLAS_FN(MatrixLayoutCreate) XH_BLAS_FN(MatrixLayoutDestroy)
    XH_BLAS_FN(MatmulPreferenceCreate) XH_BLAS_FN(MatmulPreferenceDestroy) XH_BLAS_FN(MatmulPreferenceSetAttribute)
    XH_BLAS_FN(MatmulAlgoGetHeuristic) XH_BLAS_FN(Matmul)
#undef XH_BLAS_FN
    bool ok = false;
    std::string err;
};
const BlasApi* blas_api(std::string* why = nullptr) {
    static BlasApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* so : {"libhipblaslt.so.1", "libhipblaslt.so", "/opt/rocm/lib/libhipblaslt.so.1"})
            if ((h = dlopen(so, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char* e = dlerror();
            api.err = e ? e : "dlopen failed";
            return;
        }
        bool all = true;
#define XH_BLAS_SYM(name)                                                                \
        api.name = reinterpret_cast<decltype(api.name)>(dlsym(h, "hipblasLt" #name)); \
        all = all && api.name;
        XH_BLAS_SYM(Create) XH_BLAS_SYM(Destroy) XH_BLAS_SYM(MatmulDescCreate) XH_BLAS_SYM(MatmulDescDestroy)
        XH_BLAS_SYM(MatmulDescSetAttribute) XH_BLAS_SYM(MatrixLayoutCreate) XH_BLAS_SYM(MatrixLayoutDestroy)
        XH_BLAS_SYM(MatmulPreferenceCreate) XH_BLAS_SYM(MatmulPreferenceDestroy) XH_BLAS_SYM(MatmulPreferenceSetAttribute)
        XH_BLAS_SYM(MatmulAlgoGetHeuristic) XH_BLAS_SYM(Matmul)
#undef XH_BLAS_SYM
        api.ok = all;
        if (!all) api.err = "hipBLASLt: missing entry points";
    });
    if (why) *why = api.err;
    return api.ok ? &api : nullptr;
}

#define BLAS_TRY(ctx, expr)                                                                          \
    do {                                                                                             \
        hipblasStatus_t _s = (expr);                                                                 \
        if (_s != HIPBLAS_STATUS_SUCCESS)                                                            \
            return set_err((ctx), XH_E_HIP, "%s failed: hipBLASLt status %d", #expr, (int)_s);       \
    } while (0)

// Plan of Y[n][rows] (f32) = X[n][K] (f16) . W[rows][K]^T on hipBLASLt.  Column-major view:
// D (rows x n, ld rows) = op(A) B with A = W stored K x rows (ld K, transposed), B = X stored
// K x n (ld K); f16 A and B, f32 compute (f16 x f16 products are exact in f32).  fp8 weights
// reach it as their exact f16 image (pf_dequant): the torch-bundled hipBLASLt, loaded first
// under the same soname in a process that imported torch, has no e4m3 / e5m2 kernels.  One
// plan per (rows, K, n) holding the heuristic's candidates; *plan = nullptr when there are none.
// At most PF_BLAS_MAX_PLANS plans per context (one per GEMM shape and pass length): a new pass length
// past that runs on gemm16.h, so the map does not grow with every prompt length seen.
constexpr size_t PF_BLAS_MAX_PLANS = 256;
int blas_plan(xh_ctx* ctx, int rows, int K, int n, xh_ctx::BlasPlan** plan) {
    *plan = nullptr;
    std::string why;
    if (!blas_api(&why)) return set_err(ctx, XH_E_HIP, "XH_OPT_PREFILL 4 needs hipBLASLt: %s", why.c_str());
    if (!ctx->blas) {
        BLAS_TRY(ctx, blas_api()->Create(&ctx->blas));
        char* ws = nullptr;
        int rc = dmalloc(ctx, &ws, PF_BLAS_WS);
        if (rc) return rc;
        ctx->blas_ws = ws;
    }
    const std::vector<int> key{rows, K, n};
    auto it = ctx->blas_plans.find(key);
    if (it == ctx->blas_plans.end() && ctx->blas_plans.size() >= PF_BLAS_MAX_PLANS) return 0;  // gemm16.h instead
    if (it == ctx->blas_plans.end()) {
        xh_ctx::BlasPlan& p = ctx->blas_plans[key];  // destroyed with the context, even half-built
        BLAS_TRY(ctx, blas_api()->MatmulDescCreate(&p.md, HIPBLAS_COMPUTE_32F, HIP_R_32F));
        const hipblasOperation_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
        BLAS_TRY(ctx, blas_api()->MatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof opT));
        BLAS_TRY(ctx, blas_api()->MatmulDescSetAttribute(p.md, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof opN));
        BLAS_TRY(ctx, blas_api()->MatrixLayoutCreate(&p.la, HIP_R_16F, K, rows, K));
        BLAS_TRY(ctx, blas_api()->MatrixLayoutCreate(&p.lb, HIP_R_16F, K, n, K));
        BLAS_TRY(ctx, blas_api()->MatrixLayoutCreate(&p.lc, HIP_R_32F, rows, n, rows));
        hipblasLtMatmulPreference_t pref;
        BLAS_TRY(ctx, blas_api()->MatmulPreferenceCreate(&pref));
        size_t wss = PF_BLAS_WS;
        constexpr int NH = 8;
        hipblasLtMatmulHeuristicResult_t heur[NH];
        int nret = 0;
        hipblasStatus_t st = blas_api()->MatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES,
                                                                   &wss, sizeof wss);
        if (st == HIPBLAS_STATUS_SUCCESS)
            st = blas_api()->MatmulAlgoGetHeuristic(ctx->blas, p.md, p.la, p.lb, p.lc, p.lc, pref, NH, heur, &nret);
        blas_api()->MatmulPreferenceDestroy(pref);
        for (int i = 0; st == HIPBLAS_STATUS_SUCCESS && i < nret; i++) p.cands.push_back(heur[i].algo);
        p.ready = true;
        it = ctx->blas_plans.find(key);
    }
    if (!it->second.ready) return set_err(ctx, XH_E_HIP, "hipBLASLt: plan %d x %d x %d failed earlier", rows, K, n);
    if (!it->second.cands.empty()) *plan = &it->second;
    return 0;
}

// the GEMM on the heuristic's first candidate for its shape: a fixed algorithm, so a prompt gives
// the same logits on every run (no run-time timing of candidates, whose tilings and split-K
// choices sum in different orders)
int blas_gemm(xh_ctx* ctx, const void* w, int K, int rows, const uint16_t* x, int n, float* y) {
    xh_ctx::BlasPlan* pp = nullptr;
    int rc = blas_plan(ctx, rows, K, n, &pp);
    if (rc) return rc;
    if (!pp) return set_err(ctx, XH_E_HIP, "hipBLASLt: no algorithm for %d x %d x %d", rows, K, n);
    const float alpha = 1.f, beta = 0.f;
    BLAS_TRY(ctx, blas_api()->Matmul(ctx->blas, pp->md, &alpha, w, pp->la, x, pp->lb, &beta, y, pp->lc, y, pp->lc,
                                  &pp->cands[0], ctx->blas_ws, PF_BLAS_WS, ctx->stream));
    return 0;
}

// K slices for a GEMM of `rows` outputs: about PF_WAVE_TARGET waves, K divisible into whole
// chunk pairs
int pf_ks(int rows, int K, int E) {
    const int n_rt = (rows + 32 * PF_RT - 1) / (32 * PF_RT);
    int ks = 1;
    // slices stay whole multiples of 4 chunk pairs (the pipelined kernel) where K allows
    const int unit = K % (8 * E) == 0 ? 8 * E : 2 * E;
    while (ks < 64 && (size_t)2 * ks * n_rt <= PF_WAVE_TARGET && K % (2 * ks * unit) == 0) ks *= 2;
    return ks;
}

template <int DT>
void pf_gemm_t(const PfGemmArgs& a, hipStream_t s) {
    const int waves = (a.rows + 32 * PF_RT - 1) / (32 * PF_RT) * a.ks;
    constexpr int E = WDec<DT>::E;
    const dim3 grid((waves + PF_WAVES - 1) / PF_WAVES);
    if ((a.K / a.ks) % (8 * E) == 0)
        hipLaunchKernelGGL((prefill_gemm_kernel<DT, true, PF_RT>), grid, dim3(PF_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL((prefill_gemm_kernel<DT, false, PF_RT>), grid, dim3(PF_THREADS), 0, s, a);
}
// split-f16 GEMM: K slices of whole 4-stage rings (8E), about PF_WAVE_TARGET waves, partials fit
int pf_ks16(int rows, int K, int E) {
    if (K % (8 * E)) return 0;
    const int n_rt = (rows + 32 * PF_RT16 - 1) / (32 * PF_RT16);
    int ks = 1;
    while (ks < 64 && (size_t)2 * ks * n_rt <= PF_WAVE_TARGET && K % (2 * ks * 8 * E) == 0) ks *= 2;
    while (ks > 1 && (size_t)ks * rows > PF_PART_ROWS) ks /= 2;
    return (size_t)ks * rows <= PF_PART_ROWS ? ks : 0;
}
template <int DT>
void pf_gemm16_t(const PfGemm16Args& a, hipStream_t s) {
    const int waves = (a.rows + 32 * PF_RT16 - 1) / (32 * PF_RT16) * a.ks;
    hipLaunchKernelGGL((prefill_gemm16_kernel<DT, PF_RT16>), dim3((waves + PF_WAVES - 1) / PF_WAVES), dim3(PF_THREADS),
                       0, s, a);
}
// weights per 16-byte chunk of the f32-input MFMA kernel's decoders (WDec<DT>::E)
int pf_elems(int dt) {
    if (dt == XH_F8_E4M3_EXACT || dt == XH_F8_E5M2_EXACT || dt == XH_Q8_0) return 16;
    return dt == XH_Q4_0 ? 32 : elems_per_16b(dt);
}
// weights the f16 GEMMs take: f16 as stored, e4m3 / e5m2 through their exact f16 image (kdt
// keeps the _EXACT dtypes, whose NaN / Inf codes the reference decodes to finite values, off it)
bool pf_f8(int dt) { return dt == XH_F8_E4M3 || dt == XH_F8_E5M2; }
bool pf_f16w(int dt) { return dt == XH_F16 || pf_f8(dt); }
// Does the GEMM over W (dtype dt, K columns) run on the row-major split input: gemm16.h
// (XH_OPT_PREFILL 1: K in whole 64-deep steps) or hipBLASLt (4: a plan for every shape)?
bool pf_lay0(const xh_ctx* ctx, int dt, int K) {
    // gguf blocks: their exact f16 hi + lo images through gemm16.h (XH_OPT_PREFILL 1)
    if (gq_dt(dt)) return ctx->prefill_gemm == 1 && K % MM_KMULT == 0;
    if (!pf_f16w(dt)) return false;
    if (ctx->prefill_gemm == 1) return K % MM_KMULT == 0;
    if (ctx->prefill_gemm == 4) return ctx->blas_ok > 0;
    return false;
}
// Once per prefill: (XH_OPT_PREFILL 4, once per context) does hipBLASLt have an f16 plan for every
// full-pass GEMM of the model (if not, every dtype keeps the MFMA kernels); and the f16 image
// buffer of the largest fp8 matrix that goes to the f16 GEMMs.
int pf_prepare(xh_ctx* ctx) {
    const xh_config& c = ctx->c;
    struct G { int dt, rows, K; };
    std::vector<G> gs;
    for (const LayerW& w : ctx->L) {
        gs.push_back({kdt(w.qkv_dt, w.qkv_x), ctx->q_dim + 2 * ctx->kv_dim, c.dim});
        gs.push_back({kdt(w.wo_dt, w.wo_x), c.dim, ctx->q_dim});
        gs.push_back({kdt(w.w13_dt, w.w13_x), 2 * c.hidden_dim, c.dim});
        gs.push_back({kdt(w.w2_dt, w.w2_x), c.dim, c.hidden_dim});
    }
    gs.push_back({kdt(ctx->wcls_dt, ctx->wcls_x), std::min(PF_CLS_CHUNK, c.vocab_size), c.dim});
    if (ctx->prefill_gemm == 4 && !ctx->blas_ok) {
        int ok = 1;
        for (const G& g : gs) {
            if (!pf_f16w(g.dt)) continue;
            xh_ctx::BlasPlan* p = nullptr;
            int rc = blas_plan(ctx, g.rows, g.K, 2 * PF_TOK_BLAS, &p);
            if (rc) return rc;
            if (!p) ok = -1;
        }
        ctx->blas_ok = ok;
    }
    size_t wdq = 0;  // fp8: one f16 image; gguf blocks: hi and lo images
    for (const G& g : gs)
        if ((pf_f8(g.dt) || gq_dt(g.dt)) && pf_lay0(ctx, g.dt, g.K))
            wdq = std::max(wdq, (size_t)g.rows * g.K * (gq_dt(g.dt) ? 2 : 1));
    if (wdq > ctx->pf_wdq_elems) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(ctx->pf_wdq);
        ctx->pf_wdq = nullptr;
        ctx->pf_wdq_elems = 0;
        int rc = dmalloc(ctx, &ctx->pf_wdq, wdq);
        if (rc) return rc;
        ctx->pf_wdq_elems = wdq;
    }
    return 0;
}
// Layout of the split-f16 input of the GEMM over W (dtype dt, [rows][K]): 0 = row-major (gemm16.h
// or hipBLASLt), E > 0 = the split-f16 register-streaming kernel's fragments, -1 = no split
// (f32-input MFMA).  XH_OPT_PREFILL 1 / 4: row-major for f16 / e4m3 / e5m2 where the GEMM fits,
// else the split kernel for fp8; 2: the split kernel for f16 and fp8; 3: never split.  The split
// kernel also needs a K slicing.
int pf_layout(const xh_ctx* ctx, int dt, int K, int rows) {
    if (pf_lay0(ctx, dt, K)) return 0;
    const bool f8 = pf_f8(dt);
    const int m = ctx->prefill_gemm;
    if (!(m == 2 || ((m == 1 || m == 4) && f8))) return -1;
    if (dt != XH_F16 && !f8) return -1;
    const int E = elems_per_16b(dt);
    return pf_ks16(rows, K, E) ? E : -1;
}
// split-f16 halves of a pass's rows: hi into pf_xh; lo into pf_xl (fragments) or right after
// the hi rows (row-major)
uint16_t* pf_lo(xh_ctx* ctx, int layout, int n, int K) {
    return layout ? ctx->pf_xl : ctx->pf_xh + (size_t)n * K;
}
// grid of the split kernels: one workgroup per token row, fragments padded to 32-token tiles
int pf_split_grid(int layout, int n) { return layout ? 32 * ((n + 31) / 32) : n; }
// Tokens per pass: PF_TOK_MM (gemm16.h) / PF_TOK_BLAS (hipBLASLt) when every layer GEMM takes the
// row-major input (the lm_head of a perplexity pass aside: it runs on 64-token slices when it
// cannot), else 64 (the register-streaming MFMA kernels' two token tiles)
int pf_pass_tokens(const xh_ctx* ctx) {
    const xh_config& c = ctx->c;
    for (const LayerW& w : ctx->L)
        if (!pf_lay0(ctx, kdt(w.qkv_dt, w.qkv_x), c.dim) || !pf_lay0(ctx, kdt(w.wo_dt, w.wo_x), ctx->q_dim) ||
            !pf_lay0(ctx, kdt(w.w13_dt, w.w13_x), c.dim) || !pf_lay0(ctx, kdt(w.w2_dt, w.w2_x), c.hidden_dim))
            return PF_TOK;
    return ctx->prefill_gemm == 4 ? PF_TOK_BLAS : PF_TOK_MM;
}
// rmsnorm of the pass's rows (pf_x) as the input of the GEMM over W (dt, [rows][dim]): written
// straight into the split-f16 halves when that GEMM takes a split input (one launch)
void pf_norm(xh_ctx* ctx, const void* nw, int ndt, int m, int dt, int rows) {
    const xh_config& c = ctx->c;
    const int lay = pf_layout(ctx, dt, c.dim, rows);
    if (lay >= 0) {
        hipLaunchKernelGGL(prefill_rmsnorm_split_kernel, dim3(pf_split_grid(lay, m)), dim3(256), 0, ctx->stream,
                           (const float*)ctx->pf_x, c.dim, nw, ndt, c.norm_eps, m, lay, ctx->pf_xh,
                           pf_lo(ctx, lay, m, c.dim), ctx->pf_xs);
        ctx->pf_split_ready = true;
    } else {
        hipLaunchKernelGGL(prefill_rmsnorm_kernel, dim3(m), dim3(256), 0, ctx->stream, (const float*)ctx->pf_x, c.dim,
                           nw, ndt, c.norm_eps, ctx->pf_xn);
    }
}
// one prompt GEMM launch (gemm16.h): the 4-wave instantiation when the launch has at least
// MM_W4_PER_CU workgroups per CU, else the default
void mm_launch(const MmArgs& a, int n_cu, hipStream_t s) {
    const int grid = a.n_rt * a.n_tt * a.ks;
    if (grid >= MM_W4_PER_CU * n_cu) {
        ensure_lds((const void*)mm_f16_kernel_w4, MM_LDS_W4);
        hipLaunchKernelGGL(mm_f16_kernel_w4, dim3(grid), dim3(MM_THREADS_W4), MM_LDS_W4, s, a);
    } else {
        ensure_lds((const void*)mm_f16_kernel, MM_LDS);
        hipLaunchKernelGGL(mm_f16_kernel, dim3(grid), dim3(MM_THREADS), MM_LDS, s, a);
    }
}
// Y partials of W[rows][K] . X[n][K] into pf_part ([ks][n][rows]).  Split-f16 paths convert x
// first unless pf_norm / the fused GLU already left its halves.  0 or an error code.
int pf_gemm(xh_ctx* ctx, const char* what, int dt, const void* w, int K, int rows, const float* x, int n, int& ks) {
    const int lay = pf_layout(ctx, dt, K, rows);
    ctx->pf_scaled = false;
    if (lay >= 0) {
        if (ctx->pf_split_ready)
            ctx->pf_split_ready = false;
        else
            hipLaunchKernelGGL(prefill_split_kernel, dim3(pf_split_grid(lay, n)), dim3(256), 0, ctx->stream, x, K, n,
                               lay, ctx->pf_xh, pf_lo(ctx, lay, n, K), ctx->pf_xs);
    }
    if (lay == 0) {
        // row-major hi rows then lo rows; partials unscaled, the epilogue multiplies by 1 / s_t
        if (pf_f8(dt)) {
            // the matrix's exact f16 image first (one streaming pass: 1 B read, 2 B written per weight)
            const size_t n16 = (size_t)rows * K / 16;
            if ((size_t)rows * K > ctx->pf_wdq_elems || K % 16)
                return set_err(ctx, XH_E_INVALID, "prefill: %s fp8 image does not fit", what);
            const int grid = (int)std::min<size_t>((n16 + 255) / 256, 8192);
            if (dt == XH_F8_E4M3)
                hipLaunchKernelGGL(pf_dequant_f16_kernel<XH_F8_E4M3>, dim3(grid), dim3(256), 0, ctx->stream,
                                   (const u32x4*)w, n16, (u32x4*)ctx->pf_wdq);
            else
                hipLaunchKernelGGL(pf_dequant_f16_kernel<XH_F8_E5M2>, dim3(grid), dim3(256), 0, ctx->stream,
                                   (const u32x4*)w, n16, (u32x4*)ctx->pf_wdq);
            w = ctx->pf_wdq;
        }
        const uint16_t* w_lo = nullptr;  // gguf blocks: the lo image, a second GEMM into more partials
        if (gq_dt(dt)) {
            if ((size_t)2 * rows * K > ctx->pf_wdq_elems || K % 32)
                return set_err(ctx, XH_E_INVALID, "prefill: %s block image does not fit", what);
            const size_t chunks = (size_t)rows * K / 8;
            const int grid = (int)std::min<size_t>((chunks + 255) / 256, 8192);
            uint16_t* hi = ctx->pf_wdq;
            uint16_t* lo = ctx->pf_wdq + (size_t)rows * K;
            if (dt == XH_Q8_0)
                hipLaunchKernelGGL(pf_dequant_gq_kernel<XH_Q8_0>, dim3(grid), dim3(256), 0, ctx->stream,
                                   (const uint8_t*)w, rows, K, hi, lo);
            else
                hipLaunchKernelGGL(pf_dequant_gq_kernel<XH_Q4_0>, dim3(grid), dim3(256), 0, ctx->stream,
                                   (const uint8_t*)w, rows, K, hi, lo);
            w = hi;
            w_lo = lo;
        }
        ctx->pf_scaled = true;
        if (ctx->prefill_gemm == 4) {
            // hi and lo rows as one B operand of 2n columns: partials [2][n][rows]; a pass length
            // hipBLASLt has no algorithm for runs on gemm16.h instead (same layout, same bound)
            xh_ctx::BlasPlan* pp = nullptr;
            int rc = blas_plan(ctx, rows, K, 2 * n, &pp);
            if (rc) return rc;
            if (pp || K % MM_KMULT) {
                rc = blas_gemm(ctx, w, K, rows, ctx->pf_xh, 2 * n, ctx->pf_part);
                if (rc) return rc;
                ks = 2;
                return 0;
            }
        }
        const int images = w_lo ? 2 : 1;
        const size_t cap = pf_part_floats(ctx, ctx->pf_cap);
        MmArgs a{};
        a.w = (const uint16_t*)w; a.xh = ctx->pf_xh; a.xl = ctx->pf_xh + (size_t)n * K; a.out = ctx->pf_part;
        a.rows = rows; a.K = K; a.n = n; a.ks = mm_pick_ks(rows, K, n, cap / images, ctx->n_cu);
        a.n_rt = mm_row_tiles(rows); a.n_tt = mm_tok_tiles(n);
        if (a.ks <= 0 || (size_t)images * a.ks * n * rows > cap)
            return set_err(ctx, XH_E_INVALID, "prefill: %s GEMM %d x %d over %d tokens does not fit", what, rows, K, n);
        mm_launch(a, ctx->n_cu, ctx->stream);
        if (w_lo) {  // partials [ks, 2 ks): W_lo . X, summed after W_hi's by the epilogue
            a.w = w_lo;
            a.out = ctx->pf_part + (size_t)a.ks * n * rows;
            mm_launch(a, ctx->n_cu, ctx->stream);
        }
        ks = images * a.ks;
        return 0;
    }
    if (lay > 0) {
        PfGemm16Args a{};
        a.w = w; a.row_bytes = (size_t)K * (16 / lay); a.K = K; a.rows = rows;
        a.xh = ctx->pf_xh; a.xl = ctx->pf_xl; a.inv_s = ctx->pf_xs; a.n = n; a.ks = pf_ks16(rows, K, lay);
        a.part = ctx->pf_part;
        switch (dt) {
            case XH_F16: pf_gemm16_t<XH_F16>(a, ctx->stream); break;
            case XH_F8_E4M3: pf_gemm16_t<XH_F8_E4M3>(a, ctx->stream); break;
            default: pf_gemm16_t<XH_F8_E5M2>(a, ctx->stream); break;
        }
        ks = a.ks;
        return 0;
    }
    const int E = pf_elems(dt);
    if (K % (2 * E) || n > PF_TOK) return set_err(ctx, XH_E_INVALID, "prefill: %s shape not supported", what);
    PfGemmArgs a{};
    a.w = w; a.K = K; a.rows = rows; a.x = x; a.n = n; a.part = ctx->pf_part;
    a.row_bytes = gq_dt(dt) ? gq_pitch(dt, K) : (size_t)K * (16 / E);
    a.ks = pf_ks(rows, K, E);
    if ((size_t)a.ks * rows > PF_PART_ROWS) return set_err(ctx, XH_E_INVALID, "prefill: %s shape not supported", what);
    hipStream_t s = ctx->stream;
    switch (dt) {
        case XH_F32: pf_gemm_t<XH_F32>(a, s); break;
        case XH_F16: pf_gemm_t<XH_F16>(a, s); break;
        case XH_BF16: pf_gemm_t<XH_BF16>(a, s); break;
        case XH_F8_E4M3: pf_gemm_t<XH_F8_E4M3>(a, s); break;
        case XH_F8_E5M2: pf_gemm_t<XH_F8_E5M2>(a, s); break;
        case XH_Q8: pf_gemm_t<XH_Q8>(a, s); break;
        case XH_Q8_0: pf_gemm_t<XH_Q8_0>(a, s); break;
        case XH_Q4_0: pf_gemm_t<XH_Q4_0>(a, s); break;
        case XH_F8_E4M3_EXACT: pf_gemm_t<XH_F8_E4M3_EXACT>(a, s); break;
        case XH_F8_E5M2_EXACT: pf_gemm_t<XH_F8_E5M2_EXACT>(a, s); break;
        default: return set_err(ctx, XH_E_INVALID, "prefill: %s dtype %d not supported", what, dt);
    }
    ks = a.ks;
    return 0;
}
void pf_epi(xh_ctx* ctx, PfEpiArgs e);
// x += the last GEMM's partials (EPI_RESID), then the rmsnorm of the updated rows as the input of
// the GEMM over W (dt, [rows][dim]): one launch when that GEMM takes the split input and the
// rows fit the LDS, else pf_epi + pf_norm (the same bits either way)
int pf_resid_norm(xh_ctx* ctx, int ks, const void* nw, int ndt, int m, int dt, int rows) {
    const xh_config& c = ctx->c;
    const int lay = pf_layout(ctx, dt, c.dim, rows);
    const size_t lds = (size_t)c.dim * sizeof(float);  // + the kernel's static red[4]
    if (lay >= 0 && ctx->pf_resid_norm && c.dim % 8 == 0 && lds + 4 * sizeof(float) <= 64 * 1024) {
        HIP_TRY(ctx, hipGetLastError());  // an earlier launch's error is reported as such
        hipLaunchKernelGGL(prefill_resid_norm_split_kernel, dim3(pf_split_grid(lay, m)), dim3(256), lds, ctx->stream,
                           (const float*)ctx->pf_part, ks, (const float*)(ctx->pf_scaled ? ctx->pf_xs : nullptr),
                           ctx->pf_x, c.dim, nw, ndt, c.norm_eps, m, lay, ctx->pf_xh, pf_lo(ctx, lay, m, c.dim),
                           ctx->pf_xs);
        HIP_TRY(ctx, hipGetLastError());
        ctx->pf_split_ready = true;
        return 0;
    }
    PfEpiArgs e{};
    e.ks = ks; e.n = m; e.rows = c.dim; e.epi = EPI_RESID; e.out = ctx->pf_x;
    pf_epi(ctx, e);
    pf_norm(ctx, nw, ndt, m, dt, rows);
    return 0;
}
void pf_epi(xh_ctx* ctx, PfEpiArgs e) {
    e.part = ctx->pf_part;
    e.part_s = ctx->pf_scaled ? ctx->pf_xs : nullptr;
    const int threads = e.n * ((e.rows + 1) / 2);
    hipLaunchKernelGGL(prefill_epi_kernel, dim3((threads + 255) / 256), dim3(256), 0, ctx->stream, e);
}
template <int HD, int QPK>
void pf_attn_t(xh_ctx* ctx, const AttnArgs& a, int n) {
    const size_t smem = attn_smem_bytes(HD, QPK, ctx->t_max, a.nsplit);
    auto k = prefill_attn_kernel<HD, QPK>;
    if (smem > 64 * 1024) ensure_lds((const void*)k);
    hipLaunchKernelGGL(k, dim3(ctx->c.n_kv_heads, a.nsplit, n), dim3(ATTN_THREADS), smem, ctx->stream, a,
                       (const StepParams*)ctx->pf_sp, ctx->q_dim, ctx->c.n_kv_heads);
}
// History splits of the shared-tile prompt attention: a pass whose (KV head, query tile)
// workgroups cannot fill two per CU (a short pass: 8 workgroups for <= 32 tokens at 8 KV heads)
// walks its history in up to that many splits of >= FA_MIN_SPLIT_STAGES ring stages each (the
// split partials live in pf_part, free between the qkv epilogue and the Wo GEMM).
constexpr int FA_MIN_SPLIT_STAGES = 4;
int pf_fa_nsplit(const xh_ctx* ctx, int nqt, int n, int pos0) {
    if (!ctx->pf_fa_split) return 1;
    const int wg = ctx->c.n_kv_heads * nqt;
    int ns = std::min((2 * ctx->n_cu + wg - 1) / wg, pos0 / (32 * FA_TPS) / FA_MIN_SPLIT_STAGES);
    const size_t per = (size_t)n * (ctx->q_dim + 2 * ctx->c.n_heads);
    ns = (int)std::min<size_t>((size_t)ns, pf_part_floats(ctx, ctx->pf_cap) / per);
    return std::max(ns, 1);
}
template <int HD, int QPK>
void pf_fa_t(xh_ctx* ctx, const AttnArgs& a, int n, int pos0) {
    constexpr int TPW = 32 / QPK;
    if constexpr (HD == 128) {
        if (ctx->pf_attn_mode == 1) {
            constexpr int NW = PF_FA_WAVES;
            auto k = prefill_fa2_kernel<QPK, NW>;
            ensure_lds((const void*)k);
            const int nqt = (n + NW * TPW - 1) / (NW * TPW);
            const int nsplit = pf_fa_nsplit(ctx, nqt, n, pos0);
            float* po = nsplit > 1 ? ctx->pf_part : nullptr;
            float2* pml = nsplit > 1 ? (float2*)(ctx->pf_part + (size_t)nsplit * n * ctx->q_dim) : nullptr;
            hipLaunchKernelGGL(k, dim3(ctx->c.n_kv_heads, nqt, nsplit), dim3(64 * NW), fa_lds_bytes(), ctx->stream, a.q,
                               a.kc, a.vc, a.out, n, pos0, ctx->q_dim, ctx->kv_dim, po, pml);
            if (nsplit > 1)
                hipLaunchKernelGGL(prefill_fa_merge_kernel, dim3(ctx->c.n_heads, n), dim3(256), 0, ctx->stream, (const float*)po,
                                   (const float2*)pml, a.out, n, nsplit, ctx->q_dim);
            return;
        }
    }
    hipLaunchKernelGGL((prefill_fa_kernel<HD, QPK>), dim3(ctx->c.n_kv_heads, (n + TPW - 1) / TPW), dim3(64), 0,
                       ctx->stream, a.q, a.kc, a.vc, a.out, n, pos0, ctx->q_dim, ctx->kv_dim);
}
// head shapes of the batched path's attention: head_dim 128 / 64 with 1, 2, 4 or 8 q heads per KV
// head (MHA through GQA), and the test fixtures' head_dim 16 x 2
bool pf_attn_shape(int hd, int qpk) {
    return ((hd == 128 || hd == 64) && (qpk == 1 || qpk == 2 || qpk == 4 || qpk == 8)) || (hd == 16 && qpk == 2);
}
template <int HD>
bool pf_attn_hd(xh_ctx* ctx, const AttnArgs& a, int n, int pos0, int qpk) {
    if (ctx->pf_attn_mode != 0) {
        switch (qpk) {
            case 1: pf_fa_t<HD, 1>(ctx, a, n, pos0); return true;
            case 2: pf_fa_t<HD, 2>(ctx, a, n, pos0); return true;
            case 4: pf_fa_t<HD, 4>(ctx, a, n, pos0); return true;
            case 8: pf_fa_t<HD, 8>(ctx, a, n, pos0); return true;
            default: return false;
        }
    }
    switch (qpk) {
        case 1: pf_attn_t<HD, 1>(ctx, a, n); return true;
        case 2: pf_attn_t<HD, 2>(ctx, a, n); return true;
        case 4: pf_attn_t<HD, 4>(ctx, a, n); return true;
        case 8: pf_attn_t<HD, 8>(ctx, a, n); return true;
        default: return false;
    }
}
// 0, XH_E_INVALID for a head shape with no prompt attention, or the split buffers' allocation error
int pf_attn(xh_ctx* ctx, const AttnArgs& a, int n, int pos0) {
    const int hd = ctx->c.head_dim, qpk = ctx->qpk;
    if (!pf_attn_shape(hd, qpk)) return set_err(ctx, XH_E_INVALID, "prefill: head shape not instantiated");
    AttnArgs b = a;
    if (ctx->pf_attn_mode == 0) {
        const int rc = pf_alloc_split_attn(ctx);  // keeps dmalloc's code and message
        if (rc) return rc;
        b.part_o = ctx->pf_po; b.part_ml = ctx->pf_pml; b.counters = ctx->pf_cnt;
    }
    bool ok = true;
    if (hd == 128) ok = pf_attn_hd<128>(ctx, b, n, pos0, qpk);
    else if (hd == 64) ok = pf_attn_hd<64>(ctx, b, n, pos0, qpk);
    else if (ctx->pf_attn_mode != 0) pf_fa_t<16, 2>(ctx, b, n, pos0);
    else pf_attn_t<16, 2>(ctx, b, n);
    return ok ? 0 : set_err(ctx, XH_E_INVALID, "prefill: head shape not instantiated");
}

// Whether the batched path covers this prompt (else the per-token loop): no ring wrap inside
// the prompt, an instantiated head shape, K multiples of the chunk pair (always, for K % 32).
bool pf_supported(const xh_ctx* ctx, int n, int pos0) {
    const xh_config& c = ctx->c;
    if (!ctx->prefill_batched || pos0 + n > c.max_seq_len) return false;
    const int hd = c.head_dim, qpk = ctx->qpk;
    if (!pf_attn_shape(hd, qpk)) return false;
    // every GEMM's K in whole chunk pairs of its decoder (f32-input kernel; the others need less)
    auto ok = [](int dt, int K) { return K % (2 * pf_elems(dt)) == 0; };
    for (const LayerW& w : ctx->L)
        if (!ok(w.qkv_dt, c.dim) || !ok(w.wo_dt, ctx->q_dim) || !ok(w.w13_dt, c.dim) || !ok(w.w2_dt, c.hidden_dim))
            return false;
    return ok(ctx->wcls_dt, c.dim) && c.dim % 32 == 0 && c.hidden_dim % 32 == 0 && ctx->q_dim % 32 == 0;
}

// tokens[0..n) at positions pos0..: HYDRATE for every token, then the last token's logits.
// probs (device, n floats) != nullptr: also every token's logits (final rmsnorm + lm_head as
// one GEMM per pass) and probs[i] = sample_prob(targets[i]) (targets: host, n ints).
int prefill_batched(xh_ctx* ctx, const int* tokens, int n, int pos0, int want_logits, const int* targets = nullptr,
                    float* probs = nullptr) {
    const xh_config& c = ctx->c;
    int rc = pf_prepare(ctx);
    if (rc) return rc;
    const int pass = ctx->pf_pass = pf_pass_tokens(ctx);
    if ((rc = pf_alloc(ctx, std::min(pass, std::max(n, PF_TOK))))) return rc;
    ctx->pf_split_ready = false;
    if (probs && !ctx->pf_logits &&
        ((rc = dmalloc(ctx, &ctx->pf_logits, (size_t)ctx->pf_cap * c.vocab_size)) ||
         (rc = dmalloc(ctx, &ctx->pf_tgt, (size_t)ctx->pf_cap))))
        return rc;
    std::vector<StepParams> sps(pass);
    for (int off = 0; off < n; off += pass) {
        const int m = std::min(n - off, pass);
        const int p0 = pos0 + off;
        HIP_TRY(ctx, hipMemcpyAsync(ctx->pf_tok, tokens + off, (size_t)m * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
        for (int t = 0; t < m; t++) {
            StepParams& h = sps[t];
            h = StepParams{};
            h.token = tokens[off + t];
            h.pos = p0 + t;
            h.kv_sink = 0;
            h.kv_pos = p0 + t;
            h.kv_len = p0 + t + 1;
            h.max_seq_len = c.max_seq_len;
        }
        HIP_TRY(ctx, hipMemcpyAsync(ctx->pf_sp, sps.data(), (size_t)m * sizeof(StepParams), hipMemcpyHostToDevice,
                                    ctx->stream));
        hipLaunchKernelGGL(prefill_embed_kernel, dim3(m), dim3(256), 0, ctx->stream, (const int*)ctx->pf_tok,
                           (const void*)ctx->embed, ctx->embed_dt, c.dim, ctx->pf_x);
        for (int l = 0; l < c.n_layers; l++) {
            const LayerW& w = ctx->L[l];
            // attention block (src/infer.cpp:380-452)
            const int qkv_rows = ctx->q_dim + 2 * ctx->kv_dim;
            int ks = 0;
            // layers after the first: the previous W2 residual and this rmsnorm ran as one launch
            if (l == 0) pf_norm(ctx, w.attn_norm, w.an_dt, m, kdt(w.qkv_dt, w.qkv_x), qkv_rows);
            if ((rc = pf_gemm(ctx, "qkv", kdt(w.qkv_dt, w.qkv_x), w.wqkv, c.dim, qkv_rows, ctx->pf_xn, m, ks))) return rc;
            PfEpiArgs e{};
            e.ks = ks; e.n = m; e.rows = qkv_rows; e.epi = EPI_QKV; e.q = ctx->pf_q;
            e.kcache = ctx->kcache(l); e.vcache = ctx->vcache(l); e.q_dim = ctx->q_dim; e.kv_dim = ctx->kv_dim;
            e.head_dim = c.head_dim; e.rope_freq = ctx->rope_freq; e.qkv_clip = c.qkv_clip; e.pos0 = p0; e.act = c.act;
            pf_epi(ctx, e);
            AttnArgs aa = attn_args(ctx, l);
            aa.q = ctx->pf_q; aa.out = ctx->pf_att;
            // splits for this pass's longest row (attn_block: >= ATTN_MIN_T slots per split)
            aa.nsplit = std::min(ctx->nsplit, std::max(1, (p0 + m + ATTN_MIN_T - 1) / ATTN_MIN_T));
            if ((rc = pf_attn(ctx, aa, m, p0))) return rc;
            if ((rc = pf_gemm(ctx, "wo", kdt(w.wo_dt, w.wo_x), w.wo, ctx->q_dim, c.dim, ctx->pf_att, m, ks))) return rc;
            // residual, then the feed-forward block's rmsnorm (src/infer.cpp:449-452, 455-494)
            if ((rc = pf_resid_norm(ctx, ks, w.ffn_norm, w.fn_dt, m, kdt(w.w13_dt, w.w13_x), 2 * c.hidden_dim))) return rc;
            if ((rc = pf_gemm(ctx, "w1/w3", kdt(w.w13_dt, w.w13_x), w.w13, c.dim, 2 * c.hidden_dim, ctx->pf_xn, m, ks)))
                return rc;
            const int lay2 = pf_layout(ctx, kdt(w.w2_dt, w.w2_x), c.hidden_dim, c.dim);
            // dynamic LDS = one f32 row of h; the kernel adds a static 16-float reduction array
            const size_t glu_lds = (size_t)c.hidden_dim * sizeof(float);
            bool glu_fused = false;
            if (lay2 >= 0 && ctx->pf_glu_split && glu_lds + 16 * sizeof(float) <= 64 * 1024) {
                // GLU epilogue straight into the W2 GEMM's split-f16 input (one launch); the size
                // check above is the launch's only precondition, so any error here is real.
                // part_s and inv_s are both pf_xs: a workgroup reads its token's factor before
                // the barrier and writes the new one after it.
                HIP_TRY(ctx, hipGetLastError());  // an earlier launch's error is reported as such
                hipLaunchKernelGGL(prefill_glu_split_kernel, dim3(pf_split_grid(lay2, m)), dim3(1024), glu_lds,
                                   ctx->stream, (const float*)ctx->pf_part, ks, m, c.hidden_dim, c.act, lay2,
                                   ctx->pf_xh, pf_lo(ctx, lay2, m, c.hidden_dim), ctx->pf_xs,
                                   (const float*)(ctx->pf_scaled ? ctx->pf_xs : nullptr));
                HIP_TRY(ctx, hipGetLastError());
                glu_fused = true;
                ctx->pf_split_ready = true;
            }
            if (!glu_fused) {
                e = PfEpiArgs{};
                e.ks = ks; e.n = m; e.rows = 2 * c.hidden_dim; e.epi = EPI_GLU; e.out = ctx->pf_h; e.act = c.act;
                pf_epi(ctx, e);
            }
            if ((rc = pf_gemm(ctx, "w2", kdt(w.w2_dt, w.w2_x), w.w2, c.hidden_dim, c.dim, ctx->pf_h, m, ks))) return rc;
            if (l + 1 < c.n_layers) {
                // residual, then the next layer's attention rmsnorm (src/infer.cpp:491-494, 380)
                const LayerW& wn = ctx->L[l + 1];
                if ((rc = pf_resid_norm(ctx, ks, wn.attn_norm, wn.an_dt, m, kdt(wn.qkv_dt, wn.qkv_x), qkv_rows))) return rc;
            } else {
                e = PfEpiArgs{};
                e.ks = ks; e.n = m; e.rows = c.dim; e.epi = EPI_RESID; e.out = ctx->pf_x;
                pf_epi(ctx, e);
            }
        }
        if (probs) {
            // Model::forward's OUTPUT_LOGITS tail (src/infer.cpp:620-637) for every token of the
            // pass, then Sampler::sample_prob of each token's target
            HIP_TRY(ctx, hipMemcpyAsync(ctx->pf_tgt, targets + off, (size_t)m * sizeof(int), hipMemcpyHostToDevice,
                                        ctx->stream));
            hipLaunchKernelGGL(prefill_rmsnorm_kernel, dim3(m), dim3(256), 0, ctx->stream, (const float*)ctx->pf_x, c.dim,
                               (const void*)ctx->final_norm, ctx->final_norm_dt, c.norm_eps, ctx->pf_xn);
            const size_t cls_rb = dev_row_bytes(ctx->wcls_dt, c.dim);
            const int cls_dt = kdt(ctx->wcls_dt, ctx->wcls_x);
            // lm_head weights off the hipBLASLt path (bf16 on the fp8 checkpoints): 64-token slices
            const int tstep = pf_lay0(ctx, cls_dt, c.dim) ? m : PF_TOK;
            for (int r0 = 0; r0 < c.vocab_size; r0 += PF_CLS_CHUNK) {
                const int rows = std::min(PF_CLS_CHUNK, c.vocab_size - r0);
                for (int t0 = 0; t0 < m; t0 += tstep) {
                    const int mt = std::min(tstep, m - t0);
                    int ks = 0;
                    if ((rc = pf_gemm(ctx, "lm_head", cls_dt, (const char*)ctx->wcls + (size_t)r0 * cls_rb, c.dim, rows,
                                      ctx->pf_xn + (size_t)t0 * c.dim, mt, ks)))
                        return rc;
                    PfEpiArgs e{};
                    e.ks = ks; e.n = mt; e.rows = rows; e.epi = EPI_STORE;
                    e.out = ctx->pf_logits + (size_t)t0 * c.vocab_size + r0;
                    e.out_stride = (size_t)c.vocab_size;
                    pf_epi(ctx, e);
                }
            }
            hipLaunchKernelGGL(token_prob_kernel, dim3(m), dim3(1024), 0, ctx->stream, (const float*)ctx->pf_logits,
                               c.vocab_size, (size_t)c.vocab_size, (const int*)ctx->pf_tgt, probs + off);
        }
        HIP_TRY(ctx, hipGetLastError());
        if (off + m == n) {
            // the last token's residual stream is the decode path's x
            HIP_TRY(ctx, hipMemcpyAsync(ctx->x, ctx->pf_x + (size_t)(m - 1) * c.dim, (size_t)c.dim * 4,
                                        hipMemcpyDeviceToDevice, ctx->stream));
        }
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // sps / token staging reused by the next pass
    }
    // step parameters of the last prompt token (as the per-token loop leaves them)
    rc = host_step_params(ctx, tokens[n - 1], pos0 + n - 1);
    if (rc) return rc;
    if (want_logits) {
        if (!launch_gemv<PRO_RMSNORM, EPI_LOGITS>(kdt(ctx->wcls_dt, ctx->wcls_x), cls_args(ctx), ctx->stream,
                                                   ctx->max_gemv_waves))
            return set_err(ctx, XH_E_INVALID, "unsupported wcls dtype");
        ctx->cand_valid = true;
    }
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

template <typename T>
int dmalloc(xh_ctx* ctx, T** p, size_t n) {
    HIP_TRY(ctx, hipMalloc((void**)p, n ? n * sizeof(T) : 16));
    HIP_TRY(ctx, fill_sync(ctx, *p, 0, n ? n * sizeof(T) : 16));
    return 0;
}

}  // namespace

// =======================================================================================
// C ABI
// =======================================================================================
extern "C" {

const char* xh_last_error(const xh_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int xh_create(const xh_config* cfg, int device_ordinal, xh_ctx** out) {
    if (!cfg || !out) return set_err(nullptr, XH_E_INVALID, "null argument");
    *out = nullptr;
    const xh_config& c = *cfg;
    if (c.dim <= 0 || c.hidden_dim <= 0 || c.head_dim <= 0 || c.n_layers <= 0 || c.n_heads <= 0 ||
        c.n_kv_heads <= 0 || c.vocab_size <= 0 || c.max_seq_len <= 2)
        return set_err(nullptr, XH_E_INVALID, "bad config dims");
    if (c.dim % 32 || c.hidden_dim % 32 || c.head_dim % 16 || (c.n_heads * c.head_dim) % 32)
        return set_err(nullptr, XH_E_INVALID, "dims must be multiples of 32 (head_dim of 16), as the reference asserts");
    if (c.n_heads % c.n_kv_heads) return set_err(nullptr, XH_E_INVALID, "n_heads %% n_kv_heads != 0");
    const int qpk = c.n_heads / c.n_kv_heads;
    if (!(qpk == 1 || qpk == 2 || qpk == 4 || qpk == 8))
        return set_err(nullptr, XH_E_INVALID, "q heads per kv head must be 1, 2, 4 or 8 (got %d)", qpk);
    if (!(c.head_dim == 16 || c.head_dim == 32 || c.head_dim == 64 || c.head_dim == 128 || c.head_dim == 256))
        return set_err(nullptr, XH_E_INVALID, "head_dim must be 16..256 power of two (got %d)", c.head_dim);
    if (c.rotary_dim > c.head_dim || c.rotary_dim < 0) return set_err(nullptr, XH_E_INVALID, "bad rotary_dim");
    {
        const int ns = attn_nsplit(c.n_kv_heads, c.max_seq_len);
        if (attn_smem_bytes(c.head_dim, qpk, attn_split_len(c.max_seq_len, ns), ns) > 160 * 1024)
            return set_err(nullptr, XH_E_INVALID, "attention tile of head_dim %d x %d q heads per kv head exceeds LDS",
                           c.head_dim, qpk);
    }
    if (c.act != XH_ACT_GELU && c.act != XH_ACT_SILU) return set_err(nullptr, XH_E_INVALID, "bad act");

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_err(nullptr, XH_E_HIP, "no HIP device available");
    if (device_ordinal < 0 || device_ordinal >= ndev)
        return set_err(nullptr, XH_E_INVALID, "device %d out of range (%d devices)", device_ordinal, ndev);

    xh_ctx* ctx = new xh_ctx();
    ctx->c = c;
    ctx->dev = device_ordinal;
    ctx->L.resize(c.n_layers);
    ctx->q_dim = c.n_heads * c.head_dim;
    ctx->kv_dim = c.n_kv_heads * c.head_dim;
    ctx->qpk = qpk;
    ctx->nsplit = attn_nsplit(c.n_kv_heads, c.max_seq_len);
    ctx->t_max = attn_split_len(c.max_seq_len, ctx->nsplit);
    ctx->t_max_aw = attn_split_len(c.max_seq_len, ctx->nsplit, attn_min_t_partials(c.head_dim, AW_THREADS));
    int rc = 0;
#define CREATE_TRY(expr) do { rc = (expr); if (rc) { g_create_error = ctx->err; xh_destroy(ctx); return rc; } } while (0)
    if (hipSetDevice(device_ordinal) != hipSuccess) { delete ctx; return set_err(nullptr, XH_E_HIP, "hipSetDevice failed"); }
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return set_err(nullptr, XH_E_HIP, "stream create failed");
    }
    CREATE_TRY(dmalloc(ctx, &ctx->kv, (size_t)c.n_layers * 2 * c.max_seq_len * ctx->kv_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->x, (size_t)c.dim));
    CREATE_TRY(dmalloc(ctx, &ctx->q, (size_t)ctx->q_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->attn_out, (size_t)ctx->q_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->hb, (size_t)c.hidden_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->logits, (size_t)c.vocab_size));
    CREATE_TRY(dmalloc(ctx, &ctx->part_o, (size_t)ctx->nsplit * ctx->q_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->part_ml, (size_t)ctx->nsplit * c.n_heads * 2));
    CREATE_TRY(dmalloc(ctx, &ctx->attn_cnt, (size_t)c.n_kv_heads));
    CREATE_TRY(dmalloc(ctx, &ctx->aw_sync, (size_t)c.n_layers * AW_SYNC_WORDS));
    CREATE_TRY(dmalloc(ctx, &ctx->cand, (size_t)ARGMAX_CANDS));
    CREATE_TRY(dmalloc(ctx, &ctx->scan_flag, (size_t)1));
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device_ordinal) != hipSuccess) {
            g_create_error = "hipGetDeviceProperties failed";
            xh_destroy(ctx);
            return XH_E_HIP;
        }
        ctx->n_cu = prop.multiProcessorCount;
    }
    ctx->aw_trace_len = (size_t)8 * ((size_t)c.n_kv_heads * ctx->nsplit + 4096);
    CREATE_TRY(dmalloc(ctx, &ctx->aw_trace, ctx->aw_trace_len));
    CREATE_TRY(dmalloc(ctx, &ctx->rope_freq, (size_t)c.head_dim / 2));
    CREATE_TRY(dmalloc(ctx, &ctx->rope_cs, (size_t)c.head_dim));
    CREATE_TRY(dmalloc(ctx, &ctx->sink_cos, (size_t)c.head_dim / 2));
    CREATE_TRY(dmalloc(ctx, &ctx->sink_sin, (size_t)c.head_dim / 2));
    CREATE_TRY(dmalloc(ctx, &ctx->sp, 1));
    ctx->dec_cap = 1 << 16;
    CREATE_TRY(dmalloc(ctx, &ctx->dec_tokens, (size_t)ctx->dec_cap));
    if (hipHostMalloc((void**)&ctx->sp_host, sizeof(StepParams), hipHostMallocDefault) != hipSuccess) {
        g_create_error = "hipHostMalloc failed";
        xh_destroy(ctx);
        return XH_E_HIP;
    }
    memset(ctx->sp_host, 0, sizeof(StepParams));
    ctx->sp_host->max_seq_len = c.max_seq_len;
    // rope frequencies with the host libm, exactly the reference expression (src/infer.cpp:310-312)
    std::vector<float> fr(c.head_dim / 2), sc(c.head_dim / 2), sn(c.head_dim / 2);
    for (int j = 0; j < c.head_dim; j += 2) {
        const float freq = j >= c.rotary_dim ? 0.f : 1.0f / powf(c.rope_theta, (float)j / (float)c.rotary_dim);
        fr[j / 2] = freq;
        const float val = 1 * freq;  // sink re-rotation: rope at pos = 1 (src/infer.cpp:426)
        sc[j / 2] = cosf(val);
        sn[j / 2] = sinf(val);
    }
    if (copy_sync(ctx, ctx->rope_freq, fr.data(), fr.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        copy_sync(ctx, ctx->sink_cos, sc.data(), sc.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        copy_sync(ctx, ctx->sink_sin, sn.data(), sn.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        copy_sync(ctx, ctx->sp, ctx->sp_host, sizeof(StepParams), hipMemcpyHostToDevice) != hipSuccess) {
        g_create_error = "initial copies failed";
        xh_destroy(ctx);
        return XH_E_HIP;
    }
#undef CREATE_TRY
    *out = ctx;
    return 0;
}

void xh_destroy(xh_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->dev);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    drop_graphs(ctx);
    for (auto& w : ctx->L) {
        hipFree(w.wqkv); hipFree(w.w13); hipFree(w.wo); hipFree(w.w2); hipFree(w.attn_norm); hipFree(w.ffn_norm);
    }
    if (ctx->wcls && ctx->wcls != ctx->embed) hipFree(ctx->wcls);
    hipFree(ctx->embed); hipFree(ctx->final_norm);
    hipFree(ctx->kv); hipFree(ctx->x); hipFree(ctx->q); hipFree(ctx->attn_out); hipFree(ctx->hb);
    hipFree(ctx->logits); hipFree(ctx->part_o); hipFree(ctx->part_ml); hipFree(ctx->attn_cnt); hipFree(ctx->aw_sync); hipFree(ctx->cand); hipFree(ctx->scan_flag);
    pf_free(ctx);
    hipFree(ctx->pf_wdq); hipFree(ctx->ppl_tgt); hipFree(ctx->ppl_prob); hipFree(ctx->rope_freq); hipFree(ctx->rope_cs);
    hipFree(ctx->aw_trace);
    for (auto& kv : ctx->blas_plans) {
        const xh_ctx::BlasPlan& p = kv.second;
        for (hipblasLtMatrixLayout_t l : {p.la, p.lb, p.lc})
            if (l) blas_api()->MatrixLayoutDestroy(l);
        if (p.md) blas_api()->MatmulDescDestroy(p.md);
    }
    if (ctx->blas) blas_api()->Destroy(ctx->blas);
    hipFree(ctx->blas_ws);
    hipFree(ctx->sink_cos); hipFree(ctx->sink_sin); hipFree(ctx->sp); hipFree(ctx->dec_tokens);
    if (ctx->sp_host) hipHostFree(ctx->sp_host);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

}  // extern "C"

namespace {

// Destination of one logical tensor [rows][cols] inside the device layout: the buffer
// (allocated on first use), the byte offset of row 0 and the byte pitch between rows.
struct Slot {
    char* base = nullptr;
    size_t pitch = 0;
    size_t rows = 0, cols = 0;
};

int tensor_slot(xh_ctx* ctx, int kind, int layer, int dtype, Slot* out) {
    const xh_config& c = ctx->c;
    const bool per_layer = !(kind == XH_EMBED || kind == XH_FINAL_NORM || kind == XH_WCLS);
    if (per_layer && (layer < 0 || layer >= c.n_layers))
        return set_err(ctx, XH_E_INVALID, "layer %d out of range", layer);
    size_t rows = 0, cols = 0;
    bool is_norm = false;
    switch (kind) {
        case XH_EMBED: case XH_WCLS: rows = c.vocab_size; cols = c.dim; break;
        case XH_ATTN_NORM: case XH_FFN_NORM: case XH_FINAL_NORM: rows = 1; cols = c.dim; is_norm = true; break;
        case XH_WQ: rows = ctx->q_dim; cols = c.dim; break;
        case XH_WK: case XH_WV: rows = ctx->kv_dim; cols = c.dim; break;
        case XH_WO: rows = c.dim; cols = ctx->q_dim; break;
        case XH_W1: case XH_W3: rows = c.hidden_dim; cols = c.dim; break;
        case XH_W2: rows = c.dim; cols = c.hidden_dim; break;
        default: return set_err(ctx, XH_E_INVALID, "unknown tensor kind %d", kind);
    }
    if (is_norm ? !(dtype == XH_F32 || dtype == XH_BF16) : !matrix_dtype_ok(dtype))
        return set_err(ctx, XH_E_INVALID, "tensor kind %d: unsupported dtype %d", kind, dtype);
    if (gq_dt(dtype) && cols % 32) return set_err(ctx, XH_E_INVALID, "tensor kind %d: %zu columns, not whole 32-element blocks", kind, cols);
    const size_t rb = dev_row_bytes(dtype, cols);
    out->rows = rows;
    out->cols = cols;
    out->pitch = rb;
    drop_graphs(ctx);
    auto plain = [&](void** dst, int* dst_dt, bool* special = nullptr) -> int {
        if (special) *special = false;  // a whole-buffer upload: rescanned after the copy
        if (*dst && *dst_dt != dtype) {
            if (*dst == ctx->wcls && *dst != ctx->embed) ctx->wcls = nullptr;
            hipFree(*dst);
            *dst = nullptr;
        }
        if (!*dst) HIP_TRY(ctx, hipMalloc(dst, rows * rb));
        *dst_dt = dtype;
        out->base = (char*)*dst;
        return 0;
    };
    if (kind == XH_EMBED) {
        const bool alias = ctx->wcls != nullptr && ctx->wcls == ctx->embed;
        if (alias) ctx->wcls = nullptr;
        int rc = plain(&ctx->embed, &ctx->embed_dt);
        if (alias) { ctx->wcls = ctx->embed; ctx->wcls_dt = ctx->embed_dt; }
        return rc;
    }
    if (kind == XH_FINAL_NORM) return plain(&ctx->final_norm, &ctx->final_norm_dt);
    if (kind == XH_WCLS) {
        if (ctx->wcls == ctx->embed) ctx->wcls = nullptr;
        return plain(&ctx->wcls, &ctx->wcls_dt, &ctx->wcls_x);
    }
    LayerW& w = ctx->L[layer];
    switch (kind) {
        case XH_ATTN_NORM: return plain(&w.attn_norm, &w.an_dt);
        case XH_FFN_NORM: return plain(&w.ffn_norm, &w.fn_dt);
        case XH_WO: return plain(&w.wo, &w.wo_dt, &w.wo_x);
        case XH_W2: return plain(&w.w2, &w.w2_dt, &w.w2_x);
        case XH_WQ: case XH_WK: case XH_WV: {
            // fused [Wq; Wk; Wv] rows, one dtype
            if (w.wqkv && w.qkv_dt != dtype) {
                if (w.qkv_have & ~(1u << (kind - XH_WQ)))
                    return set_err(ctx, XH_E_INVALID, "layer %d: q/k/v must share one dtype", layer);
                hipFree(w.wqkv); w.wqkv = nullptr; w.qkv_have = 0;
            }
            if (!(w.qkv_have & ~(1u << (kind - XH_WQ)))) w.qkv_x = false;  // no other part holds codes
            if (!w.wqkv) HIP_TRY(ctx, hipMalloc(&w.wqkv, (size_t)(ctx->q_dim + 2 * ctx->kv_dim) * rb));
            w.qkv_dt = dtype;
            const size_t row0 = kind == XH_WQ ? 0 : kind == XH_WK ? ctx->q_dim : ctx->q_dim + ctx->kv_dim;
            out->base = (char*)w.wqkv + row0 * rb;
            w.qkv_have |= 1u << (kind - XH_WQ);
            return 0;
        }
        case XH_W1: case XH_W3: {
            // fused gate/up, rows interleaved: row 2i = W1[i], row 2i+1 = W3[i]
            const unsigned bit = kind == XH_W1 ? 1u : 2u;
            if (w.w13 && w.w13_dt != dtype) {
                if (w.w13_have & ~bit) return set_err(ctx, XH_E_INVALID, "layer %d: w1/w3 must share one dtype", layer);
                hipFree(w.w13); w.w13 = nullptr; w.w13_have = 0;
            }
            if (!(w.w13_have & ~bit)) w.w13_x = false;
            if (!w.w13) HIP_TRY(ctx, hipMalloc(&w.w13, (size_t)2 * c.hidden_dim * rb));
            w.w13_dt = dtype;
            out->base = (char*)w.w13 + (kind == XH_W3 ? rb : 0);
            out->pitch = 2 * rb;
            w.w13_have |= bit;
            return 0;
        }
    }
    return set_err(ctx, XH_E_INVALID, "unhandled kind");
}

// any NaN/Inf fp8 code (f8_special) in a [rows][cols] byte matrix of row pitch `pitch`
__global__ void f8_special_scan_kernel(const uint8_t* base, size_t pitch, size_t rows, size_t cols, int e5m2, int* flag) {
    int hit = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * cols; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / cols;
        hit |= f8_special(base[r * pitch + (i - r * cols)], e5m2 != 0);
    }
    if (hit) *flag = 1;
}

// after an upload into slot s: record whether the fp8 matrix holds NaN/Inf codes
int scan_f8(xh_ctx* ctx, int kind, int layer, int dtype, const Slot& s) {
    if (dtype != XH_F8_E4M3 && dtype != XH_F8_E5M2) return 0;
    if (kind == XH_EMBED || kind == XH_ATTN_NORM || kind == XH_FFN_NORM || kind == XH_FINAL_NORM) return 0;
    HIP_TRY(ctx, hipMemsetAsync(ctx->scan_flag, 0, sizeof(int), ctx->stream));
    hipLaunchKernelGGL(f8_special_scan_kernel, dim3(2048), dim3(256), 0, ctx->stream, (const uint8_t*)s.base, s.pitch,
                       s.rows, s.cols, (int)(dtype == XH_F8_E5M2), ctx->scan_flag);
    int hit = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&hit, ctx->scan_flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (!hit) return 0;
    drop_graphs(ctx);
    if (kind == XH_WCLS) { ctx->wcls_x = true; return 0; }
    LayerW& w = ctx->L[layer];
    switch (kind) {
        case XH_WQ: case XH_WK: case XH_WV: w.qkv_x = true; break;
        case XH_W1: case XH_W3: w.w13_x = true; break;
        case XH_WO: w.wo_x = true; break;
        case XH_W2: w.w2_x = true; break;
    }
    return 0;
}

__global__ void synth_fill_kernel(char* base, size_t pitch, size_t rows, size_t cols, int dtype, uint64_t seed,
                                  float mean, float std) {
    const size_t n = rows * cols;
    const size_t esz = dtype == XH_F32 ? 4 : (dtype == XH_F16 || dtype == XH_BF16) ? 2 : 1;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / cols, cidx = i - r * cols;
        xs_store(base + r * pitch, cidx, dtype, xs_value(seed, i, mean, std));
        (void)esz;
    }
}

// gguf blocks: file layout ([rows][cols/32 blocks: f16 d, codes]) -> planar device rows
// ([codes][d per block][zero pad], pitch gq_pitch), on the host, split over threads
void gq_repack(int dt, const uint8_t* src, size_t rows, size_t cols, uint8_t* dst) {
    const size_t nb = cols / 32, bs = gq_block_bytes(dt), qb = bs - 2;
    const size_t pitch = gq_pitch(dt, cols), qbytes = gq_qbytes(dt, cols);
    auto part = [&](size_t r0, size_t r1) {
        for (size_t r = r0; r < r1; r++) {
            const uint8_t* in = src + r * nb * bs;
            uint8_t* out = dst + r * pitch;
            for (size_t b = 0; b < nb; b++) {
                memcpy(out + b * qb, in + b * bs + 2, qb);
                memcpy(out + qbytes + 2 * b, in + b * bs, 2);
            }
            memset(out + qbytes + 2 * nb, 0, pitch - qbytes - 2 * nb);
        }
    };
    const size_t nt = std::min<size_t>(16, std::max<size_t>(1, rows / 256));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; t++) th.emplace_back(part, rows * t / nt, rows * (t + 1) / nt);
    part(0, rows / nt);
    for (auto& x : th) x.join();
}

// synthetic gguf blocks: one thread per block, the values and quantizer of xalm_synth.h
// (xs_block: the oracle's bytes exactly), written straight into the planar rows of the slot
__global__ void synth_gq_kernel(char* base, size_t pitch, size_t rows, size_t cols, int dtype, uint64_t seed, float mean,
                                float std) {
    const size_t nb = cols / 32, qb = gq_block_bytes(dtype) - 2, qbytes = gq_qbytes(dtype, cols);
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * nb; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / nb, b = i - r * nb;
        uint8_t blk[34];
        xs_block(blk, dtype, seed, r, cols, b, mean, std);
        char* row = base + r * pitch;
        for (size_t k = 0; k < qb; k++) row[b * qb + k] = (char)blk[2 + k];
        row[qbytes + 2 * b] = (char)blk[0];
        row[qbytes + 2 * b + 1] = (char)blk[1];
    }
}

// the byte count of a tensor upload against the config (load_tensor's checks,
// src/model.cpp:62-76), before the device layout is touched
int check_bytes(xh_ctx* ctx, int kind, int dtype, size_t bytes) {
    const xh_config& c = ctx->c;
    size_t rows = 0, cols = 0;
    switch (kind) {
        case XH_EMBED: case XH_WCLS: rows = c.vocab_size; cols = c.dim; break;
        case XH_ATTN_NORM: case XH_FFN_NORM: case XH_FINAL_NORM: rows = 1; cols = c.dim; break;
        case XH_WQ: rows = ctx->q_dim; cols = c.dim; break;
        case XH_WK: case XH_WV: rows = ctx->kv_dim; cols = c.dim; break;
        case XH_WO: rows = c.dim; cols = ctx->q_dim; break;
        case XH_W1: case XH_W3: rows = c.hidden_dim; cols = c.dim; break;
        case XH_W2: rows = c.dim; cols = c.hidden_dim; break;
        default: return set_err(ctx, XH_E_INVALID, "unknown tensor kind %d", kind);
    }
    const size_t rb = file_row_bytes(dtype, cols);
    if (rb == 0 || (gq_dt(dtype) && cols % 32) || bytes != rows * rb)
        return set_err(ctx, XH_E_INVALID, "tensor kind %d: %zu bytes, expected %zu ([%zu,%zu] of dtype %d)", kind,
                       bytes, rows * rb, rows, cols, dtype);
    return 0;
}

}  // namespace

extern "C" {

int xh_upload(xh_ctx* ctx, int kind, int layer, int dtype, const void* host, size_t bytes) {
    if (!ctx || !host) return set_err(ctx, XH_E_INVALID, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    Slot s;
    int rc = check_bytes(ctx, kind, dtype, bytes);
    if (!rc) rc = tensor_slot(ctx, kind, layer, dtype, &s);
    if (rc) return rc;
    if (gq_dt(dtype)) {
        const size_t rb = dev_row_bytes(dtype, s.cols);
        std::vector<uint8_t> tmp(s.rows * rb);
        gq_repack(dtype, (const uint8_t*)host, s.rows, s.cols, tmp.data());
        HIP_TRY(ctx, copy2d_sync(ctx, s.base, s.pitch, tmp.data(), rb, rb, s.rows));
        return 0;
    }
    HIP_TRY(ctx, copy2d_sync(ctx, s.base, s.pitch, host, s.cols * dtype_size(dtype), s.cols * dtype_size(dtype),
                                 s.rows));
    return scan_f8(ctx, kind, layer, dtype, s);
}

// Tensor bytes straight from a file (the .xalm layout: tensor data at an absolute, 32-B
// aligned offset, convert.py:248-321) into the device slot.  The range is mapped with
// MAP_POPULATE (read ahead in one pass), registered with the runtime for the duration of
// the copy and moved by one DMA: no host copy of the tensor.  Measured on MI355X with the
// file in the page cache (tools/load_bench.py): 45 GB/s, against 16 GB/s for pread into
// two pinned staging buffers and 33 GB/s for a pageable copy of the mapping.
int xh_upload_file(xh_ctx* ctx, int kind, int layer, int dtype, const char* path, uint64_t offset, size_t bytes) {
    if (!ctx || !path) return set_err(ctx, XH_E_INVALID, "null argument");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_bytes(ctx, kind, dtype, bytes);
    if (rc) return rc;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return set_err(ctx, XH_E_INVALID, "%s: %s", path, strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0 || offset > (uint64_t)st.st_size || bytes > (uint64_t)st.st_size - offset) {
        close(fd);
        return set_err(ctx, XH_E_INVALID, "%s: %zu bytes at offset %llu run past the end of the file", path, bytes,
                       (unsigned long long)offset);
    }
    const uint64_t a0 = offset & ~(uint64_t)(sysconf(_SC_PAGESIZE) - 1);
    const size_t len = bytes + (size_t)(offset - a0);
    void* map = mmap(nullptr, len, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, (off_t)a0);
    const int map_errno = errno;
    close(fd);
    if (map == MAP_FAILED) return set_err(ctx, XH_E_INVALID, "%s: mmap: %s", path, strerror(map_errno));
    Slot s;
    rc = tensor_slot(ctx, kind, layer, dtype, &s);
    if (!rc && gq_dt(dtype)) {
        // gguf blocks: repacked on the host from the mapping (planar device rows)
        const size_t rb = dev_row_bytes(dtype, s.cols);
        std::vector<uint8_t> tmp(s.rows * rb);
        gq_repack(dtype, (const uint8_t*)map + (offset - a0), s.rows, s.cols, tmp.data());
        const hipError_t e = copy2d_sync(ctx, s.base, s.pitch, tmp.data(), rb, rb, s.rows);
        if (e != hipSuccess) rc = set_err(ctx, XH_E_HIP, "%s: copy to the device: %s", path, hipGetErrorString(e));
    } else if (!rc) {
        const size_t row_bytes = s.cols * dtype_size(dtype);
        // unregistered (e.g. a mapping the driver cannot pin) the same copy runs pageable
        const bool reg = hipHostRegister(map, len, hipHostRegisterReadOnly) == hipSuccess;
        const hipError_t e = copy2d_sync(ctx, s.base, s.pitch, (const char*)map + (offset - a0), row_bytes,
                                         row_bytes, s.rows);
        if (reg) hipHostUnregister(map);
        if (e != hipSuccess) rc = set_err(ctx, XH_E_HIP, "%s: copy to the device: %s", path, hipGetErrorString(e));
    }
    munmap(map, len);
    return rc ? rc : scan_f8(ctx, kind, layer, dtype, s);
}

int xh_upload_synthetic(xh_ctx* ctx, int kind, int layer, int dtype, uint64_t seed, float mean, float std) {
    if (!ctx) return XH_E_INVALID;
    if (dtype == XH_Q8) return set_err(ctx, XH_E_INVALID, "no synthetic Q8");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    Slot s;
    int rc = tensor_slot(ctx, kind, layer, dtype, &s);
    if (rc) return rc;
    if (gq_dt(dtype))
        hipLaunchKernelGGL(synth_gq_kernel, dim3(4096), dim3(256), 0, ctx->stream, s.base, s.pitch, s.rows, s.cols, dtype,
                           seed, mean, std);
    else
        hipLaunchKernelGGL(synth_fill_kernel, dim3(4096), dim3(256), 0, ctx->stream, s.base, s.pitch, s.rows, s.cols,
                           dtype, seed, mean, std);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return scan_f8(ctx, kind, layer, dtype, s);
}

int xh_kv_fill_synthetic(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, uint64_t seed, float std) {
    if (!ctx || layer < 0 || layer >= ctx->c.n_layers || (which != 0 && which != 1) || slot0 < 0 || n_slots < 0 ||
        slot0 + n_slots > ctx->c.max_seq_len)
        return set_err(ctx, XH_E_INVALID, "bad kv_fill_synthetic arguments");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    char* base = (char*)((which ? ctx->vcache(layer) : ctx->kcache(layer)) + (size_t)slot0 * ctx->kv_dim);
    hipLaunchKernelGGL(synth_fill_kernel, dim3(2048), dim3(256), 0, ctx->stream, base, (size_t)ctx->kv_dim * 2,
                       (size_t)n_slots, (size_t)ctx->kv_dim, (int)XH_F16, seed, 0.0f, std);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int xh_forward(xh_ctx* ctx, int token, int pos, int mode, float* logits_out) {
    if (!ctx) return XH_E_INVALID;
    if (token < 0 || token >= ctx->c.vocab_size) return set_err(ctx, XH_E_INVALID, "token %d out of range", token);
    if (pos < 0) return set_err(ctx, XH_E_INVALID, "negative pos");
    if (mode != XH_HYDRATE_KV_CACHE && mode != XH_OUTPUT_LOGITS) return set_err(ctx, XH_E_INVALID, "bad mode");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_ready(ctx);
    if (rc) return rc;
    rc = host_step_params(ctx, token, pos);
    if (!rc) rc = run_step(ctx, mode == XH_OUTPUT_LOGITS);
    if (rc) return rc;
    if (logits_out && mode == XH_OUTPUT_LOGITS)
        HIP_TRY(ctx, hipMemcpyAsync(logits_out, ctx->logits, (size_t)ctx->c.vocab_size * 4, hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_aw(ctx);
}

int xh_decode_greedy(xh_ctx* ctx, int pos, int n_steps, int stop_a, int stop_b, int* tokens_out, int* n_done) {
    if (!ctx || n_steps < 0) return XH_E_INVALID;
    if (n_done) *n_done = 0;
    if (n_steps > ctx->dec_cap) return set_err(ctx, XH_E_INVALID, "n_steps > %d", ctx->dec_cap);
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_ready(ctx);
    if (rc) return rc;
    // step counter 0, next position `pos`; token/pos fields are set by argmax_advance_kernel
    StepParams* h = ctx->sp_host;
    h->step = 0;
    h->pos_next = pos;
    h->max_seq_len = ctx->c.max_seq_len;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->sp->step, &h->step, 3 * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    if (ctx->use_graphs && n_steps > 0 && !ctx->g_decode) {
        rc = capture(ctx, 2, &ctx->g_decode);
        if (rc) return rc;
    }
    // the first token is the argmax of the logits on the device: candidates from them if the
    // launch that produced them left none (nothing yet)
    if (!ctx->cand_valid)
        hipLaunchKernelGGL(logits_cand_kernel, dim3(1), dim3(ARGMAX_CANDS), 0, ctx->stream, (const float*)ctx->logits,
                           ctx->c.vocab_size, ctx->cand);
    ctx->cand_valid = true;
    const bool stops = stop_a >= 0 || stop_b >= 0;
    int done = 0;
    for (int i = 0; i < n_steps; i++) {
        if (ctx->use_graphs) {
            HIP_TRY(ctx, hipGraphLaunch(ctx->g_decode, ctx->stream));
        } else {
            rc = eager_step(ctx, true, true);
            if (rc) return rc;
        }
        done = i + 1;
        if (stops) {
            int tok = -1;
            HIP_TRY(ctx, hipMemcpyAsync(&tok, ctx->dec_tokens + i, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            if (tok == stop_a || tok == stop_b) break;
        }
    }
    if (tokens_out && done)
        HIP_TRY(ctx, hipMemcpyAsync(tokens_out, ctx->dec_tokens, (size_t)done * sizeof(int), hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (n_done) *n_done = done;
    return check_aw(ctx);
}

int xh_get_logits(xh_ctx* ctx, float* logits_out) {
    if (!ctx || !logits_out) return XH_E_INVALID;
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    HIP_TRY(ctx, hipMemcpyAsync(logits_out, ctx->logits, (size_t)ctx->c.vocab_size * 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int xh_reset(xh_ctx* ctx) {
    if (!ctx) return XH_E_INVALID;
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    const xh_config& c = ctx->c;
    HIP_TRY(ctx, hipMemsetAsync(ctx->kv, 0, (size_t)c.n_layers * 2 * c.max_seq_len * ctx->kv_dim * 2, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->x, 0, (size_t)c.dim * 4, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->logits, 0, (size_t)c.vocab_size * 4, ctx->stream));
    // the attention + Wo hand-off words (normally zeroed by each layer's W1/W3 launch): a step
    // that failed between the two launches must not leave a stale arrival count
    HIP_TRY(ctx, hipMemsetAsync(ctx->aw_sync, 0, (size_t)c.n_layers * AW_SYNC_WORDS * 4, ctx->stream));
    HIP_TRY(ctx, hipMemsetAsync(ctx->cand, 0, ARGMAX_CANDS * 8, ctx->stream));
    ctx->cand_valid = true;  // all-zero candidates = zero logits (argmax token 0)
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int xh_kv_write(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, const uint16_t* host) {
    if (!ctx || !host || layer < 0 || layer >= ctx->c.n_layers || (which != 0 && which != 1) || slot0 < 0 ||
        n_slots < 0 || slot0 + n_slots > ctx->c.max_seq_len)
        return set_err(ctx, XH_E_INVALID, "bad kv_write arguments");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    uint16_t* base = (which ? ctx->vcache(layer) : ctx->kcache(layer)) + (size_t)slot0 * ctx->kv_dim;
    HIP_TRY(ctx, copy_sync(ctx, base, host, (size_t)n_slots * ctx->kv_dim * 2, hipMemcpyHostToDevice));
    return 0;
}

int xh_kv_read(xh_ctx* ctx, int layer, int which, int slot0, int n_slots, uint16_t* host) {
    if (!ctx || !host || layer < 0 || layer >= ctx->c.n_layers || (which != 0 && which != 1) || slot0 < 0 ||
        n_slots < 0 || slot0 + n_slots > ctx->c.max_seq_len)
        return set_err(ctx, XH_E_INVALID, "bad kv_read arguments");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint16_t* base = (which ? ctx->vcache(layer) : ctx->kcache(layer)) + (size_t)slot0 * ctx->kv_dim;
    HIP_TRY(ctx, copy_sync(ctx, host, base, (size_t)n_slots * ctx->kv_dim * 2, hipMemcpyDeviceToHost));
    return 0;
}

size_t xh_active_bytes(const xh_ctx* ctx, size_t pos) {
    // Model::active_bytes, src/model.cpp:12-35
    if (!ctx) return 0;
    const xh_config& c = ctx->c;
    size_t bytes = file_row_bytes(ctx->embed_dt, c.dim);
    bytes += (size_t)c.dim * dtype_size(ctx->final_norm_dt);
    const int wdt = ctx->wcls ? ctx->wcls_dt : ctx->embed_dt;
    bytes += (size_t)c.vocab_size * file_row_bytes(wdt, c.dim);
    const size_t kv_len = (size_t)c.max_seq_len < pos + 1 ? (size_t)c.max_seq_len : pos + 1;
    for (int l = 0; l < c.n_layers; ++l) {
        const LayerW& w = ctx->L[l];
        bytes += (size_t)c.dim * dtype_size(w.an_dt) + (size_t)c.dim * dtype_size(w.fn_dt);
        bytes += (size_t)(ctx->q_dim + 2 * ctx->kv_dim) * file_row_bytes(w.qkv_dt, c.dim);
        bytes += (size_t)c.dim * file_row_bytes(w.wo_dt, ctx->q_dim);
        bytes += (size_t)2 * c.hidden_dim * file_row_bytes(w.w13_dt, c.dim);
        bytes += (size_t)c.dim * file_row_bytes(w.w2_dt, c.hidden_dim);
        bytes += 2 * kv_len * ctx->kv_dim * 2;
    }
    return bytes;
}

int xh_prefill(xh_ctx* ctx, const int* tokens, int n, int pos0, int want_logits, float* logits_out) {
    if (!ctx || !tokens || n <= 0 || pos0 < 0) return set_err(ctx, XH_E_INVALID, "bad prefill arguments");
    for (int i = 0; i < n; i++)
        if (tokens[i] < 0 || tokens[i] >= ctx->c.vocab_size) return set_err(ctx, XH_E_INVALID, "token out of range");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_ready(ctx);
    if (rc) return rc;
    // a one-token prompt runs the decode step (one graph replay of the matvecs) rather than a
    // pass of GEMMs over one token: 3.3 vs 7.3 ms at the end of a 32k ring (tools/short_pass.py)
    if (n >= 2 && pf_supported(ctx, n, pos0)) {
        rc = prefill_batched(ctx, tokens, n, pos0, want_logits);
    } else {
        for (int i = 0; i < n && !rc; i++) {
            rc = host_step_params(ctx, tokens[i], pos0 + i);
            if (!rc) rc = run_step(ctx, i == n - 1 && want_logits);
            // the step parameters are copied from one pinned host slot: drain before reuse
            if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess)
                rc = set_err(ctx, XH_E_HIP, "hipStreamSynchronize failed");
        }
    }
    if (rc) return rc;
    if (logits_out && want_logits)
        HIP_TRY(ctx, hipMemcpyAsync(logits_out, ctx->logits, (size_t)ctx->c.vocab_size * 4, hipMemcpyDeviceToHost,
                                    ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_aw(ctx);
}

// The perplexity loop of run_perplexity (src/main.cpp:243-254): forward tokens[0..n-1) at
// positions pos0.. with logits, probs_out[i] = Sampler::sample_prob(tokens[i + 1]) after token
// i (src/sampler.cpp:3-17).  The logits never leave the device; batched passes where the
// prompt path allows, else token by token.
int xh_perplexity(xh_ctx* ctx, const int* tokens, int n, int pos0, float* probs_out) {
    if (!ctx || !tokens || !probs_out || n < 2 || pos0 < 0) return set_err(ctx, XH_E_INVALID, "bad perplexity arguments");
    for (int i = 0; i < n; i++)
        if (tokens[i] < 0 || tokens[i] >= ctx->c.vocab_size) return set_err(ctx, XH_E_INVALID, "token out of range");
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_ready(ctx);
    if (rc) return rc;
    const int m = n - 1, V = ctx->c.vocab_size;
    if (ctx->ppl_cap < m) {
        hipFree(ctx->ppl_tgt); hipFree(ctx->ppl_prob);
        ctx->ppl_tgt = nullptr; ctx->ppl_prob = nullptr; ctx->ppl_cap = 0;
        if ((rc = dmalloc(ctx, &ctx->ppl_tgt, (size_t)m)) || (rc = dmalloc(ctx, &ctx->ppl_prob, (size_t)m))) return rc;
        ctx->ppl_cap = m;
    }
    if (pf_supported(ctx, m, pos0)) {
        rc = prefill_batched(ctx, tokens, m, pos0, 0, tokens + 1, ctx->ppl_prob);
    } else {
        HIP_TRY(ctx, copy_sync(ctx, ctx->ppl_tgt, tokens + 1, (size_t)m * sizeof(int), hipMemcpyHostToDevice));
        for (int i = 0; i < m && !rc; i++) {
            rc = host_step_params(ctx, tokens[i], pos0 + i);
            if (!rc) rc = run_step(ctx, true);
            if (rc) break;
            hipLaunchKernelGGL(token_prob_kernel, dim3(1), dim3(1024), 0, ctx->stream, (const float*)ctx->logits, V,
                               (size_t)V, (const int*)ctx->ppl_tgt + i, ctx->ppl_prob + i);
            // the step parameters are copied from one pinned host slot: drain before reuse
            if (hipStreamSynchronize(ctx->stream) != hipSuccess) rc = set_err(ctx, XH_E_HIP, "hipStreamSynchronize failed");
        }
    }
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(probs_out, ctx->ppl_prob, (size_t)m * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_aw(ctx);
}

int xh_debug_trace(xh_ctx* ctx, int enable, uint64_t* out, int cap, int* len) {
    if (!ctx) return XH_E_INVALID;
    const int n = (int)ctx->aw_trace_len;
    if (len) *len = n;
    if (out && cap > 0) {
        HIP_TRY(ctx, hipSetDevice(ctx->dev));
        HIP_TRY(ctx, copy_sync(ctx, out, ctx->aw_trace, (size_t)std::min(cap, n) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    if (enable >= 0) {
        ctx->aw_trace_on = (enable & 2) != 0;
        ctx->w13_trace_on = (enable & 8) != 0;
        ctx->layer_trace_on = (enable & 16) != 0 && ctx->aw_trace_len >= LT_WORDS;
        drop_graphs(ctx);
        HIP_TRY(ctx, fill_sync(ctx, ctx->aw_trace, 0, (size_t)n * sizeof(uint64_t)));
    }
    return 0;
}

int xh_get_option(const xh_ctx* ctx, int option, int* value) {
    if (!ctx || !value) return XH_E_INVALID;
    switch (option) {
        case XH_OPT_FUSE_ATTN_WO: *value = ctx->fuse_attn_wo ? 1 : 0; return 0;
        case XH_OPT_PREFILL: *value = ctx->prefill_batched ? ctx->prefill_gemm : 0; return 0;
        case XH_OPT_PREFILL_GLU_SPLIT: *value = ctx->pf_glu_split ? 1 : 0; return 0;
        case XH_OPT_PREFILL_ATTN: *value = ctx->pf_attn_mode; return 0;
        case XH_OPT_PREFILL_ATTN_SPLIT: *value = ctx->pf_fa_split; return 0;
        default: return XH_E_INVALID;
    }
}

int xh_set_option(xh_ctx* ctx, int option, int value) {
    if (!ctx) return XH_E_INVALID;
    switch (option) {
        case XH_OPT_FUSE_ATTN_WO:
            if (value < 0 || value > 1) return set_err(ctx, XH_E_INVALID, "fuse level %d not in 0..1", value);
            ctx->fuse_attn_wo = value != 0;
            drop_graphs(ctx);
            return 0;
        case XH_OPT_PREFILL:
            if (value < 0 || value > 4) return set_err(ctx, XH_E_INVALID, "XH_OPT_PREFILL: 0 ... 4");
            ctx->prefill_batched = value != 0;
            if (value) ctx->prefill_gemm = value;
            return 0;
        case XH_OPT_PREFILL_GLU_SPLIT:
            if (value < 0 || value > 1) return set_err(ctx, XH_E_INVALID, "XH_OPT_PREFILL_GLU_SPLIT: 0 or 1");
            ctx->pf_glu_split = value != 0;
            ctx->pf_resid_norm = value != 0;
            return 0;
        case XH_OPT_PREFILL_ATTN:
            if (value < 0 || value > 2) return set_err(ctx, XH_E_INVALID, "XH_OPT_PREFILL_ATTN: 0, 1 or 2");
            ctx->pf_attn_mode = value;
            return 0;
        case XH_OPT_PREFILL_ATTN_SPLIT:
            if (value < 0 || value > 1) return set_err(ctx, XH_E_INVALID, "XH_OPT_PREFILL_ATTN_SPLIT: 0 or 1");
            ctx->pf_fa_split = value;
            return 0;
        default: return set_err(ctx, XH_E_INVALID, "unknown option %d", option);
    }
}

int xh_set_graphs(xh_ctx* ctx, int enable) {
    if (!ctx) return XH_E_INVALID;
    ctx->use_graphs = enable != 0;
    if (!ctx->use_graphs) drop_graphs(ctx);
    return 0;
}

// ---------------------------------------------------------------------------------------
// exposed-for-tests ops (host pointers).  They run the same kernels as the forward pass.
// ---------------------------------------------------------------------------------------
namespace {
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) hipFree(p); }
};
int op_alloc(DevBuf& b, size_t bytes, const void* src) {
    if (hipMalloc(&b.p, bytes ? bytes : 16) != hipSuccess) return set_err(nullptr, XH_E_HIP, "hipMalloc failed");
    if (src && hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
        return set_err(nullptr, XH_E_HIP, "hipMemcpy failed");
    return 0;
}
int op_finish(void* dst, const DevBuf& b, size_t bytes) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(nullptr, XH_E_HIP, "kernel launch failed: %s", hipGetErrorString(e));
    if (hipDeviceSynchronize() != hipSuccess) return set_err(nullptr, XH_E_HIP, "kernel failed");
    if (hipMemcpy(dst, b.p, bytes, hipMemcpyDeviceToHost) != hipSuccess)
        return set_err(nullptr, XH_E_HIP, "hipMemcpy D2H failed");
    return 0;
}
}  // namespace

int xh_op_matmul(float* xout, const float* x, const void* w, int dtype, int n, int d) {
    if (!xout || !x || !w || n <= 0 || d <= 0 || n % 16) return set_err(nullptr, XH_E_INVALID, "bad matmul args");
    if (!matrix_dtype_ok(dtype)) return set_err(nullptr, XH_E_INVALID, "unsupported dtype %d", dtype);
    DevBuf bw, bx, bo;
    int rc;
    if (gq_dt(dtype) && n % 32) return set_err(nullptr, XH_E_INVALID, "bad matmul args: n %% 32");
    // gguf blocks: w in the file layout, repacked to the planar device rows
    std::vector<uint8_t> gq_tmp;
    if (gq_dt(dtype)) {
        gq_tmp.resize((size_t)d * dev_row_bytes(dtype, n));
        gq_repack(dtype, (const uint8_t*)w, d, n, gq_tmp.data());
        w = gq_tmp.data();
    }
    const size_t wbytes = (size_t)d * dev_row_bytes(dtype, n);
    if ((rc = op_alloc(bw, wbytes, w)) || (rc = op_alloc(bx, (size_t)n * 4, x)) || (rc = op_alloc(bo, (size_t)d * 4, nullptr)))
        return rc;
    GemvArgs a{};
    a.w = bw.p; a.row_bytes = dev_row_bytes(dtype, n); a.n = n; a.rows = d;
    a.x = (const float*)bx.p; a.out = (float*)bo.p;
    bool special = false;
    if (dtype == XH_F8_E4M3 || dtype == XH_F8_E5M2)
        for (size_t i = 0; i < wbytes && !special; i++) special = f8_special(((const uint8_t*)w)[i], dtype == XH_F8_E5M2);
    launch_gemv<PRO_PLAIN, EPI_STORE>(kdt(dtype, special), a, nullptr, 4096);
    return op_finish(xout, bo, (size_t)d * 4);
}

int xh_op_rmsnorm(float* o, const float* x, const void* weight, int dtype, int size, float eps) {
    if (!o || !x || !weight || size <= 0 || size % 4 || !(dtype == XH_F32 || dtype == XH_BF16))
        return set_err(nullptr, XH_E_INVALID, "bad rmsnorm args");
    DevBuf bw, bx, bo;
    int rc;
    if ((rc = op_alloc(bw, (size_t)size * dtype_size(dtype), weight)) || (rc = op_alloc(bx, (size_t)size * 4, x)) ||
        (rc = op_alloc(bo, (size_t)size * 4, nullptr)))
        return rc;
    hipLaunchKernelGGL(rmsnorm_kernel, dim3(1), dim3(256), 0, nullptr, (float*)bo.p, (const float*)bx.p,
                       (const void*)bw.p, dtype, size, eps);
    return op_finish(o, bo, (size_t)size * 4);
}

int xh_op_rope(float* vec, int d, int head_dim, int pos, float theta, int rotary_dim) {
    if (!vec || d <= 0 || d % 2 || head_dim <= 0 || head_dim % 2) return set_err(nullptr, XH_E_INVALID, "bad rope args");
    std::vector<float> fr(head_dim / 2);
    for (int j = 0; j < head_dim; j += 2)
        fr[j / 2] = j >= rotary_dim ? 0.f : 1.0f / powf(theta, (float)j / (float)rotary_dim);
    DevBuf bv, bf;
    int rc;
    if ((rc = op_alloc(bv, (size_t)d * 4, vec)) || (rc = op_alloc(bf, fr.size() * 4, fr.data()))) return rc;
    hipLaunchKernelGGL(rope_kernel, dim3((d / 2 + 255) / 256), dim3(256), 0, nullptr, (float*)bv.p, d, head_dim, pos,
                       (const float*)bf.p);
    return op_finish(vec, bv, (size_t)d * 4);
}

int xh_op_mha(float* xout, const uint16_t* kb, const uint16_t* vb, const float* q, int head_dim, int kv_len,
              int max_seq_len, int n_heads, int n_kv_heads) {
    if (!xout || !kb || !vb || !q || kv_len <= 0 || kv_len > max_seq_len || n_kv_heads <= 0 || n_heads % n_kv_heads)
        return set_err(nullptr, XH_E_INVALID, "bad mha args");
    const int qpk = n_heads / n_kv_heads, kv_dim = n_kv_heads * head_dim;
    const int nsplit = attn_nsplit(n_kv_heads, max_seq_len);
    const int t_max = attn_split_len(max_seq_len, nsplit);
    DevBuf bk, bv, bq, bo, bpo, bpm, bsp, bcnt;
    std::vector<int> zeros((size_t)n_kv_heads, 0);
    StepParams sp{};
    sp.kv_len = kv_len;
    sp.max_seq_len = max_seq_len;
    int rc;
    const size_t kvb = (size_t)max_seq_len * kv_dim * 2;
    if ((rc = op_alloc(bk, kvb, kb)) || (rc = op_alloc(bv, kvb, vb)) || (rc = op_alloc(bq, (size_t)n_heads * head_dim * 4, q)) ||
        (rc = op_alloc(bo, (size_t)n_heads * head_dim * 4, nullptr)) ||
        (rc = op_alloc(bpo, (size_t)nsplit * n_heads * head_dim * 4, nullptr)) ||
        (rc = op_alloc(bpm, (size_t)nsplit * n_heads * 2 * 4, nullptr)) || (rc = op_alloc(bsp, sizeof sp, &sp)) ||
        (rc = op_alloc(bcnt, zeros.size() * sizeof(int), zeros.data())))
        return rc;
    AttnArgs a{};
    a.q = (const float*)bq.p; a.kc = (const uint16_t*)bk.p; a.vc = (const uint16_t*)bv.p; a.kv_dim = kv_dim;
    a.n_heads = n_heads; a.nsplit = nsplit; a.out = (float*)bo.p; a.part_o = (float*)bpo.p;
    a.part_ml = (float*)bpm.p; a.counters = (int*)bcnt.p; a.sp = (const StepParams*)bsp.p;
    if (!launch_attn(a, head_dim, qpk, n_kv_heads, t_max, nullptr))
        return set_err(nullptr, XH_E_INVALID, "unsupported head_dim %d / qpk %d", head_dim, qpk);
    return op_finish(xout, bo, (size_t)n_heads * head_dim * 4);
}

int xh_op_prompt_gemm(float* y, const uint16_t* w, const uint16_t* xh, const uint16_t* xl, int rows, int K, int n,
                      int ks) {
    if (!y || !w || !xh || !xl || rows <= 0 || n <= 0 || K <= 0 || K % MM_KMULT || ks < 0 || ks > 64)
        return set_err(nullptr, XH_E_INVALID, "bad prompt_gemm args");
    if (ks == 0) ks = mm_pick_ks(rows, K, n, (size_t)8 * n * rows);
    if (ks <= 0 || K % (ks * MM_KMULT)) return set_err(nullptr, XH_E_INVALID, "K %d not in %d slices of 64", K, ks);
    DevBuf bw, bx, bo;
    int rc;
    const size_t xe = (size_t)n * K;
    if ((rc = op_alloc(bw, (size_t)rows * K * 2, w)) || (rc = op_alloc(bx, 2 * xe * 2, nullptr)) ||
        (rc = op_alloc(bo, (size_t)ks * n * rows * 4, nullptr)))
        return rc;
    if (hipMemcpy(bx.p, xh, xe * 2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy((uint16_t*)bx.p + xe, xl, xe * 2, hipMemcpyHostToDevice) != hipSuccess)
        return set_err(nullptr, XH_E_HIP, "hipMemcpy failed");
    MmArgs a{};
    a.w = (const uint16_t*)bw.p; a.xh = (const uint16_t*)bx.p; a.xl = (const uint16_t*)bx.p + xe; a.out = (float*)bo.p;
    a.rows = rows; a.K = K; a.n = n; a.ks = ks; a.n_rt = mm_row_tiles(rows); a.n_tt = mm_tok_tiles(n);
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return set_err(nullptr, XH_E_HIP, "no device");
    mm_launch(a, n_cu, nullptr);
    std::vector<float> part((size_t)ks * n * rows);
    if ((rc = op_finish(part.data(), bo, part.size() * 4))) return rc;
    for (size_t i = 0; i < (size_t)n * rows; i++) {
        float v = 0.f;
        for (int s = 0; s < ks; s++) v += part[(size_t)s * n * rows + i];  // slice order, as prefill_epi_kernel
        y[i] = v;
    }
    return 0;
}

// ---------------------------------------------------------------------------------------
// timing hooks for bench.py
// ---------------------------------------------------------------------------------------
int xh_time_kernel(xh_ctx* ctx, int which, int iters, float* avg_us) {
    if (!ctx || !avg_us || iters <= 0 || which < 0 || which > 5) return XH_E_INVALID;
    HIP_TRY(ctx, hipSetDevice(ctx->dev));
    int rc = check_ready(ctx);
    if (rc) return rc;
    const int mb = ctx->max_gemv_waves;
    // launches rotate over the layers, so a repeat never finds its weights in the 256 MB
    // Infinity Cache (a decode step streams every layer once)
    int rot = 0;
    auto launch = [&]() -> bool {
        const int l = rot++ % ctx->c.n_layers;
        switch (which) {
            case 0: return launch_gemv<PRO_RMSNORM, EPI_GLU>(kdt(ctx->L[l].w13_dt, ctx->L[l].w13_x), w13_args(ctx, l), ctx->stream, mb);
            case 1: return launch_gemv<PRO_RMSNORM, EPI_QKV>(kdt(ctx->L[l].qkv_dt, ctx->L[l].qkv_x), qkv_args(ctx, l), ctx->stream,
                                                             qkv_launch_waves(ctx, l));
            case 2: return launch_gemv<PRO_PLAIN, EPI_RESID>(kdt(ctx->L[l].wo_dt, ctx->L[l].wo_x), wo_args(ctx, l), ctx->stream, mb);
            case 3: return launch_gemv<PRO_PLAIN, EPI_RESID>(kdt(ctx->L[l].w2_dt, ctx->L[l].w2_x), w2_args(ctx, l), ctx->stream, mb);
            case 4: return launch_gemv<PRO_RMSNORM, EPI_LOGITS>(kdt(ctx->wcls_dt, ctx->wcls_x), cls_args(ctx), ctx->stream, mb);
            default:
                return launch_attn(attn_args(ctx, l), ctx->c.head_dim, ctx->qpk, ctx->c.n_kv_heads, ctx->t_max,
                                   ctx->stream);
        }
    };
    hipEvent_t e0, e1;
    HIP_TRY(ctx, hipEventCreate(&e0));
    HIP_TRY(ctx, hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) launch();
    HIP_TRY(ctx, hipEventRecord(e0, ctx->stream));
    for (int i = 0; i < iters; i++) launch();
    HIP_TRY(ctx, hipEventRecord(e1, ctx->stream));
    HIP_TRY(ctx, hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_TRY(ctx, hipEventElapsedTime(&ms, e0, e1));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    HIP_TRY(ctx, hipGetLastError());
    *avg_us = ms * 1000.f / (float)iters;
    return 0;
}

size_t xh_kernel_bytes(const xh_ctx* ctx, int which, int kv_len) {
    if (!ctx) return 0;
    const xh_config& c = ctx->c;
    const LayerW& w = ctx->L[0];
    const size_t vec = 4;
    switch (which) {
        case 0: return (size_t)2 * c.hidden_dim * file_row_bytes(w.w13_dt, c.dim) + c.dim * (vec + dtype_size(w.fn_dt)) +
                       (size_t)c.hidden_dim * vec;
        case 1: return (size_t)(ctx->q_dim + 2 * ctx->kv_dim) * file_row_bytes(w.qkv_dt, c.dim) +
                       c.dim * (vec + dtype_size(w.an_dt)) + (size_t)ctx->q_dim * vec + 2 * ctx->kv_dim * 2;
        case 2: return (size_t)c.dim * file_row_bytes(w.wo_dt, ctx->q_dim) + ctx->q_dim * vec + 2 * c.dim * vec;
        case 3: return (size_t)c.dim * file_row_bytes(w.w2_dt, c.hidden_dim) + c.hidden_dim * vec + 2 * c.dim * vec;
        case 4: return (size_t)c.vocab_size * file_row_bytes(ctx->wcls ? ctx->wcls_dt : ctx->embed_dt, c.dim) +
                       c.dim * (vec + dtype_size(ctx->final_norm_dt)) + (size_t)c.vocab_size * vec;
        default: return (size_t)2 * kv_len * ctx->kv_dim * 2 + 2 * (size_t)ctx->q_dim * vec;
    }
}

}  // extern "C"
