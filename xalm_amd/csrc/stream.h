// stream.h — engine 2: the whole decode loop in one launch, weights streamed through an
// LDS-DMA ring per CU that runs ahead of every data dependency.
//
// Same math as the graph engine (gemv.h, attention.h), replacing Model::forward /
// _forward_cpu (jubruckne/Xalm src/model.cpp:120-122, src/infer.cpp:604-638) token after
// token, with the greedy loop of run_completion (src/main.cpp:105-115) on the device.
//
// Why: batch-1 decode reads every weight byte once per token; the graph engine loses
// ~15 us per layer to kernel boundaries, ramps and tails.  Here the weight
// stream never depends on activations, so one loader wave per CU issues it continuously into
// an LDS ring (global_load_lds_dwordx4 nt, 1 KiB per wave-instruction) while the consumer
// waves wait for the hand-offs between phases; the ring absorbs those waits
// (MI355X_MICROARCH.md price list: ldsdma-fill, prefetch-credit, engine-vs-launches).
//
// Workgroup = SE_NL loader waves + SE_NW consumer waves, one workgroup per CU, all resident.
// Per matrix, CU b owns a contiguous, balanced block of rows (pairs kept together), cut into
// tiles of <= 16 rows.  A ring slot holds one K-step of one tile: TH pieces, piece p = 1 KiB
// of row p of the tile at byte offset 1024 * ks.  K-step ks of every tile is consumed by
// consumer wave ks % SE_NW, which holds that K-step's activations in registers (the
// activation vector is never staged in LDS, so the ring gets ~150 KiB).  At the end of a
// tile the waves' partial sums meet in LDS and the last one to arrive runs the epilogue:
//   QKV : clip, rope, q (sc1) and the fp16 K/V row at kv_pos; a per-KV-head row counter
//   Wo  : x += .  (each CU keeps its own residual rows in LDS), x published as granules
//   W1/W3: hb = act(W1 x) * (W3 x), published as granules
//   W2  : x += ., published as granules
//   lm_head: logits + the CU's argmax candidate (one granule per CU per token)
// Hand-offs between CUs follow MI355X_MICROARCH.md "Valid forms": 8-byte {tag, value}
// granules written by one sc1 store and swept with sc1 loads until every tag matches (x, hb,
// attention output, argmax candidates), or sc1 payload + vmcnt(0) + an agent-scope counter
// (q and the new K/V row -> attention; split partials -> merge).  Every spin is bounded
// (2 s of s_memrealtime); a timeout sets the error word and drains every wave.
#pragma once

#include <float.h>

#include "gemv.h"

namespace xalm {

constexpr int SE_NW = 5;                        // consumer waves (8 waves in all: 256 VGPRs each)
constexpr int SE_NL = 3;                        // loader waves (waves SE_NW ..): slot seq % SE_NL
constexpr int SE_THREADS = 64 * (SE_NW + SE_NL);
constexpr int SE_SLOT = 16384;                  // ring slot: 16 pieces of 1 KiB
constexpr int SE_MAXS = 12;                     // ring slots (upper bound; host picks nslots)
constexpr int SE_DEPTH = 3;                     // slots in flight per loader wave
constexpr int SE_MAXP = 60;                     // LDS-DMA pieces in flight per loader wave (vmcnt: 6 bits)
constexpr int SE_XF = 48;                       // activation floats per lane (register slice)
constexpr int SE_NA = 4;                        // attention waves (consumer waves 0..3)
constexpr int SE_OWN_MAX = 64;                  // residual rows owned by one CU
constexpr uint64_t SE_TIMEOUT = 200000000ull;   // 2 s at 100 MHz (s_memrealtime)
enum { SE_QKV = 0, SE_WO = 1, SE_W13 = 2, SE_W2 = 3, SE_CLS = 4 };

struct SeLayer {
    const void* wqkv;  // [q_dim + 2 kv_dim][dim]
    const void* wo;    // [dim][q_dim]
    const void* w13;   // [2 hidden][dim], W1/W3 rows interleaved
    const void* w2;    // [dim][hidden]
    const void* attn_norm;
    const void* ffn_norm;
    uint16_t* kc;      // K ring [max_seq_len][kv_dim] fp16
    uint16_t* vc;
};

struct SeArgs {
    int n_layers, dim, hidden, q_dim, kv_dim, head_dim, n_heads, n_kv_heads, vocab, max_seq_len;
    float eps, qkv_clip;
    int act, norm_dt;
    const void* embed;
    int embed_dt;
    const void* final_norm;
    const void* wcls;
    const SeLayer* layers;
    const float* rope_freq;
    const float* sink_cos;
    const float* sink_sin;
    // hand-off buffers (granule buffers and counters zeroed before every launch)
    unsigned long long* xg;    // [dim]    residual stream x
    unsigned long long* hg;    // [hidden] act(W1 x) * W3 x
    unsigned long long* ag;    // [q_dim]  attention output
    unsigned long long* cg;    // [n_cu]   argmax candidate per CU
    float* q;                  // [q_dim]  (sc1, behind qcnt)
    unsigned* qcnt;            // [n_layers][n_kv_heads] q/k/v rows done (cumulative per launch)
    float* part_o;             // [max splits][n_heads][head_dim]
    float* part_ml;            // [max splits][n_heads][2]
    int* tickets;              // [n_kv_heads] split arrivals (zero between launches)
    float* logits;             // [vocab]
    int nslots;                // ring slots (<= SE_MAXS)
    int split_rows;            // attention rows per split (target)
    int max_splits;            // splits per KV head (<= n_cu / n_kv_heads)
    int rotate;                // 1: CU b streams a tile's K-steps from b % nk on (else from 0)
    int debug;                 // experiments (results invalid): 1 no FMA, 2 no hand-off waits, 4 no tile combine,
                               // 8 no per-slot loader stamps in the trace
    int* err;                  // [0] timeout flag
    // work of this launch
    const int* prompt;
    int n_prompt, n_gen, pos0, logits_last, stop_a, stop_b;
    int* tokens_out;
    int* n_done;
    // debug (null = off): [n_cu][8] sums (loader ring-full, wave 0 ring-empty, wave 0 hand-off
    // waits, wave 0 attention, loader issue->landed sum, slots, loader vmcnt-blocked, -), then
    // for the last token of CUs {0, n/2, n-1} [3][4 n_layers + 1][8] s_memrealtime stamps:
    // input wait start / end, matrix end, first slot issued by the loader, attention: q/k/v
    // counted, K/V loaded, published, -
    unsigned long long* trace;
};
// trace layout: [n_cu][8] sums, then [3 CUs][4 n_layers + 1 phases][8] stamps
constexpr int SE_TR_CU = 8, SE_TR_PH = 8;
__host__ __device__ inline int se_trace_len(int n_cu, int n_layers) {
    return SE_TR_CU * n_cu + 3 * (4 * n_layers + 1) * SE_TR_PH;
}
__device__ __forceinline__ int se_trace_cu(const int b, const int nblk) {
    return b == 0 ? 0 : b == nblk / 2 ? 1 : b == nblk - 1 ? 2 : -1;
}

// LDS control block (behind the ring)
struct SeCtl {  // part[] first: 16-byte aligned (float4 stores)
    float part[2][8][16];       // tile partial sums [parity][wave][row]
    int full[SE_MAXS];          // ring slot s % nslots holds sequence number full[.] (loader)
    int free_[SE_MAXS];         // ... and was released by its consumer at sequence number free_[.]
    int abort;                  // set by a wave that timed out: every wave leaves
    int ndone;                  // consumer waves finished (all SE_NW: the loaders leave)
    int cbar;                   // consumer-wave barrier arrivals (monotonic)
    int abar;                   // attention-wave barrier arrivals (monotonic)
    int tcnt[2];                // tile partial arrivals, by tile parity
    int tdone[2];               // tiles combined, by parity
    int cls_tiles;              // lm_head tiles combined this token
    int token;                  // broadcast of the argmax of existing logits
    int gath;                   // consumer waves gathering a hand-off (the loader thins out)
    unsigned long long best;    // packed argmax candidate of this CU (lm_head)
    float ssp[2][8];            // rmsnorm partial sums of squares, by barrier parity (SE_NW <= 8)
    float xown[SE_OWN_MAX];     // residual rows owned by this CU
};

static_assert(offsetof(SeCtl, part) % 16 == 0, "tile partials must be 16-byte aligned");
static_assert(offsetof(SeCtl, best) % 8 == 0, "candidate must be 8-byte aligned");

__host__ __device__ inline size_t se_att_floats(int qpk, int hd) { return (size_t)SE_NA * (qpk * hd + 2 * qpk); }
__host__ __device__ inline size_t se_ctl_bytes() { return (sizeof(SeCtl) + 15) & ~(size_t)15; }
__host__ __device__ inline size_t se_smem_bytes(int nslots, int qpk, int hd) {
    return (size_t)nslots * SE_SLOT + se_ctl_bytes() + se_att_floats(qpk, hd) * sizeof(float);
}

// ---- small device helpers -------------------------------------------------------------------
__device__ __forceinline__ uint64_t se_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ int se_lane() { return (int)threadIdx.x & 63; }
// LDS words shared between the waves of the workgroup.  Accessed through address-space-3
// pointers: a volatile access through a generic pointer stays a flat_* instruction (the
// address-space inference skips volatile), and the compiler then waits vmcnt(0) for it, which
// in the loader would drain every DMA in flight.
typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
__device__ __forceinline__ int vload(const int* p) { return *(volatile const lds_i32*)p; }
__device__ __forceinline__ void vstore(int* p, const int v) { *(volatile lds_i32*)p = v; }
__device__ __forceinline__ int lds_add(int* p, const int v) {
    return __hip_atomic_fetch_add((lds_i32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_max_u64(unsigned long long* p, const unsigned long long v) {
    __hip_atomic_fetch_max((lds_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// timeout: err[0] = 1; the first wave to time out also leaves err[2..5] = {code, workgroup,
// wave, awaited value} (codes: SE_W_*)
enum { SE_W_FREE = 1, SE_W_FULL = 2, SE_W_SWEEP = 3, SE_W_BAR = 4, SE_W_QCNT = 5, SE_W_CAND = 6, SE_W_TILE = 7 };
__device__ __forceinline__ void se_fail(const SeArgs& a, SeCtl* c, const int code, const int value) {
    int expect = 0;
    if (__hip_atomic_compare_exchange_strong(a.err + 2, &expect, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store(a.err + 3, (int)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.err + 4, (int)threadIdx.x >> 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.err + 5, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    vstore(&c->abort, 1);
}
// one bounded spin step: false when the wave must leave (timeout, or another wave aborted)
struct SeSpin {
    uint64_t t0;
    unsigned n = 0;
    int code, value;
    __device__ SeSpin(const int code_, const int value_) : t0(se_now()), code(code_), value(value_) {}
    __device__ __forceinline__ bool step(const SeArgs& a, SeCtl* c) {
        if (vload(&c->abort)) return false;
        if ((++n & 255) == 0) {
            if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { vstore(&c->abort, 1); return false; }
            if (se_now() - t0 > SE_TIMEOUT) { se_fail(a, c, code, value); return false; }
        }
        return true;
    }
};
// wait until an LDS word reaches v (>=)
__device__ __forceinline__ bool se_lds_wait_ge(const SeArgs& a, SeCtl* c, const int* w, const int v, const int code) {
    if (vload(w) >= v) return true;
    SeSpin sp(code, v);
    while (vload(w) < v) {
        __builtin_amdgcn_s_sleep(0);
        if (!sp.step(a, c)) return false;
    }
    return true;
}
__device__ __forceinline__ bool se_lds_wait_eq(const SeArgs& a, SeCtl* c, const int* w, const int v, const int code) {
    if (vload(w) == v) return true;
    SeSpin sp(code, v);
    while (vload(w) != v) {
        __builtin_amdgcn_s_sleep(0);
        if (!sp.step(a, c)) return false;
    }
    return true;
}

// barrier of the SE_NW consumer waves (the loader never joins): LDS arrival counter
__device__ __forceinline__ bool se_cbar(const SeArgs& a, SeCtl* c, int& gen, int* counter, const int members) {
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
    gen++;
    if (se_lane() == 0) lds_add(counter, 1);
    return se_lds_wait_ge(a, c, counter, gen * members, SE_W_BAR);
}

// 64-bit granule {tag (high), value (low)}: one 8-byte sc1 store
__device__ __forceinline__ void se_put(unsigned long long* g, const unsigned tag, const float v) {
    __hip_atomic_store(g, ((unsigned long long)tag << 32) | __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// ---- loader: global_load_lds_dwordx4 (hipcc does not model the LDS write or its vmcnt) ------
__device__ __forceinline__ void se_glds(const void* gsrc, const uint32_t lds_byte) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_byte)
        : "memory");
}
// wait until at most n (wave-uniform, 0..48) of this wave's vector-memory ops are outstanding
#define SE_VM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void se_vmcnt_le(const int n) {
    switch (n) {
        SE_VM(0) SE_VM(1) SE_VM(2) SE_VM(3) SE_VM(4) SE_VM(5) SE_VM(6) SE_VM(7) SE_VM(8) SE_VM(9) SE_VM(10)
        SE_VM(11) SE_VM(12) SE_VM(13) SE_VM(14) SE_VM(15) SE_VM(16) SE_VM(17) SE_VM(18) SE_VM(19) SE_VM(20)
        SE_VM(21) SE_VM(22) SE_VM(23) SE_VM(24) SE_VM(25) SE_VM(26) SE_VM(27) SE_VM(28) SE_VM(29) SE_VM(30)
        SE_VM(31) SE_VM(32) SE_VM(33) SE_VM(34) SE_VM(35) SE_VM(36) SE_VM(37) SE_VM(38) SE_VM(39) SE_VM(40)
        SE_VM(41) SE_VM(42) SE_VM(43) SE_VM(44) SE_VM(45) SE_VM(46) SE_VM(47) SE_VM(48)
        default: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    }
}
#undef SE_VM

// ---- the schedule (identical in the loader and the consumers) --------------------------------
struct SeMat {
    const char* w;
    size_t rb;   // row bytes (multiple of 1024)
    int rows;
    int nk;      // K-steps = rb / 1024
};
template <int ESZ, int ESZC>
__device__ __forceinline__ SeMat se_mat(const SeArgs& a, const int l, const int ph) {
    SeMat m;
    if (ph == SE_CLS) {
        m.w = (const char*)a.wcls; m.rb = (size_t)a.dim * ESZC; m.rows = a.vocab;
    } else {
        const SeLayer& ly = a.layers[l];
        switch (ph) {
            case SE_QKV: m.w = (const char*)ly.wqkv; m.rb = (size_t)a.dim * ESZ; m.rows = a.q_dim + 2 * a.kv_dim; break;
            case SE_WO: m.w = (const char*)ly.wo; m.rb = (size_t)a.q_dim * ESZ; m.rows = a.dim; break;
            case SE_W13: m.w = (const char*)ly.w13; m.rb = (size_t)a.dim * ESZ; m.rows = 2 * a.hidden; break;
            default: m.w = (const char*)ly.w2; m.rb = (size_t)a.hidden * ESZ; m.rows = a.dim; break;
        }
    }
    m.nk = (int)(m.rb >> 10);
    return m;
}
// CU b's rows of a matrix with R rows: balanced blocks of row pairs
__device__ __forceinline__ void se_part(const int R, const int nblk, const int b, int& r0, int& r1) {
    const long long U = (R + 1) >> 1;
    r0 = min(R, (int)(2 * (U * b / nblk)));
    r1 = min(R, (int)(2 * (U * (b + 1) / nblk)));
}
__device__ __forceinline__ int se_ntiles(const int n) { return (n + 15) >> 4; }
__device__ __forceinline__ void se_tile(const int r0, const int r1, const int nt, const int i, int& t0, int& t1) {
    const int U = (r1 - r0 + 1) >> 1;
    t0 = r0 + 2 * (U * i / nt);
    t1 = min(r1, r0 + 2 * (U * (i + 1) / nt));
}
__device__ __forceinline__ bool se_want_logits(const SeArgs& a, const int t, const int n_tok) {
    return (t == n_tok - 1) ? a.logits_last != 0 : (t >= a.n_prompt - 1);
}

// ---- the loader wave ----------------------------------------------------------------------------
// Streams the schedule's slots in order.  A slot is published (full[] = its sequence number)
// once a counted vmcnt shows its pieces landed.  Up to SE_DEPTH + 1 slots are in flight (the
// 64th piece waits in hardware for the first one: vmcnt holds 63); while a consumer wave
// gathers a hand-off (c->gath) only one, so the gather's loads do not queue behind the DMA
// (MI355X_MICROARCH.md price list: gather-pass).  The FIFO lives in named scalars: a
// dynamically indexed array would go to scratch, and the compiler's vmcnt(0) for a scratch
// load would drain every DMA in flight.
template <int DT, int DTC>
__device__ __forceinline__ void se_loader(const SeArgs& a, char* ring, SeCtl* c, const int li) {
    constexpr int ESZ = 16 / WDec<DT>::E, ESZC = 16 / WDec<DTC>::E;
    static_assert(SE_DEPTH == 3, "the in-flight FIFO below holds four slots");
    const uint32_t ring_lds = (uint32_t)(uintptr_t)ring;
    const int ns = a.nslots;
    const int nblk = gridDim.x, b = blockIdx.x;
    const int n_tok = a.n_prompt + a.n_gen;
    int seq = 0, slot = 0;  // next sequence number and its slot
    // in flight, oldest first: sequence numbers and piece counts
    int s0 = 0, s1 = 0, s2 = 0, s3 = 0, n0 = 0, n1 = 0, n2 = 0, n3 = 0, nfl = 0;
    uint64_t i0 = 0, i1 = 0, i2 = 0, i3 = 0;             // debug: issue times of the FIFO entries
    uint64_t tr_lat = 0, tr_cnt = 0, tr_blk = 0;
    auto publish_oldest = [&]() {
        const bool stamp = a.trace && !(a.debug & 8);
        const uint64_t tb = stamp ? se_now() : 0;
        se_vmcnt_le((nfl > 1 ? n1 : 0) + (nfl > 2 ? n2 : 0) + (nfl > 3 ? n3 : 0));
        vstore(&c->full[s0 % ns], s0);
        if (stamp) {
            const uint64_t now = se_now();
            tr_blk += now - tb;
            tr_lat += now - i0;
            tr_cnt++;
        }
        s0 = s1; n0 = n1; i0 = i1; s1 = s2; n1 = n2; i1 = i2; s2 = s3; n2 = n3; i2 = i3;
        nfl--;
    };
    auto publish_all = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (nfl > 0) vstore(&c->full[s0 % ns], s0);
        if (nfl > 1) vstore(&c->full[s1 % ns], s1);
        if (nfl > 2) vstore(&c->full[s2 % ns], s2);
        if (nfl > 3) vstore(&c->full[s3 % ns], s3);
        nfl = 0;
    };
    bool go = true;
    uint64_t tr_wait = 0;
    const int trc = a.trace ? se_trace_cu(b, nblk) : -1;
    for (int t = 0; t < n_tok && go; t++) {
        const bool logits = se_want_logits(a, t, n_tok);
        const int n_ph = a.n_layers * 4 + (logits ? 1 : 0);
        unsigned long long* tr_first =
            (trc >= 0 && t == n_tok - 1 && li == 0) ? a.trace + SE_TR_CU * nblk + trc * (4 * a.n_layers + 1) * SE_TR_PH : nullptr;
        for (int q = 0; q < n_ph && go; q++) {
            const int l = q >> 2, ph = q < a.n_layers * 4 ? (q & 3) : SE_CLS;
            const SeMat m = se_mat<ESZ, ESZC>(a, l, ph);
            int r0, r1;
            se_part(m.rows, nblk, b, r0, r1);
            const int nt = se_ntiles(r1 - r0);
            for (int i = 0; i < nt && go; i++) {
                int t0, t1;
                se_tile(r0, r1, nt, i, t0, t1);
                const int TH = t1 - t0;
                const char* src = m.w + (size_t)t0 * m.rb + se_lane() * 16;
                const int rot = a.rotate ? b % m.nk : 0;
                for (int kk = 0; kk < m.nk; kk++) {
                    const int ks = kk + rot < m.nk ? kk + rot : kk + rot - m.nk;
                    if (tr_first && kk == 0 && i == 0) tr_first[q * SE_TR_PH + 3] = se_now();
                    if (seq % SE_NL != li) {  // another loader wave's slot
                        seq++;
                        slot = slot + 1 == ns ? 0 : slot + 1;
                        continue;
                    }
                    // every consumer wave is gathering a hand-off: issue nothing (their loads
                    // would queue behind the DMA, MI355X_MICROARCH.md gather-pass); the ring
                    // covers the pause
                    if (vload(&c->gath) >= SE_NW) {
                        publish_all();
                        SeSpin sp(SE_W_FREE, -seq);
                        while (vload(&c->gath) >= SE_NW) {
                            if (vload(&c->ndone) >= SE_NW || !sp.step(a, c)) { go = false; break; }
                            __builtin_amdgcn_s_sleep(1);
                        }
                        if (!go) break;
                    }
                    // the slot's previous occupant (seq - ns) must have been released
                    if (seq >= ns && vload(&c->free_[slot]) != seq - ns) {
                        const uint64_t tw = a.trace ? se_now() : 0;
                        publish_all();  // ring full: whatever is in flight may as well be published
                        SeSpin sp(SE_W_FREE, seq);
                        while (vload(&c->free_[slot]) != seq - ns) {
                            if (vload(&c->ndone) >= SE_NW || !sp.step(a, c)) { go = false; break; }
                            __builtin_amdgcn_s_sleep(1);
                        }
                        if (a.trace) tr_wait += se_now() - tw;
                        if (!go) break;
                    }
                    const uint32_t dst = ring_lds + (uint32_t)slot * SE_SLOT;
                    for (int p = 0; p < TH; p++)
                        se_glds(src + (size_t)p * m.rb + (size_t)ks * 1024, __builtin_amdgcn_readfirstlane(dst + p * 1024));
                    const uint64_t ti = (a.trace && !(a.debug & 8)) ? se_now() : 0;
                    if (nfl == 0) { s0 = seq; n0 = TH; i0 = ti; }
                    else if (nfl == 1) { s1 = seq; n1 = TH; i1 = ti; }
                    else if (nfl == 2) { s2 = seq; n2 = TH; i2 = ti; }
                    else { s3 = seq; n3 = TH; i3 = ti; }
                    nfl++;
                    seq++;
                    slot = slot + 1 == ns ? 0 : slot + 1;
                    while (nfl > SE_DEPTH) publish_oldest();
                    // room for the next slot: at most SE_MAXP pieces in flight (vmcnt holds 63)
                    while (nfl > 0 && n0 + (nfl > 1 ? n1 : 0) + (nfl > 2 ? n2 : 0) + (nfl > 3 ? n3 : 0) + 16 > SE_MAXP)
                        publish_oldest();
                }
            }
        }
        if (vload(&c->ndone) >= SE_NW || vload(&c->abort)) go = false;
    }
    // every DMA must land before the wave (and its workgroup's LDS) goes away; what is still
    // in flight is published (a consumer may wait for it)
    publish_all();
    if (a.trace && se_lane() == 0 && li == 0) {
        a.trace[SE_TR_CU * b + 0] = tr_wait;
        a.trace[SE_TR_CU * b + 4] = tr_lat;
        a.trace[SE_TR_CU * b + 5] = tr_cnt;
        a.trace[SE_TR_CU * b + 6] = tr_blk;
    }
}

// ---- consumer waves ---------------------------------------------------------------------------
struct SeState {
    int cw;        // consumer wave index
    int seq = 0;   // sequence number of the next tile's K-step 0
    int tile = 0;  // global tile counter (partial-sum buffer parity)
    int cgen = 0;  // consumer barrier generation
    int agen = 0;  // attention barrier generation
    uint64_t w_full = 0, w_acq = 0, w_att = 0;  // debug: ticks waiting (a.trace)
};

// per-token scalars the epilogues need
struct SeTok {
    int t, pos, kv_pos;
    int own0;         // first residual row owned by this CU
    int cls_nt;       // lm_head tiles of this CU
    unsigned xtag0;   // granule tag of x before layer 0 (x after layer l's Wo / W2: + 2l+1 / + 2l+2)
    unsigned ltag0;   // tag of the attention output / hb of layer 0 (layer l: + l)
    unsigned ctag;    // tag of this token's argmax candidates (1..32767)
};

// this wave's K-step j of a row: ks = cw + j * SE_NW
__device__ __forceinline__ int se_ks(const SeState& st, const int j) { return st.cw + j * SE_NW; }

// Last arriver's view of the combined tile: row r = sum over participating waves, wave order.
__device__ __forceinline__ float se_sum(const SeCtl* c, const int buf, const int P, const int r) {
    float s = 0.f;
    for (int w = 0; w < P; w++) s += c->part[buf][w][r];
    return s;
}

// The epilogue of one combined tile, rows [row0, row0 + TH) of phase ph (last-arriving wave).
template <int HD, int QPK>
__device__ __forceinline__ void se_epilogue(const SeArgs& a, SeCtl* c, const SeTok& tk, const int l, const int ph,
                                            const int buf, const int P, const int row0, const int TH) {
    const int lane = se_lane();
    switch (ph) {
        case SE_QKV: {  // clip, rope, q / fp16 K,V row at kv_pos (src/infer.cpp:392-414)
            const SeLayer& ly = a.layers[l];
            if (2 * lane < TH) {
                const int row = row0 + 2 * lane;
                float v0 = clipf(se_sum(c, buf, P, 2 * lane), a.qkv_clip);
                float v1 = clipf(se_sum(c, buf, P, 2 * lane + 1), a.qkv_clip);
                if (row < a.q_dim) {
                    rope_pair(v0, v1, row, HD, tk.pos, a.rope_freq);
                    __hip_atomic_store((unsigned long long*)(a.q + row),
                                       ((unsigned long long)__builtin_bit_cast(uint32_t, v1) << 32) |
                                           __builtin_bit_cast(uint32_t, v0),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    const bool isk = row < a.q_dim + a.kv_dim;
                    const int kr = isk ? row - a.q_dim : row - a.q_dim - a.kv_dim;
                    if (isk) rope_pair(v0, v1, kr, HD, tk.pos, a.rope_freq);
                    uint16_t* dst = (isk ? ly.kc : ly.vc) + (size_t)tk.kv_pos * a.kv_dim + kr;
                    st_sc1_u32(dst, (uint32_t)f32_to_f16_bits(v0) | ((uint32_t)f32_to_f16_bits(v1) << 16));
                }
            }
            // every row stored (this wave only), then each KV head's rows counted
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                int g_prev = -1, n_prev = 0;
                for (int r = row0; r < row0 + TH; r++) {
                    const int gg = r < a.q_dim ? r / (QPK * HD) : ((r - a.q_dim) % a.kv_dim) / HD;
                    if (gg != g_prev) {
                        if (n_prev)
                            __hip_atomic_fetch_add(a.qcnt + (size_t)l * a.n_kv_heads + g_prev, (unsigned)n_prev,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        g_prev = gg;
                        n_prev = 0;
                    }
                    n_prev++;
                }
                if (n_prev)
                    __hip_atomic_fetch_add(a.qcnt + (size_t)l * a.n_kv_heads + g_prev, (unsigned)n_prev,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
        case SE_WO:
        case SE_W2: {  // x += W . (src/infer.cpp:447-452, 490-494); x rows of this CU in LDS
            if (lane < TH) {
                const int row = row0 + lane;
                const float v = c->xown[row - tk.own0] + se_sum(c, buf, P, lane);
                c->xown[row - tk.own0] = v;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // xown before anyone sees x
                se_put(a.xg + row, tk.xtag0 + 2 * l + (ph == SE_WO ? 1 : 2), v);
            }
            break;
        }
        case SE_W13: {  // hb = act(W1 x) * (W3 x) (src/infer.cpp:468-488), rows interleaved
            if (2 * lane < TH)
                se_put(a.hg + ((row0 >> 1) + lane), tk.ltag0 + l,
                       act_fn(a.act, se_sum(c, buf, P, 2 * lane)) * se_sum(c, buf, P, 2 * lane + 1));
            break;
        }
        default: {  // lm_head: logits and Sampler::sample_argmax candidates (src/sampler.cpp:19-30)
            // only logits > FLT_MIN compete, the first maximum wins:
            // key = orderable logit << 32 | (0x1FFFF - index) << 15 | tag
            unsigned long long key = 0;
            if (lane < TH) {
                const int row = row0 + lane;
                const float v = se_sum(c, buf, P, lane);
                a.logits[row] = v;
                if (v > FLT_MIN) {
                    uint32_t u = __builtin_bit_cast(uint32_t, v);
                    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
                    key = ((unsigned long long)u << 32) | ((unsigned long long)(0x1FFFF - row) << 15);
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long other = __shfl_xor(key, o, 64);
                key = other > key ? other : key;
            }
            if (lane == 0) {
                lds_max_u64(&c->best, key);
                const int done = lds_add(&c->cls_tiles, 1) + 1;
                if (done == tk.cls_nt) {
                    const unsigned long long bk = c->best;
                    c->best = 0;
                    c->cls_tiles = 0;
                    __hip_atomic_store(a.cg + blockIdx.x, bk | tk.ctag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            break;
        }
    }
}

// Tile end: reduce the wave's 16 per-lane accumulators over the lanes, meet the other waves'
// partials in LDS; the last wave to arrive runs the epilogue and marks the buffer free.
template <int HD, int QPK>
__device__ __forceinline__ bool se_tile_end(const SeArgs& a, SeCtl* c, SeState& st, const SeTok& tk, const int l,
                                            const int ph, float (&acc)[16], const int P, const int row0,
                                            const int TH) {
    rows_reduce_scatter<16>(acc);
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = group_reduce<16>(acc[k]);
    const int lane = se_lane();
    const int rg = lane >> 4;
    const int base = (rg & 1) * 8 + (rg >> 1) * 4;  // the 4 rows this 16-lane group holds
    const int buf = st.tile & 1;
    if (!se_lds_wait_ge(a, c, &c->tdone[buf], st.tile >> 1, SE_W_TILE)) return false;
    if ((lane & 15) == 0) *(float4*)&c->part[buf][st.cw][base] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) old = lds_add(&c->tcnt[buf], 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old == P - 1) {
        if (lane == 0) vstore(&c->tcnt[buf], 0);
        se_epilogue<HD, QPK>(a, c, tk, l, ph, buf, P, row0, TH);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) vstore(&c->tdone[buf], (st.tile >> 1) + 1);
    }
    return true;
}

// acc += dot(16 bytes of weights, x[0, E)), fp32 accumulation in element order.  f16: the
// weights feed v_fma_mix_f32 directly (f16 -> f32 is exact, one rounding per fma, as fmaf on
// the converted value), so no converted copies of the 16 pieces are held in registers.
template <int DT>
__device__ __forceinline__ float se_dot16(const u32x4 w, const float* x, float acc) {
    if constexpr (DT == XH_F16) {
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(ww[i]), "v"(x[2 * i]));
            asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(ww[i]), "v"(x[2 * i + 1]));
        }
        return acc;
    } else {
        constexpr int E = WDec<DT>::E;
        float f[E];
        WDec<DT>::dec(w, f);
#pragma unroll
        for (int e = 0; e < E; e++) acc = fmaf(f[e], x[e], acc);
        return acc;
    }
}

// xr rotated left by E floats (K-step j + 1 moves to j)
template <int E>
__device__ __forceinline__ void se_rotate(float (&xr)[SE_XF]) {
    float keep[E];
#pragma unroll
    for (int e = 0; e < E; e++) keep[e] = xr[e];
#pragma unroll
    for (int k = 0; k + E < SE_XF; k++) xr[k] = xr[k + E];
#pragma unroll
    for (int e = 0; e < E; e++) xr[SE_XF - E + e] = keep[e];
}

// All tiles of rows [r0, r1) of matrix m.  xr holds this wave's activations: K-step j at
// xr[j * E, +E).  The loader streams a tile's K-steps from rot = CU % nk on (so the CUs do
// not all read the same column offsets at once); a wave takes its own K-steps in that order
// (j from jstart, wrapping), holding the current one in xr[0, E): xr is rotated by E per
// K-step, and by jstart once per phase, instead of unrolling the K-step loop.
template <int DT, int HD, int QPK>
__device__ __forceinline__ bool se_matrix(const SeArgs& a, SeCtl* c, const char* ring, SeState& st, const SeTok& tk,
                                          const int l, const int ph, const SeMat& m, const int r0, const int r1,
                                          float (&xr)[SE_XF]) {
    constexpr int E = WDec<DT>::E;
    constexpr int MAXJ = SE_XF / E;
    const int nt = se_ntiles(r1 - r0);
    const int P = min(SE_NW, m.nk);
    const int lane = se_lane();
    const int ns = a.nslots;
    const int rot = a.rotate ? (int)blockIdx.x % m.nk : 0;  // the loader's first K-step (se_loader)
    int jstart = 0;                                         // this wave's K-steps below rot
    while (jstart < MAXJ && se_ks(st, jstart) < min(rot, m.nk)) jstart++;
    if (st.cw < P && nt > 0)
        for (int r = 0; r < jstart; r++) se_rotate<E>(xr);
    for (int i = 0; i < nt; i++) {
        int t0, t1;
        se_tile(r0, r1, nt, i, t0, t1);
        if (st.cw < P) {
            float acc[16];
#pragma unroll
            for (int p = 0; p < 16; p++) acc[p] = 0.f;
#pragma unroll 1
            for (int jj = 0; jj < MAXJ; jj++) {
                const int j = jj + jstart < MAXJ ? jj + jstart : jj + jstart - MAXJ;
                const int ks = se_ks(st, j);
                if (ks < m.nk) {
                    const int s = st.seq + (ks >= rot ? ks - rot : ks - rot + m.nk);
                    const int slot = s % ns;
                    if (a.trace && vload(&c->full[slot]) != s) {
                        const uint64_t tw = se_now();
                        if (!se_lds_wait_eq(a, c, &c->full[slot], s, SE_W_FULL)) return false;
                        st.w_full += se_now() - tw;
                    } else if (!se_lds_wait_eq(a, c, &c->full[slot], s, SE_W_FULL)) {
                        return false;
                    }
                    asm volatile("" ::: "memory");
                    const char* sp = ring + slot * SE_SLOT + lane * 16;
                    u32x4 w[16];
#pragma unroll
                    for (int p = 0; p < 16; p++) w[p] = *(const u32x4*)(sp + p * 1024);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) vstore(&c->free_[slot], s);
                    if (!(a.debug & 1)) {
#pragma unroll
                        for (int p = 0; p < 16; p++) acc[p] = se_dot16<DT>(w[p], xr, acc[p]);
                    } else {
                        acc[0] += __builtin_bit_cast(float, w[0].x & 1u);
                    }
                }
                se_rotate<E>(xr);
            }
            if (!(a.debug & 4) && !se_tile_end<HD, QPK>(a, c, st, tk, l, ph, acc, P, t0, t1 - t0)) return false;
        }
        st.seq += m.nk;
        st.tile++;
    }
    return true;
}

// Activations of this wave's K-steps from a granule buffer (tags must equal `tag`); every
// entry of xr is written (0 where the wave has no K-step).
template <int E>
__device__ __forceinline__ bool se_sweep(const SeArgs& a, SeCtl* c, const SeState& st, const unsigned long long* g,
                                         const int nk, const unsigned tag, float (&xr)[SE_XF]) {
    constexpr int MAXJ = SE_XF / E;
    const int lane = se_lane();
    SeSpin sp(SE_W_SWEEP, (int)tag);
    if (lane == 0) lds_add(&c->gath, 1);
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < MAXJ; j++) {
            const int ks = se_ks(st, j);
            const bool act = ks < nk;
            const uint32_t off = (uint32_t)((act ? ks : 0) * 64 * E + lane * E) * 8u;
#pragma unroll
            for (int e = 0; e < E; e += 2) {
                u32x4 u = {0u, tag, 0u, tag};
                if (act) u = ld_sc1_x4(g, off + e * 8);
                xr[j * E + e] = bits_f32(u.x);
                xr[j * E + e + 1] = bits_f32(u.z);
                ok = ok && u.y == tag && u.w == tag;
            }
        }
        if (__all(ok) || (a.debug & 2)) break;
        __builtin_amdgcn_s_sleep(1);
        if (!sp.step(a, c)) return false;
    }
    if (lane == 0) lds_add(&c->gath, -1);
    return true;
}

// This wave's norm weights at its K-steps of an n-vector (requested before the hand-off wait
// so their round trip overlaps it).
template <int E>
__device__ __forceinline__ void se_load_norm(const SeArgs& a, const SeState& st, const int n, const void* normw,
                                             float (&nw)[SE_XF]) {
    constexpr int MAXJ = SE_XF / E;
    const int nk = n / (64 * E);
    const int lane = se_lane();
#pragma unroll
    for (int j = 0; j < MAXJ; j++) {
        const int ks = se_ks(st, j);
        const bool act = ks < nk;
#pragma unroll
        for (int e = 0; e < E; e += 4) {
            float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (act) w4 = load_norm4(normw, a.norm_dt, (ks * 64 * E + lane * E + e) >> 2);
            nw[j * E + e] = w4.x; nw[j * E + e + 1] = w4.y; nw[j * E + e + 2] = w4.z; nw[j * E + e + 3] = w4.w;
        }
    }
}

// rmsnorm of the vector whose slices the waves hold: every consumer wave's partial sum of
// squares meets in LDS (one consumer barrier), then xr *= scale * w (src/infer.cpp:224-236)
template <int E>
__device__ __forceinline__ bool se_rmsnorm(const SeArgs& a, SeCtl* c, SeState& st, const int n, const float (&nw)[SE_XF],
                                           float (&xr)[SE_XF]) {
    const int lane = se_lane();
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < SE_XF; j++) ss = fmaf(xr[j], xr[j], ss);
    ss = wave_sum(ss);
    // double-buffered by barrier parity: a wave can only rewrite this buffer after the next
    // barrier, which every wave reaches after its reads below
    const int par = st.cgen & 1;
    if (lane == 0) c->ssp[par][st.cw] = ss;
    if (!se_cbar(a, c, st.cgen, &c->cbar, SE_NW)) return false;
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < SE_NW; w++) tot += c->ssp[par][w];
    const float scale = 1.0f / sqrtf(tot / (float)n + a.eps);
#pragma unroll
    for (int j = 0; j < SE_XF; j++) xr[j] = xr[j] * scale * nw[j];
    return true;
}

// This wave's slices of the embedding row (src/infer.cpp:553-602), 0 where it has none.
template <int E>
__device__ __forceinline__ void se_embed(const SeArgs& a, const SeState& st, const int token, float (&xr)[SE_XF]) {
    constexpr int MAXJ = SE_XF / E;
    const int nk = a.dim / (64 * E);
    const int lane = se_lane();
#pragma unroll
    for (int j = 0; j < MAXJ; j++) {
        const int ks = se_ks(st, j);
#pragma unroll
        for (int e = 0; e < E; e++)
            xr[j * E + e] = ks < nk ? dec1(a.embed_dt, a.embed, (size_t)token * a.dim + ks * 64 * E + lane * E + e) : 0.f;
    }
}

// ---- attention (consumer waves 0..SE_NA-1 of the CUs that own a (KV head, split) item) ---------
// attn(q_h, K, V) over slots [t0, t1) of KV head g, src/infer.cpp:325-359 (scores / sqrtf(hd),
// max-subtracted softmax with expf, sum of p * v), as an online softmax per wave; the waves'
// (m, l, o) meet in LDS and wave 0 finishes: one split publishes o / l, several publish
// partials and the last split of the head merges them.
template <int HD, int QPK>
__device__ __forceinline__ bool se_attention(const SeArgs& a, SeCtl* c, float* att, SeState& st, const int l, const int t,
                                          const int g, const int s, const int S, const int T, const int kv_sink,
                                          const int kv_len, unsigned long long* trq) {
    constexpr int LPR = HD / 8;       // lanes per K/V row (8 elements each)
    constexpr int RPW = 64 / LPR;     // rows per wave-instruction
    constexpr int NB = 4;             // row groups per batch
    constexpr int NO = QPK * HD;
    const SeLayer& ly = a.layers[l];
    const int lane = se_lane(), w = st.cw;
    const int sub = lane % LPR, rr = lane / LPR;
    // q, k, v of this head, this token: every producer's rows counted
    {
        if (lane == 0) lds_add(&c->gath, 1);
        const unsigned target = (unsigned)(t + 1) * (unsigned)(NO + 2 * HD);
        unsigned* cnt = a.qcnt + (size_t)l * a.n_kv_heads + g;
        SeSpin sp(SE_W_QCNT, (int)target);
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (!sp.step(a, c)) return false;
        }
        if (trq) trq[4] = se_now();
    }
    const uint32_t rowb = (uint32_t)a.kv_dim * 2;
    const uint32_t colb = (uint32_t)((g * HD + sub * 8) * 2);
    // StreamingLLM sink re-rotation (src/infer.cpp:421-431) of this head's columns, split 0
    if (kv_sink && s == 0) {
        if (w == 0) {
            for (int r = 0; r < kv_sink; r++) {
                for (int p = lane; p < HD / 2; p += 64) {
                    const int i = g * HD + 2 * p;
                    uint16_t* kp = ly.kc + (size_t)r * a.kv_dim + i;
                    const uint32_t pr = ld_sc1_u32(kp);
                    const float k0 = f16_bits_to_f32((uint16_t)(pr & 0xffffu)), k1 = f16_bits_to_f32((uint16_t)(pr >> 16));
                    const float fcr = a.sink_cos[p], fci = a.sink_sin[p];
                    st_sc1_u32(kp, (uint32_t)f32_to_f16_bits(k0 * fcr - k1 * fci) |
                                       ((uint32_t)f32_to_f16_bits(k0 * fci + k1 * fcr) << 16));
                }
            }
        }
        if (!se_cbar(a, c, st.agen, &c->abar, SE_NA)) return false;
    }
    float qv[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++) {
        const float* qp = a.q + (size_t)(g * QPK + h) * HD + sub * 8;
        const u32x4 q0 = ld_sc1_x4(qp, 0), q1 = ld_sc1_x4(qp, 16);
        qv[h][0] = bits_f32(q0.x); qv[h][1] = bits_f32(q0.y); qv[h][2] = bits_f32(q0.z); qv[h][3] = bits_f32(q0.w);
        qv[h][4] = bits_f32(q1.x); qv[h][5] = bits_f32(q1.y); qv[h][6] = bits_f32(q1.z); qv[h][7] = bits_f32(q1.w);
    }
    const float scale = 1.0f / sqrtf((float)HD);
    const int t0 = s * T, t1 = min(kv_len, t0 + T);
    float M[QPK], lsum[QPK], o[QPK][8];
#pragma unroll
    for (int h = 0; h < QPK; h++) {
        M[h] = -FLT_MAX;
        lsum[h] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; i++) o[h][i] = 0.f;
    }
    // rows of this wave: t0 + (w + SE_NA * (k * NB + b)) * RPW + rr
    for (int base = t0 + w * RPW; base < t1; base += SE_NA * RPW * NB) {
        u32x4 kk[NB], vv[NB];
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            const int row = base + bb * SE_NA * RPW + rr;
            const int rc = min(row, t1 - 1);
            kk[bb] = ld_sc1_x4(ly.kc, (uint32_t)rc * rowb + colb);
            vv[bb] = ld_sc1_x4(ly.vc, (uint32_t)rc * rowb + colb);
        }
        float sc[QPK][NB];
        if (trq && base == t0 + w * RPW) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            trq[5] = se_now();
        }
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            const int row = base + bb * SE_NA * RPW + rr;
            float kf[8];
            WDec<XH_F16>::dec(kk[bb], kf);
#pragma unroll
            for (int h = 0; h < QPK; h++) {
                float pr = 0.f;
#pragma unroll
                for (int i = 0; i < 8; i++) pr = fmaf(qv[h][i], kf[i], pr);
                pr = group_reduce<LPR>(pr);
                sc[h][bb] = row < t1 ? pr * scale : -FLT_MAX;
            }
        }
#pragma unroll
        for (int h = 0; h < QPK; h++) {
            float mb = sc[h][0];
#pragma unroll
            for (int bb = 1; bb < NB; bb++) mb = fmaxf(mb, sc[h][bb]);
            mb = wave_max(mb);
            const float Mn = fmaxf(M[h], mb);
            const float f = expf(M[h] - Mn);  // 0 on the first batch (M = -FLT_MAX)
            M[h] = Mn;
            lsum[h] *= f;
#pragma unroll
            for (int i = 0; i < 8; i++) o[h][i] *= f;
        }
#pragma unroll
        for (int bb = 0; bb < NB; bb++) {
            const int row = base + bb * SE_NA * RPW + rr;
            float vf[8];
            WDec<XH_F16>::dec(vv[bb], vf);
#pragma unroll
            for (int h = 0; h < QPK; h++) {
                const float p = row < t1 ? expf(sc[h][bb] - M[h]) : 0.f;
                lsum[h] += p;
#pragma unroll
                for (int i = 0; i < 8; i++) o[h][i] = fmaf(p, vf[i], o[h][i]);
            }
        }
    }
    // over the row groups of the wave (lanes sub, sub + LPR, ...)
#pragma unroll
    for (int h = 0; h < QPK; h++) {
        lsum[h] = strided_reduce<LPR>(lsum[h]);
#pragma unroll
        for (int i = 0; i < 8; i++) o[h][i] = strided_reduce<LPR>(o[h][i]);
    }
    // this wave's (m, l, o) -> LDS; a wave with no rows has m = -FLT_MAX, l = 0
    float* aw = att + (size_t)w * (NO + 2 * QPK);
    if (lane < LPR) {
#pragma unroll
        for (int h = 0; h < QPK; h++) {
            *(float4*)&aw[h * HD + sub * 8] = make_float4(o[h][0], o[h][1], o[h][2], o[h][3]);
            *(float4*)&aw[h * HD + sub * 8 + 4] = make_float4(o[h][4], o[h][5], o[h][6], o[h][7]);
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int h = 0; h < QPK; h++) { aw[NO + 2 * h] = M[h]; aw[NO + 2 * h + 1] = lsum[h]; }
    }
    if (lane == 0) lds_add(&c->gath, -1);
    if (!se_cbar(a, c, st.agen, &c->abar, SE_NA)) return false;
    if (w != 0) return true;
    // wave 0: merge the SE_NA waves (max, then rescaled sums, wave order)
    const unsigned tag = (unsigned)(t * a.n_layers + l + 1);
    for (int idx = lane; idx < NO; idx += 64) {
        const int h = idx / HD;
        float Mx = -FLT_MAX;
#pragma unroll
        for (int v = 0; v < SE_NA; v++) Mx = fmaxf(Mx, att[v * (NO + 2 * QPK) + NO + 2 * h]);
        float num = 0.f, den = 0.f;
#pragma unroll
        for (int v = 0; v < SE_NA; v++) {
            const float* av = att + v * (NO + 2 * QPK);
            const float f = expf(av[NO + 2 * h] - Mx);
            den = fmaf(f, av[NO + 2 * h + 1], den);
            num = fmaf(f, av[idx], num);
        }
        if (S == 1) {
            se_put(a.ag + (size_t)g * NO + idx, tag, num / den);
        } else {
            float* po = a.part_o + ((size_t)s * a.n_heads + g * QPK) * HD;
            st_sc1_f(po + idx, num);
            if (idx % HD == 0) {
                float* pml = a.part_ml + ((size_t)s * a.n_heads + g * QPK + h) * 2;
                st_sc1_f(pml, Mx);
                st_sc1_f(pml + 1, den);
            }
        }
    }
    if (trq) trq[6] = se_now();
    if (S == 1) return true;
    // split partials: drained, then the head's ticket; the last split merges
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(a.tickets + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    if (ticket != S - 1) return true;
    if (lane == 0) __hip_atomic_store(a.tickets + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int idx = lane; idx < NO; idx += 64) {
        const int h = idx / HD;
        float Mx = -FLT_MAX;
        for (int j = 0; j < S; j++) Mx = fmaxf(Mx, ld_sc1_f(a.part_ml + ((size_t)j * a.n_heads + g * QPK + h) * 2));
        float num = 0.f, den = 0.f;
        for (int j = 0; j < S; j++) {
            const float* pml = a.part_ml + ((size_t)j * a.n_heads + g * QPK + h) * 2;
            const float f = expf(ld_sc1_f(pml) - Mx);
            den = fmaf(f, ld_sc1_f(pml + 1), den);
            num = fmaf(f, ld_sc1_f(a.part_o + ((size_t)j * a.n_heads + g * QPK) * HD + idx), num);
        }
        se_put(a.ag + (size_t)g * NO + idx, tag, num / den);
    }
    return true;
}

// ---- the kernel -----------------------------------------------------------------------------
template <int DT, int DTC, int HD, int QPK>
__global__ __launch_bounds__(SE_THREADS) void stream_decode_kernel(const SeArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* ring = smem;
    SeCtl* c = (SeCtl*)(smem + (size_t)a.nslots * SE_SLOT);
    float* att = (float*)((char*)c + se_ctl_bytes());
    const int wid = (int)threadIdx.x >> 6;
    const int lane = se_lane();
    // LDS control block: zero, ring flags -1, then everyone starts
    for (int i = threadIdx.x; i < (int)(se_ctl_bytes() / 4); i += SE_THREADS) ((int*)c)[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < SE_MAXS; i += SE_THREADS) { c->full[i] = -1; c->free_[i] = -1; }
    __syncthreads();
    if (wid >= SE_NW) {
        se_loader<DT, DTC>(a, ring, c, wid - SE_NW);
        return;
    }

    constexpr int E = WDec<DT>::E, EC = WDec<DTC>::E;
    constexpr int ESZ = 16 / E, ESZC = 16 / EC;
    const int nblk = gridDim.x, b = blockIdx.x;
    const int L = a.n_layers;
    SeState st;
    st.cw = wid;
    const int n_tok = a.n_prompt + a.n_gen;
    int own0, own1;  // residual rows of this CU (= its Wo / W2 rows)
    se_part(a.dim, nblk, b, own0, own1);
    float xr[SE_XF];

    int token = 0;
    if (a.n_prompt == 0 && n_tok > 0) {
        // decode from the logits the previous call left: first token = their argmax
        if (wid == 0) {
            unsigned long long best = 0;
            for (int i = lane; i < a.vocab; i += 64) {
                const float v = a.logits[i];
                if (v > FLT_MIN) {
                    const unsigned long long k = argmax_key(v, i);
                    best = k > best ? k : best;
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long other = __shfl_xor(best, o, 64);
                best = other > best ? other : best;
            }
            if (lane == 0) c->token = argmax_key_index(best);
        }
        if (!se_cbar(a, c, st.cgen, &c->cbar, SE_NW)) return;
        token = c->token;
    }

    for (int t = 0; t < n_tok; t++) {
        const int pos = a.pos0 + t;
        if (t < a.n_prompt) token = a.prompt[t];
        const bool gen = t >= a.n_prompt;
        if (gen && b == 0 && wid == 0 && lane == 0) {
            a.tokens_out[t - a.n_prompt] = token;
            *a.n_done = t - a.n_prompt + 1;
        }
        if (gen && (token == a.stop_a || token == a.stop_b)) break;
        const int msl = a.max_seq_len;
        const int kv_sink = pos >= msl ? 2 : 0;  // KV_SINKS, src/infer.cpp:611-613
        const int kv_len = pos >= msl ? msl : pos + 1;
        SeTok tk;
        tk.t = t;
        tk.pos = pos;
        tk.kv_pos = kv_sink + (pos - kv_sink) % (msl - kv_sink);
        tk.own0 = own0;
        tk.xtag0 = (unsigned)(t * (2 * L + 1) + 1);
        tk.ltag0 = (unsigned)(t * L + 1);
        tk.ctag = (unsigned)(t % 32767) + 1;
        {
            int c0, c1;
            se_part(a.vocab, nblk, b, c0, c1);
            tk.cls_nt = se_ntiles(c1 - c0);
        }
        const bool want_logits = se_want_logits(a, t, n_tok);
        // attention items this token: KV head x split
        int S = (kv_len + a.split_rows - 1) / a.split_rows;
        S = max(1, min(S, a.max_splits));
        const int T = (kv_len + S - 1) / S;
        S = (kv_len + T - 1) / T;

        se_embed<E>(a, st, token, xr);
        const int n_ph = 4 * L + (want_logits ? 1 : 0);
        const int trc = a.trace ? se_trace_cu(b, nblk) : -1;
        unsigned long long* trp =
            (trc >= 0 && t == n_tok - 1 && wid == 0 && lane == 0) ? a.trace + SE_TR_CU * nblk + trc * (4 * L + 1) * SE_TR_PH
                                                                   : nullptr;
        for (int q = 0; q < n_ph; q++) {
            const uint64_t t_acq = a.trace ? se_now() : 0;
            if (trp) trp[q * SE_TR_PH + 0] = t_acq;
            const int l = q >> 2;
            const int ph = q < 4 * L ? (q & 3) : SE_CLS;
            // ---- the phase's input: granules of the previous phase, rmsnorm where the
            // reference has one (src/infer.cpp:374-382, 455-463, 626-634) ----
            const unsigned long long* gbuf = a.xg;
            int gn = a.dim;
            unsigned gtag = tk.xtag0 + 2 * l;
            const void* normw = nullptr;
            if (ph == SE_QKV) {
                normw = a.layers[l].attn_norm;
            } else if (ph == SE_WO) {
                // attention (src/infer.cpp:434-444) on the CUs that own a (head, split) item
                if (b < a.n_kv_heads * S && wid < SE_NA && !(a.debug & 2)) {
                    if (!se_attention<HD, QPK>(a, c, att, st, l, t, b / S, b % S, S, T, kv_sink, kv_len,
                                               trp ? trp + q * SE_TR_PH : nullptr))
                        return;
                    if (a.trace) st.w_att += se_now() - t_acq;
                }
                gbuf = a.ag; gn = a.q_dim; gtag = tk.ltag0 + l;
            } else if (ph == SE_W13) {
                gtag = tk.xtag0 + 2 * l + 1;
                normw = a.layers[l].ffn_norm;
            } else if (ph == SE_W2) {
                gbuf = a.hg; gn = a.hidden; gtag = tk.ltag0 + l;
            } else {
                gtag = tk.xtag0 + 2 * L;
                normw = a.final_norm;
            }
            const bool cls_other = (ph == SE_CLS) && (EC != E);
            float nw[SE_XF];
            if (cls_other) {
                if constexpr (EC != E) {
                    se_load_norm<EC>(a, st, gn, normw, nw);
                    if (!se_sweep<EC>(a, c, st, gbuf, gn / (64 * EC), gtag, xr)) return;
                    if (!se_rmsnorm<EC>(a, c, st, gn, nw, xr)) return;
                }
            } else {
                if (normw) se_load_norm<E>(a, st, gn, normw, nw);
                if (!(ph == SE_QKV && l == 0) && !se_sweep<E>(a, c, st, gbuf, gn / (64 * E), gtag, xr)) return;
                if (normw && !se_rmsnorm<E>(a, c, st, gn, nw, xr)) return;
            }
            // the owned residual rows start as the embedding: written after the rmsnorm
            // barrier above, which every wave reaches after the previous token's last W2
            // epilogue, and before wave 0 arrives at its first Wo tile (the first reader)
            if (ph == SE_QKV && l == 0 && wid == 0)
                for (int r = own0 + lane; r < own1; r += 64)
                    c->xown[r - own0] = dec1(a.embed_dt, a.embed, (size_t)token * a.dim + r);
            if (a.trace) {
                const uint64_t now = se_now();
                st.w_acq += now - t_acq;
                if (trp) trp[q * SE_TR_PH + 1] = now;
            }
            // ---- the matrix ----
            const SeMat m = se_mat<ESZ, ESZC>(a, l, ph);
            int r0, r1;
            se_part(m.rows, nblk, b, r0, r1);
            if (ph == SE_CLS && tk.cls_nt == 0 && wid == 0 && lane == 0)  // no lm_head rows here
                __hip_atomic_store(a.cg + b, (unsigned long long)tk.ctag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cls_other) {
                if constexpr (EC != E)
                    if (!se_matrix<DTC, HD, QPK>(a, c, ring, st, tk, l, ph, m, r0, r1, xr)) return;
            } else {
                if (!se_matrix<DT, HD, QPK>(a, c, ring, st, tk, l, ph, m, r0, r1, xr)) return;
            }
            if (trp) trp[q * SE_TR_PH + 2] = se_now();
        }
        // ===== next token = argmax over every CU's candidate =====
        if (want_logits && t + 1 < n_tok && t + 1 >= a.n_prompt) {
            unsigned long long best = 0;
            SeSpin sp(SE_W_CAND, (int)tk.ctag);
            if (lane == 0) lds_add(&c->gath, 1);
            for (;;) {
                bool ok = true;
                unsigned long long bb = 0;
                for (int i = lane; i < nblk; i += 64) {
                    const unsigned long long k = __hip_atomic_load(a.cg + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = ok && (unsigned)(k & 0x7FFF) == tk.ctag;
                    bb = k > bb ? k : bb;
                }
                if (__all(ok) || (a.debug & 2)) { best = bb; break; }
                __builtin_amdgcn_s_sleep(1);
                if (!sp.step(a, c)) return;
            }
            if (lane == 0) lds_add(&c->gath, -1);
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long other = __shfl_xor(best, o, 64);
                best = other > best ? other : best;
            }
            token = (best >> 15) ? 0x1FFFF - (int)((best >> 15) & 0x1FFFF) : 0;
            if (token >= a.vocab) token = 0;  // only reachable with the debug switches
        }
    }
    // consumers done: release the loader if it still waits for ring slots
    if (lane == 0) lds_add(&c->ndone, 1);  // the loader leaves once every consumer wave has
    if (wid == 0 && lane == 0) {
        if (a.trace) {
            a.trace[SE_TR_CU * b + 1] = st.w_full;
            a.trace[SE_TR_CU * b + 2] = st.w_acq;
            a.trace[SE_TR_CU * b + 3] = st.w_att;
        }
    }
}

}  // namespace xalm
