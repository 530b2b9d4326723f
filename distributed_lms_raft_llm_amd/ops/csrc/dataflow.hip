// Persistent dataflow decode (latency path, 1-2 rows): ONE launch runs many greedy decode steps
// of GPT-2 (every layer, the LM head with the repetition penalty, argmax and the bookkeeping that
// decode_update does), the reference's own operating point -- one model.generate per student
// query (/root/reference/GUI_RAFT_LLM_SourceCode/tutoring_server.py:21-29).
//
// Why: at batch 1 every layer kernel of the launch-per-op path moves 1-10 MB and is bound by its
// dependency chain (launch boundary + weight round trip), not by HBM (docs/PERFORMANCE.md: 39
// kernels of 5-9 us per step against a ~40 us weight-streaming floor).  Weights do not depend on
// activations, so here every CU streams ITS weight rows into an LDS ring ahead of the dependency
// that needs them, and the phases hand off through per-phase arrival counters instead of kernel
// boundaries or grid barriers.
//
// Geometry: one 448-thread workgroup per CU (G <= #CUs, all resident: ~160 KB of LDS each):
//   wave 0      "comm": polls arrival counters / granules, loads the residual, LayerNorm, publishes
//               results (granule stores, 64-bit fixed-point atomics, counter adds).  It is the only
//               wave that waits on vmcnt for hand-off traffic.
//   waves 1-2   "loaders": stream this CU's pre-packed weight rows (global -> LDS ring by LDS-DMA,
//               global_load_lds_dwordx4), as far ahead as the ring allows.
//   waves 3..6  "compute": MFMA on the ring's weight rows: v_mfma_f32_16x16x32_bf16 for the
//               dot-product phases (row-major rows ARE the B fragments), v_mfma_f32_16x16x16_bf16
//               on K-major blocks for the out-projection / c_proj (each wave owns 16-column
//               output tiles, so no cross-wave reduction); attention for the CU's head (K/V
//               prefetched into registers before q is ready).
// Waves synchronise through LDS words only (no s_barrier, no __syncthreads).
//
// Per layer (TP=1):
//   E1  residual complete (previous MLP's atomics + counter, or the embedding) -> every CU: LN1,
//       its rows of W_qkv (dot) -> q/k/v as tagged 8-byte granules (+ K/V cache rows)
//   E2  per-head granules -> the attention CUs of that head: attention over the cache, then W_o
//       for the CU's slice of head dims (or, opt-in, of output columns) -> counted fixed-point
//       atomics into XA
//   E3  XA complete (every word's contribution count) -> every CU: x += XA + b_o, LN2, the c_fc
//       rows of its intermediate slice (h = bf16(gelu(.))), c_proj for its slice of output columns
//       -> counted fixed-point atomics into XM
//   (output-column slices: a CU adds d / GS or d / J residual words per row, not d -- the counted
//   atomics' issue and memory-side time set the publish and edge costs; ops/dataflow.py assign())
// then ln_f + this CU's LM-head rows + penalty + argmax key -> 64-bit atomicMax + counter -> every
// CU reads the token and the next step starts.  Every CU keeps its own copy of the residual stream
// as int64 fixed point (value * 2^32, DLMS_FIX_SCALE in skinny.hip) and adds each edge's summed
// contributions: integer adds commute, so results do not depend on arrival order and all copies
// agree bit for bit.
//
// Commit: CU 0 writes the row state back (lengths, tokens, penalty bitmap) only after every step it
// ran has completed; an aborted launch commits nothing, so a retry -- another launch or the
// launch-per-op path -- starts from exactly the state this launch found.
//
// Hand-off memory ("scratch") is FRESH per step (zeroed before the launch), so nothing a CU reads
// was ever cached before its final value was written; payload/counter traffic is sc1 (agent scope),
// every storing wave drains (s_waitcnt vmcnt(0)) before its counter add (cdna_hip_programming.md
// Guideline 16 / MI355X_MICROARCH.md "Valid forms", first row).  Every spin is bounded (wall clock)
// and checks a global error word, so a stuck or mis-sized launch drains with an error code instead
// of hanging the GPU.
#include "common.h"

namespace df {

constexpr int NC = 4;                 // compute waves
#ifndef DF_NL
#define DF_NL 2
#endif
#ifndef DF_INFL
#define DF_INFL 48
#endif
constexpr int NL = DF_NL;             // loader waves (A/B builds: -DDF_NL=3)
constexpr int NWAVES = NC + NL + 1;   // + comm
constexpr int NTHREADS = 64 * NWAVES;
constexpr int SHARDS = 8;             // arrival counters are sharded by blockIdx % 8
constexpr int CSTRIDE = 16;           // u64 words between shards (one 128-B line each)
constexpr int INFL = DF_INFL;         // LDS-DMA units (1 KiB) in flight per loader wave (<= 71: vmcnt is 6 bits)
#ifndef DF_COPIES
#define DF_COPIES 2
#endif
constexpr int COPIES = DF_COPIES;     // fixed-point residual copies (each CU adds into its Cu::acp / mcp)
constexpr int LDS_MAX = 160 * 1024;
// a streamed weight row: d bf16 + 32 bytes of padding, so the 16 rows of an MFMA B fragment sit on
// distinct 16-B LDS slots (a 1536-B row is 0 mod 256 B: 8-way ds_read_b128 conflicts unpadded)
#define ROW_BYTES(D) (2u * (D) + 32u)
constexpr int TR_STEPS = 4;           // traced steps (profiling builds pass a trace buffer)
constexpr int TR_EV = 32;             // stamps per (step, layer)
constexpr unsigned long long TIMEOUT_TICKS = 20000000ull;  // 0.2 s of the 100 MHz wall clock

typedef unsigned long long u64;
typedef long long i64;

struct Cu {           // per-CU assignment (host-built table, ops/dataflow.py assign() mirrors it)
    int q0, nq;       // W_qkv rows [q0, q0 + nq)
    int f0, nf;       // intermediate (c_fc row) slice [f0, f0 + nf)
    int v0, nv;       // LM-head (wte) rows [v0, v0 + nv)
    int ah;           // attention head (-1: none)
    int ao0, aon;     // its W_o output columns [ao0, ao0 + aon) ...
    int ak0, akn;     // ... over the head dims [ak0, ak0 + akn)
    int pd0, pdn;     // c_proj output columns [pd0, pd0 + pdn) of the slice
    int acp, mcp;     // residual copy of the attention / MLP contributions
    int lm_off;       // byte offset of its LM-head rows within one step's stream (after the L layers)
    long long off;    // byte offset of this CU's packed row stream
    long long step_bytes;
};

struct Layer {
    const float *ln1_g, *ln1_b, *b_qkv, *b_o, *ln2_g, *ln2_b, *b_fc, *b_p;
    bf16_t *k_cache, *v_cache;  // [slots][H][T][64]
};

struct Args {
    const bf16_t* packed;
    const Cu* cus;
    const Layer* layers;
    const bf16_t* wte;
    const bf16_t* wpe;
    const float* lnf_g;
    const float* lnf_b;
    int* lens;
    int* finished;
    int* out_tokens;
    unsigned int* seen;
    int* cur_tok;
    int* cur_pos;
    int* cur_kvlen;
    const int* slots;
    float* x_out;
    u64* scratch;
    unsigned int* err;  // [0] code, [1] block, [2] step, [3] where
    u64* trace;         // optional: [G][TR_STEPS][L + 1][TR_EV] wall-clock stamps (profiling)
    long long step_words;
    int R, D, H, L, V, T, seen_words, eos, nsteps, A, C, max_nq, swl, ring_bytes, ldx, n_slots, P, nt_weights;
    int ko, kf;  // K (padded to 16) of the per-CU W_o block and c_proj block
    int fault_step;  // test hook: >= 0 makes the last CU abort at that step as a timed-out wait would
    int pad_args1;
    int gather_pause;  // loaders pause while the comm wave waits on a hand-off (C_GATHER)
    int spec_rem;      // residual poll: start reading whole rows once the watched word lacks <= this many adds
    int argmax_slots;  // per-step argmax: every CU stores its best key in a slot of its own, all CUs read all slots
    int pad_args2;
    int exp_att[8], exp_mlp[8];  // contributions each residual copy receives (attention / MLP CUs)
    float eps, penalty;
};

// ------------------------------------------------------------------ LDS layout (host mirrors it)
struct Lay {
    int ring, ctl, st, xn, res, part, att, mrg, seen, keys, hb, fcp, xs, total;
};

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline Lay lds_layout(int D, int R, int max_nq, int swl, int ring_bytes) {
    // the small per-CU areas FIRST, the weight ring last: every LDS address the comm / compute
    // waves form with a constant offset then fits the 16-bit ds_* immediate (with the ring first
    // they sat above 64 KiB and the compiler kept one address register per unrolled access live
    // across the step loop -- the two-row kernel spilled to scratch)
    Lay o;
    int off = 0;
    o.ctl = off; off += 64 * 4;
    o.st = off; off += 8 * R * 4;
    o.xn = off; off = align16(off + R * D * 2);                          // bf16 activation (A fragments)
    o.res = off; off = align16(off + NC * R * (max_nq > 0 ? max_nq + 16 : 16) * 4);  // K-split partials
    o.part = off; off = align16(off + R * D * 4);                        // f32 [R][D], column tiles per wave
    o.att = off; off = align16(off + 3 * R * 64 * 4);
    o.mrg = off; off = align16(off + NC * R * 68 * 4);
    o.seen = off; off = align16(off + R * swl * 4);
    o.keys = off; off = align16(off + NC * R * 8);
    o.hb = off; off = align16(off + NC * R * 64 * 2);                    // per-wave A staging (bf16 [R][64])
    o.fcp = off; off = align16(off + NC * R * 64 * 4);                   // K-split c_fc partials
    o.xs = off; off = align16(off + R * D * 8);                          // the comm wave's int64 residual
    o.ring = off; off += ring_bytes;
    o.total = off;
    return o;
}

// ctl words
enum { C_READY = 0, C_ABORT = 2, C_DONE = 3, C_CONT = 4, C_GATHER = 5, C_LOADED = 8, C_PHDONE = 16, C_CONS = 24,
       C_MID = 32 };
// C_GATHER: the comm wave is waiting on a hand-off (residual edge, q/k/v granules): the loaders
// issue no new weight batches meanwhile, so the poll's loads do not queue behind this CU's own
// refill burst (MI355X_MICROARCH.md "gather-pass": 1.0-1.7 us behind an unthrottled refill vs
// 0.3-0.65 with the CU's own DMA quiet).  Args::gather_pause (always 1 from ops/dataflow.py).
// (C_LOADED + j: loader wave j's completed-batch count)
// row state words (st[b * 8 + k])
enum { S_TOK = 0, S_POS = 1, S_FIN = 2, S_LEN = 3, S_SLOT = 4 };
// error codes (err[0]); err[4] = 1 + steps run once CU 0 has committed the row state
enum { E_WAIT_CNT = 1, E_WAIT_GRAN = 2, E_WAIT_LDS = 3, E_LOADER = 4, E_INJECTED = 5 };

// scratch word offsets (per step)
struct Scr {
    long long xw, qkv0, cnt0, keys, kslots, words;
};
__host__ __device__ inline Scr scratch_layout(int R, int D, int L, int C) {
    Scr s;
    s.xw = (long long)C * R * D;
    s.qkv0 = 2LL * L * s.xw;
    long long c = s.qkv0 + (long long)L * R * 3 * D;
    s.cnt0 = (c + 15) & ~15LL;
    s.keys = s.cnt0 + (2LL * L + 1) * SHARDS * CSTRIDE;
    s.kslots = s.keys + 16 + ((R + 15) & ~15);  // [R][256] per-CU best keys (argmax_slots)
    s.words = s.kslots + 256LL * R;
    return s;
}

__host__ __device__ inline unsigned pid_of(int s, int l, int k, int L) {
    return 1u + ((unsigned)(s * (L + 1) + l) << 2) + (unsigned)k;
}

// ------------------------------------------------------------------ primitives
__device__ __forceinline__ u64 gld64(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gst64(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned gld32(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gadd64(u64* p, u64 v) { __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned lds_ld(const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's earlier LDS writes land first
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// loads through pointers held in memory (the Layer table) are FLAT unless the address space is
// spelled out; flat loads also count in lgkmcnt, so every LDS wait would wait for them too
#define AS1 __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ T gl(const T* p) { return *(const AS1 T*)p; }
__device__ __forceinline__ uint4 gl(const uint4* p) {
    const u32x4_t v = *(const AS1 u32x4_t*)p;
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ u64 clk() { return wall_clock64(); }
__device__ __forceinline__ float bf16r(float f) { return bf16_to_f32(f32_to_bf16(f)); }
__device__ __forceinline__ float fix2f(i64 v) { return (float)v * (1.0f / 4294967296.0f); }
__device__ __forceinline__ i64 f2fix(float v) { return __float2ll_rn(v * 4294967296.0f); }

// Counted fixed point: every atomic contribution to a residual word adds (1 << 56) + (v + BIAS)
// with |v| < BIAS = 2^47 (value * 2^32, |value| < 32768): the biased values never carry into the
// top byte, which therefore COUNTS the contributions.  A consumer polls the residual itself and
// knows it is final when every word's count equals the number of contributors -- no drain, no
// separate arrival counter, one round trip (each needed a dependent memory round trip before).
constexpr u64 CNT_ONE = 1ull << 56;
constexpr i64 CNT_BIAS = 1ll << 47;
constexpr u64 CNT_MASK = CNT_ONE - 1;
__device__ __forceinline__ u64 counted(i64 v) {
    v = v < -(CNT_BIAS - 1) ? -(CNT_BIAS - 1) : (v > CNT_BIAS - 1 ? CNT_BIAS - 1 : v);
    return CNT_ONE + (u64)(v + CNT_BIAS);
}

// profiling stamp (comm wave lane 0; plain store, read after the launch)
__device__ __forceinline__ void stamp(const Args& a, int s, int l, int ev, int lane) {
    if (a.trace && s < TR_STEPS && lane == 0)
        a.trace[(((size_t)blockIdx.x * TR_STEPS + s) * (a.L + 1) + l) * TR_EV + ev] = wall_clock64();
}
__device__ __forceinline__ void stamp_val(const Args& a, int s, int l, int ev, u64 v) {
    if (a.trace && s < TR_STEPS)
        a.trace[(((size_t)blockIdx.x * TR_STEPS + s) * (a.L + 1) + l) * TR_EV + ev] = v;
}

__device__ __forceinline__ void set_err(const Args& a, unsigned code, unsigned where, int s) {
    if (atomicCAS(a.err, 0u, code) == 0u) {
        __hip_atomic_store(a.err + 1, (unsigned)blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.err + 2, (unsigned)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.err + 3, where, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// LDS wait: *w >= target (false on abort / timeout; a timeout raises the abort itself)
__device__ __forceinline__ bool lds_wait_ge(unsigned* ctl, int idx, unsigned target, const Args& a, unsigned where,
                                            int s) {
    if (lds_ld(ctl + idx) >= target) return true;
    const u64 t0 = clk();
    for (;;) {
        if (lds_ld(ctl + idx) >= target) return true;
        if (lds_ld(ctl + C_ABORT)) return false;
        if (clk() - t0 > TIMEOUT_TICKS) {
            set_err(a, E_WAIT_LDS, where, s);
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// comm wave: wait until the sharded counter reaches target (false on error / timeout)
__device__ __forceinline__ bool wait_count(const u64* cnt, u64 target, const Args& a, unsigned* ctl, unsigned where,
                                           int s, int lane) {
    const u64 t0 = clk();
    for (;;) {
        u64 v = lane < SHARDS ? gld64(cnt + lane * CSTRIDE) : 0ull;
        const unsigned e = lane == SHARDS ? gld32(a.err) : 0u;
        u64 tot = 0;
#pragma unroll
        for (int k = 0; k < SHARDS; ++k) tot += lane_value_u64(v, k);
        const unsigned ee = (unsigned)__builtin_amdgcn_readlane((int)e, SHARDS);
        if (tot >= target) return true;
        if (ee || lds_ld(ctl + C_ABORT)) {
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        if (clk() - t0 > TIMEOUT_TICKS) {
            set_err(a, E_WAIT_CNT, where, s);
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// comm wave: wait until every compute wave reported phase `pid` done
__device__ __forceinline__ bool wait_phdone(unsigned* ctl, unsigned pid, const Args& a, int s) {
#pragma unroll
    for (int w = 0; w < NC; ++w)
        if (!lds_wait_ge(ctl, C_PHDONE + w, pid, a, 100 + w, s)) return false;
    return true;
}

// ------------------------------------------------------------------ comm wave
template <int D>
__device__ __forceinline__ void load_ln(const float* g, const float* b, float (&gg)[D / 64], float (&bb)[D / 64], int lane) {
#pragma unroll
    for (int i = 0; i < D / 64; ++i) {
        gg[i] = gl(g + lane + 64 * i);
        bb[i] = gl(b + lane + 64 * i);
    }
}

// d >= 1024 register diet of the comm wave (its arrays of D / 64 values per lane set the whole
// kernel's allocation: 1280 / 1600 spilled 72 / 158 VGPRs): the bias is added into this CU's residual
// copy BEFORE the poll (its load hides under the all-to-all wait) instead of being held through it,
// and gamma / beta are loaded after the poll instead of across it
template <int D>
constexpr bool big_d() { return D >= 1024; }
// the residual poll hands the updated row back as floats (the LayerNorm's input) instead of a second
// LDS pass over it: one row at d 768, 28.5-28.6 -> 28.2 ms per query; at d 1024 it took the kernel
// to 246 VGPRs and GPT-2-medium from 65.8 to 68.0 ms (profiles/r4_df_xf_slots_ab.jsonl), so not there
#ifndef DF_XF_POLL
#define DF_XF_POLL 1  // A/B build knob (-DDF_XF_POLL=0: LayerNorm input re-read from LDS)
#endif
template <int D, int R>
constexpr bool xf_from_poll() { return DF_XF_POLL && R == 1 && D <= 768; }

template <int D, int R>
__device__ __forceinline__ void add_bias_xs(i64* xs, const float* bias, int lane) {
    constexpr int EPL = D / 64;
    float b[EPL];
#pragma unroll
    for (int i = 0; i < EPL; ++i) b[i] = gl(bias + lane + 64 * i);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < EPL; ++i) xs[r * D + lane + 64 * i] += f2fix(b[i]);
}

template <int D, int R>
__device__ __forceinline__ void layer_norm(float (&x)[R][D / 64], const float (&gg)[D / 64], const float (&bb)[D / 64],
                                           float eps, bf16_t* xn_lds, int lane) {
    constexpr int EPL = D / 64;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < EPL; ++i) s += x[r][i];
        const float mean = wave_sum(s) * (1.0f / D);
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            const float d = x[r][i] - mean;
            v += d * d;
        }
        const float rstd = rsqrtf(wave_sum(v) * (1.0f / D) + eps);
#pragma unroll
        for (int i = 0; i < EPL; ++i) xn_lds[r * D + lane + 64 * i] = f32_to_bf16((x[r][i] - mean) * rstd * gg[i] + bb[i]);
    }
}

// Poll residual-update buffer X (COPIES x R rows x D counted words, sc1 buffer loads) until every
// word carries exactly expc[copy] contributions, then add the exact integer sum of the copies (+
// the bias) to this CU's own copy of the residual xs (and hand the new row back as floats in xf).  The buffer is fresh per step, so a word can
// only ever read below its final count.
template <int D, int R>
__device__ __forceinline__ bool poll_resid(const u64* X, const int* expc, const float (&bias)[D / 64],
                                           i64* xs, float (&xf)[R][D / 64], const Args& a, unsigned* ctl,
                                           unsigned where, int s, int lane) {
    constexpr int EPL = D / 64;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, COPIES * R * D * 8, 0x00020000);
    int ec[COPIES];
#pragma unroll
    for (int c = 0; c < COPIES; ++c) ec[c] = expc[c];
    if (a.gather_pause) lds_st(ctl + C_GATHER, 1u);
    const u64 t0 = clk();
    // phase 1: poll ONE word per copy -- the element every producer adds last (row R-1, element
    // D-1) -- so 256 pollers do not hammer the lines the atomics are still updating.  With
    // spec_rem > 0 phase 2 (whole rows, exact counts checked per word) starts once that word lacks at
    // most spec_rem adds: the last producers' adds then land under row reads already in flight,
    // one round trip fewer per hand-off than watching the word reach its final count first
    const int rem = a.spec_rem;
    for (;;) {
        bool done = true;
        if (lane < COPIES) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, ((lane * R + R - 1) * D + D - 1) * 8, 0, 16);
            int want = ec[0];
#pragma unroll
            for (int c = 1; c < COPIES; ++c) want = lane == c ? ec[c] : want;
            done = (int)(x[1] >> 24) >= want - rem;
        }
        if (__all(done)) break;
        if ((unsigned)__builtin_amdgcn_readfirstlane((int)gld32(a.err)) || lds_ld(ctl + C_ABORT)) {
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        if (clk() - t0 > TIMEOUT_TICKS) {
            set_err(a, E_WAIT_CNT, where, s);
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    // phase 2: the whole buffer (almost always complete by now), one ROW at a time: all COPIES x
    // EPL words of the row in flight together (one round trip); a row whose words all carry their
    // final count is final for good (the buffer is fresh per step), so it is added to xs at once
    // and never read again -- holding every row's words at once pushed the 2-row kernel into scratch
    unsigned pending = (1u << R) - 1u;
    for (;;) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!(pending & (1u << r))) continue;
            u64 v[COPIES][EPL];
#pragma unroll
            for (int c = 0; c < COPIES; ++c)
#pragma unroll
                for (int i = 0; i < EPL; ++i) {
                    const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (((c * R + r) * D) + lane + 64 * i) * 8, 0,
                                                                        16 /* sc1 */);
                    v[c][i] = ((u64)x[1] << 32) | x[0];
                }
            bool ok = true;
#pragma unroll
            for (int c = 0; c < COPIES; ++c)
#pragma unroll
                for (int i = 0; i < EPL; ++i) ok &= (int)(v[c][i] >> 56) == ec[c];
            if (__all(ok)) {
#pragma unroll
                for (int i = 0; i < EPL; ++i) {
                    i64 t = f2fix(bias[i]);
#pragma unroll
                    for (int c = 0; c < COPIES; ++c) t += (i64)(v[c][i] & CNT_MASK) - (i64)ec[c] * CNT_BIAS;
                    const i64 nx = xs[r * D + lane + 64 * i] + t;
                    xs[r * D + lane + 64 * i] = nx;
                    if constexpr (xf_from_poll<D, R>()) xf[r][i] = fix2f(nx);
                }
                pending &= ~(1u << r);
            }
        }
        if (!pending) {
            if (a.gather_pause) lds_st(ctl + C_GATHER, 0u);
            return true;
        }
        if ((unsigned)__builtin_amdgcn_readfirstlane((int)gld32(a.err)) || lds_ld(ctl + C_ABORT)) {
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        if (clk() - t0 > TIMEOUT_TICKS) {
            set_err(a, E_WAIT_CNT, where, s);
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Publish this CU's part[r][o0 .. o0 + on) as counted fixed-point atomics into X (the residual-update
// buffer of its copy): every LDS value read first (clamped index, no branch: one LDS round trip for
// the lot), then the atomics (predicated only when the CU publishes a column range, on < D)
template <int D, int R>
__device__ __forceinline__ void publish(u64* X, const float* part, int o0, int on, int lane) {
    constexpr int EPL = D / 64;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float p[EPL];
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            const int e = lane + 64 * i;
            p[i] = part[r * D + o0 + (e < on ? e : on - 1)];
        }
        if (on == D) {
#pragma unroll
            for (int i = 0; i < EPL; ++i) gadd64(X + (size_t)r * D + lane + 64 * i, counted(f2fix(p[i])));
        } else {
#pragma unroll
            for (int i = 0; i < EPL; ++i)
                if (lane + 64 * i < on) gadd64(X + (size_t)r * D + lane + 64 * i, counted(f2fix(p[i])));
        }
    }
}

template <int D, int R>
__device__ __forceinline__ void comm_wave(const Args& a, const Cu& cu, char* lds, const Lay& ly, int lane) {
    constexpr int EPL = D / 64;
    unsigned* ctl = reinterpret_cast<unsigned*>(lds + ly.ctl);
    int* st = reinterpret_cast<int*>(lds + ly.st);
    bf16_t* xn = reinterpret_cast<bf16_t*>(lds + ly.xn);
    const float* res = reinterpret_cast<const float*>(lds + ly.res);
    const float* part = reinterpret_cast<const float*>(lds + ly.part);
    float* att = reinterpret_cast<float*>(lds + ly.att);
    unsigned* seen = reinterpret_cast<unsigned*>(lds + ly.seen);
    const u64* keys = reinterpret_cast<const u64*>(lds + ly.keys);
    const int L = a.L, H = a.H, T = a.T, C = a.C, G = gridDim.x;
    const Scr sc = scratch_layout(R, D, L, C);
    const int shard = blockIdx.x % SHARDS;
    const int D3 = 3 * D;

    // ---- row state
    int tok[R], pos[R], fin[R], len[R], slot[R], len0[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        slot[r] = a.slots[r];
        len[r] = a.lens[slot[r]];
        len0[r] = len[r];
        fin[r] = a.finished[slot[r]];
        tok[r] = a.cur_tok[slot[r]];
        pos[r] = a.cur_pos[slot[r]];
        if (lane == 0) {
            st[r * 8 + S_TOK] = tok[r];
            st[r * 8 + S_POS] = pos[r];
            st[r * 8 + S_FIN] = fin[r];
            st[r * 8 + S_LEN] = len[r];
            st[r * 8 + S_SLOT] = slot[r];
        }
        // this CU's slice of the repetition-penalty bitmap, re-based to bit 0 = row v0
        for (int i0 = 0; i0 < cu.nv; i0 += 64) {
            const int i = i0 + lane;
            const int v = cu.v0 + i;
            unsigned bit = 0;
            if (i < cu.nv && (v >> 5) < a.seen_words) bit = (a.seen[(size_t)slot[r] * a.seen_words + (v >> 5)] >> (v & 31)) & 1u;
            const u64 m = __ballot(bit);
            if (lane == 0) {
                seen[r * a.swl + (i0 >> 5)] = (unsigned)m;
                seen[r * a.swl + (i0 >> 5) + 1] = (unsigned)(m >> 32);
            }
        }
    }

    bool ok = true;
    int s = 0;
    for (; s < a.nsteps && ok; ++s) {
        u64* sw = a.scratch + (size_t)s * a.step_words;
        const unsigned tag = (unsigned)s + 1u;
        // this CU's copy of the residual stream (int64 fixed point), kept in LDS: as registers it
        // pushed the kernel past 256 VGPRs at two rows (scratch spills in every phase)
        i64* xs = reinterpret_cast<i64*>(lds + ly.xs);
        for (int l = 0; l < L && ok; ++l) {
            const Layer lw = a.layers[l];
            stamp(a, s, l, 0, lane);
            if (l == 0) {
                stamp_val(a, s, 0, 26, __builtin_amdgcn_s_memtime());
                stamp_val(a, s, 0, 27, wall_clock64());
            }
            // ---------------- E1: residual in, LN1.  Every CU keeps the whole residual itself (exact
            // int64 fixed point): x += (sum of the previous MLP's contributions) + b_proj
            float xf[R][EPL];
            float gg[EPL], bb[EPL];
            if constexpr (!big_d<D>())
                load_ln<D>(lw.ln1_g, lw.ln1_b, gg, bb, lane);  // issued before the wait: off the critical path
            if (l == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < EPL; ++i) {
                        const int e = lane + 64 * i;
                        const i64 x0 = f2fix(bf16_to_f32(a.wte[(size_t)tok[r] * D + e]) +
                                             bf16_to_f32(a.wpe[(size_t)pos[r] * D + e]));
                        xs[r * D + e] = x0;
                        if constexpr (xf_from_poll<D, R>()) xf[r][i] = fix2f(x0);
                    }
            } else {
                float bp[EPL];
                if constexpr (big_d<D>()) {
                    add_bias_xs<D, R>(xs, a.layers[l - 1].b_p, lane);
#pragma unroll
                    for (int i = 0; i < EPL; ++i) bp[i] = 0.f;
                } else {
#pragma unroll
                    for (int i = 0; i < EPL; ++i) bp[i] = gl(a.layers[l - 1].b_p + lane + 64 * i);
                }
                if (!(ok = poll_resid<D, R>(sw + (2 * (l - 1) + 1) * sc.xw, a.exp_mlp, bp, xs, xf, a, ctl, 10 * l + 1,
                                            s, lane)))
                    break;
            }
            if constexpr (big_d<D>()) load_ln<D>(lw.ln1_g, lw.ln1_b, gg, bb, lane);
            if constexpr (!xf_from_poll<D, R>()) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < EPL; ++i) xf[r][i] = fix2f(xs[r * D + lane + 64 * i]);
            }
            stamp(a, s, l, 1, lane);
            layer_norm<D, R>(xf, gg, bb, a.eps, xn, lane);
            unsigned pid = pid_of(s, l, 0, L);
            lds_st(ctl + C_READY, pid);
            stamp(a, s, l, 2, lane);
            // ---------------- QKV results -> granules (+ K/V cache rows)
            const float bq = lane < cu.nq ? gl(lw.b_qkv + cu.q0 + lane) : 0.f;
            if (!(ok = wait_phdone(ctl, pid, a, s))) break;
            stamp(a, s, l, 3, lane);
            if (lane < cu.nq) {
                const int n = cu.q0 + lane;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float acc = 0.f;
#pragma unroll
                    for (int w = 0; w < NC; ++w) acc += res[(w * R + r) * (a.max_nq + 16) + lane];
                    const float v = bf16r(acc + bq);
                    gst64(sw + sc.qkv0 + ((size_t)l * R + r) * D3 + n, ((u64)tag << 32) | __float_as_uint(v));
                    if (n >= D && !fin[r]) {
                        const int which = n >= 2 * D;
                        const int hd = n - D * (1 + which);
                        bf16_t* cache = which ? lw.v_cache : lw.k_cache;
                        const size_t o = (((size_t)slot[r] * H + (hd >> 6)) * T + pos[r]) * 64 + (hd & 63);
                        __hip_atomic_store((AS1 bf16_t*)(cache + o), f32_to_bf16(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            stamp(a, s, l, 4, lane);
            // ---------------- attention CUs: gather this head's q/k/v, publish the W_o partial
            if (cu.ah >= 0) {
                const u64* g = sw + sc.qkv0 + (size_t)l * R * D3;
                const int h = cu.ah;
                if (a.gather_pause) lds_st(ctl + C_GATHER, 1u);
                const u64 t0 = clk();
                for (;;) {
                    bool all = true;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const u64 q = gld64(g + (size_t)r * D3 + h * 64 + lane);
                        const u64 k = gld64(g + (size_t)r * D3 + D + h * 64 + lane);
                        const u64 v = gld64(g + (size_t)r * D3 + 2 * D + h * 64 + lane);
                        all &= (unsigned)(q >> 32) == tag && (unsigned)(k >> 32) == tag && (unsigned)(v >> 32) == tag;
                        att[(r * 3 + 0) * 64 + lane] = __uint_as_float((unsigned)q);
                        att[(r * 3 + 1) * 64 + lane] = __uint_as_float((unsigned)k);
                        att[(r * 3 + 2) * 64 + lane] = __uint_as_float((unsigned)v);
                    }
                    if (__all(all)) break;
                    if ((unsigned)__builtin_amdgcn_readfirstlane((int)gld32(a.err)) || lds_ld(ctl + C_ABORT) ||
                        clk() - t0 > TIMEOUT_TICKS) {
                        set_err(a, E_WAIT_GRAN, 10 * l + 2, s);
                        lds_st(ctl + C_ABORT, 1u);
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (!ok) break;
                if (a.gather_pause) lds_st(ctl + C_GATHER, 0u);
                stamp(a, s, l, 5, lane);
                pid = pid_of(s, l, 1, L);
                lds_st(ctl + C_READY, pid);
                if (!(ok = wait_phdone(ctl, pid, a, s))) break;
                stamp(a, s, l, 6, lane);
                publish<D, R>(sw + (2 * l) * sc.xw + (size_t)cu.acp * R * D + cu.ao0, part, cu.ao0, cu.aon, lane);
                stamp(a, s, l, 7, lane);
            }
            // ---------------- E3: XA complete -> LN2 -> MLP
            if constexpr (!big_d<D>()) load_ln<D>(lw.ln2_g, lw.ln2_b, gg, bb, lane);
            {
                float bo[EPL];
                if constexpr (big_d<D>()) {
                    add_bias_xs<D, R>(xs, lw.b_o, lane);
#pragma unroll
                    for (int i = 0; i < EPL; ++i) bo[i] = 0.f;
                } else {
#pragma unroll
                    for (int i = 0; i < EPL; ++i) bo[i] = gl(lw.b_o + lane + 64 * i);
                }
                if (!(ok = poll_resid<D, R>(sw + (2 * l) * sc.xw, a.exp_att, bo, xs, xf, a, ctl, 10 * l + 3, s, lane)))
                    break;
            }
            if constexpr (big_d<D>()) load_ln<D>(lw.ln2_g, lw.ln2_b, gg, bb, lane);
            stamp(a, s, l, 8, lane);
            stamp(a, s, l, 25, lane);
            if constexpr (!xf_from_poll<D, R>()) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < EPL; ++i) xf[r][i] = fix2f(xs[r * D + lane + 64 * i]);
            }
            layer_norm<D, R>(xf, gg, bb, a.eps, xn, lane);
            pid = pid_of(s, l, 2, L);
            lds_st(ctl + C_READY, pid);
            stamp(a, s, l, 9, lane);
            if (!(ok = wait_phdone(ctl, pid, a, s))) break;
            stamp(a, s, l, 10, lane);
            {
                publish<D, R>(sw + (2 * l + 1) * sc.xw + (size_t)cu.mcp * R * D + cu.pd0, part, cu.pd0, cu.pdn, lane);
                stamp(a, s, l, 11, lane);
            }
        }
        if (!ok) break;
        if (s == a.fault_step && blockIdx.x == G - 1) {  // test hook: an aborted hand-off (before the argmax)
            set_err(a, E_INJECTED, 10 * L, s);
            lds_st(ctl + C_ABORT, 1u);
            ok = false;
            break;
        }
        // ---------------- ln_f + LM head + argmax
        {
            float xf[R][EPL];
            float gg[EPL], bb[EPL], bp[EPL];
            if constexpr (big_d<D>()) {
                add_bias_xs<D, R>(xs, a.layers[L - 1].b_p, lane);
#pragma unroll
                for (int i = 0; i < EPL; ++i) bp[i] = 0.f;
            } else {
                load_ln<D>(a.lnf_g, a.lnf_b, gg, bb, lane);
#pragma unroll
                for (int i = 0; i < EPL; ++i) bp[i] = gl(a.layers[L - 1].b_p + lane + 64 * i);
            }
            if (!(ok = poll_resid<D, R>(sw + (2 * (L - 1) + 1) * sc.xw, a.exp_mlp, bp, xs, xf, a, ctl, 10 * L + 1, s,
                                        lane)))
                break;
            if constexpr (big_d<D>()) load_ln<D>(a.lnf_g, a.lnf_b, gg, bb, lane);
            if constexpr (!xf_from_poll<D, R>()) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int i = 0; i < EPL; ++i) xf[r][i] = fix2f(xs[r * D + lane + 64 * i]);
            }
            stamp(a, s, L, 0, lane);
            stamp_val(a, s, L, 26, __builtin_amdgcn_s_memtime());
            stamp_val(a, s, L, 27, wall_clock64());
            layer_norm<D, R>(xf, gg, bb, a.eps, xn, lane);
        }
        unsigned pid = pid_of(s, L, 0, L);
        lds_st(ctl + C_READY, pid);
        stamp(a, s, L, 1, lane);
        if (!(ok = wait_phdone(ctl, pid, a, s))) break;
        stamp(a, s, L, 2, lane);
        u64 best_all[R];
        if (a.argmax_slots) {
            // this CU's best key per row into a slot of its own, repacked as (ordered value : 32,
            // 65535 - token : 16, 1 : 16) -- the same order, never zero -- then every CU reads all G
            // slots of the (fresh per step) scratch until none is zero: one store and one polling
            // round trip, instead of an atomic max, its drain, a counter add and the counter poll
            // followed by a separate read of the result
            if (lane < R) {
                u64 best = 0;
#pragma unroll
                for (int w = 0; w < NC; ++w) {
                    const u64 k = keys[w * R + lane];
                    best = k > best ? k : best;
                }
                const u64 packed = best ? ((best >> 32) << 32) |
                                              ((u64)(0xffffu - ((~(unsigned)(best & 0xffffffffull)) & 0xffffu)) << 16) | 1ull
                                        : 1ull;
                gst64(sw + sc.kslots + (size_t)lane * 256 + blockIdx.x, packed);
            }
            stamp(a, s, L, 3, lane);
            const u64 t0 = clk();
            for (;;) {
                bool all = true;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    u64 m = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {  // G <= 256 slots over 64 lanes
                        const int c = lane + 64 * j;
                        const u64 k = c < G ? gld64(sw + sc.kslots + (size_t)r * 256 + c) : 1ull;
                        all &= k != 0ull;
                        m = k > m ? k : m;
                    }
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) {
                        const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)m, o);
                        const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(m >> 32), o);
                        const u64 k = ((u64)hi << 32) | lo;
                        m = k > m ? k : m;
                    }
                    best_all[r] = m;
                }
                if (__all(all)) break;
                if ((unsigned)__builtin_amdgcn_readfirstlane((int)gld32(a.err)) || lds_ld(ctl + C_ABORT)) {
                    lds_st(ctl + C_ABORT, 1u);
                    ok = false;
                    break;
                }
                if (clk() - t0 > TIMEOUT_TICKS) {
                    set_err(a, E_WAIT_CNT, 10 * L + 2, s);
                    lds_st(ctl + C_ABORT, 1u);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) break;
        } else {
            if (lane < R) {
                u64 best = 0;
#pragma unroll
                for (int w = 0; w < NC; ++w) {
                    const u64 k = keys[w * R + lane];
                    best = k > best ? k : best;
                }
                if (best) __hip_atomic_fetch_max(sw + sc.keys + lane, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            drain();
            if (lane == 0) gadd64(sw + sc.cnt0 + (2 * L) * SHARDS * CSTRIDE + shard * CSTRIDE, 1ull);
            stamp(a, s, L, 3, lane);
            if (!(ok = wait_count(sw + sc.cnt0 + (2 * L) * SHARDS * CSTRIDE, (u64)G, a, ctl, 10 * L + 2, s, lane))) break;
#pragma unroll
            for (int r = 0; r < R; ++r) best_all[r] = gld64(sw + sc.keys + r);
        }
        stamp(a, s, L, 4, lane);
        // ---------------- greedy bookkeeping (decode_update's semantics, replicated in every CU)
        bool any_live = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const u64 best = best_all[r];
            const int len0 = len[r];
            const int fin0 = fin[r];
            const int live_len = fin0 ? 0 : len0;
            int p = fin0 ? len0 - 1 : live_len;
            p = p < 0 ? 0 : (p < T - 1 ? p : T - 1);
            if (!fin0) {
                int t;
                if (a.argmax_slots)  // (value : 32, 65535 - token : 16, 1 : 16); 1 = no candidate anywhere
                    t = (best >> 16) ? (int)(0xffffu - (unsigned)((best >> 16) & 0xffffull)) : a.eos;
                else
                    t = best ? (int)(~(unsigned)(best & 0xffffffffull)) : a.eos;
                t = (t >= 0 && t < a.V) ? t : a.eos;
                if (blockIdx.x == 0 && lane == 0) a.out_tokens[(size_t)slot[r] * T + live_len] = t;
                // (this CU's LDS slice only: the global bitmap is updated at the commit, so an
                // aborted launch leaves every piece of row state as it found it)
                const int rel = t - cu.v0;
                if (rel >= 0 && rel < cu.nv && lane == 0) seen[r * a.swl + (rel >> 5)] |= 1u << (rel & 31);
                len[r] = live_len + 1;
                if (t == a.eos || live_len + 1 >= T) fin[r] = 1;
                tok[r] = t;
            }
            pos[r] = p;
            any_live |= !fin[r];
            if (lane == 0) {
                st[r * 8 + S_TOK] = tok[r];
                st[r * 8 + S_POS] = pos[r];
                st[r * 8 + S_FIN] = fin[r];
                st[r * 8 + S_LEN] = len[r];
            }
        }
        const bool cont = any_live && s + 1 < a.nsteps;
        lds_st(ctl + C_CONT, cont ? 1u : 0u);
        lds_st(ctl + C_READY, pid_of(s, L, 1, L));
        if (!cont) break;
    }
    // ---- commit (CU 0, only if it ran every step it started): decode_update's outputs incl. the
    // next embedding, and the generated tokens into the global penalty bitmap.  CU 0 passed every
    // step's argmax counter, so each token it holds saw all G CUs' keys; an aborted launch commits
    // nothing (the K/V rows and out_tokens entries it wrote lie beyond the committed lengths and
    // are rewritten by whatever runs these steps again).
    if (ok && blockIdx.x == 0) {
        drain();  // this wave's out_tokens stores, read back below
#pragma unroll
        for (int r = 0; r < R; ++r) {
            for (int i = lane; i < len[r] - len0[r]; i += 64) {
                const int t = (int)gld32(reinterpret_cast<const unsigned*>(a.out_tokens + (size_t)slot[r] * T + len0[r] + i));
                atomicOr(a.seen + (size_t)slot[r] * a.seen_words + (t >> 5), 1u << (t & 31));
            }
            if (lane == 0) {
                a.lens[slot[r]] = len[r];
                a.finished[slot[r]] = fin[r];
                a.cur_tok[slot[r]] = tok[r];
                a.cur_pos[slot[r]] = pos[r];
                a.cur_kvlen[slot[r]] = pos[r] + 1;
            }
            if (a.x_out) {
#pragma unroll
                for (int i = 0; i < EPL; ++i) {
                    const int e = lane + 64 * i;
                    a.x_out[(size_t)slot[r] * a.ldx + e] =
                        bf16_to_f32(a.wte[(size_t)tok[r] * D + e]) + bf16_to_f32(a.wpe[(size_t)pos[r] * D + e]);
                }
            }
        }
        if (lane == 0) {
            drain();
            __hip_atomic_store(a.err + 4, (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    lds_st(ctl + C_DONE, 1u);
}

// ------------------------------------------------------------------ loader waves
// NL waves stream this CU's row stream into the ring in batches of LB x 1 KiB LDS-DMA units (one
// global_load_lds_dwordx4 each); wave j issues batches j, j + NL, ..., keeping up to INFL units in
// flight, and publishes how many of ITS batches have landed.  A batch is issued only when every
// compute wave has released the ring bytes it overwrites.  (One wave issuing one unit per loop
// iteration capped the loader at ~10 GB/s per CU; the LM head's ~300 KB per CU per step needs
// far more in flight.)
constexpr int LB = 8;  // units per batch (the ring is a multiple of LB KiB)
constexpr unsigned BATCH = LB * 1024u;
template <int NT>
__device__ __forceinline__ void loader_wave(const Args& a, const Cu& cu, char* lds, const Lay& ly, int j, int lane) {
    unsigned* ctl = reinterpret_cast<unsigned*>(lds + ly.ctl);
    const unsigned RB = (unsigned)a.ring_bytes;
    const unsigned SB = (unsigned)cu.step_bytes;
    const unsigned total = SB * (unsigned)a.nsteps;  // host guarantees < 2^32
    const unsigned nbatch = (total + BATCH - 1) / BATCH;
    const char* base = reinterpret_cast<const char*>(a.packed) + cu.off;
    char* ring = lds + ly.ring;
    unsigned k = 0;          // this wave's batches issued (its batch k is global batch j + NL k)
    unsigned published = 0;  // ... and published as landed
    u64 t0 = clk();
    for (;;) {
        const unsigned b = (unsigned)j + NL * k;
        if (b >= nbatch) break;
        unsigned cons = 0xffffffffu;
#pragma unroll
        for (int w = 0; w < NC; ++w) {
            const unsigned c = lds_ld(ctl + C_CONS + w);
            cons = c < cons ? c : cons;
        }
        if ((b + 1) * BATCH > cons * 16u + RB || lds_ld(ctl + C_GATHER)) {  // ring full / a hand-off in progress
            drain();
            if (published != k) {
                published = k;
                lds_st(ctl + C_LOADED + j, k);
            }
            if (lds_ld(ctl + C_ABORT) || lds_ld(ctl + C_DONE)) break;
            if (clk() - t0 > TIMEOUT_TICKS) {
                set_err(a, E_LOADER, 0, 0);
                lds_st(ctl + C_ABORT, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        t0 = clk();
        unsigned gpos = (b * BATCH) % SB;
        unsigned rpos = (b * BATCH) % RB;
        // NT 1: every weight byte non-temporal; NT 2: the layers' bytes only, the LM-head rows (the
        // batch's start decides, a wave-uniform branch: one load per unit, the counted waits hold)
        // keep the default policy, so they may stay in the Infinity Cache from one token to the next
        const bool nt_here = NT == 1 || (NT == 2 && gpos < (unsigned)cu.lm_off);
#pragma unroll
        for (int u = 0; u < LB; ++u) {
            unsigned lo = gpos + (unsigned)lane * 16u;
            if (lo >= SB) lo -= SB;
            if (nt_here)
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + lo),
                                                 (__attribute__((address_space(3))) void*)(ring + rpos), 16, 0, 2);
            else
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + lo),
                                                 (__attribute__((address_space(3))) void*)(ring + rpos), 16, 0, 0);
            gpos += 1024u;
            if (gpos >= SB) gpos -= SB;
            rpos += 1024u;
        }
        ++k;
        if (k * LB >= (unsigned)INFL) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFL - LB) : "memory");  // INFL - LB units may stay in flight
            const unsigned done = k - (INFL - LB) / LB;
            if (done > published) {
                published = done;
                lds_st(ctl + C_LOADED + j, done);
            }
        }
    }
    drain();
    lds_st(ctl + C_LOADED + j, k);
}

// ------------------------------------------------------------------ compute waves
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;

// bytes of the stream landed in the ring: the prefix every loader wave has completed (wave j
// completed its first k_j batches = global batches j, j + NL, ...: batch b = j + NL m is in iff m < k_j)
__device__ __forceinline__ unsigned loaded_bytes(unsigned* ctl) {
    unsigned p = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        const unsigned b = (unsigned)j + NL * lds_ld(ctl + C_LOADED + j);
        p = b < p ? b : p;
    }
    return p * BATCH;
}
// wait until the stream bytes [.., end) are in the ring
__device__ __forceinline__ bool wait_loaded(unsigned* ctl, unsigned end, const Args& a, int s) {
    if (loaded_bytes(ctl) >= end) return true;
    const u64 t0 = clk();
    for (;;) {
        if (loaded_bytes(ctl) >= end) return true;
        if (lds_ld(ctl + C_ABORT)) return false;
        if (clk() - t0 > TIMEOUT_TICKS) {
            set_err(a, E_WAIT_LDS, 50, s);
            lds_st(ctl + C_ABORT, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// profiling variant: adds the ticks spent waiting for the ring to *acc
__device__ __forceinline__ bool wait_loaded_t(unsigned* ctl, unsigned end, const Args& a, int s, u64* acc,
                                              bool tracing) {
    if (!tracing || loaded_bytes(ctl) >= end) return wait_loaded(ctl, end, a, s);
    const u64 t0 = wall_clock64();
    const bool ok = wait_loaded(ctl, end, a, s);
    *acc += wall_clock64() - t0;
    return ok;
}

__device__ __forceinline__ unsigned ring_wrap(unsigned off, unsigned RB) { return off >= RB ? off - RB : off; }

// 16 row-major weight rows (ring offset gro of row 0) . the activation rows m < R (bf16 in LDS),
// over the 32-deep k chunks [c0, c0 + NCH): v_mfma_f32_16x16x32_bf16 with B = the rows as they sit
// in the ring (lane l: row l & 15, k 8 (l >> 4) .. + 8 of each chunk) and A = the activation
// (lane l: row min(l & 15, R - 1); output rows >= R are ignored, so they need no zeroing).
// Result: lane l < 16 holds row l's dot with activation m in acc[m].  Fragments are read in
// batches of up to 8 chunks before their MFMAs (sched_barrier: one LDS latency per batch), and
// alternate chunks accumulate in two chains so consecutive MFMAs do not wait on each other.
template <int D, int R, int NCH>
__device__ __forceinline__ f32x4_t mfma_rows16(const char* ring, unsigned gro, unsigned RB, const bf16_t* xnb, int c0,
                                               int lane) {
    constexpr int NCK = D / 32;
    constexpr int BT = NCH < 8 ? NCH : 8;
    const int n = lane & 15, kq = lane >> 4;
    const unsigned ro = ring_wrap(gro + (unsigned)n * ROW_BYTES(D), RB) + 16u * kq;
    const bf16_t* xr = xnb + (n < R ? n : R - 1) * D + 8 * kq;
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
    for (int b0 = 0; b0 < NCH; b0 += BT) {
        bf16x8_t bv[BT], av[BT];
#pragma unroll
        for (int j = 0; j < BT; ++j) {
            const int c = c0 + b0 + j;
            const int cc = c < NCK ? c : NCK - 1;  // (ragged last batch: a valid read, zero A below)
            bv[j] = *reinterpret_cast<const bf16x8_t*>(ring + ring_wrap(ro + 64u * cc, RB));
            av[j] = *reinterpret_cast<const bf16x8_t*>(xr + 32 * cc);
            if (b0 + j >= NCH || c >= NCK) av[j] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < BT; ++j) {
            if (j & 1)
                acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[j], bv[j], acc1, 0, 0, 0);
            else
                acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[j], bv[j], acc0, 0, 0, 0);
        }
    }
    return acc0 + acc1;
}

// this wave's 16-row output tiles t = w, w + NC, ... (t < ntiles) of a K-major block [16 ntiles][KP]
// at ring offset bro (bro < RB): out[m][o0 + 16 t + l] = sum_k A[m][k] * Blk[16 t + l][k]
// (v_mfma_f32_16x16x16_bf16 per 16-deep k block; afr[kb]: this lane's A fragment, row l & 15,
// k = 16 kb + 4 (l >> 4) .. + 4); results go to part[m][o0 + ..] (lanes < 16).
// Tiles go U = 3 at a time with every B fragment of the group read before its MFMAs, and NO
// branch between those reads: a tile index past the end is clamped to the last tile (a valid
// ring address, its result discarded) -- a branch per read made the compiler wait for each
// (s_waitcnt lgkmcnt(0) at every join) and serialised the whole block (r4 trace: W_o 1.4 -> 4.8 us);
// NKB is a template constant for the same reason.  A whole-block unroll kept D / 64 f32x4
// accumulators live and pushed the kernel past 256 VGPRs into scratch.  Offsets stay below
// 2 RB (a block is smaller than the ring), so one conditional subtract wraps them.
template <int D, int R, int NKB, int U = 3>
__device__ __forceinline__ void mfma_block_k(const char* ring, unsigned bro, unsigned RB, int KP, int ntiles, int o0,
                                             const bf16x4_t* afr, float* part, int w, int lane) {
    const int n = lane & 15, kq = lane >> 4;
    const unsigned base = bro + (unsigned)((16 * w + n) * KP + 4 * kq) * 2u;
    const unsigned tstep = (unsigned)(16 * NC * KP) * 2u;
    const int mine = ntiles > w ? (ntiles - 1 - w) / NC + 1 : 0;  // tiles of this wave (uniform)
    for (int j = 0; j < mine; j += U) {
        bf16x4_t b[U][NKB];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int jj = j + u < mine ? j + u : mine - 1;
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
                b[u][kb] = *reinterpret_cast<const bf16x4_t*>(ring + ring_wrap(base + tstep * jj + 32u * kb, RB));
        }
        f32x4_t acc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(afr[kb], b[u][kb], acc[u], 0, 0, 0);
        if (lane < 16) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (j + u < mine) {
#pragma unroll
                    for (int r = 0; r < R; ++r) part[r * D + o0 + 16 * (w + NC * (j + u)) + lane] = acc[u][r];
                }
        }
    }
}

template <int D, int R, int KB>
__device__ __forceinline__ void mfma_block(const char* ring, unsigned bro, unsigned RB, int KP, int nkb, int ntiles,
                                           int o0, const bf16x4_t (&afr)[KB], float* part, int w, int lane) {
    static_assert(KB == 4, "k blocks");
    switch (nkb) {  // (uniform: the block's K from the host table)
        case 1: mfma_block_k<D, R, 1>(ring, bro, RB, KP, ntiles, o0, afr, part, w, lane); break;
        case 2: mfma_block_k<D, R, 2>(ring, bro, RB, KP, ntiles, o0, afr, part, w, lane); break;
        case 3: mfma_block_k<D, R, 3>(ring, bro, RB, KP, ntiles, o0, afr, part, w, lane); break;
        default: mfma_block_k<D, R, 4>(ring, bro, RB, KP, ntiles, o0, afr, part, w, lane); break;
    }
}

// A fragments of a bf16 vector staged in this wave's LDS slot hb[R][64] (row m = lane & 15; rows
// m >= R and k >= nvalid are zero): fragment kb holds k = 16 kb + 4 (lane >> 4) .. + 4, read at hb
// column k0 + k
template <int KB, int R>
__device__ __forceinline__ void load_afr(const bf16_t* hb, int k0, int nvalid, int nkb, bf16x4_t (&afr)[KB],
                                         int lane) {
    // every read unconditional (row clamped, k blocks past the end read LDS that lies further
    // on and are masked to zero) so the reads issue back to back; masking by select, no branch
    const int m = lane & 15, kq = lane >> 4;
    const bf16_t* row = hb + (m < R ? m : R - 1) * 64 + k0 + 4 * kq;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
        const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(row + 16 * kb);
        bf16x4_t z;
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = (kb < nkb && m < R && 16 * kb + 4 * kq + j < nvalid) ? v[j] : (short)0;
        afr[kb] = z;
    }
}

// online-softmax state of one lane (8 dims of one position group) and its update
struct OnlineS {
    float m, l, o[8];
};
__device__ __forceinline__ void os_init(OnlineS& z) {
    z.m = -INFINITY;
    z.l = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) z.o[j] = 0.f;
}
__device__ __forceinline__ void os_add(OnlineS& z, float s, bool valid, const float (&v)[8]) {
    if (!valid) return;
    const float mn = fmaxf(z.m, s);
    const float corr = z.m == -INFINITY ? 0.f : __expf(z.m - mn);
    const float p = __expf(s - mn);
    z.l = z.l * corr + p;
#pragma unroll
    for (int j = 0; j < 8; ++j) z.o[j] = z.o[j] * corr + p * v[j];
    z.m = mn;
}
__device__ __forceinline__ void os_merge(OnlineS& z, float m2, float l2, const float (&o2)[8]) {
    const float mn = fmaxf(z.m, m2);
    const float a1 = z.m == -INFINITY ? 0.f : __expf(z.m - mn);
    const float a2 = m2 == -INFINITY ? 0.f : __expf(m2 - mn);
    z.l = z.l * a1 + l2 * a2;
#pragma unroll
    for (int j = 0; j < 8; ++j) z.o[j] = z.o[j] * a1 + o2[j] * a2;
    z.m = mn;
}

template <int D, int R, int PFG>
__device__ __forceinline__ void compute_wave(const Args& a, const Cu& cu, char* lds, const Lay& ly, int w, int lane) {
    constexpr int KBMAX = 4;  // k blocks of 16 per K-major block (K <= 64: a head, a slice)
    unsigned* ctl = reinterpret_cast<unsigned*>(lds + ly.ctl);
    const int* st = reinterpret_cast<const int*>(lds + ly.st);
    const bf16_t* xnb = reinterpret_cast<const bf16_t*>(lds + ly.xn);
    float* res = reinterpret_cast<float*>(lds + ly.res);
    float* part = reinterpret_cast<float*>(lds + ly.part);
    float* fcp = reinterpret_cast<float*>(lds + ly.fcp);
    const float* att = reinterpret_cast<const float*>(lds + ly.att);
    float* mrg = reinterpret_cast<float*>(lds + ly.mrg);
    const unsigned* seen = reinterpret_cast<const unsigned*>(lds + ly.seen);
    u64* keys = reinterpret_cast<u64*>(lds + ly.keys);
    bf16_t* hb = reinterpret_cast<bf16_t*>(lds + ly.hb) + w * R * 64;
    const char* ring = lds + ly.ring;
    // every argument the loops touch, read once (kernel-argument reloads inside the loops cost a
    // scalar round trip each under SGPR pressure)
    const unsigned RB = (unsigned)a.ring_bytes;
    const int L = a.L, H = a.H, T = a.T, V = a.V, swl = a.swl, rs = a.max_nq + 16, nsteps = a.nsteps;
    const int KO = a.ko, KF = a.kf;
    const float penalty = a.penalty;
    const bool tracing = a.trace != nullptr;
    const Layer* layers = a.layers;
    const int nq = cu.nq, nf = cu.nf, nv = cu.nv, ah = cu.ah, v0 = cu.v0, f0 = cu.f0;
    const int ao0 = cu.ao0, aon = cu.aon, pd0 = cu.pd0, pdn = cu.pdn;
    constexpr unsigned ROWB = ROW_BYTES(D);
    const unsigned ko_bytes = ah >= 0 ? (unsigned)(aon * KO * 2) : 0u;
    const unsigned kf_bytes = (unsigned)(pdn * KF * 2);
    const unsigned layer_bytes = (unsigned)(nq + nf) * ROWB + ko_bytes + kf_bytes;
    const unsigned SB = (unsigned)cu.step_bytes;
    const int ts = lane >> 3, ck = lane & 7;
    const int n16 = lane & 15;
    constexpr int NCK = D / 32;                     // 32-deep k chunks of a row
    constexpr int CPW = (NCK + NC - 1) / NC;        // K split of the QKV / c_fc dot products
    const int cw0 = w * CPW;

    for (int s = 0; s < nsteps; ++s) {
        // step start: row state for this step is in LDS
        if (s > 0) {
            if (!lds_wait_ge(ctl, C_READY, pid_of(s - 1, L, 1, L), a, 60, s)) return;
            if (!lds_ld(ctl + C_CONT)) return;
        } else if (!lds_wait_ge(ctl, C_READY, pid_of(0, 0, 0, L), a, 61, s)) {
            return;
        }
        asm volatile("" ::: "memory");
        int pos[R], slot[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            pos[r] = st[r * 8 + S_POS];
            slot[r] = st[r * 8 + S_SLOT];
        }
        const unsigned sbase = (unsigned)s * SB;
        for (int l = 0; l < L; ++l) {
            const Layer lw = layers[l];
            const unsigned lbase = sbase + (unsigned)l * layer_bytes;
            const unsigned obase = lbase + (unsigned)nq * ROWB;          // W_o block [aon][KO]
            const unsigned fbase = obase + ko_bytes;                     // c_fc rows
            const unsigned pbase = fbase + (unsigned)nf * ROWB;          // c_proj block [pdn][KF]
            u64 ringwait = 0;
            // ---- attention CU: prefetch this layer's cached K/V of the head (independent of q)
            uint4 kpf[R][PFG], vpf[R][PFG];
            int t0[R], t1[R];
            if (ah >= 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int per = (pos[r] + NC - 1) / NC;
                    t0[r] = w * per;
                    t1[r] = min(pos[r], t0[r] + per);
                    const size_t hbase = ((size_t)slot[r] * H + ah) * T;
#pragma unroll
                    for (int g = 0; g < PFG; ++g) {
                        const int t = t0[r] + 8 * g + ts;
                        if (t < t1[r]) {
                            kpf[r][g] = gl(reinterpret_cast<const uint4*>(lw.k_cache + (hbase + t) * 64 + ck * 8));
                            vpf[r][g] = gl(reinterpret_cast<const uint4*>(lw.v_cache + (hbase + t) * 64 + ck * 8));
                        } else {
                            kpf[r][g] = make_uint4(0u, 0u, 0u, 0u);
                            vpf[r][g] = make_uint4(0u, 0u, 0u, 0u);
                        }
                    }
                }
            }
            // c_fc bias of intermediate column `lane`
            const float bfc = lane < nf ? gl(lw.b_fc + f0 + lane) : 0.f;
            // ---------------- phase 0: QKV dot products, 16-row groups g = w, w + NC, ...
            unsigned pid = pid_of(s, l, 0, L);
            if (!lds_wait_ge(ctl, C_READY, pid, a, 62, s)) return;
            asm volatile("" ::: "memory");
            if (w == 0) stamp(a, s, l, 16, lane);
            // (K split: wave w takes k chunks [w CPW, (w + 1) CPW) of every row; the comm wave sums
            // the NC partials in a fixed order)
            if (!wait_loaded_t(ctl, obase, a, s, &ringwait, tracing)) return;
            asm volatile("" ::: "memory");
            for (int g = 0; 16 * g < nq; ++g) {
                const int rows = min(16, nq - 16 * g);
                const f32x4_t acc =
                    mfma_rows16<D, R, CPW>(ring, (lbase + (unsigned)(16 * g) * ROWB) % RB, RB, xnb, cw0, lane);
                if (lane < rows) {
#pragma unroll
                    for (int r = 0; r < R; ++r) res[(w * R + r) * rs + 16 * g + lane] = acc[r];
                }
            }
            if (w == 0) stamp(a, s, l, 17, lane);
            lds_st(ctl + C_CONS + w, obase >> 4);
            lds_st(ctl + C_PHDONE + w, pid);
            // ---------------- phase 1: attention + this CU's W_o block
            if (ah >= 0) {
                pid = pid_of(s, l, 1, L);
                if (!lds_wait_ge(ctl, C_READY, pid, a, 63, s)) return;
                asm volatile("" ::: "memory");
                if (w == 0) stamp(a, s, l, 18, lane);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float q[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) q[j] = att[(r * 3 + 0) * 64 + ck * 8 + j] * 0.125f;
                    OnlineS z;
                    os_init(z);
                    const int ng = (t1[r] - t0[r] + 7) >> 3;
                    const size_t hbase = ((size_t)slot[r] * H + ah) * T;
#pragma unroll
                    for (int g = 0; g < PFG; ++g) {  // prefetched groups
                        if (g >= ng) break;
                        const int t = t0[r] + 8 * g + ts;
                        float kf[8], vf[8];
                        unpack8(kpf[r][g], kf);
                        unpack8(vpf[r][g], vf);
                        float sdot = 0.f;
#pragma unroll
                        for (int j = 0; j < 8; ++j) sdot += q[j] * kf[j];
                        sdot = group8_sum(sdot);
                        os_add(z, sdot, t < t1[r], vf);
                    }
                    for (int g = PFG; g < ng; ++g) {  // long caches: the rest straight from the cache
                        const int t = t0[r] + 8 * g + ts;
                        const bool valid = t < t1[r];
                        uint4 kk = make_uint4(0u, 0u, 0u, 0u), vv = kk;
                        if (valid) {
                            kk = gl(reinterpret_cast<const uint4*>(lw.k_cache + (hbase + t) * 64 + ck * 8));
                            vv = gl(reinterpret_cast<const uint4*>(lw.v_cache + (hbase + t) * 64 + ck * 8));
                        }
                        float kf[8], vf[8];
                        unpack8(kk, kf);
                        unpack8(vv, vf);
                        float sdot = 0.f;
#pragma unroll
                        for (int j = 0; j < 8; ++j) sdot += q[j] * kf[j];
                        sdot = group8_sum(sdot);
                        os_add(z, sdot, valid, vf);
                    }
                    if (w == NC - 1) {  // the current position: k/v from the granules
                        float kf[8], vf[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            kf[j] = att[(r * 3 + 1) * 64 + ck * 8 + j];
                            vf[j] = att[(r * 3 + 2) * 64 + ck * 8 + j];
                        }
                        float sdot = 0.f;
#pragma unroll
                        for (int j = 0; j < 8; ++j) sdot += q[j] * kf[j];
                        sdot = group8_sum(sdot);
                        os_add(z, sdot, ts == 0, vf);
                    }
                    // merge the 8 position lanes (xor 8, 16, 32) of each dim chunk
#pragma unroll
                    for (int o = 8; o <= 32; o <<= 1) {
                        float m2, l2, o2[8];
                        m2 = __shfl_xor(z.m, o, 64);
                        l2 = __shfl_xor(z.l, o, 64);
#pragma unroll
                        for (int j = 0; j < 8; ++j) o2[j] = __shfl_xor(z.o[j], o, 64);
                        os_merge(z, m2, l2, o2);
                    }
                    float* mb = mrg + (w * R + r) * 68;
                    if (lane < 8) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) mb[lane * 8 + j] = z.o[j];
                    }
                    if (lane == 0) {
                        mb[64] = z.m;
                        mb[65] = z.l;
                    }
                }
                if (w == 0) stamp(a, s, l, 19, lane);
                lds_st(ctl + C_MID + w, pid);
#pragma unroll
                for (int w2 = 0; w2 < NC; ++w2)
                    if (!lds_wait_ge(ctl, C_MID + w2, pid, a, 64, s)) return;
                asm volatile("" ::: "memory");
                if (w == 0) stamp(a, s, l, 20, lane);
                // merged attention output (lane d: head dim d), staged bf16 as the A operand
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float m = -INFINITY;
#pragma unroll
                    for (int w2 = 0; w2 < NC; ++w2) m = fmaxf(m, mrg[(w2 * R + r) * 68 + 64]);
                    float lsum = 0.f, osum = 0.f;
#pragma unroll
                    for (int w2 = 0; w2 < NC; ++w2) {
                        const float* mb = mrg + (w2 * R + r) * 68;
                        const float mw = mb[64];
                        const float e = mw == -INFINITY ? 0.f : __expf(mw - m);
                        lsum += mb[65] * e;
                        osum += mb[lane] * e;
                    }
                    hb[r * 64 + lane] = f32_to_bf16(osum / lsum);  // head dim lane: the A operand of W_o
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bf16x4_t afr[KBMAX];
                const int nkb = KO / 16;
                load_afr<KBMAX, R>(hb, cu.ak0, cu.akn, nkb, afr, lane);  // this CU's head dims
                if (!wait_loaded_t(ctl, fbase, a, s, &ringwait, tracing)) return;  // the whole W_o block
                asm volatile("" ::: "memory");
                mfma_block<D, R, KBMAX>(ring, obase % RB, RB, KO, nkb, aon / 16, ao0, afr, part, w, lane);
                if (w == 0) stamp(a, s, l, 21, lane);
                lds_st(ctl + C_CONS + w, fbase >> 4);
                lds_st(ctl + C_PHDONE + w, pid);
            }
            // ---------------- phase 2: MLP -- every wave computes all of this CU's c_fc rows (a
            // handful of MFMA groups), then its own 16-column tiles of the c_proj block
            pid = pid_of(s, l, 2, L);
            if (!lds_wait_ge(ctl, C_READY, pid, a, 65, s)) return;
            asm volatile("" ::: "memory");
            if (w == 0) stamp(a, s, l, 22, lane);
            {
                if (!wait_loaded_t(ctl, pbase, a, s, &ringwait, tracing)) return;  // the c_fc rows
                asm volatile("" ::: "memory");
                const unsigned fro = fbase % RB;
#pragma unroll
                for (int g = 0; g < KBMAX; ++g) {  // K split, as for QKV
                    if (16 * g >= KF) break;
                    const f32x4_t acc =
                        mfma_rows16<D, R, CPW>(ring, ring_wrap(fro + ((unsigned)(16 * g) * ROWB) % RB, RB), RB, xnb, cw0,
                                               lane);
                    if (lane < 16) {
#pragma unroll
                        for (int r = 0; r < R; ++r) fcp[(w * R + r) * 64 + 16 * g + lane] = acc[r];
                    }
                }
                // (done with the c_fc rows: the loader may overwrite them with the c_proj block, so
                // the ring needs room for the larger of the two, not both -- GPT-2-large / XL)
                lds_st(ctl + C_CONS + w, pbase >> 4);
                lds_st(ctl + C_MID + w, pid);
#pragma unroll
                for (int w2 = 0; w2 < NC; ++w2)
                    if (!lds_wait_ge(ctl, C_MID + w2, pid, a, 67, s)) return;
                asm volatile("" ::: "memory");
                // h = bf16(gelu(sum of the partials + b_fc)), lane i = intermediate column i
                if (lane < KF) {
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        float hsum = 0.f;
#pragma unroll
                        for (int w2 = 0; w2 < NC; ++w2) hsum += fcp[(w2 * R + r) * 64 + lane];
                        hb[r * 64 + lane] = lane < nf ? f32_to_bf16(gelu_tanh(hsum + bfc)) : (bf16_t)0;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bf16x4_t afr[KBMAX];
                const int nkb = KF / 16;
                load_afr<KBMAX, R>(hb, 0, nf, nkb, afr, lane);
                if (!wait_loaded_t(ctl, pbase + kf_bytes, a, s, &ringwait, tracing)) return;
                asm volatile("" ::: "memory");
                mfma_block<D, R, KBMAX>(ring, pbase % RB, RB, KF, nkb, pdn / 16, pd0, afr, part, w, lane);
                if (w == 0) stamp(a, s, l, 23, lane);
                if (w == 0 && lane == 0) stamp_val(a, s, l, 12, ringwait);
                lds_st(ctl + C_CONS + w, (pbase + kf_bytes) >> 4);
                lds_st(ctl + C_PHDONE + w, pid);
            }
        }
        // ---------------- LM head rows: 16-row groups g = w, w + NC, ...: penalty + argmax keys
        {
            const unsigned pid = pid_of(s, L, 0, L);
            if (!lds_wait_ge(ctl, C_READY, pid, a, 66, s)) return;
            asm volatile("" ::: "memory");
            u64 best[R];
            u64 ringwait = 0;
#pragma unroll
            for (int r = 0; r < R; ++r) best[r] = 0ull;
            const unsigned vbase = sbase + (unsigned)L * layer_bytes;
            for (int g = w; 16 * g < nv; g += NC) {
                const int rows = min(16, nv - 16 * g);
                const unsigned end = vbase + (unsigned)(16 * g + rows) * ROWB;
                // everything before this group is done with (this wave's earlier groups, and the
                // other waves' groups are theirs): releasing it before the wait lets the loader run
                // ahead by the whole ring, so a window of ONE 16-row group suffices (XL: 4 groups of
                // 3.2 KB rows would not fit)
                lds_st(ctl + C_CONS + w, (vbase + (unsigned)(16 * g) * ROWB) >> 4);
                if (!wait_loaded_t(ctl, end, a, s, &ringwait, tracing)) return;
                asm volatile("" ::: "memory");
                const f32x4_t acc = mfma_rows16<D, R, NCK>(ring, (vbase + (unsigned)(16 * g) * ROWB) % RB, RB, xnb, 0, lane);
                lds_st(ctl + C_CONS + w, end >> 4);
                const int i = 16 * g + n16;
                const int v = v0 + i;
                if (lane < 16 && i < nv && v < V) {
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        float x = acc[r];
                        if ((seen[r * swl + (i >> 5)] >> (i & 31)) & 1u) x = x < 0.f ? x * penalty : x / penalty;
                        const u64 key = ((u64)f32_ordered(x) << 32) | (u64)(~(unsigned)v);
                        best[r] = key > best[r] ? key : best[r];
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) best[r] = wave_max_u64(best[r]);
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) keys[w * R + r] = best[r];
                if (w == 0) stamp_val(a, s, L, 12, ringwait);
            }
            lds_st(ctl + C_CONS + w, (vbase + (unsigned)nv * ROWB) >> 4);
            lds_st(ctl + C_PHDONE + w, pid);
        }
    }
}

template <int D, int R, int PFG>
__global__ __launch_bounds__(NTHREADS, 1) void dataflow_decode_kernel(Args a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // the wave index as a wave-uniform (scalar) value: every role branch and every "this wave's
    // tiles" loop bound derived from it is then a scalar branch, not an exec mask (a VGPR-derived
    // bound made mfma_block's tile loop exec-masked and serialised its LDS reads: r4 trace)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const Cu cu = a.cus[blockIdx.x];
    const Lay ly = lds_layout(D, R, a.max_nq, a.swl, a.ring_bytes);
    unsigned* ctl = reinterpret_cast<unsigned*>(smem + ly.ctl);
    if (threadIdx.x < 64) ctl[threadIdx.x] = 0u;
    __syncthreads();  // the only workgroup barrier: control words zeroed before any role starts
    if (wave == 0) {
        comm_wave<D, R>(a, cu, smem, ly, lane);
    } else if (wave <= NL) {
        if (a.nt_weights == 1)
            loader_wave<1>(a, cu, smem, ly, wave - 1, lane);
        else if (a.nt_weights == 2)
            loader_wave<2>(a, cu, smem, ly, wave - 1, lane);
        else
            loader_wave<0>(a, cu, smem, ly, wave - 1, lane);
    } else {
        compute_wave<D, R, PFG>(a, cu, smem, ly, wave - 1 - NL, lane);
    }
}

}  // namespace df

extern "C" int dlms_df_args_size() { return (int)sizeof(df::Args); }
extern "C" int dlms_df_cu_size() { return (int)sizeof(df::Cu); }
extern "C" int dlms_df_layer_size() { return (int)sizeof(df::Layer); }

// LDS bytes a launch needs besides the ring, and the scratch words per step
extern "C" int dlms_df_lds_fixed(int D, int R, int max_nq, int swl) { return df::lds_layout(D, R, max_nq, swl, 0).total; }
extern "C" long long dlms_df_step_words(int R, int D, int L, int C) { return df::scratch_layout(R, D, L, C).words; }
extern "C" int dlms_df_threads() { return df::NTHREADS; }
extern "C" int dlms_df_copies() { return df::COPIES; }

// Every workgroup spins on the others, so the whole grid must be resident at once.  The launcher
// checks that the device can hold it (occupancy x CUs >= grid; -2 = "cannot", the host then serves
// the launch-per-op path); the bounded waits + commit-only row state are the last line (an aborted
// launch changes nothing the next launch reads).  A plain launch: hipLaunchCooperativeKernel gives
// the same residency (MI355X_MICROARCH.md "coop-launch") and reserves nothing against other
// processes either, but measured +1.1 ms per query behind a 1024-query generation on the same
// engine -- its queue hand-over held the preceding prefill's completion (prefill 0.7 -> 1.8 ms,
// profiles/r5_prefill_b1_coop_probe.jsonl).
constexpr int DF_NOT_RESIDENT = -2;
constexpr int DF_MAX_DEVICES = 64;
template <int D, int R, int PFG>
static int df_launch(df::Args a, int grid, int lds, hipStream_t stream) {
    auto k = &df::dataflow_decode_kernel<D, R, PFG>;
    static int fits_grid[DF_MAX_DEVICES];  // per device: the most workgroups it holds at once (0: not queried)
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= DF_MAX_DEVICES) return (int)hipErrorInvalidDevice;
    if (fits_grid[dev] <= 0) {
        if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     df::LDS_MAX)) != hipSuccess)
            return (int)e;
        int cus = 0, per_cu = 0;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return (int)e;
        // (occupancy at the largest LDS any launch of this instantiation asks for)
        if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k), df::NTHREADS,
                                                              df::LDS_MAX)) != hipSuccess)
            return (int)e;
        fits_grid[dev] = per_cu * cus > 0 ? per_cu * cus : -1;
    }
    if (grid > fits_grid[dev]) return DF_NOT_RESIDENT;
    hipLaunchKernelGGL(k, dim3(grid), dim3(df::NTHREADS), lds, stream, a);
    return (int)hipGetLastError();
}

extern "C" int dlms_dataflow_decode(const df::Args* args, int grid, hipStream_t stream) {
    const df::Args& a = *args;
    const int lds = df::lds_layout(a.D, a.R, a.max_nq, a.swl, a.ring_bytes).total;
    if (lds > df::LDS_MAX || a.ring_bytes % df::BATCH || a.ring_bytes < 8 * 1024 || grid <= 0 || a.R < 1 || a.R > 2 ||
        a.H * 64 != a.D || a.max_nq > 64 || a.ko % 16 || a.kf % 16 || a.ko > 64 || a.kf > 64 || a.kf < 16 || a.nsteps <= 0 || a.C != df::COPIES || a.A < 1 || a.A > grid)
        return (int)hipErrorInvalidValue;
#define DF_CASE(DD)                                                                           \
    if (a.D == DD) return a.R == 1 ? df_launch<DD, 1, 5>(a, grid, lds, stream)                 \
                                   : df_launch<DD, 2, 3>(a, grid, lds, stream);
    DF_CASE(128)
    DF_CASE(256)
    DF_CASE(768)
    DF_CASE(1024)
    // (d 1280 / 1600 -- GPT-2-large / XL -- were built and oracle-tested in round 4 but measured slower
    // than launch-per-op, 152 / 306 vs 128.5 / 218 ms per query with 11 / 76 spilled VGPRs
    // (docs/PERFORMANCE.md round 4); the instantiations are removed)
#undef DF_CASE
    return (int)hipErrorInvalidValue;
}
