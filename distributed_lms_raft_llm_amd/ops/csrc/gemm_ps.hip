// Decode GEMM for the throughput path (M = 64..1024 rows): activation panel resident in LDS,
// PRE-SHUFFLED weights streamed straight into MFMA B-operand registers.
//
//   C[M, N] = A[M, K] . W[N, K]^T,  W stored by ops.shuffle_weight as [N/16][K/32][64 lanes][8]
//
// Why not the LDS-DMA ring of gemm.hip: at K = d = 768 the tiled kernel is bound by the per-CU
// LDS-DMA fill rate (~55-60 GB/s per CU, profiles/r1_gemm_lab/README.md) of BOTH operands.  Here:
//  * each workgroup (8 waves) loads its BM x Kc activation panel ONCE into LDS (global_load_lds,
//    one row per 1-1.5 KiB of instructions; 32-B row padding makes the 16-row A-fragment reads
//    bank-conflict free) and keeps it for every column tile it computes;
//  * every wave streams its own weight columns: one wave-instruction = one contiguous KiB = one
//    16x32 B fragment of v_mfma_f32_16x16x32_bf16, double-buffered in registers chunk by chunk
//    (KBC k-blocks), no LDS and no barrier in the main loop, so the 2 waves per SIMD drift apart
//    and one's loads hide under the other's MFMAs;
//  * a wave owns NT 16-column groups x all MT 16-row tiles, so each A fragment read from LDS
//    feeds NT MFMAs and each B fragment feeds MT.
// Persistent over N: wave slot s of the grid computes column tiles s, s + slots, ... (the LM head's
// 50k columns), with the repetition-penalty + argmax epilogue folded into a running per-row key.
//
// Epilogues (column tiles staged through a wave-private LDS region -> 16-B row stores):
//   EPI_BF16 / EPI_GELU_TANH (bf16 out), EPI_QKV (q + K/V cache scatter), EPI_PARTIAL (split-K f32
//   slab: grid carries split_k K slices), EPI_ARGMAX (one key per (row, wave slot)).
#include "common.h"

enum { PS_BF16 = 0, PS_GELU_TANH = 1, PS_QKV = 4, PS_ARGMAX = 5, PS_PARTIAL = 6 };

typedef __attribute__((address_space(3))) void ps_lds_void_t;
typedef __attribute__((address_space(1))) void ps_glob_void_t;

#define PS_NW 8        // waves per workgroup
#define PS_KBC 4       // k-blocks (32 deep) per register chunk
#define PS_PAD 32      // LDS row padding (bytes): 8-bank shift per row -> conflict-free fragments
#define PS_STAGE 4096  // wave-private epilogue staging bytes

template <int EPI, int MT, int NT, int KBC = PS_KBC, int NB = 0>
__global__ __launch_bounds__(64 * PS_NW) void gemm_ps_kernel(const bf16_t* __restrict__ A, int lda,
                                                           const bf16_t* __restrict__ Wsh, int M, int N, int K,
                                                           int row_blocks, int split, int col_wgs, GemmEpi ep) {
    constexpr int BM = 16 * MT;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4, fr = lane & 15;

    // block -> (row block, K slice, column workgroup); consecutive ids share W columns (one XCD)
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % row_blocks;
    const int rest = bid / row_blocks;
    const int ks = rest % split;
    const int cw = rest / split;
    const int kc = K / split;          // K slice of this block
    const int nkb = kc >> 5;           // its k-blocks
    const int nch = nkb / KBC;      // register chunks per column tile
    const int m0 = rb * BM;
    const int row_bytes = kc * 2 + PS_PAD;

    // ---- activation panel -> LDS (rows >= M read a clamped valid row; never stored) ----
    {
        const int pieces = (kc * 2 + 1023) >> 10;  // 1-KiB LDS-DMA instructions per row
        const int tail_lanes = ((kc * 2) & 1023) >> 4;
        for (int p = wave; p < BM * pieces; p += PS_NW) {
            const int r = p / pieces, pc = p - r * pieces;
            const int gm = m0 + r < M ? m0 + r : M - 1;
            const bool partial = pc == pieces - 1 && tail_lanes != 0;
            if (!partial || lane < tail_lanes) {
                const char* src = reinterpret_cast<const char*>(A + (size_t)gm * lda + (size_t)ks * kc) + pc * 1024 + lane * 16;
                __builtin_amdgcn_global_load_lds((ps_glob_void_t*)src, (ps_lds_void_t*)(smem + r * row_bytes + pc * 1024),
                                                 16, 0, 0);
            }
        }
    }

    // ---- this wave's column tiles ----
    const int tiles = N / (16 * NT);
    const int slot = cw * PS_NW + wave;
    const int slots = col_wgs * PS_NW;
    const int my_tiles = slot < tiles ? (tiles - 1 - slot) / slots + 1 : 0;
    const int nsteps = my_tiles * nch;
    // fragment (column group cg, k-block kb) of this K slice
    const int kb_base = ks * nkb;
    const int nkb_all = K >> 5;
    auto frag_ptr = [&](int step, int kb, int t) {
        const int tile = slot + (step / nch) * slots;
        const int cg = tile * NT + t;
        const int kbi = kb_base + (step % nch) * KBC + kb;
        return reinterpret_cast<const bf16x8_t*>(Wsh) + ((size_t)cg * nkb_all + kbi) * 64 + lane;
    };
    // steps past the end re-load the last one (static load counts keep every vmcnt wait counted)
    auto load = [&](bf16x8_t (&b)[KBC][NT], int step_) {
        const int step = step_ < nsteps ? step_ : nsteps - 1;
#pragma unroll
        for (int kb = 0; kb < KBC; ++kb)
#pragma unroll
            for (int t = 0; t < NT; ++t) b[kb][t] = *frag_ptr(step, kb, t);
    };

    f32x4_t acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[i][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    // argmax: running best key per (row tile, register row) of this lane
    unsigned long long best[EPI == PS_ARGMAX ? MT : 1][4];
#pragma unroll
    for (int i = 0; i < (EPI == PS_ARGMAX ? MT : 1); ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) best[i][r] = 0ull;

    char* stage = smem + BM * row_bytes + wave * PS_STAGE;

    auto finish_tile = [&](int step, unsigned int swl, unsigned int swl2) {
        const int tile = slot + (step / nch) * slots;
        const int col0 = tile * NT * 16;  // first column of the tile
        if constexpr (EPI == PS_ARGMAX) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // the tile's (<= 32) columns share one seen-bitmap word per row; lane (g, 4i + r)
                    // loaded the word of row 16i + 4g + r
                    // (row tiles 4.. of an 80-row panel: the second word, swl2)
                    const unsigned int bits = i < 4 ? __shfl(swl, g * 16 + 4 * i + r, 64)
                                                    : __shfl(swl2, g * 16 + 4 * (i - 4) + r, 64);
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        const int gcol = col0 + 16 * t + fr + ep.col_offset;
                        float v = acc[i][t][r];
                        if ((bits >> (gcol & 31)) & 1u) v = v < 0.f ? v * ep.penalty : v / ep.penalty;
                        const unsigned long long key =
                            ((unsigned long long)f32_ordered(v) << 32) | (unsigned long long)(~(unsigned int)gcol);
                        if (gcol < ep.vocab && key > best[i][r]) best[i][r] = key;
                    }
                }
        } else {
            // stage the BM x (16 NT) tile in the wave's LDS region, then 16-B row stores
            constexpr int OB = EPI == PS_PARTIAL ? 4 : 2;
            constexpr int TW = 16 * NT * OB;        // bytes per staged row
            constexpr int RPP = PS_STAGE / TW;      // rows per staging pass
            constexpr int PASSES = (BM + RPP - 1) / RPP;
            static_assert(RPP >= 16 && RPP % 16 == 0, "staging pass holds whole 16-row tiles");
            const int ncols = 16 * NT;
#pragma unroll
            for (int ps = 0; ps < PASSES; ++ps) {
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    if (16 * i < ps * RPP || 16 * i >= (ps + 1) * RPP) continue;
#pragma unroll
                    for (int t = 0; t < NT; ++t) {
                        const int col = col0 + 16 * t + fr;
                        const float bv = (EPI != PS_PARTIAL && ep.bias) ? ep.bias[col] : 0.f;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float v = acc[i][t][r] + bv;
                            if constexpr (EPI == PS_GELU_TANH) v = gelu_tanh(v);
                            char* dst = stage + (16 * i - ps * RPP + 4 * g + r) * TW + (16 * t + fr) * OB;
                            if constexpr (OB == 4)
                                *reinterpret_cast<float*>(dst) = v;
                            else
                                *reinterpret_cast<bf16_t*>(dst) = f32_to_bf16(v);
                        }
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                constexpr int CPR = TW / 16;  // 16-B chunks per staged row
                for (int c = lane; c < RPP * CPR; c += 64) {
                    const int lr = c / CPR, ch = c - lr * CPR;
                    const int row = m0 + ps * RPP + lr;
                    if (row >= M || ps * RPP + lr >= BM) continue;
                    const uint4 val = *reinterpret_cast<const uint4*>(stage + lr * TW + ch * 16);
                    const int col = col0 + ch * (16 / OB);
                    if constexpr (EPI == PS_PARTIAL) {
                        *reinterpret_cast<uint4*>(reinterpret_cast<float*>(ep.out) + (size_t)ks * ep.split_stride +
                                                  (size_t)row * ep.ldo + col) = val;
                    } else if constexpr (EPI == PS_QKV) {
                        const int part = col / ep.d_local;
                        const int within = col - part * ep.d_local;
                        bf16_t* dst;
                        if (part == 0) {
                            dst = ep.q_out + (size_t)row * ep.ldq + within;
                        } else {
                            const int head = within >> 6, dim = within & 63;
                            const size_t sl = dlms_idx(ep.row_slot[row], ep.n_slots, CHK_QKV_SLOT);
                            const size_t pos = dlms_idx(ep.row_pos[row], ep.t_max, CHK_QKV_POS);
                            dst = (part == 1 ? ep.k_cache : ep.v_cache) + ((sl * ep.n_heads + head) * ep.t_max + pos) * 64 + dim;
                        }
                        *reinterpret_cast<uint4*>(dst) = val;
                    } else {
                        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(ep.out) + (size_t)row * ep.ldo + col) = val;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging reads done before reuse
            }
            (void)ncols;
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[i][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    };

    auto compute = [&](const bf16x8_t (&b)[KBC][NT], int step) {
        const int kb0 = (step % nch) * KBC;
        unsigned int swl = 0, swl2 = 0;
        if constexpr (EPI == PS_ARGMAX) {
            // one seen-bitmap word per lane per chunk (unconditional: a static load count keeps the
            // counted vmcnt of the double-buffered weight stream); its latency hides under the MFMAs
            const int tile = slot + (step / nch) * slots;
            int srow = m0 + 16 * (fr >> 2) + 4 * g + (fr & 3);
            srow = srow < M ? srow : M - 1;
            swl = ep.seen[(size_t)srow * ep.seen_words + ((tile * NT * 16 + ep.col_offset) >> 5)];
            static_assert(NT <= 2, "a tile's columns share one seen word per row");
            if constexpr (MT > 4) {  // a lane's word covers row tiles 0..3; tiles 4..7 take a second one
                static_assert(MT <= 8, "two seen words per lane cover at most 8 row tiles");
                int srow2 = m0 + 16 * ((fr >> 2) + 4) + 4 * g + (fr & 3);
                srow2 = srow2 < M ? srow2 : M - 1;
                swl2 = ep.seen[(size_t)srow2 * ep.seen_words + ((tile * NT * 16 + ep.col_offset) >> 5)];
            }
        }
#pragma unroll
        for (int kb = 0; kb < KBC; ++kb) {
            bf16x8_t a[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i)
                a[i] = *reinterpret_cast<const bf16x8_t*>(smem + (16 * i + fr) * row_bytes + ((kb0 + kb) * 32 + g * 8) * 2);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[kb][t], acc[i][t], 0, 0, 0);
        }
        if (step % nch == nch - 1) finish_tile(step, swl, swl2);
    };

    // register ring of weight chunks: NBUF-1 chunks in flight behind the one being computed.  The
    // argmax variant at 64 x 32 wave tiles double-buffers by default: its running keys leave no
    // registers for a deeper ring of 4-k-block chunks (3- and 4-deep rings spill there and ran 2.5x
    // slower, profiles/r2_gemm_ps_vs_tiled.log)
    constexpr int NBUF = NB > 0 ? NB : ((EPI == PS_ARGMAX && MT * NT >= 8) ? 2 : 4);
    static_assert(NBUF >= 2 && NBUF <= 4, "2..4 register chunks");
    bf16x8_t b[NBUF][KBC][NT];
    if (nsteps > 0) {
#pragma unroll
        for (int j = 0; j < NBUF - 1; ++j) load(b[j], j);
    }
    // the activation panel: every wave's LDS-DMA landed, then all waves may read it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int step = 0; step < nsteps; step += NBUF) {
#pragma unroll
        for (int j = 0; j < NBUF; ++j) {  // (compile-time buffer indices: the ring stays in registers)
            if (j > 0 && step + j >= nsteps) break;
            load(b[(j + NBUF - 1) % NBUF], step + j + NBUF - 1);
            compute(b[j], step + j);
        }
    }

    if constexpr (EPI == PS_ARGMAX) {
        // per-row max over the 16 column lanes, one key per (row, wave slot)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                unsigned long long k = best[i][r];
                k = row16_max_u64(k);  // max over the 16 lanes of this row
                const int row = m0 + 16 * i + 4 * g + r;
                if (fr == 0 && row < M) ep.argmax_out[(size_t)row * ep.ldo + slot] = k;
            }
    }
}

template <int EPI, int MT, int NT, int KBC = PS_KBC, int NB = 0>
static hipError_t launch_ps(const void* A, int lda, const void* W, int M, int N, int K, int split, int col_wgs,
                            const GemmEpi& ep, hipStream_t stream) {
    const int kc = K / split;
    const int row_blocks = (M + 16 * MT - 1) / (16 * MT);
    const size_t lds = (size_t)16 * MT * (kc * 2 + PS_PAD) + (size_t)PS_NW * PS_STAGE;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static std::atomic<uint64_t> attr_set{0};  // per device
    if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(&gemm_ps_kernel<EPI, MT, NT, KBC, NB>), 160 * 1024);
        e != hipSuccess)
        return e;
    hipLaunchKernelGGL((gemm_ps_kernel<EPI, MT, NT, KBC, NB>), dim3(row_blocks * split * col_wgs), dim3(64 * PS_NW), lds, stream,
                       reinterpret_cast<const bf16_t*>(A), lda, reinterpret_cast<const bf16_t*>(W), M, N, K, row_blocks,
                       split, col_wgs, ep);
    return hipGetLastError();
}

// Geometry: mt = 16-row tiles per block (2 or 4; 5 for the argmax), nt = 16-column groups per wave (1 or 2),
// col_wgs = column workgroups (each 8 wave slots of nt groups; tiles beyond the slots loop).
extern "C" hipError_t dlms_gemm_ps(int epi, const void* A, int lda, const void* Wsh, int M, int N, int K, int split,
                                   int mt, int nt, int col_wgs, const GemmEpi* ep, hipStream_t stream) {
    if (M <= 0 || N % (16 * nt) || split < 1 || K % split || (K / split) % (32 * PS_KBC) || col_wgs < 1)
        return hipErrorInvalidValue;
    if (epi != PS_PARTIAL && split != 1) return hipErrorInvalidValue;
    // the argmax LM head (64 x 32 wave tiles): 8-k-block register chunks, double-buffered -- 16 KiB
    // of weights in flight per wave instead of 8 (232 VGPRs, no scratch): M = 512 67.5 -> 64.0 us,
    // M = 1024 107.9 -> 99.7 us (profiles/r5_lmhead_kbc_ab.jsonl; 6-k-block chunks x 3 buffers and
    // 64 x 64 wave tiles on 4-k-block chunks measured 68.2 / 64.1 us, both with spills)
    if (epi == PS_ARGMAX && mt == 4 && nt == 2 && (K / split) % (32 * 8) == 0)
        return launch_ps<PS_ARGMAX, 4, 2, 8, 2>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream);
#define PS_GEO(E)                                                                                         \
    if (mt == 2 && nt == 1) return launch_ps<E, 2, 1>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream); \
    if (mt == 2 && nt == 2) return launch_ps<E, 2, 2>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream); \
    if (mt == 4 && nt == 1) return launch_ps<E, 4, 1>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream); \
    if (mt == 4 && nt == 2) return launch_ps<E, 4, 2>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream); \
    if (E == PS_ARGMAX && mt == 5 && nt == 2) return launch_ps<PS_ARGMAX, 5, 2>(A, lda, Wsh, M, N, K, split, col_wgs, *ep, stream); \
    return hipErrorInvalidValue;
    switch (epi) {
        case PS_BF16: PS_GEO(PS_BF16)
        case PS_GELU_TANH: PS_GEO(PS_GELU_TANH)
        case PS_QKV: PS_GEO(PS_QKV)
        case PS_ARGMAX: PS_GEO(PS_ARGMAX)
        case PS_PARTIAL: PS_GEO(PS_PARTIAL)
        default: return hipErrorInvalidValue;
    }
#undef PS_GEO
}

DLMS_CHECK_EXPORT(gemm_ps)
