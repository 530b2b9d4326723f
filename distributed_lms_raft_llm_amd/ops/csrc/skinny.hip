// Skinny (decode, M <= 32 rows) MFMA GEMMs and split-K flash-decode attention: the latency path.
//
// At batch 1-32 a decode step is a chain of ~60 weight-streaming kernels whose runtime is launch +
// memory latency, not FLOPs (a 64x64-tile GEMM puts only N/64 = 36 workgroups on the 256 CUs for
// GPT-2's QKV).  These kernels are shaped for that regime:
//
//  * weights are PRE-SHUFFLED once at load time into MFMA B-fragment order
//    (engine/weights.py: [N/16][K/32][64 lanes][8 bf16]), so every wave-instruction loads one
//    contiguous KiB straight into the B operand of v_mfma_f32_16x16x32_bf16 -- no LDS round trip for
//    the streamed operand, perfectly coalesced, and one 16-column group per wave keeps N/16
//    groups x (K split over the workgroup's waves) wave-loads in flight;
//  * the (tiny) activation is the A operand: either x (f32 residual) normalised by a fused
//    LayerNorm prologue into an LDS bf16 image (LN1 -> QKV, LN2 -> c_fc: no separate LN kernel),
//    or a bf16 activation read as A fragments straight from L2 (att -> out-proj, ff -> c_proj);
//  * K is split over the waves of a workgroup and the partial accumulators are summed in a fixed
//    order through LDS (deterministic), so one workgroup owns whole output columns: the row-parallel
//    projections add bias + residual in place (x += ...) with no split-K slabs and no add+LN pass.
//
// Epilogues: EPI_BF16 / EPI_GELU_TANH / EPI_QKV (q out + K/V scattered into the cache) /
// EPI_F32 (x += acc + bias, in place) / EPI_PARTIAL (TP: raw partial for the all-reduce) /
// EPI_ARGMAX (repetition penalty + per-row argmax key per 64 columns, the LM-head layout of gemm.hip).
#include "common.h"
#include "skinny_common.h"
#include <type_traits>
#include <stdlib.h>


#define SK_MAX_LN_V4 8  // LN prologue: K <= 64 lanes * 4 * 8 = 2048

// Weight-fragment loads: plain (default-policy) loads keep the streamed weights eligible for the
// 256 MiB Infinity Cache, which holds most of GPT-2-small's 248 MB per-step weight stream at batch
// 1 (non-temporal loads measured no better here: cdna guide nt-weights row).
__device__ __forceinline__ bf16x8_t load_wfrag(const bf16x8_t* p) { return *p; }

// The batch-1 LM head streams 77 MB once per token: non-temporal loads keep it from evicting the
// 12 layers' ~170 MB of weights out of the 256 MiB Infinity Cache (a cyclic 248 MB stream through
// an LRU cache of about that size would otherwise miss on every layer).
static int lm_head_nt() { return 1; }


// LayerNorm of rows [0, M) of x (f32, ldx) into an LDS bf16 image of 16*MT rows (rows >= M zero).
// Wave w normalises rows w, w + NW, ...; two-pass statistics in fp32 like norm.hip.
template <int NW, int MT>
__device__ __forceinline__ void ln_prologue(const float* __restrict__ x, int ldx, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, int M, int K, float eps, char* img,
                                            int row_bytes) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nv = K >> 2;
    for (int r = wave; r < 16 * MT; r += NW) {
        char* dst = img + r * row_bytes;
        if (r >= M) {
            for (int c = lane; c < nv; c += 64) *reinterpret_cast<uint2*>(dst + c * 8) = make_uint2(0u, 0u);
            continue;
        }
        const float4* xr = reinterpret_cast<const float4*>(x + (size_t)r * ldx);
        float4 v[SK_MAX_LN_V4];
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < SK_MAX_LN_V4; ++i) {
            const int c = lane + 64 * i;
            v[i] = c < nv ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        }
        const float mean = wave_sum(s) / (float)K;
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < SK_MAX_LN_V4; ++i) {
            const int c = lane + 64 * i;
            if (c < nv) {
                const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
                ss += (a * a + b * b) + (cc * cc + d * d);
            }
        }
        const float rstd = rsqrtf(wave_sum(ss) / (float)K + eps);
        const float4* g4 = reinterpret_cast<const float4*>(gamma);
        const float4* b4 = reinterpret_cast<const float4*>(beta);
#pragma unroll
        for (int i = 0; i < SK_MAX_LN_V4; ++i) {
            const int c = lane + 64 * i;
            if (c < nv) {
                const float4 gg = g4[c], bb = b4[c];
                uint2 p;
                p.x = pack_bf16x2((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
                p.y = pack_bf16x2((v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
                *reinterpret_cast<uint2*>(dst + c * 8) = p;
            }
        }
    }
}

// grid.x = column-group blocks of CG groups (16 columns each); block = 64*NW threads.
// Waves per column group WPG = NW / CG split the K/32 k-blocks evenly (fixed-order LDS reduction);
// each wave holds at most KBW k-blocks and issues ALL its B (and, without the LN prologue, A)
// fragment loads before the first MFMA -- the latency-bound regime wants every byte in flight.
template <int EPI, bool LN, int MT, int NW, int CG, int KBW>
__global__ __launch_bounds__(64 * NW) void skinny_gemm_kernel(const void* __restrict__ A, int lda,
                                                            const float* __restrict__ ln_g, const float* __restrict__ ln_b,
                                                            float eps, const bf16_t* __restrict__ Wsh, int M, int N,
                                                            int K, GemmEpi ep, int wnt) {
    constexpr int WPG = NW / CG;
    static_assert(NW % CG == 0, "whole waves per column group");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cgi = wave / WPG;       // column group within the block
    const int kpart = wave % WPG;     // K slice of this wave
    const int ng = blockIdx.x * CG + cgi;
    const int nkb = K >> 5;
    const int per = (nkb + WPG - 1) / WPG;
    const int kb0 = kpart * per < nkb ? kpart * per : nkb;
    const int nk = (kb0 + per < nkb ? kb0 + per : nkb) - kb0;  // k-blocks of this wave (<= KBW)
    const int g = lane >> 4, fr = lane & 15;
    const int row_bytes = K * 2 + 16;  // padded LN image rows: conflict-free ds_read_b128 fragments

    const int kbl = nk > 0 ? kb0 : 0;  // a wave with no k-blocks still loads (and ignores) block 0
    const bf16x8_t* wsrc = reinterpret_cast<const bf16x8_t*>(Wsh) + ((size_t)ng * nkb + kbl) * 64 + lane;
    const int last = nk > 0 ? nk - 1 : 0;
    bf16x8_t b[KBW];
#pragma unroll
    for (int u = 0; u < KBW; ++u) {
        const bf16x8_t* p = wsrc + (size_t)(u < nk ? u : last) * 64;
        b[u] = wnt ? __builtin_nontemporal_load(p) : load_wfrag(p);
    }
    bf16x8_t a[LN ? 1 : KBW][MT];
    if constexpr (!LN) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            int row = 16 * t + fr;
            row = row < M ? row : M - 1;  // rows >= M compute garbage that is never stored
            const bf16_t* ar = reinterpret_cast<const bf16_t*>(A) + (size_t)row * lda + kbl * 32 + g * 8;
#pragma unroll
            for (int u = 0; u < KBW; ++u) a[u][t] = *reinterpret_cast<const bf16x8_t*>(ar + (u < nk ? u : last) * 32);
        }
    }

    f32x4_t acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    if constexpr (LN) {
        ln_prologue<NW, MT>(reinterpret_cast<const float*>(A), lda, ln_g, ln_b, M, K, eps, smem, row_bytes);
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < KBW; ++u) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            if (u >= nk) continue;  // wave-uniform; constant register indices keep b[]/a[] in VGPRs
            bf16x8_t av;
            if constexpr (LN)
                av = lds_a_frag(smem, row_bytes, 16 * t + fr, kb0 + u, g);
            else
                av = a[u][t];
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[u], acc[t], 0, 0, 0);
        }
    }

    // ---- fixed-order reduction of the WPG K slices of each column group ----
    float* red = reinterpret_cast<float*>(smem);
    if constexpr (WPG > 1) {
        __syncthreads();  // LN image no longer read
        if (kpart > 0) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
                *reinterpret_cast<f32x4_t*>(red + ((size_t)(wave * MT + t) * 64 + lane) * 4) = acc[t];
        }
        __syncthreads();
        if (kpart == 0) {
#pragma unroll
            for (int s = 1; s < WPG; ++s)
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const f32x4_t o = *reinterpret_cast<const f32x4_t*>(red + ((size_t)((wave + s) * MT + t) * 64 + lane) * 4);
                    acc[t] += o;
                }
        }
    }

    const int col = ng * 16 + fr;
    if constexpr (EPI == SK_ARGMAX) {
        // penalty + argmax over this block's CG*16 columns -> one key per (row, 64-column group)
        static_assert(CG * 16 == 64, "argmax epilogue: one 64-column key group per block");
        __shared__ unsigned long long kred[CG][32];
        if (kpart == 0) {
            const int gcol = col + ep.col_offset;
            const bool valid = gcol < ep.vocab;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * t + g * 4 + r;
                    const int srow = row < M ? row : M - 1;
                    float v = acc[t][r];
                    const unsigned int bits = ep.seen[(size_t)srow * ep.seen_words + (gcol >> 5)];
                    if ((bits >> (gcol & 31)) & 1u) v = v < 0.f ? v * ep.penalty : v / ep.penalty;
                    unsigned long long key =
                        valid ? (((unsigned long long)f32_ordered(v) << 32) | (unsigned long long)(~(unsigned int)gcol)) : 0ull;
                    key = row16_max_u64(key);  // max over the 16 lanes of this row
                    if (fr == 0) kred[cgi][row] = key;
                }
        }
        __syncthreads();
        for (int row = threadIdx.x; row < M && row < 16 * MT; row += 64 * NW) {
            unsigned long long b = kred[0][row];
#pragma unroll
            for (int c = 1; c < CG; ++c) b = kred[c][row] > b ? kred[c][row] : b;
            ep.argmax_out[(size_t)row * ep.ldo + blockIdx.x] = b;
        }
        return;
    }
    if (kpart != 0) return;
    skinny_store<EPI, MT>(acc, M, col, g, ep);
}

template <int EPI, bool LN, int MT, int NW, int CG, int KBW>
static hipError_t launch_skinny(const void* A, int lda, const float* g, const float* b, float eps, const bf16_t* W,
                                int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
    size_t lds = 0;
    if (LN) lds = (size_t)16 * MT * (K * 2 + 16);
    const size_t red = (size_t)NW * MT * 64 * 4 * sizeof(float);
    if (NW / CG > 1 && red > lds) lds = red;
    static std::atomic<uint64_t> attr_set{0};  // per device
    if (lds > 65536)
        if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(&skinny_gemm_kernel<EPI, LN, MT, NW, CG, KBW>),
                                      160 * 1024); e != hipSuccess)
            return e;
    const int wnt = EPI == SK_ARGMAX ? lm_head_nt() : 0;
    hipLaunchKernelGGL((skinny_gemm_kernel<EPI, LN, MT, NW, CG, KBW>), dim3(N / (16 * CG)), dim3(64 * NW), lds, stream,
                       A, lda, g, b, eps, W, M, N, K, ep, wnt);
    return hipGetLastError();
}

// k-blocks per wave -> the smallest register budget KBW that holds them
template <int EPI, bool LN, int MT, int NW, int CG>
static hipError_t skinny_kbw(const void* A, int lda, const float* g, const float* b, float eps, const bf16_t* W,
                             int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
    const int per = ((K >> 5) + NW / CG - 1) / (NW / CG);
    if (per <= 4) return launch_skinny<EPI, LN, MT, NW, CG, 4>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    if (per <= 8) return launch_skinny<EPI, LN, MT, NW, CG, 8>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    if (per <= 12) return launch_skinny<EPI, LN, MT, NW, CG, 12>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    if (per <= 16) return launch_skinny<EPI, LN, MT, NW, CG, 16>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    return hipErrorInvalidValue;
}

// Geometry per epilogue family (waves split K; one 16-column group per wave group):
//   LN-fed column-parallel GEMMs (QKV, c_fc): 4 waves per group;
//   row-parallel projections (N = d: few column groups): out-proj 8 waves, c_proj (K = 4d) 16;
//   LM head: 4 column groups of 4 waves (64 columns -> one argmax key per row and block).
template <int EPI, bool LN, int MT>
static hipError_t skinny_dispatch(const void* A, int lda, const float* g, const float* b, float eps, const bf16_t* W,
                                  int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
    if constexpr (EPI == SK_ARGMAX) {
        return skinny_kbw<EPI, LN, MT, 16, 4>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    } else if constexpr (EPI == SK_F32 || EPI == SK_FIXADD || EPI == SK_PARTIAL) {
        if (K > 2048) return skinny_kbw<EPI, LN, MT, 16, 1>(A, lda, g, b, eps, W, M, N, K, ep, stream);
        return skinny_kbw<EPI, LN, MT, 8, 1>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    } else {
        return skinny_kbw<EPI, LN, MT, 4, 1>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    }
}

template <int EPI, bool LN>
static hipError_t skinny_mt(const void* A, int lda, const float* g, const float* b, float eps, const bf16_t* W, int M,
                            int N, int K, const GemmEpi& ep, hipStream_t stream) {
    if (M <= 16) return skinny_dispatch<EPI, LN, 1>(A, lda, g, b, eps, W, M, N, K, ep, stream);
    return skinny_dispatch<EPI, LN, 2>(A, lda, g, b, eps, W, M, N, K, ep, stream);
}

// A: f32 x [M][lda] when ln_g != nullptr (fused LayerNorm prologue), else bf16 [M][lda].
// Wsh: pre-shuffled [N/16][K/32][64][8] bf16.
extern "C" hipError_t dlms_skinny_gemm(int epi, const void* A, int lda, const float* ln_g, const float* ln_b, float eps,
                                       const void* Wsh, int M, int N, int K, const GemmEpi* ep, hipStream_t stream) {
    if (M <= 0 || M > 32 || N % 16 || K % 32 || K <= 0) return hipErrorInvalidValue;
    const bool ln = ln_g != nullptr;
    if (ln && (K % 4 || K > 64 * 4 * SK_MAX_LN_V4)) return hipErrorInvalidValue;
    if (epi == SK_ARGMAX && N % 64) return hipErrorInvalidValue;
    const bf16_t* W = reinterpret_cast<const bf16_t*>(Wsh);
#define SK_LN(E) \
    case E:       \
        return ln ? skinny_mt<E, true>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream) : hipErrorInvalidValue;
#define SK_NOLN(E) \
    case E:         \
        return ln ? hipErrorInvalidValue : skinny_mt<E, false>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream);
    switch (epi) {
        case SK_BF16:
            return ln ? skinny_mt<SK_BF16, true>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream)
                      : skinny_mt<SK_BF16, false>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream);
        SK_LN(SK_GELU_TANH)
        SK_LN(SK_QKV)
        SK_NOLN(SK_F32)
        SK_NOLN(SK_FIXADD)
        case SK_ARGMAX:  // with the LN prologue: ln_f fused into the latency path's LM head
            return ln ? skinny_mt<SK_ARGMAX, true>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream)
                      : skinny_mt<SK_ARGMAX, false>(A, lda, ln_g, ln_b, eps, W, M, N, K, *ep, stream);
        SK_NOLN(SK_PARTIAL)
        default: return hipErrorInvalidValue;
    }
#undef SK_LN
#undef SK_NOLN
}

// The latency path's residual stream between fused MLP kernels is int64 fixed point (value * 2^32):
// every workgroup of the MLP adds its slice's contribution with a 64-bit integer atomic, and integer
// adds commute, so the sum is bit-identical whatever order the workgroups arrive in (float atomics
// would not be).  |x| < 2^31 and a resolution of 2^-32 cover any GPT-2 residual with margin.
// The residual is held as DLMS_FIX_COPIES partial copies (workgroup j adds into copy j % COPIES,
// readers sum them): atomics to one address serialise at the memory side.  Batch-1 query in situ
// (profiles/r2_fused_mlp.txt): 1 copy 36.9 ms, 2 copies 34.8, 4 copies 34.8 (8: the QKV prologue's
// extra 6 KB per row and copy cost more than the contention saved).
#ifndef DLMS_FIX_COPIES
#define DLMS_FIX_COPIES 2
#endif
#define DLMS_FIX_SCALE 4294967296.0f
#define DLMS_FIX_INV (1.0f / 4294967296.0f)

__device__ __forceinline__ float fix_to_f32(long long v) { return (float)v * DLMS_FIX_INV; }
__device__ __forceinline__ unsigned long long f32_to_fix(float v) {
    return (unsigned long long)__float2ll_rn(v * DLMS_FIX_SCALE);
}

// 4 consecutive residual values (columns 4c..4c+3) of the row at element offset `off`: f32, or
// int64 fixed point converted on load
template <bool XFIX>
__device__ __forceinline__ float4 load_resid4(const void* __restrict__ x, size_t off, int c, long long cs) {
    if constexpr (XFIX) {  // sum of the copies (exact integer adds), then one rounding to f32
        const long long* base = reinterpret_cast<const long long*>(x) + off + 4 * c;
        longlong2 a[DLMS_FIX_COPIES], b[DLMS_FIX_COPIES];
#pragma unroll
        for (int k = 0; k < DLMS_FIX_COPIES; ++k) {
            a[k] = reinterpret_cast<const longlong2*>(base + k * cs)[0];
            b[k] = reinterpret_cast<const longlong2*>(base + k * cs)[1];
        }
#pragma unroll
        for (int k = 1; k < DLMS_FIX_COPIES; ++k) {
            a[0].x += a[k].x; a[0].y += a[k].y; b[0].x += b[k].x; b[0].y += b[k].y;
        }
        return make_float4(fix_to_f32(a[0].x), fix_to_f32(a[0].y), fix_to_f32(b[0].x), fix_to_f32(b[0].y));
    } else {
        return reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + off)[c];
    }
}

template <bool XFIX>
__device__ __forceinline__ float load_resid1(const void* __restrict__ x, size_t off, long long cs) {
    if constexpr (XFIX) {
        long long a = 0;
#pragma unroll
        for (int k = 0; k < DLMS_FIX_COPIES; ++k) a += reinterpret_cast<const long long*>(x)[off + k * cs];
        return fix_to_f32(a);
    } else
        return reinterpret_cast<const float*>(x)[off];
}

// ---------------------------------------------------------------------------------------------
// Fused residual update + LayerNorm + skinny GEMM: the decode path's LN1 -> QKV and LN2 -> c_fc at
// M <= 4 * RPW rows (one 16-row MFMA tile; rows >= M are never stored).
//
//   v = x_in + res_bias + sum_{s < NSPLIT} parts[s]        (the pending row-parallel update:
//                                                           split-K slabs, or the TP all-reduce)
//   block 0 writes x_out = v  -- the residual stream moves to the OTHER ping-pong buffer, so no
//                                block ever reads a row another block has already advanced;
//   A = bf16(LN(v) * gamma + beta) -> LDS -> v_mfma_f32_16x16x32_bf16 against pre-shuffled W.
//
// Load order: all weight fragments of the wave first (HBM), then the activation rows (L2), so
// both are in flight together -- one memory round trip before the LayerNorm, not two.
// Fused-kernel prologue: rows [0, M) of v = x_in + res_bias + sum_{s < NSPLIT} parts[s] (wave w owns
// rows w, w + 4, ...), written to x_out by block 0 when given, LayerNormed into the LDS bf16 image
// (rows >= M are left as they are: their MFMA results are never stored).
struct NoOp {
    __device__ void operator()() const {}
};

// (after_loads() runs once the activation loads are issued: a caller's own loads issued there stay in
// flight under the LayerNorm instead of delaying it)
template <int NSPLIT, int NV4, int RPW, bool XFIX, bool LATE_GB = (XFIX && NV4 >= 7), typename AfterLoads = NoOp>
__device__ __forceinline__ void addln_rows_lds(const void* __restrict__ x_in, float* __restrict__ x_out, int ldx,
                                               const float* __restrict__ parts, int ldp, long long split_stride,
                                               const float* __restrict__ res_bias, const float* __restrict__ gamma,
                                               const float* __restrict__ beta, float eps, int M, int K, char* smem,
                                               int row_bytes, long long xcs, float* v_lds = nullptr,
                                               AfterLoads after_loads = AfterLoads()) {
    constexpr int NW = 4;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int nv = K >> 2;
    int cidx[NV4];
    bool valid[NV4];
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        const int c = lane + 64 * i;
        valid[i] = c < nv;
        cidx[i] = valid[i] ? c : nv - 1;
    }
    float4 v[RPW][NV4];
    float4 pv[RPW][NSPLIT > 0 ? NSPLIT : 1][NV4];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        int row = wave + NW * i;
        row = row < M ? row : M - 1;
#pragma unroll
        for (int c = 0; c < NV4; ++c) v[i][c] = load_resid4<XFIX>(x_in, (size_t)row * ldx, cidx[c], xcs);
#pragma unroll
        for (int s = 0; s < NSPLIT; ++s) {
            const float4* pr = reinterpret_cast<const float4*>(parts + (size_t)s * split_stride + (size_t)row * ldp);
#pragma unroll
            for (int c = 0; c < NV4; ++c) pv[i][s][c] = pr[cidx[c]];
        }
    }
    // GPT-2-XL's fixed-point variant (d 1600, two int64 copies per element in flight) loads gamma /
    // beta only once the residual is summed: held from the start they took it to 292 registers, one
    // wave per SIMD, and its 300 QKV workgroups ran in two rounds on 256 CUs; the late load is one
    // L2 round trip under the variance reduction.
    float4 gv[NV4], bv[NV4], rb[NV4];
#pragma unroll
    for (int c = 0; c < NV4; ++c) {
        if constexpr (!LATE_GB) {
            gv[c] = reinterpret_cast<const float4*>(gamma)[cidx[c]];
            bv[c] = reinterpret_cast<const float4*>(beta)[cidx[c]];
        }
        rb[c] = res_bias ? reinterpret_cast<const float4*>(res_bias)[cidx[c]] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    after_loads();

#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int row = wave + NW * i;
        if (row >= M) continue;  // wave-uniform
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NV4; ++c) {
            float4 t = v[i][c];
            t.x += rb[c].x; t.y += rb[c].y; t.z += rb[c].z; t.w += rb[c].w;
#pragma unroll
            for (int sp = 0; sp < NSPLIT; ++sp) {
                t.x += pv[i][sp][c].x; t.y += pv[i][sp][c].y; t.z += pv[i][sp][c].z; t.w += pv[i][sp][c].w;
            }
            if (!valid[c]) t = make_float4(0.f, 0.f, 0.f, 0.f);
            v[i][c] = t;
            s += (t.x + t.y) + (t.z + t.w);
        }
        if (x_out != nullptr && blockIdx.x == 0) {
#pragma unroll
            for (int c = 0; c < NV4; ++c)
                if (valid[c]) reinterpret_cast<float4*>(x_out + (size_t)row * ldx)[cidx[c]] = v[i][c];
        }
        if (v_lds != nullptr) {
#pragma unroll
            for (int c = 0; c < NV4; ++c)
                if (valid[c]) reinterpret_cast<float4*>(v_lds + (size_t)row * K)[cidx[c]] = v[i][c];
        }
        const float mean = wave_sum(s) / (float)K;
        if constexpr (LATE_GB) {
            if (i == 0) {
                asm volatile("" ::: "memory");  // issued here, not hoisted beside the residual loads
#pragma unroll
                for (int c = 0; c < NV4; ++c) {
                    gv[c] = reinterpret_cast<const float4*>(gamma)[cidx[c]];
                    bv[c] = reinterpret_cast<const float4*>(beta)[cidx[c]];
                }
            }
        }
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < NV4; ++c) {
            if (valid[c]) {
                const float a0 = v[i][c].x - mean, a1 = v[i][c].y - mean, a2 = v[i][c].z - mean, a3 = v[i][c].w - mean;
                ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
            }
        }
        const float rstd = rsqrtf(wave_sum(ss) / (float)K + eps);
        char* dst = smem + row * row_bytes;
#pragma unroll
        for (int c = 0; c < NV4; ++c) {
            if (valid[c]) {
                const float4 t = v[i][c];
                uint2 p;
                p.x = pack_bf16x2((t.x - mean) * rstd * gv[c].x + bv[c].x, (t.y - mean) * rstd * gv[c].y + bv[c].y);
                p.y = pack_bf16x2((t.z - mean) * rstd * gv[c].z + bv[c].z, (t.w - mean) * rstd * gv[c].w + bv[c].w);
                *reinterpret_cast<uint2*>(dst + cidx[c] * 8) = p;
            }
        }
    }
}

template <int EPI, int NSPLIT, int NV4, int RPW, int KBW, bool XFIX>
__device__ __forceinline__ void skinny_addln_impl(const void* __restrict__ x_in, float* __restrict__ x_out,
                                                         int ldx, const float* __restrict__ parts, int ldp,
                                                         long long split_stride, const float* __restrict__ res_bias,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float eps, const bf16_t* __restrict__ Wsh, int M, int N, int K,
                                                         GemmEpi ep, uint4* __restrict__ zero_buf, int zero_chunks,
                                                         long long xcs) {
    constexpr int NW = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ng = blockIdx.x;
    const int nkb = K >> 5;
    const int per = (nkb + NW - 1) / NW;
    const int kb0 = wave * per < nkb ? wave * per : nkb;
    const int nk = (kb0 + per < nkb ? kb0 + per : nkb) - kb0;
    const int kbl = nk > 0 ? kb0 : 0;
    const int last = nk > 0 ? nk - 1 : 0;
    const int g = lane >> 4, fr = lane & 15;
    const int row_bytes = K * 2 + 16;

    const bf16x8_t* wsrc = reinterpret_cast<const bf16x8_t*>(Wsh) + ((size_t)ng * nkb + kbl) * 64 + lane;
    bf16x8_t b[KBW];
#pragma unroll
    for (int u = 0; u < KBW; ++u) b[u] = load_wfrag(wsrc + (size_t)(u < nk ? u : last) * 64);
    // the fixed-point accumulator the following fused MLP adds into starts from zero (grid-stride)
    if (zero_buf != nullptr)
        for (int z = blockIdx.x * 256 + threadIdx.x; z < zero_chunks; z += gridDim.x * 256) zero_buf[z] = make_uint4(0u, 0u, 0u, 0u);

    addln_rows_lds<NSPLIT, NV4, RPW, XFIX>(x_in, x_out, ldx, parts, ldp, split_stride, res_bias, gamma, beta, eps, M, K,
                                           smem, row_bytes, xcs);
    __syncthreads();

    f32x4_t acc[1] = {(f32x4_t){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int u = 0; u < KBW; ++u) {
        if (u >= nk) continue;
        const bf16x8_t av = lds_a_frag(smem, row_bytes, fr, kb0 + u, g);  // rows >= M: never stored
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[u], acc[0], 0, 0, 0);
    }
    __syncthreads();  // LN image no longer read: reuse it for the K-slice reduction
    float* red = reinterpret_cast<float*>(smem);
    if (wave > 0) *reinterpret_cast<f32x4_t*>(red + ((size_t)wave * 64 + lane) * 4) = acc[0];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int s = 1; s < NW; ++s) acc[0] += *reinterpret_cast<const f32x4_t*>(red + ((size_t)s * 64 + lane) * 4);
    skinny_store<EPI, 1>(acc, M, ng * 16 + fr, g, ep);
}

template <int EPI, int NSPLIT, int NV4, int RPW, int KBW, bool XFIX>
__global__ __launch_bounds__(256) void skinny_addln_kernel(const void* __restrict__ x_in, float* __restrict__ x_out,
                                                         int ldx, const float* __restrict__ parts, int ldp,
                                                         long long split_stride, const float* __restrict__ res_bias,
                                                         const float* __restrict__ gamma, const float* __restrict__ beta,
                                                         float eps, const bf16_t* __restrict__ Wsh, int M, int N, int K,
                                                         GemmEpi ep, uint4* __restrict__ zero_buf, int zero_chunks,
                                                         long long xcs) {
    skinny_addln_impl<EPI, NSPLIT, NV4, RPW, KBW, XFIX>(x_in, x_out, ldx, parts, ldp, split_stride, res_bias, gamma,
                                                        beta, eps, Wsh, M, N, K, ep, zero_buf, zero_chunks, xcs);
}

// launch arguments shared by every instantiation of the fused add+LN kernels
struct AddlnArgs {
    const void* x_in;
    float* x_out;
    int ldx;
    const float* parts;
    int ldp;
    long long sstride;
    const float* rbias;
    const float* g;
    const float* b;
    float eps;
    const bf16_t* W;
    int M, N, K;
    uint4* zero_buf;
    int zero_chunks;
    long long xcs;  // copy stride of a fixed-point x_in (elements)
};

template <int EPI, int NSPLIT, int NV4, int RPW, bool XFIX>
static hipError_t launch_addln(const AddlnArgs& a, const GemmEpi& ep, hipStream_t stream) {
    constexpr int KBW = NV4 <= 2 ? 4 : (NV4 <= 4 ? 8 : (NV4 == 5 ? 12 : 16));  // >= K/32/4 for K <= 256 * NV4
    const size_t lds = (size_t)16 * (a.K * 2 + 16);
    hipLaunchKernelGGL((skinny_addln_kernel<EPI, NSPLIT, NV4, RPW, KBW, XFIX>), dim3(a.N / 16), dim3(256), lds, stream,
                       a.x_in, a.x_out, a.ldx, a.parts, a.ldp, a.sstride, a.rbias, a.g, a.b, a.eps, a.W, a.M, a.N, a.K,
                       ep, a.zero_buf, a.zero_chunks, a.xcs);
    return hipGetLastError();
}

template <int EPI, int NSPLIT, int NV4, bool XFIX = false>
static hipError_t addln_rpw(const AddlnArgs& a, const GemmEpi& ep, hipStream_t stream) {
    if (a.M <= 4) return launch_addln<EPI, NSPLIT, NV4, 1, XFIX>(a, ep, stream);
    if constexpr (NV4 <= 4 && NSPLIT <= 4) {
        if (a.M <= 8) return launch_addln<EPI, NSPLIT, NV4, 2, XFIX>(a, ep, stream);
    }
    return hipErrorInvalidValue;
}

template <int EPI, int NSPLIT>
static hipError_t addln_nv4(const AddlnArgs& a, const GemmEpi& ep, hipStream_t stream) {
    const int K = a.K;
    if constexpr (NSPLIT > 4) {  // per-head slabs of the fused attention + out-projection (M <= 4, K <= 1024)
        switch ((K / 4 + 63) / 64) {
            case 3: return addln_rpw<EPI, NSPLIT, 3>(a, ep, stream);
            case 4: return addln_rpw<EPI, NSPLIT, 4>(a, ep, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch ((K / 4 + 63) / 64) {
        case 1: return addln_rpw<EPI, NSPLIT, 1>(a, ep, stream);
        case 2: return addln_rpw<EPI, NSPLIT, 2>(a, ep, stream);
        case 3: return addln_rpw<EPI, NSPLIT, 3>(a, ep, stream);
        case 4: return addln_rpw<EPI, NSPLIT, 4>(a, ep, stream);
        case 5: return addln_rpw<EPI, NSPLIT, 5>(a, ep, stream);
        case 7: return addln_rpw<EPI, NSPLIT, 7>(a, ep, stream);
        default: return hipErrorInvalidValue;
    }
}

// Max rows of the fused add+LN skinny GEMM for a model width K (0: not supported).
extern "C" int dlms_skinny_addln_max_rows(int K) {
    const int nv4 = (K / 4 + 63) / 64;
    if (K % 32 || K <= 0 || nv4 == 6 || nv4 > 7) return 0;
    return nv4 <= 4 ? 8 : 4;
}

// xfix: x_in is the int64 fixed-point residual a fused MLP left (QKV, no slabs only); zero_buf (when
// given): zero_chunks 16-B chunks cleared for the fused MLP that follows (grid-stride over all blocks)
extern "C" hipError_t dlms_skinny_addln_gemm(int epi, const void* x_in, float* x_out, int ldx, const float* parts,
                                             int ldp, long long split_stride, int nsplit, const float* res_bias,
                                             const float* gamma, const float* beta, float eps, const void* Wsh, int M,
                                             int N, int K, const GemmEpi* ep, int xfix, long long xcs, void* zero_buf,
                                             int zero_chunks, hipStream_t stream) {
    if (M <= 0 || M > dlms_skinny_addln_max_rows(K) || N % 16) return hipErrorInvalidValue;
    if (xfix && (epi != SK_QKV || nsplit != 0 || x_out != nullptr || res_bias != nullptr)) return hipErrorInvalidValue;
    const AddlnArgs a{x_in, x_out, ldx, parts, ldp, split_stride, res_bias, gamma, beta, eps,
                      reinterpret_cast<const bf16_t*>(Wsh), M, N, K, reinterpret_cast<uint4*>(zero_buf),
                      zero_buf ? zero_chunks : 0, xcs};
    if (xfix) {
        switch ((K / 4 + 63) / 64) {
            case 3: return addln_rpw<SK_QKV, 0, 3, true>(a, *ep, stream);
            case 4: return addln_rpw<SK_QKV, 0, 4, true>(a, *ep, stream);
            case 5: return addln_rpw<SK_QKV, 0, 5, true>(a, *ep, stream);
            case 7: return addln_rpw<SK_QKV, 0, 7, true>(a, *ep, stream);
            default: return hipErrorInvalidValue;
        }
    }
#define ADDLN(E, NS) return addln_nv4<E, NS>(a, *ep, stream)
#define ADDLN_EPI(E)                    \
    switch (nsplit) {                   \
        case 0: ADDLN(E, 0);            \
        case 1: ADDLN(E, 1);            \
        case 4: ADDLN(E, 4);            \
        case 12: ADDLN(E, 12);          \
        case 16: ADDLN(E, 16);          \
        default: return hipErrorInvalidValue; \
    }
    switch (epi) {
        case SK_QKV: ADDLN_EPI(SK_QKV)
        case SK_GELU_TANH: ADDLN_EPI(SK_GELU_TANH)
        default: return hipErrorInvalidValue;
    }
#undef ADDLN_EPI
#undef ADDLN
}

// ---------------------------------------------------------------------------------------------
// Fused MLP of the latency path (TP=1, M <= 4 * RPW rows): workgroup j owns intermediate columns
// [16 j, 16 j + 16) of F = 4d (F / 16 workgroups, 4 waves):
//
//   v   = x_in + res_bias + sum_s parts[s]          (x_in f32 or fixed point; parts = attention slabs)
//   h   = bf16(gelu(bf16(LN2(v)) . W_fc[16j..16j+16)^T + b_fc))        MFMA, K split over the waves
//   out = h . W_p[:, 16j..16j+16)^T  (+ v + b_p in workgroup 0)        VALU, 16-deep dot per column
//   r_out += fix(out)                                                  64-bit integer atomics
//
// It replaces [add+LN2+c_fc kernel] -> [c_proj kernel]: one kernel boundary and one dependent round
// trip (the c_proj kernel's h read) fewer per layer.  Every weight byte (W_fc fragments and the
// workgroup's contiguous 16-column W_p slice, Wp_sl [F/16][d][16]) is in flight before the
// activation loads.  r_out (int64 fixed point, see DLMS_FIX_SCALE) must be zero on entry: the QKV
// kernel of the same layer clears it.  Atomic traffic is M * d * 8 B per workgroup, so the engine
// uses this kernel only at the smallest batches.
typedef __attribute__((address_space(3))) void sk_lds_void_t;
typedef __attribute__((address_space(1))) void sk_glob_void_t;

// CG column groups per workgroup (r3): the c_proj atomics per workgroup are M * d whatever its
// width, so a workgroup owning CG groups divides the same-address atomic depth (F / 16 / COPIES
// adds per residual word at CG = 1) by CG -- the atomics, not the weight stream, bounded the
// CG = 1 kernel (profiles/r3_fused_mlp_cg.jsonl).  The NW / CG waves of a column group split its
// K; the LayerNorm image holds only the 4 RPW rows a launch may carry.
__host__ __device__ constexpr int mlp_img_bytes(int RPW, int NKB) {
    return ((4 * RPW * (NKB * 64 + 16) + 1023) & ~1023) > 4096 ? ((4 * RPW * (NKB * 64 + 16) + 1023) & ~1023) : 4096;
}
__host__ __device__ constexpr int mlp_dyn_lds(int RPW, int NKB, int CG) {
    return mlp_img_bytes(RPW, NKB) + CG * NKB * 1024 + 4 * RPW * NKB * 32 * 4;
}
__host__ __device__ constexpr bool mlp_fits(int RPW, int NKB, int CG) {
    return mlp_dyn_lds(RPW, NKB, CG) + 16 * 16 * CG * 4 <= 160 * 1024;
}

template <int NSPLIT, int NV4, int RPW, int NKB, int CG, bool XFIX>
__global__ __launch_bounds__(256) void skinny_mlp_kernel(
    const void* __restrict__ x_in, int ldx, const float* __restrict__ parts, int ldp, long long split_stride,
    const float* __restrict__ res_bias, const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    const bf16_t* __restrict__ Wfc_sh, const float* __restrict__ b_fc, const bf16_t* __restrict__ Wp_sl,
    const float* __restrict__ b_p, unsigned long long* __restrict__ r_out, int ldr, long long rcs, long long xcs, int M,
    int base) {
    constexpr int NW = 4;
    constexpr int K = NKB * 32;
    constexpr int WPG = NW / CG;                // waves per column group: they split its K
    static_assert(NW % CG == 0, "whole waves per column group");
    constexpr int PER = (NKB + WPG - 1) / WPG;  // k-blocks per wave
    constexpr int ROWB = K * 2 + 16;            // padded LN image rows: conflict-free fragment reads
    constexpr int ROWS = 4 * RPW;
    constexpr int IMG = mlp_img_bytes(RPW, NKB);
    constexpr int WPB = CG * K * 32;            // the workgroup's W_p slices [CG][K][16] bf16
    constexpr int PIECES = WPB / 1024;
    constexpr int PPW = (PIECES + NW - 1) / NW;
    constexpr int NCP = (K + 255) / 256;        // c_proj output columns per thread
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float hs[16][16 * CG];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int cgi = wave / WPG;
    const int kpart = wave % WPG;
    const int ng = blockIdx.x * CG + cgi;       // this wave's column group (16 intermediate columns)
    const int kb0 = kpart * PER < NKB ? kpart * PER : NKB;
    const int nk = (kb0 + PER < NKB ? kb0 + PER : NKB) - kb0;
    const int kbl = nk > 0 ? kb0 : 0;
    const int last = nk > 0 ? nk - 1 : 0;
    const int g = lane >> 4, fr = lane & 15;

    // (0) weights first: W_fc B fragments into registers; the workgroup's contiguous W_p slices
    //     (CG * K * 32 B) straight into LDS by LDS-DMA (no staging registers, lands under the
    //     LayerNorm); the c_proj bias for this thread's output columns
    const bf16x8_t* wsrc = reinterpret_cast<const bf16x8_t*>(Wfc_sh) + ((size_t)ng * NKB + kbl) * 64 + lane;
    bf16x8_t b[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) b[u] = load_wfrag(wsrc + (size_t)(u < nk ? u : last) * 64);
    char* wp_lds = smem + IMG;
    float* v_lds = reinterpret_cast<float*>(wp_lds + WPB);  // block 0: [M][K] f32 residual rows
    const char* wp_src = reinterpret_cast<const char*>(Wp_sl + (size_t)blockIdx.x * CG * K * 16) + lane * 16;
    auto issue_wp = [&]() {
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int pc = wave + NW * q;
            if (PIECES % NW == 0 || pc < PIECES)
                __builtin_amdgcn_global_load_lds((sk_glob_void_t*)(wp_src + pc * 1024),
                                                 (sk_lds_void_t*)(wp_lds + pc * 1024), 16, 0, 0);
        }
    };
    float bp[NCP];
#pragma unroll
    for (int i = 0; i < NCP; ++i) {
        const int n = tid + 256 * i;
        bp[i] = (blockIdx.x == 0 && base && n < K) ? b_p[n] : 0.f;
    }

    // (1) residual rows -> LN2 -> LDS image (block 0 also keeps v); (2) c_fc slice on MFMA
    // (gamma / beta with the residual loads: a late load buys no occupancy at the default column
    // groups, only a round trip; GPT-2-XL at one group per workgroup, where it does give two waves
    // per SIMD, still ran 255 vs 217.5 ms per query at two groups, profiles/r4_xl_mlp_cg_ab.jsonl)
    addln_rows_lds<NSPLIT, NV4, RPW, XFIX, false>(x_in, nullptr, ldx, parts, ldp, split_stride, res_bias, gamma, beta, eps, M,
                                           K, smem, ROWB, xcs, blockIdx.x == 0 ? v_lds : nullptr, issue_wp);
    __syncthreads();
    f32x4_t acc = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int arow = fr < ROWS ? fr : ROWS - 1;  // rows >= M: garbage results, never stored
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        if (u >= nk) continue;
        const bf16x8_t av = lds_a_frag(smem, ROWB, arow, kb0 + u, g);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b[u], acc, 0, 0, 0);
    }
    __syncthreads();  // LN image no longer read: reuse it for the fixed-order K-slice reduction
    float* red = reinterpret_cast<float*>(smem);
    if (kpart > 0) *reinterpret_cast<f32x4_t*>(red + ((size_t)wave * 64 + lane) * 4) = acc;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's share of the W_p DMA has landed ...
    __syncthreads();                                  // ... and every other wave's
    if (kpart == 0) {
#pragma unroll
        for (int s = 1; s < WPG; ++s) acc += *reinterpret_cast<const f32x4_t*>(red + ((size_t)(wave + s) * 64 + lane) * 4);
        const float bb = b_fc[ng * 16 + fr];
#pragma unroll
        for (int r = 0; r < 4; ++r)  // bf16 rounding: the same operand the unfused c_proj reads
            hs[g * 4 + r][cgi * 16 + fr] = bf16_to_f32(f32_to_bf16(gelu_tanh(acc[r] + bb)));
    }
    __syncthreads();

    // (3) c_proj slice: thread t owns output columns (t + 256 i + rot) mod K; fixed-order dot over
    //     the workgroup's 16 CG intermediate columns per row.  rot staggers the workgroups' column
    //     order so their atomics to one address do not arrive together
    unsigned long long* rc = r_out + (size_t)(blockIdx.x % DLMS_FIX_COPIES) * rcs;
    const int rot = (int)((blockIdx.x / DLMS_FIX_COPIES) * 64 % K);
#pragma unroll
    for (int i = 0; i < NCP; ++i) {
        int n = tid + 256 * i;
        if (n >= K) continue;
        n = n + rot < K ? n + rot : n + rot - K;
        float o[ROWS];
#pragma unroll
        for (int m = 0; m < ROWS; ++m) o[m] = 0.f;
#pragma unroll
        for (int c = 0; c < CG; ++c) {
            float w[16];
            const char* wr = wp_lds + ((size_t)c * K + n) * 32;
            unpack8(*reinterpret_cast<const uint4*>(wr), w);
            unpack8(*reinterpret_cast<const uint4*>(wr + 16), w + 8);
#pragma unroll
            for (int m = 0; m < ROWS; ++m) {
                if (m >= M) break;
#pragma unroll
                for (int k = 0; k < 16; ++k) o[m] = fmaf(hs[m][16 * c + k], w[k], o[m]);
            }
        }
#pragma unroll
        for (int m = 0; m < ROWS; ++m) {
            if (m >= M) break;
            float v = o[m];
            if (blockIdx.x == 0 && base) v += v_lds[m * K + n] + bp[i];  // the residual and the c_proj bias, once
            atomicAdd(rc + (size_t)m * ldr + n, f32_to_fix(v));
        }
    }
}

template <int NSPLIT, int NV4, int RPW, int NKB, int CG, bool XFIX>
static hipError_t launch_mlp(const void* x_in, int ldx, const float* parts, int ldp, long long sstride,
                             const float* rbias, const float* g, const float* b, float eps, const bf16_t* Wfc,
                             const float* b_fc, const bf16_t* Wp, const float* b_p, unsigned long long* r_out, int ldr,
                             long long rcs, long long xcs, int M, int F, int base, hipStream_t stream) {
    if constexpr (!mlp_fits(RPW, NKB, CG)) {
        return hipErrorInvalidValue;
    } else {
        if (F % (16 * CG)) return hipErrorInvalidValue;
        constexpr int lds = mlp_dyn_lds(RPW, NKB, CG);
        static std::atomic<uint64_t> attr_set{0};  // per device
        if (lds > 65536)
            if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(&skinny_mlp_kernel<NSPLIT, NV4, RPW, NKB, CG, XFIX>),
                                          lds); e != hipSuccess)
                return e;
        hipLaunchKernelGGL((skinny_mlp_kernel<NSPLIT, NV4, RPW, NKB, CG, XFIX>), dim3(F / (16 * CG)), dim3(256), lds, stream,
                           x_in, ldx, parts, ldp, sstride, rbias, g, b, eps, Wfc, b_fc, Wp, b_p, r_out, ldr, rcs, xcs, M, base);
        return hipGetLastError();
    }
}

// x_in: f32 (xfix = 0) or int64 fixed point [M][ldx]; parts: nsplit (0 or 4) f32 slabs; Wfc_sh:
// shuffle_weight(W_fc) [F/16][K/32][64][8]; Wp_sl [F/16][K][16]; r_out int64 [M][ldr], zeroed.
extern "C" int dlms_fix_copies() { return DLMS_FIX_COPIES; }

// column groups per workgroup: DLMS_MLP_CG (1, 2 or 4; 0 = per width default)
static int mlp_cg_env() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("DLMS_MLP_CG");
        v = e ? atoi(e) : 0;
    }
    return v;
}

// the CG a launch uses: the requested one when it fits the LDS at this row count, else the widest
// that does (the kernel's CG * K * 32 B W_p slices + LN image + block 0's residual rows)
extern "C" int dlms_skinny_mlp_cg(int K, int M, int want) {
    const int nkb = K / 32;
    const int rpw = M <= 4 ? 1 : 2;
    if (rpw == 2 && K > 1024) return 0;  // mlp_rows: 8-row images only up to d 1024 (VGPR budget)
    if (want <= 0) want = mlp_cg_env();
    // per-width/rows default (in situ, bench.py --batch 1/2 on one box, profiles/r3_sweep_gemm96_mlp_cg.txt):
    // d <= 1024, 1 row: CG 2 30.9 ms vs CG 4 34.5 / CG 1 31.8; 2 rows: CG 1 33.5 vs 34.7 / 38.0
    if (want <= 0) want = K <= 1024 ? (M <= 1 ? 2 : 1) : 2;
    for (int cg = want; cg >= 1; cg /= 2)
        if (mlp_fits(rpw, nkb, cg)) return cg;
    return 0;
}

template <int NSPLIT, int NV4, int NKB, bool XFIX, int RPW>
static hipError_t mlp_cg(int cg, const void* x_in, int ldx, const float* parts, int ldp, long long sstride,
                         const float* rbias, const float* g, const float* b, float eps, const bf16_t* Wfc,
                         const float* b_fc, const bf16_t* Wp, const float* b_p, unsigned long long* R, int ldr,
                         long long rcs, long long xcs, int M, int F, int base, hipStream_t stream) {
#define MLP_GO(CG_) \
    return launch_mlp<NSPLIT, NV4, RPW, NKB, CG_, XFIX>(x_in, ldx, parts, ldp, sstride, rbias, g, b, eps, Wfc, b_fc, Wp, \
                                                       b_p, R, ldr, rcs, xcs, M, F, base, stream)
    switch (cg) {
        case 1: MLP_GO(1);
        case 2: MLP_GO(2);
        case 4: MLP_GO(4);
        default: return hipErrorInvalidValue;
    }
#undef MLP_GO
}

template <int NSPLIT, int NV4, int NKB>
static hipError_t mlp_rows(int cg, int xfix, const void* x_in, int ldx, const float* parts, int ldp, long long sstride,
                           const float* rbias, const float* g, const float* b, float eps, const bf16_t* Wfc,
                           const float* b_fc, const bf16_t* Wp, const float* b_p, unsigned long long* R, int ldr,
                           long long rcs, long long xcs, int M, int F, int base, hipStream_t stream) {
#define MLP_ARGS cg, x_in, ldx, parts, ldp, sstride, rbias, g, b, eps, Wfc, b_fc, Wp, b_p, R, ldr, rcs, xcs, M, F, base, stream
    if (M <= 4) {
        if (xfix) return mlp_cg<NSPLIT, NV4, NKB, true, 1>(MLP_ARGS);
        return mlp_cg<NSPLIT, NV4, NKB, false, 1>(MLP_ARGS);
    }
    if constexpr (NV4 <= 4 && NSPLIT <= 4) {
        if (xfix) return mlp_cg<NSPLIT, NV4, NKB, true, 2>(MLP_ARGS);
        return mlp_cg<NSPLIT, NV4, NKB, false, 2>(MLP_ARGS);
    }
    return hipErrorInvalidValue;
#undef MLP_ARGS
}

// r_out / a fixed-point x_in: DLMS_FIX_COPIES copies [copy][M][ld], copy strides rcs / xcs (elements)
extern "C" hipError_t dlms_skinny_mlp(const void* x_in, int ldx, int xfix, long long xcs, const float* parts, int ldp,
                                      long long split_stride, int nsplit, const float* res_bias, const float* gamma,
                                      const float* beta, float eps, const void* Wfc_sh, const float* b_fc,
                                      const void* Wp_sl, const float* b_p, void* r_out, int ldr, long long rcs, int M,
                                      int K, int F, int want_cg, int base, hipStream_t stream) {
    if (M <= 0 || M > 8 || F % 16 || F <= 0) return hipErrorInvalidValue;
    if (nsplit != 0 && nsplit != 1 && (nsplit != 4 || K > 1024)) return hipErrorInvalidValue;
    const int cg = dlms_skinny_mlp_cg(K, M, want_cg);
    if (cg == 0) return hipErrorInvalidValue;
    const bf16_t* Wf = reinterpret_cast<const bf16_t*>(Wfc_sh);
    const bf16_t* Wp = reinterpret_cast<const bf16_t*>(Wp_sl);
    unsigned long long* R = reinterpret_cast<unsigned long long*>(r_out);
#define MLP_K(NS, NV, NKB_) \
    return mlp_rows<NS, NV, NKB_>(cg, xfix, x_in, ldx, parts, ldp, split_stride, res_bias, gamma, beta, eps, Wf, b_fc, Wp, \
                                  b_p, R, ldr, rcs, xcs, M, F, base, stream)
    // nsplit 1: the TP all-reduced attention partial (tensor-parallel fused layer, base = 0 on the
    // ranks other than 0: they add only their c_proj partial, rank 0 also the residual + b_p)
    switch (K) {
        case 768:
            if (nsplit == 4) MLP_K(4, 3, 24);
            if (nsplit == 1) MLP_K(1, 3, 24);
            MLP_K(0, 3, 24);
        case 1024:
            if (nsplit == 4) MLP_K(4, 4, 32);
            if (nsplit == 1) MLP_K(1, 4, 32);
            MLP_K(0, 4, 32);
        case 1280:
            if (nsplit == 1) MLP_K(1, 5, 40);
            MLP_K(0, 5, 40);
        case 1600:
            if (nsplit == 1) MLP_K(1, 7, 50);
            MLP_K(0, 7, 50);
        default: return hipErrorInvalidValue;
    }
#undef MLP_K
}

// Final LayerNorm of the fixed-point residual (ln_f after a fused MLP): one wave per row -> bf16.
__global__ __launch_bounds__(64) void ln_fix_kernel(const long long* __restrict__ x, int ldx, long long xcs,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float eps, bf16_t* __restrict__ out, int ldo, int K) {
    const int lane = threadIdx.x;
    const int row = blockIdx.x;
    const int nv = K >> 2;
    float4 v[SK_MAX_LN_V4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < SK_MAX_LN_V4; ++i) {
        const int c = lane + 64 * i;
        v[i] = c < nv ? load_resid4<true>(x, (size_t)row * ldx, c, xcs) : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)K;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < SK_MAX_LN_V4; ++i) {
        if (lane + 64 * i < nv) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, d = v[i].w - mean;
            ss += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)K + eps);
#pragma unroll
    for (int i = 0; i < SK_MAX_LN_V4; ++i) {
        const int c = lane + 64 * i;
        if (c < nv) {
            const float4 gg = reinterpret_cast<const float4*>(gamma)[c], bb = reinterpret_cast<const float4*>(beta)[c];
            uint2 p;
            p.x = pack_bf16x2((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y);
            p.y = pack_bf16x2((v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
            *reinterpret_cast<uint2*>(out + (size_t)row * ldo + 4 * c) = p;
        }
    }
}

extern "C" hipError_t dlms_ln_fix(const void* x, int ldx, long long xcs, const float* gamma, const float* beta, float eps, void* out,
                                  int ldo, int M, int K, hipStream_t stream) {
    if (M <= 0 || K % 4 || K > 64 * 4 * SK_MAX_LN_V4 || ldx % 2 || ldo % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ln_fix_kernel, dim3(M), dim3(64), 0, stream, reinterpret_cast<const long long*>(x), ldx, xcs, gamma,
                       beta, eps, reinterpret_cast<bf16_t*>(out), ldo, K);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Split-K flash-decode (K5): ONE WORKGROUP per (row, head), NW waves each streaming a contiguous
// slice of the row's keys with the online softmax of attn_wave_kernel (lane (g = lane>>3, c =
// lane&7) owns dims [8c, 8c+8) of keys 8i + g), then a log-sum-exp merge of the NW partial
// (max, sum, acc[64]) triples in a fixed order through LDS.  At batch 1 and 1024 cached keys this
// puts 12 x NW waves on the KV stream instead of 12.
constexpr int ATTN_WS_STRIDE = 68;  // floats per partial: m, l, pad, pad, o[64] (16-byte aligned o)

template <int NW, int SYNC>
__global__ __launch_bounds__(64 * NW) void attn_split_kernel(const bf16_t* __restrict__ q, int ldq,
                                                           const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                                           const int* __restrict__ row_slot,
                                                           const int* __restrict__ row_kvlen, bf16_t* out, int ldo,
                                                           int H, int t_max, int n_slots, float scale_log2,
                                                           float* __restrict__ ws, int* __restrict__ cnt, int NS) {
    __shared__ float part[NW][8][10];  // per wave, per dim chunk c: m, l, acc[8]
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = blockIdx.x;
    const int r = blockIdx.y;
    const int sw = blockIdx.z;  // which of the NS workgroups of this (row, head)
    const int g = lane >> 3;
    const int c = lane & 7;
    const int slot = (int)dlms_idx(row_slot[r], n_slots, CHK_ATTN_SLOT);
    int kvlen = row_kvlen[r];
    kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);
    // keys [w_lo, w_hi) belong to this workgroup, then split evenly over its NW waves
    const int wspan = ((kvlen + NS - 1) / NS + 7) & ~7;
    const int w_lo = sw * wspan < kvlen ? sw * wspan : kvlen;
    const int w_hi = w_lo + wspan < kvlen ? w_lo + wspan : kvlen;
    const int span = ((w_hi - w_lo + NW - 1) / NW + 7) & ~7;
    const int t_lo = w_lo + wave * span < w_hi ? w_lo + wave * span : w_hi;
    const int t_hi = t_lo + span < w_hi ? t_lo + span : w_hi;
    const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
    const bf16_t* K = kc + head_off + c * 8;
    const bf16_t* V = vc + head_off + c * 8;

    float qf[8];
    unpack8(*reinterpret_cast<const uint4*>(q + (size_t)r * ldq + h * 64 + c * 8), qf);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[j] *= scale_log2;

    float m = -INFINITY, l = 0.f;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

    constexpr int U = 4;  // key groups of 8 in flight per wave (profiles/r2_attn_split_unroll.txt)
    for (int t0 = t_lo; t0 < t_hi; t0 += 8 * U) {
        uint4 kr[U], vr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int t = t0 + u * 8 + g;
            t = t < t_hi ? t : t_hi - 1;
            typedef unsigned int u32x4n_t __attribute__((ext_vector_type(4)));
            const u32x4n_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4n_t*>(K + (size_t)t * 64));
            const u32x4n_t b = __builtin_nontemporal_load(reinterpret_cast<const u32x4n_t*>(V + (size_t)t * 64));
            kr[u] = make_uint4(a.x, a.y, a.z, a.w);
            vr[u] = make_uint4(b.x, b.y, b.z, b.w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float kf[8];
            unpack8(kr[u], kf);
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) s += qf[j] * kf[j];
            s = group8_sum(s);
            if (t0 + u * 8 + g < t_hi) {
                const float m_new = fmaxf(m, s);
                const float corr = exp2f(m - m_new);
                const float p = exp2f(s - m_new);
                float vf[8];
                unpack8(vr[u], vf);
                l = l * corr + p;
#pragma unroll
                for (int j = 0; j < 8; ++j) acc[j] = acc[j] * corr + p * vf[j];
                m = m_new;
            }
        }
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
        float mx, my, lx, ly;  // (own, partner) or (lower, upper): the merge is symmetric
        lane_pair(m, o, mx, my);
        lane_pair(l, o, lx, ly);
        const float m_n = fmaxf(mx, my);
        const float a = mx == -INFINITY ? 0.f : exp2f(mx - m_n);
        const float b = my == -INFINITY ? 0.f : exp2f(my - m_n);
        l = lx * a + ly * b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float ax, ay;
            lane_pair(acc[j], o, ax, ay);
            acc[j] = ax * a + ay * b;
        }
        m = m_n;
    }
    if (g == 0) {
        part[wave][c][0] = m;
        part[wave][c][1] = l;
#pragma unroll
        for (int j = 0; j < 8; ++j) part[wave][c][2 + j] = acc[j];
    }
    __syncthreads();
    if (wave != 0) return;
    if (g == 0) {
        float M_ = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; ++w) M_ = fmaxf(M_, part[w][c][0]);
        float L = 0.f, o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            const float mw = part[w][c][0];
            if (mw == -INFINITY) continue;  // empty slice
            const float f = exp2f(mw - M_);
            L += part[w][c][1] * f;
#pragma unroll
            for (int j = 0; j < 8; ++j) o8[j] += part[w][c][2 + j] * f;
        }
        if (NS == 1) {
            const float inv = 1.f / L;
#pragma unroll
            for (int j = 0; j < 8; ++j) o8[j] *= inv;
            *reinterpret_cast<uint4*>(out + (size_t)r * ldo + h * 64 + c * 8) = pack8(o8);
            return;
        }
        // several workgroups per (row, head): publish (m, l, unnormalised o[64])
        float* my = ws + ((size_t)(r * H + h) * NS + sw) * ATTN_WS_STRIDE;
        if (SYNC == 0) {
            if (c == 0) {
                my[0] = M_;
                my[1] = L;
            }
            *reinterpret_cast<float4*>(my + 4 + c * 8) = make_float4(o8[0], o8[1], o8[2], o8[3]);
            *reinterpret_cast<float4*>(my + 8 + c * 8) = make_float4(o8[4], o8[5], o8[6], o8[7]);
        } else {  // device-coherent (write-through) stores: nothing dirty is left in this XCD's L2
            if (c == 0) {
                __hip_atomic_store(my, M_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(my + 1, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __hip_atomic_store(my + 4 + c * 8 + j, o8[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (NS == 1) return;
    // last-arriver merge (stream-K fix-up): publish our partial device-wide, count arrivals;
    // the workgroup that arrives last merges all NS partials and re-arms the counter.  Nobody
    // waits on anybody, so there is no co-residency assumption.
    if (SYNC == 2)  // our write-through stores have all been acknowledged (explicit: the compiler
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // emits no wait for a workgroup fence)
    else
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    int old = 0;
    if (lane == 0) old = atomicAdd(cnt + r * H + h, 1);
    old = __shfl(old, 0, 64);
    if (old != NS - 1) return;
    if (SYNC != 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const float* base = ws + (size_t)(r * H + h) * NS * ATTN_WS_STRIDE;
    auto ld = [](const float* p) {
        return SYNC == 0 ? *p : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    float M_ = -INFINITY;
    for (int k = 0; k < NS; ++k) M_ = fmaxf(M_, ld(base + k * ATTN_WS_STRIDE));
    float L = 0.f, o = 0.f;
    for (int k = 0; k < NS; ++k) {
        const float* pk = base + k * ATTN_WS_STRIDE;
        const float mk = ld(pk);
        if (mk == -INFINITY) continue;
        const float f = exp2f(mk - M_);
        L += ld(pk + 1) * f;
        o += ld(pk + 4 + lane) * f;
    }
    out[(size_t)r * ldo + h * 64 + lane] = f32_to_bf16(o / L);
    if (lane == 0) atomicExch(cnt + r * H + h, 0);
}

extern "C" hipError_t dlms_attention_split(const void* q, int ldq, const void* kc, const void* vc, const int* row_slot,
                                           const int* row_kvlen, void* out, int ldo, int R, int H, int t_max,
                                           int n_slots, float scale, int nw, int ns, float* ws, int* cnt,
                                           int sync, hipStream_t stream) {
    if (R <= 0 || H <= 0 || t_max <= 0 || ns < 1 || ns > 64) return hipErrorInvalidValue;
    if (ns > 1 && (ws == nullptr || cnt == nullptr)) return hipErrorInvalidValue;
    const float sl2 = scale * 1.4426950408889634f;
    auto go = [&](auto kern, int threads) {
        hipLaunchKernelGGL(kern, dim3(H, R, ns), dim3(threads), 0, stream, reinterpret_cast<const bf16_t*>(q), ldq,
                           reinterpret_cast<const bf16_t*>(kc), reinterpret_cast<const bf16_t*>(vc), row_slot,
                           row_kvlen, reinterpret_cast<bf16_t*>(out), ldo, H, t_max, n_slots, sl2, ws, cnt, ns);
    };
    auto pick = [&](auto sync_c) -> bool {
        constexpr int S = decltype(sync_c)::value;
        switch (nw) {
            case 2: go(attn_split_kernel<2, S>, 128); return true;
            case 4: go(attn_split_kernel<4, S>, 256); return true;
            case 8: go(attn_split_kernel<8, S>, 512); return true;
            case 16: go(attn_split_kernel<16, S>, 1024); return true;
            default: return false;
        }
    };
    bool ok = sync == 0 ? pick(std::integral_constant<int, 0>{})
            : sync == 1 ? pick(std::integral_constant<int, 1>{})
                        : pick(std::integral_constant<int, 2>{});
    if (!ok) return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Attention + out-projection in ONE kernel (latency path, M <= 4 rows).
//
// The batch-1 layer is a chain of latency-bound launches; this removes one: workgroup (h, j)
// computes head h's attention for all M rows (its keys split over the 4 waves, log-sum-exp merge in
// LDS) and multiplies the 64-wide result by its NT 16-column tiles of W_o (pre-shuffled; the tiles'
// k-blocks 2h, 2h+1 are loaded at kernel start, under the attention).  The J = N / (16 NT)
// workgroups of a head recompute the same attention (a few KB of K/V per row at GPT-2 lengths,
// L2-served) so that the out-projection's weights are spread over H * J workgroups.  Head h's
// contribution goes to split-K slab h with plain stores; the next fused add+LN kernel sums the H
// slabs in fixed order (deterministic).  (Summing them here instead -- write-through partials +
// an arrival counter + last-arriver reduce -- measured 11.8 us per call against 5.5 + 5.1 for the
// two kernels it replaced: three dependent global round trips cost what a launch boundary does.)
template <int NT>
__global__ __launch_bounds__(256) void attn_oproj_kernel(
    const bf16_t* __restrict__ q, int ldq, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ row_slot, const int* __restrict__ row_kvlen, int M, int H, int t_max, int n_slots,
    float scale_log2, const bf16_t* __restrict__ Wo_sh, int N, float* __restrict__ part, int ldp,
    long long split_stride) {
    constexpr int NW = 4;
    constexpr int TPW = (NT + NW - 1) / NW;  // output tiles per wave
    constexpr int U = 8;                      // key groups of 8 in flight per wave
    __shared__ float part_s[NW][8][10];
    __shared__ __attribute__((aligned(16))) bf16_t aimg[16][72];  // o as the MFMA A operand, padded rows
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int h = blockIdx.x;
    const int j = blockIdx.y;
    const int nkb = (H * 64) >> 5;

    // (0) this workgroup's W_o fragments first: they do not depend on the attention
    bf16x8_t wb[TPW][2];
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + NW * i < NT ? wave + NW * i : NT - 1;
        const bf16x8_t* src = reinterpret_cast<const bf16x8_t*>(Wo_sh) + ((size_t)(j * NT + t) * nkb + 2 * h) * 64 + lane;
        wb[i][0] = src[0];
        wb[i][1] = src[64];
    }

    // (1) attention of head h: S = 4 / M waves per row
    const int S = M == 1 ? 4 : (M == 2 ? 2 : 1);
    const int row = wave / S;
    const int sl = wave - row * S;
    const int g = lane >> 3;
    const int c = lane & 7;
    float m = -INFINITY, l = 0.f;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (row < M) {
        const int slot = (int)dlms_idx(row_slot[row], n_slots, CHK_ATTN_SLOT);
        int kvlen = row_kvlen[row];
        kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);
        const int span = ((kvlen + S - 1) / S + 7) & ~7;
        const int t_lo = sl * span < kvlen ? sl * span : kvlen;
        const int t_hi = t_lo + span < kvlen ? t_lo + span : kvlen;
        const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
        const bf16_t* K = kc + head_off + c * 8;
        const bf16_t* V = vc + head_off + c * 8;
        float qf[8];
        unpack8(*reinterpret_cast<const uint4*>(q + (size_t)row * ldq + h * 64 + c * 8), qf);
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[e] *= scale_log2;
        for (int t0 = t_lo; t0 < t_hi; t0 += 8 * U) {
            uint4 kr[U], vr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int t = t0 + u * 8 + g;
                t = t < t_hi ? t : t_hi - 1;
                kr[u] = *reinterpret_cast<const uint4*>(K + (size_t)t * 64);
                vr[u] = *reinterpret_cast<const uint4*>(V + (size_t)t * 64);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float kf[8];
                unpack8(kr[u], kf);
                float sc = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) sc += qf[e] * kf[e];
                sc = group8_sum(sc);
                if (t0 + u * 8 + g < t_hi) {
                    const float m_new = fmaxf(m, sc);
                    const float corr = exp2f(m - m_new);
                    const float p = exp2f(sc - m_new);
                    float vf[8];
                    unpack8(vr[u], vf);
                    l = l * corr + p;
#pragma unroll
                    for (int e = 0; e < 8; ++e) acc[e] = acc[e] * corr + p * vf[e];
                    m = m_new;
                }
            }
        }
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
        float mx, my, lx, ly;  // (own, partner) or (lower, upper): the merge is symmetric
        lane_pair(m, o, mx, my);
        lane_pair(l, o, lx, ly);
        const float m_n = fmaxf(mx, my);
        const float a = mx == -INFINITY ? 0.f : exp2f(mx - m_n);
        const float b = my == -INFINITY ? 0.f : exp2f(my - m_n);
        l = lx * a + ly * b;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float ax, ay;
            lane_pair(acc[e], o, ax, ay);
            acc[e] = ax * a + ay * b;
        }
        m = m_n;
    }
    if (g == 0) {
        part_s[wave][c][0] = m;
        part_s[wave][c][1] = l;
#pragma unroll
        for (int e = 0; e < 8; ++e) part_s[wave][c][2 + e] = acc[e];
    }
    __syncthreads();
    if (threadIdx.x < 128) {  // (row r, 8-dim chunk cc) -> bf16 A image; rows >= M are zero
        const int r = threadIdx.x >> 3, cc = threadIdx.x & 7;
        float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (r < M) {
            float M_ = -INFINITY;
            for (int w = r * S; w < r * S + S; ++w) M_ = fmaxf(M_, part_s[w][cc][0]);
            float L = 0.f;
            for (int w = r * S; w < r * S + S; ++w) {
                const float mw = part_s[w][cc][0];
                if (mw == -INFINITY) continue;
                const float f = exp2f(mw - M_);
                L += part_s[w][cc][1] * f;
#pragma unroll
                for (int e = 0; e < 8; ++e) o8[e] += part_s[w][cc][2 + e] * f;
            }
            const float inv = 1.f / L;
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[e] *= inv;
        }
        *reinterpret_cast<uint4*>(&aimg[r][cc * 8]) = pack8(o8);
    }
    __syncthreads();

    // (2) o[16 x 64] . W_o[tile cols, head h's 64 k]^T on MFMA -> slab h
    const int fr = lane & 15, gg = lane >> 4;
    const bf16x8_t a0 = *reinterpret_cast<const bf16x8_t*>(&aimg[fr][gg * 8]);
    const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(&aimg[fr][32 + gg * 8]);
    float* slab = part + (size_t)h * split_stride;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + NW * i;
        if (t >= NT) continue;  // wave-uniform
        f32x4_t d = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wb[i][0], d, 0, 0, 0);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb[i][1], d, 0, 0, 0);
        const int col = (j * NT + t) * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int rr = gg * 4 + r;
            if (rr < M) slab[(size_t)rr * ldp + col] = d[r];
        }
    }
}

// Head-grouped variant for ONE row (batch 1): workgroup (g, j) covers HG heads with WPH waves per
// head (keys split WPH ways, log-sum-exp merge in LDS) and their 2*HG k-blocks of its NT W_o tiles,
// so the out-projection lands in H / HG slabs instead of H -- with HG = H / 4 exactly the four
// split-K slabs the fused add+LN kernel already sums (12 slabs cost that kernel ~2 us at batch 1).
// (Groups of 5 heads at 2 waves per head for GPT-2-large / XL measured slower than the split
// attention + in-place out-projection: profiles/r5_large_xl_hg5_tiles_ab.jsonl.)
template <int HG, int NT, int WPH>
__global__ __launch_bounds__(64 * WPH * HG) void attn_oproj_hg_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ row_slot, const int* __restrict__ row_kvlen, int H, int t_max, int n_slots,
    float scale_log2, const bf16_t* __restrict__ Wo_sh, int N, float* __restrict__ part, long long split_stride) {
    constexpr int NW = WPH * HG;
    static_assert(NW <= 16 && NT <= NW && 16 * 8 * HG <= 64 * NW, "workgroup geometry");
    constexpr int U = NW >= 16 ? 4 : 8;  // 16 waves per CU leave 128 VGPRs per lane
    constexpr int AW = HG * 64 + 8;  // A image row (bf16), padded
    __shared__ float part_s[NW][8][10];
    __shared__ __attribute__((aligned(16))) bf16_t aimg[16][AW];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int grp = blockIdx.x;
    const int j = blockIdx.y;
    const int nkb = (H * 64) >> 5;
    const int fr = lane & 15, gg = lane >> 4;

    // (0) W_o fragments: wave t < NT owns output tile j*NT + t, k-blocks of the group's heads
    bf16x8_t wb[2 * HG];
    if (wave < NT) {
        const bf16x8_t* src =
            reinterpret_cast<const bf16x8_t*>(Wo_sh) + ((size_t)(j * NT + wave) * nkb + 2 * HG * grp) * 64 + lane;
#pragma unroll
        for (int k = 0; k < 2 * HG; ++k) wb[k] = src[k * 64];
    }

    // (1) attention: wave w -> head grp*HG + w/WPH, key slice w%WPH
    const int hh = wave / WPH, sl = wave % WPH;
    const int h = grp * HG + hh;
    const int g = lane >> 3, c = lane & 7;
    const int slot = (int)dlms_idx(row_slot[0], n_slots, CHK_ATTN_SLOT);
    int kvlen = row_kvlen[0];
    kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);
    const int span = ((kvlen + WPH - 1) / WPH + 7) & ~7;
    const int t_lo = sl * span < kvlen ? sl * span : kvlen;
    const int t_hi = t_lo + span < kvlen ? t_lo + span : kvlen;
    const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
    const bf16_t* K = kc + head_off + c * 8;
    const bf16_t* V = vc + head_off + c * 8;
    float qf[8];
    unpack8(*reinterpret_cast<const uint4*>(q + h * 64 + c * 8), qf);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[e] *= scale_log2;
    float m = -INFINITY, l = 0.f;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t0 = t_lo; t0 < t_hi; t0 += 8 * U) {
        uint4 kr[U], vr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int t = t0 + u * 8 + g;
            t = t < t_hi ? t : t_hi - 1;
            kr[u] = *reinterpret_cast<const uint4*>(K + (size_t)t * 64);
            vr[u] = *reinterpret_cast<const uint4*>(V + (size_t)t * 64);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float kf[8];
            unpack8(kr[u], kf);
            float sc = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) sc += qf[e] * kf[e];
            sc = group8_sum(sc);
            if (t0 + u * 8 + g < t_hi) {
                const float m_new = fmaxf(m, sc);
                const float corr = exp2f(m - m_new);
                const float p = exp2f(sc - m_new);
                float vf[8];
                unpack8(vr[u], vf);
                l = l * corr + p;
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] = acc[e] * corr + p * vf[e];
                m = m_new;
            }
        }
    }
#pragma unroll
    for (int o = 8; o < 64; o <<= 1) {
        float mx, my, lx, ly;  // (own, partner) or (lower, upper): the merge is symmetric
        lane_pair(m, o, mx, my);
        lane_pair(l, o, lx, ly);
        const float m_n = fmaxf(mx, my);
        const float a = mx == -INFINITY ? 0.f : exp2f(mx - m_n);
        const float b = my == -INFINITY ? 0.f : exp2f(my - m_n);
        l = lx * a + ly * b;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float ax, ay;
            lane_pair(acc[e], o, ax, ay);
            acc[e] = ax * a + ay * b;
        }
        m = m_n;
    }
    if (g == 0) {
        part_s[wave][c][0] = m;
        part_s[wave][c][1] = l;
#pragma unroll
        for (int e = 0; e < 8; ++e) part_s[wave][c][2 + e] = acc[e];
    }
    __syncthreads();
    if (threadIdx.x < 16 * 8 * HG) {  // (row r, head hh2, chunk cc) -> A image (row 0 real, rows 1..15 zero)
        const int r = threadIdx.x / (8 * HG);
        const int hh2 = (threadIdx.x / 8) % HG, cc = threadIdx.x & 7;
        float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (r == 0) {
            float M_ = -INFINITY;
#pragma unroll
            for (int w = 0; w < WPH; ++w) M_ = fmaxf(M_, part_s[hh2 * WPH + w][cc][0]);
            float L = 0.f;
#pragma unroll
            for (int w = 0; w < WPH; ++w) {
                const float mw = part_s[hh2 * WPH + w][cc][0];
                if (mw == -INFINITY) continue;
                const float f = exp2f(mw - M_);
                L += part_s[hh2 * WPH + w][cc][1] * f;
#pragma unroll
                for (int e = 0; e < 8; ++e) o8[e] += part_s[hh2 * WPH + w][cc][2 + e] * f;
            }
            const float inv = 1.f / L;
#pragma unroll
            for (int e = 0; e < 8; ++e) o8[e] *= inv;
        }
        *reinterpret_cast<uint4*>(&aimg[r][hh2 * 64 + cc * 8]) = pack8(o8);
    }
    __syncthreads();

    // (2) o[16 x HG*64] . W_o[tile, group k-blocks]^T -> slab grp (row 0 only)
    if (wave >= NT) return;
    f32x4_t d = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2 * HG; ++k) {
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(&aimg[fr][k * 32 + gg * 8]);
        d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[k], d, 0, 0, 0);
    }
    if (gg == 0) part[(size_t)grp * split_stride + (j * NT + wave) * 16 + fr] = d[0];  // row 0 of the tile
}

extern "C" hipError_t dlms_attention_oproj_grouped(const void* q, const void* kc, const void* vc, const int* row_slot,
                                                   const int* row_kvlen, int H, int hg, int t_max, int n_slots,
                                                   float scale, const void* wo_sh, int N, int nt, float* part,
                                                   long long split_stride, hipStream_t stream) {
    if (H < 1 || hg < 1 || H % hg || t_max < 1 || N % 16 || nt < 1 || nt > 4 * hg || (N / 16) % nt)
        return hipErrorInvalidValue;
    const float sl2 = scale * 1.4426950408889634f;
    const dim3 grid(H / hg, (N / 16) / nt);
    auto go = [&](auto kern, int threads) {
        hipLaunchKernelGGL(kern, grid, dim3(threads), 0, stream, reinterpret_cast<const bf16_t*>(q),
                           reinterpret_cast<const bf16_t*>(kc), reinterpret_cast<const bf16_t*>(vc), row_slot,
                           row_kvlen, H, t_max, n_slots, sl2, reinterpret_cast<const bf16_t*>(wo_sh), N, part,
                           split_stride);
    };
#define AOG(HG_, NT_, WPH_) \
    if (hg == HG_ && nt == NT_) { go(attn_oproj_hg_kernel<HG_, NT_, WPH_>, 64 * WPH_ * HG_); return hipGetLastError(); }
    AOG(3, 1, 4) AOG(3, 2, 4) AOG(3, 3, 4) AOG(3, 4, 4) AOG(4, 1, 4) AOG(4, 2, 4) AOG(4, 3, 4) AOG(4, 4, 4)
#undef AOG
    return hipErrorInvalidValue;
}

extern "C" hipError_t dlms_attention_oproj(const void* q, int ldq, const void* kc, const void* vc, const int* row_slot,
                                           const int* row_kvlen, int M, int H, int t_max, int n_slots, float scale,
                                           const void* wo_sh, int N, int nt, float* part, int ldp,
                                           long long split_stride, hipStream_t stream) {
    if (M < 1 || M > 4 || H < 1 || t_max < 1 || N % 16 || nt < 1 || (N / 16) % nt) return hipErrorInvalidValue;
    const float sl2 = scale * 1.4426950408889634f;
    const dim3 grid(H, (N / 16) / nt);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(q), ldq,
                           reinterpret_cast<const bf16_t*>(kc), reinterpret_cast<const bf16_t*>(vc), row_slot,
                           row_kvlen, M, H, t_max, n_slots, sl2, reinterpret_cast<const bf16_t*>(wo_sh), N, part,
                           ldp, split_stride);
    };
    switch (nt) {
        case 2: go(attn_oproj_kernel<2>); break;
        case 3: go(attn_oproj_kernel<3>); break;
        case 4: go(attn_oproj_kernel<4>); break;
        case 5: go(attn_oproj_kernel<5>); break;
        case 6: go(attn_oproj_kernel<6>); break;
        case 8: go(attn_oproj_kernel<8>); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

DLMS_CHECK_EXPORT(skinny)
