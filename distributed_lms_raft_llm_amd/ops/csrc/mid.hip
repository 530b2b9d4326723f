// Mid-batch decode (9-64 concurrent queries: BASELINE config 2's 32 students): LayerNorm fused
// into the column-parallel GEMMs of a decode layer.
//
// At 9-64 rows the tiled decode step spends 7 kernels per layer (add+LN1, QKV, attention,
// out-projection split-K partials, add+LN2, c_fc, c_proj partials; profiles/r6_base_decode_b32 --
// ~39 us per layer), and every one of them is latency-bound: the weights are the same 14 MB per
// layer as at batch 1 and the MFMA work is a rounding error.  The mid path runs 5 per layer:
//
//   [LN1 + QKV + K/V scatter] -> attention -> [out-proj, x += in place] -> [LN2 + c_fc + GELU]
//   -> [c_proj, x += in place]
//
// The row-parallel projections are the column-owning skinny GEMMs of skinny.hip (every workgroup
// owns whole output columns, so the residual is updated in place and no split-K slabs exist), so
// the residual is COMPLETE when the next LayerNorm needs it and that LayerNorm can run in the
// prologue of the GEMM that consumes it.  This file holds that fused kernel.
//
// mid_ln_gemm_kernel<EPI, MT, NW, CG, NV4, KBW>: grid = N / (16 CG) workgroups of NW waves; wave
// group cgi (NW / CG waves) owns the 16-column group blockIdx.x * CG + cgi and splits its K/32
// k-blocks; W is pre-shuffled into MFMA B-fragment order ([N/16][K/32][64][8] bf16, one contiguous
// KiB per wave instruction).  Order of work per workgroup:
//   1. every wave issues ALL its weight-fragment loads (HBM, no dependency on the activations);
//   2. the M residual rows are LayerNormed by all NW waves together: RPW = 16 MT / NW rows per
//      wave, every row's loads issued before the first reduction (one L2 round trip for the whole
//      prologue -- the skinny kernels' per-row loop paid one per row and scaled with M), two-pass
//      fp32 statistics like norm.hip, bf16 into a padded LDS image (conflict-free ds_read_b128);
//   3. v_mfma_f32_16x16x32_bf16 over the wave's k-blocks for the MT row tiles;
//   4. fixed-order K-slice reduction through LDS, then the column-owning epilogue
//      (skinny_common.h: QKV q-out + K/V cache scatter, GELU-tanh, or bf16).
// Every workgroup re-normalises the same rows (M * d * 4 B from L2: 96 KB at 32 rows); at these
// sizes that is cheaper than a separate LayerNorm launch and its round trip.
#include "common.h"
#include "skinny_common.h"

namespace mid {

constexpr int MAX_NV4 = 4;  // K <= 64 lanes * 4 * 4 = 1024 (GPT-2 small / medium)

template <int EPI, int MT, int NW, int CG, int NV4, int KBW>
__global__ __launch_bounds__(64 * NW) void mid_ln_gemm_kernel(const float* __restrict__ x, int ldx,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps,
                                                            const bf16_t* __restrict__ Wsh, int M, int N, int K,
                                                            GemmEpi ep) {
    constexpr int WPG = NW / CG;
    constexpr int RPW = 16 * MT / NW;
    static_assert(NW % CG == 0 && (16 * MT) % NW == 0, "whole waves per column group, whole rows per wave");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cgi = wave / WPG;
    const int kpart = wave % WPG;
    const int ng = blockIdx.x * CG + cgi;
    const int nkb = K >> 5;
    const int per = (nkb + WPG - 1) / WPG;
    const int kb0 = kpart * per < nkb ? kpart * per : nkb;
    const int nk = (kb0 + per < nkb ? kb0 + per : nkb) - kb0;
    const int kbl = nk > 0 ? kb0 : 0;
    const int last = nk > 0 ? nk - 1 : 0;
    const int g = lane >> 4, fr = lane & 15;
    const int row_bytes = K * 2 + 16;
    // row block blockIdx.y: rows [row0, row0 + 16 MT) of the M (a grid of several row blocks puts
    // the same weights on more CUs, each with fewer activation bytes to pull)
    const int row0 = blockIdx.y * 16 * MT;
    x += (size_t)row0 * ldx;
    M = M - row0 < 16 * MT ? M - row0 : 16 * MT;

    // 1. weights first: every fragment of this wave in flight before the activations
    const bf16x8_t* wsrc = reinterpret_cast<const bf16x8_t*>(Wsh) + ((size_t)ng * nkb + kbl) * 64 + lane;
    bf16x8_t b[KBW];
#pragma unroll
    for (int u = 0; u < KBW; ++u) b[u] = *(wsrc + (size_t)(u < nk ? u : last) * 64);

    // 2. LayerNorm of the M rows, all of this wave's row loads issued together
    const int nv = K >> 2;
    int cidx[NV4];
    bool valid[NV4];
#pragma unroll
    for (int c = 0; c < NV4; ++c) {
        const int cc = lane + 64 * c;
        valid[c] = cc < nv;
        cidx[c] = valid[c] ? cc : nv - 1;
    }
    float4 v[RPW][NV4];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        int row = wave + NW * i;
        row = row < M ? row : M - 1;  // (rows >= M: loaded, normalised, never stored)
        const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * ldx);
#pragma unroll
        for (int c = 0; c < NV4; ++c) v[i][c] = xr[cidx[c]];
    }
    float4 gv[NV4], bv[NV4];
#pragma unroll
    for (int c = 0; c < NV4; ++c) {
        gv[c] = reinterpret_cast<const float4*>(gamma)[cidx[c]];
        bv[c] = reinterpret_cast<const float4*>(beta)[cidx[c]];
    }
    __builtin_amdgcn_sched_barrier(0);  // weights, rows and LN parameters all in flight together
    const float inv_k = 1.f / (float)K;
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int row = wave + NW * i;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NV4; ++c)
            if (valid[c]) s += (v[i][c].x + v[i][c].y) + (v[i][c].z + v[i][c].w);
        const float mean = wave_sum(s) * inv_k;
        float ss = 0.f;
#pragma unroll
        for (int c = 0; c < NV4; ++c) {
            if (valid[c]) {
                const float a0 = v[i][c].x - mean, a1 = v[i][c].y - mean, a2 = v[i][c].z - mean, a3 = v[i][c].w - mean;
                ss += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
            }
        }
        const float rstd = rsqrtf(wave_sum(ss) * inv_k + eps);
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
    __syncthreads();

    // 3. MFMA over this wave's k-blocks, MT row tiles
    f32x4_t acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < KBW; ++u) {
        if (u >= nk) continue;  // wave-uniform
#pragma unroll
        for (int t = 0; t < MT; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_a_frag(smem, row_bytes, 16 * t + fr, kb0 + u, g), b[u],
                                                            acc[t], 0, 0, 0);
    }

    // 4. fixed-order reduction of the WPG K slices of each column group, then the epilogue
    if constexpr (WPG > 1) {
        __syncthreads();  // the LN image is no longer read: reuse it
        float* red = reinterpret_cast<float*>(smem);
        if (kpart > 0) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
                *reinterpret_cast<f32x4_t*>(red + ((size_t)(wave * MT + t) * 64 + lane) * 4) = acc[t];
        }
        __syncthreads();
        if (kpart != 0) return;
#pragma unroll
        for (int s = 1; s < WPG; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t)
                acc[t] += *reinterpret_cast<const f32x4_t*>(red + ((size_t)((wave + s) * MT + t) * 64 + lane) * 4);
    }
    skinny_store<EPI, MT>(acc, M, ng * 16 + fr, g, ep, row0);
}

// LDS bytes of one launch: the LN image (16 MT rows) or the K-slice partials, whichever is larger
__host__ constexpr size_t lds_bytes(int MT, int NW, int K) {
    const size_t img = (size_t)16 * MT * (K * 2 + 16);
    const size_t red = (size_t)NW * MT * 64 * 16;
    return img > red ? img : red;
}

template <int EPI, int MT, int NW, int CG, int NV4>
static hipError_t launch(const float* x, int ldx, const float* g, const float* b, float eps, const bf16_t* W, int M,
                         int N, int K, const GemmEpi& ep, hipStream_t stream) {
    constexpr int WPG = NW / CG;
    const int per = ((K >> 5) + WPG - 1) / WPG;
    if (N % (16 * CG)) return hipErrorInvalidValue;
    const size_t lds = lds_bytes(MT, NW, K);
    auto go = [&](auto kern) -> hipError_t {
        static std::atomic<uint64_t> attr_set{0};  // per device
        if (lds > 65536)
            if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(kern), (int)lds); e != hipSuccess)
                return e;
        hipLaunchKernelGGL(kern, dim3(N / (16 * CG), (M + 16 * MT - 1) / (16 * MT)), dim3(64 * NW), lds, stream, x, ldx,
                           g, b, eps, W, M, N, K, ep);
        return hipGetLastError();
    };
    if (per <= 4) return go(mid_ln_gemm_kernel<EPI, MT, NW, CG, NV4, 4>);
    if (per <= 8) return go(mid_ln_gemm_kernel<EPI, MT, NW, CG, NV4, 8>);
    if (per <= 12) return go(mid_ln_gemm_kernel<EPI, MT, NW, CG, NV4, 12>);
    return hipErrorInvalidValue;
}

// geometry: (waves per workgroup, column groups per workgroup, row tiles per workgroup).  MT = 0:
// one workgroup row block holds all M rows (up to 4 tiles); MT > 0: row blocks of 16 MT rows on
// grid.y.  geo 0 = the default: one row tile per workgroup (row blocks of 16) -- the time of these
// kernels tracks the bytes each CU pulls (the activation rows dominate: 96 KB of f32 x at 32 rows
// against 24 KB of weights), so more, thinner workgroups win (profiles/r6_mid_kernels.jsonl).
template <int EPI, int NV4>
static hipError_t pick_geometry(int geo, const float* x, int ldx, const float* g, const float* b, float eps,
                                const bf16_t* W, int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
    const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);  // all rows in one block
#define MID_LN(MT_, NW_, CG_) return launch<EPI, MT_, NW_, CG_, NV4>(x, ldx, g, b, eps, W, M, N, K, ep, stream)
#define MID_LN_ALL(NW_, CG_) \
    if (mt == 1) MID_LN(1, NW_, CG_); \
    if (mt == 2) MID_LN(2, NW_, CG_); \
    MID_LN(4, NW_, CG_)
    switch (geo) {
        case 0:  // 16-row blocks; 8 waves up to 32 rows, 4 waves (two workgroups per CU) above
            if (M <= 32) MID_LN(1, 8, 1);
            MID_LN(1, 4, 1);
        case 4: MID_LN(1, 8, 1);
        case 1: MID_LN_ALL(8, 1);
        case 2:  // (4 waves would hold 16 rows each at 64 rows)
            if (mt == 1) MID_LN(1, 4, 1);
            if (mt == 2) MID_LN(2, 4, 1);
            return hipErrorInvalidValue;
        case 3: MID_LN_ALL(8, 2);
        case 5: MID_LN(1, 4, 1);
        case 6: MID_LN(2, 8, 1);
        case 7: MID_LN(1, 16, 1);  // (16 waves: one row each)
        default: return hipErrorInvalidValue;
    }
#undef MID_LN_ALL
#undef MID_LN
}

template <int EPI>
static hipError_t by_shape(int geo, const float* x, int ldx, const float* g, const float* b, float eps, const bf16_t* W,
                           int M, int N, int K, const GemmEpi& ep, hipStream_t stream) {
    switch ((K / 4 + 63) / 64) {
        case 3: return pick_geometry<EPI, 3>(geo, x, ldx, g, b, eps, W, M, N, K, ep, stream);
        case 4: return pick_geometry<EPI, 4>(geo, x, ldx, g, b, eps, W, M, N, K, ep, stream);
        default: return hipErrorInvalidValue;
    }
}


// ---------------------------------------------------------------------------------------------
// In-place row-parallel projection of the mid path: x[M][N] += a[M][K] . W^T + bias (out-projection
// and c_proj), column-owning so the residual is complete for the next fused LayerNorm.
//
// grid = N / (16 CG) workgroups of NW waves; WPG = NW / CG waves split the K/32 k-blocks of a
// column group EXACTLY (KPW = nkb / WPG k-blocks each, a compile-time count: no per-wave trip
// conditions, so every load of the wave is one straight-line burst -- the generic skinny kernel's
// `u < nk` guards made the compiler version the loop and wait between the epilogue's stores).
// Each wave holds its KPW weight fragments and KPW x MT activation fragments in registers, all
// issued before the first MFMA; the WPG partial tiles are summed in a fixed order through LDS
// (deterministic), then the column group's wave 0 loads every old residual value of its rows in
// one burst and stores x + acc + bias.  FULL (M % 16 == 0, the engine's buckets): no row guards.
template <int MT, int NW, int CG, int KPW, bool FULL>
__global__ __launch_bounds__(64 * NW) void mid_proj_kernel(const bf16_t* __restrict__ a, int lda,
                                                         const bf16_t* __restrict__ Wsh,
                                                         const float* __restrict__ bias, float* __restrict__ x,
                                                         int ldx, int M, int K) {
    constexpr int WPG = NW / CG;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int cgi = wave / WPG;
    const int kpart = wave % WPG;
    const int ng = blockIdx.x * CG + cgi;
    const int nkb = K >> 5;
    const int kb0 = kpart * KPW;
    const int g = lane >> 4, fr = lane & 15;
    const int row0 = blockIdx.y * 16 * MT;  // row block (see mid_ln_gemm_kernel)
    a += (size_t)row0 * lda;
    x += (size_t)row0 * ldx;
    M = M - row0 < 16 * MT ? M - row0 : 16 * MT;

    const bf16x8_t* wsrc = reinterpret_cast<const bf16x8_t*>(Wsh) + ((size_t)ng * nkb + kb0) * 64 + lane;
    bf16x8_t b[KPW];
#pragma unroll
    for (int u = 0; u < KPW; ++u) b[u] = wsrc[(size_t)u * 64];
    bf16x8_t av[KPW][MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        int row = 16 * t + fr;
        if constexpr (!FULL) row = row < M ? row : M - 1;  // (rows >= M: computed, never stored)
        const bf16_t* ar = a + (size_t)row * lda + kb0 * 32 + g * 8;
#pragma unroll
        for (int u = 0; u < KPW; ++u) av[u][t] = *reinterpret_cast<const bf16x8_t*>(ar + u * 32);
    }
    // keep the whole burst ahead of the first MFMA: left alone, the scheduler sinks loads down to
    // their consumers to save registers (45-70 VGPRs), and the burst becomes several round trips
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < KPW; ++u)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[u][t], b[u], acc[t], 0, 0, 0);

    if constexpr (WPG > 1) {
        float* red = reinterpret_cast<float*>(smem);
        if (kpart > 0) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
                *reinterpret_cast<f32x4_t*>(red + ((size_t)(wave * MT + t) * 64 + lane) * 4) = acc[t];
        }
        __syncthreads();
        if (kpart != 0) return;
#pragma unroll
        for (int s = 1; s < WPG; ++s)
#pragma unroll
            for (int t = 0; t < MT; ++t)
                acc[t] += *reinterpret_cast<const f32x4_t*>(red + ((size_t)((wave + s) * MT + t) * 64 + lane) * 4);
    }
    const int col = ng * 16 + fr;
    const float bv = bias ? bias[col] : 0.f;
    float old[MT][4];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            int row = 16 * t + g * 4 + r;
            if constexpr (!FULL) row = row < M ? row : M - 1;
            old[t][r] = x[(size_t)row * ldx + col];
        }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * t + g * 4 + r;
            if (FULL || row < M) x[(size_t)row * ldx + col] = old[t][r] + (acc[t][r] + bv);
        }
}

template <int MT, int NW, int CG, int KPW>
static hipError_t launch_proj(const bf16_t* a, int lda, const bf16_t* W, const float* bias, float* x, int ldx, int M,
                              int N, int K, hipStream_t stream) {
    if (N % (16 * CG) || (K >> 5) != KPW * (NW / CG)) return hipErrorInvalidValue;
    const size_t lds = (size_t)NW * MT * 64 * 16;
    auto go = [&](auto kern) -> hipError_t {
        static std::atomic<uint64_t> attr_set{0};  // per device
        if (lds > 65536)
            if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(kern), (int)lds); e != hipSuccess)
                return e;
        hipLaunchKernelGGL(kern, dim3(N / (16 * CG), (M + 16 * MT - 1) / (16 * MT)), dim3(64 * NW), lds, stream, a, lda,
                           W, bias, x, ldx, M, K);
        return hipGetLastError();
    };
    if (M % (16 * MT) == 0) return go(mid_proj_kernel<MT, NW, CG, KPW, true>);
    return go(mid_proj_kernel<MT, NW, CG, KPW, false>);
}

// (waves, column groups, row tiles) per workgroup -- K = 768 / 1024 (out-projection), 3072 / 4096
// (c_proj); row tiles as in mid_ln_gemm's table (geo 0: row blocks of 16)
template <int MT>
static hipError_t proj_geo(int geo, const bf16_t* a, int lda, const bf16_t* W, const float* bias, float* x, int ldx,
                           int M, int N, int K, hipStream_t stream) {
    const int nkb = K >> 5;
#define MID_PROJ(NW_, CG_, KPW_) \
    if (nkb == KPW_ * (NW_ / CG_)) return launch_proj<MT, NW_, CG_, KPW_>(a, lda, W, bias, x, ldx, M, N, K, stream)
    switch (geo) {
        case 1:  // 8 waves per column group
            MID_PROJ(8, 1, 3); MID_PROJ(8, 1, 4); MID_PROJ(8, 1, 12); if constexpr (MT <= 2) { MID_PROJ(8, 1, 16); }
            break;
        case 2:  // 4 waves (spill-free up to 32 rows)
            MID_PROJ(4, 1, 6); MID_PROJ(4, 1, 8); if constexpr (MT == 1) { MID_PROJ(4, 1, 24); }
            break;
        case 3:  // 16 waves (c_proj: 6 / 8 k-blocks each)
            if constexpr (MT == 1) { MID_PROJ(16, 1, 6); MID_PROJ(16, 1, 8); }
            break;
        default: break;
    }
#undef MID_PROJ
    return hipErrorInvalidValue;
}

static hipError_t proj_shape(int geo, const bf16_t* a, int lda, const bf16_t* W, const float* bias, float* x, int ldx,
                             int M, int N, int K, hipStream_t stream) {
    const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
    switch (geo) {
        case 0:  // row blocks of 16: 16 waves where K splits into 6-8 k-blocks each (c_proj), else 4
            if ((K >> 5) % 16 == 0 && ((K >> 9) == 6 || (K >> 9) == 8))
                return proj_geo<1>(3, a, lda, W, bias, x, ldx, M, N, K, stream);
            return proj_geo<1>(2, a, lda, W, bias, x, ldx, M, N, K, stream);
        case 1:
        case 2:
        case 3:  // all rows in one block
            if (mt == 1) return proj_geo<1>(geo, a, lda, W, bias, x, ldx, M, N, K, stream);
            if (mt == 2) return proj_geo<2>(geo, a, lda, W, bias, x, ldx, M, N, K, stream);
            return proj_geo<4>(geo, a, lda, W, bias, x, ldx, M, N, K, stream);
        case 4: return proj_geo<1>(2, a, lda, W, bias, x, ldx, M, N, K, stream);  // row blocks of 16, 4 waves
        case 5: return proj_geo<1>(3, a, lda, W, bias, x, ldx, M, N, K, stream);  // row blocks of 16, 16 waves
        case 6: return proj_geo<2>(1, a, lda, W, bias, x, ldx, M, N, K, stream);  // row blocks of 32, 8 waves
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mid

// Largest M the mid-batch fused LN + GEMM takes (model width K; 0 = unsupported width)
extern "C" int dlms_mid_max_rows(int K) {
    const int nv4 = (K / 4 + 63) / 64;
    if (K % 32 || K % 4 || nv4 < 3 || nv4 > mid::MAX_NV4) return 0;
    return 64;
}

// out = epi(bf16(LN(x)) . W^T + bias): x f32 [M][ldx] (complete residual rows), W pre-shuffled
// [N/16][K/32][64][8] bf16; epi = SK_QKV / SK_GELU_TANH / SK_BF16 (skinny_common.h ids).
// geo: 0 = default geometry, 1..7 = tuning overrides (mid::pick_geometry).
extern "C" hipError_t dlms_mid_ln_gemm(int epi, const float* x, int ldx, const float* gamma, const float* beta, float eps,
                                       const void* Wsh, int M, int N, int K, const GemmEpi* ep, int geo,
                                       hipStream_t stream) {
    if (M <= 0 || M > dlms_mid_max_rows(K) || N % 16 || ldx % 4 || ldx < K) return hipErrorInvalidValue;
    const bf16_t* W = reinterpret_cast<const bf16_t*>(Wsh);
    switch (epi) {
        case SK_QKV: return mid::by_shape<SK_QKV>(geo, x, ldx, gamma, beta, eps, W, M, N, K, *ep, stream);
        case SK_GELU_TANH: return mid::by_shape<SK_GELU_TANH>(geo, x, ldx, gamma, beta, eps, W, M, N, K, *ep, stream);
        case SK_BF16: return mid::by_shape<SK_BF16>(geo, x, ldx, gamma, beta, eps, W, M, N, K, *ep, stream);
        default: return hipErrorInvalidValue;
    }
}

// x[M][N] += a[M][K] . W^T + bias in place (mid path out-projection / c_proj; a bf16 [M][lda], W
// pre-shuffled [N/16][K/32][64][8]).  geo: 0 = default, 1..6 tuning overrides (mid::proj_shape).
extern "C" hipError_t dlms_mid_proj(const void* a, int lda, const void* Wsh, const float* bias, float* x, int ldx,
                                    int M, int N, int K, int geo, hipStream_t stream) {
    if (M <= 0 || M > 64 || N % 16 || K % 32 || lda % 8 || ldx < N) return hipErrorInvalidValue;
    const bf16_t* A = reinterpret_cast<const bf16_t*>(a);
    const bf16_t* W = reinterpret_cast<const bf16_t*>(Wsh);
    return mid::proj_shape(geo, A, lda, W, bias, x, ldx, M, N, K, stream);
}
