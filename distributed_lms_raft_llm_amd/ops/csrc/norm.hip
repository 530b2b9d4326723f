// LayerNorm family (K2, K13).  One wave per row, the whole row held in registers
// (float4 loads, up to 8 per lane => d <= 2048), two-pass statistics in fp32.
#include "common.h"
#include <stdlib.h>

#define LN_MAX_V4 8  // float4 per lane -> d <= 64*4*8 = 2048

// y = LN(x) * gamma + beta.   x: f32 [M, ldx].  Writes bf16 (ldb) and/or f32 (ldf) outputs.
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int ldx,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, bf16_t* out_bf16, int ldb,
                                                        float* out_f32, int ldf, int M, int D, float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int nv = D >> 2;
    const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * ldx);
    float4 v[LN_MAX_V4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        v[i] = c < nv ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
            ss += (a * a + b * b) + (cc * cc + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    const float4* g4 = reinterpret_cast<const float4*>(gamma);
    const float4* b4 = reinterpret_cast<const float4*>(beta);
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float4 g = g4[c], b = b4[c];
            float4 y;
            y.x = (v[i].x - mean) * rstd * g.x + b.x;
            y.y = (v[i].y - mean) * rstd * g.y + b.y;
            y.z = (v[i].z - mean) * rstd * g.z + b.z;
            y.w = (v[i].w - mean) * rstd * g.w + b.w;
            if (out_f32) reinterpret_cast<float4*>(out_f32 + (size_t)row * ldf)[c] = y;
            if (out_bf16) {
                uint2 p;
                p.x = pack_bf16x2(y.x, y.y);
                p.y = pack_bf16x2(y.z, y.w);
                reinterpret_cast<uint2*>(out_bf16 + (size_t)row * ldb)[c] = p;
            }
        }
    }
}

// Gather variant: normalise only rows idx[0..M) of x (LM head on the last prompt token of each
// sequence after a packed prefill).
__global__ __launch_bounds__(256) void layernorm_gather_kernel(const float* __restrict__ x, int ldx,
                                                               const int* __restrict__ rows,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, bf16_t* out_bf16,
                                                               int ldb, int M, int D, float eps) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= M) return;
    const int row = rows[r];
    const int nv = D >> 2;
    const float4* xr = reinterpret_cast<const float4*>(x + (size_t)row * ldx);
    float4 v[LN_MAX_V4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        v[i] = c < nv ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
            ss += (a * a + b * b) + (cc * cc + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    const float4* g4 = reinterpret_cast<const float4*>(gamma);
    const float4* b4 = reinterpret_cast<const float4*>(beta);
#pragma unroll
    for (int i = 0; i < LN_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float4 g = g4[c], b = b4[c];
            uint2 p;
            p.x = pack_bf16x2((v[i].x - mean) * rstd * g.x + b.x, (v[i].y - mean) * rstd * g.y + b.y);
            p.y = pack_bf16x2((v[i].z - mean) * rstd * g.z + b.z, (v[i].w - mean) * rstd * g.w + b.w);
            reinterpret_cast<uint2*>(out_bf16 + (size_t)r * ldb)[c] = p;
        }
    }
}

extern "C" hipError_t dlms_layernorm(const float* x, int ldx, const float* gamma, const float* beta, void* out_bf16,
                                     int ldb, float* out_f32, int ldf, int M, int D, float eps, hipStream_t stream) {
    if (D % 4 != 0 || D > 64 * 4 * LN_MAX_V4 || M <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(layernorm_kernel, dim3((M + 3) / 4), dim3(256), 0, stream, x, ldx, gamma, beta,
                       reinterpret_cast<bf16_t*>(out_bf16), ldb, out_f32, ldf, M, D, eps);
    return hipGetLastError();
}

extern "C" hipError_t dlms_layernorm_gather(const float* x, int ldx, const int* rows, const float* gamma,
                                            const float* beta, void* out_bf16, int ldb, int M, int D, float eps,
                                            hipStream_t stream) {
    if (D % 4 != 0 || D > 64 * 4 * LN_MAX_V4 || M <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(layernorm_gather_kernel, dim3((M + 3) / 4), dim3(256), 0, stream, x, ldx, rows, gamma, beta,
                       reinterpret_cast<bf16_t*>(out_bf16), ldb, M, D, eps);
    return hipGetLastError();
}

// Fused residual update + LayerNorm (one wave per row, 64-thread workgroups so a decode batch of
// B rows spreads over B CUs):
//     v = x + bias + sum_{s < nsplit} parts[s]      (fixed summation order: deterministic)
//     x = v            (when anything was added; pre-LN GPT-2 residual stream)
//     x = LN(v)        (instead, when store_normed: post-LN BERT residual stream)
//     out = bf16(LN(v) * gamma + beta)               (skipped when out == nullptr)
// This consumes the split-K partial slabs of the previous projection GEMM (EPI_PARTIAL) or, under
// tensor parallelism, the all-reduced partial, so no GEMM epilogue ever read-modify-writes x.
template <int NSPLIT, int NV4>
__global__ __launch_bounds__(256) void add_layernorm_kernel(float* __restrict__ x, int ldx,
                                                           const float* __restrict__ parts, int ldp,
                                                           long long split_stride, const float* __restrict__ bias,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, bf16_t* __restrict__ out,
                                                           int ldb, unsigned int* __restrict__ out8, int ld8,
                                                           float* __restrict__ out8_scale, int M, int D, float eps,
                                                           int store_normed) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);  // one wave per row
    if (row >= M) return;
    const int nv = D >> 2;
    float4* xr = reinterpret_cast<float4*>(x + (size_t)row * ldx);
    const bool update = (NSPLIT > 0 || bias != nullptr) && !store_normed;
    // Branch-free and load-first: NV4 (= ceil(D / 256)) float4 per lane at compile time, column
    // index clamped (the tail's duplicate loads are masked afterwards), and every load of the row
    // -- residual, bias, all split-K partials -- issued before any use or store.  A data-dependent
    // `if (c < nv)` around each load made the compiler wait on each one in turn (NSPLIT x NV4
    // serialised memory latencies, ~7 us for d=768 at 8 splits).
    int cidx[NV4];
    bool valid[NV4];
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        const int c = lane + i * 64;
        valid[i] = c < nv;
        cidx[i] = valid[i] ? c : nv - 1;
    }
    float4 v[NV4];
#pragma unroll
    for (int i = 0; i < NV4; ++i) v[i] = xr[cidx[i]];
    float4 pv[NSPLIT > 0 ? NSPLIT : 1][NV4];
#pragma unroll
    for (int k = 0; k < NSPLIT; ++k) {
        const float4* pk = reinterpret_cast<const float4*>(parts + (size_t)k * split_stride + (size_t)row * ldp);
#pragma unroll
        for (int i = 0; i < NV4; ++i) pv[k][i] = pk[cidx[i]];
    }
    // gamma/beta are loaded with everything else (not after the statistics: that was a second
    // dependent memory round trip per row)
    const float4* g4 = reinterpret_cast<const float4*>(gamma);
    const float4* b4 = reinterpret_cast<const float4*>(beta);
    float4 gv[NV4], bv[NV4];
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        gv[i] = g4[cidx[i]];
        bv[i] = b4[cidx[i]];
    }
    if (bias) {
#pragma unroll
        for (int i = 0; i < NV4; ++i) {
            const float4 b = reinterpret_cast<const float4*>(bias)[cidx[i]];
            v[i].x += b.x; v[i].y += b.y; v[i].z += b.z; v[i].w += b.w;
        }
    }
#pragma unroll
    for (int k = 0; k < NSPLIT; ++k) {
#pragma unroll
        for (int i = 0; i < NV4; ++i) {
            v[i].x += pv[k][i].x; v[i].y += pv[k][i].y; v[i].z += pv[k][i].z; v[i].w += pv[k][i].w;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        if (!valid[i]) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    if (update) {
#pragma unroll
        for (int i = 0; i < NV4; ++i)
            if (valid[i]) xr[cidx[i]] = v[i];
    }
    if (out == nullptr && out8 == nullptr && !store_normed) return;
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        if (valid[i]) {
            const float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
            ss += (a * a + b * b) + (cc * cc + d * d);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        const float4 g = gv[i], b = bv[i];
        if (valid[i]) {
            const float4 y = make_float4((v[i].x - mean) * rstd * g.x + b.x, (v[i].y - mean) * rstd * g.y + b.y,
                                         (v[i].z - mean) * rstd * g.z + b.z, (v[i].w - mean) * rstd * g.w + b.w);
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(y.x), fabsf(y.y)), fmaxf(fabsf(y.z), fabsf(y.w))));
            if (out8) v[i] = y;  // kept for the fp8 pass below
            if (out) {
                uint2 p;
                p.x = pack_bf16x2(y.x, y.y);
                p.y = pack_bf16x2(y.z, y.w);
                reinterpret_cast<uint2*>(out + (size_t)row * ldb)[cidx[i]] = p;
            }
            if (store_normed) xr[cidx[i]] = y;  // post-LN residual stream (BERT): x <- LN(x + ...)
        }
    }
    if (out8) {  // row-scaled OCP e4m3 copy for the fp8 GEMMs (scale = absmax / 448)
        amax = wave_max(amax);
        const float sc = fmaxf(amax, 1e-20f) * (1.f / 448.f);
        const float inv = 1.f / sc;
        if (lane == 0) out8_scale[row] = sc;
#pragma unroll
        for (int i = 0; i < NV4; ++i) {
            if (valid[i]) {
                int w = __builtin_amdgcn_cvt_pk_fp8_f32(v[i].x * inv, v[i].y * inv, 0, false);
                w = __builtin_amdgcn_cvt_pk_fp8_f32(v[i].z * inv, v[i].w * inv, w, true);
                out8[(size_t)row * (ld8 >> 2) + cidx[i]] = (unsigned int)w;
            }
        }
    }
}

// Row-wise fp8 quantisation (prefill / tests): q[r] = e4m3(a[r] / s[r]), s[r] = absmax(a[r]) / 448.
// One wave per row; bf16 input (the LM-head input of a prefill is a gathered bf16 row).
__global__ __launch_bounds__(256) void quantize_rows_fp8_kernel(const bf16_t* __restrict__ a, int lda,
                                                                unsigned int* __restrict__ q, int ldq,
                                                                float* __restrict__ scale, int M, int D) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= M) return;
    const bf16_t* ar = a + (size_t)r * lda;
    float amax = 0.f;
    for (int c = lane * 4; c < D; c += 256)
#pragma unroll
        for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fabsf(bf16_to_f32(ar[c + j])));
    amax = wave_max(amax);
    const float sc = fmaxf(amax, 1e-20f) * (1.f / 448.f);
    const float inv = 1.f / sc;
    if (lane == 0) scale[r] = sc;
    for (int c = lane * 4; c < D; c += 256) {
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ar[c]) * inv, bf16_to_f32(ar[c + 1]) * inv, 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(bf16_to_f32(ar[c + 2]) * inv, bf16_to_f32(ar[c + 3]) * inv, w, true);
        q[(size_t)r * (ldq >> 2) + (c >> 2)] = (unsigned int)w;
    }
}

extern "C" hipError_t dlms_quantize_rows_fp8(const void* a, int lda, void* q, int ldq, float* scale, int M, int D,
                                             hipStream_t stream) {
    if (D % 4 != 0 || ldq % 4 != 0 || M <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(quantize_rows_fp8_kernel, dim3((M + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const bf16_t*>(a), lda, reinterpret_cast<unsigned int*>(q), ldq, scale, M, D);
    return hipGetLastError();
}

// one row (wave) per workgroup of add_layernorm_kernel (4 rows per workgroup measured the same:
// profiles/r2_sweep_ln_rows_per_block.jsonl)
static int ln_rows_per_block() { return 1; }

template <int NSPLIT>
static void launch_add_ln(int nv4, dim3 grid, int rpb, hipStream_t stream, float* x, int ldx, const float* parts, int ldp,
                          long long split_stride, const float* bias, const float* gamma, const float* beta,
                          bf16_t* o, int ldb, unsigned int* o8, int ld8, float* o8s, int M, int D, float eps,
                          int store_normed) {
#define ADD_LN_V(V)                                                                                            \
    case V:                                                                                                    \
        hipLaunchKernelGGL((add_layernorm_kernel<NSPLIT, V>), grid, dim3(64 * rpb), 0, stream, x, ldx, parts,  \
                           ldp, split_stride, bias, gamma, beta, o, ldb, o8, ld8, o8s, M, D, eps, store_normed); \
        break;
    switch (nv4) {
        ADD_LN_V(1) ADD_LN_V(2) ADD_LN_V(3) ADD_LN_V(4) ADD_LN_V(5) ADD_LN_V(6) ADD_LN_V(7) ADD_LN_V(8)
    }
#undef ADD_LN_V
}

extern "C" hipError_t dlms_add_layernorm(float* x, int ldx, const float* parts, int ldp, long long split_stride,
                                         int nsplit, const float* bias, const float* gamma, const float* beta,
                                         void* out_bf16, int ldb, void* out_fp8, int ld8, float* out_fp8_scale,
                                         int M, int D, float eps, int store_normed, hipStream_t stream) {
    if (D % 4 != 0 || D > 64 * 4 * LN_MAX_V4 || M <= 0 || nsplit < 0 || nsplit > 8) return hipErrorInvalidValue;
    bf16_t* o = reinterpret_cast<bf16_t*>(out_bf16);
    const int nv4 = (D / 4 + 63) / 64;
    const int rpb = ln_rows_per_block();
#define ADD_LN_CASE(NS)                                                                                       \
    case NS:                                                                                                  \
        launch_add_ln<NS>(nv4, dim3((M + rpb - 1) / rpb), rpb, stream, x, ldx, parts, ldp, split_stride, bias, \
                          gamma, beta, o, ldb,                                                                \
                          reinterpret_cast<unsigned int*>(out_fp8), ld8, out_fp8_scale, M, D, eps, store_normed); \
        break;
    switch (nsplit) {
        ADD_LN_CASE(0) ADD_LN_CASE(1) ADD_LN_CASE(2) ADD_LN_CASE(3) ADD_LN_CASE(4) ADD_LN_CASE(5) ADD_LN_CASE(6)
        ADD_LN_CASE(7) ADD_LN_CASE(8)
    }
#undef ADD_LN_CASE
    return hipGetLastError();
}
