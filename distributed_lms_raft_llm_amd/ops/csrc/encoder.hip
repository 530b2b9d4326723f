// BERT relevance-gate kernels: fused embedding gather + LayerNorm (K13), mean-pool (K16) and
// batched cosine similarity (K17).  The encoder GEMMs/attention reuse gemm.hip / attention.hip.
#include "common.h"

#define BE_MAX_V4 8

// x = LN(word[ids] + pos[positions] + type[0]); writes f32 residual and bf16 GEMM input.
__global__ __launch_bounds__(256) void bert_embed_ln_kernel(const int* __restrict__ ids,
                                                            const int* __restrict__ positions,
                                                            const float* __restrict__ word,
                                                            const float* __restrict__ pos_emb,
                                                            const float* __restrict__ type0,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* out_f32,
                                                            bf16_t* out_bf16, int R, int D, float eps, int V, int P) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int nv = D >> 2;
    const float4* a = reinterpret_cast<const float4*>(word + (size_t)dlms_idx(ids[r], V, CHK_BERT_TOKEN) * D);
    const float4* p = reinterpret_cast<const float4*>(pos_emb + (size_t)dlms_idx(positions[r], P, CHK_EMBED_POS) * D);
    const float4* t = reinterpret_cast<const float4*>(type0);
    float4 v[BE_MAX_V4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < BE_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float4 x0 = a[c], x1 = p[c], x2 = t[c];
            v[i] = make_float4(x0.x + x1.x + x2.x, x0.y + x1.y + x2.y, x0.z + x1.z + x2.z, x0.w + x1.w + x2.w);
        } else {
            v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < BE_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float q0 = v[i].x - mean, q1 = v[i].y - mean, q2 = v[i].z - mean, q3 = v[i].w - mean;
            ss += (q0 * q0 + q1 * q1) + (q2 * q2 + q3 * q3);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
    const float4* g4 = reinterpret_cast<const float4*>(gamma);
    const float4* b4 = reinterpret_cast<const float4*>(beta);
#pragma unroll
    for (int i = 0; i < BE_MAX_V4; ++i) {
        const int c = lane + i * 64;
        if (c < nv) {
            const float4 g = g4[c], b = b4[c];
            float4 y;
            y.x = (v[i].x - mean) * rstd * g.x + b.x;
            y.y = (v[i].y - mean) * rstd * g.y + b.y;
            y.z = (v[i].z - mean) * rstd * g.z + b.z;
            y.w = (v[i].w - mean) * rstd * g.w + b.w;
            reinterpret_cast<float4*>(out_f32 + (size_t)r * D)[c] = y;
            uint2 pk;
            pk.x = pack_bf16x2(y.x, y.y);
            pk.y = pack_bf16x2(y.z, y.w);
            reinterpret_cast<uint2*>(out_bf16 + (size_t)r * D)[c] = pk;
        }
    }
}

// out[s, :] = mean over rows [start[s], start[s]+len[s]) of x (f32 [R, D]).  Column per thread.
__global__ __launch_bounds__(256) void mean_pool_kernel(const float* __restrict__ x, const int* __restrict__ start,
                                                        const int* __restrict__ len, float* out, int D) {
    const int s = blockIdx.y;
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= D) return;
    const int r0 = start[s], n = len[s];
    float acc = 0.f;
    for (int i = 0; i < n; ++i) acc += x[(size_t)(r0 + i) * D + col];
    out[(size_t)s * D + col] = acc / (float)(n > 0 ? n : 1);
}

// sim[i, j] = a_i . b_j / sqrt(max(|a_i|^2 |b_j|^2, eps^2))   (torch.nn.functional.cosine_similarity)
__global__ __launch_bounds__(64) void cosine_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                    float* out, int NB, int D, float eps) {
    const int i = blockIdx.y, j = blockIdx.x;
    const float* x = a + (size_t)i * D;
    const float* y = b + (size_t)j * D;
    float dot = 0.f, nx = 0.f, ny = 0.f;
    for (int c = threadIdx.x; c < D; c += 64) {
        const float u = x[c], v = y[c];
        dot += u * v;
        nx += u * u;
        ny += v * v;
    }
    dot = wave_sum(dot);
    nx = wave_sum(nx);
    ny = wave_sum(ny);
    if (threadIdx.x == 0) out[(size_t)i * NB + j] = dot / sqrtf(fmaxf(nx * ny, eps * eps));
}

extern "C" hipError_t dlms_bert_embed_ln(const int* ids, const int* positions, const float* word, const float* pos_emb,
                                         const float* type0, const float* gamma, const float* beta, float* out_f32,
                                         void* out_bf16, int R, int D, float eps, int V, int P, hipStream_t stream) {
    if (D % 4 != 0 || D > 64 * 4 * BE_MAX_V4 || R <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bert_embed_ln_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, ids, positions, word, pos_emb,
                       type0, gamma, beta, out_f32, reinterpret_cast<bf16_t*>(out_bf16), R, D, eps, V, P);
    return hipGetLastError();
}

extern "C" hipError_t dlms_mean_pool(const float* x, const int* start, const int* len, float* out, int S, int D,
                                     hipStream_t stream) {
    if (S <= 0 || D <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mean_pool_kernel, dim3((D + 255) / 256, S), dim3(256), 0, stream, x, start, len, out, D);
    return hipGetLastError();
}

extern "C" hipError_t dlms_cosine(const float* a, const float* b, float* out, int NA, int NB, int D, float eps,
                                  hipStream_t stream) {
    if (NA <= 0 || NB <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(cosine_kernel, dim3(NB, NA), dim3(64), 0, stream, a, b, out, NB, D, eps);
    return hipGetLastError();
}

DLMS_CHECK_EXPORT(encoder)
