// Row attention over a slot-addressed KV cache (K5 decode, K6/K14 fallback path).
//
// Cache layout: [slots][H][t_max][64] bf16 for K and for V (one contiguous 128-B row per key, so a
// wave-instruction of 8 keys x 8 lanes x 16 B reads 1 KiB contiguous).
// Query row r attends keys [0, row_kvlen[r]) of slot row_slot[r]: causal GPT-2 decode/prefill passes
// kvlen = pos + 1, the bidirectional BERT encoder passes kvlen = sequence length.
// Scores for the whole row live in LDS (t_max <= 2048), so the softmax is an exact two-pass one.
#include <stdlib.h>

#include "common.h"

#define ATT_MAX_T 2048

__global__ __launch_bounds__(256) void row_attention_kernel(const bf16_t* __restrict__ q, int ldq,
                                                            const bf16_t* __restrict__ kc,
                                                            const bf16_t* __restrict__ vc,
                                                            const int* __restrict__ row_slot,
                                                            const int* __restrict__ row_kvlen, bf16_t* out,
                                                            int ldo, int H, int t_max, int n_slots, float scale) {
    __shared__ float sc[ATT_MAX_T];
    __shared__ float red[4][64];
    __shared__ float stat[2];

    const int h = blockIdx.x;
    const int r = blockIdx.y;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int kk = lane >> 3;  // key within the wave's group of 8
    const int c = lane & 7;    // 8-dim chunk of the head
    const int slot = (int)dlms_idx(row_slot[r], n_slots, CHK_ATTN_SLOT);
    int kvlen = row_kvlen[r];
    kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);

    const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
    const bf16_t* K = kc + head_off;
    const bf16_t* V = vc + head_off;

    float qf[8];
    unpack8(*reinterpret_cast<const uint4*>(q + (size_t)r * ldq + h * 64 + c * 8), qf);

    // ---- scores ----
    for (int t0 = wave * 8; t0 < kvlen; t0 += 32) {
        const int t = t0 + kk;
        float s = 0.f;
        if (t < kvlen) {
            float kf[8];
            unpack8(*reinterpret_cast<const uint4*>(K + (size_t)t * 64 + c * 8), kf);
#pragma unroll
            for (int j = 0; j < 8; ++j) s += qf[j] * kf[j];
        }
        s = group8_sum(s);
        if (c == 0 && t < kvlen) sc[t] = s * scale;
    }
    __syncthreads();

    // ---- softmax statistics ----
    float m = -INFINITY;
    for (int t = tid; t < kvlen; t += 256) m = fmaxf(m, sc[t]);
    m = wave_max(m);
    if (lane == 0) red[wave][0] = m;
    __syncthreads();
    if (tid == 0) stat[0] = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0]));
    __syncthreads();
    m = stat[0];
    float l = 0.f;
    for (int t = tid; t < kvlen; t += 256) {
        const float p = __expf(sc[t] - m);
        sc[t] = p;
        l += p;
    }
    l = wave_sum(l);
    __syncthreads();
    if (lane == 0) red[wave][1] = l;
    __syncthreads();
    if (tid == 0) stat[1] = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
    __syncthreads();

    // ---- P . V ----
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t = wave * 8 + kk; t < kvlen; t += 32) {
        float vf[8];
        unpack8(*reinterpret_cast<const uint4*>(V + (size_t)t * 64 + c * 8), vf);
        const float p = sc[t];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += p * vf[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        acc[j] += xor_lane(acc[j], 8);
        { float x_, y_; lane_pair(acc[j], 16, x_, y_); acc[j] = x_ + y_; }
        { float x_, y_; lane_pair(acc[j], 32, x_, y_); acc[j] = x_ + y_; }
    }
    __syncthreads();  // red[] reuse
    if (kk == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wave][c * 8 + j] = acc[j];
    }
    __syncthreads();
    if (tid < 64) {
        const float inv = 1.f / stat[1];
        const float o = ((red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid])) * inv;
        out[(size_t)r * ldo + h * 64 + tid] = f32_to_bf16(o);
    }
}

// Decode-shaped attention: ONE WAVE per (row, head), 4 heads of a row per workgroup (their cache
// rows are adjacent).  Lane (g = lane>>3, c = lane&7) owns dims [8c, 8c+8) of keys t = 8i + g;
// a wave-instruction therefore reads 8 whole 128-B key rows (1 KiB contiguous).  Online softmax
// in registers (exp2 with log2(e) folded into q), ATT_UNROLL key-steps of K and V loads issued
// before any use, then a shuffle merge of the 8 per-group (max, sum, acc) triples.  No LDS, no
// barriers: the kernel is a pure KV stream.
// NT: non-temporal K/V loads (the cache is streamed once per step; keep L2/MALL for weights).
template <int ATT_UNROLL, bool NT>
__global__ __launch_bounds__(256) void attn_wave_kernel(const bf16_t* __restrict__ q, int ldq,
                                                        const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                                        const int* __restrict__ row_slot,
                                                        const int* __restrict__ row_kvlen, bf16_t* out, int ldo, int H,
                                                        int t_max, int n_slots, float scale_log2) {
    const int lane = threadIdx.x & 63;
    const int h = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int r = blockIdx.y;
    if (h >= H) return;
    const int g = lane >> 3;
    const int c = lane & 7;
    const int slot = (int)dlms_idx(row_slot[r], n_slots, CHK_ATTN_SLOT);
    int kvlen = row_kvlen[r];
    kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);
    const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
    const bf16_t* K = kc + head_off + c * 8;
    const bf16_t* V = vc + head_off + c * 8;

    float qf[8];
    unpack8(*reinterpret_cast<const uint4*>(q + (size_t)r * ldq + h * 64 + c * 8), qf);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[j] *= scale_log2;

    float m = -INFINITY, l = 0.f;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t0 = 0; t0 < kvlen; t0 += 8 * ATT_UNROLL) {
        uint4 kr[ATT_UNROLL], vr[ATT_UNROLL];
#pragma unroll
        for (int u = 0; u < ATT_UNROLL; ++u) {
            int t = t0 + u * 8 + g;
            t = t < kvlen ? t : kvlen - 1;  // clamped (masked below): loads never leave the slot
            if constexpr (NT) {
                typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
                const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(K + (size_t)t * 64));
                const u32x4_t b = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(V + (size_t)t * 64));
                kr[u] = make_uint4(a.x, a.y, a.z, a.w);
                vr[u] = make_uint4(b.x, b.y, b.z, b.w);
            } else {
                kr[u] = *reinterpret_cast<const uint4*>(K + (size_t)t * 64);
                vr[u] = *reinterpret_cast<const uint4*>(V + (size_t)t * 64);
            }
        }
#pragma unroll
        for (int u = 0; u < ATT_UNROLL; ++u) {
            float kf[8];
            unpack8(kr[u], kf);
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) s += qf[j] * kf[j];
            s = group8_sum(s);
            const bool valid = t0 + u * 8 + g < kvlen;
            if (valid) {
                const float m_new = fmaxf(m, s);
                const float corr = exp2f(m - m_new);  // m == -inf -> 0 (acc and l are 0 then)
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
    // merge the 8 key groups (lanes c, c+8, ..., c+56 hold partials of the same dims)
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
        const float inv = 1.f / l;
        float o8[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o8[j] = acc[j] * inv;
        *reinterpret_cast<uint4*>(out + (size_t)r * ldo + h * 64 + c * 8) = pack8(o8);
    }
}

// Persistent, low-occupancy variant of attn_wave_kernel for the overlapped decode step: a fixed
// grid of NB workgroups x 4 waves, each wave looping over (row, head) pairs (consecutive pairs = the
// heads of one row, adjacent in the cache).  An 8-deep unroll keeps 16 KiB of K/V in flight per wave
// so ~8 waves per CU still stream HBM at full rate -- and leave the CU's other wave slots, LDS and
// MFMA pipes to the GEMMs of the other row half running on the second stream (a one-wave-per-pair
// grid of 6k waves occupies every slot and serialises the two streams at kernel granularity).
//
// BLK: the online softmax rescales once per block of U keys (one max, one correction exp2 and one
// acc*corr pass per block instead of per key), halving the exp2 count and dropping 8 multiplies per
// key from the VALU stream that shares the CU with the other stream's GEMMs.
template <int U, bool BLK>
__global__ __launch_bounds__(256) void attn_persist_kernel(const bf16_t* __restrict__ q, int ldq,
                                                           const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                                           const int* __restrict__ row_slot,
                                                           const int* __restrict__ row_kvlen, bf16_t* out, int ldo,
                                                           int R, int H, int t_max, int n_slots, float scale_log2) {
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3;
    const int c = lane & 7;
    const int nwaves = gridDim.x * 4;
    const int npairs = R * H;
    for (int pair = blockIdx.x * 4 + (threadIdx.x >> 6); pair < npairs; pair += nwaves) {
        const int r = pair / H, h = pair - r * H;
        const int slot = (int)dlms_idx(row_slot[r], n_slots, CHK_ATTN_SLOT);
        int kvlen = row_kvlen[r];
        kvlen = kvlen < 1 ? 1 : (kvlen > t_max ? t_max : kvlen);
        const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
        const bf16_t* K = kc + head_off + c * 8;
        const bf16_t* V = vc + head_off + c * 8;
        float qf[8];
        unpack8(*reinterpret_cast<const uint4*>(q + (size_t)r * ldq + h * 64 + c * 8), qf);
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[j] *= scale_log2;
        float m = -INFINITY, l = 0.f;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int t0 = 0; t0 < kvlen; t0 += 8 * U) {
            uint4 kr[U], vr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int t = t0 + u * 8 + g;
                t = t < kvlen ? t : kvlen - 1;
                const u32x4_t a = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(K + (size_t)t * 64));
                const u32x4_t b = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(V + (size_t)t * 64));
                kr[u] = make_uint4(a.x, a.y, a.z, a.w);
                vr[u] = make_uint4(b.x, b.y, b.z, b.w);
            }
            if constexpr (BLK) {
                float sv[U];
                float mb = -INFINITY;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    float kf[8];
                    unpack8(kr[u], kf);
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) s += qf[j] * kf[j];
                    s = group8_sum(s);
                    sv[u] = t0 + u * 8 + g < kvlen ? s : -INFINITY;
                    mb = fmaxf(mb, sv[u]);
                }
                if (mb != -INFINITY) {  // else every key of this lane group is past kvlen
                    const float m_new = fmaxf(m, mb);
                    const float corr = exp2f(m - m_new);  // m == -inf -> 0
                    float ps = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[j] *= corr;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const float p = exp2f(sv[u] - m_new);  // masked keys -> 0
                        float vf[8];
                        unpack8(vr[u], vf);
                        ps += p;
#pragma unroll
                        for (int j = 0; j < 8; ++j) acc[j] += p * vf[j];
                    }
                    l = l * corr + ps;
                    m = m_new;
                }
                continue;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float kf[8];
                unpack8(kr[u], kf);
                float s = 0.f;
#pragma unroll
                for (int j = 0; j < 8; ++j) s += qf[j] * kf[j];
                s = group8_sum(s);
                if (t0 + u * 8 + g < kvlen) {
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
            const float inv = 1.f / l;
            float o8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o8[j] = acc[j] * inv;
            *reinterpret_cast<uint4*>(out + (size_t)r * ldo + h * 64 + c * 8) = pack8(o8);
        }
    }
}

extern "C" hipError_t dlms_attention_persist(const void* q, int ldq, const void* kc, const void* vc,
                                             const int* row_slot, const int* row_kvlen, void* out, int ldo, int R,
                                             int H, int t_max, int n_slots, float scale, int blocks,
                                             hipStream_t stream) {
    if (R <= 0 || H <= 0 || t_max <= 0 || blocks <= 0) return hipErrorInvalidValue;
    const int need = (R * H + 3) / 4;
    // (the per-key softmax update measured the same at 1024 queries: 710/717 vs 715/710 k tok/s,
    // profiles/r4_attn_blk_ab.jsonl -- the kernel is bound by the KV stream; the block-wise one stays)
    hipLaunchKernelGGL((attn_persist_kernel<8, true>), dim3(blocks < need ? blocks : need), dim3(256), 0, stream,
                       reinterpret_cast<const bf16_t*>(q), ldq, reinterpret_cast<const bf16_t*>(kc),
                       reinterpret_cast<const bf16_t*>(vc), row_slot, row_kvlen, reinterpret_cast<bf16_t*>(out),
                       ldo, R, H, t_max, n_slots, scale * 1.4426950408889634f);
    return hipGetLastError();
}

// Default: 4-deep unroll with non-temporal K/V loads (the cache is streamed once per layer; keeping
// it out of L2/MALL leaves them to the weights): +6 % whole-step at 1024 queries, +4.5 % at 256
// (profiles/r1_attention_variants.log, in-situ A/B in profiles/r1_bench_lines.jsonl).

extern "C" hipError_t dlms_attention(const void* q, int ldq, const void* kc, const void* vc, const int* row_slot,
                                     const int* row_kvlen, void* out, int ldo, int R, int H, int t_max, int n_slots,
                                     float scale, hipStream_t stream) {
    if (R <= 0 || H <= 0 || t_max <= 0) return hipErrorInvalidValue;
    const float scale_log2 = scale * 1.4426950408889634f;
    hipLaunchKernelGGL((attn_wave_kernel<4, true>), dim3((H + 3) / 4, R), dim3(256), 0, stream,
                       reinterpret_cast<const bf16_t*>(q), ldq, reinterpret_cast<const bf16_t*>(kc),
                       reinterpret_cast<const bf16_t*>(vc), row_slot, row_kvlen, reinterpret_cast<bf16_t*>(out), ldo,
                       H, t_max, n_slots, scale_log2);
    return hipGetLastError();
}

extern "C" hipError_t dlms_row_attention(const void* q, int ldq, const void* kc, const void* vc, const int* row_slot,
                                         const int* row_kvlen, void* out, int ldo, int R, int H, int t_max,
                                         int n_slots, float scale, hipStream_t stream) {
    if (t_max > ATT_MAX_T || R <= 0 || H <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(row_attention_kernel, dim3(H, R), dim3(256), 0, stream, reinterpret_cast<const bf16_t*>(q), ldq,
                       reinterpret_cast<const bf16_t*>(kc), reinterpret_cast<const bf16_t*>(vc), row_slot, row_kvlen,
                       reinterpret_cast<bf16_t*>(out), ldo, H, t_max, n_slots, scale);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// MFMA tile attention (K6 prefill, K14 BERT encoder): ONE WAVE per (16-query tile, head), four
// heads per workgroup.  A tile is up to 16 consecutive packed rows of ONE sequence (host-built
// tile list: row0, nq); query row r attends keys [0, row_kvlen[r]) of slot row_slot[row0]
// (causal prefill passes kvlen = pos + 1, the bidirectional encoder the sequence length).
//
// Per 32-key step (v_mfma_f32_16x16x32_bf16, 8 MFMAs):
//   S^T[32 keys x 16 queries] = K . Q^T   -- "swapped" orientation: lane l holds the scores of
//       query l&15 for keys 4g..4g+3 and 16+4g..16+4g+3 (g = l>>4), so the online softmax of a
//       query is 8 in-register values + two cross-group shuffles, and the probabilities ARE the
//       A operand of the next product (k order permuted: slot 8g+j <-> those keys);
//   O[16 x 64] += P . V   -- V's key rows staged in LDS (4 KiB per wave, wave-private) and read
//       back transposed with ds_read_b64_tr_b16 into B fragments whose k slots follow the same
//       key permutation.
// K fragments and Q come straight from global memory (16-B row chunks).  The output tile is
// restaged through the wave's LDS so each lane stores whole 16-B row chunks.
// EXEC stays all-ones around the transposed reads: only whole waves leave early (h >= H), every
// loop bound is wave-uniform and out-of-range keys/queries are clamped + masked, never skipped.
typedef short tr4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) tr4_t lds_tr4_t;

__global__ __launch_bounds__(256) void attn_tile_kernel(const bf16_t* __restrict__ q, int ldq,
                                                        const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                                        const int* __restrict__ row_slot,
                                                        const int* __restrict__ row_kvlen,
                                                        const int* __restrict__ tiles, bf16_t* __restrict__ out,
                                                        int ldo, int H, int t_max, int n_slots, float scale_log2) {
    __shared__ __attribute__((aligned(16))) char smem[4 * 4096];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int h = blockIdx.y * 4 + w;
    if (h >= H) return;  // whole wave
    const int row0 = tiles[2 * blockIdx.x];
    const int nq = tiles[2 * blockIdx.x + 1];
    const int qi = lane & 15;
    const int g = lane >> 4;
    const int qrow = row0 + (qi < nq ? qi : nq - 1);
    const int slot = (int)dlms_idx(row_slot[row0], n_slots, CHK_ATTN_SLOT);
    int kvq = row_kvlen[qrow];
    kvq = kvq < 1 ? 1 : (kvq > t_max ? t_max : kvq);
    int kv_end = kvq;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        const int other = __shfl_xor(kv_end, o, 64);
        kv_end = other > kv_end ? other : kv_end;
    }
    if (qi >= nq) kvq = 0;  // padding lanes: every key masked, never stored

    const size_t head_off = ((size_t)slot * H + h) * t_max * 64;
    const bf16_t* K = kc + head_off;
    const bf16_t* V = vc + head_off;
    bf16x8_t qf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
        qf[ks] = *reinterpret_cast<const bf16x8_t*>(q + (size_t)qrow * ldq + h * 64 + 32 * ks + 8 * g);

    char* vl = smem + w * 4096;
    float m = -INFINITY, l = 0.f;
    f32x4_t o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    for (int t0 = 0; t0 < kv_end; t0 += 32) {
        // ---- V tile -> LDS (issued first: its latency overlaps the score MFMAs) ----
        uint4 vrow[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int key = t0 + (lane >> 3) + 8 * i;
            key = key < kv_end ? key : kv_end - 1;
            vrow[i] = *reinterpret_cast<const uint4*>(V + (size_t)key * 64 + (lane & 7) * 8);
        }
        // ---- S^T = K . Q^T (two 16-key tiles) ----
        f32x4_t s[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
            int key = t0 + 16 * tt + qi;
            key = key < kv_end ? key : kv_end - 1;
            const bf16x8_t k0 = *reinterpret_cast<const bf16x8_t*>(K + (size_t)key * 64 + 8 * g);
            const bf16x8_t k1 = *reinterpret_cast<const bf16x8_t*>(K + (size_t)key * 64 + 32 + 8 * g);
            s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[0], (f32x4_t){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            s[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[1], s[tt], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<uint4*>(vl + ((lane >> 3) + 8 * i) * 128 + (lane & 7) * 16) = vrow[i];
        // ---- online softmax for query qi over this lane's 8 keys ----
        float sv[8];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int key = t0 + 16 * (j >> 2) + 4 * g + (j & 3);
            const float v = key < kvq ? s[j >> 2][j & 3] * scale_log2 : -INFINITY;
            sv[j] = v;
            mx = fmaxf(mx, v);
        }
        { float x_, y_; lane_pair(mx, 16, x_, y_); mx = fmaxf(x_, y_); }
        { float x_, y_; lane_pair(mx, 32, x_, y_); mx = fmaxf(x_, y_); }
        const float m_new = fmaxf(m, mx);
        const bool none = m_new == -INFINITY;  // no valid key yet for this query
        const float corr = none ? 1.f : exp2f(m - m_new);
        float psum = 0.f;
        bf16x8_t pa;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float p = none ? 0.f : exp2f(sv[j] - m_new);
            psum += p;
            pa[j] = (short)f32_to_bf16(p);
        }
        { float x_, y_; lane_pair(psum, 16, x_, y_); psum = x_ + y_; }
        { float x_, y_; lane_pair(psum, 32, x_, y_); psum = x_ + y_; }
        l = l * corr + psum;
        m = m_new;
        // O rows are queries 4g + r: fetch their correction factors from lanes 4g + r
        float cr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) cr[r] = __shfl(corr, 4 * g + r, 64);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[c][r] *= cr[r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // V tile stored (wave-private region)
        // ---- O += P . V: B fragment slot 8g+j <-> key 4g+j (j<4) / 16+4g+(j-4), column 16c + qi ----
        const int trow = 4 * g + (qi >> 2);  // this lane supplies row (4g + q) of its group's 4x16 block
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int col = 16 * c + 4 * (qi & 3);
            const tr4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_tr4_t*)(vl + trow * 128 + col * 2));
            const tr4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_tr4_t*)(vl + (16 + trow) * 128 + col * 2));
            const bf16x8_t vb = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[c], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's stores
    }
    // ---- normalise (queries 4g + r), restage through LDS as [16 rows][64 dims] bf16, 16-B stores ----
    float inv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float lr = __shfl(l, 4 * g + r, 64);
        inv[r] = lr > 0.f ? 1.f / lr : 0.f;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<bf16_t*>(vl + (4 * g + r) * 128 + (16 * c + qi) * 2) = f32_to_bf16(o[c][r] * inv[r]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int chunk = lane + 64 * i;  // 16 rows x 8 chunks
        const int r = chunk >> 3, ch = chunk & 7;
        const uint4 val = *reinterpret_cast<const uint4*>(vl + r * 128 + ch * 16);
        if (r < nq) *reinterpret_cast<uint4*>(out + (size_t)(row0 + r) * ldo + h * 64 + ch * 8) = val;
    }
}

extern "C" hipError_t dlms_tile_attention(const void* q, int ldq, const void* kc, const void* vc, const int* row_slot,
                                          const int* row_kvlen, const int* tiles, int ntiles, void* out, int ldo, int H,
                                          int t_max, int n_slots, float scale, hipStream_t stream) {
    if (ntiles <= 0 || H <= 0 || t_max <= 0) return hipErrorInvalidValue;
    const float scale_log2 = scale * 1.4426950408889634f;
    hipLaunchKernelGGL(attn_tile_kernel, dim3(ntiles, (H + 3) / 4), dim3(256), 0, stream,
                       reinterpret_cast<const bf16_t*>(q), ldq, reinterpret_cast<const bf16_t*>(kc),
                       reinterpret_cast<const bf16_t*>(vc), row_slot, row_kvlen, tiles, reinterpret_cast<bf16_t*>(out),
                       ldo, H, t_max, n_slots, scale_log2);
    return hipGetLastError();
}

DLMS_CHECK_EXPORT(attention)
