// Token/position embedding (K1) and the per-step greedy bookkeeping that closes the decode loop
// on the device (K11/K12 consumer), so a whole decode step replays as one hipGraph with no host
// round trip: argmax key -> token -> output buffer, seen-bitmap, stop flags, next embedding.
#include "common.h"

// x[r] = wte[tokens[r]] + wpe[positions[r]]   (bf16 tables, f32 residual stream).  Wave per row.
__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ tokens, const int* __restrict__ positions,
                                                    const bf16_t* __restrict__ wte, const bf16_t* __restrict__ wpe,
                                                    float* x, int ldx, int R, int D, int V, int P) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const bf16_t* a = wte + (size_t)dlms_idx(tokens[r], V, CHK_EMBED_TOKEN) * D;
    const bf16_t* b = wpe + (size_t)dlms_idx(positions[r], P, CHK_EMBED_POS) * D;
    float* o = x + (size_t)r * ldx;
    for (int c = lane; c < D / 8; c += 64) {
        float fa[8], fb[8];
        unpack8(*reinterpret_cast<const uint4*>(a + c * 8), fa);
        unpack8(*reinterpret_cast<const uint4*>(b + c * 8), fb);
        float4 lo = make_float4(fa[0] + fb[0], fa[1] + fb[1], fa[2] + fb[2], fa[3] + fb[3]);
        float4 hi = make_float4(fa[4] + fb[4], fa[5] + fb[5], fa[6] + fb[6], fa[7] + fb[7]);
        reinterpret_cast<float4*>(o + c * 8)[0] = lo;
        reinterpret_cast<float4*>(o + c * 8)[1] = hi;
    }
}

// max over a row's partial argmax keys, one wave per row (keys(b, p) = keys[b * sb + p * sp])
__device__ __forceinline__ unsigned long long wave_key_max(const unsigned long long* __restrict__ keys, int b,
                                                           int nparts, long long sb, long long sp, int lane) {
    // 16 independent loads in flight per lane per round: the LM head leaves ~800 partial keys per
    // row at TP=1, one round trip (a one-load-at-a-time loop paid ~13 dependent round trips)
    unsigned long long best = 0ull;
    for (int p0 = 0; p0 < nparts; p0 += 64 * 16) {
        unsigned long long k[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int p = p0 + lane + 64 * u;
            k[u] = p < nparts ? keys[(size_t)b * sb + (size_t)p * sp] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) best = k[u] > best ? k[u] : best;
    }
    return wave_max_u64(best);  // identical in every lane
}

// argmax partials [B][nparts] -> one key per row (before the cross-rank all-gather under TP)
__global__ __launch_bounds__(256) void argmax_reduce_kernel(const unsigned long long* __restrict__ keys, int nparts,
                                                            long long sb, unsigned long long* out, int B) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const unsigned long long best = wave_key_max(keys, b, nparts, sb, 1, lane);
    if (lane == 0) out[b] = best;
}

#define DU_MAXV4 8  // float4 chunks of the new row per lane: D <= 64 * 8 * 4 = 2048

// One wave per live sequence b.
//   keys(b, p)   packed (ordered value, ~index) argmax keys: the LM head's per-column-tile
//                partials (TP=1) or the all-gathered per-rank keys (TP>1); max over p
//   lens[b]      tokens so far (prompt + generated);  finished[b] stop flag
//   out_tokens   [B][max_len] full sequences (prompt already written by the host)
//   seen         [B][seen_words] repetition-penalty bitmap
// Writes the next forward's token/position/kv-length for row b and its embedding into x.
// slot_map (optional): key row i updates sequence slot slot_map[i] -- used when a prefill of new
// requests lands in arbitrary free slots of a running continuous batch.
// Dependency chain: everything that does not depend on the new token -- the row's length and stop
// flag, its positional-embedding row, a finished row's last token -- is loaded together with the
// keys, so the step pays two memory round trips (keys -> token embedding row), not five.
__global__ __launch_bounds__(256) void decode_update_kernel(const unsigned long long* __restrict__ keys, int nparts,
                                                            long long sb, long long sp,
                                                            const int* __restrict__ slot_map, int* lens,
                                                            int* finished, int* out_tokens, int max_len,
                                                            unsigned int* seen, int seen_words, int* cur_tok,
                                                            int* cur_pos, int* cur_kvlen,
                                                            const bf16_t* __restrict__ wte,
                                                            const bf16_t* __restrict__ wpe, float* x, int ldx, int B,
                                                            int D, int eos, int t_max, int n_slots, int V,
                                                            const float* __restrict__ ln_g,
                                                            const float* __restrict__ ln_b, float eps, bf16_t* h,
                                                            int ldh) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= B) return;
    const int b = slot_map ? (int)dlms_idx(slot_map[i], n_slots, CHK_UPDATE_SLOT) : i;
    // row state (every lane reads the same words: one request each)
    const int len0 = (int)dlms_idx(lens[b], max_len + 1, CHK_UPDATE_LEN);
    const int fin = finished[b];
    // where a live row's token goes (a finished row may sit at len == max_len: not an index then)
    const int live_len = fin ? 0 : (int)dlms_idx(len0, max_len, CHK_UPDATE_LEN);
    int pos = fin ? len0 - 1 : live_len;  // (length after this step) - 1
    pos = pos < 0 ? 0 : (pos < t_max - 1 ? pos : t_max - 1);
    const int last_tok = fin ? out_tokens[(size_t)b * max_len + (len0 > 0 ? len0 - 1 : 0)] : 0;
    // the row in float4 chunks c = lane + 64 j -- add_layernorm_kernel's partition, so the fused
    // LayerNorm below computes exactly what that kernel would on the stored row
    const int nv = D >> 2;
    uint2 pe[DU_MAXV4];
#pragma unroll
    for (int j = 0; j < DU_MAXV4; ++j) {
        const int c = lane + 64 * j;
        pe[j] = c < nv ? *reinterpret_cast<const uint2*>(wpe + (size_t)pos * D + c * 4) : make_uint2(0u, 0u);
    }
    const unsigned long long best = wave_key_max(keys, i, nparts, sb, sp, lane);

    int tok;
    if (!fin) {
        // best == 0 means no shard produced a candidate (cannot happen for vocab >= 1); stay in
        // bounds anyway by emitting EOS.
        tok = best ? (int)(~(unsigned int)(best & 0xffffffffull)) : eos;
        tok = (int)dlms_idx(tok, V, CHK_UPDATE_TOKEN);
    } else {
        tok = (int)dlms_idx(last_tok, V, CHK_UPDATE_TOKEN);
    }
    if (lane == 0) {
        if (!fin) {
            out_tokens[(size_t)b * max_len + live_len] = tok;
            atomicOr(seen + (size_t)b * seen_words + (tok >> 5), 1u << (tok & 31));  // no read-back wait
            lens[b] = live_len + 1;
            if (tok == eos || live_len + 1 >= max_len) finished[b] = 1;
        }
        cur_tok[b] = tok;
        cur_pos[b] = pos;
        cur_kvlen[b] = pos + 1;
    }
    const bf16_t* a = wte + (size_t)tok * D;
    float4* o = reinterpret_cast<float4*>(x + (size_t)b * ldx);
    float4 v[DU_MAXV4];
#pragma unroll
    for (int j = 0; j < DU_MAXV4; ++j) {
        const int c = lane + 64 * j;
        v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c >= nv) continue;
        const uint2 e = *reinterpret_cast<const uint2*>(a + c * 4);
        v[j] = make_float4(bf16_to_f32((bf16_t)(e.x & 0xffffu)) + bf16_to_f32((bf16_t)(pe[j].x & 0xffffu)),
                           bf16_to_f32((bf16_t)(e.x >> 16)) + bf16_to_f32((bf16_t)(pe[j].x >> 16)),
                           bf16_to_f32((bf16_t)(e.y & 0xffffu)) + bf16_to_f32((bf16_t)(pe[j].y & 0xffffu)),
                           bf16_to_f32((bf16_t)(e.y >> 16)) + bf16_to_f32((bf16_t)(pe[j].y >> 16)));
        o[c] = v[j];
    }
    if (h == nullptr) return;
    // layer 0's LN1 of the new row (the overlapped decode step then skips that launch): the same
    // statistics order as add_layernorm_kernel -- per-lane float4 sums, wave sums, two passes
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < DU_MAXV4; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < DU_MAXV4; ++j) {
        if (lane + 64 * j < nv) {
            const float p = v[j].x - mean, q = v[j].y - mean, r = v[j].z - mean, t = v[j].w - mean;
            ss += (p * p + q * q) + (r * r + t * t);
        }
    }
    const float rstd = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
    for (int j = 0; j < DU_MAXV4; ++j) {
        const int c = lane + 64 * j;
        if (c >= nv) continue;
        const float4 g = reinterpret_cast<const float4*>(ln_g)[c], be = reinterpret_cast<const float4*>(ln_b)[c];
        uint2 pk;
        pk.x = pack_bf16x2((v[j].x - mean) * rstd * g.x + be.x, (v[j].y - mean) * rstd * g.y + be.y);
        pk.y = pack_bf16x2((v[j].z - mean) * rstd * g.z + be.z, (v[j].w - mean) * rstd * g.w + be.w);
        reinterpret_cast<uint2*>(h + (size_t)b * ldh)[c] = pk;
    }
}

extern "C" hipError_t dlms_embed(const int* tokens, const int* positions, const void* wte, const void* wpe, float* x,
                                 int ldx, int R, int D, int V, int P, hipStream_t stream) {
    if (D % 8 != 0 || R <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(embed_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, tokens, positions,
                       reinterpret_cast<const bf16_t*>(wte), reinterpret_cast<const bf16_t*>(wpe), x, ldx, R, D, V, P);
    return hipGetLastError();
}

extern "C" hipError_t dlms_decode_update(const unsigned long long* keys, int nparts, long long sb, long long sp,
                                         const int* slot_map, int* lens, int* finished, int* out_tokens, int max_len,
                                         unsigned int* seen, int seen_words, int* cur_tok, int* cur_pos,
                                         int* cur_kvlen, const void* wte, const void* wpe, float* x, int ldx, int B,
                                         int D, int eos, int t_max, int n_slots, int V, const float* ln_g,
                                         const float* ln_b, float eps, void* h, int ldh, hipStream_t stream) {
    if (D % 8 != 0 || D > 64 * DU_MAXV4 * 4 || B <= 0 || nparts <= 0 || (h && (!ln_g || !ln_b || ldh % 4)))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(decode_update_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, keys, nparts, sb, sp, slot_map,
                       lens, finished, out_tokens, max_len, seen, seen_words, cur_tok, cur_pos, cur_kvlen,
                       reinterpret_cast<const bf16_t*>(wte), reinterpret_cast<const bf16_t*>(wpe), x, ldx, B, D, eos,
                       t_max, n_slots, V, ln_g, ln_b, eps, reinterpret_cast<bf16_t*>(h), ldh);
    return hipGetLastError();
}

extern "C" hipError_t dlms_argmax_reduce(const unsigned long long* keys, int nparts, long long sb,
                                         unsigned long long* out, int B, hipStream_t stream) {
    if (B <= 0 || nparts <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(argmax_reduce_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, keys, nparts, sb, out, B);
    return hipGetLastError();
}

// Prefill bookkeeping on the device: set the repetition-penalty bit of every prompt token in its
// sequence's seen bitmap (rows pre-zeroed by the caller).  One thread per packed prompt token;
// duplicate tokens of a row OR the same bit, so the result does not depend on the order.
__global__ __launch_bounds__(256) void seen_set_kernel(const int* __restrict__ tokens, const int* __restrict__ rows,
                                                       int R, unsigned int* seen, int seen_words, int n_rows) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R) return;
    const int t = tokens[i];
    if (t < 0 || (t >> 5) >= seen_words) {  // the host validates ids; never write out of the row
        dlms_idx(t, (long long)seen_words * 32, CHK_SEEN_TOKEN);
        return;
    }
    const size_t row = dlms_idx(rows[i], n_rows, CHK_SEEN_ROW);
    atomicOr(seen + row * seen_words + (t >> 5), 1u << (t & 31));
}

extern "C" hipError_t dlms_seen_set(const int* tokens, const int* rows, int R, unsigned int* seen, int seen_words,
                                    int n_rows, hipStream_t stream) {
    if (R <= 0 || seen_words <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(seen_set_kernel, dim3((R + 255) / 256), dim3(256), 0, stream, tokens, rows, R, seen, seen_words,
                       n_rows);
    return hipGetLastError();
}

DLMS_CHECK_EXPORT(decode)
