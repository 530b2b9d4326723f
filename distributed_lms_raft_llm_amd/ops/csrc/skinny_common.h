// Shared pieces of the skinny (few-row decode) MFMA kernels: skinny.hip (M <= 32 latency path)
// and mid.hip (9-64-row decode).  Epilogue ids, the LDS A-fragment read and the column-owning
// epilogue of one wave.
#pragma once
#include "common.h"

#include <type_traits>

// SK_FIXADD: like SK_F32 (x += acc + bias, column-owning, in place) into copy 0 of the int64
// fixed-point residual the fused MLP accumulates (see DLMS_FIX_SCALE below)
enum { SK_BF16 = 0, SK_GELU_TANH = 1, SK_F32 = 3, SK_QKV = 4, SK_ARGMAX = 5, SK_PARTIAL = 6, SK_FIXADD = 7 };

// A fragment of rows [16 mt, 16 mt + 16) at k-block kb from the LDS LayerNorm image
__device__ __forceinline__ bf16x8_t lds_a_frag(const char* img, int row_bytes, int row, int kb, int g) {
    return *reinterpret_cast<const bf16x8_t*>(img + row * row_bytes + (kb * 32 + g * 8) * 2);
}

// Column-owning epilogue of one wave: accumulator element r of row tile t is (row 16t + 4g + r, col)
// of the block's rows; ``row0`` offsets every global row index (row-blocked grids: mid.hip), rows
// >= M (block-local) are not stored.
template <int EPI, int MT>
__device__ __forceinline__ void skinny_store(const f32x4_t* acc, int M, int col, int g, const GemmEpi& ep,
                                             int row0 = 0) {
    const float bv = (EPI != SK_PARTIAL && ep.bias) ? ep.bias[col] : 0.f;
    if constexpr (EPI == SK_F32 || EPI == SK_FIXADD) {
        // in-place residual update: every old value is loaded before the first store, so the
        // wave pays ONE memory round trip, not one per row (interleaved load / store pairs to
        // possibly-aliasing addresses are kept in program order by the compiler: 8 serial round
        // trips per lane at 32 rows)
        typedef std::conditional_t<EPI == SK_F32, float, long long> T;
        T* base = reinterpret_cast<T*>(ep.out);
        T old[MT][4];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * t + g * 4 + r;
                old[t][r] = row < M ? base[(size_t)(row0 + row) * ep.ldo + col] : T(0);
            }
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * t + g * 4 + r;
                if (row >= M) continue;
                const float v = acc[t][r] + bv;
                if constexpr (EPI == SK_F32)
                    base[(size_t)(row0 + row) * ep.ldo + col] = old[t][r] + v;
                else
                    base[(size_t)(row0 + row) * ep.ldo + col] = old[t][r] + __float2ll_rn(v * 4294967296.0f);  // DLMS_FIX_SCALE
            }
        return;
    }
    if constexpr (EPI == SK_QKV) {
        // K/V rows go to each row's cache slot / position: both index loads of every row are issued
        // before the first store (interleaved with the stores they were one round trip per row)
        const int part = col / ep.d_local;
        const int within = col - part * ep.d_local;
        if (part == 0) {
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 16 * t + g * 4 + r;
                    if (row < M) ep.q_out[(size_t)(row0 + row) * ep.ldq + within] = f32_to_bf16(acc[t][r] + bv);
                }
            return;
        }
        int sl[MT][4], ps[MT][4];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * t + g * 4 + r;
                const int rr = row < M ? row : M - 1;
                sl[t][r] = ep.row_slot[row0 + rr];
                ps[t][r] = ep.row_pos[row0 + rr];
            }
        bf16_t* cache = part == 1 ? ep.k_cache : ep.v_cache;
        const int head = within >> 6, dim = within & 63;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * t + g * 4 + r;
                if (row >= M) continue;
                const size_t slot = dlms_idx(sl[t][r], ep.n_slots, CHK_QKV_SLOT);
                const size_t pos = dlms_idx(ps[t][r], ep.t_max, CHK_QKV_POS);
                cache[((slot * ep.n_heads + head) * ep.t_max + pos) * 64 + dim] = f32_to_bf16(acc[t][r] + bv);
            }
        return;
    }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * t + g * 4 + r;
            if (row >= M) continue;
            float v = acc[t][r] + bv;
            const size_t grow = (size_t)(row0 + row);
            if constexpr (EPI == SK_BF16) {
                reinterpret_cast<bf16_t*>(ep.out)[grow * ep.ldo + col] = f32_to_bf16(v);
            } else if constexpr (EPI == SK_GELU_TANH) {
                reinterpret_cast<bf16_t*>(ep.out)[grow * ep.ldo + col] = f32_to_bf16(gelu_tanh(v));
            } else if constexpr (EPI == SK_PARTIAL) {
                reinterpret_cast<float*>(ep.out)[grow * ep.ldo + col] = acc[t][r];
            }
        }
}

