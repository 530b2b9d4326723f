// MFMA bf16 "TN" GEMM for gfx950 with fused epilogues.
//
//   C[M, N] = A[M, K] . W[N, K]^T  (+ bias[N]) -> epilogue
//
// A is the activation (row-major, K contiguous), W the weight stored [N][K] (K contiguous) so
// that both MFMA operands are read as contiguous 16-byte fragments.  One workgroup = 4 waves
// (256 threads) computes a BM x BN tile with v_mfma_f32_16x16x32_bf16; K advances in 64-deep
// steps staged through a double-buffered, padded LDS image (one barrier per K-step, the next
// step's global loads in flight behind the current step's MFMAs).
//
// Epilogues (all fused, no extra pass over C):
//   EPI_BF16        out = bf16(acc + bias)
//   EPI_GELU_TANH   out = bf16(gelu_tanh(acc + bias))            GPT-2 c_fc (K8)
//   EPI_GELU_ERF    out = bf16(gelu_erf(acc + bias))             BERT intermediate (K15)
//   EPI_F32         out = f32(acc + bias + resid)                residual projections (K7/K9);
//                                                                in-place when out == resid
//   EPI_QKV         q -> q_out, k/v scattered into the KV cache at (slot,pos) of each row (K3+K4)
//   EPI_ARGMAX      repetition-penalised logits -> per-row packed (value,index) atomicMax (K10-K12)
#include "common.h"

enum { EPI_BF16 = 0, EPI_GELU_TANH = 1, EPI_GELU_ERF = 2, EPI_F32 = 3, EPI_QKV = 4, EPI_ARGMAX = 5 };

// struct GemmEpi lives in common.h (shared with the ABI probe in api.hip)

#define GEMM_BK 64
#define GEMM_LDS_STRIDE (GEMM_BK + 8)  // +16 B pad per row breaks the 128-B row bank aliasing

template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(256) void gemm_tn_kernel(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W, int ldw, int M, int N,
                                                      int K, GemmEpi ep) {
    static_assert(WM * WN == 4, "4 waves per workgroup");
    constexpr int WTM = BM / WM;  // rows per wave
    constexpr int WTN = BN / WN;  // cols per wave
    constexpr int TM = WTM / 16;
    constexpr int TN = WTN / 16;
    static_assert(TM >= 1 && TN >= 1, "wave tile must hold at least one 16x16 MFMA tile");
    constexpr int A_CHUNKS = BM * GEMM_BK / 8;  // 16-byte chunks per A tile
    constexpr int W_CHUNKS = BN * GEMM_BK / 8;
    constexpr int A_PER_T = (A_CHUNKS + 255) / 256;
    constexpr int W_PER_T = (W_CHUNKS + 255) / 256;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* As = reinterpret_cast<bf16_t*>(smem);                     // [2][BM][STRIDE]
    bf16_t* Ws = As + 2 * BM * GEMM_LDS_STRIDE;                        // [2][BN][STRIDE]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;

    const int tiles_m = (M + BM - 1) / BM;
    const int nwg = gridDim.x;
    const int bid = xcd_remap(blockIdx.x, nwg);
    const int tile_m = bid % tiles_m;
    const int tile_n = bid / tiles_m;
    const int m0 = tile_m * BM;
    const int n0 = tile_n * BN;

    uint4 ra[A_PER_T];
    uint4 rw[W_PER_T];

    auto load_tile = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            const int c = tid + i * 256;
            if (c < A_CHUNKS) {
                const int r = c >> 3, kc = c & 7;
                const int gm = m0 + r;
                ra[i] = (gm < M) ? *reinterpret_cast<const uint4*>(A + (size_t)gm * lda + k0 + kc * 8)
                                 : make_uint4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int i = 0; i < W_PER_T; ++i) {
            const int c = tid + i * 256;
            if (c < W_CHUNKS) {
                const int r = c >> 3, kc = c & 7;
                rw[i] = *reinterpret_cast<const uint4*>(W + (size_t)(n0 + r) * ldw + k0 + kc * 8);
            }
        }
    };
    auto store_tile = [&](int buf) {
        bf16_t* as = As + buf * BM * GEMM_LDS_STRIDE;
        bf16_t* ws = Ws + buf * BN * GEMM_LDS_STRIDE;
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            const int c = tid + i * 256;
            if (c < A_CHUNKS) {
                const int r = c >> 3, kc = c & 7;
                *reinterpret_cast<uint4*>(as + r * GEMM_LDS_STRIDE + kc * 8) = ra[i];
            }
        }
#pragma unroll
        for (int i = 0; i < W_PER_T; ++i) {
            const int c = tid + i * 256;
            if (c < W_CHUNKS) {
                const int r = c >> 3, kc = c & 7;
                *reinterpret_cast<uint4*>(ws + r * GEMM_LDS_STRIDE + kc * 8) = rw[i];
            }
        }
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int nk = K / GEMM_BK;
    load_tile(0);
    store_tile(0);
    __syncthreads();

    const int frag_row = lane & 15;
    const int frag_k = (lane >> 4) * 8;

    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tile((kt + 1) * GEMM_BK);
        const bf16_t* as = As + buf * BM * GEMM_LDS_STRIDE + (wm * WTM) * GEMM_LDS_STRIDE;
        const bf16_t* ws = Ws + buf * BN * GEMM_LDS_STRIDE + (wn * WTN) * GEMM_LDS_STRIDE;
#pragma unroll
        for (int ks = 0; ks < GEMM_BK / 32; ++ks) {
            bf16x8_t af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frag_row) * GEMM_LDS_STRIDE + ks * 32 + frag_k);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frag_row) * GEMM_LDS_STRIDE + ks * 32 + frag_k);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_tile(buf ^ 1);
        __syncthreads();
    }

    // ---------------- epilogue ----------------
    // accumulator element r of tile (i,j): row = (lane>>4)*4 + r, col = lane & 15
    const int row_base = m0 + wm * WTM + (lane >> 4) * 4;
    const int col_base = n0 + wn * WTN + (lane & 15);

    if constexpr (EPI == EPI_ARGMAX) {
        unsigned long long best[TM][4];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) best[i][r] = 0ull;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row_base + i * 16 + r;
                if (row >= M) continue;
                const unsigned int* srow = ep.seen + (size_t)row * ep.seen_words;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = col_base + j * 16;
                    const int gcol = col + ep.col_offset;
                    if (gcol >= ep.vocab) continue;
                    float v = acc[i][j][r];
                    if ((srow[gcol >> 5] >> (gcol & 31)) & 1u) v = v < 0.f ? v * ep.penalty : v / ep.penalty;
                    const unsigned long long key =
                        ((unsigned long long)f32_ordered(v) << 32) | (unsigned long long)(~(unsigned int)gcol);
                    best[i][r] = key > best[i][r] ? key : best[i][r];
                }
            }
        }
        // reduce across the 16 lanes that share rows (lane bits 0..3 = column)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                unsigned long long b = best[i][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    unsigned long long other = __shfl_xor(b, o, 64);
                    b = other > b ? other : b;
                }
                const int row = row_base + i * 16 + r;
                if ((lane & 15) == 0 && row < M && b != 0ull) atomicMax(ep.argmax_out + row, b);
            }
        return;
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = col_base + j * 16;
        const float bv = ep.bias ? ep.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row_base + i * 16 + r;
                if (row >= M) continue;
                float v = acc[i][j][r] + bv;
                if constexpr (EPI == EPI_BF16) {
                    reinterpret_cast<bf16_t*>(ep.out)[(size_t)row * ep.ldo + col] = f32_to_bf16(v);
                } else if constexpr (EPI == EPI_GELU_TANH) {
                    reinterpret_cast<bf16_t*>(ep.out)[(size_t)row * ep.ldo + col] = f32_to_bf16(gelu_tanh(v));
                } else if constexpr (EPI == EPI_GELU_ERF) {
                    reinterpret_cast<bf16_t*>(ep.out)[(size_t)row * ep.ldo + col] = f32_to_bf16(gelu_erf(v));
                } else if constexpr (EPI == EPI_F32) {
                    if (ep.resid) v += ep.resid[(size_t)row * ep.ldr + col];
                    reinterpret_cast<float*>(ep.out)[(size_t)row * ep.ldo + col] = v;
                } else if constexpr (EPI == EPI_QKV) {
                    const int part = col / ep.d_local;
                    const int within = col - part * ep.d_local;
                    const bf16_t hv = f32_to_bf16(v);
                    if (part == 0) {
                        ep.q_out[(size_t)row * ep.ldq + within] = hv;
                    } else {
                        const int head = within >> 6, dim = within & 63;
                        const size_t idx =
                            (((size_t)ep.row_slot[row] * ep.n_heads + head) * ep.t_max + ep.row_pos[row]) * 64 + dim;
                        (part == 1 ? ep.k_cache : ep.v_cache)[idx] = hv;
                    }
                }
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int EPI>
static hipError_t launch_gemm_cfg(const bf16_t* A, int lda, const bf16_t* W, int ldw, int M, int N, int K,
                                  const GemmEpi& ep, hipStream_t stream) {
    const int tiles = ((M + BM - 1) / BM) * (N / BN);
    const size_t lds = (size_t)2 * (BM + BN) * GEMM_LDS_STRIDE * sizeof(bf16_t);
    hipLaunchKernelGGL((gemm_tn_kernel<BM, BN, WM, WN, EPI>), dim3(tiles), dim3(256), lds, stream, A, lda, W, ldw, M,
                       N, K, ep);
    return hipGetLastError();
}

// Tile selection: decode GEMMs (M = live batch) are latency-bound, so favour enough workgroups
// to cover the 256 CUs; prefill/encoder GEMMs (M in the thousands) take 128x64 tiles.
template <int EPI>
static hipError_t launch_gemm_epi(const bf16_t* A, int lda, const bf16_t* W, int ldw, int M, int N, int K,
                                  const GemmEpi& ep, hipStream_t stream) {
    if (M <= 16) {
        if (N % 64 == 0) return launch_gemm_cfg<16, 64, 1, 4, EPI>(A, lda, W, ldw, M, N, K, ep, stream);
        return launch_gemm_cfg<16, 64, 1, 4, EPI>(A, lda, W, ldw, M, N, K, ep, stream);
    }
    if (M <= 32) return launch_gemm_cfg<32, 64, 2, 2, EPI>(A, lda, W, ldw, M, N, K, ep, stream);
    const long tiles64 = (long)((M + 63) / 64) * (N / 64);
    if (M <= 256 || tiles64 < 512) return launch_gemm_cfg<64, 64, 2, 2, EPI>(A, lda, W, ldw, M, N, K, ep, stream);
    return launch_gemm_cfg<128, 64, 2, 2, EPI>(A, lda, W, ldw, M, N, K, ep, stream);
}

extern "C" hipError_t dlms_gemm(int epi, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                const GemmEpi* ep, hipStream_t stream) {
    if (K % GEMM_BK != 0 || N % 64 != 0 || M <= 0) return hipErrorInvalidValue;
    const bf16_t* a = reinterpret_cast<const bf16_t*>(A);
    const bf16_t* w = reinterpret_cast<const bf16_t*>(W);
    switch (epi) {
        case EPI_BF16: return launch_gemm_epi<EPI_BF16>(a, lda, w, ldw, M, N, K, *ep, stream);
        case EPI_GELU_TANH: return launch_gemm_epi<EPI_GELU_TANH>(a, lda, w, ldw, M, N, K, *ep, stream);
        case EPI_GELU_ERF: return launch_gemm_epi<EPI_GELU_ERF>(a, lda, w, ldw, M, N, K, *ep, stream);
        case EPI_F32: return launch_gemm_epi<EPI_F32>(a, lda, w, ldw, M, N, K, *ep, stream);
        case EPI_QKV: return launch_gemm_epi<EPI_QKV>(a, lda, w, ldw, M, N, K, *ep, stream);
        case EPI_ARGMAX: return launch_gemm_epi<EPI_ARGMAX>(a, lda, w, ldw, M, N, K, *ep, stream);
        default: return hipErrorInvalidValue;
    }
}
