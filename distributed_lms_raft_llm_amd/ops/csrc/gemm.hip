// MFMA bf16 "TN" GEMM for gfx950 with fused epilogues.
//
//   C[M, N] = A[M, K] . W[N, K]^T  (+ bias[N]) -> epilogue
//
// A is the activation (row-major, K contiguous), W the weight stored [N][K] (K contiguous) so
// that both MFMA operands are read as contiguous 16-byte fragments.  One workgroup = 4 waves
// (256 threads) computes a BM x BN tile with v_mfma_f32_16x16x32_bf16; K advances in 64-deep
// steps through a 3-stage LDS ring filled by LDS-DMA (two steps of loads in flight behind the
// MFMAs of the current one, one raw barrier per step).
//
// Epilogues (all fused, no extra pass over C):
//   EPI_BF16        out = bf16(acc + bias)
//   EPI_GELU_TANH   out = bf16(gelu_tanh(acc + bias))            GPT-2 c_fc (K8)
//   EPI_GELU_ERF    out = bf16(gelu_erf(acc + bias))             BERT intermediate (K15)
//   EPI_F32         out = f32(acc + bias + resid)                residual projections (K7/K9);
//                                                                in-place when out == resid
//   EPI_QKV         q -> q_out, k/v scattered into the KV cache at (slot,pos) of each row (K3+K4)
//   EPI_ARGMAX      repetition-penalised logits -> per-row packed (value,index) atomicMax (K10-K12)
//   (IN = IN_FP8: A and W are OCP e4m3 with per-row / per-output-channel fp32 scales; the same
//   128-B LDS rows then hold 128 k-elements, each 16-B fragment feeds two
//   v_mfma_f32_16x16x32_fp8_fp8, and acc is rescaled by a_scale[row] * w_scale[col] before the
//   epilogue.  W8A8 halves the weight bytes the latency-bound decode GEMMs stream.)
//   EPI_PARTIAL     split-K: slice s stores its raw fp32 partial tile; the following fused
//                   residual-add + LayerNorm kernel sums the slices in a fixed order (deterministic,
//                   no atomics) -- the decode projections with N = d are split 2-4 ways so the
//                   latency-bound skinny GEMMs put enough workgroups on the 256 CUs.
#include "common.h"
#include <atomic>
#include <stdlib.h>

enum { EPI_BF16 = 0, EPI_GELU_TANH = 1, EPI_GELU_ERF = 2, EPI_F32 = 3, EPI_QKV = 4, EPI_ARGMAX = 5, EPI_PARTIAL = 6 };
enum { MODE_REGPF = 1, MODE_GROUPED = 2 };

// struct GemmEpi lives in common.h (shared with the ABI probe in api.hip)

#define GEMM_BK 64  // k-elements per ring step for bf16 (128 for fp8: the row is 128 B either way)
enum { IN_BF16 = 0, IN_FP8 = 1 };

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Main loop: K advances in 64-deep steps through a STAGES-deep LDS ring (STAGES-1 steps of loads in
// flight: the decode GEMMs are HBM-latency-bound, so the ring is as deep as the LDS allows) filled by
// global_load_lds_dwordx4 (LDS-DMA, no staging registers).  Each 1-KiB wave-instruction lands 8 tile
// rows of 128 B; the 16-B chunks of a row are XOR-swizzled (phys = logical ^ (row & 7)) by permuting
// the per-lane SOURCE address, and the fragment reads apply the same involution, which makes the
// ds_read_b128 fragment loads bank-conflict free (cdna_hip_programming.md rule 21 / T2).
// Synchronisation: counted `s_waitcnt vmcnt` + raw s_barrier (a __syncthreads() would drain the
// in-flight DMA every step); out-of-range A rows read a clamped valid row (their results are never
// stored), so the DMA never needs predication.
//
// MODE (big prefill GEMMs, 256x256 tiles; see launch_gemm_epi):
//   bit 0  REGPF: a whole K-tile's fragments go LDS -> registers right after its barrier, so its
//          buffer is free one barrier later and the DMA of tile t+2 is issued before tile t's
//          MFMAs (two K-tiles of loads in flight with two LDS buffers, instead of one)
//   bit 1  GROUPED: tiles enumerated in groups of GROUP_M row tiles x all column tiles, so the 32
//          workgroups an XCD runs at once share 4 A panels and 8 W panels through its L2 (the
//          column-major order gave every one of them its own A panel: 32 panels from beyond L2)
#define GROUP_M 4
// Write-out of an LDS-staged bf16 QKV tile (rows [r0, r0 + CHUNKS / CPR), columns from c0, CPR
// 16-B chunks per row): q columns go to q_out, K/V columns to each row's cache slot / position.
// Every chunk's slot / position index is loaded before the first store -- interleaved with the
// stores they cost one dependent L2 round trip per chunk (3-8 per thread per tile).
template <int CHUNKS, int NT, int CPR>
__device__ __forceinline__ void qkv_staged_store(const char* smem, int srow, int tid, int r0, int c0, int M,
                                                 const GemmEpi& ep) {
    constexpr int ITER = (CHUNKS + NT - 1) / NT;
    int sl[ITER], ps[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        int c = tid + it * NT;
        c = c < CHUNKS ? c : CHUNKS - 1;
        int row = r0 + c / CPR;
        row = row < M ? row : M - 1;
        sl[it] = ep.row_slot[row];
        ps[it] = ep.row_pos[row];
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int c = tid + it * NT;
        if (c >= CHUNKS) break;
        const int lr = c / CPR, ch = c - lr * CPR;
        const int row = r0 + lr;
        if (row >= M) continue;
        const uint4 val = *reinterpret_cast<const uint4*>(smem + lr * srow + ch * 16);
        const int col = c0 + ch * 8;
        const int part = col / ep.d_local;
        const int within = col - part * ep.d_local;
        bf16_t* dst;
        if (part == 0) {
            dst = ep.q_out + (size_t)row * ep.ldq + within;
        } else {
            const int head = within >> 6, dim = within & 63;
            const size_t slot = dlms_idx(sl[it], ep.n_slots, CHK_QKV_SLOT);
            const size_t pos = dlms_idx(ps[it], ep.t_max, CHK_QKV_POS);
            dst = (part == 1 ? ep.k_cache : ep.v_cache) + ((slot * ep.n_heads + head) * ep.t_max + pos) * 64 + dim;
        }
        *reinterpret_cast<uint4*>(dst) = val;
    }
}

template <int BM, int BN, int WM, int WN, int STAGES, int EPI, int IN, int MODE = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_tn_kernel(const void* __restrict__ A, int lda,
                                                      const void* __restrict__ W, int ldw, int M, int N,
                                                      int K, GemmEpi ep) {
    constexpr int EB = IN == IN_FP8 ? 1 : 2;    // bytes per element
    constexpr int BKE = GEMM_BK * 2 / EB;       // k-elements per ring step
    constexpr int NW = WM * WN;  // waves per workgroup (4 or 8)
    constexpr int NT = 64 * NW;
    static_assert(NW == 4 || NW == 8, "4 or 8 waves per workgroup");
    constexpr int WTM = BM / WM;  // rows per wave
    constexpr int WTN = BN / WN;  // cols per wave
    constexpr int TM = WTM / 16;
    constexpr int TN = WTN / 16;
    static_assert(TM >= 1 && TN >= 1, "wave tile must hold at least one 16x16 MFMA tile");
    constexpr int ROWB = GEMM_BK * 2;  // 128 B per tile row
    constexpr int A_BYTES = BM * ROWB;
    constexpr int STAGE_BYTES = (BM + BN) * ROWB;
    constexpr int PIECES = STAGE_BYTES / 1024;
    static_assert(PIECES % NW == 0, "(BM + BN) * 128 B must split evenly into 1-KiB pieces per wave");
    constexpr int PPW = PIECES / NW;  // LDS-DMA instructions per wave per stage

    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN;
    const int wn = wave % WN;

    const int tiles_m = (M + BM - 1) / BM;
    const int nwg = gridDim.x;
    const int nsplit = EPI == EPI_PARTIAL ? ep.split_k : 1;
    const int tiles = nwg / nsplit;
    const int bid0 = xcd_remap(blockIdx.x, nwg);
    const int split = bid0 / tiles;
    const int bid = bid0 - split * tiles;
    constexpr bool REGPF = (MODE & MODE_REGPF) != 0;
    constexpr bool GROUPED = (MODE & MODE_GROUPED) != 0;
    static_assert(!REGPF || (STAGES == 2 && IN == IN_BF16), "REGPF: 2 bf16 stages");
    int tile_m, tile_n;
    if constexpr (GROUPED) {
        const int tiles_n = N / BN;
        const int per_group = GROUP_M * tiles_n;
        const int g = bid / per_group, r = bid - g * per_group;
        const int gm0 = g * GROUP_M;
        const int gsz = tiles_m - gm0 < GROUP_M ? tiles_m - gm0 : GROUP_M;
        tile_m = gm0 + r % gsz;
        tile_n = r / gsz;
    } else {
        tile_m = bid % tiles_m;
        tile_n = bid / tiles_m;
    }
    const int m0 = tile_m * BM;
    const int n0 = tile_n * BN;
    const int k_len = K / nsplit;
    const int k_base = split * k_len;

    // per-lane DMA sources (fixed for the K loop; byte addresses)
    const char* src[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int piece = wave + NW * i;
        const int row = piece * 8 + (lane >> 3);
        const int lchunk = (lane & 7) ^ (lane >> 3);
        if (row < BM) {
            const int gm = m0 + row < M ? m0 + row : M - 1;
            src[i] = reinterpret_cast<const char*>(A) + ((size_t)gm * lda + k_base) * EB + lchunk * 16;
        } else {
            src[i] = reinterpret_cast<const char*>(W) + ((size_t)(n0 + row - BM) * ldw + k_base) * EB + lchunk * 16;
        }
    }
    auto issue = [&](int stage, int k0) {
        char* dst = smem + stage * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < PPW; ++i)
            __builtin_amdgcn_global_load_lds((glob_void_t*)(src[i] + (size_t)k0 * EB),
                                             (lds_void_t*)(dst + (wave + NW * i) * 1024), 16, 0, 0);
    };

    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int nk = k_len / BKE;
    const int frow = lane & 15;
    const int fk = lane >> 4;
    const int fsw = lane & 7;  // == row & 7 for every fragment row this lane reads

    if constexpr (REGPF) {
        // tiles t and t+1 in flight at the top of iteration t; tile t+2 issued into tile t's buffer
        // once every wave holds tile t's fragments in registers
        issue(0, 0);
        if (nk > 1) issue(1, BKE);
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk)
                wait_vmcnt<PPW>();
            else
                wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();  // tile kt has landed for every lane
            asm volatile("" ::: "memory");
            const char* as = smem + (kt & 1) * STAGE_BYTES + (wm * WTM) * ROWB;
            const char* ws = smem + (kt & 1) * STAGE_BYTES + A_BYTES + (wn * WTN) * ROWB;
            bf16x8_t af[2][TM], bfr[2][TN];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int coff = (((ks * 4 + fk) ^ fsw) << 4);
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[ks][i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frow) * ROWB + coff);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[ks][j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frow) * ROWB + coff);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // every wave's reads of buffer kt & 1 are done
            asm volatile("" ::: "memory");
            if (kt + 2 < nk) issue(kt & 1, (kt + 2) * BKE);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
        }
    }
    // prologue: up to STAGES-1 steps in flight; no step is ever loaded twice (short split-K slices
    // would otherwise multiply their traffic)
    if constexpr (!REGPF) {
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if (s < nk) issue(s, s * BKE);
    }

    for (int kt = 0; kt < (REGPF ? 0 : nk); ++kt) {
        // this lane's share of step kt has landed (steady state: STAGES-2 younger steps may stay in
        // flight; in the tail fewer were issued, so drain everything) ...
        if (nk - kt >= STAGES - 1)
            wait_vmcnt<(STAGES - 2) * PPW>();
        else
            wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // ... and every other lane's; all reads of step kt-1 are done
        asm volatile("" ::: "memory");
        {
            const int kn = kt + STAGES - 1;
            if (kn < nk) issue(kn % STAGES, kn * BKE);
        }
        const char* as = smem + (kt % STAGES) * STAGE_BYTES + (wm * WTM) * ROWB;
        const char* ws = smem + (kt % STAGES) * STAGE_BYTES + A_BYTES + (wn * WTN) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = (((ks * 4 + fk) ^ fsw) << 4);
            if constexpr (IN == IN_FP8) {
                // a 16-B chunk = 16 k-elements: bytes 0-7 feed one fp8 MFMA, bytes 8-15 the next.
                // A and W use the same k permutation, so the dot products are unchanged.
                long af[TM][2], bfr[TN][2];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const uint4 v = *reinterpret_cast<const uint4*>(as + (i * 16 + frow) * ROWB + coff);
                    af[i][0] = (long)(((unsigned long long)v.y << 32) | v.x);
                    af[i][1] = (long)(((unsigned long long)v.w << 32) | v.z);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ws + (j * 16 + frow) * ROWB + coff);
                    bfr[j][0] = (long)(((unsigned long long)v.y << 32) | v.x);
                    bfr[j][1] = (long)(((unsigned long long)v.w << 32) | v.z);
                }
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i][h], bfr[j][h], acc[i][j],
                                                                                   0, 0, 0);
            } else {
                bf16x8_t af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frow) * ROWB + coff);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frow) * ROWB + coff);
                // (s_setprio(1)/(0) around this cluster, cdna guide T5, measured null on this 1-barrier
                // loop: prefill shapes and the whole decode within noise)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    wait_vmcnt<0>();  // drain the tail DMA before the workgroup may exit / LDS be reused

    if constexpr (IN == IN_FP8) {  // dequantise: per-row activation scale x per-channel weight scale
        const int rb = m0 + wm * WTM + (lane >> 4) * 4;
        const int cb = n0 + wn * WTN + (lane & 15);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const float wsc = ep.w_scale[cb + j * 16];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = rb + i * 16 + r;
                    acc[i][j][r] *= ep.a_scale[row < M ? row : M - 1] * wsc;
                }
            }
    }

    // ---------------- epilogue ----------------
    // accumulator element r of tile (i,j): row = (lane>>4)*4 + r, col = lane & 15
    const int row_base = m0 + wm * WTM + (lane >> 4) * 4;
    const int col_base = n0 + wn * WTN + (lane & 15);

    if constexpr (EPI == EPI_ARGMAX) {
        // Fused repetition penalty + argmax (K11/K12).  The block's BM x BN slice of the seen
        // bitmap is staged in LDS (BN/32 words per row; tile columns are 32-aligned), each row's
        // best (ordered value, ~index) key is reduced across lanes by shuffles and across the WN
        // column-waves through LDS, and ONE key per (row, column tile) is stored -- no atomics.
        // The consumer (decode_update / argmax_reduce) takes the max over the tiles of a row.
        constexpr int WPR = BN / 32;  // bitmap words per tile row
        unsigned int* sbits = reinterpret_cast<unsigned int*>(smem);
        unsigned long long* sred = reinterpret_cast<unsigned long long*>(smem + BM * WPR * 4 + 16);
        __syncthreads();  // every wave is done reading the last ring stage
        const int wbase = (n0 + ep.col_offset) >> 5;
        for (int e = tid; e < BM * WPR; e += NT) {
            const int r = e / WPR, w = e % WPR;
            const int row = m0 + r < M ? m0 + r : M - 1;
            const int word = wbase + w;
            sbits[e] = word < ep.seen_words ? ep.seen[(size_t)row * ep.seen_words + word] : 0u;
        }
        __syncthreads();
        const int lrow0 = wm * WTM + (lane >> 4) * 4;
        const int lcol0 = wn * WTN + (lane & 15);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int lr = lrow0 + i * 16 + r;
                unsigned long long b = 0ull;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int lc = lcol0 + j * 16;
                    const int gcol = n0 + lc + ep.col_offset;
                    float v = acc[i][j][r];
                    if ((sbits[lr * WPR + (lc >> 5)] >> (lc & 31)) & 1u) v = v < 0.f ? v * ep.penalty : v / ep.penalty;
                    const unsigned long long key =
                        ((unsigned long long)f32_ordered(v) << 32) | (unsigned long long)(~(unsigned int)gcol);
                    b = (gcol < ep.vocab && key > b) ? key : b;
                }
                b = row16_max_u64(b);  // max over the 16 lanes of this row
                if ((lane & 15) == 0) sred[wn * BM + lr] = b;
            }
        }
        __syncthreads();
        for (int lr = tid; lr < BM; lr += NT) {
            unsigned long long b = sred[lr];
#pragma unroll
            for (int w = 1; w < WN; ++w) {
                const unsigned long long o = sred[w * BM + lr];
                b = o > b ? o : b;
            }
            if (m0 + lr < M) {
                // one key per 64-column group: a BN > 64 tile also zeroes the groups it covers, so
                // keys left by an earlier, narrower tile config can never win the consumer's max
                unsigned long long* o = ep.argmax_out + (size_t)(m0 + lr) * ep.ldo + (n0 >> 6);
                o[0] = b;
#pragma unroll
                for (int g = 1; g < BN / 64; ++g) o[g] = 0ull;
            }
        }
        return;
    }

    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF || EPI == EPI_PARTIAL ||
                  EPI == EPI_QKV) {
        // LDS-staged store: the MFMA layout puts 16 consecutive columns on 16 lanes (2-4 B each), so
        // direct stores write 32-64 B pieces; staging the tile through LDS (padded rows: the four
        // lane groups' rows land 64 B apart, conflict-free) turns the write-out into full 16-B-per-lane
        // row stores.  The QKV scatter moves whole 8-column chunks (a chunk never straddles a head).
        constexpr int OB = EPI == EPI_PARTIAL ? 4 : 2;
        constexpr int SROW = BN * OB + 16;
        constexpr int CPR = BN * OB / 16;  // 16-B chunks per tile row
        __syncthreads();                   // every wave is done reading the last ring stage
        const int lrow0 = wm * WTM + (lane >> 4) * 4;
        const int lcol0 = wn * WTN + (lane & 15);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const float bv = (EPI != EPI_PARTIAL && ep.bias) ? ep.bias[n0 + lcol0 + j * 16] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[i][j][r] + bv;
                    if constexpr (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
                    if constexpr (EPI == EPI_GELU_ERF) v = gelu_erf(v);
                    char* dst = smem + (lrow0 + i * 16 + r) * SROW + (lcol0 + j * 16) * OB;
                    if constexpr (OB == 4)
                        *reinterpret_cast<float*>(dst) = v;
                    else
                        *reinterpret_cast<bf16_t*>(dst) = f32_to_bf16(v);
                }
        }
        __syncthreads();
        if constexpr (EPI == EPI_QKV) {
            qkv_staged_store<BM * CPR, NT, CPR>(smem, SROW, tid, m0, n0, M, ep);
            return;
        }
        for (int c = tid; c < BM * CPR; c += NT) {
            const int lr = c / CPR, ch = c - lr * CPR;
            const int row = m0 + lr;
            if (row >= M) continue;
            const uint4 val = *reinterpret_cast<const uint4*>(smem + lr * SROW + ch * 16);
            const int col = n0 + ch * (16 / OB);
            if constexpr (EPI == EPI_PARTIAL) {
                *reinterpret_cast<uint4*>(reinterpret_cast<float*>(ep.out) + (size_t)split * ep.split_stride +
                                          (size_t)row * ep.ldo + col) = val;
            } else {
                *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(ep.out) + (size_t)row * ep.ldo + col) = val;
            }
        }
        return;
    }

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = col_base + j * 16;
        const float bv = (EPI != EPI_PARTIAL && ep.bias) ? ep.bias[col] : 0.f;
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
                } else if constexpr (EPI == EPI_PARTIAL) {
                    reinterpret_cast<float*>(ep.out)[(size_t)split * ep.split_stride + (size_t)row * ep.ldo + col] =
                        acc[i][j][r];
                } else if constexpr (EPI == EPI_QKV) {
                    const int part = col / ep.d_local;
                    const int within = col - part * ep.d_local;
                    const bf16_t hv = f32_to_bf16(v);
                    if (part == 0) {
                        ep.q_out[(size_t)row * ep.ldq + within] = hv;
                    } else {
                        const int head = within >> 6, dim = within & 63;
                        const size_t slot = dlms_idx(ep.row_slot[row], ep.n_slots, CHK_QKV_SLOT);
                        const size_t pos = dlms_idx(ep.row_pos[row], ep.t_max, CHK_QKV_POS);
                        const size_t idx = ((slot * ep.n_heads + head) * ep.t_max + pos) * 64 + dim;
                        (part == 1 ? ep.k_cache : ep.v_cache)[idx] = hv;
                    }
                }
            }
        }
    }
}

// host-side launch census by tile shape (tests assert which instantiation a path dispatches;
// counted when the launch is issued, so graph captures count once per capture)
static std::atomic<long> g_tile_count[4][4];  // [BM 32/64/128/256][BN 64/96/128/256]

// ------------------------------------------------------------------------------------------------
// Big prefill GEMMs (M >= 16384 packed prompt rows): 256x256 tiles, 8 waves, an 8-phase K loop that
// keeps LDS-DMA half-tiles in flight ACROSS its barriers (cdna_hip_programming.md §5 "The 256² 8-phase
// template": counted vmcnt, raw s_barrier, all LDS in one dynamic array, the two wave rows a barrier
// apart so one row's fragment reads run under the other row's MFMAs).
//
// LDS: 2 buffers (even / odd K-tile) x {A rows 0-127, A rows 128-255, W rows 0-127, W rows 128-255}
// half-tiles of 128 rows x 64 k (128-B rows, 16-B chunks XOR-swizzled by row & 7) = 8 x 16 KiB.
// A phase computes one 128x128 block quadrant (mq, nq) of one K-tile: every wave its 64x32 piece
// (rows mq*128 + wr*64, cols nq*128 + wc*32; wr = w >> 2, wc = w & 3): 8 A / 4 W fragment reads
// (skipped when the previous phase read the same half), 16 MFMAs between two barriers.  Quadrant
// order (0,0) (0,1) (1,1) (1,0) reads a buffer's halves from LDS last in the order A0, W1, A1, W0
// (fragments are reused in registers between consecutive phases); each phase issues ONE half-tile
// (2 DMA instructions per thread) into the half whose last read was the phase before:
//   ph0 odd.W0 (K-tile 2i+1)  ph1 even.A0 (2i+2)  ph2 even.W1 (2i+2)  ph3 even.A1 (2i+2)
//   ph4 even.W0 (2i+2)        ph5 odd.A0 (2i+3)   ph6 odd.W1 (2i+3)   ph7 odd.A1 (2i+3)
// and the waits in ph3 / ph7 (vmcnt(6): the three younger half-tiles stay in flight) retire
// everything the next buffer's four phases read.  K must be a multiple of 128 (an even number of
// K-tiles).  It sums every output in the same k order as gemm_tn_kernel, so its results are
// bit-identical to the 128x128 tiles' (tests/test_kernels_gpu.py).
template <int EPI>
__global__ __launch_bounds__(512) void gemm8p_kernel(const bf16_t* __restrict__ A, int lda,
                                                     const bf16_t* __restrict__ W, int ldw, int M, int N, int K,
                                                     GemmEpi ep) {
    constexpr int BM = 256, BN = 256, HALF = 16384, ROWB = 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 2, wc = w & 3;

    const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
    const int nsplit = EPI == EPI_PARTIAL ? ep.split_k : 1;
    const int tiles = tiles_m * tiles_n;
    const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
    const int split = bid0 / tiles;
    const int bid = bid0 - split * tiles;
    // groups of GROUP_M row tiles x all column tiles (an XCD's workgroups share A / W panels in L2)
    const int per_group = GROUP_M * tiles_n;
    const int g = bid / per_group, rg = bid - g * per_group;
    const int gm0 = g * GROUP_M;
    const int gsz = tiles_m - gm0 < GROUP_M ? tiles_m - gm0 : GROUP_M;
    const int m0 = (gm0 + rg % gsz) * BM, n0 = (rg / gsz) * BN;
    const int k_len = K / nsplit, k_base = split * k_len;
    const int nk = k_len / 64, niter = nk / 2;

    // DMA sources: thread t of wave w fills pieces w and w + 8 (8 rows x 128 B each) of a half
    // tile; byte offsets (32 bit: operands < 4 GiB) from A / W, before the k offset
    unsigned aoff[2][2], woff[2][2];  // [half][piece]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
            const int r = (w + 8 * pc) * 8 + (lane >> 3);
            const int chunk = (lane & 7) ^ (lane >> 3);
            int gm = m0 + h * 128 + r;
            gm = gm < M ? gm : M - 1;
            aoff[h][pc] = (unsigned)((size_t)gm * lda * 2 + (size_t)k_base * 2 + chunk * 16);
            woff[h][pc] = (unsigned)((size_t)(n0 + h * 128 + r) * ldw * 2 + (size_t)k_base * 2 + chunk * 16);
        }
    const char* Ab = reinterpret_cast<const char*>(A);
    const char* Wb = reinterpret_cast<const char*>(W);
    // half-tile slots: buffer b, part q (0 A0, 1 A1, 2 W0, 3 W1)
    auto issue = [&](int b, int q, int kt) {
        char* dst = smem + (b * 4 + q) * HALF;
        const int h = q & 1;
        const unsigned kb = (unsigned)kt * 128u;  // 64 bf16 per K-tile
#pragma unroll
        for (int pc = 0; pc < 2; ++pc) {
            const char* src = q < 2 ? Ab + aoff[h][pc] + kb : Wb + woff[h][pc] + kb;
            __builtin_amdgcn_global_load_lds((glob_void_t*)src, (lds_void_t*)(dst + (w + 8 * pc) * 1024), 16, 0, 0);
        }
    };

    f32x4_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    bf16x8_t af[4][2], bfr[2][2];
    const int frow = lane & 15, fk = lane >> 4, fsw = lane & 7;

    auto read_a = [&](int b, int mq) {
        const char* base = smem + (b * 4 + mq) * HALF + (wr * 64) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = ((ks * 4 + fk) ^ fsw) << 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][ks] = *reinterpret_cast<const bf16x8_t*>(base + (i * 16 + frow) * ROWB + coff);
        }
    };
    auto read_w = [&](int b, int nq) {
        const char* base = smem + (b * 4 + 2 + nq) * HALF + (wc * 32) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = ((ks * 4 + fk) ^ fsw) << 4;
#pragma unroll
            for (int j = 0; j < 2; ++j) bfr[j][ks] = *reinterpret_cast<const bf16x8_t*>(base + (j * 16 + frow) * ROWB + coff);
        }
    };
    auto mfma = [&](int mq, int nq) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[mq * 4 + i][nq * 2 + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bfr[j][ks], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };

    // prologue: what iteration -1 would have issued -- the even buffer <- K-tile 0 (ph1-ph4) and
    // odd.A0 / odd.W1 / odd.A1 <- K-tile 1 (ph5-ph7); retire K-tile 0, three halves stay in flight
    issue(0, 0, 0);
    issue(0, 3, 0);
    issue(0, 1, 0);
    issue(0, 2, 0);
    issue(1, 0, 1);
    issue(1, 3, 1);
    issue(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the two wave rows run one barrier apart (two barriers per phase): row 1's fragment reads
    // overlap row 0's MFMAs and the other way round on every SIMD (cdna guide, 8-phase template)
    if (wr == 1) __builtin_amdgcn_s_barrier();

    // a phase: LDS fragment reads -> this phase's DMA -> [the K-tile wait] -> reads land -> barrier
    // -> 16 MFMAs -> barrier.  A wait sits BEFORE the first barrier of the phase ahead of the reads
    // it guards: with the rows a barrier apart, the other row passes its own wait before the
    // barrier this row crosses next (RAW); a half is refilled one phase after its last LDS read,
    // which both rows retired (lgkmcnt(0)) before the barrier ending that phase (WAR).
    auto sync1 = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    auto wait_ktile = [&](bool more) {
        if (more)
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // three younger half-tiles stay in flight
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };

    for (int it = 0; it < niter; ++it) {
        const bool more = it + 1 < niter;  // K-tiles 2it+2 / 2it+3 exist
        const int k0 = 2 * it;
        // ---- even buffer, K-tile k0 (LDS reads: A0 + W0, W1, A1, W0)
        read_a(0, 0);
        read_w(0, 0);
        issue(1, 2, k0 + 1);  // ph0: odd.W0 (its last read was ph7)
        sync1();
        mfma(0, 0);
        __builtin_amdgcn_s_barrier();
        read_w(0, 1);
        if (more) issue(0, 0, k0 + 2);  // ph1: even.A0 (last read ph0)
        sync1();
        mfma(0, 1);
        __builtin_amdgcn_s_barrier();
        read_a(0, 1);
        if (more) issue(0, 3, k0 + 2);  // ph2: even.W1 (last read ph1)
        sync1();
        mfma(1, 1);
        __builtin_amdgcn_s_barrier();
        read_w(0, 0);
        if (more) issue(0, 1, k0 + 2);  // ph3: even.A1 (last read ph2)
        wait_ktile(more);                // through ph0: the odd K-tile (read from ph4) has landed
        sync1();
        mfma(1, 0);
        __builtin_amdgcn_s_barrier();
        // ---- odd buffer, K-tile k0 + 1
        read_a(1, 0);
        read_w(1, 0);
        if (more) issue(0, 2, k0 + 2);  // ph4: even.W0 (last read ph3)
        sync1();
        mfma(0, 0);
        __builtin_amdgcn_s_barrier();
        read_w(1, 1);
        if (more) issue(1, 0, k0 + 3);  // ph5: odd.A0 (last read ph4)
        sync1();
        mfma(0, 1);
        __builtin_amdgcn_s_barrier();
        read_a(1, 1);
        if (more) issue(1, 3, k0 + 3);  // ph6: odd.W1 (last read ph5)
        sync1();
        mfma(1, 1);
        __builtin_amdgcn_s_barrier();
        read_w(1, 0);
        if (more) issue(1, 1, k0 + 3);  // ph7: odd.A1 (last read ph6)
        wait_ktile(more);                // through ph4: the next even K-tile has landed
        sync1();
        mfma(1, 0);
        __builtin_amdgcn_s_barrier();
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // realign the rows

    // ---------------- epilogue: one 128x128 block quadrant at a time through LDS ----------------
    // (accumulator element r of tile (i, j) of quadrant (mq, nq): row mq*128 + wr*64 + i*16 +
    // (lane>>4)*4 + r, column nq*128 + wc*32 + j*16 + (lane&15))
    constexpr int OB = EPI == EPI_PARTIAL ? 4 : 2;
    constexpr int SROW = 128 * OB + 16;
    constexpr int CPR = 128 * OB / 16;
#pragma unroll
    for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int nq = 0; nq < 2; ++nq) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int lc = wc * 32 + j * 16 + (lane & 15);
                const float bv = (EPI != EPI_PARTIAL && ep.bias) ? ep.bias[n0 + nq * 128 + lc] : 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = acc[mq * 4 + i][nq * 2 + j][r] + bv;
                        if constexpr (EPI == EPI_GELU_TANH) v = gelu_tanh(v);
                        char* dst = smem + (wr * 64 + i * 16 + (lane >> 4) * 4 + r) * SROW + lc * OB;
                        if constexpr (OB == 4)
                            *reinterpret_cast<float*>(dst) = v;
                        else
                            *reinterpret_cast<bf16_t*>(dst) = f32_to_bf16(v);
                    }
            }
            __syncthreads();
            if constexpr (EPI == EPI_QKV) {
                qkv_staged_store<128 * CPR, 512, CPR>(smem, SROW, tid, m0 + mq * 128, n0 + nq * 128, M, ep);
                __syncthreads();
                continue;
            }
            for (int c = tid; c < 128 * CPR; c += 512) {
                const int lr = c / CPR, ch = c - lr * CPR;
                const int row = m0 + mq * 128 + lr;
                if (row >= M) continue;
                const uint4 val = *reinterpret_cast<const uint4*>(smem + lr * SROW + ch * 16);
                const int col = n0 + nq * 128 + ch * (16 / OB);
                if constexpr (EPI == EPI_PARTIAL) {
                    *reinterpret_cast<uint4*>(reinterpret_cast<float*>(ep.out) + (size_t)split * ep.split_stride +
                                              (size_t)row * ep.ldo + col) = val;
                } else {
                    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(ep.out) + (size_t)row * ep.ldo + col) = val;
                }
            }
            __syncthreads();
        }
}

// the kernel addresses its operands with 32-bit byte offsets
static bool gemm8p_fits(int M, int lda, int N, int ldw) {
    return (size_t)M * lda * 2 < (1ull << 32) && (size_t)N * ldw * 2 < (1ull << 32);
}

template <int EPI>
static hipError_t launch_gemm8p(const void* A, int lda, const void* W, int ldw, int M, int N, int K, const GemmEpi& ep,
                                hipStream_t stream) {
    const int split = EPI == EPI_PARTIAL ? ep.split_k : 1;
    if (N % 256 != 0 || (K / split) % 128 != 0 || K % split != 0 || !gemm8p_fits(M, lda, N, ldw))
        return hipErrorInvalidValue;
    const size_t lds = 8 * 16384;  // >= the 128 x (128 x 4 + 16) B staged fp32 epilogue quadrant
    static std::atomic<uint64_t> attr_set{0};  // per device
    if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(&gemm8p_kernel<EPI>), (int)lds); e != hipSuccess)
        return e;
    g_tile_count[3][3].fetch_add(1, std::memory_order_relaxed);
    const int tiles = ((M + 255) / 256) * (N / 256) * split;
    hipLaunchKernelGGL(gemm8p_kernel<EPI>, dim3(tiles), dim3(512), lds, stream, reinterpret_cast<const bf16_t*>(A), lda,
                       reinterpret_cast<const bf16_t*>(W), ldw, M, N, K, ep);
    return hipGetLastError();
}


template <int BM, int BN, int WM, int WN, int STAGES, int EPI, int IN, int MODE = 0>
static hipError_t launch_gemm_cfg(const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                  const GemmEpi& ep, hipStream_t stream) {
    g_tile_count[BM <= 32 ? 0 : BM <= 64 ? 1 : BM <= 128 ? 2 : 3][BN <= 64 ? 0 : BN <= 96 ? 1 : BN <= 128 ? 2 : 3]
        .fetch_add(1, std::memory_order_relaxed);
    const int tiles = ((M + BM - 1) / BM) * (N / BN) * (EPI == EPI_PARTIAL ? ep.split_k : 1);
    size_t lds = (size_t)STAGES * (BM + BN) * GEMM_BK * 2;  // 128-B rows for both input types
    const size_t stage_out = (size_t)BM * (BN * (EPI == EPI_PARTIAL ? 4 : 2) + 16);  // LDS-staged epilogue
    if (EPI != EPI_ARGMAX && EPI != EPI_F32 && stage_out > lds) lds = stage_out;
    static std::atomic<uint64_t> attr_set{0};  // > 64 KiB of dynamic LDS: opted into once per kernel and device
    if (hipError_t e = lds_opt_in(attr_set, reinterpret_cast<const void*>(&gemm_tn_kernel<BM, BN, WM, WN, STAGES, EPI, IN, MODE>),
                                  (int)lds); e != hipSuccess)
        return e;
    hipLaunchKernelGGL((gemm_tn_kernel<BM, BN, WM, WN, STAGES, EPI, IN, MODE>), dim3(tiles), dim3(64 * WM * WN), lds, stream, A,
                       lda, W,
                       ldw, M, N, K, ep);
    return hipGetLastError();
}

// Tile selection, fit to the COLD-weight graph-replay sweep (profiles/r1_gemm_tile_sweep_cold.jsonl:
// weights rotated over >= 768 MB so they stream from HBM as in the 12-layer decode step; an
// L2-hot sweep favours shallow rings and misled an earlier version).  Decode GEMMs below ~400
// 64x64 workgroups are latency-bound on the K loop: keep 4-6 stages of LDS-DMA in flight; above
// that, occupancy hides latency better than ring depth (2 stages, two workgroups per CU).  The LM
// head (N = vocab) and prefill grids amortise 128x128 tiles.  8-wave variants stay tuning-only.
static int g_force_tile = -1;
static bool gemm96_on() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("DLMS_GEMM96");
        v = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    return v == 1;
}  // tuning override (dlms_gemm_force_tile), -1 = heuristic
template <int EPI, int IN>
static hipError_t launch_forced(int id, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                const GemmEpi& ep, hipStream_t stream, bool* done) {
    *done = true;
    switch (id) {
        case 0: return launch_gemm_cfg<32, 64, 2, 2, 6, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        case 1: return launch_gemm_cfg<64, 64, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        case 2: return launch_gemm_cfg<128, 64, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        case 4: return launch_gemm_cfg<64, 64, 2, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        case 7: return launch_gemm_cfg<64, 64, 2, 2, 6, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        default: break;
    }
    if (N % 128 == 0) {
        switch (id) {
            case 3: return launch_gemm_cfg<128, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 5: return launch_gemm_cfg<64, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 6: return launch_gemm_cfg<128, 128, 2, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            // 8-wave workgroups: two waves per SIMD, one's LDS reads under the other's MFMAs
            case 8: return launch_gemm_cfg<256, 128, 4, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 10: return launch_gemm_cfg<128, 128, 4, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 11: return launch_gemm_cfg<128, 128, 2, 4, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            // big per-wave tiles (128x64 per wave): more MFMA work per LDS byte read (64x64 wave
            // tiles sit exactly at the CU's LDS-bandwidth : MFMA-rate balance)
            case 12: return launch_gemm_cfg<256, 128, 2, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 13: return launch_gemm_cfg<256, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            // few-row LM head: 32-row A tiles (a 64-row tile at batch 1 fills a third of every
            // ring stage with clamped copies of the same row)
            case 15: return launch_gemm_cfg<32, 128, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 16: return launch_gemm_cfg<32, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            default: break;
        }
    }
    // 64x96 tiles (waves 32x48): decode row halves (M 512) get one round of <= 256 workgroups on the
    // GPT-2 widths (N 2304 -> 192 tiles, N 3072 -> 256), so no CU streams two tiles' operands
    if (N % 96 == 0) {
        switch (id) {
            case 17: return launch_gemm_cfg<64, 96, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 18: return launch_gemm_cfg<64, 96, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            case 19: return launch_gemm_cfg<64, 96, 2, 2, 6, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
            default: break;
        }
    }
    if (N % 256 == 0 && id == 9) return launch_gemm_cfg<128, 256, 2, 4, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    // 256x256, 8 waves of 128x64 (the cdna guide's big-tile geometry, on this kernel's 1-barrier loop)
    // (not for the fp32 split-K epilogue: its 256 x 1 KiB staged rows exceed the LDS)
    if (N % 256 == 0 && id == 14 && EPI != EPI_PARTIAL)
        return launch_gemm_cfg<256, 256, 2, 4, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    // the big-GEMM modes on 128x128 tiles (the prefill default; REGPF = 1, GROUPED = 2, both = 3) for
    // the forced-tile tests: 24 = both, 25 = GROUPED.  (Round 4's 256x256 / 256x128 mode variants and
    // the one-row-tile LM heads, all measured slower, were removed: profiles/r4_prefill_gemm_modes.jsonl,
    // r4_lmhead_tiles_m512.jsonl.)
    if constexpr (IN == IN_BF16 && (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_QKV || EPI == EPI_PARTIAL)) {
        if (id == 26 && N % 256 == 0 && (K / (EPI == EPI_PARTIAL ? ep.split_k : 1)) % 128 == 0 &&
            gemm8p_fits(M, lda, N, ldw))
            return launch_gemm8p<EPI>(A, lda, W, ldw, M, N, K, ep, stream);
    }
    if constexpr (IN == IN_BF16) {
        if (N % 128 == 0) {
            switch (id) {
                case 24: return launch_gemm_cfg<128, 128, 2, 2, 2, EPI, IN, 3>(A, lda, W, ldw, M, N, K, ep, stream);
                case 25: return launch_gemm_cfg<128, 128, 2, 2, 2, EPI, IN, 2>(A, lda, W, ldw, M, N, K, ep, stream);
                default: break;
            }
        }
    }
    *done = false;
    return hipSuccess;
}

template <int EPI, int IN>
static hipError_t launch_gemm_epi(const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                  const GemmEpi& ep, hipStream_t stream) {
    const int split = EPI == EPI_PARTIAL ? ep.split_k : 1;
    if (g_force_tile >= 0) {
        bool done = false;
        hipError_t e = launch_forced<EPI, IN>(g_force_tile, A, lda, W, ldw, M, N, K, ep, stream, &done);
        if (done) return e;
    }
    const long t64 = (long)((M + 63) / 64) * (N / 64) * split;
    const long t128 = (long)((M + 127) / 128) * (N / 128) * split;
    // big prefill GEMMs (1024 prompts x 32 tokens = 32768 rows): 128x128 tiles with a whole K-tile
    // of fragments in registers (the DMA two K-tiles ahead) and tiles in groups of 4 row tiles (the
    // 32 workgroups an XCD runs at once share their A and W panels in its L2); two workgroups per
    // CU, so one's epilogue runs under the other's K loop.  profiles/r4_prefill_gemm_modes.jsonl at
    // M = 32768: QKV 180.2 -> 153.5 us (256x256 tiles before), out-projection 82.4 -> 66.1, c_proj
    // 199.6 -> 172.3, c_fc with a plain bf16 epilogue 206.1 -> 199.4 (hipBLASLt, plain bf16 out:
    // 146.0 / 64.7 / 139.9 / 148.4)
    if constexpr (IN == IN_BF16 && (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_QKV || EPI == EPI_PARTIAL)) {
        // ... and on 256x256 tiles with the 8-phase K loop where that is faster (bit-identical
        // results): QKV 179.7 -> 155.2 us, c_fc (plain epilogue) 191.4 -> 173.0, c_proj 170.1 ->
        // 154.5; the out-projection (K = 768, 384 tiles: 1.5 rounds of workgroups) keeps the 128x128
        // tiles, 60.0 vs 62.3 (profiles/r5_prefill_gemm_8phase.jsonl).  The engine splits the prefill
        // c_proj 2 ways (K slices of 1536: three full rounds of 256 workgroups)
        // In the bench: prefill 11.2-11.9 -> 10.5-11.2 ms per 1024-query generation
        // (profiles/r5_prefill_8phase_ab.jsonl)
        const int kc = K / split;
        if (M >= 16384 && N % 256 == 0 && kc % 128 == 0 && (EPI != EPI_PARTIAL || kc >= 1536) &&
            gemm8p_fits(M, lda, N, ldw))
            return launch_gemm8p<EPI>(A, lda, W, ldw, M, N, K, ep, stream);
    }
    if constexpr (IN == IN_BF16 && (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF ||
                                    EPI == EPI_QKV || EPI == EPI_PARTIAL)) {
        // (only at the measured size class: 1024-prompt packed prefills; smaller admissions keep the
        // tiles below, e.g. a 4096-row out-projection would put 192 128x128 tiles on 256 CUs)
        if (M >= 16384 && N % 128 == 0)
            return launch_gemm_cfg<128, 128, 2, 2, 2, EPI, IN, 3>(A, lda, W, ldw, M, N, K, ep, stream);
    }
    // big prefill GEMMs with a bf16 epilogue: 256x256 tiles, 8 waves of 128x64 (one workgroup per
    // CU: its 128 KiB ring + 135 KiB staged epilogue), unless the last round of tiles would run
    // nearly empty (profiles/r1_gemm_256tile.jsonl: c_fc M=32768 247 -> 192 us, QKV 184 -> 154 us;
    // QKV at M=8192 = 288 tiles loses 6 %)
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF || EPI == EPI_QKV) {
        const long t256 = (long)((M + 255) / 256) * (N / 256);
        if (N % 256 == 0 && M >= 4096 && (t256 <= 256 || t256 % 256 >= 128 || t256 >= 512)) {
            return launch_gemm_cfg<256, 256, 2, 4, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
        }
    }
    // (LM head on a 512-row decode half: 256x256 tiles are 86.4 -> 78.3 us alone (N = 50432,
    // profiles/r1_gemm_256tile.jsonl) but 1 % slower in the two-stream decode step, where the
    // one-workgroup-per-CU tile starves the other half's kernels: profiles/r1_lmhead_256_ab.log)
    // decode GEMMs of the wider models (K = d >= 1024: GPT-2-medium/large/XL QKV and c_fc on 256-512
    // row halves): 128x64 tiles with a 3-deep ring while they fit in one round of workgroups
    // (profiles/r1_gemm_wide_models.jsonl: medium M=512 c_fc 15.0 -> 11.6 us, XL M=256 QKV 17.3 ->
    // 15.6 us / c_fc 17.8 -> 15.8 us; at 300-400 tiles 64x64 wins again)
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_GELU_ERF || EPI == EPI_QKV) {
        const long t128x64 = (long)((M + 127) / 128) * (N / 64);
        if (K >= 1024 && M >= 256 && t128x64 <= 256)
            return launch_gemm_cfg<128, 64, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    }
    // decode row halves of the overlapped step (256 < M <= 512, K = 768 / 3072): 64x96 tiles in ONE
    // round of <= 256 workgroups -- QKV 192, c_fc 256, c_proj split 4 -> 256 -- so no CU streams two
    // tiles' operands (profiles/r3_kern_sweep_m512.jsonl: QKV 9.7 -> 8.5 us, c_fc 10.2 -> 8.7 us,
    // c_proj split-2 10.5 -> split-4 8.5 us); DLMS_GEMM96=0 turns it off (A/B)
    if (gemm96_on() && N % 96 == 0 && M > 256 && M <= 512 && N != 768 &&
        (EPI == EPI_BF16 || EPI == EPI_GELU_TANH || EPI == EPI_QKV ||
         (EPI == EPI_PARTIAL && split == 4)) &&
        (long)((M + 63) / 64) * (N / 96) * split <= 256)
        return launch_gemm_cfg<64, 96, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    if (EPI == EPI_PARTIAL && gemm96_on() && N == 768 && split == 4 && M > 256 && M <= 512 && K >= 2048)
        return launch_gemm_cfg<64, 96, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    if (N % 128 == 0 && (t128 >= 1024 || (N >= 8192 && M >= 256)))
        return launch_gemm_cfg<128, 128, 2, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    // few-row LM head (latency path, B <= 32): 32-row A tiles, so clamped copies of the few real rows
    // take a fifth of each ring stage instead of a third (batch 1: 34.86 -> 34.46 ms per query,
    // profiles/r2_lm_head_tiles_b1.txt)
    if (EPI == EPI_ARGMAX && M <= 32 && N % 128 == 0 && N >= 8192)
        return launch_gemm_cfg<32, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    if (N % 128 == 0 && N >= 8192) return launch_gemm_cfg<64, 128, 2, 2, 3, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    if (M <= 64) return launch_gemm_cfg<32, 64, 2, 2, 6, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    if (t64 <= 400) return launch_gemm_cfg<64, 64, 2, 2, 4, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
    return launch_gemm_cfg<64, 64, 2, 2, 2, EPI, IN>(A, lda, W, ldw, M, N, K, ep, stream);
}

extern "C" void dlms_gemm_force_tile(int id) { g_force_tile = id; }
// launches issued so far with a BM x BN tile (BM in 32/64/128/256, BN in 64/96/128/256); reset: -1, -1
extern "C" long dlms_gemm_tile_count(int bm, int bn) {
    const int BMS[4] = {32, 64, 128, 256}, BNS[4] = {64, 96, 128, 256};
    if (bm < 0) {
        for (auto& row : g_tile_count)
            for (auto& c : row) c.store(0);
        return 0;
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            if (BMS[i] == bm && BNS[j] == bn) return g_tile_count[i][j].load();
    return -1;
}

extern "C" hipError_t dlms_gemm(int epi, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                const GemmEpi* ep, hipStream_t stream) {
    if (K % GEMM_BK != 0 || N % 64 != 0 || M <= 0) return hipErrorInvalidValue;
    if (epi == EPI_PARTIAL && (ep->split_k < 1 || K % (ep->split_k * GEMM_BK) != 0)) return hipErrorInvalidValue;
    switch (epi) {
        case EPI_BF16: return launch_gemm_epi<EPI_BF16, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_GELU_TANH: return launch_gemm_epi<EPI_GELU_TANH, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_GELU_ERF: return launch_gemm_epi<EPI_GELU_ERF, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_F32: return launch_gemm_epi<EPI_F32, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_QKV: return launch_gemm_epi<EPI_QKV, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_ARGMAX: return launch_gemm_epi<EPI_ARGMAX, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_PARTIAL: return launch_gemm_epi<EPI_PARTIAL, IN_BF16>(A, lda, W, ldw, M, N, K, *ep, stream);
        default: return hipErrorInvalidValue;
    }
}

// W8A8 fp8 (OCP e4m3) GEMM: A [M][K] and W [N][K] e4m3, ep->a_scale[M] / ep->w_scale[N] fp32.
// The decode path uses it for the GEMMs fed by a LayerNorm (QKV, c_fc, LM head), whose
// producer emits the row-scaled fp8 activation directly.
extern "C" hipError_t dlms_gemm_fp8(int epi, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                                    const GemmEpi* ep, hipStream_t stream) {
    if (K % (2 * GEMM_BK) != 0 || N % 64 != 0 || M <= 0 || !ep->a_scale || !ep->w_scale) return hipErrorInvalidValue;
    if (epi == EPI_PARTIAL && (ep->split_k < 1 || K % (ep->split_k * 2 * GEMM_BK) != 0)) return hipErrorInvalidValue;
    switch (epi) {
        case EPI_BF16: return launch_gemm_epi<EPI_BF16, IN_FP8>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_GELU_TANH: return launch_gemm_epi<EPI_GELU_TANH, IN_FP8>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_QKV: return launch_gemm_epi<EPI_QKV, IN_FP8>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_ARGMAX: return launch_gemm_epi<EPI_ARGMAX, IN_FP8>(A, lda, W, ldw, M, N, K, *ep, stream);
        case EPI_PARTIAL: return launch_gemm_epi<EPI_PARTIAL, IN_FP8>(A, lda, W, ldw, M, N, K, *ep, stream);
        default: return hipErrorInvalidValue;
    }
}

DLMS_CHECK_EXPORT(gemm)
