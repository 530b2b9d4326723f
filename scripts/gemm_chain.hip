// Persistent GEMM-chain prototype: one 512-row half-layer of GPT-2-124M --
//   out-projection (x += attn Wo^T + bo) -> LN2 -> c_fc + GELU -> c_proj (x += h Wp^T + bp) -> LN1'
// as ONE persistent kernel with row-block hand-offs, against the same work as five launches.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I distributed_lms_raft_llm_amd/ops/csrc \
//         scripts/gemm_chain.hip -o scripts/gemm_chain && ./scripts/gemm_chain
//
// Design (MI355X-first, no split-K seams):
//   * work is a list of jobs in dependency order: OUT tiles (64x96), LN row groups (8 rows), FC tiles
//     (64x96, GELU), PROJ tiles (64x32 -- K = 3072 without a split), LN' row groups.  Each job of
//     row block r (64 rows) only waits for jobs of the same row block in the previous phase, so
//     the FC tiles of row block 0 run while the out-projection of row block 7 is still in flight.
//   * workgroups take jobs from one atomic ticket, in order: a job only waits for lower tickets
//     that resident workgroups already hold, so the grid needs no co-residency (a workgroup that
//     is scheduled late simply takes a later job) and every wave reaches the exit (ticket >= jobs).
//     Waits are bounded: a timeout writes an error word and the job is skipped.
//   * completion: one counter per (phase, row block), bumped once per finished job.
//     SYNC 0: plain stores, agent-scope release fence before the bump, acquire fence after the wait.
//     SYNC 1: the chain's intermediates (x, ln, h) are written and read coherently at agent scope
//     (relaxed atomic stores / loads, and sc1 LDS-DMA loads for the GEMM A operand), so the
//     hand-off needs no L2 write-back or invalidate -- only the store counter drain.
// The tile main loop is the production 3-stage LDS-DMA ring of gemm.hip (gemm_tn_kernel), as a
// device function.  Times both variants alone and beside a streaming kernel on a second stream (the
// other half's attention in the overlapped throughput step).  Prints one JSON line per variant.
#include "gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <unistd.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

#ifndef CH_PBM
#define CH_PBM 64  // rows of a c_proj tile (64: 64x32 tiles, 32: 32x32 tiles; K = 3072 unsplit either way)
#endif
constexpr int CH_M = 512, CH_D = 768, CH_F = 3072, CH_RB = CH_M / 64;
constexpr int N_OUT = CH_RB * (CH_D / 96), N_LN = CH_RB * 8, N_FC = CH_RB * (CH_F / 96),
              N_PROJ_RB = (64 / CH_PBM) * (CH_D / 32), N_PROJ = CH_RB * N_PROJ_RB, N_LN2 = CH_RB * 8;
constexpr int N_JOBS = N_OUT + N_LN + N_FC + N_PROJ + N_LN2;
constexpr int CH_THREADS = 256, CH_STAGES = 3;
constexpr int CH_LDS = CH_STAGES * (64 + 96) * GEMM_BK * 2;  // 60 KiB: two workgroups per CU
constexpr int AUX_SC1 = 16;                                  // cache-policy bit sc1 of a global load
constexpr int AUX_SC0 = 1;                                   // sc0: miss the CU's L1, hit the XCD's L2

struct ChainArgs {
    const bf16_t* attn;  // [M][D] attention output (chain input)
    const bf16_t* Wo;    // [D][D] (N x K, K contiguous)
    const float* bo;
    float* x;  // [M][D] f32 residual stream, updated in place
    const float *g2, *b2, *g1, *b1;
    bf16_t* ln;  // [M][D] LN2(x) -> c_fc input
    const bf16_t* Wfc;
    const float* bfc;
    bf16_t* h;  // [M][F] GELU(c_fc)
    const bf16_t* Wp;
    const float* bp;
    bf16_t* ln_next;  // [M][D] LN1 of the next layer (chain output)
    int* cnt;         // [5][RB]
    int* ticket;
    int* err;
    int* dbg;  // [N_JOBS] host-visible job state (1 started, 2 math done, 3 published)
};

__device__ __forceinline__ void dbg_mark(const ChainArgs& a, int j, int v) {
    if (threadIdx.x == 0) __hip_atomic_store(a.dbg + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int SYNC>
__device__ __forceinline__ float ld_f32(const float* p) {
    if constexpr (SYNC == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}
template <int SYNC>
__device__ __forceinline__ void st_f32(float* p, float v) {
    if constexpr (SYNC == 1)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}
template <int SYNC>
__device__ __forceinline__ void st_bf16(bf16_t* p, float v) {
    if constexpr (SYNC == 1)
        __hip_atomic_store(p, f32_to_bf16(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = f32_to_bf16(v);
}

// The 3-stage LDS-DMA ring main loop of gemm_tn_kernel (bf16, no split), one BM x BN tile.
template <int BM, int BN, int WM, int WN, int AUX>
__device__ __forceinline__ void tile_mma(const bf16_t* A, int lda, const bf16_t* W, int ldw, int m0, int n0, int K,
                                         char* smem, f32x4_t (&acc)[BM / WM / 16][BN / WN / 16]) {
    constexpr int NW = WM * WN, WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    static_assert(NW * 64 == CH_THREADS, "4 waves");
    constexpr int ROWB = GEMM_BK * 2, A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;
    constexpr int PPW = STAGE_BYTES / 1024 / NW;
    static_assert((STAGE_BYTES / 1024) % NW == 0, "pieces per wave");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
    const char* src[PPW];
    bool is_a[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int piece = wave + NW * i, row = piece * 8 + (lane >> 3), lchunk = (lane & 7) ^ (lane >> 3);
        is_a[i] = row < BM;
        src[i] = row < BM ? reinterpret_cast<const char*>(A) + (size_t)(m0 + row) * lda * 2 + lchunk * 16
                          : reinterpret_cast<const char*>(W) + (size_t)(n0 + row - BM) * ldw * 2 + lchunk * 16;
    }
    auto issue = [&](int stage, int k0) {
        char* dst = smem + stage * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            if (is_a[i])
                __builtin_amdgcn_global_load_lds((glob_void_t*)(src[i] + (size_t)k0 * 2),
                                                 (lds_void_t*)(dst + (wave + NW * i) * 1024), 16, 0, AUX);
            else
                __builtin_amdgcn_global_load_lds((glob_void_t*)(src[i] + (size_t)k0 * 2),
                                                 (lds_void_t*)(dst + (wave + NW * i) * 1024), 16, 0, 0);
        }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int nk = K / GEMM_BK, frow = lane & 15, fk = lane >> 4, fsw = lane & 7;
#pragma unroll
    for (int s = 0; s < CH_STAGES - 1; ++s)
        if (s < nk) issue(s, s * GEMM_BK);
    for (int kt = 0; kt < nk; ++kt) {
        if (nk - kt >= CH_STAGES - 1)
            wait_vmcnt<(CH_STAGES - 2) * PPW>();
        else
            wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        {
            const int kn = kt + CH_STAGES - 1;
            if (kn < nk) issue(kn % CH_STAGES, kn * GEMM_BK);
        }
        const char* as = smem + (kt % CH_STAGES) * STAGE_BYTES + (wm * WTM) * ROWB;
        const char* ws = smem + (kt % CH_STAGES) * STAGE_BYTES + A_BYTES + (wn * WTN) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = (((ks * 4 + fk) ^ fsw) << 4);
            bf16x8_t af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frow) * ROWB + coff);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frow) * ROWB + coff);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    wait_vmcnt<0>();
}

typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// 16-B / 8-B accesses to the chain's intermediates: SYNC 1 = sc1 (agent-coherent) buffer ops
template <int SYNC>
__device__ __forceinline__ u32x4_t ld16(const void* base, unsigned off) {
    if constexpr (SYNC == 1) return __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(base), off, 0, AUX_SC1);
    if constexpr (SYNC == 2) return __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(base), off, 0, AUX_SC0);
    return *reinterpret_cast<const u32x4_t*>(reinterpret_cast<const char*>(base) + off);
}
template <int SYNC>
__device__ __forceinline__ void st16(void* base, unsigned off, u32x4_t v) {
    if constexpr (SYNC == 1)
        __builtin_amdgcn_raw_buffer_store_b128(v, buf_rsrc(base), off, 0, AUX_SC1);
    else
        *reinterpret_cast<u32x4_t*>(reinterpret_cast<char*>(base) + off) = v;
}
template <int SYNC>
__device__ __forceinline__ void st8(void* base, unsigned off, u32x2_t v) {
    if constexpr (SYNC == 1)
        __builtin_amdgcn_raw_buffer_store_b64(v, buf_rsrc(base), off, 0, AUX_SC1);
    else
        *reinterpret_cast<u32x2_t*>(reinterpret_cast<char*>(base) + off) = v;
}

// x[tile] += acc + bias (f32, in place): the tile is staged through LDS so x moves in 16-B pieces,
// all old values loaded before any store (one round trip)
template <int BM, int BN, int WM, int WN, int SYNC>
__device__ __forceinline__ void epi_add(f32x4_t (&acc)[BM / WM / 16][BN / WN / 16], float* x, const float* bias,
                                        int m0, int n0, char* smem) {
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16, SROW = BN + 4;
    constexpr int CPR = BN / 4, PER = BM * CPR / CH_THREADS;
    static_assert(BM * CPR % CH_THREADS == 0, "chunks per thread");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
    const int lr0 = wm * WTM + (lane >> 4) * 4, lc0 = wn * WTN + (lane & 15);
    float* t = reinterpret_cast<float*>(smem);
    u32x4_t old[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int c = tid + q * CH_THREADS, lr = c / CPR, ch = c - lr * CPR;
        old[q] = ld16<SYNC>(x, ((m0 + lr) * CH_D + n0 + ch * 4) * 4);
    }
    __syncthreads();  // every wave is done reading the ring
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const float bv = bias[n0 + lc0 + j * 16];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) t[(lr0 + i * 16 + r) * SROW + lc0 + j * 16] = acc[i][j][r] + bv;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int c = tid + q * CH_THREADS, lr = c / CPR, ch = c - lr * CPR;
        const f32x4_t d = *reinterpret_cast<const f32x4_t*>(t + lr * SROW + ch * 4);
        f32x4_t o = __builtin_bit_cast(f32x4_t, old[q]);
        o += d;
        st16<SYNC>(x, ((m0 + lr) * CH_D + n0 + ch * 4) * 4, __builtin_bit_cast(u32x4_t, o));
    }
}

// h[tile] = bf16(GELU(acc + bias)), staged through LDS into 16-B row pieces
template <int BM, int BN, int WM, int WN, int SYNC>
__device__ __forceinline__ void epi_gelu(f32x4_t (&acc)[BM / WM / 16][BN / WN / 16], bf16_t* out, int ldo,
                                         const float* bias, int m0, int n0, char* smem) {
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16, SROWB = BN * 2 + 16;
    constexpr int CPR = BN * 2 / 16, PER = BM * CPR / CH_THREADS;
    static_assert(BM * CPR % CH_THREADS == 0, "chunks per thread");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
    const int lr0 = wm * WTM + (lane >> 4) * 4, lc0 = wn * WTN + (lane & 15);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const float bv = bias[n0 + lc0 + j * 16];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                *reinterpret_cast<bf16_t*>(smem + (lr0 + i * 16 + r) * SROWB + (lc0 + j * 16) * 2) =
                    f32_to_bf16(gelu_tanh(acc[i][j][r] + bv));
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int c = tid + q * CH_THREADS, lr = c / CPR, ch = c - lr * CPR;
        st16<SYNC>(out, ((m0 + lr) * ldo + n0 + ch * 8) * 2, *reinterpret_cast<const u32x4_t*>(smem + lr * SROWB + ch * 16));
    }
}

// LayerNorm of 8 rows of x (768 f32) -> bf16, two rows per wave, 3 x 16 B per lane
template <int SYNC>
__device__ __forceinline__ void ln_rows(const float* x, const float* g, const float* b, bf16_t* out, int row0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x4_t v[2][3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int i = 0; i < 3; ++i)
            v[rr][i] = __builtin_bit_cast(f32x4_t, ld16<SYNC>(x, ((row0 + wave * 2 + rr) * CH_D + i * 256 + lane * 4) * 4));
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int row = row0 + wave * 2 + rr;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) s += v[rr][i][0] + v[rr][i][1] + v[rr][i][2] + v[rr][i][3];
        const float mu = wave_sum(s) * (1.f / CH_D);
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) q += (v[rr][i][e] - mu) * (v[rr][i][e] - mu);
        const float rstd = rsqrtf(wave_sum(q) * (1.f / CH_D) + 1e-5f);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int c = i * 256 + lane * 4;
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (v[rr][i][e] - mu) * rstd * g[c + e] + b[c + e];
            st8<SYNC>(out, (row * CH_D + c) * 2, (u32x2_t){pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
        }
    }
}

template <int SYNC>
__device__ __forceinline__ bool wait_count(const ChainArgs& a, const int* p, int target) {
    __shared__ int ok;
    if (threadIdx.x == 0) {
        int it = 0;
        while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && it < (1 << 16)) {
            __builtin_amdgcn_s_sleep(2);
            ++it;
        }
        ok = it < (1 << 16);
        if (!ok) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if constexpr (SYNC == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return __builtin_amdgcn_readfirstlane(ok);
}

template <int SYNC>
__device__ __forceinline__ void publish(int* p) {
    if constexpr (SYNC == 0)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's coherent stores have completed
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// WAIT = false: the per-phase launches (stream order is the dependency).
template <int SYNC, bool WAIT>
__device__ void run_job(const ChainArgs& a, int j, char* smem) {
    constexpr int AUX = SYNC == 1 ? AUX_SC1 : SYNC == 2 ? AUX_SC0 : 0;
    __syncthreads();  // the previous job's LDS reads are done
    if (j < N_OUT) {
        const int r = j / (CH_D / 96), c = j % (CH_D / 96);
        f32x4_t acc[2][3];
        tile_mma<64, 96, 2, 2, 0>(a.attn, CH_D, a.Wo, CH_D, r * 64, c * 96, CH_D, smem, acc);
        epi_add<64, 96, 2, 2, SYNC>(acc, a.x, a.bo, r * 64, c * 96, smem);
        if (WAIT) dbg_mark(a, j, 2);
        if (WAIT) publish<SYNC>(a.cnt + 0 * CH_RB + r);
        return;
    }
    j -= N_OUT;
    if (j < N_LN) {
        const int r = j / 8, s = j % 8;
        if (WAIT && !wait_count<SYNC>(a, a.cnt + 0 * CH_RB + r, CH_D / 96)) return;
        ln_rows<SYNC>(a.x, a.g2, a.b2, a.ln, r * 64 + s * 8);
        if (WAIT) publish<SYNC>(a.cnt + 1 * CH_RB + r);
        return;
    }
    j -= N_LN;
    if (j < N_FC) {
        const int r = j / (CH_F / 96), c = j % (CH_F / 96);
        if (WAIT && !wait_count<SYNC>(a, a.cnt + 1 * CH_RB + r, 8)) return;
        f32x4_t acc[2][3];
        tile_mma<64, 96, 2, 2, AUX>(a.ln, CH_D, a.Wfc, CH_D, r * 64, c * 96, CH_D, smem, acc);
        epi_gelu<64, 96, 2, 2, SYNC>(acc, a.h, CH_F, a.bfc, r * 64, c * 96, smem);
        if (WAIT) publish<SYNC>(a.cnt + 2 * CH_RB + r);
        return;
    }
    j -= N_FC;
    if (j < N_PROJ) {
        const int r = j / N_PROJ_RB, k = j % N_PROJ_RB, m0 = r * 64 + (k / (CH_D / 32)) * CH_PBM, c = k % (CH_D / 32);
        if (WAIT && !wait_count<SYNC>(a, a.cnt + 2 * CH_RB + r, CH_F / 96)) return;
        constexpr int PWM = CH_PBM == 64 ? 4 : 2, PWN = 4 / PWM;
        f32x4_t acc[CH_PBM / PWM / 16][32 / PWN / 16];
        tile_mma<CH_PBM, 32, PWM, PWN, AUX>(a.h, CH_F, a.Wp, CH_F, m0, c * 32, CH_F, smem, acc);
        epi_add<CH_PBM, 32, PWM, PWN, SYNC>(acc, a.x, a.bp, m0, c * 32, smem);
        if (WAIT) publish<SYNC>(a.cnt + 3 * CH_RB + r);
        return;
    }
    j -= N_PROJ;
    {
        const int r = j / 8, s = j % 8;
        if (WAIT && !wait_count<SYNC>(a, a.cnt + 3 * CH_RB + r, N_PROJ_RB)) return;
        ln_rows<SYNC>(a.x, a.g1, a.b1, a.ln_next, r * 64 + s * 8);
    }
}

// ticket -> job: ORDER 0 phase-major, ORDER 1 row-block-major (all five phases of row block 0, then 1, ...)
template <int ORDER>
__device__ __forceinline__ int job_of(int t) {
    if constexpr (ORDER == 0) return t;
    constexpr int PER_RB = N_JOBS / CH_RB, O = CH_D / 96, L = 8, F = CH_F / 96, P = N_PROJ_RB;
    const int r = t / PER_RB, k = t - r * PER_RB;
    if (k < O) return r * O + k;
    if (k < O + L) return N_OUT + r * L + (k - O);
    if (k < O + L + F) return N_OUT + N_LN + r * F + (k - O - L);
    if (k < O + L + F + P) return N_OUT + N_LN + N_FC + r * P + (k - O - L - F);
    return N_OUT + N_LN + N_FC + N_PROJ + r * L + (k - O - L - F - P);
}

template <int SYNC, int ORDER>
__global__ __launch_bounds__(CH_THREADS) void chain_persistent(ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int job;
    for (;;) {
        if (threadIdx.x == 0) job = __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        // readfirstlane: the job id is wave-uniform in the compiler's eyes (scalar branches)
        const int j = __builtin_amdgcn_readfirstlane(job);
        __syncthreads();
        if (j >= N_JOBS) return;  // every workgroup reaches this once the tickets run out
        dbg_mark(a, job_of<ORDER>(j), 1);
        run_job<SYNC, true>(a, job_of<ORDER>(j), smem);
        dbg_mark(a, job_of<ORDER>(j), 3);
        // a barrier between this job's thread-0 regions (publish, mark) and the next ticket fetch:
        // without it the compiler merges them across the loop back-edge into one lane-divergent
        // region, and the structurized loop parks lane 0 while the wave's other lanes re-enter the
        // job (the first runs of this prototype hung exactly so: every job published, no second
        // ticket ever taken)
        __syncthreads();
    }
}

// XCD-local chain: row block r runs entirely on XCD r (workgroups are dispatched round-robin over
// the 8 XCDs, so blockIdx.x % 8 is the XCD), so every hand-off stays inside one XCD's L2 -- the
// producer's plain stores land in that L2 and the consumer reads with sc0 (missing only its own
// CU's L1): no write-back, no invalidate, no L2 bypass.  One ticket per XCD.
__global__ __launch_bounds__(CH_THREADS) void chain_xcd(ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int job;
    constexpr int PER_RB = N_JOBS / CH_RB;
    const int xcd = blockIdx.x % 8;
    for (;;) {
        if (threadIdx.x == 0)
            job = __hip_atomic_fetch_add(a.ticket + 2 + xcd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(job);
        __syncthreads();
        if (t >= PER_RB) return;
        run_job<2, true>(a, job_of<1>(xcd * PER_RB + t), smem);
        dbg_mark(a, job_of<1>(xcd * PER_RB + t), 3);
        __syncthreads();  // see chain_persistent
    }
}

// Column-local coherent chain: XCD x owns the column tiles c with c % 8 == x in every phase (the
// launch-per-phase schedule's weight locality: each weight byte is pulled into one L2), and the
// activations cross XCDs coherently (sc1, as chain_persistent<1>).  Per-XCD queue, phase-major:
// OUT (1 per row block), LN (1), FC (4), PROJ (3 per 24 column tiles), LN' (1).  Every job waits
// only on jobs of earlier phases, all of which are within the first 64 tickets of their XCD's queue
// (64 workgroups per XCD), so the queues cannot block each other.
__device__ __forceinline__ int collocal_job(int xcd, int t) {
    constexpr int O = CH_D / 96, L = 8, F = CH_F / 96, P = N_PROJ_RB;
    constexpr int nO = CH_RB * O / 8, nL = CH_RB * L / 8, nF = CH_RB * F / 8, nP = CH_RB * P / 8;
    if (t < nO) return (t / (O / 8)) * O + xcd + 8 * (t % (O / 8));
    t -= nO;
    if (t < nL) return N_OUT + (t / (L / 8)) * L + xcd + 8 * (t % (L / 8));
    t -= nL;
    if (t < nF) return N_OUT + N_LN + (t / (F / 8)) * F + xcd + 8 * (t % (F / 8));
    t -= nF;
    if (t < nP) return N_OUT + N_LN + N_FC + (t / (P / 8)) * P + xcd + 8 * (t % (P / 8));
    t -= nP;
    return N_OUT + N_LN + N_FC + N_PROJ + (t / (L / 8)) * L + xcd + 8 * (t % (L / 8));
}

__global__ __launch_bounds__(CH_THREADS) void chain_collocal(ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int job;
    constexpr int PER_XCD = N_JOBS / 8;
    const int xcd = blockIdx.x % 8;
    for (;;) {
        if (threadIdx.x == 0)
            job = __hip_atomic_fetch_add(a.ticket + 2 + xcd, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(job);
        __syncthreads();
        if (t >= PER_XCD) return;
        run_job<1, true>(a, collocal_job(xcd, t), smem);
        dbg_mark(a, collocal_job(xcd, t), 3);
        __syncthreads();  // see chain_persistent
    }
}

__global__ __launch_bounds__(CH_THREADS) void chain_phase(ChainArgs a, int j0) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    run_job<0, false>(a, j0 + blockIdx.x, smem);
}

// a streaming reader on another stream: the other half's attention (reads K/V at HBM rate)
__global__ __launch_bounds__(256) void stream_read(const u32x4_t* p, size_t n, unsigned* sink) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u32x4_t v = __builtin_nontemporal_load(p + i);
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) sink[0] = s;
}

// ---------------- host ----------------
static unsigned g_rng = 12345;
static float frand() {
    g_rng = g_rng * 1664525u + 1013904223u;
    return ((g_rng >> 8) & 0xffff) / 65536.f - 0.5f;
}
static bf16_t h_bf16(float f) {
    unsigned u;
    memcpy(&u, &f, 4);
    u += 0x7fff + ((u >> 16) & 1);
    return (bf16_t)(u >> 16);
}
static float h_f32(bf16_t b) {
    unsigned u = (unsigned)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static float h_gelu(float x) { return 0.5f * x * (1.f + tanhf(0.7978845608f * (x + 0.044715f * x * x * x))); }

template <class T>
static T* dev_upload(const std::vector<T>& v) {
    T* p;
    CK(hipMalloc(&p, v.size() * sizeof(T)));
    CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

static void host_ln(const float* x, const float* g, const float* b, float* out) {
    double s = 0, q = 0;
    for (int c = 0; c < CH_D; ++c) s += x[c];
    const double mu = s / CH_D;
    for (int c = 0; c < CH_D; ++c) q += (x[c] - mu) * (x[c] - mu);
    const double rstd = 1.0 / sqrt(q / CH_D + 1e-5);
    for (int c = 0; c < CH_D; ++c) out[c] = h_f32(h_bf16((float)((x[c] - mu) * rstd * g[c] + b[c])));
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    setvbuf(stdout, nullptr, _IOLBF, 0);
    std::vector<bf16_t> attn(CH_M * CH_D), Wo(CH_D * CH_D), Wfc((size_t)CH_F * CH_D), Wp((size_t)CH_D * CH_F);
    std::vector<float> x0(CH_M * CH_D), bo(CH_D), bfc(CH_F), bp(CH_D), g1(CH_D), b1(CH_D), g2(CH_D), b2(CH_D);
    for (auto& v : attn) v = h_bf16(frand() * 2.f);
    for (auto& v : Wo) v = h_bf16(frand() * 0.08f);
    for (auto& v : Wfc) v = h_bf16(frand() * 0.08f);
    for (auto& v : Wp) v = h_bf16(frand() * 0.04f);
    for (auto& v : x0) v = frand() * 4.f;
    for (auto& v : bo) v = frand() * 0.1f;
    for (auto& v : bfc) v = frand() * 0.1f;
    for (auto& v : bp) v = frand() * 0.1f;
    for (int c = 0; c < CH_D; ++c) g1[c] = 1.f + frand() * 0.2f, b1[c] = frand() * 0.1f, g2[c] = 1.f + frand() * 0.2f,
                             b2[c] = frand() * 0.1f;

    ChainArgs a{};
    a.attn = dev_upload(attn);
    a.Wo = dev_upload(Wo);
    a.Wfc = dev_upload(Wfc);
    a.Wp = dev_upload(Wp);
    a.bo = dev_upload(bo);
    a.bfc = dev_upload(bfc);
    a.bp = dev_upload(bp);
    a.g1 = dev_upload(g1);
    a.b1 = dev_upload(b1);
    a.g2 = dev_upload(g2);
    a.b2 = dev_upload(b2);
    float* x0d = dev_upload(x0);
    CK(hipMalloc(&a.x, x0.size() * 4));
    CK(hipMalloc(&a.ln, (size_t)CH_M * CH_D * 2));
    CK(hipMalloc(&a.h, (size_t)CH_M * CH_F * 2));
    CK(hipMalloc(&a.ln_next, (size_t)CH_M * CH_D * 2));
    int* ctl;  // [5*RB counters][ticket][err]
    CK(hipMalloc(&ctl, (5 * CH_RB + 10) * 4));  // + ticket, err, 8 per-XCD tickets
    a.cnt = ctl;
    a.ticket = ctl + 5 * CH_RB;
    a.err = ctl + 5 * CH_RB + 1;
    CK(hipMalloc(&a.dbg, N_JOBS * 4));
    CK(hipFuncSetAttribute((const void*)chain_persistent<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    CK(hipFuncSetAttribute((const void*)chain_persistent<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    CK(hipFuncSetAttribute((const void*)chain_persistent<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    CK(hipFuncSetAttribute((const void*)chain_phase, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    CK(hipFuncSetAttribute((const void*)chain_xcd, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    CK(hipFuncSetAttribute((const void*)chain_collocal, hipFuncAttributeMaxDynamicSharedMemorySize, CH_LDS));
    int occ0 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, (const void*)chain_persistent<1, 0>, CH_THREADS, CH_LDS));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount * std::max(1, occ0);

    const size_t sbytes = (size_t)512 << 20;  // the streaming kernel's buffer (512 MiB, > MALL)
    u32x4_t* sbuf;
    unsigned* sink;
    CK(hipMalloc(&sbuf, sbytes));
    CK(hipMemset(sbuf, 1, sbytes));
    CK(hipMalloc(&sink, 4));
    hipStream_t s1, s2, s3;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    constexpr int NV = 6;
    const char* names[NV] = {"five_launches", "persistent_fence", "persistent_coherent", "persistent_coherent_rbmajor",
                             "persistent_xcd_local", "persistent_coherent_column_local"};
    auto reset = [&](hipStream_t s) {
        CK(hipMemcpyAsync(a.x, x0d, x0.size() * 4, hipMemcpyDeviceToDevice, s));
        CK(hipMemsetAsync(ctl, 0, (5 * CH_RB + 10) * 4, s));
        CK(hipMemsetAsync(a.dbg, 0, N_JOBS * 4, s));
    };
    auto launch = [&](int variant, hipStream_t s) {
        if (variant == 0) {
            const int starts[6] = {0, N_OUT, N_OUT + N_LN, N_OUT + N_LN + N_FC, N_OUT + N_LN + N_FC + N_PROJ, N_JOBS};
            for (int p = 0; p < 5; ++p)
                chain_phase<<<starts[p + 1] - starts[p], CH_THREADS, CH_LDS, s>>>(a, starts[p]);
        } else if (variant == 1) {
            chain_persistent<0, 0><<<grid, CH_THREADS, CH_LDS, s>>>(a);
        } else if (variant == 2) {
            chain_persistent<1, 0><<<grid, CH_THREADS, CH_LDS, s>>>(a);
        } else if (variant == 3) {
            chain_persistent<1, 1><<<grid, CH_THREADS, CH_LDS, s>>>(a);
        } else if (variant == 4) {
            chain_xcd<<<grid, CH_THREADS, CH_LDS, s>>>(a);
        } else {
            chain_collocal<<<grid, CH_THREADS, CH_LDS, s>>>(a);
        }
        CK(hipGetLastError());
    };
    // watchdog: a chain still running after 5 s is reported (counters, job states) and the
    // program stops; the bounded waits let the grid drain
    auto finish = [&](int v) {
        for (int w = 0; hipStreamQuery(s1) == hipErrorNotReady; ++w) {
            usleep(500);
            if (w == 10000) {
                int h[5 * CH_RB + 2];
                std::vector<int> st(N_JOBS);
                CK(hipMemcpyAsync(h, ctl, sizeof(h), hipMemcpyDeviceToHost, s3));
                CK(hipMemcpyAsync(st.data(), a.dbg, N_JOBS * 4, hipMemcpyDeviceToHost, s3));
                CK(hipStreamSynchronize(s3));
                fprintf(stderr, "%s still running after 5 s: ticket %d err %d counters", names[v], h[5 * CH_RB],
                        h[5 * CH_RB + 1]);
                for (int i = 0; i < 5 * CH_RB; ++i) fprintf(stderr, " %d", h[i]);
                fprintf(stderr, "\n");
                const int starts[6] = {0, N_OUT, N_OUT + N_LN, N_OUT + N_LN + N_FC, N_OUT + N_LN + N_FC + N_PROJ, N_JOBS};
                for (int p = 0; p < 5; ++p) {
                    int c[4] = {0, 0, 0, 0};
                    for (int j = starts[p]; j < starts[p + 1]; ++j) c[std::min(3, std::max(0, st[j]))]++;
                    fprintf(stderr, "  phase %d: new %d started %d math-done %d finished %d\n", p, c[0], c[1], c[2], c[3]);
                }
                CK(hipStreamSynchronize(s1));
                exit(3);
            }
        }
        CK(hipStreamSynchronize(s1));
        int err = 0;
        CK(hipMemcpy(&err, a.err, 4, hipMemcpyDeviceToHost));
        if (err) {
            fprintf(stderr, "%s: wait timeout\n", names[v]);
            exit(1);
        }
    };

    // numerics: host fp32 reference (bf16 rounding where the kernels round) on 16 rows
    std::vector<bf16_t> ref_out[NV];
    for (int v = 0; v < NV; ++v) {
        reset(s1);
        CK(hipStreamSynchronize(s1));
        fprintf(stderr, "numerics run %s (grid %d, jobs %d)\n", names[v], grid, N_JOBS);
        launch(v, s1);
        finish(v);
        ref_out[v].resize((size_t)CH_M * CH_D);
        CK(hipMemcpy(ref_out[v].data(), a.ln_next, ref_out[v].size() * 2, hipMemcpyDeviceToHost));
    }
    double max_err = 0;
    const int check_rows[] = {0, 1, 7, 63, 64, 130, 200, 255, 256, 311, 383, 400, 447, 480, 510, 511};
    for (int row : check_rows) {
        std::vector<float> xr(CH_D), ln(CH_D), h(CH_F), out(CH_D);
        for (int c = 0; c < CH_D; ++c) {
            double s = 0;
            for (int k = 0; k < CH_D; ++k) s += (double)h_f32(attn[row * CH_D + k]) * h_f32(Wo[c * CH_D + k]);
            xr[c] = x0[row * CH_D + c] + (float)s + bo[c];
        }
        host_ln(xr.data(), g2.data(), b2.data(), ln.data());
        for (int f = 0; f < CH_F; ++f) {
            double s = 0;
            for (int k = 0; k < CH_D; ++k) s += (double)ln[k] * h_f32(Wfc[(size_t)f * CH_D + k]);
            h[f] = h_f32(h_bf16(h_gelu((float)s + bfc[f])));
        }
        for (int c = 0; c < CH_D; ++c) {
            double s = 0;
            for (int k = 0; k < CH_F; ++k) s += (double)h[k] * h_f32(Wp[(size_t)c * CH_F + k]);
            xr[c] += (float)s + bp[c];
        }
        host_ln(xr.data(), g1.data(), b1.data(), out.data());
        for (int c = 0; c < CH_D; ++c)
            max_err = std::max(max_err, (double)fabsf(h_f32(ref_out[0][(size_t)row * CH_D + c]) - out[c]));
    }
    long mism[NV] = {0, 0, 0, 0, 0, 0};
    for (int v = 1; v < NV; ++v)
        for (size_t i = 0; i < ref_out[0].size(); ++i) mism[v] += ref_out[v][i] != ref_out[0][i];
    printf("{\"check\": \"numerics\", \"rows_vs_host_fp32\": 16, \"max_abs_err\": %.5f, \"bit_mismatch_vs_five_launches\": "
           "[%ld, %ld, %ld, %ld, %ld], \"grid\": %d, \"jobs\": %d, \"proj_tile_rows\": %d}\n",
           max_err, mism[1], mism[2], mism[3], mism[4], mism[5], grid, N_JOBS, CH_PBM);
    fflush(stdout);
    if (max_err > 0.1) return 2;

    for (int beside = 0; beside < 2; ++beside) {
        for (int v = 0; v < NV; ++v) {
            std::vector<float> t;
            for (int it = 0; it < iters + 3; ++it) {
                reset(s1);
                CK(hipStreamSynchronize(s1));
                if (beside) {
                    stream_read<<<1024, 256, 0, s2>>>(sbuf, sbytes / 16, sink);
                    CK(hipGetLastError());
                }
                CK(hipEventRecord(e0, s1));
                launch(v, s1);
                CK(hipEventRecord(e1, s1));
                finish(v);
                CK(hipStreamSynchronize(s2));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 3) t.push_back(ms * 1e3f);
            }
            const int err = 0;  // finish() stops the program on a wait timeout
            std::vector<bf16_t> last((size_t)CH_M * CH_D);  // the last timed run's output, vs the first
            CK(hipMemcpy(last.data(), a.ln_next, last.size() * 2, hipMemcpyDeviceToHost));
            long bad = 0;
            for (size_t i = 0; i < last.size(); ++i) bad += last[i] != ref_out[0][i];
            std::sort(t.begin(), t.end());
            printf("{\"variant\": \"%s\", \"beside_stream\": %s, \"us_median\": %.2f, \"us_min\": %.2f, \"us_p90\": %.2f, "
                   "\"iters\": %d, \"wait_timeout\": %d, \"bit_mismatch_last_run\": %ld, \"proj_tile_rows\": %d}\n",
                   names[v], beside ? "true" : "false", t[t.size() / 2], t[0], t[t.size() * 9 / 10], iters, err, bad,
                   CH_PBM);
            fflush(stdout);
        }
    }
    return 0;
}
