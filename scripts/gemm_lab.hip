// GEMM lab: standalone HIP microbenchmark for the decode / prefill / LM-head GEMM shapes.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I distributed_lms_raft_llm_amd/ops/csrc \
//         scripts/gemm_lab.hip -o scripts/gemm_lab && ./scripts/gemm_lab [filter]
//
// Times the production kernel (ops/csrc/gemm.hip, included verbatim) in several tile configs and
// a PROBE copy of its main loop that can drop parts of the work, to attribute the time:
//   mode 0 full, 1 loads only (LDS-DMA ring + waits + barriers, no ds_read / MFMA),
//   2 no global loads (ds_read + MFMA on whatever the LDS holds), 3 MFMA only (register operands).
// Weights rotate over >= 600 MB of copies so they stream from HBM as in a 12-layer decode step.
// Prints one JSON line per (shape, config, mode).
#include "gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

static int g_pad = 0;  // leading-dimension padding (elements) of A and W

template <int BM, int BN, int WM, int WN, int STAGES, int PROBE>
__global__ __launch_bounds__(64 * WM * WN) void probe_kernel(const bf16_t* __restrict__ A, int lda,
                                                             const bf16_t* __restrict__ W, int ldw, int M, int N,
                                                             int K, bf16_t* __restrict__ C, int ldc,
                                                             unsigned long long* __restrict__ stamps) {
    const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
    constexpr int NW = WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int ROWB = 128, A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;
    constexpr int PPW = STAGE_BYTES / 1024 / NW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave / WN, wn = wave % WN;
    const int tiles_m = (M + BM - 1) / BM;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int m0 = (bid % tiles_m) * BM, n0 = (bid / tiles_m) * BN;
    const char* src[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int piece = wave + NW * i, row = piece * 8 + (lane >> 3), lchunk = (lane & 7) ^ (lane >> 3);
        if (row < BM) {
            const int gm = m0 + row < M ? m0 + row : M - 1;
            src[i] = reinterpret_cast<const char*>(A) + (size_t)gm * lda * 2 + lchunk * 16;
        } else {
            src[i] = reinterpret_cast<const char*>(W) + (size_t)(n0 + row - BM) * ldw * 2 + lchunk * 16;
        }
    }
    auto issue = [&](int stage, int k0) {
        if constexpr (PROBE == 2 || PROBE == 3) return;
        char* dst = smem + stage * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < PPW; ++i)
            __builtin_amdgcn_global_load_lds((glob_void_t*)(src[i] + (size_t)k0 * 2),
                                             (lds_void_t*)(dst + (wave + NW * i) * 1024), 16, 0, 0);
    };
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int nk = K / 64;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) issue(s, s * 64);
    const int frow = lane & 15, fk = lane >> 4, fsw = lane & 7;
    bf16x8_t reg_a = *reinterpret_cast<const bf16x8_t*>(A + (size_t)(lane & 15) * lda);
    unsigned long long t_first = 0;
    for (int kt = 0; kt < nk; ++kt) {
        if (nk - kt >= STAGES - 1)
            wait_vmcnt<(STAGES - 2) * PPW>();
        else
            wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt == 0) t_first = __builtin_amdgcn_s_memrealtime();
        {
            const int kn = kt + STAGES - 1;
            if (kn < nk) issue(kn % STAGES, kn * 64);
        }
        if constexpr (PROBE == 1) continue;
        const char* as = smem + (kt % STAGES) * STAGE_BYTES + (wm * WTM) * ROWB;
        const char* ws = smem + (kt % STAGES) * STAGE_BYTES + A_BYTES + (wn * WTN) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = (((ks * 4 + fk) ^ fsw) << 4);
            bf16x8_t af[TM], bfr[TN];
            if constexpr (PROBE == 3) {
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = reg_a;
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = reg_a;
            } else {
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frow) * ROWB + coff);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frow) * ROWB + coff);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    wait_vmcnt<0>();
    const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
    const int row_base = m0 + wm * WTM + (lane >> 4) * 4, col_base = n0 + wn * WTN + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row_base + i * 16 + r;
                if (row < M) C[(size_t)row * ldc + col_base + j * 16] = f32_to_bf16(acc[i][j][r]);
            }
    if (stamps && tid < 4) {  // vector stores from 4 lanes of wave 0
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const unsigned long long v = tid == 0 ? t_entry : tid == 1 ? t_first : tid == 2 ? t_loop : t_end;
        stamps[(size_t)blockIdx.x * 4 + tid] = v;
    }
}

template <int BM, int BN, int WM, int WN, int STAGES, int PROBE>
static void launch_probe(const bf16_t* A, const bf16_t* W, bf16_t* C, int M, int N, int K, hipStream_t s,
                         unsigned long long* stamps = nullptr) {
    const size_t lds = (size_t)STAGES * (BM + BN) * 128;
    static bool set = false;
    if (!set) {
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_kernel<BM, BN, WM, WN, STAGES, PROBE>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        set = true;
    }
    const int tiles = ((M + BM - 1) / BM) * (N / BN);
    hipLaunchKernelGGL((probe_kernel<BM, BN, WM, WN, STAGES, PROBE>), dim3(tiles), dim3(64 * WM * WN), lds, s, A, K, W,
                       K, M, N, K, C, N, stamps);
}


// Warp-specialised variant: WM x WN MFMA waves + NL loader waves per workgroup.  Loader waves
// only issue the LDS-DMA ring (and wait for it); MFMA waves only ds_read + MFMA.  One raw barrier
// per k-step orders both groups (loaders: wait own DMA -> barrier -> issue next stage).
template <int BM, int BN, int WM, int WN, int STAGES, int NL>
__global__ __launch_bounds__(64 * (WM * WN + NL)) void ws_kernel(const bf16_t* __restrict__ A, int lda,
                                                                 const bf16_t* __restrict__ W, int ldw, int M, int N,
                                                                 int K, bf16_t* __restrict__ C, int ldc) {
    constexpr int NM = WM * WN;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int ROWB = 128, A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;
    constexpr int PIECES = STAGE_BYTES / 1024;
    static_assert(PIECES % NL == 0, "pieces must split over the loader waves");
    constexpr int PPW = PIECES / NL;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tiles_m = (M + BM - 1) / BM;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int m0 = (bid % tiles_m) * BM, n0 = (bid / tiles_m) * BN;
    const int nk = K / 64;
    if (wave >= NM) {  // ---------------- loader waves ----------------
        const int lw = wave - NM;
        const char* src[PPW];
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int piece = lw + NL * i, row = piece * 8 + (lane >> 3), lchunk = (lane & 7) ^ (lane >> 3);
            if (row < BM) {
                const int gm = m0 + row < M ? m0 + row : M - 1;
                src[i] = reinterpret_cast<const char*>(A) + (size_t)gm * lda * 2 + lchunk * 16;
            } else {
                src[i] = reinterpret_cast<const char*>(W) + (size_t)(n0 + row - BM) * ldw * 2 + lchunk * 16;
            }
        }
        auto issue = [&](int stage, int k0) {
            char* dst = smem + stage * STAGE_BYTES;
#pragma unroll
            for (int i = 0; i < PPW; ++i)
                __builtin_amdgcn_global_load_lds((glob_void_t*)(src[i] + (size_t)k0 * 2),
                                                 (lds_void_t*)(dst + (lw + NL * i) * 1024), 16, 0, 0);
        };
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if (s < nk) issue(s, s * 64);
        for (int kt = 0; kt < nk; ++kt) {
            if (nk - kt >= STAGES - 1)
                wait_vmcnt<(STAGES - 2) * PPW>();
            else
                wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            const int kn = kt + STAGES - 1;
            if (kn < nk) issue(kn % STAGES, kn * 64);
        }
        return;
    }
    // ---------------- MFMA waves ----------------
    const int wm = wave / WN, wn = wave % WN;
    f32x4_t acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int frow = lane & 15, fk = lane >> 4, fsw = lane & 7;
    for (int kt = 0; kt < nk; ++kt) {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* as = smem + (kt % STAGES) * STAGE_BYTES + (wm * WTM) * ROWB;
        const char* ws = smem + (kt % STAGES) * STAGE_BYTES + A_BYTES + (wn * WTN) * ROWB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int coff = (((ks * 4 + fk) ^ fsw) << 4);
            bf16x8_t af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const bf16x8_t*>(as + (i * 16 + frow) * ROWB + coff);
#pragma unroll
            for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8_t*>(ws + (j * 16 + frow) * ROWB + coff);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    const int row_base = m0 + wm * WTM + (lane >> 4) * 4, col_base = n0 + wn * WTN + (lane & 15);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = row_base + i * 16 + r;
                if (row < M) C[(size_t)row * ldc + col_base + j * 16] = f32_to_bf16(acc[i][j][r]);
            }
}

template <int BM, int BN, int WM, int WN, int STAGES, int NL>
static void launch_ws(const bf16_t* A, const bf16_t* W, bf16_t* C, int M, int N, int K, hipStream_t s) {
    const size_t lds = (size_t)STAGES * (BM + BN) * 128;
    static bool set = false;
    if (!set) {
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&ws_kernel<BM, BN, WM, WN, STAGES, NL>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        set = true;
    }
    const int tiles = ((M + BM - 1) / BM) * (N / BN);
    hipLaunchKernelGGL((ws_kernel<BM, BN, WM, WN, STAGES, NL>), dim3(tiles), dim3(64 * (WM * WN + NL)), lds, s, A,
                       K + g_pad, W, K + g_pad, M, N, K, C, N);
}

struct Shape {
    const char* name;
    int M, N, K;
};

struct Bufs {
    bf16_t* A;
    std::vector<bf16_t*> W;
    bf16_t* C;
};

static float time_it(const std::function<void(const bf16_t*)>& run, const Bufs& b, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) run(b.W[i % b.W.size()]);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) run(b.W[i % b.W.size()]);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms * 1000.f / iters;
}

__global__ void fill_kernel(bf16_t* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)(i * 2654435761u) ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = f32_to_bf16(((int)(x & 0xffff) - 32768) * (1.0f / 65536.f));
    }
}

static float bf(bf16_t v) {
    unsigned u = ((unsigned)v) << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// spot-check 64 outputs of C = A W^T against a host double reference
static double check(const Bufs& b, const bf16_t* W, int M, int N, int K) {
    const int ld = K + g_pad;
    std::vector<bf16_t> hA((size_t)M * ld), hW((size_t)N * ld), hC((size_t)M * N);
    CK(hipMemcpy(hA.data(), b.A, hA.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hW.data(), W, hW.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hC.data(), b.C, hC.size() * 2, hipMemcpyDeviceToHost));
    double worst = 0;
    unsigned s = 12345;
    for (int t = 0; t < 64; ++t) {
        s = s * 1103515245u + 12345u;
        const int m = (s >> 8) % M;
        s = s * 1103515245u + 12345u;
        const int n = (s >> 8) % N;
        double ref = 0;
        for (int k = 0; k < K; ++k) ref += (double)bf(hA[(size_t)m * ld + k]) * bf(hW[(size_t)n * ld + k]);
        const double err = fabs(ref - bf(hC[(size_t)m * N + n])) / (fabs(ref) + 0.05);
        worst = err > worst ? err : worst;
    }
    return worst;
}

int main(int argc, char** argv) {
    const std::string filt = argc > 1 ? argv[1] : "";
    const Shape shapes[] = {{"qkv", 1024, 2304, 768},   {"fc", 1024, 3072, 768},    {"proj", 1024, 768, 3072},
                            {"oproj", 1024, 768, 768},  {"lmhead", 1024, 50304, 768}, {"qkv512", 512, 2304, 768},
                            {"pf_fc", 32768, 3072, 768}, {"pf_qkv", 32768, 2304, 768}};
    hipStream_t st = 0;
    for (const Shape& sh : shapes) {
        if (!filt.empty() && filt.find(sh.name) == std::string::npos) continue;
        const int M = sh.M, N = sh.N, K = sh.K;
        Bufs b;
        CK(hipMalloc(&b.A, (size_t)M * (K + 128) * 2));
        CK(hipMalloc(&b.C, (size_t)M * N * 2));
        fill_kernel<<<1024, 256>>>(b.A, (size_t)M * (K + 128), 7u);
        const size_t wbytes = (size_t)N * (K + 128) * 2;
        const int copies = (int)((600ull << 20) / wbytes) + 1;
        for (int c = 0; c < copies; ++c) {
            bf16_t* w;
            CK(hipMalloc(&w, wbytes));
            fill_kernel<<<1024, 256>>>(w, (size_t)N * (K + 128), 100u + c);
            b.W.push_back(w);
        }
        CK(hipDeviceSynchronize());
        const double flops = 2.0 * M * N * K;
        const int iters = M >= 8192 || N >= 8192 ? 20 : 200;
        auto report = [&](const char* cfg, int mode, float us, int bm, int bn) {
            const double tiles = (double)((M + bm - 1) / bm) * (N / bn);
            const double l2bytes = tiles * (K / 64) * (bm + bn) * 128.0;
            printf("{\"pad\": %d, \"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"cfg\": \"%s\", \"mode\": %d, \"us\": %.2f, "
                   "\"tflops\": %.1f, \"wgs\": %d, \"lds_fill_TBps\": %.2f}\n",
                   g_pad, sh.name, M, N, K, cfg, mode, us, flops / us * 1e-6, (int)tiles, l2bytes / us * 1e-6);
            fflush(stdout);
        };
        GemmEpi ep;
        memset(&ep, 0, sizeof(ep));
        float* part = nullptr;
        CK(hipMalloc(&part, (size_t)8 * M * N * 4));
        ep.out = b.C;
        ep.ldo = N;
#define PROD(BM, BN, WM, WN, S)                                                                                   \
    {                                                                                                             \
        auto run = [&](const bf16_t* w) {                                                                         \
            CK((launch_gemm_cfg<BM, BN, WM, WN, S, EPI_BF16, IN_BF16>(b.A, K + g_pad, w, K + g_pad, M, N, K, ep, st)));           \
        };                                                                                                        \
        const float us = time_it(run, b, iters);                                                                  \
        const double err = check(b, b.W[(iters - 1) % b.W.size()], M, N, K);                                     \
        if (err > 0.02) printf("{\"error\": \"prod %dx%d w%dx%d s%d rel err %.4f\"}\n", BM, BN, WM, WN, S, err); \
        char nm[64];                                                                                              \
        snprintf(nm, sizeof nm, "prod %dx%d w%dx%d s%d", BM, BN, WM, WN, S);                                      \
        report(nm, 0, us, BM, BN);                                                                                \
    }
#define PSPLIT(BM, BN, WM, WN, S, SPLIT)                                                                      \
    {                                                                                                         \
        GemmEpi ep2 = ep;                                                                                     \
        ep2.out = part;                                                                                       \
        ep2.ldo = N;                                                                                          \
        ep2.split_k = SPLIT;                                                                                  \
        ep2.split_stride = (long long)M * N;                                                                  \
        auto run = [&](const bf16_t* w) {                                                                     \
            CK((launch_gemm_cfg<BM, BN, WM, WN, S, EPI_PARTIAL, IN_BF16>(b.A, K + g_pad, w, K + g_pad, M, N, K, ep2, st)));   \
        };                                                                                                    \
        const float us = time_it(run, b, iters);                                                              \
        char nm[64];                                                                                          \
        snprintf(nm, sizeof nm, "split%d %dx%d w%dx%d s%d", SPLIT, BM, BN, WM, WN, S);                        \
        report(nm, 0, us, BM, BN);                                                                            \
    }
#define WS(BM, BN, WM, WN, S, NL)                                                                             \
    {                                                                                                         \
        auto run = [&](const bf16_t* w) { launch_ws<BM, BN, WM, WN, S, NL>(b.A, w, b.C, M, N, K, st); };      \
        const float us = time_it(run, b, iters);                                                              \
        const double err = check(b, b.W[(iters - 1) % b.W.size()], M, N, K);                                 \
        if (err > 0.02) printf("{\"error\": \"ws %dx%d rel err %.4f\"}\n", BM, BN, err);                     \
        char nm[64];                                                                                          \
        snprintf(nm, sizeof nm, "ws %dx%d w%dx%d s%d L%d", BM, BN, WM, WN, S, NL);                            \
        report(nm, 0, us, BM, BN);                                                                            \
    }
#define STAMP(BM, BN, WM, WN, S)                                                                              \
    {                                                                                                         \
        const int tiles = ((M + BM - 1) / BM) * (N / BN);                                                     \
        unsigned long long* dst;                                                                              \
        CK(hipMalloc(&dst, (size_t)tiles * 32));                                                              \
        for (int it = 0; it < 20; ++it) launch_probe<BM, BN, WM, WN, S, 0>(b.A, b.W[it % b.W.size()], b.C, M, N, K, st, dst); \
        CK(hipDeviceSynchronize());                                                                           \
        std::vector<unsigned long long> h((size_t)tiles * 4);                                                 \
        CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));                                   \
        unsigned long long t0 = ~0ull, tend = 0;                                                              \
        for (int t = 0; t < tiles; ++t) { t0 = std::min(t0, h[t * 4]); tend = std::max(tend, h[t * 4 + 3]); } \
        double s_pro = 0, s_loop = 0, s_epi = 0, s_start = 0, mx_start = 0;                                  \
        for (int t = 0; t < tiles; ++t) {                                                                     \
            s_pro += h[t * 4 + 1] - h[t * 4]; s_loop += h[t * 4 + 2] - h[t * 4 + 1]; s_epi += h[t * 4 + 3] - h[t * 4 + 2]; \
            s_start += h[t * 4] - t0; mx_start = std::max(mx_start, (double)(h[t * 4] - t0));               \
        }                                                                                                     \
        printf("{\"stamp\": \"%s %dx%d w%dx%d s%d\", \"span_us\": %.2f, \"prologue_us\": %.2f, \"loop_us\": %.2f, \"epi_us\": %.2f, \"mean_start_us\": %.2f, \"max_start_us\": %.2f}\n", \
               sh.name, BM, BN, WM, WN, S, (tend - t0) / 100.0, s_pro / tiles / 100.0, s_loop / tiles / 100.0, s_epi / tiles / 100.0, \
               s_start / tiles / 100.0, mx_start / 100.0);                                                  \
        fflush(stdout);                                                                                       \
        CK(hipFree(dst));                                                                                     \
    }
#define PROBE4(BM, BN, WM, WN, S)                                                                               \
    {                                                                                                           \
        char nm[64];                                                                                            \
        snprintf(nm, sizeof nm, "probe %dx%d w%dx%d s%d", BM, BN, WM, WN, S);                                   \
        report(nm, 0, time_it([&](const bf16_t* w) { launch_probe<BM, BN, WM, WN, S, 0>(b.A, w, b.C, M, N, K, st); }, b, iters), BM, BN); \
        report(nm, 1, time_it([&](const bf16_t* w) { launch_probe<BM, BN, WM, WN, S, 1>(b.A, w, b.C, M, N, K, st); }, b, iters), BM, BN); \
        report(nm, 2, time_it([&](const bf16_t* w) { launch_probe<BM, BN, WM, WN, S, 2>(b.A, w, b.C, M, N, K, st); }, b, iters), BM, BN); \
        report(nm, 3, time_it([&](const bf16_t* w) { launch_probe<BM, BN, WM, WN, S, 3>(b.A, w, b.C, M, N, K, st); }, b, iters), BM, BN); \
    }
        PROD(64, 64, 2, 2, 2)
        PROD(64, 64, 2, 2, 3)
        PROD(64, 64, 2, 2, 4)
        if (sh.N % 96 == 0) {
            PROD(128, 96, 2, 2, 3)
            PROD(128, 96, 2, 2, 4)
            PROD(64, 96, 2, 2, 3)
        }
        if (sh.N == 768) {
            for (int split : {2, 3, 4, 6}) {
                if ((sh.K / 64) % split) continue;
                PSPLIT(64, 64, 2, 2, 2, split)
                PSPLIT(64, 64, 2, 2, 3, split)
                PSPLIT(64, 64, 2, 2, 4, split)
                PSPLIT(128, 96, 2, 2, 4, split)
            }
        }
        for (bf16_t* w : b.W) CK(hipFree(w));
        CK(hipFree(b.A));
        CK(hipFree(b.C));
        CK(hipFree(part));
    }
    return 0;
}
