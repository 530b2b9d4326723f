// One-shot all-reduce / all-gather over xGMI peer memory for tensor-parallel decode.
//
// Why: a TP decode step of GPT-2 issues 2 all-reduces per layer (attention out-proj and c_proj,
// row-parallel) on tiny messages (rows x d fp32: 64 x 1280 x 4 B = 320 KB at B = 64).  A ring
// all-reduce over RCCL pays 2(W-1) dependent link hops per call; on MI355X every GPU has a direct
// xGMI link to each of its 7 peers, so a ONE-SHOT scheme -- every rank reads every peer's
// partial straight out of the peer's HBM and sums locally -- costs one barrier round trip plus
// one parallel read over all links.  The reference has no
// GPU path at all (its tutor is a CPU `model.generate`, /root/reference/tutoring_server.py:21-29).
//
// Memory: each rank owns ONE uncached allocation (hipDeviceMallocUncached: stores go straight to
// HBM, remote reads never hit a stale L2 line), shared with its peers through hipIpc handles:
//
//   [ flag board: XGMI_MAX_BLOCKS x 8 u32 ][ epoch u32 ][ arrive u32 ][ err u32 ] ... (64 KiB)
//   [ slab 0: slab_bytes ][ slab 1: slab_bytes ]
//
// Protocol of one call (block b of rank r, all ranks launch the identical grid):
//   e = epoch + 1                     call counter kept on the device (the last block of a call
//                                     to finish advances it), so the same kernel works eagerly
//                                     AND replayed from a hipGraph, with no host-side state
//   copy chunk b of `in` -> slab[e & 1] of rank r
//   flag[p].board[b][r] = e  (system-scope release store, for every peer p)
//   spin until my board[b][p] >= e for every p   (bounded: sets *err and gives up after ~1 s)
//   acquire fence (system scope), then out chunk b = sum_p slab_p[e & 1] chunk b, p = 0..W-1 in
//   rank order -- every rank computes bit-identical sums (the greedy argmax must agree across TP
//   ranks, exactly as with a ring all-reduce).
// Slab reuse: rank r writes slab[e & 1] only at call e, after finishing call e-1 -- whose barrier
// proved that every peer had STARTED call e-1, hence (stream order) finished call e-2, the last
// reader of that parity.  So one barrier per call is enough.  (The counter is per CALL, not per
// block: grids differ between calls, and a per-block parity would let one call's block overwrite
// a range a peer's differently-sized previous call is still reading.)
#include <cstring>

#include "common.h"

#define XGMI_MAX_RANKS 8
#define XGMI_MAX_BLOCKS 128
#define XGMI_THREADS 256
#define XGMI_HEADER_BYTES 65536
#define XGMI_SPIN_LIMIT (1u << 24)

struct XgmiArgs {
    char* base[XGMI_MAX_RANKS];  // every rank's allocation (IPC-mapped; [rank] is the local one)
    const void* in;
    void* out;
    long long n;                 // fp32 elements (sum) or 8-byte words per rank (gather)
    long long slab_bytes;
    int rank;
    int world;
};

__device__ __forceinline__ unsigned* xgmi_board(char* base) { return reinterpret_cast<unsigned*>(base); }
#define XGMI_EPOCH_WORD (XGMI_MAX_BLOCKS * XGMI_MAX_RANKS)
#define XGMI_ARRIVE_WORD (XGMI_EPOCH_WORD + 1)
#define XGMI_ERR_WORD (XGMI_EPOCH_WORD + 2)
__device__ __forceinline__ unsigned* xgmi_word(char* base, int w) { return reinterpret_cast<unsigned*>(base) + w; }

// This call's number (1, 2, ...): the local counter + 1 (advanced by xgmi_finish).
__device__ __forceinline__ unsigned xgmi_epoch(const XgmiArgs& a) {
    __shared__ unsigned s_epoch;
    if (threadIdx.x == 0) s_epoch = *xgmi_word(a.base[a.rank], XGMI_EPOCH_WORD) + 1;
    __syncthreads();
    return s_epoch;
}

// The last block of the call to get here advances the counter for the next call (every block has
// read it by then: it is read before the barrier, and this runs after it).
__device__ __forceinline__ void xgmi_finish(const XgmiArgs& a, unsigned e) {
    __syncthreads();
    if (threadIdx.x == 0) {
        char* me = a.base[a.rank];
        if (atomicAdd(xgmi_word(me, XGMI_ARRIVE_WORD), 1u) == gridDim.x - 1) {
            *xgmi_word(me, XGMI_ARRIVE_WORD) = 0;
            *xgmi_word(me, XGMI_EPOCH_WORD) = e;
        }
    }
}

// Per-block cross-GPU barrier: announce call e to every peer's board, wait for theirs.
template <int W>
__device__ __forceinline__ void xgmi_signal_and_wait(const XgmiArgs& a, unsigned e) {
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    // every wave's slab stores complete (and L2 written back) before any flag goes out: a
    // workgroup barrier alone does not wait for other waves' stores to land
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (t < W) {
        // release at system scope: this block's slab stores are visible to every peer first
        __hip_atomic_store(xgmi_board(a.base[t]) + b * XGMI_MAX_RANKS + a.rank, e, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned* mine = xgmi_board(a.base[a.rank]) + b * XGMI_MAX_RANKS + t;
        unsigned spins = 0;
        while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > XGMI_SPIN_LIMIT) {  // a peer never arrived: report, never hang the GPU
                atomicOr(xgmi_word(a.base[a.rank], XGMI_ERR_WORD), 1u);
                break;
            }
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: peers' slab stores now visible
}

// [lo, hi) of this block, in vector units (float4 for the sum, u64 for the gather)
__device__ __forceinline__ void xgmi_chunk(long long n16, long long& lo, long long& hi) {
    const long long per = (n16 + gridDim.x - 1) / gridDim.x;
    lo = (long long)blockIdx.x * per;
    hi = lo + per < n16 ? lo + per : n16;
}

template <int W>
__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allreduce_f32_kernel(XgmiArgs a) {
    const unsigned e = xgmi_epoch(a);
    const long long slab_off = XGMI_HEADER_BYTES + (long long)(e & 1) * a.slab_bytes;
    long long lo, hi;
    xgmi_chunk(a.n / 4, lo, hi);
    const float4* in = reinterpret_cast<const float4*>(a.in);
    float4* mine = reinterpret_cast<float4*>(a.base[a.rank] + slab_off);
    for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) mine[i] = in[i];
    xgmi_signal_and_wait<W>(a, e);
    const float4* src[W];
#pragma unroll
    for (int p = 0; p < W; ++p) src[p] = reinterpret_cast<const float4*>(a.base[p] + slab_off);
    float4* out = reinterpret_cast<float4*>(a.out);
    for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) {
        float4 v[W];
#pragma unroll
        for (int p = 0; p < W; ++p) v[p] = src[p][i];  // all W loads in flight, one per link
        float4 s = v[0];
#pragma unroll
        for (int p = 1; p < W; ++p) {
            s.x += v[p].x; s.y += v[p].y; s.z += v[p].z; s.w += v[p].w;
        }
        out[i] = s;
    }
    xgmi_finish(a, e);
}

// Integer all-reduce of int64 words (the TP fused decode's fixed-point residual partials,
// value * 2^32): integer adds are exact and order-independent, so every rank holds the identical
// residual without relying on a summation order.  n: int64 words, a multiple of 2.
template <int W>
__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allreduce_i64_kernel(XgmiArgs a) {
    const unsigned e = xgmi_epoch(a);
    const long long slab_off = XGMI_HEADER_BYTES + (long long)(e & 1) * a.slab_bytes;
    long long lo, hi;
    xgmi_chunk(a.n / 2, lo, hi);
    const longlong2* in = reinterpret_cast<const longlong2*>(a.in);
    longlong2* mine = reinterpret_cast<longlong2*>(a.base[a.rank] + slab_off);
    for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) mine[i] = in[i];
    xgmi_signal_and_wait<W>(a, e);
    const longlong2* src[W];
#pragma unroll
    for (int p = 0; p < W; ++p) src[p] = reinterpret_cast<const longlong2*>(a.base[p] + slab_off);
    longlong2* out = reinterpret_cast<longlong2*>(a.out);
    for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) {
        longlong2 v[W];
#pragma unroll
        for (int p = 0; p < W; ++p) v[p] = src[p][i];
        longlong2 s = v[0];
#pragma unroll
        for (int p = 1; p < W; ++p) {
            s.x += v[p].x;
            s.y += v[p].y;
        }
        out[i] = s;
    }
    xgmi_finish(a, e);
}

// out[p * n + i] = in_p[i]: n 8-byte words from every rank (the LM head's packed argmax keys).
template <int W>
__global__ __launch_bounds__(XGMI_THREADS) void xgmi_allgather_u64_kernel(XgmiArgs a) {
    const unsigned e = xgmi_epoch(a);
    const long long slab_off = XGMI_HEADER_BYTES + (long long)(e & 1) * a.slab_bytes;
    long long lo, hi;
    xgmi_chunk(a.n, lo, hi);
    const unsigned long long* in = reinterpret_cast<const unsigned long long*>(a.in);
    unsigned long long* mine = reinterpret_cast<unsigned long long*>(a.base[a.rank] + slab_off);
    for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) mine[i] = in[i];
    xgmi_signal_and_wait<W>(a, e);
    unsigned long long* out = reinterpret_cast<unsigned long long*>(a.out);
#pragma unroll
    for (int p = 0; p < W; ++p) {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.base[p] + slab_off);
        for (long long i = lo + threadIdx.x; i < hi; i += XGMI_THREADS) out[(long long)p * a.n + i] = src[i];
    }
    xgmi_finish(a, e);
}

static int xgmi_blocks(long long units) {
    // ~4 KiB of each rank's message per block: a 320 KB decode all-reduce spreads over 80 blocks
    long long b = (units + 255) / 256;
    if (b < 1) b = 1;
    if (b > XGMI_MAX_BLOCKS) b = XGMI_MAX_BLOCKS;
    return (int)b;
}

#define XGMI_DISPATCH(KERNEL, W, GRID, ARGS, STREAM)                                                   \
    switch (W) {                                                                                       \
        case 1: KERNEL<1><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 2: KERNEL<2><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 3: KERNEL<3><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 4: KERNEL<4><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 5: KERNEL<5><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 6: KERNEL<6><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 7: KERNEL<7><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        case 8: KERNEL<8><<<GRID, XGMI_THREADS, 0, STREAM>>>(ARGS); break;                             \
        default: return (int)hipErrorInvalidValue;                                                     \
    }

static int xgmi_check(const XgmiArgs* a, long long bytes) {
    if (a->world < 1 || a->world > XGMI_MAX_RANKS || a->rank < 0 || a->rank >= a->world) return (int)hipErrorInvalidValue;
    if (bytes > a->slab_bytes || a->n < 0) return (int)hipErrorInvalidValue;
    for (int p = 0; p < a->world; ++p)
        if (!a->base[p]) return (int)hipErrorInvalidValue;
    return 0;
}

// ---------------------------------------------------------------- host ABI
extern "C" long long dlms_xgmi_header_bytes() { return XGMI_HEADER_BYTES; }
extern "C" int dlms_xgmi_max_blocks() { return XGMI_MAX_BLOCKS; }
extern "C" int dlms_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Zeroed allocation of XGMI_HEADER_BYTES + 2 * slab_bytes, uncached unless cached != 0.
extern "C" int dlms_xgmi_alloc(long long slab_bytes, int cached, void** out) {
    void* p = nullptr;
    const size_t bytes = (size_t)XGMI_HEADER_BYTES + 2 * (size_t)slab_bytes;
    hipError_t e = hipExtMallocWithFlags(&p, bytes, cached ? hipDeviceMallocDefault : hipDeviceMallocUncached);
    if (e != hipSuccess) return (int)e;
    e = hipMemset(p, 0, bytes);
    if (e != hipSuccess) {
        (void)hipFree(p);
        return (int)e;
    }
    *out = p;
    return 0;
}

extern "C" int dlms_xgmi_free(void* p) { return (int)hipFree(p); }

extern "C" int dlms_ipc_get_handle(void* p, void* handle_out) {
    return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), p);
}

extern "C" int dlms_ipc_open(const void* handle, void** out) {
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int dlms_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// Error word of the local board (non-zero: a barrier timed out); reset by reading with clear=1.
extern "C" int dlms_xgmi_error(void* base, int clear, unsigned* out) {
    unsigned* e = reinterpret_cast<unsigned*>(base) + XGMI_ERR_WORD;
    hipError_t r = hipMemcpy(out, e, sizeof(unsigned), hipMemcpyDeviceToHost);
    if (r != hipSuccess || !clear) return (int)r;
    return (int)hipMemset(e, 0, sizeof(unsigned));
}

// The error word copied to (pinned) host memory behind the work already on ``stream`` -- the
// serving loop polls it once per decode chunk without a device-wide synchronise.
extern "C" int dlms_xgmi_error_async(void* base, unsigned* dst, hipStream_t stream) {
    unsigned* e = reinterpret_cast<unsigned*>(base) + XGMI_ERR_WORD;
    return (int)hipMemcpyAsync(dst, e, sizeof(unsigned), hipMemcpyDeviceToHost, stream);
}

extern "C" int dlms_xgmi_allreduce_f32(const XgmiArgs* a, hipStream_t stream) {
    if (int r = xgmi_check(a, a->n * 4)) return r;
    if (a->n % 4) return (int)hipErrorInvalidValue;
    const int grid = xgmi_blocks(a->n / 4);
    XGMI_DISPATCH(xgmi_allreduce_f32_kernel, a->world, grid, *a, stream);
    return (int)hipGetLastError();
}

extern "C" int dlms_xgmi_allreduce_i64(const XgmiArgs* a, hipStream_t stream) {
    if (int r = xgmi_check(a, a->n * 8)) return r;
    if (a->n % 2) return (int)hipErrorInvalidValue;
    const int grid = xgmi_blocks(a->n / 2);
    XGMI_DISPATCH(xgmi_allreduce_i64_kernel, a->world, grid, *a, stream);
    return (int)hipGetLastError();
}

extern "C" int dlms_xgmi_allgather_u64(const XgmiArgs* a, hipStream_t stream) {
    if (int r = xgmi_check(a, a->n * 8)) return r;
    const int grid = xgmi_blocks(a->n);
    XGMI_DISPATCH(xgmi_allgather_u64_kernel, a->world, grid, *a, stream);
    return (int)hipGetLastError();
}

extern "C" int dlms_xgmi_args_size() { return (int)sizeof(XgmiArgs); }
