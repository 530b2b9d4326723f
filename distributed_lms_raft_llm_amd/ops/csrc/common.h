// Shared device helpers for the CDNA4 (gfx950) kernel library.
// Wave = 64 lanes everywhere; bf16 is carried as raw ushort and converted in-register.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#define DLMS_WAVE 64

typedef unsigned short bf16_t;
typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // one 16x16x32 MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // one 16x16x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
    return __uint_as_float(((unsigned int)v) << 16);
}

// Round-to-nearest-even f32 -> bf16 (inputs are finite activations; NaN handling not needed
// on this path, but keep NaN a NaN anyway by forcing the quiet bit).
// f32 -> bf16, round to nearest even (NaN stays NaN): gfx950's v_cvt_pk_bf16_f32, one VALU op for
// two values.  (The integer rounding sequence it replaces compiled to ~18 instructions with an
// exec-mask branch per element: 1-1.5 us of every LayerNorm prologue at 32 rows.)  Same results
// for every finite input, f32 denormals included (HIP keeps them unflushed).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

__device__ __forceinline__ unsigned int pack_bf16x2(float lo, float hi) {
    typedef __bf16 bf16x2_hw_t __attribute__((ext_vector_type(2)));
    const bf16x2_hw_t v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(unsigned int, v);
}

// unpack 8 bf16 held in a uint4 into floats
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
    uint4 r;
    r.x = pack_bf16x2(f[0], f[1]); r.y = pack_bf16x2(f[2], f[3]);
    r.z = pack_bf16x2(f[4], f[5]); r.w = pack_bf16x2(f[6], f[7]);
    return r;
}

// Lane permute within 16-lane rows by DPP (a VALU operand modifier: no LDS round trip, unlike the
// ds_bpermute_b32 that __shfl_xor compiles to -- six of those per reduction sat on the critical path
// of every LayerNorm).  CTRL: 0xB1 quad_perm[1,0,3,2], 0x4E quad_perm[2,3,0,1], 0x141 row_half_mirror,
// 0x140 row_mirror.
template <int CTRL>
__device__ __forceinline__ float dpp_perm(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_perm_u64(unsigned long long v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned int)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned int)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
}

// v from lane (lane ^ o): DPP for o in {1, 2, 8} (quad_perm [1,0,3,2] / [2,3,0,1], row_ror:8 -- the
// same permutations, bit for bit), ds_bpermute otherwise.  o must fold to a constant.
__device__ __forceinline__ float xor_lane(float v, int o) {
    if (o == 1) return dpp_perm<0xB1>(v);
    if (o == 2) return dpp_perm<0x4E>(v);
    if (o == 8) return dpp_perm<0x128>(v);
    return __shfl_xor(v, o, 64);
}

// This lane's value and its lane ^ o partner's, as (x, y): for o in {16, 32} from one gfx950
// v_permlane{16,32}_swap (x = the lower row's / half's value, y = the upper's, the same pair in both
// partner lanes), otherwise x = own, y = partner (xor_lane).  Callers combine x and y symmetrically
// (sums, the online-softmax merge), which gives the same result as (own, partner) bit for bit.
__device__ __forceinline__ void lane_pair(float v, int o, float& x, float& y) {
    if (o == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        x = __uint_as_float(r[0]);
        y = __uint_as_float(r[1]);
    } else if (o == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        x = __uint_as_float(r[0]);
        y = __uint_as_float(r[1]);
    } else {
        x = v;
        y = xor_lane(v, o);
    }
}

// Sum over aligned 8-lane groups, in every lane of the group: bit-identical to the xor 1, 2, 4
// butterfly (after two steps every quad holds one value, so the half-row mirror pairs each lane
// with the other quad exactly as xor 4 does), without an LDS round trip.
__device__ __forceinline__ float group8_sum(float s) {
    s += dpp_perm<0xB1>(s);
    s += dpp_perm<0x4E>(s);
    s += dpp_perm<0x141>(s);
    return s;
}

// Max over each 16-lane row (xor 1, 2, 4, 8 butterfly by DPP; max is order-free)
__device__ __forceinline__ unsigned long long row16_max_u64(unsigned long long k) {
    unsigned long long o;
    o = dpp_perm_u64<0xB1>(k); k = o > k ? o : k;
    o = dpp_perm_u64<0x4E>(k); k = o > k ? o : k;
    o = dpp_perm_u64<0x141>(k); k = o > k ? o : k;
    o = dpp_perm_u64<0x128>(k); k = o > k ? o : k;
    return k;
}

__device__ __forceinline__ unsigned long long lane_value_u64(unsigned long long v, int lane) {
    const unsigned int lo = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)v, lane);
    const unsigned int hi = (unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)(v >> 32), lane);
    return ((unsigned long long)hi << 32) | lo;
}

// Max over the wave, the same value in every lane
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long k) {
    k = row16_max_u64(k);
    unsigned long long a = lane_value_u64(k, 0), b = lane_value_u64(k, 16);
    const unsigned long long c = lane_value_u64(k, 32), d = lane_value_u64(k, 48);
    a = b > a ? b : a;
    a = c > a ? c : a;
    return d > a ? d : a;
}

__device__ __forceinline__ float lane_value(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Full-wave reductions: butterflies inside each 16-lane row by DPP, then the four row results
// combined in a fixed order from scalar registers (the same value in every lane, deterministic).
// (the former ds_bpermute butterflies measured slower on every path: profiles/r2_sweep_dpp_reduce.jsonl)
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_perm<0xB1>(v);
    v += dpp_perm<0x4E>(v);
    v += dpp_perm<0x141>(v);
    v += dpp_perm<0x140>(v);
    return (lane_value(v, 0) + lane_value(v, 16)) + (lane_value(v, 32) + lane_value(v, 48));
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_perm<0xB1>(v));
    v = fmaxf(v, dpp_perm<0x4E>(v));
    v = fmaxf(v, dpp_perm<0x141>(v));
    v = fmaxf(v, dpp_perm<0x140>(v));
    return fmaxf(fmaxf(lane_value(v, 0), lane_value(v, 16)), fmaxf(lane_value(v, 32), lane_value(v, 48)));
}

__device__ __forceinline__ float gelu_tanh(float x) {
    const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
    const float k1 = 0.044715f;
    float u = k0 * (x + k1 * x * x * x);
    // 0.5 x (1 + tanh(u)) == x * sigmoid(2u) == x / (1 + e^(-2u)): one v_exp_f32 + one v_rcp_f32
    // instead of libm tanhf (~40 VALU ops: the GELU epilogue of the 32768-row prefill c_fc was
    // VALU-bound).  |rel err| ~1e-6 before the bf16 rounding of every consumer; e^(-2u) = inf for
    // very negative u gives x * 0 = -0, the limit.
    const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * u);  // e^(-2u) = 2^(-2u log2 e)
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f));
}

// Order-preserving map f32 -> u32 (larger float => larger unsigned).
__device__ __forceinline__ unsigned int f32_ordered(float f) {
    unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float f32_from_ordered(unsigned int o) {
    unsigned int u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    return __uint_as_float(u);
}

// argmax key: high 32 bits = ordered value (xor sign so the int64 compare is monotone),
// low 32 bits = ~index so that ties resolve to the LOWEST index (torch.argmax semantics).
__device__ __forceinline__ long long argmax_key(float v, int idx) {
    unsigned long long hi = (unsigned long long)(f32_ordered(v) ^ 0x80000000u);
    unsigned long long lo = (unsigned long long)(~(unsigned int)idx);
    return (long long)((hi << 32) | lo);
}

__device__ __forceinline__ int argmax_key_index(long long k) {
    return (int)(~(unsigned int)((unsigned long long)k & 0xffffffffull));
}

// XCD-aware bijective remap of a linear block id so that consecutive logical tiles land on one
// XCD (8 XCDs, private L2 each; dispatch is round-robin over XCDs).  Speed only, never needed
// for correctness (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8;
    const int xcd = orig % 8;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + orig / 8;
}

// ------------------------------------------------------------------ checked (debug) build
// libdlms_hip_checked.so is compiled with -DDLMS_DEVICE_CHECKS=1 (ops.build(checked=True), used
// when DLMS_KERNEL_CHECKS=1): every data-dependent index a kernel reads from a tensor (token ids,
// positions, KV slots, sequence lengths) is range-checked on the device.  A violation is recorded
// (first site / value / bound + a count) and the index is clamped to 0, so a bad input never
// becomes an out-of-bounds access that could fault the GPU; the host reads the record with
// dlms_check_<unit>() (ops.device_errors()).  The production build compiles the checks away.
#ifndef DLMS_DEVICE_CHECKS
#define DLMS_DEVICE_CHECKS 0
#endif

enum {
    CHK_EMBED_TOKEN = 1, CHK_EMBED_POS = 2, CHK_UPDATE_SLOT = 3, CHK_UPDATE_TOKEN = 4, CHK_UPDATE_LEN = 5,
    CHK_SEEN_ROW = 6, CHK_QKV_SLOT = 7, CHK_QKV_POS = 8, CHK_ATTN_SLOT = 9, CHK_BERT_TOKEN = 10,
    CHK_SEEN_TOKEN = 11,
};

struct DlmsCheckRecord {
    unsigned int count;
    int site;
    long long value;
    long long bound;
};

// one record per translation unit (the library is built without relocatable device code)
static __device__ DlmsCheckRecord dlms_check_rec;

// v if 0 <= v < bound; otherwise (checked build) record the violation and return 0
__device__ __forceinline__ long long dlms_idx(long long v, long long bound, int site) {
#if DLMS_DEVICE_CHECKS
    if (v < 0 || v >= bound) {
        if (atomicAdd(&dlms_check_rec.count, 1u) == 0) {
            dlms_check_rec.site = site;
            dlms_check_rec.value = v;
            dlms_check_rec.bound = bound;
        }
        return 0;
    }
#else
    (void)bound;
    (void)site;
#endif
    return v;
}

#define DLMS_CHECK_EXPORT(unit)                                                                     \
    extern "C" int dlms_check_##unit(int clear, DlmsCheckRecord* out) {                             \
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(dlms_check_rec), sizeof(DlmsCheckRecord)); \
        if (e != hipSuccess || !clear) return (int)e;                                               \
        const DlmsCheckRecord zero = {0, 0, 0, 0};                                                  \
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(dlms_check_rec), &zero, sizeof(DlmsCheckRecord));  \
    }

// Epilogue parameters of the MFMA GEMM (gemm.hip).  Mirrored field-for-field by the ctypes
// binding (ops/__init__.py); dlms_gemm_epi_size() lets Python assert the layouts agree.
struct GemmEpi {
    const float* bias;   // [N] or nullptr
    void* out;           // bf16 or f32 output
    int ldo;
    const float* resid;  // f32 residual (EPI_F32) or nullptr
    int ldr;
    // EPI_QKV
    bf16_t* q_out;
    int ldq;
    bf16_t* k_cache;
    bf16_t* v_cache;
    const int* row_slot;
    const int* row_pos;
    int n_heads;
    int t_max;
    int d_local;
    // EPI_ARGMAX
    unsigned long long* argmax_out;
    const unsigned int* seen;
    int seen_words;
    int vocab;       // number of valid global vocab ids
    int col_offset;  // global id of local column 0 (vocab-parallel shards)
    float penalty;
    // split-K (EPI_PARTIAL): the grid carries split_k K-slices; slice s writes its fp32 partial tile
    // at out + s * split_stride (elements).  Summed later by the fused add+LayerNorm kernel.
    int split_k;
    long long split_stride;
    // fp8 inputs (dlms_gemm_fp8): per-row activation and per-output-channel weight scales
    const float* a_scale;
    const float* w_scale;
    int n_slots;  // EPI_QKV: KV-cache slots (the checked build range-checks row_slot against it)
};

// Opt a kernel into > 64 KiB of dynamic LDS on the CURRENT device, once per (call site, device):
// the attribute is per device, so a process-wide "done" flag would skip it on a second GPU.  A
// race between two first launches only sets the attribute twice (idempotent).
inline hipError_t lds_opt_in(std::atomic<uint64_t>& done_mask, const void* func, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done_mask.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(func, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done_mask.fetch_or(bit, std::memory_order_acq_rel);
    return e;
}
