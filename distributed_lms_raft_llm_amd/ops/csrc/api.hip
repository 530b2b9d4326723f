// Library-level entry points (version/arch probe, error strings) for the ctypes binding.
#include "common.h"

extern "C" const char* dlms_error_string(int err) { return hipGetErrorString((hipError_t)err); }

extern "C" int dlms_abi_version() { return 1; }

// Size of the GemmEpi struct as compiled, so the Python binding can assert its mirror matches.
extern "C" int dlms_gemm_epi_size() { return (int)sizeof(GemmEpi); }

// A HIP stream whose kernels may only use ``n_cus`` compute units of the current device, spread
// evenly (every ``stride``-th CU in the driver's numbering, which interleaves the XCDs): spatial
// partitioning of the GPU between co-located services -- the relevance gate's encoder passes run on
// a few CUs while the tutor's latency-bound decode keeps the rest, so a decode kernel never waits
// for gate workgroups to drain.  *out receives the hipStream_t (wrapped by torch.cuda.ExternalStream).
#include <hip/hip_ext.h>
extern "C" hipError_t dlms_stream_create_cumask(int n_cus, void** out) {
    int dev = 0, total = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if (n_cus <= 0 || n_cus > total) return hipErrorInvalidValue;
    const int words = (total + 31) / 32;
    uint32_t mask[64] = {0};
    if (words > 64) return hipErrorInvalidValue;
    const int stride = total / n_cus;
    for (int k = 0; k < n_cus; ++k) {
        const int cu = k * stride;
        mask[cu / 32] |= 1u << (cu % 32);
    }
    hipStream_t s = nullptr;
    if ((e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask)) != hipSuccess) return e;
    *out = reinterpret_cast<void*>(s);
    return hipSuccess;
}

extern "C" hipError_t dlms_stream_destroy(void* s) { return hipStreamDestroy(reinterpret_cast<hipStream_t>(s)); }
