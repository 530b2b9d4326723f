// Library-level entry points (version/arch probe, error strings) for the ctypes binding.
#include "common.h"

extern "C" const char* dlms_error_string(int err) { return hipGetErrorString((hipError_t)err); }

extern "C" int dlms_abi_version() { return 1; }

// Size of the GemmEpi struct as compiled, so the Python binding can assert its mirror matches.
extern "C" int dlms_gemm_epi_size() { return (int)sizeof(GemmEpi); }
