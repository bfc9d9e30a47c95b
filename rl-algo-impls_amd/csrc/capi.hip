// ABI introspection and error strings for the C boundary (include/rai_amd.h).
#include "common.h"

extern "C" int rai_abi_version(void) { return RAI_ABI_VERSION; }

extern "C" const char* rai_strerror(int code) {
  switch (code) {
    case RAI_OK: return "ok";
    case RAI_E_NULLPTR: return "null pointer argument";
    case RAI_E_SHAPE: return "invalid shape argument";
    case RAI_E_MODE: return "invalid mode argument";
    case RAI_E_TOO_MANY_COLUMNS: return "K exceeds RAI_MAX_K";
    case RAI_E_WORKSPACE: return "workspace too small";
    case RAI_E_UNSUPPORTED: return "unsupported configuration";
    default: break;
  }
  if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
  if (code <= RAI_E_DP_BASE) return "RCCL call failed (ncclResult_t = RAI_E_DP_BASE - code)";
  return "unknown error";
}
