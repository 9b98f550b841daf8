// ABI housekeeping (status strings, device count).
#include "bo_common.h"

extern "C" {

int bo_abi_version(void) { return BO_ABI_VERSION; }

const char* bo_status_string(int s) {
  switch (s) {
    case BO_OK: return "ok";
    case BO_ERR_ARG: return "invalid argument";
    case BO_ERR_UNSUPPORTED: return "unsupported configuration";
    case BO_ERR_WORKSPACE: return "workspace missing or too small";
    case BO_ERR_HIP: return "HIP runtime error";
    case BO_ERR_NOT_PD: return "Matrix is not positive definite";
    case BO_ERR_SINGULAR: return "Singular matrix";
    default: return "unknown status";
  }
}

int bo_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

}  // extern "C"
