// Error reporting and version entry points of libscgpu.so (include/scgpu.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "scg_common.h"
#include "scgpu.h"

namespace scg {

namespace {
thread_local char g_err[512] = "";
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SCG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return SCG_OK;
}

const char* last_error() { return g_err; }

}  // namespace scg

extern "C" {

int scg_abi_version(void) { return SCG_ABI_VERSION; }

const char* scg_last_error(void) { return scg::last_error(); }

}  // extern "C"
