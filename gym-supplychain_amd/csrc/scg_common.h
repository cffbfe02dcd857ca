// Shared host helpers of libscgpu.so: the thread-local error message behind
// scg_last_error() and HIP launch checks.
#pragma once

namespace scg {

// Record a printf-style message for scg_last_error() and return `code`.
int fail(int code, const char* fmt, ...);

// SCG_ERR_HIP (with the HIP error string) if the last launch failed, else SCG_OK.
int check_launch(const char* what);

}  // namespace scg
