// Error reporting and version entry points of libscgpu.so (include/scgpu.h).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
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

// STREAM copy for the measured HBM peak (bench.py roofline.measured_peak). The copy shapes
// measured on MI355X (tools/copy_probe.hip, profiles/r03b_copy_probe.log, 1 GiB): one
// 16-byte vector per lane with a grid covering the buffer, non-temporal, 6.59 TB/s (plain
// 6.25); the same with 2-4 vectors per lane 6.05-6.43; grid-stride loops with 4 loads in
// flight per lane 4.6-5.3 whatever the grid. blocks == 0 launches the first shape, blocks > 0
// the grid-stride loop over that many workgroups.
constexpr int kCopyBlock = 256;
typedef int v4i __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kCopyBlock) void stream_copy_kernel(const v4i* __restrict__ src, v4i* __restrict__ dst,
                                                                 int64_t n16) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kCopyBlock + threadIdx.x;
  if (i < n16) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

__global__ __launch_bounds__(kCopyBlock) void stream_copy_stride_kernel(const v4i* __restrict__ src,
                                                                        v4i* __restrict__ dst, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kCopyBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kCopyBlock + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

}  // namespace scg

extern "C" {

int scg_stream_copy(const void* src, void* dst, int64_t bytes, int32_t blocks, void* stream) {
  if (!src || !dst || bytes <= 0 || bytes % 16 != 0 || blocks < 0)
    return scg::fail(SCG_ERR_INVALID, "stream_copy needs non-null buffers, bytes > 0 and a multiple of 16, blocks >= 0");
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16 != 0)
    return scg::fail(SCG_ERR_INVALID, "stream_copy buffers must be 16-byte aligned");
  const int64_t n16 = bytes / 16;
  const int64_t grid = blocks > 0 ? blocks : (n16 + scg::kCopyBlock - 1) / scg::kCopyBlock;
  if (grid > 0x7fffffff) return scg::fail(SCG_ERR_INVALID, "stream_copy: %lld bytes need blocks > 0", (long long)bytes);
  hipLaunchKernelGGL(blocks > 0 ? scg::stream_copy_stride_kernel : scg::stream_copy_kernel, dim3(static_cast<unsigned>(grid)),
                     dim3(scg::kCopyBlock), 0, static_cast<hipStream_t>(stream), static_cast<const scg::v4i*>(src),
                     static_cast<scg::v4i*>(dst), n16);
  return scg::check_launch("stream_copy_kernel");
}

int scg_abi_version(void) { return SCG_ABI_VERSION; }

const char* scg_last_error(void) { return scg::last_error(); }

}  // extern "C"
