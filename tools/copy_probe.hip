// HBM copy-bandwidth probe: which copy shape measures the achievable peak that bench.py
// reports as roofline.measured_peak (scg_stream_copy). Standalone; build and run:
//   hipcc --offload-arch=gfx950 -O3 -o tools/copy_probe tools/copy_probe.hip && tools/copy_probe
// Prints GB/s (read + write bytes / time, 20 back-to-back launches) per variant and size.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

// one 16-byte vector per lane, grid covers the buffer
template <bool NT>
__global__ __launch_bounds__(256) void copy_one(const v4i* __restrict__ s, v4i* __restrict__ d, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  if (NT)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
  else
    d[i] = s[i];
}

// U vectors per lane, block-contiguous chunks of U * 256 vectors (all loads issued first)
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk(const v4i* __restrict__ s, v4i* __restrict__ d, int64_t n) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * (U * 256) + threadIdx.x;
  v4i v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n) {
      if (NT)
        __builtin_nontemporal_store(v[u], d + i);
      else
        d[i] = v[u];
    }
  }
}

// grid-stride, 4 loads in flight per lane (the round-2 scg_stream_copy shape)
template <bool NT>
__global__ __launch_bounds__(256) void copy_stride(const v4i* __restrict__ s, v4i* __restrict__ d, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    v4i a, b, c, e;
    if (NT) {
      a = __builtin_nontemporal_load(s + i);
      b = __builtin_nontemporal_load(s + i + stride);
      c = __builtin_nontemporal_load(s + i + 2 * stride);
      e = __builtin_nontemporal_load(s + i + 3 * stride);
      __builtin_nontemporal_store(a, d + i);
      __builtin_nontemporal_store(b, d + i + stride);
      __builtin_nontemporal_store(c, d + i + 2 * stride);
      __builtin_nontemporal_store(e, d + i + 3 * stride);
    } else {
      a = s[i]; b = s[i + stride]; c = s[i + 2 * stride]; e = s[i + 3 * stride];
      d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

template <class F>
double time_gbs(F launch, int64_t bytes, int iters = 20) {
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int k = 0; k < iters; ++k) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 2.0 * bytes / (ms / iters * 1e-3) / 1e9;
}

int main() {
  const int64_t sizes[] = {int64_t(1) << 30, int64_t(4) << 30};
  for (int64_t bytes : sizes) {
    v4i *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 7, bytes));
    const int64_t n = bytes / 16;
    const unsigned g1 = static_cast<unsigned>((n + 255) / 256);
    printf("size %lld MiB\n", (long long)(bytes >> 20));
    printf("  one/plain        %8.0f GB/s\n", time_gbs([&] { copy_one<false><<<g1, 256>>>(s, d, n); }, bytes));
    printf("  one/nt           %8.0f GB/s\n", time_gbs([&] { copy_one<true><<<g1, 256>>>(s, d, n); }, bytes));
#define CH(U, NT)                                                                                               \
  printf("  chunk%-2d/%-5s     %8.0f GB/s\n", U, NT ? "nt" : "plain",                                          \
         time_gbs([&] { copy_chunk<U, NT><<<static_cast<unsigned>((n + U * 256 - 1) / (U * 256)), 256>>>(s, d, n); }, \
                  bytes));
    CH(2, false) CH(4, false) CH(8, false) CH(2, true) CH(4, true) CH(8, true)
    for (int per_cu : {8, 16, 32, 64}) {
      const unsigned g = 256 * per_cu;
      printf("  stride%2d/plain   %8.0f GB/s\n", per_cu, time_gbs([&] { copy_stride<false><<<g, 256>>>(s, d, n); }, bytes));
      printf("  stride%2d/nt      %8.0f GB/s\n", per_cu, time_gbs([&] { copy_stride<true><<<g, 256>>>(s, d, n); }, bytes));
    }
    CK(hipFree(s));
    CK(hipFree(d));
  }
  return 0;
}
