// FETCH_SIZE / WRITE_SIZE calibration for the access shapes of this repo's kernels
// (MI355X_MICROARCH.md: only 16-B-per-lane streaming reads and writes are calibrated).
// Each kernel moves a known byte count over a 1 GiB buffer (past the 256 MiB Infinity
// Cache); run once per counter and compare the counter with the bytes printed here:
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -o pmc -- tools/pmc_calib
// Kernels:
//   rd<W>     every lane reads W bytes per instruction, coalesced (W = 4, 8, 16)
//   wr<W>     every lane writes W bytes per instruction, coalesced
//   wr_rows<O> 64 lanes write O consecutive 4-byte words each (row n*O + o, o = 0..O-1), one
//             store instruction per o: the per-env observation row pattern; the 64 rows cover
//             a contiguous 256*O-byte span per wave
//   rd_rows<A> the same pattern as loads (per-env action rows)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

template <class T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ s, int64_t n, int* __restrict__ sink) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const T v = s[i];
  const int* p = reinterpret_cast<const int*>(&v);
  int x = 0;
  for (unsigned k = 0; k < sizeof(T) / 4; ++k) x ^= p[k];
  if (x == 0x12345678) sink[0] = x;  // never true for the fill below: keeps the load
}

template <class T>
__global__ __launch_bounds__(256) void wr(T* __restrict__ d, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  T v;
  int* p = reinterpret_cast<int*>(&v);
  for (unsigned k = 0; k < sizeof(T) / 4; ++k) p[k] = static_cast<int>(i) + k;
  d[i] = v;
}

template <int O>
__global__ __launch_bounds__(256) void wr_rows(float* __restrict__ d, int64_t rows) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r >= rows) return;
#pragma unroll
  for (int o = 0; o < O; ++o) d[r * O + o] = static_cast<float>(o);
}

template <int A>
__global__ __launch_bounds__(256) void rd_rows(const float* __restrict__ s, int64_t rows, int* __restrict__ sink) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r >= rows) return;
  float x = 0.f;
#pragma unroll
  for (int o = 0; o < A; ++o) x += s[r * A + o];
  if (x == 1234.5f) sink[0] = 1;
}

int main() {
  const int64_t bytes = int64_t(1) << 30;
  char* buf;
  int* sink;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, bytes));
  auto grid = [](int64_t n) { return dim3(static_cast<unsigned>((n + 255) / 256)); };
  printf("kernel bytes\n");
  rd<int><<<grid(bytes / 4), 256>>>(reinterpret_cast<int*>(buf), bytes / 4, sink);
  printf("rd4 %lld\n", (long long)bytes);
  rd<int2><<<grid(bytes / 8), 256>>>(reinterpret_cast<int2*>(buf), bytes / 8, sink);
  printf("rd8 %lld\n", (long long)bytes);
  rd<int4><<<grid(bytes / 16), 256>>>(reinterpret_cast<int4*>(buf), bytes / 16, sink);
  printf("rd16 %lld\n", (long long)bytes);
  wr<int><<<grid(bytes / 4), 256>>>(reinterpret_cast<int*>(buf), bytes / 4);
  printf("wr4 %lld\n", (long long)bytes);
  wr<int2><<<grid(bytes / 8), 256>>>(reinterpret_cast<int2*>(buf), bytes / 8);
  printf("wr8 %lld\n", (long long)bytes);
  wr<int4><<<grid(bytes / 16), 256>>>(reinterpret_cast<int4*>(buf), bytes / 16);
  printf("wr16 %lld\n", (long long)bytes);
  const int64_t rows27 = bytes / (27 * 4), rows14 = bytes / (14 * 4);
  wr_rows<27><<<grid(rows27), 256>>>(reinterpret_cast<float*>(buf), rows27);
  printf("wr_rows27 %lld\n", (long long)(rows27 * 27 * 4));
  rd_rows<14><<<grid(rows14), 256>>>(reinterpret_cast<const float*>(buf), rows14, sink);
  printf("rd_rows14 %lld\n", (long long)(rows14 * 14 * 4));
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
