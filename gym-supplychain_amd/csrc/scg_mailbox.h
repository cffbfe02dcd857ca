// The step servers' mailbox protocol (include/scgpu.h scg_bg_server_*, scg_sc_server_*),
// shared by the BeerGame and SupplyChain servers: a request is one (or two) 64-byte lines of
// host-mapped memory, 16 (32) words, word 7 a mixing hash of the others (multiply, xor and
// rotate per word), so a read of the lines that mixes two requests is detected whatever the
// words' differences; and the host's clock and spin hint.
#pragma once

#include <cstdint>
#include <ctime>

namespace scg {

template <int N>
__host__ __device__ inline uint32_t mailbox_check(const uint32_t (&w)[N]) {
  uint32_t h = 0x9E3779B9u;
  for (int i = 0; i < N; ++i) {
    if (i == 7) continue;
    h ^= w[i] * 0x85EBCA6Bu + static_cast<uint32_t>(i);
    h = (h << 13) | (h >> 19);
    h = h * 5u + 0xE6546B64u;
  }
  h ^= h >> 16;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 13);
}

inline int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000 + ts.tv_nsec;
}

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

}  // namespace scg
