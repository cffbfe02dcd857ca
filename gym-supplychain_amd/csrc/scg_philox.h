// Philox4x32-10 counter-based RNG (Salmon et al., SC'11; Random123's published
// algorithm), __host__ __device__ so the C-ABI host helpers and the gfx950 kernels draw
// identical words. On device mulhi is one v_mul_hi_u32; the 10 rounds are fully unrolled
// into ~60 VALU ops, i.e. free next to the HBM traffic of a step.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace scg {

struct U4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return static_cast<uint32_t>((static_cast<uint64_t>(a) * b) >> 32);
#endif
}

__host__ __device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// Word j of the (env, tag, stream) sequence: philox(ctr=(env, tag, j/4, stream))[j%4].
__host__ __device__ __forceinline__ uint32_t philox_word(uint32_t k0, uint32_t k1, uint32_t env,
                                                         uint32_t tag, uint32_t j, uint32_t stream) {
  const U4 r = philox4x32_10(U4{env, tag, j >> 2, stream}, k0, k1);
  const uint32_t s = j & 3u;
  return s == 0 ? r.x : s == 1 ? r.y : s == 2 ? r.z : r.w;
}

}  // namespace scg
