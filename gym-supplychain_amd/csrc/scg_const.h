// Launch-uniform read-only tables (SupplyChain node records, Poisson / lead-time threshold
// and sinusoid tables) are read through the constant address space on the device: a
// wave-uniform index into one becomes a scalar load through the scalar cache, which the
// compiler batches, instead of a vector load that waits on vmcnt before every use (the
// compiler cannot prove a plain pointer unwritten, so it never picks a scalar load for
// one). Scalar loads also count on lgkmcnt, not vmcnt, so they do not queue behind a
// kernel's row loads. No kernel writes these tables, so the non-coherent scalar cache is
// safe. On the host the qualifier is empty.
#pragma once

#include <hip/hip_runtime.h>

#if defined(__HIP_DEVICE_COMPILE__)
#define SCG_CONST_AS __attribute__((address_space(4)))
#else
#define SCG_CONST_AS
#endif

namespace scg {

template <class T>
using ConstTab = const SCG_CONST_AS T*;

template <class T>
__host__ __device__ __forceinline__ ConstTab<T> const_tab(const T* p) {
  return (ConstTab<T>)p;
}

}  // namespace scg
