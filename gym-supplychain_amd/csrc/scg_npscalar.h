// NumPy-2 scalar semantics (NEP 50) for the SupplyChain step, __host__ __device__.
//
// SupplyChainEnv's arithmetic mixes Python ints (capacities, costs), np.float32 (actions
// and everything derived from them), np.float64 (stock) and np.int64 (demand), and the
// result type of each operation decides whether it is rounded to float32 (SURVEY F10;
// e.g. supply amount = np.float32 action * int capacity, supplychain_env.py:56, is a
// float32; a ship amount is float32 or float64 depending on whether min(capacity, stock)
// returned the int or the float, :61-64). To reproduce the reference's values bit for
// bit, every scalar carries its NumPy kind and each operation promotes and rounds like
// NumPy does. Values are held in a double: every float32, and every integer below 2^53,
// is exact in it.
#pragma once

#include <hip/hip_runtime.h>

namespace scg {

// Kind codes form a bit lattice, so NEP 50 promotion is one bitwise OR (np_promote):
// Python scalars adopt the other side's kind, float32 with float64 or int64 is float64,
// Python float with int64 is float64. float64 has two codes, 7 and 5 (= PYF | I64); every
// test below treats them alike, and ABI-facing kinds go through np_kind_abi/np_kind_int.
enum NpKind : int {
  NK_INT = 0,  // Python int   (weak)
  NK_PYF = 1,  // Python float (weak float64)
  NK_F32 = 3,  // np.float32
  NK_F64 = 7,  // np.float64 (also 5)
  NK_I64 = 4   // np.int64
};

struct Num {
  double v;
  int k;
};

__host__ __device__ __forceinline__ Num pyint(double v) { return Num{v, NK_INT}; }
__host__ __device__ __forceinline__ Num f64(double v) { return Num{v, NK_F64}; }

// Result kind of a binary arithmetic op. A select-free OR: kinds are per-lane data, and on
// the GPU every select or branch on them is an instruction in each scalar operation.
__host__ __device__ __forceinline__ int np_promote(int a, int b) { return a | b; }

// The ABI's kind numbering (scgpu.h ledger_kind: 0 int, 1 float, 2 float32, 3 float64,
// 4 int64) to and from the lattice codes.
__host__ __device__ __forceinline__ int np_kind_abi(int k) { return k == NK_F32 ? 2 : ((k & 5) == 5 ? 3 : k); }
__host__ __device__ __forceinline__ int np_kind_int(int a) { return a == 2 ? NK_F32 : (a == 3 ? NK_F64 : a); }

// float32 rounding of an operation whose NumPy result kind is float32: operands are cast
// to float32 (exact for float32 values, round-to-nearest for Python scalars), then the
// operation is done in float32. Both roundings are computed and the kind selects one.
__host__ __device__ __forceinline__ Num np_add(Num a, Num b) {
  const int k = np_promote(a.k, b.k);
  const double r32 = static_cast<double>(static_cast<float>(a.v) + static_cast<float>(b.v));
  const double r64 = a.v + b.v;
  return Num{k == NK_F32 ? r32 : r64, k};
}

__host__ __device__ __forceinline__ Num np_sub(Num a, Num b) {
  const int k = np_promote(a.k, b.k);
  const double r32 = static_cast<double>(static_cast<float>(a.v) - static_cast<float>(b.v));
  const double r64 = a.v - b.v;
  return Num{k == NK_F32 ? r32 : r64, k};
}

__host__ __device__ __forceinline__ Num np_mul(Num a, Num b) {
  const int k = np_promote(a.k, b.k);
  const double r32 = static_cast<double>(static_cast<float>(a.v) * static_cast<float>(b.v));
  const double r64 = a.v * b.v;
  return Num{k == NK_F32 ? r32 : r64, k};
}

// True division: int/int -> Python float, int64/int -> float64: the kind OR 1 (0 -> 1,
// 4 -> 5; float kinds keep theirs).
__host__ __device__ __forceinline__ Num np_div(Num a, Num b) {
  const int k = np_promote(a.k, b.k) | NK_PYF;
  if (k == NK_F32) return Num{static_cast<double>(static_cast<float>(a.v) / static_cast<float>(b.v)), k};
  return Num{a.v / b.v, k};
}

__host__ __device__ __forceinline__ Num np_neg(Num a) { return Num{-a.v, a.k}; }

// Comparisons: a float32 against a Python scalar compares in float32 (the Python value
// is cast); every other pairing compares the exact values. Two float32 values compare the
// same either way (both exact in a double), so "the kinds OR to float32" is the test.
__host__ __device__ __forceinline__ bool np_f32_cmp(const Num& a, const Num& b) { return (a.k | b.k) == NK_F32; }

__host__ __device__ __forceinline__ bool np_lt(Num a, Num b) {
  const bool c32 = static_cast<float>(a.v) < static_cast<float>(b.v);
  return np_f32_cmp(a, b) ? c32 : a.v < b.v;
}

__host__ __device__ __forceinline__ bool np_eq(Num a, Num b) {
  const bool c32 = static_cast<float>(a.v) == static_cast<float>(b.v);
  return np_f32_cmp(a, b) ? c32 : a.v == b.v;
}

// Python's builtin min(a, b): b if b < a else a (keeps the chosen operand's kind).
__host__ __device__ __forceinline__ Num py_min(Num a, Num b) { return np_lt(b, a) ? b : a; }

// The same operations where the caller knows that no promoted kind in the region is float32
// (kNo32: the operands are float64, Python or int64 scalars, or a float32 meeting a float64):
// then each is the plain double operation with the promoted kind, and a comparison is the
// exact one — one instruction where the kind-generic form computes both roundings and
// selects. Identical values and kinds.
template <bool kNo32>
__host__ __device__ __forceinline__ Num np_add_k(Num a, Num b) {
  if constexpr (kNo32) return Num{a.v + b.v, np_promote(a.k, b.k)};
  return np_add(a, b);
}
template <bool kNo32>
__host__ __device__ __forceinline__ Num np_sub_k(Num a, Num b) {
  if constexpr (kNo32) return Num{a.v - b.v, np_promote(a.k, b.k)};
  return np_sub(a, b);
}
template <bool kNo32>
__host__ __device__ __forceinline__ Num np_mul_k(Num a, Num b) {
  if constexpr (kNo32) return Num{a.v * b.v, np_promote(a.k, b.k)};
  return np_mul(a, b);
}
template <bool kNo32>
__host__ __device__ __forceinline__ Num np_div_k(Num a, Num b) {
  if constexpr (kNo32) return Num{a.v / b.v, np_promote(a.k, b.k) | NK_PYF};
  return np_div(a, b);
}
template <bool kNo32>
__host__ __device__ __forceinline__ bool np_lt_k(Num a, Num b) {
  if constexpr (kNo32) return a.v < b.v;
  return np_lt(a, b);
}

// True when every active lane of the wave has `p` (the host build runs one env: p itself).
// A kind test made wave-uniform this way picks one instantiation for the whole wave.
__host__ __device__ __forceinline__ bool wave_all(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
  return __all(p);
#else
  return p;
#endif
}

}  // namespace scg
