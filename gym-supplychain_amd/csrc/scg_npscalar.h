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

enum NpKind : int {
  NK_INT = 0,  // Python int   (weak)
  NK_PYF = 1,  // Python float (weak float64)
  NK_F32 = 2,  // np.float32
  NK_F64 = 3,  // np.float64
  NK_I64 = 4   // np.int64
};

struct Num {
  double v;
  int k;
};

__host__ __device__ __forceinline__ Num pyint(double v) { return Num{v, NK_INT}; }
__host__ __device__ __forceinline__ Num f64(double v) { return Num{v, NK_F64}; }

// Result kind of a binary arithmetic op (NEP 50: Python scalars adopt the other side's
// dtype kind when it is a NumPy scalar; int64 with any float is float64). Written as
// selects, not branches: kinds are per-lane data, and on the GPU a branch on them costs
// exec-mask bookkeeping even when every lane agrees.
__host__ __device__ __forceinline__ int np_promote(int a, int b) {
  const int lo = a < b ? a : b, hi = a < b ? b : a;
  const int pyf = hi == NK_I64 ? NK_F64 : hi;
  const int r = lo == NK_INT ? hi : (lo == NK_PYF ? pyf : NK_F64);
  return a == b ? a : r;
}

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

// True division: int/int -> Python float, int64/int -> float64.
__host__ __device__ __forceinline__ Num np_div(Num a, Num b) {
  int k = np_promote(a.k, b.k);
  if (k == NK_INT) k = NK_PYF;
  if (k == NK_I64) k = NK_F64;
  if (k == NK_F32) return Num{static_cast<double>(static_cast<float>(a.v) / static_cast<float>(b.v)), k};
  return Num{a.v / b.v, k};
}

__host__ __device__ __forceinline__ Num np_neg(Num a) { return Num{-a.v, a.k}; }

// Comparisons: a float32 against a Python scalar compares in float32 (the Python value
// is cast); every other pairing compares the exact values.
__host__ __device__ __forceinline__ bool np_f32_cmp(const Num& a, const Num& b) {
  return (a.k == NK_F32 && (b.k == NK_INT || b.k == NK_PYF)) || (b.k == NK_F32 && (a.k == NK_INT || a.k == NK_PYF));
}

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

}  // namespace scg
