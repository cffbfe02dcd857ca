// CPython heapq on fixed-capacity arrays, __host__ __device__.
//
// SupplyChainEnv keeps every node's in-transit material as a heapq list of
// (time, amount) tuples (supplychain_env.py:398-400, pops :222-225) and its observation
// walks that list in STORAGE order, as if it were sorted (:445-461; SURVEY F9: on the
// 2-per-stage chain 328 of 360 observations differ from a time-sorted binning). So the
// storage order is part of the observable state, and this is a restatement of CPython's
// heappush / heappop / _siftdown / _siftup (Lib/heapq.py, the same algorithm as the C
// accelerator _heapq.c) over an array, with Python's tuple ordering: compare times, and
// only when they are equal compare the amounts with NumPy scalar semantics.
//
// Layout: entry j of a heap lives at index j*stride of `tk` (time << 3 | NumPy kind) and
// `val` (amount as double), so env-major strided heaps of many envs can share arrays. The
// functions below take any view type with get / put / time_at (HeapView here; the staged
// kernel's byte-packed HeapView8 in scg_supplychain_staged.h).
#pragma once

#include "scg_npscalar.h"

namespace scg {

struct HeapEntry {
  int32_t tk;  // time << 3 | kind
  double v;
};

__host__ __device__ __forceinline__ int32_t he_time(int32_t tk) { return tk >> 3; }
__host__ __device__ __forceinline__ int he_kind(int32_t tk) { return tk & 7; }
__host__ __device__ __forceinline__ int32_t he_pack(int32_t time, int kind) { return (time << 3) | kind; }

// Python tuple (t1, a1) < (t2, a2): times first; on equal times the amounts (equal amounts
// are not less, and np_lt already says so). Evaluated without branches: inside a sift loop
// each early return was a divergent branch with its exec-mask bookkeeping.
//
// kPlain: the caller knows that neither entry is a Python int or float (kind codes 0 and 1).
// NumPy compares at float32 precision only when the kinds OR to float32, i.e. a float32
// against a float32 (both exact in a double: the same answer as comparing the doubles) or
// against a Python scalar; without the latter the tuple order is the doubles' order, one
// compare instead of the kind lattice's conversions and selects.
template <bool kPlain = false>
__host__ __device__ __forceinline__ bool he_less(const HeapEntry& x, const HeapEntry& y) {
  const int32_t tx = he_time(x.tk), ty = he_time(y.tk);
  if constexpr (kPlain) return (tx < ty) | ((tx == ty) & (x.v < y.v));
  const Num ax{x.v, he_kind(x.tk)}, ay{y.v, he_kind(y.tk)};
  return (tx < ty) | ((tx == ty) & np_lt(ax, ay));
}

// An entry he_less<true> may compare: its kind is neither a Python int nor a Python float.
__host__ __device__ __forceinline__ bool he_plain(int32_t tk) { return (tk & 6) != 0; }

struct HeapView {
  int32_t* tk;
  double* val;
  int64_t stride;

  __host__ __device__ __forceinline__ HeapEntry get(int i) const { return HeapEntry{tk[i * stride], val[i * stride]}; }
  __host__ __device__ __forceinline__ void put(int i, const HeapEntry& e) const {
    tk[i * stride] = e.tk;
    val[i * stride] = e.v;
  }
  __host__ __device__ __forceinline__ int32_t time_at(int i) const { return he_time(tk[i * stride]); }
};

// heapq._siftdown(heap, startpos, pos) with the moving item (the entry at pos) held in
// registers: it is written once, at its final position. Every variant below keeps the
// entries being moved in registers the same way, so each heap slot is read once per sift
// level (the heap is in LDS in every kernel but the lane one on HBM heaps: these reads are
// a chain of dependent latencies).
template <bool kPlain = false, class HV>
__host__ __device__ inline void py_siftdown_item(const HV& h, int startpos, int pos, const HeapEntry& item) {
  while (pos > startpos) {
    const int parentpos = (pos - 1) >> 1;
    const HeapEntry parent = h.get(parentpos);
    if (he_less<kPlain>(item, parent)) {
      h.put(pos, parent);
      pos = parentpos;
      continue;
    }
    break;
  }
  h.put(pos, item);
}

template <class HV>
__host__ __device__ inline void py_siftdown(const HV& h, int startpos, int pos) {
  py_siftdown_item(h, startpos, pos, h.get(pos));
}

// heapq._siftup(heap, pos) for `item` standing at pos: move the smaller child up to a leaf,
// then sift the item down from there (CPython's bottom-up variant).
template <class HV>
__host__ __device__ inline void py_siftup_item(const HV& h, int size, int pos, const HeapEntry& item) {
  const int startpos = pos;
  int childpos = 2 * pos + 1;
  while (childpos < size) {
    const int rightpos = childpos + 1;
    HeapEntry child = h.get(childpos);
    if (rightpos < size) {
      const HeapEntry right = h.get(rightpos);
      if (!he_less(child, right)) {
        childpos = rightpos;
        child = right;
      }
    }
    h.put(pos, child);
    pos = childpos;
    childpos = 2 * pos + 1;
  }
  py_siftdown_item(h, startpos, pos, item);
}

template <class HV>
__host__ __device__ inline void py_siftup(const HV& h, int size, int pos) {
  py_siftup_item(h, size, pos, h.get(pos));
}

// heapq.heappop on a non-empty heap whose root the caller holds in registers (`root` =
// heap[0]); returns the popped entry and leaves the new heap[0] in `root` (defined when the
// heap is not empty afterwards), so a loop of pops reads no slot twice: the bottom-up
// sift's first move puts the smaller child at the root, and the re-seated last entry lands
// there only if it climbs all the way back.
template <bool kPlain = false, class HV>
__host__ __device__ inline HeapEntry py_heappop_root(const HV& h, int32_t& size, HeapEntry& root) {
  --size;
  const HeapEntry last = h.get(size);
  const HeapEntry ret = root;
  if (size == 0) return last;
  int pos = 0, childpos = 1;
  bool moved = false;
  while (childpos < size) {
    const int rightpos = childpos + 1;
    HeapEntry child = h.get(childpos);
    if (rightpos < size) {
      const HeapEntry right = h.get(rightpos);
      if (!he_less<kPlain>(child, right)) {
        childpos = rightpos;
        child = right;
      }
    }
    h.put(pos, child);
    if (!moved) root = child;
    moved = true;
    pos = childpos;
    childpos = 2 * pos + 1;
  }
  while (pos > 0) {  // _siftdown(heap, 0, pos) of `last`
    const int parentpos = (pos - 1) >> 1;
    const HeapEntry parent = h.get(parentpos);
    if (he_less<kPlain>(last, parent)) {
      h.put(pos, parent);
      pos = parentpos;
      continue;
    }
    break;
  }
  h.put(pos, last);
  if (pos == 0) root = last;
  return ret;
}

// heapq.heappush. Returns false (and pushes nothing) when the heap is full.
template <class HV>
__host__ __device__ inline bool py_heappush(const HV& h, int32_t& size, int cap, const HeapEntry& e) {
  if (size >= cap) return false;
  ++size;
  py_siftdown_item(h, 0, size - 1, e);  // heap.append(e); _siftdown(heap, 0, len - 1)
  return true;
}

// heapq.heappop on a non-empty heap.
template <class HV>
__host__ __device__ inline HeapEntry py_heappop(const HV& h, int32_t& size) {
  --size;
  const HeapEntry last = h.get(size);
  if (size > 0) {
    const HeapEntry ret = h.get(0);
    py_siftup_item(h, size, 0, last);  // heap[0] = last; _siftup(heap, 0)
    return ret;
  }
  return last;
}

}  // namespace scg
