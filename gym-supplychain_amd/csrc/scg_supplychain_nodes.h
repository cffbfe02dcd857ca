// Node-parallel SupplyChainEnv.step: every node of an env acts at once, __host__ __device__.
//
// supplychain_env.py walks the nodes in nodes_info order (:714-736). What a node's act
// reads is its own stock and what its own heaps release at time t (:220-228); the pushes
// other nodes make into its heaps this step are due at t + lead time >= t + 1 (:347,
// lead times are >= 1), so they never change what it receives. Only the storage order of
// its heaps depends on them, and that order is rebuilt exactly afterwards. So a step is
//
//   stage    each heap (i, p) copied from HBM into fast memory, and the sum it releases
//            now computed WITHOUT popping (sc_recv_scan)
//   act      every node at once: stock += released, then the rest of SC_Node.act
//            (:230-396) with no heap access (kHeapsDone), shipments written to the
//            destinations' inbox entries (the staged kernel's layout, sources in node
//            order), the node's cost kept for the reward
//   heaps    every heap at once, the reference's operation order on it: the pushes
//            earlier nodes made (inbox, source order, :347), the pops due now (:222-225),
//            the node's own SUPPLY push (:254), then its in-transit bins (:445-461) and
//            the copy back
//   reward   -(sum of the node costs in node order) (:735-738)
//
// The released sum is the due amounts added in heappop order. Pops return a minimum under
// the tuple order; every due entry has the same time, so the order is by amount, and the
// heap's shape only decides between amounts neither of which is less than the other. Such
// amounts add to the same double unless NumPy compares them at float32 precision (a
// float32 against a Python scalar) while their doubles differ; sc_recv_scan reports that
// case, and the kernel then steps that env alone, node after node (sc_nodes_serial).
#pragma once

#include "scg_supplychain_core.h"

// The node-parallel kernel's streaming stores (the heap copy-back; at 2 also the stock and
// observation rows of the batch kernel) as write-through stores (sc1: the line leaves the
// L2 with the store instead of staying dirty until evicted or written back at the launch's
// end): sc-2perstage 37.2-37.5 -> 35.7-37.0 us, the two-product chain 86-88 -> 82-84 us
// (profiles/r06t_nodes_wt_ab*.log, r06u_*, r06v_*); 0 keeps the non-temporal stores.
#ifndef SCG_NODES_WT
#define SCG_NODES_WT 2
#endif

namespace scg {

__host__ __device__ __forceinline__ int sc_ctz64(uint64_t m) { return __builtin_ctzll(m); }

// Shipments into the destinations' inbox entries (scg_sc_node in_slot / in_stride, as the
// staged kernel's), entry q of this env at [q * stride]; one act per node, so the split
// runs in registers (MAXD-unrolled) and a store per destination.
struct NodesInbox {
  int32_t* tk;  // time << 3 | kind, -1 = no shipment
  double* val;
  int64_t stride;

  static constexpr bool kUnroll = true;
  static constexpr bool kUniformNode = true;  // a wave per node
  static constexpr bool kLdsSplit = false;
  static constexpr bool kVecActions = false;  // actions come from an LDS tile
  static constexpr bool kClearInAct = false;  // cleared before the act
  static constexpr bool kShipBits = false;
  __host__ __device__ Num scratch_get(int) const { return pyint(0); }
  __host__ __device__ void noship(const ScCtx&, int, int, int) const {}
  __host__ __device__ void noship_all(const ScCtx&, int, int) const {}
  __host__ __device__ __forceinline__ void ship(const ScCtx& c, ScEnv&, int src, int d, int /*dest*/, int p,
                                                int32_t time, Num amount) const {
    ScNode& nd = c.nodes[src];
    const int64_t q = nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d];
    tk[q * stride] = he_pack(time, amount.k);
    val[q * stride] = amount.v;
  }
  __host__ __device__ __forceinline__ void clear(const ScCtx& c, int src) const {
    ScNode& nd = c.nodes[src];
    for (int d = 0; d < nd.n_dests; ++d)
      for (int p = 0; p < c.P; ++p) tk[(nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d]) * stride] = -1;
  }
};

// What receive (:220-228) takes out of heap h at time t, without popping: the due entries
// added in heappop order (0.0 + a1 + a2 ..., the float64 array element of :225). Returns
// false when that order is not determined by the amounts (see the header), or when an entry
// is overdue (time < t: the reference's loop would stop at it), or the heap is wider than
// the 64-bit due mask.
__host__ __device__ inline bool sc_recv_scan(const HeapView& h, int32_t sz, int t, double& recv) {
  recv = 0.0;
  if (sz > 64) return false;
  uint64_t due = 0;
  bool ok = true;
  for (int j = 0; j < sz; ++j) {
    const int32_t tj = h.time_at(j);
    due |= static_cast<uint64_t>(tj == t) << j;
    ok &= tj >= t;
  }
  double r = 0.0;
  while (due) {
    int best = sc_ctz64(due);
    HeapEntry be = h.get(best);
    for (uint64_t m = due & (due - 1); m; m &= m - 1) {
      const int j = sc_ctz64(m);
      const HeapEntry x = h.get(j);
      if (he_less(x, be)) {
        best = j;
        be = x;
      }
    }
    due &= ~(uint64_t(1) << best);
    for (uint64_t m = due; m; m &= m - 1) {  // tied with the minimum (not greater) yet another double
      const HeapEntry x = h.get(sc_ctz64(m));
      ok &= he_less(be, x) | (x.v == be.v);
    }
    r = r + be.v;
  }
  recv = r;
  return ok;
}

// Heap copy of the stage phase, shared by the kernel (scg_sc_nodes.hip) and the host
// harness: the slots of heap view gh (HBM) with size sz into lh (LDS), kChunk at a time.
// The first chunk does not depend on sz (slots past the size are read and stored, never
// used), so it is requested together with the size — one memory round for a heap of at
// most kChunk entries — and a longer heap costs a round per further chunk.
#ifndef SCG_NODES_STAGE_CHUNK
#define SCG_NODES_STAGE_CHUNK 4
#endif
template <int kChunk = SCG_NODES_STAGE_CHUNK>
__host__ __device__ __forceinline__ void sc_nodes_copy_heap(const HeapView& gh, const HeapView& lh, int H, int32_t sz) {
  HeapEntry b[kChunk];
#pragma unroll
  for (int u = 0; u < kChunk; ++u)
    if (u < H) b[u] = gh.get(u);
#pragma unroll
  for (int u = 0; u < kChunk; ++u)
    if (u < H) lh.put(u, b[u]);
  for (int j0 = kChunk; j0 < sz; j0 += kChunk) {
#pragma unroll
    for (int u = 0; u < kChunk; ++u)
      if (j0 + u < sz) b[u] = gh.get(j0 + u);
#pragma unroll
    for (int u = 0; u < kChunk; ++u)
      if (j0 + u < sz) lh.put(j0 + u, b[u]);
  }
}

// stage: heap (i, p) from the env's state into `lh` (its size into lsz), and what it
// releases at t.
__host__ __device__ inline bool sc_nodes_stage(const ScCtx& c, const ScEnv& g, const HeapView& lh, int32_t& lsz,
                                               int t, int i, int p, double& recv) {
  const int32_t sz = sc_size(c, g, i, p);
  sc_nodes_copy_heap(sc_heap(c, g, i, p), lh, c.H, sz);
  lsz = sz;
  return sc_recv_scan(lh, sz, t, recv);
}

// act: node i receives (recv[p * rstride], from its stage) and acts; its heaps are not
// touched, its shipments go to the inbox. Returns the node's cost with its NumPy kind.
template <int MAXD, bool kKindPaths = false>
__host__ __device__ inline Num sc_nodes_act(const ScCtx& c, ScEnv& g, const NodesInbox& in, const double* recv,
                                            int64_t rstride, const float* act, int t, int i) {
  for (int p = 0; p < c.P; ++p) {
    double& st = sc_stock(c, g, i, p);
    st = st + recv[p * rstride];  // self.stock += arrived_material (:228)
  }
  if (!c.nodes[i].last_level) in.clear(c, i);
  sc_led_begin_node(c, g, i);
  SCG_ACCP(g.dbg, 7);
  WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
  return sc_node_act<MAXD, NodesInbox, true, kKindPaths>(c, g, ltc, dmc, i, act, t, in);
}

// heaps: everything heap (i, p), staged in `lh` with size sz, sees in step t, in the
// reference's order — the inbox pushes of earlier nodes in source order, the pops due now,
// the SUPPLY push (the supply-action index a_i and lead-time cursor lt_i advanced as act
// advances them, :243-259) — then its in-transit bins and the copy back to the env's state.
// The popped sum went into the stock already (sc_nodes_act), unless `receive`: then it is
// added here (:225-228), as the serial walk below needs.
// kStream (device): the copy back with non-temporal stores (written once per step, read
// next step: evict-first in the caches, so they do not push out what this step reads again).
template <bool kStream = false, class Sink>
__host__ __device__ inline void sc_nodes_heap(const ScCtx& c, ScEnv& g, const HeapView& lh, int32_t& sz,
                                              const NodesInbox& in, WordCache& ltc, const float* act, int t, int i,
                                              int p, int& a_i, int& lt_i, Sink& out, bool receive = false) {
  ScNode& nd = c.nodes[i];
  const int64_t q0 = nd.in_base + static_cast<int64_t>(p) * nd.in_deg;
  for (int k = 0; k < nd.in_deg; ++k) {  // in source order (:347)
    const HeapEntry e{in.tk[(q0 + k) * in.stride], in.val[(q0 + k) * in.stride]};
    if (e.tk >= 0 && !py_heappush(lh, sz, c.H, e)) g.overflow = 1;
  }
  SCG_ACCP(g.dbg, 0);
  if (receive) {
    double& st = sc_stock(c, g, i, p);
    st = st + sc_receive(lh, sz, t);
  } else if (sz > 0) {  // the root travels in registers from pop to pop (py_heappop_root)
    HeapEntry root = lh.get(0);
    while (sz > 0 && he_time(root.tk) == t) py_heappop_root(lh, sz, root);
  }
  SCG_ACCP(g.dbg, 1);
  if (nd.n_supply > 0 && nd.supply_capacity[p] > 0) {
    const Num amount = np_mul(sc_action(act, nd.action_offset + a_i), pyint(nd.supply_capacity[p]));
    ++a_i;
    if (np_lt(pyint(0), amount)) {
      const HeapEntry e{he_pack(t + node_leadtime(c, g, ltc, nd, t, lt_i), amount.k), amount.v};
      if (!py_heappush(lh, sz, c.H, e)) g.overflow = 1;
      ++lt_i;
    }
  }
  SCG_ACCP(g.dbg, 2);
  const HeapView gh = sc_heap(c, g, i, p);
  sc_observe_bins(c, lh, sz, t, i, p, out, [&](int k, const HeapEntry& e) {  // copy back
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (kStream) {
#if SCG_NODES_WT
      // write-through (sc1): the line leaves the L2 now instead of staying dirty for the
      // kernel's end-of-launch write-back
      __hip_atomic_store(&gh.tk[k * gh.stride], e.tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gh.val[k * gh.stride], e.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
      __builtin_nontemporal_store(e.tk, &gh.tk[k * gh.stride]);
      __builtin_nontemporal_store(e.v, &gh.val[k * gh.stride]);
#endif
      return;
    }
#endif
    gh.put(k, e);
  });
  sc_size(c, g, i, p) = sz;
  SCG_ACCP(g.dbg, 3);
}

// The step of an env whose receive order sc_recv_scan could not prove, on the same staged
// heaps and inbox: the nodes one after another in nodes_info order (:714-736), each first
// doing its heaps' work with the real pops — after the pushes earlier nodes made this step,
// as the reference does — then the rest of its act (the staged kernel's order). Returns
// the reward.
template <int MAXD, bool kKindPaths = false, class HeapAt, class Sink>
__host__ __device__ inline double sc_nodes_serial(const ScCtx& c, ScEnv& g, const HeapAt& heap_at, int32_t* sz,
                                                  int64_t sz_stride, const NodesInbox& in, const float* act, int t,
                                                  Sink& out) {
  Num total = pyint(0);
  for (int i = 0; i < c.n_nodes; ++i) {
    WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
    int a_i = 0, lt_i = 0;
    for (int p = 0; p < c.P; ++p) {
      const int hp = i * c.P + p;
      sc_nodes_heap(c, g, heap_at(hp), sz[hp * sz_stride], in, ltc, act, t, i, p, a_i, lt_i, out, true);
    }
    if (!c.nodes[i].last_level) in.clear(c, i);
    sc_led_begin_node(c, g, i);
    total = np_add(total, sc_node_act<MAXD, NodesInbox, true, kKindPaths>(c, g, ltc, dmc, i, act, t, in));
    for (int p = 0; p < c.P; ++p) sc_observe_stock(c, g, i, p, out);
  }
  return np_neg(total).v;
}

}  // namespace scg
