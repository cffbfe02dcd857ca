// Node-staged SupplyChainEnv.step for ONE env, __host__ __device__.
//
// supplychain_env.py walks the nodes in nodes_info order (:714-736) and every shipment of a
// node goes into the heap of a LATER node (:344-348, the reference's chains all ship one
// echelon down). So when node i acts, every push it will ever receive this step has been
// made, and after it acts its heaps are final for the step. The lane kernel on HBM heaps
// pays a chain of dependent global loads for every heap operation (a push sifts through
// up to log2(H) parents); here, per node in order:
//
//   stage    node i's heaps (P x H entries) from HBM into fast memory (LDS on the device)
//   drain    the shipments earlier nodes made to i this step, from i's inbox, in source
//            order — the order in which the reference pushed them — with heappush
//   act      SC_Node.act (:208-396) on the staged heaps; i's own shipments are written to
//            the inbox entries of its destinations (plain stores, one per destination and
//            product, -1 when nothing is shipped) instead of being pushed
//   observe  i's stock share and in-transit bins (:428-463) — its heaps are final
//   store    the heaps back to HBM
//
// Heap storage order, float rounding and the lead-time cursor are the reference's (the
// pushes into a heap happen in the same order, before the same pops). The inbox is a
// per-env HBM array laid out by scg_sc_prepare (scg_sc_node in_base/in_deg/in_slot).
#pragma once

#include "scg_supplychain_core.h"

namespace scg {

// Shipments into the destinations' inbox entries; entry q of this env at [q * stride].
struct StagedInbox {
  int32_t* tk;  // time << 3 | kind, -1 = no shipment
  double* val;
  int64_t stride;

  static constexpr bool kUnroll = true;  // a store per destination
  __host__ __device__ __forceinline__ void ship(const ScCtx& c, ScEnv&, int src, int d, int /*dest*/, int p,
                                                int32_t time, Num amount) const {
    const scg_sc_node& nd = c.nodes[src];
    const int64_t q = nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d];
    tk[q * stride] = he_pack(time, amount.k);
    val[q * stride] = amount.v;
  }
  // node src ships nothing this step unless its act writes an entry
  __host__ __device__ __forceinline__ void clear(const ScCtx& c, int src) const {
    const scg_sc_node& nd = c.nodes[src];
    for (int d = 0; d < nd.n_dests; ++d)
      for (int p = 0; p < c.P; ++p) tk[(nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d]) * stride] = -1;
  }
};

// Copy node i's heaps (live entries) and sizes between two env views.
__host__ __device__ inline void sc_copy_node_heaps(const ScCtx& c, const ScEnv& from, ScEnv& to, int i) {
  for (int p = 0; p < c.P; ++p) {
    const int32_t sz = sc_size(c, from, i, p);
    sc_size(c, to, i, p) = sz;
    const HeapView a = sc_heap(c, from, i, p), b = sc_heap(c, to, i, p);
    for (int j = 0; j < sz; ++j) b.put(j, a.get(j));
  }
}

// SupplyChainEnv.step body (:704-738) plus the node part of _build_observation (:762-791)
// for time t. `g` views the env's state in HBM; `loc` views the same env with heap arrays
// that hold one node's heaps (its hnode0 is set per node). out(o, x) receives the node
// observation elements (the caller adds the demand and time-to-go ones). Returns the reward.
template <int MAXD, class Sink>
__host__ __device__ inline double sc_staged_step(const ScCtx& c, ScEnv& g, ScEnv& loc, const StagedInbox& in,
                                                 const float* act, int t, Sink& out) {
  WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
  Num total = pyint(0);
  for (int i = 0; i < c.n_nodes; ++i) {
    const scg_sc_node& nd = c.nodes[i];
    loc.hnode0 = i;
    sc_copy_node_heaps(c, g, loc, i);
    for (int p = 0; p < c.P; ++p) {  // the shipments of earlier nodes, in their order (:347)
      int32_t& sz = sc_size(c, loc, i, p);
      const HeapView h = sc_heap(c, loc, i, p);
      for (int k = 0; k < nd.in_deg; ++k) {
        const int64_t q = nd.in_base + static_cast<int64_t>(p) * nd.in_deg + k;
        const int32_t tk = in.tk[q * in.stride];
        if (tk >= 0 && !py_heappush(h, sz, c.H, HeapEntry{tk, in.val[q * in.stride]})) loc.overflow = 1;
      }
    }
    if (!nd.last_level) in.clear(c, i);
    total = np_add(total, sc_node_act<MAXD, StagedInbox>(c, loc, ltc, dmc, i, act, t, in));
    for (int p = 0; p < c.P; ++p) sc_observe_heap(c, loc, t, i, p, out);
    sc_copy_node_heaps(c, loc, g, i);
  }
  g.overflow |= loc.overflow;
  return np_neg(total).v;
}

}  // namespace scg
