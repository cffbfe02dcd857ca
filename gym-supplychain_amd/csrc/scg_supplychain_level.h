// Level-parallel SupplyChainEnv.step: a group of G lanes per env, one lane per node of a
// level, __host__ __device__.
//
// supplychain_env.py walks the nodes in nodes_info order (:714-736). In every chain the
// reference's factories build (2-per-stage, N-per-stage, multi-product) the nodes form
// levels — runs of consecutive nodes (suppliers, factories, wholesalers, retailers) — and
// every shipment goes from one level to the next. Within a step a node's act reads only
// its own stock and heaps; its pushes into the next level's heaps (times >= t+1) happen
// before those nodes act. So the nodes of a level act independently, and the reference's
// order is reproduced exactly by:
//
//   for each level l:
//     drain: each heap of level l receives the pushes of level l-1 in source-node order
//            (what the reference did while walking level l-1, :347)
//     act:   each node of level l clears its inbox row, then runs SC_Node.act (:208-396) —
//            pops, supply pushes into its own heap, stock, costs — writing its shipments
//            into the inbox (one buffer, reused by every transition) instead of the
//            destination heaps
//   reward: -(sum of the node costs in node order) (:735-738)
//
// so heap storage order, float rounding order and the lead-time cursor are the
// reference's. The schedule is a Sched policy: on the device a phase is one lambda call by
// each lane followed by a block barrier; the test-only host build runs the lambda for every
// lane in turn, which is the same computation.
#pragma once

#include "scg_supplychain_core.h"

namespace scg {

struct ScLevels {
  int32_t n;
  int32_t start[SCG_SC_MAX_LEVELS + 1];
};

// One env's shipment inbox for a level transition: entry (p, src, dst) at
// (p * wsrc + src) * wdst + dst, src/dst relative to their level's first node.
struct LevelInbox {
  int32_t* tk;  // time << 3 | kind; -1 = no shipment
  double* val;
  int32_t src0, dst0, wsrc, wdst;

  static constexpr bool kUnroll = true;  // an LDS store per destination
  static constexpr bool kUniformNode = false;  // the group's lanes act different nodes
  static constexpr bool kLdsSplit = false;
  static constexpr bool kVecActions = false;
  static constexpr bool kClearInAct = false;  // cleared before the act
  static constexpr bool kShipBits = false;
  __host__ __device__ Num scratch_get(int) const { return pyint(0); }
  __host__ __device__ void noship(const ScCtx&, int, int, int) const {}
  __host__ __device__ void noship_all(const ScCtx&, int, int) const {}
  __host__ __device__ __forceinline__ void ship(const ScCtx&, ScEnv&, int src, int /*d*/, int dest, int p, int32_t time,
                                                Num amount) const {
    const int idx = (p * wsrc + (src - src0)) * wdst + (dest - dst0);
    tk[idx] = he_pack(time, amount.k);
    val[idx] = amount.v;
  }
};

// One env as the level kernel sees it: heaps/stock (env-major, stride 1), the inbox
// (cfg->inbox_size entries), the node costs of this step.
struct ScLevelEnv {
  ScEnv e;
  int32_t* in_tk;
  double* in_val;
  Num* cost;  // [n_nodes]
  const float* act;
};

// inbox of the transition l -> l+1
__host__ __device__ __forceinline__ LevelInbox level_inbox(const ScLevels& lv, const ScLevelEnv& x, int l) {
  if (l + 1 >= lv.n) return LevelInbox{x.in_tk, x.in_val, lv.start[l], lv.start[l + 1], 0, 0};
  return LevelInbox{x.in_tk, x.in_val, lv.start[l], lv.start[l + 1], lv.start[l + 1] - lv.start[l],
                    lv.start[l + 2] - lv.start[l + 1]};
}

// drain: pushes of transition (l-1 -> l) into level l's heaps, per (node, product) in
// source order (lane s of G takes every G-th heap)
__host__ __device__ inline void sc_level_drain(const ScCtx& c, ScEnv& e, const LevelInbox& in, int s, int G) {
  const int n_heaps = in.wdst * c.P;
  for (int q = s; q < n_heaps; q += G) {
    const int dl = q / c.P, p = q % c.P;
    const int j = in.dst0 + dl;
    int32_t& sz = sc_size(c, e, j, p);
    const HeapView h = sc_heap(c, e, j, p);
    for (int sl = 0; sl < in.wsrc; ++sl) {
      const int idx = (p * in.wsrc + sl) * in.wdst + dl;
      const int32_t tk = in.tk[idx];
      if (tk >= 0 && !py_heappush(h, sz, c.H, HeapEntry{tk, in.val[idx]})) e.overflow = 1;
    }
  }
}

template <int MAXD>
__host__ __device__ inline void sc_level_act(const ScCtx& c, ScLevelEnv& x, const LevelInbox& out, int b0, int b1,
                                             int t, int s, int G) {
  for (int i = b0 + s; i < b1; i += G) {
    for (int p = 0; p < c.P; ++p)  // this node's row: no shipment unless act writes one
      for (int dl = 0; dl < out.wdst; ++dl) out.tk[(p * out.wsrc + (i - b0)) * out.wdst + dl] = -1;
    WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
    x.cost[i] = sc_node_act<MAXD, LevelInbox>(c, x.e, ltc, dmc, i, x.act, t, out);
  }
}

// SupplyChainEnv.step body (:704-738) for time t; the reward is returned on lane 0.
template <int MAXD, class Sched>
__host__ __device__ inline double sc_level_step(const ScCtx& c, const ScLevels& lv, ScLevelEnv& x, int t, Sched& sch) {
  const int G = sch.G;
  for (int l = 0; l < lv.n; ++l) {
    if (l > 0) {
      const LevelInbox prev = level_inbox(lv, x, l - 1);
      sch.phase([&](int s) { sc_level_drain(c, x.e, prev, s, G); });
    }
    const LevelInbox next = level_inbox(lv, x, l);
    sch.phase([&](int s) { sc_level_act<MAXD>(c, x, next, lv.start[l], lv.start[l + 1], t, s, G); });
  }
  double reward = 0.0;
  sch.phase([&](int s) {
    if (s != 0) return;
    Num total = pyint(0);
    for (int i = 0; i < c.n_nodes; ++i) total = np_add(total, x.cost[i]);
    reward = np_neg(total).v;
  });
  return reward;
}

// Observation row at time t, pieces spread over the group's lanes.
template <class Sink>
__host__ __device__ inline void sc_level_observe_lane(const ScCtx& c, const ScEnv& e, int t, Sink& out, int s, int G) {
  for (int k = s; k < c.R * c.P; k += G) sc_observe_demand(c, e, t, k, out);
  for (int hp = s; hp < c.n_nodes * c.P; hp += G) sc_observe_heap(c, e, t, hp / c.P, hp % c.P, out);
  if (s == 0) sc_observe_tail(c, t, out);
}

__host__ __device__ inline void sc_level_reset_lane(const ScCtx& c, ScEnv& e, int s, int G) {
  for (int hp = s; hp < c.n_nodes * c.P; hp += G) sc_reset_heap(c, e, hp / c.P, hp % c.P);
}

}  // namespace scg
