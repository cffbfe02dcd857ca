// SupplyChainEnv step / reset / observation for ONE env, __host__ __device__.
//
// Restates supplychain_env.py (snapshot 2024-08-07): SC_Node.act (:208-396) with
// SC_Action.apply (:42-98), the heapq pipeline (:398-400), SC_Node.reset (:402-412),
// SC_Node.build_observation (:428-463) and SupplyChainEnv.step/_build_observation
// (:703-791). Every scalar is a scg::Num carrying its NumPy kind (scg_npscalar.h) so the
// float32/float64 rounding of the reference is reproduced; heaps follow CPython's heapq
// (scg_pyheap.h). The kernel (scg_supplychain.hip) runs one env per lane with these
// functions over env-fastest SoA arrays.
#pragma once

#include <type_traits>

#include <stdint.h>

#include "scg_const.h"
#include "scg_npscalar.h"
#include "scg_philox.h"
#include "scg_pyheap.h"
#include "scgpu.h"

// Diagnostic phase stamps (SCG_SC_STAMPS builds only, scg_supplychain.hip): no-ops here.
// SCG_STAMP(k) records the clock in slot k; SCG_ACC(k) adds the cycles since the previous
// SCG_ACC to accumulator k (declared by SCG_ACC_DECL, stored by SCG_ACC_STORE).
#ifndef SCG_STAMP
#define SCG_STAMP(k)
#define SCG_ACC_DECL scg::ScAcc scg_acc_{};
#define SCG_ACC(k)
#define SCG_ACC_STORE
#define SCG_ACCP(ptr, k)
namespace scg {
struct ScAcc {};
}
#endif

namespace scg {

// Compile-time destination bound used for a chain whose widest node ships to d nodes.
__host__ __device__ constexpr int sc_maxd_bucket(int d) { return d <= 2 ? 2 : d <= 4 ? 4 : d <= 8 ? 8 : d <= 16 ? 16 : 32; }

// Node records and threshold/sinusoid tables are read through the constant address space
// (scg_const.h): their wave-uniform fields become batched scalar loads.
using ScNode = const SCG_CONST_AS scg_sc_node;

// Launch-uniform view of the configuration.
struct ScCtx {
  ScNode* nodes;
  ConstTab<uint32_t> lt_thr;
  const int32_t* dem_tab;  // [N][T+1][R][P] or null (Philox)
  const int32_t* lt_tab;   // [N][T][n_lt] or null (Philox)
  int32_t n_nodes, P, R, A, O, H, T;
  int32_t avg_lt, max_lt, stochastic, n_lt, lt_thr_len;
  int32_t pen_unmet, pen_stock, pen_proc, pen_ship;
  uint32_t key0, key1;
  // per-product demand models (scg_sc_config demand_*; demands_generator.py:3-89)
  int32_t dkind[SCG_SC_MAX_PRODUCTS], dlo[SCG_SC_MAX_PRODUCTS], dhi[SCG_SC_MAX_PRODUCTS];
  int32_t dpert_lo[SCG_SC_MAX_PRODUCTS], dpert_n[SCG_SC_MAX_PRODUCTS];
  int64_t doff[SCG_SC_MAX_PRODUCTS];
  ConstTab<uint32_t> dthr;
  ConstTab<double> dbase;
};

// A wave-uniform pointer the compiler cannot follow across the call (device, kOpaque): loads
// through it are issued where they are used, not hoisted to a loop's or an unrolled
// sequence's top with their values held in scalar registers throughout, where a node's many
// per-destination fields spilled into VGPR lanes. Identity otherwise.
#ifndef SCG_SC_OPAQUE_DEST
#define SCG_SC_OPAQUE_DEST 0
#endif
template <bool kOpaque, class T>
__host__ __device__ __forceinline__ T* sc_opaque(T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kOpaque) asm volatile("" : "+s"(p));
#endif
  return p;
}

// A wave-uniform integer the compiler cannot follow (device): its multiples and the addresses
// derived from it are computed where used rather than hoisted out of a loop and held — or
// spilled — across it. Identity on the host.
template <class T>
__host__ __device__ __forceinline__ T sc_opaque_val(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}

// The context of a loop over nodes as a callable (sc_staged_step_ctx): the caller's own. The
// kernels pass KernargCtx (scg_supplychain_args.h) instead.
struct HostCtx {
  const ScCtx& c;
  __host__ __device__ __forceinline__ const ScCtx& operator()() const { return c; }
};

// The demand models of a config: per product, or every product uniform on
// [demand_lo, demand_hi] when the config gives none (host side of the launch).
inline void sc_ctx_demand(ScCtx& c, const scg_sc_config* cfg) {
  for (int p = 0; p < SCG_SC_MAX_PRODUCTS; ++p) {
    const bool m = cfg->demand_models != 0;
    c.dkind[p] = m ? cfg->demand_kind[p] : SCG_SC_DEMAND_UNIFORM;
    c.dlo[p] = m ? cfg->demand_lo_p[p] : cfg->demand_lo;
    c.dhi[p] = m ? cfg->demand_hi_p[p] : cfg->demand_hi;
    c.dpert_lo[p] = m ? cfg->demand_pert_lo[p] : 0;
    c.dpert_n[p] = m ? cfg->demand_pert_n[p] : 0;
    c.doff[p] = m ? cfg->demand_off[p] : 0;
  }
  c.dthr = const_tab(cfg->demand_thr);
  c.dbase = const_tab(cfg->demand_base);
}

// One env's state: element i of a per-env array lives at [i * stride] (stock) or
// [i * hstride] (heap arrays, which the LDS-staged kernel keeps in shared memory).
struct ScEnv {
  double* stock;     // [NP]
  int32_t* tk;       // [NP][H]
  double* val;       // [NP][H]
  int32_t* size;     // [NP]
  int64_t stride;    // envs in the batch
  int64_t hstride;   // heap-array stride: the batch (global) or the block (LDS)
  uint32_t env_id;   // global id (Philox counter)
  int64_t local;     // index in this shard (caller tables)
  uint32_t episode;
  int32_t overflow;  // set when a push met a full heap (the push is dropped)
  // build_info ledgers (info['sc_episode']), entry q at [q * led_stride]; null when off
  double* led_v = nullptr;
  int32_t* led_k = nullptr;
  int64_t led_stride = 0;
  int32_t hnode0 = 0;  // first node whose heaps the heap arrays hold (staged kernel: the current one)
  ScAcc* dbg = nullptr;  // diagnostic builds only (SCG_ACCP)
  // Element offset of this env added to every stock / ledger index (soff) and heap / size
  // index (hoff): 0 when the pointers above already point at the env's first element; the
  // env's column when they are the batch's base pointers (node-parallel kernel), which keeps
  // them wave-uniform (SGPRs) instead of one 64-bit VGPR pair per pointer and lane.
  int64_t soff = 0;
  int64_t hoff = 0;
  // Ledger entries by node (node-parallel kernel, where the nodes act at once): with led_word
  // set, sc_note stores the value of node led_node's entry in its own slot ((node * 2 + part)
  // * 8 + key) * P + p of led_v, and marks it, with its NumPy type, in the node's per-product
  // word led_word[(node * P + p) * led_word_stride] (bit pk = part * 8 + key, the type in
  // bits 16 + 3 pk ..); sc_ledger_reduce(_pair) adds the marked slots to the ledger in node order
  // afterwards, as _update_statistics does (:750-760).
  int32_t led_node = 0;
  uint64_t* led_word = nullptr;
  int64_t led_word_stride = 0;
};

// info['sc_episode'] categories in the reference's dict order (:416-417)
enum ScLedgerKey : int {
  LK_STOCK = 0, LK_STOCK_PEN, LK_SUPPLY, LK_PROCESS, LK_PROCESS_PEN, LK_SHIP, LK_SHIP_PEN, LK_UNMET
};

// One cost/unit entry a node's act sets (est_costs/est_units[key][p], :236-394), added to
// the episode ledger as _update_statistics does (:750-760): the reference sums the nodes'
// entries after the step in node order, and each entry is set at most once per act, so
// adding it where it is set gives the same sums; entries an act leaves at the Python int 0
// change neither value nor type of a sum, so they are skipped — and so is an entry the act
// sets to the Python int 0 (a penalty of nothing: int 0 + x is x, value and type).
__host__ __device__ __forceinline__ void sc_note(const ScCtx& c, ScEnv& e, int key, int p, Num cost, Num units) {
  if (!e.led_v) return;
  if (cost.k == NK_INT && units.k == NK_INT && cost.v == 0.0 && units.v == 0.0) return;
  if (e.led_word) {  // by node: the slot of this node's entry, reduced in node order later
    const int64_t s0 = ((static_cast<int64_t>(e.led_node) * 2 * SCG_SC_LEDGER_KEYS + key) * c.P + p) * e.led_stride + e.soff;
    const int64_t s1 = s0 + static_cast<int64_t>(SCG_SC_LEDGER_KEYS) * c.P * e.led_stride;
    e.led_v[s0] = cost.v;
    e.led_v[s1] = units.v;
    const uint64_t k0 = static_cast<uint64_t>(np_kind_abi(cost.k)), k1 = static_cast<uint64_t>(np_kind_abi(units.k));
    e.led_word[(static_cast<int64_t>(e.led_node) * c.P + p) * e.led_word_stride] |=
        (uint64_t(1) << key) | (uint64_t(1) << (8 + key)) | (k0 << (16 + 3 * key)) | (k1 << (16 + 3 * (8 + key)));
    return;
  }
  const int64_t i0 = (static_cast<int64_t>(key) * c.P + p) * e.led_stride + e.soff;
  const int64_t i1 = (static_cast<int64_t>(SCG_SC_LEDGER_KEYS + key) * c.P + p) * e.led_stride + e.soff;
  const Num a = np_add(Num{e.led_v[i0], np_kind_int(e.led_k[i0])}, cost);
  const Num b = np_add(Num{e.led_v[i1], np_kind_int(e.led_k[i1])}, units);
  e.led_v[i0] = a.v;
  e.led_k[i0] = np_kind_abi(a.k);
  e.led_v[i1] = b.v;
  e.led_k[i1] = np_kind_abi(b.k);
}

// A node is about to act (node-parallel kernel with ledgers): its entries go to its slots.
__host__ __device__ __forceinline__ void sc_led_begin_node(const ScCtx& c, ScEnv& e, int node) {
  if (!e.led_v || !e.led_word) return;
  e.led_node = node;
  for (int p = 0; p < c.P; ++p) e.led_word[(static_cast<int64_t>(node) * c.P + p) * e.led_word_stride] = 0;
}

// Ledger entries q0 and q1 (q = (part * 8 + key) * P + p; q1 < 0: q0 alone) of one env after
// the step: the nodes' marked entries added in node order (:750-760) to (lv, lk). cv: the
// slot values (stride cstride); words: the per-(node, product) marks and types (stride
// wstride). The slots of a batch of nodes are requested together for both entries, so the
// two chains of adds wait on memory once per batch, not once per batch and entry.
__host__ __device__ inline void sc_ledger_reduce_pair(const ScCtx& c, int q0, int q1, const double* cv,
                                                      int64_t cstride, const uint64_t* words, int64_t wstride,
                                                      double& lv0, int32_t& lk0, double& lv1, int32_t& lk1) {
  const bool two = q1 >= 0;
  const int p0 = q0 % c.P, pk0 = q0 / c.P;        // pk = part * 8 + key
  const int p1 = two ? q1 % c.P : p0, pk1 = two ? q1 / c.P : pk0;
  constexpr int kBatch = 8;
  Num acc0{lv0, np_kind_int(lk0)}, acc1{lv1, np_kind_int(lk1)};
  auto slot = [&](int i, int pk, int p) { return ((static_cast<int64_t>(i) * 2 * SCG_SC_LEDGER_KEYS + pk) * c.P + p) * cstride; };
  for (int i0 = 0; i0 < c.n_nodes; i0 += kBatch) {
    double v0[kBatch], v1[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u)
      if (i0 + u < c.n_nodes) {
        v0[u] = cv[slot(i0 + u, pk0, p0)];
        v1[u] = two ? cv[slot(i0 + u, pk1, p1)] : 0.0;
      }
#pragma unroll
    for (int u = 0; u < kBatch; ++u) {
      if (i0 + u >= c.n_nodes) break;
      const uint64_t w0 = words[(static_cast<int64_t>(i0 + u) * c.P + p0) * wstride];
      if ((w0 >> pk0) & 1) acc0 = np_add(acc0, Num{v0[u], np_kind_int(static_cast<int>((w0 >> (16 + 3 * pk0)) & 7))});
      if (two) {
        const uint64_t w1 = words[(static_cast<int64_t>(i0 + u) * c.P + p1) * wstride];
        if ((w1 >> pk1) & 1) acc1 = np_add(acc1, Num{v1[u], np_kind_int(static_cast<int>((w1 >> (16 + 3 * pk1)) & 7))});
      }
    }
  }
  lv0 = acc0.v;
  lk0 = np_kind_abi(acc0.k);
  if (two) {
    lv1 = acc1.v;
    lk1 = np_kind_abi(acc1.k);
  }
}

// One entry (sc_ledger_reduce_pair without the second).
__host__ __device__ inline void sc_ledger_reduce(const ScCtx& c, int q, const double* cv, int64_t cstride,
                                                 const uint64_t* words, int64_t wstride, double& lv, int32_t& lk) {
  double lv1 = 0.0;
  int32_t lk1 = 0;
  sc_ledger_reduce_pair(c, q, -1, cv, cstride, words, wstride, lv, lk, lv1, lk1);
}

// est_episode at reset (:684-695): every entry the Python int 0
__host__ __device__ inline void sc_reset_ledger(const ScCtx& c, ScEnv& e) {
  if (!e.led_v) return;
  for (int q = 0; q < 2 * SCG_SC_LEDGER_KEYS * c.P; ++q) {
    e.led_v[q * e.led_stride + e.soff] = 0.0;
    e.led_k[q * e.led_stride + e.soff] = np_kind_abi(NK_INT);
  }
}

__host__ __device__ __forceinline__ HeapView sc_heap(const ScCtx& c, const ScEnv& e, int node, int p) {
  const int64_t hp = static_cast<int64_t>(node - e.hnode0) * c.P + p;
  return HeapView{e.tk + hp * c.H * e.hstride + e.hoff, e.val + hp * c.H * e.hstride + e.hoff, e.hstride};
}

__host__ __device__ __forceinline__ int32_t& sc_size(const ScCtx& c, const ScEnv& e, int node, int p) {
  return e.size[(static_cast<int64_t>(node - e.hnode0) * c.P + p) * e.hstride + e.hoff];
}

__host__ __device__ __forceinline__ double& sc_stock(const ScCtx& c, const ScEnv& e, int node, int p) {
  return e.stock[(static_cast<int64_t>(node) * c.P + p) * e.stride + e.soff];
}

// Philox word cache: consecutive words of one (env, episode, stream) come 4 per call.
struct WordCache {
  uint32_t blk;
  U4 w;
  bool valid;
};

__host__ __device__ __forceinline__ uint32_t cached_word(const ScCtx& c, const ScEnv& e, WordCache& wc, uint32_t j,
                                                         uint32_t stream) {
  const uint32_t blk = j >> 2;
  if (!wc.valid || wc.blk != blk) {
    wc.w = philox4x32_10(U4{e.env_id, e.episode, blk, stream}, c.key0, c.key1);
    wc.blk = blk;
    wc.valid = true;
  }
  const uint32_t s = j & 3u;
  return s == 0 ? wc.w.x : s == 1 ? wc.w.y : s == 2 ? wc.w.z : wc.w.w;
}

// #{k < n : thr[k] <= u} over a nondecreasing table (upper bound)
__host__ __device__ __forceinline__ int32_t sc_count_le(ConstTab<uint32_t> thr, int32_t n, uint32_t u) {
  int32_t a = 0, b = n;
  while (a < b) {
    const int32_t m = (a + b) >> 1;
    if (thr[m] <= u)
      a = m + 1;
    else
      b = m;
  }
  return a;
}

// customer_demands[row, r, p] (np.int64) of the product's model (envs/demand.py): one
// Philox word per entry whatever the model.
__host__ __device__ __forceinline__ int32_t sc_demand(const ScCtx& c, const ScEnv& e, WordCache& wc, int row, int r,
                                                      int p) {
  const uint32_t j = static_cast<uint32_t>((row * c.R + r) * c.P + p);
  if (c.dem_tab) return c.dem_tab[e.local * (static_cast<int64_t>(c.T + 1) * c.R * c.P) + j];
  const uint32_t u = cached_word(c, e, wc, j, SCG_STREAM_SC_DEMAND);
  const int32_t lo = c.dlo[p], hi = c.dhi[p];
  switch (c.dkind[p]) {
    case SCG_SC_DEMAND_NORMAL:  // rint(clip(normal(mean, std))) by its exact CDF (:38-49)
      return lo + sc_count_le(c.dthr + c.doff[p], hi - lo, u);
    case SCG_SC_DEMAND_SINE_NORMAL:  // per period: rint(clip(b_t + normal(0, std))) (:51-89)
      return lo + sc_count_le(c.dthr + c.doff[p] + static_cast<int64_t>(row) * (hi - lo), hi - lo, u);
    case SCG_SC_DEMAND_SINE_UNIFORM: {  // rint(clip(b_t + randint(-3 std, 3 std + 1))) (:74-86)
      const int32_t jj = c.dpert_lo[p] + static_cast<int32_t>((static_cast<uint64_t>(u) * static_cast<uint32_t>(c.dpert_n[p])) >> 32);
      double x = c.dbase[c.doff[p] + row] + static_cast<double>(jj);
      x = x < lo ? static_cast<double>(lo) : (x > hi ? static_cast<double>(hi) : x);
      return static_cast<int32_t>(rint(x));
    }
    default: {  // randint(lo, hi + 1) (:33-36)
      const uint64_t span = static_cast<uint64_t>(hi - lo + 1);
      return lo + static_cast<int32_t>((static_cast<uint64_t>(u) * span) >> 32);
    }
  }
}

// leadtimes[t-1, k]: clip(1 + Poisson(avg-1), 1, max)   (:670-672)
__host__ __device__ __forceinline__ int32_t sc_leadtime(const ScCtx& c, const ScEnv& e, WordCache& wc, int t, int k) {
  const uint32_t j = static_cast<uint32_t>((t - 1) * c.n_lt + k);
  int32_t x;
  if (c.lt_tab) {  // caller table (validated on the host); clamped too, so no value can
                   // exceed the proven heap capacity or land at/before the current step
    x = c.lt_tab[e.local * (static_cast<int64_t>(c.T) * c.n_lt) + j];
  } else {
    const uint32_t u = cached_word(c, e, wc, j, SCG_STREAM_SC_LEADTIME);
    x = 0;
    for (int i = 0; i < c.lt_thr_len; ++i) x += (c.lt_thr[i] <= u) ? 1 : 0;
    x += 1;
  }
  return x < 1 ? 1 : (x > c.max_lt ? c.max_lt : x);
}

// Lead time #i of a node in step t (deterministic: avg_leadtime for every action, :724).
__host__ __device__ __forceinline__ int32_t node_leadtime(const ScCtx& c, const ScEnv& e, WordCache& wc,
                                                          ScNode& nd, int t, int i) {
  if (!c.stochastic) return c.avg_lt;
  return sc_leadtime(c, e, wc, t, nd.leadtime_offset + i);
}

__host__ __device__ __forceinline__ void sc_push(const ScCtx& c, ScEnv& e, int node, int p, int32_t time, Num amount) {
  int32_t& sz = sc_size(c, e, node, p);
  if (!py_heappush(sc_heap(c, e, node, p), sz, c.H, HeapEntry{he_pack(time, amount.k), amount.v})) e.overflow = 1;
}

// Where SHIP pushes go (:347): straight into the destination heap when one lane walks the
// whole chain in node order (sc_step_env), or into a level inbox that the destination's
// lane drains in source order before its own act (scg_supplychain_level.h).
// A Push also says whether the per-destination loop of SHIP unrolls (a plain store per
// destination does; a heap push keeps the loop rolled to bound code size).
struct DirectPush {
  static constexpr bool kUnroll = false;
  static constexpr bool kUniformNode = false;
  static constexpr bool kLdsSplit = false;  // see sc_split_scratch
  static constexpr bool kVecActions = false;  // see sc_ship_vals
  static constexpr bool kClearInAct = false;  // see StagedInbox::noship
  static constexpr bool kShipBits = false;    // see ShipLeftBits
  __host__ __device__ Num scratch_get(int) const { return pyint(0); }
  __host__ __device__ void noship(const ScCtx&, int, int, int) const {}
  __host__ __device__ void noship_all(const ScCtx&, int, int) const {}
  __host__ __device__ __forceinline__ void ship(const ScCtx& c, ScEnv& e, int /*src*/, int /*d*/, int dest, int p,
                                                int32_t time, Num amount) const {
    sc_push(c, e, dest, p, time, amount);
  }
};

// SC_Node.reset (:402-412) for one (node, product): stock back to initial_stock, the heap
// re-seeded at times 1..k (initial_supply entries first, then initial_shipments, each
// pushed with heappush). Heaps are independent, so any lane may reset any of them.
__host__ __device__ inline void sc_reset_heap(const ScCtx& c, ScEnv& e, int i, int p) {
  ScNode& nd = c.nodes[i];
  sc_stock(c, e, i, p) = static_cast<double>(nd.initial_stock[p]);
  sc_size(c, e, i, p) = 0;
  for (int j = 0; j < nd.n_init[p]; ++j) sc_push(c, e, i, p, nd.init_time[p][j], pyint(nd.init_amount[p][j]));
}

__host__ __device__ inline void sc_reset_env(const ScCtx& c, ScEnv& e) {
  for (int i = 0; i < c.n_nodes; ++i)
    for (int p = 0; p < c.P; ++p) sc_reset_heap(c, e, i, p);
  sc_reset_ledger(c, e);
}

// MAXD scalars with their NumPy kinds, the kinds packed 4 bits per entry so an unrolled
// array costs 2 VGPRs per entry plus one word per 8 entries (not 3 per entry as Num[]).
template <int MAXD>
struct NumVec {
  double v[MAXD];
  uint32_t kw[(MAXD + 7) / 8];
  __host__ __device__ __forceinline__ Num get(int i) const {
    return Num{v[i], static_cast<int>((kw[i >> 3] >> (4 * (i & 7))) & 15u)};
  }
  __host__ __device__ __forceinline__ void set(int i, Num x) {
    v[i] = x.v;
    const uint32_t sh = 4u * static_cast<uint32_t>(i & 7);
    kw[i >> 3] = (kw[i >> 3] & ~(15u << sh)) | (static_cast<uint32_t>(x.k) << sh);
  }
  // Runtime index without dynamic register indexing (which would put the array in
  // scratch): an unrolled select; constant-folds to get()/set() when i is known.
  __host__ __device__ __forceinline__ Num get_dyn(int i) const {
    double x = 0.0;
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) x = (j == i) ? v[j] : x;
#pragma unroll
    for (int j = 0; j < (MAXD + 7) / 8; ++j) w = (j == (i >> 3)) ? kw[j] : w;
    return Num{x, static_cast<int>((w >> (4 * (i & 7))) & 15u)};
  }
  __host__ __device__ __forceinline__ void set_dyn(int i, Num x) {
    const uint32_t sh = 4u * static_cast<uint32_t>(i & 7);
#pragma unroll
    for (int j = 0; j < MAXD; ++j) v[j] = (j == i) ? x.v : v[j];
#pragma unroll
    for (int j = 0; j < (MAXD + 7) / 8; ++j)
      kw[j] = (j == (i >> 3)) ? ((kw[j] & ~(15u << sh)) | (static_cast<uint32_t>(x.k) << sh)) : kw[j];
  }
};

// available_ship_capacities (:265), shared by a node's products: destination i's ship
// capacity, cut only when a product's shipment overflows it (:312-328), to the capacity minus
// what left (the shipment re-set to the capacity, times the processing ratio at a factory).
// Every value it takes is a Python int (an int capacity, minus an int times an int), so the
// kind never rounds anything to float32.
//   ShipLeftVec: the values themselves, one register pair per destination.
//   ShipLeftBits: one bit per (earlier product, destination) saying the capacity overflowed;
//     the value is rebuilt from the capacity by the same int operations in product order (a
//     destination is visited once per product). For the staged kernel, whose MAXD = 16
//     values were 48 of its 249 VGPRs; needs (P - 1) * MAXD <= 64 (scg_sc_prepare).
template <int MAXD>
struct ShipLeftVec {
  NumVec<MAXD> v;
  __host__ __device__ __forceinline__ void init(ScNode& nd, int D) {
#pragma unroll
    for (int i = 0; i < MAXD; ++i) v.set(i, pyint(i < D ? nd.ship_capacity[i] : 0));
  }
  __host__ __device__ __forceinline__ Num get(ScNode&, bool, int i, int) const { return v.get_dyn(i); }
  __host__ __device__ __forceinline__ void overflowed(int i, int, Num left) { v.set_dyn(i, left); }
  __host__ __device__ __forceinline__ bool any_f32() const {
    bool f = false;
#pragma unroll
    for (int j = 0; j < MAXD; ++j) f |= v.get(j).k == NK_F32;
    return f;
  }
};

template <int MAXD>
struct ShipLeftBits {
  uint64_t ovf;
  __host__ __device__ __forceinline__ void init(ScNode&, int) { ovf = 0; }
  __host__ __device__ __forceinline__ Num get(ScNode& nd, bool factory, int i, int p) const {
    double c = static_cast<double>(nd.ship_capacity[i]);
    for (int q = 0; q < p; ++q)
      if ((ovf >> (q * MAXD + i)) & 1u) c = c - (factory ? c * static_cast<double>(nd.processing_ratio[q]) : c);
    return pyint(c);
  }
  // (the last product's overflows are never read back, and need no bit)
  __host__ __device__ __forceinline__ void overflowed(int i, int p, Num) {
    if ((p + 1) * MAXD <= 64) ovf |= uint64_t(1) << (p * MAXD + i);
  }
  __host__ __device__ __forceinline__ bool any_f32() const { return false; }
};

// SC_Action.apply for SHIP (:58-96): the cut [0, limit] split at the destinations'
// sorted action values; amount_i = (v_(k) - v_(k-1)) * limit, clamped to what is left.
// Sorting (value, index) tuples is done by ranks so every array index is a compile-time
// constant (MAXD-unrolled loops): the arrays stay in registers instead of scratch. K <= MAXD
// bounds the loops (a node with D <= K destinations runs the K-sized split; D is uniform).
template <int MAXD, int K = MAXD, bool kNo32 = false>
__host__ __device__ inline void sc_split(const float (&vals)[MAXD], int D, Num limit, NumVec<MAXD>& out) {
#pragma unroll
  for (int i = 0; i < MAXD; ++i) out.set(i, pyint(0));
  Num left = limit;
  if (!np_lt(pyint(0), left)) return;
  // rank[i] = #{j : (vals[j], j) < (vals[i], i)}, each pair compared once
  int rank[K];
#pragma unroll
  for (int i = 0; i < K; ++i) rank[i] = 0;
#pragma unroll
  for (int i = 0; i < K; ++i)
#pragma unroll
    for (int j = i + 1; j < K; ++j)
      if (j < D) {
        const bool j_first = vals[j] < vals[i];  // on a tie the lower index i comes first
        rank[i] += j_first ? 1 : 0;
        rank[j] += j_first ? 0 : 1;
      }
  float prev = 0.0f;
  bool first = true;  // the first cut starts at the Python int 0
#pragma unroll
  for (int s = 0; s < K; ++s) {
    if (s >= D) continue;
    float v = 0.0f;
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (i < D && rank[i] == s) v = vals[i];
    const Num diff = first ? np_sub(Num{v, NK_F32}, pyint(0)) : np_sub(Num{v, NK_F32}, Num{prev, NK_F32});
    Num amt = np_mul_k<kNo32>(diff, limit);  // kNo32: a float64 limit, so a float64 amount
    if (np_lt_k<kNo32>(left, amt)) amt = left;
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (i < D && rank[i] == s) out.set(i, amt);
    left = np_sub_k<kNo32>(left, amt);
    prev = v;
    first = false;
  }
}

// The same split with its working arrays in per-lane scratch slots (the staged kernel's
// heap staging area, free while a node acts): each value is written to the slot of its
// rank, the cut is walked in slot order, and amount s is left in slot s, where destination
// i reads it at rank[i] — no O(D^2) selects and no per-destination amount registers.
// Returns false when nothing is cut (limit <= 0: every amount is the Python int 0).
template <int MAXD, bool kNo32 = false, class Scratch>
__host__ __device__ inline bool sc_split_scratch(const float (&vals)[MAXD], int D, Num limit, const Scratch& scr,
                                                 int (&rank)[MAXD]) {
  Num left = limit;
  if (!np_lt(pyint(0), left)) return false;
#pragma unroll
  for (int i = 0; i < MAXD; ++i) rank[i] = 0;
#pragma unroll
  for (int i = 0; i < MAXD; ++i)
#pragma unroll
    for (int j = i + 1; j < MAXD; ++j)
      if (j < D) {
        const bool j_first = vals[j] < vals[i];  // on a tie the lower index i comes first
        rank[i] += j_first ? 1 : 0;
        rank[j] += j_first ? 0 : 1;
      }
#pragma unroll
  for (int i = 0; i < MAXD; ++i)
    if (i < D) scr.scratch_put_value(rank[i], vals[i]);
  float prev = 0.0f;
  for (int s = 0; s < D; ++s) {
    const float v = scr.scratch_value(s);
    const Num diff = s == 0 ? np_sub(Num{v, NK_F32}, pyint(0)) : np_sub(Num{v, NK_F32}, Num{prev, NK_F32});
    Num amt = np_mul_k<kNo32>(diff, limit);
    if (np_lt_k<kNo32>(left, amt)) amt = left;
    scr.scratch_put(s, amt);
    left = np_sub_k<kNo32>(left, amt);
    prev = v;
  }
  return true;
}

// The split sized to the node: chains mixing narrow and wide nodes (ntom: 8 and 16
// destinations) run the narrow nodes' O(D^2) ranking at their own size.
template <int MAXD, bool kNo32 = false>
__host__ __device__ __forceinline__ void sc_split_d(const float (&vals)[MAXD], int D, Num limit, NumVec<MAXD>& out) {
  if constexpr (MAXD > 8) {
    if (D <= 8) {
      sc_split<MAXD, 8, kNo32>(vals, D, limit, out);
      return;
    }
  }
  sc_split<MAXD, MAXD, kNo32>(vals, D, limit, out);
}

// Action k of this env, denormalised like _denormalize_action (:697-698): (a + 1) / 2 on
// a float32 array stays float32.
__host__ __device__ __forceinline__ float sc_denorm(float a) { return (a + 1.0f) / 2.0f; }
__host__ __device__ __forceinline__ Num sc_action(const float* raw, int k) {
  return Num{static_cast<double>(sc_denorm(raw[k])), NK_F32};
}

// The D ship actions of a node and product, raw[base .. base + D), denormalised into
// vals[0 .. D) (0 past D). Every load is unconditional (a clamped index stays inside the
// row), so all of them are in flight before the first is waited for; guarded loads were
// waited one by one (a memory round trip each on the staged kernel's HBM action rows).
// K <= MAXD bounds the loads (a node with D <= K destinations loads K).
template <int MAXD, int K>
__host__ __device__ __forceinline__ void sc_ship_vals_k(const float* raw, int base, int D, float (&vals)[MAXD]) {
  float x[K];
#pragma unroll
  for (int i = 0; i < K; ++i) x[i] = raw[base + (i < D ? i : 0)];
#pragma unroll
  for (int i = 0; i < MAXD; ++i) vals[i] = (i < K && i < D) ? sc_denorm(x[i < K ? i : 0]) : 0.0f;
}
// Four destinations' actions per 16-byte load (global memory is dword-aligned here, which the
// loads need), for nodes whose destination count is a multiple of four: an env-major action
// row is one cache line apart per lane, so a quarter of the load instructions is a quarter of
// the lines the vector memory pipeline looks up. Only chunks inside the node's actions are read.
template <int MAXD, int K>
__host__ __device__ __forceinline__ void sc_ship_vals_v4(const float* raw, int base, int D, float (&vals)[MAXD]) {
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  f4u x[K / 4];
#pragma unroll
  for (int j = 0; j < K / 4; ++j)
    x[j] = 4 * j < D ? *reinterpret_cast<const f4u*>(raw + base + 4 * j) : f4u{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < MAXD; ++i) vals[i] = (i < K && i < D) ? sc_denorm(x[(i < K ? i : 0) / 4][i % 4]) : 0.0f;
}

template <int MAXD, bool kVec = false>
__host__ __device__ __forceinline__ void sc_ship_vals(const float* raw, int base, int D, float (&vals)[MAXD]) {
  if constexpr (kVec && MAXD >= 4) {
    if ((D & 3) == 0) {
      if constexpr (MAXD > 8) {
        if (D <= 8) {
          sc_ship_vals_v4<MAXD, 8>(raw, base, D, vals);
          return;
        }
      }
      sc_ship_vals_v4<MAXD, MAXD>(raw, base, D, vals);
      return;
    }
  }
  if constexpr (MAXD > 8) {
    if (D <= 8) {
      sc_ship_vals_k<MAXD, 8>(raw, base, D, vals);
      return;
    }
  }
  sc_ship_vals_k<MAXD, MAXD>(raw, base, D, vals);
}

// receive (:220-228) for one heap: pop every entry due now, summed in a float64 array
template <bool kPlain = false, class HV>
__host__ __device__ __forceinline__ double sc_receive(const HV& h, int32_t& sz, int t) {
  double recv = 0.0;
  // the root travels in registers from pop to pop (py_heappop_root): no slot read twice
  if (sz == 0) return recv;
  HeapEntry root = h.get(0);
  while (sz > 0 && he_time(root.tk) == t) recv = recv + py_heappop_root<kPlain>(h, sz, root).v;
  return recv;
}

// SC_Node.act (:208-396) for node `ni` at time t; `act` = this env's raw float32 action
// row. Returns the node's cost with its NumPy kind. MAXD bounds the node's destinations.
// kKindPaths: the ship part also has a plain double instantiation for waves whose kinds
// never round to float32 (below); on in the staged and node-parallel kernels without
// ledgers, off where its registers or code size would cost occupancy or inlining.
// kHeapsDone: the caller already did this node's heap work — the receive pops with their
// stock update and the SUPPLY pushes (sc_staged_heap) — so act touches no heap of its own;
// a node's heaps are independent of everything else act computes, so only the order of
// operations on each heap has to be the reference's, and it is.
template <int MAXD, class Push = DirectPush, bool kHeapsDone = false, bool kKindPaths = false>
__host__ __device__ __forceinline__ Num sc_node_act(const ScCtx& c, ScEnv& e, WordCache& ltc, WordCache& dmc, int ni,
                                           const float* act, int t, const Push& push = Push()) {
  ScNode& nd = c.nodes[ni];
  const int P = c.P;
  Num cost = pyint(0);
  int lt_i = 0;
  if constexpr (!kHeapsDone) {
    for (int p = 0; p < P; ++p) {
      int32_t& sz = sc_size(c, e, ni, p);
      sc_stock(c, e, ni, p) = sc_stock(c, e, ni, p) + sc_receive(sc_heap(c, e, ni, p), sz, t);
    }
  }
  // over stock capacity: penalty, excess discarded (:232-240)
  for (int p = 0; p < P; ++p) {
    double& st = sc_stock(c, e, ni, p);
    if (st > static_cast<double>(nd.stock_capacity[p])) {
      const Num over = np_sub(f64(st), pyint(nd.stock_capacity[p]));
      const Num pen = np_mul(pyint(c.pen_stock), over);
      cost = np_add(cost, pen);
      sc_note(c, e, LK_STOCK_PEN, p, pen, over);
      st = static_cast<double>(nd.stock_capacity[p]);
    }
  }
  // SUPPLY (:243-259)
  int a_i = 0;
  if (nd.n_supply > 0) {
    for (int p = 0; p < P; ++p) {
      if (nd.supply_capacity[p] <= 0) continue;
      const Num amount = np_mul(sc_action(act, nd.action_offset + a_i), pyint(nd.supply_capacity[p]));
      const Num cst = np_mul(amount, pyint(nd.supply_cost[p]));
      ++a_i;
      if (np_lt(pyint(0), amount)) {
        if constexpr (!kHeapsDone) sc_push(c, e, ni, p, t + node_leadtime(c, e, ltc, nd, t, lt_i), amount);
        ++lt_i;  // the lead-time cursor moves only when something was supplied (:252-254)
      }
      cost = np_add(cost, cst);
      sc_note(c, e, LK_SUPPLY, p, cst, amount);
    }
  }
  SCG_ACCP(e.dbg, 8);
  if (!nd.last_level) {
    // SHIP (:262-375)
    const int D = nd.n_dests;
    // available_ship_capacities, shared by the products (:265)
    typename std::conditional<Push::kShipBits, ShipLeftBits<MAXD>, ShipLeftVec<MAXD>>::type ship_left;
    ship_left.init(nd, D);
    Num proc_left = pyint(nd.processing_capacity);
    const int lt_base = lt_i;
    const bool factory = nd.processing_capacity > 0;
    for (int p = 0; p < P; ++p) {
      if (!(nd.stock_capacity[p] > 0)) {  // no SHIP action for this product
        if constexpr (Push::kClearInAct) push.noship_all(c, ni, p);
        continue;
      }
      Num over_ship = pyint(0), over_proc = pyint(0);
      const Num material = f64(sc_stock(c, e, ni, p));
      if (np_lt(pyint(0), material)) {
        const Num limit = py_min(pyint(nd.stock_capacity[p]), material);  // :61-64
        // The split and the per-destination passes below round to float32 only through a
        // float32 amount, which comes from an int limit (float32 action * int, :56-57, 86), or
        // through a float32 left in proc_left or ship_left by an earlier product. Without
        // either (the stock is the limit, or nothing is cut) every promoted kind is float64 or
        // a Python / int64 scalar, and the whole wave runs the plain double instantiation.
        bool f32_left = proc_left.k == NK_F32;
        f32_left |= ship_left.any_f32();
        const bool no32 = kKindPaths && wave_all(!f32_left && (limit.k != NK_INT || !np_lt(pyint(0), limit)));
        auto ship_product = [&](auto no32_tag) __attribute__((always_inline)) {
          constexpr bool kNo32 = decltype(no32_tag)::value;
          float vals[MAXD];
          NumVec<MAXD> out;
          int rank[MAXD];
          bool cut = false;  // kLdsSplit: the split's amounts are in the scratch slots
          sc_ship_vals<MAXD, Push::kVecActions>(act, nd.action_offset + a_i, D, vals);
          if constexpr (Push::kLdsSplit) {
            cut = sc_split_scratch<MAXD, kNo32>(vals, D, limit, push, rank);
          } else {
            sc_split_d<MAXD, kNo32>(vals, D, limit, out);
          }
          SCG_ACCP(e.dbg, 9);
          // The reference's per-destination passes — processing capacity and ratio
          // (:298-310), ship capacity (:312-328), sum(amounts) (:331), the pushes (:344-348)
          // and sum(calculate_costs(amounts_to_ship)) (:352) — each carry their own
          // accumulator in destination order and read only destination i's values; the
          // stock update between them (:332) touches none of them. So they run fused, one
          // destination at a time, every accumulator seeing the reference's order, and no
          // per-destination array besides the split's output stays live.
          Num leaving = pyint(0), ship_cost = pyint(0), ship_units = pyint(0);
          auto dest_step = [&](int i) {
            // this destination's node fields, loaded here (Push::kUniformNode: the node is
            // wave-uniform, so the laundered pointer stays in scalar registers)
            ScNode& nd = *sc_opaque<Push::kUniformNode && SCG_SC_OPAQUE_DEST>(&c.nodes[ni]);
            Num o;
            if constexpr (Push::kLdsSplit)
              o = cut ? push.scratch_get(rank[i]) : pyint(0);
            else
              o = out.get_dyn(i);
            Num snt = o;  // amounts_to_ship = amounts.copy() (:292)
            if (factory) {
              if (np_lt_k<kNo32>(pyint(0), o)) {
                if (np_lt_k<kNo32>(proc_left, o)) {
                  over_proc = np_add_k<kNo32>(over_proc, np_sub_k<kNo32>(o, proc_left));
                  o = proc_left;
                }
                proc_left = np_sub_k<kNo32>(proc_left, o);
              }
              snt = np_div_k<kNo32>(o, pyint(nd.processing_ratio[p]));
            }
            const Num cap = ship_left.get(nd, factory, i, p);
            if (np_lt_k<kNo32>(pyint(0), snt) && np_lt_k<kNo32>(cap, snt)) {
              over_ship = np_add_k<kNo32>(over_ship, np_sub_k<kNo32>(snt, cap));
              snt = cap;
              o = factory ? np_mul_k<kNo32>(snt, pyint(nd.processing_ratio[p])) : snt;
              ship_left.overflowed(i, p, np_sub_k<kNo32>(cap, o));  // only on overflow, by the new amount
            }
            leaving = np_add_k<kNo32>(leaving, o);
            if (np_lt_k<kNo32>(pyint(0), snt))
              push.ship(c, e, ni, i, nd.dests[i], p, t + node_leadtime(c, e, ltc, nd, t, lt_base + i), snt);
            else if constexpr (Push::kClearInAct)
              push.noship(c, ni, i, p);
            ship_cost = np_add_k<kNo32>(ship_cost, np_mul_k<kNo32>(snt, pyint(nd.dest_costs[p][i])));
            ship_units = np_add_k<kNo32>(ship_units, snt);  // sum(amounts_to_ship) (:356)
          };
          if constexpr (Push::kUnroll) {  // every index static: the NumVecs stay in registers
#pragma unroll
            for (int i = 0; i < MAXD; ++i)
              if (i < D) dest_step(i);
          } else {
            for (int i = 0; i < D; ++i) dest_step(i);
          }
          SCG_ACCP(e.dbg, 10);
          // float64 array element minus the promoted scalar (:332); nothing above wrote it
          sc_stock(c, e, ni, p) = material.v - leaving.v;
          if (factory) {
            const Num proc = np_mul(leaving, pyint(nd.processing_cost[p]));
            cost = np_add(cost, proc);
            sc_note(c, e, LK_PROCESS, p, proc, leaving);
          }
          cost = np_add(cost, ship_cost);
          sc_note(c, e, LK_SHIP, p, ship_cost, ship_units);
        };
        if constexpr (kKindPaths) {
          if (no32)
            ship_product(std::true_type{});
          else
            ship_product(std::false_type{});
        } else {
          ship_product(std::false_type{});
        }
      } else {
        if constexpr (Push::kClearInAct) push.noship_all(c, ni, p);
      }
      const Num pen_proc = np_mul(pyint(c.pen_proc), over_proc);  // :361
      cost = np_add(cost, pen_proc);
      sc_note(c, e, LK_PROCESS_PEN, p, pen_proc, over_proc);
      const Num pen_ship = np_mul(pyint(c.pen_ship), over_ship);  // :366
      cost = np_add(cost, pen_ship);
      sc_note(c, e, LK_SHIP_PEN, p, pen_ship, over_ship);
      a_i += D;
    }
  } else {
    // retailer: serve what stock allows, lost sales cost the rest (:379-387)
    for (int p = 0; p < P; ++p) {
      const Num dem = Num{static_cast<double>(sc_demand(c, e, dmc, t - 1, nd.retailer_index, p)), NK_I64};
      double& st = sc_stock(c, e, ni, p);
      const Num served = py_min(f64(st), dem);
      st = st - served.v;
      const Num unmet = np_sub(dem, served);
      const Num pen = np_mul(pyint(c.pen_unmet), unmet);
      cost = np_add(cost, pen);
      sc_note(c, e, LK_UNMET, p, pen, unmet);
    }
  }
  SCG_ACCP(e.dbg, 11);
  for (int p = 0; p < P; ++p) {  // holding (:390-394)
    const Num held = f64(sc_stock(c, e, ni, p));
    const Num hold = np_mul(held, pyint(nd.stock_cost[p]));
    cost = np_add(cost, hold);
    sc_note(c, e, LK_STOCK, p, hold, held);
  }
  return cost;
}

// SupplyChainEnv.step body (:704-738) for time t (already incremented). Actions are the
// raw float32 row in [-1, 1]; returns the reward. MAXD >= every node's destinations.
template <int MAXD>
__host__ __device__ inline double sc_step_env(const ScCtx& c, ScEnv& e, const float* act, int t) {
  WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
  Num total = pyint(0);
  for (int i = 0; i < c.n_nodes; ++i) {
    total = np_add(total, sc_node_act<MAXD>(c, e, ltc, dmc, i, act, t));
    SCG_STAMP(2 + (i < 20 ? i : 20));
  }
  return np_neg(total).v;
}

// Observation at time t (:762-791): normalised next demands, per node stock share and
// in-transit bins (storage-order walk, :445-461), time to go; 2x-1 clipped to [-1, 1].
// Element o of the row is written by out(o, value); the pieces below write disjoint
// elements, so lanes may emit different pieces of one row in any order.
__host__ __device__ __forceinline__ double sc_obs_norm(double x) {
  const double y = x * 2.0 - 1.0;
  return y < -1.0 ? -1.0 : (y > 1.0 ? 1.0 : y);
}

// demand element k = r * P + p
template <class Sink>
__host__ __device__ inline void sc_observe_demand(const ScCtx& c, const ScEnv& e, int t, int k, Sink& out) {
  WordCache dmc{0, U4{0, 0, 0, 0}, false};
  const int p = k % c.P;
  const double range = static_cast<double>(c.dhi[p] - c.dlo[p]);
  out(k, sc_obs_norm(static_cast<double>(sc_demand(c, e, dmc, t, k / c.P, p) - c.dlo[p]) / range));
}

// node i, product p: stock share (:433)
template <class Sink>
__host__ __device__ __forceinline__ void sc_observe_stock(const ScCtx& c, const ScEnv& e, int i, int p, Sink& out) {
  const int base = c.R * c.P + i * (c.P + c.P * c.avg_lt);
  out(base + p, sc_obs_norm(sc_stock(c, e, i, p) / static_cast<double>(c.nodes[i].stock_capacity[p])));
}

struct NoVisit {
  __host__ __device__ __forceinline__ void operator()(int, const HeapEntry&) const {}
};
template <class V>
inline constexpr bool kNoVisit = false;
template <>
inline constexpr bool kNoVisit<NoVisit> = true;

// node i, product p: avg_leadtime in-transit bins over heap h of size sz (:445-461). The
// walk reads every entry once, in storage order; visit(k, entry) sees each of them.
template <class Sink, class Visit = NoVisit, class HV>
__host__ __device__ inline void sc_observe_bins(const ScCtx& c, const HV& h, int32_t sz, int t, int i, int p,
                                                Sink& out, const Visit& visit = Visit()) {
  ScNode& nd = c.nodes[i];
  const int nb = c.avg_lt;
  const int base = c.R * c.P + i * (c.P + c.P * nb);
  int o = base + c.P + p * nb;
  const int first = t + 1, last = t + c.avg_lt;
  if (sz == 0) {
    for (int b = first; b <= last; ++b) out(o++, sc_obs_norm(0.0));
    return;
  }
  if constexpr (!kNoVisit<Visit>) {  // the kernels' step walks (their copy-back rides on it)
    // The same walk as one pass over the entries in storage order with a bin cursor that
    // only moves forward: entry k closes the bins before its time (while the cursor is short
    // of the last bin), then joins the cursor's bin, so every bin sums the same entries in
    // the same order. The entries are read kBatch at a time, all requested before the first
    // is tested (the walk below waits on each slot's read before deciding on the next).
    constexpr int kBatch = 8;
    int when = first;
    Num bin = pyint(0);
    for (int k0 = 0; k0 < sz; k0 += kBatch) {
      HeapEntry b[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        if (k0 + u < sz) b[u] = h.get(k0 + u);
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        if (k0 + u < sz) {
          visit(k0 + u, b[u]);
          const int32_t tm = he_time(b[u].tk);
          while (when < last && tm != when) {
            out(o++, sc_obs_norm(np_div(bin, pyint(nd.max_ship[p])).v));
            bin = pyint(0);
            ++when;
          }
          bin = np_add(bin, Num{b[u].v, he_kind(b[u].tk)});
        }
    }
    for (; when < last; ++when) {
      out(o++, sc_obs_norm(np_div(bin, pyint(nd.max_ship[p])).v));
      bin = pyint(0);
    }
    out(o, sc_obs_norm(np_div(bin, pyint(nd.max_ship[p] * (c.max_lt - (last - first)))).v));
    return;
  }
  int k = 0;
  for (int when = first; when < last; ++when) {
    Num bin = pyint(0);
    while (k < sz && h.time_at(k) == when) {
      const HeapEntry en = h.get(k);
      visit(k, en);
      bin = np_add(bin, Num{en.v, he_kind(en.tk)});
      ++k;
    }
    out(o++, sc_obs_norm(np_div(bin, pyint(nd.max_ship[p])).v));
  }
  Num bin = pyint(0);
  while (k < sz) {
    const HeapEntry en = h.get(k);
    visit(k, en);
    bin = np_add(bin, Num{en.v, he_kind(en.tk)});
    ++k;
  }
  out(o, sc_obs_norm(np_div(bin, pyint(nd.max_ship[p] * (c.max_lt - (last - first)))).v));
}

// node i, product p: stock share, then avg_leadtime in-transit bins
template <class Sink>
__host__ __device__ inline void sc_observe_heap(const ScCtx& c, const ScEnv& e, int t, int i, int p, Sink& out) {
  sc_observe_stock(c, e, i, p, out);
  sc_observe_bins(c, sc_heap(c, e, i, p), sc_size(c, e, i, p), t, i, p, out);
}

template <class Sink>
__host__ __device__ inline void sc_observe_tail(const ScCtx& c, int t, Sink& out) {
  out(c.O - 1, sc_obs_norm(static_cast<double>(c.T - t) / static_cast<double>(c.T)));
}

template <class Sink>
__host__ __device__ inline void sc_observe(const ScCtx& c, ScEnv& e, int t, Sink& out) {
  for (int k = 0; k < c.R * c.P; ++k) sc_observe_demand(c, e, t, k, out);
  for (int i = 0; i < c.n_nodes; ++i)
    for (int p = 0; p < c.P; ++p) sc_observe_heap(c, e, t, i, p, out);
  sc_observe_tail(c, t, out);
}

}  // namespace scg
