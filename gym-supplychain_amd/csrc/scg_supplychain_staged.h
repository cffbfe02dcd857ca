// Node-staged SupplyChainEnv.step for ONE env, __host__ __device__.
//
// supplychain_env.py walks the nodes in nodes_info order (:714-736) and every shipment of a
// node goes into the heap of a LATER node (:344-348, the reference's chains all ship one
// echelon down). So when node i acts, every push it will ever receive this step has been
// made, and after it acts its heaps are final for the step. The lane kernel on HBM heaps
// pays a chain of dependent global loads for every heap operation (a push sifts through
// up to log2(H) parents); here, per node in order:
//
//   per product p, heap (i, p) alone (H entries, so the LDS a lane needs is one heap):
//     stage    the heap from HBM into fast memory (LDS on the device)
//     drain    the shipments earlier nodes made to (i, p) this step, from i's inbox, in
//              source order — the order in which the reference pushed them — with heappush
//     receive  the pops due now and the stock update (:220-228)
//     supply   the SUPPLY push (:243-259) — the heap's last operation of the step
//     observe  its in-transit bins (:445-461), then store it back to HBM
//   act      the rest of SC_Node.act (:208-396), touching no heap of i; i's own shipments
//            are written to the inbox entries of its destinations (plain stores, one per
//            destination and product, -1 when nothing is shipped) instead of being pushed
//   observe  i's stock shares
//
// Heap storage order, float rounding and the lead-time cursor are the reference's (the
// pushes into a heap happen in the same order, before the same pops). The inbox is a
// per-env HBM array laid out by scg_sc_prepare (scg_sc_node in_base/in_deg/in_slot).
//
// Byte-packed entries: inside the step, every time a staged heap or the inbox holds lies in
// [t, t + max_leadtime], so both keep an entry's time RELATIVE to t with its NumPy kind in
// one byte (rel << 3 | kind; max_leadtime <= kStagedMaxRel) next to its float64 amount:
// 9 bytes instead of 12, in LDS (the staged heap: 64 lanes x slots x 9 B, which lets 11
// waves share a CU instead of 8) and in HBM (the inbox: a quarter less traffic). Relative
// times order, compare and bin exactly as the absolute ones (the step's own time is 0);
// they are made absolute again only where a heap goes back to HBM.
#pragma once

#include "scg_supplychain_core.h"

namespace scg {

// Largest relative time a byte-packed entry holds (5 bits); 0xFF (relative time 31, kind 7)
// marks an empty inbox entry. scg_sc_prepare keeps chains with max_leadtime > 30 off this
// kernel.
constexpr int kStagedMaxRel = 30;
constexpr uint8_t kStagedNone = 0xFF;

// A heap of byte-packed entries (rel << 3 | kind, then the amount), entry j at [j * stride].
struct HeapView8 {
  uint8_t* tk;
  double* val;
  int64_t stride;

  __host__ __device__ __forceinline__ HeapEntry get(int i) const {
    return HeapEntry{static_cast<int32_t>(tk[i * stride]), val[i * stride]};
  }
  __host__ __device__ __forceinline__ void put(int i, const HeapEntry& e) const {
    tk[i * stride] = static_cast<uint8_t>(e.tk);
    val[i * stride] = e.v;
  }
  __host__ __device__ __forceinline__ int32_t time_at(int i) const { return he_time(tk[i * stride]); }
};

// Shipments into the destinations' inbox entries; entry q of this env at [q * stride].
#ifndef SCG_STAGED_OPAQUE_STRIDE
#define SCG_STAGED_OPAQUE_STRIDE 0
#endif
struct StagedInbox {
  uint8_t* tk;  // (time - t) << 3 | kind, kStagedNone = no shipment
  double* val;
  int64_t stride;
  HeapView8 scr;  // the heap staging area, scratch for sc_split_scratch while a node acts
  int32_t t;      // the step's time: shipments are stored relative to it

  static constexpr bool kUnroll = true;  // a store per destination
  static constexpr bool kUniformNode = true;  // one lane per env, nodes in turn: the node is wave-uniform
  static constexpr bool kLdsSplit = true;
  static constexpr bool kVecActions = true;  // the env's action row in HBM
#ifndef SCG_STAGED_NOSHIP
#define SCG_STAGED_NOSHIP 1
#endif
  // Entries the act does not ship to are marked empty by the act itself (noship /
  // noship_all: one store per destination and product in all), instead of a clear of the
  // node's every entry before it acts followed by the shipments' stores over most of them.
  static constexpr bool kClearInAct = SCG_STAGED_NOSHIP != 0;
#ifndef SCG_STAGED_SHIP_BITS
#define SCG_STAGED_SHIP_BITS 0
#endif
  // available_ship_capacities as overflow bits (ShipLeftBits): (P - 1) * MAXD <= 64
  static constexpr bool kShipBits = SCG_STAGED_SHIP_BITS != 0;
  // the split's sorted values go to the amounts' slots (a float is exact in the double),
  // each read back before the amount of its rank overwrites it
  __host__ __device__ __forceinline__ void scratch_put_value(int s, float v) const {
    scr.val[s * scr.stride] = static_cast<double>(v);
  }
  __host__ __device__ __forceinline__ float scratch_value(int s) const {
    return static_cast<float>(scr.val[s * scr.stride]);
  }
  __host__ __device__ __forceinline__ void scratch_put(int s, Num x) const {
    scr.tk[s * scr.stride] = static_cast<uint8_t>(x.k);
    scr.val[s * scr.stride] = x.v;
  }
  __host__ __device__ __forceinline__ Num scratch_get(int s) const {
    return Num{scr.val[s * scr.stride], static_cast<int>(scr.tk[s * scr.stride])};
  }
  __host__ __device__ __forceinline__ void ship(const ScCtx& c, ScEnv&, int src, int d, int /*dest*/, int p,
                                                int32_t time, Num amount) const {
    ScNode& nd = *sc_opaque<SCG_SC_OPAQUE_DEST != 0>(&c.nodes[src]);
    const int64_t q = nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d];
    tk[q * stride] = static_cast<uint8_t>(he_pack(time - t, amount.k));
    val[q * stride] = amount.v;
  }
  __host__ __device__ __forceinline__ void noship(const ScCtx& c, int src, int d, int p) const {
    ScNode& nd = c.nodes[src];
    tk[(nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d]) * stride] = kStagedNone;
  }
  __host__ __device__ __forceinline__ void noship_all(const ScCtx& c, int src, int p) const {
    ScNode& nd = c.nodes[src];
    for (int d = 0; d < nd.n_dests; ++d)
      tk[(nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d]) * stride] = kStagedNone;
  }
  // node src ships nothing this step unless its act writes an entry
  __host__ __device__ __forceinline__ void clear(const ScCtx& c, int src) const {
    ScNode& nd = c.nodes[src];
    for (int d = 0; d < nd.n_dests; ++d)
      for (int p = 0; p < c.P; ++p)
        tk[(nd.in_slot[d] + static_cast<int64_t>(p) * nd.in_stride[d]) * stride] = kStagedNone;
  }
};

// Everything node i does to heap (i, p) in step t, on a copy staged in `lh` (one heap,
// H entries): the drain of the shipments earlier nodes made to it, in source order (:347);
// the receive pops and the stock update (:220-228); the SUPPLY push (:243-259, the
// lead-time cursor `lt_i` and supply-action index `a_i` advanced as act advances them);
// then, the heap being final for the step, its in-transit bins (:445-461). Heap storage
// order is the reference's: the same pushes and pops happen in the same order.
template <class Sink>
__host__ __device__ inline void sc_staged_heap(const ScCtx& c, ScEnv& g, const HeapView8& lh, const StagedInbox& in,
                                               WordCache& ltc, const float* act, int t, int i, int p, int& a_i,
                                               int& lt_i, Sink& out, ScAcc& scg_acc_) {
  ScNode& nd = c.nodes[i];
  const HeapView gh = sc_heap(c, g, i, p);
  int32_t& gsz = sc_size(c, g, i, p);
  double& st = sc_stock(c, g, i, p);
  const double st0 = st;
  // Global loads go out kChunk at a time (all issued before the first is used), so a heap
  // copy or an inbox drain waits on memory once per chunk instead of once per entry; the
  // heap size, the stock and the first inbox chunk are requested together up front.
  // (kChunk = 8 pushed the kernel to 256 VGPRs, one wave per SIMD, and ran slower.)
  constexpr int kChunk = 4;
#ifndef SCG_STAGED_HCHUNK
#define SCG_STAGED_HCHUNK 8
#endif
  constexpr int kHeapChunk = SCG_STAGED_HCHUNK;  // heap slots per memory round
#ifndef SCG_STAGED_PLAIN
#define SCG_STAGED_PLAIN 1
#endif
  const int64_t q0 = nd.in_base + static_cast<int64_t>(p) * nd.in_deg;
  const int32_t t0 = t << 3;  // an absolute time<<3|kind minus t0 is the relative one
  HeapEntry ib[kChunk];
#pragma unroll
  for (int u = 0; u < kChunk; ++u)
    if (u < nd.in_deg) ib[u] = HeapEntry{in.tk[(q0 + u) * in.stride], in.val[(q0 + u) * in.stride]};
  // the heap's first kHeapChunk slots are requested with its size (slots past the size are
  // read but not used), the rest kHeapChunk at a time
  HeapEntry b[kHeapChunk];
#pragma unroll
  for (int u = 0; u < kHeapChunk; ++u)
    if (u < c.H) b[u] = gh.get(u);
  int32_t sz = gsz;
  SCG_ACC(7);
  bool plain = true;  // no Python int or float amount in the heap (he_less<true> applies)
#pragma unroll
  for (int u = 0; u < kHeapChunk; ++u)
    if (u < sz) {
      lh.put(u, HeapEntry{b[u].tk - t0, b[u].v});
      plain &= he_plain(b[u].tk);
    }
  for (int j0 = kHeapChunk; j0 < sz; j0 += kHeapChunk) {
#pragma unroll
    for (int u = 0; u < kHeapChunk; ++u)
      if (j0 + u < sz) b[u] = gh.get(j0 + u);
#pragma unroll
    for (int u = 0; u < kHeapChunk; ++u)
      if (j0 + u < sz) {
        lh.put(j0 + u, HeapEntry{b[u].tk - t0, b[u].v});
        plain &= he_plain(b[u].tk);
      }
  }
  SCG_ACC(0);
  for (int k0 = 0; k0 < nd.in_deg; k0 += kChunk) {
    if (k0 > 0) {
#pragma unroll
      for (int u = 0; u < kChunk; ++u)
        if (k0 + u < nd.in_deg)
          ib[u] = HeapEntry{in.tk[(q0 + k0 + u) * in.stride], in.val[(q0 + k0 + u) * in.stride]};
    }
#pragma unroll
    for (int u = 0; u < kChunk; ++u)  // in source order (:347)
      if (k0 + u < nd.in_deg && ib[u].tk != kStagedNone) {
        plain &= he_plain(ib[u].tk);
        if (!py_heappush(lh, sz, c.H, ib[u])) g.overflow = 1;
      }
  }
  SCG_ACC(1);
  // the pops, the phase's longest part, compare the doubles when no lane of the wave holds
  // a Python int or float amount (a wave-uniform choice, so no lane runs both bodies)
#if SCG_STAGED_PLAIN && defined(__HIP_DEVICE_COMPILE__)
  if (__all(plain))
    st = st0 + sc_receive<true>(lh, sz, 0);
  else
    st = st0 + sc_receive(lh, sz, 0);
#else
  st = st0 + (SCG_STAGED_PLAIN && plain ? sc_receive<true>(lh, sz, 0) : sc_receive(lh, sz, 0));
#endif
  SCG_ACC(2);
  if (nd.n_supply > 0 && nd.supply_capacity[p] > 0) {
    const Num amount = np_mul(sc_action(act, nd.action_offset + a_i), pyint(nd.supply_capacity[p]));
    ++a_i;
    if (np_lt(pyint(0), amount)) {
      const HeapEntry e{he_pack(node_leadtime(c, g, ltc, nd, t, lt_i), amount.k), amount.v};  // relative
      if (!py_heappush(lh, sz, c.H, e)) g.overflow = 1;
      ++lt_i;
    }
  }
  SCG_ACC(3);
  // relative times: the step is time 0; the copy back makes them absolute again
  sc_observe_bins(c, lh, sz, 0, i, p, out, [&](int k, const HeapEntry& e) { gh.put(k, HeapEntry{e.tk + t0, e.v}); });
  gsz = sz;
  SCG_ACC(4);
}

// SupplyChainEnv.step body (:704-738) plus the node part of _build_observation (:762-791)
// for time t. `g` views the env's state in HBM; `lh` is the one-heap staging area. Per
// node in order: its heaps one product at a time (sc_staged_heap), then act on everything
// else (no heap access: kHeapsDone), its shipments going to the inbox, then its stock
// shares. out(o, x) receives the node observation elements (the caller adds the demand and
// time-to-go ones). Returns the reward. (Staging the node's stocks in LDS as well measured
// no faster on MI355X: stock accesses are few and cache-resident.)
// ctx() gives the launch-uniform context; each node's iteration asks for it again (the
// kernel's KernargCtx re-reads it through a pointer the compiler cannot see across
// iterations, so nothing derived from it is held in registers across the node loop).
template <int MAXD, bool kKindPaths = false, class CtxFn, class Sink>
__host__ __device__ inline double sc_staged_step_ctx(const CtxFn& ctx, ScEnv& g, const HeapView8& lh,
                                                     const StagedInbox& in, const float* act, int t, Sink& out) {
  WordCache ltc{0, U4{0, 0, 0, 0}, false}, dmc{0, U4{0, 0, 0, 0}, false};
  Num total = pyint(0);
  SCG_ACC_DECL
#ifdef SCG_SC_STAMPS
  g.dbg = &scg_acc_;
#endif
  const int NN = ctx().n_nodes;
  for (int i = 0; i < NN; ++i) {
    const ScCtx& c = ctx();
    ScNode& nd = c.nodes[i];
    // the batch strides (uniform: the env-fastest layout) made opaque per node, so their many
    // multiples (slot and entry offsets) are formed where used, not held across the loop
    StagedInbox inl = in;
#if SCG_STAGED_OPAQUE_STRIDE
    g.stride = sc_opaque_val(g.stride);
    g.hstride = sc_opaque_val(g.hstride);
    inl.stride = sc_opaque_val(inl.stride);
#endif
    int a_i = 0, lt_i = 0;
    for (int p = 0; p < c.P; ++p) sc_staged_heap(c, g, lh, inl, ltc, act, t, i, p, a_i, lt_i, out, scg_acc_);
    if (!StagedInbox::kClearInAct && !nd.last_level) inl.clear(c, i);
    SCG_ACC(7);
    total = np_add(total, sc_node_act<MAXD, StagedInbox, true, kKindPaths>(c, g, ltc, dmc, i, act, t, inl));
    SCG_ACC(5);
    for (int p = 0; p < c.P; ++p) sc_observe_stock(c, g, i, p, out);
    SCG_ACC(6);
  }
  SCG_ACC_STORE;
  return np_neg(total).v;
}

template <int MAXD, bool kKindPaths = false, class Sink>
__host__ __device__ inline double sc_staged_step(const ScCtx& c, ScEnv& g, const HeapView8& lh, const StagedInbox& in,
                                                 const float* act, int t, Sink& out) {
  return sc_staged_step_ctx<MAXD, kKindPaths>(HostCtx{c}, g, lh, in, act, t, out);
}

}  // namespace scg
