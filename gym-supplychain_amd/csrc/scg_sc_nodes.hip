// Node-parallel SupplyChain step kernel for gfx950 (scg_supplychain_nodes.h).
//
// A block is 64 envs x W waves. Wave w owns nodes w, w + W, ... of all 64 envs, lane l env
// blockIdx.x * 64 + l: every wave runs one node's code (no divergence between node kinds)
// and every state access is a 64-env row of the env-fastest layout (coalesced). The lane
// kernel walks an env's whole chain on one lane, a chain of dependent LDS and FP64
// latencies at one or two waves per SIMD; here the chain is cut into W waves that run at
// once, so the same work hides its latencies behind W times as many waves.
//
// LDS per block (doubles first): the block's heaps [NP][H][64], released sums [NP][64],
// shipment inbox [E][64], node costs [NN][64], the observation tile [64][O|1] (float or
// double); then the int32 heap times/kinds, heap sizes, inbox times/kinds, cost kinds, the
// per-wave "order not provable" flags [W][64] and the action tile [64][A|1].
//   stage  (wave w, its nodes)  heaps HBM -> LDS, released sums, flags; every thread
//                               loads a share of the block's action rows (one contiguous
//                               span) into the action tile                    | barrier
//   act    (wave w, its nodes)  stock, costs, shipments -> inbox, stock obs   | barrier
//   heaps  (wave w, its nodes)  inbox pushes, pops, supply push, bins, copy back
//   reward (wave 0)             -(costs in node order), return, demand / time obs
//                                                                             | barrier
//   out    (every thread)       the observation tile -> HBM, one contiguous span per block;
//                               wave 0 resets its envs at an auto-reset step
// The grid is persistent: as many blocks as the device holds at once (two per CU), each
// stepping tiles of 64 envs in turn, with the launch arguments re-read per tile through a
// pointer the compiler cannot carry across tiles (nothing derived from them is held, or
// spilled, across the loop).
// An env any wave flagged skips act and heaps; wave 0 steps it alone on its staged heaps,
// node after node in the reference's order (sc_nodes_serial). Observations and actions go
// through LDS tiles so HBM sees whole rows; the state pointers stay the batch's base
// pointers (ScEnv soff/hoff) so they live in SGPRs.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "scg_common.h"
#include "scg_mailbox.h"
#if defined(SCG_NODES_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
// Diagnostic build only: every stamp (the phase boundaries NSTAMP below, and the end of each
// section of the act and heaps phases, SCG_ACCP(ptr, k) in scg_supplychain_core.h / _nodes.h)
// goes to the wave's slots in a static LDS array, and lane 0 copies them to HBM once, at the
// tile's end: a global store per stamp would make the next wait on the vector memory counter
// (loads and stores share it on gfx950) sit out that store's latency.
// LDS slots per wave: 0-7 phase stamps, 8 real-time clock at the start, 9 + j section j
// (sections k = 0..3 -> j = k, k = 7..13 -> j = k - 3).
constexpr int kNLdsSlots = 20;
__shared__ unsigned long long s_nodes_stamps[8 * kNLdsSlots];
#define SCG_STAMP(k)
#define SCG_ACC_DECL
#define SCG_ACC(k)
#define SCG_ACC_STORE
namespace scg {
struct ScAcc {  // a marker: a non-null ScEnv::dbg turns the section stamps on
  int unused;
};
}  // namespace scg
#define SCG_ACCP(ptr, k)                                                                              \
  do {                                                                                                \
    if (ptr) {                                                                                        \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();                                   \
      if ((threadIdx.x & 63u) == 0)                                                                   \
        s_nodes_stamps[(threadIdx.x / 64u) * kNLdsSlots + 9 + ((k) < 4 ? (k) : (k) - 3)] = now_;      \
    }                                                                                                 \
  } while (0)
#endif
#include "scg_supplychain_core.h"
#include "scg_supplychain_args.h"
#include "scg_supplychain_nodes.h"

// Diagnostic build only (-DSCG_NODES_STAMPS, tools/nodes_stamps.py): lane 0 of every wave
// records the shader clock at the phase boundaries (0 start, 5 heaps staged, 6 past the first
// barrier, 1 acted, 2 past the second, 3 heaps done, 7 past the third, 4 end) into a buffer of its own that scg_nodes_debug_stamps copies
// out; nothing else reads it. In the product build NSTAMP is empty.
#ifdef SCG_NODES_STAMPS
// Global record per wave: slots 0-7 the phase stamps, 8 and 9 the real-time clock (100 MHz,
// one clock for the chip) at start and end, 10 and 11 the wave's HW_ID and XCC_ID registers
// (where the block was placed), 12 + k the end of section k of the act and heaps phases.
constexpr int kNStampSlots = 28;
constexpr int kNStampWaves = 1 << 14;
__device__ unsigned long long g_nodes_stamps[kNStampWaves * kNStampSlots];
#if defined(__HIP_DEVICE_COMPILE__)
#define NSTAMP(k)                                                                                   \
  do {                                                                                              \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                                   \
    unsigned long long* l_ = s_nodes_stamps + (threadIdx.x / 64u) * kNLdsSlots;                     \
    if ((threadIdx.x & 63u) == 0) {                                                                 \
      l_[(k)] = now_;                                                                               \
      if ((k) == 0) l_[8] = __builtin_amdgcn_s_memrealtime();                                       \
    }                                                                                               \
    if ((k) == 4) {                                                                                 \
      const unsigned long long rt_ = __builtin_amdgcn_s_memrealtime();                              \
      const unsigned w_ = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;                      \
      if ((threadIdx.x & 63u) == 0 && w_ < static_cast<unsigned>(kNStampWaves)) {                   \
        unsigned long long* s_ = g_nodes_stamps + w_ * kNStampSlots;                                \
        for (int j_ = 0; j_ < 9; ++j_) s_[j_] = l_[j_];                                             \
        s_[9] = rt_;                                                                                \
        s_[10] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                                         \
        s_[11] = __builtin_amdgcn_s_getreg((31 << 11) | 20);                                        \
        for (int j_ = 0; j_ < 4; ++j_) s_[12 + j_] = l_[9 + j_];                                    \
        for (int j_ = 4; j_ < 11; ++j_) s_[12 + 3 + j_] = l_[9 + j_];                               \
      }                                                                                             \
    }                                                                                               \
  } while (0)
#else
#define NSTAMP(k)
#endif
#else
#define NSTAMP(k)
#endif

namespace scg {

constexpr int kNodesMaxWaves = 8;

// Row and column (r, k) of element q = r * width + k of a row-major tile, walked from q0 in
// steps of `step` with one division up front (the step's share is wave-uniform).
struct TileWalk {
  int r, k, dr, dk, width;
  __device__ __forceinline__ TileWalk(int q0, int step, int w) : width(w) {
    r = q0 / w;
    k = q0 - r * w;
    dr = step / w;
    dk = step - dr * w;
  }
  __device__ __forceinline__ void next() {
    r += dr;
    k += dk;
    if (k >= width) {
      k -= width;
      ++r;
    }
  }
};

// Ledger reduce right after each wave's heaps phase (1) or after the last barrier (0, the
// round-3 placement; A/B in DESIGN §6.7).
#ifndef SCG_NODES_LED_EARLY
#define SCG_NODES_LED_EARLY 1
#endif

#ifndef SCG_NODES_WPE
#define SCG_NODES_WPE 4
#endif
// Streaming (non-temporal) stores for the rows a step writes once and only the next step
// reads (heap copy-back, stocks, observations): 0 off, 1 the ledger instantiation only, 2
// every instantiation (sc-2perstage 37.4 -> 36.7 us; the ledger run within noise,
// profiles/r05j_nodes_nt_ab.log); write-through rather than non-temporal by SCG_NODES_WT
// (scg_supplychain_nodes.h).
#ifndef SCG_NODES_NT
#define SCG_NODES_NT 2
#endif
// One tile of 64 envs (tile * 64 ...): the step described at the top, on the kernel arguments
// `a`, except the step's time, flags and episode, which come from `sp` (sp.t(), sp.flags(),
// sp.episode(): the batch kernel's launch arguments, read where used as before; the step
// server's request), and the action rows (sp.act(a)). With sp.keep_state() the stage reads no
// state: the step server's block stepped this env last and its LDS still holds the stocks,
// sizes, heaps and episode return that step left. lane is the thread's lane, opaque to the
// compiler; w the wave index.
struct NodesLaunchStep {  // the batch kernel: the step fields of the launch arguments
  static constexpr bool kKeepsState = false;
  const ScArgs& a;
  __device__ __forceinline__ int t() const { return a.t; }
  __device__ __forceinline__ int flags() const { return a.flags; }
  __device__ __forceinline__ uint32_t episode() const { return a.episode; }
  __device__ __forceinline__ const float* act(const ScArgs& x) const { return x.act; }
  __device__ __forceinline__ bool keep_state() const { return false; }
};

template <int MAXD, bool F64, bool LED, class Step>
__device__ __forceinline__ void sc_nodes_tile(const ScArgs& a, int64_t tile, int lane, int w, int W, int E,
                                              const Step& sp) {
  using ObsT = typename std::conditional<F64, double, float>::type;
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr bool ledgers = LED;
  // streaming stores for the heap copy-back and the observation and stock rows (SCG_NODES_NT)
  constexpr bool kStream = SCG_NODES_NT == 2 || (SCG_NODES_NT == 1 && LED);
  const ScCtx& c = a.c;
  const int NN = c.n_nodes, P = c.P, NP = NN * P, H = c.H;
  const int Ap = c.A | 1, Op = c.O | 1;  // odd row strides: lanes hit distinct banks
  double* hval = reinterpret_cast<double*>(smem);
  double* recv = hval + static_cast<int64_t>(NP) * H * 64;  // released sums [NP][64]
  double* ibval = recv + NP * 64;
  double* cost_v = ibval + static_cast<int64_t>(E) * 64;
  double* stk = cost_v + NN * 64;  // the tile's stocks [NP][64] for the step
  double* ret0 = stk + NP * 64;    // episode returns [64] (wave 0's prefetch)
  ObsT* obs_t = reinterpret_cast<ObsT*>(ret0 + 64);
  int32_t* htk = reinterpret_cast<int32_t*>(obs_t + 64 * Op);
  int32_t* hsz = htk + static_cast<int64_t>(NP) * H * 64;
  int32_t* ibtk = hsz + NP * 64;
  int32_t* cost_k = ibtk + static_cast<int64_t>(E) * 64;
  int32_t* amb = cost_k + NN * 64;
  uint64_t* lword = reinterpret_cast<uint64_t*>(amb + W * 64);  // ledger entry marks and types [NP][64]
  float* act_t = reinterpret_cast<float*>(lword + NP * 64);
  const bool terminal = sp.flags() & 1;
  const bool autoreset = sp.flags() & 2;
  const int64_t n0 = tile * 64;
  const int64_t n = n0 + lane;
  const int nb = a.n - n0 < 64 ? static_cast<int>(a.n - n0) : 64;  // envs of this tile
  const bool live = lane < nb;
  auto lheap = [&](int hp) { return HeapView{htk + hp * H * 64 + lane, hval + hp * H * 64 + lane, 64}; };
  // heaps and sizes in HBM (the batch's base pointers, column n); stocks in the LDS copy
  ScEnv g{stk, a.tk, a.val, a.size, 64, a.n, static_cast<uint32_t>(a.env_offset + n), n, sp.episode(), 0};
  g.soff = lane;
  g.hoff = n;
  if (ledgers) {  // the nodes' entries to their slots (column n = base + n0 + soff), reduced below
    g.led_v = a.ledp_v + n0;
    g.led_stride = a.n;
    g.led_word = lword + lane;
    g.led_word_stride = 64;
  }
  NSTAMP(0);
#if defined(SCG_NODES_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
  ScAcc acc_{};
  g.dbg = &acc_;
#define NACC(k) SCG_ACCP(&acc_, k)
#else
#define NACC(k)
#endif

  // the step's observation row, whichever buffer(s) it goes to (chosen at the copy-out)
  ObsT* const orow = obs_t + lane * Op;
  auto sink = [&](int o, double x) { orow[o] = static_cast<ObsT>(x); };
  const NodesInbox in{ibtk + lane, ibval + lane, 64};
  const float* act = act_t + lane * Ap;

  // stage, one memory round: every thread requests its share of the tile's action rows
  // (one contiguous span), every wave its node's stocks, heap sizes and the first kStage
  // slots of each heap, wave 0 the episode returns; nothing is waited for until all are in
  // flight. Then everything to LDS, the rest of a longer heap, and what each heap releases.
  bool bad = false;
  {
    constexpr int kAct = 4;  // action elements per thread per round
    const float* src = sp.act(a) + n0 * c.A;
    const int na = nb * c.A;
    // the step server's state kept in LDS since its previous request (NodesServerStep)
    const bool keep = sp.keep_state();
    float av[kAct];
#pragma unroll
    for (int u = 0; u < kAct; ++u)
      if (static_cast<int>(threadIdx.x) + u * static_cast<int>(blockDim.x) < na) av[u] = src[threadIdx.x + u * blockDim.x];
    const double r0 = (w == 0 && live && a.ep_ret && !keep) ? a.ep_ret[n] : 0.0;
    for (int i = w; i < NN; i += W)
      for (int p = 0; p < P; ++p) {
        const int hp = i * P + p;
        if (!live) continue;
        if (keep) {  // stocks, sizes and heaps are this env's, as the last step left them
          bad |= !sc_recv_scan(lheap(hp), hsz[hp * 64 + lane], sp.t(), recv[hp * 64 + lane]);
          continue;
        }
        const int64_t r = static_cast<int64_t>(hp) * a.n + n;
        const double st = a.stock[r];
        const int32_t sz = a.size[r];
        stk[hp * 64 + lane] = st;
        hsz[hp * 64 + lane] = sz;
        const HeapView lh = lheap(hp);
        // the heap's first slots are requested with the size (sc_nodes_copy_heap, shared
        // with the host harness); a longer heap costs a round more
        sc_nodes_copy_heap(HeapView{a.tk + static_cast<int64_t>(hp) * H * a.n + n,
                                    a.val + static_cast<int64_t>(hp) * H * a.n + n, a.n},
                           lh, H, sz);
        bad |= !sc_recv_scan(lh, sz, sp.t(), recv[hp * 64 + lane]);
      }
    {
      TileWalk tw(threadIdx.x, blockDim.x, c.A);
#pragma unroll
      for (int u = 0; u < kAct; ++u, tw.next())
        if (static_cast<int>(threadIdx.x) + u * static_cast<int>(blockDim.x) < na) act_t[tw.r * Ap + tw.k] = av[u];
      for (int q = threadIdx.x + kAct * blockDim.x; q < na; q += blockDim.x, tw.next()) act_t[tw.r * Ap + tw.k] = src[q];
    }
    if (w == 0 && live && a.ep_ret && !keep) ret0[lane] = r0;
  }
  amb[w * 64 + lane] = bad ? 1 : 0;
  NSTAMP(5);
  __syncthreads();
  NSTAMP(6);
  bool flagged = (sp.flags() & 4) != 0;
  for (int v = 0; v < W; ++v) flagged |= amb[v * 64 + lane] != 0;
  const bool go = live && !flagged;

  // act: every node at once (a node's act needs only what its own heaps release)
  if (go)
    for (int i = w; i < NN; i += W) {
      const Num cst = sc_nodes_act<MAXD, !LED>(c, g, in, recv + i * P * 64 + lane, 64, act, sp.t(), i);
      NACC(12);
      cost_v[i * 64 + lane] = cst.v;
      cost_k[i * 64 + lane] = cst.k;
      for (int p = 0; p < P; ++p) sc_observe_stock(c, g, i, p, sink);
      NACC(13);
    }
  NSTAMP(1);
  __syncthreads();
  NSTAMP(2);

  // heaps
  if (go)
    for (int i = w; i < NN; i += W) {
      WordCache ltc{0, U4{0, 0, 0, 0}, false};
      int a_i = 0, lt_i = 0;
      for (int p = 0; p < P; ++p) {
        const int hp = i * P + p;
        sc_nodes_heap<kStream>(c, g, lheap(hp), hsz[hp * 64 + lane], in, ltc, act, sp.t(), i, p, a_i, lt_i, sink);
      }
    }
  NSTAMP(3);

  // ledgers: entry q of an env, the nodes' entries added in node order (:750-760); at an
  // auto-reset the finished episode's ledger is kept and the new one starts at int 0
  auto ledger_put = [&](int q, double lv, int32_t lk) {
    const int64_t at = q * a.n + n;
    if (autoreset) {
      if (a.led_fv) {
        a.led_fv[at] = lv;
        a.led_fk[at] = lk;
      }
      lv = 0.0;
      lk = np_kind_abi(NK_INT);
    }
    a.led_v[at] = lv;
    a.led_k[at] = lk;
  };
  // entries first, first + step, ... of an env, two at a time (their loads in flight together)
  auto ledger_entries = [&](int first, int step) {
    const int nq = 2 * SCG_SC_LEDGER_KEYS * P;
    for (int q0 = first; q0 < nq; q0 += 2 * step) {
      const int q1 = q0 + step < nq ? q0 + step : -1;
      const int64_t at0 = q0 * a.n + n, at1 = (q1 >= 0 ? q1 : q0) * a.n + n;
      double lv0 = a.led_v[at0], lv1 = a.led_v[at1];
      int32_t lk0 = a.led_k[at0], lk1 = a.led_k[at1];
      sc_ledger_reduce_pair(c, q0, q1, a.ledp_v + n, a.n, lword + lane, 64, lv0, lk0, lv1, lk1);
      ledger_put(q0, lv0, lk0);
      if (q1 >= 0) ledger_put(q1, lv1, lk1);
    }
  };
#if SCG_NODES_LED_EARLY
  // Every slot and mark of an acted env is in place since the act barrier, so each wave
  // reduces its share of the entries as soon as its heaps are done: the slot loads overlap
  // the other waves' heaps and wave 0's reward instead of forming a phase of their own after
  // the last barrier. A flagged env's slots are written by wave 0's serial walk below, which
  // then reduces that env's entries itself.
  if (ledgers && live && !flagged) ledger_entries(w, W);
#endif

  // reward
  if (w == 0 && live) {
    double reward;
    if (flagged) {  // untouched by act and heaps: the serial walk on its staged heaps
      reward = sc_nodes_serial<MAXD, !LED>(c, g, lheap, hsz + lane, 64, in, act, sp.t(), sink);
#if SCG_NODES_LED_EARLY
      if (ledgers) ledger_entries(0, 1);
#endif
    } else {
      Num total = pyint(0);
      for (int i = 0; i < NN; ++i) total = np_add(total, Num{cost_v[i * 64 + lane], cost_k[i * 64 + lane]});
      reward = np_neg(total).v;
    }
    a.rew[n] = reward;
    if (a.ep_ret) {
      const double r = ret0[lane] + reward;  // episode_rewards += current_reward (:739)
      if (terminal && a.final_ret) a.final_ret[n] = r;
      a.ep_ret[n] = autoreset ? 0.0 : r;
      if constexpr (Step::kKeepsState) ret0[lane] = autoreset ? 0.0 : r;  // the next request's
    }
    for (int k = 0; k < c.R * c.P; ++k) sc_observe_demand(c, g, sp.t(), k, sink);  // (:771)
    sc_observe_tail(c, sp.t(), sink);                                               // (:786)
  }
  __syncthreads();
  NSTAMP(7);

#if !SCG_NODES_LED_EARLY
  if (ledgers && live) ledger_entries(w, W);
#endif

  // out: the tile is this step's observation — obs, or the terminal observation when the
  // env resets now (then wave 0 writes the reset observation to obs), or both
  ObsT* const dst0 = static_cast<ObsT*>(autoreset ? a.term_obs : a.obs);
  ObsT* const dst1 = (terminal && !autoreset) ? static_cast<ObsT*>(a.term_obs) : nullptr;
  TileWalk tw(threadIdx.x, blockDim.x, c.O);
  for (int q = threadIdx.x; q < nb * c.O; q += blockDim.x, tw.next()) {
    const ObsT x = obs_t[tw.r * Op + tw.k];
    // (the step server's rows go to host-mapped memory: plain stores there)
    if constexpr (kStream && !Step::kKeepsState && SCG_NODES_WT >= 2) {
      if (dst0) __hip_atomic_store(&dst0[n0 * c.O + q], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (dst1) __hip_atomic_store(&dst1[n0 * c.O + q], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (kStream && !Step::kKeepsState) {
      if (dst0) __builtin_nontemporal_store(x, &dst0[n0 * c.O + q]);
      if (dst1) __builtin_nontemporal_store(x, &dst1[n0 * c.O + q]);
    } else {
      if (dst0) dst0[n0 * c.O + q] = x;
      if (dst1) dst1[n0 * c.O + q] = x;
    }
  }
  if (autoreset) {  // after the barrier every wave's heap copy-back has landed
    if (w == 0 && live) {
      g.episode = sp.episode() + 1;
      g.led_v = nullptr;   // the ledger was restarted above
      sc_reset_env(c, g);  // heaps in HBM, stocks in the LDS copy
      ObsRow out{a.obs, n * c.O, F64 ? 1 : 0};
      sc_observe(c, g, 0, out);
    }
    __syncthreads();
  }
  if (live) {  // the stocks of this wave's nodes back, one 64-env row per instruction (the
               // next tile's stage rewrites these rows: the same wave)
    for (int i = w; i < NN; i += W)
      for (int p = 0; p < P; ++p) {
        if constexpr (kStream && SCG_NODES_WT >= 2)
          __hip_atomic_store(&a.stock[(i * P + p) * a.n + n], stk[(i * P + p) * 64 + lane], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        else if constexpr (kStream)
          __builtin_nontemporal_store(stk[(i * P + p) * 64 + lane], &a.stock[(i * P + p) * a.n + n]);
        else
          a.stock[(i * P + p) * a.n + n] = stk[(i * P + p) * 64 + lane];
      }
    if (g.overflow) atomicOr(a.err, 1);
  }
  NSTAMP(4);
#undef NACC
  // the next tile's stage rewrites the action tile, ret0 and, per wave, only the stock, size
  // and heap rows of its own nodes (whose stocks it copied back just above); the rows other
  // waves read (the observation tile) are next written after that tile's first barrier
}

// Four waves per SIMD (<= 128 VGPRs): two blocks of eight waves per CU, which is also what
// their LDS allows.
// F64: float64 observations; LED: build_info ledgers (a separate instantiation, so the
// ledger code costs the common run nothing).
// Persistent: block b steps tiles b, b + gridDim.x, ... (64 envs each); the launch sizes the
// grid to the blocks the device holds at once, so the second round of tiles needs no new
// blocks and each block's next tile follows its last without a dispatch.
template <int MAXD, bool F64, bool LED>
__global__ __launch_bounds__(64 * kNodesMaxWaves) __attribute__((amdgpu_waves_per_eu(SCG_NODES_WPE)))
void sc_step_nodes_kernel(const ScArgs a_arg, int W, int E) {
  // the wave index is wave-uniform: said so, node records are read with scalar loads
  const int lane0 = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_tiles = (a_arg.n + 63) / 64;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    // the lane index, opaque to the compiler inside each tile: the per-lane LDS and HBM
    // addresses derived from it are computed where used, not hoisted out of the tile loop
    // and held in registers across it (which spilled the kernel at its 128-VGPR budget)
    int lane;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane0));
    // the launch arguments through a pointer the compiler cannot see across tiles: each tile
    // reads them (scalar loads) and derives its addresses itself, instead of every derived
    // value being hoisted out of the loop and held in scalar registers across it
    typedef const __attribute__((address_space(4))) ScArgs* KArgPtr;
    KArgPtr ap = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    const ScArgs& a = *(const ScArgs*)ap;
    sc_nodes_tile<MAXD, F64, LED>(a, tile, lane, w, W, E, NodesLaunchStep{a});
  }
}

// ---- step server for the drop-in SupplyChainEnv (include/scgpu.h scg_sc_server_*) --------
// One block of the batch kernel's shape, resident: wave 0 polls the mailbox's request lines
// (the request and the inline action row, lanes 0-31, system scope, with the exit word) and
// puts what it found in LDS; after a barrier every wave either exits, sleeps and polls again,
// or runs tile 0 of the step with the request's time, flags, episode and action row
// (NodesServerStep) — the batch kernel's code, minus the state loads when the block's LDS
// still holds the state of this env's previous step — and then, past a barrier, thread 0
// publishes the request number with a system-scope release store (wave 0 acquired when it
// found the request: one cache invalidation and one L2 write-back per step for the block). At launch the
// last request served is the answer word, so a request posted while no block ran is served
// first. It exits when exit_req changes or after idle_ticks of the 100 MHz real-time clock
// without a request, and writes the exit word it saw as it goes.
__shared__ int32_t s_srv_req[5];  // t, flags, episode, command (0 none, 1 / 3 step, 2 exit), keep
__shared__ float s_srv_act[16];   // env 0's action row when it travelled in the request
#ifdef SCG_NODES_STAMPS
// Diagnostic build only (tools/sc_server_phase_probe.py): per wave, the shader clocks of each
// phase of every served step summed — [0] request seen -> tile start, then the tile's phases
// in order (stamps 0 -> 5 -> 6 -> 1 -> 2 -> 3 -> 7 -> 4), [8] tile end -> past the closing
// barrier, [9] the steps served — read without a device sync by scg_sc_server_debug_phases.
__device__ unsigned long long g_srv_phases[kNodesMaxWaves][10];
__shared__ unsigned long long s_srv_seen;
#endif
struct NodesServerStep {
  static constexpr bool kKeepsState = true;
  bool inline_act;
  __device__ __forceinline__ int t() const { return s_srv_req[0]; }
  __device__ __forceinline__ int flags() const { return s_srv_req[1]; }
  __device__ __forceinline__ uint32_t episode() const { return static_cast<uint32_t>(s_srv_req[2]); }
  __device__ __forceinline__ const float* act(const ScArgs& x) const { return inline_act ? s_srv_act : x.act; }
  __device__ __forceinline__ bool keep_state() const { return s_srv_req[4] != 0; }
};

template <int MAXD>
__global__ __launch_bounds__(64 * kNodesMaxWaves) void sc_nodes_server_kernel(const ScArgs a, int W, int E,
                                                                               scg_sc_server_box* box,
                                                                               uint32_t exit_seen, uint32_t idle_ticks) {
  const int lane0 = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t* line = reinterpret_cast<const uint32_t*>(box);
  uint32_t last = __hip_atomic_load(&box->done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint32_t ex = exit_seen;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // wave 0: whether the LDS holds an env state this block stepped, and that step's episode
  // and time (a request for the next time of the same episode finds its state there)
  bool have = false;
  uint32_t last_ep = 0;
  int32_t last_t = 0;
  for (;;) {
    if (w == 0) {
      // the request (line 0) and the inline action row (line 1) in one load, with the exit word
      const uint32_t v = lane0 < 32 ? __hip_atomic_load(line + lane0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
      ex = __hip_atomic_load(&box->exit_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint32_t q[32];
#pragma unroll
      for (int i = 0; i < 32; ++i) q[i] = __builtin_amdgcn_readlane(v, i);
      int cmd = 0;
      if (ex != exit_seen) {
        cmd = 2;
      } else if (q[0] != last && q[7] == mailbox_check(q)) {
        cmd = (q[5] & 1u) ? 3 : 1;  // 3: a step whose action row came in line 1
        last = q[0];
        const int32_t t = static_cast<int32_t>(q[2]);
        const bool keep = have && !(q[5] & 2u) && q[4] == last_ep && t == last_t + 1;
        if (lane0 == 0) {
          s_srv_req[0] = t;
          s_srv_req[1] = static_cast<int32_t>(q[3]);
          s_srv_req[2] = static_cast<int32_t>(q[4]);
          s_srv_req[4] = keep ? 1 : 0;
        }
        if (lane0 >= 16 && lane0 < 32) s_srv_act[lane0 - 16] = __uint_as_float(v);
        // the acquire for the whole block: one wave's invalidation of the CU's caches and the
        // L2 serves every wave, which the barrier below orders after it
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#ifdef SCG_NODES_STAMPS
        if (lane0 == 0) s_srv_seen = __builtin_amdgcn_s_memtime();
#endif
        have = true;
        last_ep = q[4];
        last_t = t;
      } else if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
        cmd = 2;
      }
      if (lane0 == 0) s_srv_req[3] = cmd;
    }
    __syncthreads();
    const int cmd = __builtin_amdgcn_readfirstlane(s_srv_req[3]);
    __syncthreads();  // every wave has read the command before wave 0 writes the next one
    if (cmd == 2) break;
    if (cmd == 0) {
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    int lane;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane0));
    sc_nodes_tile<MAXD, true, false>(a, 0, lane, w, W, E, NodesServerStep{cmd == 3});
    // every wave's stores happen before thread 0's system-scope release store through the
    // barrier, so one write-back of the L2 (the store's release) publishes them all; a fence in
    // each of the W waves would write the L2 back W times (2.5 us per step for W = 8)
    __syncthreads();
#if defined(SCG_NODES_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
    {
      const unsigned long long past = __builtin_amdgcn_s_memtime();
      const unsigned long long* l_ = s_nodes_stamps + w * kNLdsSlots;
      if (lane0 == 0 && w < kNodesMaxWaves) {
        const int order[8] = {0, 5, 6, 1, 2, 3, 7, 4};
        unsigned long long* acc = g_srv_phases[w];
        acc[0] += l_[0] - s_srv_seen;
        for (int k = 1; k < 8; ++k) acc[k] += l_[order[k]] - l_[order[k - 1]];
        acc[8] += past - l_[4];
        acc[9] += 1;
      }
    }
#endif
    if (threadIdx.x == 0) __hip_atomic_store(&box->done_seq, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    t0 = __builtin_amdgcn_s_memrealtime();
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (threadIdx.x == 0) __hip_atomic_store(&box->exit_seq, ex, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LDS bytes of one block (the layout above); obs_bytes 4 (float) or 8 (double).
size_t sc_nodes_lds_bytes(int n_nodes, int P, int H, int E, int W, int A, int O, int obs_bytes) {
  const size_t NP = static_cast<size_t>(n_nodes) * P;
  return 64 * ((NP * H + 2 * NP + E + n_nodes + 1) * 8 + static_cast<size_t>(O | 1) * obs_bytes +
               (NP * H + NP + E + n_nodes + W) * 4 + NP * 8 + static_cast<size_t>(A | 1) * 4);
}

// Widest destination list the kernel is instantiated for (its split runs in registers).
int sc_nodes_max_dests() { return 8; }

// Waves per block for a chain: one per node up to kNodesMaxWaves.
int sc_nodes_waves(int n_nodes) { return n_nodes < kNodesMaxWaves ? n_nodes : kNodesMaxWaves; }

// A block may use up to the CU's whole LDS (gfx950: 160 KiB; asked of the device once, the
// gfx950 figure when no device answers, e.g. scg_sc_prepare on a host without a GPU); past
// 64 KiB the kernel is told once per device that it may.
constexpr size_t kNodesLdsGfx950 = 160 * 1024;
size_t sc_nodes_lds_max() {
  static std::atomic<size_t> cached{0};
  size_t v = cached.load(std::memory_order_relaxed);
  if (v) return v;
  int dev = 0, bytes = 0;
  v = (hipGetDevice(&dev) == hipSuccess &&
       hipDeviceGetAttribute(&bytes, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) == hipSuccess && bytes > 0)
          ? static_cast<size_t>(bytes)
          : kNodesLdsGfx950;
  cached.store(v, std::memory_order_relaxed);
  return v;
}

// Blocks the device holds at once for this instantiation (occupancy x CUs), asked once per
// device and shape; the persistent grid is that many blocks, or one per tile when fewer.
template <int MAXD, bool F64, bool LED>
int64_t sc_nodes_resident_blocks(int dev, int W, size_t lds) {
  struct Entry {
    int dev, W;
    size_t lds;
    int64_t blocks;
  };
  static std::mutex mu;
  static std::vector<Entry> cache;
  std::lock_guard<std::mutex> lock(mu);
  for (const Entry& e : cache)
    if (e.dev == dev && e.W == W && e.lds == lds) return e.blocks;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&sc_step_nodes_kernel<MAXD, F64, LED>),
                                                   64 * W, lds) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1 || cus < 1)
    return 0;  // unknown: one block per tile
  cache.push_back(Entry{dev, W, lds, static_cast<int64_t>(per_cu) * cus});
  return cache.back().blocks;
}

#ifndef SCG_NODES_PERSISTENT
#define SCG_NODES_PERSISTENT 1
#endif

#ifndef SCG_NODES_LED_PERSISTENT
#define SCG_NODES_LED_PERSISTENT 0
#endif

std::atomic<int> g_nodes_max_blocks{0};  // scg_sc_nodes_max_blocks (tests)
#ifdef SCG_NODES_STAMPS
constexpr size_t kNodesStaticLds = 8 * 20 * sizeof(unsigned long long);  // s_nodes_stamps
#else
constexpr size_t kNodesStaticLds = 0;
#endif

template <int MAXD, bool F64, bool LED>
int sc_launch_nodes_d(const ScArgs& a, int W, int E, hipStream_t s) {
  static std::atomic<bool> raised[64] = {};  // per device
  const size_t lds = sc_nodes_lds_bytes(a.c.n_nodes, a.c.P, a.c.H, E, W, a.c.A, a.c.O, F64 ? 8 : 4);
  if (lds > sc_nodes_lds_max()) return fail(SCG_ERR_INVALID, "node-parallel kernel: %zu B of LDS per block", lds);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > 64 * 1024 && !raised[dev].load(std::memory_order_acquire)) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&sc_step_nodes_kernel<MAXD, F64, LED>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(sc_nodes_lds_max() - kNodesStaticLds)) != hipSuccess)
      return fail(SCG_ERR_HIP, "node-parallel kernel: cannot raise its LDS limit");
    raised[dev].store(true, std::memory_order_release);
  }
  const int64_t tiles = (a.n + 63) / 64;
  int64_t blocks = tiles;
  // the ledger instantiation keeps one block per tile (persistent measured 55.4 -> 56.7 us,
  // profiles/r05f_nodes_persistent_ab.log)
  if (SCG_NODES_PERSISTENT && (!LED || SCG_NODES_LED_PERSISTENT)) {
    const int64_t resident = sc_nodes_resident_blocks<MAXD, F64, LED>(dev, W, lds);
    if (resident > 0 && resident < tiles) blocks = resident;
  }
  const int cap = g_nodes_max_blocks.load(std::memory_order_relaxed);
  if (cap > 0 && cap < blocks) blocks = cap;
  hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_step_nodes_kernel<MAXD, F64, LED>), dim3(static_cast<unsigned>(blocks)),
                     dim3(64 * W), lds, s, a, W, E);
  return check_launch("sc_step_nodes_kernel");
}

int sc_launch_nodes(const ScArgs& a, int maxd_bucket, int W, int E, hipStream_t s) {
  if (W < 1 || W > kNodesMaxWaves) return fail(SCG_ERR_INVALID, "node-parallel kernel: %d waves per block", W);
  const int v = (a.obs_f64 ? 1 : 0) | (a.led_v && a.ledp_v ? 2 : 0);
#define SCG_NODES_CASES(D)                                  \
  switch (v) {                                              \
    case 0: return sc_launch_nodes_d<D, false, false>(a, W, E, s); \
    case 1: return sc_launch_nodes_d<D, true, false>(a, W, E, s);  \
    case 2: return sc_launch_nodes_d<D, false, true>(a, W, E, s);  \
    default: return sc_launch_nodes_d<D, true, true>(a, W, E, s);  \
  }
  switch (maxd_bucket) {
    case 2: SCG_NODES_CASES(2)
    case 4: SCG_NODES_CASES(4)
    case 8: SCG_NODES_CASES(8)
    default: return fail(SCG_ERR_INVALID, "node-parallel kernel: nodes ship to at most 8 destinations");
  }
#undef SCG_NODES_CASES
}

// The step server's block for a config the batch kernel runs (float64 observations, no
// ledgers): one block of W waves with the batch kernel's LDS.
int sc_launch_nodes_server(const ScArgs& a, int maxd_bucket, int W, int E, hipStream_t s, scg_sc_server_box* box,
                           uint32_t exit_seen, uint32_t idle_ticks) {
  if (W < 1 || W > kNodesMaxWaves) return fail(SCG_ERR_INVALID, "node-parallel server: %d waves per block", W);
  if (!a.obs_f64 || a.led_v) return fail(SCG_ERR_INVALID, "the SupplyChain step server runs float64 observations, no ledgers");
  const size_t lds = sc_nodes_lds_bytes(a.c.n_nodes, a.c.P, a.c.H, E, W, a.c.A, a.c.O, 8);
  const size_t cap = sc_nodes_lds_max() - kNodesStaticLds - 1024;  // room for the static request words and action row
  if (lds > cap) return fail(SCG_ERR_INVALID, "node-parallel server: %zu B of LDS per block", lds);
  static std::atomic<bool> raised[3][64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
#define SCG_SERVER_LAUNCH(D, K)                                                                                     \
  if (lds > 64 * 1024 && !raised[K][dev].load(std::memory_order_acquire)) {                                         \
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&sc_nodes_server_kernel<D>),                             \
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(cap)) != hipSuccess)       \
      return fail(SCG_ERR_HIP, "node-parallel server: cannot raise its LDS limit");                                 \
    raised[K][dev].store(true, std::memory_order_release);                                                          \
  }                                                                                                                 \
  hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_nodes_server_kernel<D>), dim3(1), dim3(64 * W), lds, s, a, W, E, box,       \
                     exit_seen, idle_ticks);                                                                        \
  break;
  switch (maxd_bucket) {
    case 2: SCG_SERVER_LAUNCH(2, 0)
    case 4: SCG_SERVER_LAUNCH(4, 1)
    case 8: SCG_SERVER_LAUNCH(8, 2)
    default: return fail(SCG_ERR_INVALID, "node-parallel server: nodes ship to at most 8 destinations");
  }
#undef SCG_SERVER_LAUNCH
  return check_launch("sc_nodes_server_kernel");
}

}  // namespace scg

extern "C" __attribute__((visibility("default"))) int scg_sc_nodes_max_blocks(int32_t blocks) {
  return scg::g_nodes_max_blocks.exchange(blocks < 0 ? 0 : blocks);
}

#ifdef SCG_NODES_STAMPS
// Diagnostic build only: copy the stamps of the first `waves` waves to host memory.
extern "C" __attribute__((visibility("default"))) int scg_nodes_debug_stamps(unsigned long long* host, int waves) {
  if (waves > kNStampWaves) waves = kNStampWaves;
  if (hipDeviceSynchronize() != hipSuccess) return scg::fail(SCG_ERR_HIP, "sync");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nodes_stamps), sizeof(unsigned long long) * kNStampSlots * waves) !=
      hipSuccess)
    return scg::fail(SCG_ERR_HIP, "stamp copy");
  return SCG_OK;
}

// Diagnostic build only: the step server's per-wave phase sums (g_srv_phases) to host memory
// (8 x 10 words), on a stream of its own, without waiting for the resident server block;
// reset != 0 clears them afterwards.
extern "C" __attribute__((visibility("default"))) int scg_sc_server_debug_phases(unsigned long long* host, int reset) {
  (void)hipGetLastError();  // an error an earlier call left behind is not this probe's
  static unsigned long long* pinned = nullptr;
  if (!pinned && hipHostMalloc(reinterpret_cast<void**>(&pinned), sizeof(scg::g_srv_phases), 0) != hipSuccess)
    return scg::fail(SCG_ERR_HIP, "phase probe: pinned buffer");
  void* dev = nullptr;
  if (hipGetSymbolAddress(&dev, HIP_SYMBOL(scg::g_srv_phases)) != hipSuccess) return scg::fail(SCG_ERR_HIP, "symbol");
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return scg::fail(SCG_ERR_HIP, "stream");
  int rc = SCG_OK;
  hipError_t e = hipMemcpyAsync(pinned, dev, sizeof(scg::g_srv_phases), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) rc = scg::fail(SCG_ERR_HIP, "phase copy: %s", hipGetErrorString(e));
  if (rc == SCG_OK) {
    std::memcpy(host, pinned, sizeof(scg::g_srv_phases));
    if (reset) {
      e = hipMemsetAsync(dev, 0, sizeof(scg::g_srv_phases), s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) rc = scg::fail(SCG_ERR_HIP, "phase reset: %s", hipGetErrorString(e));
    }
  }
  (void)hipStreamDestroy(s);
  return rc;
}
#endif
