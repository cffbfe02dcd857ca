// SupplyChainEnv hot path for gfx950: reset / step kernels + their C-ABI launchers.
//
// Reference: gym_supplychain/envs/supplychain_env.py (snapshot 2024-08-07). One lane owns
// one env (its whole chain, every node in nodes_info order, as SupplyChainEnv.step walks
// them, :714-736); the per-env body is scg_supplychain_core.h. State arrays are
// env-fastest ([slot][N]) so lanes touching the same node/heap slot read one contiguous
// row; heap positions are data-dependent, so heap traffic is row-gathered through L2.
// The chain description (scg_sc_node[]) is wave-uniform and read with scalar loads (constant
// address space, ScNode in scg_supplychain_core.h).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "scg_common.h"
#include "scg_mailbox.h"

// Diagnostic build only (-DSCG_SC_STAMPS, tools/sc_stamps.py): lane 0 of every wave of the
// LDS lane kernel records the shader clock at phase boundaries into a buffer of its own
// (g_sc_stamps, read back by scg_sc_debug_stamps); nothing else reads it. 0 start, 1 heaps
// staged, 2.. after each node's act (node i at 2 + min(i, 20)), 23 return, 24 observation,
// 25 heaps stored. In the product build SCG_STAMP is empty.
#ifdef SCG_SC_STAMPS
constexpr int kStampSlots = 32;
constexpr int kStampWaves = 1 << 16;
__device__ unsigned long long g_sc_stamps[kStampWaves * kStampSlots];
#if defined(__HIP_DEVICE_COMPILE__)
#define SCG_STAMP(k)                                                                                  \
  do {                                                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                                     \
    const unsigned w_ = blockIdx.x * ((blockDim.x + 63u) / 64u) + threadIdx.x / 64u;                 \
    if ((threadIdx.x & 63u) == 0 && w_ < static_cast<unsigned>(kStampWaves)) g_sc_stamps[w_ * kStampSlots + (k)] = now_; \
  } while (0)
namespace scg {
struct ScAcc {
  unsigned long long a[16];
  unsigned long long last;
};
}  // namespace scg
#define SCG_ACC_DECL scg::ScAcc scg_acc_{{0}, __builtin_amdgcn_s_memtime()};
#define SCG_ACCP(ptr, k)                                           \
  do {                                                             \
    if (ptr) {                                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
      (ptr)->a[k] += now_ - (ptr)->last;                           \
      (ptr)->last = now_;                                          \
    }                                                              \
  } while (0)
#define SCG_ACC(k)                                               \
  do {                                                           \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    scg_acc_.a[k] += now_ - scg_acc_.last;                       \
    scg_acc_.last = now_;                                        \
  } while (0)
#define SCG_ACC_STORE                                                                             \
  do {                                                                                            \
    const unsigned w_ = blockIdx.x * ((blockDim.x + 63u) / 64u) + threadIdx.x / 64u;             \
    if ((threadIdx.x & 63u) == 0 && w_ < static_cast<unsigned>(kStampWaves))                      \
      for (int k_ = 0; k_ < 16; ++k_) g_sc_stamps[w_ * kStampSlots + 16 + k_] = scg_acc_.a[k_];          \
  } while (0)
#endif
#endif

#ifndef SCG_SC_LDS_PROBE
#define SCG_SC_LDS_PROBE 0
#endif
#include "scg_supplychain_core.h"
#include "scg_supplychain_args.h"
#include "scg_supplychain_level.h"
#include "scg_supplychain_staged.h"
#include "scgpu.h"

namespace scg {

// scg_sc_nodes.hip
size_t sc_nodes_lds_bytes(int n_nodes, int P, int H, int E, int W, int A, int O, int obs_bytes);
int sc_nodes_waves(int n_nodes);
int sc_nodes_max_dests();
size_t sc_nodes_lds_max();
int sc_launch_nodes(const ScArgs& a, int maxd_bucket, int W, int E, hipStream_t s);
int sc_launch_nodes_server(const ScArgs& a, int maxd_bucket, int W, int E, hipStream_t s, scg_sc_server_box* box,
                           uint32_t exit_seen, uint32_t idle_ticks);

__global__ __launch_bounds__(kScBlock) void sc_reset_kernel(const ScArgs a) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kScBlock + threadIdx.x;
  if (n >= a.n) return;
  ScEnv e = env_view(a, n, a.episode);
  sc_reset_env(a.c, e);
  if (a.obs) {
    ObsRow out{a.obs, n * a.c.O, a.obs_f64};
    sc_observe(a.c, e, 0, out);
  }
  if (a.ep_ret) a.ep_ret[n] = 0.0;
  if (e.overflow) atomicOr(a.err, 1);
}

template <int MAXD>
__global__ __launch_bounds__(kScBlock) void sc_step_kernel(const ScArgs a) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kScBlock + threadIdx.x;
  if (n >= a.n) return;
  sc_lane_step<MAXD>(a, n);
}

// The same step with this block's EPB env heaps staged in LDS: heap pushes/pops/walks are
// chains of dependent accesses, so they run at LDS latency instead of L2/HBM latency.
// Layout [slot][lane] (lane fastest): any mix of per-lane heap positions is bank-conflict
// free. Stock stays in HBM (a few accesses per node). Rows are staged in and out with
// coalesced transfers, copying only the live entries (< heap size) of each lane.
// EPB (envs = threads per block) is 64, or 32 when the batch is too small to give every
// SIMD two full waves: a step is one long dependent chain per lane, and at one wave per
// SIMD nothing hides its latency, so two half-full waves finish sooner than one full one.
template <int MAXD, int EPB>
__global__ __launch_bounds__(EPB) void sc_step_lds_kernel(const ScArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * EPB + lane;
  const ScCtx& c = a.c;
  const int NP = c.n_nodes * c.P;
  const int slots = NP * c.H;
  SCG_STAMP(0);
  double* lval = reinterpret_cast<double*>(smem);
  int32_t* ltk = reinterpret_cast<int32_t*>(lval + static_cast<int64_t>(slots) * EPB);
  int32_t* lsize = ltk + static_cast<int64_t>(slots) * EPB;
  const bool live = n < a.n;
  if (live) {
    for (int hp = 0; hp < NP; ++hp) {
      const int32_t sz = a.size[hp * a.n + n];
      lsize[hp * EPB + lane] = sz;
      for (int j = 0; j < sz; ++j) {
        const int64_t g = (static_cast<int64_t>(hp) * c.H + j) * a.n + n;
        ltk[(hp * c.H + j) * EPB + lane] = a.tk[g];
        lval[(hp * c.H + j) * EPB + lane] = a.val[g];
      }
    }
  }
#if SCG_SC_LDS_PROBE
  double* lstock = reinterpret_cast<double*>(lsize + NP * EPB);
  float* lact = reinterpret_cast<float*>(lstock + NP * EPB);
  if (live) {
    for (int k = 0; k < NP; ++k) lstock[k * EPB + lane] = a.stock[k * a.n + n];
    for (int k = 0; k < c.A; ++k) lact[lane * c.A + k] = a.act[n * c.A + k];
  }
  const float* act_row = lact + lane * c.A;
  double* stock_col = lstock + lane;
  const int64_t stock_stride = EPB;
#else
  const float* act_row = a.act + n * c.A;
  double* stock_col = a.stock + n;
  const int64_t stock_stride = a.n;
#endif
  SCG_STAMP(1);
  if (!live) return;  // no block-wide sync below: every lane only touches its own column
  ScEnv e{stock_col, ltk + lane, lval + lane, lsize + lane, stock_stride, EPB,
          static_cast<uint32_t>(a.env_offset + n), n, a.episode, 0};
  if (a.led_v) {
    e.led_v = a.led_v + n;
    e.led_k = a.led_k + n;
    e.led_stride = a.n;
  }
  const double reward = sc_step_env<MAXD>(c, e, act_row, a.t);
  a.rew[n] = reward;
  const bool terminal = a.flags & 1;
  if (a.ep_ret) {
    const double r = a.ep_ret[n] + reward;
    if (terminal && a.final_ret) a.final_ret[n] = r;
    a.ep_ret[n] = (a.flags & 2) ? 0.0 : r;
  }
  SCG_STAMP(23);
  if (a.flags & 2) {
    if (a.term_obs) {
      ObsRow tout{a.term_obs, n * c.O, a.obs_f64};
      sc_observe(c, e, a.t, tout);
    }
    snapshot_ledger(a, c, n);
    e.episode = a.episode + 1;
    sc_reset_env(c, e);
    ObsRow out{a.obs, n * c.O, a.obs_f64};
    sc_observe(c, e, 0, out);
  } else {
    ObsRow out{a.obs, n * c.O, a.obs_f64};
    sc_observe(c, e, a.t, out);
    if (terminal && a.term_obs) {
      ObsRow tout{a.term_obs, n * c.O, a.obs_f64};
      sc_observe(c, e, a.t, tout);
    }
  }
  SCG_STAMP(24);
#if SCG_SC_LDS_PROBE
  for (int k = 0; k < NP; ++k) a.stock[k * a.n + n] = lstock[k * EPB + lane];
#endif
  if (e.overflow) atomicOr(a.err, 1);
  for (int hp = 0; hp < NP; ++hp) {
    const int32_t sz = lsize[hp * EPB + lane];
    a.size[hp * a.n + n] = sz;
    for (int j = 0; j < sz; ++j) {
      const int64_t g = (static_cast<int64_t>(hp) * c.H + j) * a.n + n;
      a.tk[g] = ltk[(hp * c.H + j) * EPB + lane];
      a.val[g] = lval[(hp * c.H + j) * EPB + lane];
    }
  }
  SCG_STAMP(25);
}

// Node-staged step (scg_supplychain_staged.h): one lane per env; the heap being worked on
// is staged in LDS ([slot][lane], lane fastest: conflict free), the
// shipments go through the env's HBM inbox, the node's observation is written while its
// heaps are staged. No block-wide barrier: every lane only touches its own LDS column.
#ifndef SCG_STAGED_WPE
#define SCG_STAGED_WPE 0  // 0: the compiler's choice
#endif
// LED: build_info ledgers kept (a separate instantiation: without it every ledger note,
// and the per-destination unit sums only ledgers read, compile away).
// The staged kernel's context re-read per node (KernargCtx): 249 -> 199 VGPRs and a third of
// the SGPR spill reloads, yet 2.3 % slower on ntom (3.97 -> 4.07 ms, profiles/r05e_*), so off.
#ifndef SCG_STAGED_KARG_CTX
#define SCG_STAGED_KARG_CTX 0
#endif
template <int MAXD, bool LED>
__global__ __launch_bounds__(kScBlock)
#if SCG_STAGED_WPE
__attribute__((amdgpu_waves_per_eu(SCG_STAGED_WPE)))
#endif
void sc_step_staged_kernel(const ScArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kScBlock + lane;
  if (n >= a.n) return;
  const ScCtx& c = a.c;
  double* lval = reinterpret_cast<double*>(smem);
  const int slots = c.H > MAXD ? c.H : MAXD;  // sc_staged_lds_bytes: 9 bytes per slot and lane
  uint8_t* ltk = reinterpret_cast<uint8_t*>(lval + static_cast<int64_t>(slots) * kScBlock);
  ScEnv g = env_view(a, n, a.episode);
  if constexpr (!LED) {
    g.led_v = nullptr;
    g.led_k = nullptr;
  }
  const HeapView8 lh{ltk + lane, lval + lane, kScBlock};
  const StagedInbox in{a.inbox_tk + n, a.inbox_val + n, a.n, lh, a.t};
  const bool terminal = a.flags & 1;
  const bool autoreset = a.flags & 2;
  // node observations go to obs, or to the terminal observation when the env resets now
  void* node_obs = autoreset ? a.term_obs : a.obs;
  ObsRow main{node_obs ? node_obs : a.obs, n * c.O, a.obs_f64};
  ObsRow extra{a.term_obs, n * c.O, a.obs_f64};
  const bool both = terminal && !autoreset && a.term_obs;
  auto sink = [&](int o, double x) {
    if (node_obs) main(o, x);
    if (both) extra(o, x);
  };
#if SCG_STAGED_KARG_CTX
  const double reward = sc_staged_step_ctx<MAXD, !LED>(KernargCtx{}, g, lh, in, a.act + n * c.A, a.t, sink);
#else
  const double reward = sc_staged_step<MAXD, !LED>(c, g, lh, in, a.act + n * c.A, a.t, sink);
#endif
  a.rew[n] = reward;
  if (a.ep_ret) {
    const double r = a.ep_ret[n] + reward;
    if (terminal && a.final_ret) a.final_ret[n] = r;
    a.ep_ret[n] = autoreset ? 0.0 : r;
  }
  auto rest = [&](ObsRow& row, int t) {  // demand and time-to-go elements (:771, :786)
    for (int k = 0; k < c.R * c.P; ++k) sc_observe_demand(c, g, t, k, row);
    sc_observe_tail(c, t, row);
  };
  if (autoreset) {
    if (a.term_obs) rest(extra, a.t);
    snapshot_ledger(a, c, n);
    g.episode = a.episode + 1;
    sc_reset_env(c, g);
    ObsRow out{a.obs, n * c.O, a.obs_f64};
    sc_observe(c, g, 0, out);
  } else {
    rest(main, a.t);
    if (both) rest(extra, a.t);
  }
  if (g.overflow) atomicOr(a.err, 1);
}

// Level-parallel step (scg_supplychain_level.h): G lanes per env, 64 / G envs per block,
// env-major state so one env's heaps are a contiguous block that stays cache-resident
// while its group works on it; the level inbox and node costs live in LDS.
struct DevSched {
  int G, s;
  bool live;
  template <class F>
  __device__ __forceinline__ void phase(F&& f) {
    if (live) f(s);
    __syncthreads();
  }
};

// LDS of one env in the level kernel: node costs and the inbox, plus — when staged — the
// env's whole mutable state (heaps, sizes, stock), so every heap walk of the step runs at
// LDS latency. Doubles first, then 32-bit arrays, each 16-byte aligned.
struct LevelLds {
  size_t cost, in_val, hval, stock, in_tk, htk, hsize, total;
};

__host__ __device__ __forceinline__ size_t a16(size_t b) { return (b + 15) / 16 * 16; }

__host__ __device__ inline LevelLds level_lds(int n_nodes, int P, int H, int inbox, bool staged) {
  const size_t NP = static_cast<size_t>(n_nodes) * P;
  LevelLds l;
  l.cost = 0;
  l.in_val = l.cost + a16(static_cast<size_t>(n_nodes) * sizeof(Num));
  l.hval = l.in_val + a16(static_cast<size_t>(inbox) * 8);
  l.stock = l.hval + (staged ? a16(NP * H * 8) : 0);
  l.in_tk = l.stock + (staged ? a16(NP * 8) : 0);
  l.htk = l.in_tk + a16(static_cast<size_t>(inbox) * 4);
  l.hsize = l.htk + (staged ? a16(NP * H * 4) : 0);
  l.total = l.hsize + (staged ? a16(NP * 4) : 0);
  return l;
}

template <int MAXD, bool STAGED>
__global__ __launch_bounds__(kScBlock) void sc_level_kernel(const ScArgs a, const ScLevels lv, int G, int inbox) {
  extern __shared__ __align__(16) unsigned char smem[];
  const ScCtx& c = a.c;
  const int g = threadIdx.x / G;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * (kScBlock / G) + g;
  DevSched sch{G, static_cast<int>(threadIdx.x) % G, n < a.n};
  const LevelLds L = level_lds(c.n_nodes, c.P, c.H, inbox, STAGED);
  unsigned char* mine = smem + g * L.total;
  ScLevelEnv x;
  x.cost = reinterpret_cast<Num*>(mine + L.cost);
  x.in_val = reinterpret_cast<double*>(mine + L.in_val);
  x.in_tk = reinterpret_cast<int32_t*>(mine + L.in_tk);
  const int64_t m = sch.live ? n : 0;  // idle groups (tail block) only join the barriers
  const ScEnv ge = env_view(a, m, a.episode);  // the env's block in HBM
  const int NP = c.n_nodes * c.P, H = c.H;
  if (STAGED) {  // copy in the live part of the env's state, coalesced over the group
    x.e = ScEnv{reinterpret_cast<double*>(mine + L.stock), reinterpret_cast<int32_t*>(mine + L.htk),
                reinterpret_cast<double*>(mine + L.hval), reinterpret_cast<int32_t*>(mine + L.hsize), 1, 1,
                ge.env_id, ge.local, ge.episode, 0};
    sch.phase([&](int s) {
      for (int k = s; k < NP; k += G) {
        x.e.size[k] = ge.size[k];
        x.e.stock[k] = ge.stock[k];
      }
    });
    sch.phase([&](int s) {
      for (int q = s; q < NP * H; q += G)
        if (q % H < x.e.size[q / H]) {
          x.e.tk[q] = ge.tk[q];
          x.e.val[q] = ge.val[q];
        }
    });
  } else {
    x.e = ge;
  }
  x.act = a.act + m * c.A;
  const double reward = sc_level_step<MAXD>(c, lv, x, a.t, sch);
  const bool terminal = a.flags & 1;
  if (sch.live && sch.s == 0) {
    a.rew[n] = reward;
    if (a.ep_ret) {
      const double r = a.ep_ret[n] + reward;
      if (terminal && a.final_ret) a.final_ret[n] = r;
      a.ep_ret[n] = (a.flags & 2) ? 0.0 : r;
    }
  }
  ObsRow out{a.obs, m * c.O, a.obs_f64};
  ObsRow tout{a.term_obs, m * c.O, a.obs_f64};
  if (a.flags & 2) {
    if (a.term_obs) sch.phase([&](int s) { sc_level_observe_lane(c, x.e, a.t, tout, s, G); });
    x.e.episode = a.episode + 1;
    sch.phase([&](int s) { sc_level_reset_lane(c, x.e, s, G); });
    sch.phase([&](int s) { sc_level_observe_lane(c, x.e, 0, out, s, G); });
  } else {
    sch.phase([&](int s) {
      sc_level_observe_lane(c, x.e, a.t, out, s, G);
      if (terminal && a.term_obs) sc_level_observe_lane(c, x.e, a.t, tout, s, G);
    });
  }
  if (STAGED) {  // copy the live part back
    sch.phase([&](int s) {
      for (int k = s; k < NP; k += G) {
        ge.size[k] = x.e.size[k];
        ge.stock[k] = x.e.stock[k];
      }
      for (int q = s; q < NP * H; q += G)
        if (q % H < x.e.size[q / H]) {
          ge.tk[q] = x.e.tk[q];
          ge.val[q] = x.e.val[q];
        }
    });
  }
  if (sch.live && x.e.overflow) atomicOr(a.err, 1);
}

__global__ __launch_bounds__(kScBlock) void sc_tables_kernel(const ScArgs a, int32_t* __restrict__ demand,
                                                             int32_t* __restrict__ leadtimes) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kScBlock + threadIdx.x;
  if (n >= a.n) return;
  ScEnv e = env_view(a, n, a.episode);
  WordCache wc{0, U4{0, 0, 0, 0}, false};
  const ScCtx& c = a.c;
  const int64_t per_dem = static_cast<int64_t>(c.T + 1) * c.R * c.P;
  for (int row = 0; row <= c.T; ++row)
    for (int r = 0; r < c.R; ++r)
      for (int p = 0; p < c.P; ++p) demand[n * per_dem + (row * c.R + r) * c.P + p] = sc_demand(c, e, wc, row, r, p);
  if (leadtimes && c.stochastic) {
    WordCache lc{0, U4{0, 0, 0, 0}, false};
    const int64_t per_lt = static_cast<int64_t>(c.T) * c.n_lt;
    for (int t = 1; t <= c.T; ++t)
      for (int k = 0; k < c.n_lt; ++k) leadtimes[n * per_lt + (t - 1) * c.n_lt + k] = sc_leadtime(c, e, lc, t, k);
  }
}

namespace {

int sc_check(const scg_sc_config* cfg, const scg_sc_state* st) {
  if (!cfg || !st) return fail(SCG_ERR_INVALID, "null config/state");
  if (!cfg->nodes || cfg->heap_capacity <= 0 || cfg->n_obs <= 0)
    return fail(SCG_ERR_INVALID, "config not prepared (call scg_sc_prepare) or no device node table");
  if (cfg->stochastic_leadtimes && !cfg->leadtime_poisson && !cfg->leadtime_table)
    return fail(SCG_ERR_INVALID, "stochastic lead times need the Poisson threshold table");
  if (st->n_envs <= 0) return fail(SCG_ERR_INVALID, "n_envs must be > 0");
  if (st->env_offset < 0 || st->env_offset + st->n_envs > (int64_t(1) << 32))
    return fail(SCG_ERR_INVALID, "global env ids must fit in 32 bits");
  if (!st->stock || !st->heap_tk || !st->heap_val || !st->heap_size || !st->error_flags)
    return fail(SCG_ERR_INVALID, "state buffers stock/heap_tk/heap_val/heap_size/error_flags are required");
  if (!st->ledger != !st->ledger_kind || !st->final_ledger != !st->final_ledger_kind)
    return fail(SCG_ERR_INVALID, "ledger values and kinds come in pairs");
  if (st->ledger && cfg->kernel == SCG_SC_KERNEL_LEVEL)
    return fail(SCG_ERR_INVALID, "build_info ledgers need the lane kernel");
  return SCG_OK;
}

ScArgs sc_args(const scg_sc_config* cfg, const scg_sc_state* st) {
  ScArgs a;
  std::memset(&a, 0, sizeof(a));
  ScCtx& c = a.c;
  c.nodes = const_tab(cfg->nodes);
  c.lt_thr = const_tab(cfg->leadtime_poisson);
  c.dem_tab = cfg->demand_table;
  c.lt_tab = cfg->leadtime_table;
  c.n_nodes = cfg->n_nodes;
  c.P = cfg->n_products;
  c.R = cfg->n_retailers;
  c.A = cfg->n_actions;
  c.O = cfg->n_obs;
  c.H = cfg->heap_capacity;
  c.T = cfg->total_time_steps;
  c.avg_lt = cfg->avg_leadtime;
  c.max_lt = cfg->max_leadtime;
  c.stochastic = cfg->stochastic_leadtimes;
  c.n_lt = cfg->n_leadtimes;
  c.lt_thr_len = cfg->leadtime_poisson_len;
  sc_ctx_demand(c, cfg);
  c.pen_unmet = cfg->unmet_demand_cost;
  c.pen_stock = cfg->exceeded_stock_capacity_cost;
  c.pen_proc = cfg->exceeded_process_capacity_cost;
  c.pen_ship = cfg->exceeded_ship_capacity_cost;
  c.key0 = static_cast<uint32_t>(st->seed & 0xffffffffu);
  c.key1 = static_cast<uint32_t>(st->seed >> 32);
  a.stock = st->stock;
  a.tk = st->heap_tk;
  a.val = st->heap_val;
  a.size = st->heap_size;
  a.ep_ret = st->episode_return;
  a.final_ret = st->final_return;
  a.err = st->error_flags;
  a.inbox_tk = st->inbox_tk;
  a.inbox_val = st->inbox_val;
  a.led_v = st->ledger;
  a.led_k = st->ledger_kind;
  a.led_fv = st->final_ledger;
  a.led_fk = st->final_ledger_kind;
  a.ledp_v = st->ledger_part;
  a.n = st->n_envs;
  a.env_offset = st->env_offset;
  a.episode = st->episode;
  a.obs_f64 = cfg->obs_f64;
  a.layout = cfg->layout;
  return a;
}

dim3 sc_grid(int64_t n) { return dim3(static_cast<unsigned>((n + kScBlock - 1) / kScBlock)); }

// LDS the staged step kernel needs per 64-env block; staged only while >= 2 blocks fit a CU.
constexpr size_t kScLdsMax = 64 * 1024;

// LDS of the level kernel per block: (64 / G) envs x level_lds.
size_t sc_level_lds_bytes(const scg_sc_config* cfg) {
  return static_cast<size_t>(kScBlock / cfg->group) *
         level_lds(cfg->n_nodes, cfg->n_products, cfg->heap_capacity, cfg->inbox_size, cfg->level_staged).total;
}

// The level schedule of a chain (scg_supplychain_level.h), or false when it has none:
// every shipment must go from a node to a later node exactly one level down, levels must be
// runs of consecutive nodes, and no node may list a destination twice.
bool sc_level_schedule(scg_sc_config* cfg, const scg_sc_node* nodes) {
  const int NN = cfg->n_nodes;
  std::vector<int> lvl(NN, 0);
  for (int i = 0; i < NN; ++i)
    for (int d = 0; d < nodes[i].n_dests; ++d) {
      const int j = nodes[i].dests[d];
      if (j <= i) return false;
      for (int d2 = 0; d2 < d; ++d2)
        if (nodes[i].dests[d2] == j) return false;
      lvl[j] = std::max(lvl[j], lvl[i] + 1);
    }
  for (int i = 0; i < NN; ++i) {
    if (i > 0 && lvl[i] != lvl[i - 1] && lvl[i] != lvl[i - 1] + 1) return false;
    for (int d = 0; d < nodes[i].n_dests; ++d)
      if (lvl[nodes[i].dests[d]] != lvl[i] + 1) return false;
  }
  if (lvl[0] != 0 || lvl[NN - 1] + 1 > SCG_SC_MAX_LEVELS) return false;
  const int L = lvl[NN - 1] + 1;
  int wmax = 1, inbox = 1;
  for (int l = 0, i = 0; l < L; ++l) {
    cfg->level_start[l] = i;
    while (i < NN && lvl[i] == l) ++i;
  }
  cfg->level_start[L] = NN;
  for (int l = 0; l < L; ++l) {
    const int w = cfg->level_start[l + 1] - cfg->level_start[l];
    wmax = std::max(wmax, w);
    if (l + 1 < L) inbox = std::max(inbox, cfg->n_products * w * (cfg->level_start[l + 2] - cfg->level_start[l + 1]));
  }
  int G = 1;
  while (G < wmax && G < kScBlock) G *= 2;
  cfg->n_levels = L;
  cfg->group = G;
  cfg->inbox_size = inbox;
  // Stage each env's state in LDS when a block's share fits; widen the group (fewer envs
  // per block) until it does.
  cfg->level_staged = 1;
  while (sc_level_lds_bytes(cfg) > kScLdsMax && cfg->group < kScBlock) cfg->group *= 2;
  if (sc_level_lds_bytes(cfg) > kScLdsMax) {
    cfg->level_staged = 0;
    cfg->group = G;
  }
  return sc_level_lds_bytes(cfg) <= kScLdsMax;
}
// Heaps and sizes only: staging stock and action rows as well (+12 B per heap, +4 B per
// action) costs sc-2perstage-v0 a block per CU (3 instead of 4 at 65,536 envs), which
// measured 127 us against 70 us per step on MI355X (profiles/r01f_sc_variants.log).
size_t sc_lds_bytes(const scg_sc_config* cfg, int epb = kScBlock) {
  const size_t NP = static_cast<size_t>(cfg->n_nodes) * cfg->n_products;
  return epb * NP * (static_cast<size_t>(cfg->heap_capacity) * 12 + 4) +
         (SCG_SC_LDS_PROBE ? epb * (NP * 8 + static_cast<size_t>(cfg->n_actions) * 4) : 0);
}

// Envs per block of the LDS lane kernel for a batch of n: half-full waves when full ones
// would leave a SIMD with fewer than two (the CU count is read once per device).
#ifndef SCG_SC_LDS_EPB
#define SCG_SC_LDS_EPB 0  // 0 = by batch size; 32 or 64 forces one
#endif
int sc_lds_epb(int64_t n) {
  if (SCG_SC_LDS_EPB) return SCG_SC_LDS_EPB;
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return n < static_cast<int64_t>(cus[dev]) * 4 * 2 * 64 ? 32 : 64;
}
// Staged kernel: one heap per lane, or the split's scratch (sc_split_scratch) when wider.
size_t sc_staged_lds_bytes(const scg_sc_config* cfg) {
  return kScBlock * static_cast<size_t>(std::max(cfg->heap_capacity, sc_maxd_bucket(cfg->max_dests))) * 9;
}

// The staged kernel's inbox (scg_supplychain_staged.h): every shipment must go to a later
// node, at most once per destination list. Fills in_deg/in_base/in_slot/in_stride and
// returns the entries per env, or -1 when the chain does not qualify.
int sc_inbox_layout(const scg_sc_config* cfg, scg_sc_node* nodes) {
  const int NN = cfg->n_nodes, P = cfg->n_products;
  std::vector<int> deg(NN, 0);
  for (int i = 0; i < NN; ++i)
    for (int d = 0; d < nodes[i].n_dests; ++d) {
      const int j = nodes[i].dests[d];
      if (j <= i) return -1;
      for (int d2 = 0; d2 < d; ++d2)
        if (nodes[i].dests[d2] == j) return -1;
      ++deg[j];
    }
  int base = 0;
  for (int j = 0; j < NN; ++j) {
    nodes[j].in_deg = deg[j];
    nodes[j].in_base = base;
    base += deg[j] * P;
  }
  std::vector<int> next(NN, 0);  // sources enumerated in node order
  for (int i = 0; i < NN; ++i)
    for (int d = 0; d < nodes[i].n_dests; ++d) {
      const int j = nodes[i].dests[d];
      nodes[i].in_slot[d] = nodes[j].in_base + next[j]++;
      nodes[i].in_stride[d] = nodes[j].in_deg;
    }
  return base;
}

}  // namespace
}  // namespace scg

using namespace scg;

extern "C" {

int scg_sc_struct_sizes(size_t* node_size, size_t* config_size, size_t* state_size) {
  if (node_size) *node_size = sizeof(scg_sc_node);
  if (config_size) *config_size = sizeof(scg_sc_config);
  if (state_size) *state_size = sizeof(scg_sc_state);
  return SCG_OK;
}

int scg_sc_prepare(scg_sc_config* cfg, scg_sc_node* nodes) {
  if (!cfg || !nodes) return fail(SCG_ERR_INVALID, "null config/node table");
  const int NN = cfg->n_nodes, P = cfg->n_products;
  if (NN < 1 || NN > SCG_SC_MAX_NODES) return fail(SCG_ERR_INVALID, "n_nodes=%d outside 1..%d", NN, SCG_SC_MAX_NODES);
  if (P < 1 || P > SCG_SC_MAX_PRODUCTS)
    return fail(SCG_ERR_INVALID, "num_products=%d outside 1..%d", P, SCG_SC_MAX_PRODUCTS);
  if (cfg->total_time_steps < 1 || cfg->total_time_steps > (1 << 20))
    return fail(SCG_ERR_INVALID, "total_time_steps=%d out of range", cfg->total_time_steps);
  if (cfg->avg_leadtime < 1 || cfg->max_leadtime < 1)
    return fail(SCG_ERR_INVALID, "lead times must be >= 1 (avg %d, max %d)", cfg->avg_leadtime, cfg->max_leadtime);
  if (!cfg->demand_models && cfg->demand_hi <= cfg->demand_lo)
    return fail(SCG_ERR_INVALID, "demand_range (%d, %d) must have lo < hi", cfg->demand_lo, cfg->demand_hi);
  for (int p = 0; cfg->demand_models && p < P; ++p) {
    const int k = cfg->demand_kind[p];
    if (k < SCG_SC_DEMAND_UNIFORM || k > SCG_SC_DEMAND_SINE_UNIFORM)
      return fail(SCG_ERR_INVALID, "product %d: demand kind %d is not a SCG_SC_DEMAND_* value", p, k);
    if (cfg->demand_hi_p[p] <= cfg->demand_lo_p[p])
      return fail(SCG_ERR_INVALID, "product %d: demand range (%d, %d) must have lo < hi", p, cfg->demand_lo_p[p],
                  cfg->demand_hi_p[p]);
    if ((k == SCG_SC_DEMAND_NORMAL || k == SCG_SC_DEMAND_SINE_NORMAL) && !cfg->demand_thr && !cfg->demand_table)
      return fail(SCG_ERR_INVALID, "product %d: normal demand needs the threshold table", p);
    if (k == SCG_SC_DEMAND_SINE_UNIFORM && ((!cfg->demand_base && !cfg->demand_table) || cfg->demand_pert_n[p] < 1))
      return fail(SCG_ERR_INVALID, "product %d: sinusoidal demand needs the base table and a perturbation range", p);
  }
  int n_act = 0, n_lt = 0, n_ret = 0;
  for (int i = 0; i < NN; ++i) {
    const scg_sc_node& nd = nodes[i];
    if (nd.action_offset != n_act) return fail(SCG_ERR_INVALID, "node %d: action_offset %d != %d", i, nd.action_offset, n_act);
    if (cfg->stochastic_leadtimes && nd.leadtime_offset != n_lt)
      return fail(SCG_ERR_INVALID, "node %d: leadtime_offset %d != %d", i, nd.leadtime_offset, n_lt);
    if (nd.n_dests < 0 || nd.n_dests > SCG_SC_MAX_DESTS)
      return fail(SCG_ERR_INVALID, "node %d: %d destinations (max %d)", i, nd.n_dests, SCG_SC_MAX_DESTS);
    if (!nd.last_level && nd.n_dests == 0) return fail(SCG_ERR_INVALID, "node %d ships but has no destinations", i);
    for (int d = 0; d < nd.n_dests; ++d)
      if (nd.dests[d] < 0 || nd.dests[d] >= NN) return fail(SCG_ERR_INVALID, "node %d: bad destination", i);
    for (int p = 0; p < P; ++p) {
      if (nd.n_init[p] < 0 || nd.n_init[p] > SCG_SC_MAX_INIT)
        return fail(SCG_ERR_INVALID, "node %d: %d initial pipeline entries (max %d)", i, nd.n_init[p], SCG_SC_MAX_INIT);
      // the reference pushes its initial pipeline at times 1..k (SC_Node.reset :402-412);
      // the ABI takes any time in [1, SCG_SC_MAX_INIT + lead time], which the heap-capacity
      // simulation below indexes
      for (int j = 0; j < nd.n_init[p]; ++j)
        if (nd.init_time[p][j] < 1 || nd.init_time[p][j] > SCG_SC_MAX_INIT + std::max(cfg->avg_leadtime, cfg->max_leadtime))
          return fail(SCG_ERR_INVALID, "node %d: initial pipeline time %d outside 1..%d", i, nd.init_time[p][j],
                      SCG_SC_MAX_INIT + std::max(cfg->avg_leadtime, cfg->max_leadtime));
      if (nd.stock_capacity[p] <= 0) return fail(SCG_ERR_INVALID, "node %d: stock_capacity must be > 0", i);
      if (nd.processing_capacity > 0 && nd.processing_ratio[p] == 0)
        return fail(SCG_ERR_INVALID, "node %d: processing node with zero processing ratio", i);
    }
    if (nd.last_level) {
      if (nd.retailer_index != n_ret) return fail(SCG_ERR_INVALID, "node %d: retailer_index", i);
      ++n_ret;
    }
    n_act += nd.n_supply + nd.n_ship;
    n_lt += (nd.n_supply > 0 ? P : 0) + nd.n_dests;
  }
  if (n_ret != cfg->n_retailers || n_ret < 1) return fail(SCG_ERR_INVALID, "retailer count mismatch");
  // Heap capacity: the peak occupancy of every (node, product) heap when every possible
  // push happens with the longest lead time, simulated in the step's node order (pops
  // of a node happen after its upstream nodes pushed). Shorter lead times and skipped
  // (non-positive) shipments only lower occupancy, so this bounds every run; the
  // kernels still flag an overflow (error_flags bit 0) instead of writing past it.
  const int lmax = cfg->stochastic_leadtimes ? cfg->max_leadtime : cfg->avg_leadtime;
  const int horizon = std::min(cfg->total_time_steps, 4 * (lmax + 2) + SCG_SC_MAX_INIT);
  const int span = horizon + lmax + SCG_SC_MAX_INIT + 2;
  std::vector<int> due(static_cast<size_t>(NN) * P * span, 0), occ(static_cast<size_t>(NN) * P, 0);
  int H = 1, maxd = 0;
  for (int i = 0; i < NN; ++i) maxd = std::max(maxd, nodes[i].n_dests);
  for (int i = 0; i < NN; ++i)
    for (int p = 0; p < P; ++p)
      for (int j = 0; j < nodes[i].n_init[p]; ++j) {
        due[(static_cast<size_t>(i) * P + p) * span + nodes[i].init_time[p][j]] += 1;
        H = std::max(H, ++occ[i * P + p]);
      }
  auto push = [&](int node, int p, int when) {
    due[(static_cast<size_t>(node) * P + p) * span + when] += 1;
    H = std::max(H, ++occ[node * P + p]);
  };
  for (int t = 1; t <= horizon; ++t)
    for (int i = 0; i < NN; ++i) {
      const scg_sc_node& nd = nodes[i];
      for (int p = 0; p < P; ++p) occ[i * P + p] -= due[(static_cast<size_t>(i) * P + p) * span + t];
      for (int p = 0; p < P; ++p)
        if (nd.n_supply > 0 && nd.supply_capacity[p] > 0) push(i, p, t + lmax);
      if (!nd.last_level)
        for (int p = 0; p < P; ++p)
          if (nd.stock_capacity[p] > 0)
            for (int d = 0; d < nd.n_dests; ++d) push(nd.dests[d], p, t + lmax);
    }
  cfg->n_actions = n_act;
  cfg->n_leadtimes = n_lt;
  cfg->n_obs = n_ret * P + NN * P + NN * P * cfg->avg_leadtime + 1;
  cfg->heap_capacity = H;
  cfg->max_dests = maxd;
  // kernel: as asked, the level-parallel one only when asked for (it is the slowest on the
  // reference's chains as measured on MI355X)
  int want = cfg->kernel;
  if (want != SCG_SC_KERNEL_AUTO && want != SCG_SC_KERNEL_LANE && want != SCG_SC_KERNEL_LEVEL &&
      want != SCG_SC_KERNEL_STAGED && want != SCG_SC_KERNEL_NODES)
    return fail(SCG_ERR_INVALID, "kernel=%d is not a SCG_SC_KERNEL_* value", want);
  cfg->n_levels = 0;
  cfg->group = 1;
  cfg->inbox_size = 0;
  cfg->level_staged = 0;
  // auto: the node-parallel kernel when every node gets a wave of its own and two blocks
  // fit a CU's LDS (sc-2perstage-v0: 48 us against the LDS lane kernel's 68 us per step on
  // MI355X), or one block does and nothing but the staged kernel would take
  // the chain; else the lane kernel with every heap in LDS when a block's heaps
  // fit; else the node-staged kernel when the chain qualifies (measured faster than the lane
  // kernel on HBM heaps); else the lane kernel on HBM heaps
  // One block per CU (a block's LDS past half the CU's) still beats the node-staged kernel:
  // sc-2perstage-multiproduct-v0 at 65,536 envs 92.5 against 126 us (profiles/r03x_*), so
  // the node-parallel kernel is also taken then, unless the lane kernel's heaps fit LDS
  // (a case not measured at one block per CU).
  if (want == SCG_SC_KERNEL_AUTO && NN <= sc_nodes_waves(NN) && maxd <= sc_nodes_max_dests() && H <= 64) {
    std::vector<scg_sc_node> probe(nodes, nodes + NN);
    const int entries = sc_inbox_layout(cfg, probe.data());
    const size_t lds = entries < 0 ? 0
                                   : sc_nodes_lds_bytes(NN, P, H, entries, sc_nodes_waves(NN), n_act, cfg->n_obs,
                                                        cfg->obs_f64 ? 8 : 4);
    if (entries >= 0 && (2 * lds <= sc_nodes_lds_max() || (lds <= sc_nodes_lds_max() && sc_lds_bytes(cfg) > kScLdsMax)))
      want = SCG_SC_KERNEL_NODES;
  }
  // the staged kernel's byte-packed entries hold times up to kStagedMaxRel after the step's
  // (scg_supplychain_staged.h): lead times, and the initial pipeline's times (1..k from the
  // reference's reset, any validated time from a C-ABI caller)
  int rel_max = std::max(cfg->avg_leadtime, cfg->max_leadtime);
  for (int i = 0; i < NN; ++i)
    for (int p = 0; p < P; ++p)
      for (int j = 0; j < nodes[i].n_init[p]; ++j) rel_max = std::max(rel_max, nodes[i].init_time[p][j]);
  // ... and its ship capacities as overflow bits (ShipLeftBits): (P - 1) * MAXD <= 64
  const bool staged_ok = rel_max <= kStagedMaxRel && (!SCG_STAGED_SHIP_BITS || (P - 1) * sc_maxd_bucket(maxd) <= 64);
  if (want == SCG_SC_KERNEL_AUTO && staged_ok && sc_lds_bytes(cfg) > kScLdsMax && sc_staged_lds_bytes(cfg) <= kScLdsMax) {
    std::vector<scg_sc_node> probe(nodes, nodes + NN);
    if (sc_inbox_layout(cfg, probe.data()) >= 0) want = SCG_SC_KERNEL_STAGED;
  }
  if (want == SCG_SC_KERNEL_NODES) {
    const int entries = sc_inbox_layout(cfg, nodes);
    if (entries < 0)
      return fail(SCG_ERR_INVALID, "the node-parallel kernel needs every shipment to go to a later node, once per list");
    const int W = sc_nodes_waves(NN);
    if (maxd > sc_nodes_max_dests())
      return fail(SCG_ERR_INVALID, "the node-parallel kernel takes nodes with at most %d destinations", sc_nodes_max_dests());
    if (H > 64 || sc_nodes_lds_bytes(NN, P, H, entries, W, n_act, cfg->n_obs, cfg->obs_f64 ? 8 : 4) > sc_nodes_lds_max())
      return fail(SCG_ERR_INVALID, "a block's heaps and inbox (%d nodes x %d products x %d slots, %d entries) exceed "
                  "the node-parallel kernel's LDS", NN, P, H, entries);
    cfg->inbox_size = entries;
    cfg->group = W;
    cfg->kernel = SCG_SC_KERNEL_NODES;
    cfg->layout = SCG_SC_LAYOUT_ENV_FASTEST;
    return SCG_OK;
  }
  if (want == SCG_SC_KERNEL_STAGED) {
    const int entries = sc_inbox_layout(cfg, nodes);
    if (entries < 0)
      return fail(SCG_ERR_INVALID, "the staged kernel needs every shipment to go to a later node, once per list");
    if (sc_staged_lds_bytes(cfg) > kScLdsMax)
      return fail(SCG_ERR_INVALID, "one node's heaps (%d products x %d slots) exceed the staged kernel's LDS", P, H);
    if (rel_max > kStagedMaxRel)
      return fail(SCG_ERR_INVALID, "the staged kernel holds lead times up to %d (this chain: %d)", kStagedMaxRel, rel_max);
    if (!staged_ok)
      return fail(SCG_ERR_INVALID, "the staged kernel takes (products - 1) x destinations <= 64 (this chain: %d x %d)",
                  P - 1, sc_maxd_bucket(maxd));
    cfg->inbox_size = entries;
    cfg->kernel = SCG_SC_KERNEL_STAGED;
    cfg->layout = SCG_SC_LAYOUT_ENV_FASTEST;
    return SCG_OK;
  }
  const bool levels = want == SCG_SC_KERNEL_LEVEL && sc_level_schedule(cfg, nodes);
  if (want == SCG_SC_KERNEL_LEVEL && !levels)
    return fail(SCG_ERR_INVALID, "the chain has no level schedule (shipments must go to the next run of nodes)");
  cfg->kernel = levels ? SCG_SC_KERNEL_LEVEL : SCG_SC_KERNEL_LANE;
  cfg->layout = levels ? SCG_SC_LAYOUT_ENV_MAJOR : SCG_SC_LAYOUT_ENV_FASTEST;
  return SCG_OK;
}

int scg_sc_reset(const scg_sc_config* cfg, scg_sc_state* st, void* obs, void* stream) {
  if (int rc = sc_check(cfg, st)) return rc;
  if (st->time_step >= 0) st->episode += 1;
  ScArgs a = sc_args(cfg, st);
  a.obs = obs;
  hipLaunchKernelGGL(sc_reset_kernel, sc_grid(st->n_envs), dim3(kScBlock), 0, static_cast<hipStream_t>(stream), a);
  if (int rc = check_launch("sc_reset_kernel")) return rc;
  st->time_step = 0;
  return SCG_OK;
}

int scg_sc_step(const scg_sc_config* cfg, scg_sc_state* st, const float* action, void* obs, double* reward,
                void* terminal_obs, uint32_t flags, int32_t* done, void* stream) {
  if (int rc = sc_check(cfg, st)) return rc;
  if (!action || !obs || !reward) return fail(SCG_ERR_INVALID, "action/obs/reward buffers are required");
  if (st->time_step < 0) return fail(SCG_ERR_NOT_RESET, "step() before reset()");
  const int T = cfg->total_time_steps;
  if (st->time_step >= T) return fail(SCG_ERR_PAST_HORIZON, "step() after the terminal step %d", T);
  const int t = st->time_step + 1;
  const bool terminal = t == T;
  const bool autoreset = terminal && (flags & SCG_BG_AUTORESET);
  ScArgs a = sc_args(cfg, st);
  a.act = action;
  a.obs = obs;
  a.term_obs = terminal_obs;
  a.rew = reward;
  a.t = t;
  a.flags = (terminal ? 1 : 0) | (autoreset ? 2 : 0) | ((flags & SCG_SC_SERIAL) ? 4 : 0);
  const dim3 grid = sc_grid(st->n_envs);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t lds = sc_lds_bytes(cfg);
  if (cfg->kernel == SCG_SC_KERNEL_LEVEL) {
    if (cfg->layout != SCG_SC_LAYOUT_ENV_MAJOR || cfg->n_levels < 1 || cfg->group < 1 || cfg->group > kScBlock)
      return fail(SCG_ERR_INVALID, "level kernel needs the schedule scg_sc_prepare derives");
    ScLevels lv;
    lv.n = cfg->n_levels;
    for (int l = 0; l <= SCG_SC_MAX_LEVELS; ++l) lv.start[l] = cfg->level_start[l];
    const int per_block = kScBlock / cfg->group;
    const dim3 lgrid(static_cast<unsigned>((st->n_envs + per_block - 1) / per_block));
    const size_t llds = sc_level_lds_bytes(cfg);
    const int G = cfg->group, IB = cfg->inbox_size;
#define SCG_LEVEL_LAUNCH(D)                                                                               \
  if (cfg->level_staged)                                                                                  \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_level_kernel<D, true>), lgrid, dim3(kScBlock), llds, s, a, lv, G, IB); \
  else                                                                                                    \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_level_kernel<D, false>), lgrid, dim3(kScBlock), llds, s, a, lv, G, IB)
    switch (sc_maxd_bucket(cfg->max_dests)) {
      case 2: SCG_LEVEL_LAUNCH(2); break;
      case 4: SCG_LEVEL_LAUNCH(4); break;
      case 8: SCG_LEVEL_LAUNCH(8); break;
      case 16: SCG_LEVEL_LAUNCH(16); break;
      default: SCG_LEVEL_LAUNCH(32); break;
    }
#undef SCG_LEVEL_LAUNCH
  } else if (cfg->kernel == SCG_SC_KERNEL_NODES && (!st->ledger || st->ledger_part)) {
    if (cfg->layout != SCG_SC_LAYOUT_ENV_FASTEST || cfg->inbox_size < 0)
      return fail(SCG_ERR_INVALID, "node-parallel kernel needs the layout and inbox scg_sc_prepare derives");
    if (int rc = sc_launch_nodes(a, sc_maxd_bucket(cfg->max_dests), cfg->group, cfg->inbox_size, s)) return rc;
  } else if (cfg->kernel == SCG_SC_KERNEL_STAGED) {
    if (!st->inbox_tk || !st->inbox_val || cfg->inbox_size < 0)
      return fail(SCG_ERR_INVALID, "the staged kernel needs the inbox buffers [inbox_size][N]");
    const size_t slds = sc_staged_lds_bytes(cfg);
    switch (sc_maxd_bucket(cfg->max_dests)) {
#define SCG_STAGED_LAUNCH(D)                                                                                   \
  if (a.led_v)                                                                                                 \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_step_staged_kernel<D, true>), grid, dim3(kScBlock), slds, s, a);    \
  else                                                                                                         \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_step_staged_kernel<D, false>), grid, dim3(kScBlock), slds, s, a)
      case 2: SCG_STAGED_LAUNCH(2); break;
      case 4: SCG_STAGED_LAUNCH(4); break;
      case 8: SCG_STAGED_LAUNCH(8); break;
      case 16: SCG_STAGED_LAUNCH(16); break;
      default: SCG_STAGED_LAUNCH(32); break;
#undef SCG_STAGED_LAUNCH
    }
  } else if (cfg->layout != SCG_SC_LAYOUT_ENV_FASTEST) {
    return fail(SCG_ERR_INVALID, "lane kernel needs the env-fastest layout");
  } else if (lds <= kScLdsMax) {
    const int epb = sc_lds_epb(st->n_envs);
    const dim3 g2(static_cast<unsigned>((st->n_envs + epb - 1) / epb));
    const size_t l2 = sc_lds_bytes(cfg, epb);
#define SCG_LDS_LAUNCH(D)                                                                     \
  if (epb == 32)                                                                              \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_step_lds_kernel<D, 32>), g2, dim3(32), l2, s, a);   \
  else                                                                                        \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(sc_step_lds_kernel<D, 64>), g2, dim3(64), l2, s, a)
    switch (sc_maxd_bucket(cfg->max_dests)) {
      case 2: SCG_LDS_LAUNCH(2); break;
      case 4: SCG_LDS_LAUNCH(4); break;
      case 8: SCG_LDS_LAUNCH(8); break;
      case 16: SCG_LDS_LAUNCH(16); break;
      default: SCG_LDS_LAUNCH(32); break;
    }
#undef SCG_LDS_LAUNCH
  } else switch (sc_maxd_bucket(cfg->max_dests)) {
    case 2: hipLaunchKernelGGL(sc_step_kernel<2>, grid, dim3(kScBlock), 0, s, a); break;
    case 4: hipLaunchKernelGGL(sc_step_kernel<4>, grid, dim3(kScBlock), 0, s, a); break;
    case 8: hipLaunchKernelGGL(sc_step_kernel<8>, grid, dim3(kScBlock), 0, s, a); break;
    case 16: hipLaunchKernelGGL(sc_step_kernel<16>, grid, dim3(kScBlock), 0, s, a); break;
    default: hipLaunchKernelGGL(sc_step_kernel<32>, grid, dim3(kScBlock), 0, s, a); break;
  }
  if (int rc = check_launch("sc_step_kernel")) return rc;
  if (autoreset) {
    st->time_step = 0;
    st->episode += 1;
  } else {
    st->time_step = t;
  }
  if (done) *done = terminal ? 1 : 0;
  return SCG_OK;
}

#ifdef SCG_SC_STAMPS
// Diagnostic build only: copy the phase stamps of the first `waves` waves to host memory.
__attribute__((visibility("default"))) int scg_sc_debug_stamps(unsigned long long* host, int waves) {
  if (waves > kStampWaves) waves = kStampWaves;
  if (hipDeviceSynchronize() != hipSuccess) return fail(SCG_ERR_HIP, "sync");
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sc_stamps), sizeof(unsigned long long) * kStampSlots * waves) != hipSuccess)
    return fail(SCG_ERR_HIP, "stamp copy");
  return SCG_OK;
}
#endif

// ---- step server (include/scgpu.h scg_sc_server_*) --------------------------------------
static_assert(sizeof(scg_sc_server_box) == 192 && offsetof(scg_sc_server_box, action) == 64 &&
                  offsetof(scg_sc_server_box, done_seq) == 128,
              "SupplyChain mailbox");
static_assert(sizeof(scg_sc_server) == 104, "SupplyChain server struct");
static int sc_server_stop_now(scg_sc_server* sv) {
  if (!sv->running) return SCG_OK;
  __atomic_store_n(&sv->box_host->exit_req, sv->box_host->exit_req + 1, __ATOMIC_RELEASE);
  sv->running = 0;
  if (hipStreamSynchronize(static_cast<hipStream_t>(sv->stream)) != hipSuccess)
    return fail(SCG_ERR_HIP, "SupplyChain step server: hipStreamSynchronize failed");
  return SCG_OK;
}

int scg_sc_server_stop(scg_sc_server* sv) {
  if (!sv || !sv->box_host || !sv->box_dev) return fail(SCG_ERR_INVALID, "null server/mailbox");
  return sc_server_stop_now(sv);
}

static int sc_server_launch(const scg_sc_config* cfg, const scg_sc_state* st, scg_sc_server* sv) {
  ScArgs a = sc_args(cfg, st);
  a.act = sv->action;
  a.obs = sv->obs;
  a.rew = sv->reward;
  a.term_obs = nullptr;
  const uint32_t exit_seen = __atomic_load_n(&sv->box_host->exit_req, __ATOMIC_ACQUIRE);
  if (int rc = sc_launch_nodes_server(a, sc_maxd_bucket(cfg->max_dests), cfg->group, cfg->inbox_size,
                                      static_cast<hipStream_t>(sv->stream), sv->box_dev, exit_seen,
                                      static_cast<uint32_t>(sv->idle_us) * 100u))
    return rc;
  sv->running = 1;
  sv->launches += 1;
  sv->last_ns = mono_ns();
  return SCG_OK;
}

int scg_sc_server_post(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv) {
  if (int rc = sc_check(cfg, st)) return rc;
  if (!sv || !sv->box_host || !sv->box_dev || !sv->action || !sv->obs || !sv->reward)
    return fail(SCG_ERR_INVALID, "SupplyChain step server: mailbox, action, obs and reward are required");
  if (!sv->stream) return fail(SCG_ERR_INVALID, "SupplyChain step server: needs a (non-blocking) stream of its own");
  if (sv->idle_us < 100 || sv->idle_us > 10000000) return fail(SCG_ERR_INVALID, "idle_us outside 100..10^7");
  if (st->n_envs > kScBlock) return fail(SCG_ERR_INVALID, "the SupplyChain step server runs up to %d envs", kScBlock);
  if (cfg->kernel != SCG_SC_KERNEL_NODES || cfg->layout != SCG_SC_LAYOUT_ENV_FASTEST || cfg->inbox_size < 0)
    return fail(SCG_ERR_INVALID, "the SupplyChain step server runs the node-parallel kernel's configs");
  if (!cfg->obs_f64 || st->ledger) return fail(SCG_ERR_INVALID, "the SupplyChain step server runs float64 observations, no ledgers");
  if (st->time_step < 0) return fail(SCG_ERR_NOT_RESET, "step() before reset()");
  const int T = cfg->total_time_steps;
  if (st->time_step >= T) return fail(SCG_ERR_PAST_HORIZON, "step() after the terminal step %d", T);
  scg_sc_server_box* b = sv->box_host;
  if (__atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) != sv->seq)
    return fail(SCG_ERR_INVALID, "SupplyChain step server: a post while the last request is unanswered");
  const int t = st->time_step + 1;
  // a block idle for more than half its time-out may be exiting: retire it before posting
  if (sv->running && mono_ns() - sv->last_ns > static_cast<int64_t>(sv->idle_us) * 500)
    if (int rc = sc_server_stop_now(sv)) return rc;
  // the request line and the inline action row: one env of at most 16 actions travels in
  // the request, so the block does not read it across PCIe
  uint32_t line[32] = {0};
  const uint32_t seq = sv->seq + 1;
  const bool inline_act = sv->action_host && st->n_envs == 1 && cfg->n_actions <= 16;
  line[0] = seq;
  line[2] = static_cast<uint32_t>(t);
  line[3] = t == T ? 1u : 0u;
  line[4] = st->episode;
  line[5] = (inline_act ? 1u : 0u) | (sv->reload ? 2u : 0u);
  if (inline_act) std::memcpy(&line[16], sv->action_host, sizeof(float) * cfg->n_actions);
  line[7] = mailbox_check(line);
  sv->reload = 0;
  uint32_t* dst = reinterpret_cast<uint32_t*>(b);
  for (int i = 1; i < 32; ++i) __atomic_store_n(&dst[i], line[i], __ATOMIC_RELAXED);
  __atomic_store_n(&dst[0], seq, __ATOMIC_RELEASE);
  sv->seq = seq;
  sv->t = t;
  sv->done = t == T ? 1 : 0;
  sv->last_ns = mono_ns();
  if (!sv->running)
    if (int rc = sc_server_launch(cfg, st, sv)) return rc;
  return SCG_OK;
}

int scg_sc_server_wait(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv, int64_t spin_us, int32_t* done) {
  if (int rc = sc_check(cfg, st)) return rc;
  if (!sv || !sv->box_host) return fail(SCG_ERR_INVALID, "null server/mailbox");
  scg_sc_server_box* b = sv->box_host;
  const uint32_t seq = sv->seq;
  const int64_t start = mono_ns();
  const int64_t check_ns = (sv->check_us > 0 ? sv->check_us : 2000000) * int64_t(1000);
  int64_t check = start + check_ns;
  int gone = 0;
  for (uint32_t spins = 0;; ++spins) {
    if (__atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) == seq) break;
    cpu_relax();
    if ((spins & 255u) != 255u) continue;
    const int64_t now = mono_ns();
    if (spin_us >= 0 && now - start > spin_us * 1000) return SCG_PENDING;
    if (now < check) continue;
    check = now + check_ns;
    // the BeerGame server's checks (scg_bg_server_wait): a HIP error at once; a block gone
    // without answering launched again once (it serves the pending request first)
    const hipError_t q = hipStreamQuery(static_cast<hipStream_t>(sv->stream));
    if (q != hipSuccess && q != hipErrorNotReady)
      return fail(SCG_ERR_HIP, "SupplyChain step server: the stream reports %s (step %d)", hipGetErrorString(q), sv->t);
    if (__atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) == seq) break;
    if (q == hipSuccess) {
      if (gone++ > 0)
        return fail(SCG_ERR_HIP, "SupplyChain step server: the block exits without answering (step %d)", sv->t);
      sv->running = 0;
      sv->relaunches += 1;
      if (int rc = sc_server_launch(cfg, st, sv)) return rc;
    }
    if (now - start > 60000000000LL) return fail(SCG_ERR_HIP, "SupplyChain step server: no answer for 60 s (step %d)", sv->t);
  }
  sv->last_ns = mono_ns();
  st->time_step = sv->t;  // no auto-reset on this path
  if (done) *done = sv->done;
  return SCG_OK;
}

int scg_sc_server_step(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv, int32_t* done) {
  if (int rc = scg_sc_server_post(cfg, st, sv)) return rc;
  return scg_sc_server_wait(cfg, st, sv, -1, done);
}

int scg_sc_draw_tables(const scg_sc_config* cfg, const scg_sc_state* st, uint32_t episode, int32_t* demand,
                       int32_t* leadtimes, void* stream) {
  if (int rc = sc_check(cfg, st)) return rc;
  if (!demand) return fail(SCG_ERR_INVALID, "null demand buffer");
  ScArgs a = sc_args(cfg, st);
  a.episode = episode;
  hipLaunchKernelGGL(sc_tables_kernel, sc_grid(st->n_envs), dim3(kScBlock), 0, static_cast<hipStream_t>(stream), a,
                     demand, leadtimes);
  return check_launch("sc_tables_kernel");
}

}  // extern "C"
