// BeerGame hot path for gfx950: reset / step / rollout kernels + their C-ABI launchers.
//
// Reference: gym_supplychain/envs/beergame_env.py (BeerGameEnv), snapshot 2024-08-07.
// One lane owns one env for the whole launch; every per-env array is env-major [N][L]
// int32, so for the default L = 4 each state row is one 16-byte global_load_dwordx4 /
// global_store_dwordx4 per lane and a wavefront moves 1 KiB per instruction, fully
// coalesced. The path is HBM/launch bound integer work (≈35 int ops per env-step);
// there is no contraction, so no MFMA and no LDS tiling — see DESIGN.md.
//
// The reference keeps an absolute-week shipment table (beergame_env.py:46-52) that is
// never shifted (:73-74). Here it is a ring of R = max delay + 1 week slots; the host
// plan (scg_bg_prepare) decides per week whether the due slot holds deliveries and
// whether the scheduled slot is written fresh (store) or accumulated (read-modify-write),
// so the common constant-delay case moves exactly one due row in and one row out.

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "scg_common.h"
#include "scg_const.h"
#include "scg_philox.h"
#include "scgpu.h"

namespace scg {

// ---- per-week plan word (host computed, uniform per launch) -------------------------
enum : int32_t { MODE_DIRECT = 0, MODE_STORE = 1, MODE_ADD = 2, MODE_DROP = 3 };
constexpr int32_t PLAN_ARRIVE = 4;
inline int32_t plan_mode(int32_t p) { return p & 3; }
inline bool plan_arrive(int32_t p) { return (p & PLAN_ARRIVE) != 0; }
inline int32_t plan_delay(int32_t p) { return (p >> 8) & 0xff; }

constexpr int kBlock = 256;

// ---- kernel arguments (passed by value, ≈300 B of the 4 KiB argument segment) -------
struct BgArgs {
  int32_t* inv;
  int32_t* bk;
  int32_t* op;
  int32_t* ring;
  int32_t* inv_acc;
  int32_t* bk_acc;
  int32_t* hist;
  int64_t* ep_ret;
  int64_t* final_ret;
  const int32_t* act;
  int32_t* obs;
  int32_t* rew;
  int32_t* term_obs;
  const int32_t* demand_table;
  const uint32_t* pthr;
  int64_t n;           // envs in this shard
  int64_t env_offset;  // global id of env 0
  uint32_t key0, key1;
  uint32_t episode;
  int32_t demand_mode;
  int32_t pthr_len;
  int32_t h, b;        // inv_cost, backlog_cost
  int32_t ship_value, orders_value;
  int32_t init_slots;  // weeks 1..init_slots hold the initial pipeline (:52)
  int32_t ring_slots;
  int32_t init_inv[SCG_BG_MAX_LEVELS];
  // BeerGameEnv2 (beergame2_env.py)
  int32_t* pen_acc;    // penalty_costs ledger (:184)
  int32_t max_stock, penalty;
  int32_t demand_lo, demand_hi;
  int32_t stochastic_delays, delay_lo, delay_hi, max_weeks;
};

// ---- row helpers: L contiguous int32 per env, widest aligned vector access ----------
template <int L>
__device__ __forceinline__ void load_row(const int32_t* __restrict__ p, int32_t (&v)[L]) {
  if constexpr (L % 4 == 0) {
#pragma unroll
    for (int c = 0; c < L / 4; ++c) {
      const int4 t = reinterpret_cast<const int4*>(p)[c];
      v[4 * c] = t.x; v[4 * c + 1] = t.y; v[4 * c + 2] = t.z; v[4 * c + 3] = t.w;
    }
  } else if constexpr (L % 2 == 0) {
#pragma unroll
    for (int c = 0; c < L / 2; ++c) {
      const int2 t = reinterpret_cast<const int2*>(p)[c];
      v[2 * c] = t.x; v[2 * c + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) v[l] = p[l];
  }
}

template <int L>
__device__ __forceinline__ void store_row(int32_t* __restrict__ p, const int32_t (&v)[L]) {
  if constexpr (L % 4 == 0) {
#pragma unroll
    for (int c = 0; c < L / 4; ++c)
      reinterpret_cast<int4*>(p)[c] = make_int4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);
  } else if constexpr (L % 2 == 0) {
#pragma unroll
    for (int c = 0; c < L / 2; ++c) reinterpret_cast<int2*>(p)[c] = make_int2(v[2 * c], v[2 * c + 1]);
  } else {
#pragma unroll
    for (int l = 0; l < L; ++l) p[l] = v[l];
  }
}

template <int L>
__device__ __forceinline__ void fill_row(int32_t* __restrict__ p, int32_t x) {
  int32_t v[L];
#pragma unroll
  for (int l = 0; l < L; ++l) v[l] = x;
  store_row<L>(p, v);
}

// Inverse CDF on uint32 thresholds, #{k : thr[k] <= u}, with the table read through the
// scalar cache (constant address space), eight entries per scalar load: the table index is
// wave-uniform, and the count waits on lgkmcnt only, so it runs while a kernel's row loads
// are still in flight instead of after them (a vector load of the table waited on vmcnt,
// i.e. for every row first).
__device__ __forceinline__ int32_t poisson_count_scalar(ConstTab<uint32_t> thr, int32_t len, uint32_t u) {
  int32_t x = 0;
  int k = 0;
  for (; k + 8 <= len; k += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x += (thr[k + j] <= u) ? 1 : 0;
  }
  for (; k < len; ++k) x += (thr[k] <= u) ? 1 : 0;
  return x;
}

__device__ __forceinline__ int32_t poisson_invert(const BgArgs& a, uint32_t u) {
  return poisson_count_scalar(const_tab(a.pthr), a.pthr_len, u);
}

// Customer demand of env n for `week` (1-based): beergame_env.py:79 reads
// customer_demand[week-1]; here per env from a table (TABLE) or drawn on device
// (POISSON, UNIFORM). The shared FIXED list arrives as a per-week kernel argument instead.
// DM: the demand mode when the kernel is specialised on it, -1 to read a.demand_mode.
template <int DM = -1>
__device__ __forceinline__ int32_t week_demand(const BgArgs& a, int64_t n, int32_t week,
                                               uint32_t episode) {
  const int32_t mode = DM >= 0 ? DM : a.demand_mode;
  if (mode == SCG_DEMAND_TABLE) return a.demand_table[(int64_t)(week - 1) * a.n + n];
  if (mode == SCG_DEMAND_UNIFORM) {  // randint(lo, hi), hi exclusive (beergame2_env.py:76-77)
    const uint32_t w = scg::philox_word(a.key0, a.key1, static_cast<uint32_t>(a.env_offset + n), episode,
                                        static_cast<uint32_t>(week - 1), SCG_STREAM_BG2_DEMAND);
    return a.demand_lo + static_cast<int32_t>((static_cast<uint64_t>(w) * static_cast<uint32_t>(a.demand_hi - a.demand_lo)) >> 32);
  }
  const uint32_t u = scg::philox_word(a.key0, a.key1, static_cast<uint32_t>(a.env_offset + n),
                                      episode, static_cast<uint32_t>(week - 1), SCG_STREAM_DEMAND);
  return poisson_invert(a, u);
}

// reset() of one env (beergame_env.py:140-156), writing the device state rows.
template <int L>
__device__ __forceinline__ void reset_env(const BgArgs& a, int64_t n, int32_t* __restrict__ obs_out) {
  const int64_t row = n * L;
  const int64_t stride = a.n * L;
  int32_t inv[L];
#pragma unroll
  for (int l = 0; l < L; ++l) inv[l] = a.init_inv[l];
  store_row<L>(a.inv + row, inv);
  fill_row<L>(a.bk + row, 0);
  fill_row<L>(a.op + row, a.orders_value);
  if (a.stochastic_delays)  // per-lane delays read-modify-write every slot: start clean
    for (int s = 0; s < a.ring_slots; ++s) fill_row<L>(a.ring + s * stride + row, 0);
  for (int t = 1; t <= a.init_slots; ++t) fill_row<L>(a.ring + (t % a.ring_slots) * stride + row, a.ship_value);
  if (a.inv_acc) fill_row<L>(a.inv_acc + row, 0);
  if (a.bk_acc) fill_row<L>(a.bk_acc + row, 0);
  if (a.pen_acc) fill_row<L>(a.pen_acc + row, 0);
  if (a.hist) fill_row<L>(a.hist + row, a.orders_value);  // all_orders_placed[:, 0] (:152)
  if (a.ep_ret) a.ep_ret[n] = 0;
  if (obs_out) {  // inventory - backlog with backlog = 0 (v2: + max_stock, beergame2_env.py:112)
#pragma unroll
    for (int l = 0; l < L; ++l) inv[l] += a.max_stock;
    store_row<L>(obs_out + row, inv);
  }
}

template <int L>
__global__ __launch_bounds__(kBlock) void bg_reset_kernel(const BgArgs a) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= a.n) return;
  reset_env<L>(a, n, a.obs);
}

// One week of one env (beergame_env.py:66-138), pure register arithmetic. The caller
// moves the rows: `due` is the pipeline row arriving this week (zeros when none), `ship`
// comes back as the row scheduled `delay` weeks ahead (or is already added into the
// inventory when the week's delay is 0, `direct`). Shared by the step kernel (state
// from/to HBM every launch) and the rollout kernel (state held in registers).
struct WeekInfo {
  int32_t week;        // 1..T
  int32_t read_slot;   // -1: nothing due
  int32_t write_slot;
  int32_t mode;        // MODE_*
  int32_t demand_fixed;
  int32_t flags;       // bit0 terminal, bit1 autoreset
};

template <int L>
__device__ __forceinline__ int32_t step_core(int32_t h, int32_t b, int32_t demand, bool direct,
                                             const int32_t (&due)[L], int32_t (&inv)[L], int32_t (&bk)[L],
                                             int32_t (&op)[L], const int32_t (&act)[L], int32_t (&ship)[L],
                                             int32_t (&obs)[L], int32_t (&ic)[L], int32_t (&bc)[L]) {
  // 1. receive the shipments due this week (:72)
  // 2. order slips: customer demand at level 0, the previous orders above (:79-81)
  int32_t inc[L];
  inc[0] = demand;
#pragma unroll
  for (int l = 1; l < L; ++l) inc[l] = op[l - 1];
  // fill what inventory allows (:85-89); ship[l] = what level l receives: deliver[l+1]
  // from the level above it, and for the factory its own orders_placed[-1] from before
  // this step (:93-96, :111-114)
  int32_t fill[L], del[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    inv[l] += due[l];
    fill[l] = inc[l] + bk[l];
    del[l] = min(inv[l], fill[l]);
  }
#pragma unroll
  for (int l = 0; l + 1 < L; ++l) ship[l] = del[l + 1];
  ship[L - 1] = op[L - 1];
  // 3. inventory / backlog (:101-103); 5. place orders (:121); obs (:127,:180); cost (:130)
  int32_t cost = 0;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    inv[l] += (direct ? ship[l] : 0) - del[l];
    bk[l] = fill[l] - del[l];
    op[l] = inc[l] + act[l];
    obs[l] = inv[l] - bk[l];
    ic[l] = h * inv[l];
    bc[l] = b * bk[l];
    cost += ic[l] + bc[l];
  }
  return -cost;
}

template <int L>
__device__ __forceinline__ void zero_row(int32_t (&v)[L]) {
#pragma unroll
  for (int l = 0; l < L; ++l) v[l] = 0;
}

// Week plan packed into one dword for the step kernel's preloaded arguments:
// bits 0-7 read_slot + 1 (0: nothing due), 8-15 write_slot, 16-17 mode, 18-19 flags.
inline uint32_t pack_week(const WeekInfo& wk) {
  return static_cast<uint32_t>(wk.read_slot + 1) | (static_cast<uint32_t>(wk.write_slot) << 8) |
         (static_cast<uint32_t>(wk.mode) << 16) | (static_cast<uint32_t>(wk.flags) << 18);
}

// step(action) for one env per lane: every row this launch reads is loaded up front (one
// round of memory latency), the week is computed in registers, then every row is stored.
// The leading scalar arguments (the four state rows' and the ring's base pointers, the env
// count and the packed week plan: 12 dwords) are preloaded into SGPRs at wave launch
// (gfx950 kernarg preload, build flag -amdgpu-kernarg-preload-count), so the first row
// loads issue without waiting on the kernarg segment; the rest of the arguments arrive
// through scalar loads that overlap those rows, and the Poisson inversion reads its
// thresholds through the scalar cache, so it too runs while the rows are in flight.
template <int L, int DM>
__global__ __launch_bounds__(kBlock) void bg_step_kernel(int32_t* __restrict__ inv_p, int32_t* __restrict__ bk_p,
                                                         int32_t* __restrict__ op_p, const int32_t* __restrict__ act_p,
                                                         int32_t* __restrict__ ring_p, uint32_t n32, uint32_t wpack,
                                                         const BgArgs a, const WeekInfo wk) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const int32_t read_slot = static_cast<int32_t>(wpack & 0xffu) - 1;
  const int32_t write_slot = static_cast<int32_t>((wpack >> 8) & 0xffu);
  const int32_t mode = static_cast<int32_t>((wpack >> 16) & 3u);
  const bool terminal = wpack & (1u << 18);
  const bool autoreset = wpack & (2u << 18);
  const int64_t row = n * L;
  const int64_t stride = static_cast<int64_t>(n32) * L;
  if (n >= static_cast<int64_t>(n32)) return;

  int32_t inv[L], bk[L], op[L], act[L], due[L], cur[L], iacc[L], bacc[L];
  zero_row<L>(due);
  zero_row<L>(cur);
  load_row<L>(inv_p + row, inv);
  load_row<L>(bk_p + row, bk);
  load_row<L>(op_p + row, op);
  load_row<L>(act_p + row, act);
  if (read_slot >= 0) load_row<L>(ring_p + read_slot * stride + row, due);
  if (mode == MODE_ADD) load_row<L>(ring_p + write_slot * stride + row, cur);
  // The remaining arguments are left to the compiler's scalar loads: they issue after
  // these rows and overlap them (forcing them up front made the register allocator reuse
  // a kernarg SGPR and wait on the kernarg segment before the first row load).
  zero_row<L>(iacc);
  zero_row<L>(bacc);
  if (!autoreset && a.inv_acc) load_row<L>(a.inv_acc + row, iacc);
  if (!autoreset && a.bk_acc) load_row<L>(a.bk_acc + row, bacc);
  const int64_t ret0 = a.ep_ret ? a.ep_ret[n] : 0;
  int32_t demand;
  if constexpr (DM == SCG_DEMAND_FIXED) {
    demand = wk.demand_fixed;
  } else if constexpr (DM == SCG_DEMAND_POISSON) {
    const uint32_t u = scg::philox_word(a.key0, a.key1, static_cast<uint32_t>(a.env_offset + n), a.episode,
                                        static_cast<uint32_t>(wk.week - 1), SCG_STREAM_DEMAND);
    demand = poisson_invert(a, u);
  } else {
    demand = week_demand<DM>(a, n, wk.week, a.episode);
  }

  int32_t ship[L], obs[L], ic[L], bc[L];
  const int32_t reward = step_core<L>(a.h, a.b, demand, mode == MODE_DIRECT, due, inv, bk, op, act, ship, obs, ic, bc);

  if (mode == MODE_STORE) {
    store_row<L>(ring_p + write_slot * stride + row, ship);
  } else if (mode == MODE_ADD) {
#pragma unroll
    for (int l = 0; l < L; ++l) cur[l] += ship[l];
    store_row<L>(ring_p + write_slot * stride + row, cur);
  }  // MODE_DROP: arrives after the horizon, never observable
  a.rew[n] = reward;
  if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);  // :123
  if (terminal && a.term_obs) store_row<L>(a.term_obs + row, obs);
  const int64_t ret = ret0 + reward;
  if (terminal && a.final_ret) a.final_ret[n] = ret;
  if (autoreset) {  // the next step starts a fresh episode (reset() in the same launch)
    reset_env<L>(a, n, a.obs);
    return;
  }
  store_row<L>(inv_p + row, inv);
  store_row<L>(bk_p + row, bk);
  store_row<L>(op_p + row, op);
  store_row<L>(a.obs + row, obs);
  if (a.inv_acc) {  // :131
#pragma unroll
    for (int l = 0; l < L; ++l) iacc[l] += ic[l];
    store_row<L>(a.inv_acc + row, iacc);
  }
  if (a.bk_acc) {  // :132
#pragma unroll
    for (int l = 0; l < L; ++l) bacc[l] += bc[l];
    store_row<L>(a.bk_acc + row, bacc);
  }
  if (a.ep_ret) a.ep_ret[n] = ret;
}

// BeerGameEnv2.step (beergame2_env.py:114-192): the v1 week with absolute orders
// (:168), the observation offset by max_stock (:112), a penalty on stock and backlog
// beyond max_stock (:179-180, :184), and optionally per-episode random shipment delays
// (:90-92): then each lane draws its own delay, the due ring slot is cleared after it is
// received and the scheduled slot is always read-modify-written (no shared week plan).
template <int L>
__global__ __launch_bounds__(kBlock) void bg2_step_kernel(const BgArgs a, const WeekInfo wk) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= a.n) return;
  const int64_t row = n * L;
  const int64_t stride = a.n * L;
  const bool terminal = wk.flags & 1;
  const bool autoreset = wk.flags & 2;
  int32_t read_slot = wk.read_slot, write_slot = wk.write_slot, mode = wk.mode;
  if (a.stochastic_delays) {
    const uint32_t u = scg::philox_word(a.key0, a.key1, static_cast<uint32_t>(a.env_offset + n), a.episode,
                                        static_cast<uint32_t>(wk.week - 1), SCG_STREAM_BG2_DELAY);
    const int32_t d = a.delay_lo + static_cast<int32_t>((static_cast<uint64_t>(u) * static_cast<uint32_t>(a.delay_hi - a.delay_lo)) >> 32);
    read_slot = wk.week % a.ring_slots;
    write_slot = (wk.week + d) % a.ring_slots;
    mode = d == 0 ? MODE_DIRECT : (wk.week + d > a.max_weeks ? MODE_DROP : MODE_ADD);
  }
  int32_t inv[L], bk[L], op[L], act[L], due[L], cur[L], iacc[L], bacc[L], pacc[L];
  load_row<L>(a.inv + row, inv);
  load_row<L>(a.bk + row, bk);
  load_row<L>(a.op + row, op);
  load_row<L>(a.act + row, act);
  zero_row<L>(due);
  zero_row<L>(cur);
  zero_row<L>(iacc);
  zero_row<L>(bacc);
  zero_row<L>(pacc);
  if (read_slot >= 0) load_row<L>(a.ring + read_slot * stride + row, due);
  if (mode == MODE_ADD) load_row<L>(a.ring + write_slot * stride + row, cur);
  if (!autoreset && a.inv_acc) load_row<L>(a.inv_acc + row, iacc);
  if (!autoreset && a.bk_acc) load_row<L>(a.bk_acc + row, bacc);
  if (!autoreset && a.pen_acc) load_row<L>(a.pen_acc + row, pacc);
  const int64_t ret0 = a.ep_ret ? a.ep_ret[n] : 0;
  const int32_t demand = a.demand_mode == SCG_DEMAND_FIXED ? wk.demand_fixed : week_demand(a, n, wk.week, a.episode);

  int32_t inc[L], fill[L], del[L], ship[L], obs[L];
  inc[0] = demand;
#pragma unroll
  for (int l = 1; l < L; ++l) inc[l] = op[l - 1];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    inv[l] += due[l];
    fill[l] = inc[l] + bk[l];
    del[l] = min(inv[l], fill[l]);
  }
#pragma unroll
  for (int l = 0; l + 1 < L; ++l) ship[l] = del[l + 1];
  ship[L - 1] = op[L - 1];
  int32_t cost = 0, pen = 0;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    inv[l] += (mode == MODE_DIRECT ? ship[l] : 0) - del[l];
    bk[l] = fill[l] - del[l];
    op[l] = act[l];                                   // absolute orders (:168)
    obs[l] = a.max_stock + inv[l] - bk[l];
    const int32_t over = max(inv[l] - a.max_stock, 0) + max(bk[l] - a.max_stock, 0);
    iacc[l] += a.h * inv[l];
    bacc[l] += a.b * bk[l];
    pacc[l] += a.penalty * over;
    cost += a.h * inv[l] + a.b * bk[l];
    pen += a.penalty * over;
  }
  const int32_t reward = -cost - pen;                 // :177-180

  if (a.stochastic_delays) {  // consumed: the slot is reused R weeks on
    int32_t z[L];
    zero_row<L>(z);
    store_row<L>(a.ring + read_slot * stride + row, z);
  }
  if (mode == MODE_STORE) {
    store_row<L>(a.ring + write_slot * stride + row, ship);
  } else if (mode == MODE_ADD) {
#pragma unroll
    for (int l = 0; l < L; ++l) cur[l] += ship[l];
    store_row<L>(a.ring + write_slot * stride + row, cur);
  }
  a.rew[n] = reward;
  if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);
  if (terminal && a.term_obs) store_row<L>(a.term_obs + row, obs);
  const int64_t ret = ret0 + reward;
  if (terminal && a.final_ret) a.final_ret[n] = ret;
  if (autoreset) {
    reset_env<L>(a, n, a.obs);
    return;
  }
  store_row<L>(a.inv + row, inv);
  store_row<L>(a.bk + row, bk);
  store_row<L>(a.op + row, op);
  store_row<L>(a.obs + row, obs);
  if (a.inv_acc) store_row<L>(a.inv_acc + row, iacc);
  if (a.bk_acc) store_row<L>(a.bk_acc + row, bacc);
  if (a.pen_acc) store_row<L>(a.pen_acc + row, pacc);
  if (a.ep_ret) a.ep_ret[n] = ret;
}

struct RolloutWeeks {
  WeekInfo wk[SCG_BG_ROLLOUT_MAX];
};

// Pipeline ring views for the rollout kernel: rows in HBM ([slot][N][L], the state
// layout) or staged in LDS for the whole launch ([slot*L + l][lane], lane fastest, so
// per-lane slot choices never conflict on banks).
template <int L>
struct RingHbm {
  int32_t* base;
  int64_t stride, row;
  __device__ __forceinline__ void load(int s, int32_t (&v)[L]) const { load_row<L>(base + s * stride + row, v); }
  __device__ __forceinline__ void store(int s, const int32_t (&v)[L]) const { store_row<L>(base + s * stride + row, v); }
};

template <int L>
struct RingLds {
  int32_t* base;  // LDS + lane
  __device__ __forceinline__ void load(int s, int32_t (&v)[L]) const {
#pragma unroll
    for (int l = 0; l < L; ++l) v[l] = base[(s * L + l) * kBlock];
  }
  __device__ __forceinline__ void store(int s, const int32_t (&v)[L]) const {
#pragma unroll
    for (int l = 0; l < L; ++l) base[(s * L + l) * kBlock] = v[l];
  }
};

// K weeks per launch, inventory/backlog/orders/ledgers/return in registers; per week only
// the action row in and the obs/reward (and history) rows out touch HBM. With LDS the
// pipeline ring is staged in shared memory for the whole launch (loaded once, stored
// once); otherwise its rows are read-modify-written through L2.
// Weeks run in groups of kRolloutGroup: the group's action rows are all requested before
// its first week, so a launch waits on memory once per group instead of once per week.
constexpr int kRolloutGroup = 8;

template <int L, class Ring>
__device__ __forceinline__ void rollout_body(const BgArgs& a, int64_t n, int32_t K, const RolloutWeeks& weeks,
                                             const int32_t* __restrict__ acts, int32_t* __restrict__ obs_out,
                                             int32_t* __restrict__ rew_out, const Ring& ring) {
  const int64_t row = n * L;
  const int64_t stride = a.n * L;
  int32_t inv[L], bk[L], op[L], iacc[L], bacc[L];
  load_row<L>(a.inv + row, inv);
  load_row<L>(a.bk + row, bk);
  load_row<L>(a.op + row, op);
  zero_row<L>(iacc);
  zero_row<L>(bacc);
  if (a.inv_acc) load_row<L>(a.inv_acc + row, iacc);
  if (a.bk_acc) load_row<L>(a.bk_acc + row, bacc);
  int64_t ret = a.ep_ret ? a.ep_ret[n] : 0;
  uint32_t episode = a.episode;
  for (int32_t k0 = 0; k0 < K; k0 += kRolloutGroup) {
  int32_t group_act[kRolloutGroup][L];
#pragma unroll
  for (int u = 0; u < kRolloutGroup; ++u)
    if (k0 + u < K) load_row<L>(acts + (k0 + u) * stride + row, group_act[u]);
#pragma unroll
  for (int u = 0; u < kRolloutGroup; ++u) {
    const int32_t k = k0 + u;
    if (k >= K) break;
    const WeekInfo wk = weeks.wk[k];
    int32_t due[L], obs[L], ic[L], bc[L], ship[L];
    int32_t(&act)[L] = group_act[u];
    zero_row<L>(due);
    if (wk.read_slot >= 0) ring.load(wk.read_slot, due);
    int32_t demand;
    if (a.demand_mode == SCG_DEMAND_FIXED)
      demand = wk.demand_fixed;
    else
      demand = week_demand(a, n, wk.week, episode);
    const int32_t reward = step_core<L>(a.h, a.b, demand, wk.mode == MODE_DIRECT, due, inv, bk, op, act, ship, obs, ic, bc);
    if (wk.mode == MODE_STORE) {
      ring.store(wk.write_slot, ship);
    } else if (wk.mode == MODE_ADD) {
      int32_t cur[L];
      ring.load(wk.write_slot, cur);
#pragma unroll
      for (int l = 0; l < L; ++l) cur[l] += ship[l];
      ring.store(wk.write_slot, cur);
    }
    if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);
    ret += reward;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      iacc[l] += ic[l];
      bacc[l] += bc[l];
    }
    if ((wk.flags & 1) && a.final_ret) a.final_ret[n] = ret;
    if (wk.flags & 2) {  // auto-reset in registers (:140-156)
#pragma unroll
      for (int l = 0; l < L; ++l) {
        inv[l] = a.init_inv[l];
        bk[l] = 0;
        op[l] = a.orders_value;
        iacc[l] = bacc[l] = 0;
        obs[l] = inv[l];
      }
      int32_t init[L];
#pragma unroll
      for (int l = 0; l < L; ++l) init[l] = a.ship_value;
      for (int t = 1; t <= a.init_slots; ++t) ring.store(t % a.ring_slots, init);
      if (a.hist) fill_row<L>(a.hist + row, a.orders_value);
      ret = 0;
      ++episode;
    }
    if (obs_out) store_row<L>(obs_out + k * stride + row, obs);
    if (rew_out) rew_out[k * a.n + n] = reward;
  }
  }
  store_row<L>(a.inv + row, inv);
  store_row<L>(a.bk + row, bk);
  store_row<L>(a.op + row, op);
  if (a.inv_acc) store_row<L>(a.inv_acc + row, iacc);
  if (a.bk_acc) store_row<L>(a.bk_acc + row, bacc);
  if (a.ep_ret) a.ep_ret[n] = ret;
}

template <int L>
__global__ __launch_bounds__(kBlock) void bg_rollout_kernel(const BgArgs a, int32_t K, const RolloutWeeks weeks,
                                                            const int32_t* __restrict__ acts, int32_t* __restrict__ obs_out,
                                                            int32_t* __restrict__ rew_out) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= a.n) return;
  rollout_body<L>(a, n, K, weeks, acts, obs_out, rew_out, RingHbm<L>{a.ring, a.n * L, n * L});
}

template <int L>
__global__ __launch_bounds__(kBlock) void bg_rollout_lds_kernel(const BgArgs a, int32_t K, const RolloutWeeks weeks,
                                                                const int32_t* __restrict__ acts,
                                                                int32_t* __restrict__ obs_out,
                                                                int32_t* __restrict__ rew_out) {
  extern __shared__ int32_t lds_ring[];
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= a.n) return;  // lanes only touch their own LDS column: no block barrier needed
  const RingHbm<L> hbm{a.ring, a.n * L, n * L};
  const RingLds<L> lds{lds_ring + threadIdx.x};
  for (int s = 0; s < a.ring_slots; ++s) {
    int32_t v[L];
    hbm.load(s, v);
    lds.store(s, v);
  }
  rollout_body<L>(a, n, K, weeks, acts, obs_out, rew_out, lds);
  for (int s = 0; s < a.ring_slots; ++s) {
    int32_t v[L];
    lds.load(s, v);
    hbm.store(s, v);
  }
}

// Philox draws for tests/benchmarks ------------------------------------------------------
__global__ __launch_bounds__(kBlock) void poisson_demand_kernel(const BgArgs a, int32_t weeks,
                                                                int32_t* __restrict__ out) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= a.n) return;
  for (int32_t w = 1; w <= weeks; ++w) out[(int64_t)(w - 1) * a.n + n] = week_demand(a, n, w, a.episode);
}

__global__ __launch_bounds__(kBlock) void uniform_ints_kernel(uint32_t k0, uint32_t k1, int64_t env_offset,
                                                              int64_t n_envs, int32_t rows, int32_t width,
                                                              uint32_t tag, int32_t lo, uint32_t range,
                                                              int32_t* __restrict__ out) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= n_envs) return;
  const uint32_t env = static_cast<uint32_t>(env_offset + n);
  const int32_t words = rows * width;
  for (int32_t j0 = 0; j0 < words; j0 += 4) {
    const scg::U4 r = scg::philox4x32_10(scg::U4{env, tag, static_cast<uint32_t>(j0 >> 2), SCG_STREAM_ACTION}, k0, k1);
    const uint32_t w4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int32_t j = j0 + s;
      if (j < words) {
        const uint32_t v = static_cast<uint32_t>((static_cast<uint64_t>(w4[s]) * range) >> 32);
        const int32_t rrow = j / width, col = j - rrow * width;
        out[((int64_t)rrow * n_envs + n) * width + col] = lo + static_cast<int32_t>(v);
      }
    }
  }
}

// ---- host helpers ---------------------------------------------------------------------
#define SCG_LEVEL_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

int launch_reset(int L, dim3 grid, hipStream_t s, const BgArgs& a) {
  switch (L) {
#define X(l) case l: hipLaunchKernelGGL(bg_reset_kernel<l>, grid, dim3(kBlock), 0, s, a); break;
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
  return check_launch("bg_reset_kernel");
}

int launch_step2(int L, dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk) {
  switch (L) {
#define X(l) case l: hipLaunchKernelGGL(bg2_step_kernel<l>, grid, dim3(kBlock), 0, s, a, wk); break;
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
  return check_launch("bg2_step_kernel");
}

template <int DM>
int launch_step_dm(int L, dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk, hipEvent_t ev0,
                   hipEvent_t ev1) {
  switch (L) {
#define X(l) case l: hipExtLaunchKernelGGL(HIP_KERNEL_NAME(bg_step_kernel<l, DM>), grid, dim3(kBlock), 0, s, ev0, ev1, 0, a.inv, a.bk, a.op, a.act, a.ring, static_cast<uint32_t>(a.n), pack_week(wk), a, wk); break;
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
  return check_launch("bg_step_kernel");
}

int launch_step(int L, dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk, hipEvent_t ev0,
                hipEvent_t ev1) {
  // hipExtLaunchKernelGGL ties the optional events to this dispatch's own start/end
  // timestamps (the numbers rocprofv3 reports), not to separate event packets.
  switch (a.demand_mode) {
    case SCG_DEMAND_FIXED: return launch_step_dm<SCG_DEMAND_FIXED>(L, grid, s, a, wk, ev0, ev1);
    case SCG_DEMAND_TABLE: return launch_step_dm<SCG_DEMAND_TABLE>(L, grid, s, a, wk, ev0, ev1);
    case SCG_DEMAND_UNIFORM: return launch_step_dm<SCG_DEMAND_UNIFORM>(L, grid, s, a, wk, ev0, ev1);
    default: return launch_step_dm<SCG_DEMAND_POISSON>(L, grid, s, a, wk, ev0, ev1);
  }
}

int launch_rollout(int L, dim3 grid, hipStream_t s, const BgArgs& a, int32_t K, const RolloutWeeks& weeks,
                   const int32_t* acts, int32_t* obs, int32_t* rew) {
  const size_t lds = static_cast<size_t>(a.ring_slots) * L * kBlock * sizeof(int32_t);
  if (lds <= 64 * 1024) {  // ring staged in LDS for the launch
    switch (L) {
#define X(l) case l: hipLaunchKernelGGL(bg_rollout_lds_kernel<l>, grid, dim3(kBlock), lds, s, a, K, weeks, acts, obs, rew); break;
      SCG_LEVEL_CASES(X)
#undef X
      default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
    }
    return check_launch("bg_rollout_lds_kernel");
  }
  switch (L) {
#define X(l) case l: hipLaunchKernelGGL(bg_rollout_kernel<l>, grid, dim3(kBlock), 0, s, a, K, weeks, acts, obs, rew); break;
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
  return check_launch("bg_rollout_kernel");
}

int check_state(const scg_bg_config* cfg, const scg_bg_state* st) {
  if (!cfg || !st) return fail(SCG_ERR_INVALID, "null config/state");
  if (!cfg->plan || cfg->ring_slots <= 0) return fail(SCG_ERR_INVALID, "config not prepared (call scg_bg_prepare)");
  if (st->n_envs <= 0) return fail(SCG_ERR_INVALID, "n_envs must be > 0");
  if (st->n_envs > INT32_MAX) return fail(SCG_ERR_INVALID, "n_envs must be <= %d per shard", INT32_MAX);
  if (st->env_offset < 0 || st->env_offset + st->n_envs > (int64_t(1) << 32))
    return fail(SCG_ERR_INVALID, "global env ids must fit in 32 bits");
  if (!st->inventory || !st->backlog || !st->orders_placed || !st->shipments)
    return fail(SCG_ERR_INVALID, "state buffers inventory/backlog/orders_placed/shipments are required");
  if (cfg->demand_mode == SCG_DEMAND_TABLE && !cfg->demand_table)
    return fail(SCG_ERR_INVALID, "TABLE demand mode needs demand_table");
  if (cfg->demand_mode == SCG_DEMAND_POISSON && !cfg->poisson_thresholds)
    return fail(SCG_ERR_INVALID, "POISSON demand mode needs poisson_thresholds");
  return SCG_OK;
}

BgArgs make_args(const scg_bg_config* cfg, const scg_bg_state* st) {
  BgArgs a;
  std::memset(&a, 0, sizeof(a));
  a.inv = st->inventory;
  a.bk = st->backlog;
  a.op = st->orders_placed;
  a.ring = st->shipments;
  a.inv_acc = st->inventory_costs;
  a.bk_acc = st->backlog_costs;
  a.hist = st->orders_history;
  a.ep_ret = st->episode_return;
  a.final_ret = st->final_return;
  a.demand_table = cfg->demand_table;
  a.pthr = cfg->poisson_thresholds;
  a.n = st->n_envs;
  a.env_offset = st->env_offset;
  a.key0 = static_cast<uint32_t>(st->seed & 0xffffffffu);
  a.key1 = static_cast<uint32_t>(st->seed >> 32);
  a.episode = st->episode;
  a.demand_mode = cfg->demand_mode;
  a.pthr_len = cfg->poisson_len;
  a.h = cfg->inv_cost;
  a.b = cfg->backlog_cost;
  a.ship_value = cfg->initial_shipment_value;
  a.orders_value = cfg->initial_orders_value;
  a.init_slots = std::min(cfg->shipment_delays ? cfg->shipment_delays[0] : 0, cfg->max_weeks);
  a.ring_slots = cfg->ring_slots;
  for (int l = 0; l < cfg->levels; ++l) a.init_inv[l] = cfg->initial_inventory[l];
  a.demand_lo = cfg->demand_lo;
  a.demand_hi = cfg->demand_hi;
  a.max_weeks = cfg->max_weeks;
  if (cfg->variant == 2) {
    a.pen_acc = st->penalty_costs;
    a.max_stock = cfg->max_stock;
    a.penalty = cfg->exceeded_capacity_penalty;
    a.stochastic_delays = cfg->stochastic_delays;
    a.delay_lo = cfg->delay_lo;
    a.delay_hi = cfg->delay_hi;
  }
  return a;
}

inline dim3 grid_for(int64_t n) { return dim3(static_cast<unsigned>((n + kBlock - 1) / kBlock)); }

}  // namespace scg

using namespace scg;

// ========================================================================================
extern "C" {

int scg_bg_struct_sizes(size_t* config_size, size_t* state_size) {
  if (config_size) *config_size = sizeof(scg_bg_config);
  if (state_size) *state_size = sizeof(scg_bg_state);
  return SCG_OK;
}

int scg_poisson_table(double lam, uint32_t* out, int32_t cap) {
  if (!(lam >= 0.0) || std::isinf(lam)) return -fail(SCG_ERR_INVALID, "poisson lambda must be finite and >= 0");
  if (!out || cap <= 0) return -fail(SCG_ERR_INVALID, "null/empty threshold buffer");
  double p = std::exp(-lam);
  double c = p;
  for (int32_t k = 0; k < cap; ++k) {
    const double t = c * 4294967296.0;
    const uint32_t v = t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
    out[k] = v;
    if (v == 0xffffffffu) return k + 1;
    p = p * lam / static_cast<double>(k + 1);
    c = c + p;
  }
  return -fail(SCG_ERR_INVALID, "poisson lambda %g needs more than %d thresholds", lam, cap);
}

int scg_bg_prepare(scg_bg_config* cfg) {
  if (!cfg) return fail(SCG_ERR_INVALID, "null config");
  const int32_t L = cfg->levels, T = cfg->max_weeks;
  if (L < 1 || L > SCG_BG_MAX_LEVELS) return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  if (T < 1 || T > SCG_BG_MAX_WEEKS) return fail(SCG_ERR_INVALID, "max_weeks=%d outside 1..%d", T, SCG_BG_MAX_WEEKS);
  if (!cfg->shipment_delays || !cfg->plan) return fail(SCG_ERR_INVALID, "shipment_delays and plan are required");
  if (cfg->variant == 0) cfg->variant = 1;
  if (cfg->variant != 1 && cfg->variant != 2) return fail(SCG_ERR_INVALID, "variant must be 1 or 2");
  if (cfg->demand_mode < SCG_DEMAND_FIXED || cfg->demand_mode > SCG_DEMAND_UNIFORM)
    return fail(SCG_ERR_INVALID, "unknown demand_mode %d", cfg->demand_mode);
  if (cfg->demand_mode == SCG_DEMAND_UNIFORM && !(cfg->demand_hi > cfg->demand_lo))
    return fail(SCG_ERR_INVALID, "uniform demand needs demand_lo < demand_hi");
  if (cfg->variant == 1 && cfg->stochastic_delays)
    return fail(SCG_ERR_INVALID, "stochastic shipment delays are a BeerGameEnv2 option");
  if (cfg->demand_mode == SCG_DEMAND_FIXED && !cfg->customer_demand)
    return fail(SCG_ERR_INVALID, "FIXED demand mode needs customer_demand");
  if (cfg->demand_mode == SCG_DEMAND_POISSON && (cfg->poisson_len < 1 || cfg->poisson_len > SCG_POISSON_MAX))
    return fail(SCG_ERR_INVALID, "poisson_len=%d outside 1..%d", cfg->poisson_len, SCG_POISSON_MAX);
  int32_t max_delay = 0;
  for (int32_t w = 0; w <= T; ++w) {
    const int32_t d = cfg->shipment_delays[w];
    if (d < 0 || d > SCG_BG_MAX_DELAY)
      return fail(SCG_ERR_INVALID, "shipment_delays[%d]=%d outside 0..%d", w, d, SCG_BG_MAX_DELAY);
    max_delay = std::max(max_delay, d);
  }
  int32_t R = max_delay + 1;
  if (cfg->stochastic_delays) {  // per-lane randint(lo, hi) delays: ring covers hi - 1 and the initial 2
    if (cfg->delay_lo < 0 || cfg->delay_hi <= cfg->delay_lo || cfg->delay_hi > SCG_BG_MAX_DELAY + 1)
      return fail(SCG_ERR_INVALID, "stochastic delays need 0 <= delay_lo < delay_hi <= %d", SCG_BG_MAX_DELAY + 1);
    R = std::max(R, cfg->delay_hi);
  }
  // Which arrival weeks have been written, in week order (writes only target later weeks).
  std::vector<uint8_t> written(static_cast<size_t>(T) + 2, 0);
  const int32_t d0 = cfg->shipment_delays[0];
  for (int32_t t = 1; t <= std::min(d0, T); ++t) written[t] = 1;  // initial pipeline (:52)
  cfg->plan[0] = 0;
  for (int32_t w = 1; w <= T; ++w) {
    const int32_t d = cfg->shipment_delays[w];
    int32_t mode;
    if (d == 0) {
      mode = MODE_DIRECT;                 // :93-94, :111-112
    } else if (w + d > T) {
      mode = MODE_DROP;                   // lands after the last step: never received
    } else if (written[w + d]) {
      mode = MODE_ADD;                    // several weeks ship into one arrival week
    } else {
      mode = MODE_STORE;
      written[w + d] = 1;
    }
    cfg->plan[w] = mode | (written[w] ? PLAN_ARRIVE : 0) | (d << 8);
  }
  cfg->ring_slots = R;
  return SCG_OK;
}

int scg_bg_reset(const scg_bg_config* cfg, scg_bg_state* st, int32_t* obs, void* stream) {
  if (int rc = check_state(cfg, st)) return rc;
  if (st->week >= 0) st->episode += 1;  // the previous episode (finished or not) is discarded
  BgArgs a = make_args(cfg, st);
  a.obs = obs;
  if (int rc = launch_reset(cfg->levels, grid_for(st->n_envs), static_cast<hipStream_t>(stream), a)) return rc;
  st->week = 0;
  return SCG_OK;
}

// Per-week launch info for week w of the current episode.
static scg::WeekInfo week_info(const scg_bg_config* cfg, int32_t w, uint32_t flags) {
  const int32_t p = cfg->plan[w];
  const int32_t R = cfg->ring_slots;
  WeekInfo wk;
  wk.week = w;
  wk.read_slot = plan_arrive(p) ? w % R : -1;
  wk.write_slot = (w + plan_delay(p)) % R;
  wk.mode = plan_mode(p);
  wk.demand_fixed = cfg->demand_mode == SCG_DEMAND_FIXED ? cfg->customer_demand[w - 1] : 0;
  const bool terminal = (w == cfg->max_weeks);
  wk.flags = (terminal ? 1 : 0) | ((terminal && (flags & SCG_BG_AUTORESET)) ? 2 : 0);
  return wk;
}

static int check_step(const scg_bg_config* cfg, const scg_bg_state* st) {
  if (st->week < 0) return fail(SCG_ERR_NOT_RESET, "step() before reset()");
  if (st->week >= cfg->max_weeks)
    return fail(SCG_ERR_PAST_HORIZON, "step() after the terminal week %d (customer_demand has %d weeks)",
                cfg->max_weeks, cfg->max_weeks);
  return SCG_OK;
}

int scg_bg_step(const scg_bg_config* cfg, scg_bg_state* st, const int32_t* action, int32_t* obs,
                int32_t* reward, int32_t* terminal_obs, uint32_t flags, int32_t* done, void* stream) {
  return scg_bg_step_timed(cfg, st, action, obs, reward, terminal_obs, flags, done, nullptr, nullptr, stream);
}

int scg_bg_step_timed(const scg_bg_config* cfg, scg_bg_state* st, const int32_t* action, int32_t* obs,
                      int32_t* reward, int32_t* terminal_obs, uint32_t flags, int32_t* done, void* start_event,
                      void* stop_event, void* stream) {
  if (int rc = check_state(cfg, st)) return rc;
  if (!action || !obs || !reward) return fail(SCG_ERR_INVALID, "action/obs/reward buffers are required");
  if (int rc = check_step(cfg, st)) return rc;
  const int32_t w = st->week + 1;
  const WeekInfo wk = week_info(cfg, w, flags);
  BgArgs a = make_args(cfg, st);
  a.act = action;
  a.obs = obs;
  a.rew = reward;
  a.term_obs = terminal_obs;
  if (cfg->variant == 2) {
    if (int rc = launch_step2(cfg->levels, grid_for(st->n_envs), static_cast<hipStream_t>(stream), a, wk)) return rc;
  } else if (int rc = launch_step(cfg->levels, grid_for(st->n_envs), static_cast<hipStream_t>(stream), a, wk,
                                  static_cast<hipEvent_t>(start_event), static_cast<hipEvent_t>(stop_event))) {
    return rc;
  }
  if (wk.flags & 2) {
    st->week = 0;
    st->episode += 1;
  } else {
    st->week = w;
  }
  if (done) *done = (wk.flags & 1) ? 1 : 0;
  return SCG_OK;
}

int scg_bg_rollout(const scg_bg_config* cfg, scg_bg_state* st, int32_t n_weeks, const int32_t* actions,
                   int32_t* obs, int32_t* rewards, uint32_t flags, void* stream) {
  if (int rc = check_state(cfg, st)) return rc;
  if (!actions || n_weeks < 0) return fail(SCG_ERR_INVALID, "rollout needs actions and n_weeks >= 0");
  if (cfg->variant == 2) return fail(SCG_ERR_INVALID, "rollout is not implemented for BeerGameEnv2");
  if (int rc = check_step(cfg, st)) return rc;
  if (!(flags & SCG_BG_AUTORESET) && st->week + static_cast<int64_t>(n_weeks) > cfg->max_weeks)
    return fail(SCG_ERR_PAST_HORIZON, "rollout of %d weeks from week %d passes the terminal week %d", n_weeks,
                st->week, cfg->max_weeks);
  const int64_t stride = st->n_envs * cfg->levels;
  int32_t done_k = 0;
  while (done_k < n_weeks) {
    // one launch covers up to SCG_BG_ROLLOUT_MAX weeks; without auto-reset it stops at T
    RolloutWeeks weeks;
    int32_t K = 0;
    scg_bg_state probe = *st;
    BgArgs a = make_args(cfg, st);
    while (K < SCG_BG_ROLLOUT_MAX && done_k + K < n_weeks) {
      const int32_t w = probe.week + 1;
      weeks.wk[K] = week_info(cfg, w, flags);
      if (weeks.wk[K].flags & 2) {
        probe.week = 0;
        probe.episode += 1;
      } else {
        probe.week = w;
      }
      ++K;
    }
    if (int rc = launch_rollout(cfg->levels, grid_for(st->n_envs), static_cast<hipStream_t>(stream), a, K, weeks,
                                actions + done_k * stride, obs ? obs + done_k * stride : nullptr,
                                rewards ? rewards + done_k * st->n_envs : nullptr))
      return rc;
    st->week = probe.week;
    st->episode = probe.episode;
    done_k += K;
  }
  return SCG_OK;
}

int scg_bg_poisson_demand(const scg_bg_config* cfg, const scg_bg_state* st, uint32_t episode, int32_t* out,
                          void* stream) {
  if (int rc = check_state(cfg, st)) return rc;
  if (!out) return fail(SCG_ERR_INVALID, "null output");
  if (cfg->demand_mode != SCG_DEMAND_POISSON) return fail(SCG_ERR_INVALID, "config is not in POISSON demand mode");
  BgArgs a = make_args(cfg, st);
  a.episode = episode;
  hipLaunchKernelGGL(poisson_demand_kernel, grid_for(st->n_envs), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     a, cfg->max_weeks, out);
  return check_launch("poisson_demand_kernel");
}

int scg_uniform_ints(uint64_t seed, int64_t env_offset, int64_t n_envs, int32_t rows, int32_t width, uint32_t tag,
                     int32_t lo, int32_t hi, int32_t* out, void* stream) {
  if (!out || n_envs <= 0 || rows <= 0 || width <= 0 || hi < lo)
    return fail(SCG_ERR_INVALID, "bad uniform_ints arguments");
  const uint32_t range = static_cast<uint32_t>(static_cast<int64_t>(hi) - lo + 1);  // 0 means 2^32
  if (range == 0) return fail(SCG_ERR_INVALID, "uniform_ints range must be < 2^32");
  hipLaunchKernelGGL(uniform_ints_kernel, grid_for(n_envs), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint32_t>(seed & 0xffffffffu), static_cast<uint32_t>(seed >> 32), env_offset, n_envs,
                     rows, width, tag, lo, range, out);
  return check_launch("uniform_ints_kernel");
}

}  // extern "C"
