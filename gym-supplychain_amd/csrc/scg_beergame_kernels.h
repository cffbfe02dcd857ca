// BeerGame kernels of libscgpu.so (included by scg_beergame.hip and the per-level
// instantiation units scg_bg_levels_*.hip): the reset / step / slab step / BeerGameEnv2 /
// rollout kernels, templated on the level count L, and one launcher per kernel family and
// L. scg_beergame.hip dispatches on L at run time; the launchers are instantiated in four
// units (levels 1-4, 5-8, 9-12, 13-16) that compile in parallel.
//
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
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "scg_common.h"
#include "scg_mailbox.h"
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
  int32_t* err;        // sticky error word (bit 0: an int64 result left int32), may be null
  int32_t guard;       // week_guard(L, h, b)
  int32_t* err_host;   // host-mapped copy of the error word, refreshed at terminal weeks (may be null)
};

// The reference computes in int64 (beergame_env.py:33,35,130-132); the kernels compute each
// week in int64 too and store int32, noting whether every stored value fits.
#ifndef SCG_BG_OVERFLOW_CHECK
#define SCG_BG_OVERFLOW_CHECK 1  // 0 only for A/B timing builds (tools/exp_build.py -D)
#endif
__device__ __forceinline__ bool fits32(int64_t x) {
  return !SCG_BG_OVERFLOW_CHECK || x == static_cast<int64_t>(static_cast<int32_t>(x));
}
__device__ __forceinline__ int out32(int64_t x) { return fits32(x) ? 0 : 1; }

// Sets bit 0 of the error word when this lane saw a value outside int32: a plain vector
// store from the lanes that overflowed (idempotent, so concurrent lanes need no atomics).
__device__ __forceinline__ void note_overflow(int32_t* err, bool ovf) {
  if (ovf && err) *reinterpret_cast<volatile int32_t*>(err) = 1;
}

// At a terminal week one lane copies the error word (final for every earlier launch) to the
// caller's host-mapped word, which the host can then read without a synchronisation.
__device__ __forceinline__ void export_error(int64_t n, bool terminal, const int32_t* err, int32_t* err_host) {
  if (terminal && n == 0 && err && err_host)
    *reinterpret_cast<volatile int32_t*>(err_host) = *reinterpret_cast<const volatile int32_t*>(err);
}

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

// Row stores of the slab kernel, by policy (SCG_BG_STORE): 0 plain, 1 non-temporal (nt),
// 2 write-through (sc1: the bytes leave L2 as they are stored and the line is dropped).
// A/B on one box (profiles/r02j_bg_store_ab.log, 65,536 envs): back-to-back launches 4.73-4.79
// (plain) / 4.61 (nt) / 5.05-5.07 µs (sc1) per step; launches run alone 5.36-5.41 / 5.16 /
// 4.73 µs. The bench and a training loop run launches back to back, so nt is the default.
#ifndef SCG_BG_STORE
#define SCG_BG_STORE 1
#endif
typedef int v4i32 __attribute__((ext_vector_type(4)));

template <int L>
__device__ __forceinline__ void store_row_p(int32_t* __restrict__ p, const int32_t (&v)[L]) {
  if constexpr (SCG_BG_STORE != 0 && L % 4 == 0) {
#pragma unroll
    for (int c = 0; c < L / 4; ++c) {
      const v4i32 x = {v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
      if constexpr (SCG_BG_STORE == 1) {
        __builtin_nontemporal_store(x, reinterpret_cast<v4i32*>(p) + c);
      } else {
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(reinterpret_cast<v4i32*>(p) + c), "v"(x)
                     : "memory");
      }
    }
  } else {
    store_row<L>(p, v);
  }
}

template <int L>
__device__ __forceinline__ void fill_row_p(int32_t* __restrict__ p, int32_t x) {
  int32_t v[L];
#pragma unroll
  for (int l = 0; l < L; ++l) v[l] = x;
  store_row_p<L>(p, v);
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
  // reset() starts clean: the int32-overflow word (and its host-mapped copy) is scoped to
  // the episodes since the last reset, in stream order after every earlier launch
  if (n == 0) {
    if (a.err) *reinterpret_cast<volatile int32_t*>(a.err) = 0;
    if (a.err_host) *reinterpret_cast<volatile int32_t*>(a.err_host) = 0;
  }
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
                                             int32_t (&obs)[L], int64_t (&ic)[L], int64_t (&bc)[L], bool& ovf) {
  // 1. receive the shipments due this week (:72)
  // 2. order slips: customer demand at level 0, the previous orders above (:79-81)
  int64_t inc[L];
  inc[0] = demand;
#pragma unroll
  for (int l = 1; l < L; ++l) inc[l] = op[l - 1];
  // fill what inventory allows (:85-89); ship[l] = what level l receives: deliver[l+1]
  // from the level above it, and for the factory its own orders_placed[-1] from before
  // this step (:93-96, :111-114)
  int64_t iv[L], fill[L], del[L], sh[L];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    iv[l] = static_cast<int64_t>(inv[l]) + due[l];
    fill[l] = inc[l] + bk[l];
    del[l] = iv[l] < fill[l] ? iv[l] : fill[l];
  }
#pragma unroll
  for (int l = 0; l + 1 < L; ++l) sh[l] = del[l + 1];
  sh[L - 1] = op[L - 1];
  // 3. inventory / backlog (:101-103); 5. place orders (:121); obs (:127,:180); cost (:130)
  int64_t cost = 0;
  int bad = 0;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    iv[l] += (direct ? sh[l] : 0) - del[l];
    const int64_t b64 = fill[l] - del[l];
    const int64_t o64 = inc[l] + act[l];
    const int64_t ob = iv[l] - b64;
    ic[l] = static_cast<int64_t>(h) * iv[l];
    bc[l] = static_cast<int64_t>(b) * b64;
    cost += ic[l] + bc[l];
    bad |= out32(iv[l]) | out32(b64) | out32(o64) | out32(ob) | out32(sh[l]);
    inv[l] = static_cast<int32_t>(iv[l]);
    bk[l] = static_cast<int32_t>(b64);
    op[l] = static_cast<int32_t>(o64);
    obs[l] = static_cast<int32_t>(ob);
    ship[l] = static_cast<int32_t>(sh[l]);
  }
  bad |= out32(-cost);
  ovf |= bad != 0;
  return static_cast<int32_t>(-cost);
}

// The same week in int32 arithmetic: exact when week_update's guard holds.
template <int L>
__device__ __forceinline__ int32_t step_core32(int32_t h, int32_t b, int32_t demand, bool direct,
                                               const int32_t (&due)[L], int32_t (&inv)[L], int32_t (&bk)[L],
                                               int32_t (&op)[L], const int32_t (&act)[L], int32_t (&ship)[L],
                                               int32_t (&obs)[L], int32_t (&ic)[L], int32_t (&bc)[L]) {
  int32_t inc[L];
  inc[0] = demand;
#pragma unroll
  for (int l = 1; l < L; ++l) inc[l] = op[l - 1];
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

// Largest magnitude a week's state inputs may have for int32 arithmetic to be exact:
// with every input (state rows, action, due and accumulating ring rows, demand) in
// (-G, G) each intermediate stays below 10 G and the cost below 10 L G max(|h|, |b|, 1),
// so G = 2^30 / (10 L max(|h|, |b|, 1)) keeps all of them, and the ledgers (inputs below
// 2^30, week costs below 2^30), inside int32.
inline int32_t week_guard(int L, int32_t h, int32_t b) {
  const int64_t m = std::max<int64_t>({std::llabs(h), std::llabs(b), int64_t(1)});
  return static_cast<int32_t>((int64_t(1) << 30) / (10 * static_cast<int64_t>(L) * m));
}

template <int L>
__device__ __forceinline__ void range_of(const int32_t (&v)[L], int32_t& lo, int32_t& hi) {
#pragma unroll
  for (int l = 0; l < L; ++l) {
    lo = min(lo, v[l]);
    hi = max(hi, v[l]);
  }
}

// One week of one env plus its pipeline-slot accumulation (cur += ship, used for MODE_ADD)
// and ledger updates (:131-132): the int32 path when every input lies inside the config's
// guard (nothing can then overflow), else the exact int64 path, which notes in `ovf` any
// stored value that does not fit int32. Bit-identical results while nothing overflows.
template <int L>
__device__ __forceinline__ int32_t week_update(int32_t h, int32_t b, int32_t guard, int32_t demand, bool direct,
                                               const int32_t (&due)[L], int32_t (&inv)[L], int32_t (&bk)[L],
                                               int32_t (&op)[L], const int32_t (&act)[L], int32_t (&ship)[L],
                                               int32_t (&obs)[L], int32_t (&cur)[L], int32_t (&iacc)[L],
                                               int32_t (&bacc)[L], bool& ovf) {
  int32_t lo = demand, hi = demand, llo = 0, lhi = 0;
  range_of<L>(inv, lo, hi);
  range_of<L>(bk, lo, hi);
  range_of<L>(op, lo, hi);
  range_of<L>(act, lo, hi);
  range_of<L>(due, lo, hi);
  range_of<L>(cur, lo, hi);
  range_of<L>(iacc, llo, lhi);
  range_of<L>(bacc, llo, lhi);
  constexpr int32_t kLedger = 1 << 30;
  if (hi < guard && lo > -guard && lhi < kLedger && llo > -kLedger) {
    int32_t ic[L], bc[L];
    const int32_t r = step_core32<L>(h, b, demand, direct, due, inv, bk, op, act, ship, obs, ic, bc);
#pragma unroll
    for (int l = 0; l < L; ++l) {
      cur[l] += ship[l];
      iacc[l] += ic[l];
      bacc[l] += bc[l];
    }
    return r;
  }
  int64_t ic[L], bc[L];
  const int32_t r = step_core<L>(h, b, demand, direct, due, inv, bk, op, act, ship, obs, ic, bc, ovf);
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int64_t c = static_cast<int64_t>(cur[l]) + ship[l];
    const int64_t x = static_cast<int64_t>(iacc[l]) + ic[l], y = static_cast<int64_t>(bacc[l]) + bc[l];
    ovf |= (out32(c) | out32(x) | out32(y)) != 0;
    cur[l] = static_cast<int32_t>(c);
    iacc[l] = static_cast<int32_t>(x);
    bacc[l] = static_cast<int32_t>(y);
  }
  return r;
}

// pipeline slot accumulation (several weeks shipping into one arrival week, :95-96)
template <int L>
__device__ __forceinline__ void add_ship(int32_t (&cur)[L], const int32_t (&ship)[L], bool& ovf) {
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const int64_t x = static_cast<int64_t>(cur[l]) + ship[l];
    ovf |= out32(x) != 0;
    cur[l] = static_cast<int32_t>(x);
  }
}

template <int L>
__device__ __forceinline__ void zero_row(int32_t (&v)[L]) {
#pragma unroll
  for (int l = 0; l < L; ++l) v[l] = 0;
}

// Week plan packed into one dword for the step kernel's preloaded arguments:
// bits 0-13 read_slot + 1 (0: nothing due), 14-27 write_slot, 28-29 mode, 30-31 flags
// (slots < 2^14 > SCG_BG_MAX_WEEKS + SCG_BG_MAX_DELAY + 2, the longest full table).
constexpr uint32_t kWeekSlotBits = 14, kWeekSlotMask = (1u << kWeekSlotBits) - 1;
static_assert(SCG_BG_MAX_WEEKS + SCG_BG_MAX_DELAY + 2 < (1 << kWeekSlotBits), "ring slot field too narrow");
inline uint32_t pack_week(const WeekInfo& wk) {
  return static_cast<uint32_t>(wk.read_slot + 1) | (static_cast<uint32_t>(wk.write_slot) << kWeekSlotBits) |
         (static_cast<uint32_t>(wk.mode) << 28) | (static_cast<uint32_t>(wk.flags) << 30);
}

// The slab kernel's week plan (its ring has at most 127 slots, scg_bg_slab_layout): bits 0-7
// read_slot + 1, 8-15 write_slot, 16-17 mode; the launcher adds the SW_* option bits and R.
inline uint32_t pack_week_slab(const WeekInfo& wk) {
  return static_cast<uint32_t>(wk.read_slot + 1) | (static_cast<uint32_t>(wk.write_slot) << 8) |
         (static_cast<uint32_t>(wk.mode) << 16);
}

// step(action) for one env per lane: every row this launch reads is loaded up front (one
// round of memory latency), the week is computed in registers, then every row is stored.
// The leading scalar arguments (the four state rows' and the ring's base pointers, the env
// count and the packed week plan: 12 dwords) are preloaded into SGPRs at wave launch
// (gfx950 kernarg preload, build flag -amdgpu-kernarg-preload-count), so the first row
// loads issue without waiting on the kernarg segment; the rest of the arguments arrive
// through scalar loads that overlap those rows, and the Poisson inversion reads its
// thresholds through the scalar cache, so it too runs while the rows are in flight.
// (the week of env n < n32: the body of bg_step_kernel and of the step server below)
// kActIn: the action row is act_in (already in registers), not read from act_p.
template <int L, int DM, bool kActIn = false>
__device__ __forceinline__ void bg_step_env(int64_t n, int32_t* __restrict__ inv_p, int32_t* __restrict__ bk_p,
                                            int32_t* __restrict__ op_p, const int32_t* __restrict__ act_p,
                                            int32_t* __restrict__ ring_p, uint32_t n32, uint32_t wpack,
                                            const BgArgs& a, const WeekInfo& wk, const int32_t* act_in = nullptr) {
  const int32_t read_slot = static_cast<int32_t>(wpack & kWeekSlotMask) - 1;
  const int32_t write_slot = static_cast<int32_t>((wpack >> kWeekSlotBits) & kWeekSlotMask);
  const int32_t mode = static_cast<int32_t>((wpack >> 28) & 3u);
  const bool terminal = wpack & (1u << 30);
  const bool autoreset = wpack & (2u << 30);
  const int64_t row = n * L;
  const int64_t stride = static_cast<int64_t>(n32) * L;

  int32_t inv[L], bk[L], op[L], act[L], due[L], cur[L], iacc[L], bacc[L];
  zero_row<L>(due);
  zero_row<L>(cur);
  load_row<L>(inv_p + row, inv);
  load_row<L>(bk_p + row, bk);
  load_row<L>(op_p + row, op);
  if constexpr (kActIn) {
#pragma unroll
    for (int l = 0; l < L; ++l) act[l] = act_in[l];
  } else {
    load_row<L>(act_p + row, act);
  }
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
  export_error(n, terminal, a.err, a.err_host);
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

  int32_t ship[L], obs[L];
  bool ovf = false;
  const int32_t reward = week_update<L>(a.h, a.b, a.guard, demand, mode == MODE_DIRECT, due, inv, bk, op, act, ship,
                                        obs, cur, iacc, bacc, ovf);

  if (mode == MODE_STORE) {
    store_row<L>(ring_p + write_slot * stride + row, ship);
  } else if (mode == MODE_ADD) {
    store_row<L>(ring_p + write_slot * stride + row, cur);
  }  // MODE_DROP: arrives after the horizon, never observable
  a.rew[n] = reward;
  if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);  // :123
  if (terminal && a.term_obs) store_row<L>(a.term_obs + row, obs);
  const int64_t ret = ret0 + reward;
  if (terminal && a.final_ret) a.final_ret[n] = ret;
  if (autoreset) {  // the next step starts a fresh episode (reset() in the same launch)
    reset_env<L>(a, n, a.obs);
    note_overflow(a.err, ovf);
    return;
  }
  store_row<L>(inv_p + row, inv);
  store_row<L>(bk_p + row, bk);
  store_row<L>(op_p + row, op);
  store_row<L>(a.obs + row, obs);
  if (a.inv_acc) store_row<L>(a.inv_acc + row, iacc);  // :131
  if (a.bk_acc) store_row<L>(a.bk_acc + row, bacc);    // :132
  if (a.ep_ret) a.ep_ret[n] = ret;
  note_overflow(a.err, ovf);
}

template <int L, int DM>
__global__ __launch_bounds__(kBlock) void bg_step_kernel(int32_t* __restrict__ inv_p, int32_t* __restrict__ bk_p,
                                                         int32_t* __restrict__ op_p, const int32_t* __restrict__ act_p,
                                                         int32_t* __restrict__ ring_p, uint32_t n32, uint32_t wpack,
                                                         const BgArgs a, const WeekInfo wk) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= static_cast<int64_t>(n32)) return;
  bg_step_env<L, DM>(n, inv_p, bk_p, op_p, act_p, ring_p, n32, wpack, a, wk);
}

// ---- step server (scg_bg_server_*: the drop-in BeerGameEnv) -------------------------------
// A request is one 64-byte line of the mailbox (scg_bg_server_line, scg_mailbox.h).
inline __host__ __device__ uint32_t server_line_check(const uint32_t (&w)[16]) { return mailbox_check(w); }

constexpr int kServerBlock = 64;
constexpr int kServerSlots = SCG_BG_SERVER_SLOTS;
constexpr int kServerArgWords = (sizeof(BgArgs) + 15) / 16 * 4;  // rows 16-byte aligned
static_assert(sizeof(BgArgs) <= SCG_BG_SERVER_ARGS_BYTES, "BgArgs outgrew the mailbox's argument blocks");
static_assert(kServerSlots <= 16 && kServerArgWords <= 2 * kServerBlock, "server layout");

// One wave serves every slot of the mailbox: env n of a slot on lane n (a slot's a.n <= 64).
// Each poll reads the request lines of slots 0 .. n_slots - 1 in up to four loads (lane l
// reads word l % 16 of slot 4r + l / 16; system scope: past the caches, from host memory)
// together with the control words; for every slot whose line carries a new, consistent request the wave loads
// the slot's kernel arguments into LDS if their generation changed, runs the week body above
// with the posted plan — env 0's action row from the line itself when n_inline says it
// travelled there — and publishes the request number in the slot's answer word with a
// system-scope release store after every lane's stores. At launch every slot's last served
// request is its answer word, so requests posted while no wave ran are served first. It exits
// when exit_req changes, or when no request has come for idle_ticks of the 100 MHz real-time
// clock, so it never outlives its host process; as it exits it writes the exit word it saw.
template <int L, int DM>
__global__ __launch_bounds__(kServerBlock) void bg_server_kernel(scg_bg_server_box* box, uint32_t exit_seen,
                                                                 uint32_t idle_ticks) {
  __shared__ __align__(16) uint32_t s_args[kServerSlots][kServerArgWords];
  __shared__ uint32_t s_last[16], s_gen[16];
  const int lane = threadIdx.x;
  if (lane < 16) {
    s_last[lane] = __hip_atomic_load(&box->done_seq[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    s_gen[lane] = 0;  // hosts publish generations from 1
  }
  __syncthreads();
  const uint32_t* lines = reinterpret_cast<const uint32_t*>(box->req);
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t ex = exit_seen;
  // the slot count a poll reads lines by is the one the previous poll read (requested beside
  // the lines, so a poll is one round trip to host memory): a slot attached since is polled
  // one round later
  uint32_t ns = __hip_atomic_load(&box->n_slots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    const int n_slots = __builtin_amdgcn_readfirstlane(static_cast<int>(ns < kServerSlots ? ns : kServerSlots));
    ns = __hip_atomic_load(&box->n_slots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ex = __hip_atomic_load(&box->exit_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int slot = 4 * r + (lane >> 4);
      if (slot < n_slots)
        v[r] = __hip_atomic_load(lines + slot * 16 + (lane & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    bool served = false;
    for (int slot = 0; slot < n_slots; ++slot) {
      const int base = (slot & 3) * 16, r = slot >> 2;
      const uint32_t vr = r == 0 ? v[0] : r == 1 ? v[1] : r == 2 ? v[2] : v[3];
      const uint32_t seq = __builtin_amdgcn_readlane(vr, base);
      if (seq == s_last[slot]) continue;
      uint32_t w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_readlane(vr, base + i);
      if (w[7] != server_line_check(w)) continue;  // a torn read: the next poll reads it again
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (w[6] != s_gen[slot]) {  // the slot's arguments changed (a new env or a reset): reload
        const uint32_t* src = reinterpret_cast<const uint32_t*>(box->args[slot]);
        for (int k = lane; k < kServerArgWords; k += kServerBlock)
          s_args[slot][k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        if (lane == 0) s_gen[slot] = w[6];
      }
      const BgArgs& a = *reinterpret_cast<const BgArgs*>(s_args[slot]);
      WeekInfo wk{};
      wk.week = static_cast<int32_t>(w[3]);
      wk.demand_fixed = static_cast<int32_t>(w[4]);
      const int64_t n = lane;
      if (n < a.n) {
        if (L <= 8 && static_cast<int32_t>(w[5]) == L) {  // the action row came with the request
          int32_t act_in[L];
#pragma unroll
          for (int l = 0; l < L; ++l) act_in[l] = static_cast<int32_t>(w[8 + (l < 8 ? l : 0)]);
          bg_step_env<L, DM, true>(n, a.inv, a.bk, a.op, a.act, a.ring, static_cast<uint32_t>(a.n), w[2], a, wk, act_in);
        } else {
          bg_step_env<L, DM>(n, a.inv, a.bk, a.op, a.act, a.ring, static_cast<uint32_t>(a.n), w[2], a, wk);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // every lane's stores before the answer
      if (lane == 0) {
        __hip_atomic_store(&box->done_seq[slot], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        s_last[slot] = seq;
      }
      __syncthreads();
      served = true;
    }
    if (ex != exit_seen) break;
    if (served) {
      t0 = __builtin_amdgcn_s_memrealtime();
      continue;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (lane == 0) __hip_atomic_store(&box->exit_seq, ex, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- slab step kernel -------------------------------------------------------------------
// The same week with every state row at a fixed offset from one base pointer (the slab,
// scg_bg_slab_layout): inventory, backlog, orders, both ledgers, the terminal observation,
// the ring slots, both returns and the history. The leading arguments — slab, actions,
// outputs (obs rows then rewards), env count, week plan, week, episode and the Philox key
// (12 dwords) — are preloaded into SGPRs at wave launch, so every row load and store is
// addressed without reading the kernarg segment; only the costs, the Poisson table pointer
// and the reset values arrive through scalar loads, which overlap the rows in flight.
struct BgSlabArgs {
  const uint32_t* pthr;
  const int32_t* demand_table;
  int32_t pthr_len;
  int32_t h, b;
  int32_t demand_fixed;
  int32_t demand_lo, demand_hi;
  int32_t ship_value, orders_value, init_slots;
  int64_t env_offset;
  int32_t guard;
  int32_t* err_host;
  int32_t init_inv[SCG_BG_MAX_LEVELS];
};


// wpack bits of the slab kernel
constexpr uint32_t SW_TERMINAL = 1u << 18, SW_AUTORESET = 1u << 19, SW_LEDGERS = 1u << 20, SW_RETURNS = 1u << 21,
                   SW_HISTORY = 1u << 22;
constexpr int kSlabHeader = 4;  // int32 words before the first row (the error word + padding)

template <int L, int DM>
__global__ __launch_bounds__(kBlock) void bg_step_slab_kernel(int32_t* __restrict__ slab, const int32_t* __restrict__ act_p,
                                                              int32_t* __restrict__ out, uint32_t n32, uint32_t wpack,
                                                              uint32_t week, uint32_t episode, uint32_t key0,
                                                              uint32_t key1, const BgSlabArgs a) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (n >= static_cast<int64_t>(n32)) return;
  const int32_t read_slot = static_cast<int32_t>(wpack & 0xffu) - 1;
  const int32_t write_slot = static_cast<int32_t>((wpack >> 8) & 0xffu);
  const int32_t mode = static_cast<int32_t>((wpack >> 16) & 3u);
  const int32_t R = static_cast<int32_t>((wpack >> 24) & 0x7fu);
  const bool terminal = wpack & SW_TERMINAL, autoreset = wpack & SW_AUTORESET;
  const bool ledgers = wpack & SW_LEDGERS, returns = wpack & SW_RETURNS, history = wpack & SW_HISTORY;
  const int64_t NL = static_cast<int64_t>(n32) * L;
  const int64_t row = n * L;
  int32_t* const rows = slab + kSlabHeader;           // row field f of env n: rows + f * NL + row
  int32_t* const inv_p = rows, *const bk_p = rows + NL, *const op_p = rows + 2 * NL;
  int32_t* const iacc_p = rows + 3 * NL, *const bacc_p = rows + 4 * NL, *const term_p = rows + 5 * NL;
  int32_t* const ring_p = rows + 6 * NL;
  int64_t* const ret_p = reinterpret_cast<int64_t*>(rows + (6 + R) * NL);   // 8-byte aligned: NL*4 % 16 == 0 or padded
  int64_t* const fret_p = ret_p + n32;
  int32_t* const hist_p = reinterpret_cast<int32_t*>(fret_p + n32);

  int32_t inv[L], bk[L], op[L], act[L], due[L], cur[L], iacc[L], bacc[L];
  zero_row<L>(due);
  zero_row<L>(cur);
  zero_row<L>(iacc);
  zero_row<L>(bacc);
  load_row<L>(inv_p + row, inv);
  load_row<L>(bk_p + row, bk);
  load_row<L>(op_p + row, op);
  load_row<L>(act_p + row, act);
  if (read_slot >= 0) load_row<L>(ring_p + read_slot * NL + row, due);
  if (mode == MODE_ADD) load_row<L>(ring_p + write_slot * NL + row, cur);
  if (ledgers && !autoreset) {
    load_row<L>(iacc_p + row, iacc);
    load_row<L>(bacc_p + row, bacc);
  }
  const int64_t ret0 = returns ? ret_p[n] : 0;
  export_error(n, terminal, slab, a.err_host);
  int32_t demand;
  if constexpr (DM == SCG_DEMAND_FIXED) {
    demand = a.demand_fixed;
  } else if constexpr (DM == SCG_DEMAND_TABLE) {
    demand = a.demand_table[static_cast<int64_t>(week - 1) * n32 + n];
  } else if constexpr (DM == SCG_DEMAND_UNIFORM) {
    const uint32_t w = scg::philox_word(key0, key1, static_cast<uint32_t>(a.env_offset + n), episode, week - 1,
                                        SCG_STREAM_BG2_DEMAND);
    demand = a.demand_lo + static_cast<int32_t>((static_cast<uint64_t>(w) * static_cast<uint32_t>(a.demand_hi - a.demand_lo)) >> 32);
  } else {
    const uint32_t u = scg::philox_word(key0, key1, static_cast<uint32_t>(a.env_offset + n), episode, week - 1,
                                        SCG_STREAM_DEMAND);
    demand = poisson_count_scalar(const_tab(a.pthr), a.pthr_len, u);
  }

  int32_t ship[L], obs[L];
  bool ovf = false;
  const int32_t reward = week_update<L>(a.h, a.b, a.guard, demand, mode == MODE_DIRECT, due, inv, bk, op, act, ship,
                                        obs, cur, iacc, bacc, ovf);
  if (mode == MODE_STORE) {
    store_row_p<L>(ring_p + write_slot * NL + row, ship);
  } else if (mode == MODE_ADD) {
    store_row_p<L>(ring_p + write_slot * NL + row, cur);
  }
  out[NL + n] = reward;                                                      // rewards follow the obs rows
  if (history) store_row_p<L>(hist_p + static_cast<int64_t>(week) * NL + row, op);   // :123
  const int64_t ret = ret0 + reward;
  if (terminal) {
    store_row_p<L>(term_p + row, obs);
    if (returns) fret_p[n] = ret;
  }
  if (autoreset) {  // reset() in the same launch (:140-156)
    int32_t v[L];
#pragma unroll
    for (int l = 0; l < L; ++l) v[l] = a.init_inv[l];
    store_row_p<L>(inv_p + row, v);
    store_row_p<L>(out + row, v);                                              // reset obs: inventory - 0
    fill_row_p<L>(bk_p + row, 0);
    fill_row_p<L>(op_p + row, a.orders_value);
    for (int t = 1; t <= a.init_slots; ++t) fill_row_p<L>(ring_p + (t % R) * NL + row, a.ship_value);
    if (ledgers) {
      fill_row_p<L>(iacc_p + row, 0);
      fill_row_p<L>(bacc_p + row, 0);
    }
    if (history) fill_row_p<L>(hist_p + row, a.orders_value);
    if (returns) ret_p[n] = 0;
    note_overflow(slab, ovf);
    return;
  }
  store_row_p<L>(inv_p + row, inv);
  store_row_p<L>(bk_p + row, bk);
  store_row_p<L>(op_p + row, op);
  store_row_p<L>(out + row, obs);
  if (ledgers) {  // :131-132
    store_row_p<L>(iacc_p + row, iacc);
    store_row_p<L>(bacc_p + row, bacc);
  }
  if (returns) ret_p[n] = ret;
  note_overflow(slab, ovf);
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
  export_error(n, terminal, a.err, a.err_host);
  const int32_t demand = a.demand_mode == SCG_DEMAND_FIXED ? wk.demand_fixed : week_demand(a, n, wk.week, a.episode);

  // the week in int64, as the reference computes it; stored values checked against int32
  int64_t inc[L], iv[L], fill[L], del[L], sh[L];
  int32_t ship[L], obs[L];
  bool ovf = false;
  inc[0] = demand;
#pragma unroll
  for (int l = 1; l < L; ++l) inc[l] = op[l - 1];
#pragma unroll
  for (int l = 0; l < L; ++l) {
    iv[l] = static_cast<int64_t>(inv[l]) + due[l];
    fill[l] = inc[l] + bk[l];
    del[l] = iv[l] < fill[l] ? iv[l] : fill[l];
  }
#pragma unroll
  for (int l = 0; l + 1 < L; ++l) sh[l] = del[l + 1];
  sh[L - 1] = op[L - 1];
  int64_t cost = 0, pen = 0;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    iv[l] += (mode == MODE_DIRECT ? sh[l] : 0) - del[l];
    const int64_t b64 = fill[l] - del[l];
    const int64_t ob = static_cast<int64_t>(a.max_stock) + iv[l] - b64;
    const int64_t over = (iv[l] > a.max_stock ? iv[l] - a.max_stock : 0) + (b64 > a.max_stock ? b64 - a.max_stock : 0);
    const int64_t i_c = static_cast<int64_t>(a.h) * iv[l], b_c = static_cast<int64_t>(a.b) * b64;
    const int64_t p_c = static_cast<int64_t>(a.penalty) * over;
    const int64_t ia = iacc[l] + i_c, ba = bacc[l] + b_c, pa = pacc[l] + p_c;
    cost += i_c + b_c;
    pen += p_c;
    ovf |= out32(iv[l]) | out32(b64) | out32(ob) | out32(sh[l]) | out32(ia) | out32(ba) | out32(pa);
    inv[l] = static_cast<int32_t>(iv[l]);
    bk[l] = static_cast<int32_t>(b64);
    op[l] = act[l];                                   // absolute orders (:168)
    obs[l] = static_cast<int32_t>(ob);
    ship[l] = static_cast<int32_t>(sh[l]);
    iacc[l] = static_cast<int32_t>(ia);
    bacc[l] = static_cast<int32_t>(ba);
    pacc[l] = static_cast<int32_t>(pa);
  }
  const int64_t reward64 = -cost - pen;               // :177-180
  ovf |= out32(reward64);
  const int32_t reward = static_cast<int32_t>(reward64);

  if (a.stochastic_delays) {  // consumed: the slot is reused R weeks on
    int32_t z[L];
    zero_row<L>(z);
    store_row<L>(a.ring + read_slot * stride + row, z);
  }
  if (mode == MODE_STORE) {
    store_row<L>(a.ring + write_slot * stride + row, ship);
  } else if (mode == MODE_ADD) {
    add_ship<L>(cur, ship, ovf);
    store_row<L>(a.ring + write_slot * stride + row, cur);
  }
  a.rew[n] = reward;
  if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);
  if (terminal && a.term_obs) store_row<L>(a.term_obs + row, obs);
  const int64_t ret = ret0 + reward;
  if (terminal && a.final_ret) a.final_ret[n] = ret;
  note_overflow(a.err, ovf);
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
  bool ovf = false;
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
    int32_t due[L], obs[L], ship[L], cur[L];
    int32_t(&act)[L] = group_act[u];
    zero_row<L>(due);
    if (wk.read_slot >= 0) ring.load(wk.read_slot, due);
    int32_t demand;
    if (a.demand_mode == SCG_DEMAND_FIXED)
      demand = wk.demand_fixed;
    else
      demand = week_demand(a, n, wk.week, episode);
    zero_row<L>(cur);
    if (wk.mode == MODE_ADD) ring.load(wk.write_slot, cur);
    const int32_t reward = week_update<L>(a.h, a.b, a.guard, demand, wk.mode == MODE_DIRECT, due, inv, bk, op, act, ship,
                                          obs, cur, iacc, bacc, ovf);
    if (wk.mode == MODE_STORE) {
      ring.store(wk.write_slot, ship);
    } else if (wk.mode == MODE_ADD) {
      ring.store(wk.write_slot, cur);
    }
    if (a.hist) store_row<L>(a.hist + static_cast<int64_t>(wk.week) * stride + row, op);
    ret += reward;
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
  note_overflow(a.err, ovf);
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

#ifndef SCG_MODULE_LAUNCH
#define SCG_MODULE_LAUNCH 1  // 0: unstamped slab launches through hipLaunchKernelGGL (A/B builds)
#endif

// hipModuleLaunchKernel with the kernel's function handle resolved once per instantiation,
// skipping the host-stub lookup of hipLaunchKernel on every step: ≈0.5 µs less host time
// per step (tools/short_region.py, profiles/r02h_short_region.log).
template <int L, int DM>
int launch_slab_module(dim3 grid, hipStream_t s, int32_t* slab, const int32_t* act, int32_t* out, uint32_t n32,
                       uint32_t wpack, uint32_t week, uint32_t episode, uint32_t k0, uint32_t k1, const BgSlabArgs& a) {
  static hipFunction_t fn = nullptr;
  if (!fn && hipGetFuncBySymbol(&fn, reinterpret_cast<const void*>(&bg_step_slab_kernel<L, DM>)) != hipSuccess)
    return fail(SCG_ERR_HIP, "hipGetFuncBySymbol(bg_step_slab_kernel) failed");
  BgSlabArgs args = a;
  void* params[] = {&slab, &act, &out, &n32, &wpack, &week, &episode, &k0, &k1, &args};
  if (hipModuleLaunchKernel(fn, grid.x, 1, 1, kBlock, 1, 1, 0, s, params, nullptr) != hipSuccess)
    return fail(SCG_ERR_HIP, "hipModuleLaunchKernel(bg_step_slab_kernel) failed");
  return SCG_OK;
}

// ---- per-level launchers (explicitly instantiated in scg_bg_levels_*.hip) ---------------
template <int L>
int bg_launch_reset(dim3 grid, hipStream_t s, const BgArgs& a) {
  hipLaunchKernelGGL(bg_reset_kernel<L>, grid, dim3(kBlock), 0, s, a);
  return check_launch("bg_reset_kernel");
}

template <int L>
int bg_launch_step2(dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk) {
  hipLaunchKernelGGL(bg2_step_kernel<L>, grid, dim3(kBlock), 0, s, a, wk);
  return check_launch("bg2_step_kernel");
}

// hipExtLaunchKernelGGL ties the optional events to this dispatch's own start/end
// timestamps (the numbers rocprofv3 reports), not to separate event packets.
template <int L, int DM>
int bg_launch_step_dm(dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk, hipEvent_t ev0, hipEvent_t ev1) {
  hipExtLaunchKernelGGL(HIP_KERNEL_NAME(bg_step_kernel<L, DM>), grid, dim3(kBlock), 0, s, ev0, ev1, 0, a.inv, a.bk, a.op,
                        a.act, a.ring, static_cast<uint32_t>(a.n), pack_week(wk), a, wk);
  return check_launch("bg_step_kernel");
}

template <int L>
int bg_launch_step(dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk, hipEvent_t ev0, hipEvent_t ev1) {
  switch (a.demand_mode) {
    case SCG_DEMAND_FIXED: return bg_launch_step_dm<L, SCG_DEMAND_FIXED>(grid, s, a, wk, ev0, ev1);
    case SCG_DEMAND_TABLE: return bg_launch_step_dm<L, SCG_DEMAND_TABLE>(grid, s, a, wk, ev0, ev1);
    case SCG_DEMAND_UNIFORM: return bg_launch_step_dm<L, SCG_DEMAND_UNIFORM>(grid, s, a, wk, ev0, ev1);
    default: return bg_launch_step_dm<L, SCG_DEMAND_POISSON>(grid, s, a, wk, ev0, ev1);
  }
}

template <int L>
int bg_launch_server(hipStream_t s, int demand_mode, scg_bg_server_box* box, uint32_t exit_seen, uint32_t idle_ticks) {
  switch (demand_mode) {
    case SCG_DEMAND_FIXED:
      hipLaunchKernelGGL(HIP_KERNEL_NAME(bg_server_kernel<L, SCG_DEMAND_FIXED>), dim3(1), dim3(kServerBlock), 0, s, box,
                         exit_seen, idle_ticks);
      break;
    case SCG_DEMAND_TABLE:
      hipLaunchKernelGGL(HIP_KERNEL_NAME(bg_server_kernel<L, SCG_DEMAND_TABLE>), dim3(1), dim3(kServerBlock), 0, s, box,
                         exit_seen, idle_ticks);
      break;
    case SCG_DEMAND_UNIFORM:
      hipLaunchKernelGGL(HIP_KERNEL_NAME(bg_server_kernel<L, SCG_DEMAND_UNIFORM>), dim3(1), dim3(kServerBlock), 0, s, box,
                         exit_seen, idle_ticks);
      break;
    default:
      hipLaunchKernelGGL(HIP_KERNEL_NAME(bg_server_kernel<L, SCG_DEMAND_POISSON>), dim3(1), dim3(kServerBlock), 0, s, box,
                         exit_seen, idle_ticks);
  }
  return check_launch("bg_server_kernel");
}

template <int L, int DM>
int bg_launch_slab_dm(dim3 grid, hipStream_t s, int32_t* slab, const int32_t* act, int32_t* out, uint32_t n32,
                      uint32_t wpack, uint32_t week, uint32_t episode, uint32_t k0, uint32_t k1, const BgSlabArgs& a,
                      hipEvent_t ev0, hipEvent_t ev1) {
  if (ev0 || ev1) {
    hipExtLaunchKernelGGL(HIP_KERNEL_NAME(bg_step_slab_kernel<L, DM>), grid, dim3(kBlock), 0, s, ev0, ev1, 0, slab, act,
                          out, n32, wpack, week, episode, k0, k1, a);
    return check_launch("bg_step_slab_kernel");
  }
  if (SCG_MODULE_LAUNCH) return launch_slab_module<L, DM>(grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(bg_step_slab_kernel<L, DM>), grid, dim3(kBlock), 0, s, slab, act, out, n32, wpack,
                     week, episode, k0, k1, a);
  return check_launch("bg_step_slab_kernel");
}

template <int L>
int bg_launch_slab(int demand_mode, dim3 grid, hipStream_t s, int32_t* slab, const int32_t* act, int32_t* out,
                   uint32_t n32, uint32_t wpack, uint32_t week, uint32_t episode, uint32_t k0, uint32_t k1,
                   const BgSlabArgs& a, hipEvent_t ev0, hipEvent_t ev1) {
  switch (demand_mode) {
    case SCG_DEMAND_FIXED:
      return bg_launch_slab_dm<L, SCG_DEMAND_FIXED>(grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a, ev0, ev1);
    case SCG_DEMAND_TABLE:
      return bg_launch_slab_dm<L, SCG_DEMAND_TABLE>(grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a, ev0, ev1);
    case SCG_DEMAND_UNIFORM:
      return bg_launch_slab_dm<L, SCG_DEMAND_UNIFORM>(grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a, ev0,
                                                      ev1);
    default:
      return bg_launch_slab_dm<L, SCG_DEMAND_POISSON>(grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a, ev0,
                                                      ev1);
  }
}

template <int L>
int bg_launch_rollout(dim3 grid, hipStream_t s, const BgArgs& a, int32_t K, const RolloutWeeks& weeks,
                      const int32_t* acts, int32_t* obs, int32_t* rew) {
  const size_t lds = static_cast<size_t>(a.ring_slots) * L * kBlock * sizeof(int32_t);
  if (lds <= 64 * 1024) {  // ring staged in LDS for the launch
    hipLaunchKernelGGL(bg_rollout_lds_kernel<L>, grid, dim3(kBlock), lds, s, a, K, weeks, acts, obs, rew);
    return check_launch("bg_rollout_lds_kernel");
  }
  hipLaunchKernelGGL(bg_rollout_kernel<L>, grid, dim3(kBlock), 0, s, a, K, weeks, acts, obs, rew);
  return check_launch("bg_rollout_kernel");
}

#define SCG_LEVEL_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

// Explicit instantiation (definition or, with `extern`, declaration) of level l's launchers.
#define SCG_BG_LAUNCHERS(EXT, l)                                                                                     \
  EXT template int bg_launch_reset<l>(dim3, hipStream_t, const BgArgs&);                                            \
  EXT template int bg_launch_step2<l>(dim3, hipStream_t, const BgArgs&, const WeekInfo&);                           \
  EXT template int bg_launch_step<l>(dim3, hipStream_t, const BgArgs&, const WeekInfo&, hipEvent_t, hipEvent_t);    \
  EXT template int bg_launch_server<l>(hipStream_t, int, scg_bg_server_box*, uint32_t, uint32_t);                   \
  EXT template int bg_launch_slab<l>(int, dim3, hipStream_t, int32_t*, const int32_t*, int32_t*, uint32_t, uint32_t, \
                                     uint32_t, uint32_t, uint32_t, uint32_t, const BgSlabArgs&, hipEvent_t,         \
                                     hipEvent_t);                                                                    \
  EXT template int bg_launch_rollout<l>(dim3, hipStream_t, const BgArgs&, int32_t, const RolloutWeeks&,             \
                                        const int32_t*, int32_t*, int32_t*);
#define SCG_BG_EXTERN_LEVEL(l) SCG_BG_LAUNCHERS(extern, l)
SCG_LEVEL_CASES(SCG_BG_EXTERN_LEVEL)
#undef SCG_BG_EXTERN_LEVEL

}  // namespace scg
