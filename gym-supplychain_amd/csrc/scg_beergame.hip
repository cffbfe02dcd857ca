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

#include <cstdarg>
#include <cstdio>
#include <ctime>
#include <vector>

#include "scg_beergame_kernels.h"

namespace scg {

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

// ---- host helpers: run-time dispatch on the level count ----------------------------------
int launch_reset(int L, dim3 grid, hipStream_t s, const BgArgs& a) {
  switch (L) {
#define X(l) case l: return bg_launch_reset<l>(grid, s, a);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

int launch_step2(int L, dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk) {
  switch (L) {
#define X(l) case l: return bg_launch_step2<l>(grid, s, a, wk);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

int launch_step(int L, dim3 grid, hipStream_t s, const BgArgs& a, const WeekInfo& wk, hipEvent_t ev0,
                hipEvent_t ev1) {
  switch (L) {
#define X(l) case l: return bg_launch_step<l>(grid, s, a, wk, ev0, ev1);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

int launch_server(int L, int demand_mode, hipStream_t s, scg_bg_server_box* box, uint32_t exit_seen,
                  uint32_t idle_ticks) {
  switch (L) {
#define X(l) case l: return bg_launch_server<l>(s, demand_mode, box, exit_seen, idle_ticks);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

int launch_slab(int demand_mode, int L, dim3 grid, hipStream_t s, int32_t* slab, const int32_t* act, int32_t* out,
                uint32_t n32, uint32_t wpack, uint32_t week, uint32_t episode, uint32_t k0, uint32_t k1,
                const BgSlabArgs& a, hipEvent_t ev0, hipEvent_t ev1) {
  switch (L) {
#define X(l) case l: return bg_launch_slab<l>(demand_mode, grid, s, slab, act, out, n32, wpack, week, episode, k0, k1, a, ev0, ev1);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

int launch_rollout(int L, dim3 grid, hipStream_t s, const BgArgs& a, int32_t K, const RolloutWeeks& weeks,
                   const int32_t* acts, int32_t* obs, int32_t* rew) {
  switch (L) {
#define X(l) case l: return bg_launch_rollout<l>(grid, s, a, K, weeks, acts, obs, rew);
    SCG_LEVEL_CASES(X)
#undef X
    default: return fail(SCG_ERR_INVALID, "levels=%d outside 1..%d", L, SCG_BG_MAX_LEVELS);
  }
}

// Word offsets of a state slab (scg_bg_slab_layout); the slab kernel derives the same ones
// from (N, L, R) and the wpack option bits.
int slab_layout(int L, int64_t N, int32_t R, int32_t T, bool history, int64_t* off) {
  const int64_t NL = N * L;
  if (NL % 4 != 0) return fail(SCG_ERR_INVALID, "slab layout needs n_envs * levels %% 4 == 0 (got %lld)", (long long)NL);
  if (R < 1 || R > 127) return fail(SCG_ERR_INVALID, "slab layout needs 1 <= ring_slots <= 127");
  off[SCG_SLAB_ERROR] = 0;
  for (int f = 0; f < 6; ++f) off[SCG_SLAB_INVENTORY + f] = kSlabHeader + f * NL;
  off[SCG_SLAB_RING] = kSlabHeader + 6 * NL;
  off[SCG_SLAB_EPISODE_RETURN] = kSlabHeader + (6 + R) * NL;
  off[SCG_SLAB_FINAL_RETURN] = off[SCG_SLAB_EPISODE_RETURN] + 2 * N;
  off[SCG_SLAB_HISTORY] = off[SCG_SLAB_FINAL_RETURN] + 2 * N;
  off[SCG_SLAB_TOTAL] = off[SCG_SLAB_HISTORY] + (history ? static_cast<int64_t>(T + 1) * NL : 0);
  return SCG_OK;
}

// The slab kernel runs when st->slab is set, its views are where the layout puts them and
// the rewards follow the observation rows in one allocation.
bool slab_ready(const scg_bg_config* cfg, const scg_bg_state* st, const int32_t* obs, const int32_t* reward,
                const int32_t* terminal_obs) {
  if (!st->slab || cfg->variant != 1) return false;
  int64_t off[SCG_SLAB_FIELDS];
  const bool hist = st->orders_history != nullptr;
  if (slab_layout(cfg->levels, st->n_envs, cfg->ring_slots, cfg->max_weeks, hist, off) != SCG_OK) return false;
  int32_t* b = st->slab;
  const bool ledgers = st->inventory_costs != nullptr, returns = st->episode_return != nullptr;
  return st->inventory == b + off[SCG_SLAB_INVENTORY] && st->backlog == b + off[SCG_SLAB_BACKLOG] &&
         st->orders_placed == b + off[SCG_SLAB_ORDERS] && st->shipments == b + off[SCG_SLAB_RING] &&
         (!ledgers || (st->inventory_costs == b + off[SCG_SLAB_INV_COSTS] &&
                       st->backlog_costs == b + off[SCG_SLAB_BACKLOG_COSTS])) &&
         ledgers == (st->backlog_costs != nullptr) &&
         (!returns || (reinterpret_cast<int32_t*>(st->episode_return) == b + off[SCG_SLAB_EPISODE_RETURN] &&
                       reinterpret_cast<int32_t*>(st->final_return) == b + off[SCG_SLAB_FINAL_RETURN])) &&
         (!hist || st->orders_history == b + off[SCG_SLAB_HISTORY]) &&
         st->error_flags == b + off[SCG_SLAB_ERROR] && reward == obs + st->n_envs * cfg->levels &&
         (!terminal_obs || terminal_obs == b + off[SCG_SLAB_TERMINAL_OBS]);
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

// Weeks 1..init_slots hold the initial pipeline (beergame_env.py:52); the ring keeps those
// within the horizon, a full table all of them.
inline int32_t init_slots(const scg_bg_config* cfg) {
  const int32_t d0 = cfg->shipment_delays ? cfg->shipment_delays[0] : 0;
  return cfg->full_table ? d0 : std::min(d0, cfg->max_weeks);
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
  a.init_slots = init_slots(cfg);
  a.ring_slots = cfg->ring_slots;
  for (int l = 0; l < cfg->levels; ++l) a.init_inv[l] = cfg->initial_inventory[l];
  a.demand_lo = cfg->demand_lo;
  a.demand_hi = cfg->demand_hi;
  a.max_weeks = cfg->max_weeks;
  a.err = st->error_flags;
  a.guard = week_guard(cfg->levels, cfg->inv_cost, cfg->backlog_cost);
  a.err_host = st->error_host;
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
  const bool full = cfg->full_table != 0;
  if (full) {  // the reference's table: rows max(T+1, max_w(w+d_w+1)) + 1 (:46-50), slot s = week s
    if (cfg->variant != 1) return fail(SCG_ERR_INVALID, "full_table is a BeerGameEnv (variant 1) option");
    int32_t last = T + 1;
    for (int32_t w = 0; w <= T; ++w) last = std::max(last, w + cfg->shipment_delays[w] + 1);
    R = last + 1;  // <= T + SCG_BG_MAX_DELAY + 2: fits pack_week's slot fields
  }
  // Which arrival weeks have been written, in week order (writes only target later weeks).
  // (a full table also keeps the rows past T: week T + 1 + max delay at most)
  std::vector<uint8_t> written(static_cast<size_t>(T) + SCG_BG_MAX_DELAY + 2, 0);
  for (int32_t t = 1; t <= init_slots(cfg); ++t) written[t] = 1;  // initial pipeline (:52)
  cfg->plan[0] = 0;
  for (int32_t w = 1; w <= T; ++w) {
    const int32_t d = cfg->shipment_delays[w];
    int32_t mode;
    if (d == 0) {
      mode = MODE_DIRECT;                 // :93-94, :111-112
    } else if (w + d > T && !full) {
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

int scg_bg_slab_layout(const scg_bg_config* cfg, int64_t n_envs, int32_t with_history,
                       int64_t offsets[SCG_SLAB_FIELDS]) {
  if (!cfg || !offsets) return fail(SCG_ERR_INVALID, "null config/offsets");
  if (cfg->ring_slots <= 0) return fail(SCG_ERR_INVALID, "config not prepared (call scg_bg_prepare)");
  if (n_envs <= 0 || n_envs > INT32_MAX) return fail(SCG_ERR_INVALID, "n_envs must be in 1..%d", INT32_MAX);
  return slab_layout(cfg->levels, n_envs, cfg->ring_slots, cfg->max_weeks, with_history != 0, offsets);
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
  if (slab_ready(cfg, st, obs, reward, terminal_obs)) {
    BgSlabArgs sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.pthr = cfg->poisson_thresholds;
    sa.demand_table = cfg->demand_table;
    sa.pthr_len = cfg->poisson_len;
    sa.h = cfg->inv_cost;
    sa.b = cfg->backlog_cost;
    sa.demand_fixed = wk.demand_fixed;
    sa.demand_lo = cfg->demand_lo;
    sa.demand_hi = cfg->demand_hi;
    sa.ship_value = cfg->initial_shipment_value;
    sa.orders_value = cfg->initial_orders_value;
    sa.init_slots = init_slots(cfg);
    sa.env_offset = st->env_offset;
    sa.guard = week_guard(cfg->levels, cfg->inv_cost, cfg->backlog_cost);
    sa.err_host = st->error_host;
    for (int l = 0; l < cfg->levels; ++l) sa.init_inv[l] = cfg->initial_inventory[l];
    uint32_t wpack = pack_week_slab(wk);  // R <= 127 (slab_layout)
    wpack |= (wk.flags & 1) ? SW_TERMINAL : 0u;
    wpack |= (wk.flags & 2) ? SW_AUTORESET : 0u;
    wpack |= st->inventory_costs ? SW_LEDGERS : 0u;
    wpack |= st->episode_return ? SW_RETURNS : 0u;
    wpack |= st->orders_history ? SW_HISTORY : 0u;
    wpack |= static_cast<uint32_t>(cfg->ring_slots) << 24;
    if (int rc = launch_slab(cfg->demand_mode, cfg->levels, grid_for(st->n_envs), static_cast<hipStream_t>(stream),
                             st->slab, action, obs, static_cast<uint32_t>(st->n_envs), wpack, static_cast<uint32_t>(w),
                             st->episode, static_cast<uint32_t>(st->seed & 0xffffffffu),
                             static_cast<uint32_t>(st->seed >> 32), sa, static_cast<hipEvent_t>(start_event),
                             static_cast<hipEvent_t>(stop_event)))
      return rc;
    if (wk.flags & 2) {
      st->week = 0;
      st->episode += 1;
    } else {
      st->week = w;
    }
    if (done) *done = (wk.flags & 1) ? 1 : 0;
    return SCG_OK;
  }
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

// ---- step server (include/scgpu.h: scg_bg_server_*) -------------------------------------
// the layouts the Python binding (_native.py) mirrors
static_assert(sizeof(scg_bg_server_line) == 64, "request line");
static_assert(sizeof(scg_bg_server_box) == 17 * 64 + 64 + SCG_BG_SERVER_SLOTS * SCG_BG_SERVER_ARGS_BYTES, "mailbox");
static_assert(offsetof(scg_bg_server_box, done_seq) == 16 * 64 && offsetof(scg_bg_server_box, args) == 18 * 64,
              "mailbox lines");
static_assert(sizeof(scg_bg_server) == 72 && sizeof(scg_bg_server_slot) == 64, "server structs");
// The server's host bookkeeping (launch, retire, slots, argument blocks) under a spin lock in
// the struct itself: posts and waits of different slots may come from different threads.
struct ServerLock {
  int32_t* w;
  explicit ServerLock(scg_bg_server* sv) : w(&sv->lock) {
    for (;;) {
      int32_t z = 0;
      if (__atomic_compare_exchange_n(w, &z, 1, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED)) return;
      cpu_relax();
    }
  }
  ~ServerLock() { __atomic_store_n(w, 0, __ATOMIC_RELEASE); }
};

static bool server_ok(const scg_bg_server* sv) { return sv && sv->box_host && sv->box_dev; }

// Launch the wave (lock held). It serves, first, every slot whose request is newer than its answer.
static int server_launch_locked(scg_bg_server* sv) {
  const uint32_t exit_seen = __atomic_load_n(&sv->box_host->exit_req, __ATOMIC_ACQUIRE);
  const uint32_t idle_ticks = static_cast<uint32_t>(sv->idle_us) * 100u;  // 100 MHz real-time clock
  if (int rc = launch_server(sv->levels, sv->demand_mode, static_cast<hipStream_t>(sv->stream), sv->box_dev,
                             exit_seen, idle_ticks))
    return rc;
  sv->running = 1;
  sv->launches += 1;
  sv->last_ns = mono_ns();
  return SCG_OK;
}

static int server_stop_locked(scg_bg_server* sv) {
  if (!sv->running) return SCG_OK;
  __atomic_store_n(&sv->box_host->exit_req, sv->box_host->exit_req + 1, __ATOMIC_RELEASE);
  sv->running = 0;
  if (hipStreamSynchronize(static_cast<hipStream_t>(sv->stream)) != hipSuccess)
    return fail(SCG_ERR_HIP, "step server: hipStreamSynchronize failed");
  return SCG_OK;
}

int scg_bg_server_stop(scg_bg_server* sv) {
  if (!server_ok(sv)) return fail(SCG_ERR_INVALID, "null server/mailbox");
  ServerLock lk(sv);
  return server_stop_locked(sv);
}

uint32_t scg_bg_server_line_check(const scg_bg_server_line* line) {
  uint32_t w[16];
  std::memcpy(w, line, sizeof(w));
  return server_line_check(w);
}

int scg_bg_server_attach(scg_bg_server* sv, scg_bg_server_slot* slot) {
  if (!server_ok(sv) || !slot) return fail(SCG_ERR_INVALID, "null server/mailbox/slot");
  if (!slot->action || !slot->obs || !slot->reward) return fail(SCG_ERR_INVALID, "step server: slot action, obs and reward are required");
  if (!sv->stream) return fail(SCG_ERR_INVALID, "step server: needs a (non-blocking) stream of its own, not the null stream");
  if (sv->levels < 1 || sv->levels > SCG_BG_MAX_LEVELS) return fail(SCG_ERR_INVALID, "step server: levels=%d", sv->levels);
  if (sv->demand_mode < SCG_DEMAND_FIXED || sv->demand_mode > SCG_DEMAND_UNIFORM)
    return fail(SCG_ERR_INVALID, "step server: unknown demand_mode %d", sv->demand_mode);
  if (sv->idle_us < 100 || sv->idle_us > 10000000) return fail(SCG_ERR_INVALID, "idle_us outside 100..10^7");
  ServerLock lk(sv);
  int k = 0;
  while (k < kServerSlots && (sv->slots_used >> k & 1u)) ++k;
  if (k == kServerSlots) return fail(SCG_ERR_INVALID, "step server: all %d slots are taken", kServerSlots);
  scg_bg_server_box* b = sv->box_host;
  sv->slots_used |= 1u << k;
  slot->server = sv;
  slot->index = k;
  // a slot taken again continues its line's numbering; its arguments are published on the
  // first post (cleared here, they differ from any real ones: a new generation)
  slot->seq = __atomic_load_n(&b->req[k].req_seq, __ATOMIC_RELAXED);
  slot->gen = b->req[k].gen;
  std::memset(b->args[k], 0, sizeof(b->args[k]));
  slot->week = 0;
  slot->done = 0;
  slot->relaunches = 0;
  __atomic_store_n(&b->done_seq[k], slot->seq, __ATOMIC_RELEASE);
  uint32_t ns = 0;
  for (int j = 0; j < kServerSlots; ++j)
    if (sv->slots_used >> j & 1u) ns = j + 1;
  __atomic_store_n(&b->n_slots, ns, __ATOMIC_RELEASE);
  return SCG_OK;
}

int scg_bg_server_detach(scg_bg_server_slot* slot) {
  if (!slot || !server_ok(slot->server)) return fail(SCG_ERR_INVALID, "null slot or server");
  scg_bg_server* sv = slot->server;
  if (slot->index < 0) return SCG_OK;
  scg_bg_server_box* b = sv->box_host;
  const int k = slot->index;
  if (__atomic_load_n(&b->done_seq[k], __ATOMIC_ACQUIRE) != slot->seq)
    return fail(SCG_ERR_INVALID, "step server: detach with a request of slot %d unanswered", k);
  ServerLock lk(sv);
  sv->slots_used &= ~(1u << k);
  uint32_t ns = 0;
  for (int j = 0; j < kServerSlots; ++j)
    if (sv->slots_used >> j & 1u) ns = j + 1;
  __atomic_store_n(&b->n_slots, ns, __ATOMIC_RELEASE);
  slot->index = -1;
  return SCG_OK;
}

int scg_bg_server_post(const scg_bg_config* cfg, scg_bg_state* st, scg_bg_server_slot* slot) {
  if (int rc = check_state(cfg, st)) return rc;
  if (!slot || !server_ok(slot->server) || slot->index < 0 || slot->index >= kServerSlots)
    return fail(SCG_ERR_INVALID, "step server: the slot is not attached");
  scg_bg_server* sv = slot->server;
  if (st->n_envs > kServerBlock) return fail(SCG_ERR_INVALID, "the step server runs up to %d envs per slot", kServerBlock);
  if (cfg->variant != 1) return fail(SCG_ERR_INVALID, "the step server runs BeerGameEnv (variant 1)");
  if (st->slab) return fail(SCG_ERR_INVALID, "the step server runs on separate state buffers (no slab)");
  if (cfg->levels != sv->levels || cfg->demand_mode != sv->demand_mode)
    return fail(SCG_ERR_INVALID, "step server: the config (levels %d, demand mode %d) is not the server's (%d, %d)",
                cfg->levels, cfg->demand_mode, sv->levels, sv->demand_mode);
  if (int rc = check_step(cfg, st)) return rc;
  scg_bg_server_box* b = sv->box_host;
  const int k = slot->index;
  if (__atomic_load_n(&b->done_seq[k], __ATOMIC_ACQUIRE) != slot->seq)
    return fail(SCG_ERR_INVALID, "step server: slot %d posts while its last request is unanswered", k);
  const int32_t w = st->week + 1;
  const WeekInfo wk = week_info(cfg, w, 0);
  BgArgs a = make_args(cfg, st);
  a.act = slot->action;
  a.obs = slot->obs;
  a.rew = slot->reward;
  a.term_obs = nullptr;
  ServerLock lk(sv);
  // the slot's arguments: a new generation whenever they differ from the published ones (the
  // wave reloads them only then; nothing of the slot is in flight, so rewriting is safe)
  if (std::memcmp(b->args[k], &a, sizeof(a)) != 0) {
    std::memcpy(b->args[k], &a, sizeof(a));
    slot->gen = slot->gen + 1 ? slot->gen + 1 : 1;  // 0 is the wave's "none loaded"
  }
  // a wave idle for more than half its time-out may be exiting: retire it before posting
  if (sv->running && mono_ns() - sv->last_ns > static_cast<int64_t>(sv->idle_us) * 500)
    if (int rc = server_stop_locked(sv)) return rc;
  uint32_t line[16] = {0};
  const uint32_t seq = slot->seq + 1;
  const int32_t n_inline = (slot->action_host && st->n_envs == 1 && cfg->levels <= 8) ? cfg->levels : 0;
  line[0] = seq;
  line[2] = pack_week(wk);
  line[3] = static_cast<uint32_t>(w);
  line[4] = static_cast<uint32_t>(wk.demand_fixed);
  line[5] = static_cast<uint32_t>(n_inline);
  line[6] = slot->gen;
  for (int l = 0; l < n_inline; ++l) line[8 + l] = static_cast<uint32_t>(slot->action_host[l]);
  line[7] = server_line_check(line);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&b->req[k]);
  for (int i = 1; i < 16; ++i) __atomic_store_n(&dst[i], line[i], __ATOMIC_RELAXED);
  __atomic_store_n(&dst[0], seq, __ATOMIC_RELEASE);
  slot->seq = seq;
  slot->week = w;
  slot->done = (wk.flags & 1) ? 1 : 0;
  sv->last_ns = mono_ns();
  if (!sv->running)
    if (int rc = server_launch_locked(sv)) return rc;
  return SCG_OK;
}

int scg_bg_server_wait(scg_bg_state* st, scg_bg_server_slot* slot, int64_t spin_us, int32_t* done) {
  if (!st || !slot || !server_ok(slot->server) || slot->index < 0 || slot->index >= kServerSlots)
    return fail(SCG_ERR_INVALID, "step server: the slot is not attached");
  scg_bg_server* sv = slot->server;
  scg_bg_server_box* b = sv->box_host;
  const int k = slot->index;
  const uint32_t seq = slot->seq;
  const int64_t start = mono_ns();
  const int64_t check_ns = (sv->check_us > 0 ? sv->check_us : 2000000) * int64_t(1000);
  int64_t check = start + check_ns;
  int gone = 0;
  for (uint32_t spins = 0;; ++spins) {
    if (__atomic_load_n(&b->done_seq[k], __ATOMIC_ACQUIRE) == seq) break;
    cpu_relax();
    if ((spins & 255u) != 255u) continue;
    const int64_t now = mono_ns();
    if (spin_us >= 0 && now - start > spin_us * 1000) return SCG_PENDING;
    if (now < check) continue;
    check = now + check_ns;
    // Every check interval: a wave that has exited without serving the request (its stream
    // idle: a host stall past its time-out, an exit another thread asked for) is launched
    // again — it serves pending requests first — once per wait; a HIP error on the stream
    // fails at once; a wave still queued or running is waited for, up to 60 s in all.
    ServerLock lk(sv);
    const hipError_t q = hipStreamQuery(static_cast<hipStream_t>(sv->stream));
    if (q != hipSuccess && q != hipErrorNotReady)
      return fail(SCG_ERR_HIP, "step server: the wave's stream reports %s (week %d)", hipGetErrorString(q), slot->week);
    if (__atomic_load_n(&b->done_seq[k], __ATOMIC_ACQUIRE) == seq) break;
    if (q == hipSuccess) {
      if (gone++ > 0) return fail(SCG_ERR_HIP, "step server: the wave exits without answering (week %d)", slot->week);
      sv->running = 0;
      slot->relaunches += 1;
      if (int rc = server_launch_locked(sv)) return rc;
    }
    if (now - start > 60000000000LL) return fail(SCG_ERR_HIP, "step server: no answer for 60 s (week %d)", slot->week);
  }
  sv->last_ns = mono_ns();
  st->week = slot->week;  // no auto-reset on this path
  if (done) *done = slot->done;
  return SCG_OK;
}

int scg_bg_server_step(const scg_bg_config* cfg, scg_bg_state* st, scg_bg_server_slot* slot, int32_t* done) {
  if (int rc = scg_bg_server_post(cfg, st, slot)) return rc;
  return scg_bg_server_wait(st, slot, -1, done);
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
  // The Philox env counter is 32-bit: global env ids past 2^32 would reuse another env's draws.
  if (env_offset < 0 || env_offset + n_envs > (int64_t(1) << 32))
    return fail(SCG_ERR_INVALID, "uniform_ints env ids must lie in [0, 2^32)");
  if (static_cast<int64_t>(rows) * width > INT32_MAX)
    return fail(SCG_ERR_INVALID, "uniform_ints rows * width must fit int32");
  const uint32_t range = static_cast<uint32_t>(static_cast<int64_t>(hi) - lo + 1);  // 0 means 2^32
  if (range == 0) return fail(SCG_ERR_INVALID, "uniform_ints range must be < 2^32");
  hipLaunchKernelGGL(uniform_ints_kernel, grid_for(n_envs), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     static_cast<uint32_t>(seed & 0xffffffffu), static_cast<uint32_t>(seed >> 32), env_offset, n_envs,
                     rows, width, tag, lo, range, out);
  return check_launch("uniform_ints_kernel");
}

}  // extern "C"
