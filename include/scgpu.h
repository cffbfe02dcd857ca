/*
 * scgpu — MI355X-native (gfx950) vectorised supply-chain environments: C ABI.
 *
 * This is the drop-in boundary for the hot path of caburu/gym-supplychain
 * (reference snapshot 2024-08-07, mounted at /root/reference): the per-env
 * step()/reset() dynamics of BeerGameEnv, run as fused HIP kernels over a batch of
 * N envs held in caller-owned device buffers.
 *
 * The reference is pure Python; its "interface" for this path is the gym.Env
 * surface of BeerGameEnv (gym_supplychain/envs/beergame_env.py):
 *     __init__(env_init_info)  beergame_env.py:11-60   -> scg_bg_config + scg_bg_prepare
 *     reset()                  beergame_env.py:140-156 -> scg_bg_reset
 *     step(action)             beergame_env.py:66-138  -> scg_bg_step / scg_bg_rollout
 *     _observation()           beergame_env.py:180-181 -> fused into the step epilogue
 * The Python package gym_supplychain_amd binds these entry points with ctypes
 *  and re-exposes the reference's class names and gym API.
 *
 * Conventions
 *   - Every function returns an int status (scg_status). Nothing throws across the ABI.
 *     On failure scg_last_error() describes the problem (thread-local).
 *   - The library never allocates device memory and never synchronises: all buffers
 *     are owned by the caller, every launch is asynchronous on the caller's stream
 *     (`stream` is a hipStream_t passed as void*; NULL = the null stream).
 *   - Integer state is int32; the reference's int64 values are reproduced exactly while
 *     every value stays within int32 range (DESIGN.md "Integer range").
 *   - Layouts are env-major: a [N][L] int32 array holds env n's L levels contiguously.
 */
#ifndef SCGPU_H
#define SCGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5 (round 4): scg_sc_state.inbox_tk is uint8 [inbox_size][N] (byte-packed entries);
 *   shipment delays up to SCG_BG_MAX_DELAY = 4096; full_table of any row count.
 * 6 (round 5): the BeerGame step server (scg_bg_server_box, scg_bg_server, scg_bg_server_step,
 *   scg_bg_server_stop) and the testing hook scg_sc_nodes_max_blocks.
 * 7 (round 6): the step server serves up to SCG_BG_SERVER_SLOTS envs from one wave
 *   (scg_bg_server_slot, attach / detach / post / wait), mixing-hash check word; the
 *   SupplyChain step server (scg_sc_server_box, scg_sc_server, scg_sc_server_*). */
#define SCG_ABI_VERSION 7

#if defined(__GNUC__)
#define SCG_API __attribute__((visibility("default")))
#else
#define SCG_API
#endif

#define SCG_BG_MAX_LEVELS 16   /* template instantiations of the step kernel        */
#define SCG_BG_MAX_WEEKS 4096  /* episode horizon (len(customer_demand), :37)        */
#define SCG_BG_MAX_DELAY 4096  /* shipment delay bound: ring slots R = max delay + 1 */
#define SCG_POISSON_MAX 256    /* CDF threshold table entries                        */
#define SCG_BG_ROLLOUT_MAX 128 /* weeks per rollout launch (host loops beyond)       */

typedef enum scg_status {
  SCG_OK = 0,
  SCG_ERR_INVALID = 1,      /* bad argument or config              -> ValueError    */
  SCG_ERR_PAST_HORIZON = 2, /* step after the terminal week        -> IndexError    */
                            /* (the reference raises IndexError on customer_demand[T], :79) */
  SCG_ERR_NOT_RESET = 3,    /* step before reset                   -> RuntimeError  */
  SCG_ERR_HIP = 4           /* HIP launch/runtime error            -> RuntimeError  */
} scg_status;

typedef enum scg_demand_mode {
  SCG_DEMAND_FIXED = 0,   /* one list shared by all envs: customer_demand (beergame_env.py:33) */
  SCG_DEMAND_TABLE = 1,   /* per-env device table int32 [T][N] (caller-drawn demand)            */
  SCG_DEMAND_POISSON = 2, /* per-(env, episode, week) Poisson draw on device, Philox4x32-10     */
  SCG_DEMAND_UNIFORM = 3  /* per-(env, episode, week) randint(demand_lo, demand_hi), Philox     */
} scg_demand_mode;

/* Step flags */
#define SCG_BG_AUTORESET 1u /* at the terminal week reset in the same launch (VecEnv semantics) */
#define SCG_SC_SERIAL 2u    /* node-parallel SupplyChain kernel: step every env with its serial
                               walk (the path of envs whose receive order it cannot prove; tests) */

/* Philox streams (counter word 3) */
#define SCG_STREAM_DEMAND 0u
#define SCG_STREAM_ACTION 1u
#define SCG_STREAM_BG2_DEMAND 4u
#define SCG_STREAM_BG2_DELAY 5u

/*
 * Env configuration, the resolved form of BeerGameEnv's env_init_info
 * (beergame_env.py:16-58). Host memory, owned by the caller.
 */
typedef struct scg_bg_config {
  int32_t levels;                 /* L, :26                                            */
  int32_t max_weeks;              /* T = len(customer_demand), :37                     */
  int32_t inv_cost;               /* :28                                               */
  int32_t backlog_cost;           /* :30                                               */
  int32_t initial_shipment_value; /* :41                                               */
  int32_t initial_orders_value;   /* :43                                               */
  int32_t initial_inventory[SCG_BG_MAX_LEVELS]; /* :35                                 */
  int32_t demand_mode;            /* scg_demand_mode                                   */
  int32_t poisson_len;            /* entries in poisson_thresholds (POISSON mode)      */
  const int32_t* shipment_delays; /* HOST [T+1]: [2] + user list, exactly :39          */
  const int32_t* customer_demand; /* HOST [T]: FIXED mode demand, :33                  */
  const int32_t* demand_table;    /* DEVICE [T][N]: TABLE mode demand                   */
  const uint32_t* poisson_thresholds; /* DEVICE [poisson_len] (scg_poisson_table)       */
  int32_t* plan;                  /* HOST [T+1] workspace, filled by scg_bg_prepare     */
  int32_t ring_slots;             /* out of scg_bg_prepare: R = max delay + 1           */
  /* BeerGameEnv2 (beergame2_env.py:5-211) when variant == 2 ----------------------------- */
  int32_t variant;                /* 1: BeerGameEnv, 2: BeerGameEnv2                    */
  int32_t max_stock;              /* v2: observation offset and capacity (:24, :112)    */
  int32_t exceeded_capacity_penalty; /* v2: per unit beyond max_stock (:35, :179-180)  */
  int32_t demand_lo, demand_hi;   /* SCG_DEMAND_UNIFORM: randint(lo, hi) per week (:77) */
  int32_t stochastic_delays;      /* v2: per-episode randint(delay_lo, delay_hi) (:91)  */
  int32_t delay_lo, delay_hi;
  /* In (BeerGameEnv only): 1 = keep the reference's whole absolute-week shipment table
   * instead of the ring — ring_slots becomes its row count max(T+1, max_w(w+d_w+1)) + 1
   * (beergame_env.py:46-50), slot s holds week s, and shipments that land after the
   * horizon are stored as the reference stores them. Rows are not cleared between
   * episodes: a row not yet scheduled in the current episode holds a stale value (the
   * reference's is 0; scg_bg_prepare's plan says which rows are scheduled by each week).
   * Any row count (T + max delay + 2 at most); the state slab, and so the slab step kernel,
   * takes ring_slots <= 127, a longer table separate buffers and the general step kernel. */
  int32_t full_table;
} scg_bg_config;

/*
 * Batch state: caller-owned device buffers plus host-side counters the library
 * advances. Optional buffers may be NULL (then that output is not produced).
 */
typedef struct scg_bg_state {
  int64_t n_envs;           /* N envs in this shard                                   */
  int64_t env_offset;       /* global id of env 0 of this shard (multi-GPU sharding)   */
  uint64_t seed;            /* Philox key                                             */
  uint32_t episode;         /* episode counter (Philox); advanced by reset/auto-reset  */
  int32_t week;             /* 0 after reset, T at the terminal week; -1 = not reset   */
  int32_t* inventory;       /* [N][L]  self.inventory      :72,:101                    */
  int32_t* backlog;         /* [N][L]  self.backlog        :103                        */
  int32_t* orders_placed;   /* [N][L]  self.orders_placed  :121                        */
  int32_t* shipments;       /* [R][N][L] ring over absolute weeks (self.shipments :50)  */
  int32_t* inventory_costs; /* [N][L]  self.inventory_costs :131   (optional)           */
  int32_t* backlog_costs;   /* [N][L]  self.backlog_costs   :132   (optional)           */
  int32_t* orders_history;  /* [T+1][N][L] self.all_orders_placed :123 (optional)       */
  int64_t* episode_return;  /* [N] running sum of rewards (optional)                   */
  int64_t* final_return;    /* [N] episode_return at the terminal week (optional)      */
  int32_t* penalty_costs;   /* [N][L]  v2 self.penalty_costs :184 (optional)           */
  /* Sticky DEVICE int32 error word (optional): bit 0 is set by any kernel whose int64
   * result (state, pipeline row, ledger, observation or reward; the reference computes in
   * int64, beergame_env.py:33,35,130-132) does not fit the int32 it is stored in. The
   * stored values are then invalid; the flag stays set (across auto-resets too) until
   * scg_bg_reset, whose kernel clears it and error_host in stream order, or the caller. */
  int32_t* error_flags;
  /* Optional HOST-mapped int32 (pinned, device-accessible): every terminal-week launch copies
   * error_flags there as the launch starts, so a host can poll earlier episodes' overflow
   * without synchronising (read it after a later episode's terminal step has completed). */
  int32_t* error_host;
  /* Optional state slab (scg_bg_slab_layout): when non-NULL, every buffer above must be
   * the slab view the layout names, and scg_bg_step launches the slab step kernel, which
   * addresses every row from this one base. */
  int32_t* slab;
} scg_bg_state;

/* Slab fields, in order: word offsets filled by scg_bg_slab_layout. */
enum scg_bg_slab_field {
  SCG_SLAB_ERROR = 0,     /* int32 error word (16-byte header)              */
  SCG_SLAB_INVENTORY,     /* [N][L]                                          */
  SCG_SLAB_BACKLOG,       /* [N][L]                                          */
  SCG_SLAB_ORDERS,        /* [N][L]                                          */
  SCG_SLAB_INV_COSTS,     /* [N][L]                                          */
  SCG_SLAB_BACKLOG_COSTS, /* [N][L]                                          */
  SCG_SLAB_TERMINAL_OBS,  /* [N][L]                                          */
  SCG_SLAB_RING,          /* [R][N][L]                                       */
  SCG_SLAB_EPISODE_RETURN,/* int64 [N] (word offset, 8-byte aligned)         */
  SCG_SLAB_FINAL_RETURN,  /* int64 [N]                                       */
  SCG_SLAB_HISTORY,       /* [T+1][N][L] when requested, else == total       */
  SCG_SLAB_TOTAL,         /* words in the slab                               */
  SCG_SLAB_FIELDS
};

/*
 * STREAM copy of `bytes` (a multiple of 16, 16-byte aligned DEVICE buffers): the
 * achievable-HBM-bandwidth probe bench.py reports beside the 8 TB/s spec
 * (roofline.measured_peak). blocks == 0: one 16-byte vector per lane, the grid covering the
 * buffer (the fastest shape measured); blocks > 0: a grid-stride loop over that many
 * workgroups of 256 lanes. Not part of the env path.
 */
SCG_API int scg_stream_copy(const void* src, void* dst, int64_t bytes, int32_t blocks, void* stream);

/* ABI version (SCG_ABI_VERSION of the built library). */
SCG_API int scg_abi_version(void);

/* sizeof(scg_bg_config) and sizeof(scg_bg_state) as compiled, to check FFI bindings. */
SCG_API int scg_bg_struct_sizes(size_t* config_size, size_t* state_size);

/* Last error message of the calling thread ("" if none). */
SCG_API const char* scg_last_error(void);

/*
 * Poisson(lam) inverse-CDF table: out[k] = min(floor(CDF(k) * 2^32), 2^32-1) for
 * k = 0..len-1, ending at the first saturated entry. Returns len (>0) or -SCG_ERR_INVALID.
 * Host function; the caller uploads the table for SCG_DEMAND_POISSON.
 */
SCG_API int scg_poisson_table(double lam, uint32_t* out, int32_t cap);

/*
 * Validate cfg and fill cfg->plan / cfg->ring_slots from cfg->shipment_delays
 * (replaces the shipment-table sizing of beergame_env.py:46-52). Host only.
 */
SCG_API int scg_bg_prepare(scg_bg_config* cfg);

/*
 * Word offsets of one state slab for n_envs envs of a prepared cfg (ring_slots known),
 * with the order history when with_history != 0. Host only; the caller allocates
 * offsets[SCG_SLAB_TOTAL] int32 words of DEVICE memory (16-byte aligned, zeroed), points
 * the scg_bg_state buffers at base + offsets[field] and sets st->slab = base.
 */
SCG_API int scg_bg_slab_layout(const scg_bg_config* cfg, int64_t n_envs, int32_t with_history,
                               int64_t offsets[SCG_SLAB_FIELDS]);

/* reset() for all N envs (beergame_env.py:140-156). obs: DEVICE int32 [N][L] or NULL. */
SCG_API int scg_bg_reset(const scg_bg_config* cfg, scg_bg_state* st, int32_t* obs, void* stream);

/*
 * step(action) for all N envs (beergame_env.py:66-138), one fused kernel.
 *   action       DEVICE int32 [N][L]
 *   obs          DEVICE int32 [N][L]   inventory - backlog (:127,:180); with
 *                SCG_BG_AUTORESET at the terminal week: the reset observation
 *   reward       DEVICE int32 [N]      -sum(inv_cost*inv + backlog_cost*backlog) (:130)
 *   terminal_obs DEVICE int32 [N][L] or NULL: observation at the terminal week
 * Returns SCG_ERR_PAST_HORIZON when called after the terminal week without auto-reset.
 * Sets *done (host, may be NULL) to 1 when this step was the terminal week (:134).
 * With st->slab set, reward == obs + N*L (one output allocation) and terminal_obs NULL or the
 * slab's SCG_SLAB_TERMINAL_OBS view, the slab kernel runs (terminal obs into the slab).
 */
SCG_API int scg_bg_step(const scg_bg_config* cfg, scg_bg_state* st, const int32_t* action,
                int32_t* obs, int32_t* reward, int32_t* terminal_obs, uint32_t flags,
                int32_t* done, void* stream);

/*
 * scg_bg_step with the step kernel's own dispatch timestamps recorded into two
 * caller-created hipEvent_t (passed as void*, either may be NULL), via
 * hipExtLaunchKernel: hipEventElapsedTime(start, stop) is the kernel's duration as
 * rocprofv3 reports it. Used by bench.py for the roofline's measured kernel time.
 */
SCG_API int scg_bg_step_timed(const scg_bg_config* cfg, scg_bg_state* st, const int32_t* action,
                              int32_t* obs, int32_t* reward, int32_t* terminal_obs, uint32_t flags,
                              int32_t* done, void* start_event, void* stop_event, void* stream);

/*
 * Step server for drop-in envs stepped one week per host call (BeerGameEnv:
 * beergame_env.py:66-138 is one Python call per week). A launch plus a stream
 * synchronisation per week costs more than the reference's whole step, so instead one wave
 * stays resident per server: it polls a mailbox in host-mapped memory and runs the week body
 * of bg_step_kernel (the same code) on the state of whichever env posted a week. One server
 * serves up to SCG_BG_SERVER_SLOTS envs (a slot each: its request line, its answer word and
 * its kernel arguments), so a process that steps many drop-in envs in turn (a DummyVecEnv)
 * keeps ONE resident wave and one stream per device, not one per env. Every slot's config
 * must have the server's levels and demand mode; up to 64 envs per slot; variant 1, separate
 * state buffers (no slab), no auto-reset.
 *
 * The wave exits on scg_bg_server_stop, or by itself after idle_us without a request on any
 * slot, so it never outlives its process; scg_bg_server_post (re)launches it when it is not
 * running or may have timed out (idle for more than idle_us / 2 on the host's clock). When it
 * starts, every slot whose request is newer than its answer is served. Work the caller
 * launches on an env's state (reset, other steps) must be complete before that env's next
 * post, and must not start while one of its posts is unanswered; the mailbox must outlive
 * the wave. post/wait/step of different slots may run on different host threads.
 */
#define SCG_BG_SERVER_SLOTS 15
#define SCG_BG_SERVER_ARGS_BYTES 512
#define SCG_PENDING 5 /* scg_bg_server_wait: not answered within spin_us (not an error) */

typedef struct scg_bg_server_line { /* one 64-byte request line, read by the wave in one load */
  uint32_t req_seq;      /* request number (a new number is a new request)                      */
  int32_t cmd;           /* 0: step                                                            */
  uint32_t wpack;        /* the week's plan, as bg_step_kernel's packed word                   */
  int32_t week;          /* the week being stepped (1..max_weeks)                              */
  int32_t demand_fixed;  /* customer_demand[week - 1] for SCG_DEMAND_FIXED                     */
  int32_t n_inline;      /* L when env 0's action row travels in action[] (one env, L <= 8)    */
  uint32_t gen;          /* generation of the slot's kernel arguments (args[slot] below)       */
  uint32_t check;        /* scg mixing hash of the line's other 15 words: a read of the line
                            that mixes two requests is read again                            */
  int32_t action[8];
} scg_bg_server_line;

typedef struct scg_bg_server_box { /* host-mapped (hipHostMalloc mapped + coherent) */
  scg_bg_server_line req[SCG_BG_SERVER_SLOTS + 1]; /* slot k's request line is req[k]       */
  uint32_t done_seq[16];  /* slot k's last request served (written by the wave)             */
  uint32_t n_slots;       /* the wave polls slots 0 .. n_slots - 1                          */
  uint32_t exit_req;      /* the wave exits when this differs from its launch value         */
  uint32_t exit_seq;      /* written by the wave as it exits: the exit_req it saw last     */
  uint32_t pad[13];
  unsigned char args[SCG_BG_SERVER_SLOTS][SCG_BG_SERVER_ARGS_BYTES]; /* opaque, per slot    */
} scg_bg_server_box;

typedef struct scg_bg_server {
  scg_bg_server_box* box_host; /* the mailbox's host address                                */
  scg_bg_server_box* box_dev;  /* its device address (hipHostGetDevicePointer)              */
  void* stream;                /* the wave's stream: a non-blocking one of the caller's (a
                                  high-priority one keeps the parked wave off the hardware
                                  queues of normal-priority streams)                         */
  int32_t levels;              /* the wave's instantiation: every slot's config must match  */
  int32_t demand_mode;
  int32_t idle_us;             /* the wave exits after this long without a request          */
  int32_t check_us;            /* a waiting step checks this often whether the wave has
                                  gone (0: 2 s)                                              */
  /* host bookkeeping: zero before first use */
  int32_t lock;
  int32_t running;             /* the wave may be running                                   */
  uint32_t slots_used;         /* bit k: slot k attached                                    */
  int32_t pad;
  int64_t last_ns;             /* host monotonic time of the last request posted or served  */
  int64_t launches;            /* waves launched so far                                     */
} scg_bg_server;

typedef struct scg_bg_server_slot {
  scg_bg_server* server;       /* set by scg_bg_server_attach                               */
  const int32_t* action;       /* DEVICE-visible int32 [N][L], read each request            */
  const int32_t* action_host;  /* its host address, or NULL: with one env of L <= 8 the row
                                  is copied into the request line (no second read)         */
  int32_t* obs;                /* DEVICE-visible int32 [N][L]                               */
  int32_t* reward;             /* DEVICE-visible int32 [N]                                  */
  int32_t index;               /* out: the slot, -1 when detached                           */
  uint32_t gen;                /* out: generation of the arguments last published           */
  uint32_t seq;                /* out: the request last posted                              */
  int32_t week;                /* out: the week it steps                                    */
  int32_t done;                /* out: that week is the terminal one                        */
  int32_t relaunches;          /* out: waves this slot's waits launched again (wave gone)   */
} scg_bg_server_slot;

/* Take a free slot of `sv` for one env (slot->action/obs/reward set by the caller). */
SCG_API int scg_bg_server_attach(scg_bg_server* sv, scg_bg_server_slot* slot);
/* Give the slot back (no request of it may be unanswered). */
SCG_API int scg_bg_server_detach(scg_bg_server_slot* slot);
/* Post step(action) for the st->n_envs <= 64 envs of the slot; launches the wave if needed. */
SCG_API int scg_bg_server_post(const scg_bg_config* cfg, scg_bg_state* st, scg_bg_server_slot* slot);
/* Wait for the slot's posted step: SCG_OK (st->week advanced, *done as scg_bg_step),
 * SCG_PENDING after spin_us (< 0: no limit; the wait then fails after 60 s), or an error
 * (a HIP error of the wave's stream at once; a wave gone twice without answering). */
SCG_API int scg_bg_server_wait(scg_bg_state* st, scg_bg_server_slot* slot, int64_t spin_us, int32_t* done);
/* post + wait without limit. */
SCG_API int scg_bg_server_step(const scg_bg_config* cfg, scg_bg_state* st, scg_bg_server_slot* slot, int32_t* done);
/* Ask the wave to exit and wait for it (a no-op when it is not running). */
SCG_API int scg_bg_server_stop(scg_bg_server* sv);
/* The request line's check word (the mixing hash the wave recomputes). */
SCG_API uint32_t scg_bg_server_line_check(const scg_bg_server_line* line);

/*
 * K consecutive steps in one launch per <= SCG_BG_ROLLOUT_MAX weeks, state held in
 * registers/LDS (open-loop action plans, evaluation sweeps). Same results as K calls
 * of scg_bg_step with the same flags (SCG_BG_AUTORESET may cross episode ends).
 *   actions DEVICE int32 [K][N][L]; obs DEVICE int32 [K][N][L] or NULL;
 *   rewards DEVICE int32 [K][N] or NULL.
 */
SCG_API int scg_bg_rollout(const scg_bg_config* cfg, scg_bg_state* st, int32_t n_weeks,
                   const int32_t* actions, int32_t* obs, int32_t* rewards, uint32_t flags,
                   void* stream);

/*
 * Device-side Philox draws for tests and benchmarks (no host round trip):
 *  scg_bg_poisson_demand: out DEVICE int32 [T][N], the demand scg_bg_step draws
 *    for episode `episode` in SCG_DEMAND_POISSON mode.
 *  scg_uniform_ints: out DEVICE int32 [rows][N][width], uniform in [lo, hi],
 *    word j of env n from philox(ctr=(env_offset+n, tag, j/4, SCG_STREAM_ACTION))[j%4]
 *    with j = row*width + col.
 */
SCG_API int scg_bg_poisson_demand(const scg_bg_config* cfg, const scg_bg_state* st, uint32_t episode,
                          int32_t* out, void* stream);
SCG_API int scg_uniform_ints(uint64_t seed, int64_t env_offset, int64_t n_envs, int32_t rows,
                     int32_t width, uint32_t tag, int32_t lo, int32_t hi, int32_t* out,
                     void* stream);

/* ======================================================================================
 * SupplyChainEnv (supplychain_env.py:478-813): generic multi-echelon, multi-product chain.
 *
 *   SupplyChainEnv.__init__(nodes_info, ...)  :482-628  -> scg_sc_config + scg_sc_node[] + scg_sc_prepare
 *   SupplyChainEnv.reset()                    :630-682  -> scg_sc_reset
 *   SupplyChainEnv.step(action)               :703-748  -> scg_sc_step
 *     SC_Node.act :208-396, SC_Action.apply :42-98, heapq pipeline :398-400,
 *     _build_observation :762-791, SC_Node.build_observation :428-463 (all fused)
 * Per-episode randomness (customer demand table, stochastic lead times; the reference
 * draws both with RandomState at reset, :644-672) is drawn on device with Philox:
 * demand word (t*R + r)*P + p on stream 2, lead-time word (t-1)*n_lt + k on stream 3.
 * ====================================================================================== */

#define SCG_SC_MAX_PRODUCTS 16
#define SCG_SC_MAX_DESTS 32
#define SCG_SC_MAX_INIT 16
#define SCG_SC_MAX_NODES 256
#define SCG_SC_MAX_LEVELS 16
#define SCG_SC_LEDGER_KEYS 8 /* info['sc_episode'] cost/unit categories (:416-417) */

/* SupplyChain kernels (scg_sc_config.kernel) and the state layouts they use. */
#define SCG_SC_KERNEL_AUTO 0
#define SCG_SC_KERNEL_LANE 1  /* one lane walks one env's whole chain; env-fastest state       */
#define SCG_SC_KERNEL_LEVEL 2 /* a lane group per env, one lane per node of a level; env-major */
#define SCG_SC_KERNEL_STAGED 3 /* one lane per env, one node's heaps in LDS at a time, shipments
                                  through a per-env global inbox; env-fastest                 */
#define SCG_SC_KERNEL_NODES 4  /* 64 envs x W waves per block, a wave per node: all nodes act at
                                  once, heaps and shipments in LDS; env-fastest               */
#define SCG_SC_LAYOUT_ENV_FASTEST 0 /* stock [NP][N], heaps [NP][H][N], sizes [NP][N]          */
#define SCG_SC_LAYOUT_ENV_MAJOR 1   /* stock [N][NP], heaps [N][NP][H], sizes [N][NP]          */
#define SCG_STREAM_SC_DEMAND 2u
#define SCG_STREAM_SC_LEADTIME 3u

/* One chain node (SC_Node :106-206 after define_destinations), in nodes_info order. */
typedef struct scg_sc_node {
  int32_t last_level;           /* retailer: serves customer demand (:379-387)             */
  int32_t n_supply;             /* SUPPLY actions: products with supply_capacity > 0       */
  int32_t n_ship;               /* SHIP actions: n_dests per product with stock_capacity>0 */
  int32_t n_dests;
  int32_t processing_capacity;  /* > 0: a factory (:298-310, :337-341)                     */
  int32_t retailer_index;       /* customer_demands column, -1 if not a retailer           */
  int32_t action_offset;        /* first action of this node in the action vector (:716)  */
  int32_t leadtime_offset;      /* first lead time of this node in a step's row (:720-722) */
  int32_t supply_capacity[SCG_SC_MAX_PRODUCTS];
  int32_t supply_cost[SCG_SC_MAX_PRODUCTS];
  int32_t stock_capacity[SCG_SC_MAX_PRODUCTS];
  int32_t stock_cost[SCG_SC_MAX_PRODUCTS];
  int32_t processing_ratio[SCG_SC_MAX_PRODUCTS];
  int32_t processing_cost[SCG_SC_MAX_PRODUCTS];
  int32_t max_ship[SCG_SC_MAX_PRODUCTS];       /* observation normaliser (:147, :206)     */
  int32_t initial_stock[SCG_SC_MAX_PRODUCTS];
  int32_t n_init[SCG_SC_MAX_PRODUCTS];         /* initial pipeline entries (:402-412)     */
  int32_t init_time[SCG_SC_MAX_PRODUCTS][SCG_SC_MAX_INIT];
  int32_t init_amount[SCG_SC_MAX_PRODUCTS][SCG_SC_MAX_INIT];
  int32_t dests[SCG_SC_MAX_DESTS];             /* node indices                            */
  int32_t ship_capacity[SCG_SC_MAX_DESTS];
  int32_t dest_costs[SCG_SC_MAX_PRODUCTS][SCG_SC_MAX_DESTS];
  /* out of scg_sc_prepare (staged kernel): this node's shipment inbox — one entry per
   * (product, source node) at in_base + p * in_deg + k, sources k in node order — and, per
   * destination d, where this node's shipment lands in the destination's inbox:
   * in_slot[d] + p * in_stride[d]. */
  int32_t in_deg, in_base;
  int32_t in_slot[SCG_SC_MAX_DESTS];
  int32_t in_stride[SCG_SC_MAX_DESTS];
} scg_sc_node;

typedef struct scg_sc_config {
  int32_t n_nodes, n_products, n_retailers;
  int32_t n_actions;            /* action_space size (:608-610)                            */
  int32_t n_obs;                /* observation_space size (:617-621)                       */
  int32_t n_leadtimes;          /* lead times per step when stochastic (:601-605)          */
  int32_t total_time_steps;     /* T                                                       */
  int32_t avg_leadtime, max_leadtime, stochastic_leadtimes;
  int32_t demand_lo, demand_hi; /* uniform demand range (demands_generator.py:33-36)       */
  int32_t unmet_demand_cost, exceeded_stock_capacity_cost;
  int32_t exceeded_process_capacity_cost, exceeded_ship_capacity_cost;
  int32_t heap_capacity;        /* H: entries per (node, product) heap (scg_sc_prepare)    */
  int32_t leadtime_poisson_len;
  int32_t obs_f64;              /* observation dtype: 0 float32, 1 float64                 */
  int32_t max_dests;            /* out of scg_sc_prepare: most destinations of any node    */
  const scg_sc_node* nodes;     /* DEVICE [n_nodes]                                        */
  const uint32_t* leadtime_poisson; /* DEVICE Poisson(avg_leadtime-1) thresholds           */
  const int32_t* demand_table;  /* DEVICE [N][T+1][R][P] caller tables instead of Philox    */
                                /* (NULL = draw; e.g. to replay RandomState episodes)       */
  const int32_t* leadtime_table;/* DEVICE [N][T][n_leadtimes] likewise (stochastic only)    */
  /* Kernel choice (in: SCG_SC_KERNEL_*, 0 = auto; out: the kernel scg_sc_step launches) and
   * what scg_sc_prepare derives for it: the state layout, lanes per env and the level
   * schedule (levels are runs of consecutive nodes; every shipment goes from a level to
   * the next one, so a level's nodes never depend on each other within a step). */
  int32_t kernel;
  int32_t layout;               /* out: SCG_SC_LAYOUT_*                                     */
  int32_t group;                /* out: lanes per env (level kernel), waves per block (nodes)*/
  int32_t n_levels;             /* out: 0 when the chain has no such schedule               */
  int32_t level_start[SCG_SC_MAX_LEVELS + 1];
  int32_t inbox_size;           /* out: shipment inbox entries per env (level/staged/nodes) */
  int32_t level_staged;         /* out: 1 = the level kernel stages each env's state in LDS */
  /* Per-product demand models (demands_generator.py:3-89). demand_models = 0: every
   * product is uniform on [demand_lo, demand_hi]. Otherwise per product p: kind
   * SCG_SC_DEMAND_*, range [lo_p, hi_p] (also the observation's normalisation, :771-777),
   * NORMAL / SINE_NORMAL: a draw is lo_p + #{k : thr[off_p + row * (hi_p - lo_p) + k] <= u}
   * (row 0 for NORMAL, the period for SINE_NORMAL); SINE_UNIFORM: rint(clip(base[off_p +
   * period] + j, lo_p, hi_p)) with j = pert_lo_p + floor(u * pert_n_p / 2^32). */
  int32_t demand_models;
  int32_t demand_kind[SCG_SC_MAX_PRODUCTS];
  int32_t demand_lo_p[SCG_SC_MAX_PRODUCTS], demand_hi_p[SCG_SC_MAX_PRODUCTS];
  int32_t demand_pert_lo[SCG_SC_MAX_PRODUCTS], demand_pert_n[SCG_SC_MAX_PRODUCTS];
  int64_t demand_off[SCG_SC_MAX_PRODUCTS];
  const uint32_t* demand_thr;   /* DEVICE thresholds of the NORMAL / SINE_NORMAL products  */
  const double* demand_base;    /* DEVICE [T+1] sinusoid bases of the SINE_UNIFORM products */
} scg_sc_config;

#define SCG_SC_DEMAND_UNIFORM 0
#define SCG_SC_DEMAND_NORMAL 1
#define SCG_SC_DEMAND_SINE_NORMAL 2
#define SCG_SC_DEMAND_SINE_UNIFORM 3

/* Batch state. NP = n_nodes * n_products; per-env arrays follow cfg->layout (shapes below
 * are the env-fastest ones; env-major puts the env index first). */
typedef struct scg_sc_state {
  int64_t n_envs;
  int64_t env_offset;
  uint64_t seed;
  uint32_t episode;
  int32_t time_step;            /* 0 after reset; -1 = not reset                           */
  double* stock;                /* [NP][N]     float64 stock (:228)                        */
  int32_t* heap_tk;             /* [NP][H][N]  time << 3 | NumPy kind of the amount        */
  double* heap_val;             /* [NP][H][N]  amount                                       */
  int32_t* heap_size;           /* [NP][N]                                                  */
  double* episode_return;       /* [N] optional                                             */
  double* final_return;         /* [N] optional: return at the terminal step                */
  int32_t* error_flags;         /* [1] DEVICE, sticky: bit 0 = a heap exceeded capacity    */
  uint8_t* inbox_tk;            /* [inbox_size][N] staged kernel: shipment (time - t)<<3|kind, 0xFF = none */
  double* inbox_val;            /* [inbox_size][N] staged kernel: shipment amount               */
  /* build_info ledgers, info['sc_episode'] (:684-695, :750-760): optional (every kernel but
     the level kernel).
     Entry ((part * SCG_SC_LEDGER_KEYS + key) * P + p), part 0 = costs, 1 = units, keys in
     the reference's order (stock, stock_pen, supply, process, process_pen, ship, ship_pen,
     unmet_dem); value in ledger, NumPy type (0 int, 1 float, 2 float32, 3 float64, 4 int64)
     in ledger_kind. The final_* pair receives the terminal step's ledger on auto-reset. */
  double* ledger;               /* [2 * 8 * P][N] */
  int32_t* ledger_kind;         /* [2 * 8 * P][N] */
  double* final_ledger;         /* [2 * 8 * P][N] optional */
  int32_t* final_ledger_kind;   /* [2 * 8 * P][N] optional */
  /* Node-parallel kernel with ledgers: each node's entry values of the step, float64
   * [n_nodes * 2 * 8 * P][N] (slot ((node * 2 + part) * 8 + key) * P + p; their NumPy types
   * stay in LDS), added to the ledger in node order after the step (:750-760). Without it a
   * ledger step of a SCG_SC_KERNEL_NODES config runs the lane kernel on the same state. */
  double* ledger_part;
} scg_sc_state;

/* sizeof(scg_sc_node), sizeof(scg_sc_config), sizeof(scg_sc_state), to check FFI bindings. */
SCG_API int scg_sc_struct_sizes(size_t* node_size, size_t* config_size, size_t* state_size);

/* Validate cfg against the host copy of the node table; fills n_actions, n_obs,
 * n_leadtimes, heap_capacity and max_dests. Host only. */
SCG_API int scg_sc_prepare(scg_sc_config* cfg, scg_sc_node* host_nodes);

/* reset() for all envs (:630-682). obs: DEVICE [N][n_obs] (float32 or float64) or NULL. */
SCG_API int scg_sc_reset(const scg_sc_config* cfg, scg_sc_state* st, void* obs, void* stream);

/* step(action) for all envs (:703-748).
 *   action DEVICE float32 [N][n_actions], in the reference's [-1, 1] convention (:697-698)
 *   obs    DEVICE [N][n_obs]; reward DEVICE float64 [N]; terminal_obs optional.
 * Returns SCG_ERR_PAST_HORIZON after the terminal step without SCG_BG_AUTORESET. */
SCG_API int scg_sc_step(const scg_sc_config* cfg, scg_sc_state* st, const float* action, void* obs,
                        double* reward, void* terminal_obs, uint32_t flags, int32_t* done, void* stream);

/* The per-episode tables scg_sc_step draws (for tests): demand DEVICE int32
 * [N][T+1][R][P], leadtimes DEVICE int32 [N][T][n_leadtimes] (NULL when deterministic). */
SCG_API int scg_sc_draw_tables(const scg_sc_config* cfg, const scg_sc_state* st, uint32_t episode,
                               int32_t* demand, int32_t* leadtimes, void* stream);

/*
 * Step server for the drop-in SupplyChainEnv (one env stepped per Python call,
 * supplychain_env.py:703-748): one resident block of the node-parallel kernel's shape (a wave
 * per node) polls a host-mapped mailbox and runs the node-parallel step of tile 0 for each
 * posted step, on the state and buffers the launch arguments named when it started — the
 * config's kernel must be SCG_SC_KERNEL_NODES, float64 observations, no ledgers, up to 64
 * envs. The same protocol as the BeerGame server: post the step (its time, flags and
 * episode travel in the request, and one env's action row too), wait for the answer word;
 * the block exits on scg_sc_server_stop or after idle_us without a request, and the next post
 * launches it again (with the then-current state pointers and action / obs / reward
 * buffers). Between two steps of an episode the block keeps the env's state in its LDS (it
 * still writes every step's state back to memory), so a step reads no state from memory;
 * a reset (a new episode) or `reload` makes it read the state again.
 */
typedef struct scg_sc_server_box { /* host-mapped (hipHostMalloc mapped + coherent), 192 B */
  /* the request: two 64-byte lines, which the block reads in one load */
  uint32_t req_seq;   /* request number                                                   */
  int32_t cmd;        /* 0: step                                                          */
  int32_t t;          /* the step's time (1..T)                                           */
  int32_t flags;      /* bit0 terminal (as scg_sc_step's kernel flags)                    */
  uint32_t episode;   /* the state's episode                                              */
  uint32_t opts;      /* bit0: env 0's action row travels in action[] (one env, A <= 16);
                         bit1: read the state from memory (not the block's LDS copy)      */
  int32_t pad0;
  uint32_t check;     /* scg mixing hash of the two lines' other 31 words                 */
  int32_t pad1[8];
  float action[16];   /* line 1: the inline action row                                    */
  /* the answer, on its own line */
  uint32_t done_seq;  /* the last request served (written by the block)                   */
  uint32_t exit_req;  /* the block exits when this differs from its launch value          */
  uint32_t exit_seq;  /* written by the block as it exits: the exit_req it saw last       */
  uint32_t pad2[13];
} scg_sc_server_box;

typedef struct scg_sc_server {
  scg_sc_server_box* box_host; /* the mailbox's host address                              */
  scg_sc_server_box* box_dev;  /* its device address                                      */
  void* stream;                /* a non-blocking stream of the caller's (high priority)   */
  const float* action;         /* DEVICE-visible float32 [N][A]                           */
  const float* action_host;    /* its host address, or NULL: with one env of A <= 16 the
                                  row is copied into the request (no read across PCIe)   */
  void* obs;                   /* DEVICE-visible float64 [N][O]                           */
  double* reward;              /* DEVICE-visible float64 [N]                              */
  int32_t idle_us;             /* the block exits after this long without a request       */
  int32_t check_us;            /* a waiting step checks this often for a gone block (0: 2 s) */
  int32_t reload;              /* set by the caller when something else wrote the state (it
                                  has no launch of its own on it otherwise): the next post
                                  makes the block read it from memory; cleared by the post */
  /* host bookkeeping: zero before first use */
  int32_t running;
  uint32_t seq;                /* the request last posted                                 */
  int32_t t;                   /* the step it runs                                        */
  int32_t done;                /* that step is the terminal one                           */
  int32_t relaunches;          /* blocks a wait launched again (block gone)               */
  int64_t last_ns;
  int64_t launches;
} scg_sc_server;

/* Post step(action) of the st->n_envs <= 64 envs (launches the block if needed). */
SCG_API int scg_sc_server_post(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv);
/* Wait for it: SCG_OK (st->time_step advanced, *done), SCG_PENDING after spin_us (< 0: no
 * limit; the wait then fails after 60 s), or an error. */
SCG_API int scg_sc_server_wait(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv, int64_t spin_us,
                               int32_t* done);
/* post + wait without limit. */
SCG_API int scg_sc_server_step(const scg_sc_config* cfg, scg_sc_state* st, scg_sc_server* sv, int32_t* done);
/* Ask the block to exit and wait for it (a no-op when it is not running). */
SCG_API int scg_sc_server_stop(scg_sc_server* sv);

/* Testing hook: cap the node-parallel kernel's persistent grid at `blocks` blocks (0, the
 * default: as many as the device holds at once), so a small batch runs several 64-env tiles
 * per block and the next-tile prefetch runs (scg_sc_nodes.hip). Returns the previous cap. */
SCG_API int scg_sc_nodes_max_blocks(int32_t blocks);

#ifdef __cplusplus
}
#endif

#endif /* SCGPU_H */
