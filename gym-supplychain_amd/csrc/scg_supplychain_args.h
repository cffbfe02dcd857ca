// Launch arguments and per-env views shared by the SupplyChain kernels (scg_supplychain.hip,
// scg_sc_nodes.hip): the ScArgs block every step/reset kernel takes, observation rows, the
// env-fastest / env-major state views, and the one-lane step on HBM heaps.
#pragma once

#include "scg_supplychain_core.h"
#include "scgpu.h"

namespace scg {

constexpr int kScBlock = 64;

struct ScArgs {
  ScCtx c;
  double* stock;
  int32_t* tk;
  double* val;
  int32_t* size;
  const float* act;
  void* obs;
  void* term_obs;
  double* rew;
  double* ep_ret;
  double* final_ret;
  int32_t* err;
  uint8_t* inbox_tk;  // staged kernel: shipment inbox [inbox_size][N] (scg_supplychain_staged.h)
  double* inbox_val;
  double* led_v;     // build_info ledgers [2*8*P][N] (lane kernels) or null
  int32_t* led_k;
  double* led_fv;    // terminal-step ledger on auto-reset
  int32_t* led_fk;
  double* ledp_v;    // node-parallel kernel: the nodes' ledger entry values of the step [NN*2*8*P][N]
  int64_t n;
  int64_t env_offset;
  uint32_t episode;
  int32_t t;       // the step being simulated (1..T) / 0 for reset
  int32_t flags;   // bit0 terminal, bit1 autoreset, bit2 serial walk (node-parallel kernel)
  int32_t obs_f64;
  int32_t layout;  // SCG_SC_LAYOUT_*
};

// The launch's ScCtx (the first member of ScArgs, the kernel's first argument) re-read
// through the kernel-argument pointer laundered by an empty asm: the compiler cannot prove two
// calls return the same object, so a loop over nodes loads context fields (scalar loads,
// cached) where each iteration uses them instead of hoisting them and everything derived from
// them out of the loop and holding them in scalar registers across it, which spilled them
// into VGPR lanes. Only for kernels whose first argument is `const ScArgs`.
struct KernargCtx {
  __device__ __forceinline__ const ScCtx& operator()() const {
    typedef const __attribute__((address_space(4))) ScArgs* KArgPtr;
    KArgPtr ap = (KArgPtr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    return ((const ScArgs*)ap)->c;
  }
};

struct ObsRow {
  void* base;
  int64_t row;
  int f64;
  __device__ __forceinline__ void operator()(int o, double x) const {
    if (f64)
      static_cast<double*>(base)[row + o] = x;
    else
      static_cast<float*>(base)[row + o] = static_cast<float>(x);
  }
};

__device__ __forceinline__ ScEnv env_view(const ScArgs& a, int64_t n, uint32_t episode) {
  if (a.layout == SCG_SC_LAYOUT_ENV_MAJOR) {  // env n's block: [NP], [NP][H]
    const int64_t NP = static_cast<int64_t>(a.c.n_nodes) * a.c.P;
    return ScEnv{a.stock + n * NP, a.tk + n * NP * a.c.H, a.val + n * NP * a.c.H, a.size + n * NP, 1, 1,
                 static_cast<uint32_t>(a.env_offset + n), n, episode, 0};
  }
  ScEnv e{a.stock + n, a.tk + n, a.val + n, a.size + n, a.n, a.n, static_cast<uint32_t>(a.env_offset + n), n, episode, 0};
  if (a.led_v) {
    e.led_v = a.led_v + n;
    e.led_k = a.led_k + n;
    e.led_stride = a.n;
  }
  return e;
}

// Auto-reset keeps the finished episode's ledger (the info of the terminal step, :744-746).
__device__ __forceinline__ void snapshot_ledger(const ScArgs& a, const ScCtx& c, int64_t n) {
  if (!a.led_v || !a.led_fv) return;
  for (int q = 0; q < 2 * SCG_SC_LEDGER_KEYS * c.P; ++q) {
    a.led_fv[q * a.n + n] = a.led_v[q * a.n + n];
    a.led_fk[q * a.n + n] = a.led_k[q * a.n + n];
  }
}

// One env's whole step on HBM heaps, one lane walking the chain in node order: the lane
// kernel's body (sc_step_kernel), and the node-parallel kernel's path for an env whose
// receive order it cannot prove (scg_sc_nodes.hip).
template <int MAXD>
__device__ inline void sc_lane_step(const ScArgs& a, int64_t n) {
  ScEnv e = env_view(a, n, a.episode);
  const double reward = sc_step_env<MAXD>(a.c, e, a.act + n * a.c.A, a.t);
  a.rew[n] = reward;
  const bool terminal = a.flags & 1;
  if (a.ep_ret) {
    const double r = a.ep_ret[n] + reward;  // episode_rewards += current_reward (:739)
    if (terminal && a.final_ret) a.final_ret[n] = r;
    a.ep_ret[n] = (a.flags & 2) ? 0.0 : r;
  }
  if (a.flags & 2) {  // auto-reset: terminal observation aside, fresh episode in place
    if (a.term_obs) {
      ObsRow tout{a.term_obs, n * a.c.O, a.obs_f64};
      sc_observe(a.c, e, a.t, tout);
    }
    snapshot_ledger(a, a.c, n);
    e.episode = a.episode + 1;
    sc_reset_env(a.c, e);
    ObsRow out{a.obs, n * a.c.O, a.obs_f64};
    sc_observe(a.c, e, 0, out);
  } else {
    ObsRow out{a.obs, n * a.c.O, a.obs_f64};
    sc_observe(a.c, e, a.t, out);
    if (terminal && a.term_obs) {
      ObsRow tout{a.term_obs, n * a.c.O, a.obs_f64};
      sc_observe(a.c, e, a.t, tout);
    }
  }
  if (e.overflow) atomicOr(a.err, 1);
}

}  // namespace scg
