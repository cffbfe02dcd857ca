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
// shipment inbox [E][64], node costs [NN][64], the stocks a step started from [NP][64]; then
// the int32 heap times/kinds, heap sizes, inbox times/kinds, cost kinds and the per-wave
// "order not provable" flags [W][64].
//   stage  (wave w, its nodes)  heaps HBM -> LDS, released sums, flags
//   act    (wave w, its nodes)  stock, costs, shipments -> inbox, stock obs | barrier
//   heaps  (wave w, its nodes)  inbox pushes, pops, supply push, bins, copy back
//   reward (wave 0)             -(costs in node order), return, demand / time obs, reset
// An env any wave flagged skips heaps; wave 0 puts its stocks back and steps it alone on its
// staged heaps, node after node in the reference's order (sc_nodes_serial).
#include <hip/hip_runtime.h>

#include "scg_common.h"
#include "scg_supplychain_core.h"
#include "scg_supplychain_args.h"
#include "scg_supplychain_nodes.h"

// Diagnostic build only (-DSCG_NODES_STAMPS, tools/nodes_stamps.py): lane 0 of every wave
// records the shader clock at the phase boundaries (0 start, 5 heaps staged, 1 acted, 2 past
// the barrier, 3 heaps done, 4 end) into a buffer of its own that scg_nodes_debug_stamps copies
// out; nothing else reads it. In the product build NSTAMP is empty.
#ifdef SCG_NODES_STAMPS
constexpr int kNStampSlots = 8;
constexpr int kNStampWaves = 1 << 14;
__device__ unsigned long long g_nodes_stamps[kNStampWaves * kNStampSlots];
#define NSTAMP(k)                                                                                   \
  do {                                                                                              \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                                   \
    const unsigned w_ = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;                        \
    if ((threadIdx.x & 63u) == 0 && w_ < static_cast<unsigned>(kNStampWaves))                       \
      g_nodes_stamps[w_ * kNStampSlots + (k)] = now_;                                               \
  } while (0)
#else
#define NSTAMP(k)
#endif

namespace scg {

constexpr int kNodesMaxWaves = 8;

#ifndef SCG_NODES_WPE
#define SCG_NODES_WPE 4
#endif
// Four waves per SIMD (<= 128 VGPRs): two blocks of eight waves per CU, which is also what
// their LDS allows.
template <int MAXD>
__global__ __launch_bounds__(64 * kNodesMaxWaves) __attribute__((amdgpu_waves_per_eu(SCG_NODES_WPE)))
void sc_step_nodes_kernel(const ScArgs a, int W, int E) {
  extern __shared__ __align__(16) unsigned char smem[];
  const ScCtx& c = a.c;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const bool live = n < a.n;
  const int NN = c.n_nodes, P = c.P, NP = NN * P, H = c.H;
  double* hval = reinterpret_cast<double*>(smem);
  double* recv = hval + static_cast<int64_t>(NP) * H * 64;
  double* ibval = recv + NP * 64;
  double* cost_v = ibval + static_cast<int64_t>(E) * 64;
  double* stock0 = cost_v + NN * 64;
  int32_t* htk = reinterpret_cast<int32_t*>(stock0 + NP * 64);
  int32_t* hsz = htk + static_cast<int64_t>(NP) * H * 64;
  int32_t* ibtk = hsz + NP * 64;
  int32_t* cost_k = ibtk + static_cast<int64_t>(E) * 64;
  int32_t* amb = cost_k + NN * 64;
  ScEnv g = env_view(a, n, a.episode);
  auto lheap = [&](int hp) { return HeapView{htk + hp * H * 64 + lane, hval + hp * H * 64 + lane, 64}; };
  NSTAMP(0);

  // node observations go to obs, or to the terminal observation when the env resets now
  const bool terminal = a.flags & 1;
  const bool autoreset = a.flags & 2;
  void* node_obs = autoreset ? a.term_obs : a.obs;
  ObsRow main{node_obs ? node_obs : a.obs, n * c.O, a.obs_f64};
  ObsRow extra{a.term_obs, n * c.O, a.obs_f64};
  const bool both = terminal && !autoreset && a.term_obs;
  auto sink = [&](int o, double x) {
    if (node_obs) main(o, x);
    if (both) extra(o, x);
  };
  const NodesInbox in{ibtk + lane, ibval + lane, 64};
  const float* act = a.act + n * c.A;

  // stage, then act at once (no barrier between): a node's act needs only what its own heaps
  // release. The stock it starts from is kept, so an env some wave flags is put back and
  // stepped by the serial walk below.
  bool bad = false;
  if (live)
    for (int i = w; i < NN; i += W) {
      for (int p = 0; p < P; ++p) {
        const int hp = i * P + p;
        stock0[hp * 64 + lane] = a.stock[hp * a.n + n];
        bad |= !sc_nodes_stage(c, g, lheap(hp), hsz[hp * 64 + lane], a.t, i, p, recv[hp * 64 + lane]);
      }
      NSTAMP(5);  // (the last node of the wave's) heaps staged, act next
      const Num cst = sc_nodes_act<MAXD>(c, g, in, recv + i * P * 64 + lane, 64, act, a.t, i);
      cost_v[i * 64 + lane] = cst.v;
      cost_k[i * 64 + lane] = cst.k;
      for (int p = 0; p < P; ++p) sc_observe_stock(c, g, i, p, sink);
    }
  amb[w * 64 + lane] = bad ? 1 : 0;
  NSTAMP(1);
  __syncthreads();
  NSTAMP(2);
  bool flagged = (a.flags & 4) != 0;
  for (int v = 0; v < W; ++v) flagged |= amb[v * 64 + lane] != 0;
  const bool go = live && !flagged;

  // heaps
  if (go)
    for (int i = w; i < NN; i += W) {
      WordCache ltc{0, U4{0, 0, 0, 0}, false};
      int a_i = 0, lt_i = 0;
      for (int p = 0; p < P; ++p) {
        const int hp = i * P + p;
        sc_nodes_heap(c, g, lheap(hp), hsz[hp * 64 + lane], in, ltc, act, a.t, i, p, a_i, lt_i, sink);
      }
    }
  NSTAMP(3);
  if (autoreset) __syncthreads();  // the reset below rewrites heaps the other waves store

  // reward
  if (w == 0 && live) {
    double reward;
    if (flagged) {  // its stocks back as they were; no wave touched its heaps: they are as staged
      for (int hp = 0; hp < NP; ++hp) a.stock[hp * a.n + n] = stock0[hp * 64 + lane];
      reward = sc_nodes_serial<MAXD>(c, g, lheap, hsz + lane, 64, in, act, a.t, sink);
    } else {
      Num total = pyint(0);
      for (int i = 0; i < NN; ++i) total = np_add(total, Num{cost_v[i * 64 + lane], cost_k[i * 64 + lane]});
      reward = np_neg(total).v;
    }
    a.rew[n] = reward;
    if (a.ep_ret) {
      const double r = a.ep_ret[n] + reward;  // episode_rewards += current_reward (:739)
      if (terminal && a.final_ret) a.final_ret[n] = r;
      a.ep_ret[n] = autoreset ? 0.0 : r;
    }
    auto rest = [&](ObsRow& row, int t) {  // demand and time-to-go elements (:771, :786)
      for (int k = 0; k < c.R * c.P; ++k) sc_observe_demand(c, g, t, k, row);
      sc_observe_tail(c, t, row);
    };
    if (autoreset) {
      if (a.term_obs) rest(extra, a.t);
      g.episode = a.episode + 1;
      sc_reset_env(c, g);
      ObsRow out{a.obs, n * c.O, a.obs_f64};
      sc_observe(c, g, 0, out);
    } else {
      rest(main, a.t);
      if (both) rest(extra, a.t);
    }
  }
  if (live && g.overflow) atomicOr(a.err, 1);
  NSTAMP(4);
}

// LDS bytes of one block (the layout above).
size_t sc_nodes_lds_bytes(int n_nodes, int P, int H, int E, int W) {
  const size_t NP = static_cast<size_t>(n_nodes) * P;
  return 64 * ((NP * H + 2 * NP + E + n_nodes) * 8 + (NP * H + NP + E + n_nodes + W) * 4);
}

// Widest destination list the kernel is instantiated for (its split runs in registers).
int sc_nodes_max_dests() { return 8; }

// Waves per block for a chain: one per node up to kNodesMaxWaves.
int sc_nodes_waves(int n_nodes) { return n_nodes < kNodesMaxWaves ? n_nodes : kNodesMaxWaves; }

// A block may hold up to the CU's whole LDS (gfx950: 160 KiB); past 64 KiB the kernel is
// told once that it may.
constexpr size_t kNodesLdsMax = 160 * 1024;
size_t sc_nodes_lds_max() { return kNodesLdsMax; }

template <int MAXD>
int sc_launch_nodes_d(const ScArgs& a, int W, int E, hipStream_t s) {
  static bool raised[64] = {};  // per device; setting it twice from racing threads is harmless
  const size_t lds = sc_nodes_lds_bytes(a.c.n_nodes, a.c.P, a.c.H, E, W);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (lds > 64 * 1024 && !raised[dev]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&sc_step_nodes_kernel<MAXD>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kNodesLdsMax)) != hipSuccess)
      return fail(SCG_ERR_HIP, "node-parallel kernel: cannot raise its LDS limit");
    raised[dev] = true;
  }
  hipLaunchKernelGGL(sc_step_nodes_kernel<MAXD>, dim3(static_cast<unsigned>((a.n + 63) / 64)), dim3(64 * W), lds, s,
                     a, W, E);
  return check_launch("sc_step_nodes_kernel");
}

int sc_launch_nodes(const ScArgs& a, int maxd_bucket, int W, int E, hipStream_t s) {
  if (W < 1 || W > kNodesMaxWaves) return fail(SCG_ERR_INVALID, "node-parallel kernel: %d waves per block", W);
  switch (maxd_bucket) {
    case 2: return sc_launch_nodes_d<2>(a, W, E, s);
    case 4: return sc_launch_nodes_d<4>(a, W, E, s);
    case 8: return sc_launch_nodes_d<8>(a, W, E, s);
    default: return fail(SCG_ERR_INVALID, "node-parallel kernel: nodes ship to at most 8 destinations");
  }
}

}  // namespace scg

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
#endif
