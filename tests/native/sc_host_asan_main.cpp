// TEST-ONLY: the host build of the SupplyChain kernel body (sc_host_harness.cpp) as an
// executable, for the AddressSanitizer / UndefinedBehaviorSanitizer build that
// tests/test_sc_sanitizers.py makes and runs (SURVEY §5 "race detection / sanitizers": GPU
// sanitizers are not available on the pool, so the kernels' bodies are checked on the host).
//
//   sc_host_asan JOBS OUT
// JOBS holds a sequence of jobs, each one episode of one env in one kernel body (mode: 0
// lane, 1 level, 2 staged, 3 node-parallel phases with the nodes in reverse order, 4 the
// node-parallel serial walk, 5 lane; ledgers kept from mode 2 on); OUT receives, per job, the
// return code and every snapshot the shared library's sch_episode_* entry points return.
// Layout of a job (little endian): int32 magic 0x53434A42, mode, cfg_bytes, node_bytes,
// n_nodes, thr_len, dthr_len, dbase_len, steps, A, O, NP, H, P; uint64 seed; uint32 env_id,
// episode; then the scg_sc_config bytes, the scg_sc_node table, the uint32 lead-time
// thresholds, the uint32 demand thresholds, the float64 demand bases and float32 actions.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sc_host_harness.cpp"

namespace {

template <class T>
bool rd(FILE* f, T* p, size_t n) {
  return n == 0 || fread(p, sizeof(T), n, f) == n;
}

template <class T>
void wr(FILE* f, const T* p, size_t n) {
  if (n) fwrite(p, sizeof(T), n, f);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s JOBS OUT\n", argv[0]);
    return 2;
  }
  FILE* in = fopen(argv[1], "rb");
  FILE* out = fopen(argv[2], "wb");
  if (!in || !out) return 2;
  int jobs = 0;
  for (;;) {
    int32_t h[14];
    if (fread(h, sizeof(int32_t), 14, in) != 14) break;
    if (h[0] != 0x53434A42) return 3;
    const int mode = h[1], cfg_bytes = h[2], node_bytes = h[3], n_nodes = h[4], thr_len = h[5], dthr_len = h[6],
              dbase_len = h[7], steps = h[8], A = h[9], O = h[10], NP = h[11], H = h[12], P = h[13];
    if (cfg_bytes != static_cast<int>(sizeof(scg_sc_config)) || node_bytes != static_cast<int>(sizeof(scg_sc_node)))
      return 4;
    uint64_t seed;
    uint32_t ids[2];
    scg_sc_config cfg;
    std::vector<scg_sc_node> nodes(n_nodes);
    std::vector<uint32_t> thr(thr_len > 0 ? thr_len : 1, 0), dthr(dthr_len);
    std::vector<double> dbase(dbase_len);
    std::vector<float> acts(static_cast<size_t>(steps) * A);
    if (!rd(in, &seed, 1) || !rd(in, ids, 2) || !rd(in, &cfg, 1) || !rd(in, nodes.data(), n_nodes) ||
        !rd(in, thr.data(), thr_len) || !rd(in, dthr.data(), dthr_len) || !rd(in, dbase.data(), dbase_len) ||
        !rd(in, acts.data(), acts.size()))
      return 5;
    // the host pointers of the process that wrote the job mean nothing here
    cfg.nodes = nullptr;
    cfg.leadtime_poisson = nullptr;
    cfg.demand_table = nullptr;
    cfg.leadtime_table = nullptr;
    cfg.demand_thr = dthr_len ? dthr.data() : nullptr;
    cfg.demand_base = dbase_len ? dbase.data() : nullptr;
    std::vector<double> obs(static_cast<size_t>(steps + 1) * O), rew(steps), stock(static_cast<size_t>(steps + 1) * NP),
        val(static_cast<size_t>(steps + 1) * NP * H), led_v(static_cast<size_t>(steps) * 2 * 8 * P);
    std::vector<int32_t> tk(static_cast<size_t>(steps + 1) * NP * H), sz(static_cast<size_t>(steps + 1) * NP),
        led_k(led_v.size());
    const bool ledger = mode >= 2;  // staged, node-parallel (by-node slots) and lane kernels
    const int impl = mode == 5 ? 0 : mode;
    const int32_t rc = episode_impl(impl, &cfg, nodes.data(), thr.data(), seed, ids[0], ids[1], steps, acts.data(),
                                    obs.data(), rew.data(), stock.data(), tk.data(), val.data(), sz.data(),
                                    ledger ? led_v.data() : nullptr, ledger ? led_k.data() : nullptr);
    const int32_t fallbacks = sch_nodes_fallbacks();
    wr(out, &rc, 1);
    wr(out, &fallbacks, 1);
    wr(out, obs.data(), obs.size());
    wr(out, rew.data(), rew.size());
    wr(out, stock.data(), stock.size());
    wr(out, tk.data(), tk.size());
    wr(out, val.data(), val.size());
    wr(out, sz.data(), sz.size());
    wr(out, led_v.data(), led_v.size());
    wr(out, led_k.data(), led_k.size());
    ++jobs;
  }
  fclose(in);
  fclose(out);
  fprintf(stderr, "sc_host_asan: %d jobs\n", jobs);
  return 0;
}
