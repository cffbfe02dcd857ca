"""bench.py — env-steps/s of beergame-v0 at 65,536 envs per GPU (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one BeerGameVecEnv.step() over this rank's 65,536 envs: one fused HIP step
kernel through the C ABI (include/scgpu.h) — receive, order slips, fill, ship, backlog,
orders, observation, reward, cost ledgers, order history and episode return, with
Poisson(8) demand drawn on device (Philox4x32-10) and auto-reset at week 35. Actions are
synthetic uniform integers in [0, 8], generated on device before timing (the policy's
output, resident in HBM). Envs shard across ranks by global id; the only collective is the
async RCCL all-gather of per-env episode returns at each episode end.

Timing (rank 0 prints ONE JSON line):
  * warm-up: max(W, 35) untimed steps — at least one whole 35-week episode, so every week
    kind of the plan and the auto-reset have run before timing — then one untimed region of
    the timed region's shape (synchronize, K steps, synchronize); "warmup_steps_run" counts
    both. The collector is off from there on;
  * the timed region is exactly K steps, bracketed by barrier + synchronize, max over
    ranks; `value` = envs of all ranks x K / that wall time. Nothing inside is stamped
    (stamping the first and last launch cost a K = 20 region 0.3-0.6 us per step,
    profiles/r02s_stamped_headline_ab.log); `headline_split` says what bounds it: the host's
    enqueue time per step (the loop's wall time up to the final synchronize / K), the wait
    after it, the same brackets around zero steps (the region's fixed cost) and the GPU
    time per step of the 100-episode region below;
  * `episodes_timed`: the same over 100 whole episodes (3,500 steps), as SURVEY §8(d)
    asks, with its first and last launch stamped (hipExtLaunchKernel dispatch begin / end):
    that GPU time / 3,500 is `roofline.avg_kernel_us`;
  * `roofline`: algorithmic bytes of those 3,500 launches (DESIGN.md §6, 260 B per env on a
    regular week, summed week by week) / their GPU time, against the 8 TB/s spec and the
    peak a STREAM copy measures in the same run (`measured_peak`, `frac_measured_peak`);
    `traffic` = HBM bytes per launch from the committed rocprofv3 PMC summary of this
    kernel; `isolated_kernel_us` = launches timed one at a time; `beyond_cache` = the same
    kernel at 1,048,576 envs (272 MB per step, past the 256 MiB Infinity Cache);
  * `cpu_baseline` (rank 0, N = 1): oracle.beergame.BeerGameOracle — the per-env NumPy
    restatement of the reference step(), calibrated against the reference by
    tools/cpu_calibration.py — on the host's cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd"))
sys.path.insert(0, REPO)

N_ENVS = 65536
LEVELS = 4
WEEKS = 35
LAMBDA = 8.0
SEED = 0x5EED0000
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)
EPISODES_TIMED = 100   # >= 100 episodes timed
KERNEL = "bg_step_slab_kernel<4, 2>"
BEYOND_CACHE_ENVS = 1 << 20


def step_bytes_per_env(plan_word, week, T, L, ring_initial_slots, ledgers, history, returns, autoreset):
    """Algorithmic HBM bytes one env moves in one step launch (mirrors the kernel).

    Regular week of the bench config (due row arrives, scheduled row stored, ledgers,
    history and returns on): 4 rows in (action, inventory, backlog, orders) + due row +
    scheduled row + history row + 4 rows out (state, obs) + 2 ledger rows RMW + reward
    + episode return RMW = 64+16+16+16+64+64+4+16 = 260 B at L = 4.
    """
    row = 4 * L
    mode, arrive = plan_word & 3, bool(plan_word & 4)
    terminal = week == T
    b = 4 * row + 4                                 # action/inventory/backlog/orders in, reward out
    b += row if arrive else 0                       # due pipeline row in
    b += {0: 0, 1: row, 2: 2 * row, 3: 0}[mode]     # scheduled row: store / read-modify-write
    b += row if history else 0                      # all_orders_placed row out
    b += row if terminal else 0                     # terminal observation out
    if returns:
        b += 16 + (8 if terminal else 0)            # episode return RMW, final return out
    if terminal and autoreset:                      # reset in the same launch
        b += 3 * row + ring_initial_slots * row + row
        b += 2 * row if ledgers else 0
        b += row if history else 0
    else:
        b += 4 * row                                # inventory/backlog/orders/obs out
        b += 4 * row if ledgers else 0              # two ledger rows read + write
    return b


def profile_tag_key(path):
    """Sort key of a profiles/ file by its session tag rNN<letters>: round number, then the
    letters as a bijective base-26 count (a..z, aa..az, ...), so r02al is newer than r02z."""
    import re
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    if not m:
        return (-1, -1)
    n = 0
    for ch in m.group(2):
        n = n * 26 + (ord(ch) - ord("a") + 1)
    return (int(m.group(1)), n)


# The sources each kernel family is compiled from: a PMC summary counts for a kernel only if
# it was collected on exactly these bytes (tools/pmc_summary.py records the hash).
KERNEL_SOURCES = {
    "bg": ["scg_beergame.hip", "scg_beergame_kernels.h", "scg_bg_levels_1.hip", "scg_bg_levels_2.hip",
           "scg_bg_levels_3.hip", "scg_bg_levels_4.hip", "scg_common.h", "scg_common.hip", "scg_const.h",
           "scg_philox.h"],
    "sc": ["scg_supplychain.hip", "scg_sc_nodes.hip", "scg_supplychain_core.h", "scg_supplychain_nodes.h",
           "scg_supplychain_staged.h", "scg_supplychain_level.h", "scg_supplychain_args.h", "scg_npscalar.h",
           "scg_pyheap.h", "scg_common.h", "scg_common.hip", "scg_const.h", "scg_philox.h"],
}


def kernel_sources_hash(family):
    """sha256 (16 hex digits) of a kernel family's sources and the shared header, in order."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.environ.get("SCG_PKG_ROOT") or os.path.join(REPO, "gym-supplychain_amd")
    for f in KERNEL_SOURCES[family]:
        with open(os.path.join(pkg, "csrc", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(REPO, "include", "scgpu.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_lookup(family, workload, kernel_substr):
    """HBM bytes per launch of `kernel_substr` from the newest committed PMC summary
    (profiles/rNN*_pmc_summary.json, tools/pmc_summary.py: separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM,
    calibrated for this repo's access shapes in profiles/r03b_pmc_calib_*.csv) whose
    recorded workload equals `workload` (every key) and whose source hash is this tree's
    for `family` — a summary of another workload, or of a kernel since changed, never
    counts. Returns (bytes, path) or (None, None)."""
    import glob
    src = kernel_sources_hash(family)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary.json")), key=profile_tag_key,
                       reverse=True):
        with open(path) as f:
            summ = json.load(f)
        meta = summ.get("workload") or {}
        if summ.get("src_hash", {}).get(family) != src or any(meta.get(k) != v for k, v in workload.items()):
            continue
        for name, t in summ.get("traffic", {}).items():
            if kernel_substr in name and t.get("hbm_bytes_per_launch"):
                return t["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
    return None, None


def pmc_traffic(kernel_substr=KERNEL, n_envs=N_ENVS):
    """The bench kernel's HBM bytes per launch at this batch size (pmc_lookup)."""
    return pmc_lookup("bg", {"bench": "beergame-v0", "n_envs": n_envs}, kernel_substr)


# ---- CPU baseline ------------------------------------------------------------------------
def cpu_worker_inputs(idx, n_episodes):
    """Per-episode inputs of CPU worker `idx`, drawn before timing: Poisson(8) demand lists
    (the device's Philox draws of env `idx`) and uniform [0, 8] actions [E, 35, L]."""
    import numpy as np

    from oracle.philox import STREAM_DEMAND, draw_words
    from oracle.poisson import poisson_invert, poisson_thresholds
    thr = poisson_thresholds(LAMBDA)
    demands = [poisson_invert(draw_words(SEED, [idx], ep, WEEKS, STREAM_DEMAND), thr)[0].tolist()
               for ep in range(n_episodes)]
    acts = np.random.RandomState(idx).randint(0, 9, size=(n_episodes, WEEKS, LEVELS))
    return demands, acts


def _cpu_worker(idx, budget_s, start):
    sys.path.insert(0, REPO)
    from oracle.beergame import BeerGameOracle
    demands, acts = cpu_worker_inputs(idx, 64)
    start()  # every worker's inputs are drawn: the timed part starts together
    steps, ep = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:  # construct + reset + 35 steps per episode
        k = ep % len(demands)
        env = BeerGameOracle({"customer_demand": demands[k]})
        env.reset()
        for w in range(WEEKS):
            env.step(acts[k, w])
        steps += WEEKS
        ep += 1
    return steps, time.perf_counter() - t0


def _cgroup_cpu_quota():
    """CPUs this process group may use per the cgroup CPU quota (v2 cpu.max, v1 cfs), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        return None if quota <= 0 else quota / period
    except (OSError, ValueError):
        return None


def host_cpus():
    """The host CPUs a baseline may use: the CPU model (/proc/cpuinfo), the cores in this
    process's affinity mask, the cgroup CPU quota if one is set, and the worker count: every
    core of the affinity mask (P = os.cpu_count() processes), down to the quota
    when one caps the job below it (processes past the quota would only share its CPU time)."""
    import math
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = _cgroup_cpu_quota()
    procs = affinity if quota is None else max(1, min(affinity, math.ceil(quota)))
    return {"cpu_model": model, "affinity_cores": affinity, "os_cpu_count": os.cpu_count(),
            "cgroup_quota_cpus": quota, "procs": procs}


def cpu_note(cpus):
    """How the worker count was chosen, for the baseline's `sample` text."""
    if cpus["procs"] < cpus["affinity_cores"]:
        return (f"the job's cgroup CPU quota of {cpus['cgroup_quota_cpus']:g} CPUs caps it below the "
                f"{cpus['affinity_cores']} cores of its affinity mask; {cpus['cpu_model']}")
    return f"one per core of the affinity mask; {cpus['cpu_model']}"


def _pool_entry(fn, idx, budget_s, barrier, q):
    try:
        q.put((idx, fn(idx, budget_s, lambda: barrier.wait(600))))
    except BaseException as exc:  # a worker that fails must not leave the others at the barrier
        barrier.abort()
        q.put((idx, repr(exc)))


def cpu_pool(fn, budget_s, procs):
    """fn(idx, budget_s, start) -> (steps, wall s) on `procs` spawned processes (no GPU use;
    each calls start() once its inputs are ready, so the timed parts overlap). Returns
    (sum of steps / max of wall, sum of steps)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(procs), ctx.Queue()
    ps = [ctx.Process(target=_pool_entry, args=(fn, i, budget_s, barrier, q), daemon=True) for i in range(procs)]
    for p in ps:
        p.start()
    try:
        res = [q.get(timeout=budget_s + 900)[1] for _ in ps]
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    bad = [r for r in res if not isinstance(r, tuple)]
    if bad:
        raise RuntimeError(f"CPU baseline worker failed: {bad[0]}")
    steps = sum(r[0] for r in res)
    return steps / max(r[1] for r in res), steps


def cpu_baseline(budget_s=2.5):
    """Per-env NumPy restatement of BeerGameEnv.step on every host core (oracle, 'port')."""
    cpus = host_cpus()
    procs = cpus["procs"]
    value, steps = cpu_pool(_cpu_worker, budget_s, procs)
    return {"value": value, "unit": "env-steps/s", "cores": procs, "kind": "port", **cpus,
            "budget_s": budget_s,
            "sample": f"{procs} processes ({cpu_note(cpus)}) x {budget_s:.1f} s "
                      f"of beergame-v0 episodes (construct + reset + 35 steps; Poisson(8) demand, uniform [0,8] "
                      f"actions drawn before timing, timed parts started together), one env per process, "
                      f"oracle.beergame.BeerGameOracle (the reference step() statement for statement; "
                      f"profiles/r04_cpu_calibration.json); {steps} env-steps total"}


# ---- the step loop (GPU VecEnv, or a CPU stand-in in tests/test_bench_distributed.py) -----
class StepLoop:
    """Steps `env` with the resident action row of each week; at episode ends hands the
    finished returns to `gather` (the async all-gather)."""

    def __init__(self, env, week_actions, gather=None):
        self.env, self.week_actions, self.gather = env, week_actions, gather
        self.episodes = 0

    def run(self, k, first=None, last=None, each=None, sync_each=None):
        env, acts = self.env, self.week_actions
        if first is None and last is None and each is None and sync_each is None:
            step, gather, T = env.step, self.gather, len(acts)
            w = env.week
            for _ in range(k):  # the timed path: one action row and one step call per week
                info = step(acts[w])[3]
                w = w + 1 if w + 1 < T else 0
                if info:
                    self.episodes += 1
                    if gather is not None:
                        gather.on_episode_end(info["episode_return"])
            return
        for i in range(k):
            stamp = each[i] if each is not None else ((first, None) if i == 0 and first else None)
            if i == k - 1 and last is not None:
                stamp = (stamp[0] if stamp else None, last)
            _, _, _, info = env.step(acts[env.week], stamp) if stamp else env.step(acts[env.week])
            if info:
                self.episodes += 1
                if self.gather is not None:
                    self.gather.on_episode_end(info["episode_return"])
            if sync_each is not None:
                sync_each()


def region(loop, k, world, barrier, sync, stamps=None, split=None):
    """Time exactly k steps: barrier + sync on both sides. Returns (wall s, GPU ms between
    the first launch's start and the last one's end, or None without stamps). With a dict
    `split`, also its host side: split["enqueue_s"] = the step loop's wall time up to the
    final synchronize (the host enqueueing k launches), split["drain_s"] = the rest (the
    synchronize waiting for the GPU, and the closing barrier)."""
    if barrier is not None:
        barrier()
    sync()
    t0 = time.perf_counter()
    loop.run(k, first=stamps[0] if stamps else None, last=stamps[1] if stamps else None)
    t1 = time.perf_counter()
    sync()
    if barrier is not None:
        barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = stamps[2](stamps[0], stamps[1]) if stamps else None
    if split is not None:
        split["enqueue_s"], split["drain_s"] = t1 - t0, elapsed - (t1 - t0)
    return elapsed, gpu_ms


def max_over_ranks(values, world, device, collective=None):
    """Elementwise max of a list of floats over ranks (all_reduce MAX; None stays None).
    collective: run the all_reduce even on one rank (the rehearsal, GpuPlatform)."""
    if not (world > 1 if collective is None else collective):
        return values
    import torch
    import torch.distributed as dist
    t = torch.tensor([-1.0 if v is None else float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [None if v is None else float(x) for v, x in zip(values, t.tolist())]


def stream_copy_peak(device, nbytes=1 << 30, iters=20):
    """Achievable HBM bandwidth: scg_stream_copy of nbytes (past every cache), GB/s of
    read + write traffic averaged over `iters` back-to-back copies."""
    import ctypes

    import torch

    from gym_supplychain_amd import _native as nat
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=device).fill_(7)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(device)
    blocks = 0             # one 16-byte vector per lane over the whole buffer (profiles/r03b_copy_probe.log)

    def copy():
        nat.check(nat.lib.scg_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, blocks,
                                          ctypes.c_void_p(stream.cuda_stream)))
    copy()
    torch.cuda.synchronize(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        copy()
    e1.record(stream)
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / iters
    assert bool((dst[:: (1 << 20)] == 7).all())
    del src, dst
    return 2 * nbytes / (ms / 1e3) / 1e9


def beyond_cache_point(device, n_envs=BEYOND_CACHE_ENVS, episodes=2):
    """The bench kernel at n_envs (one step = 272 MB at 2^20 envs, past the 256 MiB
    Infinity Cache): GPU timeline of `episodes` whole episodes after one warm-up episode."""
    import ctypes

    import torch

    from gym_supplychain_amd import BeerGameVecEnv
    from gym_supplychain_amd import _native as nat
    env = BeerGameVecEnv(n_envs, {}, demand="poisson", poisson_lambda=LAMBDA, seed=SEED, device=device,
                         auto_reset=True, track_costs=True, track_history=True, track_returns=True)
    stream = torch.cuda.current_stream(device)
    acts = torch.empty((WEEKS, n_envs, LEVELS), dtype=torch.int32, device=device)
    nat.check(nat.lib.scg_uniform_ints(SEED, 0, n_envs, WEEKS, LEVELS, 0, 0, 8, acts.data_ptr(),
                                       ctypes.c_void_p(stream.cuda_stream)))
    week = list(acts.unbind(0))
    env.reset()
    for _ in range(WEEKS):
        env.step(week[env.week])
    plan = list(env._plan)
    k = episodes * WEEKS
    nbytes = sum(n_envs * step_bytes_per_env(plan[w % WEEKS + 1], w % WEEKS + 1, WEEKS, LEVELS, 2, True, True, True,
                                             True) for w in range(k))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(device)
    e0.record(stream)
    for _ in range(k):
        env.step(week[env.week])
    e1.record(stream)
    torch.cuda.synchronize(device)
    env.check_errors()
    ms = e0.elapsed_time(e1)
    del env, acts, week
    torch.cuda.empty_cache()
    return {"n_envs": n_envs, "steps": k, "avg_kernel_us": ms * 1e3 / k, "bytes_per_launch": nbytes / k,
            "achieved": nbytes / (ms / 1e3) / 1e9, "frac": nbytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS,
            "env_steps_per_s_gpu": n_envs * k / (ms / 1e3)}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3500)
    ap.add_argument("--warmup", type=int, default=350)
    ap.add_argument("--envs", type=int, default=N_ENVS, help="envs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the STREAM peak and beyond-cache point")
    ap.add_argument("--cpu-budget", type=float, default=2.5, help="seconds of CPU-baseline work per process")
    ap.add_argument("--kernel-samples", type=int, default=350,
                    help="launches timed one at a time with kernel-stamped events after the timed region")
    ap.add_argument("--no-dry-region", action="store_true",
                    help="skip the untimed K-step region (sync, K steps, sync) run right before the timed one")
    return ap.parse_args(argv)


class NodeBarrier:
    """The region brackets' barrier for the ranks of one node: they meet on a shared page
    (`_scgpu_fast.node_barrier`, a sense-reversing counter; about a microsecond) instead of an
    RCCL all-reduce plus stream synchronisation (20-60 us on one GPU, profiles/r04o_*), which
    the closing barrier would add to every timed region of an N > 1 line. Rank 0 creates the
    page in /dev/shm and unlinks it once every rank has it mapped, so nothing is left behind
    even if a rank dies. `agree(ok)` (gym_supplychain_amd.distributed.agree) is the setup's
    collective: a step that fails on any rank raises OSError on every rank."""

    def __init__(self, rank, world, agree, timeout_s=600.0):
        import ctypes
        import mmap

        from gym_supplychain_amd import _native as nat
        self.world, self._sense = int(world), 0
        self._timeout_us = int(timeout_s * 1e6)
        self._fast = nat.fast.node_barrier
        path = "/dev/shm/scg_bench_barrier_%s_%s" % (os.environ.get("TORCHELASTIC_RUN_ID", "none"),
                                                      os.environ.get("MASTER_PORT", "0"))
        ok = True
        if rank == 0:
            try:
                try:
                    os.unlink(path)
                except FileNotFoundError:
                    pass
                fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
                os.ftruncate(fd, 64)
                os.close(fd)
            except OSError:
                ok = False
        if not agree(ok):
            raise OSError("the barrier page could not be created")
        try:
            fd = os.open(path, os.O_RDWR)
            try:
                self._mm = mmap.mmap(fd, 64)
            finally:
                os.close(fd)
        except OSError:
            ok = False
        ok = agree(ok)
        if rank == 0:
            os.unlink(path)
        if not ok:
            raise OSError("the barrier page could not be mapped on every rank")
        self._words = (ctypes.c_int32 * 2).from_buffer(self._mm)
        self._addr = ctypes.addressof(self._words)

    def __call__(self):
        if self._sense is None:
            raise RuntimeError("the node barrier timed out earlier; its page is no longer usable")
        try:
            self._sense = self._fast(self._addr, self.world, self._sense, self._timeout_us)
        except TimeoutError:
            # this rank's arrival stays counted on the page and its sense did not advance, so
            # every later barrier on it would release early or never: the page is dropped
            self._sense = None
            raise


class Platform:
    """What the measurement flow needs from the machine: the rank layout, the batch env and
    its resident week actions, the collective device, synchronisation and kernel-stamped
    events. GpuPlatform is the real one; tests/test_bench_distributed.py runs the same flow
    (run()) on gloo ranks with a CPU stand-in."""
    world, rank, device = 1, 0, None
    collectives = False  # barriers, max over ranks and the return all-gather run (world > 1)

    def make_env(self, n_envs, env_offset):
        raise NotImplementedError

    def week_actions(self, env, n_envs):
        raise NotImplementedError

    def sync(self):
        pass

    def barrier(self):
        import torch.distributed as dist
        dist.barrier()

    def new_event(self):
        raise NotImplementedError

    def elapsed_ms(self, start, stop):
        raise NotImplementedError

    def destroy_event(self, ev):
        pass

    def extras(self):
        return {}

    def cpu_baseline(self, budget):
        return cpu_baseline(budget)


class GpuPlatform(Platform):
    def __init__(self):
        import torch
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # SCG_BENCH_PG=1 (under torch.distributed.run, one rank): the process group and every
        # RCCL call of the flow run at N = 1 too, a rehearsal of the multi-GPU path on one GPU
        self.collectives = self.world > 1 or os.environ.get("SCG_BENCH_PG") == "1"
        if self.collectives:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        self.device = torch.device("cuda", local_rank)
        torch.cuda.set_device(self.device)
        from gym_supplychain_amd import _native as nat
        self.nat = nat
        self._node_barrier = None
        if self.collectives:
            from gym_supplychain_amd.distributed import agree
            try:
                self._node_barrier = NodeBarrier(self.rank, self.world, lambda ok: agree(ok, device=self.device))
            except OSError as exc:  # every rank takes the same branch
                print(f"bench: node barrier unavailable ({exc}); using dist.barrier", file=sys.stderr)

    def barrier(self):
        if self._node_barrier is not None:
            self._node_barrier()
        else:
            import torch.distributed as dist
            dist.barrier()

    def make_env(self, n_envs, env_offset):
        from gym_supplychain_amd import BeerGameVecEnv
        return BeerGameVecEnv(n_envs, {}, demand="poisson", poisson_lambda=LAMBDA, seed=SEED, device=self.device,
                              env_offset=env_offset, auto_reset=True, track_costs=True, track_history=True,
                              track_returns=True)

    def week_actions(self, env, n_envs):
        import ctypes

        import torch
        stream = torch.cuda.current_stream(self.device)
        actions = torch.empty((WEEKS, n_envs, LEVELS), dtype=torch.int32, device=self.device)
        self.nat.check(self.nat.lib.scg_uniform_ints(SEED, env.env_offset, n_envs, WEEKS, LEVELS, 0, 0, 8,
                                                     actions.data_ptr(), ctypes.c_void_p(stream.cuda_stream)))
        return list(actions.unbind(0))  # the policy output of each week, resident in HBM

    def sync(self):
        import torch
        torch.cuda.synchronize(self.device)

    def new_event(self):
        return self.nat.hip_event()

    def elapsed_ms(self, start, stop):
        return self.nat.hip_event_elapsed_ms(start, stop)

    def destroy_event(self, ev):
        self.nat.hip_event_destroy(ev)

    def extras(self):
        return {"measured_peak": stream_copy_peak(self.device), "beyond_cache": beyond_cache_point(self.device)}


def run(args, plat):
    """The measurement flow of every rank (module docstring); returns rank 0's JSON line as
    a dict (None on other ranks)."""
    from gym_supplychain_amd.distributed import EpisodeReturnGather, shard_offset
    world, rank, device = plat.world, plat.rank, plat.device
    N = args.envs
    env = plat.make_env(N, shard_offset(N, rank))
    coll = world > 1 or plat.collectives
    gather = EpisodeReturnGather(N, device, collective=coll)
    env.reset()
    loop = StepLoop(env, plat.week_actions(env, N), gather)
    plan = list(env._plan)

    def week_bytes(w):
        return N * step_bytes_per_env(plan[w], w, WEEKS, LEVELS, 2, True, True, True, True)

    def bytes_of(k):  # launches run weeks env.week+1, +2, ... (mod 35)
        w0 = env.week
        return sum(week_bytes((w0 + i) % WEEKS + 1) for i in range(k))

    barrier = plat.barrier if coll else None
    ev = [plat.new_event() for _ in range(4)]

    warmup_run = max(args.warmup, WEEKS)
    loop.run(warmup_run)
    if not args.no_dry_region:  # one untimed region of the same shape (sync, K steps, sync) right
        region(loop, args.steps, world, barrier, plat.sync)  # before: 7.9e9-9.8e9 -> 1.01e10-1.04e10 at K = 20
        warmup_run += args.steps                             # (profiles/r02m_dry_region.log)
    import gc
    gc.disable()  # no collector pass inside a timed region
    try:
        # headline: exactly K steps, unstamped (profiles/r02s_stamped_headline_ab.log)
        split = {}
        elapsed, _ = region(loop, args.steps, world, barrier, plat.sync, split=split)
        gather.result()
        # the fixed cost of a region: the same brackets around zero steps
        empty, _ = region(loop, 0, world, barrier, plat.sync)
        # 100 whole episodes, from an episode boundary
        loop.run((WEEKS - env.week) % WEEKS)
        k_ep = EPISODES_TIMED * WEEKS
        ep_bytes = bytes_of(k_ep)
        ep_elapsed, ep_gpu_ms = region(loop, k_ep, world, barrier, plat.sync, (ev[2], ev[3], plat.elapsed_ms))
        gather.result()
        # isolated launches: whole 35-week cycles, each stamped and run alone
        k_samples = max(WEEKS, args.kernel_samples // WEEKS * WEEKS)
        sampled_bytes = bytes_of(k_samples)
        iso = [(plat.new_event(), plat.new_event()) for _ in range(k_samples)]
        loop.run(k_samples, each=iso, sync_each=plat.sync)
        iso_ms = sum(plat.elapsed_ms(a, b) for a, b in iso)
    finally:
        gc.enable()
    for e in ev + [x for pair in iso for x in pair]:
        plat.destroy_event(e)
    env.check_errors()
    # the last episode end's all-gather against every rank's own returns (a collective)
    gcheck = gather.verify()
    gather.close()
    elapsed, ep_elapsed, ep_gpu_ms, iso_ms, enq_s, drain_s, empty = max_over_ranks(
        [elapsed, ep_elapsed, ep_gpu_ms, iso_ms, split["enqueue_s"], split["drain_s"], empty], world, device, coll)
    extras = plat.extras() if rank == 0 and world == 1 and not args.no_extras else {}
    if rank != 0:
        return None
    achieved = ep_bytes / (ep_gpu_ms / 1e3) / 1e9
    traffic, traffic_src = pmc_traffic(n_envs=N)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
            "kernel": f"scg::{KERNEL} (L = 4, Poisson demand, state slab)",
            "avg_kernel_us": ep_gpu_ms * 1e3 / k_ep,
            "avg_kernel_source": "the 100-episode timed region: first launch's dispatch begin to last launch's "
                                 "end (hipExtLaunchKernel stamps, nothing stamped in between) / launches",
            "bytes_per_launch": ep_bytes / k_ep, "launches_timed": k_ep,
            "isolated_kernel_us": iso_ms * 1e3 / k_samples, "isolated_launches": k_samples,
            "isolated_frac": sampled_bytes / (iso_ms / 1e3) / 1e9 / HBM_PEAK_GBS}
    if "measured_peak" in extras:
        roof["measured_peak"] = extras["measured_peak"]
        roof["frac_measured_peak"] = achieved / extras["measured_peak"]
        roof["measured_peak_source"] = ("scg_stream_copy of 1 GiB (read + write; one non-temporal 16-B "
                                        "vector per lane), 20 launches, same run")
        roof["beyond_cache"] = extras["beyond_cache"]
    line = {
        "metric": "env-steps/sec at 65536 envs/GPU, beergame-v0; 1/2/4/8 MI355X",
        "value": N * world * args.steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warmup_run,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: Poisson(8) demand drawn on device (Philox4x32-10), uniform int [0,8] actions",
        "config": {"workload": "beergame-v0 step() x 65536 envs/GPU (BASELINE configs[1]; configs[4] at N=8)",
                   "n_envs_per_gpu": N, "levels": LEVELS, "weeks": WEEKS, "auto_reset": True,
                   "ledgers": True, "orders_history": True, "episode_return_allgather": coll,
                   "parallelism": f"env-shard x{world}"},
        "episodes_timed": {"episodes": EPISODES_TIMED, "steps": k_ep, "value": N * world * k_ep / ep_elapsed,
                           "ms_per_step": ep_elapsed * 1e3 / k_ep, "avg_kernel_us": ep_gpu_ms * 1e3 / k_ep,
                           "frac": ep_bytes / (ep_gpu_ms / 1e3) / 1e9 / HBM_PEAK_GBS},
        "roofline": roof,
        # what bounds the headline region: the host enqueueing K launches, or the GPU
        # draining them (max over ranks of each part)
        "headline_split": {"host_enqueue_us_per_step": enq_s * 1e6 / args.steps,
                           "drain_after_enqueue_us": drain_s * 1e6,
                           "empty_region_us": empty * 1e6,
                           "gpu_kernel_us_per_step": ep_gpu_ms * 1e3 / k_ep,
                           "bound": "host" if enq_s * 1e6 / args.steps > ep_gpu_ms * 1e3 / k_ep else "gpu"},
        "episode_returns_gathered": gather.gathers,
        # the last gather: slice r == rank r's returns (EpisodeReturnGather.verify); main()
        # exits non-zero when it does not hold
        "allgather_ok": gcheck["allgather_ok"],
        "gather_path": gcheck["gather_path"],
        "allgather_envs_checked": gcheck["envs_checked"],
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = plat.cpu_baseline(args.cpu_budget)
    return line


def main(argv=None):
    args = parse_args(argv)
    plat = GpuPlatform()
    line = run(args, plat)
    if line is not None:
        print(json.dumps(line), flush=True)
    if plat.collectives:
        import torch.distributed as dist
        dist.destroy_process_group()
    if line is not None and not line["allgather_ok"]:
        sys.exit("bench: the episode-return all-gather does not hold every rank's returns in rank order")


if __name__ == "__main__":
    main()
