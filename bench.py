"""Benchmark: BASELINE.json's headline metric on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]

Workload (BASELINE.json configs[2]): Schmidl-Cox [A][A] float32 metric + CFO,
N = 1024 (L = 512), cir1 multipath + AWGN + CFO, 65536 streams x 1024 complex64 samples per
GPU.  One step = one pass of the product's ``sync_aa.AABatchDetector.run`` (one
``ofs_aa_detect`` launch) over the resident batch: P, R, M streams + gate/peak/CFO events.

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) every rank runs its shard;
invoked as ``python bench.py --gpus N`` without torchrun, this process starts
``torch.distributed.run`` with N ranks as a CHILD (before touching the GPU) and exits with its
code.  Streams are independent, so ranks share no data: "weak" (default) gives every rank its
own 65536-stream batch; "strong" splits --global-batch streams over the ranks
(shard.shard_bounds).  Timing: barrier + synchronize on both sides of the K timed steps, MAX
over ranks.

Rank 0 prints one JSON line with `roofline` (dominant kernel vs HBM peak), `cpu_baseline`
(C port of the reference loop + NumPy + literal Python loop on the host cores) and `parity`
(every stream's events against the C oracle, oracle/parity.py criterion).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

from ofdm_sync_amd import shard  # noqa: E402

METRIC = "complex Msamples/s through S&C metric kernel @ batch=65536; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
BYTES_PER_SAMPLE = 8 + 8 + 4 + 4   # read c64 x; write c64 P, f32 R, f32 M
BYTES_PER_STREAM = 4               # n_events
BYTES_PER_EVENT = 64               # 4 x int64 + 4 x f64


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--batch", type=int, default=65536, help="streams per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="streams over all GPUs (strong scaling; default 65536 x gpus)")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--max-events", type=int, default=4)
    ap.add_argument("--placement", choices=("auto", "contiguous", "plain"), default="auto",
                    help="AABatchDetector placement of the detector's buffers (the product default "
                         "'auto'; the JSON line records the placement actually used)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=3.0, help="seconds per CPU leg")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="launcher self-test on CPU (gloo, no HIP): exercises rank start-up, sharding, "
                         "barriers and MAX-of-times; prints the same JSON line with selftest=true")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------
# launcher
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a, argv, script: str | None = None) -> int:
    """Start N ranks of `script` (default: this file) under torch.distributed.run as a child
    process (nothing here has touched the GPU; torch.cuda.device_count() does not initialise
    it on this image)."""
    if not a.selftest_cpu:
        n = torch.cuda.device_count()
        if n < a.gpus:
            raise SystemExit(f"bench.py --gpus {a.gpus}: only {n} GPU(s) visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script or os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


# ------------------------------------------------------------------------------------------
# CPU baseline (reference-equivalent C port, NumPy restatement, literal Python loop) + parity
# ------------------------------------------------------------------------------------------
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share() -> int:
    """Host CPUs this process may use: the scheduler affinity, capped by OMP_NUM_THREADS (the
    GPU box sets 16 = its per-GPU CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, env) if env > 0 else n


def _cgroup_cpus():
    """CPUs the cgroup's quota allows (cgroup v2 cpu.max 'quota period', v1 cfs files), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // per)
    except (OSError, ValueError):
        return None


def _pool_leg(xh, L, form, workers, budget):
    sys_dir = os.path.join(ROOT, "oracle")
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "x.npy")
        n = min(len(xh), 8192 if form == "numpy" else 2048)
        np.save(path, np.ascontiguousarray(xh[:n]))
        out = subprocess.run([sys.executable, os.path.join(sys_dir, "cpu_pool.py"), path, str(L), form,
                              str(workers), str(budget)], capture_output=True, text=True, check=True)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    label = {"numpy": "NumPy restatement (ofdm_oracle.aa_detect: vectorised prefix sums + the reference's "
                      "gate loop, fp64)",
             "loop": "literal per-sample Python loop (ofdm_oracle.aa_detect_loop: the reference's "
                     "DelayLine/RunningSum streaming form, sync_aa.py:458-568)"}[form]
    return dict(value=r["value"], unit="Msamples/s", cores=workers, kind="port",
                sample=f"{r['streams']} stream runs x {r['T']} c64 (cycling over {n} streams of the same batch), "
                       f"L={L}, {label}, "
                       f"pool of {workers} processes, {r['seconds']:.2f} s wall")


def cpu_baseline(det, L: int, threads: int, budget: float):
    """Time the CPU ports on the host cores and check every stream's events against the C
    oracle (parity)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    import parity
    res = det.result
    xh = det.x.cpu().numpy()
    threads = threads if threads > 0 else _cpu_share()
    B, na, T = xh.shape
    oracle_c.aa_detect(xh[:64], L, nthreads=threads)                   # warm (page-in, thread pool)
    # C port: the full batch, repeated to ~budget s of wall time
    reps, dt, r = 0, 0.0, None
    while dt < budget and reps < 50:
        t0 = time.perf_counter()
        r = oracle_c.aa_detect(xh, L, nthreads=threads, max_events=det.max_events, want_arrays=reps == 0)
        dt += time.perf_counter() - t0
        reps += 1
        if reps == 1:
            full = r
    par = parity.classify_aa(res.M.cpu().numpy().astype(np.float64), res.n_events.cpu().numpy(),
                             res.ev_int.cpu().numpy(), res.ev_real.cpu().numpy(), full["P"], full["M"],
                             full["n_events"], full["ev_int"], full["ev_real"], L)
    par["max_abs_err_P_rel_R"] = float(np.max(np.abs(res.P.cpu().numpy() - full["P"]).max(axis=1)
                                              / np.maximum(np.abs(full["R"]).max(axis=1), 1e-30)))
    del full
    out = dict(value=reps * B * T / dt / 1e6, unit="Msamples/s", cores=threads, kind="port",
               sample=f"full per-GPU batch x{reps}: {B} streams x {T} c64 (same synthetic input), L={L}, "
                      f"C restatement of the reference's per-sample loop (oracle/csrc/ofs_oracle.c) with "
                      f"OpenMP over streams, {threads} threads, {dt:.2f} s wall",
               host=dict(cpu_model=_cpu_model(), os_cpu_count=os.cpu_count(),
                         affinity=len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
                         omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                         note="threads = this process's CPU share (affinity capped by OMP_NUM_THREADS; "
                              "the GPU box grants 16 host CPUs per GPU)"))
    # one thread, measured (a single-core rate next to the all-core pool)
    n1 = min(B, 4096)
    reps1, dt1 = 0, 0.0
    while dt1 < min(budget, 2.0) and reps1 < 50:
        t0 = time.perf_counter()
        oracle_c.aa_detect(xh[:n1], L, nthreads=1, max_events=det.max_events)
        dt1 += time.perf_counter() - t0
        reps1 += 1
    out["single_core"] = dict(value=reps1 * n1 * T / dt1 / 1e6, unit="Msamples/s", cores=1, kind="port",
                              sample=f"{n1} streams x {T} c64 x{reps1} (first streams of the same batch), "
                                     f"the same C port on one thread, {dt1:.2f} s wall")
    out["per_core_Msamples_s"] = out["single_core"]["value"]
    # every core the process may run on (one worker per core), beside the per-GPU share:
    # the affinity, capped by the cgroup's CPU quota (cpu.max) - threads beyond the quota only queue
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = _cgroup_cpus()
    n_all = min(n_aff, quota) if quota else n_aff
    out["host"]["cgroup_cpu_quota"] = quota
    out["host"]["loadavg_1m"] = round(os.getloadavg()[0], 2) if hasattr(os, "getloadavg") else None
    if n_all <= threads:
        out["all_cores"] = dict(value=out["value"], unit="Msamples/s", cores=threads, kind="port",
                                sample=f"the per-GPU leg above already uses every CPU this process may run "
                                       f"(affinity {n_aff}, cgroup quota {quota})")
    if n_all > threads:
        oracle_c.aa_detect(xh[:n_all], L, nthreads=n_all)                # warm the larger pool
        reps_a, dt_a = 0, 0.0
        while dt_a < min(budget, 2.0) and reps_a < 50:
            t0 = time.perf_counter()
            oracle_c.aa_detect(xh, L, nthreads=n_all, max_events=det.max_events, want_arrays=False)
            dt_a += time.perf_counter() - t0
            reps_a += 1
        out["all_cores"] = dict(value=reps_a * B * T / dt_a / 1e6, unit="Msamples/s", cores=n_all, kind="port",
                                sample=f"full per-GPU batch x{reps_a}: {B} streams x {T} c64, the same C port with "
                                       f"OpenMP over streams on every CPU of the process's affinity ({n_all} threads; "
                                       f"the box's other GPUs' shares included), {dt_a:.2f} s wall")
    out["numpy"] = _pool_leg(xh, L, "numpy", threads, budget)
    out["literal_loop"] = _pool_leg(xh, L, "loop", threads, budget)
    out["other_configs"] = other_config_baselines(threads, budget)
    return out, par


def other_config_baselines(workers: int, budget: float):
    """CPU rates of BASELINE.json's other configs: the NumPy restatement of each
    config's path on seeded synthetic streams of its shape, pool of `workers` processes
    (oracle/cpu_pool.py --config).  GPU rates of the same configs: tools/bench_configs.py."""
    res = {}
    for name in ("cfg2a", "cfg2b", "cfg4", "cfg5"):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_pool.py"), "--config", name,
                            str(workers), str(budget)], capture_output=True, text=True, check=True)
        r = json.loads(p.stdout.strip().splitlines()[-1])
        res[name] = dict(value=round(r["value"], 3), unit="Msamples/s", cores=workers, kind="port",
                         sample=f"{r['streams']} streams x {r['samples'] // max(r['streams'], 1)} samples, {r['form']}, "
                                f"pool of {workers} processes, {r['seconds']:.2f} s wall")
    return res


# ------------------------------------------------------------------------------------------
# measurement
# ------------------------------------------------------------------------------------------
def kernel_label(plan: int) -> str:
    if plan >= 1000:
        e, mr = (plan - 1000) // 10, (plan - 1000) % 10
        kind = "streaming" if plan >= 1100 else "register-staged"
        cap = ", 10 workgroups per CU" if plan < 1100 else ""
        return f"aa_fast_kernel<E={e},MR={mr}> (wave per stream, {kind}, fused metric + events{cap})"
    return {1: "win_kernel<C64,fp32,AA> (fused events)", 2: "win_kernel<C64,fp32,AA> + aa_events_kernel"}.get(plan, str(plan))


def pmc_traffic(workload_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one exists for this
    workload (collected in separate --pmc passes, corrected per MI355X_MICROARCH.md §HBM)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        e = d.get(workload_key)
        return None if e is None else e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


class _SelftestDetector:
    """--selftest-cpu stand-in for the HIP detector: a rank-dependent sleep, so MAX-over-ranks
    is observable.  Never used without --selftest-cpu."""

    def __init__(self, rank):
        self.delay = 0.002 * (rank + 1)

    def run(self):
        time.sleep(self.delay)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)
    info = shard.rank_info()
    rank, world, local = info.rank, info.world, info.local_rank
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    B_glob = a.global_batch or a.batch * world
    if a.scaling == "weak":
        B, lo = a.batch, rank * a.batch
        B_glob = a.batch * world
    else:
        lo, hi = shard.shard_bounds(B_glob, rank, world)
        B = hi - lo
    T, L, E = a.T, a.L, a.max_events

    if a.selftest_cpu:
        dev = torch.device("cpu")
        dist = shard.init("gloo")
        det = _SelftestDetector(rank)
        step = det.run
        sync = lambda: None                                     # noqa: E731
    else:
        from ofdm_sync_amd import sync_aa, synth
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        dist = shard.init("nccl", dev)          # RCCL; control plane only (barrier + MAX of times)
        det = sync_aa.AABatchDetector(B, T, 1, L, precision="fp32", outputs=("P", "R", "M"), max_events=E,
                                      placement=a.placement, device=dev)
        # synthetic shard: per-rank seed = the stream range it owns (weak: fresh streams per rank)
        det.x.copy_(synth.headline_batch(B, T, L, seed=shard.shard_seed(2026, rank), device=dev))
        torch.cuda.empty_cache()
        stream = torch.cuda.current_stream(dev)
        step = det.run
        sync = torch.cuda.synchronize

    for _ in range(a.warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    t_host0 = time.perf_counter()
    if not a.selftest_cpu:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
    for _ in range(a.steps):
        step()
    if not a.selftest_cpu:
        e1.record(stream)
    sync()
    t_host = time.perf_counter() - t_host0
    ms = t_host * 1e3 if a.selftest_cpu else e0.elapsed_time(e1)
    if dist:
        dist.barrier()
    ms_max = shard.max_over_ranks(ms, dist, dev)
    ms_per_step = ms_max / a.steps
    census = shard.rank_census(dist, dev, ms, (lo, lo + B))     # ranks the collective saw, per-rank device + ms
    if census["ranks_seen"] != world or not census["distinct_devices"]:
        raise SystemExit(f"bench.py: rank census disagrees with WORLD_SIZE={world}: {census}")

    total_samples = B_glob * T * a.steps
    value = total_samples / (ms_max / 1e3) / 1e6
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "f32 (c64 in, f64 prefix sums)",
        "data": "synthetic (ofs_synth_frames on the GPU): per-stream sync_aa.run_single_test frames - [A][A] "
                "ZC preamble + own random-QPSK pilot/data symbols, * cir1 RX ch1 (1100 taps) + AWGN U[0,15] dB + "
                "CFO U[-5,5] kHz @ 15.36 MHz; 1024-sample window at a random offset around the preamble",
        "config": {"workload": "cfg3 Schmidl-Cox float32 metric+CFO, N=1024 (L=512), cir1, "
                               f"{B} streams x {T} c64 per GPU",
                   "global_batch": B_glob, "seq_len": T, "L": L,
                   "parallelism": f"stream-shard x{world} (no collectives)",
                   "placement": a.placement if a.selftest_cpu else f"{a.placement} -> {det.placement}"},
        "ranks_seen": census["ranks_seen"],
        "rank_devices": [r["device"] for r in census["ranks"]],
        "rank_ms": [r["ms"] for r in census["ranks"]],
        "rank_shards": [r["shard"] for r in census["ranks"]],
    }
    if a.selftest_cpu:
        out.update(selftest=True, shard=[lo, lo + B])
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return 0

    res = det.result
    stored = int(torch.clamp(res.n_events, max=E).sum().item())
    alg_bytes = B * T * BYTES_PER_SAMPLE + B * BYTES_PER_STREAM + stored * BYTES_PER_EVENT
    launch_s = (ms / a.steps) / 1e3                       # this rank's average launch duration
    achieved = alg_bytes / launch_s / 1e9
    out["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                       "traffic": pmc_traffic(f"aa_fp32_B{B}_T{T}_L{L}"),
                       "kernel": kernel_label(det.plan()), "alg_bytes_per_launch": alg_bytes,
                       "avg_launch_ms": round(ms / a.steps, 5)}
    out["events_per_stream"] = round(float(res.n_events.float().mean().item()), 3)
    out["host_wall_s"] = round(t_host, 4)
    if rank == 0:
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"], out["parity"] = cpu_baseline(det, L, a.cpu_threads, a.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
