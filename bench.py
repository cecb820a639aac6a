"""Benchmark: BASELINE.json's headline metric on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload (BASELINE.json configs[2]): Schmidl-Cox [A][A] float32 metric + CFO,
N = 1024 (L = 512), cir1 multipath + AWGN + CFO, 65536 streams x 1024 complex64 samples per
GPU (weak scaling: each rank runs its own shard, no data-path collective).  One step = one
pass of ofs_aa_detect over the resident batch: P, R, M streams + gate/peak/CFO events.

Prints one JSON line (rank 0) with `roofline` (dominant kernel vs HBM peak) and
`cpu_baseline` (the C port of the reference loop, oracle/csrc, on the host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

from ofdm_sync_amd import _lib, shard, synth  # noqa: E402

METRIC = "complex Msamples/s through S&C metric kernel @ batch=65536; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
BYTES_PER_SAMPLE = 8 + 8 + 4 + 4   # read c64 x; write c64 P, f32 R, f32 M
BYTES_PER_STREAM = 4               # n_events
BYTES_PER_EVENT = 64               # 4 x int64 + 4 x f64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=65536, help="streams per GPU")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--max-events", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--alloc", choices=("contiguous4", "contiguous", "plain"), default="contiguous4",
                    help="batch backing: one physically contiguous block per stream (x, P, R, M), one "
                         "contiguous arena for all four, or one plain allocation")
    return ap.parse_args()


def cpu_baseline(x_dev: torch.Tensor, L: int, threads: int, gpu_M: torch.Tensor):
    """Time the C port of the reference's streaming loop (oracle/csrc/ofs_oracle.c) on the
    host cores over the full batch, repeated to ~1 s of wall time.  Also spot-checks the GPU
    metric against it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c
    xh = x_dev.cpu().numpy()
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    B, na, T = xh.shape
    oracle_c.aa_detect(xh[:64], L, nthreads=threads)          # warm (page-in, thread pool)
    # repeat the full batch until ~1 s of wall time (>= ~10 s of CPU work at 16 threads)
    reps, dt = 0, 0.0
    while dt < 1.0 and reps < 50:
        t0 = time.perf_counter()
        r = oracle_c.aa_detect(xh, L, nthreads=threads, max_events=4)
        dt += time.perf_counter() - t0
        reps += 1
    idx = np.linspace(0, B - 1, 16).astype(int)
    err = float(np.max(np.abs(gpu_M[idx].cpu().numpy() - r["M"][idx])))
    cores = os.cpu_count()
    return dict(value=reps * B * T / dt / 1e6, unit="Msamples/s", cores=threads, kind="port",
                sample=f"full per-GPU batch x{reps}: {B} streams x {T} c64 (same synthetic input), "
                       f"L={L}, C restatement of sync_aa.aa_detect_streaming with OpenMP over "
                       f"streams, {threads} threads of {cores} host CPUs, {dt:.2f} s wall",
                max_abs_err_M_vs_gpu=err, numpy=numpy_baseline(xh, L))


def numpy_baseline(xh: np.ndarray, L: int, budget_s: float = 3.0):
    """The NumPy restatement of the path (oracle/ofdm_oracle.aa_detect: vectorised prefix sums +
    the reference's gate loop), one process, streams of the same batch one after another until
    ~budget_s of wall time: the north star's "NumPy CPU path" beside the C port."""
    import ofdm_oracle
    B, _, T = xh.shape
    ofdm_oracle.aa_detect(xh[0].astype(np.complex128), L)                 # warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n < B:
        ofdm_oracle.aa_detect(xh[n].astype(np.complex128), L)
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n * T / dt / 1e6, unit="Msamples/s", cores=1, kind="port",
                sample=f"{n} streams x {T} c64 of the same batch, L={L}, NumPy restatement "
                       f"(ofdm_oracle.aa_detect, fp64), one process, {dt:.2f} s wall")


def kernel_label(plan: int) -> str:
    if plan >= 1000:
        e, mr = (plan - 1000) // 10, (plan - 1000) % 10
        return f"aa_fast_kernel<E={e},MR={mr}> (wave per stream, register-staged, fused metric + events)"
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


def main():
    a = parse()
    info = shard.rank_info()
    rank, world, local = info.rank, info.world, info.local_rank
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = shard.init("nccl", dev)          # RCCL; control plane only (barrier + MAX of times)

    # weak scaling: every rank owns its own B-stream shard (independent streams)
    B, T, L, E = a.batch, a.T, a.L, a.max_events
    # input and outputs of one batch: each stream in its own physically contiguous block
    # (default), one arena, or plain; the synthetic batch is generated, then copied in
    specs = [((B, 1, T), torch.complex64), ((B, T), torch.complex64), ((B, T), torch.float32),
             ((B, T), torch.float32)]
    alloc = a.alloc
    try:
        if alloc == "contiguous4":          # 0.267-0.272 vs 0.298-0.300 ms (one arena)
            x, P, R, M = [_lib.arena(dev, [sp], contiguous=True)[0] for sp in specs]
        else:
            x, P, R, M = _lib.arena(dev, specs, contiguous=alloc == "contiguous")
    except MemoryError:                     # the driver could not back it contiguously
        alloc = "plain (contiguous refused)"
        x, P, R, M = _lib.arena(dev, specs, contiguous=False)
    x.copy_(synth.make_aa_batch(B, T, L, seed=shard.shard_seed(2026, rank), device=dev))
    torch.cuda.empty_cache()
    n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    lib = _lib.lib()
    stream = torch.cuda.current_stream(dev)
    args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(),
            None, 1, 0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(),
            stream.cuda_stream)
    fn = lib.ofs_aa_detect

    def step():
        rc = fn(*args)
        if rc:
            raise RuntimeError(f"ofs_aa_detect failed: {rc}")

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t_host0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    t_host = time.perf_counter() - t_host0
    if dist:
        dist.barrier()
    ms = e0.elapsed_time(e1)
    ms_max = shard.max_over_ranks(ms, dist, dev)
    ms_per_step = ms_max / a.steps

    # algorithmic bytes of one launch
    stored = int(torch.clamp(n_ev, max=E).sum().item())
    alg_bytes = B * T * BYTES_PER_SAMPLE + B * BYTES_PER_STREAM + stored * BYTES_PER_EVENT
    launch_s = (ms / a.steps) / 1e3                       # this rank's average launch duration
    achieved = alg_bytes / launch_s / 1e9
    workload_key = f"aa_fp32_B{B}_T{T}_L{L}"
    traffic = pmc_traffic(workload_key)

    total_samples = world * B * T * a.steps
    value = total_samples / (ms_max / 1e3) / 1e6
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (c64 in, f64 prefix sums)",
            "data": "synthetic (ofs_synth_batch on the GPU): [A][A] ZC preamble (sync_aa.build_aa_preamble "
                    "restated) * cir1 ch1 + AWGN U[0,15] dB + CFO U[-5,5] kHz @ 15.36 MHz, random window offset",
            "config": {"workload": "cfg3 Schmidl-Cox float32 metric+CFO, N=1024 (L=512), cir1, "
                                   f"{B} streams x {T} c64 per GPU",
                       "global_batch": world * B, "seq_len": T, "L": L,
                       "parallelism": f"stream-shard x{world} (no collectives)", "alloc": alloc},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": kernel_label(lib.ofs_aa_plan(_lib.C64, _lib.FP32, 1, T, L)),
                         "alg_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(ms / a.steps, 5)},
            "events_per_stream": round(float(n_ev.float().mean().item()), 3),
            "host_wall_s": round(t_host, 4),
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(x, L, a.cpu_threads, M)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
