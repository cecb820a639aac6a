"""Secondary BASELINE.json configurations (cfg2, cfg4, cfg5, ...), one GPU or N.

bench.py measures the headline (cfg3).  This script times the other configs named in
BASELINE.json with the same method (warm-up, then K launches bracketed by HIP events on the
launch stream, inputs resident in HBM) and prints one JSON line per config with the
algorithmic bytes per launch and the achieved fraction of the
8 TB/s HBM peak.  Synthetic inputs of the config's shape; not the driver's headline line.

Multi-GPU (BASELINE configs[3] "262144 streams sharded across 8 x MI355X", configs[4] "1M
sequences, 1 -> 8 GPU scaling"): ``--gpus N`` starts N ranks (torch.distributed.run child,
as bench.py); cfg4 / cfg5 / cfg5_rocfft are STRONG-scaled: the fixed global batch
(--cfg4-global, --cfg5-global) is split by shard.shard_bounds, each rank runs its shard with
no data-path collective, the timed region is bracketed by a barrier and the reported time is
the MAX over ranks; value = global samples / that time.  The other configs run per rank
(weak) and are reported by rank 0.

    python tools/bench_configs.py [--configs cfg2a,cfg2b,cfg4,cfg5] [--steps K] [--warmup W] [--gpus N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ofdm_sync_amd import _lib, shard, synth, zc_freq  # noqa: E402
if os.environ.get("OFS_LIB"):   # a tools/variants.py tuning build, named explicitly (not a product switch)
    _lib.use_tuning_library(os.environ["OFS_LIB"])

HBM = 8000.0
VPEAK = {"fp32": 157.3, "fp64": 78.6}    # MI355X vector FMA peaks, TFLOP/s (spec; no MFMA: no contraction)
_DIST = None                     # torch.distributed when run with N ranks (barrier before timing)
_LAST_HOST_MS = None             # host time per step of the last timed() (enqueue only; > ms = host-bound)


WARM_MS = 100.0      # untimed calls continue until this much wall time has passed (clock ramp)


def timed(step, steps, warmup, stream):
    """HIP events over `steps` calls after `warmup` untimed calls, continued until WARM_MS of wall
    time have passed: sub-millisecond kernels reach steady clocks only after some tens of ms of load
    (zc_freq_refshape 0.62 ms after 5 calls vs 0.553 ms steady, tools/lib_ab.py rounds)."""
    step()                          # first call: plan creation / lazy set-up outside the warm-up clock
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    n = 1
    while n < warmup or (time.perf_counter() - t_w) * 1e3 < WARM_MS:
        step()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    if _DIST is not None:
        _DIST.barrier()
        torch.cuda.synchronize()
    global _LAST_HOST_MS
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _LAST_HOST_MS = (time.perf_counter() - t0) * 1e3 / steps      # host time to enqueue one step
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def batch_arena(dev, specs, contiguous):
    """Input + outputs of a config in one allocation; physically contiguous where measured
    faster (cfg5: 6.05 vs 6.14 ms; cfg4 is the opposite - 1.41 vs 0.69-0.75 ms with its 7
    streams - and keeps separate allocations),
    falling back to a plain allocation if the driver cannot provide a contiguous one."""
    if contiguous:
        try:
            return _lib.arena(dev, specs, contiguous=True)
        except MemoryError:
            pass
    return _lib.arena(dev, specs, contiguous=False)


def dbuf(dev, shape, dtype):
    """A config buffer: its own physically contiguous block when OFS_BENCH_ALLOC=contig (the
    headline's layout since r01i), else a plain torch allocation."""
    if os.environ.get("OFS_BENCH_ALLOC", "plain") == "contig":
        try:
            return _lib.arena(dev, [(tuple(shape), dtype)], contiguous=True)[0]
        except MemoryError:
            pass
    return torch.empty(shape, dtype=dtype, device=dev)


def dput(dev, t):
    """Move an input batch into a dbuf."""
    b = dbuf(dev, t.shape, t.dtype)
    b.copy_(t)
    return b


def chk(rc, what):
    if rc:
        raise RuntimeError(f"{what}: status {rc}")


def int12(x):
    s = 2046.0 / float(x.abs().amax())
    re = torch.clamp(torch.round(x.real * s), -2048, 2047).to(torch.int16)
    im = torch.clamp(torch.round(x.imag * s), -2048, 2047).to(torch.int16)
    return torch.stack([re, im], dim=-1).contiguous()


def packed(x):
    """int16 I/Q [B, n_ch, T, 2] (device) -> packed 12-bit AXIS words [B, T, 3 n_ch] (OFS_CP12)."""
    from ofdm_sync_amd import wire
    return torch.from_numpy(wire.pack_axis(x.cpu().numpy())).to(x.device)


def cfg2a(dev, st, steps, warmup, cp12=False):
    """cfg2 (aa side): sync_aa detector, L=128, int12 I/Q, B=4096 x T=1024, fp64 (bit-exact);
    cp12: the same samples as packed 12-bit AXIS words (3 B/sample instead of 4)."""
    B, T, L = 4096, 1024, 128
    x = int12(synth.make_aa_batch(B, T, L, seed=7, device=dev))
    x = dput(dev, packed(x) if cp12 else x)
    P = dbuf(dev, (B, T), torch.complex128)
    R = dbuf(dev, (B, T), torch.float64)
    M = dbuf(dev, (B, T), torch.float64)
    V = dbuf(dev, (B, T), torch.uint8)
    E = 4
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    fmt = _lib.CP12 if cp12 else _lib.CI16
    args = (fmt, x.data_ptr(), B, 1, T, L, _lib.FP64, P.data_ptr(), R.data_ptr(), M.data_ptr(),
            V.data_ptr(), 1, 0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(),
            st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_aa_detect(*args), "aa"), steps, warmup, st)
    insz = 3 if cp12 else 4
    nbytes = B * T * (insz + 16 + 8 + 8 + 1)
    plan = L_.ofs_aa_plan(fmt, _lib.FP64, 1, T, L)
    kernel = (f"aa_exact_kernel<E={(plan - 2000) // 10},MR={plan % 10}> (integer-exact, wave per stream, "
              "fused events)" if plan > 2000 else "win_kernel<CI16,fp64,AA> (fused events)")
    return dict(config="cfg2a_cp12" if cp12 else "cfg2a",
                workload=f"sync_aa detector L={L}, int12 {'packed AXIS words' if cp12 else 'I/Q'}, {B} x {T}, fp64",
                kernel=kernel, samples=B * T, ms=ms, alg_bytes=nbytes,
                bytes_per_sample=f"{insz} in + P 16 + R 8 + M 8 + valid 1")


def cfg2b(dev, st, steps, warmup, cp12=False, B=4096):
    """cfg2 (minn_rtl side): Q=64, int12 I/Q, B=4096 x T=1024, fused IIR + threshold + gate;
    cp12: packed 12-bit AXIS words.  B: batch sweep (``--configs cfg2b@B=65536``)."""
    T, Q = 1024, 64
    x = int12(synth.make_aa_batch(B, T, 128, seed=9, device=dev))
    if cp12:
        x = packed(x)
    f = lambda: torch.empty((B, T), dtype=torch.float64, device=dev)   # noqa: E731
    b = lambda: torch.empty((B, T), dtype=torch.bool, device=dev)      # noqa: E731
    o = [f(), f(), f(), f(), f(), f(), b(), b()]
    E = 16
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    og = torch.empty(B, dtype=torch.int64, device=dev)
    L_ = _lib.lib()
    parts = os.environ.get("OFS_CFG2B_PARTS", "full")       # diagnostic: metric | smooth | full
    ptrs = [t.data_ptr() for t in o]
    if parts == "metric":
        ptrs = [ptrs[0], ptrs[1], None, ptrs[3], None, ptrs[5], ptrs[6], None]
    det = 0 if parts in ("metric", "smooth") else 1
    fmt = _lib.CP12 if cp12 else _lib.CI16
    smode = int(os.environ.get("OFS_CFG2B_MODE", "0"))     # 1: the RTL floor-shift smoothing
    args = (fmt, x.data_ptr(), B, 1, T, Q, 3, smode, 3276, 15, *ptrs, det, 2, 0, E,
            n_ev.data_ptr(), ev.data_ptr(), og.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_minn_rtl(*args), "minn_rtl"), steps, warmup, st)
    insz = 3 if cp12 else 4
    nbytes = B * T * (insz + 6 * 8 + 2)
    plan = L_.ofs_rtl_plan(fmt, 1, T, Q)
    kernel = (f"rtl_exact_kernel<E={(plan - 2000) // 10},MW={plan % 10}> (integer-exact metric + in-wave "
              "IIR + closed-form gate)" if plan else "win_kernel<CI16,fp64,RTL> + rtl_iir_kernel")
    return dict(config=("cfg2b_cp12" if cp12 else "cfg2b") + ("" if B == 4096 else f"@B={B}"),
                workload=f"minn_rtl Q={Q}, int12 {'packed AXIS words' if cp12 else 'I/Q'}, {B} x {T}, fp64 + "
                         "sequential IIR/gate",
                kernel=kernel, samples=B * T, ms=ms, alg_bytes=nbytes,
                bytes_per_sample=f"{insz} in + 6 x f64 8 + 2 flags")


def cfg4(dev, st, steps, warmup, B=32768, seed=4):
    """cfg4: combined S&C (both-halves R) + Minn, N=2048, B x 4096 c64, fp32 (B = this rank's
    shard of the global 262144 streams)."""
    T, N = 4096, 2048
    x = dput(dev, synth.make_aa_batch(B, T, N // 2, seed=seed, device=dev))
    n_out = T - N + 1
    outs = [dbuf(dev, (B, n_out), dt) for dt in (torch.float32, torch.complex64, torch.float32) * 2]
    L_ = _lib.lib()

    fused = os.environ.get("OFS_CFG4_SEPARATE", "0") != "1"

    def step():
        if fused:
            chk(L_.ofs_sc_minn_metric(_lib.C64, x.data_ptr(), B, 1, T, N, _lib.FP32,
                                      *[t.data_ptr() for t in outs], st.cuda_stream), "sc_minn")
            return
        chk(L_.ofs_sc_metric(_lib.C64, x.data_ptr(), B, 1, T, N, 1, _lib.FP32, outs[0].data_ptr(),
                             outs[1].data_ptr(), outs[2].data_ptr(), st.cuda_stream), "sc")
        chk(L_.ofs_minn_metric(_lib.C64, x.data_ptr(), B, 1, T, N, _lib.FP32, outs[3].data_ptr(),
                               outs[4].data_ptr(), outs[5].data_ptr(), st.cuda_stream), "minn")
    ms = timed(step, steps, warmup, st)
    nbytes = B * T * 8 + 2 * B * n_out * 16
    return dict(config="cfg4", workload=f"combined_sc_min S&C + Minn, N={N}, {B} x {T} c64 per GPU, fp32",
                kernel=("sc_minn_fast_kernel (fused, one pass)" if fused else
                        "win_fast_kernel<COMB> + win_fast_kernel<MINN>"), samples=B * T, ms=ms,
                alg_bytes=nbytes, bytes_per_sample="8 in (once) + 2 x (M 4 + P 8 + R 4) per output")


def cfg5(dev, st, steps, warmup, n_seq=1 << 20, seed=5):
    """cfg5: zc_freq metric, N=4096, one window per sequence (cp=0), n_seq sequences x 4096 c64
    (n_seq = this rank's shard of the global 1M)."""
    N = 4096
    g = torch.Generator(device=dev).manual_seed(seed)
    prec = int(os.environ.get("OFS_CFG5_PREC", "0"))           # 0 fp32 window FFT, 1 fp64 sliding DFT
    x, out = batch_arena(dev, [((n_seq, N), torch.complex64),
                               ((n_seq, 1), torch.float32 if prec == 0 else torch.float64)], contiguous=True)
    for i in range(0, n_seq, 1 << 17):                          # fill in chunks (no 32 GiB temporary)
        x[i:i + (1 << 17)].copy_(torch.randn((min(1 << 17, n_seq - i), N), dtype=torch.complex64, device=dev,
                                             generator=g))
    idx, t, e = zc_freq.make_pss_frequency_template()
    idx32 = np.ascontiguousarray(idx.astype(np.int32))
    tb = np.ascontiguousarray(t.astype(np.complex128))
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), n_seq, 1, N, N, 0, prec, 62, idx32.ctypes.data, tb.ctypes.data, e,
            out.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_zc_freq_metric(*args), "zc_freq"), steps, warmup, st)
    nbytes = n_seq * (N * 8 + (4 if prec == 0 else 8))
    plan = L_.ofs_zc_freq_plan(_lib.C64, prec, N, N, 0)
    kernel = {1: "zc_freq_kernel (fp64 sliding DFT)", 2: "zc_win_kernel<64> (fp32 window FFT, LDS transpose)",
              3: "zc_win64_kernel (fp32 window FFT, lane reduce-scatter, LDS-DMA prefetch)"}.get(plan, str(plan))
    return dict(config="cfg5", workload=f"zc_freq 62-bin metric, N={N}, cp=0, {n_seq} sequences x {N} c64",
                kernel=kernel,
                samples=n_seq * N, ms=ms, alg_bytes=nbytes,
                bytes_per_sample="8 in + 4|8 B per sequence out")


def backend(dev, st, steps, warmup, B=16384, N=2048, n_used=1200, name="backend"):
    """Receiver back-end (sc.py:274-311 chain) over a batch of frames: 2 branches, N = 2048,
    CP = min(N/4, 512), c64 input; CP CFO, two N-point FFTs, LS, phase-slope STO, EQ, EVM per frame."""
    from ofdm_sync_amd import core
    nb, cp = 2, min(N // 4, 512)                                # the fast kernel's cp <= 512
    T = 2 * (N + cp) + 64
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    k = core.centered_subcarrier_indices(n_used)
    U = k.size
    ps = torch.full((B,), 32, dtype=torch.int64, device=dev)
    ds = ps + N + cp
    pil = torch.ones((U,), dtype=torch.complex128, device=dev)
    kb = torch.as_tensor(k.astype(np.int32)).to(dev)
    outs = [torch.empty((B,), dtype=torch.float64, device=dev) for _ in range(5)]
    h = torch.empty((B, U), dtype=torch.complex128, device=dev)
    xa = torch.empty_like(h)
    gain = torch.empty((B,), dtype=torch.complex128, device=dev)
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), B, nb, T, N, cp, 30.72e6, ps.data_ptr(), ds.data_ptr(), None, U, kb.data_ptr(),
            pil.data_ptr(), 0, pil.data_ptr(), 0, outs[0].data_ptr(), h.data_ptr(), xa.data_ptr(), gain.data_ptr(),
            outs[1].data_ptr(), outs[2].data_ptr(), outs[3].data_ptr(), outs[4].data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_rx_backend(*args), "rx_backend"), steps, warmup, st)
    nbytes = B * (nb * (2 * N + 2 * cp) * 8 + 2 * U * 16 + 5 * 8 + 16)
    # fp64 flops per frame (DESIGN.md §7 back-end roofline): CP correlation 8 per branch-sample;
    # two windows: per branch a complex tone product + accumulate (8) and the tone rotation (6) per
    # sample; two radix-2 FFTs 5 N log2 N; per used bin: two numpy divisions (11 each), unwrap +
    # fit (~12), vdot / EVM sums and the gain product (~20)
    lg = int(np.log2(N))
    flops = 8 * cp * nb + 2 * (N * nb * 8 + N * 6) + 2 * 5 * N * lg + U * (11 + 11 + 12 + 20)
    return _flops(dict(config=name,
                       workload=f"receiver back-end, {B} frames x {nb} branches, N={N}, CP={cp}, c64 in, fp64",
                       kernel=f"rx_backend_fast_kernel<SPT={N // 256}> (LDS FFTs, one workgroup per frame)", samples=B * nb * 2 * N,
                       ms=ms, alg_bytes=nbytes, bytes_per_sample="windows read once (8 B) + 2 x 16 B per used bin out",
                       frames_per_s=round(B / (ms / 1e3), 1), flops_per_frame=flops), B * flops, "fp64")


def cfg3_2ant(dev, st, steps, warmup):
    """cfg3 with two receive antennas per stream (sync_aa's run_single_test uses 2 RX): 65536 x
    2 x 1024 c64, L=512, fp32 fast path, events fused."""
    B, T, L, E = 65536, 1024, 512, 4
    x = dput(dev, synth.synth_batch(synth.faded_base(L, "cir1", (0, 1)), B, T, seed=32, device=dev))
    P = dbuf(dev, (B, T), torch.complex64)
    R = dbuf(dev, (B, T), torch.float32)
    M = dbuf(dev, (B, T), torch.float32)
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), B, 2, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_aa_detect(*args), "aa 2ant"), steps, warmup, st)
    plan = L_.ofs_aa_plan(_lib.C64, _lib.FP32, 2, T, L)
    return dict(config="cfg3_2ant", workload=f"sync_aa S&C fp32, L={L}, {B} streams x 2 antennas x {T} c64",
                kernel=f"aa_fast_kernel<E={(plan - 1000) // 10},MR={plan % 10},NA=2>" if plan >= 1000 else str(plan),
                samples=B * 2 * T, ms=ms, alg_bytes=B * T * (16 + 16) + B * 4,
                bytes_per_sample="2 x 8 in + P 8 + R 4 + M 4 per time index")


def cfg4_2br(dev, st, steps, warmup):
    """cfg4 with two receive branches per stream (combined_sc_min.run_simulation feeds cir1[:2]):
    16384 x 2 x 4096 c64, N = 2048, fused S&C + Minn."""
    B, T, N = 16384, 4096, 2048
    x = dput(dev, synth.synth_batch(synth.faded_base(N // 2, "cir1", (0, 1)), B, T, seed=42, device=dev))
    n_out = T - N + 1
    outs = [dbuf(dev, (B, n_out), dt) for dt in (torch.float32, torch.complex64, torch.float32) * 2]
    L_ = _lib.lib()
    ms = timed(lambda: chk(L_.ofs_sc_minn_metric(_lib.C64, x.data_ptr(), B, 2, T, N, _lib.FP32,
                                                 *[t.data_ptr() for t in outs], st.cuda_stream), "sc_minn 2br"),
               steps, warmup, st)
    return dict(config="cfg4_2br", workload=f"combined_sc_min S&C + Minn, N={N}, {B} x 2 branches x {T} c64, fp32",
                kernel="sc_minn_fast_kernel<NB=2> (fused, one pass)", samples=B * 2 * T, ms=ms,
                alg_bytes=B * 2 * T * 8 + 2 * B * n_out * 16, bytes_per_sample="2 x 8 in + 2 x 16 per output")


def cfg3_fp64(dev, st, steps, warmup):
    """cfg3 shape in the reference's float64 (complex128 in, f64/c128 out: the numpy drop-in's
    precision), 65536 x 1024, L = 512, events fused."""
    B, T, L, E = 65536, 1024, 512, 4
    x = dput(dev, synth.make_aa_batch(B, T, L, seed=33, device=dev, dtype=torch.complex128))
    P = dbuf(dev, (B, T), torch.complex128)
    R = dbuf(dev, (B, T), torch.float64)
    M = dbuf(dev, (B, T), torch.float64)
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    args = (_lib.C128, x.data_ptr(), B, 1, T, L, _lib.FP64, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_aa_detect(*args), "aa fp64"), steps, warmup, st)
    plan = L_.ofs_aa_plan(_lib.C128, _lib.FP64, 1, T, L)
    return dict(config="cfg3_fp64", workload=f"sync_aa S&C fp64, L={L}, {B} x {T} c128", kernel=f"plan {plan}",
                samples=B * T, ms=ms, alg_bytes=B * T * (16 + 16 + 8 + 8) + B * 4,
                bytes_per_sample="16 in + P 16 + R 8 + M 8")


def cfg5_rocfft(dev, st, steps, warmup, n_seq=1 << 20, seed=5, pruned=None, chunked=False):
    """cfg5 through the rocFFT leg (ofs_zc_freq_metric_fft: batched rocFFT of every window into a
    dense spectrum, then the HIP gather/metric kernel and the per-sequence argmax), same input as
    cfg5.  alg_bytes counts the same 8 B/sample + output as cfg5 so Msamples/s and frac compare
    directly; the path itself also writes and re-reads the spectrum (traffic_bytes)."""
    N = 4096
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.empty((n_seq, N), dtype=torch.complex64, device=dev)
    for i in range(0, n_seq, 1 << 17):
        x[i:i + (1 << 17)].copy_(torch.randn((min(1 << 17, n_seq - i), N), dtype=torch.complex64, device=dev,
                                             generator=g))
    if pruned is None:
        pruned = True
    idx, t, e = zc_freq.make_pss_frequency_template()
    idx32 = np.ascontiguousarray(idx.astype(np.int32))
    tb = np.ascontiguousarray(t.astype(np.complex128))
    nb_ = len(idx32)
    chunk = 0
    if chunked:
        chunk = int(os.environ.get("OFS_ZC_FFT_CHUNK", "0")) or zc_freq.default_chunk(n_seq, 1, N, 8)
    plan = zc_freq.FFTPlan(_lib.FP32, N, n_seq, N, nb_ if pruned else 0, min(chunk, n_seq))
    spec = torch.empty((plan.chunk, nb_ if pruned else N), dtype=torch.complex64, device=dev)
    out = torch.empty((n_seq, 1), dtype=torch.float32, device=dev)
    pk = torch.empty((n_seq,), dtype=torch.int64, device=dev)
    work = torch.empty((max(plan.work_bytes, 1),), dtype=torch.uint8, device=dev) if plan.work_bytes else None
    L_ = _lib.lib()
    args = (plan.handle, _lib.C64, x.data_ptr(), n_seq, 1, N, N, 0, 62, idx32.ctypes.data, tb.ctypes.data, e,
            spec.data_ptr(), _lib.ptr(work), out.data_ptr(), pk.data_ptr(), None, st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_zc_freq_metric_fft(*args), "zc_freq rocfft"), steps, warmup, st)
    name = "cfg5_rocfft" if pruned else "cfg5_rocfft_dense"
    if chunked:
        name = ("cfg5_rocfft_pruned_chunked" if pruned else "cfg5_rocfft_chunked")
    return dict(config=name, chunk_windows=plan.chunk,
                workload=f"zc_freq 62-bin metric via rocFFT, N={N}, cp=0, {n_seq} sequences x {N} c64",
                kernel=("rocFFT fp32 C2C + pruning store callback (template bins only) + zc_gather_kernel + "
                        "row_argmax_kernel" if pruned else
                        "rocFFT fp32 C2C (batched, out-of-place, dense spectrum) + zc_gather_kernel + row_argmax_kernel"),
                samples=n_seq * N, ms=ms, alg_bytes=n_seq * (N * 8 + 4),
                traffic_bytes=(n_seq * (N * 8 + 2 * 62 * 8 + 4 + 8) if pruned else
                               n_seq * (2 * N * 8 + 62 * 8 + 4 + 8)),
                bytes_per_sample="8 in + 4 B per sequence out (as cfg5); spectrum write + gather on top")


def cfg3_detect(dev, st, steps, warmup):
    """cfg3 detect-only: the headline kernel with P/R/M not stored (null outputs),
    events (gate, peak, P at peak, CFO, frame start) only: 8 B/sample + 4 B/stream + 64 B/event."""
    B, T, L, E = 65536, 1024, 512, 4
    x = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, None, None, None, None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_aa_detect(*args), "aa detect-only"), steps, warmup, st)
    stored = int(torch.clamp(n_ev, max=E).sum().item())
    ed = _lib.get_variant("FAST_E_DO") or 4
    scan = "fp64" if _lib.get_variant("FAST_SCAN_DO") == 64 else "fp32"
    return dict(config="cfg3_detect", workload=f"sync_aa S&C fp32 detect-only, L={L}, {B} x {T} c64 (events only)",
                kernel=f"aa_fast_kernel<E={ed},MR={L // (64 * ed)},DO,{scan} row scans> (P/R/M stores off)",
                samples=B * T, ms=ms,
                alg_bytes=B * T * 8 + B * 4 + stored * 64,
                bytes_per_sample="8 in + 4 B/stream + 64 B/event", events_per_stream=round(stored / B, 3))


def cfg3(dev, st, steps, warmup):
    """cfg3 = bench.py's headline launch (sync_aa storing kernel: P, R, M + events, 65536 x 1024 c64,
    L = 512) on plain caching-allocator buffers, for variant A/Bs (tools/variant_ab.py); bench.py's
    own line (AABatchDetector, contiguous placement) is the number of record."""
    B, T, L, E = 65536, 1024, 512, 4
    x = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
    P = torch.empty((B, T), dtype=torch.complex64, device=dev)
    R = torch.empty((B, T), dtype=torch.float32, device=dev)
    M = torch.empty_like(R)
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    ms = timed(lambda: chk(L_.ofs_aa_detect(*args), "aa"), steps, warmup, st)
    return dict(config="cfg3", workload=f"sync_aa S&C fp32 + events, L={L}, {B} x {T} c64",
                kernel="aa_fast_kernel<2,4,1> (P, R, M + events)", samples=B * T, ms=ms, alg_bytes=B * T * 24,
                bytes_per_sample="8 in + 16 out")


def cfg3_pcie(dev, st, steps, warmup):
    """cfg3 with the batch handed over in host memory (the numpy drop-in's situation): pinned host
    x -> HBM, the headline kernel, P/R/M back to pinned host, all on one stream.  The PCIe-inclusive
    rate DESIGN.md quotes beside the HBM-resident headline; never the bench value."""
    B, T, L, E = 65536, 1024, 512, 4
    xh = synth.make_aa_batch(B, T, L, seed=2026, device=dev).cpu().pin_memory()
    x = torch.empty((B, 1, T), dtype=torch.complex64, device=dev)
    P = torch.empty((B, T), dtype=torch.complex64, device=dev)
    R = torch.empty((B, T), dtype=torch.float32, device=dev)
    M = torch.empty_like(R)
    Ph, Rh, Mh = (torch.empty(t.shape, dtype=t.dtype).pin_memory() for t in (P, R, M))
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
    L_ = _lib.lib()
    args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)

    def step():
        x.copy_(xh, non_blocking=True)
        chk(L_.ofs_aa_detect(*args), "aa")
        Ph.copy_(P, non_blocking=True)
        Rh.copy_(R, non_blocking=True)
        Mh.copy_(M, non_blocking=True)

    ms = timed(step, steps, warmup, st)
    return dict(config="cfg3_pcie", workload=f"cfg3 with host-resident input/outputs (pinned), {B} x {T} c64",
                kernel="H2D copy + aa_fast_kernel + 3 x D2H copy (one stream)", samples=B * T, ms=ms,
                alg_bytes=B * T * 24, bytes_per_sample="8 H2D + 16 D2H (PCIe) per sample")


def _aa_cfg(dev, st, steps, warmup, name, B, na, T, L, dtype, prec, workload, seed):
    """sync_aa detector on a [B, na, T] batch through the product's AABatchDetector (its default
    placement="auto", the placement used is recorded), P/R/M + events; algorithmic bytes = input +
    P/R/M per time index."""
    from ofdm_sync_amd import sync_aa
    det = sync_aa.AABatchDetector(B, T, na, L, precision=prec, in_dtype=dtype, outputs=("P", "R", "M"),
                                  max_events=4, device=dev)
    base = synth.faded_base(L, "cir1", tuple(range(na)) if na > 1 else (1,))
    det.x.copy_(synth.synth_batch(base, B, T, seed=seed, device=dev, dtype=dtype))
    ms = timed(lambda: det.run(), steps, warmup, st)
    esz = 8 if dtype == torch.complex64 else 16
    osz = 16 if prec == "fp32" else 32                       # P + R + M per time index
    plan = det.plan()
    stored = int(torch.clamp(det.result.n_events, max=4).sum().item())
    kern = {10: "aa_fast_kernel (register-staged)", 11: "aa_stream_kernel (streaming)",
            30: "aa_exact_kernel<C128> (fp64 wave per stream)"}.get(plan // 100, "general engine")
    return dict(config=name, workload=workload, kernel=f"{kern}, plan {plan}", placement=det.placement,
                samples=B * na * T, ms=ms,
                alg_bytes=B * T * (na * esz + osz) + B * 4 + stored * 64,
                bytes_per_sample=f"{na} x {esz} in + P/R/M {osz} per time index + events")


def cfg3_T4096(dev, st, steps, warmup):
    """SURVEY §8d sensitivity run: cfg3 with T = 4096 (65536 x 4096 c64, L = 512, fp32)."""
    return _aa_cfg(dev, st, steps, warmup, "cfg3_T4096", 65536, 1, 4096, 512, torch.complex64, "fp32",
                   "sync_aa S&C fp32 L=512, 65536 x 4096 c64 (T=4096 sensitivity)", 41)


def aa_refshape_c64(dev, st, steps, warmup):
    """The reference's own detector input shape (sync_aa.run_single_test, preamble 1024 + cir1:
    2 antennas x 5315 samples, sync_aa.py:699-738), batched 16384 streams, c64 / fp32."""
    return _aa_cfg(dev, st, steps, warmup, "aa_refshape_c64", 16384, 2, 5315, 512, torch.complex64, "fp32",
                   "sync_aa S&C fp32 L=512, 16384 x 2 ant x 5315 c64 (reference run_single_test shape)", 43)


def aa_refshape_c128(dev, st, steps, warmup):
    """As aa_refshape_c64 in the reference's float64 (complex128 in, fp64 out)."""
    return _aa_cfg(dev, st, steps, warmup, "aa_refshape_c128", 16384, 2, 5315, 512, torch.complex128, "fp64",
                   "sync_aa S&C fp64 L=512, 16384 x 2 ant x 5315 c128 (reference run_single_test shape)", 43)


# ---- vector-FMA-bound kernels (Park, ZC matched filter, zc_freq sliding DFT) + the zc_v2 FSM ----
def _flops(r, flops, prec):
    r.update(alg_flops=flops, flop_prec=prec)
    return r


def park(dev, st, steps, warmup, prec="fp32"):
    """park.park_streaming_metric (park.py:64-114), N = 2048: B = 2048 x T = 8192, one branch.
    Direct sums per output d: P = Σ_{k<N/2} x[d-k]·x[d+k] (N/2 complex MACs = 4N flops) and
    E = Σ_{k<N/2} |x[d+k]|² (N/2 x 2 FMA = 2N flops): 6N flops / output."""
    from ofdm_sync_amd import park as pk
    B, T, N = 2048, 8192, 2048
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn((B, 1, T), dtype=torch.complex64 if prec == "fp32" else torch.complex128, device=dev, generator=g)
    ms = timed(lambda: pk.park_streaming_metric_batched(x, N, precision=prec), steps, warmup, st)
    nout = T - 2 * (N // 2)
    esz = 8 if prec == "fp32" else 16
    return _flops(dict(config=f"park_{prec}", workload=f"park N={N}, {B} x {T} c{esz * 8}, {prec}",
                       kernel=f"park_kernel<{prec}> (LDS tile, 8 outputs per thread)", samples=B * T, ms=ms,
                       alg_bytes=B * T * esz + B * nout * (2 * esz + esz // 2 * 2), bytes_per_sample="in + P, E, M out"),
                  B * nout * 6 * N, prec)


def zc_mf(dev, st, steps, warmup, method="fft"):
    """zc_v2 matched filter + normaliser (zc_v2.py:244-271, OFS_ZC_V2), 2048-tap PSS reference, fp64:
    B = 512 x T = 16384 c128, outputs T + N - 1.  Per output: N complex MACs (8N flops) + the
    sliding |x|² window (2 FMA)."""
    from ofdm_sync_amd import zc_v2
    B, T = 512, 16384
    ref = zc_v2.build_pss_symbol(include_cp=False)
    N = len(ref)
    g = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn((B, 1, T), dtype=torch.complex128, device=dev, generator=g)
    ms = timed(lambda: zc_v2.correlate_batched(x, ref, zc_v2.OFS_ZC_V2, want_corr=True, want_mag=True,
                                               method=method), steps, warmup, st)
    nout = T + N - 1
    # traffic model of the FFT path (bytes every pass moves): blocks of M samples
    # (ofs_zc_mf_plan_create's pick_m: power of two >= 2N minimising nblk·M), rows = B·nblk spectra
    M, best = 0, None
    for m in (1 << e for e in range(1, 17)):
        if m < 2 * N or m < 1024:
            continue
        nblk_m = -(-nout // (m - N + 1))
        if best is None or nblk_m * m < best:
            best, M = nblk_m * m, m
    nblk = -(-nout // (M - N + 1))
    fused = method == "fft" and M == 8192 and _lib.get_variant("MC_FUSED") != 0
    if fused:
        # one LDS kernel per block (zc_fftcorr.hip mc_fused_kernel, extract fused for one branch): x read
        # once per block (M samples incl. the N-1 overlap), corr + |corr| written once; no scratch
        traffic = B * nblk * M * 16 + B * nout * 24
        model = "x read once per block (M = 8192 incl. the N-1 overlap) + corr 16 B + |corr| 8 B out"
        kern = ("mc_fused_kernel<C128, fused extract>: load + DIF FFT + xH/M + DIT inverse + normalise in LDS"
                if _lib.get_variant("MC_PERS") == 0 else
                "mc_pers_kernel<C128, fused extract>: persistent, one 512-thread workgroup per CU; next block "
                "prefetched; DIF FFT + xH/M + DIT inverse + normalise in LDS")
    else:
        spec = B * nblk * M * 16
        traffic = (B * T * 16 + spec) + 2 * spec + 2 * spec + 2 * spec + (B * nout * 16 + B * T * 16 + B * nout * 24)
        model = ("pack (x in, spectra out) + rocFFT fwd (r+w) + xH (r+w) + rocFFT inv (r+w) + extract "
                 "(valid spectra + x for the energy prefix in, corr + |corr| out)")
        kern = "FFT overlap-save: pack + rocFFT fwd + xH + rocFFT inv + extract/normalise (fp64)"
    r = dict(config="zc_mf" if method == "fft" else "zc_mf_direct",
             workload=f"zc_v2 matched filter + normalise, N={N} taps, {B} x {T} c128, fp64",
             kernel=kern if method == "fft" else "zc_mf_kernel<fp64> (direct correlation, LDS tile)",
             samples=B * T, ms=ms, alg_bytes=B * T * 16 + B * nout * 24,
             bytes_per_sample="16 in + corr 16 + |corr| 8 out")
    if method == "fft":
        # the FFT path's own work: per block two M-point complex FFTs (5·M·log2 M flops each), the
        # pointwise product with H/M (6 flops per point) and the normalisation (~10 per output)
        fft_flops = B * nblk * (2 * 5 * M * (M.bit_length() - 1) + 6 * M) + B * nout * 10
        r.update(fft_block=M, fft_blocks=nblk, traffic_model_bytes=traffic, traffic_model=model,
                 traffic_frac=round(traffic / (ms / 1e3) / 1e9 / HBM, 4),
                 direct_equivalent_flops=B * nout * (8 * N + 4),
                 direct_equivalent_tflops=round(B * nout * (8 * N + 4) / (ms / 1e3) / 1e12, 2))
        return _flops(r, fft_flops, "fp64")
    # the direct sums: 8N flops per output (the reference's algorithm) + the |x|^2 window
    return _flops(r, B * nout * (8 * N + 4), "fp64")


def zc_freq_fp64(dev, st, steps, warmup):
    """zc_freq.compute_frequency_metric (zc_freq.py:62-99) at the reference's N = 2048, cp = 512, fp64
    sliding DFT: B = 256 x T = 16384 c128.  Work unit (algorithm-independent, like the direct-sum
    count of the FFT matched filter): the first-order sliding DFT per offset and template bin -
    window update (x[s+N] - x[s])·w^{ks} (6 + 2 flops), twiddle advance (6), vdot term (8): ~22 flops
    x 62 bins.  The pair kernel (±k resonators, Goertzel block DFTs) issues fewer instructions than
    this model counts; its VALU issue share is in the SQ counters (profiles/)."""
    B, T, N, cp = 256, 16384, 2048, 512
    g = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn((B, 1, T), dtype=torch.complex128, device=dev, generator=g)
    ms = timed(lambda: zc_freq.compute_frequency_metric_batched(x, N=N, cp=cp), steps, warmup, st)
    noff = T - (N + cp) + 1
    plan = _lib.lib().ofs_zc_freq_plan(_lib.C128, _lib.FP64, T, N, cp)
    kern = {4: "zc_pair_kernel (±k Goertzel resonators, 8 chunks x 4 pairs per lane, Goertzel block DFTs)",
            1: "zc_freq_kernel (lane = bin, one chunk per wave)"}.get(plan, str(plan))
    return _flops(dict(config="zc_freq_fp64", workload=f"zc_freq N={N} cp={cp}, {B} x {T} c128, fp64 sliding DFT",
                       kernel=f"plan {plan}: {kern}", samples=B * T, ms=ms,
                       alg_bytes=B * T * 16 + B * noff * 8, bytes_per_sample="16 in + 8 out per offset"),
                  B * noff * 62 * 22, "fp64")


def zc_freq_refshape(dev, st, steps, warmup, B=4096):
    """zc_freq.compute_frequency_metric on the reference's own stream shape (zc_freq.run_simulation:
    ~4.2k samples x 2 RX branches, N = 2048, cp = 512, ~1.7k offsets, zc_freq.py:102-147), complex64
    batch of B streams -> float32 metric (plan 5: the fp64 sliding DFT, rounded to fp32).  Flops as
    zc_freq_fp64 per (offset, bin) and branch-summed X."""
    T, N, cp, nb = 4242, 2048, 512, 2
    g = torch.Generator(device=dev).manual_seed(8)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    ms = timed(lambda: zc_freq.compute_frequency_metric_batched(x, N=N, cp=cp), steps, warmup, st)
    noff = T - (N + cp) + 1
    plan = _lib.lib().ofs_zc_freq_plan(_lib.C64, _lib.FP32, T, N, cp)
    return _flops(dict(config="zc_freq_refshape", workload=f"zc_freq N={N} cp={cp}, {B} x {nb} x {T} c64 -> f32",
                       kernel=f"plan {plan}: zc_pair_kernel (fp64 ±k Goertzel resonators, 4 chunks x 2 pairs per lane, f32 out)",
                       samples=B * nb * T, ms=ms, alg_bytes=B * nb * T * 8 + B * noff * 4,
                       bytes_per_sample="8 in + 4 out per offset"),
                  B * noff * 62 * (12 * nb + 10), "fp64")


def zc_freq_refshape_rocfft(dev, st, steps, warmup, B=256, layout="rows", pruned=False, rpe=0):
    """The north-star rocFFT formulation of zc_freq.compute_frequency_metric (zc_freq.py:62-99: one FFT per
    window) at the reference's own sliding shape (T = 4242, 2 branches, N = 2048, cp = 512: 1683 offsets
    per stream), complex64, B streams.  layout "rows": ofs_zc_fft_plan_create_rows - every offset of a row
    group in one rocFFT execution (windows one sample apart; T windows per row are transformed for n_off
    used), dense spectrum rows (default) or, with pruned, compact ones through rocFFT's store callback
    (which blocks the host per execution); "offsets": one execution + gather per offset (2 x 1683
    launches per row group).  Bound: the FFT flops (5 N log2 N per transformed window) against the fp32 vector
    peak - the sliding DFT (zc_freq_refshape) does O(62) work per offset instead of O(N log N)."""
    T, N, cp, nb = 4242, 2048, 512, 2
    g = torch.Generator(device=dev).manual_seed(8)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    pr = True if layout == "offsets" else pruned
    kw = {"rows_per_execution": rpe} if (layout == "rows" and rpe) else {}
    ms = timed(lambda: zc_freq.compute_frequency_metric_rocfft_batched(x, N=N, cp=cp, layout=layout,
                                                                       pruned=pr, **kw), steps, warmup, st)
    noff = T - (N + cp) + 1
    windows = B * nb * (T if layout == "rows" else noff)
    fft_flops = windows * 5 * N * 11
    name = "zc_freq_refshape_rocfft" + ("" if layout == "rows" else "_offsets") + ("_pruned" if layout == "rows" and pr else "")
    r = dict(config=name,
             workload=f"zc_freq N={N} cp={cp}, {B} x {nb} x {T} c64 -> f32 via rocFFT ({layout} layout)",
             kernel=("rocFFT fp32 C2C over every offset of a row group per execution (in_dist 1, "
                     + ("pruning store callback" if pr else "dense spectrum rows, no callback")
                     + ") + zc_gather_rows_kernel" if layout == "rows" else
                     "per offset: rocFFT fp32 C2C (pruned) + zc_gather_kernel"),
             samples=B * nb * T, ms=ms, alg_bytes=B * nb * T * 8 + B * noff * 4, transformed_windows=windows,
             launches_per_call=(2 * -(-B * nb // (rpe or zc_freq.rows_per_exec(B * nb, nb, T, 62 if pr else N, 8)))
                                if layout == "rows" else 2 * noff), rows_per_execution=rpe or None,
             bytes_per_sample="8 in + 4 out per offset")
    r.update(fft_flops=fft_flops, fft_tflops=round(fft_flops / (ms / 1e3) / 1e12, 2),
             fft_flop_frac_fp32=round(fft_flops / (ms / 1e3) / 157.3e12, 4))
    return r


def zc_freq_fewoff_rocfft(dev, st, steps, warmup, B=4096, layout="auto"):
    """A few-offsets shape for the rocFFT leg's layout choice (advisor, round 5): N = 4096, cp = 0,
    T = 4103 (8 offsets per stream), one branch, complex64, B streams.  "auto" takes the offsets plan
    here (T / offsets = 513 > zc_freq.ROWS_MAX_RATIO); "rows" forces the rows plan, which transforms
    T windows per stream for the 8 used."""
    T, N, cp, nb = 4103, 4096, 0, 1
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    noff = T - (N + cp) + 1
    rows = zc_freq.pick_rows_layout(layout, True, None, T, noff)
    ms = timed(lambda: zc_freq.compute_frequency_metric_rocfft_batched(x, N=N, cp=cp, layout=layout),
               steps, warmup, st)
    windows = B * nb * (T if rows else noff)
    return dict(config="zc_freq_fewoff_rocfft" + ("_rows" if layout == "rows" else ""),
                workload=f"zc_freq N={N} cp={cp}, {B} x {nb} x {T} c64 -> f32 via rocFFT ({layout} layout -> "
                         f"{'rows' if rows else 'offsets'})",
                kernel="rocFFT fp32 C2C + gather", samples=B * nb * T, ms=ms, alg_bytes=B * nb * T * 8 + B * noff * 4,
                transformed_windows=windows, fft_flops=windows * 5 * N * 12,
                bytes_per_sample="8 in + 4 out per offset")


def zc_detect(dev, st, steps, warmup, state=False, seq=False):
    """zc_v2 CFAR + gate (zc_v2.py:300-446) on |corr| rows: B = 4096 x 16384 f64.  Default kernel:
    zc_cfar_kernel (lane-per-stream exact recursion + closed-form gate, zc_cfar.hip); seq=True times
    the sequential one-wave-per-stream kernel (debug variant ZC_SEQ).  state=True also stores the five state
    arrays (local_sum, corr_scaled, thresh_scaled 8 B each, above, valid 1 B each)."""
    from ofdm_sync_amd import zc_v2
    B, n = 4096, 16384
    g = torch.Generator(device=dev).manual_seed(7)
    mag = torch.rand((B, n), dtype=torch.float64, device=dev, generator=g) * 0.5
    mag[:, 5000:5100] += 2.0
    with _lib.variants(ZC_SEQ=1 if seq else None):
        ms = timed(lambda: zc_v2._detect_run(mag, zc_v2.CORR_WINDOW_SIZE, zc_v2.THRESH_VALUE, zc_v2.THRESH_FRAC_BITS,
                                             zc_v2.MIN_CORR_MAG, 2048, zc_v2.HYSTERESIS, 4, want_state=state),
                   steps, warmup, st)
    name = "zc_detect" + ("_state" if state else "") + ("_seq" if seq else "")
    return dict(config=name, workload=f"zc_v2 CFAR + gate, {B} x {n} f64 |corr| (events + gate mask"
                + (" + state arrays)" if state else ")"),
                kernel=("zc_detect_kernel (one wave per stream, sequential recursion)" if seq else
                        "zc_cfar_kernel (16 streams per workgroup, 1 walker + 11 helper waves: lane-per-stream recursion + closed-form gate)"),
                samples=B * n, ms=ms, alg_bytes=B * n * (8 + 1 + (26 if state else 0)),
                bytes_per_sample="8 in + gate 1 out" + (" + 3 x 8 + 2 x 1 state out" if state else ""))


CONFIGS = {"zc_mf_direct": lambda *a, **k: zc_mf(*a, method="direct", **k), "park_fp32": park, "park_fp64": lambda *a, **k: park(*a, prec="fp64", **k), "zc_mf": zc_mf,
           "zc_freq_fp64": zc_freq_fp64, "zc_freq_refshape": zc_freq_refshape, "zc_detect": zc_detect,
           "zc_freq_refshape_rocfft": zc_freq_refshape_rocfft,
           "zc_freq_refshape_rocfft_offsets": lambda *a, **k: zc_freq_refshape_rocfft(*a, layout="offsets", **k),
           "zc_freq_refshape_rocfft_pruned": lambda *a, **k: zc_freq_refshape_rocfft(*a, pruned=True, **k),
           "zc_freq_fewoff_rocfft": zc_freq_fewoff_rocfft,
           "zc_freq_fewoff_rocfft_rows": lambda *a, **k: zc_freq_fewoff_rocfft(*a, layout="rows", **k),
           "zc_detect_state": lambda *a, **k: zc_detect(*a, state=True, **k),
           "zc_detect_seq": lambda *a, **k: zc_detect(*a, seq=True, **k),
           "cfg5_rocfft_dense": lambda *a, **k: cfg5_rocfft(*a, pruned=False, **k),
           "cfg5_rocfft_chunked": lambda *a, **k: cfg5_rocfft(*a, pruned=False, chunked=True, **k),
           "cfg2a_cp12": lambda *a, **k: cfg2a(*a, cp12=True, **k),
           "cfg2b_cp12": lambda *a, **k: cfg2b(*a, cp12=True, **k), "cfg3_T4096": cfg3_T4096, "aa_refshape_c64": aa_refshape_c64, "aa_refshape_c128": aa_refshape_c128,
"cfg2a": cfg2a, "cfg3": cfg3, "cfg3_2ant": cfg3_2ant, "cfg4_2br": cfg4_2br, "cfg3_fp64": cfg3_fp64, "cfg2b": cfg2b, "cfg4": cfg4, "cfg5": cfg5, "cfg5_rocfft": cfg5_rocfft, "cfg3_detect": cfg3_detect, "cfg3_pcie": cfg3_pcie, "backend": backend,
"backend_n1024": lambda d, s_, k, w: backend(d, s_, k, w, B=32768, N=1024, n_used=600, name="backend_n1024"),
"backend_n4096": lambda d, s_, k, w: backend(d, s_, k, w, B=8192, N=4096, n_used=2400, name="backend_n4096")}


def _selftest_config(name):
    """--selftest-cpu stand-in for a config: a rank-dependent sleep per step instead of the HIP
    launch (rank r sleeps 2·(r+1) ms), host-timed between barriers, same result fields, so the
    launcher, the strong-scaling shard split, the sums over ranks and MAX-of-times are exercised
    on CPU (gloo).  Never used without --selftest-cpu."""
    def run(dev, st, steps, warmup, B=None, n_seq=None, seed=0):
        n = B if B is not None else (n_seq if n_seq is not None else 4096)
        delay = 0.002 * (shard.rank_info().rank + 1)
        for _ in range(warmup):
            time.sleep(delay)
        if _DIST is not None:
            _DIST.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            time.sleep(delay)
        ms = (time.perf_counter() - t0) * 1e3 / steps
        return dict(config=name, workload="selftest (sleep)", kernel="none", samples=n * 4096, ms=ms,
                    alg_bytes=n * 4096 * 8, selftest=True, seed=seed)
    return run


# strong-scaled configs: global batch and the keyword that receives the rank's shard
SHARDED = {"cfg4": ("cfg4_global", "B"), "cfg5": ("cfg5_global", "n_seq"), "cfg5_rocfft": ("cfg5_global", "n_seq"),
           "cfg5_rocfft_dense": ("cfg5_global", "n_seq"), "cfg5_rocfft_chunked": ("cfg5_global", "n_seq")}


def main(argv=None):
    global _DIST
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5, help="untimed calls first, at least; they continue until "
                                                          "WARM_MS of wall time (sub-ms kernels reach steady "
                                                          "clocks only after tens of ms of load)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--cfg4-global", type=int, default=262144, help="cfg4 streams over all GPUs")
    ap.add_argument("--cfg5-global", type=int, default=1 << 20, help="cfg5 sequences over all GPUs")
    ap.add_argument("--selftest-cpu", action="store_true",
                    help="launcher self-test on CPU (gloo, a rank-dependent sleep per config instead of the HIP "
                         "launch): rank start-up, strong-scaling shards, sums over ranks, MAX-of-times")
    a = ap.parse_args(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.path.insert(0, ROOT)
        import bench
        return bench.launch_ranks(argparse.Namespace(gpus=a.gpus, selftest_cpu=a.selftest_cpu), argv,
                                  script=os.path.abspath(__file__))
    info = shard.rank_info()
    if info.world != a.gpus:
        raise SystemExit(f"bench_configs.py: --gpus {a.gpus} but WORLD_SIZE={info.world}")
    if a.selftest_cpu:
        dev = torch.device("cpu")
        _DIST = shard.init("gloo")
        st = None
    else:
        torch.cuda.set_device(info.local_rank)
        dev = torch.device("cuda", info.local_rank)
        _DIST = shard.init("nccl", dev)
        st = torch.cuda.current_stream(dev)
    for spec in a.configs.split(","):
        t0 = time.perf_counter()
        name, _, params = spec.partition("@")           # "cfg2b@B=65536": keyword overrides
        kw = {k: int(v) for k, v in (p.split("=") for p in params.split(";") if p)}
        if name in SHARDED:
            gkey, arg = SHARDED[name]
            total = getattr(a, gkey)
            lo, hi = shard.shard_bounds(total, info.rank, info.world)
            kw.update({arg: hi - lo, "seed": shard.shard_seed(5, info.rank)})
        fn = _selftest_config(name) if a.selftest_cpu else CONFIGS[name]
        r = fn(dev, st, a.steps, a.warmup, **kw)
        ms_rank = r["ms"]
        ms = shard.max_over_ranks(ms_rank, _DIST, dev)
        if name in SHARDED:
            # global samples: every rank's shard (sum); alg bytes likewise
            tot = torch.tensor([r["samples"], r["alg_bytes"]], dtype=torch.float64, device=dev)
            if _DIST is not None:
                _DIST.all_reduce(tot)
            r["samples"], r["alg_bytes"] = int(tot[0].item()), int(tot[1].item())
            census = shard.rank_census(_DIST, dev, ms_rank, (lo, hi))
            r.update(scaling="strong", global_batch=getattr(a, SHARDED[name][0]), n_gpus=info.world,
                     shard=[lo, hi])
        else:
            census = shard.rank_census(_DIST, dev, ms_rank, (0, 0))
            r.update(scaling="per-rank", n_gpus=info.world)
        if census["ranks_seen"] != info.world or not census["distinct_devices"]:
            raise SystemExit(f"bench_configs.py: rank census disagrees with WORLD_SIZE={info.world}: {census}")
        r.update(ranks_seen=census["ranks_seen"], rank_devices=[c["device"] for c in census["ranks"]],
                 rank_ms=[c["ms"] for c in census["ranks"]])
        if name in SHARDED:
            r["rank_shards"] = [c["shard"] for c in census["ranks"]]
        r["ms"] = ms
        if _LAST_HOST_MS is not None:
            r["host_ms_per_step"] = round(_LAST_HOST_MS, 4)
        gbs = r["alg_bytes"] / (ms / 1e3) / 1e9
        if "alg_flops" in r:
            tf = r["alg_flops"] / (ms / 1e3) / 1e12
            r.update(achieved_TFLOPs=round(tf, 2), vector_peak_TFLOPs=VPEAK[r["flop_prec"]],
                     flop_frac=round(tf / VPEAK[r["flop_prec"]], 4))
        r.update(value=round(r["samples"] / (ms / 1e3) / 1e6, 1), unit="Msamples/s",
                 ms=round(ms, 4), achieved_GBs=round(gbs, 1),
                 hbm_frac=round(gbs / (HBM * (info.world if name in SHARDED else 1)), 4),
                 wall_s=round(time.perf_counter() - t0, 1))
        if info.rank == 0:
            print(json.dumps(r), flush=True)
        if not a.selftest_cpu:
            torch.cuda.empty_cache()
    if _DIST is not None:
        _DIST.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
