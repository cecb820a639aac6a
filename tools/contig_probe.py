"""hipMalloc vs hipExtMallocWithFlags(hipDeviceMallocContiguous) for the headline batch
(x, P, R, M in one raw allocation): does physically contiguous backing fix the slow mode?
Diagnostic only."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
import torch
from ofdm_sync_amd import _lib, synth

B, T, L, E = 65536, 1024, 512, 4
dev = torch.device("cuda", 0)
lib = _lib.lib()
hip = ctypes.CDLL("libamdhip64.so")
st = torch.cuda.current_stream(dev)
x0 = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
torch.cuda.synchronize()
MiB = 1 << 20
NX, NR = B * T * 8, B * T * 4
SZ = NX * 2 + NR * 2


def alloc(flags):
    p = ctypes.c_void_p()
    if flags is None:
        rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(SZ))
    else:
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(SZ), ctypes.c_uint(flags))
    return rc, p.value


def run(base, steps=int(os.environ.get("PROBE_STEPS", "60"))):
    hip.hipMemcpy(ctypes.c_void_p(base), ctypes.c_void_p(x0.data_ptr()), ctypes.c_size_t(NX), 3)
    args = (_lib.C64, base, B, 1, T, L, _lib.FP32, base + NX, base + 2 * NX, base + 2 * NX + NR, None, 1,
            0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
    for _ in range(5):
        lib.ofs_aa_detect(*args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        lib.ofs_aa_detect(*args)
    e1.record(st)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / steps, 4)


held = []
for r in range(5):
    if r:
        xs_new = synth.make_aa_batch(B, T, L, seed=2026 + r, device=dev)   # as aa_ab.py's rounds
        held.append(xs_new)
    for name, fl in (("hipMalloc", None), ("contiguous", 4)):
        rc, p = alloc(fl)
        if rc:
            print(json.dumps({"round": r, "alloc": name, "rc": rc}), flush=True)
            continue
        print(json.dumps({"round": r, "alloc": name, "ms": run(p), "ptr": hex(p)}), flush=True)
        held.append(p)
        torch.cuda.synchronize()
