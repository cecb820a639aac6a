"""Which buffer's physical placement decides the headline kernel's fast/slow mode?  Allocates
4 candidates of each of x, P, R, M and times ofs_aa_detect with one buffer varied at a time.
Diagnostic only."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
import torch
from ofdm_sync_amd import _lib, synth

B, T, L, E = 65536, 1024, 512, 4
dev = torch.device("cuda", 0)
lib = _lib.lib()
st = torch.cuda.current_stream(dev)
x0 = synth.make_aa_batch(B, T, L, seed=2026, device=dev)
xs = [x0] + [x0.clone() for _ in range(3)]
Ps = [torch.empty((B, T), dtype=torch.complex64, device=dev) for _ in range(4)]
Rs = [torch.empty((B, T), dtype=torch.float32, device=dev) for _ in range(4)]
Ms = [torch.empty((B, T), dtype=torch.float32, device=dev) for _ in range(4)]
n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)


def t(x, P, R, M, steps=60):
    args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
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


for which in "xPRM":
    row = []
    for i in range(4):
        sel = dict(x=0, P=0, R=0, M=0)
        sel[which] = i
        row.append(t(xs[sel["x"]], Ps[sel["P"]], Rs[sel["R"]], Ms[sel["M"]]))
    print(json.dumps({"vary": which, "ms": row}), flush=True)
print(json.dumps({"addr": {k: [hex(v.data_ptr()) for v in vv] for k, vv in (("x", xs), ("P", Ps), ("R", Rs), ("M", Ms))}}))
