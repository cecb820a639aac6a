"""Headline kernel on a physically contiguous arena (x | P | R | M) with a gap after each large
buffer: does the relative physical placement select the timing mode?  Diagnostic only."""
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
n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
MiB = 1 << 20
gaps = [int(g) for g in os.environ.get("GAPS", "0,4096,65536,1048576,2097152,6291456,12582912,33554432").split(",")]
for rep in range(2):
    for gap in gaps:
        x, P, R, M = _lib.arena(dev, [((B, 1, T), torch.complex64), ((B, T), torch.complex64), ((B, T), torch.float32),
                                      ((B, T), torch.float32)], contiguous=True, gap=gap)
        x.copy_(x0)
        args = (_lib.C64, x.data_ptr(), B, 1, T, L, _lib.FP32, P.data_ptr(), R.data_ptr(), M.data_ptr(), None, 1,
                0.15, 128, 15.36e6, E, n_ev.data_ptr(), ev_i.data_ptr(), ev_r.data_ptr(), st.cuda_stream)
        for _ in range(5):
            lib.ofs_aa_detect(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(60):
            lib.ofs_aa_detect(*args)
        e1.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"rep": rep, "gap": gap, "ms": round(e0.elapsed_time(e1) / 60, 4)}), flush=True)
        del x, P, R, M
        torch.cuda.synchronize()
