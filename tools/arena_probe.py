"""Does the relative placement of x, P, R, M inside one allocation decide the headline
kernel's fast/slow mode?  One arena per round; the four buffers carved at chosen offsets.
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
n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
NX, NP, NR = B * T * 8, B * T * 8, B * T * 4
MB2 = 2 << 20


def run(gap, rounds=3, steps=60, ev_mode="before"):
    global n_ev, ev_i, ev_r
    out = []
    for _ in range(rounds):
        if ev_mode == "after_fresh":
            del n_ev, ev_i, ev_r
        arena = torch.empty(NX + NP + 2 * NR + 4 * MB2 + 3 * gap, dtype=torch.uint8, device=dev)
        base = (arena.data_ptr() + MB2 - 1) // MB2 * MB2 - arena.data_ptr()
        ox = base
        op = ox + NX + gap
        orr = op + NP + gap
        om = orr + NR + gap
        if ev_mode == "after_fresh":
            n_ev = torch.zeros((B,), dtype=torch.int32, device=dev)
            ev_i = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
            ev_r = torch.empty((B, E, 4), dtype=torch.float64, device=dev)
        x = arena[ox:ox + NX].view(torch.complex64).view(B, 1, T)
        x.copy_(x0)
        ptr = arena.data_ptr()
        args = (_lib.C64, ptr + ox, B, 1, T, L, _lib.FP32, ptr + op, ptr + orr, ptr + om, None, 1,
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
        out.append(round(e0.elapsed_time(e1) / steps, 4))
        del arena, x
    return out


for mode in ("before", "after_fresh", "before", "after_fresh"):
    for gap in [0, 4096]:
        print(json.dumps({"ev": mode, "gap": gap, "ms": run(gap, rounds=4, ev_mode=mode)}), flush=True)
