"""Relative placement of x, P, R, M inside ONE 4 GiB allocation vs the headline kernel's time:
the same physical pages, only the offsets change.  Diagnostic only."""
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
torch.cuda.empty_cache()
MiB = 1 << 20
arena = torch.empty(4096 * MiB, dtype=torch.uint8, device=dev)
base = arena.data_ptr()
NX, NR = B * T * 8, B * T * 4


def run(ox, op, orr, om, steps=60):
    xv = arena[ox:ox + NX].view(torch.complex64)
    xv.copy_(x0.reshape(-1))
    args = (_lib.C64, base + ox, B, 1, T, L, _lib.FP32, base + op, base + orr, base + om, None, 1,
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


layouts = {
    "packed x|P|R|M": (0, 512 * MiB, 1024 * MiB, 1280 * MiB),
    "packed P|R|M|x": (1024 * MiB + 512 * MiB, 0, 512 * MiB, 768 * MiB),
    "x|P|R|M +gaps 6MiB": (0, 518 * MiB, 1036 * MiB, 1298 * MiB),
    "x|P|R|M +gaps 2MiB+4KiB": (0, 514 * MiB + 4096, 1028 * MiB + 8192, 1286 * MiB + 12288),
    "spread 1GiB": (0, 1024 * MiB, 2048 * MiB, 3072 * MiB),
    "spread odd": (96 * MiB, 1000 * MiB, 2222 * MiB, 3500 * MiB),
}
for rep in range(2):
    for name, offs in layouts.items():
        print(json.dumps({"layout": name, "ms": run(*offs)}), flush=True)
