"""Multi-GPU layout: one process per GPU, independent stream shards, no data-path collective.

Receive streams are independent: a batch is split into contiguous per-rank
shards and every rank runs the hot path on its own shard.  The only collectives are
control-plane: a barrier around the timed region and a MAX over per-rank times (bench.py),
plus an optional gather of per-stream results for validation.  torch.distributed's "nccl"
backend is RCCL on ROCm; tests exercise the same code with "gloo" on CPU.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world: int
    local_rank: int


def rank_info() -> RankInfo:
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) of `total` streams owned by `rank` (remainder to low ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_seed(seed: int, rank: int) -> int:
    """Per-rank RNG seed for synthetic shards (weak scaling: every rank owns fresh streams)."""
    return seed + 1_000_003 * rank


def init(backend: str = "nccl", device: torch.device | None = None):
    """Initialise torch.distributed from the torchrun environment; returns the module or None."""
    info = rank_info()
    if info.world <= 1:
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return dist


def max_over_ranks(x: float, dist, device) -> float:
    """Control-plane reduction used for timing: every rank's value -> the maximum."""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rank_census(dist, device, rank_ms: float, shard: tuple[int, int]) -> dict:
    """Self-verification of a multi-rank run (control plane only): an all-reduce of ones over the
    ranks (how many ranks the collective actually saw) and an all-gather of each rank's
    (rank, local rank, device ordinal, PCI domain/bus/device, timed ms, shard bounds).  On a GPU
    the PCI address is the HIP device's (torch.cuda.get_device_properties); on CPU (gloo
    self-test) the "device" is the rank's process, labelled cpu:<local rank>.  Returns
    {"ranks_seen": n, "ranks": [{...} per rank in rank order], "distinct_devices": bool}."""
    info = rank_info()
    on_gpu = device is not None and device.type == "cuda"
    if on_gpu:
        p = torch.cuda.get_device_properties(device)
        ident = [float(device.index), float(getattr(p, "pci_domain_id", -1)), float(getattr(p, "pci_bus_id", -1)),
                 float(getattr(p, "pci_device_id", -1))]
    else:
        ident = [float(info.local_rank), -1.0, -1.0, -1.0]
    row = torch.tensor([float(info.rank), float(info.local_rank), *ident, float(rank_ms), float(shard[0]),
                        float(shard[1])], dtype=torch.float64, device=device)
    one = torch.ones(1, dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(one, op=dist.ReduceOp.SUM)
        rows = [torch.zeros_like(row) for _ in range(dist.get_world_size())]
        dist.all_gather(rows, row)
    else:
        rows = [row]
    ranks = []
    for r in rows:
        v = r.cpu().tolist()
        dev = (f"cuda:{int(v[2])} pci {int(v[3]):04x}:{int(v[4]):02x}:{int(v[5]):02x}" if on_gpu
               else f"cpu:{int(v[2])}")
        ranks.append(dict(rank=int(v[0]), local_rank=int(v[1]), device=dev, ms=round(v[6], 5),
                          shard=[int(v[7]), int(v[8])]))
    return dict(ranks_seen=int(round(float(one.item()))), ranks=ranks,
                distinct_devices=len({r["device"] for r in ranks}) == len(ranks))


def gather_counts(counts: torch.Tensor, dist) -> torch.Tensor:
    """Concatenate per-rank 1-D result tensors in rank order (validation only)."""
    if dist is None:
        return counts
    n = torch.tensor([counts.numel()], dtype=torch.int64, device=counts.device)
    sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
    dist.all_gather(sizes, n)
    mx = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros(mx, dtype=counts.dtype, device=counts.device)
    pad[: counts.numel()] = counts
    bufs = [torch.zeros_like(pad) for _ in sizes]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)])
