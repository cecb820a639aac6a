"""CPU, world_size 2 over gloo: the multi-GPU layout of bench.py (contiguous stream shards,
no data-path collective, MAX-over-ranks timing) produces exactly the single-process result.
Each rank runs the C oracle (the CPU checker) on its shard; on the GPU box the same code
path runs ofs_aa_detect per rank over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ofdm_sync_amd import shard, synth

B_TOTAL, T, L = 37, 1024, 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import oracle_c
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    d = shard.init("gloo")
    x = synth.make_aa_batch_torch(B_TOTAL, T, L, seed=5, device="cpu").numpy()
    lo, hi = shard.shard_bounds(B_TOTAL, rank, world)
    r = oracle_c.aa_detect(x[lo:hi], L, max_events=4, nthreads=1)
    counts = shard.gather_counts(torch.from_numpy(r["n_events"].astype(np.int64)), d)
    peaks = shard.gather_counts(torch.from_numpy(r["ev_int"][:, 0, 0].copy()), d)
    tmax = shard.max_over_ranks(float(rank + 1), d, "cpu")
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"), counts=counts.numpy(), peaks=peaks.numpy(), tmax=tmax)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover_exactly():
    for total in (0, 1, 7, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_bounds(10, 2, 2)


def test_world2_gloo_matches_single_process(tmp_path):
    import oracle_c
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "dist.npz")
    x = synth.make_aa_batch_torch(B_TOTAL, T, L, seed=5, device="cpu").numpy()
    ref = oracle_c.aa_detect(x, L, max_events=4, nthreads=1)
    assert np.array_equal(got["counts"], ref["n_events"])
    assert np.array_equal(got["peaks"], ref["ev_int"][:, 0, 0])
    assert float(got["tmax"]) == 2.0          # MAX over ranks 1.0, 2.0
