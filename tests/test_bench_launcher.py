"""CPU: bench.py's multi-GPU launch path as the driver invokes it (``python bench.py --gpus N``
without torchrun): the launcher starts N ranks (torch.distributed.run child), every rank
takes its shard, the timed region is MAX over ranks, rank 0 prints one JSON line.  Runs with
--selftest-cpu (gloo, a rank-dependent sleep instead of the HIP launch)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--selftest-cpu", *args],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout           # one JSON line, rank 0 only
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_gpus2_weak_launches_two_ranks():
    steps = 3
    r = _bench("--gpus", "2", "--steps", str(steps), "--warmup", "1", "--batch", "64")
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 2 * 64
    assert r["shard"] == [0, 64]
    # rank 1 sleeps 4 ms per step, rank 0 2 ms: the reported time is rank 1's (MAX over ranks)
    assert r["ms_per_step"] >= 0.95 * 4.0
    # rank census: the all-reduce saw both ranks, each on its own device, with its own time and shard
    assert r["ranks_seen"] == 2
    assert len(r["rank_devices"]) == 2 and len(set(r["rank_devices"])) == 2
    assert r["rank_devices"] == ["cpu:0", "cpu:1"]
    assert r["rank_shards"] == [[0, 64], [64, 128]]
    assert r["rank_ms"][1] > r["rank_ms"][0]
    assert r["ms_per_step"] * steps == pytest.approx(max(r["rank_ms"]), rel=1e-4)
    assert r["value"] == pytest.approx(2 * 64 * 1024 * steps / (r["ms_per_step"] * steps / 1e3) / 1e6, abs=0.11)


@pytest.mark.timeout(300)
def test_gpus2_strong_splits_global_batch():
    r = _bench("--gpus", "2", "--steps", "2", "--warmup", "0", "--scaling", "strong", "--global-batch", "101")
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["global_batch"] == 101
    assert r["shard"] == [0, 51]                 # shard.shard_bounds(101, 0, 2)
    assert r["ranks_seen"] == 2 and r["rank_shards"] == [[0, 51], [51, 101]]


@pytest.mark.timeout(300)
def test_gpus3_census_counts_every_rank():
    r = _bench("--gpus", "3", "--steps", "1", "--warmup", "0", "--batch", "16")
    assert r["ranks_seen"] == 3 and r["n_gpus"] == 3
    assert r["rank_devices"] == ["cpu:0", "cpu:1", "cpu:2"]
    assert r["rank_shards"] == [[0, 16], [16, 32], [32, 48]]


def test_gpus1_runs_in_process():
    r = _bench("--gpus", "1", "--steps", "2", "--warmup", "0", "--batch", "8")
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == 8
    assert r["ranks_seen"] == 1 and r["rank_devices"] == ["cpu:0"]


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--selftest-cpu", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
