"""CPU: tools/bench_configs.py's multi-GPU path as the driver's SCALE run would use it
(``--gpus N`` without torchrun): the launcher starts N ranks, cfg4 / cfg5 are strong-scaled over
their fixed global batch (shard.shard_bounds), every rank's samples and bytes are summed, the
time is the MAX over ranks.  --selftest-cpu: gloo, a rank-dependent sleep instead of the kernel."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_configs.py"), "--selftest-cpu", *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


@pytest.mark.timeout(300)
def test_gpus2_strong_scaling_cfg4_cfg5():
    steps = 3
    rs = _run("--gpus", "2", "--configs", "cfg4,cfg5", "--cfg4-global", "1001", "--cfg5-global", "77",
              "--steps", str(steps), "--warmup", "1")
    assert [r["config"] for r in rs] == ["cfg4", "cfg5"]          # one line per config, rank 0 only
    for r, total in zip(rs, (1001, 77)):
        assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["global_batch"] == total
        assert r["shard"] == [0, (total + 1) // 2]                # shard.shard_bounds(total, 0, 2)
        assert r["samples"] == total * 4096                       # both ranks' shards summed
        assert r["alg_bytes"] == total * 4096 * 8
        # rank 1 sleeps 4 ms per step, rank 0 2 ms: the reported time is rank 1's (MAX over ranks)
        assert r["ms"] >= 0.95 * 4.0 and r["rank_ms"][0] < r["ms"]
        assert r["ms"] == pytest.approx(max(r["rank_ms"]), rel=1e-4)
        assert r["ranks_seen"] == 2 and r["rank_devices"] == ["cpu:0", "cpu:1"]
        assert r["rank_shards"] == [[0, (total + 1) // 2], [(total + 1) // 2, total]]
        assert r["value"] == pytest.approx(total * 4096 / (r["ms"] / 1e3) / 1e6, rel=1e-3)
        assert r["hbm_frac"] == pytest.approx(r["achieved_GBs"] / (8000.0 * 2), abs=1e-4)   # vs 2 GPUs of HBM


@pytest.mark.timeout(300)
def test_gpus2_per_rank_config_and_overrides():
    rs = _run("--gpus", "2", "--configs", "cfg2b@B=100", "--steps", "1", "--warmup", "0")
    assert len(rs) == 1 and rs[0]["scaling"] == "per-rank" and rs[0]["n_gpus"] == 2
    assert rs[0]["samples"] == 100 * 4096                         # keyword override reached the config
    assert rs[0]["ranks_seen"] == 2 and len(set(rs[0]["rank_devices"])) == 2


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_configs.py"), "--selftest-cpu",
                        "--gpus", "2"], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
