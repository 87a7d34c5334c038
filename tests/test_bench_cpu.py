"""bench.py's launcher on the CPU (gloo, stand-in renderer): `--gpus N` starts
N ranks itself when no torch.distributed launcher set WORLD_SIZE, the JSON
line reports the rank count, and the config-5 frame assembled from the ranks'
64-ray tiles equals the single-rank frame."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", *args],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    return p


def _line(p):
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_n_ranks(n):
    one = _line(_bench("--gpus", "1", "--config", "5", "--frame", "48", "--steps", "2", "--warmup", "1"))
    many = _line(_bench("--gpus", str(n), "--frame", "48", "--steps", "2", "--warmup", "1"))
    assert one["n_gpus"] == 1 and many["n_gpus"] == n
    # N > 1 defaults to BASELINE config 5 (fixed 4 views per step: strong scaling)
    assert many["scaling"] == "strong" and many["config"]["rays_per_step"] == 4 * 48 * 48
    assert many["checksum"] == one["checksum"]
    # ranks > 0 start from another scene; broadcast_scene hands them rank 0's
    assert many["scene_checksum"] == one["scene_checksum"]
    assert many["scene_broadcast"]["bytes"] > 27e6 and "scene_broadcast" not in one
    # the N > 1 line attributes the step (VERDICT r04 missing 3): per-rank render / all_gather / reassembly
    # ms per step (min / max over ranks) and the gather's size
    ph = many["shard_phases"]
    for k in ("render_ms_per_step", "all_gather_ms_per_step", "reassembly_ms_per_step"):
        assert len(ph[k]["per_rank"]) == n and 0.0 <= ph[k]["min"] <= ph[k]["max"], (k, ph[k])
    assert ph["render_ms_per_step"]["max"] > 0 and ph["all_gather_ms_per_step"]["max"] > 0
    tiles = -(-4 * 48 * 48 // 64)
    assert ph["rays_per_rank_max"] == -(-tiles // n) * 64
    assert ph["gather_bytes_per_step"] == n * ph["rays_per_rank_max"] * 28
    assert "shard_phases" not in one


def test_bench_default_is_config3_weak():
    # without --device cpu's stand-in the default config at one rank is config 3; the stand-in reports it too
    one = _line(_bench("--gpus", "1", "--frame", "32", "--steps", "1", "--warmup", "0"))
    assert one["scaling"] == "weak" and one["n_gpus"] == 1


def test_bench_rejects_world_size_mismatch():
    p = _bench("--gpus", "2", "--steps", "1", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in (p.stderr + p.stdout)
