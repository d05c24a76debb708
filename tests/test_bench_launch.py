"""bench.py launch contract: ``--gpus N`` outside a launcher re-launches N ranks under
torch.distributed.run (before any device call) and rank 0 prints ONE JSON line with
``n_gpus == N`` and the whole-job throughput; inside a launcher ``WORLD_SIZE`` must equal
``--gpus``.  Runs on the CPU (gloo, fp32, tiny batch / image) — the reference harness is
``DL/models/utils/DistriOptimizerPerf.scala:32-146``."""
import json
import os
import subprocess
import sys

import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, env_extra=None):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    cmd = [sys.executable, os.path.join(_REPO, "bench.py"), "--device", "cpu", "--batch", "2", "--image-size", "64",
           "--steps", "2", "--warmup", "1", "--phase-steps", "1"] + extra
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=_REPO)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [1, 2])
def test_bench_gpus_flag_spawns_ranks(n):
    r = _run(["--gpus", str(n)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == n
    assert j["config"]["global_batch"] == 2 * n
    assert j["config"]["parallelism"] == f"dp{n}"
    assert j["config"]["driver"] == ("DistriOptimizer" if n > 1 else "LocalOptimizer")
    assert j["steps"] == 2 and j["warmup"] == 1
    assert j["value"] > 0 and j["ms_per_step"] > 0
    # value is the whole-job aggregate: global batch × steps / elapsed
    assert abs(j["value"] - 2 * n * 1e3 / j["ms_per_step"]) / j["value"] < 0.02
    ph = j["phase_ms_max_over_ranks"]
    assert "forward" in ph and "backward" in ph and "compute weight" in ph
    if n > 1:
        assert "aggregate gradient" in ph


def test_bench_world_size_mismatch_rejected():
    r = _run(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in (r.stdout + r.stderr)
