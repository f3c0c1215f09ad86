"""bench.py output contract (one JSON line; metric/config as BASELINE.json names) on the CPU at tiny shapes,
single process and 2 ranks over gloo, for each job-scheduling mode."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("extra", [[], ["--overlap", "before"], ["--overlap", "after"], ["--two-job"],
                                   ["--single-job"]])
def test_bench_single_process(extra):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "bench.py", "--small", "--steps", "2", "--warmup", "2"] + extra, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["dtype"] == "bf16"
    assert d["config"]["check"]["ok"] is True and d["config"]["check"]["ff_max_rel_err"] < 1e-2


def test_bench_two_ranks_gloo():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2", "--small",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * (64 + 4)
    assert d["config"]["check"]["ok"] is True
    # weak scaling with a replicated model: the timed steps are rank-local (no collective inside a step; the
    # conv job's single-source plan skips the cluster-wide source sizing)
    assert d["config"]["collectives_per_step"] == 0


def test_bench_self_launches_ranks():
    """``bench.py --gpus 2`` without torchrun spawns its own two ranks (gloo on this CPU host) and reports n_gpus 2."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--small", "--steps", "2", "--warmup", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * (64 + 4)
    assert d["config"]["check"]["ok"] is True
