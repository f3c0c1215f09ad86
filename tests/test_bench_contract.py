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


def test_bench_launcher_parent_makes_no_gpu_call():
    """The ``--gpus N`` parent counts GPUs from the environment / KFD topology and only spawns ranks: with every
    torch.cuda entry point that could initialise HIP replaced by one that raises, the launch still completes."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    code = (
        "import sys, runpy, torch\n"
        "def boom(*a, **k):\n"
        "    raise RuntimeError('GPU call in the launching parent')\n"
        "for f in ('device_count', 'is_available', 'init', 'set_device', 'current_device', 'synchronize'):\n"
        "    setattr(torch.cuda, f, boom)\n"
        "sys.argv = ['bench.py', '--gpus', '2', '--small', '--steps', '1', '--warmup', '1']\n"
        "runpy.run_path('bench.py', run_name='__main__')\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert _last_json(r.stdout)["n_gpus"] == 2


def test_visible_gpus_reads_environment(monkeypatch):
    from netsdb_amd.parallel import launch

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    assert launch.visible_gpus() == 4
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert launch.visible_gpus() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "5")
    assert launch.visible_gpus() == 1


def test_xgmi_model():
    from netsdb_amd.parallel.comm import XGMI_ALPHA_S, XGMI_LINK_BPS, xgmi_seconds

    assert xgmi_seconds("all_to_all", 1 << 30, 1) == 0.0
    # all-to-all of 8 GB per rank over 8 GPUs: 1 GB per link
    assert abs(xgmi_seconds("all_to_all", 8e9, 8) - (XGMI_ALPHA_S + 1e9 / XGMI_LINK_BPS)) < 1e-12
    assert xgmi_seconds("all_gather", 1e9, 8) > xgmi_seconds("reduce_scatter", 1e9, 8)
    assert abs(xgmi_seconds("all_reduce", 8e9, 8) - 2 * (XGMI_ALPHA_S + 1e9 / XGMI_LINK_BPS)) < 1e-12


@pytest.mark.timeout(900)
@pytest.mark.parametrize("script,n", [("bench_la_matmul.py", 2), ("bench_la_matmul.py", 8), ("bench_dedup.py", 2),
                                      ("bench_dedup.py", 8)])
def test_secondary_bench_self_launch(script, n):
    """The configs that move data over xGMI (BASELINE.json: LA 64k^2 on 8 GPUs, dedup across 8 GPUs) start their own
    ranks with ``--gpus N`` like bench.py (gloo on this CPU host), report n_gpus N, a correct result, and their
    per-step collective bytes with the modelled xGMI time next to the compute time."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join("scripts", script), "--small", "--gpus", str(n)], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=800)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == n
    if script == "bench_la_matmul.py":
        assert d["rel_err_sampled"] < 1e-2 and any("matmul" in f for f in d["fused"]), d
        assert d["coll_MB_per_multiply_per_rank"] > 0 and d["xgmi_pred_ms_per_multiply"] > 0 and d["local_gemm_ms"] > 0
    else:
        assert d["rel_err_model0"] < 1e-2 and d["dedup_ratio"] < 0.5, d
        assert d["add_coll_MB_per_rank"] > 0 and d["materialize_coll_MB_per_rank"] > 0
        assert d["add_xgmi_pred_ms"] > 0
