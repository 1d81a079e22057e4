"""bench.py's rank handling: `python bench.py --gpus N` must time N ranks under any launcher.

* CPU tier: a --gpus / WORLD_SIZE mismatch exits non-zero before anything is imported that touches a GPU; a spawned
  rank that fails (no GPU here) makes the parent exit non-zero instead of hanging; resolve_world's rules.
* GPU tier: a plain `python bench.py --gpus 2` (no torch.distributed.run) on the one-GPU box, both ranks on device 0
  over gloo (IS3D_BENCH_BACKEND / IS3D_BENCH_DEVICE, the rehearsal knobs), prints one JSON line with n_gpus 2 -- the
  config-2 workload, and the PTMA chained path (config 5 miniature: warm-start chains split over the two ranks, the
  gloo branch of launch_chained with host boundary buffers).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def test_resolve_world_rules():
    import bench
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(4, {}) == (4, True)
    assert bench.resolve_world(None, {"WORLD_SIZE": "8"}) == (8, False)
    assert bench.resolve_world(8, {"WORLD_SIZE": "8"}) == (8, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"], env=_env(WORLD_SIZE=2, RANK=0),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert r.stdout.strip() == ""


def test_spawned_rank_failure_propagates():
    """Here there is no GPU: each spawned rank stops at its device check, and the parent returns non-zero (and
    returns at all: a rank left waiting in the rendezvous is terminated)."""
    try:
        import torch
    except ImportError:
        pytest.skip("torch not importable")
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the rank would not fail")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--no-cpu-baseline"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "needs GPU" in r.stderr
    assert r.stdout.strip() == ""


def _run_two_ranks(extra):
    env = _env(IS3D_BENCH_BACKEND="gloo", IS3D_BENCH_DEVICE=0)
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--north-star-steps", "0", "--no-cpu-baseline", "--no-per-species"] + extra,
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout           # rank 0 prints the one JSON line
    return json.loads(lines[0])


@pytest.mark.gpu
def test_plain_bench_gpus_2_runs_two_ranks():
    res = _run_two_ranks(["--cells", "20000"])
    assert res["n_gpus"] == 2
    assert res["value"] > 0
    cfg = res["config"]
    assert cfg["backend"] == "gloo" and "gloo all-reduce" in cfg["parallelism"] and "RCCL" not in cfg["parallelism"]
    assert cfg["launcher"] == "bench.py --gpus"
    assert cfg["cells_per_gpu"] == 20000


@pytest.mark.gpu
def test_plain_bench_gpus_2_chained_ptma():
    res = _run_two_ranks(["--config", "config5", "--cells", "20000"])
    assert res["n_gpus"] == 2
    cfg = res["config"]
    assert "PTMA chain positions split" in cfg["parallelism"]
    assert cfg["cells_per_gpu"] < 20000          # each rank integrates its own chain positions
