"""bench.py --gpus N without torchrun starts the N ranks itself (the way the driver runs the
scaling bench); CPU only: the ranks rendezvous over gloo and rank 0 prints one JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_starts_n_ranks(n):
    p = _run(["--gpus", str(n), "--backend", "gloo", "--selftest-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["world"] == n and d["gpus"] == n
    assert d["rank_sum"] == n * (n + 1) / 2


def test_single_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--selftest-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["world"] == 1


def test_failing_rank_fails_the_launch():
    # rank 1 exits with status 3 before the rendezvous: the launcher stops rank 0 (which
    # would wait for it forever) and reports the failure
    p = _run(["--gpus", "2", "--backend", "gloo", "--selftest-launch"],
             {"BICOS_SELFTEST_FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["rccl", "dma"])
def test_two_rank_gloo_line_has_every_field(gather):
    """The N>1 bench line is self-contained: two gloo ranks sharing the
    box's GPU run the row-band path; rank 0's line carries the search roofline with its PMC
    traffic lookup, the gather timed on its own, the gathered frames verified against the
    oracle's whole-frame hash, and a "gloo rehearsal" label (the CPU baseline is an N = 1
    field, null here). gather=dma: the copy-engine gather (rank 1 maps rank 0's receive
    slots through IPC and copies its band into them with hipMemcpyAsync), the same check."""
    p = _run(["--gpus", "2", "--backend", "gloo", "--gather", gather, "--steps", "3",
              "--warmup", "1", "--cpu-seconds", "2", "--kernel-reps", "2", "--no-host-path"],
             timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "gloo rehearsal" in d["config"]["parallelism"]
    assert d["config"]["rows_per_rank"] == 768
    assert d["cpu_baseline"] is None
    roof = d["roofline"]
    assert roof["bound"] == "mfma" and 0 < roof["frac"] < 1
    assert "traffic" in roof and roof["traffic_source"]
    assert roof["match_hbm_read"]["peak_GBps"] == 16000.0
    g = d["gather"]
    if gather == "dma":
        assert "copy-engine" in d["config"]["parallelism"]
        assert g["mode"] == "dma" and g["ms_per_exchange"] > 0
    else:
        assert "gloo gather" in d["config"]["parallelism"]
        assert g["ms"] > 0
    assert g["bytes_to_root"] == g["bytes_per_rank"]
    v = d["verify_gather"]
    assert v["ok"] and v["slots"] >= (4 if gather == "dma" else 2) and v["bands"] == 2
    assert "frames.json" in v["check"]


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["cfg2", "cfg3"])
def test_rccl_gather_rehearsal(config):
    """The RCCL branch of the N>1 bench on the one-GPU box: a 1-rank nccl
    process group runs the whole gather path -- the match writing its band straight into the
    packed device buffer (int16 disparities with the NXC stage, float32 with subpixel), the
    async RCCL gather issued from the frames' streams, the int16 landing on rank 0, the
    gather timed with HIP events, and every gathered slot verified against the oracle's
    whole-frame hash. What it cannot cover is the transport between distinct GPUs."""
    p = _run(["--config", config, "--gather-rehearsal", "--steps", "3", "--warmup", "1",
              "--spinup-ms", "0", "--no-cpu-baseline", "--kernel-reps", "0", "--no-host-path"],
             timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert "rehearsal" in d["config"]["parallelism"] and "RCCL" in d["config"]["parallelism"]
    assert d["config"]["backend"] == "nccl"
    g = d["gather"]
    assert g["ms"] > 0 and g["bytes_to_root"] == 0
    v = d["verify_gather"]
    assert v["ok"] and v["slots"] >= 2 and v["bands"] == 1
    assert "frames.json" in v["check"]
