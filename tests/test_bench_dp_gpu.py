"""bench.py's N > 1 launch path end to end on one GPU: one torchrun rank over RCCL
(``MMAD_DP_SELFTEST=1`` runs the gradient all-reduce path at world size 1) with
``--collectives auto`` -- each candidate mode (staged, staged1, after) captured, timed and
dropped in turn, the fastest rebuilt and benched.  Checked: one JSON line, the chosen mode is
one of the probed ones and the fastest of them, every candidate was timed, and the step
launch string names it.  (The numerics of the modes: tests/test_dp_graph_world2_gpu.py.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_dp_auto_one_rank():
    port = 29600 + os.getpid() % 300
    env = dict(os.environ, MMAD_DP_SELFTEST="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", "bench.py", "--steps", "3",
           "--warmup", "1", "--batch", "2", "--size", "64", "--no-cpu-baseline",
           "--no-roofline"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    dp = res["dp"]
    probe = dp["auto_probe_ms_per_step"]
    assert set(probe) == {"staged", "staged1", "after"}
    assert dp["collectives"] == min(probe, key=probe.get)
    assert res["value"] > 0 and res["config"]["parallelism"] == "dp1"
    n_stages = {"staged": 4, "staged1": 2}.get(dp["collectives"])
    if n_stages:
        assert f"{n_stages} backward-stage graphs" in res["config"]["step_launch"]
    else:
        assert "eager RCCL all-reduce" in res["config"]["step_launch"]
