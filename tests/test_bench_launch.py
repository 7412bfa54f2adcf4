"""bench.py --gpus N: the launcher's argument and environment handling (CPU).

The driver runs `python bench.py --gpus N` as well as the torch.distributed.run form; both
must end in N ranks or fail loudly (reference: engine/trainer.py:256-258 reaches every visible
GPU from one command).  No GPU is touched here: launch_plan only reads the environment and
the visible-device count.
"""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, 1, ["--steps", "3"]) == ("run", None)
    assert bench.launch_plan(1, {}, 0, []) == ("run", None)   # the CPU container: N=1 is not refused here


def test_multi_gpu_spawns_torchrun_children():
    what, cmd = bench.launch_plan(4, {}, 8, ["--gpus", "4", "--steps", "7"], port=29555)
    assert what == "launch"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "7"]      # the children see the same arguments


def test_launched_rank_runs_when_world_matches():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_plan(8, env, 8, []) == ("run", None)


def test_world_mismatch_fails():
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.launch_plan(8, {"WORLD_SIZE": "2"}, 8, [])
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_plan(1, {"WORLD_SIZE": "4"}, 8, [])


def test_more_ranks_than_gpus_fails_under_rccl():
    with pytest.raises(SystemExit, match="visible"):
        bench.launch_plan(8, {}, 1, [])
    with pytest.raises(SystemExit, match="visible"):
        bench.launch_plan(2, {"WORLD_SIZE": "2"}, 1, [])
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, 1, [])


def test_gloo_rehearsal_may_share_a_gpu():
    what, cmd = bench.launch_plan(2, {"IMGCOMP_DIST_BACKEND": "gloo"}, 1, ["--gpus", "2"], port=29556)
    assert what == "launch" and "--nproc-per-node=2" in cmd


def test_cli_refuses_silent_smaller_run():
    """`python bench.py --gpus N` on a box with fewer GPUs exits non-zero before any step."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("IMGCOMP_DIST_BACKEND", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4096", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "visible GPU" in p.stderr
