"""bench.py's multi-rank launch, on CPU (no GPU call: OCFFM_BENCH_DRY=1 stops
every rank after the gloo rendezvous and one all-reduce).

The driver's scale command is `python bench.py --gpus N`: without torchrun's
environment the script must start N ranks itself, and rank 0 must report
n_gpus = N with every rank accounted for.  Under torchrun (WORLD_SIZE set)
it must not spawn again, and a --gpus that disagrees with WORLD_SIZE is an
error rather than a mislabelled line.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ, OCFFM_BENCH_DRY="1", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=REPO)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_n_ranks(n):
    r = _run(["--gpus", str(n)])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    assert lines[0] == {"n_gpus": n, "ranks_seen": n, "launcher": "spawn"}


def test_single_gpu_does_not_spawn():
    r = _run(["--gpus", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == {"n_gpus": 1, "ranks_seen": 1, "launcher": "none"}


def test_torchrun_world_is_used():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29631", BENCH, "--gpus", "2"],
                       capture_output=True, text=True, timeout=240, cwd=REPO,
                       env=dict(os.environ, OCFFM_BENCH_DRY="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"n_gpus": 2, "ranks_seen": 2, "launcher": "torchrun"}]


def test_gpus_disagreeing_with_world_is_an_error():
    r = _run(["--gpus", "4"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)
