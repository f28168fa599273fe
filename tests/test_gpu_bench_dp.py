"""bench.py's multi-process path as the driver launches it
(``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N``),
rehearsed with 2 ranks sharing cuda:0 over gloo (PINSAGE_DIST_BACKEND=gloo):
the run must exit 0 and rank 0 must print one JSON line for the whole job
(sharded precompute with its all-gather, data-parallel steps, max-over-ranks
timing), for both scaling modes."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_torchrun_two_ranks_gloo(scaling):
    env = dict(os.environ, PINSAGE_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--scaling", scaling]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["value"] > 0
    assert res["scaling"] == scaling
    per_gpu = res["config"]["batch_per_gpu"]
    assert res["config"]["global_batch"] == (2 * per_gpu if scaling == "weak" else 512)


def test_gpus_two_without_launcher_starts_the_ranks():
    """`bench.py --gpus 2` run directly (no torch.distributed.run) starts the
    two ranks itself and still prints one whole-job JSON line with n_gpus 2."""
    env = dict(os.environ, PINSAGE_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 3 and res["value"] > 0
