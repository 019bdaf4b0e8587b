"""bench.py's multi-rank launch on the GPU (replicas only).

The driver's scaling run is `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`,
one replica per GPU.  A one-GPU box cannot run that placement, so this runs the same launch with
two ranks on device 0 (XALM_BENCH_DEVICE=0): both replicas load, decode through the HIP library,
meet at the gloo barriers, and rank 0 prints the job line.  The two replicas share one GPU's HBM,
so the aggregate rate is not a scaling measurement; the test checks the launch and the line.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_replicas_on_one_gpu():
    steps = 16
    env = dict(os.environ, XALM_BENCH_DEVICE="0", TMPDIR="/tmp")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", str(steps), "--warmup", "2", "--no-cpu-baseline", "--kernel-iters", "2",
           "--prefill-tokens", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "replicas x2"
    # value = both replicas' tokens / the slowest rank's timed region
    assert d["value"] == pytest.approx(2 * 1000.0 / d["ms_per_step"], rel=1e-3)
    assert d["value"] > 100  # two 7B replicas on one GPU: each well above the CPU path
