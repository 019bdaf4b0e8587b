"""bench.py's multi-GPU contract on CPU: two gloo ranks (replicas only).

The driver launches `bench.py --gpus N` under torch.distributed.run; each rank decodes its own
replica and the job reports world * steps / (max over ranks of the timed region).  This runs
the same timed_region / job_value code on world_size 2 with uneven per-rank work and checks
that both ranks see the slowest rank's time.
"""
import os
import socket
import sys
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r "decodes" for 0.1 (r + 1) s; the job time is the slowest rank's
        out, elapsed = bench.timed_region(dist, None, lambda: (time.sleep(0.1 * (rank + 1)), rank)[1])
        q.put((rank, out, elapsed, bench.job_value(world, 64, elapsed)))
    finally:
        dist.destroy_process_group()


def test_timed_region_max_over_two_gloo_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [0, 1]  # each rank's own result comes back
    e0, e1 = res[0][2], res[1][2]
    assert e0 == e1  # every rank reports the same (max) time
    assert 0.2 <= e0 < 2.0  # at least the slow rank's 0.2 s
    assert res[0][3] == pytest.approx(2 * 64 / e0)  # weak scaling: both replicas' tokens


def test_timed_region_single_process():
    out, elapsed = bench.timed_region(None, None, lambda: 7)
    assert out == 7 and 0 <= elapsed < 1.0
    assert bench.job_value(1, 10, 2.0) == 5.0
