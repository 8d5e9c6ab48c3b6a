"""World-size-2 gloo rehearsal of bench.py's multi-GPU bookkeeping (CPU only):
each rank times its own GOP shard; the job time is the max over ranks, parity
the min, and the value counts every rank's units."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        wall = [0.50, 0.75][rank]
        exact = [334560, 334559][rank]
        w, e = bench.reduce_over_ranks(wall, exact, ws, torch.device("cpu"))
        got_ws, got_rank, _ = bench.dist_env()
        q.put((rank, w, e, got_ws, got_rank))
    finally:
        dist.destroy_process_group()


def test_bench_reductions_world_size_2():
    ws, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, w, e, got_ws, got_rank in res:
        assert w == 0.75 and e == 334559          # slowest rank, worst parity
        assert got_ws == ws and got_rank == rank
    # weak scaling: 2 ranks x 8160 units x 10 steps in the slowest rank's time
    assert bench.job_value(8160, 10, 2, 0.75) == pytest.approx(2 * 8160 * 10 / 0.75)


def test_single_rank_is_identity():
    assert bench.reduce_over_ranks(1.25, 7, 1, torch.device("cpu")) == (1.25, 7)
