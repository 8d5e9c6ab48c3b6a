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
        wall = [0.50, 0.75, 0.60][rank]
        exact = [334560, 334559, 334560][rank]
        w, e = bench.reduce_over_ranks(wall, exact, ws, torch.device("cpu"))
        got_ws, got_rank, _ = bench.dist_env()
        per = bench.gather_rank_parity([2024 + 1000 * rank, 100 + rank, 100 + rank - (rank == 2), int(rank > 0)], ws,
                                       torch.device("cpu"))
        q.put((rank, w, e, got_ws, got_rank, per))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_bench_reductions(ws):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, w, e, got_ws, got_rank, per in res:
        assert w == 0.75 and e == 334559          # slowest rank, worst parity
        assert got_ws == ws and got_rank == rank
        # every rank holds every rank's own parity record, in rank order
        assert per == [[2024 + 1000 * r, 100 + r, 100 + r - (r == 2), int(r > 0)] for r in range(ws)]
    # weak scaling: 2 ranks x 8160 units x 10 steps in the slowest rank's time
    assert bench.job_value(8160, 10, 2, 0.75) == pytest.approx(2 * 8160 * 10 / 0.75)


def test_single_rank_is_identity():
    assert bench.reduce_over_ranks(1.25, 7, 1, torch.device("cpu")) == (1.25, 7)


def test_single_rank_parity_record():
    assert bench.gather_rank_parity([2024, 5, 5, 0], 1, torch.device("cpu")) == [[2024, 5, 5, 0]]


def test_ranks_search_distinct_gop_frames():
    """GOP sharding: rank 0 keeps the captured frame, every other rank gets the
    P-frame of its own seeded GOP; the oracle check of a rank's output counts
    every searched partition of its sample (here: the oracle's own answers)."""
    import numpy as np
    import oracle_lib as ol
    from jmme import BLOCK_RES, NSLOT
    cur, ref, req, unit_of, slots, expect, meta = bench.load_workload()
    c0, r0, s0 = bench.rank_frames(0, cur, ref, meta)
    assert c0 is cur and r0 is ref and s0 == meta["seed"]
    frames = [bench.rank_frames(r, cur, ref, meta) for r in (1, 2)]
    for c, r, sd in frames:
        assert c.shape == cur.shape and c.dtype == np.uint8 and not np.array_equal(c, cur)
    assert frames[0][2] != frames[1][2] and not np.array_equal(frames[0][0], frames[1][0])
    # a rank's result array filled with the oracle's answers for the sampled units
    c, r, _ = frames[0]
    sel = np.sort(np.random.default_rng(5).choice(len(req), 8, replace=False))
    mv, cost = ol.full_search_batch(c, r, bench._oracle_rows(req[sel]))
    out = np.zeros((len(req), NSLOT), BLOCK_RES)
    k = 0
    for u in sel:
        for s in range(NSLOT):
            if (int(req[u]["slot_mask"]) >> s) & 1:
                out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"] = mv[k, 0], mv[k, 1], cost[k]
                k += 1
    checked, exact = bench.oracle_parity(c, r, req, out, sample=8)
    assert checked == k and exact == k
    out[sel[0], 0]["cost"] += 1
    assert bench.oracle_parity(c, r, req, out, sample=8) == (k, k - 1)
