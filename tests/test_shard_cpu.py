"""World-size-2/3 gloo rehearsal of the band-sharded stream (jmme/shard.py,
bench.py --shard band) on the CPU: rank 0 owns the frame and broadcasts the
current and reference planes, each rank searches its macroblock-row band
(here with the C restatement standing in for the HIP engine, reading the
planes it received), the bands are all-gathered, and the assembled results
equal a single-process search of every unit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import oracle_lib as ol

W, H, R = 96, 80, 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _workload():
    from jmme import MB_REQ, NSLOT, synth
    luma = synth.luma_sequence(W, H, 2, seed=3, gmv=(2, 1))
    rng = np.random.default_rng(4)
    ys, xs = np.mgrid[0:H:16, 0:W:16]
    req = np.zeros(xs.size, MB_REQ)
    req["mb_x"], req["mb_y"] = xs.ravel(), ys.ravel()
    req["slot_mask"] = (1 << NSLOT) - 1
    for u in range(len(req)):
        for s in range(NSLOT):
            b = req["blk"][u, s]
            c = rng.integers(-2, 3, size=2) * 4
            b["center_x"], b["center_y"] = c
            b["pred_x"], b["pred_y"] = c + rng.integers(-3, 4, size=2)
            b["search_range"] = R
            b["lambda"] = rng.integers(0, 200)
            req["blk"][u, s] = b
    return luma[1].astype(np.uint8), luma[0].astype(np.uint8), req


def _search_cpu(cur, ref, req):
    """stand-in for the engine: BLOCK_RES [n, NSLOT] from the restatement"""
    from jmme import BLOCK_RES, NSLOT
    out = np.zeros((len(req), NSLOT), BLOCK_RES)
    if len(req) == 0:
        return out
    mv, cost = ol.full_search_batch(cur, ref, bench._oracle_rows(req))
    k = 0
    for u in range(len(req)):
        for s in range(NSLOT):
            out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"] = mv[k, 0], mv[k, 1], cost[k]
            k += 1
    return out


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from jmme import BLOCK_RES, NSLOT, shard
        cur, ref, req = _workload()
        bands = [shard.band_units(req["mb_y"], r, ws, H // 16) for r in range(ws)]
        counts = [len(b) for b in bands]
        mine = bands[rank]
        # only the owner holds the frame; the others must get it from the broadcast
        t_cur = torch.from_numpy(cur.copy()) if rank == 0 else torch.zeros((H, W), dtype=torch.uint8)
        t_ref = torch.from_numpy(ref.copy()) if rank == 0 else torch.zeros((H, W), dtype=torch.uint8)
        t_req = torch.from_numpy(req[mine].view(np.uint8).copy())
        rec = NSLOT * BLOCK_RES.itemsize
        t_out = torch.zeros((len(mine), rec), dtype=torch.uint8)

        def search(d_req, n, d_out):
            r = d_req.numpy().view(req.dtype)[:n]
            res = _search_cpu(t_cur.numpy(), t_ref.numpy(), r)
            d_out[:n] = torch.from_numpy(res.view(np.uint8).reshape(n, rec))

        full = shard.band_step([t_cur, t_ref], t_req, len(mine), t_out, counts, search)
        order = np.concatenate(bands)
        got = np.zeros((len(req), NSLOT), BLOCK_RES)
        got[order] = full.numpy().reshape(-1).view(BLOCK_RES).reshape(len(req), NSLOT)
        q.put((rank, counts, mine.tolist(), got.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_band_shard_equals_single_process(ws):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cur, ref, req = _workload()
    want = _search_cpu(cur, ref, req).tobytes()
    seen = []
    for rank, counts, mine, got in res:
        assert sum(counts) == len(req)
        seen += mine
        assert got == want, f"rank {rank}: assembled band results differ from the single-process search"
    assert sorted(seen) == list(range(len(req)))       # every unit searched exactly once


def test_band_rows_partition():
    from jmme import shard
    for rows, ws in [(68, 8), (5, 8), (135, 3), (1, 1)]:
        spans = [shard.band_rows(rows, r, ws) for r in range(ws)]
        assert spans[0][0] == 0 and spans[-1][1] == rows
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        sizes = [b - a for a, b in spans]
        assert max(sizes) - min(sizes) <= 1
    assert [shard.gop_owner(g, 4) for g in range(6)] == [0, 1, 2, 3, 0, 1]


# ---- fractal P-frame, MB-row bands -----------------------
FW, FH, FVIEWS = 96, 80, 2


def _fractal_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from fractal_scenes import gate_scene
        from jmme import FRACTAL_MB, shard
        org, views = gate_scene(FW, FH, 5, FVIEWS, scale=6)
        rows = [shard.band_rows(FH // 16, r, ws) for r in range(ws)]
        counts = [(b - a) * (FW // 16) for a, b in rows]
        # only the owner holds the frame; the others get it from the broadcast
        planes = [torch.from_numpy(p.copy()) if rank == 0 else torch.zeros((FH, FW), dtype=torch.uint8)
                  for p in [org] + views]
        rec = FRACTAL_MB.itemsize
        t_out = torch.zeros((counts[rank], rec), dtype=torch.uint8)

        def encode_band(d_out):
            # stand-in for the HIP band encoder: the restatement of the planes this
            # rank received, restricted to its rows (the GPU test checks that the
            # HIP band form equals the whole-plane rows)
            t = ol.fractal_encode_mbs(planes[0].numpy(), [p.numpy() for p in planes[1:]], 7, 8.0, 5.0)
            a, b = rows[rank]
            d_out[:] = torch.from_numpy(t[a * (FW // 16):b * (FW // 16)].view(np.uint8).reshape(-1, rec).copy())

        full = shard.fractal_band_step(planes, t_out, counts, encode_band)
        q.put((rank, counts, full.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_fractal_band_shard_equals_single_process(ws):
    from fractal_scenes import gate_scene
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fractal_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    org, views = gate_scene(FW, FH, 5, FVIEWS, scale=6)
    want = ol.fractal_encode_mbs(org, views, 7, 8.0, 5.0)
    want = np.array(want, copy=True)
    for rank, counts, got in res:
        assert sum(counts) == (FW // 16) * (FH // 16)
        g = np.frombuffer(got, want.dtype).copy()
        for t in (g, want):
            t["chun"][np.isnan(t["chun"])] = 0
        assert g.tobytes() == want.tobytes(), f"rank {rank}: gathered trees differ from the single-process encode"
