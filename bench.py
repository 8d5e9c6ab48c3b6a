#!/usr/bin/env python3
"""Headline benchmark: macroblocks/sec of JM 18.5 full-search integer-pel ME
(+-32, SAD, 1 reference) on a synthetic 1080p frame, bit-exact vs JM 18.5.

One "step" = the whole integer-pel search of one 1080p P-frame against one
reference: 8160 macroblock x reference units, each covering JM's 41 partition
searches (334,560 IntPelME calls), in one launch of the gfx950 unit kernel.

Workload (BASELINE.json configs[1]): the seeded synthetic clip and the exact
search requests (predictors, centres, lambda, ranges) JM 18.5 issued for that
frame, captured from the unmodified encoder (tests/golden/c2_syn_1080p_fs32).
After timing, the HIP results are compared with JM's own (mv, cost) outputs.

CPU baseline: the real JM 18.5 lencod (oracle/_ref/lencod, built from the
reference sources) encodes the same 2-frame clip with the same ME settings,
as N concurrent processes on the host cores this process may use (N <= 16,
the GPU box's share per GPU) and as one process alone; JM's own "Total ME
time" gives MB/s.  Falls back to the C restatement (oracle/) on a sample when
the JM build is absent.

Multi-GPU (torchrun): GOPs shard across ranks (weak scaling): rank r searches
the P-frame of its own seeded GOP (rank 0 the captured one), no collective on
the data path; barrier + max-over-ranks timing; every rank's parity is gathered
and reported (rank 0 against JM, the others against the oracle on a sample).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "--h.264-by-zhaodongyu_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

CASE = "c2_syn_1080p_fs32"
ALG_BYTES_PER_UNIT = 1516          # per MB x ref
ABSDIFF_PER_UNIT = 65 * 65 * 256   # (2R+1)^2 * 256 at R=32, SURVEY.md §8(d)
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md (spec)
# VALU ceiling for the SAD: v_sad_u8 lane-ops/s measured on MI355X by
# tools/ubench_valu.hip (profiles/round1/ubench_valu.jsonl), 4 abs-diffs each
VSAD_LANE_OPS = 35.5e12
VSAD_PEAK = VSAD_LANE_OPS * 4


def plan_items(req: np.ndarray) -> tuple[int, int]:
    """(items, abs-diffs) the plan kernel makes of a batch: per unit, the searched
    partitions with the same predictor, lambda, range and (FS) centre share one
    window sweep (me_plan_kernel, csrc/jmme_search.hip); an item sweeps its
    (2 rs + 1)^2 positions x 256 pels whatever partitions it serves.  The
    work-normalised VALU fraction divides the kernel's time by THIS work, not by
    one window per macroblock: JM's predictors give an adversarial frame's
    macroblocks up to 41 windows each."""
    items = absd = 0
    for r in req:
        mask = int(r["slot_mask"])
        keys = set()
        for s in range(41):
            if (mask >> s) & 1:
                b = r["blk"][s]
                keys.add((int(b["pred_x"]), int(b["pred_y"]), int(b["lambda"]), int(b["search_range"]),
                          int(b["center_x"]), int(b["center_y"])))
        items += len(keys)
        absd += sum((2 * k[3] + 1) ** 2 * 256 for k in keys)
    return items, absd

JM_CFG = """# minimal JM 18.5 lencod configuration written by bench.py (unlisted keys: JM defaults)
ProfileIDC            = 66
LevelIDC              = 40
IntraPeriod           = 0
QPISlice              = 28
QPPSlice              = 28
NumberReferenceFrames = 1
SearchMode            = -1
SearchRange           = 32
DisableSubpelME       = 1
EPZSSubPelGrid        = 0
RDOptimization        = 0
MDDistortion          = 0
LeakyBucketParamFile  = "leakybucketparam.cfg"
"""


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def load_workload(case: str = CASE):
    import golden_io as g
    c = g.Case(case)
    (f, lst, rf, idx), = list(c.groups())
    from jmme import FULL_SEARCH
    req, unit_of, slots = c.units(idx, FULL_SEARCH)
    expect = (c.r["out_mv_x"][idx], c.r["out_mv_y"][idx], c.r["out_cost"][idx])
    return c.cur[f], c.ref[(f, lst, rf)], req, unit_of, slots, expect, c.meta


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """Cores this process may use, capped at 16 (the GPU box's CPU share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline_jm(meta, procs: int = 1) -> dict | None:
    """JM 18.5 lencod on the same clip: `procs` independent encoder processes at
    once (JM is single-threaded; N processes on disjoint streams is how a host
    spends N cores on it).  Aggregate MB/s = all processes'
    MB x ref / the slowest one's own 'Total ME time'."""
    lencod = os.path.join(REPO, "oracle", "_ref", "lencod")
    if not os.path.exists(lencod):
        return None
    from jmme import synth
    w, h, frames = meta["w"], meta["h"], meta["frames"]
    with tempfile.TemporaryDirectory() as d:
        luma = synth.luma_sequence(w, h, frames, seed=meta["seed"], gmv=tuple(meta["gmv"]))
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, luma)
        cfg = os.path.join(d, "enc.cfg")
        open(cfg, "w").write(JM_CFG)
        runs = []
        t0 = time.time()
        for i in range(procs):
            wd = os.path.join(d, f"p{i}")
            os.makedirs(wd)
            args = [lencod, "-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
                    "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}", "-p", f"FramesToBeEncoded={frames}",
                    "-p", f"OutputFile={os.path.join(wd, 'o.264')}", "-p", f"ReconFile={os.path.join(wd, 'r.yuv')}"]
            runs.append(subprocess.Popen(args, cwd=wd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True))
        me = []
        for r in runs:
            out, _ = r.communicate(timeout=300)
            m = re.search(r"Total ME time for sequence\s*:\s*([0-9.]+) sec", out)
            if r.returncode != 0 or not m:
                return None
            me.append(float(m.group(1)))
        wall = time.time() - t0
    units = (w // 16) * ((h + 15) // 16) * (frames - 1)
    me_s = max(me)
    who = "one process" if procs == 1 else f"{procs} concurrent processes (slowest 'Total ME time' {me_s:.3f} s, " \
                                            f"fastest {min(me):.3f} s)"
    return {"value": round(procs * units / me_s, 2), "unit": "macroblocks/sec", "cores": procs, "kind": "reference",
            "cpu": cpu_model(),
            "sample": f"JM 18.5 lencod (gcc -O3) encoding the same synthetic 1080p clip, 1 I + {frames - 1} P frame, "
                      f"FS +-32, 1 ref, RDO off, {who}: {units} MB x ref per process in JM 'Total ME time' "
                      f"{me_s:.3f} s (wall {wall:.1f} s)"}


def _oracle_rows(req_units):
    from jmme import slot_of
    geo = {}
    for bt, (bw, bh) in {1: (16, 16), 2: (16, 8), 3: (8, 16), 4: (8, 8), 5: (8, 4), 6: (4, 8), 7: (4, 4)}.items():
        for by in range(0, 16, bh):
            for bx in range(0, 16, bw):
                geo[slot_of(bt, bx // 4, by // 4)] = (bx, by, bw, bh)
    rows = []
    for q in req_units:
        for s in range(41):
            if (int(q["slot_mask"]) >> s) & 1:
                b = q["blk"][s]
                bx, by, bw, bh = geo[s]
                rows.append([q["mb_x"] + bx, q["mb_y"] + by, bw, bh, b["pred_x"], b["pred_y"], b["center_x"],
                             b["center_y"], b["search_range"], b["lambda"], int(b["flags"] & 1)])
    return np.array(rows, np.int32)


def cpu_baseline_oracle(cur, ref, req, nunits=64) -> dict:
    import oracle_lib as ol
    rows = _oracle_rows(req[:nunits])
    t0 = time.time()
    ol.full_search_batch(cur, ref, rows)
    dt = time.time() - t0
    return {"value": round(nunits / dt, 2), "unit": "macroblocks/sec", "cores": 1, "kind": "port",
            "sample": f"C restatement of JM FS (oracle/me_oracle.c, early-exit SAD like JM) on the first "
                      f"{nunits} units of the workload: {dt:.2f} s"}


def pmc_traffic():
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(p):
        d = json.load(open(p))
        if d.get("case") == CASE:
            return d.get("bytes_per_launch")
    return None


SUBPEL_CASE = "subpel_syn_1080p_fs32"


def subpel_block(dev, local: int, iters: int = 20) -> dict | None:
    """JM's sub-pel half of the same ME, measured on rank 0:
    getSubImagesLuma of the 1080p reference + the 334,560 sub_pel_motion_estimation
    calls JM ran for the frame (FS +-32, SATD), with JM's inputs, parity vs JM."""
    import golden_io as g
    from jmme import BLOCK_RES, SP_CHECK0, SP_TEST8x8, SUBPEL_REQ, MotionEstimator, _lib
    if SUBPEL_CASE not in g.manifest():
        return None
    from subpel_cases import SubpelCase
    c = SubpelCase(SUBPEL_CASE)
    (f, lst, rf, idx), = list(c.groups())
    r = c.r
    q = np.zeros(len(idx), SUBPEL_REQ)
    for k in ("pos_x", "pos_y", "blocktype", "pred_x", "pred_y", "lambda_h", "lambda_q", "subthres", "metric_h",
              "metric_q", "start_hp", "start_qp", "search_pos2", "search_pos4"):
        q[k] = r[k][idx]
    q["ref_slot"] = r["list"][idx] * 32 + r["ref"][idx]
    q["mv_x"], q["mv_y"], q["min_mcost"], q["variant"] = r["mv_in_x"][idx], r["mv_in_y"][idx], r["min_mcost_in"][idx], \
        r["kind"][idx]
    q["flags"] = (np.where(r["test8x8"][idx] != 0, SP_TEST8x8, 0) |
                  np.where((r["rdopt"][idx] == 0) & (r["slice_type"][idx] != 1), SP_CHECK0, 0))
    me = MotionEstimator(device=local)
    me.upload_cur(c.cur[f])
    me.upload_ref(lst, rf, c.ref[(f, lst, rf)])
    me.subpel_validate(q)
    d_q = torch.from_numpy(q.view(np.uint8).copy()).to(dev)
    d_o = torch.zeros(len(q) * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / iters
    ms_i = timed(lambda: _lib.check(_lib.lib().jmme_interpolate_ref(me._ctx, lst, rf, st.cuda_stream)))
    ms_r = timed(lambda: me.subpel_refine_async(d_q.data_ptr(), len(q), 0, d_o.data_ptr(), st.cuda_stream))
    got = d_o.cpu().numpy().view(BLOCK_RES)
    emv, ecost = c.expected(idx)
    exact = int(np.sum((got["mv_x"] == emv[:, 0]) & (got["mv_y"] == emv[:, 1]) & (got["cost"] == ecost)))
    me.close()
    h, w = c.cur[f].shape
    ibytes = w * h + 16 * (w + 64) * (h + 40)
    # the same kernel on a 2160p reference: with the 1080p point, the launch's
    # fixed cost and the marginal streaming rate (t = fixed + bytes / rate)
    h4, w4 = 2160, 3840
    pic4 = np.random.default_rng(4).integers(0, 256, (h4, w4)).astype(np.uint16)
    with MotionEstimator({"SourceWidth": w4, "SourceHeight": h4}, device=local) as me4:
        me4.upload_cur(pic4)
        me4.upload_ref(0, 0, pic4)
        ms_i4 = timed(lambda: _lib.check(_lib.lib().jmme_interpolate_ref(me4._ctx, 0, 0, st.cuda_stream)))
    ibytes4 = w4 * h4 + 16 * (w4 + 64) * (h4 + 40)
    marginal = (ibytes4 - ibytes) / max((ms_i4 - ms_i) * 1e-3, 1e-9)   # bytes/s
    fixed_us = (ms_i - ibytes / marginal * 1e3) * 1e3
    return {"workload": "JM 18.5 sub_pel_motion_estimation for one 1080p P-frame (FS +-32, SATD half/quarter-pel)",
            "refinements": int(len(q)), "refine_ms": round(ms_r, 4), "interpolate_ms": round(ms_i, 4),
            "mb_per_s": round((w // 16) * (h // 16) / ((ms_r + ms_i) * 1e-3), 1),
            "interpolate_hbm_frac": round(ibytes / (ms_i * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "interpolate_2160p_ms": round(ms_i4, 4),
            "interpolate_2160p_hbm_frac": round(ibytes4 / (ms_i4 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "interpolate_marginal_hbm_frac": round(marginal / 1e9 / HBM_PEAK_GBS, 4),
            "interpolate_fixed_us": round(fixed_us, 2),
            "parity": {"reference": "JM 18.5 lencod (captured)", "refinements": int(len(q)), "bit_exact": exact},
            "jm_me_time_with_subpel": c.meta.get("jm_me_time")}


UHD_CASE = "c2_syn_4k_fs32"
ADV_CASE = "c2_syn_1080p_adv_fs32"
HBD_CASE = "c2_syn_1080p_fs32_10bit"


def case_block(dev, local: int, case: str, workload: str, iters: int = 10) -> dict | None:
    """The same full search on another captured frame, measured on rank 0 with
    JM 18.5's own requests for it, parity vs JM: the 4K frame (3840x2160, 32,400
    MB x ref) and the adversarial 1080p frame (every macroblock moved by its own
    random vector: the window centre is no good bound, so the exact elimination
    prunes little -- SURVEY §8(d)'s adversarial variant)."""
    import golden_io as g
    from jmme import BLOCK_RES, FULL_SEARCH, MotionEstimator, NSLOT
    if case not in g.manifest():
        return None
    cur, ref, req, unit_of, slots, expect, meta = load_workload(case)
    n = len(req)
    cfg = {"SearchRange": 32, "SearchMode": -1, "RDOptimization": 0}
    if meta.get("bits", 8) > 8:   # 16-bit planes: the 64-bit-key v_sad_u16 item kernel
        cfg["SourceBitDepthLuma"] = meta["bits"]
    me = MotionEstimator(cfg, device=local)
    me.upload_cur(cur)
    me.upload_ref(0, 0, ref)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    me.search_async(FULL_SEARCH, d_req.data_ptr(), n, d_out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize(dev)
    out = d_out.cpu().numpy().view(BLOCK_RES).reshape(n, NSLOT)[unit_of, slots]
    exact = int(np.sum((out["mv_x"] == expect[0]) & (out["mv_y"] == expect[1]) & (out["cost"] == expect[2])))
    outs = timed_buffers(d_out, iters)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kms = []
    e0.record(st)
    for i in range(iters):
        me.search_async(FULL_SEARCH, d_req.data_ptr(), n, outs[i % len(outs)].data_ptr(), st.cuda_stream)
        kms.append(me.last_kernel_ms())
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / iters
    timed = timed_parity(outs, min(iters, len(outs)), n, unit_of, slots, expect, "JM 18.5 lencod (captured)")
    me.close()
    kernel_ms = float(np.mean(kms))
    items, absd = plan_items(req)
    return {"workload": workload, "mb_per_step": n, "ms_per_frame": round(ms, 4),
            "kernel_ms": round(kernel_ms, 4), "mb_per_s": round(n / (ms * 1e-3), 1),
            "valu_frac": round(ABSDIFF_PER_UNIT * n / (kernel_ms * 1e-3) / VSAD_PEAK, 4),
            "items_per_step": items,
            "valu_frac_items": round(absd / (kernel_ms * 1e-3) / VSAD_PEAK, 4),
            "hbm_frac": round(ALG_BYTES_PER_UNIT * n / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
            "parity": {"reference": "JM 18.5 lencod (captured)", "searches": int(len(expect[0])),
                       "bit_exact": exact},
            "parity_timed": timed,
            "jm_me_time_at_capture": meta.get("jm_me_time")}


def uhd_block(dev, local: int, iters: int = 10) -> dict | None:
    return case_block(dev, local, UHD_CASE, "4K (3840x2160) FS +-32 SAD integer-pel, 1 ref, 32,400 MB x ref per "
                                            "frame, JM 18.5's own requests", iters)


def hbd_block(dev, local: int, iters: int = 10) -> dict | None:
    """configs[1] at 10 bits (High 10: JM's uint16 planes hold 10-bit samples):
    JM 18.5's own requests for the seeded clip at 10 bits, parity vs JM's capture.
    HBM bytes per unit double (16-bit samples); the VALU fraction is against the
    same v_sad_u8 ceiling, so a v_sad_u16 pass (half the samples per op) reads
    about half of it."""
    return case_block(dev, local, HBD_CASE, "1080p FS +-32 SAD integer-pel at 10 bits (SourceBitDepthLuma 10), "
                                            "1 ref, 8160 MB x ref, JM 18.5's own requests", iters)


def adversarial_block(dev, local: int, iters: int = 10) -> dict | None:
    return case_block(dev, local, ADV_CASE, "1080p FS +-32, adversarial content (per-MB random motion, no global "
                                            "motion), 8160 MB x ref, JM 18.5's own requests", iters)


def reduce_over_ranks(wall: float, exact: int, ws: int, dev) -> tuple[float, int]:
    """Job time = the slowest rank's time; parity = the worst rank's count.
    The only collectives of the run (no data-path exchange: ranks own whole GOPs)."""
    if ws == 1:
        return wall, exact
    import torch.distributed as dist
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    e = torch.tensor([exact], dtype=torch.int64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MIN)
    return float(t.item()), int(e.item())


def gather_rank_parity(info: list[int], ws: int, dev) -> list[list[int]]:
    """Every rank's own parity record ([frame seed, searches checked, bit-exact,
    reference: 0 JM / 1 oracle]) on every rank, in rank order: with GOP
    sharding each rank searches different frames, so each is checked on its own."""
    if ws == 1:
        return [list(info)]
    import torch.distributed as dist
    t = torch.tensor(info, dtype=torch.int64, device=dev)
    out = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return [[int(v) for v in x.tolist()] for x in out]


def rank_frames(rank: int, cur, ref, meta):
    """GOP sharding: the frames rank `rank` searches.  Rank 0 takes the captured
    P-frame (JM 18.5's own results for it are checked on every search); rank r > 0
    the P-frame of its own seeded GOP (clip seed + 1000 r, the same global
    motion), searched with the same requests and checked against the oracle on a
    sample.  Returns (cur, ref, clip seed)."""
    if rank == 0:
        return cur, ref, int(meta["seed"])
    from jmme import synth
    H, W = cur.shape
    seed = int(meta["seed"]) + 1000 * rank
    luma = synth.luma_sequence(W, H, 2, seed=seed, gmv=tuple(meta["gmv"]))
    return luma[1], luma[0], seed


def oracle_parity(cur, ref, req, out, sample: int = 96, seed: int = 5) -> tuple[int, int]:
    """(searches checked, bit-exact) of a seeded sample of units against the C
    restatement (oracle/me_oracle.c, itself pinned to JM 18.5's captures)."""
    import oracle_lib as ol
    from jmme import NSLOT
    sel = np.sort(np.random.default_rng(seed).choice(len(req), min(sample, len(req)), replace=False))
    mv, cost = ol.full_search_batch(cur, ref, _oracle_rows(req[sel]))
    got = [(out[u, s]["mv_x"], out[u, s]["mv_y"], out[u, s]["cost"]) for u in sel for s in range(NSLOT)
           if (int(req[u]["slot_mask"]) >> s) & 1]
    got = np.array(got, np.int64).reshape(-1, 3)
    exp = np.column_stack([mv[:, 0], mv[:, 1], cost]).astype(np.int64)
    return len(exp), int(np.sum(np.all(got == exp, axis=1)))


def timed_buffers(d_out, steps: int, cap_bytes: int = 2 << 30) -> list:
    """One output buffer per timed launch (up to cap_bytes in all, then reused
    round-robin), filled with 0xFF -- no valid result record -- so a launch that
    skipped or half-wrote a partition cannot pass for the one before it."""
    k = max(1, min(steps, cap_bytes // max(1, d_out.numel())))
    return [torch.full_like(d_out, 0xFF) for _ in range(k)]


def timed_parity(outs, launches: int, n: int, unit_of, slots, expect, reference: str) -> dict:
    """Bit-exactness of every timed launch's output, per partition search:
    (mv, cost) against `expect` -- JM 18.5's captured results on rank 0, the
    post-warm-up output (itself checked against the oracle) on the other ranks."""
    from jmme import BLOCK_RES, NSLOT
    ok = wrong = 0
    for d_o in outs[:launches]:
        g = d_o.cpu().numpy().view(BLOCK_RES).reshape(n, NSLOT)[unit_of, slots]
        bad = int(np.sum((g["mv_x"] != expect[0]) | (g["mv_y"] != expect[1]) | (g["cost"] != expect[2])))
        ok += bad == 0
        wrong += bad
    return {"reference": reference, "launches": launches, "launches_exact": ok,
            "searches_per_launch": int(len(expect[0])), "wrong_searches": wrong,
            "note": "every timed launch wrote its own 0xFF-poisoned output buffer"}


def job_value(units_per_rank_step: int, steps: int, ws: int, wall: float) -> float:
    """Whole-job throughput: every rank's units over the max-over-ranks time."""
    return units_per_rank_step * steps * ws / wall


def run_band(args, ws: int, rank: int, local: int, dev) -> None:
    """Strong scaling of one stream (jmme/shard.py): per step rank 0 -- the rank
    that owns the encoder loop -- broadcasts the current frame and the
    reconstructed reference over RCCL, each rank searches its macroblock-row
    band of the frame's 8160 units against the whole reference, and the results
    are all-gathered in raster order; rank 0 checks them against JM."""
    from jmme import BLOCK_RES, FULL_SEARCH, MotionEstimator, NSLOT, shard
    cur, ref, req, unit_of, slots, expect, meta = load_workload()
    n = len(req)
    H, W = cur.shape
    mb_rows = H // 16
    bands = [shard.band_units(req["mb_y"], r, ws, mb_rows) for r in range(ws)]
    counts = [len(b) for b in bands]
    mine = bands[rank]
    if rank == 0:
        d_cur = torch.from_numpy(np.ascontiguousarray(cur, np.uint8)).to(dev)
        d_ref = torch.from_numpy(np.ascontiguousarray(ref, np.uint8)).to(dev)
    else:
        d_cur = torch.empty((H, W), dtype=torch.uint8, device=dev)
        d_ref = torch.empty((H, W), dtype=torch.uint8, device=dev)
    me = MotionEstimator({"SearchRange": 32, "SearchMode": -1, "RDOptimization": 0}, device=local)
    d_req = torch.from_numpy(req[mine].view(np.uint8).copy()).to(dev)
    rec = NSLOT * BLOCK_RES.itemsize
    d_out = torch.zeros((len(mine), rec), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def search(d_r, nb, d_o):
        me.search_planes_async(FULL_SEARCH, d_cur.data_ptr(), d_ref.data_ptr(), W, W, H, d_r.data_ptr(), nb,
                               d_o.data_ptr(), stream.cuda_stream)

    def step():
        return shard.band_step([d_cur, d_ref], d_req, len(mine), d_out, counts, search)

    for _ in range(args.warmup):
        full = step()
    torch.cuda.synchronize(dev)
    order = np.concatenate(bands)
    out = np.zeros((n, NSLOT), BLOCK_RES)
    out[order] = full.cpu().numpy().reshape(-1).view(BLOCK_RES).reshape(n, NSLOT)
    res = out[unit_of, slots]
    exact = int(np.sum((res["mv_x"] == expect[0]) & (res["mv_y"] == expect[1]) & (res["cost"] == expect[2])))
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    wall, exact = reduce_over_ranks(wall, exact, ws, dev)
    me.close()
    if rank == 0:
        print(json.dumps({
            "metric": "macroblocks/sec full-search ME @1080p; bit-exact MV/SAD vs JM18.5",
            "value": round(n * args.steps / wall, 1), "unit": "macroblocks/sec", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded 1080p clip; JM 18.5's own search requests for it)",
            "config": {"workload": "1080p FS +-32 SAD integer-pel, 1 ref, 8160 MB x ref per step (configs[1])",
                       "search_range": 32, "mb_per_step": n, "band_units": counts,
                       "parallelism": f"mb-row-band x{ws}, planes broadcast + results all-gathered over RCCL"},
            "parity": {"reference": "JM 18.5 lencod (captured)", "searches": int(len(expect[0])),
                       "bit_exact": exact}}))


def run_fractal(args, ws: int, rank: int, local: int, dev) -> None:
    """BASELINE configs[2] over N GPUs: every 4x4 range block
    of a 1080p frame against the full domain pool.  Range blocks are independent
    (encode_Oneframe, ZL/src/image.c:1108-1127), so each rank takes a band of
    range-block rows: rank 0 -- the frame's owner -- broadcasts the range plane
    and the reference (domain) plane over RCCL, every rank builds its own domain
    images from the received reference and searches its band against the whole
    pool, and the per-block results are all-gathered in raster order.  Strong
    scaling (one frame per step); rank 0 checks a seeded sample of the gathered
    results against the restatement (parity with the thesis unpinned)."""
    from jmme import FRACTAL_REQ, FRACTAL_RES, MotionEstimator, shard, synth
    W, H = 1920, 1080
    rows = H // 4
    if rank == 0:
        luma = synth.luma_sequence(W, H, 2, seed=77, gmv=(3, 2))
        d_org = torch.from_numpy(luma[1].astype(np.uint8)).to(dev)
        d_ref = torch.from_numpy(luma[0].astype(np.uint8)).to(dev)
    else:
        d_org = torch.empty((H, W), dtype=torch.uint8, device=dev)
        d_ref = torch.empty((H, W), dtype=torch.uint8, device=dev)
    spans = [shard.band_rows(rows, r, ws) for r in range(ws)]
    counts = [(b - a) * (W // 4) for a, b in spans]
    a, b = spans[rank]
    ys, xs = np.mgrid[4 * a:4 * b:4, 0:W:4]
    req = np.zeros(xs.size, FRACTAL_REQ)
    req["block_x"], req["block_y"], req["bsx"], req["bsy"] = xs.ravel(), ys.ravel(), 4, 4
    n = len(req)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_words = torch.empty(W * H, dtype=torch.int32, device=dev)
    d_out = torch.zeros((max(n, 1), FRACTAL_RES.itemsize), dtype=torch.uint8, device=dev)
    me = MotionEstimator(device=local)
    st = torch.cuda.current_stream(dev).cuda_stream

    def encode_band(out):
        me.fractal_words_async(d_ref.data_ptr(), W, W, H, d_words.data_ptr(), st)
        if n:
            me.fractal_search_async(d_org.data_ptr(), W, d_words.data_ptr(), W, H, max(W, H), d_req.data_ptr(), n,
                                    out.data_ptr(), st)

    def step():
        return shard.band_exchange([d_org, d_ref], d_out, counts, lambda: encode_band(d_out))

    for _ in range(args.warmup):
        full = step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        full = step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    exact = 1 << 30                     # rank 0 checks; the MIN over ranks is its count
    if rank == 0:
        import oracle_lib as ol
        got = full.cpu().numpy().reshape(-1).view(FRACTAL_RES)
        n_all = (W // 4) * rows
        sel = np.sort(np.random.default_rng(3).choice(n_all, 128, replace=False))
        bx, by = (sel % (W // 4)) * 4, (sel // (W // 4)) * 4
        rq = np.stack([bx, by, np.full_like(bx, 4), np.full_like(bx, 4)], 1).astype(np.int32)
        exp, xy = ol.fractal_search_batch_par(d_org.cpu().numpy(), d_ref.cpu().numpy(), max(W, H), rq)
        g = got[sel]
        exact = int(np.sum((g["rms"] == exp[:, 0]) & (g["scale"] == exp[:, 1]) & (g["offset"] == exp[:, 2]) &
                           (g["x"] == xy[:, 0]) & (g["y"] == xy[:, 1])))
    wall, exact = reduce_over_ranks(wall, exact, ws, dev)
    me.close()
    if rank == 0:
        nblk = (W // 4) * rows
        print(json.dumps({
            "metric": "fractal range blocks/sec (1080p, 4x4, full domain pool; configs[2])",
            "value": round(nblk * args.steps / wall, 1), "unit": "range blocks/sec", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded 1080p pair)",
            "config": {"workload": "1080p fractal full_search, 129,600 4x4 range blocks vs 2,064,609 domain positions "
                                   "each (configs[2])", "band_blocks": counts,
                       "parallelism": f"range-block-row band x{ws}, planes broadcast + results all-gathered over RCCL"},
            "parity": {"reference": "oracle/fractal_oracle.c (parity with the thesis unpinned)", "sample": 128,
                       "bit_exact": exact}}))


def run_encoder(args, ws: int, rank: int, local: int) -> None:
    """The product's own multi-GPU form (`--shard encoder`):
    each rank runs JM 18.5 lencod_jmme over its own closed GOPs on its GPU
    (integration/jmme_gop.c: one encoder process per GOP, StartFrame /
    FramesToBeEncoded, the device fixed in the child's environment before the
    encoder starts) -- weak scaling, no data-path collective; this process never
    touches the GPU, so the ranks meet over gloo for the barrier and the
    max-over-ranks time.  value = every rank's encoded macroblocks / the slowest
    rank's wall time.  After timing, each rank's GOPs go through the stock
    lencod with the same arguments (its host share, concurrent processes) and
    every GOP's bitstream and reconstruction are compared byte for byte."""
    import bench_blocks
    if ws > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        dist.barrier()
    params, psize, ptext = bench_blocks.encoder_preset(args.enc_preset)
    w, h = (int(x) for x in args.enc_size.split("x")) if args.enc_size else psize
    # host placement: each rank's encoders on its GPU's NUMA-local cores (its share
    # of them when GPUs share a node), one core per running encoder
    local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", ws))
    cpus, source = bench_blocks.gpu_local_cpus(local, local_ws) if (ws > 1 or args.enc_pin) else (None, "unpinned")
    # the timed region is the launcher's own run (clip generation excluded); the
    # stock encodes (parity, host baseline) follow once every rank's run is done
    blk = bench_blocks.encoder_gop_block(device=local, rank=rank, gops=args.enc_gops, gop=args.enc_gop, size=(w, h),
                                         per_gpu=args.enc_per_gpu, check_stock=True, encoder=args.enc_encoder,
                                         between=(lambda: dist.barrier()) if ws > 1 else None,
                                         preset=args.enc_preset, cpus=cpus)
    if blk is None:
        raise SystemExit("--shard encoder needs integration/_build/{lencod_jmme,jmme_gop} and oracle/_ref/lencod")
    blk["host_placement"]["source"] = source
    wall = blk["wall_s"]
    ok = blk["parity"]["byte_identical_gops"]
    rec = [wall, float(ok), float(blk["host_baseline"]["encoder_mb_per_s"]), float(blk["macroblocks"])]
    cores = cpus or []
    core_rec = torch.zeros(256, dtype=torch.int64)   # this rank's cores (-1 padded), gathered for the report
    core_rec.fill_(-1)
    core_rec[:min(256, len(cores))] = torch.tensor(cores[:256], dtype=torch.int64)
    if ws > 1:
        t = torch.tensor(rec, dtype=torch.float64)
        allr = [torch.zeros_like(t) for _ in range(ws)]
        dist.all_gather(allr, t)
        recs = [x.tolist() for x in allr]
        allc = [torch.zeros_like(core_rec) for _ in range(ws)]
        dist.all_gather(allc, core_rec)
        core_sets = [[int(c) for c in x.tolist() if c >= 0] for x in allc]
    else:
        recs = [rec]
        core_sets = [list(cores)]
    if rank == 0:
        job_wall = max(r[0] for r in recs)
        mbs = sum(r[3] for r in recs)
        print(json.dumps({
            "metric": f"encoder macroblocks/sec (JM 18.5 lencod_jmme, closed GOPs, ME on the GPU; preset "
                      f"{args.enc_preset})",
            "value": round(mbs / job_wall, 1), "unit": "macroblocks/sec", "n_gpus": ws, "steps": 1, "warmup": 0,
            "ms_per_step": round(job_wall * 1e3, 1), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic (a seeded {w}x{h} clip per rank)",
            "config": {"workload": f"{args.enc_gops} closed GOPs x {args.enc_gop} frames per GPU through lencod_jmme, "
                                   f"{w}x{h}, {ptext}", "preset": args.enc_preset, "per_gpu_encoders": args.enc_per_gpu,
                       "parallelism": f"closed-GOP shard x{ws} (integration/jmme_gop.c per rank, no collective)"},
            "per_rank": [{"rank": r, "wall_s": round(x[0], 3), "byte_identical_gops": int(x[1]),
                          "macroblocks": int(x[3]), "host_encoder_mb_per_s": x[2],
                          "cpus": bench_blocks._cpulist_text(core_sets[r]) if core_sets[r] else "unpinned"}
                         for r, x in enumerate(recs)],
            "parity": {"reference": "JM 18.5 lencod (stock, same GOP arguments)", "gops": args.enc_gops * ws,
                       "byte_identical_gops": int(sum(x[1] for x in recs))},
            "cpu_baseline": {"value": round(sum(x[2] for x in recs), 1), "unit": "macroblocks/sec",
                             "cores": blk["host_baseline"]["procs"] * ws, "kind": "reference",
                             "sample": "the same GOPs through the stock lencod, concurrent processes per rank"},
            "rank0": blk}))
    if ws > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-subpel", action="store_true")
    ap.add_argument("--no-uhd", action="store_true")
    ap.add_argument("--no-adversarial", action="store_true")
    ap.add_argument("--no-hbd", action="store_true")
    ap.add_argument("--no-fractal", action="store_true", help="skip the configs[2] block (fractal full pool)")
    ap.add_argument("--no-hybrid", action="store_true", help="skip the configs[4] block (joint codec frame)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the in-encoder block (lencod vs lencod_jmme)")
    ap.add_argument("--headline-only", action="store_true", help="the headline line alone (no CPU baseline, no "
                                                                  "side blocks): profiling runs")
    ap.add_argument("--workload", choices=["me", "fractal"], default="me",
                    help="me: the headline (configs[1]); fractal: configs[2] range-block bands over the ranks")
    ap.add_argument("--shard", choices=["gop", "band", "encoder"], default="gop",
                    help="gop: each rank searches its own frames (weak, default); band: rank 0 broadcasts "
                         "each frame's planes over RCCL and every rank searches an MB-row band (strong); encoder: "
                         "each rank runs the drop-in encoder (lencod_jmme) over its own closed GOPs on its GPU "
                         "(integration/jmme_gop.c, weak)")
    ap.add_argument("--no-encoder", action="store_true", help="skip the GOP-sharded encoder block of the N=1 line")
    ap.add_argument("--no-f3", action="store_true", help="skip the (f)3 block (inter residual coding on the GPU)")
    ap.add_argument("--enc-gops", type=int, default=16, help="--shard encoder / encoder block: GOPs per GPU")
    ap.add_argument("--enc-gop", type=int, default=4, help="frames per GOP (1 I + P)")
    ap.add_argument("--enc-per-gpu", type=int, default=8, help="encoder processes at once per GPU")
    ap.add_argument("--enc-size", default=None, help="clip size WxH (default: the preset's)")
    ap.add_argument("--enc-preset", choices=["fs", "epzs4k"], default="fs",
                    help="fs: configs[1]'s settings at 1080p; epzs4k: configs[3] as configured (4K, "
                         "encoder_baseline.cfg's EPZS keys, RDO on)")
    ap.add_argument("--enc-pin", action="store_true", help="pin the encoders at N=1 too (N>1 always pins)")
    ap.add_argument("--no-encoder-4k", action="store_true", help="skip the configs[3] GOP-encoder block of the N=1 line")
    ap.add_argument("--enc4k-gops", type=int, default=8, help="encoder_gop_epzs4k block: GOPs (of 2 frames)")
    ap.add_argument("--enc-encoder", default=None, help="encoder binary (default integration/_build/lencod_jmme; "
                                                         "a CPU rehearsal passes the stock oracle/_ref/lencod)")
    args = ap.parse_args()
    if args.headline_only:
        for k in ("no_cpu_baseline", "no_subpel", "no_uhd", "no_adversarial", "no_hbd", "no_fractal", "no_hybrid",
                  "no_dropin", "no_encoder", "no_encoder_4k", "no_f3"):
            setattr(args, k, True)

    ws, rank, local = dist_env()
    if args.shard == "encoder":   # before anything touches the GPU: this process only launches encoders
        run_encoder(args, ws, rank, local)
        return
    # N = 1: the GOP-encoder blocks run first, before this process touches the
    # GPU.  Its own hardware queues would otherwise join the encoders' (8 x 2)
    # on the device and oversubscribe the queues the hardware maps: the
    # encoders' queues are then time-sliced and their resident EPZS servers wait
    # seconds (profiles/round6/gop_queues/).
    pre = {}
    if ws == 1 and args.workload == "me" and args.shard == "gop":
        import bench_blocks
        if not args.no_encoder:
            # the product's multi-GPU form at N = 1: closed GOPs through lencod_jmme
            # (the same as --shard encoder on one GPU), with the host baseline
            size = tuple(int(x) for x in args.enc_size.split("x")) if args.enc_size else None
            pre["encoder_gop"] = bench_blocks.encoder_gop_block(device=local, rank=0, gops=args.enc_gops,
                                                                gop=args.enc_gop, size=size,
                                                                per_gpu=args.enc_per_gpu, encoder=args.enc_encoder,
                                                                preset=args.enc_preset)
        if not args.no_encoder_4k:
            # configs[3] as configured: 4K, encoder_baseline.cfg's EPZS keys, RDO on
            # (--shard encoder --enc-preset epzs4k is the same over N GPUs)
            pre["encoder_gop_epzs4k"] = bench_blocks.encoder_gop_block(device=local, rank=0, gops=args.enc4k_gops,
                                                                       gop=2, per_gpu=min(8, args.enc4k_gops),
                                                                       encoder=args.enc_encoder, preset="epzs4k")
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    if args.workload == "fractal":
        run_fractal(args, ws, rank, local, dev)
        if ws > 1:
            torch.distributed.destroy_process_group()
        return
    if args.shard == "band":
        run_band(args, ws, rank, local, dev)
        if ws > 1:
            torch.distributed.destroy_process_group()
        return

    from jmme import BLOCK_RES, FULL_SEARCH, MotionEstimator, NSLOT
    cur, ref, req, unit_of, slots, expect, meta = load_workload()
    n = len(req)
    cur, ref, clip_seed = rank_frames(rank, cur, ref, meta)
    me = MotionEstimator({"SearchRange": 32, "SearchMode": -1, "RDOptimization": 0}, device=local)
    me.upload_cur(cur)
    me.upload_ref(0, 0, ref)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n * NSLOT * BLOCK_RES.itemsize, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step(d_o=d_out):
        me.search_async(FULL_SEARCH, d_req.data_ptr(), n, d_o.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    # parity of this rank's output: JM 18.5's own results (rank 0, the captured
    # frame) or the oracle on a sample (its own GOP's frame)
    full = d_out.cpu().numpy().view(BLOCK_RES).reshape(n, NSLOT)
    if rank == 0:
        out = full[unit_of, slots]
        checked = len(expect[0])
        exact = int(np.sum((out["mv_x"] == expect[0]) & (out["mv_y"] == expect[1]) & (out["cost"] == expect[2])))
    else:
        checked, exact = oracle_parity(cur, ref, req, full)
    per_rank = gather_rank_parity([clip_seed, checked, exact, int(rank != 0)], ws, dev)

    # kernel duration: HIP events around the unit kernel, on its stream
    kms = []
    for _ in range(min(args.steps, 20)):
        step()
        kms.append(me.last_kernel_ms())
    kernel_ms = float(np.mean(kms))

    # every timed launch writes its own output buffer, poisoned beforehand, so the
    # work inside the timed region is checked too (parity_timed), not only the
    # post-warm-up launch above
    timed_outs = timed_buffers(d_out, args.steps)
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(timed_outs[i % len(timed_outs)])
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if ws > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    wall, _ = reduce_over_ranks(wall, exact, ws, dev)
    own = full[unit_of, slots]
    timed = timed_parity(timed_outs, min(args.steps, len(timed_outs)), n, unit_of, slots,
                         expect if rank == 0 else (own["mv_x"], own["mv_y"], own["cost"]),
                         "JM 18.5 lencod (captured)" if rank == 0 else "post-warm-up output (oracle-checked)")
    timed_worst = reduce_over_ranks(0.0, timed["launches_exact"] - timed["launches"], ws, dev)[1]

    if rank == 0:
        value = job_value(n, args.steps, ws, wall)
        ms_per_step = wall * 1e3 / args.steps
        ach = ALG_BYTES_PER_UNIT * n / (kernel_ms * 1e-3) / 1e9
        items_step, absd_step = plan_items(req)
        cpu = None
        if not args.no_cpu_baseline and ws == 1:       # the CPU baseline is an N=1 figure
            # every host core the GPU's share allows, each running JM (the headline
            # baseline), and one core alone beside it
            ncpu = host_cores()
            cpu = cpu_baseline_jm(meta, ncpu) if ncpu > 1 else None
            one = cpu_baseline_jm(meta, 1)
            if cpu is None:
                cpu = one or cpu_baseline_oracle(cur, ref, req)
            elif one is not None:
                cpu["single_core"] = {"value": one["value"], "sample": one["sample"]}
        line = {
            "metric": "macroblocks/sec full-search ME @1080p; bit-exact MV/SAD vs JM18.5",
            "value": round(value, 1),
            "unit": "macroblocks/sec",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded 1080p clip; JM 18.5's own search requests for it)",
            "config": {"workload": "1080p FS +-32 SAD integer-pel, 1 ref, 8160 MB x ref per step (configs[1])",
                       "search_range": 32, "mb_per_step": n,
                       "partition_searches_per_step": int(sum(bin(int(m)).count("1") for m in req["slot_mask"])),
                       "parallelism": f"frame-shard x{ws}" + ("" if ws == 1 else
                                                                  ": rank r searches the P-frame of its own GOP")},
            "parity": {"reference": "JM 18.5 lencod (captured)", "searches": int(len(expect[0])),
                       "bit_exact": exact},
            "parity_timed": dict(timed, all_ranks_exact=timed_worst == 0),
            "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": pmc_traffic(),
                         "kernel_ms": round(kernel_ms, 4),
                         "note": "integer SAD search is VALU-bound, see valu"},
            "valu": {"achieved_absdiff_per_s": round(ABSDIFF_PER_UNIT * n / (kernel_ms * 1e-3), 1),
                     "peak_absdiff_per_s": VSAD_PEAK,
                     "peak_source": "measured v_sad_u8 rate (tools/ubench_valu.hip) x 4 abs-diffs",
                     "frac": round(ABSDIFF_PER_UNIT * n / (kernel_ms * 1e-3) / VSAD_PEAK, 4),
                     "items_per_step": items_step,
                     "frac_items": round(absd_step / (kernel_ms * 1e-3) / VSAD_PEAK, 4),
                     "note": "frac: one (2R+1)^2 window per MB (SURVEY 8(d)); frac_items: the windows the plan "
                             "kernel really sweeps (plan_items)"},
            "event_ms_per_step": round(ev_ms / args.steps, 4),
            "per_rank": [{"rank": r, "clip_seed": sd, "searches_checked": ck, "bit_exact": ex,
                          "reference": "JM 18.5 lencod (captured)" if kind == 0 else
                          "oracle/me_oracle.c (pinned to JM), seeded sample of 96 units"}
                         for r, (sd, ck, ex, kind) in enumerate(per_rank)],
            "cpu_baseline": cpu,
        }
        if not args.no_subpel and ws == 1:
            line["subpel"] = subpel_block(dev, local)
        if not args.no_uhd and ws == 1:
            line["uhd"] = uhd_block(dev, local)
        if not args.no_adversarial and ws == 1:
            line["adversarial"] = adversarial_block(dev, local)
        if not args.no_hbd and ws == 1:
            line["hbd"] = hbd_block(dev, local)
        if not args.no_fractal and ws == 1:
            import bench_blocks
            line["fractal"] = bench_blocks.fractal_block(dev, local)
        if not args.no_hybrid and ws == 1:
            import bench_blocks
            line["hybrid"] = bench_blocks.hybrid_block(dev, local, load_workload)
        for k in ("encoder_gop", "encoder_gop_epzs4k"):   # (measured before the GPU was touched, above)
            if k in pre:
                line[k] = pre[k]
        if not args.no_f3 and ws == 1:
            import bench_blocks
            # mode decision's inter residual coding from the GPU (off by default in the product)
            line["f3"] = bench_blocks.f3_block()
        if not args.no_dropin and ws == 1:
            import bench_blocks
            # FS / FFS (configs[1] settings), FS / FFS with encoder_baseline.cfg's
            # sub-pel keys, EPZS (configs[3]'s algorithm, the same file's EPZS keys);
            # each against one core and against host_cores() concurrent encoders
            line["dropin"] = bench_blocks.dropin_block()
        print(json.dumps(line))
    me.close()
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
