"""bench.py's blocks for the BASELINE configs other than the headline one, each
measured on rank 0 at N = 1 and printed inside the same JSON line:

* fractal_block -- configs[2]: the thesis's full_search (ZL/src/block_enc.c:
  1933-1977) of every 4x4 range block of a 1080p frame against the full domain
  pool, on the pruned MFMA pool search (csrc/jmme_fractal_pool.hip);
* hybrid_block  -- configs[4]: one frame of the joint fractal + H.264 codec
  (jmme/hybrid.py): Y/U/V quadtrees over 4 views at the thesis's R = 7, their
  reconstruction, and JM's FS +-32 ME of the bench frame;
* dropin_block  -- the drop-in encoder itself: JM 18.5 lencod, stock vs
  lencod_jmme (integration/), FS and FFS at 1080p, JM's own "Total ME time"
  per P-frame and byte identity of the outputs.

Each block reports its own parity against the restatement (fractal, parity
with the thesis unpinned) or JM (ME), and a CPU baseline of the restatement on
a bounded sample ("port").  The oracle is the checker only, never timed as
the GPU's work."""
from __future__ import annotations

import time

import numpy as np
import torch

MFMA_BF16_PEAK = 2.5e15        # MI355X_MICROARCH.md: dense BF16 MFMA
FLOPS_PER_PAIR_44 = 64         # bound test of one (domain position, 4x4 range block) pair: 16 MACs x 2 (hi, lo)


def _timed(fn, iters, dev):
    fn()
    torch.cuda.synchronize(dev)
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / iters


def fractal_block(dev, local: int, iters: int = 5, sample: int = 256) -> dict:
    """configs[2]: 1920x1080, 129,600 4x4 range blocks, full domain pool
    ((W-3)(H-3) = 2,064,609 positions per block).  One step = the reference's
    words image + the search of every block (seeds, pool images, bound test,
    exact survivors), inputs resident."""
    import oracle_lib as ol
    from jmme import FRACTAL_REQ, FRACTAL_RES, MotionEstimator, synth
    W, H = 1920, 1080
    luma = synth.luma_sequence(W, H, 2, seed=77, gmv=(3, 2))
    org, ref = luma[1].astype(np.uint8), luma[0].astype(np.uint8)
    ys, xs = np.mgrid[0:H:4, 0:W:4]
    req = np.zeros(xs.size, FRACTAL_REQ)
    req["block_x"], req["block_y"], req["bsx"], req["bsy"] = xs.ravel(), ys.ravel(), 4, 4
    n, R = len(req), max(W, H)
    st = torch.cuda.current_stream(dev).cuda_stream
    d_org, d_ref = torch.from_numpy(org).to(dev), torch.from_numpy(ref).to(dev)
    d_words = torch.empty(W * H, dtype=torch.int32, device=dev)
    d_req = torch.from_numpy(req.view(np.uint8).copy()).to(dev)
    d_out = torch.empty(n * FRACTAL_RES.itemsize, dtype=torch.uint8, device=dev)
    me = MotionEstimator(device=local)

    def step():
        me.fractal_words_async(d_ref.data_ptr(), W, W, H, d_words.data_ptr(), st)
        me.fractal_search_async(d_org.data_ptr(), W, d_words.data_ptr(), W, H, R, d_req.data_ptr(), n,
                                d_out.data_ptr(), st)
    step()
    torch.cuda.synchronize(dev)
    me.fractal_pool_survivors()
    ms = _timed(step, iters, dev)
    surv = me.fractal_pool_survivors() / (iters + 1)
    got = d_out.cpu().numpy().view(FRACTAL_RES)
    me.close()
    # parity + CPU baseline: the restatement's brute force on a seeded sample,
    # over the host threads this process may use
    threads = ol.host_threads()
    sel = np.sort(np.random.default_rng(7).choice(n, sample, replace=False))
    rq = np.stack([req["block_x"][sel], req["block_y"][sel], req["bsx"][sel], req["bsy"][sel]], 1).astype(np.int32)
    t0 = time.time()
    exp, xy = ol.fractal_search_batch_par(org, ref, R, rq, threads)
    cpu_s = time.time() - t0
    g = got[sel]
    exact = int(np.sum((g["rms"] == exp[:, 0]) & (g["scale"] == exp[:, 1]) & (g["offset"] == exp[:, 2]) &
                       (g["x"] == xy[:, 0]) & (g["y"] == xy[:, 1])))
    pairs = n * (W - 3) * (H - 3)
    flops = pairs * FLOPS_PER_PAIR_44
    return {"workload": "configs[2]: 1080p (1920x1080) fractal full_search, every 4x4 range block (129,600) vs the "
                        "full domain pool (2,064,609 positions each), thesis compute_rms / QUAN_A, pruned exact "
                        "search (MFMA bound test)",
            "range_blocks": n, "ms_per_frame": round(ms, 3), "range_blocks_per_s": round(n / (ms * 1e-3), 1),
            "pairs_per_s": round(pairs / (ms * 1e-3), 1),
            "exact_evals_per_block": round(surv / n, 3),
            "roofline": {"bound": "mfma", "achieved": round(flops / (ms * 1e-3) / 1e12, 1),
                         "peak": MFMA_BF16_PEAK / 1e12, "unit": "TFLOP/s",
                         "frac": round(flops / (ms * 1e-3) / MFMA_BF16_PEAK, 4),
                         "note": "algorithmic bound-test flops (64 per pair, bf16 hi/lo split) over the whole "
                                 "frame time (words image, seeds and exact survivors included)"},
            "parity": {"reference": "oracle/fractal_oracle.c (parity with the thesis unpinned)",
                       "sample": int(sample), "bit_exact": exact},
            "cpu_baseline": {"value": round(sample / cpu_s, 2), "unit": "range blocks/sec", "cores": threads,
                             "kind": "port",
                             "sample": f"{sample} seeded blocks of the same frame, thesis full_search restated "
                                       f"(oracle/fractal_oracle.c), brute force over the full pool, {threads} "
                                       f"threads: {cpu_s:.2f} s"}}


def hybrid_block(dev, local: int, load_workload, iters: int = 10) -> dict:
    """configs[4] per GPU: one 1080p frame of the joint codec (jmme/hybrid.py)."""
    import oracle_lib as ol
    from fractal_scenes import gate_scene
    from jmme.hybrid import HybridFrameCoder
    W, H = 1920, 1088
    scene = [gate_scene(W, H, 11, 4, scale=6), gate_scene(W // 2, H // 2, 12, 4, scale=6),
             gate_scene(W // 2, H // 2, 13, 4, scale=6)]
    cur, ref, req, unit_of, slots, expect, meta = load_workload()
    st = torch.cuda.current_stream(dev).cuda_stream
    with HybridFrameCoder(W, H, n_views=4, fractal_range=7, tol_16=8.0, tol_8=5.0, device=local) as hc:
        hc.load_fractal(scene)
        hc.load_me(cur, ref, req)
        ms_enc = _timed(lambda: hc.fractal_encode(st), iters, dev)
        ms_dec = _timed(lambda: hc.fractal_decode(st), iters, dev)
        ms_me = _timed(lambda: hc.motion_search(st), iters, dev)
        ms = _timed(lambda: hc.step(st), iters, dev)
        res = hc.me_results()[unit_of, slots]
        me_exact = int(np.sum((res["mv_x"] == expect[0]) & (res["mv_y"] == expect[1]) & (res["cost"] == expect[2])))
        pu = hc.planes[1]
        got = np.array(pu.trees_host(), copy=True)
        rec = pu.rec.cpu().numpy()
        split = [int((p.trees_host()["mb"]["partition"] == 3).sum()) for p in hc.planes]
    org_u, views_u = scene[1]
    t0 = time.time()
    exp = np.array(ol.fractal_encode_mbs(org_u, views_u, 7, 8.0, 5.0), copy=True)
    cpu_s = time.time() - t0
    for t in (got, exp):
        t["chun"][np.isnan(t["chun"])] = 0
    tree_exact = int((got.view(np.uint8).reshape(len(got), -1) == exp.view(np.uint8).reshape(len(exp), -1))
                     .all(1).sum())
    rc, rec_exp = ol.fractal_decode_mbs(exp, views_u, 2)
    n_mb = sum(p.n_mb for p in hc.planes)
    return {"workload": "configs[4] per GPU: one 1080p frame of the joint fractal + H.264 codec -- Y 1920x1088 and "
                        "U, V 960x544 quadtrees (4 views, R 7, tol 8/5), their reconstruction, JM FS +-32 ME of "
                        "8160 MB x ref",
            "frames_per_s": round(1e3 / ms, 1), "ms_per_frame": round(ms, 4),
            "stages_ms": {"fractal_encode_YUV": round(ms_enc, 4), "fractal_decode_YUV": round(ms_dec, 4),
                          "h264_fs32_me": round(ms_me, 4)},
            "fractal_macroblocks": n_mb, "split_macroblocks_YUV": split,
            "parity": {"h264_me_vs_jm": {"searches": int(len(expect[0])), "bit_exact": me_exact},
                       "u_trees_vs_restatement": {"macroblocks": len(exp), "bit_exact": tree_exact},
                       "u_reconstruction_vs_restatement": bool(rc == 0 and np.array_equal(rec, rec_exp))},
            "cpu_baseline": {"value": round(len(exp) / cpu_s, 1), "unit": "fractal macroblocks/sec", "cores": 1,
                             "kind": "port", "sample": f"the U plane's quadtree ({len(exp)} MBs, 4 views), "
                                                       f"oracle/fractal_oracle.c: {cpu_s:.2f} s"},
            "scaling": "GOP replicas: a frame's P-frame refers to the previous reconstruction"}


# ---- the drop-in encoder (JM 18.5 lencod with libjmme behind IntPelME) -----------
def _progress(msg):
    """a line on stderr per encode: long blocks keep showing signs of life"""
    import sys
    print(msg, file=sys.stderr, flush=True)


def _lencod_args(binary, d, tag, yuv, w, h, frames, params, cfg_text):
    import os
    cfg = os.path.join(d, "enc.cfg")
    open(cfg, "w").write(cfg_text)
    out, rec = os.path.join(d, f"{tag}.264"), os.path.join(d, f"{tag}_rec.yuv")
    args = [binary, "-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
            "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}", "-p", f"FramesToBeEncoded={frames}",
            "-p", f"OutputFile={out}", "-p", f"ReconFile={rec}"]
    for k, v in params.items():
        args += ["-p", f"{k}={v}"]
    return args, out, rec


def _lencod_host(binary, d, yuv, w, h, frames, params, cfg_text, procs):
    """`procs` stock encoders at once, each in its own directory on the same clip
    (JM is single-threaded: N concurrent encodes are how the host spends N cores,
    SURVEY §8(d)).  Returns every process's own 'Total ME time' (s)."""
    import os
    import re
    import subprocess
    runs = []
    for i in range(procs):
        wd = os.path.join(d, f"host{i}")
        os.makedirs(wd, exist_ok=True)
        args, _, _ = _lencod_args(binary, wd, "h", yuv, w, h, frames, params, cfg_text)
        runs.append(subprocess.Popen(args, cwd=wd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True))
    me = []
    for r in runs:
        out, _ = r.communicate(timeout=900)
        m = re.search(r"Total ME time for sequence\s*:\s*([0-9.]+) sec", out)
        if r.returncode != 0 or not m:
            raise RuntimeError("host encoder failed: " + out[-800:])
        me.append(float(m.group(1)))
    return me


def _lencod(binary, d, tag, yuv, w, h, frames, params, cfg_text, env=None):
    import hashlib
    import os
    import re
    import subprocess
    args, out, rec = _lencod_args(binary, d, tag, yuv, w, h, frames, params, cfg_text)
    t0 = time.time()
    r = subprocess.run(args, cwd=d, capture_output=True, text=True, timeout=900, env=dict(os.environ, **(env or {})))
    wall = time.time() - t0
    if r.returncode != 0:
        raise RuntimeError(r.stdout[-1500:] + r.stderr[-1500:])
    me = re.search(r"Total ME time for sequence\s*:\s*([0-9.]+) sec", r.stdout)
    calls = re.search(r"jm_gpu_me: (\d+) integer-pel searches on the GPU \(libjmme\): (\d+) from (\d+) speculative",
                      r.stderr)
    stats = re.search(r"integer batches: (\d+) past the batch, (\d+) failed guesses; (\d+) units; ([0-9.]+) ms building, "
                      r"([0-9.]+) ms in jmme_search_mbs", r.stderr)
    sp = re.search(r"(\d+) sub-pel refinements: (\d+) cached, (\d+) batches, (\d+) on the CPU(?:; ([\d.]+) ms)?", r.stderr)
    ep = re.search(r"(\d+) EPZS searches on the GPU \(libjmme\); (\d+) on the CPU; (\d+) predictors, "
                   r"(\d+) pre-stamped map cells, (\d+) switches to window scans; ([\d.]+) ms in the EPZS wrapper, "
                   r"([\d.]+) ms in the engine", r.stderr)
    esp = re.search(r"(\d+) EPZS sub-pel refinements on the GPU \((\d+) chained[^)]*\), (\d+) on the CPU", r.stderr)
    ch = re.search(r"chained guesses: (\d+) chains, (\d+) steps, (\d+) calls answered, (\d+) head mismatches; "
                   r"(\d+) chain-only calls \((\d+) fell back[^;]*(?:; ([\d.]+) ms in chain-only calls)?", r.stderr)
    chsp = re.search(r"chained sub-pel: (\d+) refinements, (\d+) calls answered; (\d+) misses without", r.stderr)
    res = dict(wall_s=round(wall, 3), me_s=float(me.group(1)) if me else None, stderr=r.stderr[-4000:],
               md5=(hashlib.md5(open(out, "rb").read()).hexdigest(), hashlib.md5(open(rec, "rb").read()).hexdigest()))
    if calls:
        res.update(gpu_searches=int(calls.group(1)), batches=int(calls.group(3)),
                   searches_from_cache=int(calls.group(2)) - int(calls.group(3)))
    if stats:
        res.update(batches_past_end=int(stats.group(1)), batches_failed_guess=int(stats.group(2)),
                   batch_units=int(stats.group(3)), host_build_ms=float(stats.group(4)),
                   engine_call_ms=float(stats.group(5)))
    if ch:
        res["chains"] = dict(zip(("chains", "steps", "calls_answered", "head_mismatches", "chain_only_calls",
                                  "chain_only_fallbacks"), map(int, ch.groups()[:6])))
        if ch.group(7):
            res["chains"]["chain_only_ms"] = float(ch.group(7))
        if chsp:
            res["chains"]["subpel"] = dict(zip(("refinements", "calls_answered", "no_lambdas"), map(int, chsp.groups())))
    if sp:
        res["subpel"] = dict(zip(("calls", "cached", "batches", "cpu"), map(int, sp.groups()[:4])))
        if sp.group(5):
            res["subpel"]["batch_ms"] = float(sp.group(5))
    if ep:
        g = ep.groups()
        res["epzs"] = dict(gpu_searches=int(g[0]), cpu_searches=int(g[1]), predictors=int(g[2]),
                           pre_stamped_cells=int(g[3]), window_scan_switches=int(g[4]), wrapper_ms=float(g[5]),
                           engine_call_ms=float(g[6]),
                           us_per_search=round(float(g[5]) * 1e3 / max(1, int(g[0])), 2) if float(g[5]) > 0 else None)
        if float(g[5]) == 0:   # (the adapter's per-call clock runs only under JMME_PHASES / JMME_EPZS_TRACE)
            del res["epzs"]["wrapper_ms"], res["epzs"]["us_per_search"]
    if esp:
        res["epzs_subpel"] = dict(gpu=int(esp.group(1)), chained=int(esp.group(2)), cpu=int(esp.group(3)))
    spec = re.search(r"EPZS speculation: (\d+) searches answered from (\d+) batches \((\d+) guesses\), (\d+) searched "
                     r"alone; (\d+) not speculated; guesses refused: (\d+) inputs, (\d+) bounds, (\d+) map cells; "
                     r"([\d.]+) ms building batches", r.stderr)
    if spec:
        res["epzs_speculation"] = dict(zip(("answered_from_batches", "batches", "guesses", "searched_alone",
                                            "not_speculated", "refused_inputs", "refused_bounds", "refused_cells"),
                                           map(int, spec.groups()[:8])), build_ms=float(spec.group(9)))
    # JMME_PHASES=1: the library's own clocks (server phases, calls by kind), as printed
    lib_lines = [ln for ln in r.stderr.splitlines() if ln.startswith(("jmme EPZS", "jm_gpu_me: EPZS misses", "jm_gpu_me: EPZS host"))]
    if lib_lines:
        res["lib_clocks"] = lib_lines
    return res


# the drop-in rows of bench.py: (tag, JM parameters, frames).  FS / FFS with
# sub-pel off and RDO off are configs[1]'s settings; the "_subpel" rows are
# JM/bin/encoder_baseline.cfg's ME keys (sub-pel on, SATD half/quarter-pel and
# mode decision, RDO on, adaptive rounding) with FS / FFS and one reference; EPZS
# is configs[3]'s algorithm with the same file's EPZS section.
BASELINE_SUBPEL = {"DisableSubpelME": 0, "MEDistortionFPel": 0, "MEDistortionHPel": 2, "MEDistortionQPel": 2,
                   "MDDistortion": 2, "RestrictSearchRange": 2, "RDOptimization": 1, "AdaptiveRounding": 1}


def dropin_modes():
    from test_jm_dropin_epzs_gpu import BASELINE_EPZS
    return (("FS", {"SearchMode": -1, "RDOptimization": 0}, 3),
            ("FFS", {"SearchMode": 0, "RDOptimization": 0}, 3),
            ("FS_subpel", dict(BASELINE_SUBPEL, SearchMode=-1), 2),
            ("FFS_subpel", dict(BASELINE_SUBPEL, SearchMode=0), 2),
            ("EPZS", dict(BASELINE_EPZS), 2))


def dropin_block(modes=None, size=(1920, 1080), search_range=32, reps=3, host_procs=None) -> dict | None:
    """JM 18.5 lencod, stock (CPU) and lencod_jmme (the same JM objects, the ME
    through libjmme) on the same seeded clip: JM's own 'Total ME time' per
    P-frame, and byte identity of bitstream and reconstruction.  The GPU engine is
    created and warmed in init_motion_search_module (encoder start-up, before any
    frame is timed).  The drop-in runs `reps` times (median ME time reported, the
    spread beside it); the stock encoder runs once alone (one core) and as
    `host_procs` concurrent encoders (the host's cores, default the headline
    baseline's host_cores()), so every row states its speed against one core and
    against the whole host."""
    import os
    import tempfile
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stock = os.path.join(repo, "oracle", "_ref", "lencod")
    gpu = os.path.join(repo, "integration", "_build", "lencod_jmme")
    floor = os.path.join(repo, "integration", "_build", "lencod_noop_me")
    if not (os.path.exists(stock) and os.path.exists(gpu)):
        return None
    if host_procs is None:
        from bench import host_cores, cpu_model
        host_procs, cpu = host_cores(), cpu_model()
    else:
        cpu = None
    from jmme import synth
    from test_jm_dropin_gpu import CFG
    w, h = size
    mbs = (w // 16) * ((h + 15) // 16)
    out = {"workload": f"JM 18.5 lencod encoding a seeded {w}x{h} clip (1 I + P frames), +-{search_range}, 1 ref: "
                       f"stock (CPU) vs the drop-in (ME on the GPU)",
           "p_frame_macroblocks": mbs, "host_procs": host_procs, "host_cpu": cpu}
    with tempfile.TemporaryDirectory() as d:
        for tag, mparams, frames in (modes or dropin_modes()):
            yuv = os.path.join(d, f"in{frames}.yuv")
            if not os.path.exists(yuv):
                synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=2024, gmv=(5, 3)))
            params = dict(mparams, SearchRange=search_range, NumberReferenceFrames=1)
            mode = params["SearchMode"]
            p = frames - 1
            cpu = _lencod(stock, d, f"cpu_{tag}", yuv, w, h, frames, params, CFG)
            _progress(f"dropin {tag}: stock {cpu['me_s']:.3f} s of ME")
            host = _lencod_host(stock, d, yuv, w, h, frames, params, CFG, host_procs) if host_procs > 1 else None
            if host:
                _progress(f"dropin {tag}: {host_procs} concurrent stock encoders, slowest {max(host):.3f} s of ME")
            gs = []
            for r in range(reps):
                gs.append(_lencod(gpu, d, f"gpu_{tag}_{r}", yuv, w, h, frames, params, CFG))
                _progress(f"dropin {tag}: drop-in run {r}: {gs[-1]['me_s']:.3f} s of ME")
            gs.sort(key=lambda x: x["me_s"])
            g = gs[len(gs) // 2]
            # JM's own loop around the search (integration/jm_noop_me.c: a zero-cost IntPelME)
            fl = _lencod(floor, d, f"floor_{tag}", yuv, w, h, frames, params, CFG) \
                if mode in (-1, 0) and os.path.exists(floor) else None
            row = {
                "stock_me_ms_per_p_frame": round(cpu["me_s"] * 1e3 / p, 2),
                "dropin_me_ms_per_p_frame": round(g["me_s"] * 1e3 / p, 2),
                "me_speedup": round(cpu["me_s"] / g["me_s"], 2) if g["me_s"] else None,
                "dropin_mb_per_s": round(mbs * p / g["me_s"], 1) if g["me_s"] else None,
                "byte_identical": all(cpu["md5"] == x["md5"] for x in gs), "params": params, "p_frames": p,
                "dropin_me_ms_per_p_frame_runs": [round(x["me_s"] * 1e3 / p, 2) for x in gs],
                "jm_loop_floor_ms_per_p_frame": round(fl["me_s"] * 1e3 / p, 2) if fl and fl["me_s"] else None,
                "stock_wall_s": cpu["wall_s"], "dropin_wall_s": g["wall_s"],
                "dropin": {k: v for k, v in g.items() if k not in ("md5", "me_s", "wall_s", "stderr")}}
            if host:
                # the host's rate: every encoder's P-frame macroblocks over the slowest one's ME time
                host_rate = host_procs * mbs * p / max(host)
                row.update(host_mb_per_s=round(host_rate, 1),
                           host_me_ms_per_p_frame_slowest=round(max(host) * 1e3 / p, 2),
                           me_speedup_vs_host=round(row["dropin_mb_per_s"] / host_rate, 3) if g["me_s"] else None)
            out[tag] = row
    return out


# ---- mode decision's inter residual coding on the GPU --------------
F3_PARAMS = {"SearchMode": -1, "SearchRange": 16, "NumberReferenceFrames": 1, "RDOptimization": 1,
             "DisableSubpelME": 0, "MEDistortionHPel": 2, "MEDistortionQPel": 2, "MDDistortion": 2,
             "AdaptiveRounding": 0}
_F3_RE = r"jm_f3_gpu: (\d+) 4x4 residual calls: (\d+) served from (\d+) GPU batches; on JM's code: (\d+) intra, " \
         r"(\d+) other forms, (\d+) input mismatches"


def f3_block(size=(352, 288), frames=3) -> dict | None:
    """lencod_jmme with and without JMME_F3=1 (integration/jm_f3_gpu.c: every inter
    residual_transform_quant_luma_4x4 call of mode decision answered from one GPU
    launch per macroblock and mode) against the stock encoder on the same clip:
    byte identity, the served share and the encode-time delta.  The plain
    quantiser (adaptive rounding off) is the one served."""
    import os
    import re
    import tempfile
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stock = os.path.join(repo, "oracle", "_ref", "lencod")
    gpu = os.path.join(repo, "integration", "_build", "lencod_jmme")
    if not (os.path.exists(stock) and os.path.exists(gpu)):
        return None
    from jmme import synth
    from test_jm_dropin_gpu import CFG
    w, h = size
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=77, gmv=(2, -1)))
        ref = _lencod(stock, d, "cpu", yuv, w, h, frames, F3_PARAMS, CFG)
        off = _lencod(gpu, d, "off", yuv, w, h, frames, F3_PARAMS, CFG)
        on = _lencod(gpu, d, "on", yuv, w, h, frames, F3_PARAMS, CFG, env={"JMME_F3": "1"})
        _progress(f"f3 block: encode {off['wall_s']:.2f} s without, {on['wall_s']:.2f} s with the GPU residuals")
    out = {"workload": f"JM 18.5 lencod_jmme, seeded {w}x{h} clip, 1 I + {frames - 1} P, FS +-16 + sub-pel, RDO on, "
                       f"adaptive rounding off: inter 4x4 residual coding of mode decision from the GPU (JMME_F3=1)",
           "params": F3_PARAMS, "byte_identical": ref["md5"] == off["md5"] == on["md5"],
           "encode_wall_s": {"stock": ref["wall_s"], "dropin": off["wall_s"], "dropin_f3": on["wall_s"]},
           "f3_delta_s": round(on["wall_s"] - off["wall_s"], 3)}
    m = re.search(_F3_RE, on.get("stderr", ""))
    if m:
        calls, served, batches, intra, other, mism = map(int, m.groups())
        out.update(calls=calls, served=served, batches=batches, intra_on_cpu=intra, other_on_cpu=other,
                   input_mismatches=mism, us_per_batch_delta=round((on["wall_s"] - off["wall_s"]) * 1e6 /
                                                                   max(1, batches), 1))
    return out


# ---- the encoder itself sharded by closed GOPs ----------
# JM's ME is sequential inside a GOP (frame t searches the reconstruction of t-1,
# store_picture_in_dpb, JM/lencod/src/mbuffer.c:1905), so the product scales by
# closed GOPs: integration/jmme_gop.c starts one encoder per GOP (StartFrame /
# FramesToBeEncoded, JM/lencod/inc/configfile.h:39,47), its GPU fixed in the
# child's environment before the encoder starts and, when given a core list, its
# host cores too.  Two presets:
#   fs     -- configs[1]'s settings (FS +-32, 1 ref, RDO off, sub-pel off), 1080p;
#   epzs4k -- configs[3] as configured: 3840x2160, JM/bin/encoder_baseline.cfg's
#             EPZS keys (quarter-pel grid, SATD sub-pel, RDO on, adaptive
#             rounding; the file's EPZS section, tests/test_jm_dropin_epzs_gpu.py
#             BASELINE_EPZS) at level 5.1.
ENCODER_PARAMS = {"SearchMode": -1, "SearchRange": 32, "NumberReferenceFrames": 1, "RDOptimization": 0}


def encoder_preset(name: str):
    """(JM parameters, (w, h), text for the report) of a GOP-encoder preset"""
    if name == "fs":
        return ENCODER_PARAMS, (1920, 1080), "FS +-32, 1 ref, RDO off, sub-pel off (configs[1]'s settings)"
    if name == "epzs4k":
        from test_jm_dropin_epzs_gpu import BASELINE_EPZS
        return (dict(BASELINE_EPZS, NumberReferenceFrames=1, LevelIDC=51), (3840, 2160),
                "EPZS +-32 (encoder_baseline.cfg's EPZS keys: quarter-pel grid, SATD sub-pel, RDO on, adaptive "
                "rounding), 1 ref, level 5.1 (configs[3])")
    raise ValueError(f"unknown encoder preset {name!r}")


def _cpulist(text: str) -> list[int]:
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def _kfd_gpu_cpus(index: int) -> list[int] | None:
    """The host cores local to HIP device `index` (its PCI device's NUMA node),
    read from sysfs -- the KFD topology's GPU nodes in order, their PCI address,
    then the device's local_cpulist -- without initialising the GPU.  None when
    the topology is not readable (CPU containers)."""
    import os
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = sorted((int(n) for n in os.listdir(root)), key=int)
        gpus = []
        for n in nodes:
            props = dict(ln.split() for ln in open(f"{root}/{n}/properties") if len(ln.split()) == 2)
            if int(props.get("simd_count", 0)) > 0:
                gpus.append(props)
        vis = os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
        if vis:
            gpus = [gpus[int(v)] for v in vis.split(",") if v.strip()]
        props = gpus[index]
        loc, dom = int(props["location_id"]), int(props.get("domain", 0))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
        return _cpulist(open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read())
    except (OSError, ValueError, KeyError, IndexError):
        return None


def gpu_local_cpus(local: int, local_ws: int) -> tuple[list[int], str]:
    """The host cores rank `local` of `local_ws` runs its encoders on: its GPU's
    NUMA-local cores that this process may use, split evenly among the local
    ranks whose GPUs share that NUMA node; without a readable topology, an even
    split of this process's affinity by local rank.  Returns (cores, source)."""
    import os
    allowed = sorted(os.sched_getaffinity(0))
    mine = _kfd_gpu_cpus(local)
    if mine:
        node = [c for c in allowed if c in set(mine)]
        peers = [r for r in range(local_ws) if _kfd_gpu_cpus(r) == mine]
        if node and local in peers:
            k, i = len(peers), peers.index(local)
            share = node[i * len(node) // k:(i + 1) * len(node) // k] or node
            return share, "numa"
    k = max(1, local_ws)
    share = allowed[local * len(allowed) // k:(local + 1) * len(allowed) // k] or allowed
    return share, "affinity"


def _cpulist_text(cores) -> str:
    cores = sorted(cores)
    runs, i = [], 0
    while i < len(cores):
        j = i
        while j + 1 < len(cores) and cores[j + 1] == cores[j] + 1:
            j += 1
        runs.append(str(cores[i]) if i == j else f"{cores[i]}-{cores[j]}")
        i = j + 1
    return ",".join(runs)


def _gop_launch(launcher, encoder, d, tag, yuv, w, h, frames, gop, slots, per_slot, devices, cfg_text, params,
                timeout=1200, cpus=None):
    """One jmme_gop run over the clip: returns (report, per-GOP md5 pairs)."""
    import hashlib
    import json
    import os
    import subprocess
    wd = os.path.join(d, tag)
    os.makedirs(wd, exist_ok=True)
    cfg = os.path.join(wd, "enc.cfg")
    open(cfg, "w").write(cfg_text)
    enc_args = ["-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={w}", "-p", f"SourceHeight={h}",
                "-p", f"OutputWidth={w}", "-p", f"OutputHeight={h}"]
    for k, v in params.items():
        enc_args += ["-p", f"{k}={v}"]
    prefix = os.path.join(wd, "g")
    cmd = [launcher, "--encoder", encoder, "--gpus", str(slots), "--per-gpu", str(per_slot), "--gop", str(gop),
           "--frames", str(frames), "--prefix", prefix]
    if devices is not None:
        cmd += ["--devices", ",".join(str(x) for x in devices)]
    if cpus:
        cmd += ["--cpus", _cpulist_text(cpus)]
    t0 = time.time()
    r = subprocess.run(cmd + ["--"] + enc_args, cwd=wd, capture_output=True, text=True, timeout=timeout)
    wall = time.time() - t0
    if r.returncode != 0:
        raise RuntimeError(f"jmme_gop ({tag}) failed: " + r.stdout[-800:] + r.stderr[-800:])
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    rep["python_wall_s"] = round(wall, 3)
    md5 = []
    for g in range(rep["gops"]):
        md5.append(tuple(hashlib.md5(open(f"{prefix}_gop{g:03d}{sfx}", "rb").read()).hexdigest()
                         for sfx in (".264", "_rec.yuv")))
    return rep, md5


def encoder_gop_block(device: int = 0, rank: int = 0, gops: int = 16, gop: int = 4, size=None,
                      per_gpu: int = 8, host_procs=None, check_stock: bool = True, encoder=None,
                      between=None, preset: str = "fs", cpus=None) -> dict | None:
    """One rank's share of the GOP-sharded encoder: `gops` closed GOPs of `gop`
    frames of a seeded clip (its own seed per rank; the preset's size unless
    `size` is given) through lencod_jmme on HIP device `device` (`per_gpu`
    encoders at once; pinned one to a core of `cpus` when given), timed wall to
    wall, then -- outside the timed region -- the same GOPs through the stock
    lencod as concurrent CPU processes (the host baseline: `host_procs` at once,
    on the same cores when `cpus` is given), and every GOP's bitstream and
    reconstruction compared byte for byte.  The caller (this process) never
    touches the GPU."""
    import os
    import tempfile
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stock = os.path.join(repo, "oracle", "_ref", "lencod")
    gpu = os.path.abspath(encoder) if encoder else os.path.join(repo, "integration", "_build", "lencod_jmme")
    # (a CPU rehearsal passes the stock encoder here)
    launcher = os.path.join(repo, "integration", "_build", "jmme_gop")
    if not all(os.path.exists(p) for p in (stock, gpu, launcher)):
        return None
    if host_procs is None:
        from bench import host_cores
        host_procs = host_cores() if not cpus else len(cpus)
    from jmme import synth
    from test_jm_dropin_gpu import CFG
    params, psize, ptext = encoder_preset(preset)
    w, h = size or psize
    frames = gops * gop
    mbs = (w // 16) * ((h + 15) // 16)
    seed = 3000 + rank
    with tempfile.TemporaryDirectory() as d:
        yuv = os.path.join(d, "in.yuv")
        synth.write_yuv420(yuv, synth.luma_sequence(w, h, frames, seed=seed, gmv=(5, 3)))
        _progress(f"encoder gop block ({preset}) rank {rank}: {gops} GOPs x {gop} frames on device {device}")
        g_rep, g_md5 = _gop_launch(launcher, gpu, d, "gpu", yuv, w, h, frames, gop, 1, per_gpu, [device], CFG,
                                   params, cpus=cpus)
        out = {"encoder": os.path.basename(gpu), "preset": preset,
               "workload": f"JM 18.5 lencod_jmme (ME on the GPU) encoding {gops} closed GOPs of {gop} frames "
                           f"(1 I + {gop - 1} P) of a seeded {w}x{h} clip, {ptext}; one encoder process per GOP "
                           f"(integration/jmme_gop.c), {per_gpu} at once on the GPU",
               "device": device, "clip_seed": seed, "gops": gops, "gop": gop, "frames": frames,
               "macroblocks": frames * mbs, "wall_s": g_rep["python_wall_s"],
               "encoder_mb_per_s": round(frames * mbs / g_rep["python_wall_s"], 1),
               "me_s_per_gop": [r["me_s"] for r in g_rep["runs"]],
               "me_mb_per_s": round(gops * (gop - 1) * mbs / max(1e-9, sum(r["me_s"] for r in g_rep["runs"])), 1),
               "hw_queues_per_encoder": g_rep.get("hw_queues"),
               "host_placement": {"cpus": _cpulist_text(cpus) if cpus else "unpinned (scheduler)",
                                  "per_gop": [r.get("cpus") for r in g_rep["runs"]]}}
        if between is not None:   # (ranks meet here: no rank's stock encodes overlap another's timed run)
            between()
        if check_stock:
            _progress(f"encoder gop block ({preset}) rank {rank}: the same GOPs through the stock encoder, "
                      f"{min(host_procs, gops)} at once")
            s_rep, s_md5 = _gop_launch(launcher, stock, d, "stock", yuv, w, h, frames, gop, min(host_procs, gops), 1,
                                       None, CFG, params, cpus=cpus)
            same = [a == b for a, b in zip(g_md5, s_md5)]
            out["parity"] = {"reference": "JM 18.5 lencod (stock, same GOP arguments)", "gops": gops,
                             "byte_identical_gops": int(sum(same))}
            out["host_baseline"] = {"procs": min(host_procs, gops), "wall_s": s_rep["python_wall_s"],
                                    "encoder_mb_per_s": round(frames * mbs / s_rep["python_wall_s"], 1),
                                    "me_mb_per_s": round(gops * (gop - 1) * mbs /
                                                         max(1e-9, sum(r["me_s"] for r in s_rep["runs"])), 1),
                                    "me_s_per_gop": [r["me_s"] for r in s_rep["runs"]],
                                    "kind": "reference"}
            out["encoder_speedup_vs_host"] = round(s_rep["python_wall_s"] / g_rep["python_wall_s"], 2)
            out["me_speedup_vs_host"] = round(sum(r["me_s"] for r in s_rep["runs"]) /
                                              max(1e-9, sum(r["me_s"] for r in g_rep["runs"])), 2)
    return out
