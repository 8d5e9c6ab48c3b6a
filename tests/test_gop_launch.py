"""Closed-GOP sharding of the encoder (integration/jmme_gop.c, SURVEY §8(e)
row 1): a sequence cut into GOPs, one fresh encoder process per GOP, its GPU
fixed in the child's environment before it starts.  The concatenated GOP
reconstructions must equal one encoder run over the whole sequence with
IntraPeriod = IDRPeriod = the GOP length (JM/lencod/inc/configfile.h:39-47).

CPU rehearsal: the stock JM 18.5 lencod (oracle/_ref/lencod) under the
launcher with 2 "GPUs" (concurrent processes).  GPU: lencod_jmme under the
launcher (2 encoders sharing the box's GPU) against the stock single run."""
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STOCK = os.path.join(REPO, "oracle", "_ref", "lencod")
GPU_ENC = os.path.join(REPO, "integration", "_build", "lencod_jmme")
LAUNCHER = os.path.join(REPO, "integration", "_build", "jmme_gop")
W, H, FRAMES, GOP = 352, 288, 7, 3


def _clip(d):
    from jmme import synth
    from test_jm_dropin_gpu import CFG
    yuv = os.path.join(d, "in.yuv")
    synth.write_yuv420(yuv, synth.luma_sequence(W, H, FRAMES, seed=21, gmv=(3, -1)))
    cfg = os.path.join(d, "enc.cfg")
    open(cfg, "w").write(CFG)
    return ["-d", cfg, "-p", f"InputFile={yuv}", "-p", f"SourceWidth={W}", "-p", f"SourceHeight={H}",
            "-p", f"OutputWidth={W}", "-p", f"OutputHeight={H}", "-p", "SearchMode=-1", "-p", "SearchRange=16",
            "-p", "NumberReferenceFrames=2", "-p", "RDOptimization=0"]


def _cpulist(text):
    out = []
    for part in text.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def _md5(p):
    return hashlib.md5(open(p, "rb").read()).hexdigest()


def _single(d, args):
    rec = os.path.join(d, "single_rec.yuv")
    r = subprocess.run([STOCK] + args + ["-p", f"FramesToBeEncoded={FRAMES}", "-p", f"IntraPeriod={GOP}",
                                         "-p", f"IDRPeriod={GOP}", "-p", f"OutputFile={os.path.join(d, 'single.264')}",
                                         "-p", f"ReconFile={rec}"], cwd=d, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-1000:]
    return rec


def _sharded(d, encoder, gpus, per_gpu):
    prefix = os.path.join(d, "shard")
    r = subprocess.run([LAUNCHER, "--encoder", encoder, "--gpus", str(gpus), "--per-gpu", str(per_gpu), "--gop",
                        str(GOP), "--frames", str(FRAMES), "--prefix", prefix, "--concat", "--"] + _clip(d),
                       cwd=d, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-1500:])
    return json.loads(r.stdout.strip().splitlines()[-1]), prefix + "_rec.yuv"


@pytest.mark.skipif(not (os.path.exists(STOCK) and os.path.exists(LAUNCHER)), reason="JM build / launcher absent")
def test_gop_launcher_cpu_rehearsal():
    with tempfile.TemporaryDirectory() as d:
        rep, rec = _sharded(d, STOCK, gpus=2, per_gpu=1)
        want = _single(d, _clip(d))
        assert rep["gops"] == 3 and rep["failed"] == 0
        assert [r["frames"] for r in rep["runs"]] == [3, 3, 1]
        assert sorted({r["gpu"] for r in rep["runs"]}) == [0, 1]
        assert all(r["me_s"] >= 0 for r in rep["runs"])
        assert _md5(rec) == _md5(want)


@pytest.mark.gpu
def test_gop_launcher_gpu_dropin_matches_single_cpu_run(gpu):
    """lencod_jmme per GOP (two encoders sharing the one GPU) == stock single run."""
    with tempfile.TemporaryDirectory() as d:
        rep, rec = _sharded(d, GPU_ENC, gpus=1, per_gpu=2)
        want = _single(d, _clip(d))
        assert rep["failed"] == 0
        assert _md5(rec) == _md5(want)
        for r in rep["runs"]:
            log = open(os.path.join(d, f"shard_gop{r['gop']:03d}.log")).read()
            assert "Total ME time" in log


@pytest.mark.skipif(not (os.path.exists(STOCK) and os.path.exists(LAUNCHER)), reason="JM build / launcher absent")
def test_bench_shard_encoder_two_ranks_cpu_rehearsal():
    """bench.py --shard encoder under torch.distributed.run at world size 2 (gloo,
    no GPU: the stock encoder stands in for lencod_jmme): each rank encodes its
    own closed GOPs through the launcher, the job time is the slowest rank's, and
    every GOP is checked against the stock encoder byte for byte."""
    import socket
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                        "--gpus", "2", "--shard", "encoder", "--enc-encoder", STOCK, "--enc-size", "176x144",
                        "--enc-gops", "2", "--enc-gop", "2", "--enc-per-gpu", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-2500:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["parity"] == {"reference": "JM 18.5 lencod (stock, same GOP arguments)", "gops": 4,
                              "byte_identical_gops": 4}
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    # host placement: each rank's encoders on its own cores (its GPU's NUMA-local
    # share, or its share of the affinity here), disjoint between the ranks
    sets = [set(_cpulist(p["cpus"])) for p in line["per_rank"]]
    assert all(sets) and not (sets[0] & sets[1]), line["per_rank"]
    assert sets[0] | sets[1] <= set(os.sched_getaffinity(0))
    placed = line["rank0"]["host_placement"]
    assert placed["source"] in ("numa", "affinity")
    assert all(set(_cpulist(c)) <= sets[0] for c in placed["per_gop"]), placed
    mbs = sum(p["macroblocks"] for p in line["per_rank"])
    assert mbs == 2 * 2 * 2 * (176 // 16) * (144 // 16)
    assert abs(line["value"] - mbs / max(p["wall_s"] for p in line["per_rank"])) < 0.01 * line["value"] + 1


@pytest.mark.skipif(not os.path.exists(LAUNCHER), reason="launcher absent")
def test_gop_launcher_device_map(tmp_path):
    """--devices maps the launcher's GPU slots to HIP device indices (a rank-per-GPU
    caller passes its own device alone); each encoder sees its device in
    HIP_VISIBLE_DEVICES, set before it starts.  A stand-in encoder script reports
    its environment and arguments into the GOP's log."""
    enc = tmp_path / "fake_enc.sh"
    enc.write_text("#!/bin/sh\necho \"dev=$HIP_VISIBLE_DEVICES hq=$GPU_MAX_HW_QUEUES args=$*\"\n"
                   "echo 'Total ME time for sequence        :   0.125 sec'\n")
    enc.chmod(0o755)
    prefix = str(tmp_path / "g")
    r = subprocess.run([LAUNCHER, "--encoder", str(enc), "--gpus", "2", "--devices", "5,7", "--gop", "2",
                        "--frames", "5", "--prefix", prefix, "--", "-d", "x.cfg"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    assert rep["gops"] == 3 and rep["failed"] == 0
    assert [g["frames"] for g in rep["runs"]] == [2, 2, 1]
    for g in rep["runs"]:
        log = open(f"{prefix}_gop{g['gop']:03d}.log").read()
        assert f"dev={g['device']}" in log and g["device"] == (5, 7)[g["gpu"]], (g, log)
        assert "hq=4" in log, log   # (one encoder per GPU: the runtime's default queue count, set explicitly)
        assert f"StartFrame={g['first']}" in log and f"FramesToBeEncoded={g['frames']}" in log
        assert g["me_s"] == 0.125
    bad = subprocess.run([LAUNCHER, "--encoder", str(enc), "--gpus", "2", "--devices", "5", "--gop", "2",
                          "--frames", "4", "--prefix", prefix, "--"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 2 and "fewer devices" in bad.stderr


@pytest.mark.skipif(not os.path.exists(LAUNCHER), reason="launcher absent")
def test_gop_launcher_pins_host_cores(tmp_path):
    """--cpus: the list is cut into one contiguous share per GPU slot and every
    running encoder holds a core of its slot's share to itself (set with
    sched_setaffinity between fork and exec); a freed core goes to the next GOP.
    The stand-in encoder reports the cores it was allowed to run on."""
    cores = sorted(os.sched_getaffinity(0))
    if len(cores) < 4:
        pytest.skip("needs 4 host cores")
    use = cores[:4]
    enc = tmp_path / "fake_enc.sh"
    enc.write_text("#!/bin/sh\ngrep Cpus_allowed_list /proc/self/status\nsleep 0.2\n")
    enc.chmod(0o755)
    prefix = str(tmp_path / "g")
    r = subprocess.run([LAUNCHER, "--encoder", str(enc), "--gpus", "2", "--per-gpu", "2", "--cpus",
                        ",".join(map(str, use)), "--gop", "1", "--frames", "6", "--prefix", prefix, "--"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    assert rep["pinned"] == 1 and rep["host_cores"] == 4 and rep["failed"] == 0
    share = {0: set(use[:2]), 1: set(use[2:])}
    for g in rep["runs"]:
        log = open(f"{prefix}_gop{g['gop']:03d}.log").read()
        allowed = log.split(":", 1)[1].strip()
        assert allowed == g["cpus"] and int(allowed) in share[g["gpu"]], (g, log)
    # two encoders of a slot run at once: never on the same core
    first = [g for g in rep["runs"] if g["gop"] < 4]
    assert len({g["cpus"] for g in first}) == 4, first
    unpinned = subprocess.run([LAUNCHER, "--encoder", str(enc), "--gpus", "1", "--gop", "1", "--frames", "1",
                               "--prefix", prefix, "--"], capture_output=True, text=True, timeout=60)
    assert json.loads(unpinned.stdout.strip().splitlines()[-1])["pinned"] == 0
    # 8 encoders on one GPU: 2 hardware queues each (16 in all), so the GPU's scheduler
    # keeps every encoder's queues mapped (tools/exp_gop_queues.py)
    eight = subprocess.run([LAUNCHER, "--encoder", str(enc), "--gpus", "1", "--per-gpu", "8", "--gop", "1",
                            "--frames", "1", "--prefix", prefix, "--"], capture_output=True, text=True, timeout=60)
    assert json.loads(eight.stdout.strip().splitlines()[-1])["hw_queues"] == 2
