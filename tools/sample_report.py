#!/usr/bin/env python3
"""Attribute a JMME_SAMPLE profile (integration/jm_sample.c) to functions.
Usage: python3 tools/sample_report.py <samples file> [top N]
Each sample is an instruction pointer taken every 20 us of wall time while
JM's encoding thread was inside its timed ME region; /proc/self/maps at exit
maps it to an object, `nm` to a function (text p_vaddr == p_offset assumed, as
gcc/ld lay out these objects).  Paths under the GPU box's repository copy are
read from this repository."""
import bisect
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local(path):
    m = re.search(r"/repo/(.*)$", path)
    if m and not os.path.exists(path):
        return os.path.join(REPO, m.group(1))
    return path


_syms = {}


def symbols(path):
    if path not in _syms:
        tab = []
        for flags in (["-n", "--defined-only"], ["-n", "-D", "--defined-only"]):
            try:
                out = subprocess.run(["nm", *flags, path], capture_output=True, text=True).stdout
            except OSError:
                out = ""
            for ln in out.splitlines():
                p = ln.split()
                if len(p) >= 3 and p[1] in "tTwW":
                    tab.append((int(p[0], 16), p[2]))
            if tab:
                break
        tab.sort()
        _syms[path] = ([a for a, _ in tab], [n for _, n in tab])
    return _syms[path]


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    pcs, maps, period = [], [], 20
    in_maps = False
    for ln in open(path):
        if ln.startswith("# samples"):
            period = int(ln.split()[-1])
            continue
        if ln.startswith("# maps"):
            in_maps = True
            continue
        if not in_maps:
            pcs.append(int(ln, 16))
        else:
            p = ln.split()
            if len(p) >= 6 and "x" in p[1]:
                a, b = (int(x, 16) for x in p[0].split("-"))
                maps.append((a, b, int(p[2], 16), p[5]))
    maps.sort()
    starts = [m[0] for m in maps]
    by_fn, by_obj = collections.Counter(), collections.Counter()
    for pc in pcs:
        i = bisect.bisect_right(starts, pc) - 1
        if i < 0 or pc >= maps[i][1]:
            by_fn["?"] += 1
            by_obj["?"] += 1
            continue
        a, _, off, obj = maps[i]
        name = os.path.basename(obj)
        by_obj[name] += 1
        addrs, names = symbols(local(obj))
        j = bisect.bisect_right(addrs, pc - a + off) - 1
        by_fn[f"{name}:{names[j] if j >= 0 else '?'}"] += 1
    # source lines of the hottest functions of the encoder binary (objects built with -g)
    lines = collections.Counter()
    for pc in pcs:
        i = bisect.bisect_right(starts, pc) - 1
        if i >= 0 and pc < maps[i][1] and os.path.basename(maps[i][3]).startswith("lencod"):
            lines[(local(maps[i][3]), pc - maps[i][0] + maps[i][2])] += 1
    n = max(1, len(pcs))
    print(f"{len(pcs)} samples ({len(pcs) * period / 1e3:.1f} ms of ME region wall time)")
    print("by object:")
    for k, v in by_obj.most_common():
        print(f"  {100 * v / n:5.1f}%  {v * period / 1e3:8.2f} ms  {k}")
    print("by function:")
    for k, v in by_fn.most_common(top):
        print(f"  {100 * v / n:5.1f}%  {v * period / 1e3:8.2f} ms  {k}")
    if lines:
        hot = lines.most_common(400)
        binp = hot[0][0][0]
        out = subprocess.run(["addr2line", "-e", binp, *[hex(o) for (_, o), _ in hot]], capture_output=True,
                             text=True).stdout.split("\n")
        by_line = collections.Counter()
        for ((_, _), v), src in zip(hot, out):
            by_line[os.path.basename(src.strip()) or "?"] += v
        print("encoder source lines:")
        for k, v in by_line.most_common(top):
            print(f"  {100 * v / n:5.1f}%  {v * period / 1e3:8.2f} ms  {k}")


if __name__ == "__main__":
    main()
