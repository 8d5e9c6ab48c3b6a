#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: mean per dispatch of each counter for a kernel.
Usage: pmc_summary.py PMCDIR [kernel-substring] [--traffic-json OUT]
With --traffic-json, writes HBM bytes per launch of the kernel:
FETCH_SIZE x 2 (gfx950 tallies 128-B read requests at 64 B, MI355X_MICROARCH.md
"HBM") + WRITE_SIZE, both reported in KiB by rocprofv3."""
import collections, csv, glob, json, os, sys
import argparse
ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("kernel", nargs="?", default="me_items_kernel<true, false, false")
ap.add_argument("--traffic-json")
a_ = ap.parse_args()
root, kern, out_json = a_.root, a_.kernel, a_.traffic_json
means = {}
for f in sorted(set(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        means[k] = sum(v) / len(v)
        print(f"{k:24s} {means[k]:14.6g}  (n={len(v)})  {os.path.relpath(f, root)}")
if out_json and "FETCH_SIZE" in means and "WRITE_SIZE" in means:
    fetch = means["FETCH_SIZE"] * 1024 * 2
    write = means["WRITE_SIZE"] * 1024
    json.dump({"case": "c2_syn_1080p_fs32", "kernel": kern, "fetch_size_kib": means["FETCH_SIZE"],
               "write_size_kib": means["WRITE_SIZE"], "bytes_per_launch": round(fetch + write),
               "note": "FETCH_SIZE doubled per the gfx950 correction (calibrated for 16 B/lane reads; "
                       "this kernel fetches 4 B/lane LDS-DMA dwords -- uncalibrated width). The whole "
                       "working set (cur + ref planes, 4.2 MB) is Infinity-Cache resident across launches."},
              open(out_json, "w"), indent=1)
    print("wrote", out_json)
