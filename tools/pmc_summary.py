#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: mean per dispatch of each counter for a kernel."""
import collections, csv, glob, os, sys
root = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "me_units_kernel"
for f in sorted(glob.glob(os.path.join(root, "*", "p_counter_collection.csv"))):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{os.path.basename(os.path.dirname(f)):6s} {k:24s} {sum(v)/len(v):14.4g}  (n={len(v)})")
