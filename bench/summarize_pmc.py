#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/<target>_<set>/p_counter_collection.csv)
into a markdown table of per-dispatch averages for the stencil kernels."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
print("| target | counter | mean per dispatch |\n|---|---|---|")
for tgt in sorted({p.split("/")[-2].rsplit("_", 1)[0] for p in glob.glob(f"{root}/*_*/p_counter_collection.csv")}):
    agg = collections.defaultdict(list)
    kname = ""
    for f in sorted(glob.glob(f"{root}/{tgt}_*/p_counter_collection.csv")):
        if not f.split("/")[-2][len(tgt) + 1:].isdigit():  # another target sharing the prefix
            continue
        for r in csv.DictReader(open(f)):
            if "advdiff" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                kname = r["Kernel_Name"].split("(")[0]
    for k, v in sorted(agg.items()):
        print(f"| {tgt} | {k} | {sum(v) / len(v):.4g} |")
    print(f"| {tgt} | kernel | `{kname}` |")
