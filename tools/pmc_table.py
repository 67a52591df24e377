#!/usr/bin/env python3
"""Per-kernel (by name + grid size) median of every PMC counter over rocprofv3 CSV passes.
usage: python3 tools/pmc_table.py gpurun_out/pmc_<tag> [filter]"""
import csv, glob, statistics, sys
from collections import defaultdict

d = defaultdict(lambda: defaultdict(list))
for path in glob.glob(sys.argv[1] + "/p*/*_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("void ", "").split("(")[0].replace("ppfs::", "").replace("wg::", "")
        if len(sys.argv) > 2 and sys.argv[2] not in n:
            continue
        key = f'{n} g{int(r["Grid_Size"]) // int(r["Workgroup_Size"])}'
        d[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for k in d for c in d[k]})
for k in sorted(d):
    m = {c: statistics.median(d[k][c]) for c in d[k]}
    print(k)
    print("   " + "  ".join(f"{c}={m[c]:.4g}" for c in cols if c in m))
