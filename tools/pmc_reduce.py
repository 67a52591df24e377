#!/usr/bin/env python3
"""Reduce rocprofv3 PMC pass outputs on the GPU box to a small JSON (the raw per-dispatch CSVs are
tens of MB): {kernel short name: {counter: median over dispatches}}.
usage: python3 tools/pmc_reduce.py <prof dir with fetch/ write/ sq/ sq2/ subdirs> <out.json>"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").split("(")[0]
    return n.replace("ppfs::", "").replace("wg::", "").replace("pair::", "").replace("bf::", "")


def main():
    d, out = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, f"{sub}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as f:
            for row in csv.DictReader(f):
                per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    red = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in per.items()}
    json.dump(red, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
