#!/usr/bin/env python3
"""Reduce a rocprofv3 kernel trace (<dir>/trace_kernel_trace.csv, one row per dispatch) on the GPU box
to per-kernel durations, split the way bench.py measures them:

  all       every dispatch of the kernel (rewarm loops, standalone launches, warmup, timed steps)
  in_step   the dispatches that run inside a bench step: an encode followed by inject_kernel, a
            decode preceded by inject_kernel (the warmup, timed and in-step-timed steps) -- the
            launches bench.py's kernels_ms / roofline.achieved are the mean of

usage: python3 tools/trace_reduce.py <trace csv> <out.json>"""
import csv
import json
import statistics
import sys


def short(name):
    n = name.replace("void ", "").split("(")[0]
    return n.replace("ppfs::", "").replace("wg::", "").replace("pair::", "").replace("bf::", "")


def stats(us):
    if not us:
        return None
    return {"n": len(us), "mean_us": round(statistics.fmean(us), 3), "median_us": round(statistics.median(us), 3),
            "min_us": round(min(us), 3), "max_us": round(max(us), 3)}


def main():
    src, out = sys.argv[1], sys.argv[2]
    rows = []
    with open(src) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    names = [r[2] for r in rows]
    dur = [(r[1] - r[0]) / 1000.0 for r in rows]
    res = {}
    for k in sorted(set(names)):
        idx = [i for i, n in enumerate(names) if n == k]
        step = [i for i in idx
                if (i + 1 < len(names) and names[i + 1].startswith("inject_kernel") and "encode" in k)
                or (i > 0 and names[i - 1].startswith("inject_kernel") and "decode" in k)]
        res[k] = {"all": stats([dur[i] for i in idx]), "in_step": stats([dur[i] for i in step])}
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
