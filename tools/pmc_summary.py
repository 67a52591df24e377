#!/usr/bin/env python3
"""Summarise a tools/profile_box.sh run (rocprofv3 kernel trace + separate PMC passes).

usage: python3 tools/pmc_summary.py gpurun_out/prof_<tag> <tag> [--blocks N]

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats table), profiles/<tag>_summary.md
(per-kernel duration, HBM bytes per launch, counters) and profiles/pmc_latest.json (what
bench.py reports as roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half of the bytes of a wide coalesced streaming read,
so it is doubled; WRITE_SIZE is exact for 16-byte-per-lane streaming stores.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH_ARGS = "bench.py --steps 50 --warmup 5 --prewarm-s 0.3 --no-cpu-baseline --no-host-inclusive"


def short(name):
    # "void ppfs::rs255_encode_kernel<6, 0, 1, 1, 0>(unsigned char const*, ...)" -> rs255_encode_kernel<6, 0, 1, 1, 0>
    n = name.replace("void ", "")
    n = n.split("(")[0]
    return (n.replace("ppfs::", "").replace("wg::", "").replace("pair::", "").replace("bf::", "")
            .replace("bs::", "").replace("w1::", ""))


def counters(path):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    if not os.path.exists(path):
        return per
    with open(path) as f:
        for row in csv.DictReader(f):
            per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    d, tag = sys.argv[1], sys.argv[2]
    blocks = 1 << 20
    if "--blocks" in sys.argv:
        blocks = int(sys.argv[sys.argv.index("--blocks") + 1])
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(d, "trace_kernel_stats.csv")
    if not os.path.exists(stats):
        stats = os.path.join(d, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    merged = defaultdict(dict)
    red = os.path.join(d, "counters_median.json")  # tools/pmc_reduce.py, reduced on the box
    if os.path.exists(red):
        for k, cs in json.load(open(red)).items():
            merged[short(k)].update(cs)
    for sub in ("fetch", "write", "sq", "sq2"):
        for k, cs in counters(os.path.join(d, sub, f"{sub}_counter_collection.csv")).items():
            for c, v in cs.items():
                merged[k][c] = statistics.median(v)
    lines = [f"# rocprofv3 summary: {tag}", "",
             "Command: `tools/profile_box.sh` (" + BENCH_ARGS + ", 2^20 blocks)", "",
             "| kernel | calls | avg us | min us | HBM read MB (2xFETCH) | HBM write MB | traffic MB/launch |",
             "|---|---|---|---|---|---|---|"]
    latest = {}
    for r in rows:
        k = short(r["Name"])
        if not k.startswith(("rs255", "rs_wg", "rs_pair", "rs_solo", "rs_bs", "rs_w1", "inject", "crc", "ham", "parity", "rs_generic")):
            continue
        c = merged.get(k, {})
        fetch = 2 * c.get("FETCH_SIZE", float("nan")) * 1024
        write = c.get("WRITE_SIZE", float("nan")) * 1024
        lines.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} "
                     f"| {fetch / 1e6:.1f} | {write / 1e6:.1f} | {(fetch + write) / 1e6:.1f} |")
        base = k.split(",")[0] + ">" if "," in k else k
        latest[base] = {"kernel": base, "kernel_full": k, "blocks": blocks,
                        "avg_launch_ns": float(r["AverageNs"]),
                        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
                        "hbm_bytes_per_launch": fetch + write, "counters": c}
    # per-dispatch durations (tools/trace_reduce.py): the in-step launches apart from the rest
    durs = {}
    tdp = os.path.join(d, "trace_durations.json")
    if os.path.exists(tdp):
        shutil.copy(tdp, os.path.join(prof, f"{tag}_trace_durations.json"))
        for k, v in json.load(open(tdp)).items():
            durs[short(k)] = v
        for k, v in latest.items():
            st = (durs.get(v["kernel_full"]) or {}).get("in_step")
            if st:
                v["avg_launch_ns_in_step"] = st["mean_us"] * 1e3
                v["in_step_launches"] = st["n"]
    # the same command's untraced bench line (tools/profile_box.sh bench_line_untraced.json): the
    # profile's in-step averages reproduce its roofline.frac
    ul = os.path.join(d, "bench_line_untraced.json")
    if os.path.exists(ul) and os.path.getsize(ul) > 0:
        line = json.loads(open(ul).read().strip().splitlines()[-1])
        shutil.copy(ul, os.path.join(prof, f"{tag}_bench_untraced.json"))
        km, alg = line.get("kernels_ms", {}), line.get("roofline", {}).get("algorithmic_bytes_per_launch")
        lines += ["", f"Untraced bench line of the same command (same box, just before the trace): value {line.get('value')} "
                  f"GiB/s, roofline.frac {line.get('roofline', {}).get('frac')}, in-step frac {line.get('in_step_frac')}"]
        for kind, pref in step_kernels(line):
            for k, v in latest.items():
                if k.startswith(pref) and km.get(kind) and alg and "avg_launch_ns_in_step" in v:
                    ri = v["avg_launch_ns_in_step"] / 1e6
                    lines.append(f"- {kind}: untraced in-step {km[kind] * 1e3:.2f} us (frac {alg / (km[kind] * 1e-3) / 8e12:.4f}) vs "
                                 f"rocprofv3 in-step-launch avg {ri * 1e3:.2f} us (frac {alg / (ri * 1e-3) / 8e12:.4f}); "
                                 f"ratio {km[kind] / ri:.4f}")
    # the traced run's own bench line (tools/profile_box.sh bench_line.json): its in-step kernel
    # times (dispatch packets) against the rocprofv3 averages of the same invocation
    bl = os.path.join(d, "bench_line.json")
    if os.path.exists(bl) and os.path.getsize(bl) > 0:
        line = json.loads(open(bl).read().strip().splitlines()[-1])
        km = line.get("kernels_ms", {})
        lines += ["", f"Bench line of the traced run: value {line.get('value')} GiB/s, in-step frac "
                  f"{line.get('in_step_frac')}, roofline.frac {line.get('roofline', {}).get('frac')}"]
        alg = line.get("roofline", {}).get("algorithmic_bytes_per_launch")
        for kind, pref in step_kernels(line):
            for k, v in latest.items():
                if k.startswith(pref) and km.get(kind) and alg:
                    ra = v["avg_launch_ns"] / 1e6
                    lines.append(f"- {kind}: in-step {km[kind] * 1e3:.2f} us (frac {alg / (km[kind] * 1e-3) / 8e12:.4f}) vs "
                                 f"rocprofv3 avg {ra * 1e3:.2f} us over all launches (frac {alg / (ra * 1e-3) / 8e12:.4f}); "
                                 f"ratio {km[kind] / ra:.4f}")
                    if "avg_launch_ns_in_step" in v:
                        ri = v["avg_launch_ns_in_step"] / 1e6
                        lines.append(f"  - rocprofv3 avg over the {v['in_step_launches']} in-step launches (tools/trace_reduce.py): "
                                     f"{ri * 1e3:.2f} us (frac {alg / (ri * 1e-3) / 8e12:.4f}); ratio {km[kind] / ri:.4f}")
    lines += ["", "Counters (median per dispatch):", ""]
    for k, v in latest.items():
        lines.append(f"- `{v['kernel_full']}`: " + ", ".join(f"{a}={b:.4g}" for a, b in sorted(v["counters"].items())))
    open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    sha_path = os.path.join(d, "lib.sha256")  # the library build the counters were collected on
    lib_sha = open(sha_path).read().strip() if os.path.exists(sha_path) else None
    # profiles of other workloads on the SAME library build (e.g. the cfg5 bench) merge into it, so
    # bench.py finds traffic for each of their kernels; a new build starts it afresh
    path = os.path.join(prof, "pmc_latest.json")
    try:
        old = json.load(open(path))
    except Exception:
        old = {}
    json.dump(merge_latest(old, latest, lib_sha, tag), open(path, "w"), indent=1)
    print("\n".join(lines))


def step_kernels(line):
    """(kind, kernel-name prefix) of the bench step's encode and decode: the 2t = 32 byte-slice kernels
    when the line's roofline names one, else the t <= 4 ticket kernels (the configs leg's other
    kernels in the same profile are not the step's)."""
    bs = "rs_bs" in str(line.get("roofline", {}).get("kernel", ""))
    return (("encode", "rs_bs_encode" if bs else "rs_wg_encode_tk"), ("decode", "rs_bs_decode" if bs else "rs_wg_decode_tk"))


def merge_latest(old, latest, lib_sha, tag):
    """pmc_latest.json after a profile `tag` of library `lib_sha`: a new build starts afresh; on the
    same build, a kernel profiled in both runs keeps the entry of the run whose bench step launched it
    (more in-step launches) -- the headline profile's 1-error t = 3 decode, not the cfg5 run's clean
    configs-leg decode of the same kernel."""
    if not (lib_sha and old.get("lib_sha256") == lib_sha):
        return {"tag": tag, "lib_sha256": lib_sha, "kernels": latest}
    merged_k = dict(old.get("kernels", {}))
    for k, v in latest.items():
        if v.get("in_step_launches", 0) >= merged_k.get(k, {}).get("in_step_launches", 0):
            merged_k[k] = v
    tags = old.get("tag", "")
    return {"tag": tags if tag in tags.split("+") else tags + "+" + tag, "lib_sha256": lib_sha, "kernels": merged_k}


if __name__ == "__main__":
    main()
