"""Build profiles/<tag>/summary.json from a scripts/gpu_profile.sh run: per-kernel calls and
average duration (rocprofv3 --kernel-trace --stats) and HBM bytes per launch from the separate
--pmc FETCH_SIZE / WRITE_SIZE passes.  gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3):
FETCH_SIZE counts half of wide streaming reads, so read bytes = 2 x FETCH_SIZE KiB x 1024.

    python scripts/profile_summary.py gpurun_out/r02 profiles/r02 "<note>"
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys


def one(pattern):
    hits = glob.glob(pattern, recursive=True)
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


def counters(path, name):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


def per_launch(path, name):
    """kernel -> [counter value of its 1st, 2nd, ... launch] (dispatch order)."""
    per = collections.defaultdict(list)
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name]
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def size_classes(trace_path, fetch_path, write_path):
    """One kernel launched at several sizes (e.g. a whole round and its column chunks): its
    launches grouped by HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, two significant digits), each
    class with its launch count, bytes and the average duration of the same launches in the
    trace pass (the program is deterministic: the k-th launch of a kernel is the same launch in
    every pass)."""
    durs = collections.defaultdict(list)
    rows = list(csv.DictReader(open(trace_path)))
    for t in sorted(rows, key=lambda t: int(t["Start_Timestamp"])):
        durs[t["Kernel_Name"]].append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3)
    fe, wr = per_launch(fetch_path, "FETCH_SIZE"), per_launch(write_path, "WRITE_SIZE")
    out = {}
    for k in fe:
        n = min(len(fe[k]), len(wr.get(k, [])), len(durs.get(k, [])))
        if n == 0:
            continue
        cls = collections.defaultdict(list)
        for i in range(n):
            b = 2 * fe[k][i] * 1024 + wr[k][i] * 1024
            cls[float(f"{b:.2g}")].append((b, durs[k][i]))
        if len(cls) < 2:
            continue
        out[k] = [{"launches": len(v), "hbm_bytes_per_launch": sum(x[0] for x in v) / len(v),
                   "avg_us": sum(x[1] for x in v) / len(v)}
                  for _, v in sorted(cls.items(), reverse=True)]
    return out


def main(src, dst, note):
    os.makedirs(dst, exist_ok=True)
    stats = one(f"{src}/trace/**/*kernel_stats.csv")
    trace = one(f"{src}/trace/**/*kernel_trace.csv")
    shutil.copy(stats, f"{dst}/kernel_stats.csv")
    shutil.copy(trace, f"{dst}/kernel_trace.csv")
    fetch = counters(one(f"{src}/fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    write = counters(one(f"{src}/write/**/*counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for r in csv.DictReader(open(stats)):
        e = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
        durs = sorted((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3
                      for t in csv.DictReader(open(trace)) if t["Kernel_Name"] == r["Name"])
        if durs:
            e["median_us"] = durs[len(durs) // 2]
        if r["Name"] in fetch and r["Name"] in write:
            e["FETCH_SIZE_KiB"] = fetch[r["Name"]]
            e["WRITE_SIZE_KiB"] = write[r["Name"]]
            e["hbm_read_bytes_corrected"] = 2 * fetch[r["Name"]] * 1024
            e["hbm_write_bytes"] = write[r["Name"]] * 1024
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_corrected"] + e["hbm_write_bytes"]
        kernels[r["Name"]] = e
    out = {"note": note, "kernels": kernels}
    sc = size_classes(trace, one(f"{src}/fetch/**/*counter_collection.csv"),
                      one(f"{src}/write/**/*counter_collection.csv"))
    if sc:
        out["size_classes"] = sc
    last = int(os.environ.get("LAST", "0"))
    if last:   # the timed steps: the last LAST launches of every kernel launched that often
        per = collections.defaultdict(list)
        for t in csv.DictReader(open(trace)):
            per[t["Kernel_Name"]].append((int(t["Start_Timestamp"]),
                                          (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3))
        g = {"note": f"the last {last} launches of each kernel in kernel_trace.csv (the timed steps)"}
        for name, v in per.items():
            if len(v) >= last:
                d = [x[1] for x in sorted(v)[-last:]]
                m = re.search(r"(\w+)\s*[<(]", name.replace("(anonymous namespace)", ""))
                short = m.group(1) if m else name
                g.setdefault(f"{short}_avg_us", sum(d) / last)
                g.setdefault(f"{short}_kernels", []).append(name)
        out["graph_step_launches"] = g
    json.dump(out, open(f"{dst}/summary.json", "w"), indent=1)
    print(f"wrote {dst}/summary.json ({len(kernels)} kernels)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
