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
