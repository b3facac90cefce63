"""Kernel statistics and launch timelines from a rocprofv3 --kernel-trace SQLite result
(`rocprofv3 --kernel-trace -d DIR -o NAME -- ...` writes DIR/NAME_results.db).

python scripts/kernel_timeline.py DB [--timeline PATTERN --first N --count K] [--json OUT]

--timeline: print K consecutive launches starting at the N-th launch of a kernel whose name
contains PATTERN, with each launch's duration and the idle gap before it (the GPU-side cost of
launch boundaries that HIP events around a whole round do not separate)."""
import argparse
import collections
import json
import re
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    return [(re.sub(r"\(dl::TileArgs\)$", "", n), s, e) for n, s, e in rows]


def stats(rows):
    agg = collections.OrderedDict()
    for n, s, e in rows:
        agg.setdefault(n, []).append((e - s) / 1e3)
    out = {}
    for n, v in agg.items():
        v2 = sorted(v)
        out[n] = {"count": len(v), "median_us": v2[len(v2) // 2], "mean_us": sum(v) / len(v),
                  "min_us": v2[0]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", default=None)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=20)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    rows = load(args.db)
    st = stats(rows)
    for n, d in st.items():
        print(f"{d['count']:5d}  med {d['median_us']:9.1f}  mean {d['mean_us']:9.1f}  "
              f"min {d['min_us']:9.1f} us  {n[:110]}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"kernels": st}, f, indent=1)
    if args.timeline:
        idx = [i for i, (n, _, _) in enumerate(rows) if args.timeline in n]
        if len(idx) > args.first:
            i0 = idx[args.first]
            prev_end = rows[i0 - 1][2] if i0 > 0 else rows[i0][1]
            print(f"\ntimeline from launch {args.first} of '{args.timeline}':")
            for n, s, e in rows[i0:i0 + args.count]:
                print(f"  gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f} us  {n[:90]}")
                prev_end = e


if __name__ == "__main__":
    main()
