#!/usr/bin/env python3
"""Longest HIP API calls of a rocprofv3 ``*_hip_api_trace.csv`` (per function: count, total,
max; then the N longest single calls) -- where a host thread blocked."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            except (TypeError, ValueError):
                continue                       # a row torn by two writers
            rows.append((e - s, r.get("Function") or r.get("Operation"), r.get("Thread_Id"), s))
    agg = defaultdict(lambda: [0, 0, 0])
    for d, fn, _t, _s in rows:
        a = agg[fn]
        a[0] += 1
        a[1] += d
        a[2] = max(a[2], d)
    t0 = min(r[3] for r in rows) if rows else 0
    print("| function | calls | total ms | max ms |\n|---|---:|---:|---:|")
    for fn, (c, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| {fn} | {c} | {tot / 1e6:.1f} | {mx / 1e6:.2f} |")
    print("\n| longest calls: function | thread | ms | at s |\n|---|---|---:|---:|")
    for d, fn, t, s in sorted(rows, reverse=True)[:top]:
        print(f"| {fn} | {t} | {d / 1e6:.2f} | {(s - t0) / 1e9:.3f} |")


if __name__ == "__main__":
    main()
