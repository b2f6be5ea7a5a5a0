#!/usr/bin/env python3
"""Why does the main stream sit idle?  Joins a rocprofv3 kernel trace with its HIP API trace
(``--kernel-trace --hip-trace``) by correlation id and, for every idle gap > ``--min-us`` on
the busiest stream inside the last ``--steps`` steps, asks whether the host issued the next
kernel's launch AFTER the previous kernel had already finished (host-bound gap) or before it
(the GPU held the kernel back: a cross-stream event wait or a dependency).

    python scripts/launch_lag.py x_kernel_trace.csv x_hip_api_trace.csv --delim sgd_kernel
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("api")
    ap.add_argument("--delim", default="sgd_kernel")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--min-us", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    launch = {}
    with open(a.api) as f:
        for r in csv.DictReader(f):
            fn = r.get("Function") or r.get("Operation") or ""
            if "Launch" in fn or "launch" in fn:
                launch[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fn)
    rows = []
    with open(a.kernels) as f:
        for r in csv.DictReader(f):
            sid = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], sid,
                         r.get("Correlation_Id")))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.delim in r[2]]
    starts = [m for j, m in enumerate(marks) if j == 0 or m != marks[j - 1] + 1]
    lo, hi = starts[-a.steps - 1] + 1, starts[-1] + 1
    win = rows[lo:hi]
    busy = defaultdict(float)
    for s, e, _n, sid, _c in win:
        busy[sid] += e - s
    main_sid = max(busy, key=busy.get)
    ms = [r for r in win if r[3] == main_sid]
    host_late = defaultdict(lambda: [0.0, 0])
    gpu_held = defaultdict(lambda: [0.0, 0])
    no_api = 0.0
    for prev, nxt in zip(ms, ms[1:]):
        gap = (nxt[0] - prev[1]) / 1e3
        if gap < a.min_us:
            continue
        key = (prev[2][:50], nxt[2][:50])
        lz = launch.get(nxt[4])
        if lz is None:
            no_api += gap
            continue
        if lz[1] > prev[1]:          # the launch call returned after the previous kernel ended
            late = min(gap, (lz[1] - prev[1]) / 1e3)
            host_late[key][0] += late
            host_late[key][1] += 1
            if gap > late:
                gpu_held[key][0] += gap - late
        else:
            gpu_held[key][0] += gap
            gpu_held[key][1] += 1
    n = a.steps
    tl = sum(v[0] for v in host_late.values()) / n
    tg = sum(v[0] for v in gpu_held.values()) / n
    print(f"main stream {main_sid}: idle gaps > {a.min_us} us per step: host-late {tl:.0f} us, "
          f"GPU-held (launch issued before the previous kernel ended) {tg:.0f} us, no API record {no_api / n:.0f} us\n")
    for title, d in (("host-late", host_late), ("GPU-held", gpu_held)):
        print(f"| {title}: gap before | gap after | us/step | count/step |\n|---|---|---:|---:|")
        for (b, nx), (t, c) in sorted(d.items(), key=lambda kv: -kv[1][0])[:a.top]:
            print(f"| `{b}` | `{nx}` | {t / n:.0f} | {c / n:.1f} |")
        print()


if __name__ == "__main__":
    main()
