#!/usr/bin/env python3
"""Steady-state per-step kernel summary from a rocprofv3 ``*_kernel_trace.csv``.

Warmup (MIOpen find, TunableOp tuning, first-call JIT) swamps ``--stats`` totals.  This tool
cuts the trace at a kernel that runs exactly once per training step (the fused optimizer by
default), keeps the last ``--steps`` complete steps, and prints per-step kernel time by name,
the GPU-busy time and the wall span of a step (busy / span = how launch- or host-bound the
step is).

    python scripts/steady_profile.py gpurun_out/prof/x_kernel_trace.csv --delim sgd_kernel --steps 5
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--delim", default="sgd_kernel", help="substring of the once-per-step kernel name")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    ap.add_argument("--gaps", type=int, default=0, help="list the N largest idle-gap kinds of the main stream")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            sid = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], sid))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.delim in r[2]]
    # the optimizer may be split over several launches per step: keep the first of each run
    starts = [m for j, m in enumerate(marks) if j == 0 or m != marks[j - 1] + 1]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} '{a.delim}' launches; need {a.steps + 1}")
    lo, hi = starts[-a.steps - 1] + 1, starts[-1] + 1
    win = rows[lo:hi]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    per_stream = defaultdict(float)
    for s, e, n, sid in win:
        per_stream[sid] += (e - s) / 1e3
        tot[n] += (e - s) / 1e3
        cnt[n] += 1
    # wall time with at least one kernel running (union of the kernel intervals)
    cover, cur_s, cur_e = 0.0, None, None
    for s, e, _n, _sid in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                cover += (cur_e - cur_s) / 1e3
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        cover += (cur_e - cur_s) / 1e3
    busy = sum(tot.values()) / a.steps
    span = (rows[starts[-1]][1] - rows[starts[-a.steps - 1]][1]) / 1e3 / a.steps
    print(f"## {a.title or a.csv}\n")
    print(f"Steady state over the last {a.steps} steps (cut at `{a.delim}`): GPU-busy {busy / 1e3:.2f} ms "
          f"per step, step span {span / 1e3:.2f} ms ({100 * busy / span:.0f}% busy), "
          f"{len(win) / a.steps:.0f} kernels per step.\n")
    if len(per_stream) > 1:
        parts = ", ".join(f"stream {k}: {v / a.steps / 1e3:.2f} ms" for k, v in
                          sorted(per_stream.items(), key=lambda kv: -kv[1]))
        print(f"Per stream kernel time per step: {parts}; wall time with >= 1 kernel running "
              f"{cover / a.steps / 1e3:.2f} ms per step.\n")
    if len(per_stream) > 1 or a.gaps:
        # idle gaps of the busiest stream (the main one): where it waits on the host or on an
        # event of another stream
        main = max(per_stream.items(), key=lambda kv: kv[1])[0]
        ms = [r for r in win if r[3] == main]
        gaps = [(ms[i + 1][0] - ms[i][1], ms[i][2], ms[i + 1][2]) for i in range(len(ms) - 1)]
        tot_gap = sum(g for g, _, _ in gaps if g > 0) / 1e3 / a.steps
        big = sorted([g for g in gaps if g[0] > 5000], key=lambda g: -g[0])
        print(f"Stream {main}: {tot_gap / 1e3:.2f} ms idle per step between its kernels; "
              f"{sum(g for g, _, _ in big) / 1e3 / a.steps / 1e3:.2f} ms of it in {len(big) / a.steps:.0f} gaps > 5 us "
              f"per step.\n")
        if a.gaps:
            agg = defaultdict(lambda: [0.0, 0])
            for g, b, n in big:
                k = (b[:60], n[:60])
                agg[k][0] += g / 1e3 / a.steps
                agg[k][1] += 1
            print("| gap before | gap after | us/step | count/step |\n|---|---|---:|---:|")
            for (b, n), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.gaps]:
                print(f"| `{b}` | `{n}` | {t:.0f} | {c / a.steps:.1f} |")
            print()
    print("| kernel | ms/step | calls/step | % busy |\n|---|---:|---:|---:|")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        short = n if len(n) <= 100 else n[:97] + "..."
        print(f"| `{short}` | {t / a.steps / 1e3:.3f} | {cnt[n] / a.steps:.0f} | {100 * t / a.steps / busy:.1f} |")


if __name__ == "__main__":
    main()
