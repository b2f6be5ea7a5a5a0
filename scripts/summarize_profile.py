#!/usr/bin/env python3
"""Turn a rocprofv3 ``*_kernel_stats.csv`` into a per-step markdown table for profiles/.

    python scripts/summarize_profile.py gpurun_out/prof_X/X_kernel_stats.csv --steps 7 \
        --title "BERT-large b256" > profiles/X.md
"""
import argparse
import csv
import re


def classify(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        return "GEMM (hipBLASLt)"
    if name.startswith("void ct::") or name.startswith("ct::"):
        return "cloudtik_amd HIP"
    if "rccl" in name.lower() or "nccl" in name.lower():
        return "RCCL"
    if "MIOpen" in name or "miopen" in name or re.match(r"^(igemm|naive_conv|Conv|Sp3|gridwise)", name):
        return "MIOpen"
    return "other (torch)"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, required=True, help="profiled steps (warmup + timed)")
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {a.title}\n")
    print(f"Source: `{a.csv}` (rocprofv3 --kernel-trace --stats), {a.steps} steps profiled; "
          f"GPU kernel time {tot / a.steps / 1e6:.2f} ms/step.\n")
    cats = {}
    for r in rows:
        c = classify(r["Name"])
        cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
    print("| category | ms/step | share |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {v / a.steps / 1e6:.2f} | {100 * v / tot:.1f}% |")
    print("\n| kernel | calls/step | avg us | ms/step | share |\n|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 100:
            name = name[:97] + "..."
        print(f"| `{name}` | {int(r['Calls']) / a.steps:.0f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{float(r['TotalDurationNs']) / a.steps / 1e6:.2f} | {100 * float(r['TotalDurationNs']) / tot:.1f}% |")


if __name__ == "__main__":
    main()
