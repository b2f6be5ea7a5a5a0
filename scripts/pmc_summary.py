#!/usr/bin/env python3
"""Join rocprofv3 counter passes with a kernel-trace run: per kernel (name prefix), mean
duration, mean counter values per dispatch, and derived rates (HBM TB/s from FETCH_SIZE +
WRITE_SIZE, bf16 MFMA TFLOP/s from SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512, MFMA-busy share).

    python scripts/pmc_summary.py --trace tr.csv --pmc p1.csv p2.csv ... --top 25
"""
import argparse
import collections
import csv


def short(n, k=60):
    n = n.replace("void ", "")
    return n[:k]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--pmc", nargs="+", required=True)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    ap.add_argument("--raw", action="store_true", help="also list every counter's mean per kernel")
    a = ap.parse_args()
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in a.pmc:
        for r in csv.DictReader(open(f)):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    print(f"## {a.title}\n")
    print("| kernel | calls | mean us | HBM read MB | HBM write MB | TB/s | bf16 MFMA TF/s | % of 2.5 PF peak | LDS bank conf / LDS inst |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for name, ds in rows:
        us = sum(ds) / len(ds)
        c = {k: sum(v) / len(v) for k, v in ctr.get(name, {}).items()}
        rd = c.get("FETCH_SIZE", float("nan")) / 1024     # KB -> MB
        wr = c.get("WRITE_SIZE", float("nan")) / 1024
        tbs = (rd + wr) / 1e6 / (us / 1e6) if us > 0 else float("nan")
        tf = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512 / (us / 1e6) / 1e12 if us > 0 else float("nan")
        busy = 100.0 * tf / 2500.0
        lds = (f"{c['SQ_LDS_BANK_CONFLICT']:.3g} / {c['SQ_INSTS_LDS']:.3g}"
               if "SQ_LDS_BANK_CONFLICT" in c and "SQ_INSTS_LDS" in c else "-")
        print(f"| `{name}` | {len(ds)} | {us:.1f} | {rd:.1f} | {wr:.1f} | {tbs:.2f} | {tf:.0f} | {busy:.0f} | {lds} |")
    if a.raw:
        print("\n| kernel | counter | mean per dispatch |\n|---|---|---:|")
        for name, _ in rows:
            for k, v in sorted(ctr.get(name, {}).items()):
                print(f"| `{name[:40]}` | {k} | {sum(v) / len(v):.4g} |")
    print("\nTFLOP/s = "
          "SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / duration; durations from a separate --kernel-trace run "
          "(counter runs are serialised and not timed).")


if __name__ == "__main__":
    main()
