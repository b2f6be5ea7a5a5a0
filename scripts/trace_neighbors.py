#!/usr/bin/env python3
"""For every dispatch of kernels matching PATTERN in a rocprofv3 kernel trace, count which
kernel runs right after it (and before it): who needs the fills / copies.

    python scripts/trace_neighbors.py trace.csv SubTensorOp"""
import collections
import csv
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    after, before = collections.Counter(), collections.Counter()
    for i, r in enumerate(rows):
        if pat in r["Kernel_Name"]:
            if i + 1 < len(rows):
                after[rows[i + 1]["Kernel_Name"][:90]] += 1
            if i:
                before[rows[i - 1]["Kernel_Name"][:90]] += 1
    print(f"## neighbours of {pat}\n\nnext kernel:")
    for k, v in after.most_common(12):
        print(f"  {v:5d}  {k}")
    print("previous kernel:")
    for k, v in before.most_common(12):
        print(f"  {v:5d}  {k}")


if __name__ == "__main__":
    main()
