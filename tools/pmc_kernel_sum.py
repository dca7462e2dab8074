#!/usr/bin/env python3
"""Per-launch averages of every counter collected in the passes under a profile directory
(rocprofv3 --pmc ... -d <dir>/<pass> -o run --output-format csv), for the kernels whose name
contains a pattern.  usage: tools/pmc_kernel_sum.py <dir> [pattern ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    pats = sys.argv[2:] or ["k_h_eval"]
    for pat in pats:
        acc = collections.defaultdict(float)
        n = collections.defaultdict(set)
        for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
            for r in csv.DictReader(open(f)):
                if pat not in r["Kernel_Name"]:
                    continue
                c = r["Counter_Name"]
                acc[c] += float(r["Counter_Value"])
                n[c].add(r["Dispatch_Id"])
        print(f"== {pat}")
        for c in sorted(acc):
            print(f"  {c:40s} {acc[c] / max(1, len(n[c])):16.1f}  ({len(n[c])} launches)")


if __name__ == "__main__":
    main()
