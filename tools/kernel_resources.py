#!/usr/bin/env python3
"""VGPRs, spills and scratch of the kernels in a hipcc -Rpass-analysis=kernel-resource-usage log
(design check: a per-lane array that lands in scratch memory shows as ScratchSize > 0).

usage: hipcc ... -c uampath.hip -Rpass-analysis=kernel-resource-usage 2> ru.log
       python tools/kernel_resources.py ru.log [name-substring ...]"""
import re
import sys


def main():
    log, pats = sys.argv[1], sys.argv[2:]
    info, cur = {}, None
    for line in open(log):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            info[cur] = {}
            continue
        if cur and "remark:" in line:
            body = line.split("remark:", 1)[1].strip().split(" [-Rpass")[0]
            key, _, val = body.rpartition(": ")
            info[cur][key] = val
    for name, v in info.items():
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name[:70]:70s} VGPR {v.get('VGPRs', '?'):>4} spill {v.get('VGPRs Spill', '?'):>3} "
              f"scratch {v.get('ScratchSize [bytes/lane]', '?'):>4} occ {v.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
