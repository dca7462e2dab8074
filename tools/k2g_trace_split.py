#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of tools/probe_k2g.py into its settings: the probe runs
(3 warm-up + reps) evaluations per setting in the order of its JSON lines, so the k_g_final
dispatches delimit the settings.  Prints, per setting, the median duration (us) of each K2g
kernel.  usage: k2g_trace_split.py <run_kernel_trace.csv> <probe stdout log> [--reps 10]"""
import csv
import json
import statistics
import sys


def main():
    trace, log = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    settings = [json.loads(l) for l in open(log) if l.startswith("{")]
    per = 3 + reps
    # one k_g_final per evaluation: evaluation e covers dispatches up to its k_g_final
    evals, cur = [], []
    for r in rows:
        n = r["Kernel_Name"]
        if "k_g_" not in n and "k_scan" not in n:
            continue
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        if short.startswith("k_g_eval"):
            short = "k_g_eval"
        if short.startswith("k_g_final"):
            short = "k_g_final"
        cur.append((short, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        if short == "k_g_final":
            evals.append(cur)
            cur = []
    for i, st in enumerate(settings):
        block = evals[i * per + 3:(i + 1) * per]
        if not block:
            break
        d = {}
        for ev in block:
            for k, us in ev:
                d.setdefault(k, []).append(us)
        med = {k: round(statistics.median(v), 1) for k, v in d.items()}
        tag = {k: st[k] for k in ("group", "tbits", "lds", "chunk", "minw") if k in st}
        print(json.dumps({**tag, "ms": st["ms"], **med}))


if __name__ == "__main__":
    main()
