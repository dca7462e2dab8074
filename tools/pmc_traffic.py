#!/usr/bin/env python3
"""Per-launch PMC figures of one kernel from rocprofv3 --pmc passes of a bench run, written to
profiles/traffic.json under bench.py's profile key (workload:mode:R:Q:kernel-tag), where
bench.py's roofline reads them.  Corrections as MI355X_MICROARCH.md §HBM prescribes:

  L2->fabric read bytes  = FETCH_SIZE[KiB] * 1024 * 2   (gfx950 tallies each 128-B line
                                                          request at 64 B; cross-checked with
                                                          TCC_EA0_RDREQ_128B * 128 when present)
  L2->fabric write bytes = WRITE_SIZE[KiB] * 1024
These count requests that leave L2, Infinity-Cache hits included: not proven DRAM bytes.

Optional passes: --tcc (TCC_HIT_sum, TCC_MISS_sum, TCC_EA0_RDREQ_128B_sum) -> L2 hit rate;
--sq (SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_ACTIVE_INST_VALU, ...) -> wave-cycle shares;
--flops (SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64) -> f64 FLOP per launch
(64 lanes x (2 FMA + ADD + MUL + TRANS) per instruction; an upper bound when lanes are masked).

usage: tools/pmc_traffic.py --key cfg3:raster:R4096:Q100000:raster+skip --kernel k_eval_pairs \
          [--fetch DIR] [--write DIR] [--tcc DIR] [--sq DIR] [--flops DIR] [--source TEXT]
Each DIR holds rocprofv3's *counter_collection.csv of one counter pass.

A multi-launch evaluation (K2s: sorts, two segment launches, output launch) is summarised per
step: --kernel takes comma-separated name patterns, and --per names the kernel launched once per
step; each counter is then the sum over every matching dispatch / the number of --per
dispatches (e.g. --kernel k_seg_,k_scan_ --per k_seg_final).
"""
import argparse
import csv
import glob
import json
import os
import statistics


PER = None  # --per: the once-per-step kernel of a multi-launch evaluation


def load(d, kernel, counter):
    pats = kernel.split(",")
    vals, steps = [], set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            if any(p in r["Kernel_Name"] for p in pats):
                vals.append(float(r["Counter_Value"]))
            if PER and PER in r["Kernel_Name"]:
                steps.add(r.get("Dispatch_Id", len(steps)))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel '{kernel}' in {d}")
    if PER:
        if not steps:
            raise SystemExit(f"no {counter} rows for the per-step kernel '{PER}' in {d}")
        return sum(vals) / len(steps), len(steps)
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--per", default=None)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--tcc")
    ap.add_argument("--sq")
    ap.add_argument("--flops")
    ap.add_argument("--source", default=None)
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    global PER
    PER = a.per
    rec = {"kernel": a.kernel, "source": a.source}
    if a.per:
        rec["per_step_of"] = a.per
    if a.fetch and a.write:
        fetch_kib, n1 = load(a.fetch, a.kernel, "FETCH_SIZE")
        write_kib, n2 = load(a.write, a.kernel, "WRITE_SIZE")
        read_b, write_b = fetch_kib * 1024 * 2, write_kib * 1024
        rec.update({"launches_profiled": min(n1, n2), "fetch_size_kib_raw": fetch_kib,
                    "write_size_kib_raw": write_kib,
                    "l2_fabric_read_bytes_per_launch": read_b,
                    "l2_fabric_write_bytes_per_launch": write_b,
                    "l2_fabric_bytes_per_launch": read_b + write_b,
                    "correction": "read = 2 x FETCH_SIZE (gfx950 128-B requests tallied at "
                                  "64 B); includes Infinity-Cache hits"})
    if a.tcc:
        hit, _ = load(a.tcc, a.kernel, "TCC_HIT_sum")
        miss, _ = load(a.tcc, a.kernel, "TCC_MISS_sum")
        rec.update({"tcc_hit": hit, "tcc_miss": miss,
                    "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None})
        try:
            req128, _ = load(a.tcc, a.kernel, "TCC_EA0_RDREQ_128B_sum")
            rec.update({"tcc_ea0_rdreq_128b": req128,
                        "read_bytes_from_128b_requests": req128 * 128})
        except SystemExit:
            pass
    if a.sq:
        cyc, _ = load(a.sq, a.kernel, "SQ_WAVE_CYCLES")
        out = {"sq_wave_cycles": cyc}
        for c, k in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_ACTIVE_INST_VALU", "valu_frac"),
                     ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_any_frac")):
            try:
                v, _ = load(a.sq, a.kernel, c)
                out[k] = round(v / cyc, 4) if cyc else None
            except SystemExit:
                pass
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM", "SQ_INSTS_SALU", "SQ_BUSY_CYCLES"):
            try:
                out[c.lower()], _ = load(a.sq, a.kernel, c)
            except SystemExit:
                pass
        rec.update(out)
    if a.flops:
        n = {}
        for c in ("FMA", "ADD", "MUL", "TRANS"):
            n[c], _ = load(a.flops, a.kernel, f"SQ_INSTS_VALU_{c}_F64")
        rec.update({"f64_insts": n,
                    "f64_flop_per_launch": 64 * (2 * n["FMA"] + n["ADD"] + n["MUL"] + n["TRANS"]),
                    "flop_rule": "64 lanes x (2 FMA + ADD + MUL + TRANS) per f64 VALU "
                                 "instruction (SQ_INSTS_VALU_*_F64)"})
    db = {}
    if os.path.exists(a.out):
        db = json.load(open(a.out))
    db.setdefault(a.key, {}).update({k: v for k, v in rec.items() if v is not None})
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1)
    print(json.dumps({a.key: db[a.key]}))


if __name__ == "__main__":
    main()
