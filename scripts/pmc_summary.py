#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/diag_session.sh output) for one kernel, per variant:
python scripts/pmc_summary.py KERNEL_SUBSTR OUT.json LABEL=DIR [LABEL=DIR ...]

Each DIR holds p*/pmc_counter_collection.csv passes. Counters are averaged per dispatch of the
kernels whose name contains KERNEL_SUBSTR; derived ratios:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (GRBM sums the 8 XCDs)
  wait_any  = SQ_WAIT_ANY / SQ_WAVE_CYCLES,  wait_inst = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  kernel_us = mean dispatch duration of the pass that ran the SQ group (counters serialise it)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d, kern):
    vals = defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
        seen = set()
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    g = out.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in out:
        out["mfma_busy"] = out["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
    if "SQ_WAVE_CYCLES" in out:
        for c, name in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst")):
            if c in out:
                out[name] = out[c] / out["SQ_WAVE_CYCLES"]
    if durs:
        out["dispatch_us_under_pmc"] = sum(durs) / len(durs)
    return out


def main():
    kern, dst = sys.argv[1], sys.argv[2]
    res = {"kernel": kern, "variants": {}}
    for spec in sys.argv[3:]:
        label, d = spec.split("=", 1)
        res["variants"][label] = summarise(d, kern)
    json.dump(res, open(dst, "w"), indent=1)
    for label, v in res["variants"].items():
        print(label, {k: round(v[k], 3) for k in ("mfma_busy", "wait_any", "wait_inst", "dispatch_us_under_pmc") if k in v})


if __name__ == "__main__":
    main()
