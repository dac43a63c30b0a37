#!/usr/bin/env python3
"""HBM bytes per launch of the fused kernel from rocprofv3 --pmc passes -> profiles/traffic.json.

    python scripts/traffic.py <pmc-out-dir> [B P n m K]

<pmc-out-dir> holds the FETCH_SIZE and WRITE_SIZE passes of scripts/pmc.sh (separate runs,
pmc_counter_collection.csv each). Units and gfx950 corrections per MI355X_MICROARCH.md §HBM:
both counters are in KiB; FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads
(every global read of the fused kernel is a 16-B buffer_load), so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "fused_forward_kernel"


def per_launch(pmc_dir, counter):
    vals = []
    for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    pmc_dir = sys.argv[1]
    B, P, n, m, K = (int(x) for x in (sys.argv[2:7] if len(sys.argv) > 6 else (4096, 5, 256, 64, 25)))
    fetch_kib, nf = per_launch(pmc_dir, "FETCH_SIZE")
    write_kib, nw = per_launch(pmc_dir, "WRITE_SIZE")
    if fetch_kib is None or write_kib is None:
        sys.exit(f"no {KERNEL} FETCH_SIZE/WRITE_SIZE rows under {pmc_dir}")
    read_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tr = json.load(open(path)) if os.path.exists(path) else {}
    tr[f"B{B}_P{P}_n{n}_m{m}_K{K}"] = {
        "kernel": KERNEL, "launches": min(nf, nw),
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "correction": "read = 2 x FETCH_SIZE (gfx950, 16-B/lane loads); write = WRITE_SIZE; KiB",
        "source": os.path.relpath(pmc_dir, ROOT),
    }
    json.dump(tr, open(path, "w"), indent=1)
    print(json.dumps(tr, indent=1))


if __name__ == "__main__":
    main()
