#!/usr/bin/env python3
"""Per-step kernel breakdown of a rocprofv3 --kernel-trace database (results.db) of
scripts/prof_gnn_train.py: the last complete train step (steps are delimited by the loss kernel),
its kernel count, GPU busy time and span, and the kernels grouped by (name, workgroups).
    python scripts/trace_step.py gpurun_out/<tag>/kt/run_results.db [marker | all/N]"""
import collections
import re
import sqlite3
import sys

db = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "loss::partial"
rows = sqlite3.connect(db).execute(
    "select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start").fetchall()
if marker.startswith("all"):   # "all/N": every kernel of the run, times divided by N (e.g. forwards)
    div = int(marker.split("/")[1]) if "/" in marker else 1
    step = rows
    busy = sum(r[2] - r[1] for r in step) / 1e6 / div
    print(f"whole run / {div}: {len(step) / div:.0f} kernels, GPU busy {busy:.3f} ms each (under the profiler)")
else:
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(idx) < 2:
        sys.exit(f"fewer than two '{marker}' kernels in {db}")
    step = rows[idx[-2] + 1:idx[-1] + 1]
    div = 1
    busy = sum(r[2] - r[1] for r in step) / 1e6
    span = (step[-1][2] - step[0][1]) / 1e6
    print(f"last step: {len(step)} kernels, GPU busy {busy:.3f} ms, span {span:.3f} ms (under the profiler)")
agg = collections.OrderedDict()
for r in step:
    k = (re.sub(r"\(.*", "", r[0])[:70], r[3] // max(r[5], 1), r[4])
    e = agg.setdefault(k, [0, 0.0])
    e[0] += 1
    e[1] += (r[2] - r[1]) / 1e3
for (nm, gx, gy), (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{t / div:9.1f} us {n / div:6.0f}x {t / n:7.2f} us  wg={gx}x{gy}  {nm}")
