"""Per-kernel summary (calls, total / average / min / max ns) of a rocprofv3 rocpd database
(ROCm 7.2 writes <name>_results.db by default), as the kernel_stats CSV of earlier rounds.

    python scripts/rocpd_stats.py gpurun_out/x/prof/run_results.db [out.csv]
"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), "
         "min(d.end - d.start), max(d.end - d.start) from rocpd_kernel_dispatch d join "
         "rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name "
         "order by sum(d.end - d.start) desc")
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, calls, total, avg, mn, mx in rows:
        w.writerow([name, calls, total, round(avg, 1), round(100.0 * total / tot, 2), mn, mx])


if __name__ == "__main__":
    main()
