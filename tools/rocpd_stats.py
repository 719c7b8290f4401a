#!/usr/bin/env python3
"""Export rocprofv3's per-kernel summary (--stats, rocpd SQLite output) to CSV.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rNN_rocprof_kernel_stats.csv

Durations are in microseconds (rocpd `top_kernels` view: total and average per
kernel over every dispatch in the profiled command)."""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    cur = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
    for name, calls, tot, avg, pct in cur:
        w.writerow([name, calls, f"{tot:.3f}", f"{avg:.3f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main(sys.argv[1])
