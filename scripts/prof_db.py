"""Kernel statistics (and optionally the kernel trace) from a rocprofv3 results database (the rocpd SQLite output of
`rocprofv3 --kernel-trace --stats`), in the columns of rocprofv3's kernel_stats.csv.

    python scripts/prof_db.py gpurun_out/prof/bench_results.db profiles/r04_v1_kernel_stats.csv [trace.csv]
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    rows = list(con.execute("select name, start, end from kernels"))
    by = {}
    for name, s, e in rows:
        by.setdefault(name, []).append(e - s)
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        total = sum(sum(v) for v in by.values()) or 1
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
            for name, s, e in sorted(rows, key=lambda r: r[1]):
                w.writerow([name, s, e])


if __name__ == "__main__":
    main()
