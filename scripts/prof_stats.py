"""Per-kernel statistics (calls, total/avg duration) from a rocprofv3 run.

    python scripts/prof_stats.py <rocpd .db | kernel_stats.csv> [out.csv]

rocprofv3 7.x writes a rocpd SQLite database by default; this reduces its kernel dispatch table to the
same columns as `--stats` (name, calls, total_us, avg_us, percent)."""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end - start) from kernels group by name").fetchall()
    return [(n, k, t / 1e3) for n, k, t in rows]


def main():
    src = sys.argv[1]
    rows = from_db(src)
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows) or 1.0
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["name", "calls", "total_us", "avg_us", "percent"])
    for n, k, t in rows:
        w.writerow([n, k, round(t, 3), round(t / k, 3), 100.0 * t / tot])


if __name__ == "__main__":
    main()
