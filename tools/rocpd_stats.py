#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max ns, share) from a rocprofv3 results database
(rocpd SQLite, the default output format of rocprofv3 in ROCm 7) -- the same columns as the
kernel_stats.csv that `--output-format csv --stats` writes."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        r = rows.setdefault(name, [0, 0, None, 0])
        r[0] += 1
        r[1] += dur
        r[2] = dur if r[2] is None else min(r[2], dur)
        r[3] = max(r[3], dur)
    total = sum(r[1] for r in rows.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (n, s, mn, mx) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, n, s, round(s / n, 1), round(100.0 * s / total, 3), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
