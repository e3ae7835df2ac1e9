#!/usr/bin/env python3
"""Per-(kernel, grid) duration table from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    k = (r["Kernel_Name"].split("(")[0][-16:], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]),
         r.get("VGPR_Count"), r.get("LDS_Block_Size"))
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:18s} grid {k[1]:4d}x{k[2]:<3d} vgpr {k[3]:>4s} lds {k[4]:>6s}  n={len(v):5d} mean {statistics.mean(v):7.2f} med {statistics.median(v):7.2f} us")
