"""Summarise a rocprofv3 kernel-trace CSV: per (kernel, grid) median/min duration and inter-kernel gaps."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else "sfx"
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if flt not in n:
        continue
    key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["VGPR_Count"], r["LDS_Block_Size"])
    d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v.sort()
    print(k, len(v), "median %.2f us" % (v[len(v) // 2] / 1e3), "min %.2f" % (v[0] / 1e3))
sf = sorted((r for r in rows if flt in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
gaps = sorted(int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(sf, sf[1:]))
gaps = [g for g in gaps if 0 <= g < 100000]
if gaps:
    print("gap median %.2f us  p10 %.2f  p90 %.2f" % (gaps[len(gaps) // 2] / 1e3, gaps[len(gaps) // 10] / 1e3,
                                                     gaps[9 * len(gaps) // 10] / 1e3))
