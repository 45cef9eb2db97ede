#!/usr/bin/env python3
"""Per-iteration kernel durations of the last flood in a rocprofv3 kernel-trace CSV."""
import re
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "msg::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_prep" in r["Kernel_Name"]]
seg = rows[idx[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
its, cur, pre = [], None, {}
for r in seg:
    k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].split()[-1].replace("msg::", ""))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k == "k_resolve":
        cur = {"start": int(r["Start_Timestamp"])}
        its.append(cur)
    if cur is None:
        pre[k] = d
    else:
        cur[k] = cur.get(k, 0) + d
        cur["end"] = int(r["End_Timestamp"])
print("flood span us %.1f, iterations %d, before loop %s" % ((int(seg[-1]["End_Timestamp"]) - t0) / 1e3, len(its), pre))
step = int(sys.argv[2]) if len(sys.argv) > 2 else 4
for j, it in enumerate(its):
    if j % step == 0 or max(v for k, v in it.items() if k.startswith("k_")) > 100:
        print(j, {k: round(v, 1) for k, v in it.items() if k.startswith("k_")}, round((it["end"] - it["start"]) / 1e3, 1))
