"""Per-kernel averages of the counters collected by scripts/pmc_occupancy.sh.
usage: python scripts/pmc_table.py gpurun_out/<tag> [out.json]"""
import re
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].split()[-1].replace("msg::", ""))
            c = r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = {}
    for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0)):
        row = {c: tot[k][c] / max(len(disp[k][c]), 1) for c in tot[k]}
        wc = row.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in row:
                    row[c + "/WAVE_CYCLES"] = round(row[c] / wc, 3)
        h, m = row.get("TCC_HIT_sum"), row.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            row["L2_hit_rate"] = round(h / (h + m), 3)
        out[k] = {c: round(v, 3) for c, v in row.items()}
    for k, row in out.items():
        if not k.startswith("k_"):
            continue
        keys = ["SQ_WAVES", "SQ_WAIT_INST_ANY/WAVE_CYCLES", "SQ_ACTIVE_INST_ANY/WAVE_CYCLES",
                "SQ_ACTIVE_INST_VMEM/WAVE_CYCLES", "SQ_ACTIVE_INST_LDS/WAVE_CYCLES", "L2_hit_rate",
                "SQ_LEVEL_WAVES"]
        print("%-14s " % k + "  ".join("%s=%s" % (c.replace("/WAVE_CYCLES", "/wc"), row.get(c)) for c in keys))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
