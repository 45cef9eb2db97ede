#!/usr/bin/env python3
"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (separate passes) into per-kernel HBM bytes
per launch.  FETCH_SIZE is doubled: on gfx950 it reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM/rocprofv3 section; checked here on k_untile, whose 16-B-per-lane loads
move a known 8 B per pixel).  Random 4-B and 16-B gathers, one per distinct 128-B line, calibrated
in round 2 (scripts/exp/fetch_calib.hip): TCC_EA0_RDREQ counts one request per line (as for the
coalesced reads: one per 128-B line) and FETCH_SIZE reads 64 B per line, so the same x2 holds.

  python scripts/pmc_summary.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <out.json> [note] [bench args]

The workload of the profiled command (bench.py's defaults unless bench args are given) is stored
as "config"; bench.py quotes the traffic only for that same workload.
"""
import re
import collections
import csv
import glob
import json
import os
import sys


def load(path, counter):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].split()[-1].replace("msg::", ""))
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return {k: (tot[k], n[k]) for k in tot}


def bench_config(argv):
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--pipeline", default="watershed")
    ap.add_argument("--kind", default="mosaic")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    return {"pipeline": a.pipeline, "kind": a.kind, "size": a.size, "seed": a.seed, "frames": a.frames}


def main():
    src, out = sys.argv[1], sys.argv[2]
    fetch = load(os.path.join(src, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    write = load(os.path.join(src, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fk, fn = fetch.get(k, (0.0, 1))
        wk, wn = write.get(k, (0.0, 1))
        res[k] = {"launches": max(fn, wn),
                  "fetch_bytes_per_launch": 2.0 * 1024.0 * fk / max(fn, 1),
                  "write_bytes_per_launch": 1024.0 * wk / max(wn, 1)}
        res[k]["hbm_bytes_per_launch"] = res[k]["fetch_bytes_per_launch"] + res[k]["write_bytes_per_launch"]
    cmd = " ".join(sys.argv[4:]) or "--steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --batch-frames 1"
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) of `python bench.py %s`" % cmd,
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes", "note": sys.argv[3] if len(sys.argv) > 3 else "",
           "config": bench_config(sys.argv[4:]), "kernels": res}
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in res.items():
        print("%-12s launches %6d  fetch %10.0f  write %10.0f  B/launch" % (k, v["launches"], v["fetch_bytes_per_launch"], v["write_bytes_per_launch"]))


if __name__ == "__main__":
    main()
