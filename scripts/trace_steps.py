"""Per-flood busy / idle split of a rocprofv3 kernel trace (CSV): every flood starts at a k_prep
launch; for floods first..first+n-1 (bench.py's timed steps: after the warm-up floods) the time from
its k_prep start to the next flood's, the union of its kernels' intervals, and its idle gaps by size.
usage: python scripts/trace_steps.py run_kernel_trace.csv [first=3] [n=10]"""
import csv
import re
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].split()[-1].replace("msg::", ""))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    starts = [i for i, r in enumerate(rows) if r[2].startswith("k_prep")]
    tot_span = tot_busy = 0
    hist = {}
    for f in range(first, min(first + n, len(starts) - 1)):
        seg = rows[starts[f]:starts[f + 1]]
        span = seg[-1][1] - seg[0][0]
        busy, cs, ce = 0, None, None
        for s, e, _ in seg:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                    g = s - ce
                    b = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">20us"
                    hist.setdefault(b, [0, 0])
                    hist[b][0] += 1
                    hist[b][1] += g
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        # the gap to the next flood's k_prep (host: flood_end sync, Python, flood_begin)
        inter = rows[starts[f + 1]][0] - seg[-1][1]
        print("flood %d: %d kernels, span %.3f ms, busy %.3f ms, to next flood %.1f us" % (
            f, len(seg), span / 1e6, busy / 1e6, inter / 1e3))
        tot_span += span + inter
        tot_busy += busy
    print("total %.3f ms, busy %.3f ms (%.1f%%)" % (tot_span / 1e6, tot_busy / 1e6, 100.0 * tot_busy / max(tot_span, 1)))
    for b, (c, t) in sorted(hist.items()):
        print("  gaps %-6s %6d  %.3f ms" % (b, c, t / 1e6))


if __name__ == "__main__":
    main()
