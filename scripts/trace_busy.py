"""GPU occupancy of a kernel trace (rocprofv3 --kernel-trace CSV): over the last W milliseconds
of the trace (the timed steps), the time some kernel was running (union of intervals), the sum
of kernel durations (their overlap factor = sum / union) and the idle gaps, per kernel name too.
usage: python scripts/trace_busy.py run_kernel_trace.csv [window_ms]"""
import collections
import csv
import re
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].split()[-1].replace("msg::", ""))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Queue_Id"]))
    rows.sort()
    end = max(e for _, e, _, _ in rows)
    win = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else None
    t0 = end - win if win else rows[0][0]
    rows = [(max(s, t0), e, k, q) for s, e, k, q in rows if e > t0]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _, _ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = end - t0
    tot = sum(e - s for s, e, _, _ in rows)
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, k, _ in rows:
        per[k][0] += 1
        per[k][1] += e - s
    print("window %.3f ms: busy %.3f ms (%.1f%%), kernel time %.3f ms (overlap %.2fx), %d gaps, largest %.1f us,"
          " gaps > 5 us total %.3f ms, queues %d" % (
              span / 1e6, busy / 1e6, 100.0 * busy / span, tot / 1e6, tot / max(busy, 1), len(gaps),
              max(gaps or [0]) / 1e3, sum(g for g in gaps if g > 5000) / 1e6, len({q for *_, q in rows})))
    for k, (n, t) in sorted(per.items(), key=lambda x: -x[1][1])[:10]:
        print("  %-28s %6d launches %9.3f ms  %7.2f us avg" % (k, n, t / 1e6, t / 1e3 / n))


if __name__ == "__main__":
    main()
