"""Print the key fields of bench.py's JSON line(s) from a log.  usage: python scripts/bench_summary.py <bench.log>"""
import json
import sys


def main():
    for ln in open(sys.argv[1]):
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        out = {"value": d.get("value"), "ms_per_step": d.get("ms_per_step")}
        rf = d.get("roofline") or {}
        out["roofline.frac"] = rf.get("frac")
        for k in ("batch", "batch_hwq4", "stress", "stress_random"):
            v = d.get(k)
            if isinstance(v, dict):
                out[k] = {kk: v.get(kk) for kk in ("value", "inflight", "alt_high", "executions_per_pop", "flood") if kk in v}
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
