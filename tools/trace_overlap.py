#!/usr/bin/env python3
"""Kernel concurrency from a rocprofv3 kernel trace (CSV): per kernel name, dispatches, mean duration, and how
many kernels of any kind were running at once on average while it ran; per queue, dispatch counts. Used to
check that coalesced launches on different lanes (streams) overlap on the device.

    python tools/trace_overlap.py <run_kernel_trace.csv> [--top 12]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        ev.append((s, e, r["Kernel_Name"].split("(")[0].replace("void ", ""), q))
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
    # running count sweep
    pts = sorted([(s, 1) for s, _, _, _ in ev] + [(e, -1) for _, e, _, _ in ev])
    busy = 0
    cur = 0
    last = t0
    hist = collections.Counter()
    for t, d in pts:
        if cur > 0:
            busy += t - last
        hist[cur] += t - last
        cur += d
        last = t
    by = collections.defaultdict(list)
    for s, e, n, q in ev:
        by[n].append((s, e, q))
    out = {"span_ms": (t1 - t0) / 1e6, "device_busy_frac": busy / max(1, t1 - t0),
           "time_at_concurrency": {k: round(v / max(1, t1 - t0), 4) for k, v in sorted(hist.items())},
           "queues": dict(collections.Counter(q for _, _, _, q in ev)), "kernels": {}}
    for n, lst in sorted(by.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1]))[:a.top]:
        dur = [e - s for s, e, _ in lst]
        out["kernels"][n] = {"dispatches": len(lst), "mean_ms": round(sum(dur) / len(dur) / 1e6, 4),
                             "total_ms": round(sum(dur) / 1e6, 2),
                             "queues": dict(collections.Counter(q for _, _, q in lst))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
