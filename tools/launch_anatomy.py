#!/usr/bin/env python3
"""Anatomy of coalesced launches from a rocprofv3 kernel trace (+ optional memory-copy trace) of the jobs driver:
for every launch on a lane stream (K1 ... scatter_jobs_kernel, then its downloads), the device-side phases

    upload  = first H2D copy of the launch -> K1 start  (uploads, waits, queueing)
    k1      = K1 duration (xof_* kernels of the launch)
    tail    = K1 end -> scatter end  (K3, FLP final, scatter)
    down    = scatter end -> last D2H copy end
    turn    = this launch's first H2D start - the end of the most recent earlier launch's last D2H
              (host: callers wake, copy out, accumulate, come back, copy in; the gather closes)

and the device idle time between kernels. Used to find where a closed-loop job's round trip goes.

    python tools/launch_anatomy.py <run_kernel_trace.csv> [--copies <run_memory_copy_trace.csv>]
"""
import argparse
import csv
import json
import statistics


def pct(xs, p):
    if not xs:
        return None
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(p * len(xs)))] / 1e6, 4)


def summ(xs):
    return {"n": len(xs), "mean_ms": round(statistics.fmean(xs) / 1e6, 4) if xs else None, "p50_ms": pct(xs, 0.5),
            "p90_ms": pct(xs, 0.9)}


def stream_of(r):
    for k in ("Stream_Id", "Queue_Id"):
        if r.get(k) not in (None, ""):
            return r[k]
    return "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("--copies")
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.kernels)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, stream_of(r)))
    ks.sort()
    cps = []
    if a.copies:
        for r in csv.DictReader(open(a.copies)):
            d = (r.get("Direction") or r.get("Operation") or "").upper()
            kind = "H2D" if "HOST_TO_DEVICE" in d or "H2D" in d else ("D2H" if "DEVICE_TO_HOST" in d or "D2H" in d else d)
            cps.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, stream_of(r), int(r.get("Size") or 0)))
        cps.sort()
    # launches: per stream, a K1 (jx::xof*) opens one, the scatter kernel closes its kernels
    launches = []
    open_l = {}
    for s, e, n, q in ks:
        if n.startswith("jx::xof") and "slow" not in n:
            cur = open_l.get(q)
            if cur is None or cur.get("scatter_end"):
                cur = {"stream": q, "k1_start": s, "k1_end": e, "kernels": [n]}
                open_l[q] = cur
                launches.append(cur)
            else:  # a second K1 part of the same launch (lane split + pairs)
                cur["k1_start"] = min(cur["k1_start"], s)
                cur["k1_end"] = max(cur["k1_end"], e)
                cur["kernels"].append(n)
        elif n.startswith("jx::scatter_jobs"):
            cur = open_l.get(q)
            if cur is not None and not cur.get("scatter_end"):
                cur["scatter_end"] = e
    launches = [L for L in launches if L.get("scatter_end")]
    launches.sort(key=lambda L: L["k1_start"])
    out = {"launches": len(launches), "span_ms": round((ks[-1][1] - ks[0][0]) / 1e6, 3) if ks else 0}
    k1 = [L["k1_end"] - L["k1_start"] for L in launches]
    tail = [L["scatter_end"] - L["k1_end"] for L in launches]
    out["k1"] = summ(k1)
    out["tail"] = summ(tail)
    if cps:
        h2d = [c for c in cps if c[2] == "H2D"]
        d2h = [c for c in cps if c[2] == "D2H"]
        # a launch's uploads: the H2D copies after the previous launch's K1 start on its stream and before its K1
        up, down, turn = [], [], []
        ends = []
        for i, L in enumerate(launches):
            prev_same = max((M["k1_start"] for M in launches[:i] if M["stream"] == L["stream"]), default=0)
            mine = [c for c in h2d if prev_same < c[0] < L["k1_start"] and (c[3] == L["stream"] or c[3] == "?")]
            after = [c for c in d2h if c[0] >= L["scatter_end"] and (c[3] == L["stream"] or c[3] == "?")]
            L["first_h2d"] = min((c[0] for c in mine), default=None)
            L["last_d2h"] = None
            if after:
                # the launch's downloads: the D2H copies that start within 1 ms of its scatter
                near = [c for c in after if c[0] - L["scatter_end"] < 1_000_000]
                if near:
                    L["last_d2h"] = max(c[1] for c in near)
            if L["first_h2d"] is not None:
                up.append(L["k1_start"] - L["first_h2d"])
            if L["last_d2h"] is not None:
                down.append(L["last_d2h"] - L["scatter_end"])
                ends.append(L["last_d2h"])
        for L in launches:
            if L["first_h2d"] is None:
                continue
            prev = [x for x in ends if x <= L["first_h2d"]]
            if prev:
                turn.append(L["first_h2d"] - max(prev))
        out["upload"] = summ(up)
        out["down"] = summ(down)
        out["turn"] = summ(turn)
        out["h2d_bytes_per_launch"] = round(sum(c[4] for c in h2d) / max(1, len(launches)))
    # device idle: no kernel running
    pts = sorted([(s, 1) for s, _, _, _ in ks] + [(e, -1) for _, e, _, _ in ks])
    cur, last, idle, gaps = 0, pts[0][0] if pts else 0, 0, []
    for t, d in pts:
        if cur == 0 and t > last:
            idle += t - last
            gaps.append(t - last)
        cur += d
        last = t
    out["device_idle_frac"] = round(idle / max(1, ks[-1][1] - ks[0][0]), 4) if ks else None
    out["idle_gaps"] = summ(gaps)
    out["idle_gaps_over_1ms"] = sum(1 for g in gaps if g > 1_000_000)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
