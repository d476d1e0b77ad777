#!/usr/bin/env python3
"""Per-stream idle gaps from a rocprofv3 kernel trace (CSV): for every stream (or queue), the gaps between one
kernel's end and the next kernel's start on that stream, their distribution, and the longest ones with what the
OTHER streams ran meanwhile. Used on tests/arena_trim_worker.py (two engines, a small arena budget that forces
trims) to check that one engine's stream never waits on the other engine's trim.

    python tools/stream_gaps.py <run_kernel_trace.csv> [--top 5] [--min-kernels 20]
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--min-kernels", type=int, default=20, help="ignore streams with fewer kernels")
    ap.add_argument("--trims", help="JX_ARENA_TRIM_LOG file: mark the gaps that overlap an arena trim")
    a = ap.parse_args()
    by = collections.defaultdict(list)
    allk = []
    for r in csv.DictReader(open(a.csv)):
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        by[q].append((s, e, n))
        allk.append((s, e, n, q))
    allk.sort()
    trims = []
    clock = None
    started = collections.Counter()
    if a.trims:
        rows = [ln.split() for ln in open(a.trims) if ln.strip()]
        t_lo, t_hi = allk[0][0], max(e for _, e, _, _ in allk)
        # the trace's clock: the one with more hipFree intervals inside the traced span (the frees of the final
        # teardown come after the last kernel)
        best = 0
        for name, i0 in (("monotonic", 1), ("boottime", 4)):
            iv = [(int(r[i0]), int(r[i0 + 1])) for r in rows]
            inside = [(s0, e0) for s0, e0 in iv if t_lo <= s0 <= t_hi]
            if len(inside) > best:
                best, trims, clock = len(inside), inside, name
    # per stream: kernels started while a hipFree ran (a stream that keeps launching was not held up by it)
    started = collections.Counter(q for s, _, _, q in allk if any(t0 <= s <= t1 for t0, t1 in trims))
    out = {"streams": {}, "trims": len(trims), "trim_clock": clock,
           "trim_ms_total": round(sum(e - s for s, e in trims) / 1e6, 3)}
    for q, ks in sorted(by.items()):
        if len(ks) < a.min_kernels:
            continue
        ks.sort()
        gaps = []
        for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
            if s1 > e0:
                gaps.append((s1 - e0, e0, s1, n0, n1))
        gaps.sort(reverse=True)
        top = []
        for g, t0, t1, n0, n1 in gaps[:a.top]:
            other = sorted({n for s, e, n, qq in allk if qq != q and s < t1 and e > t0})
            ov = [(s, e) for s, e in trims if s < t1 and e > t0]
            top.append({"gap_ms": round(g / 1e6, 3), "after": n0, "before": n1, "other_streams_ran": other[:6],
                        "overlapping_trims_ms": [round((min(e, t1) - max(s, t0)) / 1e6, 3) for s, e in ov]})
        out["streams"][q] = {"kernels": len(ks), "gaps": len(gaps),
                             "gap_p50_ms": round(gaps[len(gaps) // 2][0] / 1e6, 4) if gaps else 0,
                             "gaps_over_1ms": sum(1 for g in gaps if g[0] > 1_000_000),
                             "gaps_over_1ms_overlapping_a_trim": sum(
                                 1 for g in gaps if g[0] > 1_000_000 and any(s < g[2] and e > g[1] for s, e in trims)),
                             "kernels_started_during_a_free": started.get(q, 0),
                             "max_gap_ms": round(gaps[0][0] / 1e6, 3) if gaps else 0, "longest": top}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
