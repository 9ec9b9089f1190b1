#!/usr/bin/env python3
"""Kernels in flight over one frame, from a rocprofv3 --kernel-trace CSV.

usage: tools/timeline.py gpurun_out/prof_<TAG>/run_kernel_trace.csv [--bucket-ms 5]

Takes the bench's second frame (a frame ends with k_combine_partials, the streaming splat's last
launch; the frame layout, k_pixel_map included, is built once per scene), prints the mean number
of kernels in flight per bucket, the time per kernel, per-partition iteration counts (one k_bookkeep
per iteration) and where the last resolve runs.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bucket-ms", type=float, default=5.0)
    ap.add_argument("--gap-us", type=float, default=150.0)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r["Kernel_Name"].startswith(("k_", "void k_"))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_combine_partials" in r["Kernel_Name"]]
    if len(ends) < 2:
        raise SystemExit("need two frames (two k_combine_partials launches) in the trace")
    fr = rows[ends[0] + 1:ends[1] + 1]
    t0 = min(int(r["Start_Timestamp"]) for r in fr)
    t1 = max(int(r["End_Timestamp"]) for r in fr)
    bucket = int(a.bucket_ms * 1e6)
    busy = [0.0] * ((t1 - t0) // bucket + 1)
    for r in fr:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        b = s // bucket
        while s < e:
            be = min(e, (b + 1) * bucket)
            busy[b] += be - s
            s, b = be, b + 1
    print(f"frame {(t1 - t0) / 1e6:.1f} ms; kernels in flight per {a.bucket_ms:g} ms:")
    print(" ".join(f"{x / bucket:.1f}" for x in busy))
    per = {}
    for r in fr:
        n = short(r)
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c, tot = per.get(n, (0, 0.0))
        per[n] = (c + 1, tot + d)
    for n, (c, tot) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {n:28s} {c:5d} launches {tot:8.1f} ms ({tot / c * 1e3:8.1f} us each)")
    res = [r for r in fr if "k_resolve" in r["Kernel_Name"]]
    if res:
        r = res[-1]
        print(f"last resolve {(int(r['Start_Timestamp']) - t0) / 1e6:.1f} -> {(int(r['End_Timestamp']) - t0) / 1e6:.1f} ms")
    # per queue (a partition's stream): idle gaps longer than --gap-us between one kernel's end and the
    # next one's start, with the kernels on either side
    qcol = next((c for c in ("Queue_Id", "Queue_ID", "Stream_Id") if c in fr[0]), None)
    if qcol:
        byq = {}
        for r in fr:
            byq.setdefault(r[qcol], []).append(r)
        for q, rs in sorted(byq.items()):
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            gaps = []
            end = int(rs[0]["End_Timestamp"])
            for prev, r in zip(rs, rs[1:]):
                s = int(r["Start_Timestamp"])
                if s - end > a.gap_us * 1e3:
                    gaps.append(f"{(end - t0) / 1e6:.2f}->{(s - t0) / 1e6:.2f} ({(s - end) / 1e3:.0f} us, "
                                f"{short(prev)} -> {short(r)})")
                end = max(end, int(r["End_Timestamp"]))
            print(f"queue {q}: {len(rs)} kernels, {(int(rs[0]['Start_Timestamp']) - t0) / 1e6:.2f}-"
                  f"{(end - t0) / 1e6:.2f} ms, idle gaps: " + ("; ".join(gaps) or "none"))


def short(r):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "k_trace<" in n:           # k_trace<LST, REF, PH>: PH 3 merged, 1 extension, 2 shadow (rt_scene_config::shadow_launch)
        return {"1": "k_trace_ext", "2": "k_trace_shadow"}.get(n.split("<")[1].rstrip(">").split(",")[-1].strip(), "k_trace")
    return n.split("<")[0]

if __name__ == "__main__":
    main()
