#!/usr/bin/env python3
"""Per-partition iteration timeline of one frame, from a rocprofv3 --kernel-trace CSV.

usage: tools/drain.py gpurun_out/<dir>/run_kernel_trace.csv [--frame 1]

A partition is one HIP stream (the trace's Stream_Id, or Queue_Id when the stream column is
absent).  An iteration is generate -> extend -> shade -> connect -> bookkeep (+ resolve); the
script prints, per partition, each iteration's start and length and its kernels' durations, so
the frame's ramp, steady state and drain (the iterations in which the last paths finish, and the
empty iterations enqueued before the host sees a partition is done) can be read off.
"""
import argparse
import csv

SHORT = {"k_generate": "gen", "k_trace<false>": "ext", "k_shade": "shd", "k_trace<true>": "con",
         "k_bookkeep": "bk", "k_resolve_tiles": "res", "k_combine_partials": "comb", "k_pixel_map": "map",
         "k_drain_list": "dl", "k_drain": "drn"}


def kname(n):
    n = n.split("(")[0].replace("void ", "")
    if "k_trace" in n:
        return "k_trace<" + n.split("<")[1].split(",")[0] + ">"
    return n.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frame", type=int, default=1, help="which frame (0 = the first, warm-up)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r["Kernel_Name"].startswith(("k_", "void k_"))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "k_combine_partials" in r["Kernel_Name"]]
    lo = ends[a.frame - 1] + 1 if a.frame > 0 else 0
    fr = rows[lo:ends[a.frame] + 1]
    key = "Stream_Id" if "Stream_Id" in fr[0] else "Queue_Id"
    t0 = min(int(r["Start_Timestamp"]) for r in fr)
    t1 = max(int(r["End_Timestamp"]) for r in fr)
    print(f"frame {(t1 - t0) / 1e6:.2f} ms, {len(fr)} launches, partitions by {key}")
    parts = {}
    for r in fr:
        parts.setdefault(r[key], []).append(r)
    for pid, rs in sorted(parts.items(), key=lambda x: int(x[1][0]["Start_Timestamp"])):
        its, cur = [], None
        for r in rs:
            n = SHORT.get(kname(r["Kernel_Name"]), kname(r["Kernel_Name"]))
            if n == "gen" or cur is None:
                cur = []
                its.append(cur)
            cur.append((n, int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0))
        busy = sum(e - s for it in its for _, s, e in it)
        last = max(e for it in its for _, s, e in it)
        print(f"\npartition {key}={pid}: {len(its)} iterations, kernel time {busy / 1e6:.2f} ms, "
              f"ends at {last / 1e6:.2f} ms")
        print("  it  start_ms  len_ms  gap_ms | " + " ".join(f"{k:>6s}" for k in ("gen", "dl", "drn", "ext", "shd", "con", "bk", "res")))
        for i, it in enumerate(its):
            s = it[0][1]
            e = max(x[2] for x in it)
            gap = sum(max(0, it[j][1] - it[j - 1][2]) for j in range(1, len(it)))
            d = {}
            for n, ss, ee in it:
                d[n] = d.get(n, 0) + (ee - ss)
            cols = " ".join(f"{d[k] / 1e3:6.0f}" if k in d else "     -" for k in ("gen", "dl", "drn", "ext", "shd", "con", "bk", "res"))
            print(f"  {i:3d} {s / 1e6:8.2f} {(e - s) / 1e6:7.3f} {gap / 1e6:7.3f} | {cols}")


if __name__ == "__main__":
    main()
