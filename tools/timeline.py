#!/usr/bin/env python3
"""Kernels in flight over one frame, from a rocprofv3 --kernel-trace CSV.

usage: tools/timeline.py gpurun_out/prof_<TAG>/run_kernel_trace.csv [--bucket-ms 5]

Takes the frame between the first two k_resolve launches (the bench's second frame),
prints the mean number of kernels in flight per bucket and where the resolve starts.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bucket-ms", type=float, default=5.0)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if r["Kernel_Name"].startswith(("k_", "void k_"))]
    ri = [i for i, r in enumerate(rows) if "k_resolve" in r["Kernel_Name"]]
    if len(ri) < 2:
        raise SystemExit("need two frames (two k_resolve launches) in the trace")
    fr = rows[ri[0] + 1:ri[1] + 1]
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
    res = next(r for r in fr if "k_resolve" in r["Kernel_Name"])
    print(f"resolve {(int(res['Start_Timestamp']) - t0) / 1e6:.1f} -> {(int(res['End_Timestamp']) - t0) / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
