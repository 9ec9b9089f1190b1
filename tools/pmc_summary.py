#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh output) per kernel.

usage: tools/pmc_summary.py gpurun_out/<TAG> [--out profiles/<name>.md] [--traffic profiles/traffic.json
                            --config c3 --bench-log gpurun_out/<TAG>/pass1.log]

--traffic merges this run's per-kernel bytes and isolated durations into the file's "configs"[<config>]
entry (the other configurations' entries are kept), which bench.py reads for the `isolated` figures.

Counter values are summed over every dispatch of a kernel; SQ counters on gfx950 are
summed over the shader engines.  FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM
section: gfx950 reports half the bytes of a wide coalesced read); both sizes are in KiB.
"""
import argparse
import collections
import csv
import glob
import json
import os

# r06: k_trace<LST, REF, PH>: PH 3 the merged trace launch (the extension rays, then the previous iteration's
# shadow rays), 1 / 2 the separate extension / shadow launches (rt_scene_config::shadow_launch)
KERNELS = ["k_generate", "k_trace", "k_trace_ext", "k_trace_shadow", "k_shade", "k_splat", "k_resolve_tiles",
           "k_resolve", "k_combine_partials", "k_bookkeep", "k_drain_list", "k_drain"]
LABEL = {"k_trace": "k_trace (merged: extension + shadow rays)", "k_trace_ext": "k_trace_ext (extension rays)",
         "k_trace_shadow": "k_trace_shadow (shadow rays)"}
KEYS = {}


def short(name):
    if "k_trace<" in name:                      # by the phases argument: void k_trace<true, false, 3>(...)
        ph = name.split("k_trace<")[1].split(">")[0].split(",")[-1].strip()
        return {"1": "k_trace_ext", "2": "k_trace_shadow"}.get(ph, "k_trace")
    # longest names first: k_resolve_tiles before k_resolve, k_drain_list before k_drain
    for k in sorted(KERNELS, key=len, reverse=True):
        if k in name:
            return k
    return None


def load(tag_dir):
    val = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(tag_dir, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k:
                continue
            key = (f, r["Dispatch_Id"])
            val[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(key)
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    return val, disp, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag_dir")
    ap.add_argument("--out")
    ap.add_argument("--traffic")
    ap.add_argument("--bench-log")
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    val, disp, dur = load(a.tag_dir)
    lines = [f"# PMC summary: {a.tag_dir}", "",
             "Per kernel, summed over dispatches (each pass is a separate bench run; dispatch counts per pass are equal).",
             "", "| kernel | dispatches/pass | mean us | waves/launch | VALU util | wait (s_waitcnt) | issue-stall |"
             " VALU inst/wave | SALU inst/wave | VMEM inst/wave | VMEM level/inst | LDS bank-conflict | L2 hit |"
             " L1->L2 req/access | clock GHz | HBM rd MB/launch | HBM wr MB/launch |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    out = {}
    npass = max(1, len(glob.glob(os.path.join(a.tag_dir, "pass*", ""))))
    for k in KERNELS:
        if k not in val:
            continue
        v = val[k]
        n = len(disp[k]) / npass
        g = lambda c: v.get(c, float("nan"))
        wc = g("SQ_WAVE_CYCLES")
        valu = g("SQ_ACTIVE_INST_VALU") / wc if wc else float("nan")
        wait = g("SQ_WAIT_ANY") / wc if wc else float("nan")
        stall = g("SQ_WAIT_INST_ANY") / wc if wc else float("nan")
        waves = g("SQ_WAVES")
        per_wave = lambda c: g(c) / waves if waves else float("nan")
        # SQ_INST_LEVEL_VMEM accumulates the VMEM instructions in flight per (quad-)cycle, so its ratio
        # to SQ_INSTS_VMEM is a Little's-law latency in those units (uncalibrated on gfx950; compare
        # kernels, not absolutes).  SQ_ACCUM_PREV_HIRES reads 0 on gfx950 / ROCm 7.2.
        lat = g("SQ_INST_LEVEL_VMEM") / g("SQ_INSTS_VMEM") if g("SQ_INSTS_VMEM") else float("nan")
        ldsc = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE") if g("SQ_LDS_IDX_ACTIVE") else float("nan")
        hit = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")) if g("TCC_HIT_sum") == g("TCC_HIT_sum") else float("nan")
        l1 = g("TCP_TCC_READ_REQ_sum") / g("TCP_TOTAL_CACHE_ACCESSES_sum") if g("TCP_TOTAL_CACHE_ACCESSES_sum") else float("nan")
        rd = 2.0 * g("FETCH_SIZE") * 1024 / n / 1e6
        wr = g("WRITE_SIZE") * 1024 / n / 1e6
        mean_us = sum(dur[k].values()) / max(1, len(dur[k]))
        # effective clock: GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS)
        clk = g("GRBM_GUI_ACTIVE") / 8.0 / n / (mean_us * 1e3) if mean_us and n else float("nan")
        out[k] = {"dispatches": n, "mean_us": mean_us, "waves_per_launch": waves / n if n else float("nan"),
                  "valu_util": valu, "wait_frac": wait, "issue_stall_frac": stall,
                  "valu_inst_per_wave": per_wave("SQ_INSTS_VALU"), "salu_inst_per_wave": per_wave("SQ_INSTS_SALU"),
                  "vmem_inst_per_wave": per_wave("SQ_INSTS_VMEM"), "vmem_level_per_inst": lat,
                  "lds_bank_conflict_frac": ldsc, "clock_ghz": clk, "l2_hit": hit, "l1_miss_req_per_access": l1,
                  "hbm_read_mb_per_launch": rd, "hbm_write_mb_per_launch": wr}
        e = out[k]
        lines.append(f"| {LABEL.get(k, k)} | {n:.0f} | {mean_us:.1f} | {e['waves_per_launch']:.0f} | {valu:.3f} | {wait:.3f} | "
                     f"{stall:.3f} | {e['valu_inst_per_wave']:.0f} | {e['salu_inst_per_wave']:.0f} | "
                     f"{e['vmem_inst_per_wave']:.1f} | {lat:.1f} | {ldsc:.4f} | {hit:.3f} | {l1:.3f} | {clk:.2f} | "
                     f"{rd:.1f} | {wr:.1f} |")
    lines += ["", "VALU util = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (per wave); wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES;",
              "issue-stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES; inst/wave = SQ_INSTS_* / SQ_WAVES;",
              "VMEM level/inst = SQ_INST_LEVEL_VMEM / SQ_INSTS_VMEM (Little's-law latency, uncalibrated units);",
              "LDS bank-conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS);",
              "L1->L2 = TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES; clock = GRBM_GUI_ACTIVE / 8 / duration;",
              "kernels run serialized under --pmc, so durations are isolated launch times.",
              "HBM rd = 2 x FETCH_SIZE (gfx950 correction), wr = WRITE_SIZE, per launch."]
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        open(a.out, "w").write(text)
        json.dump(out, open(os.path.splitext(a.out)[0] + ".json", "w"), indent=1)
    if a.traffic and out:
        rec = {"source": a.tag_dir,
               "note": "HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 --pmc, kernels serialized), "
                       "plus the serialized mean launch duration",
               "kernels": {KEYS.get(k, k): {"hbm_bytes_per_launch": (e["hbm_read_mb_per_launch"] + e["hbm_write_mb_per_launch"]) * 1e6,
                                            "isolated_mean_us": e["mean_us"], "dispatches": e["dispatches"]}
                           for k, e in out.items()}}
        if a.bench_log and os.path.exists(a.bench_log):
            for line in open(a.bench_log):
                if line.startswith("{"):
                    b = json.loads(line)
                    if b.get("c4"):
                        raise SystemExit("the PMC bench run also rendered C4 frames (--c4-steps 0 needed): "
                                         "its dispatch counts mix two configurations")
                    rec["bench_spp"] = b["config"].get("spp")
                    # frames the PMC pass rendered, and rank 0's units per frame per kernel: bench.py
                    # normalizes the counters per frame (pmc_figures) and uses them for frames of this size
                    rec["frames_per_pass"] = b["steps"] + b["warmup"]
                    rec["units_per_frame"] = b.get("units_per_frame")
                    # the units per launch of the dominant kernel in that run: bench.py uses the isolated
                    # time only for launches of the same size
                    rf = b.get("roofline") or {}
                    if rf.get("kernel") in rec["kernels"]:
                        rec["kernels"][rf["kernel"]]["units_per_launch"] = rf.get("units_per_launch")
        try:
            allrec = json.load(open(a.traffic))
        except (OSError, ValueError):
            allrec = {}
        if "configs" not in allrec:
            allrec = {"note": "per configuration: HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE and the serialized "
                              "mean launch duration (rocprofv3 --pmc, kernels serialized); tools/pmc_summary.py --traffic",
                      "configs": {}}
        allrec["configs"][a.config] = rec
        json.dump(allrec, open(a.traffic, "w"), indent=1)
        print("wrote", a.traffic, "configs", sorted(allrec["configs"]))


if __name__ == "__main__":
    main()
