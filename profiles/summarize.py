#!/usr/bin/env python3
"""Summarize a profiles/profile.sh output directory: per-kernel average
duration (kernel trace) and per-launch PMC counter averages, and the L2
memory-side bytes per launch.

Read bytes come from the size-split request counters when that pass exists:
32 x TCC_EA0_RDREQ_32B + 64 x TCC_EA0_RDREQ_64B + 128 x TCC_EA0_RDREQ_128B.
rocprofv3's FETCH_SIZE on gfx950 counts every non-32-B request as 64 B (its
128-B term reads TCC_BUBBLE, which stays 0 here), hence MI355X_MICROARCH.md
§HBM's "x2" for wide streaming reads, which are all 128-B requests; the
request kernel's loads mix 64-B and 128-B requests, so neither x1 nor x2 is
right for it (profiles/r02ac: calibration kernels and the request kernel).
Without that pass the FETCH_SIZE x 2 upper bound is used.  WRITE_SIZE as read;
effective clock GRBM_GUI_ACTIVE / 8 / time."""
import collections
import csv
import json
import os
import sys


def short(name):
    for k in ("clock_probe_kernel", "sha256_msgs_overlap_kernel", "sha256_msgs_cu_kernel", "sha256_msgs_kernel",
              "sha256_lists_kernel", "sha256_chain_kernel",
              "sha256_chain_pair_kernel", "sha256_fused_paced_kernel",
              "gen_requests_kernel", "gen_mixed_kernel"):
        if k in name:
            return k
    return None


def main(d):
    out = {"kernels": {}}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        if k:
            out["kernels"].setdefault(k, {})["avg_ns"] = float(r["AverageNs"])
            out["kernels"][k]["calls"] = int(r["Calls"])
    # Per launch shape from the kernel trace: the bench's own launches (full
    # config grid) apart from the pipelined host calls' chunk launches.
    tr = os.path.join(d, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            k = short(r["Kernel_Name"])
            if k:
                by[(k, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for (k, g), v in by.items():
            v.sort()
            out["kernels"].setdefault(k, {}).setdefault("by_grid", {})[str(g)] = {
                "launches": len(v), "mean_us": sum(v) / len(v), "median_us": v[len(v) // 2]}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_mem", "pmc_size"):
        f = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in agg.items():
            out["kernels"].setdefault(k, {})[c] = sum(v) / len(v)
    for k, v in out["kernels"].items():
        t = v.get("avg_ns")
        sized = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
        if all(c in v for c in sized):
            v["hbm_read_bytes_sized"] = 32 * v[sized[0]] + 64 * v[sized[1]] + 128 * v[sized[2]]
        if "FETCH_SIZE" in v:
            v["hbm_read_bytes_upper"] = v["FETCH_SIZE"] * 1024 * 2  # KB units, every request taken as 128 B
        if "WRITE_SIZE" in v:
            v["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
        rd = v.get("hbm_read_bytes_sized", v.get("hbm_read_bytes_upper"))
        if rd is not None and "WRITE_SIZE" in v:
            v["hbm_bytes_per_launch"] = rd + v["hbm_write_bytes"]
            v["hbm_read_method"] = "sized requests" if "hbm_read_bytes_sized" in v else "FETCH_SIZE x 2 (upper bound)"
        if t and "GRBM_GUI_ACTIVE" in v:
            v["effective_clock_ghz"] = v["GRBM_GUI_ACTIVE"] / 8 / t
        if "SQ_WAVE_CYCLES" in v:
            wc = v["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in v:
                    v[c + "_frac"] = v[c] / wc
        if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v:
            v["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
