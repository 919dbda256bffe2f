#!/usr/bin/env python3
"""Summarize bench.py JSON lines (A/B runs): value, step, dominant-kernel time,
frac, clock, probe ceiling.  Usage: abview.py file.jsonl ..."""
import json
import sys

for f in sys.argv[1:]:
    for ln in open(f):
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        d = json.loads(ln)
        r = d["roofline"]
        m = r.get("measured_peak") or {}
        print(f"{f:34s} {d['value'] / 1e9:7.3f}G {d['ms_per_step']:.4f}ms kern={r['avg_launch_ms'] * 1e3:7.1f}us "
              f"frac={r['frac']:.3f} clk={d.get('effective_clock_ghz') or 0:.3f} "
              f"probe_cyc={m.get('cycles_per_wave_compression', 0):.0f} meas_frac={m.get('frac', 0):.3f} "
              f"batch={d.get('batch_kernel_avg_ms', 0) * 1e3:.1f}us")
