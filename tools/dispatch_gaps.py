#!/usr/bin/env python3
"""Gaps between back-to-back dispatches in a rocprofv3 kernel trace.

For every dispatch of a kernel matching REGEX that directly follows another
such dispatch on the same queue, prints the distribution of (start - previous
end) and of the durations, and lists any other kernels that ran in between.

Usage: dispatch_gaps.py <kernel_trace.csv | rocprofv3 output dir> [REGEX]"""
import csv
import glob
import os
import re
import sys

import numpy as np


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else "sha256")
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    gaps, durs, between = [], [], {}
    prev = None  # the previous matching dispatch
    others = []
    for s, e, name, q in rows:
        if rx.search(name):
            if prev is not None and prev[3] == q:
                gaps.append(s - prev[1])
                durs.append(e - s)
                for o in others:
                    between[o] = between.get(o, 0) + 1
            prev = (s, e, name, q)
            others = []
        else:
            others.append(name.split("(")[0][:80])
    if not gaps:
        print("no back-to-back dispatches of", rx.pattern)
        return
    g = np.array(gaps) / 1e3
    d = np.array(durs) / 1e3
    pct = [10, 50, 90]
    print(f"{len(g)} back-to-back dispatches of /{rx.pattern}/")
    print("gap us p10/50/90:", [round(float(x), 2) for x in np.percentile(g, pct)], "min", round(float(g.min()), 2))
    print("duration us p10/50/90:", [round(float(x), 1) for x in np.percentile(d, pct)])
    print("kernels in between:", between or "none")


if __name__ == "__main__":
    main()
