#!/usr/bin/env python3
"""Record the PMC traffic of one profiled kernel build in profiles/traffic.json,
keyed by bench.kernel_source_key(variant) (sha256 of the device sources), so
bench.py reports `roofline.traffic` only for the exact kernel it ran.

L2 memory-side bytes per launch = read bytes from the size-split request
counters (32 x TCC_EA0_RDREQ_32B + 64 x _64B + 128 x _128B; see
profiles/summarize.py: rocprofv3's FETCH_SIZE takes every request as 64 B on
gfx950) + WRITE_SIZE x 1024, averaged over every launch of the kernel in the
pass; FETCH_SIZE x 2 (upper bound) when the size pass is missing.

Usage: update_traffic.py <summary.json> --tag r02 [--config 2] [--variant 0] [--kernel sha256_msgs_kernel]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("summary")
    p.add_argument("--tag", required=True)
    p.add_argument("--config", type=int, default=2)
    p.add_argument("--variant", type=int, default=0)
    p.add_argument("--kernel", default="sha256_msgs_kernel")
    p.add_argument("--from-kernel", default=None,
                   help="summary entry to read (default --kernel); e.g. sha256_msgs_cu_kernel, the form "
                        "launch_msgs picks for 1,025-4,096 tiles, which bench.py reports as sha256_msgs_kernel")
    p.add_argument("--algorithmic", type=float, default=None, help="algorithmic bytes per launch (for the ratio)")
    a = p.parse_args()
    from bench import kernel_source_key  # noqa: E402

    k = json.load(open(a.summary))["kernels"][a.from_kernel or a.kernel]
    entry = {
        "key": kernel_source_key(a.variant), "config": a.config, "variant": a.variant, "kernel": a.kernel,
        "hbm_bytes_per_launch": k["hbm_bytes_per_launch"],
        "read_method": k.get("hbm_read_method"),
        "FETCH_SIZE_kb": k.get("FETCH_SIZE"), "WRITE_SIZE_kb": k.get("WRITE_SIZE"),
        "TCC_EA0_RDREQ_32B_sum": k.get("TCC_EA0_RDREQ_32B_sum"), "TCC_EA0_RDREQ_64B_sum": k.get("TCC_EA0_RDREQ_64B_sum"),
        "TCC_EA0_RDREQ_128B_sum": k.get("TCC_EA0_RDREQ_128B_sum"),
        "TCC_HIT_sum": k.get("TCC_HIT_sum"), "TCC_MISS_sum": k.get("TCC_MISS_sum"),
        "source": f"{a.summary} (profiles/profile.sh {a.tag})",
    }
    if a.algorithmic:
        entry["over_algorithmic"] = k["hbm_bytes_per_launch"] / a.algorithmic
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        tf = json.load(open(path))
    except (OSError, ValueError):
        tf = {}
    entries = [e for e in tf.get("entries", [])
               if not (e.get("key") == entry["key"] and e.get("config") == entry["config"]
                       and e.get("kernel") == entry["kernel"])]
    entries.append(entry)
    out = {"method": "rocprofv3 --pmc passes over bench.py (profiles/profile.sh); bytes per launch = "
                     "32*TCC_EA0_RDREQ_32B + 64*TCC_EA0_RDREQ_64B + 128*TCC_EA0_RDREQ_128B + WRITE_SIZE*1024 "
                     "(entries without read_method 'sized requests': FETCH_SIZE*1024*2 + WRITE_SIZE*1024)",
           "entries": entries}
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
