#!/usr/bin/env python3
"""HBM bytes per decode layer from a rocprofv3 --pmc FETCH_SIZE pass over bench.py's decode-layer
line (run with --no-other-mode: then every GEMV / attention dispatch of the run belongs to the
decode layers).  bytes per layer = sum over those dispatches of FETCH_SIZE x 1024 x 2 (the gfx950
correction, MI355X_MICROARCH.md HBM section) / number of attention dispatches (one per layer).
Usage: python tools/decode_traffic.py <pmc dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys

LAYER_KERNELS = ("gemv_fast_kernel", "gemv_kernel", "gemv_wrow_kernel", "gemv_rows_kernel",
                 "attn_decode_kernel")


def main():
    d, out = sys.argv[1:3]
    per = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != "FETCH_SIZE":
                continue
            name = r.get("Kernel_Name", "")
            if any(k in name for k in LAYER_KERNELS):
                per[name].append(float(r["Counter_Value"]) * 1024 * 2)
    layers = sum(len(v) for k, v in per.items() if "attn_decode_kernel" in k)
    if not layers:
        raise SystemExit("no attention dispatches: not a decode-layer pass")
    total = sum(sum(v) for v in per.values())
    res = {"workload": "decode_layer_int4_g128", "layers_dispatched": layers,
           "fetch_bytes_per_launch": total / layers,
           "per_kernel_mean_bytes": {k[:120]: sum(v) / len(v) for k, v in per.items()},
           "per_kernel_dispatches": {k[:120]: len(v) for k, v in per.items()},
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 counts half of wide streaming reads)",
           "source": "rocprofv3 --pmc FETCH_SIZE, separate pass, bench.py --no-other-mode"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
