#!/usr/bin/env python3
"""Per-launch HBM traffic of the bench's dominant kernel from a rocprofv3 --pmc FETCH_SIZE pass.

Run on the GPU box (tools/gpu_round.sh step `pmc`):
  cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- python bench.py ...
then:  python tools/pmc_traffic.py <dir> <kernel-substring> <workload> <out.json> [products]

FETCH_SIZE is reported in KiB (rocprofv3 derived counter: TCC_EA0_RDREQ x 64 B / 1024); on gfx950
it counts exactly half of the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM
section), so bytes = FETCH_SIZE x 1024 x 2.  The average over the kernel's dispatches is written
as `fetch_bytes_per_launch`; bench.py reads it into roofline.traffic.  `products` (default 1) is
the number of (1 x M) x (N x K) products one profiled launch computes (the bench ring for a batched
launch): bench.py scales the pass per product to a line whose launches are another size."""
import csv
import glob
import json
import os
import sys


def main():
    d, sub, workload, out = sys.argv[1:5]
    products = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub in r.get("Kernel_Name", "") and r.get("Counter_Name") == "FETCH_SIZE":
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no FETCH_SIZE rows for kernels matching {sub!r}")
    vals.sort()
    med = vals[len(vals) // 2]
    mean = sum(vals) / len(vals)
    res = {"workload": workload, "kernel_match": sub, "dispatches": len(vals),
           "fetch_size_kib_median": med, "fetch_size_kib_mean": mean,
           "fetch_bytes_per_launch": mean * 1024 * 2, "products_per_launch": products,
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 counts half of wide streaming reads)",
           "source": "rocprofv3 --pmc FETCH_SIZE, separate pass"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
