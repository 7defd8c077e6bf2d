#!/usr/bin/env python3
"""HBM traffic per launch of the EPnP path kernels from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC slots").

Corrections (MI355X_MICROARCH.md §HBM): both counters are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced read, so read bytes = 2 x FETCH_SIZE x 1024 (an upper estimate for
narrower accesses); WRITE_SIZE x 1024 is exact for 16-B-per-lane stores.

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv out.json [commit]"""
import csv
import json
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").strip()
        vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


fetch, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
write, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
kernels = {}
for k in sorted(set(fetch) | set(write)):
    rd = 2.0 * fetch.get(k, 0.0) * 1024.0
    wr = write.get(k, 0.0) * 1024.0
    kernels[k] = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr, "dispatches": nf.get(k, nw.get(k, 0))}
path = [k for k in kernels if k.replace("rsc::", "").startswith(("pnp_eig_group_kernel", "pnp_eig_split_kernel", "pnp_eig_quad_kernel", "pnp_betas_kernel", "pnp_scan_kernel"))]
out = {"kernels": kernels, "epnp_launch_set": path,
       "epnp_launch_set_bytes": sum(kernels[k]["bytes"] for k in path),
       "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB",
       "commit": sys.argv[4] if len(sys.argv) > 4 else None}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps({k: round(v["bytes"] / 1e6, 3) for k, v in kernels.items()}))
