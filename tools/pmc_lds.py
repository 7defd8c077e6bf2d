#!/usr/bin/env python3
"""LDS traffic of the EPnP launch set from an SQ pass summary (tools/pmc_summary.py text, e.g.
profiles/r05/pmc_sq_r6l.txt): SQ_INSTS_LDS per dispatch of each kernel x 64 lanes x 8 B, an upper
estimate of the bytes moved (every LDS instruction counted as a full-wave 8-byte access).
Usage: pmc_lds.py <pmc_sq.txt> <commit> > pmc_lds.json"""
import json
import re
import sys

SET = ("pnp_eig_split_kernel<4>", "pnp_betas_kernel<4>", "pnp_scan_kernel<8>")
per = {}
for line in open(sys.argv[1]):
    m = re.match(r"(\S+)\s+n=\d+\s+(.*)", line)
    if not m or "SQ_INSTS_LDS=" not in line:
        continue
    name = m.group(1).replace("rsc::", "")
    v = float(re.search(r"SQ_INSTS_LDS=([0-9.e+]+)", line).group(1))
    if name in SET:
        per[name] = v
out = {"kernels": {k: {"lds_instructions": v, "lds_bytes_upper": v * 64 * 8} for k, v in per.items()},
       "lds_bytes_upper_per_launch_set": sum(v * 64 * 8 for v in per.values()),
       "estimate": "SQ_INSTS_LDS x 64 lanes x 8 B per dispatch (upper: partial waves and 4-byte accesses counted full)",
       "source": sys.argv[1], "commit": sys.argv[2]}
json.dump(out, sys.stdout, indent=1)
print()
