#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (short name), mean of each counter
over dispatches, plus per-wave derived values."""
import csv
import re
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
    agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{k[:60]:60s} n={len(next(iter(cs.values())))}"
    for c, v in sorted(m.items()):
        line += f" {c}={v:.4g}"
    w = m.get("SQ_WAVES")
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"):
            if c in m:
                line += f" {c}/wave={m[c] / w:.4g}"
    print(line)
