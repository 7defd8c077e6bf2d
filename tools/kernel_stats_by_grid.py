#!/usr/bin/env python3
"""Per-(kernel, grid size) dispatch statistics from a rocprofv3 kernel_trace.csv, so the launches
of one bench section (e.g. config 2: pnp_eig_group_kernel<4> with grid 61440) can be compared with
the HIP-event durations bench.py reports.  usage: kernel_stats_by_grid.py trace.csv [out.csv]"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").strip()
    acc[(name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1][1]) if False else -sum(kv[1]))
out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["kernel", "grid_threads", "workgroup", "calls", "avg_us", "min_us", "max_us", "total_us"])
for (name, grid, wg), d in rows:
    w.writerow([name, grid, wg, len(d), round(sum(d) / len(d), 2), round(min(d), 2), round(max(d), 2), round(sum(d), 1)])
