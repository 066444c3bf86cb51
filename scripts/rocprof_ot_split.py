"""Append to a rocprofv3 --stats kernel summary the average of the Sinkhorn iteration launches
that RAN an iteration, from the same run's kernel trace:

    python scripts/rocprof_ot_split.py <kernel_trace.csv> <kernel_stats.csv>

The engine (and bench's OT calls) enqueue iteration launches past the stop rule that exit at
once (include/nfdpf.h, nfdpf_ot_resample poll / stop_at), so the summary's ot_iter_kernel
average mixes ~1 us tail launches into the 18-115 us iterations.  A launch counts as an
iteration when it lasts more than a quarter of the 90th percentile of that kernel's launches;
the row is named "<kernel>[full]" (bench.rocprof_avg_ms reads it), a "[tail]" row beside it."""
import csv
import sys

import numpy as np

trace, stats = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(trace)))
by = {}
for r in rows:
    if "ot_iter_kernel" in r["Kernel_Name"]:
        by.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
out = []
for name, d in by.items():
    d = np.array(d, dtype=np.float64)
    thr = 0.25 * np.percentile(d, 90)
    for tag, sel in (("full", d > thr), ("tail", d <= thr)):
        v = d[sel]
        if len(v):
            out.append([f"{name}[{tag}]", len(v), int(v.sum()), float(v.mean()), 0.0, int(v.min()), int(v.max()),
                        float(v.std())])
with open(stats, "a", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    for r in out:
        w.writerow(r)
print(f"{stats}: {len(out)} rows appended")
