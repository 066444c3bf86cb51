"""Median duration per kernel (substring match) from a rocprofv3 kernel trace; ot_iter launches
that exit at the stop rule (< 20 us) are counted separately."""
import csv
import sys

import numpy as np

path = sys.argv[1]
names = sys.argv[2:] or ["ot_iter", "ot_init", "ot_final", "ot_col", "ot_apply", "ot_prep", "ot_setup"]
rows = list(csv.DictReader(open(path)))
for kn in names:
    d = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if kn in r["Kernel_Name"]])
    if not len(d):
        continue
    live = d[d > 20000] if kn == "ot_iter" else d
    print(f"{kn:>12}: {len(d)} launches, {len(live)} live, median {np.median(live) / 1e3 if len(live) else 0:.1f} us,"
          f" total {d.sum() / 1e6:.2f} ms")
