"""Kernel sequence of one timed pass from a rocprofv3 --kernel-trace csv: every dispatch between
two consecutive tiled_pass_kernel launches (the graph-replayed pass), with its duration and the
gap before it (us).  python scripts/pass_sequence.py <kernel_trace.csv>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [k for k, r in enumerate(rows) if "tiled_pass_kernel" in r["Kernel_Name"]]
if len(idx) < 3:
    sys.exit("fewer than 3 pass launches in the trace")
a, b = idx[-3], idx[-2]  # a whole timed pass (the last launch is the Python-launched event pass)
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
tot_k = 0
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.split(r"[<(]", r["Kernel_Name"].replace("void ", ""), maxsplit=1)[0]
    gap = (s - prev_end) / 1000 if prev_end is not None else 0.0
    print(f"{(s - t0) / 1000:9.2f}  gap {gap:7.2f}  dur {(e - s) / 1000:8.2f}  {name[:90]}")
    prev_end = e
    tot_k += e - s
print(f"pass-to-pass {(int(rows[b]['Start_Timestamp']) - t0) / 1000:.1f} us")
