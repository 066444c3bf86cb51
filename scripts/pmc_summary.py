"""Per-kernel mean of rocprofv3 --pmc counters over dispatches (scripts/pmc.sh output).

    python scripts/pmc_summary.py gpurun_out/pmc_<tag>_* > profiles/<name>.csv
"""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
print("kernel,counter,dispatches,mean_per_dispatch")
for k in sorted(acc):
    for c in sorted(acc[k]):
        per = defaultdict(float)
        for did, v in acc[k][c]:
            per[did] += v  # sum over XCC/SE instances of one dispatch
        vals = list(per.values())
        print(f"{k},{c},{len(vals)},{sum(vals) / len(vals):.6g}")
