"""Per-kernel mean of rocprofv3 --pmc counters over dispatches (scripts/pmc.sh output).

    python scripts/pmc_summary.py gpurun_out/pmc_<tag>_* > profiles/<name>.csv
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            # base name only: template arguments hold commas, which would break the CSV
            name = re.split(r"[<(]", r["Kernel_Name"].replace("void ", ""), maxsplit=1)[0].strip()
            acc[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
print("kernel,counter,dispatches,mean_per_dispatch")
for k in sorted(acc):
    for c in sorted(acc[k]):
        per = defaultdict(float)
        for did, v in acc[k][c]:
            per[did] += v  # sum over XCC/SE instances of one dispatch
        vals = list(per.values())
        print(f"{k},{c},{len(vals)},{sum(vals) / len(vals):.6g}")
