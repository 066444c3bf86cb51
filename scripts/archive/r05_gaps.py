"""Experiment: where the wall time of the timed bench loop goes between the pass kernels -- reads
a rocprofv3 --kernel-trace CSV (of `bench.py --no-forced --no-informative --no-cpu-baseline`) and
prints, over the last K tiled_pass_kernel<0> launches, each kernel's mean duration and the mean
idle gap before it (the GPU doing nothing).  python scripts/archive/r05_gaps.py <kernel_trace.csv> [K]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "tiled_pass_kernel<0>" in r["Kernel_Name"]]
lo = idx[-K - 1]  # from the end of a pass K + 1 passes before the last
seg = rows[lo:]
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
prev_end = int(seg[0]["End_Timestamp"])
for r in seg[1:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"][:60]
    dur[n] += (e - s) / 1e3
    gap[n] += max(0, s - prev_end) / 1e3
    cnt[n] += 1
    prev_end = max(prev_end, e)
span = (prev_end - int(seg[0]["End_Timestamp"])) / 1e3
print(f"{K} passes, {span / K:.1f} us per pass")
for n in sorted(dur, key=lambda n: -dur[n]):
    print(f"  {n:60s} n/pass {cnt[n] / K:4.1f}  dur {dur[n] / cnt[n]:8.1f} us  idle before {gap[n] / cnt[n]:7.1f} us")
