"""Timeline of a rocprofv3 kernel trace: the dominant kernel's launches, what runs between two
consecutive ones, and the idle gaps (device time covered by no kernel)."""
import csv
import sys
from collections import Counter

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else "tiled_pass_kernel<0"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
dom = [i for i, e in enumerate(ev) if pat in e[2]]
print(f"{len(ev)} kernels, {len(dom)} '{pat}' launches")
periods, busy, between = [], [], Counter()
for a, b in zip(dom[-12:-1], dom[-11:]):
    t0, t1 = ev[a][0], ev[b][0]
    periods.append((t1 - t0) / 1e3)
    # union of kernel intervals in [t0, t1)
    cov, cur_s, cur_e = 0, None, None
    for s, e, n in ev[a:b]:
        s, e = max(s, t0), min(e, t1)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                cov += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    cov += cur_e - cur_s
    busy.append(cov / 1e3)
    for s, e, n in ev[a + 1:b]:
        between[(n[:90], round((e - s) / 1e3, 1))] += 1
print("period us (dominant start -> next start):", np.round(periods, 1))
print("device busy us per period:", np.round(busy, 1))
print("dominant kernel us:", np.round([(ev[i][1] - ev[i][0]) / 1e3 for i in dom[-11:]], 1))
print("between (name, us): count")
for k, v in between.most_common(25):
    print("  ", v, k)
