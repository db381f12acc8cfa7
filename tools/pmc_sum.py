"""Sum rocprofv3 counter_collection.csv per (kernel, counter); print per-dispatch means."""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    acc = defaultdict(float)
    disp = defaultdict(set)
    dur = defaultdict(float)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0]
        acc[(k, row["Counter_Name"])] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    print("==", path)
    kern = sorted(disp, key=lambda k: -acc.get((k, "SQ_WAVE_CYCLES"), 0))
    for k in kern[:12]:
        n = len(disp[k])
        vals = {c: v / n for (kk, c), v in acc.items() if kk == k}
        print(f"  {k[:70]:70s} n={n}")
        print("    " + "  ".join(f"{c.replace('SQ_', '')}={v:.4g}" for c, v in sorted(vals.items())))
