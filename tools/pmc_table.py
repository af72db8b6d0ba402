"""Print per-kernel medians of the counters collected by tools/pmc_conv.sh."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(f"{root}/pmc*/run_counter_collection.csv")):
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0][-48:]
    for (d, c), v in per.items():
        vals[names[d]][c].append(v)
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {statistics.median(v):16.1f}   (n={len(v)})")
