"""Per-iteration kernel breakdown of the Gatys hipGraph replays in a rocprofv3
kernel trace (gpurun_out/prof/run_kernel_trace.csv): kernels between consecutive
Adam launches, averaged over the last N iterations."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
a, b = idx[-n_it - 1], idx[-1]
agg = collections.defaultdict(lambda: [0, 0])
for r in rows[a + 1:b + 1]:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    blocks = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    k = f"{r['Kernel_Name'][:72]} grid={blocks},{r['Grid_Size_Y']},{r['Grid_Size_Z']}"
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{100 * v[1] / tot:6.2f}% {v[0] / n_it:4.1f}/it {v[1] / v[0] / 1e3:8.1f}us  {k}")
span = (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / n_it / 1e3
print(f"{tot / n_it / 1e3:.1f} us kernel time per iteration, {span:.1f} us wall (profiled)")
