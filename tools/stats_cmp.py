"""Two rocprofv3 kernel_stats.csv files side by side: mean duration (us) and total per
kernel name, sorted by the first file's total."""
import csv
import sys

a, b = [{r["Name"]: r for r in csv.DictReader(open(f))} for f in sys.argv[1:3]]
print(f"{'kernel':80s} {'calls':>6s} {'mean A':>9s} {'mean B':>9s} {'tot A ms':>9s} {'tot B ms':>9s}")
ta = tb = 0.0
for k, r in sorted(a.items(), key=lambda kv: -float(kv[1]["TotalDurationNs"]))[:28]:
    s = b.get(k)
    ma, tA = float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6
    mb, tB = (float(s["AverageNs"]) / 1e3, float(s["TotalDurationNs"]) / 1e6) if s else (0.0, 0.0)
    print(f"{k[:80]:80s} {r['Calls']:>6s} {ma:9.1f} {mb:9.1f} {tA:9.2f} {tB:9.2f}")
ta = sum(float(r["TotalDurationNs"]) for r in a.values()) / 1e6
tb = sum(float(r["TotalDurationNs"]) for r in b.values()) / 1e6
print(f"total kernel ms: A {ta:.2f}  B {tb:.2f}")
