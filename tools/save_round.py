"""Copy the tools/gpu_r4.sh outputs gpurun_out/<tag>_* into profiles/<tag>_*: the bench
line, the rocprofv3 --stats summaries of the bench's Gatys-Adam legs, its L-BFGS leg and
its fast_st leg, the per-iteration Gatys breakdown, and the per-grid durations of the
roofline and dominant kernels (same trace).  The calibrated PMC record is written by
tools/pmc_r3.sh itself.  usage: python tools/save_round.py r4"""
import csv
import os
import shutil
import statistics
import subprocess
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r3"
G = "gpurun_out"
shutil.copy(f"{G}/{tag}_bench.json", f"profiles/{tag}_bench.json")
shutil.copy(f"{G}/{tag}_prof/run_kernel_stats.csv", f"profiles/{tag}_bench_kernel_stats.csv")
shutil.copy(f"{G}/{tag}_profl/run_kernel_stats.csv", f"profiles/{tag}_lbfgs_kernel_stats.csv")
shutil.copy(f"{G}/{tag}_proff/run_kernel_stats.csv", f"profiles/{tag}_fast_st_kernel_stats.csv")
if os.path.exists(f"{G}/{tag}_pmc.json"):
    shutil.copy(f"{G}/{tag}_pmc.json", f"profiles/{tag}_pmc.json")
br = subprocess.check_output([sys.executable, "tools/iter_breakdown.py",
                              f"{G}/{tag}_prof/run_kernel_trace.csv"], text=True)
open(f"profiles/{tag}_gatys512_iteration_breakdown.txt", "w").write(
    "rocprofv3 --kernel-trace of `python3 bench.py --skip-cpu --skip-fast --skip-infer "
    "--lbfgs-steps 0` "
    "(tools/iter_breakdown.py: kernels between consecutive Adam launches, last 20 "
    "iterations)\n" + br)
out = [f"rocprofv3 --kernel-trace of the bench's Gatys legs (profiles/{tag}_bench_kernel_stats.csv):",
       "per-dispatch durations by grid (blocks x, y, z)",
       "kernel                                              grid            n   mean_us  median_us"]
for K in ("conv3x3_f16x3_v2_kernel<64, 1, 0, 2, 1>", "conv3x3_f16x3_v2_kernel<64, 0, 3, 2, 1>",
          "conv3x3_f16x3_v2_kernel<64, 0, 1, 2, 1>"):
    by = {}
    for r in csv.DictReader(open(f"{G}/{tag}_prof/run_kernel_trace.csv")):
        if K in r["Kernel_Name"]:
            g = tuple(int(r[f"Grid_Size_{a}"]) // int(r[f"Workgroup_Size_{a}"]) for a in "XYZ")
            by.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for g, v in sorted(by.items(), key=lambda kv: -len(kv[1])):  # (absent variants: no rows)
        out.append(f"{K:50s} {str(g):15s} {len(v):4d} {statistics.mean(v):8.2f} {statistics.median(v):10.2f}")
open(f"profiles/{tag}_bench_roofline_kernel.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
