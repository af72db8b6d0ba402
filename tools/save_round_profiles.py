"""Copy the round_profiles.sh outputs from gpurun_out/ into profiles/<tag>_* (bench line,
rocprof stats of the same command, per-grid roofline-kernel durations, PMC record,
Gatys / fast_st breakdowns).  usage: python tools/save_round_profiles.py r2"""
import csv
import json
import shutil
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r2"
G = "gpurun_out"
shutil.copy(f"{G}/bench_{tag}.json", f"profiles/{tag}_bench.json")
shutil.copy(f"{G}/prof_bench_{tag}/run_kernel_stats.csv", f"profiles/{tag}_bench_kernel_stats.csv")
shutil.copy(f"{G}/breakdown_{tag}g.txt", f"profiles/{tag}_gatys512_iteration_breakdown.txt")
shutil.copy(f"{G}/breakdown_{tag}f.txt", f"profiles/{tag}_fast_st_step_breakdown.txt")
shutil.copy(f"{G}/prof_{tag}f/run_kernel_stats.csv", f"profiles/{tag}_fast_st_kernel_stats.csv")
K = "conv3x3_f16x3_kernel<64, 1, 0, 0, 2>"
by = {}
for r in csv.DictReader(open(f"{G}/prof_bench_{tag}/run_kernel_trace.csv")):
    if K in r["Kernel_Name"]:
        g = tuple(int(r[f"Grid_Size_{a}"]) // int(r[f"Workgroup_Size_{a}"]) for a in "XYZ")
        by.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
names = {(1024, 1, 1): "conv1_2 fwd 512^2 (+ fused Gram; the roofline launch; includes the 20 + 1 "
                       "plain launches bench.py times for the fused-Gram cost)",
         (256, 2, 1): "conv2_2 fwd 256^2 (Gatys)", (256, 1, 8): "conv1_2 fwd 256^2 B8 (fast_st loss network)",
         (64, 2, 8): "conv2_2 fwd 128^2 B8 (fast_st loss network)",
         (256, 1, 64): "conv1_2 fwd B64 (fast_st_b64)", (64, 2, 64): "conv2_2 fwd B64 (fast_st_b64)"}
out = [f"rocprofv3 --kernel-trace of `python3 bench.py` (same command as profiles/{tag}_bench.json):",
       f"per-dispatch durations of {K} by grid (blocks x, y, z)",
       "grid            dispatches  mean_us  median_us  launch"]
for g, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    out.append(f"{str(g):15s} {len(v):10d} {statistics.mean(v):8.2f} {statistics.median(v):10.2f}  "
               f"{names.get(g, '')}")
open(f"profiles/{tag}_bench_roofline_kernel.txt", "w").write("\n".join(out) + "\n")
log = open(f"{G}/pmc_{tag}.log").read()
rec = json.loads(log[log.index("{"):log.rindex("}") + 1])
json.dump(rec, open(f"profiles/{tag}_pmc_conv1_2_fwd.json", "w"), indent=1)
print("\n".join(out))
