"""Summarise tools/pmc_sq.sh: per (kernel, grid) of the eager Gatys iteration, medians per
dispatch of the SQ/GRBM counters and the derived fractions:
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  clock_ghz   = GRBM_GUI_ACTIVE / 8 / kernel duration (the profiled clock)
  parked      = SQ_WAIT_ANY / SQ_WAVE_CYCLES      (s_waitcnt / barrier)
  issue_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (dependency / pipe busy)
  issuing     = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
Writes profiles/<tag>_sq.json."""
import csv
import glob
import json
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r3"
vals = {}   # (kernel, grid) -> counter -> [per dispatch]
durs = {}   # dispatch id -> ns
for f in glob.glob("gpurun_out/pmcsq_*/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        durs[(f.split("/")[1], int(r["Dispatch_Id"]))] = (int(r["End_Timestamp"]) -
                                                         int(r["Start_Timestamp"]))
per = {}
for f in glob.glob("gpurun_out/pmcsq_*/**/*counter_collection.csv", recursive=True):
    run = f.split("/")[1]
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"], int(r["Grid_Size"]))
        d = per.setdefault((key, run, int(r["Dispatch_Id"])), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for (key, run, did), d in per.items():
    v = vals.setdefault(key, {})
    for c, x in d.items():
        v.setdefault(c, []).append(x)
    if (run, did) in durs:
        v.setdefault(f"dur_ns_{run}", []).append(durs[(run, did)])
recs = []
for (k, g), v in vals.items():
    m = {c: statistics.median(x) for c, x in v.items()}
    r = {"kernel": k, "grid": g, **m}
    gui, wc = m.get("GRBM_GUI_ACTIVE"), m.get("SQ_WAVE_CYCLES")
    if gui:
        r["mfma_util"] = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024)
        d1 = m.get("dur_ns_pmcsq_1")
        if d1:
            r["clock_ghz"] = gui / 8 / d1
    if wc:
        for name, c in (("parked", "SQ_WAIT_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                        ("issuing", "SQ_ACTIVE_INST_ANY"), ("lds_issue_stall", "SQ_WAIT_INST_LDS")):
            if c in m:
                r[name] = m[c] / wc
    recs.append(r)
recs.sort(key=lambda r: -r.get("dur_ns_pmcsq_1", 0))
json.dump({"kernels": recs}, open(f"profiles/{tag}_sq.json", "w"), indent=1)
for r in recs[:16]:
    print(f"{r['kernel'][:58]:58s} g{r['grid']:8d} {r.get('dur_ns_pmcsq_1', 0)/1e3:6.1f}us "
          f"mfma {r.get('mfma_util', 0):.3f} clk {r.get('clock_ghz', 0):.2f} "
          f"park {r.get('parked', 0):.2f} stall {r.get('issue_stall', 0):.2f} "
          f"issue {r.get('issuing', 0):.2f} lds {r.get('lds_issue_stall', 0):.2f} "
          f"valu {r.get('SQ_INSTS_VALU', 0):.3g} mfma# {r.get('SQ_INSTS_MFMA', 0):.3g} "
          f"lds# {r.get('SQ_INSTS_LDS', 0):.3g} bank {r.get('SQ_LDS_BANK_CONFLICT', 0):.3g}")
