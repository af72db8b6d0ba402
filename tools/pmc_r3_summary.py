"""Summarise tools/pmc_r3.sh: calibration factors (counter bytes / true bytes for 4-B and
16-B per lane reads and 4-B stores, 512 MiB each, HBM-streamed) and, per (kernel, grid)
of the eager Gatys iteration, the median FETCH_SIZE / WRITE_SIZE per dispatch -- raw and
calibrated.  Writes profiles/<tag>_pmc.json."""
import csv
import glob
import json
import statistics
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r3"
TRUE = 512 << 20


def load(pattern, counter):
    out = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            key = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["Dispatch_Id"]))
            out[key] = out.get(key, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


cal = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = load(f"gpurun_out/pmccal_{c}/**/*counter_collection.csv", c)
    for name, tagk in (("read4_kernel", "read4"), ("read16_kernel", "read16"),
                       ("write4_kernel", "write4")):
        v = [b for (k, g, i), b in d.items() if name in k]
        if v:
            cal[f"{tagk}_{c}"] = statistics.median(v) / TRUE
f4 = cal.get("read4_FETCH_SIZE")
w4 = cal.get("write4_WRITE_SIZE")
recs = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = load(f"gpurun_out/pmctgt_{c}/**/*counter_collection.csv", c)
    groups = {}
    for (k, g, i), b in d.items():
        groups.setdefault((k, g), []).append(b)
    for (k, g), v in groups.items():
        r = recs.setdefault(f"{k} | grid {g}", {"kernel": k, "grid": g})
        r[f"{c}_bytes_raw"] = statistics.median(v)
        r["dispatches"] = len(v)
for r in recs.values():
    fr, wr = r.get("FETCH_SIZE_bytes_raw"), r.get("WRITE_SIZE_bytes_raw")
    if fr is not None and f4:
        r["fetch_bytes_cal4"] = fr / f4
    if wr is not None and w4:
        r["write_bytes_cal4"] = wr / w4
out = {"calibration": cal,
       "calibration_note": "counter bytes / true bytes over 512 MiB streamed once (tools/calib): "
                           "read4 = 4-B per lane buffer loads, read16 = 16-B per lane global "
                           "loads, write4 = 4-B per lane buffer stores; *_cal4 = raw / the "
                           "4-B factor (the width of the conv halo / Gram-backward streams)",
       "kernels": sorted(recs.values(), key=lambda r: -(r.get("FETCH_SIZE_bytes_raw", 0)
                                                       + r.get("WRITE_SIZE_bytes_raw", 0)))}
json.dump(out, open(f"profiles/{tag}_pmc.json", "w"), indent=1)
print(json.dumps(cal, indent=1))
for r in out["kernels"][:14]:
    print(f"{r['kernel'][:60]:60s} grid {r['grid']:8d} fetch {r.get('FETCH_SIZE_bytes_raw', 0)/1e6:8.1f} MB"
          f" write {r.get('WRITE_SIZE_bytes_raw', 0)/1e6:8.1f} MB")
