"""Turn the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round.sh into a per-launch
HBM-traffic record for one kernel, written under profiles/ (bench.py reports it
as roofline.traffic).

    python tools/pmc_summary.py --kernel 'conv3x3_f16x3_kernel<64, 1>' \
        --out profiles/r1_pmc_conv1_2_fwd.json [--gpurun-out gpurun_out]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3).  MI355X_MICROARCH.md
§HBM: on gfx950 FETCH_SIZE reports exactly half the bytes of a 16-B/lane streaming
read; other access widths are uncalibrated.  The record keeps the raw counters and
the bytes under both readings so the reader can see which one applies.
"""
import argparse
import csv
import json
import os
import statistics


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or kernel not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--gpurun-out", default="gpurun_out")
    ap.add_argument("--algorithmic-bytes", type=float, default=0.0)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    fe = per_dispatch(os.path.join(a.gpurun_out, "pmc_fetch", "run_counter_collection.csv"),
                      "FETCH_SIZE", a.kernel)
    wr = per_dispatch(os.path.join(a.gpurun_out, "pmc_write", "run_counter_collection.csv"),
                      "WRITE_SIZE", a.kernel)
    if not fe or not wr:
        raise SystemExit(f"no dispatches of {a.kernel!r} in the PMC passes")
    fk, wk = statistics.median(fe), statistics.median(wr)
    rec = {
        "kernel": a.kernel,
        "command": a.command,
        "dispatches": {"fetch": len(fe), "write": len(wr)},
        "FETCH_SIZE_KiB_median": fk,
        "WRITE_SIZE_KiB_median": wk,
        "bytes_raw": (fk + wk) * 1024.0,
        "bytes_fetch_x2": (2.0 * fk + wk) * 1024.0,
        "algorithmic_bytes": a.algorithmic_bytes or None,
        "note": "traffic = bytes_raw: the kernel's global reads are 4-B/lane buffer "
                "loads (uncalibrated width per MI355X_MICROARCH.md §HBM; the x2 "
                "correction is for 16-B/lane streams and is given as bytes_fetch_x2)",
    }
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
