# HBM bytes per launch of the bench's roofline kernel (conv1_2 forward as the Gatys
# iteration launches it: fused pool output + Gram partials), one rocprofv3 --pmc pass
# per counter.  gpurun -- 'bash tools/pmc_roofline.sh r2'  ->  profiles/<tag>_pmc_conv1_2_fwd.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out profiles
tag=${1:-r2}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run \
    -- python3 tools/bench_conv.py --only conv1_2 > gpurun_out/pmc_$c.log 2>&1 \
    || { echo "PMC $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
python3 - "$tag" <<'PY'
import csv, glob, json, statistics, sys
tag = sys.argv[1]
K = "conv3x3_f16x3_kernel<64, 1, 0, 0, 2>"
vals = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmc_{c}/**/*counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if K in r["Kernel_Name"] and r["Counter_Name"] == c:
            per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    # bench_conv times the plain launch (21 dispatches), then the +gram launch (21): the
    # iteration's launch is the second group
    gram_ids = ids[-19:]
    vals[c] = (statistics.median(per[i] for i in gram_ids), len(ids))
fetch, write = vals["FETCH_SIZE"][0] * 1024, vals["WRITE_SIZE"][0] * 1024
alg = (2 * 64 * 512 * 512 * 4 + 64 * 256 * 256 * 4 + 64 * 64 * 9 * 4 + 64 * 4
       + 1024 * 64 * 64 * 4)
rec = {
    "kernel": K,
    "launch": "conv1_2 forward 64->64 @512^2, ReLU loader, fused ReLU/MaxPool output, fused Gram "
              "partials (the Gatys iteration's launch)",
    "command": "rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE, separate runs) --output-format csv "
               "-- python3 tools/bench_conv.py --only conv1_2  (tools/pmc_roofline.sh)",
    "dispatches_of_kernel": {"fetch": vals["FETCH_SIZE"][1], "write": vals["WRITE_SIZE"][1]},
    "FETCH_SIZE_KiB_median": vals["FETCH_SIZE"][0],
    "WRITE_SIZE_KiB_median": vals["WRITE_SIZE"][0],
    "bytes_raw": fetch + write,
    "bytes_fetch_x2": 2 * fetch + write,
    "algorithmic_bytes": alg,
    "note": "traffic = bytes_raw: the kernel's global reads are 4-B/lane buffer loads (the "
            "guide's x2 FETCH correction is calibrated for 16-B/lane streams; given as "
            "bytes_fetch_x2 for reference)",
}
json.dump(rec, open(f"profiles/{tag}_pmc_conv1_2_fwd.json", "w"), indent=1)
print(json.dumps(rec, indent=1))
PY
