set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcg -o run -- python3 tools/bench_conv.py --only "conv1_1" > gpurun_out/pmcg.log 2>&1 || { tail -5 gpurun_out/pmcg.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_SCRATCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/pmcg2 -o run -- python3 tools/bench_conv.py --only "conv1_1" > gpurun_out/pmcg2.log 2>&1 || { tail -5 gpurun_out/pmcg2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmcg", "gpurun_out/pmcg2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    by = collections.defaultdict(lambda: collections.defaultdict(float))
    order = []
    for r in rows:
        if "fewin16" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        if did not in order:
            order.append(did)
        by[did][r["Counter_Name"]] += float(r["Counter_Value"])
    order.sort()
    for lab, ids in (("plain", order[1:20]), ("gram", order[-19:])):
        acc = collections.defaultdict(float)
        for i in ids:
            for k, v in by[i].items():
                acc[k] += v / len(ids)
        print(d, lab, {k: round(v) for k, v in sorted(acc.items())})
PY
