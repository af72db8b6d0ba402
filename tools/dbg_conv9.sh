# conv9 profiling variants (tools/bench_conv9.py) under rocprofv3 kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
p() { tag=$1; shift; env "$@" timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c9_$tag -o run -- python3 tools/bench_conv9.py > gpurun_out/c9_$tag.log 2>&1 || { tail -5 gpurun_out/c9_$tag.log; exit 1; }
  python3 - gpurun_out/c9_$tag/run_kernel_stats.csv $tag <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "conv9" in r["Name"] or "fewout" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
}
for v in ${@:-0 8 24}; do p d$v STX_CONV9_DBG=$v; done
