# L-BFGS: the GPU tests, then a rocprofv3 kernel trace of bench.py's gatys_lbfgs leg and
# the full-history (last 100) durations of the history passes.  gpurun -- 'bash tools/gpu_lbprof.sh <tag>'
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-lbp}
timeout -k 10 300 python -u -m pytest tests/test_lbfgs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1 || { tail -15 gpurun_out/${tag}_t.log; exit 1; }
tail -1 gpurun_out/${tag}_t.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag} -o run \
  -- python3 bench.py --steps 1 --warmup 1 --gatys-run-iters 0 --skip-cpu --skip-fast --skip-infer > gpurun_out/${tag}.log 2>&1 || { tail -20 gpurun_out/${tag}.log; exit 1; }
python3 - "$tag" <<'PY'
import csv, glob, json, statistics, sys
tag = sys.argv[1]
f = (glob.glob(f"gpurun_out/{tag}/*/run_kernel_trace.csv") + glob.glob(f"gpurun_out/{tag}/run_kernel_trace.csv"))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
for name in ("lb_dots_kernel", "lb_combine_kernel", "lb_solve_kernel"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    print(name, len(d), "last-100 mean %.1f us" % statistics.mean(d[-100:]))
line = [l for l in open(f"gpurun_out/{tag}.log") if l.startswith("{")][-1]
print("gatys_lbfgs", json.loads(line)["gatys_lbfgs"]["value"])
PY
