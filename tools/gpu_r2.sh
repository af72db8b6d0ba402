# Round-2 GPU check: full GPU test suite (verbose, per-test timeout), the ITN fp64
# diagnostic, a host-CPU probe and a 1-GPU bench line; then a same-device 2-rank
# bench rehearsal (gloo) of the launcher.  Usage: gpurun -- 'bash tools/gpu_r2.sh [quick]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== host"; python - <<'PY'
import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), "OMP", os.environ.get("OMP_NUM_THREADS"))
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective"):
    try: print(f, open(f).read().strip())
    except OSError as e: print(f, e)
PY
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "passed|failed|error" gpurun_out/t.log | tail -3
grep -E "^E |FAILED|Error|err |rel err|diff" gpurun_out/t.log | head -40
[ $rc -le 1 ] || exit $rc
[ "$1" = quick ] && exit $rc
echo "== diag"; timeout -k 10 120 python tools/diag_itn_grad.py > gpurun_out/diag.log 2>&1; tail -3 gpurun_out/diag.log
echo "== bench"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== bench2 (same-device rehearsal)"
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --skip-infer --fast-steps 10 > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { tail -20 gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
exit $rc
