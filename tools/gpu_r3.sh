# Round-3 GPU check: the whole -m gpu suite (verbose, prints kept, no -x so every
# failure shows), then optionally a 1-GPU bench line.  Usage:
#   gpurun -- 'bash tools/gpu_r3.sh [tests-args...]'   (BENCH=1 to add the bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== tests"
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -v -s -rA --timeout 300 --timeout-method thread "$@" > gpurun_out/t.log 2>&1
rc=$?; echo "TESTS rc=$rc"; grep -E "passed|failed|error" gpurun_out/t.log | tail -3
grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -40
[ $rc -le 1 ] || exit $rc
if [ "$BENCH" = 1 ]; then
  echo "== bench"
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --skip-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
exit $rc
