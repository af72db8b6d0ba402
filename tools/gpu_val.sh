# Validation of a fresh build on one MI355X: the -m gpu suite (quiet), smoke, one bench
# line.  gpurun --timeout 1100 -- 'bash tools/gpu_val.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread "$@" > gpurun_out/t.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
[ $rc -le 1 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --skip-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
exit $rc
