# Round-3 evidence on one MI355X: -m gpu suite, smoke, the bench line (with the CPU
# baseline), the rocprofv3 --kernel-trace --stats summary of the same bench command
# (Gatys legs) and of the fast_st leg, and the calibrated FETCH/WRITE passes
# (tools/pmc_r3.sh).  gpurun --timeout 1100 -- 'bash tools/gpu_round3.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -20
[ $rc -le 1 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== pmc"
timeout -k 10 600 bash tools/pmc_r3.sh r3 || exit 1
echo "== bench"
timeout -k 10 400 python bench.py --steps 50 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof gatys"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps 50 --warmup 5 --skip-cpu --skip-fast --skip-infer > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
echo "== rocprof fast_st"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proff -o run \
  -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/proff.log 2>&1 || { tail -20 gpurun_out/proff.log; exit 1; }
echo "== done"
exit $rc
