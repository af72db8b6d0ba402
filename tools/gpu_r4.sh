# Round-4 evidence on one MI355X: the -m gpu suite, smoke, the calibrated FETCH/WRITE
# passes (tools/pmc_r3.sh), the bench line (with the CPU baseline), and rocprofv3
# --kernel-trace --stats of the bench's Gatys-Adam legs, its L-BFGS leg and its fast_st
# leg.  Outputs gpurun_out/<tag>_*; tools/save_round.py <tag> copies them to profiles/.
#   gpurun --timeout 1150 -- 'bash tools/gpu_r4.sh r4'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-r4}
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "== tests"
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -20
  [ $rc -eq 0 ] || exit $rc
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
  tail -1 gpurun_out/${tag}_smoke.log
fi
if [ -z "${SKIP_PMC:-}" ]; then
  echo "== pmc"
  timeout -k 10 600 bash tools/pmc_r3.sh ${tag} > gpurun_out/${tag}_pmc.log 2>&1 || { tail -10 gpurun_out/${tag}_pmc.log; exit 1; }
  cp profiles/${tag}_pmc.json gpurun_out/${tag}_pmc.json
fi
echo "== bench"
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
echo "== rocprof gatys"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
  -- python3 bench.py --steps 50 --warmup 5 --skip-cpu --skip-fast --skip-infer --lbfgs-steps 0 > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
echo "== rocprof lbfgs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_profl -o run \
  -- python3 bench.py --steps 1 --warmup 1 --gatys-run-iters 0 --skip-cpu --skip-fast --skip-infer > gpurun_out/${tag}_profl.log 2>&1 || { tail -20 gpurun_out/${tag}_profl.log; exit 1; }
echo "== rocprof fast_st"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_proff -o run \
  -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/${tag}_proff.log 2>&1 || { tail -20 gpurun_out/${tag}_proff.log; exit 1; }
echo "== done"
