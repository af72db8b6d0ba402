# Round-6 GPU runs on one MI355X.  Steps chosen by env (each its own time limit, stop at
# the first failure):
#   T="<pytest args>"   run those GPU tests (default: the whole -m gpu suite when TESTS=1)
#   SQ=1                SQ counter passes (tools/pmc_sq.sh) -> profiles/<tag>_sq.json
#   PMC=1               calibrated FETCH/WRITE passes (tools/pmc_r3.sh)
#   BENCH=1             bench line (BENCH_ARGS) -> gpurun_out/<tag>_bench.json
#   PROF=1              rocprofv3 --kernel-trace --stats of the Gatys / L-BFGS / fast_st legs
#   SMOKE=1             __graft_entry__.smoke()
#   gpurun --timeout 1150 -- 'T="tests/test_lbfgs_gpu.py" SQ=1 BENCH=1 bash tools/gpu_r6.sh r6a'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out profiles
tag=${1:-r6}
if [ -n "${TESTS:-}" ] || [ -n "${T:-}" ]; then
  echo "== tests ${T:-all}"
  timeout -k 10 900 python -u -m pytest ${T:-tests/} ${K:+-k "$K"} -m gpu -x -q -rf -s --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SMOKE:-}" ]; then
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
  tail -1 gpurun_out/${tag}_smoke.log
fi
if [ -n "${SQ:-}" ]; then
  echo "== sq"
  timeout -k 10 400 bash tools/pmc_sq.sh ${tag} ${SQ_ARGS:-} > gpurun_out/${tag}_sq.log 2>&1 || { tail -10 gpurun_out/${tag}_sq.log; exit 1; }
  cp profiles/${tag}_sq.json gpurun_out/${tag}_sq.json; tail -18 gpurun_out/${tag}_sq.log
fi
if [ -n "${PMC:-}" ]; then
  echo "== pmc"
  timeout -k 10 600 bash tools/pmc_r3.sh ${tag} > gpurun_out/${tag}_pmc.log 2>&1 || { tail -10 gpurun_out/${tag}_pmc.log; exit 1; }
  cp profiles/${tag}_pmc.json gpurun_out/${tag}_pmc.json
fi
if [ -n "${AB:-}" ]; then
  echo "== ab $AB"
  timeout -k 10 400 python tools/ab_engine.py $AB ${AB_ARGS:-} > gpurun_out/${tag}_ab.log 2>&1 || { tail -20 gpurun_out/${tag}_ab.log; exit 1; }
  tail -12 gpurun_out/${tag}_ab.log
fi
if [ -n "${MICRO:-}" ]; then
  # MICRO_AB=1: the same script under libstx_prev.so as well (same box); MICRO_LIBS: the
  # library variants to run it under (default libstx.so [libstx_prev.so])
  for v in ${MICRO_LIBS:-libstx.so ${MICRO_AB:+libstx_prev.so}}; do
    L=$PWD/styletransfer_amd/$v
    echo "== micro $MICRO ($v)"
    STX_LIB_PARTIAL=1 STX_LIB=$L timeout -k 10 300 python $MICRO ${MICRO_ARGS:-} > gpurun_out/${tag}_micro_$v.log 2>&1 || { tail -20 gpurun_out/${tag}_micro_$v.log; exit 1; }
    tail -40 gpurun_out/${tag}_micro_$v.log
  done
fi
if [ -n "${PROFAB:-}" ]; then
  echo "== prof A/B $PROFAB"
  timeout -k 10 600 bash tools/prof_libs.sh ${tag}_pab $PROFAB > gpurun_out/${tag}_pab.log 2>&1 || { tail -20 gpurun_out/${tag}_pab.log; exit 1; }
  tail -40 gpurun_out/${tag}_pab.log
fi
if [ -n "${BENCH:-}" ]; then
  echo "== bench"
  timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
  cat gpurun_out/${tag}_bench.json
fi
if [ -n "${PROF:-}" ]; then
  echo "== rocprof gatys"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
    -- python3 bench.py --steps 50 --warmup 5 --skip-cpu --skip-fast --skip-infer --lbfgs-steps 0 > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
  echo "== rocprof lbfgs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_profl -o run \
    -- python3 bench.py --steps 1 --warmup 1 --gatys-run-iters 0 --skip-cpu --skip-fast --skip-infer > gpurun_out/${tag}_profl.log 2>&1 || { tail -20 gpurun_out/${tag}_profl.log; exit 1; }
  echo "== rocprof fast_st"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_proff -o run \
    -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/${tag}_proff.log 2>&1 || { tail -20 gpurun_out/${tag}_proff.log; exit 1; }
fi
echo "== done"
