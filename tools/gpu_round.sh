# Round-end evidence on one MI355X: GPU parity tests, the bench line (with the CPU
# baseline), the rocprofv3 kernel-trace summary of the same bench command, and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs) for the dominant conv kernel.
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { echo "== $*" ; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
step bench
timeout -k 10 300 python bench.py --steps 50 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps 50 --warmup 3 --skip-cpu --skip-fast --skip-infer > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
step pmc-fetch
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
  -- python3 tools/bench_conv.py --only "conv1_2" > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
step pmc-write
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run \
  -- python3 tools/bench_conv.py --only "conv1_2" > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
step done
find gpurun_out -name "*.csv" | head -20
step rocprof-fast_st
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proff -o run \
  -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/proff.log 2>&1 || { tail -20 gpurun_out/proff.log; exit 1; }
step done-fast
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
