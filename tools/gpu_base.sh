# Quick baseline on one MI355X: the bench line (no CPU leg) and the rocprofv3
# --kernel-trace --stats summaries of the Gatys and fast_st legs.
#   gpurun --timeout 900 -- 'bash tools/gpu_base.sh <tag>'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-base}
echo "== bench"
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --skip-cpu ${BENCH_ARGS:-} > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
echo "== rocprof gatys"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
  -- python3 bench.py --steps 50 --warmup 5 --skip-cpu --skip-fast --skip-infer --gatys-run-iters 0 > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
echo "== rocprof fast_st"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_proff -o run \
  -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/${tag}_proff.log 2>&1 || { tail -20 gpurun_out/${tag}_proff.log; exit 1; }
echo "== done"
