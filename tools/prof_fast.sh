# rocprofv3 kernel trace of the fast_st train step (graph replays, B=8) + per-step
# breakdown (kernels between consecutive Adam launches).
#   gpurun -- 'bash tools/prof_fast.sh [tag]'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-f}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run \
  -- python3 bench.py --fast-only --fast-steps 30 --warmup 2 > gpurun_out/prof_$tag.log 2>&1 \
  || { echo "PROF FAILED"; tail -20 gpurun_out/prof_$tag.log; exit 1; }
python3 tools/iter_breakdown.py gpurun_out/prof_$tag/run_kernel_trace.csv 20 | tee gpurun_out/breakdown_$tag.txt
