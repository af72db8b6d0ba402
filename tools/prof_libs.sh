# rocprofv3 --stats of one bench leg under the in-tree libstx.so and libstx_prev.so
# (same box), then the per-kernel mean durations side by side (tools/stats_cmp.py).
#   gpurun -- 'bash tools/prof_libs.sh <tag> fast|gatys'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export STX_AB=1  # (the host path reads its A/B switches only under STX_AB=1: N.knob)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; leg=${2:-fast}
if [ "$leg" = fast ]; then ARGS="--fast-only --steps 20 --warmup 2"; else ARGS="--steps 30 --warmup 3 --skip-cpu --skip-fast --skip-infer --lbfgs-steps 0 --gatys-run-iters 0"; fi
for v in new prev; do
  if [ $v = prev ]; then L=$PWD/styletransfer_amd/libstx_prev.so; else L=$PWD/styletransfer_amd/libstx.so; fi
  X=""; [ $v = prev ] && X="${PREV_ENV:-}"; env $X STX_LIB_PARTIAL=1 STX_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_$v -o run \
    -- python3 bench.py $ARGS > gpurun_out/${tag}_$v.log 2>&1 || { tail -20 gpurun_out/${tag}_$v.log; exit 1; }
  tail -1 gpurun_out/${tag}_$v.log
done
python3 tools/stats_cmp.py gpurun_out/${tag}_new/run_kernel_stats.csv gpurun_out/${tag}_prev/run_kernel_stats.csv
