# rocprofv3 kernel trace of the bench's Gatys-Adam leg under env variants, each followed by
# the per-iteration breakdown (tools/iter_breakdown.py).
#   gpurun -- 'bash tools/prof_iter.sh tag "STX_COMPOSE=0" "STX_COMPOSE=1"'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export STX_AB=1  # (the host path reads its A/B switches only under STX_AB=1: N.knob)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; shift
i=0
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_pi$i -o run \
    -- python3 bench.py --steps 30 --warmup 3 --skip-cpu --skip-fast --skip-infer --lbfgs-steps 0 --gatys-run-iters 0 > gpurun_out/${tag}_pi$i.log 2>&1 || { tail -20 gpurun_out/${tag}_pi$i.log; exit 1; }
  python3 tools/iter_breakdown.py gpurun_out/${tag}_pi$i/run_kernel_trace.csv 20 > gpurun_out/${tag}_pi$i.txt || exit 1
  cat gpurun_out/${tag}_pi$i.txt
  i=$((i+1))
done
