# rocprofv3 kernel traces of the Gatys leg under VAR=a and VAR=b, per-iteration breakdowns
#   gpurun -- 'bash tools/gpu_prof_env.sh <tag> VAR a b'
cd /tmp && export TMPDIR=/tmp
export STX_AB=1  # (the host path reads its A/B switches only under STX_AB=1: N.knob)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; var=$2
for v in $3 $4; do
  export $var=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_$v -o run \
    -- python3 bench.py --steps 30 --warmup 5 --skip-cpu --skip-fast --skip-infer --lbfgs-steps 0 \
    --gatys-run-iters 0 > gpurun_out/${tag}_$v.log 2>&1 || { tail -5 gpurun_out/${tag}_$v.log; exit 1; }
  f=$(ls gpurun_out/${tag}_$v/*/run_kernel_trace.csv gpurun_out/${tag}_$v/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/iter_breakdown.py "$f" 20 > gpurun_out/${tag}_$v.txt && echo "== $var=$v" && head -8 gpurun_out/${tag}_$v.txt && tail -1 gpurun_out/${tag}_$v.txt
  rm -rf gpurun_out/${tag}_$v
done
