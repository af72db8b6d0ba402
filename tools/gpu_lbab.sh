# L-BFGS leg A/B on one box (separate processes, alternating): bench.py's gatys_lbfgs
# with VAR=a vs VAR=b, after the given tests.  gpurun -- 'bash tools/gpu_lbab.sh <tag> VAR a b "<tests>"'
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; var=$2; va=$3; vb=$4; T=${5:-}
if [ -n "$T" ]; then
  timeout -k 10 400 python -u -m pytest $T -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
  rc=$?; echo "T rc=$rc"; tail -1 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -10
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for v in $va $vb; do
    env $var=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --skip-cpu --skip-fast --skip-infer --gatys-run-iters 0 --lbfgs-steps 10 > gpurun_out/${tag}_$v$i.json 2>gpurun_out/${tag}_$v$i.err || { tail -3 gpurun_out/${tag}_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${tag}_$v$i.json'));l=d['gatys_lbfgs'];print('$var=$v #$i', 'adam_ms', d['ms_per_step'], 'lbfgs evals/s', l['value'], 'ratio', l['vs_adam_iteration_rate'], 'fill', l['fill_evals_per_s'])"
  done
done
