# environment A/B on one box (separate processes, alternating): bench.py Gatys + fast_st legs
# with VAR=a vs VAR=b, after the given tests.   gpurun -- 'bash tools/gpu_envab.sh <tag> VAR a b "<tests>"'
export STX_AB=1  # (the host path reads its A/B switches only under STX_AB=1: N.knob)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; var=$2; va=$3; vb=$4; T=${5:-}
if [ -n "$T" ]; then
  timeout -k 10 400 python -u -m pytest $T -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
  rc=$?; echo "T rc=$rc"; tail -1 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -10
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for v in $va $vb; do
    env $var=$v timeout -k 10 200 python bench.py --steps 50 --warmup 5 --skip-cpu --skip-infer --lbfgs-steps 0 --gatys-run-iters 0 --fast-b64-steps 0 > gpurun_out/${tag}_$v$i.json 2>gpurun_out/${tag}_$v$i.err || { tail -3 gpurun_out/${tag}_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${tag}_$v$i.json'));print('$var=$v #$i', 'gatys_ms', d['ms_per_step'], 'fast_ms', d['fast_st']['ms_per_step'])"
  done
done
