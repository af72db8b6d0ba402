# library A/B on one box: the in-tree libstx.so against styletransfer_amd/libstx_prev.so
# (STX_LIB), alternating bench runs (Gatys leg; fast_st leg), after the given tests.
#   gpurun -- 'bash tools/gpu_libab.sh <tag> "<pytest args>"'
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-lab}; T=${2:-}
if [ -n "$T" ]; then
  timeout -k 10 400 python -u -m pytest $T -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
  rc=$?; echo "T rc=$rc"; tail -1 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -10
  [ $rc -eq 0 ] || exit $rc
fi
for i in ${ROUNDS:-1 2}; do
  for v in new prev ${EXTRA_VARIANT:-}; do
    if [ $v = prev ]; then L=$PWD/styletransfer_amd/libstx_prev.so; else L=$PWD/styletransfer_amd/libstx.so; fi; if [ $v = ppb2 ]; then export STX_IN_PPB=2; else unset STX_IN_PPB; fi
    STX_LIB=$L timeout -k 10 200 python bench.py --steps 50 --warmup 5 --skip-cpu --skip-infer --lbfgs-steps 0 --gatys-run-iters 0 --fast-b64-steps 0 > gpurun_out/${tag}_$v$i.json 2>gpurun_out/${tag}_$v$i.err || { tail -3 gpurun_out/${tag}_$v$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${tag}_$v$i.json'));print('$v$i', 'gatys_ms', d['ms_per_step'], 'fast_ms', d['fast_st']['ms_per_step'])"
  done
done
