# whole-step A/B (tools/ab_engine.py) of the variants given in $AB, then (TESTS=1) the
# -m gpu suite.   gpurun -- 'AB="STX_FIN_BATCH=0 STX_FIN_BATCH=1" TESTS=1 bash tools/gpu_ab2.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== ab: $AB"
timeout -k 10 400 python -u tools/ab_engine.py $AB > gpurun_out/ab2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab2.log | tail -20
[ $rc -eq 0 ] || exit $rc
if [ "$TESTS" = 1 ]; then
  echo "== tests"
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
fi
exit $rc
