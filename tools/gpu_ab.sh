# A/B + correctness of a kernel change on one MI355X: the v1/v2 split-conv A/B
# (tools/ab_v2.py, bitwise comparison + timings), then the -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== ab"
timeout -k 10 300 python -u tools/ab_v2.py > gpurun_out/ab.log 2>&1; rc=$?
cat gpurun_out/ab.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
if [ "$TESTS" = 1 ]; then
  echo "== tests"
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
fi
exit $rc
