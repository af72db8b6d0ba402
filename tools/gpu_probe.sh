# probes: the Gram-backward schedules per launch, then the whole-step A/B of $AB and
# (TESTS=1) the -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "== gbwd"
timeout -k 10 120 python tools/bench_gbwd.py 2>&1 | grep -v amdgpu || exit 1
if [ -n "$AB" ]; then timeout -k 10 400 python -u tools/ab_engine.py $AB 2>&1 | grep -E "^(gatys|fastst)" || exit 1; fi
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
  exit $rc
fi
