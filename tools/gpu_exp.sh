# Validation + experiments in one call: -m gpu suite (quiet), smoke, then the A/B probes
# named in $EXP (a ';'-separated list of commands run under timeouts).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "$TESTS" != 0 ]; then
  echo "== tests"
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
  [ $rc -le 1 ] || exit $rc
  echo "== smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
IFS=';' read -ra CMDS <<< "$EXP"
for c in "${CMDS[@]}"; do
  echo "== $c"
  timeout -k 10 400 bash -c "$c" 2>&1 | grep -v "^amdgpu\|UserWarning\|warnings.warn" || exit 1
done
