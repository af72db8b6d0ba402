# probes: Gram-backward stream phases (STX_GB_DBG: 1 no A staging, 2 no MFMA, 4 no stores),
# the 64->3 data gradient, then the whole-step A/B of $AB and (TESTS=1) the -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0 2 4 6; do
  echo "== gbwd dbg=$d"
  STX_GB_DBG=$d timeout -k 10 120 python tools/bench_gbwd.py 2>&1 | grep -E "^C64 512x512|^C128 256x256" || exit 1
done
echo "== conv 64->3"
timeout -k 10 120 python tools/bench_conv.py --only "dgrad1_1" 2>&1 | grep -v amdgpu || exit 1
[ -n "$AB" ] && { timeout -k 10 400 python -u tools/ab_engine.py $AB 2>&1 | grep -E "^(gatys|fastst)" || exit 1; }
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
  rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/t.log | head -30
  exit $rc
fi
