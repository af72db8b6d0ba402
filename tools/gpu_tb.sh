# -m gpu suite, then the bench line (no CPU leg) and rocprofv3 --stats of the Gatys and
# fast_st legs (tools/gpu_base.sh).   gpurun --timeout 1000 -- 'bash tools/gpu_tb.sh <tag>'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-tb}
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -rf --timeout 120 --timeout-method thread ${TEST_ARGS:-} > gpurun_out/${tag}_t.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_base.sh "$tag"
