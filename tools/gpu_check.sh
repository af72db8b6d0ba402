# one GPU round trip: split-conv + op parity tests, conv microbench, 1-GPU bench (no CPU leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
echo TESTS $rc; tail -3 gpurun_out/t.log; grep -E "^E |FAILED|Error" gpurun_out/t.log | head -20
if [ $rc -le 1 ]; then
  timeout -k 10 300 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids &&
  timeout -k 10 300 python bench.py --steps 50 --warmup 3 --skip-cpu 2>/dev/null
fi
if [ "$PROF" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
    -- python3 bench.py --steps 30 --warmup 3 --skip-cpu --skip-fast --skip-infer > gpurun_out/prof.log 2>&1
  echo PROF $?
fi
