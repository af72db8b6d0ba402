# one GPU round trip: parity tests, conv microbench, 1-GPU bench (no CPU leg)
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -q -m gpu -x > gpurun_out/t.log 2>&1
rc=$?
echo TESTS $rc; tail -2 gpurun_out/t.log; grep -E "^E |FAILED" gpurun_out/t.log | head -8
if [ $rc -le 1 ]; then
  timeout -k 10 300 python tools/bench_conv.py 2>&1 | grep -v amdgpu.ids &&
  timeout -k 10 300 python bench.py --steps 50 --warmup 3 --skip-cpu 2>/dev/null
fi
