# conv9_out3 A/B: the CLI train->convert workflow test and the 9x9 microbenchmark with the
# in-tree library and with a build of the previous conv9 kernel (STX_LIB)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=tests/test_workflows_gpu.py::test_fast_st_cli_train_then_convert
for v in new old; do
  if [ $v = old ]; then export STX_LIB=$PWD/styletransfer_amd/libstx_c9old.so; fi
  timeout -k 10 200 python -u -m pytest $T tests/test_conv9_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/c9_$v.log 2>&1
  echo "$v rc=$?"; tail -1 gpurun_out/c9_$v.log; grep "convert-image vs" gpurun_out/c9_$v.log
  timeout -k 10 120 python tools/bench_conv9.py > gpurun_out/c9b_$v.log 2>&1; tail -4 gpurun_out/c9b_$v.log
done
