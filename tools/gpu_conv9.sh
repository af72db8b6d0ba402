# conv9 check: the 9x9 split kernels' tests + the ITN / conv suites, kernel times, fast_st A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv9_gpu.py tests/test_ops_gpu.py tests/test_itn_layers_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1 || { tail -40 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
bash tools/dbg_conv9.sh ${DBGV:-0} || exit 1
bash tools/ab_fast.sh STX_CONV9 ${ABR:-1}
