# weight-gradient side stream: the trainer tests, then the same-process A/B of the fast_st step
set -o pipefail
export STX_AB=1  # (the host path reads its A/B switches only under STX_AB=1: N.knob)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-side}
timeout -k 10 500 python -u -m pytest tests/test_side_stream_gpu.py tests/test_conv9_gpu.py tests/test_itn_masks_gpu.py tests/test_dp_gpu.py tests/test_video_gpu.py tests/test_parity_gpu.py tests/test_workflows_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_engine.py "STX_WGRAD_SIDE=0" "STX_WGRAD_SIDE=1" --rounds 7 --no-gatys > gpurun_out/${tag}_ab.log 2>&1; tail -3 gpurun_out/${tag}_ab.log
timeout -k 10 120 python tools/bench_conv9.py > gpurun_out/${tag}_c9.log 2>&1; tail -5 gpurun_out/${tag}_c9.log
timeout -k 10 400 python tools/ab_engine.py "STX_LOSS_STREAM=0" "STX_LOSS_STREAM=1" --rounds 7 > gpurun_out/${tag}_ls.log 2>&1; tail -4 gpurun_out/${tag}_ls.log
