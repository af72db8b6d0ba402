# L-BFGS loop: its GPU tests, the bench leg, and rocprofv3 --stats of the leg.
#   gpurun -- 'bash tools/gpu_lb.sh <tag>'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-lb}
timeout -k 10 300 python -u -m pytest tests/test_lbfgs_gpu.py tests/test_workflows_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1
rc=$?; echo "T rc=$rc"; tail -2 gpurun_out/${tag}_t.log; grep -E "^(FAILED|ERROR)|^E  " gpurun_out/${tag}_t.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run \
  -- python3 bench.py --steps 3 --warmup 1 --gatys-run-iters 0 --skip-cpu --skip-fast --skip-infer --lbfgs-fill 40 > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --gatys-run-iters 0 --skip-cpu --skip-fast --skip-infer --lbfgs-fill 40 > gpurun_out/${tag}.json 2> gpurun_out/${tag}.err || { tail gpurun_out/${tag}.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${tag}.json'));print(d['value'], d['gatys_lbfgs'])"
