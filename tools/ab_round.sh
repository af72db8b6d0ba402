set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for v in 1 2 3; do
 echo "new  $(timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"
 echo "base $(STX_BIAS_ONEPASS=0 timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"
done
