set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for v in 1 2; do echo "fast $(timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proff -o run -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/proff.log 2>&1 || { tail -20 gpurun_out/proff.log; exit 1; }
