set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_conv.py --only "wgrad" || exit 1
for v in 1 0 1 0; do echo "fast S2=$v $(STX_WG16_S2=$v timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"; done
