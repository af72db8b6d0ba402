set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B="$GRAFT_REPO_ROOT/ab/libstx_base.so"
for v in 1 2 3; do
 echo "new  $(timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"
 echo "base $(STX_LIB=$B timeout -k 10 200 python bench.py --fast-only --steps 20 --warmup 3 2>/dev/null)"
done
