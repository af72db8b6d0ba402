# A/B a runtime switch on the fast_st train step (B=8, graph replay), alternating arms.
#   gpurun -- 'bash tools/ab_fast.sh VAR [rounds]'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in $(seq ${2:-2}); do
  for v in 0 1; do
    out=$(env $1=$v timeout -k 5 200 python bench.py --fast-only --fast-steps 50 --warmup 3 2>/dev/null) || { echo "$1=$v FAILED"; exit 1; }
    echo "$1=$v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fast_st_images_per_s"], d["ms_per_step"])')"
  done
done
