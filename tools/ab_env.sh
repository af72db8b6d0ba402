# A/B a runtime switch on the Gatys bench (alternating arms): bash tools/ab_env.sh VAR [rounds]
cd "$GRAFT_REPO_ROOT"
for r in $(seq ${2:-1}); do
for v in 0 1; do
  echo "$1=$v $(env $1=$v timeout -k 5 200 python bench.py --steps 50 --warmup 3 --skip-cpu --skip-fast --skip-infer 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["gatys_config2_run"]["value"], d["roofline"]["achieved"])')"
done
done
