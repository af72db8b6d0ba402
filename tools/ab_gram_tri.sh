cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in 256 512; do
  echo "TRI=$v $(STX_GRAM_TRI_BLOCKS=$v timeout -k 5 200 python bench.py --steps 50 --warmup 3 --skip-cpu --skip-fast --skip-infer 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["gatys_config2_run"]["value"])')"
done; done
