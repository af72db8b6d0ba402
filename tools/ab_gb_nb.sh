cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in 0 1; do
  g=$(STX_GB_NB=$v timeout -k 5 200 python bench.py --steps 50 --warmup 3 --skip-cpu --skip-fast --skip-infer 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["gatys_config2_run"]["value"])')
  f=$(STX_GB_NB=$v timeout -k 5 200 python bench.py --fast-only --fast-steps 50 --warmup 3 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["fast_st_images_per_s"])')
  echo "GB_NB=$v gatys $g fast $f"
done; done
