cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for v in 0 1 2; do
  echo "IN_CFG=$v $(STX_IN_CFG=$v timeout -k 5 200 python bench.py --fast-only --fast-steps 50 --warmup 3 2>/dev/null)"
done; done
