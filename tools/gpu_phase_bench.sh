cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2; do
for v in 0 default; do
  if [ $v = 0 ]; then export STX_V2_PHASE=0; else unset STX_V2_PHASE; fi
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --skip-cpu --skip-fast --skip-infer > gpurun_out/bab_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/bab_$v.json'));r=d['roofline']
print('$v', d['value'], 'fwd', r['fwd_ms'], r['frac'], 'dg', r['dominant_kernel']['ms'], r['dominant_kernel']['frac'], 'cfg2', d['gatys_config2_run']['value'])"
done
done
