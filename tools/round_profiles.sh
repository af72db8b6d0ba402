# End-of-round measurement set (1 GPU): default bench line, rocprofv3 kernel stats of
# the same command, PMC bytes of the roofline launch, per-iteration / per-step
# breakdowns.  gpurun -- 'bash tools/round_profiles.sh r2'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-r2}
echo "== bench"
timeout -k 10 500 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
  || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
echo "== rocprof stats of the same command"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench_$tag -o run \
  -- python3 bench.py > gpurun_out/prof_bench_$tag.log 2>&1 || { tail -20 gpurun_out/prof_bench_$tag.log; exit 1; }
tail -1 gpurun_out/prof_bench_$tag.log | cut -c1-300
echo "== pmc"
bash tools/pmc_roofline.sh $tag > gpurun_out/pmc_$tag.log 2>&1 || { tail -10 gpurun_out/pmc_$tag.log; exit 1; }
echo "== breakdowns"
bash tools/prof_gatys.sh ${tag}g > /dev/null && bash tools/prof_fast.sh ${tag}f > /dev/null
tail -1 gpurun_out/breakdown_${tag}g.txt; tail -1 gpurun_out/breakdown_${tag}f.txt
