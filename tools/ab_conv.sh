# Same-box A/B of the conv microbench: ab/libstx_base.so vs the in-tree libstx.so.
#   gpurun -- 'bash tools/ab_conv.sh "conv1_2|conv2_2|res conv"'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
pat=${1:-conv}
for rep in 1 2; do
  for lib in ab/libstx_base.so styletransfer_amd/libstx.so; do
    echo "== $lib (rep $rep)"
    for only in $(echo "$pat" | tr '|' ' '); do
      STX_LIB=$lib STX_LIB_PARTIAL=1 timeout -k 10 120 python tools/bench_conv.py --only "$only" 2>&1 | grep -v amdgpu || exit 1
    done
  done
done
