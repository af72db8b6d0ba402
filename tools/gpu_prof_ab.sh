# rocprofv3 --stats of the fast_st leg with the in-tree library and libstx_prev.so
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-pab}
for v in new prev; do
  if [ $v = prev ]; then export STX_LIB=$PWD/styletransfer_amd/libstx_prev.so; else unset STX_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_$v -o run \
    -- python3 bench.py --fast-only --steps 20 --warmup 2 > gpurun_out/${tag}_$v.log 2>&1 || { tail -5 gpurun_out/${tag}_$v.log; exit 1; }
done
