cd $GRAFT_REPO_ROOT
for d in 0 4 1 5; do STX_CONV16_DBG=$d timeout -k 5 120 python tools/bench_conv.py --only "gram C64 512" 2>&1 | grep -v amdgpu.ids | sed "s/^/dbg$d /"; done
