cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pw -o run -- python3 tools/bench_conv.py --only "wgrad res" > gpurun_out/pw.log 2>&1; echo rc $?
