cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/proff -o run -- python3 bench.py --fast-only --steps 30 --warmup 2 > gpurun_out/proff.log 2>&1; echo rc $?; tail -2 gpurun_out/proff.log
