set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export STX_BENCH_SAME_DEVICE=1 STX_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --fast-only --steps 10 --warmup 2 > gpurun_out/dp2.log 2>&1 || { tail -30 gpurun_out/dp2.log; exit 1; }
grep fast_st gpurun_out/dp2.log
STX_FAST_GRAPH=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --fast-only --steps 10 --warmup 2 > gpurun_out/dp2e.log 2>&1 || { tail -30 gpurun_out/dp2e.log; exit 1; }
grep fast_st gpurun_out/dp2e.log
