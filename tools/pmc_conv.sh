cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc1 -- python tools/bench_conv.py --only conv1_2 > gpurun_out/pmc1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/pmc2 -- python tools/bench_conv.py --only conv1_2 > gpurun_out/pmc2.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc3 -- python tools/bench_conv.py --only conv1_2 > gpurun_out/pmc3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc4 -- python tools/bench_conv.py --only conv1_2 > gpurun_out/pmc4.log 2>&1
echo rc $?
