cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export STX_CONV16_DBG=${DBG:-1}
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/$1 -o run -- python3 tools/bench_conv.py --only "${ONLY:-gram C64 512}" > gpurun_out/$1.log 2>&1; echo "$1 rc $?"; }
rm -rf gpurun_out/pmc*
run pmc1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" &&
run pmc2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES" &&
run pmc3 "SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
