# Issue/stall counters per dispatch of an eager Gatys 512^2 iteration (tools/pmc_targets.py):
# pass 1 = where the waves' cycles go (parked on s_waitcnt/barrier vs issue-stalled vs
# issuing), the MFMA pipe's busy cycles and the shader clock; pass 2 = instruction mix.
# Each pass its own run.  Summary: tools/pmc_sq_summary.py -> profiles/<tag>_sq.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out profiles
tag=${1:-r3}
shift || true
targs="$*"   # extra tools/pmc_targets.py arguments (e.g. --fast)
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmcsq_$i -o run \
    -- python3 tools/pmc_targets.py $targs > gpurun_out/pmcsq_$i.log 2>&1 \
    || { echo "SQ PMC pass $i failed"; tail -5 gpurun_out/pmcsq_$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_sq_summary.py "$tag"
