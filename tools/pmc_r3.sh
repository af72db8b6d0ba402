# HBM bytes per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass, each
# pass its own run) for (1) the calibration kernels of known byte counts
# (tools/calib: 4-B and 16-B per lane loads, 4-B stores over 512 MiB) and (2) every
# kernel of an eager Gatys 512^2 iteration (tools/pmc_targets.py).  Summary:
# profiles/<tag>_pmc.json (tools/pmc_r3_summary.py).
#   gpurun -- 'bash tools/pmc_r3.sh r3'
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out profiles
tag=${1:-r3}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmccal_$c -o run \
    -- python3 tools/calib/pmc_calib.py > gpurun_out/pmccal_$c.log 2>&1 \
    || { echo "calib PMC $c failed"; tail -5 gpurun_out/pmccal_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmctgt_$c -o run \
    -- python3 tools/pmc_targets.py > gpurun_out/pmctgt_$c.log 2>&1 \
    || { echo "targets PMC $c failed"; tail -5 gpurun_out/pmctgt_$c.log; exit 1; }
done
python3 tools/pmc_r3_summary.py "$tag"
