# Round-3 evidence (tools/gpu_round3.sh) followed by the experiments in $EXP.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round3.sh || exit $?
IFS=';' read -ra CMDS <<< "$EXP"
for c in "${CMDS[@]}"; do
  echo "== $c"
  timeout -k 10 300 bash -c "$c" 2>&1 | grep -v "^amdgpu\|UserWarning\|warnings.warn\|amdgpu.ids" || exit 1
done
