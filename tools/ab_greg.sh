# STX_GREG_FORM variants of the 256^2 IN backward on the measurement library (one process each)
cd "$GRAFT_REPO_ROOT"
for f in 0 1 2 0 1 2; do
  echo "STX_GREG_FORM=$f"
  STX_GREG_FORM=$f STX_LIB=$PWD/styletransfer_amd/libstx_ab.so timeout -k 10 120 python tools/micro_in.py 2>&1 | grep instnorm
done
