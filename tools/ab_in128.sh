# STX_IN128 block shapes of the 128^2 InstanceNorm kernels on the measurement library
cd "$GRAFT_REPO_ROOT"
for f in 0 2 3 0 2 3; do
  echo "STX_IN128=$f"
  STX_IN128=$f STX_LIB=$PWD/styletransfer_amd/libstx_ab.so timeout -k 10 120 python tools/micro_in.py 128 2>&1 | grep instnorm
done
