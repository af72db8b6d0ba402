# C = 256 Gram (gram_tri256_kernel) knob sweep on the measurement library: style_loss =
# partials + finalize (tools/bench_conv.py "gram C256"), per split target and store form
cd "$GRAFT_REPO_ROOT"
for st in 1 0; do
for b in 64 128 256; do
  echo "STX_GRAM256_BLOCKS=$b STX_GRAM256_STAGE=$st"
  STX_GRAM256_STAGE=$st STX_GRAM256_BLOCKS=$b STX_LIB=$PWD/styletransfer_amd/libstx_ab.so timeout -k 10 120 python tools/bench_conv.py --only "gram C256" 2>&1 | grep C256
done
done
echo "old kernel (STX_GRAM_TRI256=0)"
STX_GRAM_TRI256=0 STX_LIB=$PWD/styletransfer_amd/libstx_ab.so timeout -k 10 120 python tools/bench_conv.py --only "gram C256" 2>&1 | grep C256
