// fp32 k-major GEMM weight slab (the fp32 MFMA conv kernels' B operand), shared by
// stx_conv_weight_prep (conv.hip) and the batched prep (conv16.hip).
#pragma once

namespace stx {

// slab[row][col], row = ci*kk + kh*ks + kw (transpose: co*kk + flipped tap), col = co
// (transpose: ci); padded rows / columns are zero.  Elements i0, i0 + step, ...
__device__ __forceinline__ void weight_prep32_body(const float* __restrict__ w,
                                                   float* __restrict__ wt, int cout, int cin,
                                                   int ks, int transpose, int rows_pad,
                                                   int cols_pad, long long i0, long long step) {
  const int total = rows_pad * cols_pad;  // < 2^31: 32-bit index math
  const int kk = ks * ks;
  for (int i = (int)i0; i < total; i += (int)step) {
    const int col = (int)((unsigned)i % (unsigned)cols_pad);
    const int row = (int)((unsigned)i / (unsigned)cols_pad);
    const int c_in = row / kk, r = row % kk, kh = r / ks, kw = r % ks;
    float v = 0.f;
    if (!transpose) {
      if (c_in < cin && col < cout) v = w[(((size_t)col * cin + c_in) * ks + kh) * ks + kw];
    } else {
      // data-gradient weights: flipped taps, channels swapped
      if (c_in < cout && col < cin)
        v = w[(((size_t)c_in * cin + col) * ks + (ks - 1 - kh)) * ks + (ks - 1 - kw)];
    }
    wt[i] = v;
  }
}

}  // namespace stx
