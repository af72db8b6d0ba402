// Streaming split-MFMA Gram backward (gbwd16.hip), launched by stx_conv2d's 1x1 mode.
#pragma once
#include "common.h"

namespace stx {

struct Gb16 {
  const float* coef;      // [n][C][pitch]  A[c][co]
  long long coef_bs;      // floats between images
  int pitch;
  const float* z;         // [n][C][h][w]
  const float* z_amax;    // amax group >= max|z|
  const float* acc_scale; // device scalar or NULL (1)
  const float* up_dp;     // [n][C][h/2][w/2] or NULL
  const float* aux;       // [n][C][h][w] or NULL
  float aux_scale;
  float* out;             // [n][C][h][w]
  float* out_amax;        // amax group or NULL
  int h, w;
};

// C in {64, 128}, h even, w % 32 == 0 (the caller checks the contract)
int gram_bwd16_launch(const Gb16& p, int nimg, int c, hipStream_t st);

}  // namespace stx
