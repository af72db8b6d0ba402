// Convolutions with 3 input channels on the fp32 MFMA (v_mfma_f32_32x32x2_f32):
// VGG conv1_1 (3 -> 64, 3x3; torchvision vgg19().features[0] via
// stransfer/network.py:246-271), ImageTransformNet conv0 (3 -> 32, 9x9,
// stransfer/network.py:525-527) and the data gradient of conv22 (its transpose, also
// 3 -> 32 9x9).
//
// With cin = 3 the implicit GEMM has K = 27 or 243 and the generic kernels pad the
// channel tile (3 -> 4/8) and spend their loop on staging.  Here the whole input
// tile (3 x (TH + KS-1) x (64 + KS-1)) sits in LDS once and the B operand is read
// straight out of it: for K-pair step s a lane's element is im2col row
// k = 2s + l/32 = (ci, kh, kw) at its pixel, i.e. one ds_read_b32 at a per-lane base
// plus a compile-time offset.  The A operand (weights, k-major slab rows) stays in
// registers for the kernel's lifetime.  fp32 products: no scaling, exact as the
// reference's fp32 conv up to summation order.
//
// A wave owns 2 output rows x 64 columns (4 N-blocks of 32 pixels) for all cout
// (MT = cout/32 M-tiles); a block is 4 waves = 8 rows x 64 columns.  Epilogue: bias,
// optional ReLU, plain stores (128-B rows per half-wave), optional amax group.
#include "common.h"
#include "conv_epi.h"

namespace stx {

namespace {

constexpr int CF_TW = 64, CF_TH = 8, CF_CIN = 3;

template <int KS, int MT>
__global__ void __launch_bounds__(256, 2) conv_fewin_kernel(stx_conv_params p, int tiles_x) {
  constexpr int KK = KS * KS, K = CF_CIN * KK, NST = (K + 1) / 2;
  constexpr int RH = CF_TH + KS - 1, RW = CF_TW + KS - 1, RWP = RW + 1;
  // A operand in registers when it fits (3x3: 14 x MT floats), else from LDS (9x9)
  constexpr bool AREG = NST * MT <= 64;
  __shared__ float tile[CF_CIN * RH * RWP];
  __shared__ float wl[AREG ? 1 : 2 * NST * 32 * MT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const int oy0 = ty * CF_TH, ox0 = tx * CF_TW;
  const int pad = KS / 2;
  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * CF_CIN * plane_in;

  // A fragments: a[s][mt] = wt[k = 2s + h][co = 32 mt + l32] (0 past K)
  float a[AREG ? NST : 1][MT];
  if constexpr (AREG) {
#pragma unroll
    for (int s = 0; s < NST; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int k = 2 * s + h;
        a[s][mt] = k < K ? p.wt[(size_t)k * p.cout_pad + 32 * mt + l32] : 0.f;
      }
  } else {  // wl[k][32 MT] (k < 2 NST, zero rows past K)
    for (int i = tid; i < 2 * NST * 32 * MT; i += 256) {
      const int k = i / (32 * MT), c = i - k * 32 * MT;
      wl[i] = k < K ? p.wt[(size_t)k * p.cout_pad + c] : 0.f;
    }
  }
  // input tile with zero halo
  for (int i = tid; i < CF_CIN * RH * RW; i += 256) {
    const int ci = i / (RH * RW), r = (i / RW) % RH, c = i % RW;
    const int y = oy0 - pad + r, x = ox0 - pad + c;
    tile[(ci * RH + r) * RWP + c] =
        (y >= 0 && y < p.h && x >= 0 && x < p.w) ? xn[(size_t)ci * plane_in + y * p.w + x] : 0.f;
  }
  __syncthreads();

  f32x16 acc[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][b][r] = 0.f;
  // N-block b = (row j = b >> 1, half = b & 1): pixel (2 wave + j, 32 half + l32)
  const float* base = tile + (2 * wave) * RWP + l32;
#pragma unroll
  for (int s = 0; s < NST; ++s) {
    const int k = 2 * s + h;  // this lane's im2col row (lanes h = 0/1 differ by one)
    const int kc = k < K ? k : K - 1;
    const int ci = kc / KK, kh = (kc % KK) / KS, kw = kc % KS;
    const int off = (ci * RH + kh) * RWP + kw;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float bv = base[off + (b >> 1) * RWP + (b & 1) * 32];
      if (k >= K) bv = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float av = AREG ? a[AREG ? s : 0][mt] : wl[k * 32 * MT + 32 * mt + l32];
        acc[mt][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[mt][b], 0, 0, 0);
      }
    }
  }

  // epilogue: rows co = 32 mt + 8 (r/4) + 4h + r%4, pixel (oy0 + 2 wave + j, ox0 + 32 half + l32)
  const size_t plane = (size_t)p.ho * p.wo;
  float* __restrict__ yn = p.y + (size_t)n * p.cout * plane;
  uint32_t vmax_u = 0u;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int oy = oy0 + 2 * wave + (b >> 1), ox = ox0 + 32 * (b & 1) + l32;
    const bool in = oy < p.ho && ox < p.wo;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * mt + 8 * (r >> 2) + 4 * h + (r & 3);
        float v = acc[mt][b][r];
        if (p.bias) v += p.bias[co];
        if (p.relu_out) v = fmaxf(v, 0.f);
        if (in && co < p.cout) {
          yn[(size_t)co * plane + (size_t)oy * p.wo + ox] = v;
          vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
        }
      }
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

template <int KS, int MT>
int launch_fewin(const stx_conv_params& p, hipStream_t st) {
  const int tiles_x = (p.wo + CF_TW - 1) / CF_TW, tiles_y = (p.ho + CF_TH - 1) / CF_TH;
  hipLaunchKernelGGL((conv_fewin_kernel<KS, MT>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0,
                     st, p, tiles_x);
  return check_launch("stx_conv2d(fewin)");
}

}  // namespace

// cin == 3, stride 1, pad ks/2, raw input, cout in {32, 64} (9x9: 32); bias / relu_out / out_amax
// epilogue only.  Returns -1 when the shape is not covered.
int conv2d_fewin(const stx_conv_params& p, hipStream_t st) {
  const bool ok = p.cin == CF_CIN && p.stride == 1 && p.pad == p.ks / 2 &&
                  p.in_mode == STX_IN_RAW && (p.cout == 32 || p.cout == 64) &&
                  !p.mask && !p.aux && !p.accumulate && !p.p2_z && !p.up_dp && !p.pool_out &&
                  !p.acc_scale && p.wt_batch_stride == 0 && p.wt && p.hv == p.h && p.wv == p.w;
  if (!ok) return -1;
  if (p.ks == 3) return p.cout == 64 ? launch_fewin<3, 2>(p, st) : launch_fewin<3, 1>(p, st);
  if (p.ks == 9 && p.cout == 32) return launch_fewin<9, 1>(p, st);
  return -1;
}

}  // namespace stx
