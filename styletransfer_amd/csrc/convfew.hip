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
        const float v = p.wt[(size_t)min(k, K - 1) * p.cout_pad + 32 * mt + l32];
        a[s][mt] = k < K ? v : 0.f;
      }
  } else {  // wl[k][32 MT] (k < 2 NST, zero rows past K)
    for (int i = tid; i < 2 * NST * 32 * MT; i += 256) {
      const int k = i / (32 * MT), c = i - k * 32 * MT;
      const float v = p.wt[(size_t)min(k, K - 1) * p.cout_pad + c];
      wl[i] = k < K ? v : 0.f;
    }
  }
  // input tile with zero halo
  {
    const auto rx = make_srd(xn, (uint32_t)(CF_CIN * plane_in) * 4u);
    for (int i = tid; i < CF_CIN * RH * RW; i += 256) {
      const int ci = i / (RH * RW), r = (i / RW) % RH, c = i % RW;
      const int y = oy0 - pad + r, x = ox0 - pad + c;
      const bool ok = y >= 0 && y < p.h && x >= 0 && x < p.w;
      tile[(ci * RH + r) * RWP + c] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(
                     rx, ok ? (uint32_t)(ci * plane_in + y * p.w + x) * 4u : BUF_OOB, 0, 0));
    }
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


// ---------------------------------------------------------------------------------
// 3x3 convolutions with <= 3 output channels (the data gradient of VGG conv1_1 to
// the image, 64 -> 3: stransfer/network.py:246-271 through autograd) on the fp32
// MFMA as a GEMM plus col2im: D[m = (s, kh, kw)][q] = sum_c W[s][c][kh][kw] x[c][q]
// over the tile's input pixels q (27 of an MFMA's 32 rows), then
// y[s][p] = sum_{kh,kw} D[(s, kh, kw)][p + (kh-1, kw-1)] from LDS.  The generic
// path pads cout 3 -> 64 (a 21x larger GEMM) or runs a VALU kernel; here the MFMA
// rows are the 27 (channel, tap) pairs and x is read once, straight into B.
//
// Tile: 8 output rows x 64 columns; its 10 x 66 input pixels are 30 items of
// (input row, 32-column block at offsets 0, 32, 34 -- the last overlaps), spread
// over the 4 waves.  D (27 x 10 x 66 floats, 71 KB) stays in LDS; every thread then
// forms 2 rows x 3 channels of one output column.
namespace {

constexpr int FO_TH = 8, FO_TW = 64, FO_RH = FO_TH + 2, FO_RW = FO_TW + 2, FO_RWP = FO_RW + 2;

template <int CIN>
__global__ void __launch_bounds__(256, 2) conv_fewout3_kernel(stx_conv_params p, int tiles_x) {
  constexpr int NST = CIN / 2;
  __shared__ float dt[27 * FO_RH * FO_RWP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const int oy0 = ty * FO_TH, ox0 = tx * FO_TW;
  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * CIN * plane_in;
  const bool relu_in = p.in_mode == STX_IN_RELU;
  // A: a[s] = W[m = l32][c = 2s + h], m = co*9 + kh*3 + kw (rows >= 9*cout are 0)
  const int m = l32, mco = m / 9, mt = m - mco * 9;
  // (unconditional loads from a valid address, then select: a predicated load would
  // be a branch with a vmcnt(0) join per element)
  float a[NST];
  const int mcl = min(mco, p.cout - 1);
#pragma unroll
  for (int s = 0; s < NST; ++s) {
    const int c = 2 * s + h;
    const float v = p.wt[(size_t)(c * 9 + mt) * p.cout_pad + mcl];
    a[s] = mco < p.cout ? v : 0.f;
  }
  const auto rx = make_srd(xn, (uint32_t)(CIN * plane_in) * 4u);
  // items wave, wave + 4, ...: double-buffered -- item i+1's 32 loads are in flight
  // while item i's MFMA chain runs (no spills: 2 x 32 + 32 + 16 VGPRs of state)
  constexpr int NITEM = FO_RH * 3;
  auto load_item = [&](int item, float (&buf)[NST]) {
    const int r = item / 3, nb = item - r * 3;
    const int c0 = nb == 0 ? 0 : (nb == 1 ? 32 : FO_RW - 32);  // last block overlaps
    const int iy = oy0 - 1 + r, ix = ox0 - 1 + c0 + l32;
    const bool ok = iy >= 0 && iy < p.h && ix >= 0 && ix < p.w;
    // out-of-image pixels read 0 through the descriptor's range check (no branches)
    const uint32_t vo = ok ? (uint32_t)(h * plane_in + iy * p.w + ix) * 4u : BUF_OOB;
#pragma unroll
    for (int s = 0; s < NST; ++s) {
      const float v = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo, (uint32_t)(2 * s) * plane_in * 4u, 0));
      buf[s] = relu_in ? fmaxf(v, 0.f) : v;
    }
  };
  auto run_item = [&](int item, const float (&buf)[NST]) {
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
    for (int s = 0; s < NST; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], buf[s], acc, 0, 0, 0);
    const int r = item / 3, nb = item - r * 3;
    const int c0 = nb == 0 ? 0 : (nb == 1 ? 32 : FO_RW - 32);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = 8 * (q >> 2) + 4 * h + (q & 3);
      if (row < 27) dt[(row * FO_RH + r) * FO_RWP + c0 + l32] = acc[q];
    }
  };
  float b0[NST], b1[NST];
  load_item(wave, b0);
  for (int it = wave; it < NITEM; it += 8) {
    if (it + 4 < NITEM) load_item(it + 4, b1);
    run_item(it, b0);
    if (it + 8 < NITEM) load_item(it + 8, b0);
    if (it + 4 < NITEM) run_item(it + 4, b1);
  }
  __syncthreads();
  const int ox = ox0 + (tid & 63), g = tid >> 6;
  const size_t plane = (size_t)p.ho * p.wo;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ry = 2 * g + j, oy = oy0 + ry;
    if (oy >= p.ho || ox >= p.wo) continue;
    for (int co = 0; co < p.cout; ++co) {
      float v = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          v += dt[((co * 9 + kh * 3 + kw) * FO_RH + ry + kh) * FO_RWP + (tid & 63) + kw];
      const size_t o = ((size_t)n * p.cout + co) * plane + (size_t)oy * p.wo + ox;
      if (p.bias) v += p.bias[co];
      if (p.accumulate) v += p.y[o];
      if (p.relu_out) v = fmaxf(v, 0.f);
      p.y[o] = v;
    }
  }
}

}  // namespace

// cout <= 3, 3x3 stride 1 pad 1, raw/relu input, cin = 64; bias / accumulate / relu_out
// epilogue only.  Returns -1 when not covered.
int conv2d_fewout(const stx_conv_params& p, hipStream_t st) {
  const bool ok = p.cout >= 1 && p.cout <= 3 && p.ks == 3 && p.stride == 1 && p.pad == 1 &&
                  (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) && p.cin == 64 &&
                  !p.mask && !p.aux && !p.p2_z && !p.up_dp && !p.pool_out && !p.acc_scale &&
                  !p.out_amax && p.wt_batch_stride == 0 && p.wt && p.hv == p.h && p.wv == p.w;
  if (!ok) return -1;
  const int tiles_x = (p.wo + FO_TW - 1) / FO_TW, tiles_y = (p.ho + FO_TH - 1) / FO_TH;
  hipLaunchKernelGGL((conv_fewout3_kernel<64>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0, st,
                     p, tiles_x);
  return check_launch("stx_conv2d(fewout)");
}

}  // namespace stx
