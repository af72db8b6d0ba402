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
#include <stdlib.h>

#include "common.h"
#include "conv_epi.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

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

// ---------------------------------------------------------------------------------
// The same convolutions on the fp16 hi/lo split MFMA (v_mfma_f32_32x32x16_f16, three
// products per K=16 step; conv16.hip explains the split).  The scales are block-local:
// every block computes max|x| over its own input tile and max|W| over the weights
// before splitting, so no producer has to annotate the input -- each block's outputs
// depend only on its tile, and the de-scale 2^(ex + ew - 30) is exact.  The input
// tile is split once into fp16 hi/lo planes in LDS; a lane's B fragment (8 im2col
// rows k = 16t + 8h + e at its pixel) is 8 16-bit LDS reads per plane at compile-time
// offsets (one of two per element, by lane half); the A fragments (weights,
// [t][plane][h][co][8]) are one ds_read_b128 each.  A wave owns 2 output rows x 64
// columns as 4 N-blocks of 32 pixels and stores each N-block's outputs right after
// its MFMAs, so the store stream overlaps the next N-block's matrix work.  K = 27
// (3x3) is 2 steps, K = 243 (9x9) 16: 5x fewer matrix cycles than the fp32 MFMA.
template <int KS>
struct Few16 {
  static constexpr int KK = KS * KS, K = CF_CIN * KK, KST = (K + 15) / 16;
  static constexpr int RH = CF_TH + KS - 1, RW = CF_TW + KS - 1, RWP = RW + 1;
  static constexpr int NT = CF_CIN * RH * RWP;        // LDS tile elements per plane
  static constexpr int NIN = CF_CIN * RH * RW;        // loaded tile elements
  static constexpr int NR = (NIN + 255) / 256;
  // LDS offset of im2col row k relative to the pixel's (0, 0) tap, or -1 past K
  static constexpr int koff(int k) {
    return k < K ? ((k / KK) * RH + (k % KK) / KS) * RWP + (k % KS) : -1;
  }
};

template <int KS, int MT>
__global__ void __launch_bounds__(256, 2) conv_fewin16_kernel(stx_conv_params p, int tiles_x) {
  using F = Few16<KS>;
  constexpr int KST = F::KST, NCO = 32 * MT;
  constexpr int NW = KST * 2 * NCO * 8;                // A elements (t, h, co, e)
  constexpr int NWR = (NW + 255) / 256;
  __shared__ _Float16 tile16[2][F::NT];
  __shared__ __attribute__((aligned(16))) _Float16 wa[KST][2][2][NCO][8];  // [t][P][h][co][e]
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const int oy0 = ty * CF_TH, ox0 = tx * CF_TW;
  constexpr int pad = KS / 2;
  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * CF_CIN * plane_in;

  // input tile (zero halo through the descriptor's range check) and weights into
  // registers, with their maxima
  float xv[F::NR], wv[NWR];
  float mx = 0.f, mw = 0.f;
  {
    const auto rx = make_srd(xn, (uint32_t)(CF_CIN * plane_in) * 4u);
#pragma unroll
    for (int r = 0; r < F::NR; ++r) {
      const int i = tid + 256 * r;
      const int ci = i / (F::RH * F::RW), rr = (i / F::RW) % F::RH, cc = i % F::RW;
      const int y = oy0 - pad + rr, x = ox0 - pad + cc;
      const bool ok = i < F::NIN && y >= 0 && y < p.h && x >= 0 && x < p.w;
      xv[r] = buf_ld(rx, ok ? (uint32_t)(ci * plane_in + y * p.w + x) * 4u : BUF_OOB);
      mx = fmaxf(mx, fabsf(xv[r]));
    }
#pragma unroll
    for (int r = 0; r < NWR; ++r) {
      const int u = tid + 256 * r;
      const int e = u & 7, co = (u >> 3) % NCO, hh = (u / (8 * NCO)) & 1, t = u / (16 * NCO);
      const int k = 16 * t + 8 * hh + e;
      const bool ok = u < NW && k < F::K && co < p.cout;
      wv[r] = ok ? p.wt[(size_t)k * p.cout_pad + co] : 0.f;
      mw = fmaxf(mw, fabsf(wv[r]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    mw = fmaxf(mw, __shfl_xor(mw, o, 64));
  }
  if (lane == 0) {
    red[wave] = mx;
    red[4 + wave] = mw;
  }
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  mw = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
  int ex = 0, ew = 0;
  frexpf(mx, &ex);
  frexpf(mw, &ew);
  ex = min(max(ex, -60), 60);
  ew = min(max(ew, -60), 60);
  const float sx = __builtin_ldexpf(1.f, 15 - ex), sw = __builtin_ldexpf(1.f, 15 - ew);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
  // split into the LDS planes
#pragma unroll
  for (int r = 0; r < F::NR; ++r) {
    const int i = tid + 256 * r;
    if (i < F::NIN) {
      const int ci = i / (F::RH * F::RW), rr = (i / F::RW) % F::RH, cc = i % F::RW;
      const int o = (ci * F::RH + rr) * F::RWP + cc;
      const float v = xv[r] * sx;
      const _Float16 vh = (_Float16)v;
      tile16[0][o] = vh;
      tile16[1][o] = (_Float16)(v - (float)vh);
    }
  }
#pragma unroll
  for (int r = 0; r < NWR; ++r) {
    const int u = tid + 256 * r;
    if (u < NW) {
      const int e = u & 7, co = (u >> 3) % NCO, hh = (u / (8 * NCO)) & 1, t = u / (16 * NCO);
      const float v = wv[r] * sw;
      const _Float16 vh = (_Float16)v;
      wa[t][0][hh][co][e] = vh;
      wa[t][1][hh][co][e] = (_Float16)(v - (float)vh);
    }
  }
  __syncthreads();

  const size_t plane = (size_t)p.ho * p.wo;
  const uint32_t pb = (uint32_t)plane * 4u;
  // stores through a descriptor: per-lane pixel offset + per-register row constant
  const auto ry = make_srd(p.y + (size_t)n * p.cout * plane, (uint32_t)p.cout * pb);
  // this lane's output rows' biases, loaded once (not per stored element)
  float bias_r[MT][16];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = 32 * mt + 8 * (r >> 2) + 4 * h + (r & 3);
      bias_r[mt][r] = (p.bias && co < p.cout) ? p.bias[co] : 0.f;
    }
  uint32_t vmax_u = 0u;
  // fused Gram partial (stx_conv_params.gram_part; KS == 3, cout == 64): each N-block's
  // 4 x 32 pixels go to gT as fp32 [channel][pixel], waves 0..2 add their 32 x 32 block
  // of the upper triangle (fp16 hi/lo MFMA at the N-block's own power-of-two scale,
  // de-scaled into g)
  constexpr bool GRAM = KS == 3 && MT == 2;
  using GPL = GramPlanes<128>;
  __shared__ __attribute__((aligned(16))) char gsm[GRAM ? GPL::BYTES : 16];
  _Float16* gH = reinterpret_cast<_Float16*>(gsm);
  float* gred = reinterpret_cast<float*>(gsm + (GRAM ? GPL::BYTES - 16 : 0));
  const bool gram = GRAM && p.gram_part;
  f32x16 g;
#pragma unroll
  for (int q = 0; q < 16; ++q) g[q] = 0.f;
#pragma unroll 1
  for (int b = 0; b < 4; ++b) {
    const int row = 2 * wave + (b >> 1), col = 32 * (b & 1) + l32;
    const int base = row * F::RWP + col;
    f32x16 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
#pragma unroll
    for (int t = 0; t < KST; ++t) {
      f16x8 bh, bl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o0 = F::koff(16 * t + e), o1 = F::koff(16 * t + 8 + e);
        const int o = h ? o1 : o0;
        const bool ok = o >= 0;
        const int oo = ok ? o : 0;
        const _Float16 zh = (_Float16)0.f;
        bh[e] = ok ? tile16[0][base + oo] : zh;
        bl[e] = ok ? tile16[1][base + oo] : zh;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(&wa[t][0][h][32 * mt + l32][0]);
        const f16x8 al = *reinterpret_cast<const f16x8*>(&wa[t][1][h][32 * mt + l32][0]);
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[mt], 0, 0, 0);
      }
    }
    // this N-block's outputs: rows co = 32 mt + 8 (r/4) + 4h + r%4, pixel (row, col)
    const int oy = oy0 + row, ox = ox0 + col;
    const bool in = oy < p.ho && ox < p.wo;
    const uint32_t vo = in ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row_c = 32 * mt + 8 * (r >> 2) + (r & 3);  // co without the lane half
        float v = fmaf(acc[mt][r], descale, bias_r[mt][r]);
        if (p.relu_out) v = fmaxf(v, 0.f);
        buf_st(ry, vo + (uint32_t)row_c * pb, v);
        if (in && row_c + 4 * h < p.cout) vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
        if constexpr (GRAM) acc[mt][r] = in ? v : 0.f;
      }
    if constexpr (GRAM) if (gram) {
      // this N-block's 4 x 32 pixels at their own scale: max, split into the planes, then
      // waves 0..2 add their upper-triangle block (de-scaled into g)
      uint32_t m = 0u;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) m = max(m, __float_as_uint(acc[mt][r]) & 0x7fffffffu);
      const int e = gram_block_exp(m, gred);  // (its barrier also retires the last block's reads)
      const float gs = __builtin_ldexpf(1.f, 15 - e);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          gram_put(gH, GPL::HP, 32 * mt + 8 * (r >> 2) + 4 * h + (r & 3), wave * 32 + l32,
                   acc[mt][r] * gs);
      lds_sync();  // (the y stores stay in flight)
      if (wave < 3) {
        f32x16 gc;
#pragma unroll
        for (int q = 0; q < 16; ++q) gc[q] = 0.f;
        gram_mma<8>(gH, GPL::HP, wave, h, l32, gc);
        const float ginv = __builtin_ldexpf(1.f, 2 * e - 30);
#pragma unroll
        for (int q = 0; q < 16; ++q) g[q] = fmaf(gc[q], ginv, g[q]);
      }
    }
  }
  if constexpr (GRAM) if (gram) {
    if (p.gram_cnt)
      gram_store_grouped(p, blockIdx.z, blockIdx.x, gridDim.x, g, wave, h, l32, gred);
    else
      gram_store_lds<256>(p.gram_part + ((size_t)blockIdx.z * gridDim.x + blockIdx.x) * 4096, g,
                          wave, h, l32, reinterpret_cast<float*>(gsm));
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

// ---------------------------------------------------------------------------------
// conv1_1 (3x3, cin 3, cout 32 * MT) on the split MFMA with TRANSPOSED accumulators:
// the MFMA operands are swapped (A = the im2col pixel fragment, B = the weight
// fragment), so D[pixel][co] -- a lane holds one output channel and, per register r,
// pixel 8(r/4) + 4h + r%4 of its 32-pixel N-block.  Two things follow:
//  * stores are 16 B per lane (four consecutive pixels of one channel) instead of 4 B;
//  * the fused Gram partial needs no LDS transpose: with the K (pixel) order of a
//    16-deep step taken as the lane's own registers 8t..8t+7 (pixels 16t + 8(e/4) + 4h
//    + e%4 -- a bijection onto [16t, 16t + 16) shared by both operands), the A fragment
//    of channel block I and the B fragment of block J are both just the lane's split
//    registers, so each wave adds all three upper 32 x 32 blocks of its own pixels,
//    from registers, at its own power-of-two scale (no barrier per N-block); the four
//    waves' partials are summed once per block through LDS in a fixed order.
// wo % 4 == 0 (whole 16-B groups); otherwise the lane-per-pixel kernel above runs.

template <int MT>
__global__ void __launch_bounds__(256, 2) conv_fewin16t_kernel(stx_conv_params p, int tiles_x) {
  constexpr int KS = 3;
  using F = Few16<KS>;
  constexpr int KST = F::KST, NCO = 32 * MT;
  constexpr int NW = KST * 2 * NCO * 8;
  constexpr int NWR = (NW + 255) / 256;
  constexpr bool GRAM = MT == 2;
  __shared__ _Float16 tile16[2][F::NT];
  __shared__ __attribute__((aligned(16))) _Float16 wa[KST][2][2][NCO][8];  // [t][P][h][co][e]
  __shared__ float red[8];
  __shared__ __attribute__((aligned(16))) float gsum[GRAM ? 4 * 3 * 1024 : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, n = blockIdx.z;
  const int oy0 = ty * CF_TH, ox0 = tx * CF_TW;
  constexpr int pad = KS / 2;
  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * CF_CIN * plane_in;

  float xv[F::NR], wv[NWR];
  float mx = 0.f, mw = 0.f;
  {
    const auto rx = make_srd(xn, (uint32_t)(CF_CIN * plane_in) * 4u);
#pragma unroll
    for (int r = 0; r < F::NR; ++r) {
      const int i = tid + 256 * r;
      const int ci = i / (F::RH * F::RW), rr = (i / F::RW) % F::RH, cc = i % F::RW;
      const int y = oy0 - pad + rr, x = ox0 - pad + cc;
      const bool ok = i < F::NIN && y >= 0 && y < p.h && x >= 0 && x < p.w;
      xv[r] = buf_ld(rx, ok ? (uint32_t)(ci * plane_in + y * p.w + x) * 4u : BUF_OOB);
      mx = fmaxf(mx, fabsf(xv[r]));
    }
#pragma unroll
    for (int r = 0; r < NWR; ++r) {
      const int u = tid + 256 * r;
      const int e = u & 7, co = (u >> 3) % NCO, hh = (u / (8 * NCO)) & 1, t = u / (16 * NCO);
      const int k = 16 * t + 8 * hh + e;
      const bool ok = u < NW && k < F::K && co < p.cout;
      wv[r] = ok ? p.wt[(size_t)k * p.cout_pad + co] : 0.f;
      mw = fmaxf(mw, fabsf(wv[r]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    mw = fmaxf(mw, __shfl_xor(mw, o, 64));
  }
  if (lane == 0) {
    red[wave] = mx;
    red[4 + wave] = mw;
  }
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  mw = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
  int ex = 0, ew = 0;
  frexpf(mx, &ex);
  frexpf(mw, &ew);
  ex = min(max(ex, -60), 60);
  ew = min(max(ew, -60), 60);
  const float sx = __builtin_ldexpf(1.f, 15 - ex), sw = __builtin_ldexpf(1.f, 15 - ew);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
#pragma unroll
  for (int r = 0; r < F::NR; ++r) {
    const int i = tid + 256 * r;
    if (i < F::NIN) {
      const int ci = i / (F::RH * F::RW), rr = (i / F::RW) % F::RH, cc = i % F::RW;
      const int o = (ci * F::RH + rr) * F::RWP + cc;
      const float v = xv[r] * sx;
      const _Float16 vh = (_Float16)v;
      tile16[0][o] = vh;
      tile16[1][o] = (_Float16)(v - (float)vh);
    }
  }
#pragma unroll
  for (int r = 0; r < NWR; ++r) {
    const int u = tid + 256 * r;
    if (u < NW) {
      const int e = u & 7, co = (u >> 3) % NCO, hh = (u / (8 * NCO)) & 1, t = u / (16 * NCO);
      const float v = wv[r] * sw;
      const _Float16 vh = (_Float16)v;
      wa[t][0][hh][co][e] = vh;
      wa[t][1][hh][co][e] = (_Float16)(v - (float)vh);
    }
  }
  __syncthreads();

  const size_t plane = (size_t)p.ho * p.wo;
  const uint32_t pb = (uint32_t)plane * 4u;
  const auto ry = make_srd(p.y + (size_t)n * p.cout * plane, (uint32_t)p.cout * pb);
  float bias_l[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int co = 32 * mt + l32;
    bias_l[mt] = (p.bias && co < p.cout) ? p.bias[co] : 0.f;
  }
  uint32_t vmax_u = 0u;
  const bool gram = GRAM && p.gram_part;
  f32x16 g[3];
#pragma unroll
  for (int b3 = 0; b3 < 3; ++b3)
#pragma unroll
    for (int q = 0; q < 16; ++q) g[b3][q] = 0.f;
#pragma unroll 1
  for (int b = 0; b < 4; ++b) {
    const int row = 2 * wave + (b >> 1), col0 = 32 * (b & 1);
    const int base = row * F::RWP + col0 + l32;  // the B-gather pixel of this lane
    f32x16 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
#pragma unroll
    for (int t = 0; t < KST; ++t) {
      f16x8 bh, bl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o0 = F::koff(16 * t + e), o1 = F::koff(16 * t + 8 + e);
        const int o = h ? o1 : o0;
        const bool ok = o >= 0;
        const int oo = ok ? o : 0;
        const _Float16 zh = (_Float16)0.f;
        bh[e] = ok ? tile16[0][base + oo] : zh;
        bl[e] = ok ? tile16[1][base + oo] : zh;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(&wa[t][0][h][32 * mt + l32][0]);
        const f16x8 al = *reinterpret_cast<const f16x8*>(&wa[t][1][h][32 * mt + l32][0]);
        // D[pixel][co]: the pixel fragment is the A operand, the weights the B operand
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, ah, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl, ah, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh, al, acc[mt], 0, 0, 0);
      }
    }
    // outputs: lane's channel 32 mt + l32; registers 4q..4q+3 -> pixels 8q + 4h + 0..3
    const int oy = oy0 + row;
    uint32_t wmax = 0u;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int co = 32 * mt + l32;
      const bool cok = co < p.cout;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ox = ox0 + col0 + 8 * q + 4 * h;
        const bool in = cok && oy < p.ho && ox < p.wo;
        f32x4 v4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = fmaf(acc[mt][4 * q + e], descale, bias_l[mt]);
          if (p.relu_out) v = fmaxf(v, 0.f);
          v4[e] = v;
          const uint32_t bits = in ? (__float_as_uint(v) & 0x7fffffffu) : 0u;
          vmax_u = max(vmax_u, bits);
          wmax = max(wmax, bits);
          acc[mt][4 * q + e] = in ? v : 0.f;  // the Gram's copy: pixels outside count 0
        }
        const uint32_t off = in ? (uint32_t)co * pb + (uint32_t)(oy * p.wo + ox) * 4u : BUF_OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v4), ry, off, 0, 0);
      }
    }
    if constexpr (GRAM) if (gram) {
      // this wave's 64 channels x 32 pixels at the wave's own power-of-two scale
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
      int e2 = 0;
      frexpf(__uint_as_float(wmax), &e2);
      e2 = min(max(e2, -60), 60);
      const float gs = __builtin_ldexpf(1.f, 15 - e2);
      f16x8 fh[2][2], fl[2][2];  // [mt][t]
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = acc[mt][8 * t + e] * gs;
            const _Float16 vh = (_Float16)v;
            fh[mt][t][e] = vh;
            fl[mt][t][e] = (_Float16)(v - (float)vh);
          }
      const float ginv = __builtin_ldexpf(1.f, 2 * e2 - 30);
#pragma unroll
      for (int b3 = 0; b3 < 3; ++b3) {
        const int I = b3 == 2 ? 1 : 0, J = b3 == 0 ? 0 : 1;
        f32x16 gc;
#pragma unroll
        for (int q = 0; q < 16; ++q) gc[q] = 0.f;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          gc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[I][t], fh[J][t], gc, 0, 0, 0);
          gc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fh[I][t], fl[J][t], gc, 0, 0, 0);
          gc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fl[I][t], fh[J][t], gc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) g[b3][q] = fmaf(gc[q], ginv, g[b3][q]);
      }
    }
  }
  if constexpr (GRAM) if (gram) {
    // the four waves' partials, summed in wave order; waves 0..2 store one block each
#pragma unroll
    for (int b3 = 0; b3 < 3; ++b3)
      *reinterpret_cast<f32x16*>(&gsum[((wave * 3 + b3) * 64 + lane) * 16]) = g[b3];
    lds_sync();  // (the y stores stay in flight)
    f32x16 s;
#pragma unroll
    for (int q = 0; q < 16; ++q) s[q] = 0.f;
    if (wave < 3) {
      s = *reinterpret_cast<const f32x16*>(&gsum[((0 * 3 + wave) * 64 + lane) * 16]);
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const f32x16 o = *reinterpret_cast<const f32x16*>(&gsum[((w * 3 + wave) * 64 + lane) * 16]);
#pragma unroll
        for (int q = 0; q < 16; ++q) s[q] += o[q];
      }
    }
    if (p.gram_cnt)  // (gsum's first word becomes the reducer flag after the helper's barrier)
      gram_store_grouped(p, blockIdx.z, blockIdx.x, gridDim.x, s, wave, h, l32, gsum);
    else
      gram_store_lds<256>(p.gram_part + ((size_t)blockIdx.z * gridDim.x + blockIdx.x) * 4096, s,
                          wave, h, l32, gsum);
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

static bool few16t_on() {
  static const bool on = STX_KNOB("STX_FEW16T", 1) != 0;
  return on;
}

static bool few16_on() {
  static const bool on = STX_KNOB("STX_FEW16", 1) != 0;
  return on;
}

template <int KS, int MT>
int launch_fewin(const stx_conv_params& p, hipStream_t st) {
  const int tiles_x = (p.wo + CF_TW - 1) / CF_TW, tiles_y = (p.ho + CF_TH - 1) / CF_TH;
  // 9x9 (K = 243) stays on the fp32 kernel: its B gathers (16 16-bit LDS reads per
  // K step) cost more than the matrix cycles saved (150 vs 105 us, ITN conv0 B8 256^2)
  if (KS == 3 && few16_on() && few16t_on() && p.wo % 4 == 0)
    hipLaunchKernelGGL((conv_fewin16t_kernel<MT>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256),
                       0, st, p, tiles_x);
  else if (KS == 3 && few16_on())
    hipLaunchKernelGGL((conv_fewin16_kernel<KS, MT>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256),
                       0, st, p, tiles_x);
  else
    hipLaunchKernelGGL((conv_fewin_kernel<KS, MT>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0,
                       st, p, tiles_x);
  return check_launch("stx_conv2d(fewin)");
}

}  // namespace

// Gram partials per image of conv_fewin16_kernel<3, 2> (gram_part), 0 if another kernel
// would run this conv
int fewin_gram_tiles(const stx_conv_params& p) {
  const bool ok = p.cin == CF_CIN && p.ks == 3 && p.stride == 1 && p.pad == 1 &&
                  p.in_mode == STX_IN_RAW && p.cout == 64 && !p.relu_out && !p.mask && !p.aux &&
                  !p.accumulate && !p.p2_z && !p.up_dp && !p.pool_out && !p.acc_scale &&
                  p.wt_batch_stride == 0 && few16_on();
  return ok ? ((p.wo + CF_TW - 1) / CF_TW) * ((p.ho + CF_TH - 1) / CF_TH) : 0;
}

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
      buf[s] = relu_in ? relu_bits(v) : v;
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

// The same GEMM + col2im on the fp16 hi/lo split MFMA when the caller gives a bound
// on max|x| (p.in_amax, e.g. the producing conv's out_amax): K = 64 channels is 4
// K=16 steps x 3 products per item instead of 32 fp32 K=2 steps (5.3x fewer matrix
// cycles).  The weights' scale is block-local (max over the 27 x 64 slab entries).
// A lane's B fragment is 8 channels 16t + 8h + e of its pixel, loaded straight from
// global memory and split in registers.
template <int CIN, bool RELU_IN = false>  // RELU_IN: ReLU input (compile time)
__global__ void __launch_bounds__(256, 2) conv_fewout16_kernel(stx_conv_params p, int tiles_x) {
  constexpr int KST = CIN / 16;
  __shared__ float dt[27 * FO_RH * FO_RWP];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  // the blocks of one XCD (blockIdx % 8 under round-robin placement) take consecutive
  // tiles in row-major order, so the input rows two vertically adjacent tiles share are
  // fetched once into that XCD's L2 (speed only)
  const int G = gridDim.x;
  const int tile = (G & 7) == 0 ? (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3)
                                : (int)blockIdx.x;
  const int tx = tile % tiles_x, ty = tile / tiles_x, n = blockIdx.z;
  const int oy0 = ty * FO_TH, ox0 = tx * FO_TW;
  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * CIN * plane_in;
  constexpr bool relu_in = RELU_IN;
  // A: row m = co*9 + tap (rows >= 9*cout are 0), channel c = 16t + 8h + e
  const int m = l32, mco = m / 9, mt = m - mco * 9;
  const int mcl = min(mco, p.cout - 1);
  float wr[KST][8];
  float mw = 0.f;
#pragma unroll
  for (int t = 0; t < KST; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 16 * t + 8 * h + e;
      const float v = p.wt[(size_t)(c * 9 + mt) * p.cout_pad + mcl];
      wr[t][e] = mco < p.cout ? v : 0.f;
      mw = fmaxf(mw, fabsf(wr[t][e]));
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mw = fmaxf(mw, __shfl_xor(mw, o, 64));
  if (lane == 0) red[wave] = mw;
  __syncthreads();
  mw = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int ew = 0;
  frexpf(mw, &ew);
  ew = min(max(ew, -60), 60);
  int ex = 0;
  frexpf(read_amax(p.in_amax), &ex);
  ex = min(max(ex, -60), 60);
  const float sw = __builtin_ldexpf(1.f, 15 - ew), sx = __builtin_ldexpf(1.f, 15 - ex);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
  f16x8 ah[KST], al[KST];
#pragma unroll
  for (int t = 0; t < KST; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = wr[t][e] * sw;
      const _Float16 vh = (_Float16)v;
      ah[t][e] = vh;
      al[t][e] = (_Float16)(v - (float)vh);
    }
  const auto rx = make_srd(xn, (uint32_t)(CIN * plane_in) * 4u);
  constexpr int NITEM = FO_RH * 3;
  auto load_item = [&](int item, float (&buf)[KST][8]) {
    const int r = item / 3, nb = item - r * 3;
    const int c0 = nb == 0 ? 0 : (nb == 1 ? 32 : FO_RW - 32);
    const int iy = oy0 - 1 + r, ix = ox0 - 1 + c0 + l32;
    // the third column block overlaps the first two: only its last two columns (the
    // right halo) are new -- the other lanes read nothing (their D columns are written
    // by the first two blocks)
    const bool fresh = nb < 2 || c0 + l32 >= 64;
    const bool ok = fresh && iy >= 0 && iy < p.h && ix >= 0 && ix < p.w;
    const uint32_t vo = ok ? (uint32_t)(8 * h * plane_in + iy * p.w + ix) * 4u : BUF_OOB;
#pragma unroll
    for (int t = 0; t < KST; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo, (uint32_t)(16 * t + e) * plane_in * 4u, 0));
        buf[t][e] = relu_in ? relu_bits(v) : v;
      }
  };
  auto run_item = [&](int item, const float (&buf)[KST][8]) {
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
#pragma unroll
    for (int t = 0; t < KST; ++t) {
      f16x8 bh, bl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = buf[t][e] * sx;
        const _Float16 vh = (_Float16)v;
        bh[e] = vh;
        bl[e] = (_Float16)(v - (float)vh);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t], bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[t], bh, acc, 0, 0, 0);
    }
    const int r = item / 3, nb = item - r * 3;
    const int c0 = nb == 0 ? 0 : (nb == 1 ? 32 : FO_RW - 32);
    const bool fresh = nb < 2 || c0 + l32 >= 64;  // (the overlap lanes read zeros)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = 8 * (q >> 2) + 4 * h + (q & 3);
      if (row < 27 && fresh) dt[(row * FO_RH + r) * FO_RWP + c0 + l32] = acc[q] * descale;
    }
  };
  // items wave, wave + 4, ... through a ring of three register buffers: two items'
  // loads stay in flight behind the one being multiplied (12 MFMAs per item hide far
  // less than one load round trip).  The loads are unconditional (a clamped item past
  // the end re-reads the last one): a load skipped in a branch would leave the
  // compiler unsure how many are pending, and every wait would become vmcnt(0).
  constexpr int NK = (NITEM + 3) / 4;
  float bf[3][KST][8];
  load_item(min(wave, NITEM - 1), bf[0]);
  load_item(min(wave + 4, NITEM - 1), bf[1]);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int it = wave + 4 * k;
    if (k + 2 < NK) load_item(min(it + 8, NITEM - 1), bf[(k + 2) % 3]);
    if (it < NITEM) run_item(it, bf[k % 3]);
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
// epilogue only.  Returns -1 when not covered.  With p.in_amax (a device bound on
// max|x|) the split-MFMA kernel runs.
int conv2d_fewout(const stx_conv_params& p, hipStream_t st) {
  const bool ok = p.cout >= 1 && p.cout <= 3 && p.ks == 3 && p.stride == 1 && p.pad == 1 &&
                  (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) && p.cin == 64 &&
                  !p.mask && !p.aux && !p.p2_z && !p.up_dp && !p.pool_out && !p.acc_scale &&
                  !p.out_amax && p.wt_batch_stride == 0 && p.wt && p.hv == p.h && p.wv == p.w;
  if (!ok) return -1;
  const int tiles_x = (p.wo + FO_TW - 1) / FO_TW, tiles_y = (p.ho + FO_TH - 1) / FO_TH;
  if (p.in_amax && few16_on()) {
    if (p.in_mode == STX_IN_RELU)
      hipLaunchKernelGGL((conv_fewout16_kernel<64, true>), dim3(tiles_x * tiles_y, 1, p.n),
                         dim3(256), 0, st, p, tiles_x);
    else
      hipLaunchKernelGGL((conv_fewout16_kernel<64>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256),
                         0, st, p, tiles_x);
  }
  else
    hipLaunchKernelGGL((conv_fewout3_kernel<64>), dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0,
                       st, p, tiles_x);
  return check_launch("stx_conv2d(fewout)");
}

}  // namespace stx
