// The ImageTransformNet's 9x9 layers on the fp16 hi/lo split MFMA
// (v_mfma_f32_32x32x16_f16, three products per K=16 step; conv16.hip explains the
// split).  Reference: ConvLayer(3, 32, 9, 1) and ConvLayer(32, 3, 9, 1) of
// stransfer/network.py:525-527 / :607-609, forward and (through autograd) data gradient.
//
// Both shapes have three channels on one side, where an im2col GEMM either gathers
// its B fragments element by element (K = 3 x 81 = 243: 16 scalar LDS reads per K
// step) or pads an MFMA dimension 3 -> 32.  Instead the (channel, kh) pairs are
// folded into the 16-B fp16 units a lane feeds one MFMA, so every operand read is one
// aligned, conflict-free ds_read_b128:
//
// * conv9_in3 (3 -> 32: conv0 forward, conv22's data gradient).  K is walked as
//   (kw, 16 of the 27 (ci, kh) pairs): the unit of output row r at input column c for
//   pair group g holds x[ci][r + kh - 4][c - 4] for the 8 pairs q = 8g + e
//   ((ci, kh) = (q / 9, q % 9), zero past q = 26).  Tap kw of output pixel (r, x) is the
//   unit at column x + kw -- a per-lane base plus a compile-time offset.  27 of 32 K
//   rows are real: 3.6x the fp32 products in fp16 MFMAs at 16x the fp32 MFMA rate.
// * conv9_out3 (32 -> 3: conv22 forward).  The MFMA rows are (co, kw) (27 of 32) and
//   K = (kh, 16 channels): P[(co, kw)][r][c] = sum_{ci,kh} W[co][ci][kh][kw] x[ci][r+kh-4][c]
//   over the tile's input columns c, read from a plain [channel group][row][column]
//   halo; the output is the kw-shifted sum y[co][r][x] = sum_kw P[(co, kw)][r][x + kw]
//   formed from LDS after the MFMAs.  64 input columns give 56 output columns.
//
// Scales are block-local (max|x| over the block's input window, max|W| over the
// weights it stages), so no producer annotates the input and each block's outputs
// depend only on its window; the de-scale 2^(ex + ew - 30) is exact.  Weights come
// from the fp32 k-major slab (stx_conv_weight_prep: row (ci, kh, kw), column co; the
// data-gradient slab is already transposed and flipped).
#include <stdlib.h>

#include "common.h"
#include "conv_epi.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace {

__device__ __forceinline__ void split8(const float (&v)[8], float s, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t = v[e] * s;
    const _Float16 th = (_Float16)t;
    hi[e] = th;
    lo[e] = (_Float16)(t - (float)th);
  }
}

// block max of two values (4 waves), returned to every thread
__device__ __forceinline__ void block_max2(float& a, float& b, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a = fmaxf(a, __shfl_xor(a, o, 64));
    b = fmaxf(b, __shfl_xor(b, o, 64));
  }
  const int tid = threadIdx.x;
  if ((tid & 63) == 0) {
    red[tid >> 6] = a;
    red[4 + (tid >> 6)] = b;
  }
  __syncthreads();
  a = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  b = fmaxf(fmaxf(red[4], red[5]), fmaxf(red[6], red[7]));
}

__device__ __forceinline__ int exp_of(float m) {
  int e = 0;
  frexpf(m, &e);
  return min(max(e, -60), 60);
}

// ------------------------------------------------------------------ 3 -> 32
// Block: 4 waves, output tile 4 rows x 64 columns (wave w: row w, two 32-pixel
// N-blocks), all 32 output channels (one M tile).
namespace in3 {
constexpr int TH = 4, TW = 64, RW = TW + 8;           // unit columns per row
constexpr int NPOS = TH * RW;                          // 288 unit positions
constexpr int NB_ITEMS = 4 * NPOS;                     // (group, position) items
constexpr int NB_R = (NB_ITEMS + 255) / 256;           // 5
constexpr int NA_ITEMS = 9 * 2 * 2 * 32;               // (kw, s, h, co) items
constexpr int LDS_B = 2 * 4 * NPOS * 16;               // [P][g][pos] units
constexpr int LDS_A = 9 * 2 * 2 * 2 * 32 * 16;         // [kw][s][P][h][co] units
}  // namespace in3

__global__ void __launch_bounds__(256, 2) conv9_in3_kernel(stx_conv_params p, int tiles_x) {
  using namespace in3;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B + LDS_A];
  __shared__ float red[8];
  char* lb = smem;
  char* la = smem + LDS_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n = blockIdx.z;
  const int oy0 = (blockIdx.x / tiles_x) * TH, ox0 = (blockIdx.x % tiles_x) * TW;
  const int plane_in = p.h * p.w;
  const auto rx = make_srd(p.x + (size_t)n * 3 * plane_in, (uint32_t)(3 * plane_in) * 4u);
  const bool relu_in = p.in_mode == STX_IN_RELU;

  // B items i = tid + 256 k: position pos = i % NPOS (r, c), group g = i / NPOS
  float bv[NB_R][8];
  float mx = 0.f;
#pragma unroll
  for (int k = 0; k < NB_R; ++k) {
    const int i = tid + 256 * k;
    const int g = i / NPOS, pos = i - g * NPOS;
    const int r = pos / RW, c = pos - r * RW;
    const int x = ox0 - 4 + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = 8 * g + e;
      const int ci = q / 9, kh = q - 9 * (q / 9);
      const int y = oy0 + r + kh - 4;
      const bool ok = i < NB_ITEMS && q < 27 && y >= 0 && y < p.h && x >= 0 && x < p.w;
      float v = buf_ld(rx, ok ? (uint32_t)(ci * plane_in + y * p.w + x) * 4u : BUF_OOB);
      if (relu_in) v = fmaxf(v, 0.f);
      bv[k][e] = v;
      mx = fmaxf(mx, fabsf(v));
    }
  }
  // A items u = tid + 256 k: co = u % 32, h = (u / 32) % 2, s = (u / 64) % 2, kw = u / 128;
  // element e is pair q = 16 s + 8 h + e of W[co][ci][kh][kw] = wt[(ci*81 + kh*9 + kw)][co]
  constexpr int NAK = (NA_ITEMS + 255) / 256;  // 5 (the last round half idle)
  float av[NAK][8];
  float mw = 0.f;
#pragma unroll
  for (int k = 0; k < NAK; ++k) {
    const int u = tid + 256 * k;
    const int co = u & 31, hh = (u >> 5) & 1, s = (u >> 6) & 1, kw = u >> 7;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = 16 * s + 8 * hh + e;
      const int ci = q / 9, kh = q - 9 * (q / 9);
      const bool ok = u < NA_ITEMS && q < 27 && co < p.cout;
      const int row = ok ? ci * 81 + kh * 9 + kw : 0;
      const float v = p.wt[(size_t)row * p.cout_pad + (ok ? co : 0)];
      av[k][e] = ok ? v : 0.f;
      mw = fmaxf(mw, fabsf(av[k][e]));
    }
  }
  block_max2(mx, mw, red);
  const int ex = exp_of(mx), ew = exp_of(mw);
  const float sx = __builtin_ldexpf(1.f, 15 - ex), sw = __builtin_ldexpf(1.f, 15 - ew);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
#pragma unroll
  for (int k = 0; k < NB_R; ++k) {
    const int i = tid + 256 * k;
    if (i < NB_ITEMS) {
      f16x8 hi, lo;
      split8(bv[k], sx, hi, lo);
      const int g = i / NPOS, pos = i - g * NPOS;
      *reinterpret_cast<f16x8*>(lb + ((0 * 4 + g) * NPOS + pos) * 16) = hi;
      *reinterpret_cast<f16x8*>(lb + ((1 * 4 + g) * NPOS + pos) * 16) = lo;
    }
  }
#pragma unroll
  for (int k = 0; k < NAK; ++k) {
    const int u = tid + 256 * k;
    if (u < NA_ITEMS) {
      f16x8 hi, lo;
      split8(av[k], sw, hi, lo);
      const int co = u & 31, hh = (u >> 5) & 1, s = (u >> 6) & 1, kw = u >> 7;
      const int base = ((kw * 2 + s) * 2) * 2;  // [kw][s][P][h]
      *reinterpret_cast<f16x8*>(la + (((base + 0 * 2 + hh) * 32) + co) * 16) = hi;
      *reinterpret_cast<f16x8*>(la + (((base + 1 * 2 + hh) * 32) + co) * 16) = lo;
    }
  }
  __syncthreads();

  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const char* bb = lb + (wave * RW + l32) * 16;
#pragma unroll
  for (int kw = 0; kw < 9; ++kw)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int base = ((kw * 2 + s) * 2) * 2;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(la + ((base + h) * 32 + l32) * 16);
      const f16x8 al = *reinterpret_cast<const f16x8*>(la + ((base + 2 + h) * 32 + l32) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int off = (32 * j + kw) * 16;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(bb + ((0 * 4 + 2 * s + h) * NPOS) * 16 + off);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(bb + ((1 * 4 + 2 * s + h) * NPOS) * 16 + off);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
      }
    }

  // epilogue: rows co = 8 (r/4) + 4h + r%4, pixel (oy0 + wave, ox0 + 32 j + l32)
  const size_t plane = (size_t)p.ho * p.wo;
  const uint32_t pb = (uint32_t)plane * 4u;
  const auto ry = make_srd(p.y + (size_t)n * p.cout * plane, (uint32_t)p.cout * pb);
  uint32_t vmax_u = 0u;
  const int oy = oy0 + wave;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ox = ox0 + 32 * j + l32;
    const bool in = oy < p.ho && ox < p.wo;
    const uint32_t vo = in ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row_c = 8 * (r >> 2) + (r & 3);
      const int co = row_c + 4 * h;
      float v = acc[j][r] * descale;
      if (p.bias) v += p.bias[min(co, p.cout - 1)];
      if (p.relu_out) v = fmaxf(v, 0.f);
      if (co < p.cout) {
        buf_st(ry, vo + (uint32_t)row_c * pb, v);
        if (in) vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
      }
    }
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

// ------------------------------------------------------------------ 32 -> 3
// Block: 4 waves, 4 output rows x 56 output columns (wave w: row w; its two N-blocks
// are the 64 input columns ox0 - 4 .. ox0 + 59), input channels in chunks of 16.
namespace out3 {
constexpr int TH = 4, TWO = 56, TWI = 64, RH = TH + 8;
constexpr int NPOS = RH * TWI;                     // 768 halo positions
constexpr int NB_ITEMS = 2 * NPOS;                 // (channel group, position)
constexpr int NB_R = NB_ITEMS / 256;               // 6
constexpr int NA_ITEMS = 9 * 2 * 32;               // (kh, h, m)
constexpr int LDS_B = 2 * NB_ITEMS * 16;           // [P][cg][row][col]
constexpr int LDS_A = 9 * 2 * 2 * 32 * 16;         // [kh][P][h][m]
constexpr int PST = TWI + 1;                       // P row stride (floats)
static_assert(NB_ITEMS % 256 == 0, "halo items per thread");
static_assert(4 * 32 * PST * 4 <= LDS_B + LDS_A, "P planes fit");
}  // namespace out3

__global__ void __launch_bounds__(256, 2) conv9_out3_kernel(stx_conv_params p, int tiles_x) {
  using namespace out3;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B + LDS_A];
  __shared__ float red[8];
  char* lb = smem;
  char* la = smem + LDS_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n = blockIdx.z;
  const int oy0 = (blockIdx.x / tiles_x) * TH, ox0 = (blockIdx.x % tiles_x) * TWO;
  const int plane_in = p.h * p.w;
  const auto rx = make_srd(p.x + (size_t)n * p.cin * plane_in, (uint32_t)(p.cin * plane_in) * 4u);
  const bool relu_in = p.in_mode == STX_IN_RELU;
  const int nchunks = cdiv(p.cin, 16);

  // halo item i = tid + 256 k -> channel group cg = i / NPOS, position (row, col)
  uint32_t hoff[NB_R];
#pragma unroll
  for (int k = 0; k < NB_R; ++k) {
    const int i = tid + 256 * k;
    const int cg = i / NPOS, pos = i - cg * NPOS;
    const int rr = pos / TWI, cc = pos - rr * TWI;
    const int y = oy0 - 4 + rr, x = ox0 - 4 + cc;
    const bool ok = y >= 0 && y < p.h && x >= 0 && x < p.w;
    hoff[k] = ok ? (uint32_t)(8 * cg * plane_in + y * p.w + x) * 4u : BUF_OOB;
  }
  auto ld_halo = [&](int c0, int k, int e) -> float {
    const bool ok = c0 + 8 * ((tid + 256 * k) / NPOS) + e < p.cin && hoff[k] != BUF_OOB;
    float v = buf_ld(rx, ok ? hoff[k] + (uint32_t)((c0 + e) * plane_in) * 4u : BUF_OOB);
    return relu_in ? fmaxf(v, 0.f) : v;
  };
  // weight item u = tid + 256 k -> (kh, h, m): m = co * 9 + kw, element e = channel
  // c0 + 8 h + e: W[co][ci][kh][kw] = wt[(ci*81 + kh*9 + kw)][co]
  auto ld_w = [&](int c0, int k, int e) -> float {
    const int u = tid + 256 * k;
    const int m = u & 31, hh = (u >> 5) & 1, kh = u >> 6;
    const int co = m / 9, kw = m - 9 * (m / 9), ci = c0 + 8 * hh + e;
    const bool ok = u < NA_ITEMS && co < p.cout && ci < p.cin;
    const float v = p.wt[(size_t)(ok ? ci * 81 + kh * 9 + kw : 0) * p.cout_pad + (ok ? co : 0)];
    return ok ? v : 0.f;
  };
  // block-local maxima over the whole window and all weights (a read-only first pass)
  float mx = 0.f, mw = 0.f;
  for (int c = 0; c < nchunks; ++c) {
#pragma unroll
    for (int k = 0; k < NB_R; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(ld_halo(16 * c, k, e)));
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) mw = fmaxf(mw, fabsf(ld_w(16 * c, k, e)));
  }
  block_max2(mx, mw, red);
  const int ex = exp_of(mx), ew = exp_of(mw);
  const float sx = __builtin_ldexpf(1.f, 15 - ex), sw = __builtin_ldexpf(1.f, 15 - ew);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);

  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const char* bb = lb + (wave * TWI + l32) * 16;  // (row wave + kh, column 32 j + l32)
  for (int c = 0; c < nchunks; ++c) {
    const int c0 = 16 * c;
    float hv[NB_R][8], wv[3][8];
#pragma unroll
    for (int k = 0; k < NB_R; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[k][e] = ld_halo(c0, k, e);
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) wv[k][e] = ld_w(c0, k, e);
    __syncthreads();  // the previous chunk's operand reads are done
#pragma unroll
    for (int k = 0; k < NB_R; ++k) {
      f16x8 hi, lo;
      split8(hv[k], sx, hi, lo);
      const int i = tid + 256 * k;
      *reinterpret_cast<f16x8*>(lb + i * 16) = hi;
      *reinterpret_cast<f16x8*>(lb + (NB_ITEMS + i) * 16) = lo;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int u = tid + 256 * k;
      if (u < NA_ITEMS) {
        f16x8 hi, lo;
        split8(wv[k], sw, hi, lo);
        const int m = u & 31, hh = (u >> 5) & 1, kh = u >> 6;
        *reinterpret_cast<f16x8*>(la + (((kh * 2 + 0) * 2 + hh) * 32 + m) * 16) = hi;
        *reinterpret_cast<f16x8*>(la + (((kh * 2 + 1) * 2 + hh) * 32 + m) * 16) = lo;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kh = 0; kh < 9; ++kh) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(la + (((kh * 2 + 0) * 2 + h) * 32 + l32) * 16);
      const f16x8 al = *reinterpret_cast<const f16x8*>(la + (((kh * 2 + 1) * 2 + h) * 32 + l32) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int off = ((h * NPOS) + kh * TWI + 32 * j) * 16;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(bb + off);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(bb + NB_ITEMS * 16 + off);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
      }
    }
  }
  // P[(co, kw)][column] of this wave's row to LDS, then y[co][x] = sum_kw P[co*9+kw][x+kw]
  __syncthreads();
  float* pw = reinterpret_cast<float*>(smem) + wave * 32 * PST;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) pw[(8 * (r >> 2) + 4 * h + (r & 3)) * PST + 32 * j + l32] = acc[j][r] * descale;
  __syncthreads();
  const size_t plane = (size_t)p.ho * p.wo;
  const int oy = oy0 + wave;
  uint32_t vmax_u = 0u;
  for (int idx = lane; idx < p.cout * TWO; idx += 64) {
    const int co = idx / TWO, x = idx - co * TWO;
    float v = 0.f;
#pragma unroll
    for (int kw = 0; kw < 9; ++kw) v += pw[(co * 9 + kw) * PST + x + kw];
    const int ox = ox0 + x;
    if (oy < p.ho && ox < p.wo) {
      const size_t o = ((size_t)n * p.cout + co) * plane + (size_t)oy * p.wo + ox;
      if (p.bias) v += p.bias[co];
      if (p.accumulate) v += p.y[o];
      if (p.relu_out) v = fmaxf(v, 0.f);
      p.y[o] = v;
      vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
    }
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

bool conv9_on() {
  static const bool on = [] {
    const char* e = getenv("STX_CONV9");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

}  // namespace

// 9x9 stride 1 pad 4, 3 -> 32 or 32 -> 3 (any cin <= 3 / cout <= 3 side of those
// shapes), raw or ReLU input, fp32 slab (wt); bias / relu_out / out_amax (and
// accumulate for 32 -> 3) epilogues.  Returns -1 when not covered.
int conv2d_conv9(const stx_conv_params& p, hipStream_t st) {
  const bool base = p.ks == 9 && p.stride == 1 && p.pad == 4 && p.wt &&
                    (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) && !p.mask && !p.aux &&
                    !p.p2_z && !p.up_dp && !p.pool_out && !p.acc_scale && !p.gram_part &&
                    p.wt_batch_stride == 0 && p.hv == p.h && p.wv == p.w && conv9_on();
  if (!base) return -1;
  if (p.cin == 3 && p.cout >= 1 && p.cout <= 32 && !p.accumulate) {
    const int tiles_x = cdiv(p.wo, in3::TW), tiles_y = cdiv(p.ho, in3::TH);
    hipLaunchKernelGGL(conv9_in3_kernel, dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0, st, p,
                       tiles_x);
    return check_launch("stx_conv2d(conv9 3->32)");
  }
  if (p.cout >= 1 && p.cout <= 3 && p.cin >= 1 && p.cin <= 64) {
    const int tiles_x = cdiv(p.wo, out3::TWO), tiles_y = cdiv(p.ho, out3::TH);
    hipLaunchKernelGGL(conv9_out3_kernel, dim3(tiles_x * tiles_y, 1, p.n), dim3(256), 0, st, p,
                       tiles_x);
    return check_launch("stx_conv2d(conv9 32->3)");
  }
  return -1;
}

}  // namespace stx
