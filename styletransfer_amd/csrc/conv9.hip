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
// Both run persistent: one 8-wave block per CU stages the split weights once and walks
// its tiles with the next tile's (or chunk's) input loads in flight during the current
// MFMAs.  The input scale is per tile for 3 -> 32 (the tile's window max: no producer
// annotates the image or the loss-network gradient) and the producer's max|x| bound
// (p.in_amax, an InstanceNorm output) for 32 -> 3; the weight scale is max|W|.  Each
// tile's outputs depend only on its window, and the de-scale 2^(ex + ew - 30) is exact.
// Weights come from the fp32 k-major slab (stx_conv_weight_prep: row (ci, kh, kw),
// column co; the data-gradient slab is already transposed and flipped).
#include <stdlib.h>

#include "common.h"
#include "conv_epi.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr int NWV = 8, NT = 64 * NWV;  // waves / threads per block

__device__ __forceinline__ void split8(const float (&v)[8], float s, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t = v[e] * s;
    const _Float16 th = (_Float16)t;
    hi[e] = th;
    lo[e] = (_Float16)(t - (float)th);
  }
}

// block max (NWV waves), returned to every thread; red[NWV] is free again once every
// thread has passed the next barrier
template <int W = NWV>
__device__ __forceinline__ float block_max(float a, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < W; ++i) m = fmaxf(m, red[i]);
  return m;
}

// one atomic per block into slot (block id % STX_AMAX_SLOTS) of an amax group
template <int W = NWV>
__device__ __forceinline__ void block_amax_out(float* group, uint32_t m_u, float* red) {
  const float m = block_max<W>(__uint_as_float(m_u), red);
  if (threadIdx.x == 0) atomic_max_abs(group + (blockIdx.x & (STX_AMAX_SLOTS - 1)), m);
}

__device__ __forceinline__ int exp_of(float m) {
  int e = 0;
  frexpf(m, &e);
  return min(max(e, -60), 60);
}

// persistent tile walk: XCD x (block b -> x = b % 8) takes a contiguous run of each
// round's tiles, so neighbouring tiles (which share halo rows) meet in one L2
__device__ __forceinline__ int first_tile() {
  const int g = gridDim.x;
  if (g % 8) return blockIdx.x;
  return (blockIdx.x % 8) * (g / 8) + blockIdx.x / 8;
}

// ------------------------------------------------------------------ 3 -> 32
// Tile: 8 output rows x 64 columns (wave w: row w, two 32-pixel N-blocks), all
// output channels <= 32 (one M tile).
// W waves per block (8: one block per CU, LDS-limited)
template <int W>
struct In3 {
  static constexpr int NT = 64 * W;
  static constexpr int TH = W, TW = 64, RW = TW + 8;    // unit columns per row
  static constexpr int NPOS = TH * RW;                  // unit positions
  static constexpr int NB_ITEMS = 4 * NPOS;             // (pair group, position) units
  static constexpr int NB_R = (NB_ITEMS + NT - 1) / NT; // 5 (the last round partly idle)
  static constexpr int NA_ITEMS = 9 * 2 * 2 * 32;      // (kw, s, h, co) units
  static constexpr int NA_R = (NA_ITEMS + NT - 1) / NT;
  static constexpr int LDS_B = 2 * 4 * NPOS * 16;      // [P][g][pos]
  static constexpr int LDS_A = 9 * 2 * 2 * 2 * 32 * 16; // [kw][s][P][h][co]
};

template <int W = NWV>
__global__ void __launch_bounds__(64 * W, 8 / W) conv9_in3_kernel(stx_conv_params p, int tiles_x,
                                                                  int tiles_y) {
  using C = In3<W>;
  constexpr int NT = C::NT, TH = C::TH, TW = C::TW, RW = C::RW, NPOS = C::NPOS;
  constexpr int NB_ITEMS = C::NB_ITEMS, NB_R = C::NB_R, NA_ITEMS = C::NA_ITEMS, NA_R = C::NA_R;
  constexpr int LDS_B = C::LDS_B, LDS_A = C::LDS_A;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B + LDS_A];
  __shared__ float red[W];
  char* lb = smem;
  char* la = smem + LDS_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tiles_img = tiles_x * tiles_y, ntiles = tiles_img * p.n;
  const int plane_in = p.h * p.w;
  const bool relu_in = p.in_mode == STX_IN_RELU;

  // B unit i = tid + NT k: position pos = i % NPOS (r, c), pair group g = i / NPOS
  float bv[NB_R][8];
  auto load_b = [&](int tile) {
    const int n = tile / tiles_img, t = tile - n * tiles_img;
    const int oy0 = (t / tiles_x) * TH, ox0 = (t % tiles_x) * TW;
    const auto rx = make_srd(p.x + (size_t)n * 3 * plane_in, (uint32_t)(3 * plane_in) * 4u);
#pragma unroll
    for (int k = 0; k < NB_R; ++k) {
      const int i = tid + NT * k;
      const int g = i / NPOS, pos = i - g * NPOS;
      const int r = pos / RW, c = pos - r * RW;
      const int x = ox0 - 4 + c;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = 8 * g + e;
        const int ci = q / 9, kh = q - 9 * (q / 9);
        const int y = oy0 + r + kh - 4;
        const bool ok = i < NB_ITEMS && q < 27 && y >= 0 && y < p.h && x >= 0 && x < p.w;
        bv[k][e] = buf_ld(rx, ok ? (uint32_t)(ci * plane_in + y * p.w + x) * 4u : BUF_OOB);
      }
    }
  };
  int tile = first_tile();
  if (tile < ntiles) load_b(tile);

  // weights, once: unit u = tid + NT k -> co = u % 32, h = (u / 32) % 2, s = (u / 64) % 2,
  // kw = u / 128; element e is pair q = 16 s + 8 h + e of W[co][ci][kh][kw]
  int ew;
  {
    float av[NA_R][8];
    float mw = 0.f;
#pragma unroll
    for (int k = 0; k < NA_R; ++k) {
      const int u = tid + NT * k;
      const int co = u & 31, hh = (u >> 5) & 1, s = (u >> 6) & 1, kw = u >> 7;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = 16 * s + 8 * hh + e;
        const int ci = q / 9, kh = q - 9 * (q / 9);
        const bool ok = u < NA_ITEMS && q < 27 && co < p.cout;
        const float v = p.wt[(size_t)(ok ? ci * 81 + kh * 9 + kw : 0) * p.cout_pad + (ok ? co : 0)];
        av[k][e] = ok ? v : 0.f;
        mw = fmaxf(mw, fabsf(av[k][e]));
      }
    }
    ew = exp_of(block_max<W>(mw, red));
    const float sw = __builtin_ldexpf(1.f, 15 - ew);
#pragma unroll
    for (int k = 0; k < NA_R; ++k) {
      const int u = tid + NT * k;
      if (u < NA_ITEMS) {
        f16x8 hi, lo;
        split8(av[k], sw, hi, lo);
        const int co = u & 31, hh = (u >> 5) & 1, s = (u >> 6) & 1, kw = u >> 7;
        const int base = ((kw * 2 + s) * 2) * 2;  // [kw][s][P][h]
        *reinterpret_cast<f16x8*>(la + ((base + 0 * 2 + hh) * 32 + co) * 16) = hi;
        *reinterpret_cast<f16x8*>(la + ((base + 1 * 2 + hh) * 32 + co) * 16) = lo;
      }
    }
    __syncthreads();  // red[] is reused by the first tile's window max
  }
  const size_t plane = (size_t)p.ho * p.wo;
  const uint32_t pb = (uint32_t)plane * 4u;
  float bias_r[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = 8 * (r >> 2) + 4 * h + (r & 3);
    bias_r[r] = (p.bias && co < p.cout) ? p.bias[co] : 0.f;
  }
  uint32_t vmax_u = 0u;
  const char* bb = lb + (wave * RW + l32) * 16;
  for (; tile < ntiles; tile += gridDim.x) {
    // this tile's window max (the barrier inside also retires the last tile's B reads)
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < NB_R; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (relu_in) bv[k][e] = relu_bits(bv[k][e]);
        mx = fmaxf(mx, fabsf(bv[k][e]));
      }
    const int ex = exp_of(block_max<W>(mx, red));
    const float sx = __builtin_ldexpf(1.f, 15 - ex);
    const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
#pragma unroll
    for (int k = 0; k < NB_R; ++k) {
      const int i = tid + NT * k;
      if (i < NB_ITEMS) {
        f16x8 hi, lo;
        split8(bv[k], sx, hi, lo);
        *reinterpret_cast<f16x8*>(lb + i * 16) = hi;  // [P][g][pos]: i = g * NPOS + pos
        *reinterpret_cast<f16x8*>(lb + (NB_ITEMS + i) * 16) = lo;
      }
    }
    __syncthreads();
    const int cur = tile;
    if (tile + (int)gridDim.x < ntiles) load_b(tile + gridDim.x);  // in flight during the MFMAs

    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int kw = 0; kw < 9; ++kw)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int base = ((kw * 2 + s) * 2) * 2;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(la + ((base + h) * 32 + l32) * 16);
        const f16x8 al = *reinterpret_cast<const f16x8*>(la + ((base + 2 + h) * 32 + l32) * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int off = ((2 * s + h) * NPOS + 32 * j + kw) * 16;
          const f16x8 bh = *reinterpret_cast<const f16x8*>(bb + off);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(bb + NB_ITEMS * 16 + off);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
        }
      }

    // rows co = 8 (r/4) + 4h + r%4, pixel (oy0 + wave, ox0 + 32 j + l32)
    const int n = cur / tiles_img, t = cur - n * tiles_img;
    const int oy = (t / tiles_x) * TH + wave, ox0 = (t % tiles_x) * TW;
    const auto ry = make_srd(p.y + (size_t)n * p.cout * plane, (uint32_t)p.cout * pb);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ox = ox0 + 32 * j + l32;
      const bool in = oy < p.ho && ox < p.wo;
      const uint32_t vo = in ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row_c = 8 * (r >> 2) + (r & 3);
        float v = fmaf(acc[j][r], descale, bias_r[r]);
        if (p.relu_out) v = fmaxf(v, 0.f);
        // branch-free: channels past cout store out of range (a store inside a branch
        // leaves the compiler unsure how many are pending, so the next tile's wait for
        // its prefetched loads becomes a wait for every store too)
        const bool ok = row_c + 4 * h < p.cout;
        buf_st(ry, ok ? vo + (uint32_t)row_c * pb : BUF_OOB, v);
        vmax_u = max(vmax_u, (in && ok) ? (__float_as_uint(v) & 0x7fffffffu) : 0u);
      }
    }
  }
  if (p.out_amax) block_amax_out<W>(p.out_amax, vmax_u, red);
}

// ------------------------------------------------------------------ 32 -> 3
// Tile: 8 output rows x 56 output columns (wave w: row w; its two N-blocks are the 64
// input columns ox0 - 4 .. ox0 + 59); input channels in chunks of 16 (cin <= 32: the
// split weights of every chunk stay in LDS).
namespace out3 {
constexpr int TH = NWV, TWO = 56, TWI = 64, RH = TH + 8;
constexpr int NPOS = RH * TWI;                     // 1024 halo positions
constexpr int NB_ITEMS = 2 * NPOS;                 // (channel group, position) units
constexpr int NB_R = NB_ITEMS / NT;                // 4
constexpr int NA_ITEMS = 9 * 2 * 32;               // (kh, h, m) units per chunk
constexpr int NA_R = (2 * NA_ITEMS + NT - 1) / NT; // both chunks: 3 rounds
constexpr int LDS_B = 2 * NB_ITEMS * 16;           // [P][cg][row][col]
constexpr int LDS_A = 2 * 9 * 2 * 2 * 32 * 16;     // [chunk][kh][P][h][m]
constexpr int PST = TWI + 1;                       // P row stride (floats)
static_assert(NB_ITEMS % NT == 0, "halo units per thread");
static_assert(NWV * 27 * PST * 4 <= LDS_B, "P rows fit in the halo region");
}  // namespace out3

// The block walks steps s = (its tile i, chunk c) = (s / NCH, s % NCH); the halo loads of
// step s + 2 are issued right after step s is staged (two register sets: a load has two
// steps of MFMAs to land instead of one), unconditionally -- a step past the block's
// last tile loads through an empty descriptor and stores out of range -- so the wait
// before a set's staging covers exactly the older set's loads.
template <int NCH>
__global__ void __launch_bounds__(NT, 1) conv9_out3_kernel(stx_conv_params p, int tiles_x,
                                                           int tiles_y) {
  using namespace out3;
  __shared__ __attribute__((aligned(16))) char smem[LDS_B + LDS_A];
  __shared__ float red[NWV];
  char* lb = smem;
  char* la = smem + LDS_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int tiles_img = tiles_x * tiles_y, ntiles = tiles_img * p.n;
  const int plane_in = p.h * p.w;
  const bool relu_in = p.in_mode == STX_IN_RELU;

  // halo unit i = tid + NT k -> channel group cg = i / NPOS, position (row, col)
  uint32_t hpos[NB_R];
#pragma unroll
  for (int k = 0; k < NB_R; ++k) {
    const int i = tid + NT * k;
    const int cg = i / NPOS, pos = i - cg * NPOS;
    const int rr = pos / TWI, cc = pos - rr * TWI;
    hpos[k] = (uint32_t)(cg << 20 | rr << 10 | cc);
  }
  const int tile0 = first_tile();
  const int mine = tile0 < ntiles ? cdiv(ntiles - tile0, (int)gridDim.x) : 0;
  const int nsteps = rup(mine * NCH, 2);  // whole pairs of steps (a padded step is inert)
  float hv[2][NB_R][8];
  auto load_h = [&](float (&hs)[NB_R][8], int step) {
    const int it = step / NCH, c = step - it * NCH;
    const int tile = tile0 + it * (int)gridDim.x;
    const bool valid = it < mine;
    const int n = tile / tiles_img, t = tile - n * tiles_img;
    const int oy0 = (t / tiles_x) * TH, ox0 = (t % tiles_x) * TWO;
    const auto rx = make_srd(p.x + (size_t)(valid ? n : 0) * p.cin * plane_in,
                             valid ? (uint32_t)(p.cin * plane_in) * 4u : 0u);
#pragma unroll
    for (int k = 0; k < NB_R; ++k) {
      const int cg = hpos[k] >> 20, rr = (hpos[k] >> 10) & 1023, cc = hpos[k] & 1023;
      const int y = oy0 - 4 + rr, x = ox0 - 4 + cc, ch = 16 * c + 8 * cg;
      const bool ok = y >= 0 && y < p.h && x >= 0 && x < p.w;
      const uint32_t o = (uint32_t)(ch * plane_in + y * p.w + x) * 4u;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        hs[k][e] = buf_ld(rx, (ok && ch + e < p.cin) ? o + (uint32_t)(e * plane_in) * 4u : BUF_OOB);
    }
  };
  load_h(hv[0], 0);
  load_h(hv[1], 1);

  // weights of every chunk, once: unit u = tid + NT k -> chunk c = u / NA_ITEMS, (kh, h, m):
  // m = co * 9 + kw, element e = channel 16 c + 8 h + e: W[co][ci][kh][kw] = wt[(ci*81 + kh*9 + kw)][co]
  const float sx = __builtin_ldexpf(1.f, 15 - exp_of(read_amax(p.in_amax)));
  float descale;
  {
    float wv[NA_R][8];
    float mw = 0.f;
#pragma unroll
    for (int k = 0; k < NA_R; ++k) {
      const int u = tid + NT * k;
      const int c = u / NA_ITEMS, v = u - c * NA_ITEMS;
      const int m = v & 31, hh = (v >> 5) & 1, kh = v >> 6;
      const int co = m / 9, kw = m - 9 * (m / 9);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ci = 16 * c + 8 * hh + e;
        const bool ok = c < NCH && co < p.cout && ci < p.cin;
        const float w = p.wt[(size_t)(ok ? ci * 81 + kh * 9 + kw : 0) * p.cout_pad + (ok ? co : 0)];
        wv[k][e] = ok ? w : 0.f;
        mw = fmaxf(mw, fabsf(wv[k][e]));
      }
    }
    const int ew = exp_of(block_max(mw, red));
    const float sw = __builtin_ldexpf(1.f, 15 - ew);
    descale = __builtin_ldexpf(1.f, exp_of(read_amax(p.in_amax)) + ew - 30);
#pragma unroll
    for (int k = 0; k < NA_R; ++k) {
      const int u = tid + NT * k;
      if (u < 2 * NA_ITEMS) {
        f16x8 hi, lo;
        split8(wv[k], sw, hi, lo);
        const int c = u / NA_ITEMS, v = u - c * NA_ITEMS;
        const int m = v & 31, hh = (v >> 5) & 1, kh = v >> 6;
        *reinterpret_cast<f16x8*>(la + ((((c * 9 + kh) * 2 + 0) * 2 + hh) * 32 + m) * 16) = hi;
        *reinterpret_cast<f16x8*>(la + ((((c * 9 + kh) * 2 + 1) * 2 + hh) * 32 + m) * 16) = lo;
      }
    }
  }

  const size_t plane = (size_t)p.ho * p.wo;
  uint32_t vmax_u = 0u;
  const char* bb = lb + (wave * TWI + l32) * 16;  // (row wave + kh, column 32 j + l32)
  float* pw = reinterpret_cast<float*>(smem) + wave * 27 * PST;
  f32x16 acc[2];
  auto step = [&](float (&hs)[NB_R][8], int s, int c) {
    if (c == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    }
    __syncthreads();  // the previous step's operand reads / P reads are done
#pragma unroll
    for (int k = 0; k < NB_R; ++k) {
      if (relu_in)
#pragma unroll
        for (int e = 0; e < 8; ++e) hs[k][e] = relu_bits(hs[k][e]);
      f16x8 hi, lo;
      split8(hs[k], sx, hi, lo);
      const int i = tid + NT * k;
      *reinterpret_cast<f16x8*>(lb + i * 16) = hi;
      *reinterpret_cast<f16x8*>(lb + (NB_ITEMS + i) * 16) = lo;
    }
    __syncthreads();
    load_h(hs, s + 2);  // in flight during this step's and the next step's MFMAs
    const char* ac = la + c * 9 * 2 * 2 * 32 * 16;
#pragma unroll
    for (int kh = 0; kh < 9; ++kh) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(ac + (((kh * 2 + 0) * 2 + h) * 32 + l32) * 16);
      const f16x8 al = *reinterpret_cast<const f16x8*>(ac + (((kh * 2 + 1) * 2 + h) * 32 + l32) * 16);
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
    if (c != NCH - 1) return;
    // P[(co, kw)][column] of this wave's row into LDS (rows < 27), then
    // y[co][x] = sum_kw P[co*9 + kw][x + kw]
    __syncthreads();  // every wave's halo reads are done
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = 8 * (r >> 2) + 4 * h + (r & 3);
        if (m < 27) pw[m * PST + 32 * j + l32] = acc[j][r] * descale;
      }
    __syncthreads();
    const int it = s / NCH;
    const int tile = tile0 + it * (int)gridDim.x;
    const bool tok = it < mine;
    const int n = tok ? tile / tiles_img : 0, t = tile - n * tiles_img;
    const int oy = (t / tiles_x) * TH + wave, ox0 = (t % tiles_x) * TWO;
    // branch-free stores through a descriptor (see conv9_in3's epilogue): 3 x 64 lanes
    // cover the 3 x 56 outputs, the rest (and a padded step) store out of range
    const auto ry = make_srd(p.y + (size_t)n * p.cout * plane,
                             tok ? (uint32_t)(p.cout * plane) * 4u : 0u);
#pragma unroll
    for (int r3 = 0; r3 < 3; ++r3) {
      const int idx = lane + 64 * r3;
      const int co = idx / TWO, x = idx - co * TWO, coc = min(co, p.cout - 1);
      float v = 0.f;
#pragma unroll
      for (int kw = 0; kw < 9; ++kw) v += pw[(coc * 9 + kw) * PST + x + kw];
      const int ox = ox0 + x;
      const bool ok = tok && co < p.cout && oy < p.ho && ox < p.wo;
      const uint32_t o = ok ? (uint32_t)((size_t)co * plane + (size_t)oy * p.wo + ox) * 4u : BUF_OOB;
      if (p.bias) v += p.bias[coc];
      if (p.accumulate) v += buf_ld(ry, o);
      if (p.relu_out) v = fmaxf(v, 0.f);
      buf_st(ry, o, v);
      vmax_u = max(vmax_u, ok ? (__float_as_uint(v) & 0x7fffffffu) : 0u);
    }
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(hv[0], s, NCH == 2 ? 0 : 0);
    step(hv[1], s + 1, NCH == 2 ? 1 : 0);
  }
  if (p.out_amax) block_amax_out(p.out_amax, vmax_u, red);
}

bool conv9_on() {
  static const bool on = STX_KNOB("STX_CONV9", 1) != 0;
  return on;
}


int persistent_grid(int ntiles, int per_cu) {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  static const int over = STX_KNOB("STX_CONV9_GRID", 0);  // profiling override
  return std::min(ntiles, over > 0 ? over : per_cu * cus);  // LDS-limited blocks per CU
}

}  // namespace

// 9x9 stride 1 pad 4, 3 -> <= 32 channels, or <= 32 -> <= 3 channels with a max|x|
// bound (p.in_amax), raw or ReLU input, fp32 slab (wt); bias / relu_out / out_amax
// (and accumulate for the 3-output shape) epilogues.  Returns -1 when not covered.
int conv2d_conv9(const stx_conv_params& p, hipStream_t st) {
  const bool base = p.ks == 9 && p.stride == 1 && p.pad == 4 && p.wt &&
                    (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) && !p.mask && !p.aux &&
                    !p.p2_z && !p.up_dp && !p.pool_out && !p.acc_scale && !p.gram_part &&
                    p.wt_batch_stride == 0 && p.hv == p.h && p.wv == p.w && conv9_on();
  if (!base) return -1;
  if (p.cin == 3 && p.cout >= 1 && p.cout <= 32 && !p.accumulate) {
    // (4-wave blocks, two per CU, measured the same: 58.5 vs 58.2 us at B8 256^2)
    const int tx = cdiv(p.wo, In3<8>::TW), ty = cdiv(p.ho, In3<8>::TH);
    hipLaunchKernelGGL(conv9_in3_kernel<>, dim3(persistent_grid(tx * ty * p.n, 1)), dim3(NT), 0,
                       st, p, tx, ty);
    return check_launch("stx_conv2d(conv9 3->32)");
  }
  if (p.cout >= 1 && p.cout <= 3 && p.cin >= 1 && p.cin <= 32 && p.in_amax) {
    const int tx = cdiv(p.wo, out3::TWO), ty = cdiv(p.ho, out3::TH);
    const dim3 grid(persistent_grid(tx * ty * p.n, 1));
    if (p.cin > 16)
      hipLaunchKernelGGL(conv9_out3_kernel<2>, grid, dim3(NT), 0, st, p, tx, ty);
    else
      hipLaunchKernelGGL(conv9_out3_kernel<1>, grid, dim3(NT), 0, st, p, tx, ty);
    return check_launch("stx_conv2d(conv9 32->3)");
  }
  return -1;
}

}  // namespace stx
