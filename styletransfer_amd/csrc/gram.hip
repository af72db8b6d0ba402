// Gram matrix + style loss for gfx950 (fp32 MFMA 32x32x2, split-K, deterministic).
//
//   G[b] = F_b F_b^T / (C*H*W),  F_b = z[b].view(C, H*W)
//   loss = mean((G - T)^2)  over B*C*C       (T broadcast over the batch)
//
// Reference: StyleLoss.gram_matrix / forward / set_target,
// stransfer/network.py:92-131 (torch.bmm(features, features_t).div(d*h*w);
// F.mse_loss(G, target.expand_as(G))).
//
// Kernel 1 (gram_partial): one block = one 64x64 tile (I<=J, symmetry) of one
// image over one K-split of the H*W pixels.  The block stages 64 rows x 64 pixels
// of F for tile-rows I and J in LDS (pitch 65: conflict-free column reads), each
// of the 4 waves owns a 32x32 quadrant.  Partials go to a workspace slab.
// Kernel 2 (gram_finalize): sums the splits in fixed order (bit-reproducible),
// scales, mirrors, and for the style loss also forms (G-T), the per-tile squared
// sum, and the backward coefficient matrix A = cA*(G-T) + alpha*I used by the
// Gram backward dF = A F (a 1x1 MFMA conv, see stx_gram_bwd).
#include "common.h"
#include "../../include/stx.h"

namespace stx {

constexpr int GT = 64;    // tile
constexpr int GKC = 64;   // pixels per LDS stage
constexpr int GP = GKC + 1;

__device__ __forceinline__ void tile_ij(int t, int nt, int& I, int& J) {
  // enumerate upper triangle row-major: (0,0),(0,1)..(0,nt-1),(1,1)...
  int i = 0;
  while (t >= nt - i) {
    t -= nt - i;
    ++i;
  }
  I = i;
  J = i + t;
}

__global__ void __launch_bounds__(256)
gram_partial_kernel(const float* __restrict__ z, float* __restrict__ ws, int c, int hw,
                    int nsplit, int split_len) {
  __shared__ __attribute__((aligned(16))) float smem[2 * GT * GP];
  float* rI = smem;
  float* rJ = smem + GT * GP;
  const int nt = cdiv(c, GT);
  const int ntu = nt * (nt + 1) / 2;
  int I, J;
  tile_ij(blockIdx.y, nt, I, J);
  const bool diag = I == J;
  const int split = blockIdx.x, b = blockIdx.z;
  const int p_begin = split * split_len;
  const int p_end = min(hw, p_begin + split_len);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int qi = wave >> 1, qj = wave & 1;
  const float* zb = z + (size_t)b * c * hw;

  // loader: thread -> (row = tid/4, 16 consecutive pixels at (tid%4)*16)
  const int lrow = tid >> 2, lseg = (tid & 3) * 16;
  float regI[16], regJ[16];
  auto fetch = [&](int p0) {
    const int gi = I * GT + lrow, gj = J * GT + lrow;
    const float* srcI = zb + (size_t)gi * hw + p0 + lseg;
    const float* srcJ = zb + (size_t)gj * hw + p0 + lseg;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int pp = p0 + lseg + e;
      const bool ok = pp < p_end;
      regI[e] = (ok && gi < c) ? srcI[e] : 0.f;
      if (!diag) regJ[e] = (ok && gj < c) ? srcJ[e] : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      rI[lrow * GP + lseg + e] = regI[e];
      if (!diag) rJ[lrow * GP + lseg + e] = regJ[e];
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const float* Bsrc = diag ? rI : rJ;
  const int a_off = (qi * 32 + l32) * GP + h * 32;
  const int b_off = (qj * 32 + l32) * GP + h * 32;

  if (p_begin < p_end) fetch(p_begin);
  for (int p0 = p_begin; p0 < p_end; p0 += GKC) {
    __syncthreads();
    store();
    __syncthreads();
    if (p0 + GKC < p_end) fetch(p0 + GKC);
#pragma unroll
    for (int s = 0; s < 32; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(rI[a_off + s], Bsrc[b_off + s], acc, 0, 0, 0);
  }
  float* out = ws + (((size_t)b * ntu + blockIdx.y) * nsplit + split) * (GT * GT);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = qi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    out[row * GT + qj * 32 + l32] = acc[r];
  }
}

// Register-direct Gram partial (hw % 4 == 0).  No LDS staging of F: lane
// (r = l&31, h = l>>5) of a wave streams 16 consecutive pixels of its own rows
// (float4 x4 per row: lanes l and l+32 cover one full 128-B line) and feeds them
// straight to v_mfma_f32_32x32x2_f32 — the k index of step t for lane half h is
// pixel p0 + 16h + t, identical for the A (rows I) and B (rows J) operands.
// Each wave owns a full 64x64 tile over its own 32-pixel steps (waves interleave
// steps); diagonal tiles (I == J) load each row once and skip the mirrored
// quadrant.  Blocks of one split run all of its tiles on one XCD (blocks b and
// b+8 share an XCD under round-robin dispatch) so the row tiles re-read by
// several tiles come from that XCD's L2 (speed only).  The 4 wave partials are
// summed through LDS into one deterministic slab per (block, tile).
// index of tile (I, J), I <= J, in the row-major upper-triangle enumeration
__device__ __forceinline__ int tile_index(int I, int J, int nt) {
  return I * nt - I * (I - 1) / 2 + (J - I);
}

// DIAG: one launch over the diagonal tiles (each row tile loaded once, 3 of the 4
// quadrants computed: fits 4 waves/SIMD); !DIAG: the off-diagonal tiles.
template <bool DIAG>
__global__ void __launch_bounds__(256, DIAG ? 4 : 2)
gram_partial_v2_kernel(const float* __restrict__ z, float* __restrict__ ws, int c, int hw,
                       int nsplit, int split_len) {
  __shared__ __attribute__((aligned(16))) float red[2 * GT * GT];
  const int nt = cdiv(c, GT);
  const int ntu = nt * (nt + 1) / 2;
  const int nk = DIAG ? nt : ntu - nt;  // tiles of this launch
  const int L = blockIdx.x;
  const int xcd = L & 7, rest = L >> 3;
  const int k = rest % nk, split = (rest / nk) * 8 + xcd;
  int I, J;
  if (DIAG) {
    I = J = k;
  } else {  // k-th pair I < J, row-major
    int i = 0, t = k;
    while (t >= nt - 1 - i) {
      t -= nt - 1 - i;
      ++i;
    }
    I = i;
    J = i + 1 + t;
  }
  const int tileu = tile_index(I, J, nt);
  constexpr bool diag = DIAG;
  const int b = blockIdx.z;
  const int p_begin = split * split_len;
  const int p_end = min(hw, p_begin + split_len);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const float* zb = z + (size_t)b * c * hw;
  const int ra0 = I * GT + r, ra1 = I * GT + 32 + r;
  const int rb0 = J * GT + r, rb1 = J * GT + 32 + r;
  const float* pa0 = zb + (size_t)min(ra0, c - 1) * hw;
  const float* pa1 = zb + (size_t)min(ra1, c - 1) * hw;
  const float* pb0 = zb + (size_t)min(rb0, c - 1) * hw;
  const float* pb1 = zb + (size_t)min(rb1, c - 1) * hw;
  const bool va0 = ra0 < c, va1 = ra1 < c, vb0 = rb0 < c, vb1 = rb1 < c;

  f32x16 a00, a01, a10, a11;
#pragma unroll
  for (int k = 0; k < 16; ++k) a00[k] = a01[k] = a10[k] = a11[k] = 0.f;

  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  for (int p0 = p_begin + wave * 32; p0 < p_end; p0 += 128) {
    f32x4 A0[4], A1[4];
    const int base = p0 + h * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pp = base + q * 4;
      const bool ok = pp < p_end;  // hw % 4 == 0: a float4 is all in or all out
      A0[q] = (ok && va0) ? *reinterpret_cast<const f32x4*>(pa0 + pp) : zero;
      A1[q] = (ok && va1) ? *reinterpret_cast<const f32x4*>(pa1 + pp) : zero;
    }
    if (diag) {
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float x0 = A0[t >> 2][t & 3], x1 = A1[t >> 2][t & 3];
        a00 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, x0, a00, 0, 0, 0);
        a01 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, x1, a01, 0, 0, 0);
        a11 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, x1, a11, 0, 0, 0);
      }
    } else {
      f32x4 B0[4], B1[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int pp = base + q * 4;
        const bool ok = pp < p_end;
        B0[q] = (ok && vb0) ? *reinterpret_cast<const f32x4*>(pb0 + pp) : zero;
        B1[q] = (ok && vb1) ? *reinterpret_cast<const f32x4*>(pb1 + pp) : zero;
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const float x0 = A0[t >> 2][t & 3], x1 = A1[t >> 2][t & 3];
        const float y0 = B0[t >> 2][t & 3], y1 = B1[t >> 2][t & 3];
        a00 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, y0, a00, 0, 0, 0);
        a01 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0, y1, a01, 0, 0, 0);
        a10 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, y0, a10, 0, 0, 0);
        a11 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1, y1, a11, 0, 0, 0);
      }
    }
  }
  // 4 wave partials -> 2 LDS images (32 KB): waves 2,3 store, waves 0,1 add, then sum
  auto put = [&](float* img, bool add) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int row = (k & 3) + 8 * (k >> 2) + 4 * h;
      float* q00 = img + row * GT + r;
      float* q01 = img + row * GT + 32 + r;
      float* q11 = img + (32 + row) * GT + 32 + r;
      float* q10 = img + (32 + row) * GT + r;
      *q00 = add ? *q00 + a00[k] : a00[k];
      *q01 = add ? *q01 + a01[k] : a01[k];
      *q11 = add ? *q11 + a11[k] : a11[k];
      if (!diag) *q10 = add ? *q10 + a10[k] : a10[k];
    }
  };
  if (wave >= 2) put(red + (wave - 2) * GT * GT, false);
  __syncthreads();
  if (wave < 2) put(red + wave * GT * GT, true);
  __syncthreads();
  float* out = ws + (((size_t)b * ntu + tileu) * nsplit + split) * (GT * GT);
#pragma unroll
  for (int q = 0; q < (GT * GT) / 256; ++q) {
    const int e = q * 256 + tid;
    int row = e / GT, col = e % GT;
    if (diag && row >= 32 && col < 32) {  // mirrored quadrant of a diagonal tile
      const int t = row;
      row = col;
      col = t;
    }
    const int o = row * GT + col;
    out[e] = red[o] + red[GT * GT + o];
  }
}

// fp16 hi/lo split Gram partial (hw % 8 == 0, z_amax = a device bound on max|z|).
// Same tiling, split-K and deterministic LDS reduction as gram_partial_v2_kernel,
// but every F element is scaled by a power of two s (s*max|z| < 2^15) and split
// s*f = hi + lo (fp16) and each 32x32 quadrant takes hi*hi + hi*lo + lo*hi on
// v_mfma_f32_32x32x16_f16 (fp32-level accuracy, conv16.hip): the matrix pipe does
// 16 pixels in 3 x 32 cycles where the fp32 MFMA needs 8 x 64, so the kernel is
// bound by reading F.  Lane (r, h) feeds pixels [8h, 8h+8) of each 16-pixel step
// from its own rows (two float4), identical for the A (rows I) and B (rows J)
// operands; a wave walks 32-pixel groups (two steps) with the next group's loads
// in flight.  Partials are de-scaled by 1/s^2 (exact) before the reduction.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int gram_amax_exp(float a) {
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

__device__ __forceinline__ void split8(const f32x4& x0, const f32x4& x1, float s, f16x8_t& hi,
                                       f16x8_t& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float v = (e < 4 ? x0[e] : x1[e - 4]) * s;
    const _Float16 vh = (_Float16)v;
    hi[e] = vh;
    lo[e] = (_Float16)(v - (float)vh);
  }
}

#define MF16(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0)

// One launch over all upper-triangle tiles (a block-uniform branch picks the
// diagonal or off-diagonal body) so that small-C x large-HW and large-C x small-HW
// layers both fill the chip with ~512 blocks.
template <bool DIAG>
__device__ __forceinline__ void gram_f16_tile(const float* __restrict__ z, float* __restrict__ ws,
                                              int c, int hw, int nsplit, int split_len,
                                              const float* __restrict__ z_amax, int I, int J,
                                              int split, float* red);

__global__ void __launch_bounds__(256, 2)
gram_partial_f16_kernel(const float* __restrict__ z, float* __restrict__ ws, int c, int hw,
                        int nsplit, int split_len, const float* __restrict__ z_amax) {
  __shared__ __attribute__((aligned(16))) float red[2 * GT * GT];
  const int nt = cdiv(c, GT);
  const int ntu = nt * (nt + 1) / 2;
  const int L = blockIdx.x;
  const int xcd = L & 7, rest = L >> 3;
  const int k = rest % ntu, split = (rest / ntu) * 8 + xcd;
  int I, J;
  tile_ij(k, nt, I, J);
  if (I == J)
    gram_f16_tile<true>(z, ws, c, hw, nsplit, split_len, z_amax, I, J, split, red);
  else
    gram_f16_tile<false>(z, ws, c, hw, nsplit, split_len, z_amax, I, J, split, red);
}

template <bool DIAG>
__device__ __forceinline__ void gram_f16_tile(const float* __restrict__ z, float* __restrict__ ws,
                                              int c, int hw, int nsplit, int split_len,
                                              const float* __restrict__ z_amax, int I, int J,
                                              int split, float* red) {
  const int nt = cdiv(c, GT);
  const int ntu = nt * (nt + 1) / 2;
  const int tileu = tile_index(I, J, nt);
  const int b = blockIdx.z;
  const int p_begin = split * split_len;
  const int p_end = min(hw, p_begin + split_len);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const float* zb = z + (size_t)b * c * hw;
  const int ra0 = I * GT + r, ra1 = I * GT + 32 + r;
  const int rb0 = J * GT + r, rb1 = J * GT + 32 + r;
  // branch-free loads: rows past c and pixels past the split read 0 through the
  // buffer descriptor's range check (a predicated load compiles to an exec branch and
  // a vmcnt(0) join, which serialised the double-buffered groups)
  const auto rz = make_srd(zb, (uint32_t)c * (uint32_t)hw * 4u);
  const uint32_t oa0 = ra0 < c ? (uint32_t)(ra0 * hw + 8 * h) * 4u : BUF_OOB;
  const uint32_t oa1 = ra1 < c ? (uint32_t)(ra1 * hw + 8 * h) * 4u : BUF_OOB;
  const uint32_t ob0 = rb0 < c ? (uint32_t)(rb0 * hw + 8 * h) * 4u : BUF_OOB;
  const uint32_t ob1 = rb1 < c ? (uint32_t)(rb1 * hw + 8 * h) * 4u : BUF_OOB;
  const int e = gram_amax_exp(read_amax(z_amax));
  const float sx = __builtin_ldexpf(1.f, 15 - e);
  const float inv2 = __builtin_ldexpf(1.f, 2 * e - 30);

  f32x16 a00, a01, a10, a11;
#pragma unroll
  for (int q = 0; q < 16; ++q) a00[q] = a01[q] = a10[q] = a11[q] = 0.f;

  // one 32-pixel group: [step s][half of the 8 pixels] float4s per row
  struct Grp {
    f32x4 x[4][2][2];  // [row a0, a1, b0, b1][step][lo/hi float4]
  };
  auto load = [&](int p0, Grp& g) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int pp = p0 + 16 * st;       // + 8h folded into the row offsets
      const bool ok = pp + 8 * h < p_end;  // hw % 8 == 0: a lane's 8 pixels all in or out
      const uint32_t po = ok ? (uint32_t)pp * 4u : BUF_OOB;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        g.x[0][st][q] = buf_ld4(rz, (oa0 | (po & BUF_OOB)) + (po & ~BUF_OOB) + 16u * q);
        g.x[1][st][q] = buf_ld4(rz, (oa1 | (po & BUF_OOB)) + (po & ~BUF_OOB) + 16u * q);
        if (!DIAG) {
          g.x[2][st][q] = buf_ld4(rz, (ob0 | (po & BUF_OOB)) + (po & ~BUF_OOB) + 16u * q);
          g.x[3][st][q] = buf_ld4(rz, (ob1 | (po & BUF_OOB)) + (po & ~BUF_OOB) + 16u * q);
        }
      }
    }
  };
  auto compute = [&](const Grp& g) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      f16x8_t h0, l0, h1, l1;
      split8(g.x[0][st][0], g.x[0][st][1], sx, h0, l0);
      split8(g.x[1][st][0], g.x[1][st][1], sx, h1, l1);
      if (DIAG) {
        a00 = MF16(h0, h0, a00); a01 = MF16(h0, h1, a01); a11 = MF16(h1, h1, a11);
        a00 = MF16(h0, l0, a00); a01 = MF16(h0, l1, a01); a11 = MF16(h1, l1, a11);
        a00 = MF16(l0, h0, a00); a01 = MF16(l0, h1, a01); a11 = MF16(l1, h1, a11);
      } else {
        f16x8_t g0, m0, g1, m1;
        split8(g.x[2][st][0], g.x[2][st][1], sx, g0, m0);
        split8(g.x[3][st][0], g.x[3][st][1], sx, g1, m1);
        a00 = MF16(h0, g0, a00); a01 = MF16(h0, g1, a01);
        a10 = MF16(h1, g0, a10); a11 = MF16(h1, g1, a11);
        a00 = MF16(h0, m0, a00); a01 = MF16(h0, m1, a01);
        a10 = MF16(h1, m0, a10); a11 = MF16(h1, m1, a11);
        a00 = MF16(l0, g0, a00); a01 = MF16(l0, g1, a01);
        a10 = MF16(l1, g0, a10); a11 = MF16(l1, g1, a11);
      }
    }
  };
  // waves interleave 32-pixel groups: wave w takes p_begin + 32*(w + 4*i)
  int p0 = p_begin + wave * 32;
  if (p0 < p_end) {
    Grp cur, nxt;
    load(p0, cur);
    for (; p0 < p_end; p0 += 128) {
      if (p0 + 128 < p_end) load(p0 + 128, nxt);
      compute(cur);
      cur = nxt;
    }
  }
  // 4 wave partials -> 2 LDS images (32 KB): waves 2,3 store, waves 0,1 add, then sum
  auto put = [&](float* img, bool add) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
      float* q00 = img + row * GT + r;
      float* q01 = img + row * GT + 32 + r;
      float* q11 = img + (32 + row) * GT + 32 + r;
      float* q10 = img + (32 + row) * GT + r;
      *q00 = add ? *q00 + a00[q] : a00[q];
      *q01 = add ? *q01 + a01[q] : a01[q];
      *q11 = add ? *q11 + a11[q] : a11[q];
      if (!DIAG) *q10 = add ? *q10 + a10[q] : a10[q];
    }
  };
  if (wave >= 2) put(red + (wave - 2) * GT * GT, false);
  __syncthreads();
  if (wave < 2) put(red + wave * GT * GT, true);
  __syncthreads();
  float* out = ws + (((size_t)b * ntu + tileu) * nsplit + split) * (GT * GT);
#pragma unroll
  for (int q = 0; q < (GT * GT) / 256; ++q) {
    const int el = q * 256 + tid;
    int row = el / GT, col = el % GT;
    if (DIAG && row >= 32 && col < 32) {  // mirrored quadrant of a diagonal tile
      const int t = row;
      row = col;
      col = t;
    }
    const int o = row * GT + col;
    out[el] = (red[o] + red[GT * GT + o]) * inv2;
  }
}
#undef MF16

// Whole-triangle split Gram for C = 128 / 256 (the conv2_x / conv3_1 taps): a block
// takes a pixel range of one image and ALL 32 x 32 blocks of the upper triangle of
// G (10 / 36 of them), so z is read exactly once (the 64 x 64-tile kernel above reads
// every row (nt + 1) / 2 times).  Per chunk of 64 pixels the C x 64 slab is split
// into fp16 hi/lo planes in LDS ([plane][channel][pixel], pitch 72 halves: the 16-B
// fragment reads of 16 lanes hit distinct banks) -- once per element instead of once
// per tile that uses it -- with the next chunk's loads in flight; wave w owns blocks
// w, w + 4, ... (3 MFMAs per block per 16 pixels).  The partials are written in the
// 64 x 64-tile layout gram_finalize_kernel reads (diagonal tiles with the mirrored
// lower-left quadrant).
// MSE: also the content/feature sums of (z - cz)^2 and (relu z - relu cz)^2 over the
// block's pixels (the pass over z the content loss needs anyway): mparts[2 blk + 0/1]
template <int C, bool MSE = false>
__global__ void __launch_bounds__(256, 1)
gram_tri_f16_kernel(const float* __restrict__ z, float* __restrict__ ws, int hw, int nsplit,
                    int split_len, const float* __restrict__ z_amax,
                    const float* __restrict__ cz = nullptr, float* __restrict__ mparts = nullptr) {
  constexpr int NB = C / 32;                 // 32-row blocks per side
  constexpr int NBLK = NB * (NB + 1) / 2;    // upper-triangle blocks
  constexpr int PER = (NBLK + 3) / 4;        // per wave
  constexpr int NPX = 64, HP = NPX + 8;      // pixels per chunk, plane pitch (halves)
  constexpr int NL = C * NPX / 4 / 256;      // float4 loads per thread per chunk
  constexpr int NT = C / GT, NTU = NT * (NT + 1) / 2;
  __shared__ __attribute__((aligned(16))) _Float16 pl[2 * C * HP];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int split = blockIdx.x, b = blockIdx.z;
  const int p0 = split * split_len, p1 = min(hw, p0 + split_len);
  const float* zb = z + (size_t)b * C * hw;
  const auto rz = make_srd(zb, (uint32_t)C * (uint32_t)hw * 4u);
  const auto rc = make_srd(MSE ? cz + (size_t)b * C * hw : zb, (uint32_t)C * (uint32_t)hw * 4u);
  float ms = 0.f, msr = 0.f;  // MSE sums
  const int e = gram_amax_exp(read_amax(z_amax));
  const float sx = __builtin_ldexpf(1.f, 15 - e), inv2 = __builtin_ldexpf(1.f, 2 * e - 30);
  // this wave's blocks (bi <= bj), row-major over the upper triangle
  int bi[PER], bj[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    int t = wave + 4 * q, i = 0;
    if (t >= NBLK) t = 0;  // padding slot (its result is not stored)
    while (t >= NB - i) {
      t -= NB - i;
      ++i;
    }
    bi[q] = i;
    bj[q] = i + t;
  }
  f32x16 acc[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  // loads: float4 f = tid + 256 r -> (channel f / 16, pixels 4 (f % 16) ..)
  f32x4 ld[NL];
  f32x4 lc[MSE ? NL : 1];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int f = tid + 256 * r, ch = f >> 4, px = c0 + 4 * (f & 15);
      const uint32_t o = px < p1 ? (uint32_t)(ch * hw + px) * 4u : BUF_OOB;
      ld[r] = buf_ld4(rz, o);
      if constexpr (MSE) lc[r] = buf_ld4(rc, o);
    }
  };
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  auto stage = [&]() {
#pragma unroll
    for (int r = 0; r < NL; ++r) {
      const int f = tid + 256 * r, ch = f >> 4, px = 4 * (f & 15);
      f16x4 hi, lo;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = ld[r][k] * sx;
        hi[k] = (_Float16)v;
        lo[k] = (_Float16)(v - (float)hi[k]);
        if constexpr (MSE) {  // out-of-range pixels read 0 on both sides: no contribution
          const float d = ld[r][k] - lc[r][k], dr = relu_bits(ld[r][k]) - relu_bits(lc[r][k]);
          ms += d * d;
          msr += dr * dr;
        }
      }
      *reinterpret_cast<f16x4*>(pl + ch * HP + px) = hi;
      *reinterpret_cast<f16x4*>(pl + (C + ch) * HP + px) = lo;
    }
  };
  if (p0 < p1) fetch(p0);
  for (int c0 = p0; c0 < p1; c0 += NPX) {
    __syncthreads();  // the previous chunk's fragment reads are done
    stage();
    __syncthreads();
    if (c0 + NPX < p1) fetch(c0 + NPX);  // in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < NPX / 16; ++ks) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        if (wave + 4 * q >= NBLK) continue;
        const _Float16* ra = pl + (bi[q] * 32 + l32) * HP + ks * 16 + 8 * h;
        const _Float16* rb = pl + (bj[q] * 32 + l32) * HP + ks * 16 + 8 * h;
        const f16x8_t ah = *reinterpret_cast<const f16x8_t*>(ra);
        const f16x8_t al = *reinterpret_cast<const f16x8_t*>(ra + C * HP);
        const f16x8_t bh = *reinterpret_cast<const f16x8_t*>(rb);
        const f16x8_t bl = *reinterpret_cast<const f16x8_t*>(rb + C * HP);
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[q], 0, 0, 0);
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[q], 0, 0, 0);
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[q], 0, 0, 0);
      }
    }
  }
  if constexpr (MSE) {
    __shared__ float mred[4];
    ms = block_sum<256>(ms, mred);
    msr = block_sum<256>(msr, mred);
    if (tid == 0) {
      const int blk = b * nsplit + split;
      mparts[2 * blk] = ms;
      mparts[2 * blk + 1] = msr;
    }
  }
  // partials in the 64 x 64-tile layout [b][tile][split][64][64]
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (wave + 4 * q >= NBLK) continue;
    const int I = bi[q] >> 1, J = bj[q] >> 1, qi = bi[q] & 1, qj = bj[q] & 1;
    float* out = ws + (((size_t)b * NTU + tile_index(I, J, NT)) * nsplit + split) * (GT * GT);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = acc[q][r] * inv2;
      out[(qi * 32 + row) * GT + qj * 32 + l32] = v;
      if (I == J && qi != qj) out[(qj * 32 + l32) * GT + qi * 32 + row] = v;  // mirror
    }
  }
}

// C = 256 (VGG conv3_1's tap): the whole upper triangle of G per block, on 8 waves.  A
// block takes one image's pixel range and ALL 36 upper-triangle 32 x 32 blocks (row panels
// w and 7 - w to waves 2 (w % 4) .. +1, four or five blocks each, so a wave's blocks share
// their A fragments), z read once from HBM and split once into fp16 hi/lo.  Per chunk of
// 32 pixels the 256 x 32 slab goes to LDS as 16-B fragment units (8 pixels of one channel)
// at unit c * 4 + (g ^ ((c >> 2) & 3)) (g = 8-pixel group): the swizzle keeps both the
// staging stores (4 lanes per channel) and the fragment reads (32 lanes over 32
// channels) conflict-free.  Double-buffered chunks, one barrier per chunk, the next
// chunk's loads in flight during the MFMAs.  The 64 x 64-tile kernel it replaces read
// every 64-row panel (nt + 1) / 2 times and split it once per tile (640 blocks, 19 us at
// 128^2); the 4-wave triangle kernel (1 wave per SIMD, 9 accumulator blocks per wave)
// was slower still.  Partials: the 64 x 64-tile layout gram_finalize reads.
constexpr int T256_PX = 32;  // pixels per chunk
template <bool STAGED>
__global__ void __launch_bounds__(512, 1)
gram_tri256_kernel(const float* __restrict__ z, float* __restrict__ ws, int hw, int nsplit,
                   int split_len, const float* __restrict__ z_amax) {
  constexpr int C = 256, NB = 8, NT = C / GT, NTU = NT * (NT + 1) / 2;
  constexpr int UNITS = C * T256_PX / 8;       // 16-B units per plane per chunk (1024)
  constexpr int PLANE = UNITS * 16;            // bytes (16 KB)
  constexpr int BUF = 2 * PLANE;               // hi + lo
  __shared__ __attribute__((aligned(16))) char lds[2 * BUF];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int split = blockIdx.x, b = blockIdx.z;
  const int p0 = split * split_len, p1 = min(hw, p0 + split_len);
  const auto rz = make_srd(z + (size_t)b * C * hw, (uint32_t)C * (uint32_t)hw * 4u);
  const int e = gram_amax_exp(read_amax(z_amax));
  const float sx = __builtin_ldexpf(1.f, 15 - e), inv2 = __builtin_ldexpf(1.f, 2 * e - 30);
  // this wave's blocks: the 9 blocks of row panels (w, 7 - w), w = wave / 2, in order
  // (panel w: bj = w .. 7, then panel 7 - w: bj = 7 - w .. 7); the even wave takes the
  // first five, the odd wave the other four
  constexpr int PER = 5;
  int bi[PER], bj[PER];
  bool uA[PER];  // block q's A panel is 7 - pw (else pw)
  const int pw = wave >> 1, first = (wave & 1) ? 5 : 0, cnt = (wave & 1) ? 4 : 5;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    int t = min(first + q, first + cnt - 1);  // (slot past cnt: a copy, not stored)
    const int n0 = NB - pw;                   // blocks in panel pw
    uA[q] = t >= n0;
    if (t < n0) {
      bi[q] = pw;
      bj[q] = pw + t;
    } else {
      bi[q] = NB - 1 - pw;
      bj[q] = NB - 1 - pw + (t - n0);
    }
  }
  f32x16 acc[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  // staging: unit u = tid + 512 r (r = 0, 1) -> channel u >> 2, 8-pixel group u & 3
  f32x4 ld[2][2];
  uint32_t ch_off[2];
  int slot[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int u = tid + 512 * r, c = u >> 2, g = u & 3;
    ch_off[r] = (uint32_t)(c * hw + 8 * g) * 4u;
    slot[r] = (c * 4 + (g ^ ((c >> 2) & 3))) * 16;
  }
  auto fetch = [&](int c0) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int g = (tid + 512 * r) & 3;
      const uint32_t o = c0 + 8 * g < p1 ? ch_off[r] + (uint32_t)c0 * 4u : BUF_OOB;
      ld[r][0] = buf_ld4(rz, o);
      ld[r][1] = buf_ld4(rz, o + 16u);
    }
  };
  auto stage = [&](int buf) {
    char* base = lds + buf * BUF;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      f16x8_t hi, lo;
      split8(ld[r][0], ld[r][1], sx, hi, lo);
      *reinterpret_cast<f16x8_t*>(base + slot[r]) = hi;
      *reinterpret_cast<f16x8_t*>(base + PLANE + slot[r]) = lo;
    }
  };
  // fragment unit of (block row panel, k-step s) for this lane: channel 32 panel + l32,
  // group 2 s + h
  auto frag_off = [&](int panel, int s) {
    const int c = 32 * panel + l32, g = 2 * s + h;
    return (c * 4 + (g ^ ((c >> 2) & 3))) * 16;
  };
  int buf = 0;
  if (p0 < p1) {
    fetch(p0);
    stage(0);
    if (p0 + T256_PX < p1) fetch(p0 + T256_PX);
  }
  for (int c0 = p0; c0 < p1; c0 += T256_PX, buf ^= 1) {
    __syncthreads();  // buffer buf complete; the other buffer's reads (chunk c0 - 32) done
    const char* base = lds + buf * BUF;
    // per k-step every fragment first (A panels pw and 7 - pw -- uA[q]: which one block q
    // uses, wave-uniform -- and one B panel per block; a diagonal block reads its A panel
    // again), then the step's MFMAs
#pragma unroll
    for (int st = 0; st < T256_PX / 16; ++st) {
      f16x8_t fa[2][2], fb[PER][2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int oa = frag_off(a ? NB - 1 - pw : pw, st);
        fa[a][0] = *reinterpret_cast<const f16x8_t*>(base + oa);
        fa[a][1] = *reinterpret_cast<const f16x8_t*>(base + PLANE + oa);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        if (q >= cnt) break;
        const int ob = frag_off(bj[q], st);
        fb[q][0] = *reinterpret_cast<const f16x8_t*>(base + ob);
        fb[q][1] = *reinterpret_cast<const f16x8_t*>(base + PLANE + ob);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        if (q >= cnt) break;
        const int a = uA[q] ? 1 : 0;
        if (a) {
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1][0], fb[q][0], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1][0], fb[q][1], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1][1], fb[q][0], acc[q], 0, 0, 0);
        } else {
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0][0], fb[q][0], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0][0], fb[q][1], acc[q], 0, 0, 0);
          acc[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0][1], fb[q][0], acc[q], 0, 0, 0);
        }
      }
    }
    if (c0 + T256_PX < p1) {  // the next chunk -> the other buffer, its successor's loads
      stage(buf ^ 1);
      if (c0 + 2 * T256_PX < p1) fetch(c0 + 2 * T256_PX);
    }
  }
  // partials in the 64 x 64-tile layout [b][tile][split][64][64] (diagonal tiles with the
  // mirrored lower-left quadrant)
  if constexpr (STAGED) {
    // each wave's 32 x 32 block through its own LDS region (pitch 40 floats: the two lane
    // halves' rows land 32 banks apart), then 16-B stores: 8 rows x 128 B per store
    // instruction instead of 2 x 128 B
    constexpr int PITCH = 40;
    float* reg = reinterpret_cast<float*>(lds) + wave * 32 * PITCH;
    __syncthreads();  // the last chunk's fragment reads are done
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (q >= cnt) break;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        reg[((r & 3) + 8 * (r >> 2) + 4 * h) * PITCH + l32] = acc[q][r] * inv2;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS stores landed
      const int I = bi[q] >> 1, J = bj[q] >> 1, qi = bi[q] & 1, qj = bj[q] & 1;
      float* out = ws + (((size_t)b * NTU + tile_index(I, J, NT)) * nsplit + split) * (GT * GT);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int row = (lane >> 3) + 8 * k, c4 = lane & 7;
        const f32x4 v = *reinterpret_cast<const f32x4*>(reg + row * PITCH + 4 * c4);
        *reinterpret_cast<f32x4*>(out + (qi * 32 + row) * GT + qj * 32 + 4 * c4) = v;
        if (I == J && qi != qj) {  // mirror: row `row` of the transposed block
          f32x4 m;
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] = reg[(4 * c4 + e) * PITCH + row];
          *reinterpret_cast<f32x4*>(out + (qj * 32 + row) * GT + qi * 32 + 4 * c4) = m;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next stores
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (q >= cnt) break;
    const int I = bi[q] >> 1, J = bj[q] >> 1, qi = bi[q] & 1, qj = bj[q] & 1;
    float* out = ws + (((size_t)b * NTU + tile_index(I, J, NT)) * nsplit + split) * (GT * GT);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = acc[q][r] * inv2;
      out[(qi * 32 + row) * GT + qj * 32 + l32] = v;
      if (I == J && qi != qj) out[(qj * 32 + l32) * GT + qi * 32 + row] = v;  // mirror
    }
  }
}

// splits per image of gram_tri256_kernel: ~256 blocks over the batch, at least 128 pixels
// (4 chunks) per block, a multiple of 8 splits
static int gram_tri256_splits(int hw, int b) {
  static const int target = std::max(8, STX_KNOB("STX_GRAM256_BLOCKS", 256));
  int want = std::max(1, target / std::max(1, b));
  want = std::min(want, std::max(1, hw / 128));
  return want;
}

static bool gram_tri256_on(int c, int hw) {
  static const bool on = STX_KNOB("STX_GRAM_TRI256", 1) != 0;
  return on && c == 256 && hw % 32 == 0;
}

static int gram_tri_splits(int c, int hw, int b) {
  // C = 128 @ 256^2: 256 > 128 > 64 blocks (A/B)
  static const int target = std::max(8, STX_KNOB("STX_GRAM_TRI_BLOCKS", 256));
  // ~target blocks over the whole batch (the partial slab grows with b * splits)
  return std::max(1, std::min(std::max(1, target / std::max(1, b)), hw / 64));
}

static bool gram_tri_on(int c, int hw) {
  static const bool on = STX_KNOB("STX_GRAM_TRI", 1) != 0;
  // C = 256 @ 128^2 measured slower than the 64 x 64-tile kernel (36 vs 10 blocks of
  // accumulators per block: 33-37 us vs 32 us with the finalize); STX_GRAM_TRI=2 forces it
  static const bool all = STX_KNOB("STX_GRAM_TRI", 1) == 2;
  return on && (c == 128 || (all && c == 256)) && hw % 64 == 0;
}

// grid (ntu * FSUB, B), 512 threads: 64 tile elements (16 lanes x float4, one 256-B
// row segment of every partial) x 32 split-lanes.  Split-lane kl sums partials kl,
// kl + 32, ... (four float4 accumulators, so each lane keeps several loads in flight);
// the 32 lane sums of an element are added through LDS in split-lane order, so the
// result is bit-reproducible.  (64 split-lanes in 1024-thread blocks left each lane 4
// partials at fast_st's batch: the batched launch 57.2 -> 52.5 us there, Gatys 17.3 ->
// 15.4 us with 32; 16 lanes: 50.2 / 18.1 us; 16-element x 16-lane blocks reading 64-B
// segments were latency-bound: 11.8 us for the 16.8 MB of C=64 @ 512^2 partials.)
constexpr int FEL = 64, FKL = 32, FNT = FEL / 4 * FKL;  // elements, split-lanes, threads
constexpr int FSUB = GT * GT / FEL;   // 64-element sub-tiles per tile (loss partials)
// Few partials per tile (the 128 / 256-channel taps at small HW and large batch: a handful
// of splits) would leave most of a block's split-lanes idle: such a block takes G = 2 or 4
// sub-tiles with 32 / G split-lanes each (G from nsplit, so every caller of a tap picks
// the same order and the same bits).
__host__ __device__ inline int fin_groups(int nsplit) { return nsplit <= 8 ? 4 : nsplit <= 16 ? 2 : 1; }
__host__ __device__ inline int fin_blocks_per_tile(int nsplit) { return FSUB / fin_groups(nsplit); }

// block (bx, by) of a finalize over grid (ntu * fin_blocks_per_tile(nsplit), b)
template <int G>
__device__ __forceinline__ void gram_finalize_body_g(
    const float* __restrict__ ws, int c, int nsplit, float scale, float* __restrict__ g_out,
    const float* __restrict__ target, long long t_bstride, float* __restrict__ coef, int cpad,
    float cA, float alpha, float* __restrict__ loss_parts, int bx, int by, float* part,
    float* __restrict__ coef_amax) {
  constexpr int KL = FKL / G, GT_ = FNT / G;  // split-lanes and threads per sub-tile
  const int nt = cdiv(c, GT), ntu = nt * (nt + 1) / 2;
  const int tile = bx / (FSUB / G), r = threadIdx.x / GT_, sub = (bx % (FSUB / G)) * G + r;
  int I, J;
  tile_ij(tile, nt, I, J);
  const int b = by;
  const float* src = ws + ((size_t)b * ntu + tile) * nsplit * (GT * GT) + sub * FEL;
  const int t2 = threadIdx.x % GT_, q4 = t2 % (FEL / 4), kl = t2 / (FEL / 4);
  float* pr = part + (size_t)r * KL * (FEL + 1);  // this sub-tile's [KL][FEL + 1]
  {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    const f32x4* p4 = reinterpret_cast<const f32x4*>(src) + q4;
    constexpr int ST = GT * GT / 4;  // float4s per partial
    int k = kl;
    for (; k + 3 * KL < nsplit; k += 4 * KL) {
      const f32x4 a0 = p4[(size_t)(k + 0 * KL) * ST], a1 = p4[(size_t)(k + 1 * KL) * ST];
      const f32x4 a2 = p4[(size_t)(k + 2 * KL) * ST], a3 = p4[(size_t)(k + 3 * KL) * ST];
      s0 += a0;
      s1 += a1;
      s2 += a2;
      s3 += a3;
    }
    for (; k < nsplit; k += KL) s0 += p4[(size_t)k * ST];
    const f32x4 t = (s0 + s1) + (s2 + s3);
#pragma unroll
    for (int i = 0; i < 4; ++i) pr[kl * (FEL + 1) + 4 * q4 + i] = t[i];
  }
  __syncthreads();
  float sq = 0.f, ma = 0.f;
  if (t2 < FEL) {  // one wave per sub-tile
    const int el = t2, e = sub * FEL + el;
    float s = 0.f;
#pragma unroll 8
    for (int q = 0; q < KL; ++q) s += pr[q * (FEL + 1) + el];
    const int gi = I * GT + e / GT, gj = J * GT + e % GT;
    if (gi < c && gj < c) {
      const float g = s * scale;
      if (g_out) {
        g_out[((size_t)b * c + gi) * c + gj] = g;
        if (I != J) g_out[((size_t)b * c + gj) * c + gi] = g;
      }
      if (target) {
        const float d = g - target[(size_t)b * t_bstride + (size_t)gi * c + gj];
        sq = (I != J ? 2.f : 1.f) * d * d;
        if (coef) {
          const float a = cA * d;
          float* cb = coef + (size_t)b * cpad * cpad;
          const float ad = a + (gi == gj ? alpha : 0.f);
          cb[(size_t)gi * cpad + gj] = ad;
          if (I != J) cb[(size_t)gj * cpad + gi] = a;
          ma = fmaxf(fabsf(ad), fabsf(a));
        }
      }
    }
    if (target) {  // the sub-tile's loss partial: its one wave's sum
      const float t = wave_sum(sq);
      if (t2 == 0) loss_parts[(size_t)b * ntu * FSUB + (size_t)tile * FSUB + sub] = t;
    }
    if (coef_amax) {  // max|A| of the batch for the split Gram-backward phase
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ma = fmaxf(ma, __shfl_xor(ma, o, 64));
      if (t2 == 0)  // |v| >= 0: the bit pattern orders like the value
        atomicMax(reinterpret_cast<unsigned int*>(coef_amax + (bx & (STX_AMAX_SLOTS - 1))),
                  __float_as_uint(ma));
    }
  }
}

__device__ __forceinline__ void gram_finalize_body(
    const float* __restrict__ ws, int c, int nsplit, float scale, float* __restrict__ g_out,
    const float* __restrict__ target, long long t_bstride, float* __restrict__ coef, int cpad,
    float cA, float alpha, float* __restrict__ loss_parts, const float* __restrict__ mse_parts,
    int mse_nparts, double mse_n, float* __restrict__ mse_out, int bx, int by,
    float* __restrict__ coef_amax = nullptr) {
  __shared__ float part[FKL * (FEL + 1)];
  __shared__ float red[FNT / 64];
  // block (0, 0) also finalizes the content / feature MSE partials of a fused content
  // pass (gram_tri_f16_kernel<128, true>): the launch a separate mse2 finalize would take
  if (mse_out && bx == 0 && by == 0) {
    float s = 0.f, sr = 0.f;
    for (int i = threadIdx.x; i < mse_nparts; i += FNT) {
      s += mse_parts[2 * i];
      sr += mse_parts[2 * i + 1];
    }
    s = block_sum<FNT>(s, red);
    sr = block_sum<FNT>(sr, red);
    if (threadIdx.x == 0) {
      const float mr = (float)(sr / mse_n);
      mse_out[0] = (float)(s / mse_n);
      mse_out[1] = (float)((double)(mr * mr) / mse_n);
      mse_out[2] = mr;
    }
  }
  switch (fin_groups(nsplit)) {
    case 4:
      gram_finalize_body_g<4>(ws, c, nsplit, scale, g_out, target, t_bstride, coef, cpad, cA,
                              alpha, loss_parts, bx, by, part, coef_amax);
      break;
    case 2:
      gram_finalize_body_g<2>(ws, c, nsplit, scale, g_out, target, t_bstride, coef, cpad, cA,
                              alpha, loss_parts, bx, by, part, coef_amax);
      break;
    default:
      gram_finalize_body_g<1>(ws, c, nsplit, scale, g_out, target, t_bstride, coef, cpad, cA,
                              alpha, loss_parts, bx, by, part, coef_amax);
  }
}

__global__ void __launch_bounds__(FNT)
gram_finalize_kernel(const float* __restrict__ ws, int c, int nsplit, float scale,
                     float* __restrict__ g_out, const float* __restrict__ target, long long t_bstride,
                     float* __restrict__ coef, int cpad, float cA, float alpha,
                     float* __restrict__ loss_parts, const float* __restrict__ mse_parts = nullptr,
                     int mse_nparts = 0, double mse_n = 1.0, float* __restrict__ mse_out = nullptr) {
  gram_finalize_body(ws, c, nsplit, scale, g_out, target, t_bstride, coef, cpad, cA, alpha,
                     loss_parts, mse_parts, mse_nparts, mse_n, mse_out, blockIdx.x, blockIdx.y);
}

// the finalizes of several style losses (one per VGG tap) in ONE launch: block ranges
// per job, each block the body of gram_finalize_kernel (same arithmetic, same order)
struct FinBatch {
  stx_gram_fin_job job[STX_FIN_MAX];
  int blk0[STX_FIN_MAX + 1];
  int njobs;
};

__global__ void __launch_bounds__(FNT) gram_finalize_batch_kernel(FinBatch fb) {
  int j = 0;
  while (j + 1 < fb.njobs && (int)blockIdx.x >= fb.blk0[j + 1]) ++j;
  const stx_gram_fin_job& q = fb.job[j];
  const int local = blockIdx.x - fb.blk0[j];
  const int nt = cdiv(q.c, GT), nbx = nt * (nt + 1) / 2 * fin_blocks_per_tile(q.nsplit);
  gram_finalize_body(q.parts, q.c, q.nsplit, q.scale, q.g_out, q.target, q.t_bstride, q.coef,
                     q.cpad, q.cA, q.alpha, q.loss_parts, q.mse_parts, q.mse_nparts, q.mse_n,
                     q.mse_out, local % nbx, local / nbx, q.coef_amax);
}

// one wave: the fixed-order sum of n loss partials (4 lane-strided accumulators, then a
// wave tree) -- shared by sum_parts_kernel and loss_finalize_kernel so the deferred and
// direct style losses are the same bits
__device__ __forceinline__ float wave_sum_parts(const float* __restrict__ parts, int n, int lane) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int i = lane;
  for (; i + 192 < n; i += 256) {
    s0 += parts[i];
    s1 += parts[i + 64];
    s2 += parts[i + 128];
    s3 += parts[i + 192];
  }
  for (; i < n; i += 64) s0 += parts[i];
  return wave_sum((s0 + s1) + (s2 + s3));
}

// single wave: loss = inv * sum(parts)
__global__ void sum_parts_kernel(const float* __restrict__ parts, int n, float inv,
                                 float* __restrict__ out) {
  const float s = wave_sum_parts(parts, n, threadIdx.x);
  if (threadIdx.x == 0) *out = s * inv;
}

__global__ void zero_kernel(float* p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

struct LossWF {
  float w[16];
};

static void gram_geometry(int c, int hw, int b, int& nsplit, int& split_len, int& ntu) {
  const int nt = cdiv(c, GT);
  ntu = nt * (nt + 1) / 2;
  if (hw % 4 == 0) {
    // v2: splits in multiples of 8 (XCD grouping), >= 512 pixels (4 steps/wave),
    // ~4 blocks per CU
    int want = rup(cdiv(1024, ntu * b), 8);
    const int max_splits = std::max(1, cdiv(hw, 512));
    want = std::max(8, std::min(want, rup(max_splits, 8)));
    split_len = rup(cdiv(hw, want), 128);
    nsplit = rup(cdiv(hw, split_len), 8);
    return;
  }
  const int chunks = cdiv(hw, GKC);
  // aim for ~512 blocks (2 per CU), at least 8 chunks (512 pixels) per split
  int want = cdiv(512, ntu * b);
  want = std::max(1, std::min(want, cdiv(chunks, 8)));
  const int per = cdiv(chunks, want);
  split_len = per * GKC;
  nsplit = cdiv(hw, split_len);
}

// split geometry of the fp16 split kernel: 32-pixel groups interleaved over 4 waves,
// splits in multiples of 256 pixels (whole groups) and of 8 (XCD grouping), each
// wave >= 2 groups, ~640 blocks (2-3 per CU: enough bytes in flight)
static void gram_geometry16(int c, int hw, int b, int& nsplit, int& split_len, int& ntu) {
  const int nt = cdiv(c, GT);
  ntu = nt * (nt + 1) / 2;
  static const int target = std::max(8, STX_KNOB("STX_GRAM_BLOCKS", 640));
  int want = rup(cdiv(target, ntu * b), 8);
  const int max_splits = std::max(1, cdiv(hw, 256));
  want = std::max(8, std::min(want, rup(max_splits, 8)));
  split_len = rup(cdiv(hw, want), 256);
  nsplit = rup(cdiv(hw, split_len), 8);
}

// workspace layout: [partial slabs (largest geometry)][loss partials b*ntu*FSUB]; the
// loss partials sit at a geometry-independent offset so a caller can keep them for a
// deferred, fused loss reduction (stx_style_loss_parts / stx_loss_finalize)
static size_t gram_parts_offset(int b, int c, int hw, int* nparts) {
  int nsplit, split_len, ntu, ns16, sl16;
  gram_geometry(c, hw, b, nsplit, split_len, ntu);
  gram_geometry16(c, hw, b, ns16, sl16, ntu);
  nsplit = std::max(nsplit, ns16);
  if (gram_tri_on(c, hw)) nsplit = std::max(nsplit, gram_tri_splits(c, hw, b));
  if (gram_tri256_on(c, hw)) nsplit = std::max(nsplit, gram_tri256_splits(hw, b));
  if (nparts) *nparts = b * ntu * FSUB;
  return (size_t)b * ntu * nsplit * GT * GT * sizeof(float);
}

static size_t gram_ws_bytes(int b, int c, int hw) {
  int nparts;
  const size_t off = gram_parts_offset(b, c, hw, &nparts);
  return off + ((size_t)nparts + 64) * sizeof(float);
}

// content / feature MSE companion of a style loss (stx_style_content_loss)
struct MseCompanion {
  const float* content;  // [b][c][hw], the content target
  float* out;            // [3]: content mse, feature loss, feature mse (stx_mse mode 2)
  float* parts;          // 2 floats per block
  size_t parts_bytes;
};

static void fill_job(stx_gram_fin_job* job, const float* parts, int c, int nsplit, float scale,
                     float* g_out, const float* target, long long t_bstride, float* coef,
                     int cpad, float cA, float alpha, float* loss_parts, const float* mse_parts,
                     int mse_nparts, double mse_n, float* mse_out, int b) {
  *job = stx_gram_fin_job{};
  job->parts = parts;
  job->c = c;
  job->nsplit = nsplit;
  job->b = b;
  job->scale = scale;
  job->g_out = g_out;
  job->target = target;
  job->t_bstride = t_bstride;
  job->coef = coef;
  job->cpad = cpad;
  job->cA = cA;
  job->alpha = alpha;
  job->loss_parts = loss_parts;
  job->mse_parts = mse_parts;
  job->mse_nparts = mse_nparts;
  job->mse_n = mse_n;
  job->mse_out = mse_out;
}

static int gram_run(const float* z, int b, int c, int hw, float scale, float* g_out,
                    const float* target, long long t_bstride, float* coef, float cA, float alpha, float* loss,
                    float loss_inv, const float* z_amax, void* ws, size_t ws_bytes,
                    hipStream_t st, const MseCompanion* mse = nullptr,
                    stx_gram_fin_job* defer = nullptr) {
  if (b <= 0 || c <= 0 || hw <= 0 || !z) {
    set_error("gram: invalid dims");
    return STX_E_INVALID;
  }
  const bool f16 = z_amax && hw % 8 == 0 && (reinterpret_cast<uintptr_t>(z) & 15) == 0;
  int nsplit, split_len, ntu;
  if (f16)
    gram_geometry16(c, hw, b, nsplit, split_len, ntu);
  else
    gram_geometry(c, hw, b, nsplit, split_len, ntu);
  const size_t need = gram_ws_bytes(b, c, hw);
  if (!ws || ws_bytes < need) {
    set_error("gram: workspace %zu < %zu", ws_bytes, need);
    return STX_E_WORKSPACE;
  }
  float* slabs = (float*)ws;
  float* parts = (float*)((char*)ws + gram_parts_offset(b, c, hw, nullptr));
  const MseCompanion* mse_fin = nullptr;
  int mse_nparts = 0;
  if (f16 && gram_tri_on(c, hw)) {
    nsplit = gram_tri_splits(c, hw, b);
    split_len = rup(cdiv(hw, nsplit), 64);
    nsplit = cdiv(hw, split_len);
    if (c == 128 && mse && (reinterpret_cast<uintptr_t>(mse->content) & 15) == 0 &&
        mse->parts_bytes >= (size_t)2 * b * nsplit * sizeof(float)) {
      hipLaunchKernelGGL((gram_tri_f16_kernel<128, true>), dim3(nsplit, 1, b), dim3(256), 0, st,
                         z, slabs, hw, nsplit, split_len, z_amax, mse->content, mse->parts);
      mse_fin = mse;  // finalized by the Gram finalize below
      mse_nparts = b * nsplit;
      mse = nullptr;  // done
    } else if (c == 128)
      hipLaunchKernelGGL(gram_tri_f16_kernel<128>, dim3(nsplit, 1, b), dim3(256), 0, st, z, slabs,
                         hw, nsplit, split_len, z_amax);
#ifdef STX_AB  // C = 256 on the triangle kernel (measured slower; STX_GRAM_TRI=2)
    else
      hipLaunchKernelGGL(gram_tri_f16_kernel<256>, dim3(nsplit, 1, b), dim3(256), 0, st, z, slabs,
                         hw, nsplit, split_len, z_amax);
#endif
  } else if (f16 && gram_tri256_on(c, hw)) {
    nsplit = gram_tri256_splits(hw, b);
    split_len = rup(cdiv(hw, nsplit), T256_PX);
    nsplit = cdiv(hw, split_len);
    if (STX_KNOB("STX_GRAM256_STAGE", 1))
      hipLaunchKernelGGL(gram_tri256_kernel<true>, dim3(nsplit, 1, b), dim3(512), 0, st, z, slabs,
                         hw, nsplit, split_len, z_amax);
    else
      hipLaunchKernelGGL(gram_tri256_kernel<false>, dim3(nsplit, 1, b), dim3(512), 0, st, z, slabs,
                         hw, nsplit, split_len, z_amax);
  } else if (f16) {
    hipLaunchKernelGGL(gram_partial_f16_kernel, dim3(nsplit * ntu, 1, b), dim3(256), 0, st, z,
                       slabs, c, hw, nsplit, split_len, z_amax);
  } else if (hw % 4 == 0) {
    const int nt = cdiv(c, GT);
    hipLaunchKernelGGL(gram_partial_v2_kernel<true>, dim3(nsplit * nt, 1, b), dim3(256), 0, st,
                       z, slabs, c, hw, nsplit, split_len);
    if (ntu > nt)
      hipLaunchKernelGGL(gram_partial_v2_kernel<false>, dim3(nsplit * (ntu - nt), 1, b),
                         dim3(256), 0, st, z, slabs, c, hw, nsplit, split_len);
  } else
    hipLaunchKernelGGL(gram_partial_kernel, dim3(nsplit, ntu, b), dim3(256), 0, st, z, slabs, c,
                       hw, nsplit, split_len);
  const int cpad = stx_gram_coef_pitch(c);
  if (defer) {  // the finalize joins a stx_gram_finalize_batch launch
    fill_job(defer, slabs, c, nsplit, scale, g_out, target, t_bstride, coef, cpad, cA, alpha,
             parts, mse_fin ? mse_fin->parts : nullptr, mse_nparts, (double)b * c * hw,
             mse_fin ? mse_fin->out : nullptr, b);
  } else {
    hipLaunchKernelGGL(gram_finalize_kernel, dim3(ntu * fin_blocks_per_tile(nsplit), b), dim3(FNT), 0, st, slabs, c,
                       nsplit, scale, g_out, target, t_bstride, coef, cpad, cA, alpha, parts,
                       mse_fin ? mse_fin->parts : nullptr, mse_nparts, (double)b * c * hw,
                       mse_fin ? mse_fin->out : nullptr);
  }
  if (target && loss && !defer)
    hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(64), 0, st, parts, b * ntu * FSUB,
                       loss_inv, loss);
  if (mse) {  // not fused (another Gram kernel ran): the separate content pass
    const int rc = stx_mse(z, mse->content, (long long)b * c * hw, 0, 2, mse->out, nullptr, 1.f,
                           mse->parts, mse->parts_bytes, st);
    if (rc) return rc;
  }
  return check_launch("gram");
}

}  // namespace stx

using namespace stx;

extern "C" size_t stx_gram_ws(int b, int c, int hw) { return gram_ws_bytes(b, c, hw); }

extern "C" size_t stx_style_loss_parts(int b, int c, int hw, int* nparts) {
  return gram_parts_offset(b, c, hw, nparts);
}

namespace stx {
// one block: losses[i] = inv_i * sum(parts_i) (wave i, the order of sum_parts_kernel, so
// the values are identical), then the weighted total
__global__ void __launch_bounds__(512) loss_finalize_kernel(stx_loss_parts lp,
                                                           float* __restrict__ losses,
                                                           const float* __restrict__ extra,
                                                           int m, LossWF w,
                                                           float* __restrict__ total) {
  // wave i reduces loss i (the sum_parts_kernel order), all losses in parallel
  __shared__ float lv[8];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave < lp.k) {
    const float s = wave_sum_parts(lp.parts[wave], lp.nparts[wave], lane);
    if (lane == 0) lv[wave] = s * lp.inv[wave];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < lp.k; ++i) {
      losses[i] = lv[i];
      t += w.w[i] * lv[i];
    }
    for (int j = 0; j < m; ++j) t += w.w[lp.k + j] * extra[j];
    if (total) *total = t;
  }
}
}  // namespace stx

extern "C" int stx_loss_finalize(const stx_loss_parts* lp, float* losses, const float* extra,
                                 int m, const float* w_host, float* total, void* stream) {
  if (!lp || lp->k < 0 || lp->k > 8 || m < 0 || lp->k + m > 16 || !losses ||
      (m && !extra) || (total && !w_host)) {
    set_error("stx_loss_finalize: invalid arguments");
    return STX_E_INVALID;
  }
  LossWF w{};
  for (int i = 0; i < lp->k + m && w_host; ++i) w.w[i] = w_host[i];
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(512), 0, (hipStream_t)stream, *lp,
                     losses, extra, m, w, total);
  return check_launch("stx_loss_finalize");
}

extern "C" int stx_gram_coef_pitch(int c) { return c <= 64 ? rup(c, 64) : rup(c, 128); }

extern "C" int stx_gram(const float* z, float* g, int b, int c, int hw, float scale,
                        const float* z_amax, void* ws, size_t ws_bytes, void* stream) {
  return gram_run(z, b, c, hw, scale, g, nullptr, 0, nullptr, 0.f, 0.f, nullptr, 0.f, z_amax, ws,
                  ws_bytes,
                  (hipStream_t)stream);
}

static int style_loss_impl(const float* z, const float* target, float* g_out, float* coef,
                           float* loss, int b, int c, int hw, int target_batched, float weight,
                           float diag_alpha, const float* z_amax, void* ws, size_t ws_bytes,
                           void* stream, stx_gram_fin_job* defer) {
  if (!target) {  // loss == NULL: partials stay in ws (stx_style_loss_parts)
    set_error("stx_style_loss: target is required");
    return STX_E_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  const double n = (double)c * hw;
  const float scale = (float)(1.0 / n);
  // d(weight*mean((G-T)^2))/dF_b = weight * 2(G-T)/(B C^2) * 2 F_b / N   (G symmetric)
  const float cA = (float)(weight * 4.0 / ((double)b * c * c * n));
  if (coef && stx_gram_coef_pitch(c) != c) {  // zero the padding (finalize writes c x c)
    const int cpad = stx_gram_coef_pitch(c);
    const long long cnt = (long long)b * cpad * cpad;
    hipLaunchKernelGGL(zero_kernel, dim3((int)std::min<long long>((cnt + 255) / 256, 2048)),
                       dim3(256), 0, st, coef, cnt);
  }
  return gram_run(z, b, c, hw, scale, g_out, target, target_batched ? (long long)c * c : 0, coef, cA, diag_alpha, loss,
                  (float)(1.0 / ((double)b * c * c)), z_amax, ws, ws_bytes, st, nullptr, defer);
}

extern "C" int stx_style_loss(const float* z, const float* target, float* g_out, float* coef,
                              float* loss, int b, int c, int hw, int target_batched, float weight,
                              float diag_alpha, const float* z_amax, void* ws, size_t ws_bytes,
                              void* stream) {
  return style_loss_impl(z, target, g_out, coef, loss, b, c, hw, target_batched, weight,
                         diag_alpha, z_amax, ws, ws_bytes, stream, nullptr);
}

extern "C" int stx_style_loss_deferred(const float* z, const float* target, float* coef, int b,
                                       int c, int hw, int target_batched, float weight,
                                       float diag_alpha, const float* z_amax, void* ws,
                                       size_t ws_bytes, stx_gram_fin_job* job, void* stream) {
  if (!job) {
    set_error("stx_style_loss_deferred: job is required");
    return STX_E_INVALID;
  }
  return style_loss_impl(z, target, nullptr, coef, nullptr, b, c, hw, target_batched, weight,
                         diag_alpha, z_amax, ws, ws_bytes, stream, job);
}

static size_t style_content_parts_bytes(int b, int c, int hw) {
  const size_t fused = (size_t)2 * b * gram_tri_splits(c, hw, b) * sizeof(float);
  return std::max(fused, stx_mse_ws((long long)b * c * hw));
}

extern "C" size_t stx_style_content_ws(int b, int c, int hw) {
  return rup((long long)gram_ws_bytes(b, c, hw), 256) + style_content_parts_bytes(b, c, hw);
}

static int style_content_impl(const float* z, const float* target, float* coef, float* loss,
                              int b, int c, int hw, int target_batched, float weight,
                              float diag_alpha, const float* z_amax, const float* content,
                              float* mse_out, void* ws, size_t ws_bytes, void* stream,
                              stx_gram_fin_job* defer) {
  if (!target || !content || !mse_out) {
    set_error("stx_style_content_loss: target, content and mse_out are required");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_style_content_ws(b, c, hw)) {
    set_error("stx_style_content_loss: workspace too small");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const double n = (double)c * hw;
  const float scale = (float)(1.0 / n);
  const float cA = (float)(weight * 4.0 / ((double)b * c * c * n));
  const int cpad = stx_gram_coef_pitch(c);
  if (coef && cpad != c) {
    const long long cnt = (long long)b * cpad * cpad;
    hipLaunchKernelGGL(zero_kernel, dim3((int)std::min<long long>((cnt + 255) / 256, 2048)),
                       dim3(256), 0, st, coef, cnt);
  }
  const size_t gb = rup((long long)gram_ws_bytes(b, c, hw), 256);
  MseCompanion m{content, mse_out, (float*)((char*)ws + gb), ws_bytes - gb};
  return gram_run(z, b, c, hw, scale, nullptr, target, target_batched ? (long long)c * c : 0,
                  coef, cA, diag_alpha, loss, (float)(1.0 / ((double)b * c * c)), z_amax, ws, gb,
                  st, &m, defer);
}

extern "C" int stx_style_content_loss(const float* z, const float* target, float* coef,
                                      float* loss, int b, int c, int hw, int target_batched,
                                      float weight, float diag_alpha, const float* z_amax,
                                      const float* content, float* mse_out, void* ws,
                                      size_t ws_bytes, void* stream) {
  return style_content_impl(z, target, coef, loss, b, c, hw, target_batched, weight, diag_alpha,
                            z_amax, content, mse_out, ws, ws_bytes, stream, nullptr);
}

extern "C" int stx_style_content_loss_deferred(const float* z, const float* target, float* coef,
                                               int b, int c, int hw, int target_batched,
                                               float weight, float diag_alpha,
                                               const float* z_amax, const float* content,
                                               float* mse_out, void* ws, size_t ws_bytes,
                                               stx_gram_fin_job* job, void* stream) {
  if (!job) {
    set_error("stx_style_content_loss_deferred: job is required");
    return STX_E_INVALID;
  }
  return style_content_impl(z, target, coef, nullptr, b, c, hw, target_batched, weight,
                            diag_alpha, z_amax, content, mse_out, ws, ws_bytes, stream, job);
}

// gparts: [b][ntu][nparts][64 x 64] (ntu = 1 for c <= 64, 3 for c = 128: the fused conv
// epilogue tiles, stx_conv_params.gram_part); mse_parts (c = 128, the content tap): the
// epilogue's 2 sums per block, b * nparts pairs, finalized into mse_out like
// gram_tri_f16_kernel<128, true>'s
static int from_parts_impl(const float* gparts, int nparts, const float* target, float* g_out,
                           float* coef, float* loss, int b, int c, int hw, int target_batched,
                           float weight, float diag_alpha, void* ws, size_t ws_bytes,
                           void* stream, stx_gram_fin_job* defer,
                           const float* mse_parts = nullptr, float* mse_out = nullptr) {
  if (!gparts || !target || nparts <= 0 || b <= 0 || c <= 0 || (c > GT && c != 2 * GT) ||
      hw <= 0) {
    set_error("stx_style_loss_from_parts: invalid arguments (c <= 64 or c == 128)");
    return STX_E_INVALID;
  }
  if ((mse_parts != nullptr) != (mse_out != nullptr)) {
    set_error("stx_style_content_loss_from_parts: mse_parts and mse_out go together");
    return STX_E_INVALID;
  }
  const int nt = cdiv(c, GT), ntu = nt * (nt + 1) / 2;
  const size_t need = gram_ws_bytes(b, c, hw);
  if (!ws || ws_bytes < need) {
    set_error("stx_style_loss_from_parts: workspace %zu < %zu", ws_bytes, need);
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const double n = (double)c * hw;
  const float cA = (float)(weight * 4.0 / ((double)b * c * c * n));
  const int cpad = stx_gram_coef_pitch(c);
  if (coef && cpad != c) {
    const long long cnt = (long long)b * cpad * cpad;
    hipLaunchKernelGGL(zero_kernel, dim3((int)std::min<long long>((cnt + 255) / 256, 2048)),
                       dim3(256), 0, st, coef, cnt);
  }
  float* lparts = (float*)((char*)ws + gram_parts_offset(b, c, hw, nullptr));
  const int mse_nparts = mse_parts ? b * nparts : 0;
  const double mse_n = (double)b * c * hw;
  if (defer) {
    fill_job(defer, gparts, c, nparts, (float)(1.0 / n), g_out, target,
             target_batched ? (long long)c * c : 0ll, coef, cpad, cA, diag_alpha, lparts,
             mse_parts, mse_nparts, mse_n, mse_out, b);
    return check_launch("stx_style_loss_from_parts_deferred");
  }
  hipLaunchKernelGGL(gram_finalize_kernel, dim3(ntu * fin_blocks_per_tile(nparts), b), dim3(FNT),
                     0, st, gparts, c, nparts, (float)(1.0 / n), g_out, target,
                     target_batched ? (long long)c * c : 0ll, coef, cpad, cA, diag_alpha, lparts,
                     mse_parts, mse_nparts, mse_n, mse_out);
  if (loss)
    hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(64), 0, st, lparts, b * ntu * FSUB,
                       (float)(1.0 / ((double)b * c * c)), loss);
  return check_launch("stx_style_loss_from_parts");
}

extern "C" int stx_style_content_loss_from_parts(const float* gparts, int nparts,
                                                 const float* target, float* coef, float* loss,
                                                 int b, int c, int hw, int target_batched,
                                                 float weight, float diag_alpha,
                                                 const float* mse_parts, float* mse_out, void* ws,
                                                 size_t ws_bytes, void* stream) {
  if (!mse_parts || !mse_out) {
    set_error("stx_style_content_loss_from_parts: mse_parts and mse_out are required");
    return STX_E_INVALID;
  }
  return from_parts_impl(gparts, nparts, target, nullptr, coef, loss, b, c, hw, target_batched,
                         weight, diag_alpha, ws, ws_bytes, stream, nullptr, mse_parts, mse_out);
}

extern "C" int stx_style_content_loss_from_parts_deferred(
    const float* gparts, int nparts, const float* target, float* coef, int b, int c, int hw,
    int target_batched, float weight, float diag_alpha, const float* mse_parts, float* mse_out,
    void* ws, size_t ws_bytes, stx_gram_fin_job* job, void* stream) {
  if (!job || !mse_parts || !mse_out) {
    set_error("stx_style_content_loss_from_parts_deferred: job, mse_parts and mse_out are "
              "required");
    return STX_E_INVALID;
  }
  return from_parts_impl(gparts, nparts, target, nullptr, coef, nullptr, b, c, hw,
                         target_batched, weight, diag_alpha, ws, ws_bytes, stream, job, mse_parts,
                         mse_out);
}

extern "C" int stx_style_loss_from_parts(const float* gparts, int nparts, const float* target,
                                         float* g_out, float* coef, float* loss, int b, int c,
                                         int hw, int target_batched, float weight,
                                         float diag_alpha, void* ws, size_t ws_bytes,
                                         void* stream) {
  return from_parts_impl(gparts, nparts, target, g_out, coef, loss, b, c, hw, target_batched,
                         weight, diag_alpha, ws, ws_bytes, stream, nullptr);
}

extern "C" int stx_style_loss_from_parts_deferred(const float* gparts, int nparts,
                                                  const float* target, float* coef, int b, int c,
                                                  int hw, int target_batched, float weight,
                                                  float diag_alpha, void* ws, size_t ws_bytes,
                                                  stx_gram_fin_job* job, void* stream) {
  if (!job) {
    set_error("stx_style_loss_from_parts_deferred: job is required");
    return STX_E_INVALID;
  }
  return from_parts_impl(gparts, nparts, target, nullptr, coef, nullptr, b, c, hw,
                         target_batched, weight, diag_alpha, ws, ws_bytes, stream, job);
}

extern "C" int stx_gram_finalize_batch(const stx_gram_fin_job* jobs, int njobs, void* stream) {
  if (!jobs || njobs <= 0 || njobs > STX_FIN_MAX) {
    set_error("stx_gram_finalize_batch: 1 <= njobs <= %d required", STX_FIN_MAX);
    return STX_E_INVALID;
  }
  FinBatch fb{};
  int blocks = 0;
  for (int j = 0; j < njobs; ++j) {
    const stx_gram_fin_job& q = jobs[j];
    if (!q.parts || q.c <= 0 || q.nsplit <= 0 || q.b <= 0 || !q.loss_parts) {
      set_error("stx_gram_finalize_batch: job %d invalid", j);
      return STX_E_INVALID;
    }
    const int nt = cdiv(q.c, GT);
    fb.job[j] = q;
    fb.blk0[j] = blocks;
    blocks += nt * (nt + 1) / 2 * fin_blocks_per_tile(q.nsplit) * q.b;
  }
  fb.blk0[njobs] = blocks;
  fb.njobs = njobs;
  hipLaunchKernelGGL(gram_finalize_batch_kernel, dim3(blocks), dim3(FNT), 0, (hipStream_t)stream,
                     fb);
  return check_launch("stx_gram_finalize_batch");
}

extern "C" int stx_gram_bwd(const float* coef, const float* z, float* dz, int b, int c, int h,
                            int w, const float* acc_scale_dev, const float* mask,
                            const float* aux, float aux_scale, int accumulate, void* stream) {
  stx_conv_params p = {};
  p.x = z;
  p.wt = coef;
  p.y = dz;
  p.mask = mask;
  p.aux = aux;
  p.aux_scale = aux_scale;
  p.acc_scale = acc_scale_dev;
  p.accumulate = accumulate;
  p.n = b;
  p.cin = c;
  p.h = h;
  p.w = w;
  p.cout = c;
  p.ks = 1;
  p.stride = 1;
  p.pad = 0;
  p.in_mode = STX_IN_RAW;
  p.hv = h;
  p.wv = w;
  p.ho = h;
  p.wo = w;
  stx_conv_weight_dims(c, c, 1, &p.cin_pad, &p.cout_pad);
  const int cpad = stx_gram_coef_pitch(c);
  if (p.cout_pad != cpad || p.cin_pad > cpad) {
    set_error("stx_gram_bwd: pitch mismatch");
    return STX_E_INVALID;
  }
  p.wt_batch_stride = (long long)cpad * cpad;
  return stx_conv2d(&p, stream);
}
