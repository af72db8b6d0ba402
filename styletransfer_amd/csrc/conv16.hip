// 3x3 stride-1 implicit-GEMM convolution on the fp16 MFMA pipe with an exact-ish
// fp32 emulation: v_mfma_f32_32x32x16_f16 over hi/lo split operands.
//
// Every fp32 operand v (input halo element, weight) is scaled by a per-tensor
// power of two s (s*max|v| < 2^15, so no fp16 overflow) and split
//     s*v = hi + lo,   hi = fp16(s*v),  lo = fp16(s*v - hi)
// which keeps 22 significant bits.  The product of two operands is taken as
//     hi_a*hi_b + hi_a*lo_b + lo_a*hi_b      (dropped lo_a*lo_b ~ 2^-22 relative)
// with every fp16 x fp16 product exact in the fp32 MFMA accumulator; the result is
// de-scaled by 1/(s_x s_w) (exact, a power of two).  Against an fp64 ground truth
// this is as accurate as fp32 arithmetic (tools/split_numerics.py: Gatys losses,
// Gram matrices and image gradients within 2-4e-7 of fp64, the same as the fp32
// reference), and it runs three fp16 MFMAs (3 x 32 cycles for K=16) where the fp32
// MFMA needs 8 x 64 cycles: a 5.3x higher matrix-pipe ceiling than
// v_mfma_f32_32x32x2_f32.  bf16 would need a three-way split (6 products) for the
// same accuracy — its 8-bit mantissa halves lose the ReLU/argmax decisions.
//
// GEMM view: M = cout (block tile 64), N = 256 output pixels (TH x TW), K = cin*9.
// K walks chunks of 16 input channels; per chunk and tap (kh, kw) one K=16 MFMA
// step.  LDS images are [plane hi/lo][channel group of 8][item][8 x fp16], i.e. each
// 16-B unit holds the 8 channels one lane feeds one MFMA (A: lane = cout row,
// B: lane = pixel column; lane half h = channel group), so every operand read is
// one conflict-free ds_read_b128 at (lane base + compile-time offset):
//   halo    [P][cg][pos]   pos = r*RW + c of the (TH+2) x (TW+2) input window
//   weights [tap][P][cg][co]
//
// Reference: the torchvision vgg19 Conv2d(3x3, p1) layers sliced by StyleNetwork
// (stransfer/network.py:246-314) and the ImageTransformNet 3x3 convs
// (stransfer/network.py:468-481, 525-609), forward and data-gradient.
#include <stdlib.h>
#include <type_traits>

#include "common.h"
#include "conv_epi.h"
#include "wprep.h"
#include "../../include/stx.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));


// Split Gram-backward phase: acc (the de-scaled, masked main result) gets
//   + s2 * sum_c A[n][c][co] * z2[n][c][pixel]
// on the fp16 hi/lo MFMA.  z2 is scaled by sz = 2^(15 - e(p2_amax)); A' = s2 * A
// (small, L2 resident) by its block-wide max.  The products accumulate straight into
// acc (no second accumulator: register budget): acc is first brought to the common
// power-of-two scale S = 2^(30 - ea - ez) (capped so |acc| * S < 2^100), A' is
// staged with sa = S / sz (<= 2^(15 - ea): no fp16 overflow) and acc is de-scaled
// by 1/S at the end -- all factors are powers of two, so the only roundings are
// those of fp32 accumulation.  Per chunk of 16
// channels: z2 tile -> LDS [P][cg][pixel], A' -> LDS [P][cg][co] (16-B units of 8
// channels), 3 MFMAs per 32x32 tile; the next chunk's loads are in flight meanwhile.
template <int TW>
__device__ __forceinline__ void phase2_f16(f32x16 (&acc)[2][2], const stx_conv_params& p, int n,
                                           int co0, int ty0, int tx0, int wave, int h, int l32,
                                           char* smem) {
  constexpr int NPIX = 256, BM = 64;
  constexpr bool RP = TW == 64;
  const int tid = threadIdx.x;
  const size_t plane = (size_t)p.ho * p.wo;
  const float* __restrict__ A = p.p2_wt + (size_t)n * p.p2_wt_batch_stride;
  const int C2 = p.p2_c;
  const float s2 = p.p2_scale ? *p.p2_scale : 1.f;
  char* lz = smem;                     // [P][cg][256 px] x 16 B = 16 KB
  char* la = smem + 4 * NPIX * 16;     // [P][cg][64 co]  x 16 B = 4 KB
  // z2 staging: thread -> pixel quad q (4 consecutive tile pixels of one row) x
  // channel quad cq (4 channels) of the 16-channel chunk: 4 float4 loads per chunk
  const int q = tid & 63, cq = tid >> 6;
  const int qp = 4 * q, qrow = qp / TW, qcol = qp - qrow * TW;
  const int qy = ty0 + qrow, qx = tx0 + qcol;
  const bool vec = (p.wo & 3) == 0;    // rows 16-B aligned: a quad is all in or all out
  const uint32_t zq_off = (qy < p.ho && qx < p.wo) ? (uint32_t)(qy * p.wo + qx) * 4u : BUF_OOB;
  const uint32_t pb = (uint32_t)plane * 4u;
  const float* __restrict__ z2 = p.p2_z + (size_t)n * C2 * plane;
  int bpix[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, RP>(wave, j, l32, ty, tx);
    bpix[j] = ty * TW + tx;
  }
  const int acg = tid >> 6, aco = tid & 63;  // A' staging: threads 0..127 -> (cg, co)
  struct Stage {
    f32x4 z[4];  // [channel e of the quad] x 4 pixels
    float a[8];
  };
  auto fetch = [&](int c0, Stage& g) {
    const auto rz = make_srd(z2 + (size_t)c0 * plane, (uint32_t)max(0, C2 - c0) * pb);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t o = zq_off + (uint32_t)(4 * cq + e) * pb;
      if (vec) {
        g.z[e] = buf_ld4(rz, o);
      } else {  // ragged width: per-pixel loads, pixels past the row end read 0
#pragma unroll
        for (int k = 0; k < 4; ++k)
          g.z[e][k] = (qx + k < p.wo) ? buf_ld(rz, o + 4u * k) : 0.f;
      }
    }
    if (tid < 128) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + acg * 8 + e, co = co0 + aco;
        g.a[e] = (c < C2 && co < p.cout_pad) ? A[(size_t)c * p.cout_pad + co] : 0.f;
      }
    }
  };
  // the first two chunks' loads are in flight during the scale reductions below
  Stage s0, s1;
  fetch(0, s0);
  if (16 < C2) fetch(16, s1);
  // max |A[c][co0 .. co0+63]| over c < C2 (float4 rows of the padded [c][cout_pad] layout)
  float m = 0.f;
  for (int base = 0; base < C2 * (BM / 4); base += 1024) {
    f32x4 v[4];  // four independent loads in flight, then reduce
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int idx = base + tid + 256 * u;
      const int c = idx / (BM / 4), q4 = idx - c * (BM / 4);
      const int co = co0 + 4 * q4;
      const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
      v[u] = (c < C2 && co < p.cout_pad)
                 ? *reinterpret_cast<const f32x4*>(A + (size_t)c * p.cout_pad + co)
                 : zero;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(v[u][e]));
  }
  __shared__ float red2[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) red2[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red2[0], red2[1]), fmaxf(red2[2], red2[3])) * fabsf(s2);
  // max |acc| bounds how far acc may be scaled up (|acc| * S < 2^100)
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) am = fmaxf(am, fabsf(acc[i][j][r]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  __syncthreads();
  if ((tid & 63) == 0) red2[tid >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red2[0], red2[1]), fmaxf(red2[2], red2[3]));
  const int ea = amax_exp(m), ez = amax_exp(read_amax(p.p2_amax)), eacc = amax_exp(am);
  const int ls = min(min(30 - ea - ez, 100 - eacc), 120);  // log2 S
  const float sz = __builtin_ldexpf(1.f, 15 - ez);
  const float sa = __builtin_ldexpf(s2, ls - (15 - ez));  // S / sz, with s2 folded in
  {
    const float up = __builtin_ldexpf(1.f, ls);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= up;
  }

  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  auto stage = [&](const Stage& g) {
    const int cg = cq >> 1, half = cq & 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = g.z[e][k] * sz;
        const _Float16 vh = (_Float16)v;
        hi[e] = vh;
        lo[e] = (_Float16)(v - (float)vh);
      }
      *reinterpret_cast<f16x4*>(lz + ((0 * 2 + cg) * NPIX + qp + k) * 16 + half * 8) = hi;
      *reinterpret_cast<f16x4*>(lz + ((1 * 2 + cg) * NPIX + qp + k) * 16 + half * 8) = lo;
    }
    if (tid < 128) {
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = g.a[e] * sa;
        const _Float16 vh = (_Float16)v;
        hi[e] = vh;
        lo[e] = (_Float16)(v - (float)vh);
      }
      *reinterpret_cast<f16x8*>(la + ((0 * 2 + acg) * BM + aco) * 16) = hi;
      *reinterpret_cast<f16x8*>(la + ((1 * 2 + acg) * BM + aco) * 16) = lo;
    }
  };
  // two chunks of loads in flight ahead of the chunk being multiplied
  for (int c0 = 0; c0 < C2; c0 += 16) {
    __syncthreads();  // previous chunk's operand reads done
    stage(s0);
    __syncthreads();
    s0 = s1;
    if (c0 + 32 < C2) fetch(c0 + 32, s1);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f16x8 fa[2];
#pragma unroll
      for (int P = 0; P < 2; ++P)
        fa[P] = *reinterpret_cast<const f16x8*>(la + ((P * 2 + h) * BM + i * 32 + l32) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f16x8 fb[2];
#pragma unroll
        for (int P = 0; P < 2; ++P)
          fb[P] = *reinterpret_cast<const f16x8*>(lz + ((P * 2 + h) * NPIX + bpix[j]) * 16);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[0], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // LDS handed back to the epilogue
  const float down = __builtin_ldexpf(1.f, -ls);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] *= down;
}

// Split Gram-backward phase of the v2 data-gradient conv (P2 = 3): acc -- de-scaled,
// *acc_scale, ReLU-masked and brought to the power-of-two scale S = 2^ls by `prologue`,
// which runs once chunk 0's loads are issued -- gets + S * s2 * A[n] . z2 on the fp16
// hi/lo MFMA with every scale precomputed: z2 by its amax group (p2_amax: sz =
// 2^(15 - ez)), A' = s2 * A by the batch max the Gram finalize wrote (p2_wt_amax: sa =
// S / sz <= 2^(15 - ea)).  No in-kernel reductions: the round-3 port of phase2_f16 paid
// two block-wide max passes and a re-read of A for its scales, and lost to the fp32 MFMA.
// Per 16-channel chunk, into one of two LDS buffers (one barrier per chunk: chunk c+1 is
// split and written while chunk c's MFMAs run):
//   z2 -> [P][cg][256 px] 16-B units: thread t owns tile pixel t and writes its two
//         channel groups' hi and lo units (lane-consecutive 16-B stores, conflict-free;
//         the round-5 form wrote 8-B halves at a 64-B lane stride: 896 bank-conflict
//         cycles per chunk and block) from 16 lane-coalesced dword loads;
//   A' -> [P][cg][64 co] 16-B units, split once per block by waves 0-1 (each of the four
//         waves split its own register copy of all 64 couts before);
// then 3 MFMAs per 32 x 32 tile from conflict-free ds_read_b128s.
template <int TW, bool RP, class Prologue>
__device__ __forceinline__ void phase2_pre(f32x16 (&acc)[2][2], const stx_conv_params& p,
                                           const EpiTile& t, int ls, int ez, char* smem,
                                           Prologue&& prologue) {
  constexpr int NPIX = 256, BM = 64;
  constexpr int ZB = 4 * NPIX * 16, AB_ = 4 * BM * 16, BUF = ZB + AB_;  // 20 KB per buffer
  const int tid = threadIdx.x, h = t.h, l32 = t.l32;
  const size_t plane = (size_t)p.ho * p.wo;
  const int C2 = p.p2_c;
  const float s2 = p.p2_scale ? *p.p2_scale : 1.f;
  const float sz = __builtin_ldexpf(1.f, 15 - ez);
  const float sa = __builtin_ldexpf(s2, ls - (15 - ez));
  // z2: thread -> tile pixel tid (row tid / TW), all 16 channels of the chunk
  const int zy = t.ty0 + tid / TW, zx = t.tx0 + tid % TW;
  const uint32_t z_off = (zy < p.ho && zx < p.wo) ? (uint32_t)(zy * p.wo + zx) * 4u : BUF_OOB;
  const uint32_t pb = (uint32_t)plane * 4u;
  const float* __restrict__ z2 = p.p2_z + (size_t)t.n * C2 * plane;
  // A': threads 0..127 -> (channel group acg, cout aco): 8 channels of one cout
  const bool a_thr = tid < 128;  // (waves 0 and 1: wave-uniform)
  const int acg = (tid >> 6) & 1, aco = tid & 63;
  const auto ra = make_srd(p.p2_wt + (size_t)t.n * p.p2_wt_batch_stride,
                           (uint32_t)C2 * (uint32_t)p.cout_pad * 4u);
  const uint32_t a_off = (uint32_t)((8 * acg) * p.cout_pad + t.co0 + aco) * 4u;
  const uint32_t a_row = (uint32_t)p.cout_pad * 4u;
  int bpix[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, RP, 2>(t.wn, j, l32, ty, tx);
    bpix[j] = ty * TW + tx;
  }
  struct Stage {
    float z[16];  // channel e of the chunk at this thread's pixel
    float a[8];   // channel 8 acg + e at cout aco
  };
  auto fetch = [&](int c0, Stage& g) {
    // channels past C2 read 0 (descriptor range)
    const auto rz = make_srd(z2 + (size_t)c0 * plane, (uint32_t)max(0, C2 - c0) * pb);
#pragma unroll
    for (int e = 0; e < 16; ++e) g.z[e] = buf_ld(rz, z_off + (uint32_t)e * pb);
    if (a_thr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) g.a[e] = buf_ld(ra, a_off + (uint32_t)(c0 + e) * a_row);
    }
  };
  auto split8 = [](const float* v, float s, f16x8& hi, f16x8& lo) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = v[e] * s;
      const _Float16 xh = (_Float16)x;
      hi[e] = xh;
      lo[e] = (_Float16)(x - (float)xh);
    }
  };
  auto stage = [&](const Stage& g, int b) {
    char* lz = smem + b * BUF;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
      f16x8 hi, lo;
      split8(g.z + 8 * cg, sz, hi, lo);
      *reinterpret_cast<f16x8*>(lz + ((0 * 2 + cg) * NPIX + tid) * 16) = hi;
      *reinterpret_cast<f16x8*>(lz + ((1 * 2 + cg) * NPIX + tid) * 16) = lo;
    }
    if (a_thr) {
      char* la = lz + ZB;
      f16x8 hi, lo;
      split8(g.a, sa, hi, lo);
      *reinterpret_cast<f16x8*>(la + ((0 * 2 + acg) * BM + aco) * 16) = hi;
      *reinterpret_cast<f16x8*>(la + ((1 * 2 + acg) * BM + aco) * 16) = lo;
    }
  };
  Stage g;
  fetch(0, g);
  prologue();  // the caller's scaling and mask, with chunk 0's loads in flight
  __syncthreads();  // the main loop's LDS reads done
  stage(g, 0);
  if (16 < C2) fetch(16, g);
  int b = 0;
  for (int c0 = 0; c0 < C2; c0 += 16, b ^= 1) {
    __syncthreads();  // buffer b complete; buffer b^1's reads (chunk c0 - 16) done
    const char* lz = smem + b * BUF;
    const char* la = lz + ZB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f16x8 fa[2];
#pragma unroll
      for (int P = 0; P < 2; ++P)
        fa[P] = *reinterpret_cast<const f16x8*>(la + ((P * 2 + h) * BM + i * 32 + l32) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f16x8 fb[2];
#pragma unroll
        for (int P = 0; P < 2; ++P)
          fb[P] = *reinterpret_cast<const f16x8*>(lz + ((P * 2 + h) * NPIX + bpix[j]) * 16);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[0], fb[1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[1], fb[0], acc[i][j], 0, 0, 0);
      }
    }
    if (c0 + 16 < C2) {  // the next chunk -> the other buffer, its successor's loads
      stage(g, b ^ 1);
      if (c0 + 32 < C2) fetch(c0 + 32, g);
    }
  }
  __syncthreads();  // LDS handed back to the epilogue
}

// P2 = 4 (stx_conv_params.unpool_out, include/stx.h): a pooled VGG tap's ReLU+MaxPool
// backward and Gram backward in the epilogue of the data gradient that produces the pooled
// gradient d (conv2_1^T: d = dP1, the output dZ2 = unpool(d) [Z2 > 0] + s A2 Z2).  The
// block's 32 x 4 tile of d (wave wn: row ty0 + wn, lane l32: column tx0 + l32) covers the
// full-resolution rows 2 ty0 .. +7, columns 2 tx0 .. +63 of z:
//  1. per element of acc (co, d pixel): the window's four z values (two 8-B loads) give its
//     first maximum of relu(z) (torch's max_pool2d backward index, as gram_bwd16) and the
//     ReLU mask there -> one bit per element in sel[s] (s = 2 dy + dx, the window slot);
//  2. per row parity dy: A . z over the region's 256 pixels of that parity on the fp16
//     hi / lo MFMA, N-tile dx / lane l32 <-> pixel (2 (ty0 + wn) + dy, 2 (tx0 + l32) + dx),
//     so the lane's N-tile element sits under its own element of d.  z in chunks of 16
//     channels through double-buffered LDS ([P][cg][dx][row][32] 16-B units: the
//     fragment reads are conflict-free), one barrier per chunk; A' straight from L2 into
//     fragment registers (as phase2_pre); accumulators separate from acc, so each term
//     keeps its own power-of-two scale;
//  3. y = A.z + the routed d, written as 8-B (dx pair) stores; max|y| -> out_amax.
template <int TW>
__device__ __forceinline__ void epi_unpool_gram(f32x16 (&acc)[2][1], const stx_conv_params& p,
                                                const EpiTile& t, float descale, char* smem) {
  static_assert(TW == 32, "32 x 4 tiles of d");
  constexpr int UNITS = 2 * 2 * 2 * 128;  // [P][cg][dx][4 rows x 32]: one 16 KB buffer
  const int tid = threadIdx.x, h = t.h, l32 = t.l32, wn = t.wn;
  const int C = p.cout, nch = C / 16;     // z channels (= cout: 64 or 128), K chunks
  const int H2 = 2 * p.ho, W2 = 2 * p.wo;
  const uint32_t pb2 = (uint32_t)H2 * (uint32_t)W2 * 4u;
  const size_t img = (size_t)t.n * C * H2 * W2, blk = img + (size_t)t.co0 * H2 * W2;
  const auto rz = make_srd(p.up_z + img, (uint32_t)C * pb2);   // all channels (A . z)
  const auto rw = make_srd(p.up_z + blk, 64u * pb2);           // this block's 64 (windows)
  const auto ry = make_srd(p.y + blk, 64u * pb2);
  const auto rx = make_srd(p.aux ? p.aux + blk : p.y + blk, p.aux ? 64u * pb2 : 0u);
  const int Y0 = 2 * (t.ty0 + wn), X0 = 2 * (t.tx0 + l32);
  const uint32_t win = (uint32_t)(Y0 * W2 + X0) * 4u, wrow = (uint32_t)W2 * 4u;
  auto corow = [&](int i, int r) { return i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h; };
  // 1. window first maximum and mask
  uint32_t sel[4] = {0u, 0u, 0u, 0u};
#pragma unroll 1
  for (int i = 0; i < 2; ++i) {
    f32x2_t top[16], bot[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t o = (uint32_t)corow(i, r) * pb2 + win;
      top[r] = buf_ld2(rw, o);
      bot[r] = buf_ld2(rw, o + wrow);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float z0 = top[r].x, z1 = top[r].y, z2 = bot[r].x, z3 = bot[r].y;
      const float r0 = relu_bits(z0), r1 = relu_bits(z1), r2 = relu_bits(z2), r3 = relu_bits(z3);
      int bi = 0;
      float best = r0;
      if (r1 > best) { best = r1; bi = 1; }
      if (r2 > best) { best = r2; bi = 2; }
      if (r3 > best) { bi = 3; }
      const float zs = bi == 0 ? z0 : bi == 1 ? z1 : bi == 2 ? z2 : z3;
      const uint32_t bit = zs > 0.f ? 1u << (16 * i + r) : 0u;
      sel[0] |= bi == 0 ? bit : 0u;
      sel[1] |= bi == 1 ? bit : 0u;
      sel[2] |= bi == 2 ? bit : 0u;
      sel[3] |= bi == 3 ? bit : 0u;
    }
  }
  // 2. scales: A' = s2 A 2^(15 - ea), z' = z 2^(15 - ez); A.z = acc2 2^(ea + ez - 30)
  const float s2 = p.p2_scale ? *p.p2_scale : 1.f;
  const int ea = amax_exp(read_amax(p.p2_wt_amax) * fabsf(s2));
  const int ez = amax_exp(read_amax(p.p2_amax));
  const float sa = __builtin_ldexpf(s2, 15 - ea), sz = __builtin_ldexpf(1.f, 15 - ez);
  const float down = __builtin_ldexpf(1.f, ea + ez - 30);
  // A'[c][co0 .. co0 + 63] (C x 64, both passes) split once into LDS after the z buffers:
  // [chunk][P][cg][co] 16-B units (8 channels of one cout), C x 256 B; thread t -> the
  // units (channel group of 8, cout) t, t + 256, ...
  char* la = smem + 2 * UNITS * 16;
  {
    const float* __restrict__ A = p.p2_wt + (size_t)t.n * p.p2_wt_batch_stride + t.co0;
    for (int u = tid; u < C * 8; u += 256) {
      const int co = u & 63, cg8 = u >> 6;  // channel group of 8
      float av[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = A[(size_t)(8 * cg8 + e) * p.cout_pad + co];
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = av[e] * sa;
        const _Float16 vh = (_Float16)v;
        hi[e] = vh;
        lo[e] = (_Float16)(v - (float)vh);
      }
      const int c = cg8 >> 1, cg = cg8 & 1;
      *reinterpret_cast<f16x8*>(la + (((c * 2 + 0) * 2 + cg) * 64 + co) * 16) = hi;
      *reinterpret_cast<f16x8*>(la + (((c * 2 + 1) * 2 + cg) * 64 + co) * 16) = lo;
    }
  }
  // staging thread -> (cg, row wr, column tx): 8 channels x the pixel pair dx = 0, 1
  const int scg = tid >> 7, swr = (tid >> 5) & 3, stx_ = tid & 31;
  auto fetch = [&](int dy, int c0, f32x2_t (&g)[8]) {
    const uint32_t po = (uint32_t)((2 * (t.ty0 + swr) + dy) * W2 + 2 * (t.tx0 + stx_)) * 4u;
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = buf_ld2(rz, (uint32_t)(c0 + 8 * scg + e) * pb2 + po);
  };
  auto stage = [&](const f32x2_t (&g)[8], int b) {
    char* lz = smem + b * UNITS * 16;
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      f16x8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (dx ? g[e].y : g[e].x) * sz;
        const _Float16 vh = (_Float16)v;
        hi[e] = vh;
        lo[e] = (_Float16)(v - (float)vh);
      }
      const int u = ((scg * 2 + dx) * 4 + swr) * 32 + stx_;  // [cg][dx][row][32] in plane P
      *reinterpret_cast<f16x8*>(lz + u * 16) = hi;
      *reinterpret_cast<f16x8*>(lz + (UNITS / 2 + u) * 16) = lo;
    }
  };
  uint32_t vmax_u = 0u;
#pragma unroll 1
  for (int dy = 0; dy < 2; ++dy) {
    f32x16 acc2[2][2];  // [dx][i]
#pragma unroll
    for (int dx = 0; dx < 2; ++dx)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[dx][i][r] = 0.f;
    f32x2_t g[8];
    fetch(dy, 0, g);
    __syncthreads();  // the LDS is free (main loop / the previous pass's reads done)
    stage(g, 0);
    fetch(dy, 16, g);
    for (int c = 0; c < nch; ++c) {
      const int b = c & 1;
      __syncthreads();  // buffer b (and A') complete; buffer b ^ 1's reads (chunk c - 1) done
      const char* lz = smem + b * UNITS * 16;
      f16x8 fa[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int P = 0; P < 2; ++P)
          fa[i][P] = *reinterpret_cast<const f16x8*>(la + (((c * 2 + P) * 2 + h) * 64 + 32 * i + l32) * 16);
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int u = ((h * 2 + dx) * 4 + wn) * 32 + l32;
        const f16x8 bh = *reinterpret_cast<const f16x8*>(lz + u * 16);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(lz + (UNITS / 2 + u) * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc2[dx][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i][0], bh, acc2[dx][i], 0, 0, 0);
          acc2[dx][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i][0], bl, acc2[dx][i], 0, 0, 0);
          acc2[dx][i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[i][1], bh, acc2[dx][i], 0, 0, 0);
        }
      }
      if (c + 1 < nch) {
        stage(g, b ^ 1);
        if (c + 2 < nch) fetch(dy, 16 * (c + 2), g);
      }
    }
    // 3. y = A.z (+ aux_scale aux) + the routed d (8-B stores of the dx pair); the aux
    // loads all go out before the first store (vmcnt counts stores too)
    const uint32_t sel0 = dy ? sel[2] : sel[0], sel1 = dy ? sel[3] : sel[1];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int rh = 0; rh < 16; rh += 8) {
      f32x2_t xv[16];
      if (p.aux) {
#pragma unroll
        for (int r = rh; r < rh + 8; ++r)
          xv[r] = buf_ld2(rx, (uint32_t)corow(i, r) * pb2 + win + (uint32_t)dy * wrow);
      }
#pragma unroll
      for (int r = rh; r < rh + 8; ++r) {
        const float d = acc[i][0][r] * descale;
        const uint32_t bit = 1u << (16 * i + r);
        float v0 = acc2[0][i][r] * down + ((sel0 & bit) ? d : 0.f);
        float v1 = acc2[1][i][r] * down + ((sel1 & bit) ? d : 0.f);
        if (p.aux) {
          v0 = fmaf(p.aux_scale, xv[r].x, v0);
          v1 = fmaf(p.aux_scale, xv[r].y, v1);
        }
        vmax_u = max(vmax_u, max(__float_as_uint(v0) & 0x7fffffffu,
                                 __float_as_uint(v1) & 0x7fffffffu));
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t dv = {__float_as_uint(v0), __float_as_uint(v1)};
        __builtin_amdgcn_raw_buffer_store_b64(
            dv, ry, (uint32_t)corow(i, r) * pb2 + win + (uint32_t)dy * wrow, 0, 0);
      }
    }
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u), 4);  // (4 waves: K2 too)
}

// S = 2: the stride-2 downsampling convs (raw input, loader mode LM_S2): the tile's
// input window is (2 TH + 1) x (2 TW + 1) and output pixel (ty, tx) reads its taps at
// window position (2 ty + kh, 2 tx + kw)
constexpr int LM_S2 = 16;

template <int TW, int NI, int S = 1>
struct C16 {
  static constexpr int BM = 64, NPIX = 128 * NI, TH = NPIX / TW;
  static constexpr int RH = S * (TH - 1) + 3, RW = S * (TW - 1) + 3, NPOS = RH * RW;
  static constexpr int NITEM = 2 * NPOS;                   // (channel group, position)
  static constexpr int NIT = (NITEM + 255) / 256;          // items per thread
  static constexpr int NITP = NIT * 256;                   // padded: stores unconditional
  static constexpr int WT_U = 9 * 2 * 2 * BM;              // 16-B units per weight chunk
  static constexpr int NWT = WT_U / 256;
  static constexpr int LDS_BYTES = (2 * NITP + WT_U) * 16;
  static_assert(WT_U % 256 == 0, "weight units per thread");
  static_assert(16 * NPIX * 4 + 16 * BM * 4 <= LDS_BYTES, "phase-2 staging fits");
  static_assert(TW != 64 || NI != 2 || S != 1 || GramPlanes<256>::BYTES <= LDS_BYTES,
                "fused Gram planes fit");
};

// The v1 main loop: the stride-2 downsampling convs (LM_S2) and the split
// Gram-backward phase alone (P2 = 2, the 1x1 mode with cin == 0); every other
// stride-1 launch runs the v2 loop below.
// P2: 0 plain conv, 2 the split Gram-backward phase alone (1x1 mode, cin == 0)
template <int TW, int LM, int P2 = 0, int NI = 2>
__global__ void __launch_bounds__(256, 2)
conv3x3_f16x3_kernel(stx_conv_params p, int tiles_x) {
  constexpr int S = LM == LM_S2 ? 2 : 1;
  using C = C16<TW, NI, S>;
  constexpr bool RP = TW == 64 && NI == 2 && S == 1;  // row-pair tiles (fused pool / unpool)
  static_assert(P2 == 0 || P2 == 2, "v1 kernel: plain conv or the split phase alone");
  static_assert(P2 == 0 || NI == 2, "the Gram-backward phase assumes 256-pixel tiles");
  constexpr int BM = C::BM;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS_BYTES];
  char* lds_h = smem;                       // halo, hi plane then lo plane
  char* lds_w = smem + 2 * C::NITP * 16;    // weight chunk

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;

  const int tile = blockIdx.x;
  const int ty0 = (tile / tiles_x) * C::TH, tx0 = (tile % tiles_x) * TW;
  const int co0 = blockIdx.y * BM;
  const int n = blockIdx.z;

  const int nchunks = cdiv(p.cin, 16);  // 0: Gram-backward phase only (1x1 mode)
  const int ex = nchunks ? amax_exp(read_amax(p.in_amax)) : 0;
  const int ew = nchunks ? amax_exp(read_amax(p.w_amax)) : 0;
  const float sx = __builtin_ldexpf(1.f, 15 - ex);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);

  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * p.cin * plane_in;
  const int vy0 = S * ty0 - 1, vx0 = S * tx0 - 1;

  // chunk-invariant byte offsets of channel 0 of each halo item (BUF_OOB = zero pad)
  uint32_t hoff[C::NIT];
#pragma unroll
  for (int r = 0; r < C::NIT; ++r) {
    const int idx = tid + r * 256;
    const int cg = idx / C::NPOS, pos = idx - cg * C::NPOS;
    const int rr = pos / C::RW, cc = pos - rr * C::RW;
    const int vy = vy0 + rr, vx = vx0 + cc;
    bool ok = idx < C::NITEM && vy >= 0 && vx >= 0 && vy < p.hv && vx < p.wv;
    int sy = vy, sx_ = vx;
    if (LM == STX_IN_RELU_POOL2) {
      sy = 2 * vy;
      sx_ = 2 * vx;
    } else if (LM == STX_IN_UPSAMPLE2) {
      sy = vy >> 1;
      sx_ = vx >> 1;
    } else if (LM == STX_IN_DILATE2) {
      ok = ok && !((vy | vx) & 1);
      sy = vy >> 1;
      sx_ = vx >> 1;
      ok = ok && sy < p.h && sx_ < p.w;
    }
    hoff[r] = ok ? (uint32_t)((cg * 8) * plane_in + sy * p.w + sx_) * 4u : BUF_OOB;
  }
  const uint32_t pb = (uint32_t)plane_in * 4u, wb = 4u * (uint32_t)p.w;

  // weight chunk: units u = tid + q*256 -> (seg = tap*4 + P*2 + cg, co)
  const int cout64 = rup(p.cout, 64);
  const uint32_t chunk_bytes = (uint32_t)(36 * cout64 * 16);
  uint32_t woff[C::NWT];
#pragma unroll
  for (int q = 0; q < C::NWT; ++q) {
    const int u = tid + q * 256;
    const int seg = u / BM, co = u - seg * BM;
    woff[q] = (uint32_t)((seg * cout64 + co0 + co) * 16);
  }
  const char* __restrict__ wt16 = reinterpret_cast<const char*>(p.wt16);

  float hv[C::NIT][8];
  f32x4 wreg[C::NWT];
  auto fetch = [&](int chunk) {
    const int c0 = chunk * 16;
    const auto rs = make_srd(xn + (size_t)c0 * plane_in, (uint32_t)(p.cin - c0) * pb);
#pragma unroll
    for (int r = 0; r < C::NIT; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t o = hoff[r] + (uint32_t)c * pb;
        if (LM == STX_IN_RELU_POOL2)
          hv[r][c] = pool4_bits(buf_ld(rs, o), buf_ld(rs, o + 4), buf_ld(rs, o + wb),
                                buf_ld(rs, o + wb + 4));
        else
          hv[r][c] = buf_ld(rs, o);
      }
    const auto rw = make_srd(reinterpret_cast<const float*>(wt16 + (size_t)chunk * chunk_bytes),
                             chunk_bytes);
#pragma unroll
    for (int q = 0; q < C::NWT; ++q) wreg[q] = buf_ld4(rw, woff[q]);
  };
  auto store = [&]() {
#pragma unroll
    for (int r = 0; r < C::NIT; ++r) {
      f16x8 hi, lo;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float v = hv[r][c];
        if (LM == STX_IN_RELU) v = relu_bits(v);  // (POOL2: pool4_bits applied the ReLU)
        v *= sx;
        const _Float16 vh = (_Float16)v;
        hi[c] = vh;
        lo[c] = (_Float16)(v - (float)vh);
      }
      const int idx = tid + r * 256;
      *reinterpret_cast<f16x8*>(lds_h + idx * 16) = hi;
      *reinterpret_cast<f16x8*>(lds_h + (C::NITP + idx) * 16) = lo;
    }
#pragma unroll
    for (int q = 0; q < C::NWT; ++q)
      *reinterpret_cast<f32x4*>(lds_w + (tid + q * 256) * 16) = wreg[q];
  };

  f32x16 acc[2][NI];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-lane operand bases (bytes)
  const char* bbase[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    int ty, tx;
    tile_pix<TW, RP, NI>(wave, j, l32, ty, tx);
    bbase[j] = lds_h + (h * C::NPOS + S * ty * C::RW + S * tx) * 16;
  }
  const char* abase = lds_w + (h * BM + l32) * 16;

  if (nchunks) fetch(0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();  // previous chunk's operand reads done
    store();
    __syncthreads();
    if (chunk + 1 < nchunks) fetch(chunk + 1);  // in flight across the MFMA loop
    // Operand reads run one product phase ahead of their use: a tap's three phases
    // (hi*hi, hi*lo, lo*hi; 2 x NI MFMAs each) are each preceded by the reads the NEXT
    // phase needs (B lo, then A lo, then the next tap's A hi + B hi), so every LDS
    // read has a whole phase of MFMAs (>= 4 x 32 cycles) to land, with at most
    // 2 x (2 + NI) operand registers live -- the register budget of two waves per SIMD
    // leaves no room for a whole second tap of operands.
    auto rdA = [&](int tap, int P, f16x8 (&a)[2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const f16x8*>(abase + (tap * 4 * BM + P * 2 * BM + i * 32) * 16);
    };
    auto rdB = [&](int tap, int P, f16x8 (&b)[NI]) {
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int j = 0; j < NI; ++j)
        b[j] = *reinterpret_cast<const f16x8*>(bbase[j] + (P * C::NITP + kh * C::RW + kw) * 16);
    };
    auto phase = [&](const f16x8 (&a)[2], const f16x8 (&b)[NI]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    };
    f16x8 ahi[2], alo[2], bhi[NI], blo[NI];
    rdA(0, 0, ahi);
    rdB(0, 0, bhi);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      rdB(tap, 1, blo);
      __builtin_amdgcn_sched_group_barrier(0x100, NI, 0);      // the reads, then
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);  // the phase's MFMAs
      phase(ahi, bhi);
      rdA(tap, 1, alo);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);
      phase(ahi, blo);
      f16x8 nah[2], nbh[NI];
      if (tap + 1 < 9) {
        rdA(tap + 1, 0, nah);
        rdB(tap + 1, 0, nbh);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 + NI, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);
      phase(alo, bhi);
      __builtin_amdgcn_sched_barrier(0);
      if (tap + 1 < 9) {
#pragma unroll
        for (int i = 0; i < 2; ++i) ahi[i] = nah[i];
#pragma unroll
        for (int j = 0; j < NI; ++j) bhi[j] = nbh[j];
      }
    }
  }
  __syncthreads();  // the epilogue's phase 2 re-uses the LDS
  const EpiTile et{n, co0, ty0, tx0, 0, wave, h, l32};
  if constexpr (P2 == 2) {
    // main accumulator first: de-scale, *acc_scale, ReLU mask (the order of the
    // fp32 path), then the split Gram-backward phase adds s2 * A[n] . p2_z
    const float sc = descale * (p.acc_scale ? *p.acc_scale : 1.f);
    const size_t plane = (size_t)p.ho * p.wo;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int ty, tx;
      tile_pix<TW, RP>(wave, j, l32, ty, tx);
      const int oy = min(ty0 + ty, p.ho - 1), ox = min(tx0 + tx, p.wo - 1);
      const size_t pofs = (size_t)oy * p.wo + ox;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r] * sc;
          if (p.mask) {
            const int co = min(co0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, p.cout - 1);
            if (!(p.mask[((size_t)n * p.cout + co) * plane + pofs] > 0.f)) v = 0.f;
          }
          acc[i][j][r] = v;
        }
    }
    phase2_f16<TW>(acc, p, n, co0, ty0, tx0, wave, h, l32, smem);
    stx_conv_params q = p;
    q.p2_z = nullptr;
    q.acc_scale = nullptr;
    q.mask = nullptr;
    conv_epilogue<BM, TW, C::NPIX, 16, RP, NI, false>(acc, q, et, 1.f, reinterpret_cast<float*>(smem),
                                           reinterpret_cast<float*>(smem + 16 * C::NPIX * 4));
    return;
  }
  if (conv_epilogue_plain<TW, NI, RP>(acc, p, et, descale, smem)) return;
  conv_epilogue<BM, TW, C::NPIX, 16, RP, NI, false>(acc, p, et, descale, reinterpret_cast<float*>(smem),
                                         reinterpret_cast<float*>(smem + 16 * C::NPIX * 4));
}

// ------------------------------------------------------------------ v2 main loop
// One block per 64-cout x 256 (128) pixel tile, two blocks per CU.  K
// runs in STEPS of (16-channel chunk, kernel row kh): the step's 3 taps x 64 couts of
// split weights (12 KB) and the chunk's halo sit in double-buffered LDS, so the next
// step's weights and a third of the next chunk's halo are converted and written while
// this step's MFMAs run, with ONE barrier per step (v1: two barriers per chunk and the
// whole restaging between them, and 36 KB of weights per chunk in one buffer).  Halo
// buffers are sized to the exact item count (v1 pads to a multiple of 256).  Stride 1,
// cin >= 16 only.
// WM = 2: one 8-wave block for 128 couts (waves 4..7 the second 64), the halo of the
// pixel tile staged once for both cout halves (the 128-channel layers)
template <int TW, int NI, int WM = 1, int MINLDS = 0>
struct C16v2 {
  static constexpr int NT = 256 * WM;
  static constexpr int BM = 64 * WM, NPIX = 128 * NI, TH = NPIX / TW;
  static constexpr int RH = TH + 2, RW = TW + 2, NPOS = RH * RW;
  static constexpr int NITEM = 2 * NPOS;               // (channel group, position) units
  static constexpr int NIT = (NITEM + NT - 1) / NT;    // items per thread
  static constexpr int HB = 2 * NITEM * 16;            // one halo buffer: hi plane, lo plane
  static constexpr int WU = 3 * 4 * BM;                // weight units per step: [tap][P][cg][co]
  static constexpr int NWU = WU / NT;
  static constexpr int WB = WU * 16;                   // one weight buffer
  static constexpr int LOOP_BYTES = 2 * HB + 2 * WB;
  // (the 128-channel fused Gram planes of a WM = 2, 64 x 4 tile: 135 KB, one block per CU)
  static constexpr int LDS_BYTES0 =
      WM == 2 && TW == 64 && NI == 2 && LOOP_BYTES < GramPlanes128::BYTES ? GramPlanes128::BYTES
                                                                           : LOOP_BYTES;
  // (MINLDS: the unpool epilogue's z buffers and A' for 128 channels, 64 KB)
  static constexpr int LDS_BYTES = LDS_BYTES0 < MINLDS ? MINLDS : LDS_BYTES0;
  static_assert(WU % NT == 0, "weight units per thread");
  static_assert(16 * NPIX * 4 + 16 * BM * 4 <= LDS_BYTES, "phase-2 staging fits");
  static_assert(TW != 64 || NI != 2 || GramPlanes<256>::BYTES <= LDS_BYTES, "Gram planes fit");
};

// UPP geometry: the parity-class form of a conv over a nearest x2 upsampled input
// (stx_conv_params.wt16_up).  A block takes 64 output columns x 4 output rows of ONE row
// parity a (rows ty0 + 2 wn + a), the N-tile j of a wave the column parity b = j (x =
// 2 l32 + j): every output row / column reads 2 input rows / columns, so the halo is the
// input's own 5 x 34 window, K steps are (16-channel chunk, ry) and each step holds the
// 4 (b, rx) taps' weights of parity a.
struct C16up {
  static constexpr int NT = 256, BM = 64, NPIX = 256, TH = 8;
  static constexpr int RH = 5, RW = 34, NPOS = RH * RW;
  static constexpr int NITEM = 2 * NPOS, NIT = (NITEM + NT - 1) / NT;
  static constexpr int HB = 2 * NITEM * 16;
  static constexpr int WU = 4 * 4 * BM, NWU = WU / NT, WB = WU * 16;
  static constexpr int LOOP_BYTES = 2 * HB + 2 * WB, LDS_BYTES = LOOP_BYTES;
  static_assert(16 * NPIX * 4 + 16 * BM * 4 <= LDS_BYTES, "phase-2 staging fits");
};

// K2: two groups of four waves per block (512 threads) walk alternate 16-channel chunks of
// the same tile with their own double-buffered halo / weight images and accumulators --
// two waves per SIMD in a grid of one block per CU (the unpool launch of conv3_1^T at
// B = 1); group 1 hands its sums to group 0 through LDS (acc0 + acc1, fixed order) and
// ends, group 0 runs the epilogue (waves that have ended are not counted at a barrier).
template <int TW, int LM, int P2, int NI, int WM = 1, bool K2 = false>
__global__ void __launch_bounds__(256 * WM * (K2 ? 2 : 1),
                                  (WM == 2 || K2) ? 1 : ((NI == 1 && TW <= 32 && P2 == 0) ? 3 : 2))
conv3x3_f16x3_v2_kernel(stx_conv_params p, int tiles_x, int ntiles) {
  // PAR: the zero-dilated data gradient (a stride-2 conv's input gradient) on 64 x 4 tiles
  // whose N-tiles are output parity classes: of the 9 taps x 3 kernel rows only those that
  // meet the dilated input's non-zero (even) positions run -- a quarter of the MFMAs
  constexpr bool PAR = LM == STX_IN_DILATE2 && TW == 64 && NI == 2 && WM == 1 && P2 == 0;
  // UPP: the nearest-x2 upsampled input as four output-parity 2x2 convs (C16up)
  constexpr bool UPP = LM == STX_IN_UPSAMPLE2 && TW == 64 && NI == 2 && WM == 1 && P2 == 0;
  using C = std::conditional_t<UPP, C16up, C16v2<TW, NI, WM, P2 == 4 ? 65536 : 0>>;
  constexpr int NT = C::NT;
  constexpr int KS = UPP ? 2 : 3;  // K steps per 16-channel chunk
  constexpr bool RP = TW == 64 && NI == 2 && !PAR && !UPP;  // row-pair tiles (pool / unpool)
  static_assert(P2 == 0 || P2 == 4 || NI == 2, "the Gram-backward phase assumes 256-pixel tiles");
  static_assert(P2 != 4 || (TW == 32 && NI == 1 && WM == 1 && LM == STX_IN_RAW),
                "the unpool epilogue takes 32 x 4 tiles of a raw-input conv");
  static_assert(P2 != 2, "1x1 mode: v1 kernel");
  static_assert(WM == 1 || P2 == 0, "WM = 2: plain epilogue only");
  static_assert(!K2 || (WM == 1 && !PAR && !UPP), "K2: the plain 4-wave loop");
  constexpr int BM = C::BM;
  constexpr int NG = K2 ? 2 : 1;  // chunk groups
  constexpr int LDSB = NG * C::LOOP_BYTES > C::LDS_BYTES ? NG * C::LOOP_BYTES : C::LDS_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];

  const int tid = K2 ? (int)(threadIdx.x & 255) : (int)threadIdx.x;
  const int gk = K2 ? __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 8) : 0;
  char* const sg = smem + gk * C::LOOP_BYTES;  // this group's loop buffers
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // cout half, pixel column of the wave
  const int h = lane >> 5, l32 = lane & 31;
  const int co0 = blockIdx.y * BM;
  const int n = blockIdx.z;
  // the blocks of one XCD (blockIdx % 8 under round-robin placement) take consecutive
  // tiles, so neighbouring halos meet in the same L2 (speed only)
  const int G = gridDim.x;
  const int first = (G & 7) == 0 ? (int)(blockIdx.x & 7) * (G >> 3) + (int)(blockIdx.x >> 3)
                                 : (int)blockIdx.x;
  if (first >= ntiles) return;

  // the second-dispatched half of the blocks (blockIdx >> 8 odd: the co-resident partner
  // under round-robin placement) at wave priority 1, so the two blocks of a CU drift
  // apart instead of issuing their epilogue stores together (same-process A/B:
  // Gatys 679.6 -> 674.5 us per iteration, fast_st within noise)
  if ((blockIdx.x >> 8) & 1) __builtin_amdgcn_s_setprio(1);
  // (K2: this group's chunks gch(c) = 2c + gk of an even count -- launch16_unpool)
  const int nchunks = cdiv(p.cin, 16) / NG;
  const int nsteps = KS * nchunks;
  auto gch = [&](int c) { return NG * c + gk; };  // global chunk of local chunk c
  // the parity-class forms with cout <= 32 in this block (the ITN's 32-channel layers:
  // the up conv to 32 channels, the first down conv's data gradient): the second 32-row
  // MFMA tile would only multiply the slab's zero padding
  const bool half_m = (PAR || UPP) && co0 + 32 >= p.cout;
  const int ex = amax_exp(read_amax(p.in_amax));
  const int ew = amax_exp(read_amax(p.w_amax)) + (UPP ? 2 : 0);  // (UPP: |W'| <= 4 max|w|)
  const float sx = __builtin_ldexpf(1.f, 15 - ex);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);

  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * p.cin * plane_in;
  const uint32_t pb = (uint32_t)plane_in * 4u, wrow = 4u * (uint32_t)p.w;

  // weight units of a step: u = tid + q*256 -> (seg = tap*4 + P*2 + cg, co)
  const int cout64 = rup(p.cout, 64);
  const uint32_t chunk_bytes = (uint32_t)((UPP ? 32 : 36) * cout64 * 16);
  const uint32_t step_bytes = (uint32_t)((UPP ? 16 : 12) * cout64 * 16);
  uint32_t woff[C::NWU];
#pragma unroll
  for (int q = 0; q < C::NWU; ++q) {
    const int u = tid + q * NT;
    const int seg = u / BM, co = u - seg * BM;
    woff[q] = (uint32_t)((seg * cout64 + co0 + co) * 16);
  }
  const char* __restrict__ wt16 = reinterpret_cast<const char*>(UPP ? p.wt16_up : p.wt16);

  uint32_t hoff[C::NIT];
  int ty0 = 0, tx0 = 0, upa = 0;
  auto halo_offsets = [&](int tile) {
    if constexpr (UPP) {
      // tile -> (8-row band, row parity a, 64-column band); the halo: input rows
      // ty0/2 + a - 1 .. +4, columns tx0/2 - 1 .. +33
      const int r2 = tile / tiles_x;
      upa = r2 & 1;
      ty0 = (r2 >> 1) * C::TH;
      tx0 = (tile % tiles_x) * TW;
      const int yb = (ty0 >> 1) + upa - 1, xb = (tx0 >> 1) - 1;
#pragma unroll
      for (int r = 0; r < C::NIT; ++r) {
        const int idx = tid + r * NT;
        const int cg = idx / C::NPOS, pos = idx - cg * C::NPOS;
        const int rr = pos / C::RW, cc = pos - rr * C::RW;
        const int sy = yb + rr, sx_ = xb + cc;
        const bool ok = idx < C::NITEM && sy >= 0 && sx_ >= 0 && sy < p.h && sx_ < p.w;
        hoff[r] = ok ? (uint32_t)((cg * 8) * plane_in + sy * p.w + sx_) * 4u : BUF_OOB;
      }
      return;
    }
    ty0 = (tile / tiles_x) * C::TH;
    tx0 = (tile % tiles_x) * TW;
    const int vy0 = ty0 - 1, vx0 = tx0 - 1;
#pragma unroll
    for (int r = 0; r < C::NIT; ++r) {
      const int idx = tid + r * NT;
      const int cg = idx / C::NPOS, pos = idx - cg * C::NPOS;
      const int rr = pos / C::RW, cc = pos - rr * C::RW;
      const int vy = vy0 + rr, vx = vx0 + cc;
      bool ok = idx < C::NITEM && vy >= 0 && vx >= 0 && vy < p.hv && vx < p.wv;
      int sy = vy, sx_ = vx;
      if (LM == STX_IN_RELU_POOL2) {
        sy = 2 * vy;
        sx_ = 2 * vx;
      } else if (LM == STX_IN_UPSAMPLE2) {
        sy = vy >> 1;
        sx_ = vx >> 1;
      } else if (LM == STX_IN_DILATE2) {
        ok = ok && !((vy | vx) & 1);
        sy = vy >> 1;
        sx_ = vx >> 1;
        ok = ok && sy < p.h && sx_ < p.w;
      }
      hoff[r] = ok ? (uint32_t)((cg * 8) * plane_in + sy * p.w + sx_) * 4u : BUF_OOB;
    }
  };

  float hv[C::NIT][8];
  f32x4 wreg[C::NWU];
  auto ld_halo = [&](int chunk, int r) {
    const int c0 = gch(chunk) * 16;
    const auto rs = make_srd(xn + (size_t)c0 * plane_in, (uint32_t)(p.cin - c0) * pb);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint32_t o = hoff[r] + (uint32_t)c * pb;
      if (LM == STX_IN_RELU_POOL2)
        hv[r][c] = pool4_bits(buf_ld(rs, o), buf_ld(rs, o + 4), buf_ld(rs, o + wrow),
                              buf_ld(rs, o + wrow + 4));
      else
        hv[r][c] = buf_ld(rs, o);
    }
  };
  auto st_halo = [&](int buf, int r) {
    const int idx = tid + r * NT;
    if (r + 1 < C::NIT || C::NITEM % NT == 0 || idx < C::NITEM) {
      char* hb = sg + buf * C::HB;
#ifdef STX_DIAG_NOSPLIT
      // timing-only diagnostic build (make DIAG=1, numerically meaningless): the loader's
      // values stored as raw fp32 bits in the two planes -- no scale, no fp16 conversion
      f32x4 a, b;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        a[c] = hv[r][c];
        b[c] = hv[r][c + 4];
        if (LM == STX_IN_RELU || LM == STX_IN_RELU_POOL2) {
          a[c] = fmaxf(a[c], 0.f);
          b[c] = fmaxf(b[c], 0.f);
        }
      }
      *reinterpret_cast<f32x4*>(hb + idx * 16) = a;
      *reinterpret_cast<f32x4*>(hb + (C::NITEM + idx) * 16) = b;
#else
      f16x8 hi, lo;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        // ReLU as an integer max of the bit pattern (negative floats are negative ints):
        // one v_max_i32 -- fmaxf of a loaded value costs two v_max_f32 (the first
        // canonicalises the operand)
        float v = hv[r][c];
        if (LM == STX_IN_RELU) v = relu_bits(v);  // (POOL2: pool4_bits applied the ReLU)
        v *= sx;
        const _Float16 vh = (_Float16)v;
        hi[c] = vh;
        lo[c] = (_Float16)(v - (float)vh);
      }
      *reinterpret_cast<f16x8*>(hb + idx * 16) = hi;
      *reinterpret_cast<f16x8*>(hb + (C::NITEM + idx) * 16) = lo;
#endif
    }
  };
  auto ld_w = [&](int step) {  // step = chunk * KS + kh (UPP: ry)
    const int chunk = gch(step / KS), kh = step - KS * (step / KS);
    const size_t base = UPP ? (size_t)upa * nchunks * chunk_bytes : 0;  // (UPP: parity a)
    const auto rw = make_srd(reinterpret_cast<const float*>(wt16 + base +
                                                            (size_t)chunk * chunk_bytes +
                                                            (size_t)kh * step_bytes),
                             step_bytes);
#pragma unroll
    for (int q = 0; q < C::NWU; ++q) wreg[q] = buf_ld4(rw, woff[q]);
  };
  auto st_w = [&](int buf) {
    char* wbp = sg + 2 * C::HB + buf * C::WB;
#pragma unroll
    for (int q = 0; q < C::NWU; ++q)
      *reinterpret_cast<f32x4*>(wbp + (tid + q * NT) * 16) = wreg[q];
  };

  // per-lane operand bases (bytes) relative to buffer 0
  int boff[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    int ty, tx;
    tile_pix<TW, RP, NI, PAR>(wn, j, l32, ty, tx);
    // UPP: halo row wn (+ ry), column l32 + j (+ rx) -- see C16up
    boff[j] = UPP ? (h * C::NPOS + wn * C::RW + l32 + j) * 16
                  : (h * C::NPOS + ty * C::RW + tx) * 16;
  }
  const int aoff = 2 * C::HB + (h * BM + wm * 64 + l32) * 16;

  const int tile = first;
  halo_offsets(tile);
#pragma unroll
  for (int r = 0; r < C::NIT; ++r) ld_halo(0, r);
  ld_w(0);
  {
    // chunk 0's halo and step 0's weights -> buffers 0
#pragma unroll
    for (int r = 0; r < C::NIT; ++r) st_halo(0, r);
    st_w(0);
    // staged for step 0: step 1's weights, part 0 of chunk 1's halo
    if (nsteps > 1) ld_w(1);
    if (nchunks > 1) {
#pragma unroll
      for (int r = 0; r < C::NIT; r += KS) ld_halo(1, r);
    }
    __syncthreads();

    f32x16 acc[2][NI];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    for (int c = 0; c < nchunks; ++c) {
      const int hbo = (c & 1) * C::HB;
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int s = KS * c + k;
        const int wbo = (s & 1) * C::WB;
        const char* abase = sg + aoff + wbo;
        const char* bbase[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) bbase[j] = sg + boff[j] + hbo;
        auto rdA = [&](int tl, int P, f16x8 (&a)[2]) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
            a[i] = *reinterpret_cast<const f16x8*>(abase + (tl * 4 * BM + P * 2 * BM + i * 32) * 16);
        };
        auto rdB = [&](int tl, int P, f16x8 (&b)[NI]) {
#pragma unroll
          for (int j = 0; j < NI; ++j)
            b[j] = *reinterpret_cast<const f16x8*>(bbase[j] + (P * C::NITEM + k * C::RW + tl) * 16);
        };
        auto phase = [&](const f16x8 (&a)[2], const f16x8 (&b)[NI]) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[j], acc[i][j], 0, 0, 0);
        };
        if constexpr (UPP) {
          // staging for step s+1 first, then this step's 4 taps (b = j, rx) at input row
          // wn + ry (= k) of the halo: 2 A fragments and 2 B fragments per tap
          if (s + 1 < nsteps) st_w((s + 1) & 1);
          if (c + 1 < nchunks) {
#pragma unroll
            for (int r = k; r < C::NIT; r += KS) st_halo((c + 1) & 1, r);
          }
          if (s + 2 < nsteps) ld_w(s + 2);
          {
            const int cn = k < KS - 1 ? c + 1 : c + 2;
            if (cn < nchunks) {
#pragma unroll
              for (int r = (k + 1) % KS; r < C::NIT; r += KS) ld_halo(cn, r);
            }
          }
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int rx = 0; rx < 2; ++rx) {
              f16x8 ah[2], al[2];
              rdA(2 * j + rx, 0, ah);
              rdA(2 * j + rx, 1, al);
              const f16x8 bh = *reinterpret_cast<const f16x8*>(bbase[j] + (k * C::RW + rx) * 16);
              const f16x8 bl =
                  *reinterpret_cast<const f16x8*>(bbase[j] + (C::NITEM + k * C::RW + rx) * 16);
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                if (i == 1 && half_m) break;  // (rows past cout: nothing to compute)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, acc[i][j], 0, 0, 0);
              }
            }
          __syncthreads();
          continue;
        }
        if constexpr (PAR) {
          // staging for step s+1 first (every wave), then this step's taps, only in the
          // waves whose output row meets a non-zero dilated row at this kernel row (the
          // tile's rows start even: the wave's row parity is wn's) and, per tap, only the
          // N-tile of the column parity that meets a non-zero column
          if (s + 1 < nsteps) st_w((s + 1) & 1);
          if (c + 1 < nchunks) {
#pragma unroll
            for (int r = k; r < C::NIT; r += 3) st_halo((c + 1) & 1, r);
          }
          if (s + 2 < nsteps) ld_w(s + 2);
          {
            const int cn = k < 2 ? c + 1 : c + 2;
            if (cn < nchunks) {
#pragma unroll
              for (int r = (k + 1) % 3; r < C::NIT; r += 3) ld_halo(cn, r);
            }
          }
          if (((k + wn) & 1) == 1) {
#pragma unroll
            for (int tl = 0; tl < 3; ++tl) {
              const int jt = (tl + 1) & 1;  // x + tl - 1 even <=> x parity != tl parity
              f16x8 ah[2], al[2];
              rdA(tl, 0, ah);
              rdA(tl, 1, al);
              const f16x8 bh = *reinterpret_cast<const f16x8*>(bbase[jt] + (k * C::RW + tl) * 16);
              const f16x8 bl =
                  *reinterpret_cast<const f16x8*>(bbase[jt] + (C::NITEM + k * C::RW + tl) * 16);
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                if (i == 1 && half_m) break;  // (rows past cout: nothing to compute)
                acc[i][jt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, acc[i][jt], 0, 0, 0);
                acc[i][jt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, acc[i][jt], 0, 0, 0);
                acc[i][jt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, acc[i][jt], 0, 0, 0);
              }
            }
          }
          __syncthreads();
          continue;
        }
        f16x8 ahi[2], alo[2], bhi[NI], blo[NI];
        rdA(0, 0, ahi);
        rdB(0, 0, bhi);
#pragma unroll
        for (int tl = 0; tl < 3; ++tl) {
          rdB(tl, 1, blo);
          __builtin_amdgcn_sched_group_barrier(0x100, NI, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);
          phase(ahi, bhi);
          rdA(tl, 1, alo);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);
          phase(ahi, blo);
          f16x8 nah[2], nbh[NI];
          if (tl + 1 < 3) {
            rdA(tl + 1, 0, nah);
            rdB(tl + 1, 0, nbh);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 + NI, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI, 0);
          phase(alo, bhi);
          __builtin_amdgcn_sched_barrier(0);
          if (tl == 0) {
            // staged data -> the other buffers: step s+1's weights and part k of chunk
            // c+1's halo (loaded one step ago); then the loads for step s+1's staging:
            // step s+2's weights and the next part of the halo
            if (s + 1 < nsteps) st_w((s + 1) & 1);
            if (c + 1 < nchunks) {
#pragma unroll
              for (int r = k; r < C::NIT; r += 3) st_halo((c + 1) & 1, r);
            }
            if (s + 2 < nsteps) ld_w(s + 2);
            const int cn = k < 2 ? c + 1 : c + 2;  // chunk of the next halo part
            if (cn < nchunks) {
#pragma unroll
              for (int r = (k + 1) % 3; r < C::NIT; r += 3) ld_halo(cn, r);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
          if (tl + 1 < 3) {
#pragma unroll
            for (int i = 0; i < 2; ++i) ahi[i] = nah[i];
#pragma unroll
            for (int j = 0; j < NI; ++j) bhi[j] = nbh[j];
          }
        }
        __syncthreads();  // this step's reads done; the staged buffers are complete
      }
    }
    if constexpr (K2) {
      // group 1's accumulators -> LDS (the loop buffers are dead after its last barrier),
      // group 0 adds them; group 1 ends here
      float* red = reinterpret_cast<float*>(smem);
      if (gk == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[(((wave * 2 + i) * NI + j) * 16 + r) * 64 + lane] = acc[i][j][r];
      }
      __syncthreads();
      if (gk == 1) return;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += red[(((wave * 2 + i) * NI + j) * 16 + r) * 64 + lane];
      __syncthreads();  // (the epilogue reuses this LDS)
    }

    EpiTile et{n, co0, ty0, tx0, wm, wn, h, l32};
    et.tile = tile;
    et.ntiles = ntiles;
    if constexpr (UPP) {
      // the PAR pixel mapping (x = 2 l32 + j, y = wn) with rows 2 wn + a: paired stores
      et.wn = 2 * wn;
      et.ty0 = ty0 + upa;
      conv_epilogue_plain<TW, NI, false, true>(acc, p, et, descale, smem);  // (launch16up)
    } else if constexpr (PAR) {
      conv_epilogue_plain<TW, NI, false, true>(acc, p, et, descale, smem);  // (launch16v2)
    } else if constexpr (WM == 2) {
      // (eligibility: launch16v2 / launch16_gram128)
      conv_epilogue_plain<TW, NI, RP, false, WM>(acc, p, et, descale, smem);
    } else if constexpr (P2 == 4) {
      // (eligibility: stx_conv2d -- stx_conv_params.unpool_out)
      static_assert(2 * 2 * 2 * 2 * 128 * 16 + 128 * 256 <= C::LDS_BYTES,
                    "unpool epilogue buffers fit");
      epi_unpool_gram<TW>(acc, p, et, descale, smem);
    } else if constexpr (P2 == 3) {
      // (eligibility: launch16v2 -- data gradient + mask + the phase, bias / out_amax only)
      const int ez = amax_exp(read_amax(p.p2_amax));
      const int ea = amax_exp(read_amax(p.p2_wt_amax) * fabsf(p.p2_scale ? *p.p2_scale : 1.f));
      // |acc| < 9 cin16 2^(ex + ew) |acc_scale|: every split-operand product is below 2^30
      // before the de-scale
      const int eacc = ex + ew + (32 - __builtin_clz(9 * rup(p.cin, 16))) + 1 +
                       amax_exp(p.acc_scale ? fabsf(*p.acc_scale) : 1.f);
      const int ls = max(min(min(30 - ea - ez, 100 - eacc), 120), -100);
      // de-scale, *acc_scale, ReLU mask, bring to 2^ls: run by the phase once its first
      // chunk's loads are in flight (the mask loads and those overlap)
      auto prologue = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] *= descale;
        epi_scale_mask<TW, RP, NI>(acc, p, et);
        const float up = __builtin_ldexpf(1.f, ls);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] *= up;
      };
      static_assert(2 * (4 * 256 * 16 + 4 * 64 * 16) <= C::LDS_BYTES, "phase-2 buffers fit");
      phase2_pre<TW, RP>(acc, p, et, ls, ez, smem, prologue);
      conv_epilogue_plain_body<TW, NI, RP, false>(acc, p, et, __builtin_ldexpf(1.f, -ls), smem);
    } else if constexpr (P2 == 1) {
      conv_epilogue<BM, TW, C::NPIX, 16, RP, NI, true>(acc, p, et, descale,
                                                       reinterpret_cast<float*>(smem),
                                                       reinterpret_cast<float*>(smem + 16 * C::NPIX * 4));
    } else {
      if (!conv_epilogue_plain<TW, NI, RP>(acc, p, et, descale, smem))
        conv_epilogue<BM, TW, C::NPIX, 16, RP, NI, false>(acc, p, et, descale,
                                                          reinterpret_cast<float*>(smem),
                                                          reinterpret_cast<float*>(smem + 16 * C::NPIX * 4));
    }
  }
}

static int cus16() {  // compute units (the WM = 2 form pays only in a single round of blocks)
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

static bool wm2_on() {  // STX_V2_WM2=0: 64-cout blocks for every layer (A/B)
  static const bool on = STX_KNOB("STX_V2_WM2", 1) != 0;
  return on;
}

static bool p2_split_on() {  // STX_P2_SPLIT=0: the fp32-MFMA phase even given p2_wt_amax (A/B)
  static const bool on = STX_KNOB("STX_P2_SPLIT", 1) != 0;
  return on;
}

template <int TW, int LM, int NI>
static int launch16v2(const stx_conv_params& p, hipStream_t st) {
  using C = C16v2<TW, NI>;
  const int tiles_x = cdiv(p.wo, TW), tiles_y = cdiv(p.ho, C::TH);
  const int ntiles = tiles_x * tiles_y;
  dim3 grid(ntiles, cdiv(p.cout, C::BM), p.n);
  if (p.p2_z) {
    // the fused Gram-backward phase: 256-pixel tiles of a raw-input data gradient
    if constexpr (NI == 2 && LM == STX_IN_RAW) {
      if (p.p2_wt_amax && p2_split_on() && !p.up_dp && !p.aux && !p.accumulate &&
          !p.relu_out && !p.pool_out && !p.gram_part) {
        hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<TW, LM, 3, NI>), grid, dim3(256), 0, st, p,
                           tiles_x, ntiles);
        return check_launch("stx_conv2d(f16x3 v2 + split phase 2)");
      }
      hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<TW, LM, 1, NI>), grid, dim3(256), 0, st, p,
                         tiles_x, ntiles);
      return check_launch("stx_conv2d(f16x3 v2 + phase 2)");
    }
    set_error("stx_conv2d: the fused Gram-backward phase needs a raw-input conv");
    return STX_E_INVALID;
  }
  // 128-pixel tiles of a 128-channel layer through the plain epilogue, when the grid is at
  // most one block per CU and fills (nearly) every CU (the ImageTransformNet's residual
  // convs at B = 8: 256 blocks; a 128-block grid left half the CUs idle -- Gatys' conv3_1
  // data gradient 39 -> 48 us -- and B = 1's 32 blocks lost to the 64-cout form's 64): one
  // 8-wave block per 128 couts, the tile's halo staged once for both cout halves (same-box
  // A/B: fast_st 4607/4626 -> 4570/4592 us per step; Gatys' 512-block conv3_1 lost 5 us)
  if constexpr (NI == 1)
    if (wm2_on() && p.cout % 128 == 0 && (long long)ntiles * (p.cout / 128) * p.n <= cus16() &&
        10LL * ntiles * (p.cout / 128) * p.n >= 9LL * cus16() &&  // a (nearly) full round
        !p.mask && !p.accumulate && !p.acc_scale && !p.up_dp &&
        !p.pool_out && !p.pool_sum && !p.gram_part && !(p.aux && p.relu_out)) {
      dim3 g2(ntiles, p.cout / 128, p.n);
      hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<TW, LM, 0, NI, 2>), g2, dim3(512), 0, st, p,
                         tiles_x, ntiles);
      return check_launch("stx_conv2d(f16x3 v2, 128 couts)");
    }
#ifdef STX_AB  // STX_FORCE_WM2=1: 8-wave 128-cout blocks on 64 x 4 tiles without the Gram (A/B)
  if constexpr (NI == 2 && TW == 64 && (LM == STX_IN_RAW || LM == STX_IN_RELU))
    if (STX_KNOB("STX_FORCE_WM2", 0) && p.cout % 128 == 0 && !p.mask && !p.accumulate &&
        !p.acc_scale && !p.up_dp && !p.pool_sum && !p.gram_part && !p.aux) {
      dim3 g2(ntiles, p.cout / 128, p.n);
      hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<TW, LM, 0, NI, 2>), g2, dim3(512), 0, st, p,
                         tiles_x, ntiles);
      return check_launch("stx_conv2d(f16x3 v2, 128 couts, forced)");
    }
#endif
  if constexpr (LM == STX_IN_DILATE2 && TW == 64 && NI == 2)
    if (p.mask || p.accumulate || p.acc_scale || p.up_dp || p.pool_out || p.pool_sum ||
        p.gram_part || (p.aux && p.relu_out)) {
      set_error("stx_conv2d: zero-dilated input on 64 x 4 tiles takes the plain epilogue only");
      return STX_E_INVALID;
    }
  hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<TW, LM, 0, NI>), grid, dim3(256), 0, st, p,
                     tiles_x, ntiles);
  return check_launch("stx_conv2d(f16x3 v2)");
}

template <int TW, int LM, int NI>
static int launch16(const stx_conv_params& p, hipStream_t st) {
  using C = C16<TW, NI, LM == LM_S2 ? 2 : 1>;
  // the v2 main loop: stride 1 with a 3x3 K loop (not the 1x1 Gram-backward mode)
  if constexpr (LM != LM_S2)
    if (p.cin > 0) return launch16v2<TW, LM, NI>(p, st);
  const int tiles_x = cdiv(p.wo, TW), tiles_y = cdiv(p.ho, C::TH);
  dim3 grid(tiles_x * tiles_y, cdiv(p.cout, C::BM), p.n);
  if (p.p2_z) {
    if constexpr (LM == STX_IN_RAW && NI == 2) {
      hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM, 2>), grid, dim3(256), 0, st, p, tiles_x);
      return check_launch("stx_conv2d(f16x3, split phase 2 alone)");
    }
    set_error("stx_conv2d: the fused Gram-backward phase needs a raw-input conv");
    return STX_E_INVALID;
  }
  hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM, 0, NI>), grid, dim3(256), 0, st, p, tiles_x);
  return check_launch("stx_conv2d(f16x3)");
}

// 256-pixel tiles (NI = 2) unless that grid leaves CUs idle: then 128-pixel tiles
// (twice the blocks; not with the fused pool output or the Gram-backward phase,
// which rely on the 256-pixel row-pair tile)
// the 128-channel fused Gram (conv_gram_tile128): one 8-wave block per 64 x 4 tile holds
// all 128 couts (stx_conv_gram_tiles admits only these: plain epilogue, raw / ReLU input)
template <int LM>
static int launch16_gram128(const stx_conv_params& p, hipStream_t st) {
  using C = C16v2<64, 2, 2>;
  const int tiles_x = cdiv(p.wo, 64), tiles_y = cdiv(p.ho, C::TH);
  const int ntiles = tiles_x * tiles_y;
  hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<64, LM, 0, 2, 2>), dim3(ntiles, 1, p.n), dim3(512),
                     0, st, p, tiles_x, ntiles);
  return check_launch("stx_conv2d(f16x3 v2, 128 couts + fused Gram)");
}

template <int TW, int LM>
static int launch16_ni(const stx_conv_params& p, hipStream_t st) {
  if constexpr (TW == 64 && (LM == STX_IN_RAW || LM == STX_IN_RELU))
    if (p.gram_part && p.cout == 128) return launch16_gram128<LM>(p, st);
  const long long blocks2 = (long long)cdiv(p.wo, TW) * cdiv(p.ho, 256 / TW) *
                            cdiv(p.cout, 64) * p.n;
  // 256-pixel-tile grids smaller than two resident rounds use 128-px tiles
  if (blocks2 < 512 && !p.pool_out && !p.p2_z && !p.gram_part) {
    // 128-pixel tiles as 32 x 4 rather than 64 x 2: a 34 x 6 halo instead of 66 x 4 (23 %
    // less staging per tile) -- Gatys NI=1 launches 37-40 -> 35-39 us, ITN residual convs
    // 35.3 -> 34.7 us (same-box profile)
    if constexpr (TW == 64) return launch16<32, LM, 1>(p, st);
    return launch16<TW, LM, 1>(p, st);
  }
  // 256-pixel tiles of the transforming loaders (ReLU, nearest x2, zero-dilation) without
  // a row-pair epilogue (no pool output / unpool / Gram / Gram-backward phase): 32 x 8
  // (34 x 10 halo) instead of 64 x 4 (66 x 6) -- same-box profile of the fast_st step:
  // upsampling convs 92 -> 84 and 49 -> 45 us, dilated (stride-2 dgrad) 89 -> 85 and
  // 55 -> 52, ReLU 101 -> 98; raw-input launches measured 1 % slower and keep 64 x 4.
  // the zero-dilated input (a stride-2 conv's data gradient) with the plain epilogue: 64 x 4
  // parity-class tiles (PAR in conv3x3_f16x3_v2_kernel: a quarter of the MFMAs)
  if constexpr (TW == 64 && LM == STX_IN_DILATE2)
    if (!p.mask && !p.accumulate && !p.acc_scale && !p.up_dp && !p.pool_out && !p.pool_sum &&
        !p.gram_part && !p.p2_z && !(p.aux && p.relu_out))
      return launch16<64, LM, 2>(p, st);
  if constexpr (TW == 64 && LM != STX_IN_RAW)
    if (!p.pool_out && !p.gram_part && !p.p2_z && !p.up_dp)
      return launch16<32, LM, 2>(p, st);
  if constexpr (TW == 64 && LM == STX_IN_UPSAMPLE2) {
    // (the 64 x 4 instantiation of this loader is the parity-class kernel, launch16up)
    set_error("stx_conv2d: an upsampled-input conv takes no fused pool output / Gram / "
              "unpool epilogue");
    return STX_E_INVALID;
  } else {
    return launch16<TW, LM, 2>(p, st);
  }
}

// the parity-class form of a conv over a nearest x2 upsampled input (stx_conv_params.wt16_up)
static int launch16up(const stx_conv_params& p, hipStream_t st) {
  const int tiles_x = cdiv(p.wo, 64), ntiles = tiles_x * 2 * cdiv(p.ho, C16up::TH);
  hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<64, STX_IN_UPSAMPLE2, 0, 2>),
                     dim3(ntiles, cdiv(p.cout, 64), p.n), dim3(256), 0, st, p, tiles_x, ntiles);
  return check_launch("stx_conv2d(f16x3 v2, upsampled input as parity classes)");
}

template <int LM>
static int dispatch16_tw(const stx_conv_params& p, hipStream_t st) {
  if (p.wo > 32) return launch16_ni<64, LM>(p, st);
  if (p.pool_out) {
    set_error("stx_conv2d: pool_out needs wo > 32 (row-pair tile mapping)");
    return STX_E_INVALID;
  }
  if (p.wo > 16) return launch16_ni<32, LM>(p, st);
  return launch16_ni<16, LM>(p, st);
}

// ------------------------------------------------------------ weight split prep
// slab [cin16/16][tap][P][cg][cout64][8] fp16 of the GEMM weights W'[co][ci][tap]
__device__ __forceinline__ void weight_prep16_body(const float* __restrict__ w,
                                                   _Float16* __restrict__ out,
                                                   const float* __restrict__ w_amax, int cout,
                                                   int cin, int transpose, int gin16, int gout64,
                                                   long long i0, long long step) {
  // 32-bit index math (slabs are < 2^31 elements; 64-bit div/mod is a long
  // software sequence on the GPU)
  const int total = gin16 * 9 * 2 * gout64;
  const float sw = __builtin_ldexpf(1.f, 15 - amax_exp(read_amax(w_amax)));
  for (int i = (int)i0; i < total; i += (int)step) {
    const int e = i & 7;
    unsigned r = (unsigned)i >> 3;
    const int co = (int)(r % (unsigned)gout64);
    r /= (unsigned)gout64;
    const int cg = (int)(r & 1);
    r >>= 1;
    const int P = (int)(r & 1);
    r >>= 1;
    const int tap = (int)(r % 9u);
    const int chunk = (int)(r / 9u);
    const int ci = chunk * 16 + cg * 8 + e;
    const int kh = tap / 3, kw = tap % 3;
    float v = 0.f;
    if (!transpose) {
      if (co < cout && ci < cin) v = w[(((size_t)co * cin + ci) * 3 + kh) * 3 + kw];
    } else {
      // data-gradient GEMM: W'[co'=layer ci][ci'=layer co][tap] = w[ci'][co'][2-kh][2-kw]
      if (ci < cout && co < cin) v = w[(((size_t)ci * cin + co) * 3 + (2 - kh)) * 3 + (2 - kw)];
    }
    v *= sw;
    const _Float16 vh = (_Float16)v;
    out[i] = P == 0 ? vh : (_Float16)(v - (float)vh);
  }
}

// The parity-class slab of a conv behind a nearest x2 upsampling (the ImageTransformNet's
// UpsampleConvLayer, stransfer/network.py:578-600): output pixel (2y + a, 2x + b) of the
// 3x3 conv over the upsampled input is a 2x2 conv over the input itself,
//   sum_{ry, rx} W'[a][b][ry][rx] x[y - 1 + a + ry][x - 1 + b + rx],
// W'[a][b][ry][rx] = sum of W[kh][kw] over kh in K(a, ry), kw in K(b, rx),
// K(0,0) = {0}, K(0,1) = {1,2}, K(1,0) = {0,1}, K(1,1) = {2} (rows y-1 / y or y / y+1 of the
// input: the zero padding of the upsampled image is the input's own).  Slab
// [a][cin16/16][ry][b*2+rx][P][cg][cout64][8] fp16, split at 2^(15 - e - 2) (|W'| <= 4
// max|w| < 2^(e+2)); sums in kh, kw order.
__device__ __forceinline__ void weight_prep16up_body(const float* __restrict__ w,
                                                     _Float16* __restrict__ out,
                                                     const float* __restrict__ w_amax, int cout,
                                                     int cin, int gin16, int gout64, long long i0,
                                                     long long step) {
  const int total = 2 * gin16 * 2 * 4 * 2 * 2 * gout64 * 8;
  const float sw = __builtin_ldexpf(1.f, 13 - amax_exp(read_amax(w_amax)));
  for (int i = (int)i0; i < total; i += (int)step) {
    const int e = i & 7;
    unsigned r = (unsigned)i >> 3;
    const int co = (int)(r % (unsigned)gout64);
    r /= (unsigned)gout64;
    const int cg = (int)(r & 1);
    const int P = (int)((r >> 1) & 1);
    const int t4 = (int)((r >> 2) & 3);
    const int ry = (int)((r >> 4) & 1);
    r >>= 5;
    const int chunk = (int)(r % (unsigned)gin16);
    const int a = (int)(r / (unsigned)gin16);
    const int b = t4 >> 1, rx = t4 & 1;
    const int ci = chunk * 16 + cg * 8 + e;
    const int kh0 = a == 0 ? (ry == 0 ? 0 : 1) : (ry == 0 ? 0 : 2);
    const int kh1 = a == 0 ? (ry == 0 ? 0 : 2) : (ry == 0 ? 1 : 2);
    const int kw0 = b == 0 ? (rx == 0 ? 0 : 1) : (rx == 0 ? 0 : 2);
    const int kw1 = b == 0 ? (rx == 0 ? 0 : 2) : (rx == 0 ? 1 : 2);
    float v = 0.f;
    if (co < cout && ci < cin) {
      const float* wp = w + ((size_t)co * cin + ci) * 9;
      for (int kh = kh0; kh <= kh1; ++kh)
        for (int kw = kw0; kw <= kw1; ++kw) v += wp[kh * 3 + kw];
    }
    v *= sw;
    const _Float16 vh = (_Float16)v;
    out[i] = P == 0 ? vh : (_Float16)(v - (float)vh);
  }
}

__global__ void weight_prep16up_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                       const float* __restrict__ w_amax, int cout, int cin,
                                       int gin16, int gout64) {
  weight_prep16up_body(w, out, w_amax, cout, cin, gin16, gout64,
                       blockIdx.x * (long long)blockDim.x + threadIdx.x,
                       (long long)gridDim.x * blockDim.x);
}

__global__ void weight_prep16_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                     const float* __restrict__ w_amax, int cout, int cin,
                                     int transpose, int gin16, int gout64) {
  weight_prep16_body(w, out, w_amax, cout, cin, transpose, gin16, gout64,
                     blockIdx.x * (long long)blockDim.x + threadIdx.x,
                     (long long)gridDim.x * blockDim.x);
}

// both slabs of one weight in one launch: blockIdx.y 0 = forward, 1 = data gradient
__global__ void weight_prep16_pair_kernel(const float* __restrict__ w, _Float16* __restrict__ fwd,
                                          _Float16* __restrict__ dgr,
                                          const float* __restrict__ w_amax, int cout, int cin) {
  const long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long step = (long long)gridDim.x * blockDim.x;
  if (blockIdx.y == 0)
    weight_prep16_body(w, fwd, w_amax, cout, cin, 0, rup(cin, 16), rup(cout, 64), i0, step);
  else
    weight_prep16_body(w, dgr, w_amax, cout, cin, 1, rup(cout, 16), rup(cin, 64), i0, step);
}

// -------------------------------------------------------------------- amax
__global__ void amax_zero_kernel(float* __restrict__ out) { out[threadIdx.x] = 0.f; }

__global__ void amax_kernel(const float* __restrict__ x, long long n, float* __restrict__ out) {
  float m = 0.f;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  auto upd = [&](float v) {
    const float a = fabsf(v);
    m = (a != a) ? a : fmaxf(m, a);
  };
  for (long long i = t0; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    upd(v[0]);
    upd(v[1]);
    upd(v[2]);
    upd(v[3]);
  }
  for (long long i = 4 * n4 + t0; i < n; i += stride) upd(x[i]);
  block_max_to(out, m);
}

// One launch, no clearing: exactly STX_AMAX_SLOTS blocks, block b reduces slice b of x
// and stores its max into slot b (plain store), so the group's max is max|x|.
__device__ __forceinline__ void amax_slot_body(const float* __restrict__ x, long long n,
                                               float* __restrict__ out, int slot) {
  __shared__ float red[16];
  const long long n4 = n >> 2;
  const long long per = (n4 + STX_AMAX_SLOTS - 1) / STX_AMAX_SLOTS;
  const long long b0 = slot * per, b1 = min(n4, b0 + per);
  float m = 0.f;
  auto upd = [&](float v) {
    const float a = fabsf(v);
    m = (a != a) ? a : fmaxf(m, a);
  };
#pragma unroll 4
  for (long long i = b0 + threadIdx.x; i < b1; i += 1024) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    upd(v[0]);
    upd(v[1]);
    upd(v[2]);
    upd(v[3]);
  }
  if (slot == 0)
    for (long long i = 4 * n4 + threadIdx.x; i < n; i += 1024) upd(x[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float other = __shfl_xor(m, o, 64);
    m = (other != other) ? other : fmaxf(m, other);
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) r = (red[i] != red[i]) ? red[i] : fmaxf(r, red[i]);
    out[slot] = r;
  }
}

__global__ void __launch_bounds__(1024) amax_slots_kernel(const float* __restrict__ x,
                                                          long long n, float* __restrict__ out) {
  amax_slot_body(x, n, out, blockIdx.x);
}

// ------------------------------------------------------- batched weight prep
// Every slab of a trained network re-prepped in two launches per step (the ITN: 31
// slabs of 14 weights would otherwise be ~35 launches, each a few microseconds of
// launch-bound tail): (1) the max|w| groups of the distinct split-slab weights, 32
// blocks each; (2) all conversions, a fixed block range per job.
struct WprepAmax {
  const float* w[STX_WPREP_MAX];
  float* out[STX_WPREP_MAX];
  long long n[STX_WPREP_MAX];
};

__global__ void __launch_bounds__(1024) amax_batch_kernel(WprepAmax a) {
  const int j = blockIdx.x / STX_AMAX_SLOTS;
  amax_slot_body(a.w[j], a.n[j], a.out[j], blockIdx.x % STX_AMAX_SLOTS);
}

struct WprepJobs {
  stx_wprep_job job[STX_WPREP_MAX];
  int blk0[STX_WPREP_MAX + 1];  // first block of each job (prefix sums)
  int gin[STX_WPREP_MAX], gout[STX_WPREP_MAX];  // padded GEMM dims of the slab
  int njobs;
};

__global__ void __launch_bounds__(256) weight_prep_batch_kernel(WprepJobs b) {
  int j = 0;
  while (j + 1 < b.njobs && (int)blockIdx.x >= b.blk0[j + 1]) ++j;
  const stx_wprep_job& t = b.job[j];
  const int nb = b.blk0[j + 1] - b.blk0[j];
  const long long i0 = (long long)(blockIdx.x - b.blk0[j]) * 256 + threadIdx.x;
  const long long step = (long long)nb * 256;
  if (t.kind == STX_WPREP_F16)
    weight_prep16_body(t.w, reinterpret_cast<_Float16*>(t.slab), t.w_amax, t.cout, t.cin,
                       t.transpose, b.gin[j], b.gout[j], i0, step);
  else if (t.kind == STX_WPREP_F16UP)
    weight_prep16up_body(t.w, reinterpret_cast<_Float16*>(t.slab), t.w_amax, t.cout, t.cin,
                         b.gin[j] / 16, b.gout[j], i0, step);
  else
    weight_prep32_body(t.w, reinterpret_cast<float*>(t.slab), t.cout, t.cin, t.ks, t.transpose,
                       b.gin[j], b.gout[j], i0, step);
}

// ------------------------------------------------ composed data-gradient weights
// W'[c][k] = s * sum_co A[c*pitch + co] * W[co][k]  (k = ci*9 + tap, K = cin*9): the 1x1
// Gram-backward operator A folded into the next 3x3 conv's weights, so that
//   conv^T_W(A . z) = conv^T_{W'}(z)
// (stx_conv_weight_compose16), written straight into the data-gradient split slab.  The
// split needs a power-of-two scale known before W' exists: the bound
//   max|W'| <= |s| * C * max|A| * max|W|
// (the producers' amax groups) -- a loose scale only moves hi/lo down the fp16 range (both
// keep 11 bits; what a headroom of 2^k costs is the lo floor 2^-24, far below fp32
// rounding of the sums).  Block = 16 rows c x 64 columns k, with A^T and the block's W
// columns staged in LDS (every load in flight at once); wave w sums co in [64w, 64w + 64)
// for all of them (lane: 4 rows x 4 columns), then wave 0 adds the four wave sums in wave
// order (fixed order), splits and stores 8-B runs of the slab.
constexpr int WC_R = 16, WC_K = 64;

__global__ void __launch_bounds__(256)
weight_compose16_kernel(const float* __restrict__ A, int pitch, const float* __restrict__ a_amax,
                        const float* __restrict__ W, const float* __restrict__ w_amax, int C,
                        int cin, const float* __restrict__ scale, _Float16* __restrict__ slab,
                        float* __restrict__ out_amax) {
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  const int K = cin * 9;
  __shared__ __attribute__((aligned(16))) float la[256][WC_R];  // A^T tile (C <= 256)
  // W columns k0 .. k0 + 63; after the sums, the three wave partials (80 KB per block in
  // all: two blocks per CU)
  __shared__ __attribute__((aligned(16))) float lw[256][WC_K];
  float (*red)[WC_R * WC_K] = reinterpret_cast<float (*)[WC_R * WC_K]>(&lw[0][0]);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c0 = blockIdx.y * WC_R, k0 = blockIdx.x * WC_K;
  const float sc = scale ? *scale : 1.f;
  const float bound = fabsf(sc) * (float)C * read_amax(a_amax) * read_amax(w_amax);
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid < STX_AMAX_SLOTS) out_amax[tid] = bound;
  const float sw = __builtin_ldexpf(1.f, 15 - amax_exp(bound));
  {
    // A rows c0 .. c0 + 15 (-> la, transposed) and the block's W columns [C][64] (-> lw):
    // every load issued before the first LDS store (one exposed latency per block);
    // unconditional descriptor loads (rows past C / columns past K read 0)
    constexpr int NLD = 256 * WC_K / 4 / 256;  // W float4 per thread (C <= 256)
    const auto ra = make_srd(A, (uint32_t)C * (uint32_t)pitch * 4u);
    const auto rw = make_srd(W, (uint32_t)C * (uint32_t)K * 4u);
    float av[WC_R];
#pragma unroll
    for (int r = 0; r < WC_R; ++r)
      av[r] = buf_ld(ra, (c0 + r < C && tid < C) ? (uint32_t)((c0 + r) * pitch + tid) * 4u : BUF_OOB);
    f32x4 v[NLD];  // (cin % 4 == 0: a float4 run of a row is all in or all out)
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int f = tid + 256 * u, co = f >> 4, k = k0 + 4 * (f & 15);
      v[u] = buf_ld4(rw, co < C && k < K ? (uint32_t)(co * K + k) * 4u : BUF_OOB);
    }
#pragma unroll
    for (int r = 0; r < WC_R; r += 4)
      *reinterpret_cast<f32x4*>(&la[tid][r]) = f32x4{av[r], av[r + 1], av[r + 2], av[r + 3]};
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int f = tid + 256 * u;
      *reinterpret_cast<f32x4*>(&lw[f >> 4][4 * (f & 15)]) = v[u];
    }
  }
  __syncthreads();
  const int r4 = 4 * (lane >> 4), q4 = 4 * (lane & 15);
  const int kk = k0 + q4;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  const int cb = 64 * wave, ce = min(C, cb + 64);
#pragma unroll 8
  for (int co = cb; co < ce; ++co) {
    const f32x4 a4 = *reinterpret_cast<const f32x4*>(&la[co][r4]);
    const f32x4 w4 = *reinterpret_cast<const f32x4*>(&lw[co][q4]);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(a4[a], w4[b], acc[a][b]);
  }
  __syncthreads();  // every wave's lw reads done (red aliases lw)
  if (wave > 0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) red[wave - 1][(r4 + a) * WC_K + q4 + b] = acc[a][b];
  }
  __syncthreads();
  if (wave != 0) return;
  const int gout64 = rup(cin, 64);
  // slab [ci'/16][tap][P][cg][co' < gout64][8] of the data-gradient GEMM:
  // W_T[co' = ci][ci' = c][tap'] = W'[c][ci][2 - kh][2 - kw]
  const int c = c0 + r4, chunk = c >> 4, cg = (c >> 3) & 1, e0 = c & 7;  // e0 in {0, 4}
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int k = kk + b;
    if (k >= K || c >= C) continue;
    const int ci = k / 9, tap = k - 9 * ci, tapf = 8 - tap;  // (2-kh)*3 + (2-kw)
    f16x4 hi, lo;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int o = (r4 + a) * WC_K + q4 + b;
      const float v = (((acc[a][b] + red[0][o]) + red[1][o]) + red[2][o]) * sc * sw;
      hi[a] = (_Float16)v;
      lo[a] = (_Float16)(v - (float)hi[a]);
    }
    const size_t u0 = ((((size_t)chunk * 9 + tapf) * 2 + 0) * 2 + cg) * gout64 + ci;
    const size_t u1 = ((((size_t)chunk * 9 + tapf) * 2 + 1) * 2 + cg) * gout64 + ci;
    *reinterpret_cast<f16x4*>(slab + u0 * 8 + e0) = hi;
    *reinterpret_cast<f16x4*>(slab + u1 * 8 + e0) = lo;
  }
}

// stx_conv_params.unpool_out (validated by stx_conv2d): 32 x 4 tiles of d, 64 couts
// (K2 -- two chunk groups per block -- when the grid is at most one block per CU and
// the chunk count is even)
static int launch16_unpool(const stx_conv_params& p, hipStream_t st) {
  const int tiles_x = p.wo / 32, ntiles = tiles_x * (p.ho / 4);
  const dim3 grid(ntiles, p.cout / 64, p.n);
  const bool k2 = STX_KNOB("STX_CONV_K2", 1) != 0 && cdiv(p.cin, 16) % 2 == 0 &&
                  (long long)ntiles * (p.cout / 64) * p.n <= cus16();
  if (k2)
    hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<32, STX_IN_RAW, 4, 1, 1, true>), grid, dim3(512),
                       0, st, p, tiles_x, ntiles);
  else
    hipLaunchKernelGGL((conv3x3_f16x3_v2_kernel<32, STX_IN_RAW, 4, 1>), grid, dim3(256), 0, st, p,
                       tiles_x, ntiles);
  return check_launch("stx_conv2d(f16x3 v2 + unpool / Gram-backward epilogue)");
}

int conv2d_f16x3(const stx_conv_params& p, hipStream_t st) {
  if (p.unpool_out) return launch16_unpool(p, st);
  switch (p.stride == 2 ? LM_S2 : p.in_mode) {
    case STX_IN_RAW: return dispatch16_tw<STX_IN_RAW>(p, st);
    case STX_IN_RELU: return dispatch16_tw<STX_IN_RELU>(p, st);
    case STX_IN_RELU_POOL2: return dispatch16_tw<STX_IN_RELU_POOL2>(p, st);
    case STX_IN_UPSAMPLE2:
      if (p.wt16_up) return launch16up(p, st);  // (eligibility: stx_conv2d)
      return dispatch16_tw<STX_IN_UPSAMPLE2>(p, st);
    case LM_S2:  // stride 2 (raw input): 32 x 4 output tiles, two blocks per CU
      if (p.pool_out || p.p2_z) {
        set_error("stx_conv2d: stride 2 takes no fused pool output / Gram phase");
        return STX_E_INVALID;
      }
      return launch16<32, LM_S2, 1>(p, st);
    default: return dispatch16_tw<STX_IN_DILATE2>(p, st);
  }
}

}  // namespace stx

using namespace stx;

extern "C" size_t stx_conv_weight16_bytes(int cin, int cout, int ks, int transpose) {
  if (ks != 3) return 0;
  const int gin = transpose ? cout : cin, gout = transpose ? cin : cout;
  return (size_t)rup(gin, 16) * 9 * 2 * rup(gout, 64) * sizeof(_Float16);
}

extern "C" int stx_amax(const float* x, long long n, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!out || n < 0 || (n > 0 && !x)) {
    set_error("stx_amax: invalid arguments");
    return STX_E_INVALID;
  }
  if (reinterpret_cast<uintptr_t>(x) & 15) {
    set_error("stx_amax: x must be 16-byte aligned");
    return STX_E_INVALID;
  }
  if (n <= (8ll << 20)) {  // up to 32 MB: one launch, every slot written (no clearing)
    hipLaunchKernelGGL(amax_slots_kernel, dim3(STX_AMAX_SLOTS), dim3(1024), 0, st, x, n, out);
    return check_launch("stx_amax");
  }
  // the slots are cleared by a kernel, not hipMemsetAsync: a memset node captured into a
  // hipGraph was observed to run out of order with the amax kernel on replay
  hipLaunchKernelGGL(amax_zero_kernel, dim3(1), dim3(STX_AMAX_SLOTS), 0, st, out);
  if (n == 0) return check_launch("stx_amax");
  const int blocks = (int)std::min<long long>(std::max<long long>(1, (n / 4 + 255) / 256), 512);
  hipLaunchKernelGGL(amax_kernel, dim3(blocks), dim3(256), 0, st, x, n, out);
  return check_launch("stx_amax");
}

extern "C" size_t stx_conv_weight16up_bytes(int cin, int cout) {
  if (cin <= 0 || cout <= 0) return 0;
  return (size_t)2 * rup(cin, 16) * 2 * 4 * 2 * rup(cout, 64) * sizeof(_Float16);
}

extern "C" int stx_conv_weight_prep16_up(const float* w, void* wt16_up, float* w_amax, int cout,
                                         int cin, void* stream) {
  if (!w || !wt16_up || !w_amax || cout <= 0 || cin <= 0) {
    set_error("stx_conv_weight_prep16_up: pointers non-NULL, cout / cin > 0");
    return STX_E_INVALID;
  }
  int rc = stx_amax(w, (long long)cout * cin * 9, w_amax, stream);
  if (rc) return rc;
  const long long total = (long long)rup(cin, 16) * 32 * rup(cout, 64);
  if (total >= (1ll << 31)) {
    set_error("stx_conv_weight_prep16_up: slab too large");
    return STX_E_INVALID;
  }
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(weight_prep16up_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<_Float16*>(wt16_up), w_amax, cout, cin, rup(cin, 16) / 16,
                     rup(cout, 64));
  return check_launch("stx_conv_weight_prep16_up");
}

extern "C" int stx_conv_weight_prep16_pair(const float* w, void* wt16, void* wtT16, float* w_amax,
                                           int cout, int cin, int ks, void* stream) {
  if (ks != 3 || !w || !wt16 || !wtT16 || !w_amax || cout <= 0 || cin <= 0) {
    set_error("stx_conv_weight_prep16_pair: ks must be 3 and pointers non-NULL");
    return STX_E_INVALID;
  }
  int rc = stx_amax(w, (long long)cout * cin * 9, w_amax, stream);
  if (rc) return rc;
  const long long total = std::max((long long)rup(cin, 16) * rup(cout, 64),
                                   (long long)rup(cout, 16) * rup(cin, 64)) * 9 * 2;
  if (total >= (1ll << 31)) {
    set_error("stx_conv_weight_prep16_pair: slab too large");
    return STX_E_INVALID;
  }
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(weight_prep16_pair_kernel, dim3(blocks, 2), dim3(256), 0,
                     (hipStream_t)stream, w, reinterpret_cast<_Float16*>(wt16),
                     reinterpret_cast<_Float16*>(wtT16), w_amax, cout, cin);
  return check_launch("stx_conv_weight_prep16_pair");
}

extern "C" int stx_conv_weight_prep_batch(const stx_wprep_job* jobs, int njobs, void* stream) {
  if (!jobs || njobs <= 0 || njobs > STX_WPREP_MAX) {
    set_error("stx_conv_weight_prep_batch: 1 <= njobs <= %d required", STX_WPREP_MAX);
    return STX_E_INVALID;
  }
  WprepAmax a{};
  WprepJobs b{};
  int na = 0, blocks = 0;
  b.njobs = njobs;
  for (int j = 0; j < njobs; ++j) {
    const stx_wprep_job& t = jobs[j];
    if (!t.w || !t.slab || t.cout <= 0 || t.cin <= 0 ||
        (t.kind != STX_WPREP_F32 && t.kind != STX_WPREP_F16 && t.kind != STX_WPREP_F16UP) ||
        (t.kind != STX_WPREP_F32 && (t.ks != 3 || !t.w_amax)) ||
        (t.kind == STX_WPREP_F16UP && t.transpose)) {
      set_error("stx_conv_weight_prep_batch: job %d invalid", j);
      return STX_E_INVALID;
    }
    const int gin = t.transpose ? t.cout : t.cin, gout = t.transpose ? t.cin : t.cout;
    long long total;
    if (t.kind != STX_WPREP_F32) {
      if (reinterpret_cast<uintptr_t>(t.w) & 15) {
        set_error("stx_conv_weight_prep_batch: job %d weight not 16-byte aligned", j);
        return STX_E_INVALID;
      }
      b.gin[j] = rup(gin, 16);
      b.gout[j] = rup(gout, 64);
      total = (long long)b.gin[j] * (t.kind == STX_WPREP_F16UP ? 32 : 18) * b.gout[j];
      bool seen = false;  // the forward / data-gradient slabs of a weight share one group
      for (int k = 0; k < na; ++k) {
        if (a.out[k] == t.w_amax) {
          if (a.w[k] != t.w) {
            set_error("stx_conv_weight_prep_batch: w_amax shared by two weights");
            return STX_E_INVALID;
          }
          seen = true;
        }
      }
      if (!seen) {
        a.w[na] = t.w;
        a.out[na] = t.w_amax;
        a.n[na] = (long long)t.cout * t.cin * 9;
        ++na;
      }
    } else {
      int rp, cp;
      int rc = stx_conv_weight_dims(gin, gout, t.ks, &rp, &cp);
      if (rc) return rc;
      b.gin[j] = rp * t.ks * t.ks;
      b.gout[j] = cp;
      total = (long long)b.gin[j] * cp;
    }
    if (total >= (1ll << 31)) {
      set_error("stx_conv_weight_prep_batch: job %d slab too large", j);
      return STX_E_INVALID;
    }
    b.job[j] = t;
    b.blk0[j] = blocks;
    // ~16 elements per thread: the per-thread setup (job lookup, the 32-slot max|w|
    // read) costs as much as a handful of elements
    blocks += (int)std::min<long long>((total + 4095) / 4096, 256);
  }
  b.blk0[njobs] = blocks;
  hipStream_t st = (hipStream_t)stream;
  if (na > 0)
    hipLaunchKernelGGL(amax_batch_kernel, dim3(na * STX_AMAX_SLOTS), dim3(1024), 0, st, a);
  hipLaunchKernelGGL(weight_prep_batch_kernel, dim3(blocks), dim3(256), 0, st, b);
  return check_launch("stx_conv_weight_prep_batch");
}

extern "C" int stx_conv_weight_compose16(const float* A, int pitch, const float* a_amax,
                                         const float* w, const float* w_amax, int cout, int cin,
                                         const float* scale, void* wtT16, float* out_amax,
                                         void* stream) {
  if (!A || !a_amax || !w || !w_amax || !wtT16 || !out_amax || cout <= 0 || cout > 256 ||
      cin <= 0 || cin % 4 || pitch < cout || (reinterpret_cast<uintptr_t>(w) & 15)) {
    set_error("stx_conv_weight_compose16: invalid arguments (1 <= cout <= 256, cin % 4 == 0, "
              "w 16-byte aligned)");
    return STX_E_INVALID;
  }
  const long long total = (long long)rup(cout, 16) * 9 * 2 * rup(cin, 64);
  if ((long long)cout * cin * 9 >= (1ll << 31) || total >= (1ll << 31)) {
    set_error("stx_conv_weight_compose16: weight too large");
    return STX_E_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  // slab padding (channels past cout / cin) must read as zero: cleared first when present
  if (cout % 16 || cin % 64)
    (void)hipMemsetAsync(wtT16, 0, (size_t)total * sizeof(_Float16), st);
  hipLaunchKernelGGL(weight_compose16_kernel, dim3(cdiv(cin * 9, WC_K), cdiv(cout, WC_R)), dim3(256),
                     0, st, A, pitch, a_amax, w, w_amax, cout, cin, scale,
                     reinterpret_cast<_Float16*>(wtT16), out_amax);
  return check_launch("stx_conv_weight_compose16");
}

extern "C" int stx_conv_weight_prep16(const float* w, void* wt16, float* w_amax, int cout, int cin,
                                      int ks, int transpose, void* stream) {
  if (ks != 3 || !w || !wt16 || !w_amax || cout <= 0 || cin <= 0) {
    set_error("stx_conv_weight_prep16: ks must be 3 and pointers non-NULL");
    return STX_E_INVALID;
  }
  int rc = stx_amax(w, (long long)cout * cin * 9, w_amax, stream);
  if (rc) return rc;
  const int gin = transpose ? cout : cin, gout = transpose ? cin : cout;
  const int gin16 = rup(gin, 16), gout64 = rup(gout, 64);
  const long long total = (long long)gin16 * 9 * 2 * gout64;
  if (total >= (1ll << 31)) {
    set_error("stx_conv_weight_prep16: slab too large");
    return STX_E_INVALID;
  }
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(weight_prep16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<_Float16*>(wt16), w_amax, cout, cin, transpose, gin16,
                     gout64);
  return check_launch("stx_conv_weight_prep16");
}
