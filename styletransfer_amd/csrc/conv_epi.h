// Fused epilogue shared by the implicit-GEMM conv kernels (conv.hip: fp32 MFMA,
// conv16.hip: fp16 hi/lo split MFMA).  Both keep the same accumulator tiling:
// 4 waves in a WM x WN grid, each wave 2 x 2 tiles of 32x32 (MI = NI = 2), so
//   output channel  co  = co0 + wm*64 + i*32 + (r & 3) + 8*(r >> 2) + 4*h
//   output pixel    pix = (wn*2 + j)*32 + l32   of the block's TH x TW tile
// for accumulator register r of tile (i, j) in lane (h = lane>>5, l32 = lane&31)
// (the C/D layout of every 32x32 MFMA on gfx950).
//
// Order of operations (stx_conv_params, include/stx.h):
//   v = acc * pre_scale                      (fp16-split de-scaling; 1 for fp32)
//   v *= *acc_scale; v *= (mask > 0)          (data-gradient ReLU mask)
//   v += s2 * A[n] . p2_z                     (fused Gram-backward phase, 1x1 fp32 MFMA)
//   v += bias; v += unpool(up_dp)*(up_z>0); v += aux_scale*aux; v += y; relu
//   y = v;  *out_amax = max(*out_amax, |v|)  (next fp16-split conv's input scale)
#pragma once
#include "common.h"
#include "../../include/stx.h"

namespace stx {

struct EpiTile {
  int n, co0, ty0, tx0, wm, wn, h, l32;
  int tile = -1, ntiles = 0;  // persistent kernels: the tile (blockIdx.x otherwise)
};

// (ty, tx) inside the block tile of the pixel lane l32 of wave column wn holds in
// N-tile j.  Default: the wave's two tiles are consecutive runs of 32 pixels in
// row-major tile order.  ROWPAIR (TW == 64): wave column wn covers x in
// [32*(wn&1), +32) of rows 2*(wn>>1) + {0, 1}, so every 2x2 pooling window lies in
// one wave (tiles j = 0/1 x lanes l32, l32^1) -- the fused ReLU+MaxPool output.
// PAR (TW == 64, NI == 2: the zero-dilated data gradient): wave column wn owns tile row
// wn, N-tile j the pixels of column parity j (x = 2 l32 + j) -- every N-tile is one output
// parity class, so the taps that only meet dilation zeros are skipped per N-tile
template <int TW, bool ROWPAIR, int NI = 2, bool PAR = false>
__device__ __forceinline__ void tile_pix(int wn, int j, int l32, int& ty, int& tx) {
  if (PAR) {
    static_assert(!PAR || (TW == 64 && NI == 2), "parity mapping needs 64 x 4 tiles");
    tx = 2 * l32 + j;
    ty = wn;
  } else if (ROWPAIR) {
    static_assert(!ROWPAIR || TW == 64, "row-pair mapping needs TW == 64");
    tx = (wn & 1) * 32 + l32;
    ty = (wn >> 1) * 2 + j;
  } else {
    const int pix = (wn * NI + j) * 32 + l32;
    ty = pix / TW;
    tx = pix - ty * TW;
  }
}

__device__ __forceinline__ void atomic_max_abs(float* slot, float m) {
  // |v| >= 0: the IEEE bit pattern orders like the value (NaN sorts above inf)
  atomicMax(reinterpret_cast<unsigned int*>(slot), __float_as_uint(m));
}

// max over the 256-thread block (NaN wins), then ONE device atomic per block into
// one of the group's STX_AMAX_SLOTS slots: same-address atomics serialise at
// ~12-15 ns each chip-wide (8192 of them stalled a 64 MB pass for 100 us; 1024 at a
// conv's tail cost ~15 us)
// nwaves: the waves taking part (0: the whole block; a K2 block's epilogue runs on 4)
__device__ __forceinline__ void block_max_to(float* group, float m, int nwaves = 0) {
  __shared__ float red[16];  // up to 1024-thread blocks
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float other = __shfl_xor(m, o, 64);
    m = (other != other) ? other : fmaxf(m, other);
  }
  const int tid = threadIdx.x;
  if ((tid & 63) == 0) red[tid >> 6] = m;
  lds_sync();  // (not a __syncthreads: the caller's output stores need not drain first)
  if (tid == 0) {
    float r = red[0];
    const int nw = nwaves > 0 ? nwaves : (int)(blockDim.x >> 6);
    for (int i = 1; i < nw; ++i) r = (red[i] != red[i]) ? red[i] : fmaxf(r, red[i]);
    const int bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    atomic_max_abs(group + (bid & (STX_AMAX_SLOTS - 1)), fabsf(r));
  }
}

// The forward-conv epilogue (no mask, aux, accumulate, acc_scale, unpool or Gram
// phase -- every VGG / ITN forward launch): v = acc * scale + bias [, relu]; y = v;
// optional fused ReLU + MaxPool2d output; optional out_amax.  Specialised because the
// generic epilogue's per-element feature tests and the pooled output's 64-bit
// address arithmetic cost more VALU issue per wave than the main loop's staging
// (PMC, conv1_2 fwd @ 512^2: ~3,400 VALU instructions per wave for 432 MFMAs).
// All stores go through buffer descriptors: a per-lane pixel offset plus a per-
// register row constant, rows past cout / pixels past the image dropped by the
// hardware range check.
// ---- fused Gram partials (stx_conv_params.gram_part) --------------------------------
// A producing conv's 64-channel output tile is split ONCE into fp16 hi/lo planes in LDS,
// [plane][channel][pixel] with a pitch of NPX + 8 halves (the 16-B operand reads of 16
// lanes land on distinct banks; a store's two lane halves on disjoint banks), at the
// tile's own power-of-two scale s = 2^(15 - e), max|y| < 2^e.  Waves 0..2 then each
// take one 32 x 32 block of the upper triangle of G = Z Z^T (3 MFMAs per 16 pixels),
// de-scaled by 2^(2e - 30) (exact); the lower block is the mirror of the upper one.
template <int NPX>
struct GramPlanes {
  static constexpr int HP = NPX + 8;                 // pitch (halves)
  static constexpr int BYTES = 2 * 64 * HP * 2 + 16;  // hi + lo planes, 4 floats of max
};

// block max over NW waves (IEEE bits of |y|) -> the scale exponent e (barrier inside)
template <int NW = 4>
__device__ __forceinline__ int gram_block_exp(uint32_t m, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(m);
  lds_sync();  // (the epilogue's y stores stay in flight)
  uint32_t bm = 0u;
#pragma unroll
  for (int w = 0; w < NW; ++w) bm = max(bm, __float_as_uint(red[w]));
  int e = 0;
  frexpf(__uint_as_float(bm), &e);
  return min(max(e, -60), 60);
}

// scaled value v of (channel, pixel) -> the hi and lo planes
__device__ __forceinline__ void gram_put(_Float16* H, int hp, int ch, int px, float v) {
  const _Float16 hi = (_Float16)v;
  H[ch * hp + px] = hi;
  H[(64 + ch) * hp + px] = (_Float16)(v - (float)hi);
}

// g += this wave's upper-triangle block over KS x 16 pixels (waves 0..2)
template <int KS>
__device__ __forceinline__ void gram_mma(const _Float16* H, int hp, int wave, int h, int l32,
                                         f32x16& g) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  const int I = wave == 2 ? 1 : 0, J = wave == 0 ? 0 : 1;
  const _Float16* ra = H + (I * 32 + l32) * hp + 8 * h;
  const _Float16* rb = H + (J * 32 + l32) * hp + 8 * h;
  const int lo = 64 * hp;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const h8 ah = *reinterpret_cast<const h8*>(ra + ks * 16);
    const h8 al = *reinterpret_cast<const h8*>(ra + lo + ks * 16);
    h8 bh = ah, bl = al;
    if (I != J) {
      bh = *reinterpret_cast<const h8*>(rb + ks * 16);
      bl = *reinterpret_cast<const h8*>(rb + lo + ks * 16);
    }
    g = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, g, 0, 0, 0);
    g = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, g, 0, 0, 0);
  }
}

// the 64 x 64 partial of this block (waves 0..2 hold the three upper blocks)
__device__ __forceinline__ void gram_store(float* out, const f32x16& g, int wave, int h,
                                           int l32) {
  const int I = wave == 2 ? 1 : 0, J = wave == 0 ? 0 : 1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    out[(I * 32 + row) * 64 + J * 32 + l32] = g[r];
    if (I != J) out[(J * 32 + l32) * 64 + I * 32 + row] = g[r];
  }
}

// gram_store through LDS: waves 0..2's blocks (and the mirror of (0,1)) into O (>= 64 x 68
// floats of LDS no wave reads any more once every wave is past the first barrier), then
// coalesced 16-B stores by all NT threads -- the scattered 4-B stores (the mirrored block
// a column per lane) cost ~20 us per 1024-block launch (measurement build)
template <int NT>
__device__ __forceinline__ void gram_store_lds(float* out, const f32x16& g, int wave, int h,
                                               int l32, float* O) {
  constexpr int OP = 68;
  lds_sync();
  if (wave < 3) {
    const int I = wave == 2 ? 1 : 0, J = wave == 0 ? 0 : 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      O[(I * 32 + row) * OP + J * 32 + l32] = g[r];
      if (I != J) O[(J * 32 + l32) * OP + I * 32 + row] = g[r];
    }
  }
  lds_sync();
  const auto rg = make_srd(out, 16384u);
#pragma unroll
  for (int k = 0; k < 1024 / NT; ++k) {  // 64 rows x 16 float4
    const int idx = threadIdx.x + NT * k, row = idx >> 4, c4 = idx & 15;
    const f32x4 v = *reinterpret_cast<const f32x4*>(O + row * OP + 4 * c4);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rg,
                                           (uint32_t)(row * 64 + 4 * c4) * 4u, 0, 0);
  }
}

// Grouped partials (stx_conv_params.gram_cnt): the in-launch fixed-order reduction of
// STX_GRAM_GROUP consecutive tiles' partials, so the loss finalize reads one 16 KB sum
// per group instead of one partial per tile.  Called by all four waves (waves 0..2 hold
// the blocks (0,0), (0,1), (1,1) in g).  Hand-off (cdna_hip_programming.md §6 G16, the
// sc1 form): each wave stores its block TRANSPOSED with 16-B write-through (sc1) stores --
// (0,0) and (1,1) are symmetric blocks, and (0,1) lands as its mirror (1,0), so no
// 4-byte stores -- drains them (vmcnt(0)), the block barrier, then one lane's relaxed
// agent-scope ticket add; the block that draws the group's last ticket resets the
// counter and reads the group's partials with sc1 loads (no acquire fence: every load of
// the handed-off bytes is sc1), sums them in tile order and writes the group sum
// (plain stores: read by the next launch), mirroring (1,0) into (0,1).
typedef __attribute__((address_space(1))) unsigned int gu32_t;

__device__ __forceinline__ void gram_store_grouped(const stx_conv_params& p, int n, int tix,
                                                   int ntl, const f32x16& g, int wave, int h,
                                                   int l32, float* flag) {
  constexpr int G = STX_GRAM_GROUP;
  const int grp = tix / G, g0 = grp * G, gs = min(G, ntl - g0), ng = cdiv(ntl, G);
  const auto rs = make_srd(p.gram_part + (size_t)n * ntl * 4096, (uint32_t)ntl * 16384u);
  if (wave < 3) {
    const int I = wave == 2 ? 1 : 0, J = wave == 0 ? 0 : 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = {g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]};
      const uint32_t off =
          (uint32_t)((tix * 64 + J * 32 + l32) * 64 + I * 32 + 8 * q + 4 * h) * 4u;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, off, 0, 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    gu32_t* cnt = (gu32_t*)(p.gram_cnt + (size_t)n * ng + grp);
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = t == (unsigned)(gs - 1);
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last ? 1.f : 0.f;
  }
  __syncthreads();
  if (*flag == 0.f) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float* gsum = p.gram_part + ((size_t)p.n * ntl + (size_t)n * ng + grp) * 4096;
#pragma unroll
  for (int k = 0; k < 3; ++k) {  // stored blocks (0,0), (1,0), (1,1): 256 float4 each
    const int f = threadIdx.x, rr = f >> 3, c4 = f & 7;
    const int row = (k == 0 ? 0 : 32) + rr, col = (k == 2 ? 32 : 0) + 4 * c4;
    f32x4 v[G];
#pragma unroll
    for (int m = 0; m < G; ++m) {
      const uint32_t off = (uint32_t)(((g0 + min(m, gs - 1)) * 64 + row) * 64 + col) * 4u;
      v[m] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
    }
    f32x4 s = v[0];
#pragma unroll
    for (int m = 1; m < G; ++m)
      if (m < gs) s += v[m];
    *reinterpret_cast<f32x4*>(gsum + row * 64 + col) = s;
    if (k == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) gsum[(col + e) * 64 + row] = s[e];
    }
  }
}

// conv16's 64 x 256 tile: acc holds y; lane_ok[j] marks pixels inside the image
template <int NI>
__device__ __forceinline__ void conv_gram_tile(const f32x16 (&acc)[2][NI],
                                               const stx_conv_params& p, const EpiTile& t,
                                               const bool (&lane_ok)[NI], uint32_t vmax_u,
                                               char* smem) {
  static_assert(NI == 2, "256-pixel tiles");
  using GP = GramPlanes<256>;
  _Float16* H = reinterpret_cast<_Float16*>(smem);
  float* red = reinterpret_cast<float*>(smem + GP::BYTES - 16);
  const int wave = threadIdx.x >> 6, h = t.h, l32 = t.l32;
#ifdef STX_AB  // stage cut-off for timing (aux_scale = 1..3; aux is unused with gram_part)
  const int dbg = (int)p.aux_scale;
  if (dbg == 4) return;
#else
  constexpr int dbg = 0;
#endif
  const int e = gram_block_exp(vmax_u, red);
  if (dbg == 1) return;
  const float sx = __builtin_ldexpf(1.f, 15 - e);
  // two neighbouring pixels per 4-B LDS store: for the registers (r, r+1) (channels ch,
  // ch+1) the lane pair (px even, px+1) swaps one value by DPP, then the even lane holds
  // channel ch at (px, px+1) and the odd lane channel ch+1 at (px-1, px) -- half the
  // ds_write instructions of one fp16 per store
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  const int q = l32 & 1;
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float va = lane_ok[j] ? acc[i][j][r] * sx : 0.f;
        const float vb = lane_ok[j] ? acc[i][j][r + 1] * sx : 0.f;
        const float recv = __int_as_float(
            __builtin_amdgcn_mov_dpp(__float_as_int(q ? va : vb), 0xB1, 0xF, 0xF, false));
        const float v0 = q ? recv : va, v1 = q ? vb : recv;
        const int ch = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h + q;
        const int p0 = wave * 64 + j * 32 + l32 - q;
        f16x2 hi, lo;
        hi[0] = (_Float16)v0;
        hi[1] = (_Float16)v1;
        lo[0] = (_Float16)(v0 - (float)hi[0]);
        lo[1] = (_Float16)(v1 - (float)hi[1]);
        *reinterpret_cast<f16x2*>(H + ch * GP::HP + p0) = hi;
        *reinterpret_cast<f16x2*>(H + (64 + ch) * GP::HP + p0) = lo;
      }
  lds_sync();
  if (dbg == 2) return;
  f32x16 g;
#pragma unroll
  for (int q = 0; q < 16; ++q) g[q] = 0.f;
  if (wave < 3) {
    gram_mma<16>(H, GP::HP, wave, h, l32, g);
    const float inv2 = __builtin_ldexpf(1.f, 2 * e - 30);
#pragma unroll
    for (int q = 0; q < 16; ++q) g[q] *= inv2;
  }
  const int tix = t.tile >= 0 ? t.tile : (int)blockIdx.x;
  const int ntl = t.tile >= 0 ? t.ntiles : (int)gridDim.x;
  if (dbg == 3) {
    if (g[0] == 12345.f) p.gram_part[0] = g[1];  // (keeps the MFMAs)
    return;
  }
  if (p.gram_cnt) {  // (red's block maxima were read before the barrier above)
    gram_store_grouped(p, blockIdx.z, tix, ntl, g, wave, h, l32, red);
    return;
  }
  gram_store_lds<256>(p.gram_part + ((size_t)blockIdx.z * ntl + tix) * 4096, g, wave, h, l32,
                      reinterpret_cast<float*>(smem));
}

// The 128-channel taps (VGG conv2_1 / conv2_2): an 8-wave (WM = 2) block holds all 128
// channels of its 256-pixel tile, so the whole C x C partial of the tile comes out of the
// epilogue (the standalone triangle kernel's re-read of y is gone).  Same split as the
// 64-channel tile (block-local power-of-two scale, fp16 hi/lo planes [plane][channel]
// [pixel], 3 MFMAs per 16 pixels); the 10 upper-triangle 32 x 32 blocks go to waves
// 0..7 (waves 0 and 1 take blocks 8 and 9 too) and are stored in the 64 x 64-tile layout
// of the triangle kernel: gram_part + ((n * 3 + u) * T + t) * 4096, u the tile (0,0),
// (0,1), (1,1), diagonal tiles with the mirrored lower-left quadrant.
// MSE (p.mse_ref, the content target at conv2_2): also the block's sums of (y - ref)^2
// and (relu y - relu ref)^2 over its valid outputs -> mse_parts[2 (n T + t) + 0/1] (the
// content / feature losses' pass over y, stransfer/network.py:134-201).
struct GramPlanes128 {
  static constexpr int HP = 256 + 8;                   // pitch (halves)
  static constexpr int BYTES = 2 * 128 * HP * 2 + 128;  // hi + lo planes, 32 floats of sums
};

template <int TW, bool ROWPAIR>
__device__ __forceinline__ void conv_gram_tile128(const f32x16 (&acc)[2][2],
                                                  const stx_conv_params& p, const EpiTile& t,
                                                  const bool (&lane_ok)[2],
                                                  const uint32_t (&vo)[2], uint32_t vmax_u,
                                                  char* smem) {
  using GP = GramPlanes128;
  constexpr int HP = GP::HP;
  _Float16* H = reinterpret_cast<_Float16*>(smem);
  float* red = reinterpret_cast<float*>(smem + GP::BYTES - 128);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = t.h, l32 = t.l32;
  const int tix = t.tile >= 0 ? t.tile : (int)blockIdx.x;
  const int ntl = t.tile >= 0 ? t.ntiles : (int)gridDim.x;
  // the content target's values at this lane's outputs, in flight during the staging
#ifdef STX_AB  // stage cut-off for timing (aux_scale = 1..4; aux is unused with gram_part)
  const int dbg = (int)p.aux_scale;
  if (dbg == 4) return;
#else
  constexpr int dbg = 0;
#endif
  const bool mse = p.mse_ref != nullptr;
  float rf[2][2][16];
  if (mse) {
    const size_t plane = (size_t)p.ho * p.wo;
    const uint32_t pb = (uint32_t)plane * 4u;
    const int co_w = t.co0 + t.wm * 64;
    const auto rr = make_srd(p.mse_ref + ((size_t)t.n * p.cout + co_w) * plane,
                             (uint32_t)max(0, p.cout - co_w) * pb);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rf[j][i][r] = buf_ld(rr, vo[j] + (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * pb);
  }
  const int e = gram_block_exp<8>(vmax_u, red);
  if (dbg == 1) return;
  const float sx = __builtin_ldexpf(1.f, 15 - e);
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  const int q = l32 & 1;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float va = lane_ok[j] ? acc[i][j][r] * sx : 0.f;
        const float vb = lane_ok[j] ? acc[i][j][r + 1] * sx : 0.f;
        const float recv = __int_as_float(
            __builtin_amdgcn_mov_dpp(__float_as_int(q ? va : vb), 0xB1, 0xF, 0xF, false));
        const float v0 = q ? recv : va, v1 = q ? vb : recv;
        const int ch = t.wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h + q;
        const int p0 = t.wn * 64 + j * 32 + l32 - q;  // any pixel order: a sum over pixels
        f16x2 hi, lo;
        hi[0] = (_Float16)v0;
        hi[1] = (_Float16)v1;
        lo[0] = (_Float16)(v0 - (float)hi[0]);
        lo[1] = (_Float16)(v1 - (float)hi[1]);
        *reinterpret_cast<f16x2*>(H + ch * HP + p0) = hi;
        *reinterpret_cast<f16x2*>(H + (128 + ch) * HP + p0) = lo;
      }
  if (mse) {
    float ms = 0.f, msr = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = acc[i][j][r], c = rf[j][i][r];
          const float d = lane_ok[j] ? v - c : 0.f;
          const float dr = lane_ok[j] ? fmaxf(v, 0.f) - fmaxf(c, 0.f) : 0.f;
          ms += d * d;
          msr += dr * dr;
        }
    // fixed-order block sums (the red slots were last read before the staging)
    ms = wave_sum(ms);
    msr = wave_sum(msr);
    if ((threadIdx.x & 63) == 0) {
      red[8 + wave] = ms;  // (slots 0..7: the block max, possibly still being read)
      red[16 + wave] = msr;
    }
    lds_sync();  // (also: the planes are complete)
    if (threadIdx.x == 0) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s0 += red[8 + w];
        s1 += red[16 + w];
      }
      float* mp = p.mse_parts + 2 * ((size_t)blockIdx.z * ntl + tix);
      mp[0] = s0;
      mp[1] = s1;
    }
  } else {
    lds_sync();
  }
  if (dbg == 2) return;
  const float inv2 = __builtin_ldexpf(1.f, 2 * e - 30);
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  constexpr int LO = 128 * HP;
  // the upper-triangle blocks b = wave (and 8 + wave for waves 0, 1), row-major over the
  // 4 x 4 block grid
  f32x16 g[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int b = wave + 8 * q;
    if (b >= 10) break;
    const int bi = b < 4 ? 0 : b < 7 ? 1 : b < 9 ? 2 : 3;
    const int bj = bi + b - (bi == 0 ? 0 : bi == 1 ? 4 : bi == 2 ? 7 : 9);
    const _Float16* ra = H + (bi * 32 + l32) * HP + 8 * h;
    const _Float16* rb = H + (bj * 32 + l32) * HP + 8 * h;
#pragma unroll
    for (int k = 0; k < 16; ++k) g[q][k] = 0.f;
#pragma unroll 4
    for (int ks = 0; ks < 16; ++ks) {
      const h8 ah = *reinterpret_cast<const h8*>(ra + ks * 16);
      const h8 al = *reinterpret_cast<const h8*>(ra + LO + ks * 16);
      const h8 bh = *reinterpret_cast<const h8*>(rb + ks * 16);
      const h8 bl = *reinterpret_cast<const h8*>(rb + LO + ks * 16);
      g[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, g[q], 0, 0, 0);
      g[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, g[q], 0, 0, 0);
      g[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, g[q], 0, 0, 0);
    }
  }
  if (dbg == 3) {
    if (g[0][0] == 12345.f) p.gram_part[0] = g[0][1] + g[1][1];  // (keeps the MFMAs)
    return;
  }
  lds_sync();  // every wave's plane reads are done: the planes become the output tiles
  // the three 64 x 64 tiles in LDS (pitch 68 floats: the mirrored column writes of a wave
  // spread over 16 banks), then streamed out with coalesced 16-B stores
  constexpr int OP = 68;
  float* O = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int b = wave + 8 * q;
    if (b >= 10) break;
    const int bi = b < 4 ? 0 : b < 7 ? 1 : b < 9 ? 2 : 3;
    const int bj = bi + b - (bi == 0 ? 0 : bi == 1 ? 4 : bi == 2 ? 7 : 9);
    const int I = bi >> 1, J = bj >> 1, qi = bi & 1, qj = bj & 1;
    float* T = O + (I == 0 ? J : 2) * 64 * OP;  // tile_index(I, J, 2)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = g[q][r] * inv2;
      T[(qi * 32 + row) * OP + qj * 32 + l32] = v;
      if (I == J && qi != qj) T[(qj * 32 + l32) * OP + qi * 32 + row] = v;  // mirror
    }
  }
  lds_sync();
  const auto rg = make_srd(p.gram_part + (size_t)blockIdx.z * 3 * ntl * 4096,
                           (uint32_t)(3 * ntl) * 16384u);
#pragma unroll
  for (int k = 0; k < 6; ++k) {  // 3 tiles x 64 rows x 16 float4 over 512 threads
    const int idx = threadIdx.x + 512 * k;
    const int u = idx >> 10, row = (idx >> 4) & 63, c4 = idx & 15;
    const f32x4 v = *reinterpret_cast<const f32x4*>(O + (u * 64 + row) * OP + 4 * c4);
    const uint32_t off = (uint32_t)(((u * ntl + tix) * 64 + row) * 64 + 4 * c4) * 4u;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rg, off, 0, 0);
  }
}

// AUX: value += aux_scale * aux (a residual block's skip gradient, ResLink), loaded
// through a descriptor at the store offsets
// POOLSUM: pool_out = 2x2 sum of the output and no y stores (stx_conv_params.pool_sum)
template <int TW, int NI, bool ROWPAIR, bool RELU, bool AUX = false,
          bool POOLSUM = false, bool PAR = false, int WM = 1>
__device__ __forceinline__ void conv_epilogue_plain_body(f32x16 (&acc)[2][NI],
                                                         const stx_conv_params& p,
                                                         const EpiTile& t, float scale,
                                                         char* smem) {
  const size_t plane = (size_t)p.ho * p.wo;
  const int h = t.h, l32 = t.l32;
  const int co_w = t.co0 + t.wm * 64;
  const int rows = max(0, p.cout - co_w);
  const uint32_t pb = (uint32_t)plane * 4u;
  // (y = NULL: pool_out only -- a zero-size descriptor drops every full-resolution store)
  const auto ry = make_srd(p.y ? p.y + ((size_t)t.n * p.cout + co_w) * plane : p.pool_out,
                           p.y ? (uint32_t)rows * pb : 0u);
  const auto raux = make_srd(AUX ? p.aux + ((size_t)t.n * p.cout + co_w) * plane : p.y,
                             AUX ? (uint32_t)rows * pb : 0u);
  uint32_t vo[NI];
  bool lane_ok[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    int ty, tx;
    tile_pix<TW, ROWPAIR, NI, PAR>(t.wn, j, l32, ty, tx);
    const int oy = t.ty0 + ty, ox = t.tx0 + tx;
    lane_ok[j] = oy < p.ho && ox < p.wo;
    vo[j] = lane_ok[j] ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
  }
  // biases of this lane's rows: branch-free descriptor loads (rows past cout read 0)
  float bias_r[2][16];
  {
    const auto rbias = make_srd(p.bias ? p.bias + co_w : p.y, p.bias ? (uint32_t)rows * 4u : 0u);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        bias_r[i][r] = buf_ld(rbias, (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 4u);
  }
  // max|v| over the valid outputs: a per-lane mask (pixel inside the image) ANDed
  // into the IEEE bits; rows past cout exist only in a ragged last 64-row tile, where
  // a per-row mask is added
  // the skip gradient of every element first: a load issued after one of this loop's
  // stores waits for that store (vmcnt counts both), which serialised the loop into 32 / 64
  // load -> store round trips
  float auxv[AUX ? NI : 1][2][16];
  if constexpr (AUX) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          auxv[j][i][r] = buf_ld(raux, vo[j] + (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * pb);
  }
  const bool rows_full = rows >= 64;
  // (a tile with cout <= 32 in it -- the ITN's 32-channel layers: its second 32-row MFMA
  // tile holds only padding, whose stores fall outside the descriptor anyway)
  const bool half = rows <= 32;
  uint32_t lmask[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) lmask[j] = lane_ok[j] ? 0x7fffffffu : 0u;
  uint32_t vmax_u = 0u;  // max |v| as IEEE bits: NaN (above inf) propagates
#pragma unroll
  for (int j = 0; j < NI; ++j) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && half && !ROWPAIR) break;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i * 32 + (r & 3) + 8 * (r >> 2);
        float v = fmaf(acc[i][j][r], scale, bias_r[i][r]);
        if (AUX) v += p.aux_scale * auxv[j][i][r];
        if (RELU) v = fmaxf(v, 0.f);
        if constexpr (!POOLSUM && !PAR) buf_st(ry, vo[j] + (uint32_t)row * pb, v);
        acc[i][j][r] = v;  // kept for the fused pooled output (PAR: for the paired stores)
        uint32_t m = lmask[j];
        if (!rows_full) m = (row + 4 * h < rows) ? m : 0u;
        vmax_u = max(vmax_u, __float_as_uint(v) & m);
      }
    }
  }
  if constexpr (PAR) {
    // the lane's two N-tiles are the neighbouring pixels 2 l32 and 2 l32 + 1: one 8-B store
    // per row (a 4-B store where the odd pixel is past a ragged right edge)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && half) break;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t o = vo[0] + (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * pb;
        if (lane_ok[1]) {
          typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
          const u32x2_t d = {__float_as_uint(acc[i][0][r]), __float_as_uint(acc[i][1][r])};
          __builtin_amdgcn_raw_buffer_store_b64(d, ry, o, 0, 0);
        } else {
          buf_st(ry, o, acc[i][0][r]);
        }
      }
    }
  }
  if constexpr (ROWPAIR) if (p.pool_out) {
    // relu(maxpool2x2(y)) = maxpool2x2(relu(y)) -> pool_out [n][cout][ho/2][wo/2]
    // (torch MaxPool2d floor mode: a window needs both rows and both columns).  On
    // IEEE bit patterns: relu is max_i32(bits, 0) and the max of non-negative floats
    // is the unsigned max, under which a NaN (exponent all ones, non-zero mantissa)
    // beats every number -- so the window max propagates NaN like torch.
    const int hp = p.ho >> 1, wp = p.wo >> 1;
    const int py = (t.ty0 + (t.wn >> 1) * 2) >> 1;
    const int px = (t.tx0 + (t.wn & 1) * 32 + l32) >> 1;
    const bool ok = py < hp && px < wp && !(l32 & 1);
    const uint32_t ppb = (uint32_t)hp * (uint32_t)wp * 4u;
    const auto rp = make_srd(p.pool_out + ((size_t)t.n * p.cout + co_w) * hp * wp,
                             (uint32_t)rows * ppb);
    const uint32_t po = ok ? (uint32_t)(4 * h * hp * wp + py * wp + px) * 4u : BUF_OOB;
    auto rb = [](float v) -> uint32_t {
      const int b = __float_as_int(v);
      const uint32_t a = (uint32_t)b & 0x7fffffffu;
      return a > 0x7f800000u ? a : (uint32_t)max(b, 0);  // NaN stays NaN (sign dropped)
    };
    if constexpr (POOLSUM) {
      // nearest-x2 upsampling backward: dx = (y00 + y10) + (y01 + y11) -- the window's
      // two rows are this lane's two N-tiles, its other column is lane ^ 1 (DPP)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float s2 = acc[i][0][r] + acc[i][1][r];
          const float sp = __int_as_float(
              __builtin_amdgcn_mov_dpp(__float_as_int(s2), 0xB1, 0xF, 0xF, false));
          const int row = i * 32 + (r & 3) + 8 * (r >> 2);
          buf_st(rp, po + (uint32_t)row * ppb, s2 + sp);
        }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t m2 = max(rb(acc[i][0][r]), rb(acc[i][1][r]));
        // partner column (lane ^ 1) by a DPP quad permutation [1,0,3,2]: one VALU
        // move instead of an LDS bpermute
        const uint32_t mp = (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, 0xB1, 0xF, 0xF, false);
        const uint32_t m = max(m2, mp);
        const int row = i * 32 + (r & 3) + 8 * (r >> 2);
        buf_st(rp, po + (uint32_t)row * ppb, __uint_as_float(m));
      }
  }
  if constexpr (NI == 2 && TW == 64 && !RELU && WM == 1) if (p.gram_part) {
    // the max over valid pixels of all 64 rows (cout == 64: rows_full)
    conv_gram_tile<NI>(acc, p, t, lane_ok, vmax_u, smem);
  }
  if constexpr (NI == 2 && TW == 64 && !RELU && !PAR && WM == 2) if (p.gram_part) {
    // (cout == 128: both halves rows_full)
    conv_gram_tile128<TW, ROWPAIR>(acc, p, t, lane_ok, vo, vmax_u, smem);
  }
  if (p.out_amax) block_max_to(p.out_amax, __uint_as_float(vmax_u));
}

template <int TW, int NI, bool ROWPAIR, bool PAR = false, int WM = 1>
__device__ __forceinline__ bool conv_epilogue_plain(f32x16 (&acc)[2][NI], const stx_conv_params& p,
                                                    const EpiTile& t, float scale, char* smem) {
  if (p.mask || p.accumulate || p.acc_scale || p.up_dp || p.p2_z) return false;
  if (p.pool_sum) {  // validated by stx_conv2d: plain epilogue, row-pair tiles
    if constexpr (ROWPAIR)
      conv_epilogue_plain_body<TW, NI, ROWPAIR, false, false, true, false, WM>(acc, p, t, scale,
                                                                               smem);
    return true;
  }
  if (p.aux) {
    if (p.relu_out || p.pool_out || p.gram_part) return false;
    conv_epilogue_plain_body<TW, NI, ROWPAIR, false, true, false, PAR, WM>(acc, p, t, scale, smem);
  } else if (p.relu_out) {
    conv_epilogue_plain_body<TW, NI, ROWPAIR, true, false, false, PAR, WM>(acc, p, t, scale, smem);
  } else {
    conv_epilogue_plain_body<TW, NI, ROWPAIR, false, false, false, PAR, WM>(acc, p, t, scale,
                                                                            smem);
  }
  return true;
}

// acc *= acc_scale, then the ReLU mask (acc = 0 where mask <= 0): the order of the fp32
// path, ahead of a fused Gram-backward phase
template <int TW, bool ROWPAIR, int NI>
__device__ __forceinline__ void epi_scale_mask(f32x16 (&acc)[2][NI], const stx_conv_params& p,
                                               const EpiTile& t) {
  const size_t plane = (size_t)p.ho * p.wo;
  const int n = t.n, h = t.h, l32 = t.l32;
  if (p.acc_scale) {
    const float sc = *p.acc_scale;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= sc;
  }
  if (p.mask) {
    // descriptor at this wave's first row: per-lane pixel offset + per-register row
    // constant (no 64-bit address math); rows past cout / pixels past the image
    // read 0 (their outputs are dropped by the final stores anyway)
    const int co_m = t.co0 + t.wm * 64;
    const uint32_t mpb = (uint32_t)plane * 4u;
    const auto rm = make_srd(p.mask + ((size_t)n * p.cout + co_m) * plane,
                             (uint32_t)max(0, p.cout - co_m) * mpb);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int ty, tx;
      tile_pix<TW, ROWPAIR, NI>(t.wn, j, l32, ty, tx);
      const int oy = t.ty0 + ty, ox = t.tx0 + tx;
      const uint32_t mo = (oy < p.ho && ox < p.wo)
                              ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t row = (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2));
          if (!(buf_ld(rm, mo + row * mpb) > 0.f)) acc[i][j][r] = 0.f;
        }
    }
  }
}

template <int BM, int TW, int NPIX, int CIS2, bool ROWPAIR = false, int NI = 2,
          bool HAS_P2 = true>
// (NI: 32-pixel N-tiles per wave; ROWPAIR needs NI == 2)
__device__ __forceinline__ void conv_epilogue(f32x16 (&acc)[2][NI], const stx_conv_params& p,
                                              const EpiTile& t, float pre_scale,
                                              float* __restrict__ lds_in,
                                              float* __restrict__ lds_w) {
  const int tid = threadIdx.x;
  const size_t plane = (size_t)p.ho * p.wo;
  const int n = t.n, h = t.h, l32 = t.l32;
  if (pre_scale != 1.f) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] *= pre_scale;
  }
  bool mask_done = false;
  if (HAS_P2 && p.p2_z) {
    // ---- fused second phase: acc = acc*(mask>0) + s2 * A[n] . z2 (1x1, no halo) ----
    epi_scale_mask<TW, ROWPAIR, NI>(acc, p, t);
    mask_done = true;
    const float s2 = p.p2_scale ? *p.p2_scale : 1.f;
    const float* __restrict__ z2 = p.p2_z + (size_t)n * p.p2_c * plane;
    const float* __restrict__ w2 = p.p2_wt + (size_t)n * p.p2_wt_batch_stride;
    constexpr int E2 = CIS2 * NPIX;  // staged floats per phase-2 chunk
    constexpr int N2 = (E2 + 255) / 256;
    constexpr int WQ2 = CIS2 * BM / 4;
    constexpr int NW2 = (WQ2 + 255) / 256;
    int b2_base[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int ty, tx;
      tile_pix<TW, ROWPAIR, NI>(t.wn, j, l32, ty, tx);
      b2_base[j] = h * (CIS2 / 2) * NPIX + ty * TW + tx;
    }
    const int a2_base = h * (CIS2 / 2) * BM + t.wm * 64 + l32;
    uint32_t off2[N2];  // chunk-invariant byte offsets of the staged Z elements
#pragma unroll
    for (int e = 0; e < N2; ++e) {
      const int idx = tid + e * 256;
      const int ci = idx / NPIX, px = idx % NPIX;
      const int oy = t.ty0 + px / TW, ox = t.tx0 + px % TW;
      const bool ok = idx < E2 && oy < p.ho && ox < p.wo;
      off2[e] = ok ? (uint32_t)(ci * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
    }
    for (int c0 = 0; c0 < p.p2_c; c0 += CIS2) {
      const auto rz = make_srd(z2 + (size_t)c0 * plane, (uint32_t)((p.p2_c - c0) * plane * 4));
      float v2[N2];
#pragma unroll
      for (int e = 0; e < N2; ++e) v2[e] = s2 * buf_ld(rz, off2[e]);
      f32x4 wv2[NW2];
#pragma unroll
      for (int e = 0; e < NW2; ++e) {
        const int idx = tid + e * 256;
        if (idx < WQ2) {
          const int kr = idx / (BM / 4), c4 = idx - kr * (BM / 4);
          wv2[e] = *reinterpret_cast<const f32x4*>(w2 + (size_t)(c0 + kr) * p.cout_pad + t.co0 +
                                                  c4 * 4);
        }
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < N2; ++e) {
        const int idx = tid + e * 256;
        if (idx < E2) lds_in[idx] = v2[e];
      }
#pragma unroll
      for (int e = 0; e < NW2; ++e) {
        const int idx = tid + e * 256;
        if (idx < WQ2) *reinterpret_cast<f32x4*>(lds_w + idx * 4) = wv2[e];
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < CIS2 / 2; ++s) {
        float a[2], b[NI];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = lds_w[a2_base + s * BM + i * 32];
#pragma unroll
        for (int j = 0; j < NI; ++j) b[j] = lds_in[b2_base[j] + s * NPIX];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  }

  if (HAS_P2 && mask_done && !p.up_dp && !p.aux && !p.accumulate && !p.relu_out &&
      !p.pool_out) {
    // data gradient + Gram-backward phase (the Gatys dZ1 / dZ3 launches): bias and
    // out_amax only
    conv_epilogue_plain_body<TW, NI, ROWPAIR, false>(acc, p, t, 1.f,
                                                     reinterpret_cast<char*>(lds_in));
    return;
  }

  // ReLU + MaxPool2d(2,2) backward (unpool(up_dp) * (up_z > 0), argmax of the
  // relu'd window recomputed from up_z, first max in row-major order wins).  With the
  // row-pair mapping the window is this lane's two tiles x its partner lane (l32^1):
  // two z loads and one dp load per lane per register instead of six per element.
  float dpv[2][16];
  uint32_t dsel[2] = {0u, 0u};  // bit i*16+r of dsel[j]: element (i, j, r) takes dpv
  if constexpr (ROWPAIR) {
    if (p.up_dp) {
      const int hp = p.ho >> 1, wp = p.wo >> 1;
      const int ty0r = t.ty0 + (t.wn >> 1) * 2, oxr = t.tx0 + (t.wn & 1) * 32 + l32;
      const int py = ty0r >> 1, px = oxr >> 1, par = l32 & 1;
      const bool win = py < hp && px < wp;   // both rows, both columns exist
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = min(t.co0 + t.wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h,
                             p.cout - 1);
          const float* zc = p.up_z + ((size_t)n * p.cout + co) * plane;
          const int oyc = min(ty0r, p.ho - 1), oxc = min(oxr, p.wo - 1);
          const float za = zc[(size_t)oyc * p.wo + oxc];                      // row 2py
          const float zb = zc[(size_t)min(oyc + 1, p.ho - 1) * p.wo + oxc];   // row 2py+1
          const float pa = __shfl_xor(za, 1, 64), pb = __shfl_xor(zb, 1, 64);
          const float z0 = fmaxf(par ? pa : za, 0.f), z1 = fmaxf(par ? za : pa, 0.f);
          const float z2v = fmaxf(par ? pb : zb, 0.f), z3 = fmaxf(par ? zb : pb, 0.f);
          int bi = 0;
          float best = z0;
          if (z1 > best) { best = z1; bi = 1; }
          if (z2v > best) { best = z2v; bi = 2; }
          if (z3 > best) { bi = 3; }
          dpv[i][r] = win ? p.up_dp[(((size_t)n * p.cout + co) * hp + py) * wp + px] : 0.f;
          // element (row j, column parity par) is window slot j*2 + par
          if (win && bi == par && za > 0.f) dsel[0] |= 1u << (i * 16 + r);
          if (win && bi == 2 + par && zb > 0.f) dsel[1] |= 1u << (i * 16 + r);
        }
    }
  }

  // Final pass.  All tensor accesses go through buffer descriptors based at this
  // wave's first output row co_w: the per-element byte offset is one VGPR add of a
  // per-register row constant (SGPR) to a per-lane pixel offset, rows past cout
  // fall outside num_records and pixels outside the image carry BUF_OOB, so loads
  // read 0 and stores are dropped by the hardware -- no 64-bit address math and no
  // per-element bounds branches.
  const int co_w = t.co0 + t.wm * 64;
  const uint32_t rows = (uint32_t)max(0, p.cout - co_w);
  const size_t wofs = ((size_t)n * p.cout + co_w) * plane;
  const uint32_t pb = (uint32_t)plane * 4u;
  const auto ry = make_srd(p.y + wofs, rows * pb);
  // (absent operands: zero-size descriptors, so every load below is issued unconditionally
  // -- a load inside a per-element branch gets its own vmcnt(0) wait)
  const bool has_mask = !mask_done && p.mask, has_aux = p.aux, has_acc = p.accumulate;
  const auto rmask = make_srd(has_mask ? p.mask + wofs : p.y, has_mask ? rows * pb : 0u);
  const auto raux = make_srd(has_aux ? p.aux + wofs : p.y, has_aux ? rows * pb : 0u);
  const auto racc = make_srd(p.y + wofs, has_acc ? rows * pb : 0u);
  uint32_t vo[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    int ty, tx;
    tile_pix<TW, ROWPAIR, NI>(t.wn, j, l32, ty, tx);
    const int oy = t.ty0 + ty, ox = t.tx0 + tx;
    vo[j] = (oy < p.ho && ox < p.wo) ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u
                                     : BUF_OOB;
  }
  const auto rbias = make_srd(p.bias ? p.bias + co_w : p.y, p.bias ? rows * 4u : 0u);
  const float sc = (!mask_done && p.acc_scale) ? *p.acc_scale : 1.f;
  // per group of EG elements of one (j, i) register tile: the group's loads first, then
  // its stores -- a load issued after a store waits for it (vmcnt counts both), which
  // serialised an element-at-a-time pass into a load -> store round trip per element
  constexpr int EG = 8;
  uint32_t vmax_u = 0u;  // max |v| as IEEE bits: NaN (above inf) propagates
#pragma unroll
  for (int j = 0; j < NI; ++j) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r0 = 0; r0 < 16; r0 += EG) {
      float mv[16], av[16], yv[16], bv[16];
#pragma unroll
      for (int r = r0; r < r0 + EG; ++r) {
        const uint32_t o = vo[j] + (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * pb;
        bv[r] = buf_ld(rbias, (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 4u);
        mv[r] = buf_ld(rmask, o);
        av[r] = buf_ld(raux, o);
        yv[r] = buf_ld(racc, o);
      }
#pragma unroll
      for (int r = r0; r < r0 + EG; ++r) {
        float v = acc[i][j][r];
        if (!mask_done) {
          v *= sc;
          v = (!has_mask || mv[r] > 0.f) ? v : 0.f;
        }
        v += bv[r];
        if (ROWPAIR) {
          if ((dsel[j] >> (i * 16 + r)) & 1u) v += dpv[i][r];
        } else if (p.up_dp) {
          // ReLU + MaxPool2d(2,2) backward, argmax recomputed from up_z
          const int co = co_w + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          int ty, tx;
          tile_pix<TW, ROWPAIR, NI>(t.wn, j, l32, ty, tx);
          const int oy = t.ty0 + ty, ox = t.tx0 + tx;
          if (co < p.cout && oy < p.ho && ox < p.wo) {
            const size_t pofs = (size_t)oy * p.wo + ox;
            const float* zc = p.up_z + ((size_t)n * p.cout + co) * plane;
            const int hp = p.ho >> 1, wp = p.wo >> 1;
            const int py = oy >> 1, px2 = ox >> 1;
            if (py < hp && px2 < wp && zc[pofs] > 0.f) {
              const float* q = zc + (size_t)(2 * py) * p.wo + 2 * px2;
              const float z0 = fmaxf(q[0], 0.f), z1 = fmaxf(q[1], 0.f);
              const float z2v = fmaxf(q[p.wo], 0.f), z3 = fmaxf(q[p.wo + 1], 0.f);
              int bi = 0;
              float best = z0;
              if (z1 > best) { best = z1; bi = 1; }
              if (z2v > best) { best = z2v; bi = 2; }
              if (z3 > best) { bi = 3; }
              if (bi == ((oy & 1) * 2 + (ox & 1)))
                v += p.up_dp[(((size_t)n * p.cout + co) * hp + py) * wp + px2];
            }
          }
        }
        v = has_aux ? v + p.aux_scale * av[r] : v;
        v = has_acc ? v + yv[r] : v;
        if (p.relu_out) v = fmaxf(v, 0.f);
        acc[i][j][r] = v;  // (kept for the fused pooled output)
      }
#pragma unroll
      for (int r = r0; r < r0 + EG; ++r) {
        const uint32_t o = vo[j] + (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * pb;
        const float v = acc[i][j][r];
        buf_st(ry, o, v);
        // elements outside the output (dropped stores) must not count
        if (o < rows * pb) vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
      }
    }
    }
  }
  const float vmax = __uint_as_float(vmax_u);
  if constexpr (ROWPAIR) if (p.pool_out) {
    // relu(maxpool2x2(y)) = maxpool2x2(relu(y)) -> pool_out [n][cout][ho/2][wo/2]
    // (torch MaxPool2d floor mode: a window needs both rows and both columns)
    const int hp = p.ho >> 1, wp = p.wo >> 1;
    const int py = (t.ty0 + (t.wn >> 1) * 2) >> 1;
    const int px = (t.tx0 + (t.wn & 1) * 32 + l32) >> 1;
    const bool ok = py < hp && px < wp && !(l32 & 1);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float m = fmaxf(acc[i][0][r], acc[i][1][r]);
        if (acc[i][0][r] != acc[i][0][r]) m = acc[i][0][r];
        const float o = __shfl_xor(m, 1, 64);
        m = (o != o) ? o : ((m != m) ? m : fmaxf(m, o));
        m = (m != m) ? m : fmaxf(m, 0.f);
        const int co = t.co0 + t.wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (ok && co < p.cout)
          p.pool_out[(((size_t)n * p.cout + co) * hp + py) * wp + px] = m;
      }
  }
  if (p.out_amax) block_max_to(p.out_amax, vmax);
}

}  // namespace stx
