// Implicit-GEMM convolution for gfx950 on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
//   out[n][co][oy][ox] = sum_{ci,kh,kw} W[co][ci][kh][kw] * V[n][ci][oy*S-P+kh][ox*S-P+kw]
//
// GEMM view: M = cout, N = output pixels of one image, K = cin*KS*KS.
// A block owns BM output channels x a TH x TW output-pixel tile of one image and
// walks K in chunks of CIS input channels.  Per chunk it stages
//   * the input HALO  [CIS][RH][RW]  (the virtual input V, formed on the fly from
//     x by the loader: relu / relu+maxpool / nearest-upsample / zero-dilation),
//     so each input element is read from L2 once per chunk and re-used KS*KS times
//     out of LDS ("LDS-staged 3x3 conv tiles");
//   * the weight slab [CIS*KS*KS][BM] (prepped k-major layout, coalesced rows).
// MFMA operand mapping (32x32x2, lane l, half h = l>>5): lane supplies
// A[i = l&31][k_h] and B[k_h][j = l&31].  The two k slots of each MFMA are
// assigned to the two lane halves as two different input channels
// (k = s + h*KC/2), so every LDS address is (lane base) + compile-time offset.
//
// Reference: torchvision vgg19 Conv2d(3x3,p1) used by StyleNetwork
// (stransfer/network.py:246-314) and the ImageTransformNet convs
// (stransfer/network.py:468-481, 525-609; zero padding = torch 1.1.0 semantics
// of padding_mode='reflection').
#include "common.h"
#include "conv_epi.h"
#include "gbwd16.h"
#include "wprep.h"
#include "../../include/stx.h"

namespace stx {

__device__ __forceinline__ float load_virtual(const float* __restrict__ xp, int mode, int cin,
                                              int h, int w, int hv, int wv, int ci, int vy,
                                              int vx) {
  if (ci >= cin || vy < 0 || vx < 0 || vy >= hv || vx >= wv) return 0.f;
  const float* plane = xp + (size_t)ci * h * w;
  switch (mode) {
    case STX_IN_RAW:
      return plane[vy * w + vx];
    case STX_IN_RELU:
      return fmaxf(plane[vy * w + vx], 0.f);
    case STX_IN_RELU_POOL2: {
      const float* q = plane + (2 * vy) * w + 2 * vx;
      // relu then max: every relu'd value is >= 0, start from 0
      float m = fmaxf(fmaxf(q[0], q[1]), fmaxf(q[w], q[w + 1]));
      return fmaxf(m, 0.f);
    }
    case STX_IN_UPSAMPLE2:
      return plane[(vy >> 1) * w + (vx >> 1)];
    default: {  // STX_IN_DILATE2
      if ((vy | vx) & 1) return 0.f;
      const int sy = vy >> 1, sx = vx >> 1;
      if (sy >= h || sx >= w) return 0.f;
      return plane[sy * w + sx];
    }
  }
}

template <int KS, int S, int CIS, int BM, int TW>
struct ConvCfg {
  static constexpr int WM = BM / 64;          // waves along M (each 64 rows = 2 MFMA tiles)
  static constexpr int WN = 4 / WM;           // waves along N
  static constexpr int MI = 2, NI = 2;        // MFMA tiles per wave
  static constexpr int NPIX = WN * NI * 32;   // output pixels per block
  static constexpr int TH = NPIX / TW;
  static constexpr int RH = (TH - 1) * S + KS;
  static constexpr int RW = (TW - 1) * S + KS;
  static constexpr int RWP = RW;
  static constexpr int CH = RH * RWP;
  static constexpr int KK = KS * KS;
  static constexpr int KC = CIS * KK;          // K per chunk
  static constexpr int HALO = CIS * RH * RW;
  static constexpr int NH = (HALO + 255) / 256;
  static constexpr int WQ = KC * BM / 4;       // float4 per weight slab
  static constexpr int NW = (WQ + 255) / 256;
  // halo / slab regions padded to whole 256-thread rounds: the stores are unconditional
  static constexpr int LDS_IN = NH * 256;
  static constexpr int LDS_FLOATS = LDS_IN + NW * 1024;
  static_assert(CIS % 2 == 0, "CIS must be even (two lane halves)");
  static_assert(NPIX % TW == 0, "tile");
};

// Halo element i of this thread (idx = tid + i*256) always maps to the same
// (ci_local, r, c) and, for a given block, to the same source offset within the
// input-channel plane; only the channel base moves from chunk to chunk.  So the
// per-element offsets and the in-bounds mask are computed once per block and the
// per-chunk fetch is one (or, for the fused 2x2 pool, four) loads per element.
// Halo element i of this thread (idx = tid + i*256) always maps to the same
// (ci_local, r, c) and, for a given block, to the same byte offset from the
// chunk's first input channel; only the chunk base moves.  So the offsets are
// computed once per block (BUF_OOB for zero padding) and the per-chunk fetch is
// one (or, for the fused 2x2 pool, four) unconditional buffer loads per element.
// The loads land raw in registers; the relu / pool transform runs in
// halo_store, after the MFMA loop, so no wait on them is exposed before it.
template <bool POOL, int NH>
__device__ __forceinline__ void halo_fetch(float (&hraw)[NH][4], __amdgpu_buffer_rsrc_t rs,
                                           const uint32_t (&hoff)[NH], uint32_t wb) {
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const uint32_t o = hoff[i];
    hraw[i][0] = buf_ld(rs, o);
    if (POOL) {
      hraw[i][1] = buf_ld(rs, o + 4);
      hraw[i][2] = buf_ld(rs, o + wb);
      hraw[i][3] = buf_ld(rs, o + wb + 4);
    }
  }
}

template <int MODE, int NH>
__device__ __forceinline__ void halo_store(float* __restrict__ lds_in, const float (&hraw)[NH][4],
                                           int tid) {
#pragma unroll
  for (int i = 0; i < NH; ++i) {
    const int idx = tid + i * 256;
    float v = hraw[i][0];
    if (MODE == STX_IN_RELU_POOL2)
      v = fmaxf(fmaxf(fmaxf(v, hraw[i][1]), fmaxf(hraw[i][2], hraw[i][3])), 0.f);
    else if (MODE == STX_IN_RELU)
      v = fmaxf(v, 0.f);
    lds_in[idx] = v;  // idx >= HALO lands in the padding of the halo region
  }
}

// LM: loader mode of the halo fetch -- STX_IN_RAW (also serves UPSAMPLE2 and
// DILATE2, whose index maps live in the precomputed offsets), STX_IN_RELU or
// STX_IN_RELU_POOL2 (four loads per element).
template <int KS, int S, int CIS, int BM, int TW, int LM>
__global__ void __launch_bounds__(256, 2)
conv_fwd_kernel(stx_conv_params p, int tiles_x) {
  using C = ConvCfg<KS, S, CIS, BM, TW>;
  static_assert(C::RWP == C::RW, "halo LDS index == element index");
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  float* lds_in = smem;
  float* lds_w = smem + C::LDS_IN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm = wave / C::WN, wn = wave % C::WN;

  const int tile = blockIdx.x;
  const int ty0 = (tile / tiles_x) * C::TH, tx0 = (tile % tiles_x) * TW;
  const int co0 = blockIdx.y * BM;
  const int n = blockIdx.z;

  const float* __restrict__ xn = p.x + (size_t)n * p.cin * p.h * p.w;
  const float* __restrict__ wt = p.wt + (size_t)n * p.wt_batch_stride;
  const int vy0 = ty0 * S - p.pad, vx0 = tx0 * S - p.pad;
  const int mode = p.in_mode;
  const int plane_in = p.h * p.w;

  // chunk-invariant halo byte offsets (BUF_OOB = zero padding)
  uint32_t hoff[C::NH];
#pragma unroll
  for (int i = 0; i < C::NH; ++i) {
    const int idx = tid + i * 256;
    const int ci = idx / (C::RH * C::RW);
    const int rem = idx - ci * (C::RH * C::RW);
    const int r = rem / C::RW, c = rem - r * C::RW;
    const int vy = vy0 + r, vx = vx0 + c;
    bool ok = idx < C::HALO && vy >= 0 && vx >= 0 && vy < p.hv && vx < p.wv;
    int sy = vy, sx = vx;
    if (mode == STX_IN_RELU_POOL2) {
      sy = 2 * vy;
      sx = 2 * vx;
    } else if (mode == STX_IN_UPSAMPLE2) {
      sy = vy >> 1;
      sx = vx >> 1;
    } else if (mode == STX_IN_DILATE2) {
      ok = ok && !((vy | vx) & 1);
      sy = vy >> 1;
      sx = vx >> 1;
      ok = ok && sy < p.h && sx < p.w;
    }
    hoff[i] = ok ? (uint32_t)(ci * plane_in + sy * p.w + sx) * 4u : BUF_OOB;
  }

  f32x16 acc[C::MI][C::NI];
#pragma unroll
  for (int i = 0; i < C::MI; ++i)
#pragma unroll
    for (int j = 0; j < C::NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-lane LDS bases
  // 1x1 convs (the Gram backward with the fused unpool epilogue) use the row-pair
  // pixel mapping so each 2x2 pooling window lies inside one wave
  constexpr bool ROWPAIR = KS == 1 && TW == 64;
  int b_base[C::NI];
#pragma unroll
  for (int j = 0; j < C::NI; ++j) {
    int ty, tx;
    tile_pix<TW, ROWPAIR>(wn, j, l32, ty, tx);
    b_base[j] = h * (CIS / 2) * C::CH + ty * S * C::RWP + tx * S;
  }
  const int a_base = h * (CIS / 2) * C::KK * BM + wm * 64 + l32;

  float hraw[C::NH][4];
  f32x4 wreg[C::NW];
  const int nchunks = p.cin_pad / CIS;

  // chunk-invariant weight-slab byte offsets (from the chunk's first slab row)
  uint32_t woff[C::NW];
#pragma unroll
  for (int i = 0; i < C::NW; ++i) {
    const int idx = tid + i * 256;
    const int kr = idx / (BM / 4), c4 = idx - kr * (BM / 4);
    woff[i] = idx < C::WQ ? (uint32_t)(kr * p.cout_pad + co0 + c4 * 4) * 4u : BUF_OOB;
  }
  const uint32_t wbytes = (uint32_t)p.cin_pad * C::KK * p.cout_pad * 4u;

  auto fetch = [&](int chunk) {
    const int c0 = chunk * CIS;
    // descriptor over channels [c0, cin): padding channels past cin read 0
    const auto rs = make_srd(xn + (size_t)c0 * plane_in, (uint32_t)(p.cin - c0) * plane_in * 4u);
    halo_fetch<LM == STX_IN_RELU_POOL2, C::NH>(hraw, rs, hoff, 4u * p.w);
    const uint32_t wskip = (uint32_t)c0 * C::KK * p.cout_pad * 4u;
    const auto rw = make_srd(wt + (size_t)c0 * C::KK * p.cout_pad, wbytes - wskip);
#pragma unroll
    for (int i = 0; i < C::NW; ++i) wreg[i] = buf_ld4(rw, woff[i]);
  };
  auto store = [&]() {
    halo_store<LM, C::NH>(lds_in, hraw, tid);
#pragma unroll
    for (int i = 0; i < C::NW; ++i)
      *reinterpret_cast<f32x4*>(lds_w + (tid + i * 256) * 4) = wreg[i];
  };

  fetch(0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();  // previous chunk's reads done
    store();
    __syncthreads();
    if (chunk + 1 < nchunks) fetch(chunk + 1);  // overlaps the MFMA loop below
    // Software-pipelined operand reads: a ring of PD register slots; the LDS reads
    // of step s+PD are issued right after step s's MFMAs consume slot s%PD, so an
    // LDS round trip is hidden behind PD steps (4 MFMAs = 256 cycles each).
    constexpr int NS = (CIS / 2) * C::KK;
    constexpr int PD = 3;
    float ra[PD][C::MI], rb[PD][C::NI];
    auto rd = [&](int s, float (&a)[C::MI], float (&b)[C::NI]) {
      const int cil = s / C::KK, r = s % C::KK, kh = r / KS, kw = r % KS;
#pragma unroll
      for (int i = 0; i < C::MI; ++i) a[i] = lds_w[a_base + s * BM + i * 32];
#pragma unroll
      for (int j = 0; j < C::NI; ++j) b[j] = lds_in[b_base[j] + cil * C::CH + kh * C::RWP + kw];
    };
#pragma unroll
    for (int s = 0; s < PD && s < NS; ++s) rd(s, ra[s], rb[s]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int slot = s % PD;
#pragma unroll
      for (int i = 0; i < C::MI; ++i)
#pragma unroll
        for (int j = 0; j < C::NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[slot][i], rb[slot][j], acc[i][j],
                                                           0, 0, 0);
      if (s + PD < NS) rd(s + PD, ra[slot], rb[slot]);
      // keep the prefetch reads ahead of the next step's MFMAs (the scheduler
      // otherwise sinks them next to their use and waits lgkmcnt(0) every step)
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  static_assert(CIS * C::NPIX <= C::LDS_IN && CIS * BM <= C::KC * BM, "phase-2 staging fits");
  const EpiTile et{n, co0, ty0, tx0, wm, wn, h, l32};
  conv_epilogue<BM, TW, C::NPIX, CIS, ROWPAIR>(acc, p, et, 1.f, lds_in, lds_w);
}

// ------------------------------------------------------- small-cout direct conv
// cout <= 4, stride 1 (VGG conv1_1 data-gradient 64->3, ImageTransformNet's final
// 9x9 conv 32->3).  An MFMA tile would be >= 90% padding here, so this is a VALU
// direct convolution: thread = 4 consecutive output pixels x all output channels;
// a block is G = 2 channel groups x (TH x 64 output pixels): group g takes the
// input-channel chunks g, g+2, ... (so one image tile keeps 2x the waves in flight),
// and the two partial sums are added in a fixed order at the end (deterministic).
// Per chunk of CIS channels the input halo (row pitch padded to 16 B for
// ds_read_b128) and the chunk's weights are prefetched into registers during the
// previous chunk's FMAs and staged in LDS; every FMA takes one LDS value re-used KS
// times across kw and COUT times across output channels; weights are LDS broadcasts.
constexpr int SC_TW = 64, SC_PX = 4;

template <int KS, int CIS, int TH, int SC_G>
struct SmallCfg {
  static constexpr int NT = 16 * TH;                   // threads per channel group
  static constexpr int RH = TH + KS - 1;
  static constexpr int RW = SC_TW + KS - 1;
  static constexpr int RWP = (RW + 3) / 4 * 4;
  static constexpr int CH = RH * RWP;
  static constexpr int PL = RH * RW;                   // halo elements per channel plane
  static constexpr int NE = (PL + NT - 1) / NT;
  static constexpr int NV = (SC_PX + KS - 1 + 3) / 4;  // float4 reads per row
  static constexpr int WU = CIS * KS * KS;             // f32x4 weight units per chunk
  static constexpr int NWU = (WU + NT - 1) / NT;
};

// SC_G channel groups per block split the input channels (chunk c0 = (SC_G*k + g)*CIS)
// and combine their partial sums in a fixed order at the end
template <int KS, int CIS, int TH, int SC_G, int COUT = 4>
__global__ void __launch_bounds__(SC_G * 16 * TH)
conv_smallc_kernel(stx_conv_params p, int tiles_x) {
  using C = SmallCfg<KS, CIS, TH, SC_G>;
  static_assert(COUT >= 1 && COUT <= 4, "weights are staged as 4 couts per f32x4");
  __shared__ __attribute__((aligned(16))) float halo[SC_G][CIS * C::CH];
  __shared__ __attribute__((aligned(16))) f32x4 wts[SC_G][C::WU];  // [ci][tap] -> 4 couts
  const int g = threadIdx.x / C::NT, tid = threadIdx.x % C::NT;
  const int ty = tid / 16, tx = tid % 16;
  const int tile = blockIdx.x, n = blockIdx.z;
  const int oy0 = (tile / tiles_x) * TH, ox0 = (tile % tiles_x) * SC_TW;
  const int vy0 = oy0 - p.pad, vx0 = ox0 - p.pad;
  const float* __restrict__ xn = p.x + (size_t)n * p.cin * p.h * p.w;
  const float* __restrict__ wt = p.wt + (size_t)n * p.wt_batch_stride;
  const int plane_in = p.h * p.w;
  constexpr int KK = KS * KS;
  const bool relu_in = p.in_mode == STX_IN_RELU;

  // plane-invariant halo offsets (source and LDS) of this thread's elements
  int eoff[C::NE], loff[C::NE];
  uint32_t evalid = 0;
#pragma unroll
  for (int e = 0; e < C::NE; ++e) {
    const int idx = tid + e * C::NT;
    const int r = idx / C::RW, c = idx - (idx / C::RW) * C::RW;
    const int vy = vy0 + r, vx = vx0 + c;
    const bool in_tile = idx < C::PL;
    const bool ok = in_tile && vy >= 0 && vx >= 0 && vy < p.hv && vx < p.wv;
    eoff[e] = ok ? vy * p.w + vx : 0;
    loff[e] = in_tile ? r * C::RWP + c : -1;
    if (ok) evalid |= 1u << e;
  }

  // (packed v_pk_fma_f32 over pixel pairs measured 1.37x SLOWER here: 209 vs 153 us)
  float acc[COUT][SC_PX];
#pragma unroll
  for (int c = 0; c < COUT; ++c)
#pragma unroll
    for (int q = 0; q < SC_PX; ++q) acc[c][q] = 0.f;

  float hv[CIS][C::NE];
  f32x4 wv[C::NWU];
  // branch-free fetch: out-of-tile / padding elements read 0 through the buffer
  // descriptor's range check, weights come from a clamped valid address and are
  // selected after the load (a predicated load is a branch + vmcnt(0) per element)
  const auto rx = make_srd(xn, (uint32_t)p.cin * (uint32_t)plane_in * 4u);
  auto fetch = [&](int c0) {
    const int cn = min(CIS, p.cin - c0);
#pragma unroll
    for (int cil = 0; cil < CIS; ++cil) {
      const uint32_t cofs = (uint32_t)(c0 + cil) * (uint32_t)plane_in;
#pragma unroll
      for (int e = 0; e < C::NE; ++e) {
        const bool ok = cil < cn && ((evalid >> e) & 1);
        float v = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rx, ok ? (cofs + eoff[e]) * 4u : BUF_OOB,
                                                        0, 0));
        if (relu_in) v = fmaxf(v, 0.f);
        hv[cil][e] = v;
      }
    }
#pragma unroll
    for (int k = 0; k < C::NWU; ++k) {
      const int i = tid + k * C::NT;
      const int cil = i / KK;
      const int ic = min(i, C::WU - 1), cc = min(c0 + ic / KK, p.cin - 1);
      const f32x4 v = *reinterpret_cast<const f32x4*>(wt + (size_t)(cc * KK + (ic - (ic / KK) * KK)) *
                                                               p.cout_pad);
      const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
      wv[k] = (i < C::WU && cil < cn) ? v : zero;
    }
  };
  // chunks of this group: c0 = (2k + g) * CIS
  const int nch = cdiv(p.cin, CIS);
  int chunk = g;
  if (chunk < nch) fetch(chunk * CIS);
  // every thread runs the same number of loop trips (barriers): groups idle past nch
  const int trips = cdiv(nch, SC_G);
  for (int it = 0; it < trips; ++it, chunk += SC_G) {
    const bool active = chunk < nch;
    __syncthreads();
    if (active) {
#pragma unroll
      for (int cil = 0; cil < CIS; ++cil)
#pragma unroll
        for (int e = 0; e < C::NE; ++e)
          if (loff[e] >= 0) halo[g][cil * C::CH + loff[e]] = hv[cil][e];
#pragma unroll
      for (int k = 0; k < C::NWU; ++k) {
        const int i = tid + k * C::NT;
        if (i < C::WU) wts[g][i] = wv[k];
      }
    }
    __syncthreads();
    if (!active) continue;
    const int cn = min(CIS, p.cin - chunk * CIS);
    if (chunk + SC_G < nch) fetch((chunk + SC_G) * CIS);
    for (int cil = 0; cil < cn; ++cil) {
      const f32x4* wk = wts[g] + cil * KK;
#pragma unroll
      for (int kh = 0; kh < KS; ++kh) {
        float in[C::NV * 4];
        const float* row = halo[g] + cil * C::CH + (ty + kh) * C::RWP + tx * SC_PX;
#pragma unroll
        for (int v = 0; v < C::NV; ++v) {
          const f32x4 t = *reinterpret_cast<const f32x4*>(row + 4 * v);
          in[4 * v + 0] = t[0];
          in[4 * v + 1] = t[1];
          in[4 * v + 2] = t[2];
          in[4 * v + 3] = t[3];
        }
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const f32x4 w4 = wk[kh * KS + kw];  // LDS broadcast (same address in all lanes)
#pragma unroll
          for (int c = 0; c < COUT; ++c)
#pragma unroll
            for (int q = 0; q < SC_PX; ++q) acc[c][q] = fmaf(w4[c], in[q + kw], acc[c][q]);
        }
      }
    }
  }
  // fixed-order combine: groups 1..SC_G-1 pass partial sums through LDS, group 0
  // adds them in group order
  __syncthreads();
  float* red = &halo[0][0];
  static_assert(C::NT * COUT * SC_PX * (SC_G - 1) <= SC_G * CIS * C::CH, "reduction buffer fits");
  if (g > 0) {
#pragma unroll
    for (int c = 0; c < COUT; ++c)
#pragma unroll
      for (int q = 0; q < SC_PX; ++q)
        red[((g - 1) * COUT * SC_PX + c * SC_PX + q) * C::NT + tid] = acc[c][q];
  }
  __syncthreads();
  if (g > 0) return;
#pragma unroll
  for (int gg = 1; gg < SC_G; ++gg)
#pragma unroll
    for (int c = 0; c < COUT; ++c)
#pragma unroll
      for (int q = 0; q < SC_PX; ++q)
        acc[c][q] += red[((gg - 1) * COUT * SC_PX + c * SC_PX + q) * C::NT + tid];
  const int oy = oy0 + ty;
  if (oy >= p.ho) return;
  const size_t plane = (size_t)p.ho * p.wo;
#pragma unroll
  for (int c = 0; c < COUT; ++c) {
    if (c >= p.cout) break;
#pragma unroll
    for (int q = 0; q < SC_PX; ++q) {
      const int ox = ox0 + tx * SC_PX + q;
      if (ox >= p.wo) continue;
      const size_t o = ((size_t)n * p.cout + c) * plane + (size_t)oy * p.wo + ox;
      float v = acc[c][q];
      if (p.acc_scale) v *= *p.acc_scale;
      if (p.bias) v += p.bias[c];
      if (p.mask) v = p.mask[o] > 0.f ? v : 0.f;
      if (p.aux) v += p.aux_scale * p.aux[o];
      if (p.accumulate) v += p.y[o];
      if (p.relu_out) v = fmaxf(v, 0.f);
      p.y[o] = v;
    }
  }
}

template <int KS, int TH>
static int launch_smallc(const stx_conv_params& p, hipStream_t st) {
  const int tiles_x = cdiv(p.wo, SC_TW), tiles_y = cdiv(p.ho, TH);
  dim3 grid(tiles_x * tiles_y, 1, p.n);
  constexpr int CIS = KS == 9 ? 4 : 8;
#ifdef STX_AB  // measured tilings (not in the product build)
  if constexpr (KS == 3) {
    static const int cfg = STX_KNOB("STX_SMALLC", 0);
    if (cfg == 1) {
      const int ty = cdiv(p.ho, 4);
      hipLaunchKernelGGL((conv_smallc_kernel<KS, 4, 4, 4>), dim3(tiles_x * ty, 1, p.n),
                         dim3(4 * 16 * 4), 0, st, p, tiles_x);
      return check_launch("stx_conv2d(smallc)");
    }
    if (cfg == 2) {
      hipLaunchKernelGGL((conv_smallc_kernel<KS, 4, TH, 4>), grid, dim3(4 * 16 * TH), 0, st, p,
                         tiles_x);
      return check_launch("stx_conv2d(smallc)");
    }
    if (cfg == 3) {
      const int ty = cdiv(p.ho, 4);
      hipLaunchKernelGGL((conv_smallc_kernel<KS, 8, 4, 2>), dim3(tiles_x * ty, 1, p.n),
                         dim3(2 * 16 * 4), 0, st, p, tiles_x);
      return check_launch("stx_conv2d(smallc)");
    }
    if (cfg == 4) {
      const int ty = cdiv(p.ho, 4);
      hipLaunchKernelGGL((conv_smallc_kernel<KS, 8, 4, 4>), dim3(tiles_x * ty, 1, p.n),
                         dim3(4 * 16 * 4), 0, st, p, tiles_x);
      return check_launch("stx_conv2d(smallc)");
    }
  }
#endif
  static const bool c3 = STX_KNOB("STX_SMALLC_C3", 1) != 0;
  if (p.cout == 3 && c3)  // the ITN's final conv: no idle fourth output channel
    hipLaunchKernelGGL((conv_smallc_kernel<KS, CIS, TH, 2, 3>), grid, dim3(2 * 16 * TH), 0, st,
                       p, tiles_x);
  else
    hipLaunchKernelGGL((conv_smallc_kernel<KS, CIS, TH, 2>), grid, dim3(2 * 16 * TH), 0, st, p,
                       tiles_x);
  return check_launch("stx_conv2d(smallc)");
}

// ---------------------------------------------------------------- weight prep
__global__ void weight_prep_kernel(const float* __restrict__ w, float* __restrict__ wt, int cout,
                                   int cin, int ks, int transpose, int rows_pad, int cols_pad) {
  weight_prep32_body(w, wt, cout, cin, ks, transpose, rows_pad, cols_pad,
                     blockIdx.x * (long long)blockDim.x + threadIdx.x,
                     (long long)gridDim.x * blockDim.x);
}

// input channels per K chunk; 3x3 convs over <= 4 channels (conv1_1, 3-channel
// images) use 4 so the RGB input is padded to 4, not 8
static int cis_for(int ks, int cin) {
  return ks == 9 ? 2 : (ks == 1 ? 16 : (cin <= 4 ? 4 : 8));
}

template <int KS, int S, int CIS, int BM, int TW, int LM>
static int launch_fwd(const stx_conv_params& p, hipStream_t st) {
  using C = ConvCfg<KS, S, CIS, BM, TW>;
  const int tiles_x = cdiv(p.wo, TW), tiles_y = cdiv(p.ho, C::TH);
  dim3 grid(tiles_x * tiles_y, cdiv(p.cout, BM), p.n);
  hipLaunchKernelGGL((conv_fwd_kernel<KS, S, CIS, BM, TW, LM>), grid, dim3(256), 0, st, p,
                     tiles_x);
  return check_launch("stx_conv2d");
}

template <int KS, int S, int BM, int LM>
static int dispatch_tw(const stx_conv_params& p, hipStream_t st) {
  constexpr int CIS = KS == 9 ? 2 : (KS == 1 ? 16 : 8);
  if constexpr (KS == 3 && S == 1 && BM == 64 && LM == STX_IN_RAW) {  // RGB input
    if (p.cin_pad == 4) {
      if (p.wo > 32) return launch_fwd<3, 1, 4, 64, 64, LM>(p, st);
      return launch_fwd<3, 1, 4, 64, 16, LM>(p, st);
    }
  }
  if (p.wo > 32) return launch_fwd<KS, S, CIS, BM, 64, LM>(p, st);
  if (p.wo > 16) return launch_fwd<KS, S, CIS, BM, 32, LM>(p, st);
  return launch_fwd<KS, S, CIS, BM, 16, LM>(p, st);
}

int conv2d_f16x3(const stx_conv_params& p, hipStream_t st);  // conv16.hip
int conv2d_fewin(const stx_conv_params& p, hipStream_t st);  // convfew.hip (-1: not covered)
int fewin_gram_tiles(const stx_conv_params& p);              // convfew.hip
int conv2d_fewout(const stx_conv_params& p, hipStream_t st);  // convfew.hip (-1: not covered)
int conv2d_conv9(const stx_conv_params& p, hipStream_t st);   // conv9.hip (-1: not covered)

}  // namespace stx

using namespace stx;

extern "C" int stx_conv_weight_dims(int cin, int cout, int ks, int* cin_pad, int* cout_pad) {
  if (ks != 1 && ks != 3 && ks != 9) {
    set_error("stx_conv_weight_dims: unsupported kernel size %d", ks);
    return STX_E_INVALID;
  }
  if (cin_pad) *cin_pad = rup(cin, cis_for(ks, cin));
  // BM is 64 for cout <= 64 and 128 otherwise; pad to the tile so VGG widths need none
  if (cout_pad) *cout_pad = cout <= 64 ? rup(cout, 64) : rup(cout, 128);
  return STX_OK;
}

extern "C" int stx_conv_weight_prep(const float* w, float* wt, int cout, int cin, int ks,
                                    int transpose, void* stream) {
  int rp, cp;
  // GEMM dims of the conv this slab feeds
  const int gin = transpose ? cout : cin, gout = transpose ? cin : cout;
  int rc = stx_conv_weight_dims(gin, gout, ks, &rp, &cp);
  if (rc) return rc;
  const long long total = (long long)rp * ks * ks * cp;
  if (total >= (1ll << 31)) {
    set_error("stx_conv_weight_prep: slab too large");
    return STX_E_INVALID;
  }
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(weight_prep_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wt,
                     cout, cin, ks, transpose, rp * ks * ks, cp);
  return check_launch("stx_conv_weight_prep");
}

static int device_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

extern "C" int stx_conv_gram_tiles(const stx_conv_params* pp) {
  if (!pp) return 0;
  const stx_conv_params& p = *pp;
  // conv16's 256-pixel (64 x 4) tiles through the plain epilogue (cout 128: the 8-wave
  // block of launch16_gram128, raw or ReLU input, and only for a single round of blocks:
  // with one 135 KB block per CU a second round waits for the first one's epilogue, and
  // the fast_st batch (B = 8, 512 blocks) measured no faster than the standalone triangle
  // kernel -- Gatys' 256-block conv2_x: 10.8 us per iteration saved, same-box profile)
  const int tiles = cdiv(p.wo, 64) * cdiv(p.ho, 4);
  const bool ok = p.wt16 && p.wt16 != (const void*)1 && p.ks == 3 && p.pad == 1 &&
                  p.stride == 1 && p.cin >= 16 &&
                  (p.cout == 64 ||
                   (p.cout == 128 && (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) &&
                    (long long)tiles * p.n <= device_cus())) &&
                  p.wo > 32 && p.wt_batch_stride == 0 && !p.mask && !p.aux && !p.accumulate &&
                  !p.acc_scale && !p.up_dp && !p.p2_z && !p.relu_out && !p.pool_sum;
  if (ok) return tiles;
  if (p.cout != 64) return 0;
  return fewin_gram_tiles(p);  // 3 input channels (VGG conv1_1): 64 x 8 tiles
}

extern "C" int stx_conv_gram_groups(const stx_conv_params* pp) {
  if (!pp || pp->cout != 64) return 0;  // the grouped sums: 64-channel tiles only
  const int t = stx_conv_gram_tiles(pp);
  return t > 0 ? cdiv(t, STX_GRAM_GROUP) : 0;
}

extern "C" int stx_conv2d(const stx_conv_params* pp, void* stream) {
  if (!pp) {
    set_error("stx_conv2d: null params");
    return STX_E_INVALID;
  }
  const stx_conv_params& p = *pp;
  hipStream_t st = (hipStream_t)stream;
  int cinp, coutp;
  if (stx_conv_weight_dims(p.cin, p.cout, p.ks, &cinp, &coutp)) return STX_E_INVALID;
  if (p.cin_pad != cinp || p.cout_pad != coutp || p.n <= 0 || p.ho <= 0 || p.wo <= 0 ||
      p.pad < 0 || p.in_mode < 0 || p.in_mode > 4 || !p.x || (!p.y && !p.pool_out) ||
      (!p.wt && (!p.wt16 || p.wt16 == (const void*)1))) {
    set_error("stx_conv2d: invalid params (cin_pad %d/%d cout_pad %d/%d n %d ho %d wo %d)",
              p.cin_pad, cinp, p.cout_pad, coutp, p.n, p.ho, p.wo);
    return STX_E_INVALID;
  }
  // geometry consistency: ho = (hv + 2p - ks)/s + 1
  if ((p.hv + 2 * p.pad - p.ks) / p.stride + 1 != p.ho ||
      (p.wv + 2 * p.pad - p.ks) / p.stride + 1 != p.wo) {
    set_error("stx_conv2d: inconsistent output dims");
    return STX_E_INVALID;
  }
  if (p.in_mode == STX_IN_RELU_POOL2 && (p.hv * 2 > p.h || p.wv * 2 > p.w)) {
    set_error("stx_conv2d: pool dims");
    return STX_E_INVALID;
  }
  if (p.in_mode == STX_IN_UPSAMPLE2 && (p.hv > 2 * p.h || p.wv > 2 * p.w)) {
    set_error("stx_conv2d: upsample dims");
    return STX_E_INVALID;
  }
  if (p.in_mode <= STX_IN_RELU && (p.hv != p.h || p.wv != p.w)) {
    set_error("stx_conv2d: raw dims");
    return STX_E_INVALID;
  }
  // buffer-descriptor byte counts (and the BUF_OOB sentinel) are 32-bit
  const long long in_bytes = 4LL * p.cin * p.h * p.w;
  const long long wt_bytes = 4LL * p.cin_pad * p.ks * p.ks * p.cout_pad;
  const long long p2_bytes = p.p2_z ? 4LL * p.p2_c * p.ho * p.wo : 0;
  const long long out_bytes = 4LL * p.cout * p.ho * p.wo;  // epilogue descriptors
  if (in_bytes >= (long long)BUF_OOB / 2 || wt_bytes >= (long long)BUF_OOB / 2 ||
      p2_bytes >= (long long)BUF_OOB / 2 || out_bytes >= (long long)BUF_OOB / 2) {
    set_error("stx_conv2d: per-image tensor too large (>= 1 GiB)");
    return STX_E_INVALID;
  }
  if (p.p2_z && (p.stride != 1 || !p.p2_wt || p.p2_c <= 0)) {
    set_error("stx_conv2d: fused phase 2 needs stride 1, p2_wt and p2_c > 0");
    return STX_E_INVALID;
  }
  if (p.p2_z && p.wt16 && p.wt16 != (const void*)1 && p.cin > 0 && p.in_mode != STX_IN_RAW) {
    set_error("stx_conv2d: the fused Gram-backward phase needs a raw-input conv");
    return STX_E_INVALID;
  }
  if (p.up_dp && (!p.up_z || p.ho < 2 || p.wo < 2)) {
    set_error("stx_conv2d: unpool epilogue needs up_z");
    return STX_E_INVALID;
  }
  if (p.pool_sum &&
      (!p.pool_out || !p.wt16 || p.wt16 == (const void*)1 || p.ks != 3 || p.pad != 1 ||
       p.stride != 1 || p.cin < 16 || p.cout <= 4 || p.wo <= 32 || (p.ho | p.wo) & 1 ||
       p.mask || p.aux || p.accumulate || p.acc_scale || p.up_dp || p.p2_z || p.relu_out ||
       p.gram_part || p.out_amax || p.wt_batch_stride)) {
    set_error("stx_conv2d: pool_sum needs pool_out on the split path (3x3 stride 1, wo > 32, "
              "even output dims) and the plain epilogue");
    return STX_E_INVALID;
  }
  if (p.gram_cnt && (!p.gram_part || (reinterpret_cast<uintptr_t>(p.gram_part) & 15) ||
                     (long long)stx_conv_gram_tiles(&p) * 16384 >= (1ll << 31))) {
    set_error("stx_conv2d: gram_cnt needs a 16-byte aligned gram_part slab (< 2 GB per image)");
    return STX_E_INVALID;
  }
  if (p.gram_part && !stx_conv_gram_tiles(&p)) {
    set_error("stx_conv2d: fused Gram partials need the split path, stride 1, cout 64 or 128, "
              "wo > 32 and the plain epilogue");
    return STX_E_INVALID;
  }
  if (p.gram_part && p.cout == 128 && 3LL * stx_conv_gram_tiles(&p) * 16384 >= (1ll << 31)) {
    set_error("stx_conv2d: 128-channel Gram partials per image >= 2 GB");
    return STX_E_INVALID;
  }
  if (p.gram_cnt && p.cout != 64) {
    set_error("stx_conv2d: gram_cnt (grouped Gram sums) needs cout 64");
    return STX_E_INVALID;
  }
  if (p.wt16_up &&
      (p.in_mode != STX_IN_UPSAMPLE2 || !p.wt16 || p.wt16 == (const void*)1 || p.ks != 3 ||
       p.pad != 1 || p.stride != 1 || p.cin < 16 || p.cout <= 4 || p.wo <= 32 ||
       p.hv != 2 * p.h || p.wv != 2 * p.w ||  // (the 2x2 parity taps assume the full x2 image)
       p.wt_batch_stride || p.mask || p.aux || p.accumulate || p.acc_scale || p.up_dp ||
       p.p2_z || p.pool_out || p.pool_sum || p.gram_part)) {
    set_error("stx_conv2d: wt16_up needs an upsampled-input split conv (3x3 stride 1, wo > 32, "
              "virtual size exactly 2h x 2w) with the plain epilogue (bias / relu_out / out_amax)");
    return STX_E_INVALID;
  }
  // y = NULL with pool_out: only the pooled output is written (the VGG content target's
  // conv1_2: nothing reads Z2 there) -- the split path's plain epilogue only
  if (!p.y && (!p.wt16 || p.wt16 == (const void*)1 || p.pool_sum || p.mask || p.aux ||
               p.accumulate || p.acc_scale || p.up_dp || p.p2_z || p.gram_part || p.mse_ref ||
               p.unpool_out || p.stride != 1)) {
    set_error("stx_conv2d: y = NULL (pool_out only) needs the split path's plain epilogue");
    return STX_E_INVALID;
  }
  if (p.unpool_out &&
      (!p.wt16 || p.wt16 == (const void*)1 || !p.w_amax || !p.in_amax || p.wt16_up || p.ks != 3 ||
       p.pad != 1 || p.stride != 1 || p.in_mode != STX_IN_RAW || p.cin < 16 ||
       (p.cout != 64 && p.cout != 128) || p.cout_pad != p.cout || p.p2_c != p.cout || !p.up_z ||
       !p.p2_wt || !p.p2_amax || !p.p2_wt_amax || p.p2_z || p.up_dp || p.mask || p.accumulate ||
       p.acc_scale || p.relu_out || p.bias || p.pool_out || p.pool_sum || p.gram_part ||
       p.gram_cnt || p.mse_ref || p.wt_batch_stride || p.wo % 32 || p.ho % 4 ||
       4LL * p.cout * 4 * p.ho * p.wo >= (long long)BUF_OOB / 2)) {
    set_error("stx_conv2d: unpool_out needs a raw-input split 3x3 stride-1 data gradient with "
              "cout 64 or 128 (= p2_c = cout_pad), wo %% 32 == 0, ho %% 4 == 0, up_z / p2_wt / "
              "p2_amax / p2_wt_amax, and no epilogue term but aux");
    return STX_E_INVALID;
  }
  if ((p.mse_ref || p.mse_parts) && (!p.mse_ref || !p.mse_parts || !p.gram_part || p.cout != 128)) {
    set_error("stx_conv2d: mse_ref / mse_parts go together, with gram_part on a 128-channel tap");
    return STX_E_INVALID;
  }
  // fp16 hi/lo split MFMA path (conv16.hip) for the 3x3 stride-1 layers it covers;
  // other shapes keep the fp32 MFMA kernels (wt is always required)
  if (p.wt16 && p.ks == 3 && p.pad == 1 && p.cout > 4 && p.cin >= 16 &&
      (p.stride == 1 || (p.stride == 2 && p.in_mode == STX_IN_RAW)) && p.wt_batch_stride == 0) {
    if (!p.w_amax || !p.in_amax || (p.p2_z && !p.p2_amax)) {
      set_error("stx_conv2d: the wt16 path needs w_amax, in_amax (and p2_amax with p2_z)");
      return STX_E_INVALID;
    }
    return conv2d_f16x3(p, st);
  }
  // 1x1 conv with per-image weights (Gram backward) as the split phase alone
  if (p.wt16 == (const void*)1 && p.ks == 1 && p.stride == 1 && p.pad == 0 &&
      p.wt_batch_stride != 0 && !p.p2_z) {
    if (!p.in_amax || p.mask || p.in_mode != STX_IN_RAW) {
      set_error("stx_conv2d: split 1x1 mode needs in_amax, no mask, raw input");
      return STX_E_INVALID;
    }
    if ((p.cin == 64 || p.cin == 128 || (p.cin == 256 && !p.up_dp)) && p.cout == p.cin &&
        p.cout_pad >= p.cin &&
        p.ho % 2 == 0 && p.wo % 16 == 0 && !p.bias && !p.accumulate && !p.relu_out &&
        (!p.up_dp || p.up_z == p.x) && (uint64_t)p.cin * p.ho * p.wo * 4 < (1ull << 31)) {
      Gb16 g{p.wt, p.wt_batch_stride, p.cout_pad, p.x, p.in_amax, p.acc_scale, p.up_dp,
             p.aux, p.aux_scale, p.y, p.out_amax, p.ho, p.wo};
      return gram_bwd16_launch(g, p.n, p.cin, st);
    }
    stx_conv_params q = p;
    q.p2_z = p.x;
    q.p2_wt = p.wt;
    q.p2_c = p.cin;
    q.p2_wt_batch_stride = p.wt_batch_stride;
    q.p2_scale = p.acc_scale;
    q.p2_amax = p.in_amax;
    q.acc_scale = nullptr;
    q.cin = 0;
    q.wt_batch_stride = 0;
    q.pad = 1;
    q.ks = 3;
    q.hv = p.ho;
    q.wv = p.wo;
    q.wt16 = nullptr;
    return conv2d_f16x3(q, st);
  }
  if (p.pool_out) {
    set_error("stx_conv2d: pool_out is only fused on the split (wt16) path");
    return STX_E_INVALID;
  }
  if (!p.wt) {  // only the split path may run without the fp32 slab
    set_error("stx_conv2d: this shape runs on the fp32 kernels and needs wt");
    return STX_E_INVALID;
  }
  {  // 3 input channels (VGG conv1_1, ITN conv0, conv22's data gradient)
    static const bool few_off = STX_KNOB("STX_FEWIN", 1) == 0;
    int rc = few_off ? -1 : conv2d_conv9(p, st);  // the ITN's 9x9 layers, split MFMA
    if (rc >= 0) return rc;
    rc = few_off ? -1 : conv2d_fewin(p, st);
    if (rc >= 0) return rc;
    rc = few_off ? -1 : conv2d_fewout(p, st);
    if (rc >= 0) return rc;
  }
  if (p.cout <= 4 && p.stride == 1 && (p.in_mode == STX_IN_RAW || p.in_mode == STX_IN_RELU) &&
      (p.ks == 3 || p.ks == 9) && !p.p2_z && !p.up_dp && !p.out_amax) {
    if (p.ks == 3) return launch_smallc<3, 8>(p, st);
    return launch_smallc<9, 8>(p, st);
  }
  const bool big = p.cout > 64;
  if (p.in_mode == STX_IN_RELU || p.in_mode == STX_IN_RELU_POOL2) {
    // fused relu / relu+pool loaders: the VGG 3x3 stride-1 layers
    if (p.ks != 3 || p.stride != 1 || p.cin_pad % 8) {
      set_error("stx_conv2d: relu/pool input modes need a 3x3 stride-1 conv with cin > 4");
      return STX_E_INVALID;
    }
    if (p.in_mode == STX_IN_RELU)
      return big ? dispatch_tw<3, 1, 128, STX_IN_RELU>(p, st)
                 : dispatch_tw<3, 1, 64, STX_IN_RELU>(p, st);
    return big ? dispatch_tw<3, 1, 128, STX_IN_RELU_POOL2>(p, st)
               : dispatch_tw<3, 1, 64, STX_IN_RELU_POOL2>(p, st);
  }
  constexpr int R = STX_IN_RAW;
  if (p.ks == 3 && p.stride == 1)
    return big ? dispatch_tw<3, 1, 128, R>(p, st) : dispatch_tw<3, 1, 64, R>(p, st);
  if (p.ks == 3 && p.stride == 2)
    return big ? dispatch_tw<3, 2, 128, R>(p, st) : dispatch_tw<3, 2, 64, R>(p, st);
  if (p.ks == 9 && p.stride == 1) return dispatch_tw<9, 1, 64, R>(p, st);
  if (p.ks == 1 && p.stride == 1)
    return big ? dispatch_tw<1, 1, 128, R>(p, st) : dispatch_tw<1, 1, 64, R>(p, st);
  set_error("stx_conv2d: unsupported ks=%d stride=%d", p.ks, p.stride);
  return STX_E_INVALID;
}
