// 3x3 stride-1 split-MFMA convolution with producer and consumer waves, persistent over
// a contiguous range of output tiles (the forward convs of the VGG-19 prefix and of the
// ImageTransformNet, and the plain data-gradient convs -- torchvision vgg19 Conv2d(3x3,
// p1) sliced by StyleNetwork, stransfer/network.py:246-314; the ImageTransformNet 3x3
// convs, :468-481, 525-609).
//
// Why: in the one-tile-per-block kernel (conv16.hip, v2 loop) every wave loads, splits,
// multiplies and stores; the two co-resident blocks of a CU start and end together, so
// their halo loads (prologue) and their output stores (epilogue: y, the pooled output,
// the Gram partials -- 100 MB at conv1_2 / 512^2) leave the matrix pipe idle for almost
// half of the launch, and a wave's stores are drained by the vmcnt waits of its own next
// loads.  Here one 512-thread block per CU splits the roles:
//   * waves 0-3 (consumers) own the 64-cout x 256-pixel accumulator tile and only read
//     LDS and issue MFMAs; their epilogue stores are never waited on (they issue no
//     global loads in the K loop), so tile t's stores drain under tile t+1's MFMAs;
//   * waves 4-7 (producers) load the next K step's halo third and weights, apply the
//     loader transform (ReLU / ReLU+MaxPool / nearest x2 / zero dilation), split them
//     into fp16 hi/lo 16-B operand units in double-buffered LDS, and compute the fused
//     Gram of the previous tile from its fp32 image in LDS, accumulated over the block's
//     tiles: ONE 64 x 64 partial per block instead of one per tile (4-8x fewer partial
//     bytes for stx_style_loss_from_parts to reduce).
// One __syncthreads per K step (a step = 16 input channels x one kernel row), one more per
// tile for the epilogue hand-off; max|y| is accumulated over the block's tiles and
// published with one atomic per block.
// The split arithmetic (s v = hi + lo, three MFMA products hi.hi + hi.lo + lo.hi, fp32
// accumulation, power-of-two de-scaling) and the LDS operand layout are conv16.hip's.
#include "common.h"
#include "conv_epi.h"
#include "../../include/stx.h"

namespace stx {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int TW>
struct PC {
  static constexpr int BM = 64, NPIX = 256, TH = NPIX / TW;
  static constexpr int RH = TH + 2, RW = TW + 2, NPOS = RH * RW;
  static constexpr int NITEM = 2 * NPOS;           // (channel group, halo position) units
  static constexpr int NIT = (NITEM + 255) / 256;  // per producer thread
  static constexpr int HB = 2 * NITEM * 16;        // one halo buffer: hi plane, lo plane
  static constexpr int WU = 3 * 4 * BM;            // weight units per step [tap][P][cg][co]
  static constexpr int NWU = WU / 256;
  static constexpr int WB = WU * 16;
  static constexpr int GZP = NPIX + 4;             // fp32 pitch of the Gram tile image
  static constexpr int OFF_W = 2 * HB;
  static constexpr int OFF_GZ = 2 * HB + 2 * WB;
  // the Gram tile image (64 x GZP fp32) or, for the Gram-backward data gradient, the
  // 64 KB register-major A.Z image followed by 2 KB of mask words
  static constexpr int GZ_BYTES = 64 * GZP * 4 > 64 * 1024 + 2048 ? 64 * GZP * 4 : 64 * 1024 + 2048;
  static constexpr int OFF_RED = OFF_GZ + GZ_BYTES;
  static constexpr int LDS_BYTES = OFF_RED + 64;
  static_assert(WU % 256 == 0, "weight units per thread");
  static_assert(LDS_BYTES <= 160 * 1024, "one block per CU");
};

struct PcArgs {
  int tiles_x, ntiles;  // per image
  int ncob;             // 64-cout blocks
  int per_block;        // items (tile, cout block) per block, contiguous
  int nitems;           // n * ntiles * ncob
  int gparts;           // Gram partials per image (blocks per image) when gram_part
};

// consumer epilogue: v = acc * scale + bias [, relu]; y stores (or the 2x2 sums of a
// pool_sum launch); the fused ReLU+MaxPool output; the fp32 tile image for the Gram;
// the running max|v| (IEEE bits)
template <int TW, bool RP, bool POOLSUM>
__device__ __forceinline__ void pc_epilogue(f32x16 (&acc)[2][2], const stx_conv_params& p, int n,
                                            int co0, int ty0, int tx0, int wn, int h, int l32,
                                            float scale, bool gram, float* gz, float* wred,
                                            uint32_t& vmax_run) {
  using C = PC<TW>;
  const size_t plane = (size_t)p.ho * p.wo;
  const int rows = max(0, p.cout - co0);
  // rows of this 64-cout block as a scalar (a VALU clamp would put the descriptor sizes in
  // VGPRs and every buffer access in a readfirstlane loop)
  const uint32_t nrows = (uint32_t)__builtin_amdgcn_readfirstlane(min(rows, 64));
  const uint32_t pb = (uint32_t)plane * 4u;
  const auto ry = make_srd(p.y + ((size_t)n * p.cout + co0) * plane, nrows * pb);
  uint32_t vo[2];
  bool lane_ok[2];
  int pix[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, RP, 2>(wn, j, l32, ty, tx);
    pix[j] = ty * TW + tx;
    const int oy = ty0 + ty, ox = tx0 + tx;
    lane_ok[j] = oy < p.ho && ox < p.wo;
    vo[j] = lane_ok[j] ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
  }
  float bias_r[2][16];
  {
    const auto rbias = make_srd(p.bias ? p.bias + co0 : p.y, p.bias ? nrows * 4u : 0u);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        bias_r[i][r] = buf_ld(rbias, (uint32_t)(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 4u);
  }
  const bool rows_full = rows >= 64;
  const bool relu = p.relu_out;
  uint32_t vmax_u = 0u;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint32_t lm = lane_ok[j] ? 0x7fffffffu : 0u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i * 32 + (r & 3) + 8 * (r >> 2);
        float v = fmaf(acc[i][j][r], scale, bias_r[i][r]);
        if (relu) v = fmaxf(v, 0.f);
        if constexpr (!POOLSUM) buf_st(ry, vo[j] + (uint32_t)row * pb, v);
        acc[i][j][r] = v;
        uint32_t m = lm;
        if (!rows_full) m = (row + 4 * h < rows) ? m : 0u;
        vmax_u = max(vmax_u, __float_as_uint(v) & m);
        if (gram) gz[(row + 4 * h) * C::GZP + pix[j]] = lane_ok[j] ? v : 0.f;
      }
    }
  }
  if constexpr (RP) if (p.pool_out) {
    const int hp = p.ho >> 1, wp = p.wo >> 1;
    const int py = (ty0 + (wn >> 1) * 2) >> 1;
    const int px = (tx0 + (wn & 1) * 32 + l32) >> 1;
    const bool ok = py < hp && px < wp && !(l32 & 1);
    const uint32_t ppb = (uint32_t)hp * (uint32_t)wp * 4u;
    const auto rp = make_srd(p.pool_out + ((size_t)n * p.cout + co0) * hp * wp, nrows * ppb);
    const uint32_t po = ok ? (uint32_t)(4 * h * hp * wp + py * wp + px) * 4u : BUF_OOB;
    if constexpr (POOLSUM) {
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
    } else {
      auto rb = [](float v) -> uint32_t {
        const int b = __float_as_int(v);
        const uint32_t a = (uint32_t)b & 0x7fffffffu;
        return a > 0x7f800000u ? a : (uint32_t)max(b, 0);  // NaN stays NaN (sign dropped)
      };
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t m2 = max(rb(acc[i][0][r]), rb(acc[i][1][r]));
          const uint32_t mp = (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, 0xB1, 0xF, 0xF, false);
          const int row = i * 32 + (r & 3) + 8 * (r >> 2);
          buf_st(rp, po + (uint32_t)row * ppb, __uint_as_float(max(m2, mp)));
        }
    }
  }
  // wave max -> the Gram scale (this tile) and the running max|y| (the block)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vmax_u = max(vmax_u, (uint32_t)__shfl_xor((int)vmax_u, o, 64));
  if (gram && threadIdx.x % 64 == 0) wred[wn] = __uint_as_float(vmax_u);
  vmax_run = max(vmax_run, vmax_u);
}

// producers: k-steps [k0, k1) of the tile's upper-triangle Gram blocks (producer wave
// wp = 0..2 takes block (I, J)) from the fp32 tile image, split at the tile's scale
// 2^(15 - e); the de-scaled result is added to the block's running partial g_run
template <int TW>
__device__ __forceinline__ void pc_gram_steps(const float* gz, int wp, int h, int l32, int e,
                                              int k0, int k1, f32x16& g_tile) {
  using C = PC<TW>;
  const int I = wp == 2 ? 1 : 0, J = wp == 0 ? 0 : 1;
  const float sx = __builtin_ldexpf(1.f, 15 - e);
  const float* ra = gz + (I * 32 + l32) * C::GZP + 8 * h;
  const float* rb = gz + (J * 32 + l32) * C::GZP + 8 * h;
  auto split = [&](const float* src, f16x8& hi, f16x8& lo) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(src);
    const f32x4 b = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float v = (q < 4 ? a[q] : b[q - 4]) * sx;
      const _Float16 vh = (_Float16)v;
      hi[q] = vh;
      lo[q] = (_Float16)(v - (float)vh);
    }
  };
  for (int ks = k0; ks < k1; ++ks) {
    f16x8 ah, al, bh, bl;
    split(ra + ks * 16, ah, al);
    if (I != J) {
      split(rb + ks * 16, bh, bl);
    } else {
      bh = ah;
      bl = al;
    }
    g_tile = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, g_tile, 0, 0, 0);
    g_tile = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, g_tile, 0, 0, 0);
    g_tile = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, g_tile, 0, 0, 0);
  }
}

// Data-gradient epilogue with the fused Gram-backward phase (P2): the producers computed
// s2 A[n] . Z for this tile (register-major fp32 image in LDS, the same MFMA layout as
// this wave's accumulators) and the ReLU mask [Z > 0] as ballot words
// mw[wave][j][channel] (bit l32 = the pixel of lane l32 in N-tile j):
//   v = [Z > 0] (acc * scale * acc_scale) + s2 A.Z;  y = v;  running max|v|
template <int TW>
__device__ __forceinline__ void pc_epilogue_p2(f32x16 (&acc)[2][2], const stx_conv_params& p,
                                               int n, int co0, int ty0, int tx0, int wn, int h,
                                               int l32, float scale, const float* az,
                                               const uint32_t* mw, uint32_t& vmax_run) {
  const size_t plane = (size_t)p.ho * p.wo;
  const int rows = max(0, p.cout - co0);
  const uint32_t nrows = (uint32_t)__builtin_amdgcn_readfirstlane(min(rows, 64));
  const uint32_t pb = (uint32_t)plane * 4u;
  const auto ry = make_srd(p.y + ((size_t)n * p.cout + co0) * plane, nrows * pb);
  const float sc = scale * (p.acc_scale ? *p.acc_scale : 1.f);
  const bool masked = p.mask != nullptr;
  const int lane = threadIdx.x & 63;
  uint32_t vmax_u = 0u;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, true, 2>(wn, j, l32, ty, tx);
    const int oy = ty0 + ty, ox = tx0 + tx;
    const bool ok = oy < p.ho && ox < p.wo;
    const uint32_t vo = ok ? (uint32_t)(4 * h * (int)plane + oy * p.wo + ox) * 4u : BUF_OOB;
    const uint32_t lm = ok ? 0x7fffffffu : 0u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(
            az + ((((wn * 2 + i) * 2 + j) * 4 + q) * 64 + lane) * 4);
        const uint4 mq = *reinterpret_cast<const uint4*>(
            mw + (wn * 2 + j) * 64 + i * 32 + 8 * q + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * q + e;
          const int row = i * 32 + (r & 3) + 8 * (r >> 2);
          const uint32_t word = e == 0 ? mq.x : e == 1 ? mq.y : e == 2 ? mq.z : mq.w;
          float v = acc[i][j][r] * sc;
          if (masked && !((word >> l32) & 1u)) v = 0.f;
          v += t[e];
          buf_st(ry, vo + (uint32_t)row * pb, v);
          uint32_t m = lm;
          if (row + 4 * h >= rows) m = 0u;
          vmax_u = max(vmax_u, __float_as_uint(v) & m);
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) vmax_u = max(vmax_u, (uint32_t)__shfl_xor((int)vmax_u, o, 64));
  vmax_run = max(vmax_run, vmax_u);
}

template <int TW, int LM, bool POOLSUM, bool P2 = false>
__global__ void __launch_bounds__(512, 1)
conv3x3_pc_kernel(stx_conv_params p, PcArgs a) {
  static_assert(!P2 || (TW == 64 && LM == STX_IN_RAW && !POOLSUM), "P2: raw-input dgrad");
  using C = PC<TW>;
  constexpr bool RP = TW == 64;  // row-pair tiles (fused pool output / pool_sum)
  constexpr int BM = C::BM;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS_BYTES];
  float* gz = reinterpret_cast<float*>(smem + C::OFF_GZ);
  float* red = reinterpret_cast<float*>(smem + C::OFF_RED);

  const int tid = threadIdx.x;
  // the wave index as a scalar: the role branch below is wave-uniform, so buffer
  // descriptors built inside it stay in SGPRs (no readfirstlane waterfall loops)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int h = lane >> 5, l32 = lane & 31;
  const bool consumer = wave < 4;
  const int item0 = blockIdx.x * a.per_block;
  const int nit = min(a.nitems, item0 + a.per_block) - item0;
  if (nit <= 0) return;
  const bool gram = !P2 && p.gram_part != nullptr;

  const int nchunks = cdiv(p.cin, 16);
  const int S = 3 * nchunks;           // K steps per item
  const int gtot = nit * S;
  const int ex = amax_exp(read_amax(p.in_amax));
  const int ew = amax_exp(read_amax(p.w_amax));
  const float sx = __builtin_ldexpf(1.f, 15 - ex);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);
  const int plane_in = p.h * p.w;
  const uint32_t pb = (uint32_t)plane_in * 4u, wrow = 4u * (uint32_t)p.w;
  const int cout64 = rup(p.cout, 64);
  const uint32_t chunk_bytes = (uint32_t)(36 * cout64 * 16);
  const uint32_t step_bytes = (uint32_t)(12 * cout64 * 16);
  const int per_img = a.ntiles * a.ncob;

  auto decode = [&](int item, int& n, int& ty0, int& tx0, int& co0) {
    n = item / per_img;
    const int rem = item - n * per_img;
    const int tile = rem / a.ncob;
    co0 = (rem - tile * a.ncob) * BM;
    ty0 = (tile / a.tiles_x) * C::TH;
    tx0 = (tile % a.tiles_x) * TW;
  };

  if (!consumer) {
    // ------------------------------------------------------------------ producers
    const int pt = tid - 256;
    const int wp = wave - 4;
    const char* __restrict__ wt16 = reinterpret_cast<const char*>(p.wt16);
    uint32_t hoff[C::NIT];
    int h_item = -1, h_n = 0;
    auto halo_offsets = [&](int item) {
      if (item == h_item) return;
      h_item = item;
      int ty0, tx0, co0;
      decode(item, h_n, ty0, tx0, co0);
      const int vy0 = ty0 - 1, vx0 = tx0 - 1;
#pragma unroll
      for (int r = 0; r < C::NIT; ++r) {
        const int idx = pt + r * 256;
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
    // one halo part in flight: items r = part, part + 3 (NIT <= 6)
    static_assert(C::NIT <= 6, "two items per part");
    float hv[2][8];
    f32x4 wreg[C::NWU];
    auto ld_halo = [&](int q, int part) {
      const int item = item0 + q / nchunks, c = q % nchunks;
      halo_offsets(item);
      const int c0 = c * 16;
      const auto rs = make_srd(p.x + ((size_t)h_n * p.cin + c0) * plane_in,
                               (uint32_t)(p.cin - c0) * pb);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = part + 3 * t;
        if (r >= C::NIT) continue;
        uint32_t off = hoff[0];
#pragma unroll
        for (int rr = 1; rr < C::NIT; ++rr) off = r == rr ? hoff[rr] : off;
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
          const uint32_t o = off + (uint32_t)ch * pb;
          if (LM == STX_IN_RELU_POOL2)
            hv[t][ch] = fmaxf(fmaxf(buf_ld(rs, o), buf_ld(rs, o + 4)),
                              fmaxf(buf_ld(rs, o + wrow), buf_ld(rs, o + wrow + 4)));
          else
            hv[t][ch] = buf_ld(rs, o);
        }
      }
    };
    auto st_halo = [&](int buf, int part) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = part + 3 * t;
        if (r >= C::NIT) continue;
        const int idx = pt + r * 256;
        if (idx < C::NITEM) {
          f16x8 hi, lo;
#pragma unroll
          for (int ch = 0; ch < 8; ++ch) {
            float v = hv[t][ch];
            if (LM == STX_IN_RELU || LM == STX_IN_RELU_POOL2) v = fmaxf(v, 0.f);
            v *= sx;
            const _Float16 vh = (_Float16)v;
            hi[ch] = vh;
            lo[ch] = (_Float16)(v - (float)vh);
          }
          char* hb = smem + buf * C::HB;
          *reinterpret_cast<f16x8*>(hb + idx * 16) = hi;
          *reinterpret_cast<f16x8*>(hb + (C::NITEM + idx) * 16) = lo;
        }
      }
    };
    auto ld_w = [&](int g) {  // global step g
      const int item = item0 + g / S, s = g % S;
      int n, ty0, tx0, co0;
      decode(item, n, ty0, tx0, co0);
      const int chunk = s / 3, kh = s - 3 * chunk;
      const auto rw = make_srd(reinterpret_cast<const float*>(wt16 + (size_t)chunk * chunk_bytes +
                                                              (size_t)kh * step_bytes),
                               step_bytes);
#pragma unroll
      for (int q = 0; q < C::NWU; ++q) {
        const int u = pt + q * 256;
        const int seg = u / BM, co = u - seg * BM;
        wreg[q] = buf_ld4(rw, (uint32_t)((seg * cout64 + co0 + co) * 16));
      }
    };
    auto st_w = [&](int buf) {
      char* wbp = smem + C::OFF_W + buf * C::WB;
#pragma unroll
      for (int q = 0; q < C::NWU; ++q)
        *reinterpret_cast<f32x4*>(wbp + (pt + q * 256) * 16) = wreg[q];
    };
    const int nq = gtot / 3;  // chunks in the block's sequence
    // prologue: chunk 0 and step 0's weights staged; step 1's weights and part 0 of
    // chunk 1 in flight
    ld_w(0);
#pragma unroll
    for (int part = 0; part < 3; ++part) {
      ld_halo(0, part);
      st_halo(0, part);
    }
    st_w(0);
    if (gtot > 1) ld_w(1);
    if (nq > 1) ld_halo(1, 0);
    __syncthreads();

    f32x16 g_run, g_tile;
#pragma unroll
    for (int q = 0; q < 16; ++q) g_run[q] = 0.f;
    int g_e = 0;
    constexpr int SG = 4;  // the previous tile's Gram spread over its successor's first steps
    auto gram_flush = [&](int item) {
      // the block's partial of its image: slot = block index within the image
      int n, ty0, tx0, co0;
      decode(item, n, ty0, tx0, co0);
      const int slot = blockIdx.x % a.gparts;
      if (wp < 3) gram_store(p.gram_part + ((size_t)n * a.gparts + slot) * 4096, g_run, wp, h, l32);
#pragma unroll
      for (int q = 0; q < 16; ++q) g_run[q] = 0.f;
    };
    auto gram_part = [&](int k0, int k1) {
      if (wp < 3) pc_gram_steps<TW>(gz, wp, h, l32, g_e, k0, k1, g_tile);
    };
    // ---- P2: s2 A[n] . Z of the item's tile (K = p2_c channels, 16 per MFMA step),
    // this wave's 64 couts x 64 pixels in the consumer layout; fragments loaded one K
    // step of the conv ahead of their MFMAs; A's scale from max|s2 A| over the block
    // (wave maxima through red[8..11] across one barrier)
    const int KS = P2 ? cdiv(p.p2_c, 16) : 0;
    f32x16 acc2[2][2];
    float fa[2][8], fz[2][8];
    int p2_n = 0, p2_co0 = 0, p2_ty0 = 0, p2_tx0 = 0, p2_ea = 0;
    const float s2v = P2 && p.p2_scale ? *p.p2_scale : 1.f;
    const int p2_ez = P2 ? amax_exp(read_amax(p.p2_amax)) : 0;
    const size_t zplane = (size_t)p.ho * p.wo;
    auto p2_load = [&](int ks) {
      const float* A = p.p2_wt + (size_t)p2_n * p.p2_wt_batch_stride;
      const int c0 = 16 * ks + 8 * h;
      const auto ra = make_srd(A, (uint32_t)p.p2_c * (uint32_t)p.cout_pad * 4u);
      const auto rz = make_srd(p.p2_z + (size_t)p2_n * p.p2_c * zplane,
                               (uint32_t)p.p2_c * (uint32_t)zplane * 4u);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          fa[i][e] = buf_ld(ra, (uint32_t)((c0 + e) * p.cout_pad + p2_co0 + 32 * i + l32) * 4u);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int ty, tx;
        tile_pix<TW, RP, 2>(wp, j, l32, ty, tx);
        const int oy = p2_ty0 + ty, ox = p2_tx0 + tx;
        const uint32_t zo = (oy < p.ho && ox < p.wo) ? (uint32_t)(oy * p.wo + ox) * 4u : BUF_OOB;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          fz[j][e] = buf_ld(rz, zo == BUF_OOB ? BUF_OOB : zo + (uint32_t)((c0 + e) * zplane) * 4u);
      }
    };
    uint32_t* mwords = reinterpret_cast<uint32_t*>(smem + C::OFF_GZ + 64 * 1024);
    auto p2_mma = [&](int ks) {
      const float sa = __builtin_ldexpf(s2v, 15 - p2_ea), sz = __builtin_ldexpf(1.f, 15 - p2_ez);
      f16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fa[i][e] * sa;
          const _Float16 vh = (_Float16)v;
          ah[i][e] = vh;
          al[i][e] = (_Float16)(v - (float)vh);
        }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = fz[j][e] * sz;
          const _Float16 vh = (_Float16)v;
          bh[j][e] = vh;
          bl[j][e] = (_Float16)(v - (float)vh);
        }
      if (p.mask) {
        // [Z > 0] of channels 16 ks + e (lanes 0-31) and 16 ks + 8 + e (lanes 32-63) at
        // this wave's pixels: the consumer's mask words for output channels co0 ..
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const unsigned long long b = __ballot(fz[j][e] > 0.f);
            const int c_lo = 16 * ks + e - p2_co0, c_hi = c_lo + 8;
            if (lane == 0) {
              if (c_lo >= 0 && c_lo < 64) mwords[(wp * 2 + j) * 64 + c_lo] = (uint32_t)b;
              if (c_hi >= 0 && c_hi < 64) mwords[(wp * 2 + j) * 64 + c_hi] = (uint32_t)(b >> 32);
            }
          }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc2[i][j], 0, 0, 0);
          acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc2[i][j], 0, 0, 0);
          acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc2[i][j], 0, 0, 0);
        }
    };
    auto p2_begin = [&](int item) {
      int n, ty0, tx0, co0;
      decode(item, n, ty0, tx0, co0);
      p2_n = n;
      p2_co0 = co0;
      p2_ty0 = ty0;
      p2_tx0 = tx0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc2[i][j][r] = 0.f;
      // max|A[n][c][co0 .. co0 + 63]| over c < p2_c: this wave's quarter of the rows
      const float* A = p.p2_wt + (size_t)n * p.p2_wt_batch_stride;
      float m = 0.f;
      for (int idx = wp * 64 + lane; idx < p.p2_c * 16; idx += 256) {
        const int c = idx >> 4, q4 = idx & 15;
        const f32x4 v = *reinterpret_cast<const f32x4*>(A + (size_t)c * p.cout_pad + co0 + 4 * q4);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (lane == 0) red[8 + wp] = m;
    };
    auto p2_finish = [&]() {
      // de-scale, then the register-major image for the consumers
      const float ds = __builtin_ldexpf(1.f, p2_ea + p2_ez - 30);
      float* az = gz;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            f32x4 t;
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = acc2[i][j][4 * q + e] * ds;
            *reinterpret_cast<f32x4*>(az + ((((wp * 2 + i) * 2 + j) * 4 + q) * 64 + lane) * 4) = t;
          }
    };
    for (int g = 0; g < gtot; ++g) {
      const int it = g / S, s = g - it * S;
      if (gram && it > 0 && s < SG) {
        // the Gram of item it-1 (its fp32 image and wave maxima were written by the
        // consumers' epilogue before the last barrier)
        if (s == 0) {
          uint32_t m = 0u;
#pragma unroll
          for (int w = 0; w < 4; ++w) m = max(m, __float_as_uint(red[w]));
          int e = 0;
          frexpf(__uint_as_float(m), &e);
          g_e = min(max(e, -60), 60);
#pragma unroll
          for (int q = 0; q < 16; ++q) g_tile[q] = 0.f;
        }
        const int ns = min(SG, S);
        if (s < ns) gram_part(16 * s / ns, 16 * (s + 1) / ns);
        if (s == ns - 1 && wp < 3) {
          const float inv2 = __builtin_ldexpf(1.f, 2 * g_e - 30);
#pragma unroll
          for (int q = 0; q < 16; ++q) g_run[q] = fmaf(g_tile[q], inv2, g_run[q]);
        }
      }
      if constexpr (P2) {
        // the A.Z phase of item it: step 0 starts it (A's wave maxima, fragment 0 in
        // flight), steps 1 .. KS multiply the fragment loaded one step earlier
        if (s == 0) {
          p2_begin(item0 + it);
        } else if (s <= KS && s < S - 1) {
          if (s == 1) {
            const float m = fmaxf(fmaxf(red[8], red[9]), fmaxf(red[10], red[11])) * fabsf(s2v);
            p2_ea = amax_exp(m);
          }
          p2_mma(s - 1);
        }
      }
      // stage step g+1: its weights (loaded last step) and part k of chunk q+1
      const int q = g / 3, k = g - 3 * q;
      if (g + 1 < gtot) st_w((g + 1) & 1);
      if (q + 1 < nq) st_halo((q + 1) & 1, k);
      if (g + 2 < gtot) ld_w(g + 2);
      const int qn = k < 2 ? q + 1 : q + 2;
      if (qn < nq) ld_halo(qn, (k + 1) % 3);
      if constexpr (P2) {
        if (s < KS && s + 2 < S) p2_load(s);  // multiplied at step s + 1 (< S - 1)
        if (s == S - 1) {
          // the fragments a short K loop left (loaded and multiplied here), then the
          // result handed to the consumers' epilogue of this item
          for (int ks = max(0, S - 2); ks < KS; ++ks) {
            if (ks == 0) {
              const float m = fmaxf(fmaxf(red[8], red[9]), fmaxf(red[10], red[11])) * fabsf(s2v);
              p2_ea = amax_exp(m);
            }
            p2_load(ks);
            p2_mma(ks);
          }
          p2_finish();
        }
      }
      __syncthreads();
      if (s == S - 1) __syncthreads();  // the consumers' epilogue of item it
    }
    if (gram) {
      uint32_t m = 0u;
#pragma unroll
      for (int w = 0; w < 4; ++w) m = max(m, __float_as_uint(red[w]));
      int e = 0;
      frexpf(__uint_as_float(m), &e);
      g_e = min(max(e, -60), 60);
#pragma unroll
      for (int q = 0; q < 16; ++q) g_tile[q] = 0.f;
      gram_part(0, 16);
      if (wp < 3) {
        const float inv2 = __builtin_ldexpf(1.f, 2 * g_e - 30);
#pragma unroll
        for (int q = 0; q < 16; ++q) g_run[q] = fmaf(g_tile[q], inv2, g_run[q]);
      }
      gram_flush(item0 + nit - 1);
    }
    __syncthreads();  // the consumers' max|y| is in red[4..7]
    if (tid == 256 && p.out_amax) {
      uint32_t m = 0u;
#pragma unroll
      for (int w = 0; w < 4; ++w) m = max(m, __float_as_uint(red[4 + w]));
      atomic_max_abs(p.out_amax + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(m));
    }
    return;
  }

  // -------------------------------------------------------------------- consumers
  const int wn = wave;
  int boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, RP, 2>(wn, j, l32, ty, tx);
    boff[j] = (h * C::NPOS + ty * C::RW + tx) * 16;
  }
  const int aoff = C::OFF_W + (h * BM + l32) * 16;
  uint32_t vmax_run = 0u;
  f32x16 acc[2][2];
  __syncthreads();  // the producers' prologue: step 0 staged
  for (int g = 0; g < gtot; ++g) {
    const int it = g / S, s = g - it * S;
    if (s == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
    const int kh = s % 3;
    const char* abase = smem + aoff + (g & 1) * C::WB;
    const int hbo = ((g / 3) & 1) * C::HB;
    const char* bbase[2] = {smem + boff[0] + hbo, smem + boff[1] + hbo};
    auto rdA = [&](int tl, int P, f16x8 (&av)[2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        av[i] = *reinterpret_cast<const f16x8*>(abase + (tl * 4 * BM + P * 2 * BM + i * 32) * 16);
    };
    auto rdB = [&](int tl, int P, f16x8 (&bv)[2]) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bv[j] = *reinterpret_cast<const f16x8*>(bbase[j] + (P * C::NITEM + kh * C::RW + tl) * 16);
    };
    auto phase = [&](const f16x8 (&av)[2], const f16x8 (&bv)[2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    f16x8 ahi[2], alo[2], bhi[2], blo[2];
    rdA(0, 0, ahi);
    rdB(0, 0, bhi);
#pragma unroll
    for (int tl = 0; tl < 3; ++tl) {
      rdB(tl, 1, blo);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      phase(ahi, bhi);
      rdA(tl, 1, alo);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      phase(ahi, blo);
      f16x8 nah[2], nbh[2];
      if (tl + 1 < 3) {
        rdA(tl + 1, 0, nah);
        rdB(tl + 1, 0, nbh);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      phase(alo, bhi);
      __builtin_amdgcn_sched_barrier(0);
      if (tl + 1 < 3) {
#pragma unroll
        for (int i = 0; i < 2; ++i) ahi[i] = nah[i];
#pragma unroll
        for (int j = 0; j < 2; ++j) bhi[j] = nbh[j];
      }
    }
    __syncthreads();  // this step's operand reads done; the next step is staged
    if (s == S - 1) {
      int n, ty0, tx0, co0;
      decode(item0 + it, n, ty0, tx0, co0);
      if constexpr (P2)
        pc_epilogue_p2<TW>(acc, p, n, co0, ty0, tx0, wn, h, l32, descale, gz,
                           reinterpret_cast<const uint32_t*>(smem + C::OFF_GZ + 64 * 1024),
                           vmax_run);
      else
        pc_epilogue<TW, RP, POOLSUM>(acc, p, n, co0, ty0, tx0, wn, h, l32, descale, gram, gz,
                                     red, vmax_run);
      __syncthreads();  // the Gram image and its wave maxima handed to the producers
    }
  }
  if (lane == 0) red[4 + wn] = __uint_as_float(vmax_run);
  __syncthreads();  // the producers publish max|y|
}

int cu_count() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  return cus;
}

}  // namespace

// The producer/consumer plan of a launch (pc_plan.ok false: conv16.hip's kernels run it):
// 256-pixel tiles (TW 64 for raw / ReLU input and the row-pair epilogues, else 32),
// the plain epilogue, at least two items per CU, and, with gram_part, whole images per
// block (per_block divides the tiles of an image)
struct PcPlan {
  bool ok = false;
  int tw = 64;
  PcArgs a{};
};

PcPlan pc_plan(const stx_conv_params& p, bool gram) {
  PcPlan r;
  if (!p.wt16 || p.wt16 == (const void*)1 || p.ks != 3 || p.stride != 1 || p.pad != 1 ||
      p.cin < 16 || p.cout <= 4 || p.wt_batch_stride || p.aux || p.accumulate || p.up_dp)
    return r;
  if (p.p2_z) {
    // the Gram-backward data gradient: raw input, the mask (if any) is [p2_z > 0] of the
    // output channels, plain epilogue otherwise
    if (p.in_mode != STX_IN_RAW || (p.mask && (p.mask != p.p2_z || p.p2_c != p.cout)) ||
        p.pool_out || gram || p.pool_sum || p.relu_out || p.bias || !p.p2_amax || !p.p2_wt ||
        p.wo <= 32)
      return r;
  } else if (p.mask || p.acc_scale) {
    return r;
  }
  const bool rowpair = p.pool_out || gram || p.p2_z;
  const int tw = (p.in_mode == STX_IN_RAW || rowpair || p.wo <= 32) ? 64 : 32;
  if (p.wo <= 32 && (rowpair || p.pool_sum)) return r;
  if (rowpair && p.in_mode != STX_IN_RAW && p.in_mode != STX_IN_RELU) return r;
  if (p.wo <= 32 && tw == 64) return r;  // narrow images: conv16.hip's 32 / 16-wide tiles
  const int th = 256 / tw;
  r.tw = tw;
  r.a.tiles_x = cdiv(p.wo, tw);
  r.a.ntiles = r.a.tiles_x * cdiv(p.ho, th);
  r.a.ncob = cdiv(p.cout, 64);
  r.a.nitems = p.n * r.a.ntiles * r.a.ncob;
  const int cus = cu_count();
  if (r.a.nitems < 2 * cus) return r;
  int k = cdiv(r.a.nitems, cus);
  if (gram) {
    if (p.cout != 64) return r;
    while (r.a.ntiles % k) ++k;  // every block within one image
    r.a.gparts = r.a.ntiles / k;
  }
  r.a.per_block = k;
  r.ok = true;
  return r;
}

// Gram partials per image a launch of these params with gram_part writes (0: not the
// producer/consumer kernel)
int conv16_pc_gram_parts(const stx_conv_params& p) {
  const PcPlan r = pc_plan(p, true);
  return r.ok ? r.a.gparts : 0;
}

template <int TW, int LM>
static int pc_launch(const stx_conv_params& p, const PcArgs& a, hipStream_t st) {
  const dim3 grid(cdiv(a.nitems, a.per_block));
  if (p.p2_z) {
    if constexpr (TW == 64 && LM == STX_IN_RAW) {
      hipLaunchKernelGGL((conv3x3_pc_kernel<TW, LM, false, true>), grid, dim3(512), 0, st, p, a);
      return check_launch("stx_conv2d(pc, Gram-backward phase)");
    }
    return -1;
  }
  if (p.pool_sum) {
    if constexpr (TW == 64 && LM == STX_IN_RAW) {
      hipLaunchKernelGGL((conv3x3_pc_kernel<TW, LM, true>), grid, dim3(512), 0, st, p, a);
      return check_launch("stx_conv2d(pc, pool_sum)");
    }
    return -1;
  }
  hipLaunchKernelGGL((conv3x3_pc_kernel<TW, LM, false>), grid, dim3(512), 0, st, p, a);
  return check_launch("stx_conv2d(pc)");
}

// -1: not covered (the caller runs conv16.hip's kernels)
int conv16_pc(const stx_conv_params& p, hipStream_t st) {
  const PcPlan r = pc_plan(p, p.gram_part != nullptr);
  if (!r.ok) return -1;
  if (r.tw == 64) {
    switch (p.in_mode) {
      case STX_IN_RAW: return pc_launch<64, STX_IN_RAW>(p, r.a, st);
      case STX_IN_RELU: return pc_launch<64, STX_IN_RELU>(p, r.a, st);
      default: return -1;
    }
  }
  switch (p.in_mode) {
    case STX_IN_RELU: return pc_launch<32, STX_IN_RELU>(p, r.a, st);
    case STX_IN_RELU_POOL2: return pc_launch<32, STX_IN_RELU_POOL2>(p, r.a, st);
    case STX_IN_UPSAMPLE2: return pc_launch<32, STX_IN_UPSAMPLE2>(p, r.a, st);
    case STX_IN_DILATE2: return pc_launch<32, STX_IN_DILATE2>(p, r.a, st);
    default: return -1;
  }
}

}  // namespace stx
