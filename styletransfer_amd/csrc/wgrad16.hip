// 3x3 stride-1 convolution weight gradient on the fp16 hi/lo split MFMA
// (v_mfma_f32_32x32x16_f16; numerics as conv16.hip: both operands scaled by a
// per-tensor power of two and split s*v = hi + lo, hi*hi + hi*lo + lo*hi in fp32).
//
//   dW[co][ci][kh][kw] = sum_{n,y,x} dY[n][co][y][x] * V[n][ci][y+kh-1][x+kw-1]
//
// For each tap row kh this is three GEMMs (kw = 0,1,2) with M = cout, N = cin and
// K = every output pixel, whose B operands are the same input row shifted by one
// pixel.  A wave owns one (32 couts, 32 cins, kh) unit over one K split and keeps
// the three kw accumulators: per 16-pixel step each lane loads 8 pixels of its dY
// row (two float4) and 10 pixels of its V row (two float4 + the two neighbours),
// splits them once and forms the three shifted B fragments in registers -- no LDS,
// no im2col.  The four waves of a block take four consecutive cin tiles of the
// same (cout tile, kh, split), so their identical dY loads hit L1.  Each wave
// writes its partial [split][kh][kw][co][ci]; a second kernel sums the splits in a
// fixed order (bit-reproducible; no float atomics).
//
// Reference: autograd of the ImageTransformNet 3x3 convs trained by static_train
// (stransfer/network.py:468-481, 525-609, :690-765).
//
// S2 (the stride-2 downsampling convs, stransfer/network.py:528-533): the same
// (32 couts, 32 cins, kh) units over output pixels; the lane loads 16 consecutive
// input pixels 2*x0 .. 2*x0+15 (four float4) plus 2*x0-1 and takes the even ones
// (kw = 1) and the odd ones shifted by zero / one (kw = 0 / 2) as packed pairs.
#include "common.h"

#include <mutex>
#include <unordered_map>
#include "../../include/stx.h"

namespace stx {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int wg_amax_exp(float a) {
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

struct Wg16 {
  int n, cin, h, w, cout, mode, hv, wv;  // x physical [n][cin][h][w]; V/dY are hv x wv
  int ncot, ncit, nsplit, steps, steps_per_split;
  int cout32, cin32;
  int ci2;  // cout <= 32: a wave takes 32 couts x 64 cins (two cin tiles), not 64 x 32
  int lds;  // wgrad16_lds_kernel geometry (cout 64/128, 64-cin tiles, 1 block per CU; 2: K2)
};

// Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one L2): renumber
// them so that consecutive logical blocks -- the units of one K split, which read the
// same dY rows -- sit on one XCD.  A bijection on [0, nb).
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7, x = b & 7, k = b >> 3;
  return x * per + min(x, rem) + k;
}

constexpr int WG16_S2 = 16;  // private mode: stride 2, pad 1, raw input (h = 2 hv, w = 2 wv)

template <int PF, bool S2, bool CI2 = false>
__global__ void __launch_bounds__(256)
wgrad16_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ ws,
               const float* __restrict__ x_amax, const float* __restrict__ dy_amax, Wg16 g) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  int unit = xcd_block(blockIdx.x, gridDim.x) * 4 + wave;
  const int cit = unit % g.ncit;
  unit /= g.ncit;
  const int cot = unit % g.ncot;  // pair of 32-cout tiles (64 couts)
  unit /= g.ncot;
  const int kh = unit % 3;
  const int split = unit / 3;
  if (split >= g.nsplit) return;  // (no barriers in this kernel)

  const int ex = wg_amax_exp(read_amax(x_amax)), ed = wg_amax_exp(read_amax(dy_amax));
  const float sv = __builtin_ldexpf(1.f, 15 - ex), sd = __builtin_ldexpf(1.f, 15 - ed);
  const float descale = __builtin_ldexpf(1.f, ex + ed - 30);

  const int co = cot * (CI2 ? 32 : 64) + l32, ci = cit * (CI2 ? 64 : 32) + l32;
  const bool co_ok = co < g.cout, co2_ok = co + 32 < g.cout, ci_ok = ci < g.cin;
  const bool ci2_ok = ci + 32 < g.cin;
  const int H = g.hv, W = g.wv, wsteps = W / 16;
  const bool relu = g.mode == STX_IN_RELU, up = g.mode == STX_IN_UPSAMPLE2;

  f32x16 acc[2][3];  // [cout tile][kw]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  const auto rdy = make_srd(dy, (uint32_t)((size_t)g.n * g.cout * H * W * 4u));
  const auto rx = make_srd(x, (uint32_t)((size_t)g.n * g.cin * g.h * g.w * 4u));
  struct Step {
    f32x4 a0, a1;   // dY[co][y][x0+8h .. +7]
    f32x4 c0, c1;   // dY[co+32][y][x0+8h .. +7]
    f32x4 b0, b1;   // V[ci][vy][x0+8h .. +7] (b1 unused for the upsample loader)
    float bl, br;   // V at x0+8h-1 and x0+8h+8
    f32x4 b2, b3;   // S2: x[ci][2y+kh-1][2x0+8 .. +15] (b0/b1: 2x0 .. 2x0+7; bl: 2x0-1)
    float bl2, br2; // CI2: neighbours of the second cin row (c0/c1 hold its 8 pixels)
  };
  // running (image, row, 16-pixel column step) of the next load: loads are issued in
  // step order, so no integer division per step
  int ln, ly, lxs;
  auto load = [&](Step& t) {
    const int n = ln, y = ly, x0 = lxs * 16 + 8 * h;
    if (++lxs == wsteps) {
      lxs = 0;
      if (++ly == H) {
        ly = 0;
        ++ln;
      }
    }
    // branch-free: invalid rows / taps / neighbours read 0 through the descriptors'
    // range check (predicated loads compiled to exec branches with vmcnt(0) joins,
    // which serialised the prefetch ring)
    const uint32_t oa = (uint32_t)((((size_t)n * g.cout + co) * H + y) * W + x0) * 4u;
    t.a0 = buf_ld4(rdy, co_ok ? oa : BUF_OOB);
    t.a1 = buf_ld4(rdy, co_ok ? oa + 16u : BUF_OOB);
    if constexpr (!CI2) {
      const uint32_t oc = oa + (uint32_t)32 * H * W * 4u;
      t.c0 = buf_ld4(rdy, co2_ok ? oc : BUF_OOB);
      t.c1 = buf_ld4(rdy, co2_ok ? oc + 16u : BUF_OOB);
    }
    if constexpr (S2) {
      const int vy = 2 * y + kh - 1;
      const bool bok = ci_ok && vy >= 0 && vy < g.h;
      const uint32_t ob = (uint32_t)((((size_t)n * g.cin + ci) * g.h + vy) * g.w + 2 * x0) * 4u;
      t.b0 = buf_ld4(rx, bok ? ob : BUF_OOB);
      t.b1 = buf_ld4(rx, bok ? ob + 16u : BUF_OOB);
      t.b2 = buf_ld4(rx, bok ? ob + 32u : BUF_OOB);
      t.b3 = buf_ld4(rx, bok ? ob + 48u : BUF_OOB);
      t.bl = buf_ld(rx, (bok && x0 > 0) ? ob - 4u : BUF_OOB);
      return;
    }
    const int vy = y + kh - 1;
    const bool bok = ci_ok && vy >= 0 && vy < H;
    if (!up) {
      const uint32_t ob = (uint32_t)((((size_t)n * g.cin + ci) * g.h + vy) * g.w + x0) * 4u;
      t.b0 = buf_ld4(rx, bok ? ob : BUF_OOB);
      t.b1 = buf_ld4(rx, bok ? ob + 16u : BUF_OOB);
      t.bl = buf_ld(rx, (bok && x0 > 0) ? ob - 4u : BUF_OOB);
      t.br = buf_ld(rx, (bok && x0 + 8 < W) ? ob + 32u : BUF_OOB);
      if constexpr (CI2) {  // the same row of cin + 32
        const bool bok2 = ci2_ok && vy >= 0 && vy < H;
        const uint32_t ob2 = ob + (uint32_t)32 * g.h * g.w * 4u;
        t.c0 = buf_ld4(rx, bok2 ? ob2 : BUF_OOB);
        t.c1 = buf_ld4(rx, bok2 ? ob2 + 16u : BUF_OOB);
        t.bl2 = buf_ld(rx, (bok2 && x0 > 0) ? ob2 - 4u : BUF_OOB);
        t.br2 = buf_ld(rx, (bok2 && x0 + 8 < W) ? ob2 + 32u : BUF_OOB);
      }
    } else {  // V[vy][vx] = x[vy/2][vx/2]; x0 is even
      const uint32_t ob =
          (uint32_t)((((size_t)n * g.cin + ci) * g.h + (vy >> 1)) * g.w + (x0 >> 1)) * 4u;
      t.b0 = buf_ld4(rx, bok ? ob : BUF_OOB);
      t.b1 = zero4;
      t.bl = buf_ld(rx, (bok && x0 > 0) ? ob - 4u : BUF_OOB);
      t.br = buf_ld(rx, (bok && x0 + 8 < W) ? ob + 16u : BUF_OOB);
      if constexpr (CI2) {
        const bool bok2 = ci2_ok && vy >= 0 && vy < H;
        const uint32_t ob2 = ob + (uint32_t)32 * g.h * g.w * 4u;
        t.c0 = buf_ld4(rx, bok2 ? ob2 : BUF_OOB);
        t.c1 = zero4;
        t.bl2 = buf_ld(rx, (bok2 && x0 > 0) ? ob2 - 4u : BUF_OOB);
        t.br2 = buf_ld(rx, (bok2 && x0 + 8 < W) ? ob2 + 16u : BUF_OOB);
      }
    }
  };
  // Packed split: pairs of scaled values -> (hi, lo) fp16 pairs with 2-wide VALU
  // (v_pk_mul/v_pk_add_f32, v_cvt_pkrtz_f16_f32: hi rounded toward zero, lo = v - hi
  // exactly as before, so hi + lo keeps ~22 significant bits); the three kw-shifted B
  // fragments reuse the packed pairs (kw = 0, 2) or one v_alignbit per dword (kw = 1).
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  auto split2 = [](f2 v, uint32_t& hi, uint32_t& lo) {
    const auto h = __builtin_amdgcn_cvt_pkrtz(v.x, v.y);
    hi = __builtin_bit_cast(uint32_t, h);
    const f2 hf = {(float)h[0], (float)h[1]};
    const f2 r = v - hf;
    lo = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.x, r.y));
  };
  auto compute = [&](const Step& t) {
    // A: dY rows co and co+32 (8 pixels each)
    uint32_t ahs[2][4], als[2][4];
    const f2 sd2 = {sd, sd};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f2 va = {q < 2 ? t.a0[2 * q] : t.a1[2 * q - 4], q < 2 ? t.a0[2 * q + 1] : t.a1[2 * q - 3]};
      const f2 vc = {q < 2 ? t.c0[2 * q] : t.c1[2 * q - 4], q < 2 ? t.c0[2 * q + 1] : t.c1[2 * q - 3]};
      split2(va * sd2, ahs[0][q], als[0][q]);
      if constexpr (!CI2) split2(vc * sd2, ahs[1][q], als[1][q]);
      else ahs[1][q] = als[1][q] = 0u;
    }
    u4v ahu[2], alu[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ahu[i] = u4v{ahs[i][0], ahs[i][1], ahs[i][2], ahs[i][3]};
      alu[i] = u4v{als[i][0], als[i][1], als[i][2], als[i][3]};
    }
    if constexpr (S2) {
      // even inputs 2(x0+e) -> kw = 1; odd sequence o = [2x0-1, 2x0+1, .., 2x0+15]:
      // o[0..7] -> kw = 0, o[1..8] -> kw = 2 (one v_alignbit per dword)
      const float xs[16] = {t.b0[0], t.b0[1], t.b0[2], t.b0[3], t.b1[0], t.b1[1], t.b1[2], t.b1[3],
                            t.b2[0], t.b2[1], t.b2[2], t.b2[3], t.b3[0], t.b3[1], t.b3[2], t.b3[3]};
      const float od[10] = {t.bl, xs[1], xs[3], xs[5], xs[7], xs[9], xs[11], xs[13], xs[15], 0.f};
      uint32_t eh[4], el[4], oh[5], ol[5];
      const f2 sv2 = {sv, sv};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f2 v = {xs[4 * q], xs[4 * q + 2]};
        split2(v * sv2, eh[q], el[q]);
      }
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const f2 v = {od[2 * q], od[2 * q + 1]};
        split2(v * sv2, oh[q], ol[q]);
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        uint32_t fh4[4], fl4[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (kw == 0) {
            fh4[q] = oh[q];
            fl4[q] = ol[q];
          } else if (kw == 1) {
            fh4[q] = eh[q];
            fl4[q] = el[q];
          } else {
            fh4[q] = __builtin_amdgcn_alignbit(oh[q + 1], oh[q], 16);
            fl4[q] = __builtin_amdgcn_alignbit(ol[q + 1], ol[q], 16);
          }
        }
        const u4v fhu = {fh4[0], fh4[1], fh4[2], fh4[3]}, flu = {fl4[0], fl4[1], fl4[2], fl4[3]};
        const h8 fh = __builtin_bit_cast(h8, fhu), fl = __builtin_bit_cast(h8, flu);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const h8 ah = __builtin_bit_cast(h8, ahu[i]), al = __builtin_bit_cast(h8, alu[i]);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fh, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fl, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, fh, acc[i][kw], 0, 0, 0);
        }
      }
      return;
    }
    // B: V[ci] at x0-1 .. x0+8 (10 values) -> 5 packed pairs
    const f2 sv2 = {sv, sv};
    auto bpairs = [&](const f32x4& b0, const f32x4& b1, float bl, float br, uint32_t (&ph)[5],
                      uint32_t (&pl)[5]) {
      float bv[10];
      bv[0] = bl;
      bv[9] = br;
      if (!up) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bv[1 + e] = b0[e];
          bv[5 + e] = b1[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[1 + 2 * e] = bv[2 + 2 * e] = b0[e];
      }
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        f2 v = {bv[2 * q], bv[2 * q + 1]};
        if (relu) {
          v.x = relu_bits(v.x);
          v.y = relu_bits(v.y);
        }
        split2(v * sv2, ph[q], pl[q]);
      }
    };
    // kw-shifted fragments: kw = 0, 2 reuse the pairs, kw = 1 takes halves (2q+1, 2q+2)
    auto kwfrag = [&](const uint32_t (&ph)[5], const uint32_t (&pl)[5], int kw, h8& fh, h8& fl) {
      uint32_t fh4[4], fl4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (kw == 0) {
          fh4[q] = ph[q];
          fl4[q] = pl[q];
        } else if (kw == 2) {
          fh4[q] = ph[q + 1];
          fl4[q] = pl[q + 1];
        } else {
          fh4[q] = __builtin_amdgcn_alignbit(ph[q + 1], ph[q], 16);
          fl4[q] = __builtin_amdgcn_alignbit(pl[q + 1], pl[q], 16);
        }
      }
      const u4v fhu = {fh4[0], fh4[1], fh4[2], fh4[3]}, flu = {fl4[0], fl4[1], fl4[2], fl4[3]};
      fh = __builtin_bit_cast(h8, fhu);
      fl = __builtin_bit_cast(h8, flu);
    };
    if constexpr (CI2) {  // one dY row against two cin rows: acc[cin tile][kw]
      uint32_t ph[2][5], pl[2][5];
      bpairs(t.b0, t.b1, t.bl, t.br, ph[0], pl[0]);
      bpairs(t.c0, t.c1, t.bl2, t.br2, ph[1], pl[1]);
      const h8 ah = __builtin_bit_cast(h8, ahu[0]), al = __builtin_bit_cast(h8, alu[0]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          h8 fh, fl;
          kwfrag(ph[i], pl[i], kw, fh, fl);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fh, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fl, acc[i][kw], 0, 0, 0);
          acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, fh, acc[i][kw], 0, 0, 0);
        }
      return;
    }
    uint32_t ph[5], pl[5];
    bpairs(t.b0, t.b1, t.bl, t.br, ph, pl);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      h8 fh, fl;
      kwfrag(ph, pl, kw, fh, fl);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const h8 ah = __builtin_bit_cast(h8, ahu[i]), al = __builtin_bit_cast(h8, alu[i]);
        acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fh, acc[i][kw], 0, 0, 0);
        acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, fl, acc[i][kw], 0, 0, 0);
        acc[i][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, fh, acc[i][kw], 0, 0, 0);
      }
    }
  };

  // four steps of loads in flight (HBM latency >> one step of 9 MFMAs)
  const int s0 = split * g.steps_per_split;
  const int s1 = min(g.steps, s0 + g.steps_per_split);
  {
    const int r0 = s0 / wsteps;
    lxs = s0 - r0 * wsteps;
    ln = r0 / H;
    ly = r0 - ln * H;
  }
  Step ring[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (s0 + k < s1) load(ring[k]);
  for (int s = s0; s < s1; s += PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (s + k < s1) {
        compute(ring[k]);
        if (s + k + PF < s1) load(ring[k]);
      }
    }
  }
  // partial [split][kh*3+kw][co (cout32)][ci (cin32)], descaled (exact)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int orow = CI2 ? cot * 32 : cot * 64 + i * 32;
      const int ocol = CI2 ? cit * 64 + i * 32 : cit * 32;
      float* out = ws + (((size_t)split * 9 + kh * 3 + kw) * g.cout32 + orow) * g.cin32 + ocol + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(size_t)row * g.cin32] = acc[i][kw][r] * descale;
      }
    }
}

// dW[co][ci][kh][kw] (+)= sum over splits (fixed order); thread -> (tap, co, ci), ci fastest
__global__ void wgrad16_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                      Wg16 g, int accumulate) {
  // 32-bit index math (the 64-bit div/mod is a long software sequence per element;
  // weights are < 2^31 / 9 elements)
  const int per = g.cout * g.cin;
  const int total = per * 9;
  const size_t sstride = (size_t)9 * g.cout32 * g.cin32;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int tap = i / per;
    const int rem = i - tap * per;
    const int co = rem / g.cin, ci = rem - co * g.cin;
    const float* src = ws + ((size_t)tap * g.cout32 + co) * g.cin32 + ci;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = 0;
    for (; k + 7 < g.nsplit; k += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += src[(size_t)(k + u) * sstride];
    }
    for (int u = 0; k < g.nsplit; ++k, ++u) a[u] += src[(size_t)k * sstride];
    const float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    float* d = dw + ((size_t)co * g.cin + ci) * 9 + tap;
    *d = accumulate ? *d + s : s;
  }
}

// Small outputs with many splits (the cout <= 64 layers: < 512 blocks of the kernel
// above, latency-bound): 4 thread groups per output each sum a contiguous quarter of
// the splits (8 running sums), combined in LDS as (q0 + q1) + (q2 + q3) -- fixed order
__global__ void __launch_bounds__(256)
wgrad16_reduce4_kernel(const float* __restrict__ ws, float* __restrict__ dw, Wg16 g,
                       int accumulate) {
  __shared__ float part[4][64];
  const int per = g.cout * g.cin;  // 32-bit index math (see wgrad16_reduce_kernel)
  const int total = per * 9;
  const int q = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.f;
  int tap = 0, co = 0, ci = 0;
  if (i < total) {
    tap = i / per;
    const int rem = i - tap * per;
    co = rem / g.cin;
    ci = rem - co * g.cin;
    const size_t sstride = (size_t)9 * g.cout32 * g.cin32;
    const float* src = ws + ((size_t)tap * g.cout32 + co) * g.cin32 + ci;
    const int quarter = (g.nsplit + 3) / 4;
    const int k0 = q * quarter, k1 = min(g.nsplit, k0 + quarter);
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int k = k0;
    for (; k + 7 < k1; k += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += src[(size_t)(k + u) * sstride];
    }
    for (int u = 0; k < k1; ++k, ++u) a[u] += src[(size_t)k * sstride];
    s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  }
  part[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && i < total) {
    const int j = threadIdx.x;
    const float t = (part[0][j] + part[1][j]) + (part[2][j] + part[3][j]);
    float* d = dw + ((size_t)co * g.cin + ci) * 9 + tap;
    *d = accumulate ? *d + t : t;
  }
}

// ---- parity classes of an upsampled-input conv (UpsampleConvLayer, stransfer/network.py
// :578-600).  Output pixel (2y + a, 2x + b) of the conv over the nearest x2 upsampled input
// reads input rows y - 1 + a + ry and columns x - 1 + b + rx (ry, rx in {0, 1}), so
//   dW'[a][b][ry][rx] = sum over the class-(a, b) outputs of dY * x[..][..]
// takes 4 instead of 9 MACs per output, and dW[kh][kw] = sum of dW' over the (a, ry) with
// kh in K(a, ry) and the (b, rx) with kw in K(b, rx) (K(0,0) = {0}, K(0,1) = {1,2},
// K(1,0) = {0,1}, K(1,1) = {2}) -- wgrad16up_reduce_kernel.  A wave owns (64 couts |
// CI2: 32 couts x 64 cins, 32 cins, ry, a) over a K split of the parity-a output rows; a
// step is 32 output columns of one row: the lane's 16 dY pixels split into the b = 0 / 1
// halves (evens / odds: two A fragments) and its 10 input pixels give the three shifted B
// fragments, shift b + rx (the kw fragments of the plain kernel).  Partials
// [split][a*6 + ry*3 + kw][co][ci] (the column taps assembled in registers).
constexpr int WG16_UPP = 17;  // private mode: the parity-class form of STX_IN_UPSAMPLE2

template <int PF, bool CI2>
__global__ void __launch_bounds__(256)
wgrad16up_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ ws,
                 const float* __restrict__ x_amax, const float* __restrict__ dy_amax, Wg16 g) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  int unit = xcd_block(blockIdx.x, gridDim.x) * 4 + wave;
  const int cit = unit % g.ncit;
  unit /= g.ncit;
  const int cot = unit % g.ncot;
  unit /= g.ncot;
  const int q4 = unit % 4, ry = q4 >> 1, a = q4 & 1;
  const int split = unit / 4;
  if (split >= g.nsplit) return;  // (no barriers in this kernel)

  const int ex = wg_amax_exp(read_amax(x_amax)), ed = wg_amax_exp(read_amax(dy_amax));
  const float sv = __builtin_ldexpf(1.f, 15 - ex), sd = __builtin_ldexpf(1.f, 15 - ed);
  const float descale = __builtin_ldexpf(1.f, ex + ed - 30);
  const int co = cot * (CI2 ? 32 : 64) + l32, ci = cit * (CI2 ? 64 : 32) + l32;
  const bool co_ok = co < g.cout, co2_ok = !CI2 && co + 32 < g.cout, ci_ok = ci < g.cin;
  const bool ci2_ok = CI2 && ci + 32 < g.cin;
  const int H = g.hv, W = g.wv, hin = g.h, win = g.w, wsteps = W / 32;

  f32x16 acc[2][4];  // [cout tile | CI2: cin tile][b * 2 + rx]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

  const auto rdy = make_srd(dy, (uint32_t)((size_t)g.n * g.cout * H * W * 4u));
  const auto rx_ = make_srd(x, (uint32_t)((size_t)g.n * g.cin * hin * win * 4u));
  struct Step {
    f32x4 d[2][4];  // dY rows co (, co + 32): output columns X0 + 16h .. +15
    f32x4 b[2][2];  // input rows ci (, ci + 32 for CI2): columns c0 + 1 .. c0 + 8
    float bl[2], br[2];  // columns c0 and c0 + 9 (c0 = X0 / 2 + 8h - 1)
  };
  int ln, ly, lxs;  // image, input row y (output row 2y + a), 32-column step
  auto load = [&](Step& t) {
    const int n = ln, y = ly, X0 = lxs * 32;
    if (++lxs == wsteps) {
      lxs = 0;
      if (++ly == hin) {
        ly = 0;
        ++ln;
      }
    }
    const int Y = 2 * y + a;
    const uint32_t oa = (uint32_t)((((size_t)n * g.cout + co) * H + Y) * W + X0 + 16 * h) * 4u;
#pragma unroll
    for (int k = 0; k < 4; ++k) t.d[0][k] = buf_ld4(rdy, co_ok ? oa + 16u * k : BUF_OOB);
    if constexpr (!CI2) {
      const uint32_t oc = oa + (uint32_t)32 * H * W * 4u;
#pragma unroll
      for (int k = 0; k < 4; ++k) t.d[1][k] = buf_ld4(rdy, co2_ok ? oc + 16u * k : BUF_OOB);
    }
    const int iy = y - 1 + a + ry, c1 = X0 / 2 + 8 * h;  // c1 = c0 + 1
#pragma unroll
    for (int j = 0; j < (CI2 ? 2 : 1); ++j) {
      const bool bok = (j ? ci2_ok : ci_ok) && iy >= 0 && iy < hin;
      const uint32_t ob =
          (uint32_t)((((size_t)n * g.cin + ci + 32 * j) * hin + iy) * win + c1) * 4u;
      t.b[j][0] = buf_ld4(rx_, bok ? ob : BUF_OOB);
      t.b[j][1] = buf_ld4(rx_, bok ? ob + 16u : BUF_OOB);
      t.bl[j] = buf_ld(rx_, (bok && c1 > 0) ? ob - 4u : BUF_OOB);
      t.br[j] = buf_ld(rx_, (bok && c1 + 8 < win) ? ob + 32u : BUF_OOB);
    }
  };
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  auto split2 = [](f2 v, uint32_t& hi, uint32_t& lo) {
    const auto hh = __builtin_amdgcn_cvt_pkrtz(v.x, v.y);
    hi = __builtin_bit_cast(uint32_t, hh);
    const f2 hf = {(float)hh[0], (float)hh[1]};
    const f2 r = v - hf;
    lo = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.x, r.y));
  };
  auto compute = [&](const Step& t) {
    const f2 sd2 = {sd, sd}, sv2 = {sv, sv};
    // A fragments [cout tile][b]: the even (b = 0) / odd (b = 1) columns of the lane's 16
    h8 ah[2][2], al[2][2];
#pragma unroll
    for (int i = 0; i < (CI2 ? 1 : 2); ++i) {
      float dv[16];
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) dv[4 * k + e] = t.d[i][k][e];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        uint32_t hs[4], ls[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f2 v = {dv[4 * q + b], dv[4 * q + 2 + b]};
          split2(v * sd2, hs[q], ls[q]);
        }
        ah[i][b] = __builtin_bit_cast(h8, u4v{hs[0], hs[1], hs[2], hs[3]});
        al[i][b] = __builtin_bit_cast(h8, u4v{ls[0], ls[1], ls[2], ls[3]});
      }
    }
    // B: input columns c0 .. c0 + 9 -> 5 packed pairs; shift s in {0, 1, 2} = b + rx
    uint32_t ph[2][5], pl[2][5];
#pragma unroll
    for (int j = 0; j < (CI2 ? 2 : 1); ++j) {
      float bv[10];
      bv[0] = t.bl[j];
      bv[9] = t.br[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bv[1 + e] = t.b[j][0][e];
        bv[5 + e] = t.b[j][1][e];
      }
#pragma unroll
      for (int q = 0; q < 5; ++q) split2(f2{bv[2 * q], bv[2 * q + 1]} * sv2, ph[j][q], pl[j][q]);
    }
    auto frag = [&](int j, int sft, h8& fh, h8& fl) {
      uint32_t fh4[4], fl4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (sft == 0) {
          fh4[q] = ph[j][q];
          fl4[q] = pl[j][q];
        } else if (sft == 2) {
          fh4[q] = ph[j][q + 1];
          fl4[q] = pl[j][q + 1];
        } else {
          fh4[q] = __builtin_amdgcn_alignbit(ph[j][q + 1], ph[j][q], 16);
          fl4[q] = __builtin_amdgcn_alignbit(pl[j][q + 1], pl[j][q], 16);
        }
      }
      fh = __builtin_bit_cast(h8, u4v{fh4[0], fh4[1], fh4[2], fh4[3]});
      fl = __builtin_bit_cast(h8, u4v{fl4[0], fl4[1], fl4[2], fl4[3]});
    };
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int rx = 0; rx < 2; ++rx)
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // cout tile (CI2: cin tile)
          h8 fh, fl;
          frag(CI2 ? i : 0, b + rx, fh, fl);
          const h8 xh = ah[CI2 ? 0 : i][b], xl = al[CI2 ? 0 : i][b];
          f32x16& c = acc[i][b * 2 + rx];
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, fh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, fl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, fh, c, 0, 0, 0);
        }
  };

  const int s0 = split * g.steps_per_split;
  const int s1 = min(g.steps, s0 + g.steps_per_split);
  {
    const int r0 = s0 / wsteps;
    lxs = s0 - r0 * wsteps;
    ln = r0 / hin;
    ly = r0 - ln * hin;
  }
  Step ring[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (s0 + k < s1) load(ring[k]);
  for (int s_ = s0; s_ < s1; s_ += PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      if (s_ + k < s1) {
        compute(ring[k]);
        if (s_ + k + PF < s1) load(ring[k]);
      }
    }
  }
  // the column taps assembled here (kw = 0: (b, rx) = (0,0) + (1,0); 1: (0,1) + (1,0);
  // 2: (0,1) + (1,1)), so the partial is [split][a*6 + ry*3 + kw][co (cout32)][ci (cin32)],
  // descaled (exact)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int orow = CI2 ? cot * 32 : cot * 64 + i * 32;
      const int ocol = CI2 ? cit * 64 + i * 32 : cit * 32;
      const int k0 = kw == 0 ? 0 : 1, k1 = kw == 2 ? 3 : 2;
      float* out = ws + (((size_t)split * 12 + a * 6 + ry * 3 + kw) * g.cout32 + orow) * g.cin32 +
                   ocol + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(size_t)row * g.cin32] = (acc[i][k0][r] + acc[i][k1][r]) * descale;
      }
    }
}

// dW[co][ci][kh][kw] (+)= sum over splits of the tap's two row-parity partials (fixed
// order: split quarters by thread group, a = 0 and a = 1 sums added last); 4 thread groups
// per output as wgrad16_reduce4_kernel
__global__ void __launch_bounds__(256)
wgrad16up_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, Wg16 g,
                        int accumulate) {
  __shared__ float part[4][64];
  const int per = g.cout * g.cin, total = per * 9;
  const int q = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  float s = 0.f;
  int tap = 0, co = 0, ci = 0;
  if (i < total) {
    tap = i / per;
    const int rem = i - tap * per;
    co = rem / g.cin;
    ci = rem - co * g.cin;
    const int kh = tap / 3, kw = tap - 3 * kh;
    // the two row partials of (kh, kw): (a = 0, ry = kh > 0) and (a = 1, ry = kh == 2)
    const size_t plane = (size_t)g.cout32 * g.cin32, sstride = 12 * plane;
    const size_t p0 = (size_t)((kh == 0 ? 0 : 1) * 3 + kw) * plane;
    const size_t p1 = (size_t)(6 + (kh == 2 ? 1 : 0) * 3 + kw) * plane;
    const float* src = ws + (size_t)co * g.cin32 + ci;
    const int quarter = (g.nsplit + 3) / 4;
    const int k0 = q * quarter, k1 = min(g.nsplit, k0 + quarter);
    float s0 = 0.f, s1 = 0.f;
    for (int k = k0; k < k1; ++k) {
      const float* sp = src + (size_t)k * sstride;
      s0 += sp[p0];
      s1 += sp[p1];
    }
    s = s0 + s1;
  }
  part[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && i < total) {
    const int j = threadIdx.x;
    const float t = (part[0][j] + part[1][j]) + (part[2][j] + part[3][j]);
    float* d = dw + ((size_t)co * g.cin + ci) * 9 + tap;
    *d = accumulate ? *d + t : t;
  }
}

// LDS-staged variant for the ITN's stride-1 layers with cout in {64, 128} and
// cin % 64 == 0 (the residual convs 128 -> 128, the up convs 128 -> 64): a block
// owns (all couts, 64 cins, kh) over a K split and steps through 16-pixel rows.
// The V row segment (64 cins x 18 pixels incl. the kw halo) is split ONCE per block
// into fp16 hi/lo and written to LDS as the three kw-shifted copies the B fragments
// need ([kw][plane][h][ci][8 fp16]: every fragment one conflict-free ds_read_b128);
// each wave keeps its own 32 couts of dY register-direct (A fragments, split in
// registers).  Double-buffered V images, one barrier per step, the next steps'
// global loads in flight.  Against wgrad16_kernel this removes the 4x redundant
// V conversion of its four waves and halves the number of K splits (1 block per CU
// instead of 8 waves), so the split-K slab the reduce kernel reads is half as big.
// CIB = cins per block (64; 128 for cout = 64, so each wave still owns two 32 x 32
// (co, ci) tiles: 18 MFMAs per barrier instead of 9)
// RL: ReLU input (compile time: no per-element select)
// K2: two groups of four waves per block (512 threads) take alternate 16-pixel steps of the
// block's K range, each with its own double-buffered V images and accumulators, so two waves
// per SIMD share the MFMA pipe (the 4-wave block has one: its staging, barrier and operand
// latency leave the pipe idle); group 1's sums are added to group 0's through LDS at the
// end (fixed order), the partial slab and the split count stay those of the 4-wave block.
template <int WCO, bool UP, int PF, int CIB = 64, bool RL = false, bool K2 = false>
__global__ void __launch_bounds__(K2 ? 512 : 256, 1)  // WCO = couts / 32; UP: nearest x2
wgrad16_lds_kernel(const float* __restrict__ x, const float* __restrict__ dy,  // upsampled
                   float* __restrict__ ws, const float* __restrict__ x_amax,   // input; PF + 1
                   const float* __restrict__ dy_amax, Wg16 g) {               // steps in flight
  constexpr int NCI = CIB / 64;            // staged cin rows per thread
  constexpr int NPAIR = WCO * 2 * NCI / 4;  // (co tile, ci tile) pairs per wave
  constexpr int NG = K2 ? 2 : 1;           // step groups
  static_assert((PF + 1) % 2 == 0, "ring slot k stages into V image k & 1");
  constexpr int IMG = 3 * 2 * 2 * CIB * 16;  // one V image: 12|24 KB
  constexpr int RED = K2 ? 4 * NPAIR * 3 * 16 * 64 * 4 : 0;  // group 1's accumulators
  constexpr int LDSB = 2 * NG * IMG > RED ? 2 * NG * IMG : RED;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  const int gk = K2 ? (int)(threadIdx.x >> 8) : 0;  // this thread's step group
  auto vimg = [&](int b) { return smem + (b * NG + gk) * IMG; };
  const int h = lane >> 5, l32 = lane & 31;
  int unit = xcd_block(blockIdx.x, gridDim.x);
  const int cit = unit % g.ncit;           // CIB-cin tile
  unit /= g.ncit;
  const int kh = unit % 3;
  const int split = unit / 3;
  const int ex = wg_amax_exp(read_amax(x_amax)), ed = wg_amax_exp(read_amax(dy_amax));
  const float sv = __builtin_ldexpf(1.f, 15 - ex), sd = __builtin_ldexpf(1.f, 15 - ed);
  const float descale = __builtin_ldexpf(1.f, ex + ed - 30);
  const int H = g.hv, W = g.wv, wsteps = W / 16;
  constexpr bool relu = RL;
  // this wave's (co tile, ci tile) pairs: WCO = 4 -> co tile = wave, ci tiles 0, 1;
  // WCO = 2 -> co tile = wave & 1, ci tile(s) (wave >> 1) * NCI + 0 .. NCI - 1
  const int cot = WCO == 4 ? wave : (wave & 1);
  const int co = cot * 32 + l32;
  // V staging: thread -> (ci = tid / 4, quad q = tid % 4): pixels x0 + 4q - 1 .. x0 + 4q + 4
  const int sci = tid >> 2, q = tid & 3;
  const int ci_g = cit * CIB + sci;        // (+ 64 r for row r < NCI)
  const auto rdy = make_srd(dy, (uint32_t)((size_t)g.n * g.cout * H * W * 4u));
  const auto rx = make_srd(x, (uint32_t)((size_t)g.n * g.cin * g.h * g.w * 4u));
  // byte offsets = a per-lane part (channel row, pixel within the step) + a per-step
  // uniform part (image, row, column step) -- 32-bit: the plan bounds every tensor < 2 GB
  const uint32_t la = (uint32_t)(co * H * W + 8 * h) * 4u;
  uint32_t lb[NCI];
#pragma unroll
  for (int r = 0; r < NCI; ++r)
    lb[r] = (uint32_t)((ci_g + 64 * r) * g.h * g.w + (UP ? 2 * q : 4 * q)) * 4u;
  const bool lft = q > 0;  // (x0 + 4q > 0 when x0 == 0)
  struct Ld {
    f32x4 a0, a1;        // dY[co][y][x0 + 8h .. +7]
    f32x4 v[NCI];        // V[ci][vy][x0 + 4q .. +3] (upsample: x[.][vy/2][(x0+4q)/2 .. +1] in v.xy)
    float vl[NCI], vr[NCI];  // V at x0 + 4q - 1 and x0 + 4q + 4
  };
  // Every load is issued unconditionally (steps past the split's end read zeros
  // through out-of-range offsets) so the wait counts stay exact: no branch around a
  // load, no vmcnt(0) before the LDS staging.
  int ln, ly, lxs, lleft;  // running (image, row, 16-px column step) of the next load, steps left
  auto load = [&](Ld& t) {
    const int n = ln, y = ly, x0 = lxs * 16;
    const bool live = lleft-- > 0;
#pragma unroll
    for (int i = 0; i < NG; ++i) {  // (this group's next step: NG steps on)
      if (++lxs == wsteps) {
        lxs = 0;
        if (++ly == H) {
          ly = 0;
          ++ln;
        }
      }
    }
    const uint32_t oa = (uint32_t)(((n * g.cout) * H + y) * W + x0) * 4u + la;
    t.a0 = buf_ld4(rdy, live ? oa : BUF_OOB);
    t.a1 = buf_ld4(rdy, live ? oa + 16u : BUF_OOB);
    const int vy = y + kh - 1;
    const bool rok = live && vy >= 0 && vy < H;
    const bool lok = rok && (x0 > 0 || lft);             // V[x0 + 4q - 1] exists
    const bool rgt = rok && x0 + 4 * q + 4 < W;          // V[x0 + 4q + 4] exists
    // (UP: V[vy][vx] = x[vy/2][vx/2]; x0 + 4q is even)
    const uint32_t sb = UP ? (uint32_t)(((n * g.cin) * g.h + (vy >> 1)) * g.w + (x0 >> 1)) * 4u
                           : (uint32_t)(((n * g.cin) * g.h + vy) * g.w + x0) * 4u;
#pragma unroll
    for (int r = 0; r < NCI; ++r) {
      const uint32_t ob = sb + lb[r];
      if constexpr (!UP) {
        t.v[r] = buf_ld4(rx, rok ? ob : BUF_OOB);
        t.vl[r] = buf_ld(rx, lok ? ob - 4u : BUF_OOB);
        t.vr[r] = buf_ld(rx, rgt ? ob + 16u : BUF_OOB);
      } else {
        t.v[r].x = buf_ld(rx, rok ? ob : BUF_OOB);
        t.v[r].y = buf_ld(rx, rok ? ob + 4u : BUF_OOB);
        t.vl[r] = buf_ld(rx, lok ? ob - 4u : BUF_OOB);
        t.vr[r] = buf_ld(rx, rgt ? ob + 8u : BUF_OOB);
      }
    }
  };
  // V -> the three kw-shifted fp16 hi/lo copies in LDS (thread: 4 pixels of NCI cins)
  auto stage = [&](const Ld& t, char* img) {
#pragma unroll
    for (int r = 0; r < NCI; ++r) {
      float v6[6];
      v6[0] = t.vl[r];
      v6[5] = t.vr[r];
      if constexpr (!UP) {
        v6[1] = t.v[r].x; v6[2] = t.v[r].y; v6[3] = t.v[r].z; v6[4] = t.v[r].w;
      } else {
        v6[1] = v6[2] = t.v[r].x;
        v6[3] = v6[4] = t.v[r].y;
      }
      _Float16 hi[6], lo[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        float v = v6[e];
        if (relu) v = fmaxf(v, 0.f);
        v *= sv;
        hi[e] = (_Float16)v;
        lo[e] = (_Float16)(v - (float)hi[e]);
      }
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      const int ci_l = sci + 64 * r;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        // copy kw, element e = 4q + j holds V[x0 + e + kw - 1] = v6[j + kw]
        const h4 ph = {hi[kw], hi[kw + 1], hi[kw + 2], hi[kw + 3]};
        const h4 pl = {lo[kw], lo[kw + 1], lo[kw + 2], lo[kw + 3]};
        const int base = (((kw * 2 + 0) * 2 + (q >> 1)) * CIB + ci_l) * 16 + (q & 1) * 8;
        const int base_l = (((kw * 2 + 1) * 2 + (q >> 1)) * CIB + ci_l) * 16 + (q & 1) * 8;
        *reinterpret_cast<h4*>(img + base) = ph;
        *reinterpret_cast<h4*>(img + base_l) = pl;
      }
    }
  };
  f32x16 acc[NPAIR][3];
#pragma unroll
  for (int i = 0; i < NPAIR; ++i)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;
  auto compute = [&](const Ld& t, const char* img) {
    h8 ah, al;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (e < 4 ? t.a0[e] : t.a1[e - 4]) * sd;
      ah[e] = (_Float16)v;
      al[e] = (_Float16)(v - (float)ah[e]);
    }
#pragma unroll
    for (int pi = 0; pi < NPAIR; ++pi) {
      // ci tile (32 cins) within the block's CIB
      const int ct = WCO == 4 ? pi : (wave >> 1) * NCI + (NPAIR > 1 ? pi : 0);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const h8 bh = *reinterpret_cast<const h8*>(img + (((kw * 2 + 0) * 2 + h) * CIB + ct * 32 + l32) * 16);
        const h8 bl = *reinterpret_cast<const h8*>(img + (((kw * 2 + 1) * 2 + h) * CIB + ct * 32 + l32) * 16);
        acc[pi][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[pi][kw], 0, 0, 0);
        acc[pi][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[pi][kw], 0, 0, 0);
        acc[pi][kw] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[pi][kw], 0, 0, 0);
      }
    }
  };
  const int s0 = split * g.steps_per_split;
  const int nst = min(g.steps, s0 + g.steps_per_split) - s0;  // >= 1
  {
    const int sg = s0 + gk;  // this group's first step (K2: steps sg, sg + 2, ...)
    const int r0 = sg / wsteps;
    lxs = sg - r0 * wsteps;
    ln = r0 / H;
    ly = r0 - ln * H;
    lleft = (nst - gk + NG - 1) / NG;
  }
  const int nit = (nst + NG - 1) / NG;  // steps per group (both groups: the same barriers)
  // steps run in groups of PF + 1 (a ring slot per step); a ragged last group computes
  // on zeros
  Ld ring[PF + 1];
#pragma unroll
  for (int k = 0; k <= PF; ++k) load(ring[k]);
  stage(ring[0], vimg(0));
  __syncthreads();
  for (int s = 0; s < nit; s += PF + 1) {
#pragma unroll
    for (int k = 0; k <= PF; ++k) {
      stage(ring[(k + 1) % (PF + 1)], vimg((k + 1) & 1));  // the next step's V image
      compute(ring[k], vimg(k & 1));
      load(ring[k]);  // step s + k + PF + 1
      __syncthreads();  // lgkmcnt(0) + s_barrier: the global loads stay in flight
    }
  }
  if constexpr (K2) {
    // group 1's accumulators -> LDS (the images are dead after the loop's last barrier);
    // group 0 adds them (acc0 + acc1) and writes the partial
    float* red = reinterpret_cast<float*>(smem);
    if (gk == 1) {
#pragma unroll
      for (int pi = 0; pi < NPAIR; ++pi)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            red[(((wave * NPAIR + pi) * 3 + kw) * 16 + r) * 64 + lane] = acc[pi][kw][r];
    }
    __syncthreads();
    if (gk == 1) return;
#pragma unroll
    for (int pi = 0; pi < NPAIR; ++pi)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          acc[pi][kw][r] += red[(((wave * NPAIR + pi) * 3 + kw) * 16 + r) * 64 + lane];
  }
  // partial [split][kh*3+kw][co (cout32)][ci (cin32)], descaled (exact)
#pragma unroll
  for (int pi = 0; pi < NPAIR; ++pi) {
    const int ct = WCO == 4 ? pi : (wave >> 1) * NCI + (NPAIR > 1 ? pi : 0);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      float* out = ws + (((size_t)split * 9 + kh * 3 + kw) * g.cout32 + cot * 32) * g.cin32 +
                   cit * CIB + ct * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
        out[(size_t)row * g.cin32] = acc[pi][kw][r] * descale;
      }
    }
  }
}

static bool wg16_lds_on() {
  static const bool on = STX_KNOB("STX_WG16_LDS", 1) != 0;
  return on;
}

// cout 64 on the LDS kernel (STX_WG16_LDS64=1): 64 cins per block measured 1.6x slower
// than the register-direct kernel, 128 cins per block (cin % 128 == 0) 5 % slower on the
// ITN up conv (188 vs 179 us, same box): off by default
static bool lds_on_64() {
  static const bool on = STX_KNOB("STX_WG16_LDS64", 0) != 0;
  return on;
}

typedef void (*Wg16Kernel)(const float*, const float*, float*, const float*, const float*, Wg16);

constexpr int WG16_K2_PF = 3;  // the K2 blocks' load ring

static int wg16_threads(const Wg16& g) { return g.lds == 2 ? 512 : 256; }

static int wg16_pf() {
  static const int pf = STX_KNOB("STX_WG16_PF", 4);
  return pf;
}

// the kernel a planned geometry launches (g.lds / g.ci2 / mode / cout / cin set)
static Wg16Kernel wg16_kernel(const Wg16& g) {
  if (g.lds) {
    const bool up = g.mode == STX_IN_UPSAMPLE2;
#ifdef STX_AB  // measured variants (not in the product build): load-ring depths, cout 64
    if (g.mode == STX_IN_RELU && g.cout != 128)
      return wgrad16_lds_kernel<2, false, 3, 64, true>;
    static const int lpf = STX_KNOB("STX_WG16_LPF", 3);
    if (g.cout == 128 && !up && lpf >= 5)
      return lpf >= 7 ? wgrad16_lds_kernel<4, false, 7> : wgrad16_lds_kernel<4, false, 5>;
    if (g.cout != 128) {
      if (g.cin % 128 == 0)
        return up ? wgrad16_lds_kernel<2, true, 3, 128> : wgrad16_lds_kernel<2, false, 3, 128>;
      return up ? wgrad16_lds_kernel<2, true, 3> : wgrad16_lds_kernel<2, false, 3>;
    }
#endif
    if (g.lds == 2)  // (K2: cout 128, not upsampled -- wg16_plan)
      return g.mode == STX_IN_RELU ? wgrad16_lds_kernel<4, false, WG16_K2_PF, 64, true, true>
                                   : wgrad16_lds_kernel<4, false, WG16_K2_PF, 64, false, true>;
    if (g.mode == STX_IN_RELU) return wgrad16_lds_kernel<4, false, 3, 64, true>;
    return up ? wgrad16_lds_kernel<4, true, 3> : wgrad16_lds_kernel<4, false, 3>;
  }
  if (g.mode == WG16_UPP) return g.ci2 ? wgrad16up_kernel<2, true> : wgrad16up_kernel<2, false>;
  if (g.ci2) return wgrad16_kernel<4, false, true>;
  if (g.mode == WG16_S2) return wgrad16_kernel<4, true>;
#ifdef STX_AB
  const int pf = wg16_pf();
  if (pf >= 8) return pf >= 12 ? wgrad16_kernel<12, false> : wgrad16_kernel<8, false>;
#endif
  return wgrad16_kernel<4, false>;
}

// resident blocks of `k` over the whole device (CUs x blocks per CU at `threads`);
// 256 x 1 when no device answers (the CPU-only build host sizing a workspace)
static int wg16_slots_query(Wg16Kernel k, int threads) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(k), threads,
                                                   0) != hipSuccess ||
      cus <= 0 || per <= 0) {
    (void)hipGetLastError();
    return 256;
  }
  return cus * per;
}

static int wg16_slots(Wg16Kernel k, int threads) {  // cached per kernel (plans run at every launch)
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(reinterpret_cast<const void*>(k));
  if (it != cache.end()) return it->second;
  const int v = wg16_slots_query(k, threads);
  cache.emplace(reinterpret_cast<const void*>(k), v);
  return v;
}

static bool wg16_plan(int n, int cin, int cout, int in_mode, int hv, int wv, Wg16& g) {
  if (wv % 16 != 0 || cin < 16 || cout < 16 || n <= 0 || hv <= 0) return false;
  // 32-bit buffer offsets over the whole dy / x tensors
  if ((size_t)n * std::max(cin, cout) * hv * wv * 4 >= (1ull << 31)) return false;
  if ((long long)cin * cout * 9 >= (1ll << 31)) return false;  // 32-bit reduce indices
  if (in_mode != STX_IN_RAW && in_mode != STX_IN_RELU && in_mode != STX_IN_UPSAMPLE2 &&
      in_mode != WG16_S2)
    return false;
  g.n = n;
  g.cin = cin;
  g.cout = cout;
  g.mode = in_mode;
  g.hv = hv;
  g.wv = wv;
  // STX_WG16_CI2=0: the 64 x 32 tiling for every cout
  static const bool ci2_on = STX_KNOB("STX_WG16_CI2", 1) != 0;
  g.ci2 = ci2_on && cout <= 32 && in_mode != WG16_S2;
  if (g.ci2) {  // 32 couts x two 32-cin tiles per wave (no all-zero second cout tile)
    g.ncot = 1;
    g.ncit = cdiv(cin, 64);
    g.cout32 = 32;
    g.cin32 = g.ncit * 64;
  } else {
    g.ncot = cdiv(cout, 64);  // a wave takes 64 couts (two 32-row MFMA tiles)
    g.ncit = cdiv(cin, 32);
    g.cout32 = g.ncot * 64;
    g.cin32 = g.ncit * 32;
  }
  g.steps = n * hv * (wv / 16);
  g.lds = wg16_lds_on() && (cout == 128 || (cout == 64 && lds_on_64())) && cin % 64 == 0 &&
          (in_mode == STX_IN_RAW || in_mode == STX_IN_RELU || in_mode == STX_IN_UPSAMPLE2);
  // (read per plan: A/B in one process; both forms run one block per CU, so the split
  // count and the workspace are the same)
  if (g.lds && cout == 128 && in_mode != STX_IN_UPSAMPLE2 && STX_KNOB("STX_WG16_K2", 1)) g.lds = 2;
  // the upsampled input as parity classes (4 instead of 9 MACs per output; STX_WG16_UPP=0:
  // the upsampled-row kernels): 32-column steps over the output rows of one row parity
  static const bool upp_on = STX_KNOB("STX_WG16_UPP", 1) != 0;
  if (upp_on && in_mode == STX_IN_UPSAMPLE2 && !g.lds && wv % 32 == 0 && hv % 2 == 0) {
    g.mode = WG16_UPP;
    g.steps = n * (hv / 2) * (wv / 32);
  }
  if (g.lds) {  // blocks of (all couts x 64 cins x kh) x K split: ~512 blocks
    g.ncot = 1;
    g.ncit = cout == 64 && cin % 128 == 0 ? cin / 128 : cin / 64;  // CIB
    g.cout32 = cout;
    g.cin32 = cin;
    g.ci2 = 0;
  }
  // K splits: as many as fill whole rounds of resident blocks (a ragged last round of a
  // few blocks costs a full block duration: 513 blocks at 256 slots ran 3 rounds)
  static const int rounds = std::max(1, STX_KNOB("STX_WG16_ROUNDS", 1));
  const int slots = rounds * wg16_slots(wg16_kernel(g), wg16_threads(g));
  // blocks per split: (kh x cin tiles) for the LDS kernel; 4 units (waves) per block
  // (parity classes: 4 (ry, a) units per cout / cin tile pair instead of 3 kh)
  const int kq = g.mode == WG16_UPP ? 4 : 3;
  int ns = g.lds ? slots / (3 * g.ncit) : slots * 4 / (kq * g.ncot * g.ncit);
  ns = std::max(1, std::min(ns, cdiv(g.steps, 8)));  // >= 8 steps per split
  g.steps_per_split = cdiv(g.steps, ns);
  g.nsplit = cdiv(g.steps, g.steps_per_split);
  return true;
}

}  // namespace stx

using namespace stx;

extern "C" size_t stx_conv2d_wgrad16_ws(int n, int cin, int cout, int in_mode, int hv, int wv) {
  Wg16 g;
  if (!wg16_plan(n, cin, cout, in_mode, hv, wv, g)) return 0;
  return (size_t)g.nsplit * (g.mode == WG16_UPP ? 12 : 9) * g.cout32 * g.cin32 * sizeof(float);
}

extern "C" int stx_conv2d_wgrad16(const float* x, const float* dy, float* dw, int accumulate,
                                  int n, int cin, int h, int w, int cout, int in_mode, int hv,
                                  int wv, const float* x_amax, const float* dy_amax, void* ws,
                                  size_t ws_bytes, void* stream) {
  Wg16 g;
  if (!x || !dy || !dw || !x_amax || !dy_amax || !wg16_plan(n, cin, cout, in_mode, hv, wv, g)) {
    set_error("stx_conv2d_wgrad16: unsupported shape/mode or NULL argument");
    return STX_E_INVALID;
  }
  g.h = h;
  g.w = w;
  if ((in_mode == STX_IN_UPSAMPLE2 && (hv != 2 * h || wv != 2 * w)) ||
      (in_mode == WG16_S2 && (h != 2 * hv || w != 2 * wv)) ||
      (in_mode != STX_IN_UPSAMPLE2 && in_mode != WG16_S2 && (hv != h || wv != w))) {
    set_error("stx_conv2d_wgrad16: virtual dims do not match the input mode");
    return STX_E_INVALID;
  }
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy)) & 15) {
    set_error("stx_conv2d_wgrad16: 16-byte aligned tensors required");
    return STX_E_INVALID;
  }
  const size_t need = stx_conv2d_wgrad16_ws(n, cin, cout, in_mode, hv, wv);
  if (!ws || ws_bytes < need) {
    set_error("stx_conv2d_wgrad16: workspace %zu < %zu", ws_bytes, need);
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int units = g.nsplit * (g.mode == WG16_UPP ? 4 : 3) * g.ncot * g.ncit;
  const int blocks = g.lds ? g.nsplit * 3 * g.ncit : cdiv(units, 4);
  hipLaunchKernelGGL(wg16_kernel(g), dim3(blocks), dim3(wg16_threads(g)), 0, st, x, dy,
                     (float*)ws, x_amax, dy_amax, g);
  const long long total = (long long)cout * cin * 9;
  if (g.mode == WG16_UPP) {
    hipLaunchKernelGGL(wgrad16up_reduce_kernel, dim3((int)((total + 63) / 64)), dim3(256), 0, st,
                       (const float*)ws, dw, g, accumulate);
    return check_launch("stx_conv2d_wgrad16 (parity classes)");
  }
  const int rblocks = (int)std::min<long long>((total + 255) / 256, 4096);
  if (rblocks < 512 && g.nsplit >= 32)
    hipLaunchKernelGGL(wgrad16_reduce4_kernel, dim3((int)((total + 63) / 64)), dim3(256), 0, st,
                       (const float*)ws, dw, g, accumulate);
  else
    hipLaunchKernelGGL(wgrad16_reduce_kernel, dim3(rblocks), dim3(256), 0, st, (const float*)ws,
                       dw, g, accumulate);
  return check_launch("stx_conv2d_wgrad16");
}

extern "C" size_t stx_conv2d_wgrad16_s2_ws(int n, int cin, int cout, int ho, int wo) {
  return stx_conv2d_wgrad16_ws(n, cin, cout, WG16_S2, ho, wo);
}

extern "C" int stx_conv2d_wgrad16_s2(const float* x, const float* dy, float* dw, int accumulate,
                                     int n, int cin, int h, int w, int cout, int ho, int wo,
                                     const float* x_amax, const float* dy_amax, void* ws,
                                     size_t ws_bytes, void* stream) {
  return stx_conv2d_wgrad16(x, dy, dw, accumulate, n, cin, h, w, cout, WG16_S2, ho, wo, x_amax,
                            dy_amax, ws, ws_bytes, stream);
}
