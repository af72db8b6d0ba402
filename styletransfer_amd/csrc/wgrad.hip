// Convolution weight gradient for gfx950 on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
//   dW[co][ci][kh][kw] = sum_{n,oy,ox} dY[n][co][oy][ox] * V[n][ci][oy*S-P+kh][ox*S-P+kw]
//
// GEMM view: M = cout, N = (ci,kh,kw), K = every output pixel of every image.
// A block owns a BM x BN output tile (BN covers CIS input channels x KS*KS taps)
// and one K-split (a contiguous run of (image, pixel-tile) pairs).  Per K tile it
// stages dY[BM][NPIX] (pitch NPIX+1) and the input halo [CIS][RH][RW] of the same
// pixels in LDS; lane j of an N tile keeps a fixed LDS offset for its (ci,kh,kw)
// column, so the B operand of K step s is halo[off_j + pixoff(s)] — no im2col.
// Split-K partial slabs are reduced in a fixed order by a second kernel
// (deterministic; no float atomics).
//
// Reference: autograd of the ImageTransformNet Conv2d layers trained by
// static_train (stransfer/network.py:520-611, :690-765).
#include "common.h"
#include "../../include/stx.h"

namespace stx {

__device__ float load_virtual_w(const float* __restrict__ xp, int mode, int cin, int h, int w,
                                int hv, int wv, int ci, int vy, int vx) {
  if (ci >= cin || vy < 0 || vx < 0 || vy >= hv || vx >= wv) return 0.f;
  const float* plane = xp + (size_t)ci * h * w;
  switch (mode) {
    case STX_IN_RAW:
      return plane[vy * w + vx];
    case STX_IN_RELU:
      return fmaxf(plane[vy * w + vx], 0.f);
    case STX_IN_RELU_POOL2: {
      const float* q = plane + (2 * vy) * w + 2 * vx;
      return fmaxf(fmaxf(fmaxf(q[0], q[1]), fmaxf(q[w], q[w + 1])), 0.f);
    }
    case STX_IN_UPSAMPLE2:
      return plane[(vy >> 1) * w + (vx >> 1)];
    default: {
      if ((vy | vx) & 1) return 0.f;
      const int sy = vy >> 1, sx = vx >> 1;
      if (sy >= h || sx >= w) return 0.f;
      return plane[sy * w + sx];
    }
  }
}

template <int KS, int S, int CIS, int WM, int WN, int NI, int NPIX, int TW>
struct WgCfg {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int BM = 32 * WM;
  static constexpr int BN = 32 * WN * NI;
  static constexpr int KK = KS * KS;
  static constexpr int TH = NPIX / TW;
  static constexpr int RH = (TH - 1) * S + KS;
  static constexpr int RW = (TW - 1) * S + KS;
  static constexpr int RWP = RW;
  static constexpr int CH = RH * RWP;
  static constexpr int HALO = CIS * RH * RW;
  static constexpr int NH = (HALO + NT - 1) / NT;
  static constexpr int DYP = NPIX + 1;
  static constexpr int DYN = BM * NPIX;
  static constexpr int ND = (DYN + NT - 1) / NT;
  static constexpr int LDS_FLOATS = CIS * CH + BM * DYP;
  static_assert(BN >= CIS * KK, "N tile must cover the chunk");
  static_assert((NPIX / 2) % TW == 0, "half K tile must be whole rows");
};

template <int KS, int S, int CIS, int WM, int WN, int NI, int NPIX, int TW>
__global__ void __launch_bounds__(64 * WM * WN)
wgrad_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ ws,
             int nimg, int cin, int h, int w, int cout, int pad, int mode, int hv, int wv, int ho,
             int wo, int tiles_x, int tiles_per_img, int nsplit) {
  using C = WgCfg<KS, S, CIS, WM, WN, NI, NPIX, TW>;
  __shared__ __attribute__((aligned(16))) float smem[C::LDS_FLOATS];
  float* halo = smem;
  float* ldy = smem + CIS * C::CH;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h2 = lane >> 5, l32 = lane & 31;
  const int wm = wave / WN, wn = wave % WN;
  const int split = blockIdx.x, cob = blockIdx.y, cc = blockIdx.z;
  const int co0 = cob * C::BM, c0 = cc * CIS;

  const long long ktiles = (long long)nimg * tiles_per_img;
  const long long kt_begin = ktiles * split / nsplit;
  const long long kt_end = ktiles * (split + 1) / nsplit;

  int boff[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int j = (wn * NI + ni) * 32 + l32;
    int off = 0;
    if (j < CIS * C::KK) {
      const int ci = j / C::KK, r = j % C::KK;
      off = ci * C::CH + (r / KS) * C::RWP + (r % KS);
    }
    boff[ni] = off + h2 * ((NPIX / 2) / TW) * S * C::RWP;
  }
  const int aoff = (wm * 32 + l32) * C::DYP + h2 * (NPIX / 2);

  f32x16 acc[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ni][r] = 0.f;

  float hreg[C::NH], dreg[C::ND];
  auto fetch = [&](long long kt) {
    const int n = (int)(kt / tiles_per_img);
    const int t = (int)(kt % tiles_per_img);
    const int ty0 = (t / tiles_x) * C::TH, tx0 = (t % tiles_x) * TW;
    const float* xn = x + (size_t)n * cin * h * w;
    const int vy0 = ty0 * S - pad, vx0 = tx0 * S - pad;
#pragma unroll
    for (int i = 0; i < C::NH; ++i) {
      const int idx = tid + i * C::NT;
      float v = 0.f;
      if (idx < C::HALO) {
        const int ci = idx / (C::RH * C::RW);
        const int rem = idx - ci * (C::RH * C::RW);
        const int r = rem / C::RW, c = rem - r * C::RW;
        v = load_virtual_w(xn, mode, cin, h, w, hv, wv, c0 + ci, vy0 + r, vx0 + c);
      }
      hreg[i] = v;
    }
    const float* dyn = dy + (size_t)n * cout * ho * wo;
#pragma unroll
    for (int i = 0; i < C::ND; ++i) {
      const int idx = tid + i * C::NT;
      float v = 0.f;
      if (idx < C::DYN) {
        const int row = idx / NPIX, px = idx % NPIX;
        const int oy = ty0 + px / TW, ox = tx0 + px % TW;
        const int co = co0 + row;
        if (co < cout && oy < ho && ox < wo) v = dyn[((size_t)co * ho + oy) * wo + ox];
      }
      dreg[i] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < C::NH; ++i) {
      const int idx = tid + i * C::NT;
      if (idx < C::HALO) {
        const int ci = idx / (C::RH * C::RW);
        const int rem = idx - ci * (C::RH * C::RW);
        const int r = rem / C::RW, c = rem - r * C::RW;
        halo[ci * C::CH + r * C::RWP + c] = hreg[i];
      }
    }
#pragma unroll
    for (int i = 0; i < C::ND; ++i) {
      const int idx = tid + i * C::NT;
      if (idx < C::DYN) {
        const int row = idx / NPIX, px = idx % NPIX;
        ldy[row * C::DYP + px] = dreg[i];
      }
    }
  };

  if (kt_begin < kt_end) fetch(kt_begin);
  for (long long kt = kt_begin; kt < kt_end; ++kt) {
    __syncthreads();
    store();
    __syncthreads();
    if (kt + 1 < kt_end) fetch(kt + 1);
    // operand reads software-pipelined PD steps ahead (see conv_fwd_kernel)
    constexpr int NS = NPIX / 2, PD = 2;
    float ra[PD], rb[PD][NI];
    auto rd = [&](int s, float& a, float (&b)[NI]) {
      const int poff = (s / TW) * S * C::RWP + (s % TW) * S;
      a = ldy[aoff + s];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) b[ni] = halo[boff[ni] + poff];
    };
#pragma unroll
    for (int s = 0; s < PD; ++s) rd(s, ra[s], rb[s]);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int slot = s % PD;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        acc[ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[slot], rb[slot][ni], acc[ni], 0, 0, 0);
      if (s + PD < NS) rd(s + PD, ra[slot], rb[slot]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  float* out = ws + (((size_t)split * gridDim.y + cob) * gridDim.z + cc) * (C::BM * C::BN);
#pragma unroll
  for (int ni = 0; ni < NI; ++ni)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h2;
      out[row * C::BN + (wn * NI + ni) * 32 + l32] = acc[ni][r];
    }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, int cout,
                                    int cin, int kk, int bm, int bn, int cis, int ncob, int ncc,
                                    int nsplit, int accumulate) {
  const long long total = (long long)cout * cin * kk;
  const size_t slab = (size_t)bm * bn;
  const size_t split_stride = (size_t)ncob * ncc * slab;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i % kk);
    const long long t = i / kk;
    const int ci = (int)(t % cin);
    const int co = (int)(t / cin);
    const int cob = co / bm, row = co % bm, cc = ci / cis, cil = ci % cis;
    const size_t o = ((size_t)cob * ncc + cc) * slab + (size_t)row * bn + cil * kk + r;
    float s = 0.f;
    // same (split) order; unrolled so the independent loads are in flight together
#pragma unroll 8
    for (int k = 0; k < nsplit; ++k) s += ws[(size_t)k * split_stride + o];
    dw[i] = accumulate ? dw[i] + s : s;
  }
}

struct WgPlan {
  int bm, bn, cis, nt, npix, tw, ncob, ncc, nsplit, tiles_x, tiles_per_img;
};

static bool wg_plan(int n, int cin, int cout, int ks, int stride, int ho, int wo, WgPlan& pl) {
  if (ks == 3) {
    pl.cis = 32;
    pl.bm = 64;
    pl.bn = 288;
    pl.nt = 384;
    pl.npix = stride == 1 ? 128 : 64;
  } else if (ks == 9 && stride == 1) {
    pl.cis = 3;
    pl.bm = 32;
    pl.bn = 256;
    pl.nt = 256;
    pl.npix = 128;
  } else {
    return false;
  }
  if (stride == 1)
    pl.tw = wo > 32 ? 64 : (wo > 16 ? 32 : 16);
  else
    pl.tw = wo > 16 ? 32 : 16;
  const int th = pl.npix / pl.tw;
  pl.tiles_x = cdiv(wo, pl.tw);
  pl.tiles_per_img = pl.tiles_x * cdiv(ho, th);
  pl.ncob = cdiv(cout, pl.bm);
  pl.ncc = cdiv(cin, pl.cis);
  const long long ktiles = (long long)n * pl.tiles_per_img;
  long long ns = cdiv(768, pl.ncob * pl.ncc);
  ns = std::max<long long>(1, std::min<long long>(ns, ktiles));
  pl.nsplit = (int)ns;
  return true;
}

template <int KS, int S, int CIS, int WM, int WN, int NI, int NPIX, int TW>
static void wg_launch(const WgPlan& pl, const float* x, const float* dy, float* ws, int n, int cin,
                      int h, int w, int cout, int pad, int mode, int hv, int wv, int ho, int wo,
                      hipStream_t st) {
  hipLaunchKernelGGL((wgrad_kernel<KS, S, CIS, WM, WN, NI, NPIX, TW>),
                     dim3(pl.nsplit, pl.ncob, pl.ncc), dim3(64 * WM * WN), 0, st, x, dy, ws, n,
                     cin, h, w, cout, pad, mode, hv, wv, ho, wo, pl.tiles_x, pl.tiles_per_img,
                     pl.nsplit);
}

}  // namespace stx

using namespace stx;

extern "C" size_t stx_conv2d_wgrad_ws(int n, int cin, int cout, int ks, int stride, int ho,
                                      int wo) {
  WgPlan pl;
  if (!wg_plan(n, cin, cout, ks, stride, ho, wo, pl)) return 0;
  return (size_t)pl.nsplit * pl.ncob * pl.ncc * pl.bm * pl.bn * sizeof(float) + 256;
}

extern "C" int stx_conv2d_wgrad(const float* x, const float* dy, float* dw, int accumulate,
                                int n, int cin, int h, int w, int cout, int ks, int stride,
                                int pad, int in_mode, int hv, int wv, int ho, int wo, void* ws,
                                size_t ws_bytes, void* stream) {
  WgPlan pl;
  if (!wg_plan(n, cin, cout, ks, stride, ho, wo, pl) || n <= 0 || !x || !dy || !dw) {
    set_error("stx_conv2d_wgrad: unsupported ks=%d stride=%d", ks, stride);
    return STX_E_INVALID;
  }
  if ((hv + 2 * pad - ks) / stride + 1 != ho || (wv + 2 * pad - ks) / stride + 1 != wo) {
    set_error("stx_conv2d_wgrad: inconsistent output dims");
    return STX_E_INVALID;
  }
  const size_t need = stx_conv2d_wgrad_ws(n, cin, cout, ks, stride, ho, wo);
  if (!ws || ws_bytes < need) {
    set_error("stx_conv2d_wgrad: workspace %zu < %zu", ws_bytes, need);
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* slabs = (float*)ws;
#define WG_ARGS pl, x, dy, slabs, n, cin, h, w, cout, pad, in_mode, hv, wv, ho, wo, st
  if (ks == 3 && stride == 1) {
    if (pl.tw == 64) wg_launch<3, 1, 32, 2, 3, 3, 128, 64>(WG_ARGS);
    else if (pl.tw == 32) wg_launch<3, 1, 32, 2, 3, 3, 128, 32>(WG_ARGS);
    else wg_launch<3, 1, 32, 2, 3, 3, 128, 16>(WG_ARGS);
  } else if (ks == 3 && stride == 2) {
    if (pl.tw == 32) wg_launch<3, 2, 32, 2, 3, 3, 64, 32>(WG_ARGS);
    else wg_launch<3, 2, 32, 2, 3, 3, 64, 16>(WG_ARGS);
  } else {
    if (pl.tw == 64) wg_launch<9, 1, 3, 1, 4, 2, 128, 64>(WG_ARGS);
    else if (pl.tw == 32) wg_launch<9, 1, 3, 1, 4, 2, 128, 32>(WG_ARGS);
    else wg_launch<9, 1, 3, 1, 4, 2, 128, 16>(WG_ARGS);
  }
#undef WG_ARGS
  const long long total = (long long)cout * cin * ks * ks;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, (const float*)slabs, dw,
                     cout, cin, ks * ks, pl.bm, pl.bn, pl.cis, pl.ncob, pl.ncc, pl.nsplit,
                     accumulate);
  return check_launch("stx_conv2d_wgrad");
}
