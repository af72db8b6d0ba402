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

#include "common.h"
#include "conv_epi.h"
#include "../../include/stx.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// e with |a| < 2^e (frexp), clamped so 2^(15-e) and 2^(ex+ew-30) stay normal floats
__device__ __forceinline__ int amax_exp(float a) {
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

template <int TW>
struct C16 {
  static constexpr int BM = 64, NPIX = 256, TH = NPIX / TW;
  static constexpr int RH = TH + 2, RW = TW + 2, NPOS = RH * RW;
  static constexpr int NITEM = 2 * NPOS;                   // (channel group, position)
  static constexpr int NIT = (NITEM + 255) / 256;          // items per thread
  static constexpr int NITP = NIT * 256;                   // padded: stores unconditional
  static constexpr int WT_U = 9 * 2 * 2 * BM;              // 16-B units per weight chunk
  static constexpr int NWT = WT_U / 256;
  static constexpr int LDS_BYTES = (2 * NITP + WT_U) * 16;
  static_assert(WT_U % 256 == 0, "weight units per thread");
  static_assert(16 * NPIX * 4 + 16 * BM * 4 <= LDS_BYTES, "phase-2 staging fits");
};

// DBG (profiling experiments only, tools/bench_conv.py --dbg): bit 0 skips the
// epilogue, bit 1 skips the per-chunk restaging after chunk 0
template <int TW, int LM, int DBG = 0>
__global__ void __launch_bounds__(256, 2)
conv3x3_f16x3_kernel(stx_conv_params p, int tiles_x) {
  using C = C16<TW>;
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

  const int ex = amax_exp(*p.in_amax), ew = amax_exp(*p.w_amax);
  const float sx = __builtin_ldexpf(1.f, 15 - ex);
  const float descale = __builtin_ldexpf(1.f, ex + ew - 30);

  const int plane_in = p.h * p.w;
  const float* __restrict__ xn = p.x + (size_t)n * p.cin * plane_in;
  const int vy0 = ty0 - 1, vx0 = tx0 - 1;

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
  const int nchunks = cdiv(p.cin, 16);
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
          hv[r][c] = fmaxf(fmaxf(buf_ld(rs, o), buf_ld(rs, o + 4)),
                           fmaxf(buf_ld(rs, o + wb), buf_ld(rs, o + wb + 4)));
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
        if (LM == STX_IN_RELU || LM == STX_IN_RELU_POOL2) v = fmaxf(v, 0.f);
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

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // per-lane operand bases (bytes)
  const char* bbase[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int ty, tx;
    tile_pix<TW, (TW == 64)>(wave, j, l32, ty, tx);
    bbase[j] = lds_h + (h * C::NPOS + ty * C::RW + tx) * 16;
  }
  const char* abase = lds_w + (h * BM + l32) * 16;

  fetch(0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();  // previous chunk's operand reads done
    if (!(DBG & 2) || chunk == 0) store();
    __syncthreads();
    if (chunk + 1 < nchunks && !(DBG & 2)) fetch(chunk + 1);  // in flight across the MFMA loop
    f16x8 ra[2][2][2], rb[2][2][2];            // [slot][tile][hi/lo]
    auto rd = [&](int tap, f16x8 (&a)[2][2], f16x8 (&b)[2][2]) {
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int P = 0; P < 2; ++P)
          a[i][P] = *reinterpret_cast<const f16x8*>(abase + (tap * 4 * BM + P * 2 * BM + i * 32) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int P = 0; P < 2; ++P)
          b[j][P] = *reinterpret_cast<const f16x8*>(bbase[j] +
                                                    (P * C::NITP + kh * C::RW + kw) * 16);
    };
    rd(0, ra[0], rb[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int s = tap & 1;
      if (tap + 1 < 9) rd(tap + 1, ra[s ^ 1], rb[s ^ 1]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][i][0], rb[s][j][0], acc[i][j],
                                                             0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][i][0], rb[s][j][1], acc[i][j],
                                                             0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[s][i][1], rb[s][j][0], acc[i][j],
                                                             0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (DBG & 1) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    if (t == 12345.f) p.y[tid] = t;
    return;
  }
  __syncthreads();  // the epilogue's phase 2 re-uses the LDS
  const EpiTile et{n, co0, ty0, tx0, 0, wave, h, l32};
  conv_epilogue<BM, TW, C::NPIX, 16, (TW == 64)>(acc, p, et, descale, reinterpret_cast<float*>(smem),
                                     reinterpret_cast<float*>(smem + 16 * C::NPIX * 4));
}

static int dbg_mode() {
  static const int m = [] {
    const char* e = getenv("STX_CONV16_DBG");
    return e ? atoi(e) : 0;
  }();
  return m;
}

template <int TW, int LM>
static int launch16(const stx_conv_params& p, hipStream_t st) {
  using C = C16<TW>;
  const int tiles_x = cdiv(p.wo, TW), tiles_y = cdiv(p.ho, C::TH);
  dim3 grid(tiles_x * tiles_y, cdiv(p.cout, C::BM), p.n);
  if constexpr (TW == 64 && LM == STX_IN_RELU) {
    switch (dbg_mode()) {
      case 1: hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM, 1>), grid, dim3(256), 0, st, p, tiles_x); return check_launch("dbg");
      case 2: hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM, 2>), grid, dim3(256), 0, st, p, tiles_x); return check_launch("dbg");
      case 3: hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM, 3>), grid, dim3(256), 0, st, p, tiles_x); return check_launch("dbg");
      default: break;
    }
  }
  hipLaunchKernelGGL((conv3x3_f16x3_kernel<TW, LM>), grid, dim3(256), 0, st, p, tiles_x);
  return check_launch("stx_conv2d(f16x3)");
}

template <int LM>
static int dispatch16_tw(const stx_conv_params& p, hipStream_t st) {
  if (p.wo > 32) return launch16<64, LM>(p, st);
  if (p.pool_out) {
    set_error("stx_conv2d: pool_out needs wo > 32 (row-pair tile mapping)");
    return STX_E_INVALID;
  }
  if (p.wo > 16) return launch16<32, LM>(p, st);
  return launch16<16, LM>(p, st);
}

// ------------------------------------------------------------ weight split prep
// slab [cin16/16][tap][P][cg][cout64][8] fp16 of the GEMM weights W'[co][ci][tap]
__global__ void weight_prep16_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                     const float* __restrict__ w_amax, int cout, int cin,
                                     int transpose, int gin16, int gout64) {
  const long long total = (long long)gin16 * 9 * 2 * gout64;
  const float sw = __builtin_ldexpf(1.f, 15 - amax_exp(*w_amax));
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7);
    long long r = i >> 3;
    const int co = (int)(r % gout64);
    r /= gout64;
    const int cg = (int)(r & 1);
    r >>= 1;
    const int P = (int)(r & 1);
    r >>= 1;
    const int tap = (int)(r % 9);
    const int chunk = (int)(r / 9);
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

// -------------------------------------------------------------------- amax
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

int conv2d_f16x3(const stx_conv_params& p, hipStream_t st) {
  switch (p.in_mode) {
    case STX_IN_RAW: return dispatch16_tw<STX_IN_RAW>(p, st);
    case STX_IN_RELU: return dispatch16_tw<STX_IN_RELU>(p, st);
    case STX_IN_RELU_POOL2: return dispatch16_tw<STX_IN_RELU_POOL2>(p, st);
    case STX_IN_UPSAMPLE2: return dispatch16_tw<STX_IN_UPSAMPLE2>(p, st);
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
  hipError_t e = hipMemsetAsync(out, 0, sizeof(float), st);
  if (e != hipSuccess) {
    set_error("stx_amax: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (n == 0) return STX_OK;
  const int blocks = (int)std::min<long long>(std::max<long long>(1, (n / 4 + 255) / 256), 512);
  hipLaunchKernelGGL(amax_kernel, dim3(blocks), dim3(256), 0, st, x, n, out);
  return check_launch("stx_amax");
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
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(weight_prep16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<_Float16*>(wt16), w_amax, cout, cin, transpose, gin16,
                     gout64);
  return check_launch("stx_conv_weight_prep16");
}
