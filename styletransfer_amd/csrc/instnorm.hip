// InstanceNorm2d(affine=True) forward/backward for gfx950, with the ResidualBlock
// add and the following ReLU fused.
//
// Reference: nn.InstanceNorm2d(num_features, affine=True) in ImageTransformNet /
// ResidualBlock (stransfer/network.py:474,483,531,541,551,588,600; eps 1e-5,
// biased variance, per-instance statistics in train and eval, no running stats),
// residual `out += residual` (stransfer/network.py:502) and nn.ReLU.
//
// One 256-thread block per (n, c) plane.  Forward: u = x (+ res); two passes
// over u (mean, then sum of squared deviations: numerically like torch's
// two-pass CPU kernel), then y = (u-mean)*rstd*gamma + beta (relu).  The plane
// (<= 256 KB at 256x256) stays L2-resident between the passes.
#include "common.h"
#include "conv_epi.h"
#include "../../include/stx.h"

namespace stx {

constexpr int NB = 256;

// y = fma(u, gsc, sh) with gsc = gamma rstd, sh = fma(-mean, gsc, beta): every forward
// kernel forms the output this way, with explicit fmas (no contraction left to the
// compiler), so a backward recomputes the ReLU decision y > 0 from u = x (+ res) and the
// saved mean / rstd bit for bit instead of reading y (one plane-read fewer per element)
__device__ __forceinline__ void in_coefs(const float* gamma, const float* beta, int ch,
                                         float mean, float rstd, float& gsc, float& sh) {
  gsc = gamma ? gamma[ch] * rstd : rstd;
  sh = __builtin_fmaf(-mean, gsc, beta ? beta[ch] : 0.f);
}

__global__ void __launch_bounds__(NB)
instnorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ res,
                    const float* __restrict__ gamma, const float* __restrict__ beta,
                    float* __restrict__ y, float* __restrict__ mean_out,
                    float* __restrict__ rstd_out, int c, int hw, float eps, int relu,
                    float* __restrict__ out_amax) {
  __shared__ float red[NB / 64];
  const size_t base = (size_t)blockIdx.x * hw;
  const int ch = blockIdx.x % c;
  const float* xp = x + base;
  const float* rp = res ? res + base : nullptr;
  const bool vec = ((hw & 3) == 0);
  float s = 0.f;
  if (vec) {
    for (int i = threadIdx.x * 4; i < hw; i += NB * 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(xp + i);
      if (rp) v += *reinterpret_cast<const f32x4*>(rp + i);
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += NB) s += xp[i] + (rp ? rp[i] : 0.f);
  }
  const float mean = block_sum<NB>(s, red) / (float)hw;
  float q = 0.f;
  if (vec) {
    for (int i = threadIdx.x * 4; i < hw; i += NB * 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(xp + i);
      if (rp) v += *reinterpret_cast<const f32x4*>(rp + i);
      v -= mean;
      q += (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += NB) {
      const float d = xp[i] + (rp ? rp[i] : 0.f) - mean;
      q += d * d;
    }
  }
  const float var = block_sum<NB>(q, red) / (float)hw;
  const float rstd = 1.f / sqrtf(var + eps);
  float gsc, sh;
  in_coefs(gamma, beta, ch, mean, rstd, gsc, sh);
  float* yp = y + base;
  uint32_t om = 0u;  // max |y| as IEEE bits (NaN sorts above inf)
  if (vec) {
    for (int i = threadIdx.x * 4; i < hw; i += NB * 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(xp + i);
      if (rp) v += *reinterpret_cast<const f32x4*>(rp + i);
      f32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = __builtin_fmaf(v[k], gsc, sh);
        if (relu) o[k] = fmaxf(o[k], 0.f);
        om = max(om, __float_as_uint(o[k]) & 0x7fffffffu);
      }
      *reinterpret_cast<f32x4*>(yp + i) = o;
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += NB) {
      float o = __builtin_fmaf(xp[i] + (rp ? rp[i] : 0.f), gsc, sh);
      o = relu ? fmaxf(o, 0.f) : o;
      yp[i] = o;
      om = max(om, __float_as_uint(o) & 0x7fffffffu);
    }
  }
  if (out_amax) block_max_to(out_amax, __uint_as_float(om));
  if (threadIdx.x == 0) {
    if (mean_out) mean_out[blockIdx.x] = mean;
    if (rstd_out) rstd_out[blockIdx.x] = rstd;
  }
}

// Backward.  g = dy * (y > 0 if relu);  xh = (u-mean)*rstd
//   dgamma_nc = sum g*xh ; dbeta_nc = sum g
//   du = gamma*rstd/HW * (HW*g - dbeta_nc - xh*dgamma_nc)
// max |.| over an NT-thread block, then one atomic into slot (block id & 31)
template <int NT>
__device__ __forceinline__ void block_max_to_nt(float* group, uint32_t mu, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mu = max(mu, (uint32_t)__shfl_xor((int)mu, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(mu);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = 0u;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) r = max(r, __float_as_uint(red[i]));
    atomic_max_abs(group + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
  }
}

template <int NBT>
__global__ void __launch_bounds__(NBT)
instnorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ beta,
                    const float* __restrict__ x, const float* __restrict__ res,
                    const float* __restrict__ gamma, const float* __restrict__ mean,
                    const float* __restrict__ rstd, float* __restrict__ du,
                    float* __restrict__ parts, int c, int hw, int relu,
                    float* __restrict__ out_amax) {
  __shared__ float red[NBT / 64];
  const size_t base = (size_t)blockIdx.x * hw;
  const int ch = blockIdx.x % c;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  float gsc, sh;  // the forward's y = fma(u, gsc, sh): the ReLU decision recomputed
  in_coefs(gamma, beta, ch, mu, rs, gsc, sh);
  const float* dyp = dy + base;
  const float* xp = x + base;
  const float* rp = res ? res + base : nullptr;
  float sg = 0.f, sgx = 0.f;
  const bool vec = ((hw & 3) == 0) &&
                   ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
                     reinterpret_cast<uintptr_t>(res) | reinterpret_cast<uintptr_t>(du)) & 15) == 0;
  // float4 path (16-B aligned planes): 4x fewer loads, two float4 groups per trip so
  // each thread keeps 8 loads in flight
  auto ld4 = [](const float* p, int i) { return *reinterpret_cast<const f32x4*>(p + i); };
  if (vec) {
    for (int i = threadIdx.x * 4; i < hw; i += NBT * 4) {
      const f32x4 d4 = ld4(dyp, i);
      const f32x4 x4 = ld4(xp, i);
      const f32x4 r4 = rp ? ld4(rp, i) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u = x4[e] + r4[e];
        const float g = (relu && !(__builtin_fmaf(u, gsc, sh) > 0.f)) ? 0.f : d4[e];
        const float xh = (u - mu) * rs;
        sg += g;
        sgx += g * xh;
      }
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += NBT) {
      float g = dyp[i];
      const float u = xp[i] + (rp ? rp[i] : 0.f);
      if (relu && !(__builtin_fmaf(u, gsc, sh) > 0.f)) g = 0.f;
      const float xh = (u - mu) * rs;
      sg += g;
      sgx += g * xh;
    }
  }
  sg = block_sum<NBT>(sg, red);
  sgx = block_sum<NBT>(sgx, red);
  const float gm = gamma ? gamma[ch] : 1.f;
  const float k = gm * rs / (float)hw;
  float* dup = du + base;
  uint32_t om = 0u;  // max |du| as IEEE bits
  float sdu = 0.f;   // sum du: the gradient of the producing conv's bias
  if (vec) {
    for (int i = threadIdx.x * 4; i < hw; i += NBT * 4) {
      const f32x4 d4 = ld4(dyp, i);
      const f32x4 x4 = ld4(xp, i);
      const f32x4 r4 = rp ? ld4(rp, i) : f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u = x4[e] + r4[e];
        const float g = (relu && !(__builtin_fmaf(u, gsc, sh) > 0.f)) ? 0.f : d4[e];
        const float xh = (u - mu) * rs;
        o[e] = k * ((float)hw * g - sg - xh * sgx);
        om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
        sdu += o[e];
      }
      *reinterpret_cast<f32x4*>(dup + i) = o;
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += NBT) {
      float g = dyp[i];
      const float u = xp[i] + (rp ? rp[i] : 0.f);
      if (relu && !(__builtin_fmaf(u, gsc, sh) > 0.f)) g = 0.f;
      const float xh = (u - mu) * rs;
      const float o = k * ((float)hw * g - sg - xh * sgx);
      dup[i] = o;
      om = max(om, __float_as_uint(o) & 0x7fffffffu);
      sdu += o;
    }
  }
  sdu = block_sum<NBT>(sdu, red);
  if (threadIdx.x == 0) {
    parts[3 * blockIdx.x] = sgx;
    parts[3 * blockIdx.x + 1] = sg;
    parts[3 * blockIdx.x + 2] = sdu;
  }
  if (out_amax) block_max_to_nt<NBT>(out_amax, om, red);
}

// Register-resident variants for planes of up to 4*NT*R4 floats (the ImageTransformNet
// planes: 64^2, 128^2, 256^2): each thread loads its R4 float4s of u = x (+res) once,
// and the statistics and the output come from registers -- one HBM read and one write
// per element instead of three passes (the loop kernels above re-read the plane).
// Same arithmetic; block reductions in a fixed order (bit-reproducible).
template <int NT>
__device__ __forceinline__ float block_sum_nt(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

template <int NT, int R4>
__global__ void __launch_bounds__(NT)
instnorm_fwd_reg_kernel(const float* __restrict__ x, const float* __restrict__ res,
                        const float* __restrict__ gamma, const float* __restrict__ beta,
                        float* __restrict__ y, float* __restrict__ mean_out,
                        float* __restrict__ rstd_out, int c, int hw, float eps, int relu,
                        float* __restrict__ out_amax) {
  __shared__ float red[NT / 64];
  const size_t base = (size_t)blockIdx.x * hw;
  const int ch = blockIdx.x % c;
  const int n4 = hw >> 2;
  const f32x4* xp = reinterpret_cast<const f32x4*>(x + base);
  const f32x4* rp = res ? reinterpret_cast<const f32x4*>(res + base) : nullptr;
  f32x4 u[R4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    const int i = threadIdx.x + k * NT;
    u[k] = i < n4 ? xp[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    if (rp && i < n4) u[k] += rp[i];
  }
#pragma unroll
  for (int k = 0; k < R4; ++k) s += (u[k][0] + u[k][1]) + (u[k][2] + u[k][3]);
  const float mean = block_sum_nt<NT>(s, red) / (float)hw;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    if (threadIdx.x + k * NT < n4) {
      const f32x4 d = u[k] - mean;
      q += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
    }
  }
  const float var = block_sum_nt<NT>(q, red) / (float)hw;
  const float rstd = 1.f / sqrtf(var + eps);
  float gsc, sh;
  in_coefs(gamma, beta, ch, mean, rstd, gsc, sh);
  f32x4* yp = reinterpret_cast<f32x4*>(y + base);
  uint32_t om = 0u;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < n4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = __builtin_fmaf(u[k][e], gsc, sh);
        if (relu) o[e] = fmaxf(o[e], 0.f);
        om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
      }
      yp[i] = o;
    }
  }
  if (threadIdx.x == 0) {
    if (mean_out) mean_out[blockIdx.x] = mean;
    if (rstd_out) rstd_out[blockIdx.x] = rstd;
  }
  if (out_amax) {
    uint32_t m = om;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) r = max(r, __float_as_uint(red[i]));
      atomic_max_abs(out_amax + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

template <int NT, int R4>
__global__ void __launch_bounds__(NT)
instnorm_bwd_reg_kernel(const float* __restrict__ dy, const float* __restrict__ beta,
                        const float* __restrict__ x, const float* __restrict__ res,
                        const float* __restrict__ gamma, const float* __restrict__ mean,
                        const float* __restrict__ rstd, float* __restrict__ du,
                        float* __restrict__ parts, int c, int hw, int relu,
                        float* __restrict__ out_amax) {
  __shared__ float red[NT / 64];
  const size_t base = (size_t)blockIdx.x * hw;
  const int ch = blockIdx.x % c;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  float gsc, sh;  // the forward's y = fma(u, gsc, sh): the ReLU decision recomputed
  in_coefs(gamma, beta, ch, mu, rs, gsc, sh);
  const int n4 = hw >> 2;
  const f32x4* dyp = reinterpret_cast<const f32x4*>(dy + base);
  const f32x4* xp = reinterpret_cast<const f32x4*>(x + base);
  const f32x4* rp = res ? reinterpret_cast<const f32x4*>(res + base) : nullptr;
  f32x4 g[R4], xh[R4];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    const int i = threadIdx.x + k * NT;
    const bool in = i < n4;
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 d4 = in ? dyp[i] : z4;
    f32x4 u4 = in ? xp[i] : z4;
    if (rp && in) u4 += rp[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      g[k][e] = (relu && !(__builtin_fmaf(u4[e], gsc, sh) > 0.f)) ? 0.f : d4[e];
      xh[k][e] = in ? (u4[e] - mu) * rs : 0.f;
    }
  }
#pragma unroll
  for (int k = 0; k < R4; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sg += g[k][e];
      sgx += g[k][e] * xh[k][e];
    }
  sg = block_sum_nt<NT>(sg, red);
  sgx = block_sum_nt<NT>(sgx, red);
  const float gm = gamma ? gamma[ch] : 1.f;
  const float kk = gm * rs / (float)hw;
  f32x4* dup = reinterpret_cast<f32x4*>(du + base);
  uint32_t om = 0u;
  float sdu = 0.f;  // sum du: the gradient of the producing conv's bias
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    const int i = threadIdx.x + k * NT;
    if (i < n4) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = kk * ((float)hw * g[k][e] - sg - xh[k][e] * sgx);
        om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
      }
      dup[i] = o;
      sdu += (o[0] + o[1]) + (o[2] + o[3]);
    }
  }
  sdu = block_sum_nt<NT>(sdu, red);
  if (threadIdx.x == 0) {
    parts[3 * blockIdx.x] = sgx;
    parts[3 * blockIdx.x + 1] = sg;
    parts[3 * blockIdx.x + 2] = sdu;
  }
  if (out_amax) {
    uint32_t m = om;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) r = max(r, __float_as_uint(red[i]));
      atomic_max_abs(out_amax + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

// Pipelined register variants for planes of exactly 4*NT*R4 floats (the ITN's 64^2
// planes, 1024 of them at B = 8): a block walks PPB consecutive planes and issues the
// next plane's loads before this plane's reductions and stores, so the chip's load and
// store phases overlap instead of every block loading, reducing and storing in lockstep
// (one-plane blocks all resident at once: 13 us for 34 MB).  Loads are unconditional
// (exact plane size, compile-time residual / ReLU) so each wait covers one plane's loads.
// Same arithmetic and reduction order per plane as the one-plane kernels (same bits).
template <int NT, int R4, int PPB, bool RES>
__global__ void __launch_bounds__(NT)
instnorm_fwd_pipe_kernel(const float* __restrict__ x, const float* __restrict__ res,
                         const float* __restrict__ gamma, const float* __restrict__ beta,
                         float* __restrict__ y, float* __restrict__ mean_out,
                         float* __restrict__ rstd_out, int c, float eps, int relu,
                         float* __restrict__ out_amax) {
  constexpr int HW = 4 * NT * R4;
  __shared__ float red[NT / 64];
  const int p0 = blockIdx.x * PPB;
  f32x4 xb[2][R4], rb[2][R4];
  auto load = [&](int b, int plane) {
    const f32x4* xp = reinterpret_cast<const f32x4*>(x + (size_t)plane * HW);
#pragma unroll
    for (int k = 0; k < R4; ++k) xb[b][k] = xp[threadIdx.x + k * NT];
    if constexpr (RES) {
      const f32x4* rp = reinterpret_cast<const f32x4*>(res + (size_t)plane * HW);
#pragma unroll
      for (int k = 0; k < R4; ++k) rb[b][k] = rp[threadIdx.x + k * NT];
    }
  };
  uint32_t om = 0u;
  load(0, p0);
#pragma unroll
  for (int j = 0; j < PPB; ++j) {
    const int b = j & 1, plane = p0 + j;
    if (j + 1 < PPB) load(b ^ 1, plane + 1);
    f32x4 u[R4];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      u[k] = xb[b][k];
      if constexpr (RES) u[k] += rb[b][k];
    }
#pragma unroll
    for (int k = 0; k < R4; ++k) s += (u[k][0] + u[k][1]) + (u[k][2] + u[k][3]);
    const float mean = block_sum_nt<NT>(s, red) / (float)HW;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      const f32x4 d = u[k] - mean;
      q += (d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]);
    }
    const float var = block_sum_nt<NT>(q, red) / (float)HW;
    const float rstd = 1.f / sqrtf(var + eps);
    const int ch = plane % c;
    float gsc, sh;
    in_coefs(gamma, beta, ch, mean, rstd, gsc, sh);
    f32x4* yp = reinterpret_cast<f32x4*>(y + (size_t)plane * HW);
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = __builtin_fmaf(u[k][e], gsc, sh);
        if (relu) o[e] = fmaxf(o[e], 0.f);
        om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
      }
      yp[threadIdx.x + k * NT] = o;
    }
    if (threadIdx.x == 0) {
      if (mean_out) mean_out[plane] = mean;
      if (rstd_out) rstd_out[plane] = rstd;
    }
  }
  if (out_amax) {
    uint32_t m = om;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) r = max(r, __float_as_uint(red[i]));
      atomic_max_abs(out_amax + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

template <int NT, int R4, int PPB, bool RELU, bool RES>
__global__ void __launch_bounds__(NT)
instnorm_bwd_pipe_kernel(const float* __restrict__ dy, const float* __restrict__ beta,
                         const float* __restrict__ x, const float* __restrict__ res,
                         const float* __restrict__ gamma, const float* __restrict__ mean,
                         const float* __restrict__ rstd, float* __restrict__ du,
                         float* __restrict__ parts, int c, float* __restrict__ out_amax) {
  constexpr int HW = 4 * NT * R4;
  __shared__ float red[NT / 64];
  const int p0 = blockIdx.x * PPB;
  f32x4 db[2][R4], xb[2][R4], rb[2][R4];
  auto load = [&](int b, int plane) {
    const size_t base = (size_t)plane * HW;
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      const int i = threadIdx.x + k * NT;
      db[b][k] = reinterpret_cast<const f32x4*>(dy + base)[i];
      xb[b][k] = reinterpret_cast<const f32x4*>(x + base)[i];
      if constexpr (RES) rb[b][k] = reinterpret_cast<const f32x4*>(res + base)[i];
    }
  };
  uint32_t om = 0u;
  load(0, p0);
#pragma unroll
  for (int j = 0; j < PPB; ++j) {
    const int b = j & 1, plane = p0 + j;
    if (j + 1 < PPB) load(b ^ 1, plane + 1);
    const float mu = mean[plane], rs = rstd[plane];
    float gsc, sh;  // the forward's y = fma(u, gsc, sh): the ReLU decision recomputed
    in_coefs(gamma, beta, plane % c, mu, rs, gsc, sh);
    f32x4 g[R4], xh[R4];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      f32x4 u4 = xb[b][k];
      if constexpr (RES) u4 += rb[b][k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (RELU) g[k][e] = !(__builtin_fmaf(u4[e], gsc, sh) > 0.f) ? 0.f : db[b][k][e];
        else g[k][e] = db[b][k][e];
        xh[k][e] = (u4[e] - mu) * rs;
      }
    }
#pragma unroll
    for (int k = 0; k < R4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sg += g[k][e];
        sgx += g[k][e] * xh[k][e];
      }
    sg = block_sum_nt<NT>(sg, red);
    sgx = block_sum_nt<NT>(sgx, red);
    const float gm = gamma ? gamma[plane % c] : 1.f;
    const float kk = gm * rs / (float)HW;
    f32x4* dup = reinterpret_cast<f32x4*>(du + (size_t)plane * HW);
    float sdu = 0.f;
#pragma unroll
    for (int k = 0; k < R4; ++k) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = kk * ((float)HW * g[k][e] - sg - xh[k][e] * sgx);
        om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
      }
      dup[threadIdx.x + k * NT] = o;
      sdu += (o[0] + o[1]) + (o[2] + o[3]);
    }
    sdu = block_sum_nt<NT>(sdu, red);
    if (threadIdx.x == 0) {
      parts[3 * plane] = sgx;
      parts[3 * plane + 1] = sg;
      parts[3 * plane + 2] = sdu;
    }
  }
  if (out_amax) {
    uint32_t m = om;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = __uint_as_float(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) r = max(r, __float_as_uint(red[i]));
      atomic_max_abs(out_amax + (blockIdx.x & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

// block shape of the planes between 4 x 256 x 4 and 4 x 1024 x 4 floats (the ITN's 128^2
// layers: 512 planes at B = 8): 0 = 256 x 16 float4 (2 blocks, 8 waves per CU), 1 = 1024 x
// 4, 2 = 512 x 8, 3 = the pipelined kernels on two planes per 512-thread block (A/B:
// STX_IN128; B8 x 64 @ 128^2 ReLU, same box: fwd / bwd 13.9 / 18.9, 13.7 / 21.7, 13.5 /
// 18.0, 14.6 / 19.0 us -- none pays, 0 is kept)
static int in128_form() {
  static const int v = STX_KNOB("STX_IN128", 0);
  return v;
}

static int in_ppb() {  // planes per block of the pipelined 64^2 kernels (1: one-plane kernels)
  // 1, 2 or 4 (the launches below instantiate these; anything else means 1)
  static const int v = [] {
    const int k = STX_KNOB("STX_IN_PPB", 4);
    return k == 2 || k == 4 ? k : 1;
  }();
  return v;
}

// Large planes (the ITN's 256^2 layers: 64 K floats, 1024 threads x 16 float4): g stays
// in registers (64 VGPRs) and u = x (+ res) is kept too -- its first XL float4s per thread
// in registers, the rest in LDS (XL = 8: 32 VGPRs + 128 KB of LDS, one block per CU) -- so
// the plane is read once: dy and u in, du out (the round-5 form re-read u in its second
// pass: 4 plane-reads + 1 write instead of 2 + 1).  The ReLU decision is recomputed from u.
// Same arithmetic as instnorm_bwd_reg_kernel.
template <int NT, int R4, bool RELU, bool RES, int XL>
__global__ void __launch_bounds__(NT)
instnorm_bwd_greg_kernel(const float* __restrict__ dy, const float* __restrict__ beta,
                         const float* __restrict__ x, const float* __restrict__ res,
                         const float* __restrict__ gamma, const float* __restrict__ mean,
                         const float* __restrict__ rstd, float* __restrict__ du,
                         float* __restrict__ parts, int c, int hw, int relu,
                         float* __restrict__ out_amax) {
  __shared__ float red[NT / 64];
  // u of steps XL .. R4-1 ([step][thread]); XL < 0: u not kept, re-read in the second pass
  __shared__ f32x4 ul[XL < 0 ? 1 : (R4 - XL) * NT];
  const size_t base = (size_t)blockIdx.x * hw;
  const int ch = blockIdx.x % c;
  const float mu = mean[blockIdx.x], rs = rstd[blockIdx.x];
  float gsc, sh;  // the forward's y = fma(u, gsc, sh): the ReLU decision recomputed
  in_coefs(gamma, beta, ch, mu, rs, gsc, sh);
  // per-plane buffer descriptors: one lane offset, the per-k step in the scalar offset
  // (64-bit addresses per k would take 2 VGPRs each and spill); elements past the
  // plane read 0 and their stores are dropped by the range check
  const uint32_t pbytes = (uint32_t)hw * 4u;
  const auto rdy = make_srd(dy + base, pbytes);
  const auto rx = make_srd(x + base, pbytes);
  const auto rr = make_srd(RES ? res + base : x + base, pbytes);
  const auto rdu = make_srd(du + base, pbytes);
  const uint32_t lo = threadIdx.x * 16u;
  constexpr uint32_t KSTEP = NT * 16u;
  const int n4 = hw >> 2;
  f32x4 g[R4], ur[XL > 0 ? XL : 1];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    const f32x4 d4 = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(rdy, lo, k * KSTEP, 0));
    f32x4 u4 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, lo, k * KSTEP, 0));
    if (RES) u4 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, lo, k * KSTEP, 0));
    const bool in = (int)threadIdx.x + k * NT < n4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      g[k][e] = (RELU && !(__builtin_fmaf(u4[e], gsc, sh) > 0.f)) ? 0.f : d4[e];
      const float xh = in ? (u4[e] - mu) * rs : 0.f;
      sg += g[k][e];
      sgx += g[k][e] * xh;
    }
    if constexpr (XL >= 0) {
      if (k < XL)
        ur[k < XL ? k : 0] = u4;
      else
        ul[(k - XL) * NT + threadIdx.x] = u4;
    }
    // at most 2 steps of loads in flight (g and u take 96 VGPRs; the scheduler would
    // hoist more loads and spill)
    if ((k & 1) == 1) __builtin_amdgcn_sched_barrier(0);
  }
  sg = block_sum_nt<NT>(sg, red);   // (its barriers also order the LDS stores of u)
  sgx = block_sum_nt<NT>(sgx, red);
  const float gm = gamma ? gamma[ch] : 1.f;
  const float kk = gm * rs / (float)hw;
  uint32_t om = 0u;
  float sdu = 0.f;
#pragma unroll
  for (int k = 0; k < R4; ++k) {
    f32x4 u4;
    if constexpr (XL < 0) {
      if ((k & 3) == 0) __builtin_amdgcn_sched_barrier(0);
      u4 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, lo, k * KSTEP, 0));
      if (RES) u4 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, lo, k * KSTEP, 0));
    } else {
      u4 = k < XL ? ur[k < XL ? k : 0] : ul[(k - XL) * NT + threadIdx.x];
    }
    const bool in = (int)threadIdx.x + k * NT < n4;
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xh = (u4[e] - mu) * rs;
      o[e] = in ? kk * ((float)hw * g[k][e] - sg - xh * sgx) : 0.f;
      om = max(om, __float_as_uint(o[e]) & 0x7fffffffu);
    }
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rdu, lo, k * KSTEP, 0);
    sdu += (o[0] + o[1]) + (o[2] + o[3]);
  }
  sdu = block_sum_nt<NT>(sdu, red);
  if (threadIdx.x == 0) {
    parts[3 * blockIdx.x] = sgx;
    parts[3 * blockIdx.x + 1] = sg;
    parts[3 * blockIdx.x + 2] = sdu;
  }
  if (out_amax) block_max_to_nt<NT>(out_amax, om, red);
}

// dgamma, dbeta and the producing conv's bias gradient: fixed-order sums over n
__global__ void instnorm_param_grad_kernel(const float* __restrict__ parts, int n, int c,
                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                           float* __restrict__ dbias, int accumulate) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  float a = 0.f, b = 0.f, d = 0.f;
  for (int k = 0; k < n; ++k) {
    const float* p = parts + 3 * ((size_t)k * c + ch);
    a += p[0];
    b += p[1];
    d += p[2];
  }
  if (dgamma) dgamma[ch] = accumulate ? dgamma[ch] + a : a;
  if (dbeta) dbeta[ch] = accumulate ? dbeta[ch] + b : b;
  if (dbias) dbias[ch] = accumulate ? dbias[ch] + d : d;
}

// many layers' parameter reductions in one launch (stx_instnorm_param_grads): thread ->
// (job, channel) in job order; the same fixed-order sums as instnorm_param_grad_kernel
struct PGradJobs {
  stx_in_pgrad_job job[STX_PGRAD_MAX];
  int ch0[STX_PGRAD_MAX + 1];  // first channel of each job (prefix sums)
  int njobs;
};

__global__ void __launch_bounds__(256) instnorm_param_grads_kernel(PGradJobs b) {
  const int gc = blockIdx.x * blockDim.x + threadIdx.x;
  if (gc >= b.ch0[b.njobs]) return;
  int j = 0;
  while (j + 1 < b.njobs && gc >= b.ch0[j + 1]) ++j;
  const stx_in_pgrad_job& t = b.job[j];
  const int ch = gc - b.ch0[j];
  float a = 0.f, bb = 0.f, d = 0.f;
  for (int k = 0; k < t.n; ++k) {
    const float* p = t.parts + 3 * ((size_t)k * t.c + ch);
    a += p[0];
    bb += p[1];
    d += p[2];
  }
  const bool acc = t.accumulate != 0;
  if (t.dgamma) t.dgamma[ch] = acc ? t.dgamma[ch] + a : a;
  if (t.dbeta) t.dbeta[ch] = acc ? t.dbeta[ch] + bb : bb;
  if (t.dbias_in) t.dbias_in[ch] = acc ? t.dbias_in[ch] + d : d;
}

}  // namespace stx

using namespace stx;

extern "C" int stx_instnorm_param_grads(const stx_in_pgrad_job* jobs, int njobs, void* stream) {
  if (!jobs || njobs <= 0 || njobs > STX_PGRAD_MAX) {
    set_error("stx_instnorm_param_grads: 1 <= njobs <= %d required", STX_PGRAD_MAX);
    return STX_E_INVALID;
  }
  PGradJobs b{};
  int ch = 0;
  for (int j = 0; j < njobs; ++j) {
    if (!jobs[j].parts || jobs[j].n <= 0 || jobs[j].c <= 0) {
      set_error("stx_instnorm_param_grads: job %d invalid", j);
      return STX_E_INVALID;
    }
    b.job[j] = jobs[j];
    b.ch0[j] = ch;
    ch += jobs[j].c;
  }
  b.ch0[njobs] = ch;
  b.njobs = njobs;
  hipLaunchKernelGGL(instnorm_param_grads_kernel, dim3(cdiv(ch, 256)), dim3(256), 0,
                     (hipStream_t)stream, b);
  return check_launch("stx_instnorm_param_grads");
}

extern "C" int stx_instnorm_fwd(const float* x, const float* res, const float* gamma,
                                const float* beta, float* y, float* mean, float* rstd, int n,
                                int c, int hw, float eps, int relu, float* out_amax,
                                void* stream) {
  if (n <= 0 || c <= 0 || hw <= 0 || !x || !y) {
    set_error("stx_instnorm_fwd: invalid args");
    return STX_E_INVALID;
  }
  if ((((uintptr_t)x) | ((uintptr_t)y) | ((uintptr_t)res)) & 15) {
    set_error("stx_instnorm_fwd: 16-byte alignment required");
    return STX_E_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  // 64^2 planes: 512 threads x 2 float4 per thread (fast_st 1801 -> 1811 img/s same box
  // against 256 x 4; 128 x 8 was 0.6 % slower); STX_IN_CFG=0 restores 256 x 4, 1 = 128 x 8
  static const int cfg = STX_KNOB("STX_IN_CFG", 2);
#ifdef STX_AB  // 128 x 8 blocks for the 64^2 planes (measured 0.6 % slower)
  if (cfg == 1 && hw % 4 == 0 && hw <= 4 * 128 * 8)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<128, 8>), dim3(n * c), dim3(128), 0, st, x, res,
                       gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else
#endif
  if (cfg == 2 && hw == 4 * 512 * 2 && in_ppb() > 1 && (n * c) % in_ppb() == 0 &&
           n * c / in_ppb() >= 256 &&  // enough blocks to fill the chip (B = 8: 256)
           ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(res) |
             reinterpret_cast<uintptr_t>(y)) & 15) == 0) {
    const int ppb = in_ppb();
    const dim3 grid(n * c / ppb);
#define STX_IN_FWD_PIPE(P, R)                                                                   \
  hipLaunchKernelGGL((instnorm_fwd_pipe_kernel<512, 2, P, R>), grid, dim3(512), 0, st, x, res, \
                     gamma, beta, y, mean, rstd, c, eps, relu, out_amax)
    if (ppb == 4) {
      if (res) STX_IN_FWD_PIPE(4, true); else STX_IN_FWD_PIPE(4, false);
    } else {
      if (res) STX_IN_FWD_PIPE(2, true); else STX_IN_FWD_PIPE(2, false);
    }
#undef STX_IN_FWD_PIPE
  } else if (cfg == 2 && hw % 4 == 0 && hw <= 4 * 512 * 2)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<512, 2>), dim3(n * c), dim3(512), 0, st, x, res,
                       gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else if (hw % 4 == 0 && hw <= 4 * 256 * 4)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<256, 4>), dim3(n * c), dim3(256), 0, st, x, res,
                       gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else if (in128_form() == 3 && hw == 4 * 512 * 8 && !res && (n * c) % 2 == 0 && n * c / 2 >= 256)
    hipLaunchKernelGGL((instnorm_fwd_pipe_kernel<512, 8, 2, false>), dim3(n * c / 2), dim3(512), 0,
                       st, x, res, gamma, beta, y, mean, rstd, c, eps, relu, out_amax);
  else if (in128_form() == 1 && hw % 4 == 0 && hw <= 4 * 1024 * 4)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<1024, 4>), dim3(n * c), dim3(1024), 0, st, x,
                       res, gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else if (in128_form() == 2 && hw % 4 == 0 && hw <= 4 * 512 * 8)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<512, 8>), dim3(n * c), dim3(512), 0, st, x,
                       res, gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else if (hw % 4 == 0 && hw <= 4 * 256 * 16)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<256, 16>), dim3(n * c), dim3(256), 0, st, x, res,
                       gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else if (hw % 4 == 0 && hw <= 4 * 1024 * 16)
    hipLaunchKernelGGL((instnorm_fwd_reg_kernel<1024, 16>), dim3(n * c), dim3(1024), 0, st, x,
                       res, gamma, beta, y, mean, rstd, c, hw, eps, relu, out_amax);
  else
    hipLaunchKernelGGL(instnorm_fwd_kernel, dim3(n * c), dim3(NB), 0, st, x, res, gamma, beta, y,
                       mean, rstd, c, hw, eps, relu, out_amax);
  return check_launch("stx_instnorm_fwd");
}

static bool greg_on() {
  static const bool on = STX_KNOB("STX_IN_GREG", 1) != 0;
  return on;
}

extern "C" size_t stx_instnorm_bwd_ws(int n, int c) {
  return (size_t)3 * n * c * sizeof(float) + 64;
}

extern "C" int stx_instnorm_bwd(const float* dy, const float* beta, const float* x,
                                const float* res, const float* gamma, const float* mean,
                                const float* rstd,
                                float* du, float* dgamma, float* dbeta, float* dbias_in, int n,
                                int c, int hw, int relu, int accumulate_params, float* out_amax,
                                void* ws, size_t ws_bytes, void* stream) {
  if (n <= 0 || c <= 0 || hw <= 0 || !dy || !x || !du || !mean || !rstd) {
    set_error("stx_instnorm_bwd: invalid args");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_instnorm_bwd_ws(n, c)) {
    set_error("stx_instnorm_bwd: workspace too small");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const bool al = ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
                    reinterpret_cast<uintptr_t>(res) | reinterpret_cast<uintptr_t>(du)) & 15) == 0 &&
                  hw % 4 == 0;
  // block shape of the 64^2 kernels, as stx_instnorm_fwd
  static const int cfg = STX_KNOB("STX_IN_CFG", 2);
#ifdef STX_AB
  if (cfg == 1 && al && hw <= 4 * 128 * 8)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<128, 8>), dim3(n * c), dim3(128), 0, st, dy, beta, x,
                       res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else
#endif
  if (cfg == 2 && al && hw == 4 * 512 * 2 && in_ppb() > 1 && (n * c) % in_ppb() == 0 &&
           n * c / in_ppb() >= 256) {
    const int ppb = in_ppb();
    const dim3 grid(n * c / ppb);
#define STX_IN_BWD_PIPE(P, RL, R)                                                               \
  hipLaunchKernelGGL((instnorm_bwd_pipe_kernel<512, 2, P, RL, R>), grid, dim3(512), 0, st, dy, beta, \
                     x, res, gamma, mean, rstd, du, (float*)ws, c, out_amax)
    if (ppb == 4) {
      if (relu) { if (res) STX_IN_BWD_PIPE(4, true, true); else STX_IN_BWD_PIPE(4, true, false); }
      else { if (res) STX_IN_BWD_PIPE(4, false, true); else STX_IN_BWD_PIPE(4, false, false); }
    } else {
      if (relu) { if (res) STX_IN_BWD_PIPE(2, true, true); else STX_IN_BWD_PIPE(2, true, false); }
      else { if (res) STX_IN_BWD_PIPE(2, false, true); else STX_IN_BWD_PIPE(2, false, false); }
    }
#undef STX_IN_BWD_PIPE
  } else if (cfg == 2 && al && hw <= 4 * 512 * 2)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<512, 2>), dim3(n * c), dim3(512), 0, st, dy, beta, x,
                       res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else if (al && hw <= 4 * 256 * 4)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<256, 4>), dim3(n * c), dim3(256), 0, st, dy, beta, x,
                       res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else if (in128_form() == 3 && al && hw == 4 * 512 * 8 && relu && !res && (n * c) % 2 == 0 &&
           n * c / 2 >= 256)
    hipLaunchKernelGGL((instnorm_bwd_pipe_kernel<512, 8, 2, true, false>), dim3(n * c / 2),
                       dim3(512), 0, st, dy, beta, x, res, gamma, mean, rstd, du, (float*)ws, c,
                       out_amax);
  else if (in128_form() == 1 && al && hw <= 4 * 1024 * 4)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<1024, 4>), dim3(n * c), dim3(1024), 0, st, dy,
                       beta, x, res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else if (in128_form() == 2 && al && hw <= 4 * 512 * 8)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<512, 8>), dim3(n * c), dim3(512), 0, st, dy,
                       beta, x, res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else if (al && hw <= 4 * 256 * 16)
    hipLaunchKernelGGL((instnorm_bwd_reg_kernel<256, 16>), dim3(n * c), dim3(256), 0, st, dy, beta,
                       x, res, gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else if (al && hw <= 4 * 1024 * 16 && relu && !res && greg_on())  // 256^2 IN + ReLU
  {
    // u kept in registers + LDS at 512 threads per plane (STX_GREG_FORM A/B, B8 x 32 planes
    // of 256^2, same box: 0 = u re-read in the second pass at 1024 threads 51.0 us, 1 = u
    // kept at 1024 threads 44.1 us (spills 24 VGPRs), 2 = this 40.1 us)
    static const int form = STX_KNOB("STX_GREG_FORM", 2);
    if (form == 0)
      hipLaunchKernelGGL((instnorm_bwd_greg_kernel<1024, 16, true, false, -1>), dim3(n * c),
                         dim3(1024), 0, st, dy, beta, x, res, gamma, mean, rstd, du, (float*)ws,
                         c, hw, relu, out_amax);
    else if (form == 2)
      hipLaunchKernelGGL((instnorm_bwd_greg_kernel<512, 32, true, false, 14>), dim3(n * c),
                         dim3(512), 0, st, dy, beta, x, res, gamma, mean, rstd, du, (float*)ws,
                         c, hw, relu, out_amax);
    else
      hipLaunchKernelGGL((instnorm_bwd_greg_kernel<1024, 16, true, false, 7>), dim3(n * c),
                         dim3(1024), 0, st, dy, beta, x, res, gamma, mean, rstd, du, (float*)ws,
                         c, hw, relu, out_amax);
  }
  else if (hw >= 4 * 1024 * 4)  // big planes (256^2): 16 waves per plane
    hipLaunchKernelGGL(instnorm_bwd_kernel<1024>, dim3(n * c), dim3(1024), 0, st, dy, beta, x, res,
                       gamma, mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  else
    hipLaunchKernelGGL(instnorm_bwd_kernel<NB>, dim3(n * c), dim3(NB), 0, st, dy, beta, x, res, gamma,
                       mean, rstd, du, (float*)ws, c, hw, relu, out_amax);
  if (dgamma || dbeta || dbias_in)
    hipLaunchKernelGGL(instnorm_param_grad_kernel, dim3(cdiv(c, 256)), dim3(256), 0, st,
                       (const float*)ws, n, c, dgamma, dbeta, dbias_in, accumulate_params);
  return check_launch("stx_instnorm_bwd");
}
