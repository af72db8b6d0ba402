// HBM-bound kernels of the style-transfer hot path (gfx950): losses, pooling,
// ReLU, Adam, upsample, total variation, bias gradients.  All reductions are
// two-stage with a fixed block count and a fixed summation order, so results
// are bit-reproducible run to run (no float atomics).
#include "common.h"
#include "../../include/stx.h"

namespace stx {

constexpr int RB = 256;         // threads per block for reductions
constexpr int RMAXB = 1024;     // max partial blocks

static int red_blocks(long long n) {
  return (int)std::max<long long>(1, std::min<long long>((n + RB * 8 - 1) / (RB * 8), RMAXB));
}

// ------------------------------------------------------------------ MSE
// ContentLoss (stransfer/network.py:155-164): F.mse_loss(x, target) (mean)
// FeatureReconstructionLoss (stransfer/network.py:186-201): mse^2 / numel
__global__ void __launch_bounds__(RB)
sqdiff_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                      int relu, float* __restrict__ parts, float* __restrict__ grad,
                      float gscale) {
  __shared__ float red[RB / 64];
  float s = 0.f;
  const long long stride = (long long)gridDim.x * RB;
  for (long long i = blockIdx.x * (long long)RB + threadIdx.x; i < n; i += stride) {
    float x = a[i], y = b[i];
    if (relu) {
      x = fmaxf(x, 0.f);
      y = fmaxf(y, 0.f);
    }
    const float d = x - y;
    s += d * d;
    if (grad) grad[i] = gscale * d;
  }
  s = block_sum<RB>(s, red);
  if (threadIdx.x == 0) parts[blockIdx.x] = s;
}

// mode 0: mean; mode 1: mean^2 / n;  out[1] (optional, mode 1) = mean
__global__ void mse_finalize_kernel(const float* __restrict__ parts, int nparts, double n,
                                    int mode, float* __restrict__ out,
                                    float* __restrict__ mean_out) {
  __shared__ float red[RB / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += RB) s += parts[i];
  s = block_sum<RB>(s, red);
  if (threadIdx.x == 0) {
    const float mean = (float)(s / n);
    if (mode == 0) {
      *out = mean;
    } else {
      *out = (float)((double)(mean * mean) / n);
    }
    if (mean_out) *mean_out = mean;
  }
}

// ContentLoss on conv2_2 and FeatureReconstructionLoss on relu(conv2_2) read the
// same two tensors: one pass computes both sums (float4 when aligned).
__global__ void __launch_bounds__(RB)
sqdiff2_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                       float* __restrict__ parts) {
  __shared__ float red[RB / 64];
  float s = 0.f, sr = 0.f;
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * RB;
  for (long long i = blockIdx.x * (long long)RB + threadIdx.x; i < n4; i += stride) {
    const f32x4 x = reinterpret_cast<const f32x4*>(a)[i];
    const f32x4 y = reinterpret_cast<const f32x4*>(b)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = x[k] - y[k], dr = fmaxf(x[k], 0.f) - fmaxf(y[k], 0.f);
      s += d * d;
      sr += dr * dr;
    }
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)RB + threadIdx.x; i < n; i += stride) {
    const float d = a[i] - b[i], dr = fmaxf(a[i], 0.f) - fmaxf(b[i], 0.f);
    s += d * d;
    sr += dr * dr;
  }
  s = block_sum<RB>(s, red);
  sr = block_sum<RB>(sr, red);
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = s;
    parts[2 * blockIdx.x + 1] = sr;
  }
}

// out[0] = mean sq diff; out[1] = mean(relu sq diff)^2 / n; out[2] = mean relu sq diff
__global__ void mse2_finalize_kernel(const float* __restrict__ parts, int nparts, double n,
                                     float* __restrict__ out) {
  __shared__ float red[RB / 64];
  float s = 0.f, sr = 0.f;
  for (int i = threadIdx.x; i < nparts; i += RB) {
    s += parts[2 * i];
    sr += parts[2 * i + 1];
  }
  s = block_sum<RB>(s, red);
  sr = block_sum<RB>(sr, red);
  if (threadIdx.x == 0) {
    const float mr = (float)(sr / n);
    out[0] = (float)(s / n);
    out[1] = (float)((double)(mr * mr) / n);
    out[2] = mr;
  }
}

// grad = s0 * (*s1) * (*s2) * (f(a) - f(b))   (autograd backward of the MSE losses)
__global__ void diff_scale_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                  float* __restrict__ g, long long n, float s0,
                                  const float* __restrict__ s1, const float* __restrict__ s2,
                                  int relu, int accumulate) {
  float sc = s0;
  if (s1) sc *= *s1;
  if (s2) sc *= *s2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float x = a[i], y = b[i];
    if (relu) {
      const float gx = x > 0.f ? 1.f : 0.f;
      x = fmaxf(x, 0.f);
      y = fmaxf(y, 0.f);
      const float v = sc * (x - y) * gx;
      g[i] = accumulate ? g[i] + v : v;
    } else {
      const float v = sc * (x - y);
      g[i] = accumulate ? g[i] + v : v;
    }
  }
}

// ------------------------------------------------------------------ pooling
// MaxPool2d(2,2) (VGG pieces, stransfer/network.py:264-275); torch CPU kernel
// semantics: scan the window row-major, update when (v > max) || isnan(v).
__global__ void maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                   long long* __restrict__ idx, int nc, int h, int w, int relu) {
  const int ho = h / 2, wo = w / 2;
  const long long total = (long long)nc * ho * wo;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ox = (int)(i % wo);
    const long long t = i / wo;
    const int oy = (int)(t % ho);
    const long long pl = t / ho;
    const float* src = x + pl * h * w;
    float best = -INFINITY;
    int bi = (2 * oy) * w + 2 * ox;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int yy = 2 * oy + dy, xx = 2 * ox + dx;
        float v = src[yy * w + xx];
        if (relu) v = fmaxf(v, 0.f);
        if (v > best || isnan(v)) {
          best = v;
          bi = yy * w + xx;
        }
      }
    y[i] = best;
    if (idx) idx[i] = bi;
  }
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, const long long* __restrict__ idx,
                                   float* __restrict__ dx, int nc, int h, int w) {
  // gather form (no atomics): each input element checks its window's argmax
  const int ho = h / 2, wo = w / 2;
  const long long total = (long long)nc * h * w;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    const long long t = i / w;
    const int yy = (int)(t % h);
    const long long pl = t / h;
    const int oy = yy >> 1, ox = xx >> 1;
    float v = 0.f;
    if (oy < ho && ox < wo) {
      const long long o = (pl * ho + oy) * wo + ox;
      if (idx[o] == (long long)yy * w + xx) v = dy[o];
    }
    dx[i] = v;
  }
}

// dZ = unpool(dP) * (Z > 0): backward of relu+maxpool(2x2), argmax recomputed from Z
// (first max of relu(Z) in the window, row-major) — no index tensor needed.
__global__ void relupool_bwd_kernel(const float* __restrict__ dp, const float* __restrict__ z,
                                    float* __restrict__ dz, int nc, int h, int w) {
  const int ho = h / 2, wo = w / 2;
  const long long total = (long long)nc * h * w;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    const long long t = i / w;
    const int yy = (int)(t % h);
    const long long pl = t / h;
    const int oy = yy >> 1, ox = xx >> 1;
    float v = 0.f;
    const float zv = z[i];
    if (oy < ho && ox < wo && zv > 0.f) {
      const float* src = z + pl * h * w + (2 * oy) * w + 2 * ox;
      const float a0 = fmaxf(src[0], 0.f), a1 = fmaxf(src[1], 0.f);
      const float a2 = fmaxf(src[w], 0.f), a3 = fmaxf(src[w + 1], 0.f);
      int bi = 0;
      float best = a0;
      if (a1 > best) { best = a1; bi = 1; }
      if (a2 > best) { best = a2; bi = 2; }
      if (a3 > best) { best = a3; bi = 3; }
      const int me = (yy & 1) * 2 + (xx & 1);
      if (me == bi) v = dp[(pl * ho + oy) * wo + ox];
    }
    dz[i] = v;
  }
}

__global__ void relu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = fmaxf(x[i], 0.f);
}

__global__ void relu_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                float* __restrict__ dx, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

// ------------------------------------------------------------------ Adam
// torch.optim.Adam (single-tensor, torch 2.10): exp_avg.lerp_(g, 1-b1);
// exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2); denom = sqrt(v)/sqrt(bc2) + eps;
// p.addcdiv_(m, denom, -lr/bc1).  Step counter lives on the device so a captured
// graph replays correctly; scalars computed in fp64 like torch's Python floats.
struct AdamScalars {
  float step_size;   // lr / bc1
  float bc2_sqrt;    // sqrt(1 - b2^t)
};

// thread 0: the step counter and bias corrections; all threads: zero `clear` (the
// caller's per-iteration amax groups, stx_adam_step_clear) -- one launch fewer per
// iteration than a separate fill
__global__ void adam_prepare_kernel(int* step, AdamScalars* sc, double lr, double b1, double b2,
                                    float* clear, int clear_n) {
  for (int i = threadIdx.x; i < clear_n; i += blockDim.x) clear[i] = 0.f;
  if (threadIdx.x) return;
  const int t = ++(*step);
  const double bc1 = 1.0 - pow(b1, (double)t);
  const double bc2 = 1.0 - pow(b2, (double)t);
  sc->step_size = (float)(lr / bc1);
  sc->bc2_sqrt = (float)sqrt(bc2);
}

__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, long long n, float b1, float b2, float eps,
            const AdamScalars* __restrict__ sc, int vec) {
  const float step_size = sc->step_size, bc2s = sc->bc2_sqrt;
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const long long n4 = vec ? n / 4 : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    const f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = mm[k] + w1 * (gg[k] - mm[k]);
      vv[k] = vv[k] * b2 + w2 * gg[k] * gg[k];
      const float denom = sqrtf(vv[k]) / bc2s + eps;
      pp[k] = pp[k] + (-step_size * mm[k]) / denom;
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += stride) {
    const float gg = g[i];
    const float mm = m[i] + w1 * (gg - m[i]);
    const float vv = v[i] * b2 + w2 * gg * gg;
    m[i] = mm;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2s + eps;
    p[i] = p[i] + (-step_size * mm) / denom;
  }
}

// ------------------------------------------------------------------ upsample
__global__ void upsample_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int nc,
                                    int h, int w) {
  const int H = 2 * h, W = 2 * w;
  const long long total = (long long)nc * H * W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % W);
    const long long t = i / W;
    const int yy = (int)(t % H);
    const long long pl = t / H;
    y[i] = x[(pl * h + (yy >> 1)) * w + (xx >> 1)];
  }
}

__global__ void upsample_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, int nc,
                                    int h, int w) {
  const long long total = (long long)nc * h * w;
  const int W = 2 * w;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    const long long t = i / w;
    const int yy = (int)(t % h);
    const long long pl = t / h;
    const float* s = dy + (pl * 2 * h + 2 * yy) * W + 2 * xx;
    dx[i] = (s[0] + s[1]) + (s[W] + s[W + 1]);
  }
}

// ------------------------------------------------------------------ TV
// get_total_variation_regularization_loss (stransfer/network.py:621-641):
// factor * (sum|y[..., :-1] - y[..., 1:]| + sum|y[..., :-1, :] - y[..., 1:, :]|),
// summed over the whole batch.  abs'(0) = 0 (torch sign).
__device__ __forceinline__ float sgn(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// 32-bit index math (64-bit div/mod is a long software sequence per element) and
// branch-free neighbour loads / gradient stores through buffer descriptors: a load
// behind `if (xx + 1 < w)` is a branch with a vmcnt(0) at its join, one round trip per
// neighbour.  Out-of-image neighbours are selected away after the (in-range) load, so
// the sums and gradients are the same bits as the branchy form (adding +0 is exact).
__global__ void __launch_bounds__(RB)
tv_kernel(const float* __restrict__ y, float* __restrict__ parts, float* __restrict__ grad,
          float gscale, const float* __restrict__ gscale_dev, long long total, int h, int w,
          float factor) {
  __shared__ float red[RB / 64];
  float gs = gscale * factor;
  if (gscale_dev) gs *= *gscale_dev;
  float sh = 0.f, sv = 0.f;
  const int n = (int)total;  // stx_tv_loss checks total < 2^29
  const uint32_t bytes = (uint32_t)n * 4u;
  const auto ry = make_srd(y, bytes);
  const auto rg = make_srd(grad ? grad : y, grad ? bytes : 0u);
  const int stride = gridDim.x * RB;
  for (int i = blockIdx.x * RB + threadIdx.x; i < n; i += stride) {
    const int q = i / w, xx = i - q * w;
    const int yy = q % h;
    const uint32_t o = (uint32_t)i * 4u;
    const float v = buf_ld(ry, o);
    const bool r_ok = xx + 1 < w, l_ok = xx > 0, d_ok = yy + 1 < h, u_ok = yy > 0;
    const float vr = buf_ld(ry, r_ok ? o + 4u : o);
    const float vl = buf_ld(ry, l_ok ? o - 4u : o);
    const float vd = buf_ld(ry, d_ok ? o + 4u * (uint32_t)w : o);
    const float vu = buf_ld(ry, u_ok ? o - 4u * (uint32_t)w : o);
    float g = 0.f;
    const float dr = v - vr, dd = v - vd;
    sh += r_ok ? fabsf(dr) : 0.f;
    g += r_ok ? sgn(dr) : 0.f;
    g -= l_ok ? sgn(vl - v) : 0.f;
    sv += d_ok ? fabsf(dd) : 0.f;
    g += d_ok ? sgn(dd) : 0.f;
    g -= u_ok ? sgn(vu - v) : 0.f;
    buf_st(rg, o, gs * g);
  }
  sh = block_sum<RB>(sh, red);
  sv = block_sum<RB>(sv, red);
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = sh;
    parts[2 * blockIdx.x + 1] = sv;
  }
}

__global__ void tv_finalize_kernel(const float* __restrict__ parts, int nb, float factor,
                                   float* __restrict__ out) {
  __shared__ float red[RB / 64];
  float sh = 0.f, sv = 0.f;
  for (int i = threadIdx.x; i < nb; i += RB) {
    sh += parts[2 * i];
    sv += parts[2 * i + 1];
  }
  sh = block_sum<RB>(sh, red);
  sv = block_sum<RB>(sv, red);
  if (threadIdx.x == 0) *out = factor * (sh + sv);
}

// ------------------------------------------------------------------ bias grad
// per (n, c) plane sums -> ws[n][c]; then ordered sum over n
__global__ void __launch_bounds__(RB)
plane_sum_kernel(const float* __restrict__ x, float* __restrict__ out, int hw) {
  __shared__ float red[RB / 64];
  const float* src = x + (size_t)blockIdx.x * hw;
  float s = 0.f;
  if ((hw & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    // float4 loads, several in flight per thread (fixed order: 4 running sums)
    const f32x4* s4 = reinterpret_cast<const f32x4*>(src);
    const int n4 = hw >> 2;
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int i = threadIdx.x; i < n4; i += RB) a += s4[i];
    s = (a[0] + a[1]) + (a[2] + a[3]);
  } else {
    for (int i = threadIdx.x; i < hw; i += RB) s += src[i];
  }
  s = block_sum<RB>(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// small planes: one block per channel sums its n planes in one pass (fixed order:
// per-thread float4 running sums over the planes in order, then the block tree)
__global__ void __launch_bounds__(RB)
bias_grad_c_kernel(const float* __restrict__ x, float* __restrict__ db, int n, int c, int hw,
                   int accumulate) {
  __shared__ float red[RB / 64];
  const int ch = blockIdx.x;
  const int n4 = hw >> 2;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < n; ++k) {
    const f32x4* s4 = reinterpret_cast<const f32x4*>(x + ((size_t)k * c + ch) * hw);
#pragma unroll 4
    for (int i = threadIdx.x; i < n4; i += RB) a += s4[i];
  }
  float s = (a[0] + a[1]) + (a[2] + a[3]);
  s = block_sum<RB>(s, red);
  if (threadIdx.x == 0) db[ch] = accumulate ? db[ch] + s : s;
}

__global__ void sum_over_n_kernel(const float* __restrict__ parts, float* __restrict__ out, int n,
                                  int c, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  float s = 0.f;
  for (int k = 0; k < n; ++k) s += parts[(size_t)k * c + i];
  out[i] = accumulate ? out[i] + s : s;
}

// ------------------------------------------------------------------ loss combine
// out = sum_i w_i * s[i]   (k <= 16, fixed order)
struct LossW {
  float w[16];
};
__global__ void loss_combine_kernel(const float* __restrict__ s, int k, LossW w,
                                    float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < k; ++i) t += w.w[i] * s[i];
    *out = t;
  }
}

static int ew_blocks(long long n) {
  return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192));
}

}  // namespace stx

using namespace stx;

namespace stx {
}  // namespace stx

extern "C" size_t stx_mse_ws(long long n) { return (size_t)(2 * red_blocks(n) + 4) * sizeof(float); }

extern "C" int stx_mse(const float* a, const float* b, long long n, int relu_inputs, int mode,
                       float* out, float* grad, float gscale, void* ws, size_t ws_bytes,
                       void* stream) {
  if (n <= 0 || !a || !b || !out || mode < 0 || mode > 2 || (grad && mode != 0)) {
    set_error("stx_mse: invalid args");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_mse_ws(n)) {
    set_error("stx_mse: workspace too small");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int nb = red_blocks(n);
  float* parts = (float*)ws;
  if (mode == 2) {
    if (((uintptr_t)a | (uintptr_t)b) & 15) {
      set_error("stx_mse: mode 2 needs 16-byte aligned inputs");
      return STX_E_INVALID;
    }
    hipLaunchKernelGGL(sqdiff2_partial_kernel, dim3(nb), dim3(RB), 0, st, a, b, n, parts);
    hipLaunchKernelGGL(mse2_finalize_kernel, dim3(1), dim3(RB), 0, st, parts, nb, (double)n,
                       out);
    return check_launch("stx_mse");
  }
  const float gs = (float)(gscale * 2.0 / (double)n);
  hipLaunchKernelGGL(sqdiff_partial_kernel, dim3(nb), dim3(RB), 0, st, a, b, n, relu_inputs,
                     parts, grad, gs);
  hipLaunchKernelGGL(mse_finalize_kernel, dim3(1), dim3(RB), 0, st, parts, nb, (double)n, mode,
                     out, mode == 1 ? out + 1 : (float*)nullptr);
  return check_launch("stx_mse");
}

extern "C" int stx_diff_scale(const float* a, const float* b, float* grad, long long n, float s0,
                              const float* s1_dev, const float* s2_dev, int relu, int accumulate,
                              void* stream) {
  hipLaunchKernelGGL(diff_scale_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, a,
                     b, grad, n, s0, s1_dev, s2_dev, relu, accumulate);
  return check_launch("stx_diff_scale");
}

extern "C" int stx_loss_combine(const float* s, int k, const float* w_host, float* out,
                                void* stream) {
  if (k < 1 || k > 16) {
    set_error("stx_loss_combine: k out of range");
    return STX_E_INVALID;
  }
  LossW w = {};
  for (int i = 0; i < k; ++i) w.w[i] = w_host[i];
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, s, k, w,
                     out);
  return check_launch("stx_loss_combine");
}

extern "C" int stx_maxpool2x2_fwd(const float* x, float* y, long long* idx, int nc, int h, int w,
                                  int relu_input, void* stream) {
  const long long n = (long long)nc * (h / 2) * (w / 2);
  if (n <= 0) {
    set_error("stx_maxpool2x2_fwd: empty");
    return STX_E_INVALID;
  }
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, x,
                     y, idx, nc, h, w, relu_input);
  return check_launch("stx_maxpool2x2_fwd");
}

extern "C" int stx_maxpool2x2_bwd(const float* dy, const long long* idx, float* dx, int nc, int h,
                                  int w, void* stream) {
  const long long n = (long long)nc * h * w;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream,
                     dy, idx, dx, nc, h, w);
  return check_launch("stx_maxpool2x2_bwd");
}

extern "C" int stx_relupool_bwd(const float* dp, const float* z, float* dz, int nc, int h, int w,
                                void* stream) {
  const long long n = (long long)nc * h * w;
  hipLaunchKernelGGL(relupool_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream,
                     dp, z, dz, nc, h, w);
  return check_launch("stx_relupool_bwd");
}

extern "C" int stx_relu_fwd(const float* x, float* y, long long n, void* stream) {
  hipLaunchKernelGGL(relu_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, x, y,
                     n);
  return check_launch("stx_relu_fwd");
}

extern "C" int stx_relu_bwd(const float* dy, const float* y, float* dx, long long n,
                            void* stream) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, dy,
                     y, dx, n);
  return check_launch("stx_relu_bwd");
}

extern "C" size_t stx_adam_ws(void) { return 64; }

extern "C" int stx_adam_step_clear(float* p, const float* g, float* m, float* v, long long n,
                                   float lr, float beta1, float beta2, float eps, int* step_dev,
                                   void* ws, float* clear, int clear_n, void* stream) {
  if (n <= 0 || !p || !g || !m || !v || !step_dev || !ws || clear_n < 0 ||
      (clear_n > 0 && !clear)) {
    set_error("stx_adam_step: invalid args");
    return STX_E_INVALID;
  }
  const int vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
  hipStream_t st = (hipStream_t)stream;
  AdamScalars* sc = (AdamScalars*)ws;
  hipLaunchKernelGGL(adam_prepare_kernel, dim3(1), dim3(clear_n > 0 ? 256 : 64), 0, st, step_dev,
                     sc, (double)lr, (double)beta1, (double)beta2, clear, clear_n);
  const long long units = vec ? n / 4 : n;
  const int blocks = (int)std::max<long long>(1, std::min<long long>((units + 255) / 256, 4096));
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, p, g, m, v, n, beta1, beta2,
                     eps, sc, vec);
  return check_launch("stx_adam_step");
}

extern "C" int stx_adam_step(float* p, const float* g, float* m, float* v, long long n, float lr,
                             float beta1, float beta2, float eps, int* step_dev, void* ws,
                             void* stream) {
  return stx_adam_step_clear(p, g, m, v, n, lr, beta1, beta2, eps, step_dev, ws, nullptr, 0,
                             stream);
}

extern "C" int stx_upsample2x_fwd(const float* x, float* y, int nc, int h, int w, void* stream) {
  const long long n = (long long)nc * 4 * h * w;
  hipLaunchKernelGGL(upsample_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream,
                     x, y, nc, h, w);
  return check_launch("stx_upsample2x_fwd");
}

extern "C" int stx_upsample2x_bwd(const float* dy, float* dx, int nc, int h, int w,
                                  void* stream) {
  const long long n = (long long)nc * h * w;
  hipLaunchKernelGGL(upsample_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream,
                     dy, dx, nc, h, w);
  return check_launch("stx_upsample2x_bwd");
}

extern "C" size_t stx_tv_ws(int n, int c, int h, int w) {
  return (size_t)(2 * red_blocks((long long)n * c * h * w) + 4) * sizeof(float);
}

extern "C" int stx_tv_loss(const float* y, float* loss, float* grad, float gscale,
                           const float* gscale_dev, int n, int c, int h, int w, float factor,
                           void* ws, size_t ws_bytes, void* stream) {
  const long long total = (long long)n * c * h * w;
  if (total <= 0 || !y || !loss || total >= (1ll << 29)) {
    set_error("stx_tv_loss: invalid args (or more than 2^29 elements)");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_tv_ws(n, c, h, w)) {
    set_error("stx_tv_loss: workspace too small");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int nb = red_blocks(total);
  hipLaunchKernelGGL(tv_kernel, dim3(nb), dim3(RB), 0, st, y, (float*)ws, grad, gscale,
                     gscale_dev, total, h, w, factor);
  hipLaunchKernelGGL(tv_finalize_kernel, dim3(1), dim3(RB), 0, st, (const float*)ws, nb, factor,
                     loss);
  return check_launch("stx_tv_loss");
}

extern "C" size_t stx_bias_grad_ws(int n, int c) { return (size_t)n * c * sizeof(float) + 64; }

static bool one_pass_bias() {  // STX_BIAS_ONEPASS=0: always the two-pass path (A/B)
  static const bool on = STX_KNOB("STX_BIAS_ONEPASS", 1) != 0;
  return on;
}

extern "C" int stx_bias_grad(const float* dy, float* db, int n, int c, int hw, int accumulate,
                             void* ws, size_t ws_bytes, void* stream) {
  if (!ws || ws_bytes < stx_bias_grad_ws(n, c)) {
    set_error("stx_bias_grad: workspace too small");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  if ((hw & 3) == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0 &&
      (long long)n * hw <= 64 * 1024 && c >= 16 && one_pass_bias()) {
    // <= 256 KB per channel: one launch (the two-pass path below is launch-bound there)
    hipLaunchKernelGGL(bias_grad_c_kernel, dim3(c), dim3(RB), 0, st, dy, db, n, c, hw,
                       accumulate);
    return check_launch("stx_bias_grad");
  }
  hipLaunchKernelGGL(plane_sum_kernel, dim3(n * c), dim3(RB), 0, st, dy, (float*)ws, hw);
  hipLaunchKernelGGL(sum_over_n_kernel, dim3(cdiv(c, 256)), dim3(256), 0, st, (const float*)ws,
                     db, n, c, accumulate);
  return check_launch("stx_bias_grad");
}
