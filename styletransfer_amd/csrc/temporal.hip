// Temporal loss of the video network (VideoTransformNet.get_temporal_loss,
// stransfer/network.py:885-903):
//
//     loss = ||y - y_old|| / (||x - x_old|| + 1) * w
//
// with y the stylised batch, y_old the previous stylised batch, x / x_old the content
// batches (Frobenius norms over the whole batch, as torch's Tensor.norm()).  Forward:
// both sums of squares in ONE streaming pass over the four tensors (fixed-order
// two-stage reduction: bit-reproducible), then a one-block epilogue that writes
// [loss, ||dy||, ||dx||].  Backward: d loss / d y = w / ((c + 1) a) * (y - y_old)
// (torch's norm backward: 0 where the norm is 0), scaled by the upstream gradient
// held on the device, written or accumulated into grad.  HBM-bound: 16 B/element
// forward, 12 B/element backward.
#include "common.h"
#include "../../include/stx.h"

namespace stx {

constexpr int TB = 256;      // threads per block
constexpr int TPARTS = 512;  // partial blocks (fixed: the reduction order never changes)

__global__ void __launch_bounds__(TB)
temporal_partial_kernel(const float* __restrict__ y, const float* __restrict__ yo,
                        const float* __restrict__ x, const float* __restrict__ xo, long long n,
                        float* __restrict__ parts, int vec) {
  float sy = 0.f, sx = 0.f;
  const long long n4 = vec ? n >> 2 : 0;  // a misaligned tensor: scalar loop throughout
  const long long stride = (long long)gridDim.x * TB;
  for (long long i = blockIdx.x * (long long)TB + threadIdx.x; i < n4; i += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(y)[i] - reinterpret_cast<const f32x4*>(yo)[i];
    const f32x4 b = reinterpret_cast<const f32x4*>(x)[i] - reinterpret_cast<const f32x4*>(xo)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sy = fmaf(a[e], a[e], sy);
      sx = fmaf(b[e], b[e], sx);
    }
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)TB + threadIdx.x; i < n; i += stride) {
    const float a = y[i] - yo[i], b = x[i] - xo[i];
    sy = fmaf(a, a, sy);
    sx = fmaf(b, b, sx);
  }
  __shared__ float red[TB / 64];
  sy = block_sum<TB>(sy, red);
  sx = block_sum<TB>(sx, red);
  if (threadIdx.x == 0) {
    parts[blockIdx.x] = sy;
    parts[TPARTS + blockIdx.x] = sx;
  }
}

__global__ void __launch_bounds__(TB)
temporal_final_kernel(const float* __restrict__ parts, float w, float* __restrict__ out) {
  float sy = 0.f, sx = 0.f;
  for (int i = threadIdx.x; i < TPARTS; i += TB) {  // fixed assignment, fixed order
    sy += parts[i];
    sx += parts[TPARTS + i];
  }
  __shared__ float red[TB / 64];
  sy = block_sum<TB>(sy, red);
  sx = block_sum<TB>(sx, red);
  if (threadIdx.x == 0) {
    const float a = sqrtf(sy), c = sqrtf(sx);
    out[0] = a / (c + 1.f) * w;
    out[1] = a;
    out[2] = c;
  }
}

__global__ void __launch_bounds__(TB)
temporal_bwd_kernel(const float* __restrict__ y, const float* __restrict__ yo, long long n,
                    const float* __restrict__ fwd, float w, const float* __restrict__ g,
                    float* __restrict__ grad, int accumulate, int vec) {
  const float a = fwd[1], c = fwd[2];
  const float s = a > 0.f ? (g ? *g : 1.f) * w / ((c + 1.f) * a) : 0.f;
  const long long n4 = vec ? n >> 2 : 0;
  const long long stride = (long long)gridDim.x * TB;
  for (long long i = blockIdx.x * (long long)TB + threadIdx.x; i < n4; i += stride) {
    f32x4 d = s * (reinterpret_cast<const f32x4*>(y)[i] - reinterpret_cast<const f32x4*>(yo)[i]);
    if (accumulate) d += reinterpret_cast<f32x4*>(grad)[i];
    reinterpret_cast<f32x4*>(grad)[i] = d;
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)TB + threadIdx.x; i < n; i += stride) {
    const float d = s * (y[i] - yo[i]);
    grad[i] = accumulate ? grad[i] + d : d;
  }
}

static int tgrid(long long n) {
  return (int)std::min<long long>(std::max<long long>(1, (n / 4 + TB - 1) / TB), 2048);
}

static bool aligned16(const void* p) { return !(reinterpret_cast<uintptr_t>(p) & 15); }

}  // namespace stx

using namespace stx;

extern "C" size_t stx_temporal_loss_ws(void) { return 2 * TPARTS * sizeof(float); }

extern "C" int stx_temporal_loss(const float* y, const float* y_old, const float* x,
                                 const float* x_old, long long n, float weight, float* out,
                                 void* ws, size_t ws_bytes, void* stream) {
  if (!y || !y_old || !x || !x_old || !out || n < 0) {
    set_error("stx_temporal_loss: invalid arguments");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_temporal_loss_ws()) {
    set_error("stx_temporal_loss: workspace");
    return STX_E_WORKSPACE;
  }
  // views at odd offsets (e.g. the previous frame inside a [B, 6, H, W] input at an odd
  // H*W) take the scalar loop: same result, no alignment contract on the caller
  const int vec = aligned16(y) && aligned16(y_old) && aligned16(x) && aligned16(x_old);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(temporal_partial_kernel, dim3(TPARTS), dim3(TB), 0, st, y, y_old, x, x_old,
                     n, (float*)ws, vec);
  hipLaunchKernelGGL(temporal_final_kernel, dim3(1), dim3(TB), 0, st, (const float*)ws, weight,
                     out);
  return check_launch("stx_temporal_loss");
}

extern "C" int stx_temporal_loss_bwd(const float* y, const float* y_old, long long n,
                                     const float* fwd, float weight, const float* g_dev,
                                     float* grad, int accumulate, void* stream) {
  if (!y || !y_old || !fwd || !grad || n < 0) {
    set_error("stx_temporal_loss_bwd: invalid arguments");
    return STX_E_INVALID;
  }
  const int vec = aligned16(y) && aligned16(y_old) && aligned16(grad);
  hipLaunchKernelGGL(temporal_bwd_kernel, dim3(tgrid(n)), dim3(TB), 0, (hipStream_t)stream, y,
                     y_old, n, fwd, weight, g_dev, grad, accumulate, vec);
  return check_launch("stx_temporal_loss_bwd");
}
