// Vector kernels for the on-device L-BFGS (styletransfer_amd/optim.py LBFGS, the
// optimiser of StyleNetwork.train_gatys, stransfer/network.py:411-458, which uses
// torch.optim.LBFGS defaults): deterministic reductions (dot, sum|a|, max|a|) with a
// fused scalar epilogue, a*x + b*y updates whose scalars may live on the device (so
// the two-loop recursion needs no host round trip), and a one-thread scalar kernel
// for the handful of 0-d quantities (ys, rho, H_diag, step size) torch keeps as
// device tensors.
#include "common.h"
#include "../../include/stx.h"

namespace stx {

constexpr int VB = 256;      // threads per block
constexpr int VPARTS = 256;  // partial-reduction blocks (fixed: bit-reproducible)

__device__ __forceinline__ float vred_op(int op, float acc, float a, float b) {
  if (op == 0) return fmaf(a, b, acc);
  if (op == 1) return acc + fabsf(a);
  const float m = fabsf(a);
  return (m != m || acc != acc) ? __int_as_float(0x7fc00000) : fmaxf(acc, m);
}

__device__ __forceinline__ float vred_combine(int op, float x, float y) {
  if (op == 2) return (x != x || y != y) ? __int_as_float(0x7fc00000) : fmaxf(x, y);
  return x + y;
}

__global__ void __launch_bounds__(VB)
vred_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                    int op, float* __restrict__ parts) {
  float acc = 0.f;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * VB;
  for (long long i = blockIdx.x * (long long)VB + threadIdx.x; i < n4; i += stride) {
    const f32x4 x = reinterpret_cast<const f32x4*>(a)[i];
    const f32x4 y = b ? reinterpret_cast<const f32x4*>(b)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = vred_op(op, acc, x[e], y[e]);
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)VB + threadIdx.x; i < n; i += stride)
    acc = vred_op(op, acc, a[i], b ? b[i] : 0.f);
  __shared__ float red[VB];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = VB / 2; s > 0; s >>= 1) {  // fixed tree order
    if (threadIdx.x < s) red[threadIdx.x] = vred_combine(op, red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) parts[blockIdx.x] = red[0];
}

// out = (add ? *add : 0) + sgn * r * (mul ? *mul : 1), r = the reduction
__global__ void __launch_bounds__(VB)
vred_final_kernel(const float* __restrict__ parts, int op, float* __restrict__ out,
                  const float* __restrict__ mul, const float* __restrict__ add, float sgn) {
  __shared__ float red[VB];
  red[threadIdx.x] = parts[threadIdx.x];
  __syncthreads();
  for (int s = VB / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = vred_combine(op, red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float r = red[0] * (mul ? *mul : 1.f);
    *out = (add ? *add : 0.f) + sgn * r;
  }
}

// y = alpha * x + b * y, alpha = a_dev ? a_sgn * *a_dev * a : a   (x may be NULL: y *= b)
__global__ void __launch_bounds__(VB)
vaxpby_kernel(float* __restrict__ y, const float* __restrict__ x, long long n, float a,
              const float* __restrict__ a_dev, float a_sgn, float b) {
  const float al = a_dev ? a_sgn * *a_dev * a : a;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * VB;
  for (long long i = blockIdx.x * (long long)VB + threadIdx.x; i < n4; i += stride) {
    f32x4 v = b == 0.f ? f32x4{0.f, 0.f, 0.f, 0.f} : reinterpret_cast<f32x4*>(y)[i] * b;
    if (x) v += al * reinterpret_cast<const f32x4*>(x)[i];
    reinterpret_cast<f32x4*>(y)[i] = v;
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)VB + threadIdx.x; i < n; i += stride)
    y[i] = (b == 0.f ? 0.f : b * y[i]) + (x ? al * x[i] : 0.f);
}

// s[k] = s[i] <op> s[j]:  0 div, 1 mul, 2 sub, 3 add, 4 recip(s[i]), 5 min(s[j], 1/s[i])
__global__ void scalar_kernel(float* s, int op, int i, int j, int k) {
  const float a = s[i], b = j >= 0 ? s[j] : 0.f;
  float r;
  switch (op) {
    case 0: r = a / b; break;
    case 1: r = a * b; break;
    case 2: r = a - b; break;
    case 3: r = a + b; break;
    case 4: r = 1.f / a; break;
    default: r = fminf(b, 1.f / a); break;
  }
  s[k] = r;
}

static int vgrid(long long n) {
  return (int)std::min<long long>(std::max<long long>(1, (n / 4 + VB - 1) / VB), 1024);
}

}  // namespace stx

using namespace stx;

extern "C" size_t stx_vec_ws(void) { return VPARTS * sizeof(float); }

extern "C" int stx_vec_reduce(const float* a, const float* b, long long n, int op, float* out,
                              const float* mul, const float* add, float sgn, void* ws,
                              size_t ws_bytes, void* stream) {
  if (!a || !out || n < 0 || op < 0 || op > 2 || (op == 0 && !b)) {
    set_error("stx_vec_reduce: invalid arguments");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < stx_vec_ws()) {
    set_error("stx_vec_reduce: workspace");
    return STX_E_WORKSPACE;
  }
  if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) {
    set_error("stx_vec_reduce: 16-byte aligned vectors required");
    return STX_E_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(vred_partial_kernel, dim3(VPARTS), dim3(VB), 0, st, a, b, n, op, (float*)ws);
  hipLaunchKernelGGL(vred_final_kernel, dim3(1), dim3(VB), 0, st, (const float*)ws, op, out, mul,
                     add, sgn);
  return check_launch("stx_vec_reduce");
}

extern "C" int stx_vec_axpby(float* y, const float* x, long long n, float a, const float* a_dev,
                             float a_sgn, float b, void* stream) {
  if (!y || n < 0) {
    set_error("stx_vec_axpby: invalid arguments");
    return STX_E_INVALID;
  }
  if ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(x)) & 15) {
    set_error("stx_vec_axpby: 16-byte aligned vectors required");
    return STX_E_INVALID;
  }
  hipLaunchKernelGGL(vaxpby_kernel, dim3(vgrid(n)), dim3(VB), 0, (hipStream_t)stream, y, x, n, a,
                     a_dev, a_sgn, b);
  return check_launch("stx_vec_axpby");
}

extern "C" int stx_scalar_op(float* s, int op, int i, int j, int k, void* stream) {
  if (!s || op < 0 || op > 5 || i < 0 || k < 0) {
    set_error("stx_scalar_op: invalid arguments");
    return STX_E_INVALID;
  }
  hipLaunchKernelGGL(scalar_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, s, op, i, j, k);
  return check_launch("stx_scalar_op");
}
