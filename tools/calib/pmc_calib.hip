// FETCH_SIZE / WRITE_SIZE calibration kernels (profiling tool, not part of libstx):
// streaming reads of a known byte count with 4-B-per-lane buffer loads (the access width
// of the split convs' halo staging and of gram_bwd16) and with 16-B-per-lane loads (the
// width the microarchitecture guide's FETCH_SIZE x2 correction is stated for), and
// 4-B-per-lane stores.  Each launch touches exactly `bytes` bytes once, coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

__global__ void __launch_bounds__(256) read4_kernel(const float* x, long long n, float* out) {
  float s = 0.f;
  for (long long base = 0; base < n; base += (long long)gridDim.x * 256 * 16) {
    const long long blk = base + (long long)blockIdx.x * 256 * 16;
    const auto r = srd(x + blk, (uint32_t)(min((long long)256 * 16, n - blk) * 4));
#pragma unroll
    for (int u = 0; u < 16; ++u)
      s += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                         r, (uint32_t)(u * 256 + threadIdx.x) * 4u, 0, 0));
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) read16_kernel(const float* x, long long n, float* out) {
  float s = 0.f;
  const long long n4 = n / 4;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    s += v[0] + v[1] + v[2] + v[3];
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) write4_kernel(float* y, long long n) {
  for (long long base = 0; base < n; base += (long long)gridDim.x * 256 * 16) {
    const long long blk = base + (long long)blockIdx.x * 256 * 16;
    const auto r = srd(y + blk, (uint32_t)(min((long long)256 * 16, n - blk) * 4));
#pragma unroll
    for (int u = 0; u < 16; ++u)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(1.f), r,
                                            (uint32_t)(u * 256 + threadIdx.x) * 4u, 0, 0);
  }
}

extern "C" int calib_run(int which, void* buf, long long n, void* scratch, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (which == 0)
    hipLaunchKernelGGL(read4_kernel, dim3(2048), dim3(256), 0, st, (const float*)buf, n,
                       (float*)scratch);
  else if (which == 1)
    hipLaunchKernelGGL(read16_kernel, dim3(2048), dim3(256), 0, st, (const float*)buf, n,
                       (float*)scratch);
  else
    hipLaunchKernelGGL(write4_kernel, dim3(2048), dim3(256), 0, st, (float*)buf, n);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
