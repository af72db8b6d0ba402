// Shared device helpers for libstx (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/stx.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define STX_WAVE 64

namespace stx {

// error reporting shared by every entry point (api.cpp)
void set_error(const char* fmt, ...);
int check_launch(const char* what);

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then
// s_barrier.  __syncthreads() also drains the wave's outstanding global stores (vmcnt(0)),
// which in a conv epilogue serialises the whole output write before the LDS phase that
// follows it (the fused Gram tiles).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Deterministic block-wide sum (fixed tree order). `red` must hold
// blockDim.x/64 floats. Result valid in every thread.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
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

// Raw buffer loads with the hardware range check: an offset at or past the
// descriptor's byte count returns 0.  Gather loaders address every element through
// one per-chunk descriptor and mark padding/out-of-tile elements with BUF_OOB, so
// the fetch is straight-line code (no per-element exec branches, no serialising
// vmcnt(0) per load) and channel padding past the tensor end reads as zero.
constexpr uint32_t BUF_OOB = 0x80000000u;  // callers keep byte counts below this

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_srd(const float* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

__device__ __forceinline__ f32x4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t buf_ld2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x2_t, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}

// ReLU on the IEEE bit pattern: max(bits, 0) as signed ints keeps every non-negative float
// and maps every negative one (sign bit set) to +0 -- one v_max_i32, where fmaxf(x, 0.f)
// of a loaded x is two v_max_f32 (operand canonicalisation first)
__device__ __forceinline__ float relu_bits(float x) {
  return __int_as_float(max(__float_as_int(x), 0));
}
// relu(max of a 2x2 window) = the integer max of the four bit patterns and 0 (non-negative
// floats order like their bits; a negative float loses to 0 either way): two v_max3_i32.
// Exactly relu_bits(max_pool(x)); the bare int max of four floats is NOT their float max
// when all are negative, which is why the 0 is part of it.
__device__ __forceinline__ float pool4_bits(float a, float b, float c, float d) {
  const int m = max(max(__float_as_int(a), __float_as_int(b)),
                    max(max(__float_as_int(c), __float_as_int(d)), 0));
  return __int_as_float(m);
}


__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, byte_off, 0, 0);
}

// A max|.| bound ("amax") is a group of STX_AMAX_SLOTS floats whose maximum is the
// value: producers atomicMax into slot (block id % 32) so a 1024-block kernel does
// not serialise 1024 same-address atomics at its tail; consumers take the max of
// the group (wave-uniform loads).
__device__ __forceinline__ float read_amax(const float* __restrict__ g) {
  uint32_t m = 0u;
#pragma unroll
  for (int i = 0; i < STX_AMAX_SLOTS; ++i) m = max(m, __float_as_uint(g[i]) & 0x7fffffffu);
  return __uint_as_float(m);
}

// e with |a| < 2^e (frexp), clamped so 2^(15-e) and 2^(ex+ew-30) stay normal floats
// (the power-of-two scales of the fp16 hi/lo split operands)
__device__ __forceinline__ int amax_exp(float a) {
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

// A/B switches for measurement builds only.  The product library is built without STX_AB:
// every switch is its default, a compile-time constant, so no environment variable can
// change which kernel runs (and no variable name is left in the library).  `make AB=1`
// builds the measurement library, in which STX_KNOB reads the named integer variable.
#ifdef STX_AB
}  // namespace stx
#include <cstdlib>
namespace stx {
#define STX_KNOB(name, dflt) ([] { const char* e_ = getenv(name); return e_ ? atoi(e_) : (dflt); }())
#else
#define STX_KNOB(name, dflt) (dflt)
#endif

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline int rup(int a, int b) { return cdiv(a, b) * b; }

}  // namespace stx
