// Streaming Gram backward on the fp16 hi/lo split MFMA (the "1x1 mode" of stx_conv2d
// for the VGG widths C = 64 and 128):
//
//   out[n][co][p] = s * sum_c A[n][c][co] * z[n][c][p]                 (A = dL/dG op)
//                 + unpool(up_dp)[n][co][p] * [z[n][co][p] > 0]       (ReLU+MaxPool bwd)
//                 + aux_scale * aux[n][co][p]                         (folded content)
//
// StyleLoss backward dZ = (dG + dG^T) F / N (stransfer/network.py:92-108, the autograd
// of gram_matrix) plus the MaxPool2d/ReLU backward of the next layer
// (torch.nn.functional.max_pool2d backward: the gradient goes to the first maximum of
// each 2x2 window in row-major order).
//
// Why its own kernel: the work is 2*C^2 FLOPs per pixel over (2 + 1/4)*C*4 bytes --
// 7 (C=64) to 14 (C=128) FLOP/B, far under the split MFMA ridge -- so it is an HBM
// stream, not a conv.  Mapping (no LDS for pixels, no block barriers in the loop):
//
//  * a wave owns a unit of 2 rows x 32 columns (two 32-pixel MFMA N-blocks, one per
//    row; loads of a channel row are 128-B lines per half-wave) or, NB = 1, of
//    2 rows x 16 columns in one N-block;
//  * the K (input-channel) order is permuted so that the B fragment a lane loads for
//    chunk k holds exactly the channels of the output rows the lane's accumulators
//    cover (v_mfma_f32_32x32x16_f16: lane l holds B[K=8(l/32)+e][l%32] and
//    D[8(r/4)+4(l/32)+r%4][l%32]).  With pi(16k+8h+e) = 32(k/2)+8(2(k&1)+e/4)+4h+e%4
//    the ReLU mask and the 2x2 window argmax come from registers: the vertical
//    neighbour is the other N-block (same lane, same register), the horizontal one
//    lane l^1 (one DPP move);
//  * A' = A * 2^(15 - e(max|A|)) is split into hi/lo fragments in LDS once per block
//    (C=128: 64 KB) while the first unit's z loads are in flight; z' = z * 2^(15 - e(z))
//    is split in registers.  acc = sum A'z' (3 MFMA products, fp32-equivalent) and
//    the result is acc * s * 2^(e_A + e_z - 30), exact power-of-two de-scaling.
#include "common.h"
#include "conv_epi.h"
#include "gbwd16.h"

namespace stx {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int amax_exp16(float a) {  // a < 2^e (a = 0: e = 0)
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

__device__ __forceinline__ float swap_pair(float v) {  // lane l <- lane l^1
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}

// The first version (one kernel for every pooled-gradient / aux combination, decided at
// run time): kept for C = 128, where the compile-time variants spill.
template <int C, int NB, bool AUX, int NW, int CQ = C>
__global__ void __launch_bounds__(64 * NW, (NW == 8 || (C == 128 && NB == 2)) ? 1 : 2)
gram_bwd16_v1_kernel(Gb16 p) {
  constexpr int NT = 64 * NW;
  constexpr bool PREFETCH = C * NB <= 128;
  constexpr bool A_IN_REGS = C == 64;  // 64 VGPRs of A fragments stay resident
  constexpr int NK = C / 16, NCB = CQ / 32, FRAG = 64 * 16;
  static_assert(C % CQ == 0 && CQ % 32 == 0, "co split");
  __shared__ __attribute__((aligned(16))) char la[NCB * NK * 2 * FRAG];
  __shared__ float red[NW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n = blockIdx.y / (C / CQ), co0 = (blockIdx.y % (C / CQ)) * CQ;
  constexpr int UW = 16 * NB;  // unit width (columns)
  const int W = p.w, plane = p.h * p.w, ucols = W / UW, units = (p.h >> 1) * ucols;
  // lane pixel inside the unit: row offset (NB == 1: l32/16) and column
  const int lrow = NB == 1 ? (l32 >> 4) : 0, lcol = NB == 1 ? (l32 & 15) : l32;
  const uint32_t pl4 = (uint32_t)plane * 4u;
  const size_t img = (size_t)n * C * plane;
  const auto rz = make_srd(p.z + img, (uint32_t)C * pl4);
  const auto ro = make_srd(p.out + img, (uint32_t)C * pl4);
  const auto rx = make_srd(p.aux ? p.aux + img : p.out + img, (uint32_t)C * pl4);
  const auto rdp = make_srd(p.up_dp ? p.up_dp + img / 4 : p.out + img, (uint32_t)C * pl4 / 4u);
  const bool has_dp = p.up_dp != nullptr;
  constexpr bool has_aux = AUX;

  // channel of K slot (k, e) for this half-wave, as a byte offset past plane 4h
  auto zoff = [&](int k, int e) {
    return (uint32_t)(32 * (k >> 1) + 8 * (((k & 1) << 1) | (e >> 2)) + (e & 3)) * pl4;
  };
  float zr[NK][NB][8];
  auto lane_off = [&](int u, int& ry, int& cx) {
    ry = u / ucols;
    cx = u - ry * ucols;
    return (uint32_t)(4 * h * plane + (2 * ry + lrow) * W + cx * UW + lcol) * 4u;
  };
  auto load_unit = [&](int u) {
    int ry, cx;
    const uint32_t vo = lane_off(u, ry, cx);
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          zr[k][j][e] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rz, vo + j * W * 4, zoff(k, e), 0));
  };
  int u = blockIdx.x * NW + wave;
  const int ustride = gridDim.x * NW;
  if (u < units) load_unit(u);  // in flight while A is staged

  // ---- A' hi/lo fragments -> LDS (fragment (cb, k, P): lane ln's 16 B at ln*16) ----
  int ea;
  {
    constexpr int NA = C * CQ / NT;
    const float* A = p.coef + (size_t)n * p.coef_bs;
    float av[NA];  // all loads in flight at once (A is small and L2 resident)
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + NT * i, c = idx / CQ, co = co0 + idx - c * CQ;
      av[i] = A[(size_t)c * p.pitch + co];
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) m = fmaxf(m, fabsf(av[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) red[wave] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = fmaxf(m, red[i]);
    const float sa = __builtin_ldexpf(1.f, 15 - amax_exp16(m));
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + NT * i, c = idx / CQ, co = idx - c * CQ;  // co: block-local
      const int rem = c & 31, q = rem >> 3;
      const int k = 2 * (c >> 5) + (q >> 1), e = (q & 1) * 4 + (rem & 3);
      const int ln = ((rem >> 2) & 1) * 32 + (co & 31);
      const int f = ((co >> 5) * NK + k) * 2;
      const float v = av[i] * sa;
      const _Float16 hi = (_Float16)v;
      *reinterpret_cast<_Float16*>(la + f * FRAG + ln * 16 + e * 2) = hi;
      *reinterpret_cast<_Float16*>(la + (f + 1) * FRAG + ln * 16 + e * 2) =
          (_Float16)(v - (float)hi);
    }
    __syncthreads();
    ea = amax_exp16(m);
  }
  const int ez = amax_exp16(read_amax(p.z_amax));
  const float sz = __builtin_ldexpf(1.f, 15 - ez);
  const float fout = (p.acc_scale ? *p.acc_scale : 1.f) *
                     __builtin_ldexpf(1.f, ea + ez - 30);
  const int par = l32 & 1;
  uint32_t vmax_u = 0u;

  for (; u < units; u += ustride) {
    if constexpr (!PREFETCH) {
      if (u != blockIdx.x * NW + wave) load_unit(u);
    }
    int ry, cx;
    const uint32_t vo = lane_off(u, ry, cx);
    // opaque per unit: keeps the A fragment reads inside the loop (hoisted, C = 128
    // would pin 256 VGPRs of A for the kernel's lifetime)
    int abase = lane * 16;
    if constexpr (!A_IN_REGS) asm volatile("" : "+v"(abase));
    f32x16 acc[NCB][NB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][j][r] = 0.f;
    uint32_t sel[NCB];  // bit j*16 + r: element (cb, r, row j) receives the pooled grad
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) sel[cb] = 0u;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if (CQ == C && has_dp) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int r = ((k & 1) << 3) | ((e >> 2) << 2) | (e & 3);
          // the window's top/bottom rows at this lane's column and its partner's
          float za, zb;
          if constexpr (NB == 2) {
            za = zr[k][0][e];
            zb = zr[k][1][e];
          } else {
            const float zo = zr[k][0][e], zv = __shfl_xor(zo, 16, 64);
            za = lrow ? zv : zo;
            zb = lrow ? zo : zv;
          }
          const float pa = swap_pair(za), pb = swap_pair(zb);
          const float z0 = relu_bits(par ? pa : za), z1 = relu_bits(par ? za : pa);
          const float z2 = relu_bits(par ? pb : zb), z3 = relu_bits(par ? zb : pb);
          int bi = 0;
          float best = z0;
          if (z1 > best) { best = z1; bi = 1; }
          if (z2 > best) { best = z2; bi = 2; }
          if (z3 > best) { bi = 3; }
          if constexpr (NB == 2) {
            if (bi == par && za > 0.f) sel[k >> 1] |= 1u << r;
            if (bi == 2 + par && zb > 0.f) sel[k >> 1] |= 1u << (16 + r);
          } else {
            const float zo = lrow ? zb : za;
            if (bi == 2 * lrow + par && zo > 0.f) sel[k >> 1] |= 1u << r;
          }
        }
      }
      f16x8 bh[NB], bl[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = zr[k][j][e] * sz;
          const _Float16 vh = (_Float16)v;
          bh[j][e] = vh;
          bl[j][e] = (_Float16)(v - (float)vh);
        }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int f = (cb * NK + k) * 2;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(la + f * FRAG + abase);
        const f16x8 al = *reinterpret_cast<const f16x8*>(la + (f + 1) * FRAG + abase);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[cb][j], 0, 0, 0);
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], acc[cb][j], 0, 0, 0);
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], acc[cb][j], 0, 0, 0);
        }
      }
    }
    // next unit's loads go out before this unit's epilogue (where registers allow)
    const int un = u + ustride;
    if constexpr (PREFETCH) {
      if (un < units) load_unit(un);
    }

    const uint32_t vdp =
        (uint32_t)(4 * h * (plane >> 2) + ry * (W >> 1) + ((cx * UW + lcol) >> 1)) * 4u;
    // every pooled-gradient load of the unit goes out before the first store (vmcnt
    // counts stores too: a load issued after a store waits for it)
    float dpv[NCB][16];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t so = (uint32_t)(co0 + 32 * cb + 8 * (r >> 2) + (r & 3)) * (pl4 >> 2);
        dpv[cb][r] = (CQ == C && has_dp) ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                            rdp, vdp, so, 0))
                            : 0.f;
      }
    // aux rows of co-block cb+1 are loaded before the stores of cb (software pipeline)
    float axv[2][NB][16];
    auto load_aux = [&](int cb, float (&dst)[NB][16]) {
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t so = (uint32_t)(co0 + 32 * cb + 8 * (r >> 2) + (r & 3)) * pl4;
          dst[j][r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rx, vo + j * W * 4, so, 0));
        }
    };
    if (has_aux) load_aux(0, axv[0]);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      if (has_aux && cb + 1 < NCB) load_aux(cb + 1, axv[(cb + 1) & 1]);
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t so = (uint32_t)(co0 + 32 * cb + 8 * (r >> 2) + (r & 3)) * pl4;
          const uint32_t vj = vo + j * W * 4;
          float v = acc[cb][j][r] * fout;
          if ((sel[cb] >> (j * 16 + r)) & 1u) v += dpv[cb][r];
          if (has_aux) v += p.aux_scale * axv[cb & 1][j][r];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), ro, vj, so, 0);
          vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
        }
    }
  }
  if (p.out_amax) {  // one atomic per block into slot (block id & 31) of the group
    uint32_t mu = vmax_u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mu = max(mu, (uint32_t)__shfl_xor((int)mu, o, 64));
    __syncthreads();
    if (lane == 0) red[wave] = __uint_as_float(mu);
    __syncthreads();
    if (tid == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NW; ++i) r = max(r, __float_as_uint(red[i]));
      const int bid = blockIdx.x + gridDim.x * blockIdx.y;
      atomic_max_abs(p.out_amax + (bid & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

// NB = 2: a unit is 2 rows x 32 columns, one 32-pixel N-block per row (window
//         partners: the other N-block, lane l^1);
// NB = 1: a unit is 2 rows x 16 columns in one N-block, lane l32 -> row l32/16,
//         column l32%16 (window partners: lanes l^1, l^16, l^17) -- half the
//         registers, twice the units (the C = 128 occupancy case)
// NW waves per block share one staged A (C = 128: 8 waves, one 64 KB copy per CU)
// CQ: output channels per block (C for 64/128; a quarter of C = 256, whose A slice
// 64 x 256 is 64 KB of LDS).  With CQ < C the lane's loaded channels are not its
// accumulator rows, so the fused unpool (which relies on that) needs CQ == C.
// DP / AUX: the pooled-gradient and aux terms (compile time: no branch in the loop).
// PF: the next unit's z loads go out right after this unit's MFMAs.
//
// Memory-op order per unit (vmcnt counts every vector memory op in issue order, at most
// 63 outstanding are waited for exactly, and a wait across a branch that issued loads
// degrades to vmcnt(0)): MFMAs of u -> [pooled gradient + the first AXT aux co-blocks
// of u] -> [z of the next unit] -> [the other aux co-blocks] -> stores of u (waiting
// for the pooled gradient waits for at most one prefetch load).  Every load is unconditional: a wave past the last unit
// loads through an offset beyond the descriptor's range (zeros, no memory traffic).
template <int C, int NB, bool DP, bool AUX, int NW, int CQ, bool PF, int AXT>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 1 : 2)
gram_bwd16_kernel(Gb16 p) {
  constexpr int NT = 64 * NW;
  constexpr bool A_IN_REGS = C == 64 && !AUX;  // 64 VGPRs of A fragments stay resident
  constexpr int NK = C / 16, NCB = CQ / 32, FRAG = 64 * 16;
  static_assert(C % CQ == 0 && CQ % 32 == 0, "co split");
  static_assert(!DP || CQ == C, "the fused unpool needs CQ == C");
  static_assert(AXT <= NCB, "aux split");
  constexpr uint32_t OOR = 0x80000000u;  // beyond every descriptor's num_records
  __shared__ __attribute__((aligned(16))) char la[NCB * NK * 2 * FRAG];
  __shared__ float red[NW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int n = blockIdx.y / (C / CQ), co0 = (blockIdx.y % (C / CQ)) * CQ;
  constexpr int UW = 16 * NB;  // unit width (columns)
  const int W = p.w, plane = p.h * p.w, ucols = W / UW, units = (p.h >> 1) * ucols;
  // lane pixel inside the unit: row offset (NB == 1: l32/16) and column
  const int lrow = NB == 1 ? (l32 >> 4) : 0, lcol = NB == 1 ? (l32 & 15) : l32;
  const uint32_t pl4 = (uint32_t)plane * 4u;
  const size_t img = (size_t)n * C * plane;
  const auto rz = make_srd(p.z + img, (uint32_t)C * pl4);
  const auto ro = make_srd(p.out + img, (uint32_t)C * pl4);
  const auto rx = make_srd(AUX ? p.aux + img : p.out + img, (uint32_t)C * pl4);
  const auto rdp = make_srd(DP ? p.up_dp + img / 4 : p.out + img, (uint32_t)C * pl4 / 4u);

  // channel of K slot (k, e) for this half-wave, as a byte offset past plane 4h
  auto zoff = [&](int k, int e) {
    return (uint32_t)(32 * (k >> 1) + 8 * (((k & 1) << 1) | (e >> 2)) + (e & 3)) * pl4;
  };
  float zr[NK][NB][8];
  auto lane_off = [&](int u) {
    const int ry = u / ucols, cx = u - ry * ucols;
    return (uint32_t)(4 * h * plane + (2 * ry + lrow) * W + cx * UW + lcol) * 4u;
  };
  auto load_unit = [&](uint32_t vo) {
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          zr[k][j][e] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rz, vo + j * W * 4, zoff(k, e), 0));
  };
  const int u0 = blockIdx.x * NW + wave;
  const int ustride = gridDim.x * NW;
  load_unit(u0 < units ? lane_off(u0) : OOR);  // in flight while A is staged

  // ---- A' hi/lo fragments -> LDS (fragment (cb, k, P): lane ln's 16 B at ln*16) ----
  int ea;
  {
    constexpr int NA = C * CQ / NT;
    const float* A = p.coef + (size_t)n * p.coef_bs;
    float av[NA];  // all loads in flight at once (A is small and L2 resident)
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + NT * i, c = idx / CQ, co = co0 + idx - c * CQ;
      av[i] = A[(size_t)c * p.pitch + co];
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) m = fmaxf(m, fabsf(av[i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) red[wave] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) m = fmaxf(m, red[i]);
    const float sa = __builtin_ldexpf(1.f, 15 - amax_exp16(m));
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = tid + NT * i, c = idx / CQ, co = idx - c * CQ;  // co: block-local
      const int rem = c & 31, q = rem >> 3;
      const int k = 2 * (c >> 5) + (q >> 1), e = (q & 1) * 4 + (rem & 3);
      const int ln = ((rem >> 2) & 1) * 32 + (co & 31);
      const int f = ((co >> 5) * NK + k) * 2;
      const float v = av[i] * sa;
      const _Float16 hi = (_Float16)v;
      *reinterpret_cast<_Float16*>(la + f * FRAG + ln * 16 + e * 2) = hi;
      *reinterpret_cast<_Float16*>(la + (f + 1) * FRAG + ln * 16 + e * 2) =
          (_Float16)(v - (float)hi);
    }
    __syncthreads();
    ea = amax_exp16(m);
  }
  const int ez = amax_exp16(read_amax(p.z_amax));
  const float sz = __builtin_ldexpf(1.f, 15 - ez);
  const float fout = (p.acc_scale ? *p.acc_scale : 1.f) *
                     __builtin_ldexpf(1.f, ea + ez - 30);
  const int par = l32 & 1;
  uint32_t vmax_u = 0u;
  // output-channel byte offset of accumulator element (cb, r) within a plane stack
  auto co_off = [&](int cb, int r) { return (uint32_t)(co0 + 32 * cb + 8 * (r >> 2) + (r & 3)); };

  for (int u = u0; u < units; u += ustride) {
    if constexpr (!PF) {
      if (u != u0) load_unit(lane_off(u));
    }
    const int ry = u / ucols, cx = u - ry * ucols;
    const uint32_t vo = lane_off(u);
    // opaque per unit: keeps the A fragment reads inside the loop (hoisted, C = 128
    // would pin 256 VGPRs of A for the kernel's lifetime)
    int abase = lane * 16;
    if constexpr (!A_IN_REGS) asm volatile("" : "+v"(abase));
    f32x16 acc[NCB][NB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[cb][j][r] = 0.f;
    uint32_t sel[NCB];  // bit j*16 + r: element (cb, r, row j) receives the pooled grad
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) sel[cb] = 0u;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if constexpr (DP) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int r = ((k & 1) << 3) | ((e >> 2) << 2) | (e & 3);
          // the window's top/bottom rows at this lane's column and its partner's
          float za, zb;
          if constexpr (NB == 2) {
            za = zr[k][0][e];
            zb = zr[k][1][e];
          } else {
            const float zo = zr[k][0][e], zv = __shfl_xor(zo, 16, 64);
            za = lrow ? zv : zo;
            zb = lrow ? zo : zv;
          }
          const float pa = swap_pair(za), pb = swap_pair(zb);
          const float z0 = relu_bits(par ? pa : za), z1 = relu_bits(par ? za : pa);
          const float z2 = relu_bits(par ? pb : zb), z3 = relu_bits(par ? zb : pb);
          int bi = 0;
          float best = z0;
          if (z1 > best) { best = z1; bi = 1; }
          if (z2 > best) { best = z2; bi = 2; }
          if (z3 > best) { bi = 3; }
          if constexpr (NB == 2) {
            if (bi == par && za > 0.f) sel[k >> 1] |= 1u << r;
            if (bi == 2 + par && zb > 0.f) sel[k >> 1] |= 1u << (16 + r);
          } else {
            const float zo = lrow ? zb : za;
            if (bi == 2 * lrow + par && zo > 0.f) sel[k >> 1] |= 1u << r;
          }
        }
      }
      f16x8 bh[NB], bl[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = zr[k][j][e] * sz;
          const _Float16 vh = (_Float16)v;
          bh[j][e] = vh;
          bl[j][e] = (_Float16)(v - (float)vh);
        }
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int f = (cb * NK + k) * 2;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(la + f * FRAG + abase);
        const f16x8 al = *reinterpret_cast<const f16x8*>(la + (f + 1) * FRAG + abase);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[cb][j], 0, 0, 0);
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], acc[cb][j], 0, 0, 0);
          acc[cb][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], acc[cb][j], 0, 0, 0);
        }
      }
      // one K chunk at a time: hoisting the next chunks' splits would hold them all live
      __builtin_amdgcn_sched_barrier(0);
    }
    // the unit's pooled gradients and first aux co-blocks, then the next unit's z
    const uint32_t vdp =
        (uint32_t)(4 * h * (plane >> 2) + ry * (W >> 1) + ((cx * UW + lcol) >> 1)) * 4u;
    float dpv[NCB][16];
    if constexpr (DP) {
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          dpv[cb][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rdp, vdp, co_off(cb, r) * (pl4 >> 2), 0));
    }
    float axv[NCB][NB][16];
    auto load_aux = [&](int cb) {
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          axv[cb][j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                        rx, vo + j * W * 4, co_off(cb, r) * pl4, 0));
    };
    if constexpr (AUX) {
#pragma unroll
      for (int cb = 0; cb < AXT; ++cb) load_aux(cb);
    }
    if constexpr (PF) {
      const int un = u + ustride;
      load_unit(un < units ? lane_off(un) : OOR);
    }
    if constexpr (AUX) {
#pragma unroll
      for (int cb = AXT; cb < NCB; ++cb) load_aux(cb);
    }
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[cb][j][r] * fout;
          if constexpr (DP)
            if ((sel[cb] >> (j * 16 + r)) & 1u) v += dpv[cb][r];
          if constexpr (AUX) v += p.aux_scale * axv[cb][j][r];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), ro,
                                                vo + j * W * 4, co_off(cb, r) * pl4, 0);
          vmax_u = max(vmax_u, __float_as_uint(v) & 0x7fffffffu);
        }
  }
  if (p.out_amax) {  // one atomic per block into slot (block id & 31) of the group
    uint32_t mu = vmax_u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mu = max(mu, (uint32_t)__shfl_xor((int)mu, o, 64));
    __syncthreads();
    if (lane == 0) red[wave] = __uint_as_float(mu);
    __syncthreads();
    if (tid == 0) {
      uint32_t r = 0u;
#pragma unroll
      for (int i = 0; i < NW; ++i) r = max(r, __float_as_uint(red[i]));
      const int bid = blockIdx.x + gridDim.x * blockIdx.y;
      atomic_max_abs(p.out_amax + (bid & (STX_AMAX_SLOTS - 1)), __uint_as_float(r));
    }
  }
}

template <int C, int NB, bool DP, bool AUX, int CQ, bool PF, int AXT>
static void launch_gb1(const Gb16& p, int nimg, hipStream_t st) {
  constexpr int NW = (C == 128 && NB == 1) ? 8 : 4;
  constexpr int slots = NW == 8 ? 256 : 512;  // resident blocks (2048 waves)
  constexpr int NQ = C / CQ;
  const int units = (p.h / 2) * (p.w / (16 * NB));
  const int per_img =
      std::max(1, std::min((units + NW - 1) / NW, std::max(1, slots / (nimg * NQ))));
  hipLaunchKernelGGL((gram_bwd16_kernel<C, NB, DP, AUX, NW, CQ, PF, AXT>),
                     dim3(per_img, nimg * NQ), dim3(64 * NW), 0, st, p);
}

template <int C, int NB, int CQ, bool PF, int AXT>
static void launch_gb(const Gb16& p, int nimg, hipStream_t st) {
  const bool dp = p.up_dp != nullptr, aux = p.aux != nullptr;
  if constexpr (CQ == C) {
    if (dp && aux) return launch_gb1<C, NB, true, true, CQ, PF, AXT>(p, nimg, st);
    if (dp) return launch_gb1<C, NB, true, false, CQ, PF, AXT>(p, nimg, st);
  }
  if (aux) return launch_gb1<C, NB, false, true, CQ, PF, AXT>(p, nimg, st);
  launch_gb1<C, NB, false, false, CQ, PF, AXT>(p, nimg, st);
}

// C in {64, 128, 256} (256: no up_dp), h even, w % 16 == 0, dense channels; the caller
// (stx_conv2d's split 1x1 mode) checks the rest of the contract.
template <int C, int NB, int CQ>
static void launch_gb_v1(const Gb16& p, int nimg, hipStream_t st) {
  constexpr int NW = (C == 128 && NB == 1) ? 8 : 4;
  constexpr int slots = NW == 8 ? 256 : 512;  // resident blocks (2048 waves)
  constexpr int NQ = C / CQ;
  const int units = (p.h / 2) * (p.w / (16 * NB));
  const dim3 grid(std::max(1, std::min((units + NW - 1) / NW, std::max(1, slots / (nimg * NQ)))),
                  nimg * NQ);
  if (p.aux)
    hipLaunchKernelGGL((gram_bwd16_v1_kernel<C, NB, true, NW, CQ>), grid, dim3(64 * NW), 0, st, p);
  else
    hipLaunchKernelGGL((gram_bwd16_v1_kernel<C, NB, false, NW, CQ>), grid, dim3(64 * NW), 0, st, p);
}

// C in {64, 128, 256} (256: no up_dp), h even, w % 16 == 0, dense channels; the caller
// (stx_conv2d's split 1x1 mode) checks the rest of the contract.
int gram_bwd16_launch(const Gb16& p, int nimg, int c, hipStream_t st) {
  static const int nb_env = STX_KNOB("STX_GB_NB", 0);
  // STX_GB_V1=1: the run-time-branch loop schedule (A/B)
  static const bool v1 = STX_KNOB("STX_GB_V1", 0) != 0;
  const bool two = (nb_env ? nb_env : 2) == 2 && p.w % 32 == 0;
  if (c == 64) {
    if (v1 || p.aux)
      two ? launch_gb_v1<64, 2, 64>(p, nimg, st) : launch_gb_v1<64, 1, 64>(p, nimg, st);
    else
      two ? launch_gb<64, 2, 64, true, 2>(p, nimg, st) : launch_gb<64, 1, 64, true, 2>(p, nimg, st);
  } else if (c == 128) {
    launch_gb_v1<128, 1, 128>(p, nimg, st);
  } else {  // C = 256 (conv3_1): no fused unpool
    if (v1)
      launch_gb_v1<256, 1, 64>(p, nimg, st);
    else
      launch_gb<256, 1, 64, false, 2>(p, nimg, st);
  }
  return check_launch("stx_conv2d(gram backward, split 1x1)");
}

}  // namespace stx
