// Weight gradient of the ImageTransformNet's 9x9 layers (3 <-> 32 channels) on the
// fp16 hi/lo split MFMA (numerics as conv16.hip: per-tensor power-of-two scales,
// s*v = hi + lo, hi*hi + hi*lo + lo*hi accumulated in fp32).
//
// ImageTransformNet conv0 (3 -> 32) and conv22 (32 -> 3), 9x9 stride 1 pad 4
// (stransfer/network.py:525-527, 605-609), trained by static_train (:690-765).  As a
// GEMM their wgrad has M = 3 or 32 channels, N = the other side x 81 taps and K =
// every pixel: the generic tiled kernel wastes most of a 64/128-wide tile on the
// 3-channel side and needs a large split-K reduction (1.1 ms for conv22 at B=8 256^2).
//
// Here the 3-channel tensor S is the im2col side and the 32-channel tensor L the
// other:
//   conv0:  S = x (the image), L = dY:  dW[l][s][t] = sum_p L[l][p] * S[s][p + d_t]
//   conv22: S = dY, L = x:              dW[s][l][t] = sum_q S[s][q - d_t] * L[l][q]
// with d_t = (kh - 4, kw - 4).  For one tap row kh, rows (s, kw) -- 27 of an MFMA's 32
// -- times the 32 L channels is one v_mfma_f32_32x32x16_f16 tile per 16 pixels, so a
// 16-pixel K-step is 9 tiles x 3 split products.  A block owns 4 image rows x 256
// columns: it stages S rows y0-4 .. y0+7 (zero halo) in LDS once, already scaled and
// split (one dword = fp16 hi | fp16 lo << 16), and each wave streams one row of L
// (two float4 per lane per step, split in registers).  A lane's A fragment is 8
// consecutive S pixels shifted by its (s, kw) row: 8 LDS dwords and 8 v_perm.  The
// 4 waves are summed through LDS in a fixed order into one partial per block; a
// second kernel sums the blocks in a fixed order (bit-reproducible, no atomics).
#include "common.h"
#include "../../include/stx.h"

namespace stx {

typedef _Float16 f16x8_w9 __attribute__((ext_vector_type(8)));

namespace {

constexpr int W9_TW = 256;              // columns per unit
constexpr int W9_ROWS = 4;              // rows per unit (one per wave)
constexpr int W9_SR = W9_ROWS + 8;      // staged S rows
constexpr int W9_SC = W9_TW + 8;        // staged S columns (4-column zero halo)
constexpr int W9_SCP = W9_SC + 1;       // LDS row pitch (dwords)
constexpr int W9_NS = 3;                // small-side channels (27 of 32 tile rows)
constexpr int W9_PART = 9 * 32 * 32;    // floats per block partial [kh][row][l]
constexpr int W9_LPF = 3;               // L steps in flight ahead of the MFMAs
constexpr int W9_SB = 10;               // S staging: loads per thread per batch
constexpr int W9_STG = (W9_NS * W9_SR * W9_SC + 255) / 256 + (W9_SB - 1) -
                       ((W9_NS * W9_SR * W9_SC + 255) / 256 + W9_SB - 1) % W9_SB;  // 40

struct Wf9 {
  const float* S;       // [n][ns][h][w]
  const float* L;       // [n][32][h][w]
  const float* s_amax;  // amax groups
  const float* l_amax;
  float* part;          // [blocks][9][32][32]
  int n, ns, h, w;
  int sgn;              // +1: S at p + d (conv0), -1: S at p - d (conv22)
  int tiles_x, units;
};

__device__ __forceinline__ int w9_exp(float a) {
  int e = 0;
  frexpf(a, &e);
  return min(max(e, -60), 60);
}

__device__ __forceinline__ uint32_t w9_pack(float v) {  // fp16 hi | fp16 lo << 16
  const _Float16 hi = (_Float16)v;
  const _Float16 lo = (_Float16)(v - (float)hi);
  return (uint32_t)__builtin_bit_cast(uint16_t, hi) |
         ((uint32_t)__builtin_bit_cast(uint16_t, lo) << 16);
}

__global__ void __launch_bounds__(256, 2) wgrad9_kernel(Wf9 p) {
  __shared__ uint32_t st[W9_NS * W9_SR * W9_SCP];  // 51 KB; reused for the wave sum
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int plane = p.h * p.w;
  const float sS = __builtin_ldexpf(1.f, 15 - w9_exp(read_amax(p.s_amax)));
  const int eL = w9_exp(read_amax(p.l_amax));
  const float sL = __builtin_ldexpf(1.f, 15 - eL);

  f32x16 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;

  // this lane's A row: (s, kw) = (l32 / 9, l32 % 9); rows past 3*9 (or ns*9) read a
  // valid LDS row and produce discarded tile rows
  const int s_row = min(l32 / 9, p.ns - 1), kw = l32 % 9;
  const int sgn = p.sgn;

  for (int u = blockIdx.x; u < p.units; u += gridDim.x) {
    const int rows_u = (p.h + W9_ROWS - 1) / W9_ROWS;
    const int tx = u % p.tiles_x, rest = u / p.tiles_x;
    const int ry = rest % rows_u, n = rest / rows_u;
    const int y0 = ry * W9_ROWS, x0 = tx * W9_TW;
    __syncthreads();  // previous unit's LDS reads are done
    {
      // the S window in batches of W9_SB elements per thread: every load of a batch issued
      // before the first use (unconditional descriptor loads: outside the image or past
      // ns channels read 0), then split and stored
      const auto rs = make_srd(p.S + (size_t)n * p.ns * plane, (uint32_t)(p.ns * plane) * 4u);
      const int nel = p.ns * W9_SR * W9_SC;
#pragma unroll 1
      for (int b0 = 0; b0 < W9_STG; b0 += W9_SB) {
        float v[W9_SB];
#pragma unroll
        for (int j = 0; j < W9_SB; ++j) {
          const int idx = tid + 256 * (b0 + j);
          const int s = idx / (W9_SR * W9_SC), rem = idx - s * (W9_SR * W9_SC);
          const int rr = rem / W9_SC, cc = rem - rr * W9_SC;
          const int y = y0 - 4 + rr, x = x0 - 4 + cc;
          const bool ok = idx < nel && y >= 0 && y < p.h && x >= 0 && x < p.w;
          v[j] = buf_ld(rs, ok ? (uint32_t)(s * plane + y * p.w + x) * 4u : BUF_OOB);
        }
#pragma unroll
        for (int j = 0; j < W9_SB; ++j) {
          const int idx = tid + 256 * (b0 + j);
          if (idx < nel) {
            const int s = idx / (W9_SR * W9_SC), rem = idx - s * (W9_SR * W9_SC);
            const int rr = rem / W9_SC, cc = rem - rr * W9_SC;
            st[(s * W9_SR + rr) * W9_SCP + cc] = w9_pack(v[j] * sS);
          }
        }
      }
    }
    __syncthreads();
    const int y = y0 + wave;
    if (y < p.h) {
      const float* Lrow = p.L + ((size_t)n * 32 + l32) * plane + (size_t)y * p.w;
      const int xend = min(W9_TW, p.w - x0);
      // the L row in 16-pixel steps with the next W9_LPF steps' loads in flight (one
      // exposed HBM latency per row instead of one per step); loads past the row's end
      // read the row start (valid memory, never used)
      f32x4 lr[W9_LPF + 1][2];
#pragma unroll
      for (int k = 0; k < W9_LPF; ++k) {
        const int xo = 16 * k < xend ? 16 * k : 0;
        lr[k][0] = *reinterpret_cast<const f32x4*>(Lrow + x0 + xo + 8 * h);
        lr[k][1] = *reinterpret_cast<const f32x4*>(Lrow + x0 + xo + 8 * h + 4);
      }
      for (int xs = 0; xs < xend; xs += 16 * (W9_LPF + 1)) {
#pragma unroll
      for (int k = 0; k <= W9_LPF; ++k) {
        {
          const int xn = xs + 16 * (k + W9_LPF), xo = xn < xend ? xn : 0;
          lr[(k + W9_LPF) % (W9_LPF + 1)][0] = *reinterpret_cast<const f32x4*>(Lrow + x0 + xo + 8 * h);
          lr[(k + W9_LPF) % (W9_LPF + 1)][1] = *reinterpret_cast<const f32x4*>(Lrow + x0 + xo + 8 * h + 4);
        }
        if (xs + 16 * k >= xend) break;
        // B: L[l32][y][x0 + xs + 16k + 8h .. +7], split in registers
        const f32x4 v0 = lr[k][0], v1 = lr[k][1];
        f16x8_w9 bh, bl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (e < 4 ? v0[e] : v1[e - 4]) * sL;
          const _Float16 vh = (_Float16)v;
          bh[e] = vh;
          bl[e] = (_Float16)(v - (float)vh);
        }
        // A rows (s, kw) for each tap row kh: S at pixel (y + sgn(kh-4), x + sgn(kw-4))
        const int cbase = xs + 16 * k + 8 * h + 4 + sgn * (kw - 4);
#pragma unroll
        for (int kh = 0; kh < 9; ++kh) {
          const int rr = wave + 4 + sgn * (kh - 4);
          const uint32_t* src = st + (s_row * W9_SR + rr) * W9_SCP + cbase;
          uint32_t d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = src[e];
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          u32x4 hi, lo;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            hi[q] = __builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x05040100u);
            lo[q] = __builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x07060302u);
          }
          const f16x8_w9 ah = __builtin_bit_cast(f16x8_w9, hi);
          const f16x8_w9 al = __builtin_bit_cast(f16x8_w9, lo);
          acc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[kh], 0, 0, 0);
          acc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[kh], 0, 0, 0);
          acc[kh] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[kh], 0, 0, 0);
        }
      }
      }
    }
  }
  // fixed-order sum of the 4 waves through LDS (9 x 32 x 32 floats = 36 KB), de-scaled
  __syncthreads();
  float* red = reinterpret_cast<float*>(st);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int kh = 0; kh < 9; ++kh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = 8 * (r >> 2) + 4 * h + (r & 3);
          float* d = red + (kh * 32 + row) * 32 + l32;
          *d = (w == 0 ? 0.f : *d) + acc[kh][r];
        }
    }
    __syncthreads();
  }
  const float descale = __builtin_ldexpf(1.f, w9_exp(read_amax(p.s_amax)) + eL - 30);
  float* out = p.part + (size_t)blockIdx.x * W9_PART;
  for (int i = tid; i < W9_PART; i += 256) out[i] = red[i] * descale;
}

// dW from the block partials, blocks summed in a fixed order.  A block takes 32
// consecutive partial entries; its 8 thread groups stride over the blocks' partials
// (coalesced 128-B rows) and are combined in group order.  conv0 (S = x):
// dw[l][s][kh][kw]; conv22 (S = dY): dw[s][l][kh][kw].
constexpr int W9R_OB = 32, W9R_G = 8;
__global__ void __launch_bounds__(W9R_OB * W9R_G)
wgrad9_reduce_kernel(const float* __restrict__ part, int nparts, float* dw, int ns, int s_is_x,
                     int accumulate) {
  __shared__ float red[W9R_G][W9R_OB];
  const int t = threadIdx.x, oi = t % W9R_OB, g = t / W9R_OB;
  const int o = blockIdx.x * W9R_OB + oi;  // [kh][row = s*9 + kw][l]
  float v = 0.f;
#pragma unroll 8
  for (int b = g; b < nparts; b += W9R_G) v += part[(size_t)b * W9_PART + o];
  red[g][oi] = v;
  __syncthreads();
  if (g != 0) return;
  float sum = red[0][oi];
#pragma unroll
  for (int i = 1; i < W9R_G; ++i) sum += red[i][oi];
  const int kh = o / (32 * 32), row = (o / 32) % 32, l = o % 32;
  if (row >= ns * 9) return;
  const int s = row / 9, kw = row - s * 9, tap = kh * 9 + kw;
  const size_t i = s_is_x ? ((size_t)l * ns + s) * 81 + tap : ((size_t)s * 32 + l) * 81 + tap;
  dw[i] = accumulate ? dw[i] + sum : sum;
}

bool w9_plan(int n, int cin, int cout, int ks, int h, int w, int& ns, int& s_is_x, int& units,
             int& tiles_x, int& blocks) {
  if (ks != 9 || n <= 0 || h <= 0 || w <= 0 || w % 16) return false;
  if (cin <= W9_NS && cout == 32) {
    ns = cin;
    s_is_x = 1;
  } else if (cout <= W9_NS && cin == 32) {
    ns = cout;
    s_is_x = 0;
  } else {
    return false;
  }
  if ((size_t)32 * h * w * 4 >= (1ull << 31)) return false;
  tiles_x = (w + W9_TW - 1) / W9_TW;
  units = n * ((h + W9_ROWS - 1) / W9_ROWS) * tiles_x;
  blocks = std::min(units, 512);
  return true;
}

}  // namespace
}  // namespace stx

using namespace stx;

extern "C" size_t stx_conv2d_wgrad_few16_ws(int n, int cin, int cout, int ks, int h, int w) {
  int ns, sx, units, tiles_x, blocks;
  if (!w9_plan(n, cin, cout, ks, h, w, ns, sx, units, tiles_x, blocks)) return 0;
  return (size_t)blocks * W9_PART * sizeof(float);
}

extern "C" int stx_conv2d_wgrad_few16(const float* x, const float* dy, float* dw, int accumulate,
                                      int n, int cin, int h, int w, int cout, int ks, int pad,
                                      const float* x_amax, const float* dy_amax, void* ws,
                                      size_t ws_bytes, void* stream) {
  int ns, sx, units, tiles_x, blocks;
  if (!x || !dy || !dw || !x_amax || !dy_amax || pad != ks / 2 ||
      !w9_plan(n, cin, cout, ks, h, w, ns, sx, units, tiles_x, blocks)) {
    set_error("stx_conv2d_wgrad_few16: unsupported shape (9x9 pad 4, 1..3 <-> 32 channels, "
              "w %% 16 == 0) or missing pointers");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < (size_t)blocks * W9_PART * sizeof(float)) {
    set_error("stx_conv2d_wgrad_few16: workspace");
    return STX_E_WORKSPACE;
  }
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy)) & 15) {
    set_error("stx_conv2d_wgrad_few16: 16-byte aligned x and dy required");
    return STX_E_INVALID;
  }
  Wf9 p;
  p.S = sx ? x : dy;
  p.L = sx ? dy : x;
  p.s_amax = sx ? x_amax : dy_amax;
  p.l_amax = sx ? dy_amax : x_amax;
  p.part = reinterpret_cast<float*>(ws);
  p.n = n;
  p.ns = ns;
  p.h = h;
  p.w = w;
  p.sgn = sx ? 1 : -1;
  p.tiles_x = tiles_x;
  p.units = units;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wgrad9_kernel, dim3(blocks), dim3(256), 0, st, p);
  hipLaunchKernelGGL(wgrad9_reduce_kernel, dim3(W9_PART / W9R_OB), dim3(W9R_OB * W9R_G), 0, st,
                     p.part, blocks, dw, ns, sx, accumulate);
  return check_launch("stx_conv2d_wgrad_few16");
}
