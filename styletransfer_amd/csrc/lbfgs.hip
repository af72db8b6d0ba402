// On-device L-BFGS in the compact (Byrd-Nocedal-Schnabel) form: the search direction
// of torch.optim.LBFGS (the optimiser of StyleNetwork.train_gatys,
// stransfer/network.py:411-458: lr 1, max_iter 20, tolerance_change 1e-9,
// history_size 100, no line search) in a fixed number of launches per iteration
// whatever the history length.
//
// torch's two-loop recursion walks the m stored pairs one at a time (a dot product,
// then an axpy, twice per pair: ~4m dependent vector launches per iteration).  The
// same direction, d = -H g with H the L-BFGS inverse-Hessian approximation
//   H = gI + [S gY] [[R^-T (D + g Y^T Y) R^-1, -R^-T], [-R^-1, 0]] [S^T; gY^T]
// (S, Y the pairs as columns, R_ij = s_i.y_j for i <= j, D = diag(s_i.y_i), g = H_diag),
// is two passes over the history slabs and an m x m solve:
//   dots     u = S^T g, w = Y^T g (and, for a newly accepted pair, S^T y_new, Y^T y_new:
//            the new column of R and row of Y^T Y) -- one read of S and Y
//   solve    r = R^-1 u; a = R^-T ((D + g Y^T Y) r - g w)   (one block, fp64, R^-1 kept
//            up to date: three matrix-vector products, no serial substitution)
//   combine  d = -g g - S a + g Y r; s_next = t d; g.d; max|t d| -- one read of S and Y
// so an iteration reads the 2m history vectors twice (torch: twice too, in 4m launches).
//
// History: a ring of m + 1 slots of [S | Y] (the spare slot holds the candidate pair, so a
// rejected pair (y.s <= 1e-10) never overwrites a committed one); the chronological order,
// R, Y^T Y, H_diag, the step size and torch's iteration counter live in a device state
// block, so an iteration is a fixed launch sequence (capturable in a hipGraph) and the host
// reads back only the scalars torch's control flow branches on.
#include "common.h"
#include "../../include/stx.h"

namespace stx {
namespace {

constexpr int LB_MAXM = 256;   // largest history size
constexpr int LB_CHUNK = 1024; // elements per block of the history passes (256 x float4)
constexpr int LB_G = 512;      // blocks of the grid-stride passes (fixed: fixed sum order)
constexpr int LB_NT = 256;

struct LbHdr {
  int count, n_iter, cand, flag, accepted, pad0, pad1, pad2;
  float H_diag, t, ys, yy, gtd, dmax, pad3, pad4;
  int order[LB_MAXM + 1];  // committed slots, oldest first
};

struct LbLayout {
  int m1;
  size_t sy, yy, ri, dots, coef, total;
  __host__ __device__ explicit LbLayout(int m) {
    m1 = m + 1;
    size_t o = (sizeof(LbHdr) + 255) & ~size_t(255);
    sy = o;
    o += sizeof(double) * m1 * m1;  // s_i . y_j by slot
    yy = o;
    o += sizeof(double) * m1 * m1;  // y_i . y_j by slot
    ri = o;
    o += sizeof(double) * m1 * m1;  // (R^-1)_ij by slot (upper triangle in chronological order)
    dots = o;
    o += sizeof(double) * 4 * m1;   // per chronological pair: s.g, y.g, s.yn, y.yn
    coef = o;
    o += sizeof(float) * 2 * m1;    // combination coefficients of s_k, y_k
    total = (o + 255) & ~size_t(255);
  }
};

__host__ __device__ inline long long lb_npad(long long n) {
  return (n + LB_CHUNK - 1) / LB_CHUNK * LB_CHUNK;
}

__device__ __forceinline__ f32x4 ld4g(const float* __restrict__ p, long long e, long long n) {
  if (e + 3 < n) return *reinterpret_cast<const f32x4*>(p + e);
  f32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = e + k < n ? p[e + k] : 0.f;
  return v;
}

__device__ __forceinline__ float nanmax(float a, float b) {
  return (a != a || b != b) ? __int_as_float(0x7fc00000) : fmaxf(a, b);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nanmax(v, __shfl_xor(v, o, 64));
  return v;
}

// fixed-order block reduction of two values (sum, sum | max) over 256 threads
template <bool MAX2>
__device__ __forceinline__ void block_red2(float& a, float& b, float* red) {
  a = wave_sum(a);
  b = MAX2 ? wave_max(b) : wave_sum(b);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[w] = a;
    red[4 + w] = b;
  }
  __syncthreads();
  a = (red[0] + red[1]) + (red[2] + red[3]);
  b = MAX2 ? nanmax(nanmax(red[4], red[5]), nanmax(red[6], red[7]))
           : (red[4] + red[5]) + (red[6] + red[7]);
}

// K1: y_cand = g - prev_g (into the candidate Y slot), prev_g = g; partials of y.s_cand
// and y.y (s_cand = t d of the previous iteration, written by lb_combine_kernel)
__global__ void __launch_bounds__(LB_NT)
lb_pair_kernel(const float* __restrict__ g, float* __restrict__ prev_g, float* __restrict__ hist,
               long long n, long long np, int m1, const LbHdr* __restrict__ hdr,
               float* __restrict__ parts) {
  __shared__ float red[8];
  const bool first = hdr->n_iter == 0;
  const int cand = hdr->cand;
  const float* __restrict__ s = hist + (size_t)cand * np;
  float* __restrict__ y = hist + (size_t)(m1 + cand) * np;
  float ys = 0.f, yy = 0.f;
  const long long n4 = np >> 2;
  for (long long i = blockIdx.x * (long long)LB_NT + threadIdx.x; i < n4;
       i += (long long)gridDim.x * LB_NT) {
    const long long e = 4 * i;
    const f32x4 gv = ld4g(g, e, n);
    if (!first) {
      const f32x4 pg = *reinterpret_cast<const f32x4*>(prev_g + e);
      const f32x4 sv = *reinterpret_cast<const f32x4*>(s + e);
      const f32x4 yv = gv - pg;
      *reinterpret_cast<f32x4*>(y + e) = yv;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ys = fmaf(yv[k], sv[k], ys);
        yy = fmaf(yv[k], yv[k], yy);
      }
    }
    *reinterpret_cast<f32x4*>(prev_g + e) = gv;
  }
  block_red2<false>(ys, yy, red);
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = ys;
    parts[2 * blockIdx.x + 1] = yy;
  }
}

// K2 (one block): torch's per-iteration scalar logic -- n_iter += 1; step size t (first
// iteration: min(1, 1/sum|g|) * lr, else lr); accept the candidate pair when y.s > 1e-10
// (evicting the oldest when the ring holds m), H_diag = y.s / y.y
__global__ void __launch_bounds__(LB_NT)
lb_commit_kernel(LbHdr* __restrict__ hdr, char* __restrict__ st, float* __restrict__ scal,
                 const float* __restrict__ parts, int m, float lr) {
  __shared__ float red[8];
  float ys = parts[2 * threadIdx.x] + parts[2 * (threadIdx.x + LB_NT)];
  float yy = parts[2 * threadIdx.x + 1] + parts[2 * (threadIdx.x + LB_NT) + 1];
  block_red2<false>(ys, yy, red);
  if (threadIdx.x != 0) return;
  const LbLayout L(m);
  const int n_iter = hdr->n_iter + 1;
  hdr->n_iter = n_iter;
  int accepted = 0;
  float t = lr;
  if (n_iter == 1) {
    hdr->H_diag = 1.f;
    t = fminf(1.f, 1.f / scal[2]) * lr;
  } else if (ys > 1e-10f) {
    accepted = 1;
    int count = hdr->count, evicted = -1;
    if (count == m) {
      evicted = hdr->order[0];
      for (int i = 1; i < count; ++i) hdr->order[i - 1] = hdr->order[i];
      --count;
    }
    const int slot = hdr->cand;
    hdr->order[count++] = slot;
    hdr->count = count;
    hdr->cand = evicted >= 0 ? evicted : count;
    hdr->H_diag = ys / yy;
    reinterpret_cast<double*>(st + L.sy)[(size_t)slot * L.m1 + slot] = (double)ys;
  }
  hdr->accepted = accepted;
  hdr->t = t;
  hdr->ys = ys;
  hdr->yy = yy;
  scal[7] = ys;
  scal[8] = (float)hdr->count;
  scal[9] = (float)n_iter;
  scal[10] = hdr->H_diag;
}

// Lane exchanges without the LDS pipe (gfx950 v_permlane*_swap, DPP).  swap_sum<32>(a, c):
// a + (a of lane + 32) in lanes < 32, (c of lane - 32) + c in lanes >= 32 -- the swap
// trades the upper half of its first operand for the lower half of its second, and the
// two results always hold the lane's own value and its partner's, in either order.
// swap_sum<16>: the same between rows 0/1 and 2/3.
template <int H>
__device__ __forceinline__ float swap_sum(float a, float c) {
  const auto r = H == 32 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(c),
                                                            false, false)
                         : __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(c),
                                                            false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// the sum of a 16-lane row in every lane of it: quad swaps, then the half-row and row
// mirrors pair each lane with one of the other half (every lane adds the same two values)
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

// K3: u = S^T g, w = Y^T g and the new pair's column (s_k . y_new, y_k . y_new) in one
// read of the history.  The block's four waves walk the pairs in the same order,
// each thread one float4 of the block's chunk (the combine pass's access pattern: every
// pair's chunk read as one contiguous 4 KB per vector), four pairs' loads in flight; a
// pair's four sums are packed into one wave reduction (the 32- and 16-lane swaps trade
// halves of the quantities, then one 16-lane DPP tree: 7 register-only exchanges instead
// of 24 LDS-pipe permutes) and kept in
// LDS, and after the last pair the block adds its waves' values in wave order (per-block
// partials for lb_dots_fin_kernel).  Round 4: a wave per pair subset with 16 values per
// lane and one 64-lane tree per quantity took 125.9 us at history 100, this form 118.5
__global__ void __launch_bounds__(LB_NT)
lb_dots_kernel(const float* __restrict__ g, const float* __restrict__ hist, long long n,
               long long np, int m1, const LbHdr* __restrict__ hdr, float* __restrict__ parts) {
  const int count = hdr->count;
  if (count == 0) return;
  __shared__ float wp[LB_NT / 64][LB_MAXM + 1][4];
  const int nb = (int)gridDim.x;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long e = (long long)blockIdx.x * LB_CHUNK + 4 * threadIdx.x;
  const f32x4 gv = ld4g(g, e, n);
  const f32x4 yn = hdr->accepted
                       ? *reinterpret_cast<const f32x4*>(hist + (size_t)(m1 + hdr->order[count - 1]) * np + e)
                       : f32x4{0.f, 0.f, 0.f, 0.f};
  auto dot4 = [](f32x4 a, f32x4 b) {
    return fmaf(a[3], b[3], fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])));
  };
  constexpr int PF = 4;
  f32x4 sv[PF], yv[PF];
  auto load_pair = [&](int kk, f32x4& a, f32x4& b) {  // (clamped: unconditional loads)
    const int sl = hdr->order[min(kk, count - 1)];
    a = *reinterpret_cast<const f32x4*>(hist + (size_t)sl * np + e);
    b = *reinterpret_cast<const f32x4*>(hist + (size_t)(m1 + sl) * np + e);
  };
#pragma unroll
  for (int i = 0; i < PF; ++i) load_pair(i, sv[i], yv[i]);
  for (int k0 = 0; k0 < count; k0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int k = k0 + i;
      if (k < count) {
        const float d0 = dot4(sv[i], gv), d1 = dot4(yv[i], gv);
        const float d2 = dot4(sv[i], yn), d3 = dot4(yv[i], yn);
        load_pair(k + PF, sv[i], yv[i]);
        // lanes < 32 end with quantities 0, 1, lanes >= 32 with 2, 3; then rows 0..3 with
        // quantity 0..3; then the 16-lane tree
        const float v0 = swap_sum<32>(d0, d2), v1 = swap_sum<32>(d1, d3);
        const float v = row_sum16(swap_sum<16>(v0, v1));
        if ((lane & 15) == 0) wp[w][k][lane >> 4] = v;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * count; i += LB_NT) {
    const int k = i >> 2, q = i & 3;
    float t = wp[0][k][q];
#pragma unroll
    for (int ww = 1; ww < LB_NT / 64; ++ww) t += wp[ww][k][q];
    parts[((size_t)k * 4 + q) * nb + blockIdx.x] = t;
  }
}

// K3b: the dot partials summed in a fixed order (fp64), one block per (pair, quantity)
__global__ void __launch_bounds__(LB_NT)
lb_dots_fin_kernel(const float* __restrict__ parts, int nb, const LbHdr* __restrict__ hdr,
                   char* __restrict__ st, int m) {
  const int b = blockIdx.x;
  if (b >= 4 * hdr->count) return;
  const LbLayout L(m);
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += LB_NT) acc += (double)parts[(size_t)b * nb + i];
  __shared__ double red[LB_NT];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = LB_NT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) reinterpret_cast<double*>(st + L.dots)[b] = red[0];
}

// K4 (one block, fp64): the new column of Y^T Y and of R^-1, then
//   r = R^-1 u,  z = (D + g Y^T Y) r - g w,  a = R^-T z,  coefficients  s_k: -a_k,  y_k: g r_k
// R^-1 is kept current instead of solving with R: dropping the oldest pair drops the
// first row and column of both R and R^-1 (the inverse of an upper-triangular matrix's
// trailing block is the trailing block of its inverse), and appending pair n (column
// c_i = s_i.y_n, diagonal d = s_n.y_n) appends the column -R^-1 c / d and 1 / d.  Every
// phase is a matrix-vector product: 8 neighbouring lanes per row (rows 128 apart per
// pass), each lane a strided set of columns (independent loads), a fixed-order sum over
// the 8 lanes.
constexpr int LB_SOLVE_NT = 1024;
constexpr int LB_RG = 8;  // lanes per row

__device__ __forceinline__ double group_sum8(double v) {
#pragma unroll
  for (int o = 1; o < LB_RG; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(LB_SOLVE_NT)
lb_solve_kernel(LbHdr* __restrict__ hdr, char* __restrict__ st, int m) {
  const LbLayout L(m);
  const int k = hdr->count;
  double* SY = reinterpret_cast<double*>(st + L.sy);
  double* YY = reinterpret_cast<double*>(st + L.yy);
  double* RI = reinterpret_cast<double*>(st + L.ri);
  const double* dots = reinterpret_cast<const double*>(st + L.dots);
  float* coef = reinterpret_cast<float*>(st + L.coef);
  const int m1 = L.m1, sub = threadIdx.x % LB_RG, row0 = threadIdx.x / LB_RG;
  constexpr int RPP = LB_SOLVE_NT / LB_RG;  // rows per pass
  __shared__ int slot[LB_MAXM + 1];
  __shared__ double vu[LB_MAXM + 1], vc[LB_MAXM + 1], vr[LB_MAXM + 1], vz[LB_MAXM + 1];
  for (int i = threadIdx.x; i < k; i += LB_SOLVE_NT) {
    slot[i] = hdr->order[i];
    vu[i] = dots[4 * i];
    vc[i] = dots[4 * i + 2];
  }
  __syncthreads();
  if (hdr->accepted && k > 0) {
    const int nw = slot[k - 1];
    // d = s_n.y_n from the fp64 dots (vc[k-1], shared memory): the loop below overwrites
    // SY's diagonal entry with the same value, so no lane may read SY[nw][nw] here
    const double dinv = 1.0 / vc[k - 1];
    for (int i = threadIdx.x; i < k; i += LB_SOLVE_NT) {
      const int si = slot[i];
      SY[(size_t)si * m1 + nw] = vc[i];
      YY[(size_t)si * m1 + nw] = dots[4 * i + 3];
      YY[(size_t)nw * m1 + si] = dots[4 * i + 3];
    }
    // column k-1 of R^-1: rows i < k-1 from the old R^-1 (columns i .. k-2)
    for (int i = row0; i < k - 1; i += RPP) {
      const double* row = RI + (size_t)slot[i] * m1;
      double acc = 0.0;
      for (int j = i + sub; j < k - 1; j += LB_RG) acc = fma(row[slot[j]], vc[j], acc);
      acc = group_sum8(acc);
      if (sub == 0) RI[(size_t)slot[i] * m1 + nw] = -acc * dinv;
    }
    if (threadIdx.x == 0) RI[(size_t)nw * m1 + nw] = dinv;
  }
  __syncthreads();
  const double gam = (double)hdr->H_diag;
  // r = R^-1 u
  for (int i = row0; i < k; i += RPP) {
    const double* row = RI + (size_t)slot[i] * m1;
    double acc = 0.0;
    for (int j = i + sub; j < k; j += LB_RG) acc = fma(row[slot[j]], vu[j], acc);
    acc = group_sum8(acc);
    if (sub == 0) vr[i] = acc;
  }
  __syncthreads();
  // z = (D + g Y^T Y) r - g w
  for (int i = row0; i < k; i += RPP) {
    const int si = slot[i];
    const double* row = YY + (size_t)si * m1;
    double acc = 0.0;
    for (int j = sub; j < k; j += LB_RG) acc = fma(row[slot[j]], vr[j], acc);
    acc = group_sum8(acc);
    if (sub == 0) vz[i] = SY[(size_t)si * m1 + si] * vr[i] - gam * dots[4 * i + 1] + gam * acc;
  }
  __syncthreads();
  // a = R^-T z
  for (int i = row0; i < k; i += RPP) {
    const int si = slot[i];
    double acc = 0.0;
    for (int j = sub; j <= i; j += LB_RG) acc = fma(RI[(size_t)slot[j] * m1 + si], vz[j], acc);
    acc = group_sum8(acc);
    if (sub == 0) {
      coef[i] = (float)(-acc);
      coef[m1 + i] = (float)(gam * vr[i]);
    }
  }
}

// K5: d = -H_diag g + sum_k (cs_k s_k + cy_k y_k); s_next = t d into the free slot;
// partials of g.d and max|t d|
__global__ void __launch_bounds__(LB_NT)
lb_combine_kernel(const float* __restrict__ g, float* __restrict__ hist, long long n, long long np,
                  const LbHdr* __restrict__ hdr, const char* __restrict__ st, int m,
                  float* __restrict__ parts) {
  const LbLayout L(m);
  __shared__ float cs[LB_MAXM + 1], cy[LB_MAXM + 1];
  __shared__ int slot[LB_MAXM + 1];
  __shared__ float red[8];
  const int k = hdr->count, m1 = L.m1;
  const float* coef = reinterpret_cast<const float*>(st + L.coef);
  for (int i = threadIdx.x; i < k; i += LB_NT) {
    cs[i] = coef[i];
    cy[i] = coef[m1 + i];
    slot[i] = hdr->order[i];
  }
  __syncthreads();
  const float gam = hdr->H_diag, t = hdr->t;
  const long long e = (long long)blockIdx.x * LB_CHUNK + 4 * threadIdx.x;
  const f32x4 gv = ld4g(g, e, n);
  f32x4 d = -gam * gv;
  int j = 0;
  for (; j + 1 < k; j += 2) {
    const int s0 = slot[j], s1 = slot[j + 1];
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(hist + (size_t)s0 * np + e);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(hist + (size_t)(m1 + s0) * np + e);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(hist + (size_t)s1 * np + e);
    const f32x4 b1 = *reinterpret_cast<const f32x4*>(hist + (size_t)(m1 + s1) * np + e);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[q] = fmaf(cs[j], a0[q], d[q]);
      d[q] = fmaf(cy[j], b0[q], d[q]);
      d[q] = fmaf(cs[j + 1], a1[q], d[q]);
      d[q] = fmaf(cy[j + 1], b1[q], d[q]);
    }
  }
  if (j < k) {
    const int s0 = slot[j];
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(hist + (size_t)s0 * np + e);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(hist + (size_t)(m1 + s0) * np + e);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      d[q] = fmaf(cs[j], a0[q], d[q]);
      d[q] = fmaf(cy[j], b0[q], d[q]);
    }
  }
  const f32x4 sn = t * d;
  *reinterpret_cast<f32x4*>(hist + (size_t)hdr->cand * np + e) = sn;
  float gd = 0.f, dm = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    gd = fmaf(gv[q], d[q], gd);
    dm = nanmax(dm, fabsf(sn[q]));
  }
  block_red2<true>(gd, dm, red);
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = gd;
    parts[2 * blockIdx.x + 1] = dm;
  }
}

// K6: g.d and max|t d| (every block sums the combine's partials in the same fixed order,
// so all blocks agree bit for bit); flag = (g.d > -tolerance_change): torch breaks before
// moving x; otherwise x += t d (= s_next).  Block 0 publishes the scalars.
__global__ void __launch_bounds__(LB_NT)
lb_finish_step_kernel(LbHdr* __restrict__ hdr, float* __restrict__ scal,
                      const float* __restrict__ parts, int nb, float tol_change,
                      float* __restrict__ x, const float* __restrict__ hist, long long n,
                      long long np) {
  __shared__ float red[8];
  float gd = 0.f, dm = 0.f;
  for (int i = threadIdx.x; i < nb; i += LB_NT) {  // fixed order per thread
    gd += parts[2 * i];
    dm = nanmax(dm, parts[2 * i + 1]);
  }
  block_red2<true>(gd, dm, red);
  const int flag = gd > -tol_change;
  const int cand = hdr->cand;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    hdr->flag = flag;
    hdr->gtd = gd;
    hdr->dmax = dm;
    scal[3] = gd;
    scal[4] = hdr->t;
    scal[5] = dm;
    scal[6] = (float)flag;
  }
  if (flag) return;
  const float* __restrict__ s = hist + (size_t)cand * np;
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)LB_NT + threadIdx.x; i < n4;
       i += (long long)gridDim.x * LB_NT)
    reinterpret_cast<f32x4*>(x)[i] += reinterpret_cast<const f32x4*>(s)[i];
  for (long long i = 4 * n4 + blockIdx.x * (long long)LB_NT + threadIdx.x; i < n;
       i += (long long)gridDim.x * LB_NT)
    x[i] += s[i];
}

// K7/K8: max|g| (NaN propagates, as torch's max) and sum|g| of a fresh gradient; the loss
// copied next to them (one host read); optionally zero `clear` (the Gatys engine's amax
// groups, next written by the following forward)
__global__ void __launch_bounds__(LB_NT)
lb_gstats_kernel(const float* __restrict__ g, long long n, float* __restrict__ parts) {
  __shared__ float red[8];
  float sm = 0.f, mx = 0.f;
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)LB_NT + threadIdx.x; i < n4;
       i += (long long)gridDim.x * LB_NT) {
    const f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sm += fabsf(v[q]);
      mx = nanmax(mx, fabsf(v[q]));
    }
  }
  for (long long i = 4 * n4 + blockIdx.x * (long long)LB_NT + threadIdx.x; i < n;
       i += (long long)gridDim.x * LB_NT) {
    sm += fabsf(g[i]);
    mx = nanmax(mx, fabsf(g[i]));
  }
  block_red2<true>(sm, mx, red);
  if (threadIdx.x == 0) {
    parts[2 * blockIdx.x] = sm;
    parts[2 * blockIdx.x + 1] = mx;
  }
}

__global__ void __launch_bounds__(LB_NT)
lb_gstats_fin_kernel(const float* __restrict__ parts, const float* __restrict__ loss,
                     float* __restrict__ scal, float* __restrict__ clear, int clear_n) {
  __shared__ float red[8];
  float sm = parts[2 * threadIdx.x] + parts[2 * (threadIdx.x + LB_NT)];
  float mx = nanmax(parts[2 * threadIdx.x + 1], parts[2 * (threadIdx.x + LB_NT) + 1]);
  block_red2<true>(sm, mx, red);
  if (threadIdx.x == 0) {
    if (loss) scal[0] = *loss;
    scal[1] = mx;
    scal[2] = sm;
  }
  for (int i = threadIdx.x; i < clear_n; i += LB_NT) clear[i] = 0.f;
}

struct LbWs {
  size_t p1, p3, p5, p8, total;
  LbWs(long long n, int m) {
    const long long nb = lb_npad(n) / LB_CHUNK;
    size_t o = 0;
    p1 = o;
    o += sizeof(float) * 2 * LB_G;
    p3 = o;
    o += sizeof(float) * 4 * (size_t)(m + 1) * nb;
    p5 = o;
    o += sizeof(float) * 2 * nb;
    p8 = o;
    o += sizeof(float) * 2 * LB_G;
    total = o;
  }
};

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace
}  // namespace stx

using namespace stx;

extern "C" size_t stx_lbfgs_state_bytes(int m) {
  return (m < 1 || m > LB_MAXM) ? 0 : LbLayout(m).total;
}

extern "C" size_t stx_lbfgs_hist_bytes(long long n, int m) {
  return (m < 1 || m > LB_MAXM || n <= 0) ? 0 : sizeof(float) * 2 * (size_t)(m + 1) * lb_npad(n);
}

extern "C" size_t stx_lbfgs_ws(long long n, int m) {
  return (m < 1 || m > LB_MAXM || n <= 0) ? 0 : LbWs(n, m).total;
}

extern "C" int stx_lbfgs_direction(float* x, const float* g, float* prev_g, float* hist, long long n,
                                   int m, float lr, float tol_change, void* state, float* scal,
                                   void* ws, size_t ws_bytes, void* stream) {
  if (!x || !g || !prev_g || !hist || !state || !scal || n <= 0 || m < 1 || m > LB_MAXM ||
      !aligned16(x) || !aligned16(g) || !aligned16(prev_g) || !aligned16(hist)) {
    set_error("stx_lbfgs_direction: invalid arguments (16-byte aligned vectors, 1 <= m <= %d)",
              LB_MAXM);
    return STX_E_INVALID;
  }
  const LbWs W(n, m);
  if (!ws || ws_bytes < W.total) {
    set_error("stx_lbfgs_direction: workspace");
    return STX_E_WORKSPACE;
  }
  const long long np = lb_npad(n);
  const int nb = (int)(np / LB_CHUNK);
  if ((long long)4 * (m + 1) * nb >= (1ll << 31)) {
    set_error("stx_lbfgs_direction: vector too long");
    return STX_E_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  char* w = static_cast<char*>(ws);
  LbHdr* hdr = static_cast<LbHdr*>(state);
  char* sb = static_cast<char*>(state);
  float* p1 = reinterpret_cast<float*>(w + W.p1);
  float* p3 = reinterpret_cast<float*>(w + W.p3);
  float* p5 = reinterpret_cast<float*>(w + W.p5);
  hipLaunchKernelGGL(lb_pair_kernel, dim3(LB_G), dim3(LB_NT), 0, st, g, prev_g, hist, n, np, m + 1,
                     hdr, p1);
  hipLaunchKernelGGL(lb_commit_kernel, dim3(1), dim3(LB_NT), 0, st, hdr, sb, scal, p1, m, lr);
  hipLaunchKernelGGL(lb_dots_kernel, dim3(nb), dim3(LB_NT), 0, st, g, hist, n, np, m + 1, hdr, p3);
  hipLaunchKernelGGL(lb_dots_fin_kernel, dim3(4 * (m + 1)), dim3(LB_NT), 0, st, p3, nb, hdr, sb, m);
  hipLaunchKernelGGL(lb_solve_kernel, dim3(1), dim3(LB_SOLVE_NT), 0, st, hdr, sb, m);
  hipLaunchKernelGGL(lb_combine_kernel, dim3(nb), dim3(LB_NT), 0, st, g, hist, n, np, hdr, sb, m,
                     p5);
  hipLaunchKernelGGL(lb_finish_step_kernel, dim3(LB_G), dim3(LB_NT), 0, st, hdr, scal, p5, nb,
                     tol_change, x, hist, n, np);
  return check_launch("stx_lbfgs_direction");
}

extern "C" int stx_lbfgs_grad_stats(const float* g, long long n, const float* loss, float* scal,
                                    float* clear, int clear_n, void* ws, size_t ws_bytes,
                                    void* stream) {
  if (!g || !scal || n <= 0 || !aligned16(g) || clear_n < 0 || (clear_n > 0 && !clear)) {
    set_error("stx_lbfgs_grad_stats: invalid arguments");
    return STX_E_INVALID;
  }
  if (!ws || ws_bytes < sizeof(float) * 2 * LB_G) {
    set_error("stx_lbfgs_grad_stats: workspace");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* p = static_cast<float*>(ws);
  hipLaunchKernelGGL(lb_gstats_kernel, dim3(LB_G), dim3(LB_NT), 0, st, g, n, p);
  hipLaunchKernelGGL(lb_gstats_fin_kernel, dim3(1), dim3(LB_NT), 0, st, p, loss, scal, clear,
                     clear_n);
  return check_launch("stx_lbfgs_grad_stats");
}
