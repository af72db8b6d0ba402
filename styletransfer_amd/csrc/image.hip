// Image conditioning on the GPU: the reference's image_loader_transform
// (stransfer/img_utils.py:13-44 -- CenterCrop(min side) -> Resize(IMSIZE) ->
// ToTensor -> ImageNet normalisation, stransfer/constants.py:16-17) for a batch of
// decoded 8-bit RGB images of any sizes, so the COCO loader's host workers only
// decode JPEGs (stransfer/dataset.py:141-197).
//
// The resize is the pinned image library's own arithmetic (Pillow's 8-bit
// convolution resampler, BILINEAR): separable, horizontal pass first over the rows
// the vertical pass needs, int32 coefficients with 22 fractional bits, each pass
// acc = 2^21 + sum(u8 * coeff), out = clip(acc >> 22, 0, 255) kept as 8 bits --
// integer arithmetic, so the output bytes equal PIL's exactly.  Coefficient tables
// are built on the host (stx_resample_coeffs, double precision in Pillow's operation
// order) and uploaded with the batch.  Then u8 / 255 and (x - mean) / std in fp32,
// the order torch's ToTensor + Normalize use (IEEE division, no reciprocal).
//
// Two launches per batch: (1) horizontal pass, one thread per (image, input row,
// output column) writing 3 bytes to a workspace image [m_rows][size][3]; (2)
// vertical pass + normalisation, one thread per (image, output row, output column)
// writing the three planes of the [B][3][size][size] fp32 output (coalesced along x).
#include <math.h>

#include <vector>

#include "common.h"
#include "../../include/stx.h"

namespace stx {

constexpr int RS_PREC = 22;  // 32 - 8 - 2: Pillow's PRECISION_BITS for 8-bit images

__device__ __forceinline__ uint8_t clip8(int acc) {
  const int v = acc >> RS_PREC;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// horizontal pass: tmp[b][y - y0][xo][c] for crop rows y0 <= y < y1
__global__ void __launch_bounds__(256)
resample_h_kernel(const uint8_t* __restrict__ src, const stx_image_meta* __restrict__ meta,
                  const int* __restrict__ coef, int size, uint8_t* __restrict__ tmp) {
  const stx_image_meta m = meta[blockIdx.y];
  if (!m.resize_w) return;  // no horizontal pass (and no tmp rows) for this image
  const int nrows = m.y1 - m.y0;
  const long long total = (long long)nrows * size;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int yr = (int)(i / size), xo = (int)(i - (long long)yr * size);
  const int* __restrict__ xb = coef + m.xcoef;           // [size][2] bounds
  const int* __restrict__ xk = xb + 2 * size;            // [size][xk]
  const int xmin = xb[2 * xo], n = xb[2 * xo + 1];
  const uint8_t* __restrict__ row =
      src + m.offset + ((size_t)(m.top + m.y0 + yr) * m.w + m.left + xmin) * 3;
  int a0 = 1 << (RS_PREC - 1), a1 = a0, a2 = a0;
  for (int k = 0; k < n; ++k) {
    const int c = xk[xo * m.xk + k];
    a0 += (int)row[3 * k] * c;
    a1 += (int)row[3 * k + 1] * c;
    a2 += (int)row[3 * k + 2] * c;
  }
  uint8_t* o = tmp + m.tmp_offset + ((size_t)yr * size + xo) * 3;
  o[0] = clip8(a0);
  o[1] = clip8(a1);
  o[2] = clip8(a2);
}

// vertical pass (or a copy when the height does not change) + ToTensor + Normalize
__global__ void __launch_bounds__(256)
resample_v_kernel(const uint8_t* __restrict__ src, const stx_image_meta* __restrict__ meta,
                  const int* __restrict__ coef, int size, const uint8_t* __restrict__ tmp,
                  float m0, float m1, float m2, float s0, float s1, float s2,
                  float* __restrict__ out) {
  const int b = blockIdx.y;
  const stx_image_meta m = meta[b];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= size * size) return;
  const int yo = i / size, xo = i - yo * size;
  int v0, v1, v2;
  if (m.resize_h) {
    const int* __restrict__ yb = coef + m.ycoef;
    const int* __restrict__ yk = yb + 2 * size;
    const int ymin = yb[2 * yo] - m.y0, n = yb[2 * yo + 1];
    // rows come from the horizontal pass, or straight from the crop when only the
    // height changes
    int a0 = 1 << (RS_PREC - 1), a1 = a0, a2 = a0;
    for (int k = 0; k < n; ++k) {
      const int c = yk[yo * m.yk + k];
      const uint8_t* px = m.resize_w
          ? tmp + m.tmp_offset + ((size_t)(ymin + k) * size + xo) * 3
          : src + m.offset + ((size_t)(m.top + m.y0 + ymin + k) * m.w + m.left + xo) * 3;
      a0 += (int)px[0] * c;
      a1 += (int)px[1] * c;
      a2 += (int)px[2] * c;
    }
    v0 = clip8(a0);
    v1 = clip8(a1);
    v2 = clip8(a2);
  } else {
    const uint8_t* px = m.resize_w ? tmp + m.tmp_offset + ((size_t)yo * size + xo) * 3
                                   : src + m.offset + ((size_t)(m.top + yo) * m.w + m.left + xo) * 3;
    v0 = px[0];
    v1 = px[1];
    v2 = px[2];
  }
  const size_t plane = (size_t)size * size;
  float* o = out + (size_t)b * 3 * plane + (size_t)yo * size + xo;
  o[0] = ((float)v0 / 255.f - m0) / s0;
  o[plane] = ((float)v1 / 255.f - m1) / s1;
  o[2 * plane] = ((float)v2 / 255.f - m2) / s2;
}

}  // namespace stx

using namespace stx;

// Pillow's precompute_coeffs + normalize_coeffs_8bpc for one axis (BILINEAR).
extern "C" int stx_resample_coeffs(int in_size, int out_size, int* bounds, int* kk,
                                   int kk_stride) {
  if (in_size <= 0 || out_size <= 0) return -1;
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)ceil(support) * 2 + 1;
  if (!bounds || !kk) return ksize;  // size query
  if (kk_stride < ksize) return -1;
  const double ss = 1.0 / filterscale;
  std::vector<double> w(ksize);  // any down-scale factor (a crop of ~8000 px at 256 needs > 64)
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    double ww = 0.0;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0) t = -t;
      const double v = t < 1.0 ? 1.0 - t : 0.0;
      w[x] = v;
      ww += v;
    }
    for (int x = 0; x < ksize; ++x) {
      double k = x < xmax ? (ww != 0.0 ? w[x] / ww : w[x]) : 0.0;
      kk[(size_t)xx * kk_stride + x] =
          k < 0 ? (int)(-0.5 + k * (1 << RS_PREC)) : (int)(0.5 + k * (1 << RS_PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

extern "C" int stx_image_condition(const void* src, const stx_image_meta* meta, int b,
                                   int max_rows, const int* coef, int size, const float* mean,
                                   const float* std_, float* out, void* tmp, size_t tmp_bytes,
                                   void* stream) {
  if (!src || !meta || !coef || !out || !mean || !std_ || b <= 0 || size <= 0 || max_rows < 0) {
    set_error("stx_image_condition: invalid arguments");
    return STX_E_INVALID;
  }
  if (max_rows > 0 && !tmp) {
    set_error("stx_image_condition: workspace");
    return STX_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  if (max_rows > 0) {
    const long long work = (long long)max_rows * size;
    hipLaunchKernelGGL(resample_h_kernel, dim3((unsigned)((work + 255) / 256), b), dim3(256), 0, st,
                       (const uint8_t*)src, meta, coef, size, (uint8_t*)tmp);
  }
  hipLaunchKernelGGL(resample_v_kernel, dim3((size * size + 255) / 256, b), dim3(256), 0, st,
                     (const uint8_t*)src, meta, coef, size, (const uint8_t*)tmp, mean[0], mean[1],
                     mean[2], std_[0], std_[1], std_[2], out);
  return check_launch("stx_image_condition");
}
