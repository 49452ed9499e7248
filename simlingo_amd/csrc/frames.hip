// Collate image path on the GPU: uint8 camera frames -> InternVL2 pixel tiles.
//
// Replaces, per frame, the CPU worker chain of the reference collate
//   bottom crop            dataset_base.py:464-467   rows [0, H - (H*4.8)//16)
//   dynamic_preprocess     internvl2_utils.py:231-266 aspect-ratio grid (host) + PIL Image.resize((tw, th))
//                          (Pillow's default filter for RGB = BICUBIC) + crop into 448x448 tiles
//   build_transform        internvl2_utils.py:206-214 Resize(448) (identity on a 448 tile), ToTensor, Normalize
// with ONE kernel per batch. The resize reproduces Pillow's ImagingResample (Resample.c, pinned pillow 10.2.0,
// environment.yaml:187) bit for bit: separable two-pass convolution, horizontal pass first over exactly the rows
// the vertical pass needs, each pass rounding to uint8 through 22-bit fixed-point coefficients (clip8). The
// coefficients are built on the host (slx_resample_coeffs: Pillow's precompute_coeffs in double + the 8-bpc
// normalisation), once per geometry. ToTensor / Normalize are the same f32 operations torchvision performs
// (u / 255, then (x - mean) / std, IEEE division), so the tiles are bit-identical to the reference's.
//
// Work split: one 256-thread block per (strip of RY output rows, frame). The block first runs the horizontal
// pass for the source rows its strip needs into LDS (uint8, [rows][tw*3]), then the vertical pass, the
// normalisation and the scatter into the tile layout [B][blocks][3][448][448] with x fastest (coalesced f32
// stores). Byte work, HBM-bound: 1 read of the cropped frame + 1 f32 write of the tiles.
#include <cmath>

#include "common.h"
#include "../../include/slx.h"

namespace slx {

static constexpr int kPrecisionBits = 32 - 8 - 2;  // Resample.c PRECISION_BITS

__device__ __forceinline__ int clip8(int in) {
  if (in >= (1 << kPrecisionBits << 8)) return 255;
  if (in <= 0) return 0;
  return in >> kPrecisionBits;
}

struct FrameArgs {
  const uint8_t* src;
  long sb, sy, sx, sc;
  int H, W, tw, th, tile, tiles_x, blocks, RY, lds_rows;
  const int* hb;
  const int* hk;
  int hks;
  const int* vb;
  const int* vk;
  int vks;
  int need_h, need_v;
  float mean[3], stdv[3];
  float* out;
};

__global__ __launch_bounds__(256) void frames_to_tiles_kernel(FrameArgs a) {
  extern __shared__ uint8_t rowbuf[];  // [lds_rows][tw*3]
  const int b = blockIdx.y;
  const int y0 = blockIdx.x * a.RY;
  const int y1 = min(y0 + a.RY, a.th);
  const int tid = threadIdx.x;
  // source rows this strip reads (vertical bounds are monotone in y)
  int ylo, yhi;
  if (a.need_v) {
    ylo = a.vb[2 * y0];
    yhi = 0;
    for (int y = y0; y < y1; ++y) yhi = max(yhi, a.vb[2 * y] + a.vb[2 * y + 1]);
  } else {
    ylo = y0;
    yhi = y1;
  }
  const int nrows = yhi - ylo;  // <= lds_rows (host-checked for every strip)
  const int row3 = a.tw * 3;
  const uint8_t* fb = a.src + (long)b * a.sb;
  // ---- horizontal pass (or plain copy when the width is unchanged) -> LDS ----
  for (int i = tid; i < nrows * a.tw; i += 256) {
    const int r = i / a.tw, xx = i - r * a.tw;
    const uint8_t* srow = fb + (long)(ylo + r) * a.sy;
    int s0, s1, s2;
    if (a.need_h) {
      const int xmin = a.hb[2 * xx], xl = a.hb[2 * xx + 1];
      const int* k = a.hk + (long)xx * a.hks;
      s0 = s1 = s2 = 1 << (kPrecisionBits - 1);
      for (int x = 0; x < xl; ++x) {
        const uint8_t* p = srow + (long)(xmin + x) * a.sx;
        const int kx = k[x];
        s0 += (int)p[0] * kx;
        s1 += (int)p[a.sc] * kx;
        s2 += (int)p[2 * a.sc] * kx;
      }
      s0 = clip8(s0);
      s1 = clip8(s1);
      s2 = clip8(s2);
    } else {
      const uint8_t* p = srow + (long)xx * a.sx;
      s0 = p[0];
      s1 = p[a.sc];
      s2 = p[2 * a.sc];
    }
    uint8_t* d = rowbuf + r * row3 + xx * 3;
    d[0] = (uint8_t)s0;
    d[1] = (uint8_t)s1;
    d[2] = (uint8_t)s2;
  }
  __syncthreads();
  // ---- vertical pass + ToTensor + Normalize + tile scatter ----
  const int n = (y1 - y0) * 3 * a.tw;
  const long plane = (long)a.tile * a.tile;
  for (int i = tid; i < n; i += 256) {
    const int xx = i % a.tw;
    const int t = i / a.tw;
    const int c = t % 3, y = y0 + t / 3;
    int u;
    if (a.need_v) {
      const int ymin = a.vb[2 * y], yl = a.vb[2 * y + 1];
      const int* k = a.vk + (long)y * a.vks;
      int s = 1 << (kPrecisionBits - 1);
      const uint8_t* col = rowbuf + (ymin - ylo) * row3 + xx * 3 + c;
      for (int j = 0; j < yl; ++j) s += (int)col[j * row3] * k[j];
      u = clip8(s);
    } else {
      u = rowbuf[(y - ylo) * row3 + xx * 3 + c];
    }
    const float v = ((float)u / 255.0f - a.mean[c]) / a.stdv[c];
    const int tx = xx / a.tile, ty = y / a.tile;
    const long tileix = (long)b * a.blocks + ty * a.tiles_x + tx;
    a.out[(tileix * 3 + c) * plane + (long)(y - ty * a.tile) * a.tile + (xx - tx * a.tile)] = v;
  }
}

// Pillow bicubic kernel, a = -0.5 (Resample.c bicubic_filter), support 2
static double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

}  // namespace slx

using namespace slx;

extern "C" {

int slx_resample_ksize(int in_size, int out_size) {
  if (in_size <= 0 || out_size <= 0) return -22;
  double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  return (int)std::ceil(support) * 2 + 1;
}

// Pillow precompute_coeffs (box = [0, in_size), BICUBIC) + normalize_coeffs_8bpc. Evaluated in double with
// contraction off, like Pillow's C build, so every weight rounds to the same 22-bit integer.
#pragma clang fp contract(off)
int slx_resample_coeffs(int in_size, int out_size, int kmax, int32_t* bounds, int32_t* kk) {
  SLX_CHECK_ARG(in_size > 0 && out_size > 0, "slx_resample_coeffs: sizes must be positive (%d, %d)", in_size,
                out_size);
  const int ksize = slx_resample_ksize(in_size, out_size);
  SLX_CHECK_ARG(kmax >= ksize, "slx_resample_coeffs: kmax %d < ksize %d", kmax, ksize);
  SLX_CHECK_ARG(bounds != nullptr && kk != nullptr, "slx_resample_coeffs: null output");
  const double in0 = 0.0, in1 = (double)in_size;
  const double scale = (in1 - in0) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  double k[64];
  SLX_CHECK_ARG(ksize <= 64, "slx_resample_coeffs: downscale factor too large (ksize %d)", ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    int x = 0;
    for (; x < xmax; ++x) {
      const double w = bicubic_filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    for (; x < ksize; ++x) k[x] = 0;
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
    for (x = 0; x < kmax; ++x) {
      const double v = x < ksize ? k[x] : 0.0;
      kk[(long)xx * kmax + x] = v < 0 ? (int32_t)(-0.5 + v * (1 << kPrecisionBits))
                                      : (int32_t)(0.5 + v * (1 << kPrecisionBits));
    }
  }
  return ksize;
}

int slx_frames_to_tiles(const slx_frame_desc* d, slx_stream_t stream) {
  SLX_CHECK_ARG(d != nullptr && d->src != nullptr && d->out != nullptr, "slx_frames_to_tiles: null pointer");
  SLX_CHECK_ARG(d->B >= 0 && d->H > 0 && d->W > 0 && d->tw > 0 && d->th > 0 && d->tile > 0,
                "slx_frames_to_tiles: bad sizes");
  SLX_CHECK_ARG(d->tw % d->tile == 0 && d->th % d->tile == 0, "slx_frames_to_tiles: %dx%d is not a grid of %d tiles",
                d->tw, d->th, d->tile);
  SLX_CHECK_ARG(d->need_h || d->tw == d->W, "slx_frames_to_tiles: width changes but need_h = 0");
  SLX_CHECK_ARG(d->need_v || d->th == d->H, "slx_frames_to_tiles: height changes but need_v = 0");
  SLX_CHECK_ARG(!d->need_h || (d->hbounds && d->hcoeffs && d->hksize > 0), "slx_frames_to_tiles: missing horizontal coeffs");
  SLX_CHECK_ARG(!d->need_v || (d->vbounds && d->vcoeffs && d->vksize > 0), "slx_frames_to_tiles: missing vertical coeffs");
  SLX_CHECK_ARG(d->rows_per_block > 0 && d->lds_rows > 0, "slx_frames_to_tiles: rows_per_block / lds_rows unset");
  const size_t lds = (size_t)d->lds_rows * d->tw * 3;
  SLX_CHECK_ARG(lds <= 64 * 1024, "slx_frames_to_tiles: strip needs %zu B of LDS (> 64 KiB): fewer rows_per_block",
                lds);
  if (d->B == 0) return 0;
  FrameArgs a;
  a.src = d->src;
  a.sb = d->sb; a.sy = d->sy; a.sx = d->sx; a.sc = d->sc;
  a.H = d->H; a.W = d->W; a.tw = d->tw; a.th = d->th; a.tile = d->tile;
  a.tiles_x = d->tw / d->tile;
  a.blocks = a.tiles_x * (d->th / d->tile);
  a.RY = d->rows_per_block; a.lds_rows = d->lds_rows;
  a.hb = d->hbounds; a.hk = d->hcoeffs; a.hks = d->hksize;
  a.vb = d->vbounds; a.vk = d->vcoeffs; a.vks = d->vksize;
  a.need_h = d->need_h; a.need_v = d->need_v;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = d->mean[c];
    a.stdv[c] = d->std[c];
  }
  a.out = d->out;
  const dim3 grid((unsigned)((d->th + a.RY - 1) / a.RY), (unsigned)d->B);
  hipLaunchKernelGGL(frames_to_tiles_kernel, grid, dim3(256), lds, (hipStream_t)stream, a);
  SLX_LAUNCH_CHECK("slx_frames_to_tiles");
  return 0;
}

}  // extern "C"
