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
// Work split: one 256-thread block per (RY output rows x CW output columns, frame): the source window it needs is
// staged into LDS (4-byte loads for packed HWC frames), the horizontal pass writes uint8 rows to LDS, the vertical
// pass + normalisation scatter f32 into the tile layout [B][tiles][3][448][448] with x fastest (coalesced
// stores). Byte work, HBM-bound: 1 read of the cropped frame + 1 f32 write of the tiles.
#include <cmath>

#include <vector>

#include "common.h"
#include "../../include/slx.h"

namespace slx {

static constexpr int kPrecisionBits = 32 - 8 - 2;  // Resample.c PRECISION_BITS
static constexpr int kCW = 128;                      // output columns per block (one per thread of a row group)

__device__ __forceinline__ int clip8(int in) {
  if (in >= (1 << kPrecisionBits << 8)) return 255;
  if (in <= 0) return 0;
  return in >> kPrecisionBits;
}

struct FrameArgs {
  const uint8_t* src;
  long sb, sy, sx, sc;
  int H, W, tw, th, tile, tiles_x, blocks, RY, CW, lds_rows, lds_cols;
  const int* hb;
  const int* hk;
  int hks;
  const int* vb;
  const int* vk;
  int vks;
  int need_h, need_v, packed;
  float mean[3], stdv[3];
  float* out;
};

// One 256-thread block per (RY output rows) x (CW output columns) x frame. LDS holds the source window the block
// needs ([lds_rows][lds_cols*3] bytes, staged with 4-byte loads when the frame is packed HWC) and the horizontal
// pass result ([lds_rows][CW*3] bytes); the vertical pass reads the latter and writes f32 tiles, x fastest.
template <int KH, int KV>  // tap-loop bounds (>= hks / vks): unrolled with a guard so the LDS reads batch
__global__ __launch_bounds__(256) void frames_to_tiles_kernel(FrameArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = blockIdx.z;
  const int y0 = blockIdx.y * a.RY, y1 = min(y0 + a.RY, a.th);
  const int x0 = blockIdx.x * a.CW, x1 = min(x0 + a.CW, a.tw);
  const int ncol = x1 - x0;
  const int tid = threadIdx.x;
  // source rows / columns this block reads: Pillow's first index and first+count are both non-decreasing in the
  // output index, so the window is [first of the first output, end of the last output)
  int ylo, yhi, xlo, xhi;
  if (a.need_v) {
    ylo = a.vb[2 * y0];
    yhi = a.vb[2 * (y1 - 1)] + a.vb[2 * (y1 - 1) + 1];  // window end = the last output's end (monotone)
  } else {
    ylo = y0;
    yhi = y1;
  }
  if (a.need_h) {
    xlo = a.hb[2 * x0];
    xhi = a.hb[2 * (x1 - 1)] + a.hb[2 * (x1 - 1) + 1];
  } else {
    xlo = x0;
    xhi = x1;
  }
  const int nrows = yhi - ylo, nsc = xhi - xlo;  // <= lds_rows, lds_cols: host-checked against Pillow's bounds
  if (nrows > a.lds_rows || nsc > a.lds_cols) {
    // caller-supplied bounds need a wider window than the LDS was sized for: never stage past the buffers; the
    // block's outputs become NaN so the failure is loud (slx_frames_to_tiles already rejects Pillow geometries
    // whose window exceeds lds_rows / lds_cols, so only inconsistent custom tables reach this)
    const int yl0 = y0, xl0 = x0;
    const long plane = (long)a.tile * a.tile;
    for (int i = tid; i < (y1 - y0) * ncol * 3; i += 256) {
      const int yy = yl0 + i / (ncol * 3), rem = i % (ncol * 3), xx = xl0 + rem / 3, c = rem % 3;
      const int tx = xx / a.tile, ty = yy / a.tile;
      a.out[((long)b * a.blocks + (long)ty * a.tiles_x + tx) * 3 * plane + (long)c * plane +
            (long)(yy - ty * a.tile) * a.tile + (xx - tx * a.tile)] = __builtin_nanf("");
    }
    return;
  }
  // LDS: coefficient rows of this block's outputs (int32), then the source window, then the horizontal result
  int* lhk = reinterpret_cast<int*>(smem);                  // [CW][hks]
  int* lhb = lhk + a.CW * a.hks;                            // [CW][2] (first index relative to xlo, count)
  int* lvk = lhb + 2 * a.CW;                                // [RY][vks]
  int* lvb = lvk + a.RY * a.vks;                            // [RY][2] (first index relative to ylo, count)
  uint8_t* sbuf = reinterpret_cast<uint8_t*>(lvb + 2 * a.RY);  // [lds_rows][lds_cols*3 + 4] source window
  const int sld = a.lds_cols * 3 + 4;
  uint8_t* hbuf = sbuf + a.lds_rows * sld;            // [lds_rows][CW*3] horizontal-pass result
  const int hld = a.CW * 3;
  const uint8_t* fb = a.src + (long)b * a.sb;
  if (a.need_h) {
    for (int i = tid; i < ncol * a.hks; i += 256) lhk[i] = a.hk[(long)x0 * a.hks + i];
    for (int i = tid; i < ncol; i += 256) {
      lhb[2 * i] = a.hb[2 * (x0 + i)] - xlo;
      lhb[2 * i + 1] = a.hb[2 * (x0 + i) + 1];
    }
  }
  if (a.need_v) {
    for (int i = tid; i < (y1 - y0) * a.vks; i += 256) lvk[i] = a.vk[(long)y0 * a.vks + i];
    for (int i = tid; i < y1 - y0; i += 256) {
      lvb[2 * i] = a.vb[2 * (y0 + i)] - ylo;
      lvb[2 * i + 1] = a.vb[2 * (y0 + i) + 1];
    }
  }
  // ---- stage the source window ----
  if (a.packed) {  // HWC bytes contiguous along x: dword loads from the 4-aligned start of each row segment
    const long bx0 = (long)xlo * 3;
    const int lead = (int)(bx0 & 3);  // rows and frames start 4-aligned (checked on the host)
    const int nw = (nsc * 3 + lead + 3) >> 2;
    const long rowend = (long)a.W * 3 - bx0 + lead;  // bytes of a row from the aligned start
    for (int i = tid; i < nrows * nw; i += 256) {
      const int r = i / nw, wi = i - r * nw;
      const uint8_t* rowp = fb + (long)(ylo + r) * a.sy + bx0 - lead;
      uint32_t w;
      if ((long)(wi + 1) * 4 <= rowend) {
        w = *reinterpret_cast<const uint32_t*>(rowp + wi * 4);
      } else {
        w = 0;
        for (int q = 0; q < 4; ++q)
          if ((long)wi * 4 + q < rowend) w |= (uint32_t)rowp[wi * 4 + q] << (8 * q);
      }
      uint8_t* d = sbuf + r * sld;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = wi * 4 + q - lead;
        if (o >= 0 && o < nsc * 3) d[o] = (uint8_t)(w >> (8 * q));
      }
    }
  } else {
    for (int i = tid; i < nrows * nsc * 3; i += 256) {
      const int r = i / (nsc * 3), j = i - r * (nsc * 3);
      const int x = j / 3, c = j - x * 3;
      sbuf[r * sld + j] = fb[(long)(ylo + r) * a.sy + (long)(xlo + x) * a.sx + (long)c * a.sc];
    }
  }
  __syncthreads();
  // Each thread owns one output column xl = tid % CW for both passes (CW = 128: two row groups of 128 threads, one
  // wave never straddles them), so its horizontal taps, tile column and store offset are computed once.
  const int xl = tid & (kCW - 1), rg = tid / kCW;
  const bool live = xl < ncol;
  const int xx = x0 + xl;
  // ---- horizontal pass (or copy when the width is unchanged) ----
  int hx0 = xx - xlo, hn = 0, hk[KH];
  if (a.need_h && live) {
    hx0 = lhb[2 * xl];
    hn = lhb[2 * xl + 1];
#pragma unroll
    for (int x = 0; x < KH; ++x) hk[x] = x < hn ? lhk[xl * a.hks + x] : 0;
  }
  if (live) {
    for (int r = rg; r < nrows; r += 256 / kCW) {
      const uint8_t* p = sbuf + r * sld + hx0 * 3;
      int s0, s1, s2;
      if (a.need_h) {
        s0 = s1 = s2 = 1 << (kPrecisionBits - 1);
#pragma unroll
        for (int x = 0; x < KH; ++x) {
          if (x < hn) {
            s0 += (int)p[3 * x] * hk[x];
            s1 += (int)p[3 * x + 1] * hk[x];
            s2 += (int)p[3 * x + 2] * hk[x];
          }
        }
        s0 = clip8(s0);
        s1 = clip8(s1);
        s2 = clip8(s2);
      } else {
        s0 = p[0];
        s1 = p[1];
        s2 = p[2];
      }
      uint8_t* d = hbuf + r * hld + xl * 3;
      d[0] = (uint8_t)s0;
      d[1] = (uint8_t)s1;
      d[2] = (uint8_t)s2;
    }
  }
  __syncthreads();
  if (!live) return;
  // ---- vertical pass + ToTensor + Normalize + tile scatter ----
  const long plane = (long)a.tile * a.tile;
  const int tx = xx / a.tile;
  const int xin = xx - tx * a.tile;
  float* ob = a.out + ((long)b * a.blocks + tx) * 3 * plane + xin;
  for (int t = rg; t < (y1 - y0) * 3; t += 256 / kCW) {  // t = (row, channel), uniform across the wave
    const int yl = t / 3, c = t - yl * 3, y = y0 + yl;
    int u;
    if (a.need_v) {
      const int ymin = lvb[2 * yl], n = lvb[2 * yl + 1];
      const int* k = lvk + yl * a.vks;
      int sacc = 1 << (kPrecisionBits - 1);
      const uint8_t* col = hbuf + ymin * hld + xl * 3 + c;
#pragma unroll
      for (int j = 0; j < KV; ++j)
        if (j < n) sacc += (int)col[j * hld] * k[j];
      u = clip8(sacc);
    } else {
      u = hbuf[(y - ylo) * hld + xl * 3 + c];
    }
    const float mean = c == 0 ? a.mean[0] : (c == 1 ? a.mean[1] : a.mean[2]);
    const float sd = c == 0 ? a.stdv[0] : (c == 1 ? a.stdv[1] : a.stdv[2]);
    const float v = ((float)u / 255.0f - mean) / sd;
    const int ty = y / a.tile;
    ob[((long)ty * a.tiles_x * 3 + c) * plane + (long)(y - ty * a.tile) * a.tile] = v;
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

// Largest source span any block of `per_block` consecutive outputs reads, from Pillow's bounds recomputed on the
// host (the same precompute_coeffs the caller's tables come from); per_block outputs if the size is unchanged.
static int max_block_window(int in_size, int out_size, int per_block, int need) {
  if (!need) return per_block < out_size ? per_block : out_size;
  const int ks = slx_resample_ksize(in_size, out_size);
  std::vector<int32_t> bnd(2 * (size_t)out_size), kk((size_t)out_size * ks);
  if (slx_resample_coeffs(in_size, out_size, ks, bnd.data(), kk.data()) < 0) return -1;
  int mx = 0;
  for (int o0 = 0; o0 < out_size; o0 += per_block) {
    const int o1 = (o0 + per_block < out_size ? o0 + per_block : out_size) - 1;
    const int span = bnd[2 * o1] + bnd[2 * o1 + 1] - bnd[2 * o0];
    mx = span > mx ? span : mx;
  }
  return mx;
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
  SLX_CHECK_ARG(d->rows_per_block > 0 && d->cols_per_block == kCW && d->lds_rows > 0 && d->lds_cols > 0,
                "slx_frames_to_tiles: rows_per_block, lds_rows/lds_cols must be set and cols_per_block == %d", kCW);
  const int hks = d->need_h ? d->hksize : 0, vks = d->need_v ? d->vksize : 0;
  const size_t lds = (size_t)4 * (d->cols_per_block * (hks + 2) + d->rows_per_block * (vks + 2)) +
                     (size_t)d->lds_rows * (d->lds_cols * 3 + 4) + (size_t)d->lds_rows * d->cols_per_block * 3;
  SLX_CHECK_ARG(lds <= 64 * 1024, "slx_frames_to_tiles: block window needs %zu B of LDS (> 64 KiB)", lds);
  {
    const int wr = max_block_window(d->H, d->th, d->rows_per_block, d->need_v);
    const int wc = max_block_window(d->W, d->tw, d->cols_per_block, d->need_h);
    SLX_CHECK_ARG(wr > 0 && wc > 0 && wr <= d->lds_rows && wc <= d->lds_cols,
                  "slx_frames_to_tiles: blocks of %dx%d outputs read %dx%d source pixels but the LDS window is %dx%d",
                  d->rows_per_block, d->cols_per_block, wr, wc, d->lds_rows, d->lds_cols);
  }
  if (d->B == 0) return 0;
  FrameArgs a;
  a.src = d->src;
  a.sb = d->sb; a.sy = d->sy; a.sx = d->sx; a.sc = d->sc;
  a.H = d->H; a.W = d->W; a.tw = d->tw; a.th = d->th; a.tile = d->tile;
  a.tiles_x = d->tw / d->tile;
  a.blocks = a.tiles_x * (d->th / d->tile);
  a.RY = d->rows_per_block; a.CW = d->cols_per_block; a.lds_rows = d->lds_rows; a.lds_cols = d->lds_cols;
  a.hb = d->hbounds; a.hk = d->hcoeffs; a.hks = hks;
  a.vb = d->vbounds; a.vk = d->vcoeffs; a.vks = vks;
  a.need_h = d->need_h; a.need_v = d->need_v;
  a.packed = d->sx == 3 && d->sc == 1 && d->sy % 4 == 0 && d->sb % 4 == 0 && ((uintptr_t)d->src & 3) == 0;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = d->mean[c];
    a.stdv[c] = d->std[c];
  }
  a.out = d->out;
  const dim3 grid((unsigned)((d->tw + a.CW - 1) / a.CW), (unsigned)((d->th + a.RY - 1) / a.RY), (unsigned)d->B);
  SLX_CHECK_ARG(hks <= 64 && vks <= 64, "slx_frames_to_tiles: ksize > 64");
  hipStream_t st = (hipStream_t)stream;
  if (hks <= 8 && vks <= 8) hipLaunchKernelGGL((frames_to_tiles_kernel<8, 8>), grid, dim3(256), lds, st, a);
  else if (hks <= 16 && vks <= 16) hipLaunchKernelGGL((frames_to_tiles_kernel<16, 16>), grid, dim3(256), lds, st, a);
  else hipLaunchKernelGGL((frames_to_tiles_kernel<64, 64>), grid, dim3(256), lds, st, a);
  SLX_LAUNCH_CHECK("slx_frames_to_tiles");
  return 0;
}

}  // extern "C"
