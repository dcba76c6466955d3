// Frame decode: the per-step arithmetic of the reference data path, on the GPU.
//
// The reference decodes every camera frame on the CPU each step (dataset/carla_dataset.py):
//   image  ProcessImage (:494-515): uint8 RGB crop -> fp32 / 255 -> minus ImageNet mean ->
//          over ImageNet std (torchvision ToTensor + Normalize), channels-first;
//   depth  get_depth (:114-131): uint8 CARLA depth RGB -> (R + 256 G + 65536 B) / (2^24 - 1)
//          * 1000, float64 metres;
//   seg    (:404-406) class map -> int64.
// The frame cache (dataset/frame_cache.py) keeps the cropped uint8 pixels resident in HBM;
// these kernels gather a batch out of it (optional source-frame / source-row table) and turn
// it into the reference's tensors in the same pass.  HBM-bound byte work:
// one thread per 4 pixels (3 dword loads of packed RGB, float4 / double2 stores), 26 bytes
// of traffic per camera pixel (6 read, 12 + 8 written).
#include "common.h"

namespace e2ep {

constexpr int DEC_THREADS = 256;

__device__ __forceinline__ unsigned byte_of(const unsigned w[3], int k) {
  return (w[k >> 2] >> ((k & 3) * 8)) & 0xffu;
}

// rgb/depth_rgb [*][hw][3] uint8 (either may be null); output frame f reads source frame
// src[f] (f when src is null); image [frames][3][hw] fp32; depth [frames][hw] fp64.
// hw % 4 == 0, so a quad never straddles two frames.
__global__ void __launch_bounds__(DEC_THREADS)
    k_decode_frames(const unsigned *__restrict__ rgb, const unsigned *__restrict__ depth_rgb,
                    const long long *__restrict__ src, long long quads, int hw,
                    float *__restrict__ image, double *__restrict__ depth) {
  const long long q = (long long)blockIdx.x * DEC_THREADS + threadIdx.x;
  if (q >= quads) return;
  const long long p0 = q * 4;
  const long long frame = p0 / hw;
  const int off = (int)(p0 - frame * hw);
  // source quad: 3 dwords per quad, hw / 4 quads per frame
  const long long sq = (src ? src[frame] : frame) * (hw / 4) + off / 4;
  if (rgb) {
    const unsigned w[3] = {rgb[3 * sq], rgb[3 * sq + 1], rgb[3 * sq + 2]};
    const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
    for (int c = 0; c < 3; ++c) {
      float v[4];
      for (int j = 0; j < 4; ++j) v[j] = ((float)byte_of(w, 3 * j + c) / 255.f - mean[c]) / stdv[c];
      *reinterpret_cast<float4 *>(image + (frame * 3 + c) * hw + off) =
          make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (depth_rgb) {
    const unsigned w[3] = {depth_rgb[3 * sq], depth_rgb[3 * sq + 1], depth_rgb[3 * sq + 2]};
    double d[4];
    for (int j = 0; j < 4; ++j) {
      // exact integer sum, then the reference's two float64 roundings: / (2^24 - 1), * 1000
      const double s = (double)(byte_of(w, 3 * j) + 256u * byte_of(w, 3 * j + 1) +
                                65536u * byte_of(w, 3 * j + 2));
      d[j] = 1000.0 * (s / 16777215.0);
    }
    double2 *o = reinterpret_cast<double2 *>(depth + frame * hw + off);
    o[0] = make_double2(d[0], d[1]);
    o[1] = make_double2(d[2], d[3]);
  }
}

// uint8 rows -> int64 (class maps): output row r reads source row src[r] (r when null);
// 4 bytes per thread, one dword load, two 16-byte stores.  row_len % 4 == 0.
__global__ void __launch_bounds__(DEC_THREADS)
    k_widen_u8_i64(const unsigned *__restrict__ in, const long long *__restrict__ src,
                   long long quads, int row_len, long long *__restrict__ dst) {
  const long long q = (long long)blockIdx.x * DEC_THREADS + threadIdx.x;
  if (q >= quads) return;
  const long long row = q * 4 / row_len;
  const int off = (int)(q * 4 - row * row_len);
  const unsigned w = in[((src ? src[row] : row) * row_len + off) / 4];
  longlong2 *o = reinterpret_cast<longlong2 *>(dst + q * 4);
  o[0] = make_longlong2(w & 0xff, (w >> 8) & 0xff);
  o[1] = make_longlong2((w >> 16) & 0xff, w >> 24);
}

}  // namespace e2ep

using namespace e2ep;

extern "C" {

int e2ep_decode_frames(const void *rgb, const void *depth_rgb, const long long *src_frame,
                       long long frames, int hw, float *image, double *depth, void *stream) {
  E2EP_REQUIRE(frames >= 0 && hw > 0 && hw % 4 == 0, E2EP_EINVAL,
               "e2ep_decode_frames: need hw %% 4 == 0 (hw=%d)", hw);
  E2EP_REQUIRE((!rgb || image) && (!depth_rgb || depth), E2EP_EINVAL,
               "e2ep_decode_frames: missing output");
  E2EP_REQUIRE(((uintptr_t)rgb & 3) == 0 && ((uintptr_t)depth_rgb & 3) == 0 &&
                   ((uintptr_t)image & 15) == 0 && ((uintptr_t)depth & 15) == 0,
               E2EP_EINVAL, "e2ep_decode_frames: misaligned buffer");
  const long long quads = frames * hw / 4;
  if (quads == 0 || (!rgb && !depth_rgb)) return 0;
  hipLaunchKernelGGL(k_decode_frames, dim3(cdiv(quads, DEC_THREADS)), dim3(DEC_THREADS), 0,
                     as_stream(stream), static_cast<const unsigned *>(rgb),
                     static_cast<const unsigned *>(depth_rgb), src_frame, quads, hw, image, depth);
  return launch_status("e2ep_decode_frames");
}

int e2ep_widen_u8_i64(const void *src, const long long *src_row, long long rows, int row_len,
                      long long *dst, void *stream) {
  E2EP_REQUIRE(rows >= 0 && row_len > 0 && row_len % 4 == 0, E2EP_EINVAL,
               "e2ep_widen_u8_i64: need row_len %% 4 == 0 (row_len=%d)", row_len);
  E2EP_REQUIRE(rows == 0 || (src && dst), E2EP_EINVAL, "e2ep_widen_u8_i64: null buffer");
  E2EP_REQUIRE(((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 15) == 0, E2EP_EINVAL,
               "e2ep_widen_u8_i64: misaligned buffer");
  const long long quads = rows * row_len / 4;
  if (quads == 0) return 0;
  hipLaunchKernelGGL(k_widen_u8_i64, dim3(cdiv(quads, DEC_THREADS)), dim3(DEC_THREADS), 0,
                     as_stream(stream), static_cast<const unsigned *>(src), src_row, quads,
                     row_len, dst);
  return launch_status("e2ep_widen_u8_i64");
}

}  // extern "C"
