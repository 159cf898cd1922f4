// PET-MRI early fusion and feature-map fusion glue, gfx950.
//
// Replaces the tensor plumbing of the reference's two voxel-level fusion models:
//   * PET_MRI_EF.general_step  torch.stack((x_pet, x_mri), dim=1).to(float32)
//     (pkg/models/fusion_models/early_fusion.py:77-80) feeding a Cin = 2 Conv3d (:35):
//     mmad_gather_channels writes the channel-stacked input directly in the conv's NDHWC
//     layout with the channel count padded to 8 (one 16-byte bf16 vector per voxel) and
//     zeros in the pad lanes; mmad_pad_rows pads the weight's Ci the same way and cuts the
//     weight gradient back.  Zero channels times zero weights add exact zeros, so the
//     padded conv is bit-identical in value to the unpadded one.
//   * PET_MRI_FMF.forward  torch.cat((out_pet, out_mri), dim=1) ('concatenate') and
//     torch.max(torch.stack((out_pet, out_mri)), dim=0) ('maxout')
//     (pkg/models/fusion_models/anat_pet_featuremapfusion.py:112-118):
//     mmad_concat_channels / mmad_split_channels interleave two NDHWC volumes per voxel;
//     mmad_max2_fwd / _bwd take the voxel-wise max with torch's tie and NaN rules (ties ->
//     the first operand, i.e. index 0; a NaN wins, the first NaN if both) and route the
//     gradient to the selected operand only, as MaxBackward does.
//
// All four are single-pass HBM streams (16-byte vectors where the channel counts allow).
#include "common.h"

namespace {

unsigned grid_of(int64_t n, int block = 256) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, block), 256 * 32));
}

struct Planes {
  const void* p[8];
};

template <typename TI>
__device__ __forceinline__ float load_as_f32(const TI* p, int64_t i) {
  if constexpr (sizeof(TI) == 2) return bf2f(p[i]);
  else return (float)p[i];                 // f64 -> f32 rounds once, as torch's .to(float32)
}

// dst[(b*vox + v)*CP + c] = c < nsrc ? src_c[b*bstride + v*vstride] : 0   (CP = 8)
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void gather_channels_kernel(Planes P, int nsrc, int64_t bstride,
                                                              int64_t vstride, int n,
                                                              int64_t vox, TO* __restrict__ dst) {
  const int64_t total = (int64_t)n * vox;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / vox, v = i - b * vox;
    const int64_t off = b * bstride + v * vstride;
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      f[c] = c < nsrc ? load_as_f32(reinterpret_cast<const TI*>(P.p[c]), off) : 0.f;
    if constexpr (sizeof(TO) == 2) {
      Chunk<u16>::store(dst + i * 8, f);
    } else {
      Chunk<float>::store(dst + i * 8, f);
      Chunk<float>::store(dst + i * 8 + 4, f + 4);
    }
  }
}

// dst[r][j] = j < cin ? src[r][j] : 0, j < cout   (weights: [Co][Ci*taps] rows)
__global__ void pad_rows_kernel(int rows, int cin, int cout, const float* __restrict__ src,
                                float* __restrict__ dst) {
  const int64_t total = (int64_t)rows * cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cout), j = (int)(i - (int64_t)r * cout);
    dst[i] = j < cin ? src[(int64_t)r * cin + j] : 0.f;
  }
}

// torch.max(stack((a, b)), 0): b is selected iff b > a, or b is NaN and a is not
__device__ __forceinline__ bool pick_b(float a, float b) {
  return b > a || (b != b && a == a);
}

template <typename T>
__global__ __launch_bounds__(256) void max2_fwd_kernel(int64_t nchunks, const T* __restrict__ a,
                                                       const T* __restrict__ b,
                                                       T* __restrict__ y,
                                                       uint8_t* __restrict__ sel) {
  constexpr int V = Chunk<T>::N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunks;
       i += (int64_t)gridDim.x * blockDim.x) {
    float fa[V], fb[V], o[V];
    Chunk<T>::load(a + i * V, fa);
    Chunk<T>::load(b + i * V, fb);
    uint8_t s[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const bool pb = pick_b(fa[e], fb[e]);
      o[e] = pb ? fb[e] : fa[e];
      s[e] = pb ? 1 : 0;
    }
    Chunk<T>::store(y + i * V, o);               // values pass through unchanged
#pragma unroll
    for (int e = 0; e < V; ++e) sel[i * V + e] = s[e];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void max2_bwd_kernel(int64_t nchunks, const T* __restrict__ g,
                                                       const uint8_t* __restrict__ sel,
                                                       T* __restrict__ ga, T* __restrict__ gb) {
  constexpr int V = Chunk<T>::N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nchunks;
       i += (int64_t)gridDim.x * blockDim.x) {
    float fg[V], oa[V], ob[V];
    Chunk<T>::load(g + i * V, fg);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const bool pb = sel[i * V + e] != 0;
      oa[e] = pb ? 0.f : fg[e];
      ob[e] = pb ? fg[e] : 0.f;
    }
    Chunk<T>::store(ga + i * V, oa);
    Chunk<T>::store(gb + i * V, ob);
  }
}

// NDHWC channel concat of two volumes: one thread per 16-byte chunk of the output row.
template <typename T>
__global__ __launch_bounds__(256) void concat_ch_kernel(int64_t rows, int ca, int cb,
                                                        const T* __restrict__ a,
                                                        const T* __restrict__ b,
                                                        T* __restrict__ dst) {
  constexpr int V = Chunk<T>::N;
  const int qa = ca / V, qb = cb / V, q = qa + qb;
  const int64_t total = rows * q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q;
    const int j = (int)(i - r * q);
    const T* src = j < qa ? a + (r * qa + j) * V : b + (r * qb + (j - qa)) * V;
    *reinterpret_cast<u32x4*>(dst + i * V) = *reinterpret_cast<const u32x4*>(src);
  }
}

// inverse of concat_ch_kernel; a NULL destination skips its half
template <typename T>
__global__ __launch_bounds__(256) void split_ch_kernel(int64_t rows, int ca, int cb,
                                                       const T* __restrict__ src,
                                                       T* __restrict__ a, T* __restrict__ b) {
  constexpr int V = Chunk<T>::N;
  const int qa = ca / V, qb = cb / V, q = qa + qb;
  const int64_t total = rows * q;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q;
    const int j = (int)(i - r * q);
    T* d = j < qa ? (a ? a + (r * qa + j) * V : nullptr)
                  : (b ? b + (r * qb + (j - qa)) * V : nullptr);
    if (d == nullptr) continue;
    *reinterpret_cast<u32x4*>(d) = *reinterpret_cast<const u32x4*>(src + i * V);
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int mmad_gather_channels(int in_dtype, int nsrc, const void* const* srcs, int64_t batch_stride,
                         int64_t vox_stride, int n, int64_t vox, int cpad, int out_dtype,
                         void* dst, void* stream) {
  if (nsrc <= 0 || nsrc > 8 || cpad != 8 || n <= 0 || vox <= 0 || vox_stride <= 0 ||
      batch_stride < 0)
    return MMAD_EBADSHAPE;
  if (!srcs || !dst) return MMAD_ENULL;
  Planes P{};
  for (int c = 0; c < nsrc; ++c) {
    if (!srcs[c]) return MMAD_ENULL;
    P.p[c] = srcs[c];
  }
  if (!aligned16(dst)) return MMAD_EBADSHAPE;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_of((int64_t)n * vox);
#define GATHER(TI, TO)                                                                        \
  hipLaunchKernelGGL((gather_channels_kernel<TI, TO>), dim3(grid), dim3(256), 0, st, P, nsrc, \
                     batch_stride, vox_stride, n, vox, (TO*)dst)
  if (in_dtype == MMAD_F64 && out_dtype == MMAD_F32) GATHER(double, float);
  else if (in_dtype == MMAD_F64 && out_dtype == MMAD_BF16) GATHER(double, u16);
  else if (in_dtype == MMAD_F32 && out_dtype == MMAD_F32) GATHER(float, float);
  else if (in_dtype == MMAD_F32 && out_dtype == MMAD_BF16) GATHER(float, u16);
  else if (in_dtype == MMAD_BF16 && out_dtype == MMAD_BF16) GATHER(u16, u16);
  else return MMAD_EBADDTYPE;
#undef GATHER
  return launch_status();
}

int mmad_pad_rows(int rows, int cin, int cout, const float* src, float* dst, void* stream) {
  if (rows <= 0 || cin <= 0 || cout <= 0) return MMAD_EBADSHAPE;
  if (!src || !dst) return MMAD_ENULL;
  hipLaunchKernelGGL(pad_rows_kernel, dim3(grid_of((int64_t)rows * cout)), dim3(256), 0,
                     as_stream(stream), rows, cin, cout, src, dst);
  return launch_status();
}

int mmad_max2_fwd(int dtype, int64_t n, const void* a, const void* b, void* y, uint8_t* sel,
                  void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!a || !b || !y || !sel) return MMAD_ENULL;
  if (!aligned16(a) || !aligned16(b) || !aligned16(y)) return MMAD_EBADSHAPE;
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16) {
    if (n % 8) return MMAD_EBADSHAPE;
    hipLaunchKernelGGL(max2_fwd_kernel<u16>, dim3(grid_of(n / 8)), dim3(256), 0, st, n / 8,
                       (const u16*)a, (const u16*)b, (u16*)y, sel);
  } else if (dtype == MMAD_F32) {
    if (n % 4) return MMAD_EBADSHAPE;
    hipLaunchKernelGGL(max2_fwd_kernel<float>, dim3(grid_of(n / 4)), dim3(256), 0, st, n / 4,
                       (const float*)a, (const float*)b, (float*)y, sel);
  } else {
    return MMAD_EBADDTYPE;
  }
  return launch_status();
}

int mmad_max2_bwd(int dtype, int64_t n, const void* g, const uint8_t* sel, void* ga, void* gb,
                  void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!g || !sel || !ga || !gb) return MMAD_ENULL;
  if (!aligned16(g) || !aligned16(ga) || !aligned16(gb)) return MMAD_EBADSHAPE;
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16) {
    if (n % 8) return MMAD_EBADSHAPE;
    hipLaunchKernelGGL(max2_bwd_kernel<u16>, dim3(grid_of(n / 8)), dim3(256), 0, st, n / 8,
                       (const u16*)g, sel, (u16*)ga, (u16*)gb);
  } else if (dtype == MMAD_F32) {
    if (n % 4) return MMAD_EBADSHAPE;
    hipLaunchKernelGGL(max2_bwd_kernel<float>, dim3(grid_of(n / 4)), dim3(256), 0, st, n / 4,
                       (const float*)g, sel, (float*)ga, (float*)gb);
  } else {
    return MMAD_EBADDTYPE;
  }
  return launch_status();
}

int mmad_concat_channels(int dtype, int64_t rows, int ca, const void* a, int cb, const void* b,
                         void* dst, void* stream) {
  const int V = dtype == MMAD_BF16 ? 8 : 4;
  if (dtype != MMAD_BF16 && dtype != MMAD_F32) return MMAD_EBADDTYPE;
  if (rows <= 0 || ca <= 0 || cb <= 0 || ca % V || cb % V) return MMAD_EBADSHAPE;
  if (!a || !b || !dst) return MMAD_ENULL;
  if (!aligned16(a) || !aligned16(b) || !aligned16(dst)) return MMAD_EBADSHAPE;
  const int64_t total = rows * ((ca + cb) / V);
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(concat_ch_kernel<u16>, dim3(grid_of(total)), dim3(256), 0, st, rows, ca,
                       cb, (const u16*)a, (const u16*)b, (u16*)dst);
  else
    hipLaunchKernelGGL(concat_ch_kernel<float>, dim3(grid_of(total)), dim3(256), 0, st, rows, ca,
                       cb, (const float*)a, (const float*)b, (float*)dst);
  return launch_status();
}

int mmad_split_channels(int dtype, int64_t rows, int ca, int cb, const void* src, void* a,
                        void* b, void* stream) {
  const int V = dtype == MMAD_BF16 ? 8 : 4;
  if (dtype != MMAD_BF16 && dtype != MMAD_F32) return MMAD_EBADDTYPE;
  if (rows <= 0 || ca <= 0 || cb <= 0 || ca % V || cb % V) return MMAD_EBADSHAPE;
  if (!src || (!a && !b)) return MMAD_ENULL;
  if (!aligned16(src) || !aligned16(a) || !aligned16(b)) return MMAD_EBADSHAPE;
  const int64_t total = rows * ((ca + cb) / V);
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(split_ch_kernel<u16>, dim3(grid_of(total)), dim3(256), 0, st, rows, ca, cb,
                       (const u16*)src, (u16*)a, (u16*)b);
  else
    hipLaunchKernelGGL(split_ch_kernel<float>, dim3(grid_of(total)), dim3(256), 0, st, rows, ca,
                       cb, (const float*)src, (float*)a, (float*)b);
  return launch_status();
}

}  // extern "C"
