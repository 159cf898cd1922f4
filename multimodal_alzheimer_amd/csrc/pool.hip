// 3D max pooling (with argmax) and global average pooling on NDHWC activations, gfx950.
//
// Replaces nn.MaxPool3d(3, 2, 1) of the MedicalNet stem, nn.MaxPool3d(2) of the head /
// Small_PET_CNN conv blocks (pkg/models/pet_models/pet_cnn.py:26,
// pkg/models/mri_models/anat_cnn.py:62) and nn.AdaptiveAvgPool3d(1)
// (anat_cnn.py:66, pet_cnn.py:33).
//
// Max pool: consecutive threads walk consecutive channels of one voxel (coalesced).
// Ties resolve to the FIRST window position in (kd, kh, kw) scan order with a strict
// `>` (NaN always wins), exactly torch's CPU kernel; the window index is kept as one
// byte per output so the backward is a deterministic gather (no atomics) that adds the
// contributions of the overlapping windows in output order, as torch's CPU backward does.
#include "common.h"

namespace {

struct PoolG {
  int n, c, di, hi, wi, do_, ho, wo, k, s, p;
};

template <typename T>
__global__ void maxpool_fwd_kernel(PoolG g, const T* __restrict__ x, T* __restrict__ y,
                                   uint8_t* __restrict__ am) {
  const int64_t total = (int64_t)g.n * g.do_ * g.ho * g.wo * g.c;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.c);
    int64_t v = i / g.c;
    const int ow = (int)(v % g.wo); v /= g.wo;
    const int oh = (int)(v % g.ho); v /= g.ho;
    const int od = (int)(v % g.do_);
    const int64_t nb = v / g.do_;
    const int z0 = od * g.s - g.p, y0 = oh * g.s - g.p, x0 = ow * g.s - g.p;
    float best = -__builtin_inff();
    int bi = -1;
    for (int kd = 0; kd < g.k; ++kd) {
      const int z = z0 + kd;
      if ((unsigned)z >= (unsigned)g.di) continue;
      for (int kh = 0; kh < g.k; ++kh) {
        const int yy = y0 + kh;
        if ((unsigned)yy >= (unsigned)g.hi) continue;
        for (int kw = 0; kw < g.k; ++kw) {
          const int xx = x0 + kw;
          if ((unsigned)xx >= (unsigned)g.wi) continue;
          const float val = Elt<T>::ld(x, (((nb * g.di + z) * g.hi + yy) * g.wi + xx) * g.c + c);
          const int wi = (kd * g.k + kh) * g.k + kw;
          if (bi < 0) bi = wi;
          if (val > best || val != val) { best = val; bi = wi; }
        }
      }
    }
    Elt<T>::st(y, i, best);
    am[i] = (uint8_t)bi;
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(PoolG g, const T* __restrict__ dy,
                                   const uint8_t* __restrict__ am, T* __restrict__ dx) {
  const int64_t total = (int64_t)g.n * g.di * g.hi * g.wi * g.c;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.c);
    int64_t v = i / g.c;
    const int iw = (int)(v % g.wi); v /= g.wi;
    const int ih = (int)(v % g.hi); v /= g.hi;
    const int id = (int)(v % g.di);
    const int64_t nb = v / g.di;
    // outputs whose window covers this input: o*s - p <= i <= o*s - p + k - 1
    auto lo = [&](int ii) { int t = ii + g.p - (g.k - 1); return t <= 0 ? 0 : (t + g.s - 1) / g.s; };
    auto hi = [&](int ii, int lim) { int t = (ii + g.p) / g.s; return t < lim - 1 ? t : lim - 1; };
    const int d0 = lo(id), d1 = hi(id, g.do_);
    const int h0 = lo(ih), h1 = hi(ih, g.ho);
    const int w0 = lo(iw), w1 = hi(iw, g.wo);
    float acc = 0.f;
    for (int od = d0; od <= d1; ++od)
      for (int oh = h0; oh <= h1; ++oh)
        for (int ow = w0; ow <= w1; ++ow) {
          const int wi = ((id - (od * g.s - g.p)) * g.k + (ih - (oh * g.s - g.p))) * g.k +
                         (iw - (ow * g.s - g.p));
          const int64_t o = (((nb * g.do_ + od) * g.ho + oh) * g.wo + ow) * g.c + c;
          if (am[o] == wi) acc += Elt<T>::ld(dy, o);
        }
    Elt<T>::st(dx, i, acc);
  }
}

// GAP: one block per (n, 64-channel group); 4 row-lanes per channel, fp32 partial sums
template <typename T>
__global__ __launch_bounds__(256) void gap_fwd_kernel(int64_t S, int C, const T* __restrict__ x,
                                                     float* __restrict__ y) {
  __shared__ float red[256];
  const int n = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C)
    for (int64_t v = rl; v < S; v += 4) s += Elt<T>::ld(x, ((int64_t)n * S + v) * C + c);
  red[threadIdx.x] = s;
  __syncthreads();
  if (rl == 0 && c < C)
    y[(int64_t)n * C + c] = (red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] +
                             red[threadIdx.x + 192]) / (float)S;
}

template <typename T>
__global__ void gap_bwd_kernel(int n, int64_t S, int C, const float* __restrict__ dy,
                               T* __restrict__ dx) {
  const int64_t total = (int64_t)n * S * C;
  const float inv = 1.f / (float)S;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int64_t nb = i / ((int64_t)S * C);
    Elt<T>::st(dx, i, dy[nb * C + c] * inv);
  }
}

unsigned grid_of(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 256 * 16));
}

bool pool_ok(const PoolG& g) {
  if (g.n <= 0 || g.c <= 0 || g.di <= 0 || g.hi <= 0 || g.wi <= 0 || g.k <= 0 || g.s <= 0 ||
      g.p < 0 || g.k * g.k * g.k > 255 || 2 * g.p > g.k)
    return false;
  auto ext = [&](int i) { return (i + 2 * g.p - g.k) / g.s + 1; };
  return ext(g.di) == g.do_ && ext(g.hi) == g.ho && ext(g.wi) == g.wo;
}

}  // namespace

extern "C" {

int mmad_maxpool3d_fwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                       int k, int s, int p, const void* x, void* y, uint8_t* argmax,
                       void* stream) {
  PoolG g{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(g)) return MMAD_EBADSHAPE;
  if (!x || !y || !argmax) return MMAD_ENULL;
  const unsigned grid = grid_of((int64_t)n * do_ * ho * wo * c);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<u16>, dim3(grid), dim3(256), 0, as_stream(stream), g,
                       (const u16*)x, (u16*)y, argmax);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
                       g, (const float*)x, (float*)y, argmax);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_maxpool3d_bwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                       int k, int s, int p, const void* dy, const uint8_t* argmax, void* dx,
                       void* stream) {
  PoolG g{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(g)) return MMAD_EBADSHAPE;
  if (!dy || !dx || !argmax) return MMAD_ENULL;
  const unsigned grid = grid_of((int64_t)n * di * hi * wi * c);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<u16>, dim3(grid), dim3(256), 0, as_stream(stream), g,
                       (const u16*)dy, argmax, (u16*)dx);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream),
                       g, (const float*)dy, argmax, (float*)dx);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_gap_fwd(int dtype, int n, int64_t s, int c, const void* x, float* y, void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!x || !y) return MMAD_ENULL;
  dim3 grid((unsigned)cdiv(c, 64), (unsigned)n);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(gap_fwd_kernel<u16>, grid, dim3(256), 0, as_stream(stream), s, c,
                       (const u16*)x, y);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(gap_fwd_kernel<float>, grid, dim3(256), 0, as_stream(stream), s, c,
                       (const float*)x, y);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_gap_bwd(int dtype, int n, int64_t s, int c, const float* dy, void* dx, void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!dy || !dx) return MMAD_ENULL;
  const unsigned grid = grid_of((int64_t)n * s * c);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(gap_bwd_kernel<u16>, dim3(grid), dim3(256), 0, as_stream(stream), n, s, c,
                       dy, (u16*)dx);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(grid), dim3(256), 0, as_stream(stream), n, s,
                       c, dy, (float*)dx);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

}  // extern "C"
