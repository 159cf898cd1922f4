// 3D max pooling (with argmax) and global average pooling on NDHWC activations, gfx950.
//
// Replaces nn.MaxPool3d(3, 2, 1) of the MedicalNet stem, nn.MaxPool3d(2) of the head /
// Small_PET_CNN conv blocks (pkg/models/pet_models/pet_cnn.py:26,
// pkg/models/mri_models/anat_cnn.py:62) and nn.AdaptiveAvgPool3d(1)
// (anat_cnn.py:66, pet_cnn.py:33).
//
// Every thread owns V consecutive channels of one voxel (16-byte vectors when C % VEC ==
// 0), so all loads and stores are coalesced vectors.  Max-pool ties resolve to the FIRST
// window position in (kd, kh, kw) scan order with a strict `>` (NaN always wins), exactly
// torch's CPU kernel; the window index is kept as one byte per output so the backward is
// a deterministic gather (no atomics) that adds the contributions of the overlapping
// windows in output order, as torch's CPU backward does.
#include <atomic>
#include <cstdlib>

#include "common.h"
#include "patchconv.h"

namespace {

struct PoolG {
  int n, c, di, hi, wi, do_, ho, wo, k, s, p;
};

template <typename T, int V>
__device__ __forceinline__ void load_v(const T* p, float* v) {
  if constexpr (V == Chunk<T>::N) Chunk<T>::load(p, v);
  else for (int e = 0; e < V; ++e) v[e] = Elt<T>::ld(p, e);
}
template <typename T, int V>
__device__ __forceinline__ void store_v(T* p, const float* v) {
  if constexpr (V == Chunk<T>::N) Chunk<T>::store(p, v);
  else for (int e = 0; e < V; ++e) Elt<T>::st(p, e, v[e]);
}

template <typename T, int V>
__global__ void maxpool_fwd_kernel(PoolG g, const T* __restrict__ x, T* __restrict__ y,
                                   uint8_t* __restrict__ am) {
  const int cv = g.c / V;
  const int64_t total = (int64_t)g.n * g.do_ * g.ho * g.wo * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int64_t ovox = v;
    const int ow = (int)(v % g.wo); v /= g.wo;
    const int oh = (int)(v % g.ho); v /= g.ho;
    const int od = (int)(v % g.do_);
    const int64_t nb = v / g.do_;
    const int z0 = od * g.s - g.p, y0 = oh * g.s - g.p, x0 = ow * g.s - g.p;
    float best[V];
    int bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { best[e] = -__builtin_inff(); bi[e] = -1; }
    for (int kd = 0; kd < g.k; ++kd) {
      const int z = z0 + kd;
      if ((unsigned)z >= (unsigned)g.di) continue;
      for (int kh = 0; kh < g.k; ++kh) {
        const int yy = y0 + kh;
        if ((unsigned)yy >= (unsigned)g.hi) continue;
        for (int kw = 0; kw < g.k; ++kw) {
          const int xx = x0 + kw;
          if ((unsigned)xx >= (unsigned)g.wi) continue;
          float val[V];
          load_v<T, V>(x + (((nb * g.di + z) * g.hi + yy) * g.wi + xx) * g.c + c0, val);
          const int wi = (kd * g.k + kh) * g.k + kw;
#pragma unroll
          for (int e = 0; e < V; ++e) {
            if (bi[e] < 0) bi[e] = wi;
            if (val[e] > best[e] || val[e] != val[e]) { best[e] = val[e]; bi[e] = wi; }
          }
        }
      }
    }
    store_v<T, V>(y + ovox * g.c + c0, best);
#pragma unroll
    for (int e = 0; e < V; ++e) am[ovox * g.c + c0 + e] = (uint8_t)bi[e];
  }
}

template <typename T, int V>
__global__ void maxpool_bwd_kernel(PoolG g, const T* __restrict__ dy,
                                   const uint8_t* __restrict__ am, T* __restrict__ dx) {
  const int cv = g.c / V;
  const int64_t total = (int64_t)g.n * g.di * g.hi * g.wi * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int64_t ivox = v;
    const int iw = (int)(v % g.wi); v /= g.wi;
    const int ih = (int)(v % g.hi); v /= g.hi;
    const int id = (int)(v % g.di);
    const int64_t nb = v / g.di;
    // outputs whose window covers this input: o*s - p <= i <= o*s - p + k - 1
    auto lo = [&](int ii) { int q = ii + g.p - (g.k - 1); return q <= 0 ? 0 : (q + g.s - 1) / g.s; };
    auto hi = [&](int ii, int lim) { int q = (ii + g.p) / g.s; return q < lim - 1 ? q : lim - 1; };
    const int d0 = lo(id), d1 = hi(id, g.do_);
    const int h0 = lo(ih), h1 = hi(ih, g.ho);
    const int w0 = lo(iw), w1 = hi(iw, g.wo);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int od = d0; od <= d1; ++od)
      for (int oh = h0; oh <= h1; ++oh)
        for (int ow = w0; ow <= w1; ++ow) {
          const int wi = ((id - (od * g.s - g.p)) * g.k + (ih - (oh * g.s - g.p))) * g.k +
                         (iw - (ow * g.s - g.p));
          const int64_t o = (((nb * g.do_ + od) * g.ho + oh) * g.wo + ow) * g.c + c0;
          uint8_t a[V];
          if constexpr (V == 8) {
            const uint64_t w = *reinterpret_cast<const uint64_t*>(am + o);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = (uint8_t)(w >> (8 * e));
          } else if constexpr (V == 4) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(am + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) a[e] = (uint8_t)(w >> (8 * e));
          } else {
            for (int e = 0; e < V; ++e) a[e] = am[o + e];
          }
          bool any = false;
#pragma unroll
          for (int e = 0; e < V; ++e) any |= a[e] == wi;
          if (!any) continue;
          float gv[V];
          load_v<T, V>(dy + o, gv);
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (a[e] == wi) acc[e] += gv[e];
        }
    store_v<T, V>(dx + ivox * g.c + c0, acc);
  }
}

// Fused MedicalNet stem tail: out = maxpool(relu(bn(y))) straight from the conv output y.
// The BN+ReLU value is rounded to T before the comparison, so out and the argmax equal the
// unfused scale_shift_act -> maxpool_fwd chain bit for bit.  am = window index | 0x80 when
// the max is > 0 (ReLU passed it); ymax = the raw y at the argmax (backward x-hat).
template <typename T, int V>
__global__ void bnpool_fwd_kernel(PoolG g, const T* __restrict__ y,
                                  const float* __restrict__ scale,
                                  const float* __restrict__ shift, T* __restrict__ out,
                                  uint8_t* __restrict__ am, T* __restrict__ ymax) {
  const int cv = g.c / V;
  const int64_t total = (int64_t)g.n * g.do_ * g.ho * g.wo * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int64_t ovox = v;
    const int ow = (int)(v % g.wo); v /= g.wo;
    const int oh = (int)(v % g.ho); v /= g.ho;
    const int od = (int)(v % g.do_);
    const int64_t nb = v / g.do_;
    const int z0 = od * g.s - g.p, y0 = oh * g.s - g.p, x0 = ow * g.s - g.p;
    float sc[V], sh[V], best[V], braw[V];
    int bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      sc[e] = scale[c0 + e]; sh[e] = shift[c0 + e];
      best[e] = -__builtin_inff(); braw[e] = 0.f; bi[e] = -1;
    }
    for (int kd = 0; kd < g.k; ++kd) {
      const int z = z0 + kd;
      if ((unsigned)z >= (unsigned)g.di) continue;
      for (int kh = 0; kh < g.k; ++kh) {
        const int yy = y0 + kh;
        if ((unsigned)yy >= (unsigned)g.hi) continue;
        for (int kw = 0; kw < g.k; ++kw) {
          const int xx = x0 + kw;
          if ((unsigned)xx >= (unsigned)g.wi) continue;
          float raw[V];
          load_v<T, V>(y + (((nb * g.di + z) * g.hi + yy) * g.wi + xx) * g.c + c0, raw);
          const int wi = (kd * g.k + kh) * g.k + kw;
#pragma unroll
          for (int e = 0; e < V; ++e) {
            const float val = as_stored<T>(fmaxf(bn_affine(raw[e], sc[e], sh[e]), 0.f));
            if (bi[e] < 0) { bi[e] = wi; braw[e] = raw[e]; }
            if (val > best[e] || val != val) { best[e] = val; bi[e] = wi; braw[e] = raw[e]; }
          }
        }
      }
    }
    store_v<T, V>(out + ovox * g.c + c0, best);
    store_v<T, V>(ymax + ovox * g.c + c0, braw);
#pragma unroll
    for (int e = 0; e < V; ++e)
      am[ovox * g.c + c0 + e] = (uint8_t)(bi[e] | (best[e] > 0.f ? 0x80 : 0));
  }
}

// k = 3 form of bnpool_fwd_kernel: per window plane the 9 loads are unrolled and issued
// together (clamped addresses for padding positions, masked out of the comparison); the
// argmax bytes of a channel vector leave in one store.
template <typename T, int V>
__device__ __forceinline__ void bnpool3_fwd_one(const PoolG& g, const T* __restrict__ y,
                                                const float* __restrict__ scale,
                                                const float* __restrict__ shift,
                                                T* __restrict__ out, uint8_t* __restrict__ am,
                                                T* __restrict__ ymax, int64_t nb, int od,
                                                int oh, int ow, int c0, const float* sc,
                                                const float* sh) {
  const int64_t ovox = ((nb * g.do_ + od) * g.ho + oh) * g.wo + ow;
  const int z0 = od * g.s - g.p, y0 = oh * g.s - g.p, x0 = ow * g.s - g.p;
  float best[V], braw[V];
  int bi[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    best[e] = -__builtin_inff(); braw[e] = 0.f; bi[e] = -1;
  }
  for (int kd = 0; kd < 3; ++kd) {
    const int z = z0 + kd;
    if ((unsigned)z >= (unsigned)g.di) continue;
    float raw[9][V];
    bool ok[9];
#pragma unroll
    for (int w = 0; w < 9; ++w) {
      const int yy = y0 + w / 3, xx = x0 + w % 3;
      ok[w] = (unsigned)yy < (unsigned)g.hi && (unsigned)xx < (unsigned)g.wi;
      const int yc = min(max(yy, 0), g.hi - 1), xc = min(max(xx, 0), g.wi - 1);
      load_v<T, V>(y + (((nb * g.di + z) * g.hi + yc) * g.wi + xc) * g.c + c0, raw[w]);
    }
#pragma unroll
    for (int w = 0; w < 9; ++w) {
      if (!ok[w]) continue;
      const int wi = kd * 9 + w;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float val = as_stored<T>(fmaxf(bn_affine(raw[w][e], sc[e], sh[e]), 0.f));
        if (bi[e] < 0) { bi[e] = wi; braw[e] = raw[w][e]; }
        if (val > best[e] || val != val) { best[e] = val; bi[e] = wi; braw[e] = raw[w][e]; }
      }
    }
  }
  store_v<T, V>(out + ovox * g.c + c0, best);
  store_v<T, V>(ymax + ovox * g.c + c0, braw);
  uint64_t packed = 0;
#pragma unroll
  for (int e = 0; e < V; ++e)
    packed |= (uint64_t)(uint8_t)(bi[e] | (best[e] > 0.f ? 0x80 : 0)) << (8 * e);
  if constexpr (V == 8) *reinterpret_cast<uint64_t*>(am + ovox * g.c + c0) = packed;
  else if constexpr (V == 4) *reinterpret_cast<uint32_t*>(am + ovox * g.c + c0) = (uint32_t)packed;
  else for (int e = 0; e < V; ++e) am[ovox * g.c + c0 + e] = (uint8_t)(packed >> (8 * e));
}

// k = 3 form of bnpool_fwd_kernel: per window plane the 9 loads are unrolled and issued
// together (clamped addresses for padding positions, masked out of the comparison); the
// argmax bytes of a channel vector leave in one store.
template <typename T, int V>
__global__ void bnpool3_fwd_kernel(PoolG g, const T* __restrict__ y,
                                   const float* __restrict__ scale,
                                   const float* __restrict__ shift, T* __restrict__ out,
                                   uint8_t* __restrict__ am, T* __restrict__ ymax) {
  const int cv = g.c / V;
  const int64_t total = (int64_t)g.n * g.do_ * g.ho * g.wo * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int ow = (int)(v % g.wo); v /= g.wo;
    const int oh = (int)(v % g.ho); v /= g.ho;
    const int od = (int)(v % g.do_);
    float sc[V], sh[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { sc[e] = scale[c0 + e]; sh[e] = shift[c0 + e]; }
    bnpool3_fwd_one<T, V>(g, y, scale, shift, out, am, ymax, v / g.do_, od, oh, ow, c0, sc, sh);
  }
}

// bf16 form of bnpool3_fwd_one for 8 channels, on packed words: per pair of channels one
// packed FMA, one RNE pack to bf16 and one packed 16-bit max for the ReLU (bf16 bits of a
// non-negative value order like integers), then each channel's candidate is the 32-bit key
// (bf16 bits << 16 | 31 - window index), so "larger value, else earlier position" is one
// unsigned compare.  The old per-channel float compare / index / raw bookkeeping cost ~11
// VALU ops per loaded element and made the kernel VALU-bound; this is ~7.  Padded window
// positions load their clamped in-window neighbour and carry that neighbour's index, so
// they tie with it and never win.  NaN: relu(NaN) stays NaN (as torch) and wins the window.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void bnpool3_fwd_one_bf16(const PoolG& g, const u16* __restrict__ y,
                                                     u16* __restrict__ out,
                                                     uint8_t* __restrict__ am,
                                                     u16* __restrict__ ymax, int64_t nb, int od,
                                                     int oh, int ow, int c0, const f32x2* sc2,
                                                     const f32x2* sh2) {
  const int64_t ovox = ((nb * g.do_ + od) * g.ho + oh) * g.wo + ow;
  const int z0 = od * g.s - g.p, y0 = oh * g.s - g.p, x0 = ow * g.s - g.p;
  uint32_t key[8], rb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { key[e] = 0; rb[e] = 0; }
  for (int kd = 0; kd < 3; ++kd) {
    const int z = z0 + kd;
    if ((unsigned)z >= (unsigned)g.di) continue;     // block-uniform (od is per block)
    u32x4 raw[9];
    uint32_t tag[9];
#pragma unroll
    for (int w = 0; w < 9; ++w) {
      const int yc = min(max(y0 + w / 3, 0), g.hi - 1), xc = min(max(x0 + w % 3, 0), g.wi - 1);
      tag[w] = 31 - (kd * 9 + (yc - y0) * 3 + (xc - x0));
      raw[w] = *reinterpret_cast<const u32x4*>(y + (((nb * g.di + z) * g.hi + yc) * g.wi + xc) *
                                                       g.c + c0);
    }
#pragma unroll
    for (int w = 0; w < 9; ++w) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t word = raw[w][p];
        const f32x2 a = {__uint_as_float(word << 16), __uint_as_float(word & 0xffff0000u)};
        const f32x2 s = __builtin_elementwise_fma(a, sc2[p], sh2[p]);
        const s16x2 v = __builtin_elementwise_max(
            __builtin_bit_cast(s16x2, __builtin_convertvector(s, bf16x2)), (s16x2){0, 0});
        const uint32_t pk = __builtin_bit_cast(uint32_t, v);
        const uint32_t k0 = (pk << 16) | tag[w], k1 = (pk & 0xffff0000u) | tag[w];
        if (k0 > key[2 * p]) { key[2 * p] = k0; rb[2 * p] = word; }
        if (k1 > key[2 * p + 1]) { key[2 * p + 1] = k1; rb[2 * p + 1] = word; }
      }
    }
  }
  u32x4 o, r;
  uint64_t packed = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    o[p] = (key[2 * p] >> 16) | (key[2 * p + 1] & 0xffff0000u);
    r[p] = (rb[2 * p] & 0xffffu) | (rb[2 * p + 1] & 0xffff0000u);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t vb = key[e] >> 16;            // bf16 bits, sign clear
    const bool pos = vb != 0 && vb <= 0x7f80u;   // > 0 and not NaN: ReLU passed it
    packed |= (uint64_t)((31 - (key[e] & 31)) | (pos ? 0x80 : 0)) << (8 * e);
  }
  *reinterpret_cast<u32x4*>(out + ovox * g.c + c0) = o;
  *reinterpret_cast<u32x4*>(ymax + ovox * g.c + c0) = r;
  *reinterpret_cast<uint64_t*>(am + ovox * g.c + c0) = packed;
}

// Same, one block per output row (blockIdx.y = oh, blockIdx.z = n*do + od) when the
// channel-vector count is a power of two: the per-thread index math is a shift and a mask
// instead of five 64-bit divisions (which, at 8 channels per thread, cost more VALU time
// than the kernel's memory traffic).
template <typename T, int V>
__global__ __launch_bounds__(256) void bnpool3_fwd_rows_kernel(
    PoolG g, int cv_shift, const T* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, T* __restrict__ out, uint8_t* __restrict__ am,
    T* __restrict__ ymax) {
  const int oh = blockIdx.y, od = blockIdx.z % g.do_;
  const int64_t nb = blockIdx.z / g.do_;
  const int items = g.wo << cv_shift, cmask = (1 << cv_shift) - 1;
  // cv divides 256: this thread's channel vector is the same for every item it visits
  const int c0 = (threadIdx.x & cmask) * V;
  if constexpr (sizeof(T) == 2 && V == 8) {
    f32x2 sc2[4], sh2[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      sc2[p] = (f32x2){scale[c0 + 2 * p], scale[c0 + 2 * p + 1]};
      sh2[p] = (f32x2){shift[c0 + 2 * p], shift[c0 + 2 * p + 1]};
    }
    for (int e = threadIdx.x; e < items; e += 256)
      bnpool3_fwd_one_bf16(g, y, out, am, ymax, nb, od, oh, e >> cv_shift, c0, sc2, sh2);
  } else {
    float sc[V], sh[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { sc[e] = scale[c0 + e]; sh[e] = shift[c0 + e]; }
    for (int e = threadIdx.x; e < items; e += 256)
      bnpool3_fwd_one<T, V>(g, y, scale, shift, out, am, ymax, nb, od, oh, e >> cv_shift, c0, sc,
                            sh);
  }
}

// k = 3, stride 2, pad 1 form of bnpool_bwd_apply_kernel, one thread per 2x2x2 input cell
// {2a, 2a+1}^3: input 2a lies only in window a, input 2a+1 in windows a and a+1, so the
// cell's 8 inputs share the 8 windows {a, a+1}^3, loaded once (not ~3.4x per input).  All
// 24 loads of a cell are issued before any use (raw 16-byte registers), so a thread waits
// for one memory round trip, not eight.
// Per-thread BN-backward constants of channels c0..c0+V-1:
// dy = k0 * g' - k1 - (y - mu) * kt, with kt = invstd * coef2
template <int V>
__device__ __forceinline__ void bnbwd_params(int C, int c0, const float* __restrict__ mean,
                                             const float* __restrict__ invstd,
                                             const float* __restrict__ coef, float* mu,
                                             float* k0, float* k1, float* kt) {
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = c0 + e;
    mu[e] = mean[c];
    k0[e] = coef[c]; k1[e] = coef[C + c]; kt[e] = invstd[c] * coef[2 * C + c];
  }
}

// V elements of T held packed in 32-bit words (V * sizeof(T) = 8 or 16 bytes)
template <typename T, int V>
struct Packed {
  static constexpr int W = V * (int)sizeof(T) / 4;
  uint32_t w[W];
  __device__ __forceinline__ void load(const T* p) {
    if constexpr (W == 4) {
      const u32x4 c = *reinterpret_cast<const u32x4*>(p);
      w[0] = c[0]; w[1] = c[1]; w[2] = c[2]; w[3] = c[3];
    } else {
      const uint2 c = *reinterpret_cast<const uint2*>(p);
      w[0] = c.x; w[1] = c.y;
    }
  }
  __device__ __forceinline__ float get(int e) const {
    if constexpr (sizeof(T) == 4) return __uint_as_float(w[e]);
    else return __uint_as_float((e & 1) ? (w[e >> 1] & 0xffff0000u) : (w[e >> 1] << 16));
  }
};

template <typename T, int V>
__device__ __forceinline__ void store_packed(T* p, const float* v) {
  if constexpr (sizeof(T) == 4 && V == 4) {
    f32x4 c; c[0] = v[0]; c[1] = v[1]; c[2] = v[2]; c[3] = v[3];
    *reinterpret_cast<f32x4*>(p) = c;
  } else if constexpr (V == 8) {
    u32x4 c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
    *reinterpret_cast<u32x4*>(p) = c;
  } else {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
}

// V = 4 channels per thread in both dtypes (8-byte bf16 / 16-byte fp32 accesses): the 8
// windows' argmax bytes, pooled gradients and the cell's 8 inputs stay packed, so the cell
// fits in ~100 VGPRs (4+ waves per SIMD; 8 bf16 channels per thread needed 247)
template <typename T, int V>
__device__ __forceinline__ void bnpool3s2_bwd_cell(
    const PoolG& g, const T* __restrict__ gp, const uint8_t* __restrict__ am,
    const T* __restrict__ y, T* __restrict__ dy, int64_t nb, int ad, int ah, int aw, int c0,
    const float* mu, const float* k0, const float* k1, const float* kt) {
  static_assert(V == 4, "argmax bytes are read as one 32-bit word");
  uint32_t a4[8];
  Packed<T, V> graw[8], yraw[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int qd = q >> 2, qh = (q >> 1) & 1, qw = q & 1;
    const bool ok = ad + qd < g.do_ && ah + qh < g.ho && aw + qw < g.wo;
    const int od = min(ad + qd, g.do_ - 1), oh = min(ah + qh, g.ho - 1);
    const int ow = min(aw + qw, g.wo - 1);
    const int64_t o = (((nb * g.do_ + od) * g.ho + oh) * g.wo + ow) * g.c + c0;
    const uint32_t w = *reinterpret_cast<const uint32_t*>(am + o);
    a4[q] = ok ? w : 0;          // 0: no active window (the 0x80 bit is never set)
    graw[q].load(gp + o);
    const int id = min(2 * ad + qd, g.di - 1), ih = min(2 * ah + qh, g.hi - 1);
    const int iw = min(2 * aw + qw, g.wi - 1);
    yraw[q].load(y + (((nb * g.di + id) * g.hi + ih) * g.wi + iw) * g.c + c0);
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int rd = r >> 2, rh = (r >> 1) & 1, rw = r & 1;
    const int id = 2 * ad + rd, ih = 2 * ah + rh, iw = 2 * aw + rw;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int qd = q >> 2, qh = (q >> 1) & 1, qw = q & 1;
      // an even input (r-bit 0) lies only in window a (q-bit 0); offset inside window
      // a+q: (i - 2a) + 1 - 2q
      if ((!rd && qd) || (!rh && qh) || (!rw && qw)) continue;
      const uint32_t wi = 0x80 | (((rd + 1 - 2 * qd) * 3 + (rh + 1 - 2 * qh)) * 3 + (rw + 1 - 2 * qw));
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (((a4[q] >> (8 * e)) & 0xff) == wi) acc[e] += graw[q].get(e);
    }
    if (id >= g.di || ih >= g.hi || iw >= g.wi) continue;
    float dv[V];
#pragma unroll
    for (int e = 0; e < V; ++e) dv[e] = k0[e] * acc[e] - k1[e] - (yraw[r].get(e) - mu[e]) * kt[e];
    store_packed<T, V>(dy + (((nb * g.di + id) * g.hi + ih) * g.wi + iw) * g.c + c0, dv);
  }
}

template <typename T, int V>
__global__ __launch_bounds__(256) void bnpool3s2_bwd_apply_kernel(
    PoolG g, const T* __restrict__ gp, const uint8_t* __restrict__ am, const T* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, T* __restrict__ dy) {
  const int cv = g.c / V;
  const int cd = (g.di + 1) >> 1, ch = (g.hi + 1) >> 1, cw = (g.wi + 1) >> 1;
  const int64_t total = (int64_t)g.n * cd * ch * cw * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int aw = (int)(v % cw); v /= cw;
    const int ah = (int)(v % ch); v /= ch;
    const int ad = (int)(v % cd);
    float mu[V], k0[V], k1[V], kt[V];
    bnbwd_params<V>(g.c, c0, mean, invstd, coef, mu, k0, k1, kt);
    bnpool3s2_bwd_cell<T, V>(g, gp, am, y, dy, v / cd, ad, ah, aw, c0, mu, k0, k1, kt);
  }
}

// Same, one block per row of cells (blockIdx.y = ah, blockIdx.z = n*cd + ad), power-of-two
// channel-vector count: shift/mask index math (see bnpool3_fwd_rows_kernel).
template <typename T, int V>
__global__ __launch_bounds__(256) void bnpool3s2_bwd_rows_kernel(
    PoolG g, int cv_shift, const T* __restrict__ gp, const uint8_t* __restrict__ am,
    const T* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, T* __restrict__ dy) {
  const int cd = (g.di + 1) >> 1, cw = (g.wi + 1) >> 1;
  const int ah = blockIdx.y, ad = blockIdx.z % cd;
  const int64_t nb = blockIdx.z / cd;
  const int items = cw << cv_shift, cmask = (1 << cv_shift) - 1;
  const int c0 = (threadIdx.x & cmask) * V;      // fixed per thread (cv divides 256)
  float mu[V], k0[V], k1[V], kt[V];
  bnbwd_params<V>(g.c, c0, mean, invstd, coef, mu, k0, k1, kt);
  for (int e = threadIdx.x; e < items; e += 256)
    bnpool3s2_bwd_cell<T, V>(g, gp, am, y, dy, nb, ad, ah, e >> cv_shift, c0, mu, k0, k1, kt);
}

// Fused backward, dense pass: for every input voxel, g' = sum of the pooled gradients of the
// windows whose argmax it is (and whose max passed the ReLU), then the BN input gradient
// dy = coef0 * g' - coef1 - xhat * coef2 (coef from the pooled-grid reduction).
template <typename T, int V>
__global__ void bnpool_bwd_apply_kernel(PoolG g, const T* __restrict__ gp,
                                        const uint8_t* __restrict__ am, const T* __restrict__ y,
                                        const float* __restrict__ mean,
                                        const float* __restrict__ invstd,
                                        const float* __restrict__ coef, T* __restrict__ dy) {
  const int cv = g.c / V;
  const int64_t total = (int64_t)g.n * g.di * g.hi * g.wi * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    int64_t v = t / cv;
    const int64_t ivox = v;
    const int iw = (int)(v % g.wi); v /= g.wi;
    const int ih = (int)(v % g.hi); v /= g.hi;
    const int id = (int)(v % g.di);
    const int64_t nb = v / g.di;
    auto lo = [&](int ii) { int q = ii + g.p - (g.k - 1); return q <= 0 ? 0 : (q + g.s - 1) / g.s; };
    auto hi = [&](int ii, int lim) { int q = (ii + g.p) / g.s; return q < lim - 1 ? q : lim - 1; };
    const int d0 = lo(id), d1 = hi(id, g.do_);
    const int h0 = lo(ih), h1 = hi(ih, g.ho);
    const int w0 = lo(iw), w1 = hi(iw, g.wo);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int od = d0; od <= d1; ++od)
      for (int oh = h0; oh <= h1; ++oh)
        for (int ow = w0; ow <= w1; ++ow) {
          const int wi = 0x80 | (((id - (od * g.s - g.p)) * g.k + (ih - (oh * g.s - g.p))) * g.k +
                                 (iw - (ow * g.s - g.p)));
          const int64_t o = (((nb * g.do_ + od) * g.ho + oh) * g.wo + ow) * g.c + c0;
          uint8_t a[V];
          if constexpr (V == 8) {
            const uint64_t w = *reinterpret_cast<const uint64_t*>(am + o);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = (uint8_t)(w >> (8 * e));
          } else if constexpr (V == 4) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(am + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) a[e] = (uint8_t)(w >> (8 * e));
          } else {
            for (int e = 0; e < V; ++e) a[e] = am[o + e];
          }
          bool any = false;
#pragma unroll
          for (int e = 0; e < V; ++e) any |= a[e] == wi;
          if (!any) continue;
          float gv[V];
          load_v<T, V>(gp + o, gv);
#pragma unroll
          for (int e = 0; e < V; ++e)
            if (a[e] == wi) acc[e] += gv[e];
        }
    float yv[V], dv[V];
    load_v<T, V>(y + ivox * g.c + c0, yv);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int c = c0 + e;
      const float xh = (yv[e] - mean[c]) * invstd[c];
      dv[e] = coef[c] * acc[e] - coef[g.c + c] - xh * coef[2 * g.c + c];
    }
    store_v<T, V>(dy + ivox * g.c + c0, dv);
  }
}

// GAP: one block per (n, channel chunk of up to 256); V channels per thread,
// 256 / (chunk / V) voxel lanes; fp32 partial sums folded through LDS.
template <typename T, int V>
__global__ __launch_bounds__(1024) void gap_fwd_kernel(int64_t S, int C, int CB,
                                                      const T* __restrict__ x,
                                                      float* __restrict__ y) {
  __shared__ float red[1024 * 8];
  const int n = blockIdx.y;
  // blockIdx.z > 0 (gridDim.z = P partitions): this block sums voxel slab z of P and
  // writes raw partial sums to y[(n*P + z)*C + c] (no division); see gap_fold_kernel
  const int P = gridDim.z, part = blockIdx.z;
  const int64_t v0 = S * part / P, v1 = S * (part + 1) / P;
  const int cb0 = blockIdx.x * CB;
  const int cw = min(CB, C - cb0);
  const int lpr = cw / V;
  const int rpar = (int)blockDim.x / lpr;
  const int cl = threadIdx.x % lpr, rl = threadIdx.x / lpr;
  float s[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = 0.f;
  if (rl < rpar) {
    for (int64_t v = v0 + rl; v < v1; v += rpar) {
      float val[V];
      load_v<T, V>(x + ((int64_t)n * S + v) * C + cb0 + cl * V, val);
#pragma unroll
      for (int e = 0; e < V; ++e) s[e] += val[e];
    }
#pragma unroll
    for (int e = 0; e < V; ++e) red[rl * cw + cl * V + e] = s[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cw; c += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < rpar; ++k) acc += red[k * cw + c];
    if (P == 1) y[(int64_t)n * C + cb0 + c] = acc / (float)S;
    else y[((int64_t)n * P + part) * C + cb0 + c] = acc;
  }
}

// second level of the partitioned GAP: y[n][c] = (sum over p, in order, of ws[n][p][c]) / S
__global__ void gap_fold_kernel(int n, int P, int C, int64_t S, const float* __restrict__ ws,
                                float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * C) return;
  const int64_t b = i / C, c = i % C;
  float acc = 0.f;
  // (unrolled so the P partial loads are in flight together; the sum order is unchanged)
#pragma unroll 16
  for (int p = 0; p < P; ++p) acc += ws[(b * P + p) * C + c];
  y[i] = acc / (float)S;
}

template <typename T, int V>
__global__ void gap_bwd_kernel(int n, int64_t S, int C, float inv, const float* __restrict__ dy,
                               T* __restrict__ dx) {
  const int cv = C / V;
  const int64_t total = (int64_t)n * S * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(t % cv) * V;
    const int64_t nb = t / ((int64_t)S * cv);
    float v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = dy[nb * C + c0 + e] * inv;
    store_v<T, V>(dx + (t / cv) * C + c0, v);
  }
}

// k = 3, stride 2, pad 1, bf16 (the MedicalNet stem pool, BN + ReLU fused): a block owns
// one output row (n, oh) of a z segment and walks it along z.  The 3 x 3 (y, x) max of input
// plane p is computed once and serves both outputs that read the plane (od = p / 2 and
// (p + 1) / 2): per output 18 window elements are loaded and transformed instead of 27 (the
// rows kernel ran VALU-bound: r03y counters, 85 % of its cycles issuing VALU).  Keys and tie
// order as bnpool3_fwd_one_bf16 (value << 16 | 31 - window index, the index composed as
// plane part + 9 * kd, windows clipped at the borders), so out / argmax / ymax are
// bit-identical to the rows kernel's.  Thread = (output x, 8-channel vector).
struct PlaneMax {
  uint32_t key[8], rb[8];
};
// (window loads through the sample's buffer resource: the plane's byte offset is a scalar,
// the thread's 9 in-plane byte offsets `wofs` are fixed for its whole z walk -- no per-load
// 64-bit address arithmetic in this VALU-bound loop)
__device__ __forceinline__ void plane_max(const PoolG& g, __amdgpu_buffer_rsrc_t rs,
                                          uint32_t plane_off, const uint32_t (&wofs)[9], int y0,
                                          int x0, const f32x2* sc2, const f32x2* sh2,
                                          PlaneMax& m) {
#pragma unroll
  for (int e = 0; e < 8; ++e) { m.key[e] = 0; m.rb[e] = 0; }
  u32x4 raw[9];
  uint32_t tag[9];
#pragma unroll
  for (int w = 0; w < 9; ++w) {
    const int yc = min(max(y0 + w / 3, 0), g.hi - 1), xc = min(max(x0 + w % 3, 0), g.wi - 1);
    tag[w] = 31 - 18 - ((yc - y0) * 3 + (xc - x0));     // kd = 2 part; + 9 (2 - kd) later
    raw[w] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rs, wofs[w], __builtin_amdgcn_readfirstlane(plane_off), 0));
  }
#pragma unroll
  for (int w = 0; w < 9; ++w) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t word = raw[w][q];
      const f32x2 a = {__uint_as_float(word << 16), __uint_as_float(word & 0xffff0000u)};
      const f32x2 sv = __builtin_elementwise_fma(a, sc2[q], sh2[q]);
      const s16x2 v = __builtin_elementwise_max(
          __builtin_bit_cast(s16x2, __builtin_convertvector(sv, bf16x2)), (s16x2){0, 0});
      const uint32_t pk = __builtin_bit_cast(uint32_t, v);
      const uint32_t k0 = (pk << 16) | tag[w], k1 = (pk & 0xffff0000u) | tag[w];
      if (k0 > m.key[2 * q]) { m.key[2 * q] = k0; m.rb[2 * q] = word; }
      if (k1 > m.key[2 * q + 1]) { m.key[2 * q + 1] = k1; m.rb[2 * q + 1] = word; }
    }
  }
}
__device__ __forceinline__ void zmerge(PlaneMax& best, const PlaneMax& m, uint32_t add) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t k = m.key[e] + add;
    if (k > best.key[e]) { best.key[e] = k; best.rb[e] = m.rb[e]; }
  }
}

#ifndef POOL_ZW_WAVES
#define POOL_ZW_WAVES 1
#endif
#ifndef POOL_ZW_ODS
#define POOL_ZW_ODS 4
#endif
__global__ __launch_bounds__(256, POOL_ZW_WAVES) void bnpool3s2_fwd_zwalk_kernel(
    PoolG g, int cv_shift, int ods, const u16* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, u16* __restrict__ out, uint8_t* __restrict__ am,
    u16* __restrict__ ymax) {
  const int cvn = 1 << cv_shift;
  const int ow = threadIdx.x >> cv_shift, c0 = (threadIdx.x & (cvn - 1)) * 8;
  if (ow >= g.wo) return;                          // (no barrier in this kernel)
  const int oh = blockIdx.y;
  const int64_t nb = blockIdx.z;
  const int od0 = blockIdx.x * ods, od1 = min(g.do_, od0 + ods);
  f32x2 sc2[4], sh2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    sc2[q] = (f32x2){scale[c0 + 2 * q], scale[c0 + 2 * q + 1]};
    sh2[q] = (f32x2){shift[c0 + 2 * q], shift[c0 + 2 * q + 1]};
  }
  const int y0 = 2 * oh - 1, x0 = 2 * ow - 1;
  const int64_t plane = (int64_t)g.hi * g.wi * g.c;
  const uint32_t pbytes = (uint32_t)(plane * 2);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(y + nb * g.di * plane), 0, (int)__builtin_amdgcn_readfirstlane(pbytes * g.di),
      0x00020000);
  uint32_t wofs[9];
#pragma unroll
  for (int w = 0; w < 9; ++w) {
    const int yc = min(max(y0 + w / 3, 0), g.hi - 1), xc = min(max(x0 + w % 3, 0), g.wi - 1);
    wofs[w] = (uint32_t)((yc * g.wi + xc) * g.c + c0) * 2u;
  }
  PlaneMax prev;                                   // plane 2 od - 1 (the previous od's last)
  bool prev_ok = 2 * od0 - 1 >= 0;
  if (prev_ok) plane_max(g, rs, (uint32_t)(2 * od0 - 1) * pbytes, wofs, y0, x0, sc2, sh2, prev);
  for (int od = od0; od < od1; ++od) {
    PlaneMax a, b;
    plane_max(g, rs, (uint32_t)(2 * od) * pbytes, wofs, y0, x0, sc2, sh2, a);
    const bool b_ok = 2 * od + 1 < g.di;
    if (b_ok) plane_max(g, rs, (uint32_t)(2 * od + 1) * pbytes, wofs, y0, x0, sc2, sh2, b);
    PlaneMax best;                                 // kd = 1: always inside the volume
#pragma unroll
    for (int e = 0; e < 8; ++e) { best.key[e] = a.key[e] + 9; best.rb[e] = a.rb[e]; }
    if (prev_ok) zmerge(best, prev, 18);           // kd = 0
    if (b_ok) zmerge(best, b, 0);                  // kd = 2
    const int64_t ovox = ((nb * g.do_ + od) * g.ho + oh) * g.wo + ow;
    u32x4 o, r;
    uint64_t packed = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = (best.key[2 * q] >> 16) | (best.key[2 * q + 1] & 0xffff0000u);
      r[q] = (best.rb[2 * q] & 0xffffu) | (best.rb[2 * q + 1] & 0xffff0000u);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t vb = best.key[e] >> 16;
      const bool pos = vb != 0 && vb <= 0x7f80u;
      packed |= (uint64_t)((31 - (best.key[e] & 31)) | (pos ? 0x80 : 0)) << (8 * e);
    }
    *reinterpret_cast<u32x4*>(out + ovox * g.c + c0) = o;
    *reinterpret_cast<u32x4*>(ymax + ovox * g.c + c0) = r;
    *reinterpret_cast<uint64_t*>(am + ovox * g.c + c0) = packed;
    prev = b;
    prev_ok = b_ok;
  }
}

// MMAD_POOL_ROWS=0 keeps the grid-stride fused pool kernels (A/B switch)
bool rows_on() {
  static const bool v = [] { const char* e = getenv("MMAD_POOL_ROWS"); return !e || atoi(e) != 0; }();
  return v;
}

// MMAD_POOL_RUN: 2 (default) the z-walking bnpool3s2_fwd_zwalk_kernel for the stem pool (k 3,
// s 2, p 1, bf16), any other value the per-output rows kernel; mmad_set_kernel_variant(
// "pool_run", v).  (A column-carrying form -- each thread walking a run of outputs along x --
// measured 124.5 us against the rows kernel's 110.8 at config 2, r03e: its 2 waves per SIMD
// did not keep enough loads in flight; removed.)
std::atomic<int> g_pool_run{-1};
int pool_run_mode() {
  int v = g_pool_run.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_POOL_RUN");
    int expect = -1;
    g_pool_run.compare_exchange_strong(expect, e ? atoi(e) : 2);
    v = g_pool_run.load(std::memory_order_relaxed);
  }
  return v;
}

unsigned grid_of(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 256 * 32));
}

bool pool_ok(const PoolG& g) {
  if (g.n <= 0 || g.c <= 0 || g.di <= 0 || g.hi <= 0 || g.wi <= 0 || g.k <= 0 || g.s <= 0 ||
      g.p < 0 || g.k * g.k * g.k > 255 || 2 * g.p > g.k)
    return false;
  auto ext = [&](int i) { return (i + 2 * g.p - g.k) / g.s + 1; };
  return ext(g.di) == g.do_ && ext(g.hi) == g.ho && ext(g.wi) == g.wo;
}

template <typename T>
int pool_fwd(const PoolG& g, const void* x, void* y, uint8_t* am, hipStream_t st) {
  constexpr int VEC = Chunk<T>::N;
  const int64_t vox = (int64_t)g.n * g.do_ * g.ho * g.wo;
  if (g.c % VEC == 0)
    hipLaunchKernelGGL((maxpool_fwd_kernel<T, VEC>), dim3(grid_of(vox * g.c / VEC)), dim3(256),
                       0, st, g, (const T*)x, (T*)y, am);
  else
    hipLaunchKernelGGL((maxpool_fwd_kernel<T, 1>), dim3(grid_of(vox * g.c)), dim3(256), 0, st,
                       g, (const T*)x, (T*)y, am);
  return launch_status();
}

template <typename T>
int pool_bwd(const PoolG& g, const void* dy, const uint8_t* am, void* dx, hipStream_t st) {
  constexpr int VEC = Chunk<T>::N;
  const int64_t vox = (int64_t)g.n * g.di * g.hi * g.wi;
  if (g.c % VEC == 0)
    hipLaunchKernelGGL((maxpool_bwd_kernel<T, VEC>), dim3(grid_of(vox * g.c / VEC)), dim3(256),
                       0, st, g, (const T*)dy, am, (T*)dx);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<T, 1>), dim3(grid_of(vox * g.c)), dim3(256), 0, st,
                       g, (const T*)dy, am, (T*)dx);
  return launch_status();
}

template <typename T>
int bnpool_fwd(const PoolG& g, const void* y, const float* scale, const float* shift, void* out,
               uint8_t* am, void* ymax, hipStream_t st) {
  constexpr int VEC = Chunk<T>::N;
  const int64_t vox = (int64_t)g.n * g.do_ * g.ho * g.wo;
  const int cv = g.c / VEC;
  if constexpr (sizeof(T) == 2) {
    if (g.c % VEC == 0 && g.k == 3 && g.s == 2 && g.p == 1 && is_pow2(cv) &&
        pool_run_mode() == 2 && cv * g.wo <= 256 && g.ho < 65536 && g.n < 65536 &&
        (int64_t)g.di * g.hi * g.wi * g.c * 2 < (int64_t(1) << 31)) {   // (32-bit offsets)
      // z segments of 4 outputs (one extra plane each): >= 8 blocks per CU at the stem
      const int ods = POOL_ZW_ODS;
      hipLaunchKernelGGL(bnpool3s2_fwd_zwalk_kernel,
                         dim3((unsigned)cdiv(g.do_, ods), (unsigned)g.ho, (unsigned)g.n),
                         dim3(256), 0, st, g, ilog2(cv), ods, (const u16*)y, scale, shift,
                         (u16*)out, am, (u16*)ymax);
      return launch_status();
    }
  }
  if (g.c % VEC == 0 && g.k == 3 && is_pow2(cv) && rows_on() &&
      (int64_t)g.n * g.do_ < 65536 && g.ho < 65536)
    hipLaunchKernelGGL((bnpool3_fwd_rows_kernel<T, VEC>),
                       dim3(1, (unsigned)g.ho, (unsigned)(g.n * g.do_)), dim3(256), 0, st, g,
                       ilog2(cv), (const T*)y, scale, shift, (T*)out, am, (T*)ymax);
  else if (g.c % VEC == 0 && g.k == 3)
    hipLaunchKernelGGL((bnpool3_fwd_kernel<T, VEC>), dim3(grid_of(vox * g.c / VEC)), dim3(256),
                       0, st, g, (const T*)y, scale, shift, (T*)out, am, (T*)ymax);
  else if (g.c % VEC == 0)
    hipLaunchKernelGGL((bnpool_fwd_kernel<T, VEC>), dim3(grid_of(vox * g.c / VEC)), dim3(256),
                       0, st, g, (const T*)y, scale, shift, (T*)out, am, (T*)ymax);
  else
    hipLaunchKernelGGL((bnpool_fwd_kernel<T, 1>), dim3(grid_of(vox * g.c)), dim3(256), 0, st, g,
                       (const T*)y, scale, shift, (T*)out, am, (T*)ymax);
  return launch_status();
}

template <typename T>
int bnpool_bwd_apply(const PoolG& g, const void* gp, const uint8_t* am, const void* y,
                     const float* mean, const float* invstd, const float* coef, void* dy,
                     hipStream_t st) {
  constexpr int VEC = Chunk<T>::N;
  const int64_t vox = (int64_t)g.n * g.di * g.hi * g.wi;
  const int cd = (g.di + 1) >> 1, ch = (g.hi + 1) >> 1;
  const int cv4 = g.c / 4;   // the k3 s2 cell kernels take 4 channels per thread
  if (g.c % 4 == 0 && g.k == 3 && g.s == 2 && g.p == 1 && is_pow2(cv4) && cv4 <= 256 &&
      rows_on() && (int64_t)g.n * cd < 65536 && ch < 65536)
    hipLaunchKernelGGL((bnpool3s2_bwd_rows_kernel<T, 4>),
                       dim3(1, (unsigned)ch, (unsigned)(g.n * cd)), dim3(256), 0, st, g,
                       ilog2(cv4), (const T*)gp, am, (const T*)y, mean, invstd, coef, (T*)dy);
  else if (g.c % 4 == 0 && g.k == 3 && g.s == 2 && g.p == 1)
    hipLaunchKernelGGL((bnpool3s2_bwd_apply_kernel<T, 4>), dim3(grid_of(vox * g.c / 4 / 8 + 1)),
                       dim3(256), 0, st, g, (const T*)gp, am, (const T*)y, mean, invstd, coef,
                       (T*)dy);
  else if (g.c % VEC == 0)
    hipLaunchKernelGGL((bnpool_bwd_apply_kernel<T, VEC>), dim3(grid_of(vox * g.c / VEC)),
                       dim3(256), 0, st, g, (const T*)gp, am, (const T*)y, mean, invstd, coef,
                       (T*)dy);
  else
    hipLaunchKernelGGL((bnpool_bwd_apply_kernel<T, 1>), dim3(grid_of(vox * g.c)), dim3(256), 0,
                       st, g, (const T*)gp, am, (const T*)y, mean, invstd, coef, (T*)dy);
  return launch_status();
}

// voxel-slab partitions so a (n, channel-chunk) grid of a few blocks becomes >= 512 blocks
int gap_parts(int n, int64_t s, int c) {
  const int64_t blocks = (int64_t)n * cdiv(c, std::min(c, 256));
  int64_t p = cdiv(512, blocks);
  p = std::min<int64_t>(p, std::max<int64_t>(1, s / 64));
  return (int)std::max<int64_t>(1, std::min<int64_t>(p, 1024));
}

template <typename T>
int gap_fwd(int n, int64_t s, int c, const void* x, float* y, hipStream_t st, float* ws = nullptr,
            int P = 1) {
  constexpr int VEC = Chunk<T>::N;
  if (ws != nullptr && P > 1 && c % VEC == 0) {
    const int cb = std::min(c, 256);
    if (cb % VEC) return MMAD_EUNSUPPORTED;
    hipLaunchKernelGGL((gap_fwd_kernel<T, VEC>), dim3((unsigned)cdiv(c, cb), (unsigned)n,
                       (unsigned)P), dim3(1024), 0, st, s, c, cb, (const T*)x, ws);
    hipLaunchKernelGGL(gap_fold_kernel, dim3((unsigned)cdiv((int64_t)n * c, 256)), dim3(256), 0, st,
                       n, P, c, s, ws, y);
    return launch_status();
  }
  if (c % VEC == 0) {
    const int cb = std::min(c, 256);
    if (cb % VEC) return MMAD_EUNSUPPORTED;
    hipLaunchKernelGGL((gap_fwd_kernel<T, VEC>), dim3((unsigned)cdiv(c, cb), (unsigned)n),
                       dim3(1024), 0, st, s, c, cb, (const T*)x, y);
  } else {
    const int cb = std::min(c, 1024);
    hipLaunchKernelGGL((gap_fwd_kernel<T, 1>), dim3((unsigned)cdiv(c, cb), (unsigned)n),
                       dim3(1024), 0, st, s, c, cb, (const T*)x, y);
  }
  return launch_status();
}

// dx = dy / s broadcast over s rows per sample; compact: one row per sample (the (n, c)
// values a broadcast-gradient consumer expands itself, see mmad_bn_bwd_reduce2)
template <typename T>
int gap_bwd(int n, int64_t s, int c, const float* dy, void* dx, hipStream_t st,
            bool compact = false) {
  constexpr int VEC = Chunk<T>::N;
  const float inv = 1.f / (float)s;
  const int64_t rows = compact ? 1 : s;
  const int64_t tot = (int64_t)n * rows * c;
  if (c % VEC == 0)
    hipLaunchKernelGGL((gap_bwd_kernel<T, VEC>), dim3(grid_of(tot / VEC)), dim3(256), 0, st, n,
                       rows, c, inv, dy, (T*)dx);
  else
    hipLaunchKernelGGL((gap_bwd_kernel<T, 1>), dim3(grid_of(tot)), dim3(256), 0, st, n, rows, c,
                       inv, dy, (T*)dx);
  return launch_status();
}

}  // namespace

extern "C" {

int mmad_maxpool3d_fwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                       int k, int s, int p, const void* x, void* y, uint8_t* argmax,
                       void* stream) {
  PoolG g{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(g)) return MMAD_EBADSHAPE;
  if (!x || !y || !argmax) return MMAD_ENULL;
  if (dtype == MMAD_BF16) return pool_fwd<u16>(g, x, y, argmax, as_stream(stream));
  if (dtype == MMAD_F32) return pool_fwd<float>(g, x, y, argmax, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int mmad_maxpool3d_bwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                       int k, int s, int p, const void* dy, const uint8_t* argmax, void* dx,
                       void* stream) {
  PoolG g{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(g)) return MMAD_EBADSHAPE;
  if (!dy || !dx || !argmax) return MMAD_ENULL;
  if (dtype == MMAD_BF16) return pool_bwd<u16>(g, dy, argmax, dx, as_stream(stream));
  if (dtype == MMAD_F32) return pool_bwd<float>(g, dy, argmax, dx, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int mmad_bnpool_fwd(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho, int wo,
                    int k, int s, int p, const void* y, const float* scale, const float* shift,
                    void* out, uint8_t* argmax, void* ymax, void* stream) {
  PoolG g{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(g) || k * k * k > 127) return MMAD_EBADSHAPE;
  if (!y || !scale || !shift || !out || !argmax || !ymax) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return bnpool_fwd<u16>(g, y, scale, shift, out, argmax, ymax, as_stream(stream));
  if (dtype == MMAD_F32)
    return bnpool_fwd<float>(g, y, scale, shift, out, argmax, ymax, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int mmad_bnpool_bwd_apply(int dtype, int n, int c, int di, int hi, int wi, int do_, int ho,
                          int wo, int k, int s, int p, const void* g, const uint8_t* argmax,
                          const void* y, const float* mean, const float* invstd,
                          const float* coef, void* dy, void* stream) {
  PoolG pg{n, c, di, hi, wi, do_, ho, wo, k, s, p};
  if (!pool_ok(pg) || k * k * k > 127) return MMAD_EBADSHAPE;
  if (!g || !argmax || !y || !mean || !invstd || !coef || !dy) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return bnpool_bwd_apply<u16>(pg, g, argmax, y, mean, invstd, coef, dy, as_stream(stream));
  if (dtype == MMAD_F32)
    return bnpool_bwd_apply<float>(pg, g, argmax, y, mean, invstd, coef, dy, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int mmad_gap_fwd(int dtype, int n, int64_t s, int c, const void* x, float* y, void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!x || !y) return MMAD_ENULL;
  if (dtype == MMAD_BF16) return gap_fwd<u16>(n, s, c, x, y, as_stream(stream));
  if (dtype == MMAD_F32) return gap_fwd<float>(n, s, c, x, y, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int64_t mmad_gap_fwd_ws_elems(int n, int64_t s, int c) {
  if (n <= 0 || s <= 0 || c <= 0) return -1;
  return (int64_t)n * gap_parts(n, s, c) * c;
}

int mmad_gap_fwd_ws(int dtype, int n, int64_t s, int c, const void* x, float* y, float* ws,
                    void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!x || !y || !ws) return MMAD_ENULL;
  const int P = gap_parts(n, s, c);
  if (dtype == MMAD_BF16) return gap_fwd<u16>(n, s, c, x, y, as_stream(stream), ws, P);
  if (dtype == MMAD_F32) return gap_fwd<float>(n, s, c, x, y, as_stream(stream), ws, P);
  return MMAD_EBADDTYPE;
}

int mmad_gap_parts(int n, int64_t s, int c) {
  if (n <= 0 || s <= 0 || c <= 0) return -1;
  return gap_parts(n, s, c);
}

// the first level of mmad_gap_fwd_ws only: ws[n][P][c] raw partial sums (P = mmad_gap_parts
// > 1), or the pooled means ws[n][c] when P == 1; mmad_gap_linear_fwd folds them
int mmad_gap_partial(int dtype, int n, int64_t s, int c, const void* x, float* ws,
                     void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!x || !ws) return MMAD_ENULL;
  const int P = gap_parts(n, s, c);
  const int cb = std::min(c, 256);
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16 && c % Chunk<u16>::N == 0 && cb % Chunk<u16>::N == 0)
    hipLaunchKernelGGL((gap_fwd_kernel<u16, Chunk<u16>::N>), dim3((unsigned)cdiv(c, cb),
                       (unsigned)n, (unsigned)P), dim3(1024), 0, st, s, c, cb, (const u16*)x, ws);
  else if (dtype == MMAD_F32 && c % Chunk<float>::N == 0 && cb % Chunk<float>::N == 0)
    hipLaunchKernelGGL((gap_fwd_kernel<float, Chunk<float>::N>), dim3((unsigned)cdiv(c, cb),
                       (unsigned)n, (unsigned)P), dim3(1024), 0, st, s, c, cb, (const float*)x,
                       ws);
  else
    return MMAD_EUNSUPPORTED;
  return launch_status();
}

int mmad_gap_bwd(int dtype, int n, int64_t s, int c, const float* dy, void* dx, void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!dy || !dx) return MMAD_ENULL;
  if (dtype == MMAD_BF16) return gap_bwd<u16>(n, s, c, dy, dx, as_stream(stream));
  if (dtype == MMAD_F32) return gap_bwd<float>(n, s, c, dy, dx, as_stream(stream));
  return MMAD_EBADDTYPE;
}

int mmad_gap_bwd_compact(int dtype, int n, int64_t s, int c, const float* dy, void* dx,
                         void* stream) {
  if (n <= 0 || s <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!dy || !dx) return MMAD_ENULL;
  if (dtype == MMAD_BF16) return gap_bwd<u16>(n, s, c, dy, dx, as_stream(stream), true);
  if (dtype == MMAD_F32) return gap_bwd<float>(n, s, c, dy, dx, as_stream(stream), true);
  return MMAD_EBADDTYPE;
}

}  // extern "C"

namespace mmad_pool {
int set_run_mode(int v) {
  const int prev = pool_run_mode();
  if (v >= 0) g_pool_run.store(v, std::memory_order_relaxed);
  return prev;
}
}  // namespace mmad_pool
