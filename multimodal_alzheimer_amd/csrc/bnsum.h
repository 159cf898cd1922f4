// BN-backward partial sums from a conv epilogue (round 6).  MedicalNet's BasicBlock runs
// conv1 -> bn1 -> relu -> conv2 (anat_cnn.py:30-31, MedicalNet BasicBlock); in the backward,
// conv2's input gradient g is exactly what bn1's backward reduces:
//   S = sum g',  Q = sum g' * xhat,  g' = g * (fma(y, scale, shift) > 0),  xhat = (y - mean) * invstd
// over all voxels, per channel (bn.hip colsum_kernel MODE 4, the same arithmetic per element).
// A dgrad kernel whose store loop gives each thread a fixed 8-channel vector adds its stored
// (bf16-rounded) g and the matching 16 bytes of y into per-thread sums, folds them over the
// threads of the block in a fixed order and writes one partial row per tile:
// parts[tile][2][C] -- the layout bn_bwd_finalize reads -- so the separate column-sum pass
// over g and y disappears.  Deterministic (fixed-shape sums, no atomics).
#pragma once
#include "common.h"

struct BnSum {
  float s[8], q[8], sc[8], sh[8], mu[8], is[8];

  // the BN constants of channels c0 .. c0 + 7 (16-byte aligned: c0 % 8 == 0)
  __device__ __forceinline__ void init(const float* __restrict__ scale,
                                       const float* __restrict__ shift,
                                       const float* __restrict__ mean,
                                       const float* __restrict__ invstd, int c0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(scale + c0 + 4 * h);
      const f32x4 b = *reinterpret_cast<const f32x4*>(shift + c0 + 4 * h);
      const f32x4 m = *reinterpret_cast<const f32x4*>(mean + c0 + 4 * h);
      const f32x4 v = *reinterpret_cast<const f32x4*>(invstd + c0 + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[4 * h + e] = a[e];
        sh[4 * h + e] = b[e];
        mu[4 * h + e] = m[e];
        is[4 * h + e] = v[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[e] = 0.f; q[e] = 0.f; }
  }

  // one stored 8-channel gradient vector and the BN input y at the same voxel
  __device__ __forceinline__ void add(u32x4 gv, u32x4 yv) {
    float g[8], y[8];
    Chunk<u16>::load(reinterpret_cast<const u16*>(&gv), g);
    Chunk<u16>::load(reinterpret_cast<const u16*>(&yv), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gm = bn_affine(y[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
      s[e] += gm;
      q[e] += gm * ((y[e] - mu[e]) * is[e]);
    }
  }
};

// Fold the block's per-thread sums (thread t holds channel vector t % cpr of the tile's
// cpr * 8 columns) in thread order and write the tile's partial row.  red: LDS scratch of
// nthr * 16 floats, free for the caller's purposes before (a barrier separates its last
// reads from these writes) and after.  Block-uniform call (contains a barrier).
__device__ __forceinline__ void bnsum_flush(const BnSum& a, float* red, int cpr, int nthr,
                                            float* __restrict__ parts, int64_t prow, int nd,
                                            int col0) {
  const int tid = threadIdx.x, c8 = tid % cpr, k = tid / cpr;
  float* r = red + k * (cpr * 16) + c8 * 16;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    r[e] = a.s[e];
    r[8 + e] = a.q[e];
  }
  __syncthreads();
  const int K = nthr / cpr;
  for (int c = tid; c < cpr * 8; c += nthr) {
    const int cv = c >> 3, e = c & 7;
    float S = 0.f, Q = 0.f;
    for (int kk = 0; kk < K; ++kk) {                // fixed order: deterministic
      S += red[kk * (cpr * 16) + cv * 16 + e];
      Q += red[kk * (cpr * 16) + cv * 16 + 8 + e];
    }
    parts[(prow * 2) * nd + col0 + c] = S;
    parts[(prow * 2 + 1) * nd + col0 + c] = Q;
  }
}
