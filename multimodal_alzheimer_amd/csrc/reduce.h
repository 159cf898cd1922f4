// Transposing split-K slab reductions of the weight gradients (the bodies of conv.hip's
// wgrad_reduce_t_kernel / wgrad_reduce_tz_kernel) as device functions of explicit block
// coordinates, and the job record that describes one launch of them.  Slabs
// ws[split][co][tap * Cs + ci] are summed in fixed order into dW[co][ci][tap].  (Round 4 ran
// them as extra blocks of the next BN-backward reduction launch: bit-identical, one launch
// fewer, 2 % slower -- PERF_LOG.md.)
#pragma once
#include "common.h"

namespace mmad_reduce {

enum { KIND_NONE = 0, KIND_T = 1, KIND_TZ = 2, KIND_WIDE = 3, KIND_STEM = 4 };
// the C ABI's record of one pending reduction (include/mmad.h); KIND_WIDE: 1x1x1 slabs
// [split][co][ci] (dW in the same order), gx blocks of 256 elements
using Job = mmad_wgrad_job;
// shared memory the bodies need (floats): tz's 256 f32x4 partials + the 64 x 33 tile
constexpr int SMEM_FLOATS = 256 * 4 + 64 * 33;

// one block per (co, 64-channel slice); slab reads run along ci, 16 bytes per lane (a wave
// covers 4 taps x 64 channels), and the [ci][taps] result goes out through LDS as one
// contiguous run of the torch tensor (taps <= 32)
__device__ __forceinline__ void t_body(const float* __restrict__ ws, float* __restrict__ dw,
                                       int splits, int Nd, int K, int Cs, int taps, int bx,
                                       int by, float* sm) {
  float* tile = sm;                            // [64][taps + 1]
  const int ct = min(64, Cs);                  // channels in this slice (Cs % 16 == 0)
  const int q4 = ct / 4, tpi = 256 / q4;       // lanes per tap row, taps per block pass
  const int co = by, c0 = bx * ct;
  const int e4 = threadIdx.x % q4, tg = threadIdx.x / q4;
  const int64_t total = (int64_t)Nd * K;
  const float* base = ws + (int64_t)co * K + c0 + e4 * 4;
  for (int t = tg; t < taps; t += tpi) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int sp = 0; sp < splits; ++sp)
      s += *reinterpret_cast<const f32x4*>(base + sp * total + (int64_t)t * Cs);
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[(e4 * 4 + q) * (taps + 1) + t] = s[q];
  }
  __syncthreads();
  float* out = dw + ((int64_t)co * Cs + c0) * taps;
  for (int l = threadIdx.x; l < ct * taps; l += 256)
    out[l] = tile[(l / taps) * (taps + 1) + l % taps];
}

// Same sum and layout for grids of few (co, channel-slice) blocks (the 64-channel layer1 and
// layer2 shapes: 64-128 blocks for 128-69 slabs): bz takes a group of tper taps, and each
// (tap, 4-channel) position's slabs are split over SP thread groups whose partial sums are
// added in a fixed order (deterministic; the order differs from t_body's single chain only
// in fp32 rounding)
__device__ __forceinline__ void tz_body(const float* __restrict__ ws, float* __restrict__ dw,
                                        int splits, int Nd, int K, int Cs, int taps, int tper,
                                        int bx, int by, int bz, float* sm) {
  f32x4* part = reinterpret_cast<f32x4*>(sm);  // [256]
  float* tile = sm + 256 * 4;                  // [64][tper + 1]
  const int ct = min(64, Cs);
  const int q4 = ct / 4;
  const int co = by, c0 = bx * ct;
  const int t0 = bz * tper, nt = min(taps - t0, tper);
  const int P = nt * q4;                         // (tap, 4-channel) positions of this block
  const int SP = max(1, 256 / max(P, 1));        // slab groups per position
  const int pos = threadIdx.x % P, sg = threadIdx.x / P;
  const int64_t total = (int64_t)Nd * K;
  if (nt <= 0) return;                           // (block-uniform)
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  const int e4 = pos % q4, tl = pos / q4;
  if (sg < SP) {
    const int per = (splits + SP - 1) / SP;
    const int sp0 = sg * per, sp1 = min(splits, sp0 + per);
    const float* base = ws + (int64_t)co * K + c0 + e4 * 4 + (int64_t)(t0 + tl) * Cs;
#pragma unroll 8
    for (int sp = sp0; sp < sp1; ++sp) s += *reinterpret_cast<const f32x4*>(base + sp * total);
    part[threadIdx.x] = s;
  }
  __syncthreads();
  if ((int)threadIdx.x < P) {
    f32x4 a = part[threadIdx.x];
    for (int g2 = 1; g2 < SP; ++g2) a += part[g2 * P + threadIdx.x];   // fixed order
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[(e4 * 4 + q) * (tper + 1) + tl] = a[q];
  }
  __syncthreads();
  // dW[co][c][t0 .. t0 + nt): runs of nt taps per channel
  float* out = dw + ((int64_t)co * Cs + c0) * taps + t0;
  for (int l = threadIdx.x; l < ct * nt; l += 256) {
    const int c = l / nt, t = l % nt;
    out[(int64_t)c * taps + t] = tile[c * (tper + 1) + t];
  }
}

// 1x1x1 slabs (conv.hip's wgrad_reduce_wide_kernel, stride 1, taps 1): block bx sums 256
// consecutive elements, 4 groups of 64 lanes taking every 4th slab (16 bytes per lane per
// load), the groups combined in fixed order; dW[co][ci] is the slab order itself
__device__ __forceinline__ void wide_body(const float* __restrict__ ws, float* __restrict__ dw,
                                          int splits, int64_t total, int bx, float* sm) {
  f32x4* red = reinterpret_cast<f32x4*>(sm);   // [4][64]
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t idx = ((int64_t)bx * 64 + e) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (idx < total) {
#pragma unroll 4
    for (int sp = grp; sp < splits; sp += 4)
      s += *reinterpret_cast<const f32x4*>(ws + sp * total + idx);
  }
  red[grp * 64 + e] = s;
  __syncthreads();
  if (grp != 0 || idx >= total) return;
  s = ((red[e] + red[64 + e]) + red[128 + e]) + red[192 + e];
  *reinterpret_cast<f32x4*>(dw + idx) = s;
}

// The stem's slabs (one per stem wgrad block, [co][K = (kd*KH + kh)*8 + j] on the W-unfolded
// input, dW[co][kd*KH + kh][j < unf_kw]): conv.hip's two-level sum (slab_group_sum_kernel's
// groups of 16 slabs, then the group sums in order; wgrad_reduce_kernel's scatter) in one
// pass -- 4 thread groups of 64 consecutive elements each take every 4th slab group, keep
// each group's sum, and lane group 0 adds the group sums in order: bit-identical
constexpr int STEM_G = 16;
__device__ __forceinline__ void stem_body(const float* __restrict__ ws, float* __restrict__ dw,
                                          int splits, int Nd, int K, int taps, int unf_kw, int bx,
                                          float* sm) {
  const int64_t total = (int64_t)Nd * K;
  const int e = threadIdx.x & 63, g4 = threadIdx.x >> 6;
  const int64_t idx = (int64_t)bx * 64 + e;
  const int ng = (splits + STEM_G - 1) / STEM_G;      // <= 32 (host-checked)
  if (idx < total) {
    for (int gi = g4; gi < ng; gi += 4) {
      float s = 0.f;
      const int s1 = min(splits, (gi + 1) * STEM_G);
#pragma unroll 16
      for (int sp = gi * STEM_G; sp < s1; ++sp) s += ws[sp * total + idx];
      sm[gi * 64 + e] = s;
    }
  }
  __syncthreads();
  if (g4 != 0 || idx >= total) return;
  float s = 0.f;
  for (int gi = 0; gi < ng; ++gi) s += sm[gi * 64 + e];
  const int co = (int)(idx / K), k = (int)(idx % K);
  const int j = k & 7, tkh = k >> 3;
  if (j < unf_kw) dw[((int64_t)co * taps + tkh) * unf_kw + j] = s;
}

// block `lin` of job j's own grid (x fastest)
__device__ __forceinline__ void run(const Job& j, int lin, float* sm) {
  const int bx = lin % j.gx, r = lin / j.gx, by = r % j.gy, bz = r / j.gy;
  if (j.kind == KIND_WIDE)
    wide_body(j.ws, j.dw, j.splits, (int64_t)j.nd * j.k, bx, sm);
  else if (j.kind == KIND_STEM)
    stem_body(j.ws, j.dw, j.splits, j.nd, j.k, j.taps, j.tper, bx, sm);
  else if (j.kind == KIND_TZ)
    tz_body(j.ws, j.dw, j.splits, j.nd, j.k, j.cs, j.taps, j.tper, bx, by, bz, sm);
  else
    t_body(j.ws, j.dw, j.splits, j.nd, j.k, j.cs, j.taps, bx, by, sm);
}

__host__ __device__ inline int64_t job_blocks(const Job& j) {
  return j.kind == KIND_NONE ? 0 : (int64_t)j.gx * j.gy * j.gz;
}

}  // namespace mmad_reduce
