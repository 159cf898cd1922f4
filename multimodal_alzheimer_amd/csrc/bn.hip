// BatchNorm (train / eval) + ReLU + residual add on NDHWC activations, gfx950.
//
// Replaces nn.BatchNorm3d / nn.BatchNorm1d + nn.ReLU + MedicalNet's residual
// `out += residual; out = relu(out)` (BasicBlock), the stem bn1+relu and the head BNs
// (pkg/models/mri_models/anat_cnn.py:50-51, :69-70).  Layout [m][c], m = N*D*H*W.
//
// All per-channel reductions are two-stage and deterministic: a partial pass writes
// [parts][2][c] fp32 rows (fixed row ranges per block), a finalize pass sums the parts
// in fixed order in f64.  The conv forward kernel emits the same partial layout from its
// epilogue, so a BN that follows one of our convs needs no separate statistics pass.
#include "common.h"

// rows in flight per thread of the column sums (16-byte rows; round 4 measured 2 and 8
// for the single and dual forms, neither faster)
constexpr int COLSUM_ROWS = 4;

namespace {

// Row ranges per partial-sum block: <= 1024 parts so the f64 finalize stays short, and
// >= 64 rows per part so each block streams a useful amount.
struct PartPlan {
  int64_t rpp;
  int nparts;
};
PartPlan part_plan(int64_t M) {
  int n = (int)std::min<int64_t>(1024, std::max<int64_t>(1, cdiv(M, 64)));
  const int64_t rpp = cdiv(M, n);
  return {rpp, (int)cdiv(M, rpp)};
}

// Per-channel sums over rows [p*rpp, (p+1)*rpp) of
//   MODE 0: y and y^2          (BN forward statistics)
//   MODE 1: g' and g'*xhat     (BN backward), g' = g * (relu_out > 0 | 1)
//   MODE 2: y                  (conv bias gradient)
//   MODE 3: as MODE 1 with the mask from bit 7 of act[] (fused BN+ReLU+max-pool backward,
//           rows = pooled outputs, y = the pre-BN value at each window's argmax)
// V channels per thread (16-byte vectors when C % VEC == 0), CC / V lanes per row and
// 256 / (CC / V) rows in flight per block; one LDS pass folds the row lanes.  Wide rows
// (C / V > 256, e.g. ResNet-50's 2048 channels) are split over gridDim.y channel slabs of
// CC = C / gridDim.y channels each.
// DUAL (MODE 1 only): a second BN over the same gradient and ReLU mask (the shortcut BN of
// a residual block, y2 = its input): parts2 gets (sum g', sum g' * xhat2) from the same pass,
// so g and the mask are read once for both
// G2 (MODE 1 / 3): a second gradient of the same output (the block input's other consumer,
// volume_ops twin outputs); g is then as_stored(g + g2), rounded as torch's own gradient
// accumulation rounds it, so no separate add pass is needed.  MODE 3 also stores that sum
// to gsum (the pool backward's input).
// GB (DUAL only): g is a global-average-pool gradient given compactly as [N][C] rows, row r of
// the BN input reading g[r / gS] (the pooled gradient's broadcast is never materialised)
#ifndef BN_FOLD_PROBE
#define BN_FOLD_PROBE 0
#endif
#if BN_FOLD_PROBE
// BN-finalize fold measurement (build flag, never the default): after its partial rows every
// block releases them and arrives on its 32-block group's counter; the group's last arriver
// acquires and re-reads the group's rows -- the first level of a producer-side fold -- and
// re-arms the counter.  The result goes to g_fold_sink so the reads stay.
__device__ int g_fold_cnt[4096];
__device__ float g_fold_sink[4096];
#endif

template <typename T, int MODE, int V, bool DUAL = false, bool G2 = false, bool GB = false>
__global__ __launch_bounds__(256) void colsum_kernel(int64_t M, int C, int64_t rpp,
                                                     const T* __restrict__ y,
                                                     const T* __restrict__ g,
                                                     const T* __restrict__ relu_out,
                                                     const float* __restrict__ mean,
                                                     const float* __restrict__ invstd,
                                                     float* __restrict__ parts,
                                                     const uint8_t* __restrict__ act,
                                                     const float* __restrict__ msc,
                                                     const float* __restrict__ msh,
                                                     const T* __restrict__ y2 = nullptr,
                                                     const float* __restrict__ mean2 = nullptr,
                                                     const float* __restrict__ invstd2 = nullptr,
                                                     float* __restrict__ parts2 = nullptr,
                                                     const T* __restrict__ g2 = nullptr,
                                                     T* __restrict__ gsum = nullptr,
                                                     uint32_t gS = 0) {
  static_assert(!DUAL || MODE == 1, "dual partial sums: BN backward with a relu_out mask");
  static_assert(!GB || (DUAL && V == Chunk<T>::N), "broadcast g: the pair kernel, 16-byte rows");
  __shared__ float red[DUAL ? 3 : 2][2048];
  const int tid = threadIdx.x;
  const int CC = C / (int)gridDim.y;           // this block's channel slab
  const int cb = (int)blockIdx.y * CC;
  const int lpr = CC / V;
  const int rpar = 256 / lpr;
  const int cl = tid % lpr, rl = tid / lpr;
  const int64_t r0 = (int64_t)blockIdx.x * rpp;
  const int64_t r1 = min(M, r0 + rpp);
  float s[V], q[V], q2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { s[e] = 0.f; q[e] = 0.f; q2[e] = 0.f; }
  if (rl < rpar) {
    float mu[V], is[V], sc[V], sh[V], mu2[V], is2[V];
    if (MODE == 1 || MODE == 3 || MODE == 4) {
#pragma unroll
      for (int e = 0; e < V; ++e) { mu[e] = mean[cb + cl * V + e]; is[e] = invstd[cb + cl * V + e]; }
    }
    if constexpr (DUAL) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        mu2[e] = mean2[cb + cl * V + e];
        is2[e] = invstd2[cb + cl * V + e];
      }
    }
    if (MODE == 4) {
#pragma unroll
      for (int e = 0; e < V; ++e) { sc[e] = msc[cb + cl * V + e]; sh[e] = msh[cb + cl * V + e]; }
    }
    // one row's contribution, from its y / g / relu_out values
    auto accum = [&](int64_t i, float* yv, float* gv, const float* ov, const float* y2v) {
      if (MODE == 1 || MODE == 3 || MODE == 4) {
        if (MODE == 4) {
          // ReLU mask of a BN+ReLU without residual, recomputed from its input y with the
          // forward's own affine (bn_affine): out > 0 <=> fma(y, scale, shift) > 0
#pragma unroll
          for (int e = 0; e < V; ++e) gv[e] = bn_affine(yv[e], sc[e], sh[e]) > 0.f ? gv[e] : 0.f;
        } else if (MODE == 3) {
#pragma unroll
          for (int e = 0; e < V; ++e) gv[e] = (act[i + e] & 0x80) ? gv[e] : 0.f;
        } else if (relu_out != nullptr) {
#pragma unroll
          for (int e = 0; e < V; ++e) gv[e] = ov[e] > 0.f ? gv[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
          s[e] += gv[e];
          q[e] += gv[e] * ((yv[e] - mu[e]) * is[e]);
        }
        if constexpr (DUAL) {
#pragma unroll
          for (int e = 0; e < V; ++e) q2[e] += gv[e] * ((y2v[e] - mu2[e]) * is2[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          s[e] += yv[e];
          if (MODE == 0) q[e] += yv[e] * yv[e];
        }
      }
    };
    constexpr bool NEED_G = MODE == 1 || MODE == 3 || MODE == 4;
    int64_t r = r0 + rl;
    if constexpr (V == Chunk<T>::N) {
      // 4 rows' 16-byte loads issued before any is used (the loop is load-latency bound:
      // 512-1024 blocks of 4 waves keep too few bytes in flight with one row at a time);
      // rows are still added in the same order
      constexpr int U = COLSUM_ROWS;
      for (; r + (U - 1) * rpar < r1; r += U * rpar) {
        u32x4 yr[U], gr[U], orr[U], y2r[U], g2r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = (r + u * rpar) * C + cb + cl * V;
          yr[u] = *reinterpret_cast<const u32x4*>(y + i);
          if constexpr (GB)
            gr[u] = *reinterpret_cast<const u32x4*>(
                g + (int64_t)((uint32_t)(r + u * rpar) / gS) * C + cb + cl * V);
          else if (NEED_G)
            gr[u] = *reinterpret_cast<const u32x4*>(g + i);
          if (NEED_G && G2) g2r[u] = *reinterpret_cast<const u32x4*>(g2 + i);
          if (MODE == 1 && relu_out != nullptr)
            orr[u] = *reinterpret_cast<const u32x4*>(relu_out + i);
          if constexpr (DUAL) y2r[u] = *reinterpret_cast<const u32x4*>(y2 + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = (r + u * rpar) * C + cb + cl * V;
          float yv[V], gv[V], ov[V], y2v[V];
          Chunk<T>::load(reinterpret_cast<const T*>(&yr[u]), yv);
          if (NEED_G) Chunk<T>::load(reinterpret_cast<const T*>(&gr[u]), gv);
          if constexpr (NEED_G && G2) {
            float hv[V];
            Chunk<T>::load(reinterpret_cast<const T*>(&g2r[u]), hv);
#pragma unroll
            for (int e = 0; e < V; ++e) gv[e] = as_stored<T>(gv[e] + hv[e]);
            if constexpr (MODE == 3) Chunk<T>::store(gsum + i, gv);
          }
          if (MODE == 1 && relu_out != nullptr)
            Chunk<T>::load(reinterpret_cast<const T*>(&orr[u]), ov);
          if constexpr (DUAL) Chunk<T>::load(reinterpret_cast<const T*>(&y2r[u]), y2v);
          accum(i, yv, gv, ov, y2v);
        }
      }
    }
    for (; r < r1; r += rpar) {
      const int64_t i = r * C + cb + cl * V;
      float yv[V], gv[V], ov[V], y2v[V];
      if constexpr (V == Chunk<T>::N) Chunk<T>::load(y + i, yv);
      else for (int e = 0; e < V; ++e) yv[e] = Elt<T>::ld(y, i + e);
      if (NEED_G) {
        if constexpr (GB) Chunk<T>::load(g + (int64_t)((uint32_t)r / gS) * C + cb + cl * V, gv);
        else if constexpr (V == Chunk<T>::N) Chunk<T>::load(g + i, gv);
        else for (int e = 0; e < V; ++e) gv[e] = Elt<T>::ld(g, i + e);
        if constexpr (G2) {
          float hv[V];
          if constexpr (V == Chunk<T>::N) Chunk<T>::load(g2 + i, hv);
          else for (int e = 0; e < V; ++e) hv[e] = Elt<T>::ld(g2, i + e);
#pragma unroll
          for (int e = 0; e < V; ++e) gv[e] = as_stored<T>(gv[e] + hv[e]);
          if constexpr (MODE == 3) {
            if constexpr (V == Chunk<T>::N) Chunk<T>::store(gsum + i, gv);
            else for (int e = 0; e < V; ++e) Elt<T>::st(gsum, i + e, gv[e]);
          }
        }
        if (MODE == 1 && relu_out != nullptr) {
          if constexpr (V == Chunk<T>::N) Chunk<T>::load(relu_out + i, ov);
          else for (int e = 0; e < V; ++e) ov[e] = Elt<T>::ld(relu_out, i + e);
        }
      }
      if constexpr (DUAL) {
        if constexpr (V == Chunk<T>::N) Chunk<T>::load(y2 + i, y2v);
        else for (int e = 0; e < V; ++e) y2v[e] = Elt<T>::ld(y2, i + e);
      }
      accum(i, yv, gv, ov, y2v);
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      red[0][rl * CC + cl * V + e] = s[e];
      red[1][rl * CC + cl * V + e] = q[e];
      if constexpr (DUAL) red[DUAL ? 2 : 0][rl * CC + cl * V + e] = q2[e];
    }
  }
  __syncthreads();
  for (int c = tid; c < CC; c += 256) {
    float ss = 0.f, qq = 0.f, q2q = 0.f;
    for (int k = 0; k < rpar; ++k) {
      ss += red[0][k * CC + c];
      qq += red[1][k * CC + c];
      if constexpr (DUAL) q2q += red[DUAL ? 2 : 0][k * CC + c];
    }
    parts[((int64_t)blockIdx.x * 2) * C + cb + c] = ss;
    parts[((int64_t)blockIdx.x * 2 + 1) * C + cb + c] = qq;
    if constexpr (DUAL) {
      parts2[((int64_t)blockIdx.x * 2) * C + cb + c] = ss;
      parts2[((int64_t)blockIdx.x * 2 + 1) * C + cb + c] = q2q;
    }
  }
#if BN_FOLD_PROBE
  __shared__ int last;
  const int ngx = ((int)gridDim.x + 31) >> 5;
  const int grp = (int)blockIdx.y * ngx + ((int)blockIdx.x >> 5);
  const int gsize = min(32, (int)gridDim.x - (((int)blockIdx.x >> 5) << 5));
  __threadfence();                                   // release this block's rows
  __syncthreads();
  if (tid == 0) last = atomicAdd(&g_fold_cnt[grp & 4095], 1) == gsize - 1;
  __syncthreads();
  if (last) {
    __threadfence();                                 // acquire the group's rows
    for (int c = tid; c < CC; c += 256) {
      float ss = 0.f, qq = 0.f;
      const int p0 = ((int)blockIdx.x >> 5) << 5;
      for (int k = 0; k < gsize; ++k) {
        ss += parts[((int64_t)(p0 + k) * 2) * C + cb + c];
        qq += parts[((int64_t)(p0 + k) * 2 + 1) * C + cb + c];
      }
      g_fold_sink[(grp * 64 + c) & 4095] = ss + qq;
    }
    if (tid == 0) g_fold_cnt[grp & 4095] = 0;          // re-arm
  }
#endif
}

// Fold groups of `group` partial rows into one (fixed order): keeps the finalize short
// when the parts come from the conv epilogue (one row per 128-voxel tile).
__global__ void parts_fold_kernel(int C, int nparts, int group, const float* __restrict__ in,
                                  float* __restrict__ out) {
  const int o = blockIdx.x;
  for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
    float s = 0.f;
    const int p1 = min(nparts, (o + 1) * group);
#pragma unroll 8
    for (int p = o * group; p < p1; ++p) s += in[(int64_t)p * 2 * C + c];
    out[(int64_t)o * 2 * C + c] = s;
  }
}

template <typename T, int MODE>
int launch_colsum(int64_t M, int C, const void* y, const void* g, const void* ro,
                  const float* mean, const float* invstd, float* parts, hipStream_t st,
                  const uint8_t* act = nullptr, const float* msc = nullptr,
                  const float* msh = nullptr, const void* g2 = nullptr,
                  void* gsum = nullptr) {
  const PartPlan pp = part_plan(M);
  constexpr int VEC = Chunk<T>::N;
  dim3 grid((unsigned)pp.nparts);
  // channel slabs for wide rows: the smallest power-of-two split whose slab fits one block
  int slabs = 1;
  while (C % (slabs * 2 * VEC) == 0 && C / (slabs * VEC) > 256) slabs *= 2;
  // g2: its own instantiation, so the kernels without one keep their registers
#define COLSUM(VV, G)                                                                       \
  hipLaunchKernelGGL((colsum_kernel<T, MODE, VV, false, G>), grid, dim3(256), 0, st, M, C, \
                     pp.rpp, (const T*)y, (const T*)g, (const T*)ro, mean, invstd, parts, act, \
                     msc, msh, nullptr, nullptr, nullptr, nullptr, (const T*)g2, (T*)gsum)
  if (C % (slabs * VEC) == 0 && C / (slabs * VEC) <= 256) {
    grid.y = (unsigned)slabs;
    if constexpr (MODE == 1 || MODE == 3) {
      if (g2 != nullptr) COLSUM(VEC, true); else COLSUM(VEC, false);
    } else {
      COLSUM(VEC, false);
    }
  } else if (C <= 256) {
    if constexpr (MODE == 1 || MODE == 3) {
      if (g2 != nullptr) COLSUM(1, true); else COLSUM(1, false);
    } else {
      COLSUM(1, false);
    }
  } else {
    return MMAD_EUNSUPPORTED;
  }
#undef COLSUM
  return launch_status();
}

// f64 sum of the partial rows; block = FC channels x 64 part-lanes (1024 threads), loads
// unrolled 8 deep (16 in flight per thread: the finalize kernels are load-latency bound),
// then a fixed-shape LDS tree over the part-lanes (deterministic).
constexpr int FC = 16;
__device__ __forceinline__ void sum_parts(int c, int C, int nparts, const float* parts,
                                          double* sm, double& S, double& Q) {
  const int cx = threadIdx.x % FC, py = threadIdx.x / FC;
  double s = 0.0, q = 0.0;
  if (c < C) {
    int p = py;
    constexpr int U = 8;
    for (; p + 64 * (U - 1) < nparts; p += 64 * U) {
      float a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = parts[((int64_t)(p + 64 * u) * 2) * C + c];
        b[u] = parts[((int64_t)(p + 64 * u) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) { s += a[u]; q += b[u]; }
    }
    for (; p < nparts; p += 64) {
      s += parts[((int64_t)p * 2) * C + c];
      q += parts[((int64_t)p * 2 + 1) * C + c];
    }
  }
  // the 4 part lanes of a channel inside one wave (lane bits 4-5) by shuffles, then the 16
  // waves through LDS: one barrier instead of a six-level tree (this kernel is latency-bound)
  s += __shfl_xor(s, 16, 64);
  q += __shfl_xor(q, 16, 64);
  s += __shfl_xor(s, 32, 64);
  q += __shfl_xor(q, 32, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < FC) {
    sm[w * FC + cx] = s;
    sm[1024 + w * FC + cx] = q;
  }
  __syncthreads();
  S = 0.0;
  Q = 0.0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {                 // fixed order: deterministic
    S += sm[k * FC + cx];
    Q += sm[1024 + k * FC + cx];
  }
}

__device__ __forceinline__ void finalize_body(int C, int64_t count, int nparts,
                                              const float* parts, const float* gamma,
                                              const float* beta, float* running_mean,
                                              float* running_var, float momentum, float eps,
                                              int training, float* mean_out, float* invstd_out,
                                              float* scale_out, float* shift_out, int64_t* nbt,
                                              double* sm) {
  const int c = blockIdx.x * FC + (threadIdx.x % FC);
  // the per-channel operands are loaded before the partial sums, so their memory round trip
  // overlaps the sum's instead of following it (this kernel is latency-bound)
  const bool own = threadIdx.x < FC && c < C;
  float gm = 1.f, bt = 0.f, rm = 0.f, rv = 0.f;
  if (own) {
    if (gamma) gm = gamma[c];
    if (beta) bt = beta[c];
    if (running_mean != nullptr) { rm = running_mean[c]; rv = running_var[c]; }
  }
  double S, Q;
  if (training) {
    sum_parts(c, C, nparts, parts, sm, S, Q);
  } else {
    S = Q = 0.0;
  }
  if (!own) return;
  double mean, var;
  if (training) {
    mean = S / (double)count;
    var = Q / (double)count - mean * mean;
    if (var < 0) var = 0;
    if (running_mean != nullptr) {
      if (nbt != nullptr && c == 0) *nbt += 1;
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      running_mean[c] = (float)((1.0 - momentum) * rm + momentum * mean);
      running_var[c] = (float)((1.0 - momentum) * rv + momentum * unb);
    }
  } else {
    mean = rm;
    var = rv;
  }
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  if (mean_out) mean_out[c] = (float)mean;
  if (invstd_out) invstd_out[c] = is;
  if (scale_out) scale_out[c] = gm * is;
  if (shift_out) shift_out[c] = bt - (float)mean * gm * is;
}

__global__ __launch_bounds__(1024) void bn_finalize_kernel(
    int C, int64_t count, int nparts, const float* __restrict__ parts,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* running_mean,
    float* running_var, float momentum, float eps, int training, float* mean_out,
    float* invstd_out, float* scale_out, float* shift_out, int64_t* nbt) {
  __shared__ double sm[2048];
  finalize_body(C, count, nparts, parts, gamma, beta, running_mean, running_var, momentum, eps,
                training, mean_out, invstd_out, scale_out, shift_out, nbt, sm);
}

// the two BNs of a residual pair (main and shortcut) in one launch: blockIdx.y picks the set
__global__ __launch_bounds__(1024) void bn_finalize2_kernel(int C, int64_t count, mmad_bn_fin a,
                                                            mmad_bn_fin b) {
  __shared__ double sm[2048];
  const mmad_bn_fin& f = blockIdx.y ? b : a;
  finalize_body(C, count, f.nparts, f.parts, f.gamma, f.beta, f.running_mean, f.running_var,
                f.momentum, f.eps, f.training, f.mean, f.invstd, f.scale, f.shift,
                f.num_batches_tracked, sm);
}

// eval-mode BN folded into the preceding conv: scale = gamma / sqrt(var + eps),
// bias = beta - mean*scale (+ conv_bias*scale); the same arithmetic as bn_finalize_kernel's
// running-statistics branch, so folded and unfolded eval paths use identical coefficients
__global__ void bn_fold_kernel(int C, const float* __restrict__ gamma,
                               const float* __restrict__ beta, const float* __restrict__ mean,
                               const float* __restrict__ var, float eps,
                               const float* __restrict__ conv_bias, float* __restrict__ scale,
                               float* __restrict__ bias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = (float)(1.0 / sqrt((double)var[c] + (double)eps));
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  const float sc = gm * is;
  float sh = bt - mean[c] * gm * is;
  if (conv_bias) sh += conv_bias[c] * sc;
  scale[c] = sc;
  bias[c] = sh;
}

__device__ __forceinline__ void bwd_finalize(int C, int64_t count, int nparts,
                                             const float* parts, const float* gamma,
                                             const float* invstd, int training, float* dgamma,
                                             float* dbeta, float* coef, double* sm) {
  const int c = blockIdx.x * FC + (threadIdx.x % FC);
  const bool own = threadIdx.x < FC && c < C;
  float gm = 1.f, is = 0.f;                      // loaded ahead of the partial sums
  if (own) {
    if (gamma) gm = gamma[c];
    is = invstd[c];
  }
  double S, Q;
  sum_parts(c, C, nparts, parts, sm, S, Q);
  if (!own) return;
  if (dbeta) dbeta[c] = (float)S;
  if (dgamma) dgamma[c] = (float)Q;
  const double k0 = (double)gm * is;
  coef[c] = (float)k0;
  coef[C + c] = training ? (float)(k0 * S / (double)count) : 0.f;
  coef[2 * C + c] = training ? (float)(k0 * Q / (double)count) : 0.f;
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    int C, int64_t count, int nparts, const float* __restrict__ parts,
    const float* __restrict__ gamma, const float* __restrict__ invstd, int training,
    float* dgamma, float* dbeta, float* coef) {
  __shared__ double sm[2048];
  bwd_finalize(C, count, nparts, parts, gamma, invstd, training, dgamma, dbeta, coef, sm);
}

// both BNs of a residual pair in one launch: blockIdx.y picks the set
struct BwdFin {
  const float* parts;
  const float* gamma;
  const float* invstd;
  int training;
  float* dgamma;
  float* dbeta;
  float* coef;
};

__global__ __launch_bounds__(1024) void bn_bwd_finalize2_kernel(int C, int64_t count,
                                                                int nparts, BwdFin a, BwdFin b) {
  __shared__ double sm[2048];
  const BwdFin& f = blockIdx.y ? b : a;
  bwd_finalize(C, count, nparts, f.parts, f.gamma, f.invstd, f.training, f.dgamma, f.dbeta,
               f.coef, sm);
}

__global__ void sum_only_finalize_kernel(int C, int nparts, const float* __restrict__ parts,
                                         float* out) {
  __shared__ double sm[2048];
  const int c = blockIdx.x * FC + (threadIdx.x % FC);
  double S, Q;
  sum_parts(c, C, nparts, parts, sm, S, Q);
  if (threadIdx.x >= FC || c >= C) return;
  out[c] = (float)S;
}

// out = act(y*scale + shift + R); vector path when C % EPC == 0
template <typename T, int RES>   // RES 0: none, 1: identity residual, 2: BN'ed residual
__global__ void scale_shift_act_kernel(int64_t M, int C, const T* __restrict__ y,
                                       const float* __restrict__ scale,
                                       const float* __restrict__ shift,
                                       const T* __restrict__ res,
                                       const float* __restrict__ rscale,
                                       const float* __restrict__ rshift, int relu,
                                       T* __restrict__ out) {
  constexpr int N = Chunk<T>::N;
  const int64_t nchunks = M * C / N;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nchunks;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = q * N;
    const int c0 = (int)(i0 % C);
    float v[N], r[N];
    Chunk<T>::load(y + i0, v);
    if (RES) Chunk<T>::load(res + i0, r);
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int c = c0 + e;
      float o = bn_affine(v[e], scale[c], shift[c]);
      if (RES == 1) o += r[e];
      if (RES == 2) o += r[e] * rscale[c] + rshift[c];
      v[e] = relu ? fmaxf(o, 0.f) : o;
    }
    Chunk<T>::store(out + i0, v);
  }
}

// per-channel fp32 parameters of one channel vector: N consecutive floats from a 16-byte
// aligned offset (N = 4 or 8) as 16-byte loads
template <int N>
__device__ __forceinline__ void ld_params(const float* __restrict__ p, float* v) {
#pragma unroll
  for (int h = 0; h < N / 4; ++h) {
    const f32x4 c = *reinterpret_cast<const f32x4*>(p + 4 * h);
    v[4 * h] = c[0]; v[4 * h + 1] = c[1]; v[4 * h + 2] = c[2]; v[4 * h + 3] = c[3];
  }
}

// Fixed-channel form of scale_shift_act_kernel for C / N a power of two dividing 256: the
// grid stride is a multiple of the chunks per row, so every thread always handles the same
// channel vector -- its scale/shift (and residual scale/shift) are loaded once, as 16-byte
// vectors, instead of 2-4 scalar loads per element per chunk (the per-element parameter
// loads made the old kernel VMEM-issue bound at ~2 TB/s).  Two chunks per trip, loads first.
template <typename T, int RES>
__global__ __launch_bounds__(256) void scale_shift_act_fc_kernel(
    int64_t nchunks, int cpr, const T* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, const T* __restrict__ res, const float* __restrict__ rscale,
    const float* __restrict__ rshift, int relu, T* __restrict__ out) {
  constexpr int N = Chunk<T>::N;
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int c0 = (int)(t0 & (cpr - 1)) * N;
  float sc[N], sh[N], rs[N], rh[N];
  ld_params<N>(scale + c0, sc);
  ld_params<N>(shift + c0, sh);
  if (RES == 2) {
    ld_params<N>(rscale + c0, rs);
    ld_params<N>(rshift + c0, rh);
  }
  auto apply = [&](float* v, const float* r) {
#pragma unroll
    for (int e = 0; e < N; ++e) {
      float o = bn_affine(v[e], sc[e], sh[e]);
      if (RES == 1) o += r[e];
      if (RES == 2) o += r[e] * rs[e] + rh[e];
      v[e] = relu ? fmaxf(o, 0.f) : o;
    }
  };
  int64_t q = t0;
  for (; q + stride < nchunks; q += 2 * stride) {
    float v0[N], v1[N], r0[N], r1[N];
    Chunk<T>::load(y + q * N, v0);
    Chunk<T>::load(y + (q + stride) * N, v1);
    if (RES) {
      Chunk<T>::load(res + q * N, r0);
      Chunk<T>::load(res + (q + stride) * N, r1);
    }
    apply(v0, r0);
    apply(v1, r1);
    Chunk<T>::store(out + q * N, v0);
    Chunk<T>::store(out + (q + stride) * N, v1);
  }
  if (q < nchunks) {
    float v0[N], r0[N];
    Chunk<T>::load(y + q * N, v0);
    if (RES) Chunk<T>::load(res + q * N, r0);
    apply(v0, r0);
    Chunk<T>::store(out + q * N, v0);
  }
}

template <typename T>
__global__ void scale_shift_act_scalar_kernel(int64_t M, int C, const T* __restrict__ y,
                                              const float* __restrict__ scale,
                                              const float* __restrict__ shift,
                                              const T* __restrict__ res,
                                              const float* __restrict__ rscale,
                                              const float* __restrict__ rshift, int relu,
                                              T* __restrict__ out) {
  const int64_t n = M * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    float o = bn_affine(Elt<T>::ld(y, i), scale[c], shift[c]);
    if (res) o += rscale ? Elt<T>::ld(res, i) * rscale[c] + rshift[c] : Elt<T>::ld(res, i);
    Elt<T>::st(out, i, relu ? fmaxf(o, 0.f) : o);
  }
}

// Fixed-channel form of bn_bwd_apply_kernel (C / V a power of two dividing 256): per-thread
// channel vector constant, its mean/invstd/coef loaded once as vectors; two chunks a trip.
// DUAL: also the shortcut BN of a residual pair (input y2, gradient dy2), same masked g
struct BwdApply2 {
  const void* y2;
  const float* mean2;
  const float* invstd2;
  const float* coef2;
  void* dy2;
};

template <typename T, bool MASKY = false, bool DUAL = false, bool G2 = false, bool GB = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_fc_kernel(
    int64_t nv, int cpr, int C, const T* __restrict__ g, const T* __restrict__ relu_out,
    const T* __restrict__ y, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ coef, T* __restrict__ dy, T* __restrict__ gmask,
    const float* __restrict__ msc = nullptr, const float* __restrict__ msh = nullptr,
    BwdApply2 d2 = {}, const T* __restrict__ g2 = nullptr, uint32_t gS = 0) {
  constexpr int V = Chunk<T>::N;
  // GB: g compact [N][C] (see colsum_kernel); vector q is row q / cpr, cpr a power of two
  const int cpr_shift = __builtin_ctz(cpr);
  auto g_at = [&](int64_t qq) -> const T* {
    if constexpr (GB)
      return g + (int64_t)((uint32_t)(qq >> cpr_shift) / gS) * C + (qq & (cpr - 1)) * V;
    else
      return g + qq * V;
  };
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int c0 = (int)(t0 & (cpr - 1)) * V;
  float mu[V], is[V], k0[V], k1[V], k2[V];
  ld_params<V>(mean + c0, mu);
  ld_params<V>(invstd + c0, is);
  ld_params<V>(coef + c0, k0);
  ld_params<V>(coef + C + c0, k1);
  ld_params<V>(coef + 2 * C + c0, k2);
  float sc[V], sh[V];
  if constexpr (MASKY) {
    ld_params<V>(msc + c0, sc);
    ld_params<V>(msh + c0, sh);
  }
  const T* __restrict__ y2 = static_cast<const T*>(d2.y2);
  T* __restrict__ dy2 = static_cast<T*>(d2.dy2);
  float mu2[V], is2[V], j0[V], j1[V], j2[V];
  if constexpr (DUAL) {
    ld_params<V>(d2.mean2 + c0, mu2);
    ld_params<V>(d2.invstd2 + c0, is2);
    ld_params<V>(d2.coef2 + c0, j0);
    ld_params<V>(d2.coef2 + C + c0, j1);
    ld_params<V>(d2.coef2 + 2 * C + c0, j2);
  }
  auto one = [&](int64_t q, const float* gv0, const float* yv, const float* ov,
                 const float* y2v) {
    float gv[V], dv[V], dv2[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      if constexpr (MASKY) gv[e] = bn_affine(yv[e], sc[e], sh[e]) > 0.f ? gv0[e] : 0.f;
      else gv[e] = (relu_out && !(ov[e] > 0.f)) ? 0.f : gv0[e];
      const float xh = (yv[e] - mu[e]) * is[e];
      dv[e] = k0[e] * gv[e] - k1[e] - xh * k2[e];
      if constexpr (DUAL) {
        const float xh2 = (y2v[e] - mu2[e]) * is2[e];
        dv2[e] = j0[e] * gv[e] - j1[e] - xh2 * j2[e];
      }
    }
    Chunk<T>::store(dy + q * V, dv);
    if constexpr (DUAL) Chunk<T>::store(dy2 + q * V, dv2);
    if (gmask) Chunk<T>::store(gmask + q * V, gv);
  };
  // g2 (may be NULL): second gradient of the same output, summed as torch accumulates it
  auto add_g2 = [&](int64_t qq, float* gv) {
    float hv[V];
    Chunk<T>::load(g2 + qq * V, hv);
#pragma unroll
    for (int e = 0; e < V; ++e) gv[e] = as_stored<T>(gv[e] + hv[e]);
  };
  int64_t q = t0;
  for (; q + stride < nv; q += 2 * stride) {
    float g0[V], g1[V], y0[V], y1[V], o0[V], o1[V], z0[V], z1[V];
    Chunk<T>::load(g_at(q), g0);
    Chunk<T>::load(g_at(q + stride), g1);
    if constexpr (G2) {
      add_g2(q, g0);
      add_g2(q + stride, g1);
    }
    Chunk<T>::load(y + q * V, y0);
    Chunk<T>::load(y + (q + stride) * V, y1);
    if (relu_out) {
      Chunk<T>::load(relu_out + q * V, o0);
      Chunk<T>::load(relu_out + (q + stride) * V, o1);
    }
    if constexpr (DUAL) {
      Chunk<T>::load(y2 + q * V, z0);
      Chunk<T>::load(y2 + (q + stride) * V, z1);
    }
    one(q, g0, y0, o0, z0);
    one(q + stride, g1, y1, o1, z1);
  }
  if (q < nv) {
    float g0[V], y0[V], o0[V], z0[V];
    Chunk<T>::load(g_at(q), g0);
    if constexpr (G2) add_g2(q, g0);
    Chunk<T>::load(y + q * V, y0);
    if (relu_out) Chunk<T>::load(relu_out + q * V, o0);
    if constexpr (DUAL) Chunk<T>::load(y2 + q * V, z0);
    one(q, g0, y0, o0, z0);
  }
}

template <typename T, int V>
__global__ void bn_bwd_apply_kernel(int64_t M, int C, const T* __restrict__ g,
                                    const T* __restrict__ relu_out, const T* __restrict__ y,
                                    const float* __restrict__ mean,
                                    const float* __restrict__ invstd,
                                    const float* __restrict__ coef, T* __restrict__ dy,
                                    T* __restrict__ gmask) {
  const int64_t nv = M * C / V;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nv;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q * V;
    const int c0 = (int)(i % C);
    float gv[V], yv[V], ov[V], dv[V];
    if constexpr (V == Chunk<T>::N) {
      Chunk<T>::load(g + i, gv);
      Chunk<T>::load(y + i, yv);
      if (relu_out) Chunk<T>::load(relu_out + i, ov);
    } else {
      for (int e = 0; e < V; ++e) {
        gv[e] = Elt<T>::ld(g, i + e);
        yv[e] = Elt<T>::ld(y, i + e);
        if (relu_out) ov[e] = Elt<T>::ld(relu_out, i + e);
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int c = c0 + e;
      if (relu_out && !(ov[e] > 0.f)) gv[e] = 0.f;
      const float xh = (yv[e] - mean[c]) * invstd[c];
      dv[e] = coef[c] * gv[e] - coef[C + c] - xh * coef[2 * C + c];
    }
    if constexpr (V == Chunk<T>::N) {
      Chunk<T>::store(dy + i, dv);
      if (gmask) Chunk<T>::store(gmask + i, gv);
    } else {
      for (int e = 0; e < V; ++e) {
        Elt<T>::st(dy, i + e, dv[e]);
        if (gmask) Elt<T>::st(gmask, i + e, gv[e]);
      }
    }
  }
}

template <typename T>
__global__ void relu_bwd_kernel(int64_t n, const T* __restrict__ g, const T* __restrict__ out,
                                T* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    Elt<T>::st(dx, i, Elt<T>::ld(out, i) > 0.f ? Elt<T>::ld(g, i) : 0.f);
}

template <typename T>
__global__ void relu_fwd_kernel(int64_t n, const T* __restrict__ x, T* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = Elt<T>::ld(x, i);
    Elt<T>::st(y, i, v > 0.f ? v : (v != v ? v : 0.f));
  }
}

template <typename T>
__global__ void add_kernel(int64_t n, const T* __restrict__ a, const T* __restrict__ b,
                           T* __restrict__ o) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    Elt<T>::st(o, i, Elt<T>::ld(a, i) + Elt<T>::ld(b, i));
}

unsigned ew_grid(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 256 * 16));
}

bool dt_ok(int dtype) { return dtype == MMAD_F32 || dtype == MMAD_BF16; }

}  // namespace

extern "C" {

int64_t mmad_bn_stats_parts(int64_t m, int c) {
  (void)c;
  return m > 0 ? part_plan(m).nparts : -1;
}
int64_t mmad_bn_bwd_parts(int64_t m, int c) { return mmad_bn_stats_parts(m, c); }

int mmad_bn_stats(int dtype, int64_t m, int c, const void* y, float* parts, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!y || !parts) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return launch_colsum<u16, 0>(m, c, y, nullptr, nullptr, nullptr, nullptr, parts,
                                 as_stream(stream));
  return launch_colsum<float, 0>(m, c, y, nullptr, nullptr, nullptr, nullptr, parts,
                                 as_stream(stream));
}

int mmad_bn_parts_fold(int c, int nparts, const float* parts, int group, float* out,
                       void* stream) {
  if (c <= 0 || nparts <= 0 || group <= 0) return MMAD_EBADSHAPE;
  if (!parts || !out) return MMAD_ENULL;
  hipLaunchKernelGGL(parts_fold_kernel, dim3((unsigned)cdiv(nparts, group)), dim3(256), 0,
                     as_stream(stream), c, nparts, group, parts, out);
  return launch_status();
}

// column sums (conv bias gradient) using `parts` as scratch ([parts][2][c] floats)
int mmad_colsum_ws(int dtype, int64_t m, int c, const void* y, float* parts, float* out,
                   void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!y || !parts || !out) return MMAD_ENULL;
  int rc = dtype == MMAD_BF16
               ? launch_colsum<u16, 2>(m, c, y, nullptr, nullptr, nullptr, nullptr, parts,
                                       as_stream(stream))
               : launch_colsum<float, 2>(m, c, y, nullptr, nullptr, nullptr, nullptr, parts,
                                         as_stream(stream));
  if (rc) return rc;
  hipLaunchKernelGGL(sum_only_finalize_kernel, dim3((unsigned)cdiv(c, FC)), dim3(1024), 0,
                     as_stream(stream), c, part_plan(m).nparts, parts, out);
  return launch_status();
}

int mmad_bn_finalize2(int c, int64_t count, const mmad_bn_fin* a, const mmad_bn_fin* b,
                      void* stream) {
  if (c <= 0 || count <= 0) return MMAD_EBADSHAPE;
  if (!a || !b) return MMAD_ENULL;
  for (const mmad_bn_fin* f : {a, b}) {
    if (f->training && (!f->parts || f->nparts <= 0)) return MMAD_ENULL;
    if (!f->training && (!f->running_mean || !f->running_var)) return MMAD_ENULL;
  }
  hipLaunchKernelGGL(bn_finalize2_kernel, dim3((unsigned)cdiv(c, FC), 2), dim3(1024), 0,
                     as_stream(stream), c, count, *a, *b);
  return launch_status();
}

int mmad_bn_finalize(int c, int64_t count, int nparts, const float* parts, const float* gamma,
                     const float* beta, float* running_mean, float* running_var,
                     float momentum, float eps, int training, float* mean, float* invstd,
                     float* scale, float* shift, int64_t* num_batches_tracked, void* stream) {
  if (c <= 0 || count <= 0) return MMAD_EBADSHAPE;
  if (training && (!parts || nparts <= 0)) return MMAD_ENULL;
  if (!training && (!running_mean || !running_var)) return MMAD_ENULL;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)cdiv(c, FC)), dim3(1024), 0,
                     as_stream(stream), c, count, nparts, parts, gamma, beta, running_mean,
                     running_var, momentum, eps, training, mean, invstd, scale, shift,
                     num_batches_tracked);
  return launch_status();
}

int mmad_scale_shift_act(int dtype, int64_t m, int c, const void* y, const float* scale,
                         const float* shift, const void* res, const float* rscale,
                         const float* rshift, int relu, void* out, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!y || !scale || !shift || !out) return MMAD_ENULL;
  if ((rscale == nullptr) != (rshift == nullptr)) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  const int epc = dtype == MMAD_BF16 ? 8 : 4;
  const int rk = res == nullptr ? 0 : (rscale == nullptr ? 1 : 2);
  const unsigned grid = ew_grid(m * c / epc);
#define SSA(T, R)                                                                          \
  hipLaunchKernelGGL((scale_shift_act_kernel<T, R>), dim3(grid), dim3(256), 0, st, m, c,  \
                     (const T*)y, scale, shift, (const T*)res, rscale, rshift, relu, (T*)out)
#define SSAF(T, R)                                                                         \
  hipLaunchKernelGGL((scale_shift_act_fc_kernel<T, R>), dim3(grid), dim3(256), 0, st,        \
                     m * c / epc, c / epc, (const T*)y, scale, shift, (const T*)res, rscale,  \
                     rshift, relu, (T*)out)
  if (c % epc == 0 && is_pow2(c / epc) && c / epc <= 256) {
    if (dtype == MMAD_BF16) {
      if (rk == 0) SSAF(u16, 0); else if (rk == 1) SSAF(u16, 1); else SSAF(u16, 2);
    } else {
      if (rk == 0) SSAF(float, 0); else if (rk == 1) SSAF(float, 1); else SSAF(float, 2);
    }
  } else if (c % epc == 0) {
    if (dtype == MMAD_BF16) {
      if (rk == 0) SSA(u16, 0); else if (rk == 1) SSA(u16, 1); else SSA(u16, 2);
    } else {
      if (rk == 0) SSA(float, 0); else if (rk == 1) SSA(float, 1); else SSA(float, 2);
    }
  } else if (dtype == MMAD_BF16) {
    hipLaunchKernelGGL(scale_shift_act_scalar_kernel<u16>, dim3(ew_grid(m * c)), dim3(256), 0,
                       st, m, c, (const u16*)y, scale, shift, (const u16*)res, rscale, rshift,
                       relu, (u16*)out);
  } else {
    hipLaunchKernelGGL(scale_shift_act_scalar_kernel<float>, dim3(ew_grid(m * c)), dim3(256), 0,
                       st, m, c, (const float*)y, scale, shift, (const float*)res, rscale,
                       rshift, relu, (float*)out);
  }
#undef SSA
#undef SSAF
  return launch_status();
}

int mmad_bn_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* g2,
                       const void* relu_out, const void* y, const float* mean,
                       const float* invstd, float* parts, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !y || !mean || !invstd || !parts) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return launch_colsum<u16, 1>(m, c, y, g, relu_out, mean, invstd, parts, as_stream(stream),
                                 nullptr, nullptr, nullptr, g2);
  return launch_colsum<float, 1>(m, c, y, g, relu_out, mean, invstd, parts, as_stream(stream),
                                 nullptr, nullptr, nullptr, g2);
}

// BN + ReLU (no residual) backward with the ReLU mask recomputed from y: the same partial
// sums / input gradient as mmad_bn_bwd_reduce / _apply with relu_out, without reading it
int mmad_bn_relu_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* y,
                            const float* mean, const float* invstd, const float* scale,
                            const float* shift, float* parts, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !y || !mean || !invstd || !scale || !shift || !parts) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return launch_colsum<u16, 4>(m, c, y, g, nullptr, mean, invstd, parts, as_stream(stream),
                                 nullptr, scale, shift);
  return launch_colsum<float, 4>(m, c, y, g, nullptr, mean, invstd, parts, as_stream(stream),
                                 nullptr, scale, shift);
}

int mmad_bn_relu_bwd_apply(int dtype, int64_t m, int c, const void* g, const void* y,
                           const float* mean, const float* invstd, const float* scale,
                           const float* shift, const float* coef, void* dy, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !y || !mean || !invstd || !scale || !shift || !coef || !dy) return MMAD_ENULL;
  const int vv = dtype == MMAD_BF16 ? 8 : 4;
  if (!(c % vv == 0 && is_pow2(c / vv) && c / vv <= 256)) return MMAD_EUNSUPPORTED;
  const int64_t nv = m * c / vv;
  hipStream_t st = as_stream(stream);
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_fc_kernel<u16, true>), dim3(ew_grid(nv)), dim3(256), 0, st,
                       nv, c / vv, c, (const u16*)g, (const u16*)nullptr, (const u16*)y, mean,
                       invstd, coef, (u16*)dy, (u16*)nullptr, scale, shift);
  else
    hipLaunchKernelGGL((bn_bwd_apply_fc_kernel<float, true>), dim3(ew_grid(nv)), dim3(256), 0,
                       st, nv, c / vv, c, (const float*)g, (const float*)nullptr,
                       (const float*)y, mean, invstd, coef, (float*)dy, (float*)nullptr, scale,
                       shift);
  return launch_status();
}

int mmad_bnpool_bwd_reduce(int dtype, int64_t m, int c, const void* g, const void* g2,
                           void* gsum, const uint8_t* argmax, const void* ymax,
                           const float* mean, const float* invstd, float* parts,
                           void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !argmax || !ymax || !mean || !invstd || !parts) return MMAD_ENULL;
  if (g2 && !gsum) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    return launch_colsum<u16, 3>(m, c, ymax, g, nullptr, mean, invstd, parts, as_stream(stream),
                                 argmax, nullptr, nullptr, g2, gsum);
  return launch_colsum<float, 3>(m, c, ymax, g, nullptr, mean, invstd, parts, as_stream(stream),
                                 argmax, nullptr, nullptr, g2, gsum);
}

int mmad_bn_fold(int c, const float* gamma, const float* beta, const float* running_mean,
                 const float* running_var, float eps, const float* conv_bias, float* scale,
                 float* bias, void* stream) {
  if (c <= 0) return MMAD_EBADSHAPE;
  if (!running_mean || !running_var || !scale || !bias) return MMAD_ENULL;
  hipLaunchKernelGGL(bn_fold_kernel, dim3((unsigned)cdiv(c, 256)), dim3(256), 0,
                     as_stream(stream), c, gamma, beta, running_mean, running_var, eps, conv_bias,
                     scale, bias);
  return launch_status();
}

int mmad_bn_bwd_finalize(int c, int64_t count, int nparts, const float* parts,
                         const float* gamma, const float* invstd, int training, float* dgamma,
                         float* dbeta, float* coef, void* stream) {
  if (c <= 0 || count <= 0 || nparts <= 0) return MMAD_EBADSHAPE;
  if (!parts || !invstd || !coef) return MMAD_ENULL;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((unsigned)cdiv(c, FC)), dim3(1024), 0,
                     as_stream(stream), c, count, nparts, parts, gamma, invstd, training,
                     dgamma, dbeta, coef);
  return launch_status();
}

int mmad_bn_bwd_apply(int dtype, int64_t m, int c, const void* g, const void* g2,
                      const void* relu_out, const void* y, const float* mean,
                      const float* invstd, const float* coef, void* dy, void* gmask,
                      void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !y || !mean || !invstd || !coef || !dy) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
#define APPLY(T, V)                                                                          \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, V>), dim3(ew_grid(m * c / V)), dim3(256), 0, st, \
                     m, c, (const T*)g, (const T*)relu_out, (const T*)y, mean, invstd, coef,  \
                     (T*)dy, (T*)gmask)
  const int vv = dtype == MMAD_BF16 ? 8 : 4;
  if (c % vv == 0 && is_pow2(c / vv) && c / vv <= 256) {
    const int64_t nv = m * c / vv;
#define APPLYFC(T, G)                                                                         \
  hipLaunchKernelGGL((bn_bwd_apply_fc_kernel<T, false, false, G>), dim3(ew_grid(nv)), dim3(256), \
                     0, st, nv, c / vv, c, (const T*)g, (const T*)relu_out, (const T*)y, mean,  \
                     invstd, coef, (T*)dy, (T*)gmask, nullptr, nullptr, BwdApply2{},           \
                     (const T*)g2)
    if (dtype == MMAD_BF16) {
      if (g2 != nullptr) APPLYFC(u16, true); else APPLYFC(u16, false);
    } else {
      if (g2 != nullptr) APPLYFC(float, true); else APPLYFC(float, false);
    }
#undef APPLYFC
    return launch_status();
  }
  if (g2 != nullptr) return MMAD_EUNSUPPORTED;   // generic layouts: the caller adds g2 first
  if (dtype == MMAD_BF16) {
    if (c % 8 == 0) APPLY(u16, 8); else APPLY(u16, 1);
  } else {
    if (c % 4 == 0) APPLY(float, 4); else APPLY(float, 1);
  }
#undef APPLY
  return launch_status();
}

// Residual pair (bn2(y) + bn_r(y2), then ReLU): both BNs' backward from one read of g and
// the mask.  Same values, bit for bit, as reduce / finalize / apply called once per BN with
// the same g and relu_out.  Fixed-channel layouts only (MMAD_EUNSUPPORTED otherwise: the
// caller falls back to the per-BN calls).
int mmad_bn_bwd_reduce2(int dtype, int64_t m, int c, const void* g, const void* g2,
                        int64_t g_rows, const void* relu_out, const void* y, const float* mean,
                        const float* invstd, const void* y2,
                        const float* mean2, const float* invstd2, float* parts, float* parts2,
                        void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !relu_out || !y || !mean || !invstd || !y2 || !mean2 || !invstd2 || !parts ||
      !parts2)
    return MMAD_ENULL;
  if (g_rows < 0 || (g_rows > 0 && (m % g_rows || m >= (int64_t(1) << 31))))
    return MMAD_EBADSHAPE;
  const PartPlan pp = part_plan(m);
  hipStream_t st = as_stream(stream);
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    constexpr int VEC = Chunk<T>::N;
    int slabs = 1;
    while (c % (slabs * 2 * VEC) == 0 && c / (slabs * VEC) > 256) slabs *= 2;
    if (!(c % (slabs * VEC) == 0 && c / (slabs * VEC) <= 256)) return MMAD_EUNSUPPORTED;
    auto k = g_rows > 0 ? (g2 != nullptr ? colsum_kernel<T, 1, VEC, true, true, true>
                                          : colsum_kernel<T, 1, VEC, true, false, true>)
                        : (g2 != nullptr ? colsum_kernel<T, 1, VEC, true, true>
                                          : colsum_kernel<T, 1, VEC, true, false>);
    hipLaunchKernelGGL(k, dim3((unsigned)pp.nparts, slabs), dim3(256), 0, st, m, c, pp.rpp,
                       (const T*)y, (const T*)g, (const T*)relu_out, mean, invstd, parts,
                       nullptr, nullptr, nullptr, (const T*)y2, mean2, invstd2, parts2,
                       (const T*)g2, (T*)nullptr, (uint32_t)g_rows);
    return launch_status();
  };
  return dtype == MMAD_BF16 ? go(u16{}) : go(float{});
}

int mmad_bn_bwd_finalize2(int c, int64_t count, int nparts, const float* parts,
                          const float* gamma, const float* invstd, int training, float* dgamma,
                          float* dbeta, float* coef, const float* parts2, const float* gamma2,
                          const float* invstd2, int training2, float* dgamma2, float* dbeta2,
                          float* coef2, void* stream) {
  if (c <= 0 || count <= 0 || nparts <= 0) return MMAD_EBADSHAPE;
  if (!parts || !invstd || !coef || !parts2 || !invstd2 || !coef2) return MMAD_ENULL;
  const BwdFin a{parts, gamma, invstd, training, dgamma, dbeta, coef};
  const BwdFin b{parts2, gamma2, invstd2, training2, dgamma2, dbeta2, coef2};
  hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3((unsigned)cdiv(c, FC), 2), dim3(1024), 0,
                     as_stream(stream), c, count, nparts, a, b);
  return launch_status();
}

int mmad_bn_bwd_apply2(int dtype, int64_t m, int c, const void* g, const void* g2,
                       int64_t g_rows, const void* relu_out, const void* y, const float* mean, const float* invstd, const float* coef,
                       void* dy, const void* y2, const float* mean2, const float* invstd2,
                       const float* coef2, void* dy2, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (m <= 0 || c <= 0) return MMAD_EBADSHAPE;
  if (!g || !relu_out || !y || !mean || !invstd || !coef || !dy || !y2 || !mean2 || !invstd2 ||
      !coef2 || !dy2)
    return MMAD_ENULL;
  const int vv = dtype == MMAD_BF16 ? 8 : 4;
  if (!(c % vv == 0 && is_pow2(c / vv) && c / vv <= 256)) return MMAD_EUNSUPPORTED;
  const int64_t nv = m * c / vv;
  const BwdApply2 d2{y2, mean2, invstd2, coef2, dy2};
  hipStream_t st = as_stream(stream);
  if (g_rows < 0 || (g_rows > 0 && (m % g_rows || m >= (int64_t(1) << 31))))
    return MMAD_EBADSHAPE;
#define APPLY2(T, G, B)                                                                      \
  hipLaunchKernelGGL((bn_bwd_apply_fc_kernel<T, false, true, G, B>), dim3(ew_grid(nv)),       \
                     dim3(256), 0, st, nv, c / vv, c, (const T*)g, (const T*)relu_out,        \
                     (const T*)y, mean, invstd, coef, (T*)dy, (T*)nullptr, nullptr, nullptr,  \
                     d2, (const T*)g2, (uint32_t)g_rows)
#define APPLY2G(T, B)                                                                        \
  do {                                                                                       \
    if (g2 != nullptr) APPLY2(T, true, B); else APPLY2(T, false, B);                         \
  } while (0)
  if (dtype == MMAD_BF16) {
    if (g_rows > 0) APPLY2G(u16, true); else APPLY2G(u16, false);
  } else {
    if (g_rows > 0) APPLY2G(float, true); else APPLY2G(float, false);
  }
#undef APPLY2G
#undef APPLY2
  return launch_status();
}

int mmad_relu_bwd(int dtype, int64_t n, const void* g, const void* out, void* dx, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!g || !out || !dx) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(relu_bwd_kernel<u16>, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream),
                       n, (const u16*)g, (const u16*)out, (u16*)dx);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0,
                       as_stream(stream), n, (const float*)g, (const float*)out, (float*)dx);
  return launch_status();
}

int mmad_relu_fwd(int dtype, int64_t n, const void* x, void* y, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!x || !y) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(relu_fwd_kernel<u16>, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream),
                       n, (const u16*)x, (u16*)y);
  else
    hipLaunchKernelGGL(relu_fwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0,
                       as_stream(stream), n, (const float*)x, (float*)y);
  return launch_status();
}

int mmad_add(int dtype, int64_t n, const void* a, const void* b, void* out, void* stream) {
  if (!dt_ok(dtype)) return MMAD_EBADDTYPE;
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!a || !b || !out) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(add_kernel<u16>, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), n,
                       (const u16*)a, (const u16*)b, (u16*)out);
  else
    hipLaunchKernelGGL(add_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, as_stream(stream), n,
                       (const float*)a, (const float*)b, (float*)out);
  return launch_status();
}

}  // extern "C"
