// Adam step fused with the bf16 weight repack, gfx950 (the captured training step's
// optimizer: graph_step.GraphedTrainStep with fused_optim.AdamRepack).
//
// Replaces, in one launch: torch's capturable fused Adam over every param group (the
// reference's optimizer, anat_cnn.py:111-126 -- one `_foreach_add_` of the step counters plus
// one fused multi-tensor launch per learning rate) AND the next step's weight repack
// (mmad_conv_pack_dual_batch, volume_ops.PackPlan): a conv weight's 16 co x 16 ci x taps tile
// is updated in registers and its new values leave as the fp32 master AND as both bf16
// layouts, so the fp32 weights are read once per step instead of twice.
//
// Arithmetic: ATen's fused Adam (ATen/native/cuda/fused_adam_utils.cuh, torch 2.10:
// FusedAdamMathFunctor / adam_math, ADAM_MODE::ORIGINAL, amsgrad off, maximize off, no grad
// scaler) operation for operation and type for type -- the betas, eps and weight decay are
// doubles, the bias corrections are computed in double and handed to the math as floats, lr
// is the group's device float read as a double -- so the update is bit-identical to
// torch.optim.Adam(fused=True) (tests/test_adam_repack_gpu.py).
//
// Step counters: torch increments each parameter's device `step` before its update reads it.
// Here every block reads step and updates with step + 1; the block that finishes a job last
// (a per-job arrival counter, device-scope atomics; every block has read step before it
// arrives) stores step + 1 and resets the counter for the next replay.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int FLAT = NT * 16;             // elements per block of a plain (not repacked) job

struct AdamConst {
  double lr, beta1, beta2, eps, wd;
  float bc1, bc2s;
};

// adam_math of fused_adam_utils.cuh: same expressions, same operand types
__device__ __forceinline__ float adam_elem(const AdamConst& k, float param, float grad,
                                           float& exp_avg, float& exp_avg_sq) {
  if (k.wd != 0) grad += param * k.wd;
  exp_avg = k.beta1 * exp_avg + (1 - k.beta1) * grad;
  exp_avg_sq = k.beta2 * exp_avg_sq + (1 - k.beta2) * grad * grad;
  const float step_size = k.lr / k.bc1;
  const float denom = (sqrtf(exp_avg_sq) / k.bc2s) + k.eps;
  param -= step_size * exp_avg / denom;
  return param;
}

__device__ __forceinline__ bool al16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

__global__ __launch_bounds__(NT) void adam_repack_kernel(const mmad_adam_job* __restrict__ jobs,
                                                         int njobs,
                                                         const int* __restrict__ block_job,
                                                         int* __restrict__ arrivals) {
  __shared__ float tile[16 * 27 * 17];
  int lo = 0, hi = njobs - 1;
  const int64_t bid = blockIdx.x;
  if (block_job != nullptr) {
    lo = block_job[bid];              // one load instead of a chain of ~12 dependent ones
  } else {
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
    }
  }
  const mmad_adam_job& jb = jobs[lo];
  const int64_t t = bid - jb.tile0;
  // FusedAdamMathFunctor: step read as float, bias corrections in double (pow(double,
  // double)), then narrowed to the math's opmath floats
  const float step = *jb.step + 1.0f;
  AdamConst k;
  k.lr = (double)*jb.lr;
  k.beta1 = jb.beta1;
  k.beta2 = jb.beta2;
  k.eps = jb.eps;
  k.wd = jb.weight_decay;
  const double bc1 = 1 - pow(jb.beta1, (double)step);
  const double bc2 = 1 - pow(jb.beta2, (double)step);
  k.bc1 = (float)bc1;
  k.bc2s = (float)sqrt(bc2);
  float* __restrict__ P = jb.param;
  const float* __restrict__ G = jb.grad;
  float* __restrict__ M = jb.exp_avg;
  float* __restrict__ Q = jb.exp_avg_sq;
  const bool vec = al16(P) && al16(G) && al16(M) && al16(Q);

  if (jb.w_fwd == nullptr || jb.unf_kw > 0) {
    // plain job: elements [t * FLAT, (t + 1) * FLAT); the unfolded stem: block t = output
    // channel t (its taps * unf_kw weights, then its packed row)
    const int64_t per = (int64_t)jb.taps * jb.unf_kw;
    const int64_t e0 = jb.unf_kw > 0 ? t * per : t * FLAT;
    const int64_t e1 = jb.unf_kw > 0 ? e0 + per : min(jb.numel, e0 + FLAT);
    if (vec && ((e0 | e1) & 3) == 0) {
#pragma unroll 2
      for (int64_t e = e0 + threadIdx.x * 4; e < e1; e += NT * 4) {
        const f32x4 p = *reinterpret_cast<const f32x4*>(P + e);
        const f32x4 g = *reinterpret_cast<const f32x4*>(G + e);
        f32x4 m = *reinterpret_cast<const f32x4*>(M + e);
        f32x4 v = *reinterpret_cast<const f32x4*>(Q + e);
        f32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float mq = m[q], vq = v[q];
          o[q] = adam_elem(k, p[q], g[q], mq, vq);
          m[q] = mq;
          v[q] = vq;
        }
        *reinterpret_cast<f32x4*>(P + e) = o;
        *reinterpret_cast<f32x4*>(M + e) = m;
        *reinterpret_cast<f32x4*>(Q + e) = v;
      }
    } else {
      for (int64_t e = e0 + threadIdx.x; e < e1; e += NT) {
        float m = M[e], v = Q[e];
        P[e] = adam_elem(k, P[e], G[e], m, v);
        M[e] = m;
        Q[e] = v;
      }
    }
    if (jb.unf_kw > 0) {
      // pack_weight_kernel's unfolded Cin = 1 forward layout (mode 2) of row co = t from the
      // updated weights this block just wrote: k = (kd * KH + kh) * 8 + kw, zero for kw >=
      // unf_kw and k >= taps * 8
      __syncthreads();
      u16* wf = reinterpret_cast<u16*>(jb.w_fwd) + t * jb.kpad;
      const int K = jb.taps * 8, kw = jb.unf_kw;
      for (int kk = threadIdx.x; kk < jb.kpad; kk += NT) {
        float v = 0.f;
        if (kk < K) {
          const int tap = kk >> 3, c = kk & 7;
          if (c < kw) v = P[e0 + tap * kw + c];
        }
        Elt<u16>::st(wf, kk, v);
      }
    }
  } else {
    // repacked conv weight: tile t = (co block, ci block) of 16 x 16 x taps, as
    // pack_dual_kernel (conv.hip) -- each co's 16 * T floats are contiguous
    const int T = jb.taps, CI = jb.ci, CO = jb.co;
    const int nci = CI / 16;
    const int co0 = (int)(t / nci) * 16, ci0 = (int)(t % nci) * 16;
    const int per_co = 16 * T, q4 = per_co / 4;
    if (vec) {
#pragma unroll 2
      for (int e = threadIdx.x; e < 16 * q4; e += NT) {
        const int col = e / q4, rem0 = (e % q4) * 4;
        const int64_t o = ((int64_t)(co0 + col) * CI + ci0) * T + rem0;
        const f32x4 p = *reinterpret_cast<const f32x4*>(P + o);
        const f32x4 g = *reinterpret_cast<const f32x4*>(G + o);
        f32x4 m = *reinterpret_cast<const f32x4*>(M + o);
        f32x4 v = *reinterpret_cast<const f32x4*>(Q + o);
        f32x4 w;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float mq = m[q], vq = v[q];
          w[q] = adam_elem(k, p[q], g[q], mq, vq);
          m[q] = mq;
          v[q] = vq;
          const int rem = rem0 + q, cil = rem / T, tap = rem % T;
          tile[(col * T + tap) * 17 + cil] = w[q];
        }
        *reinterpret_cast<f32x4*>(P + o) = w;
        *reinterpret_cast<f32x4*>(M + o) = m;
        *reinterpret_cast<f32x4*>(Q + o) = v;
      }
    } else {
      for (int e = threadIdx.x; e < 16 * per_co; e += NT) {
        const int col = e / per_co, rem = e % per_co;
        const int64_t o = ((int64_t)(co0 + col) * CI + ci0) * T + rem;
        float m = M[o], v = Q[o];
        const float w = adam_elem(k, P[o], G[o], m, v);
        P[o] = w;
        M[o] = m;
        Q[o] = v;
        tile[(col * T + rem % T) * 17 + rem / T] = w;
      }
    }
    __syncthreads();
    u16* wf = reinterpret_cast<u16*>(jb.w_fwd);
    u16* wd = reinterpret_cast<u16*>(jb.w_dgrad);
    const int items = 16 * T * 2;
    for (int e = threadIdx.x; e < 2 * items; e += NT) {
      const int it = e % items, half = it & 1, rest = it >> 1;
      u32x4 v;
      if (e < items) {                               // forward: [co][tap][ci]
        const int col = rest / T, tap = rest % T;
        const float* tp = tile + (col * T + tap) * 17 + half * 8;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = pack_bf16x2(tp[2 * q], tp[2 * q + 1]);
        *reinterpret_cast<u32x4*>(wf + (int64_t)(co0 + col) * T * CI + (int64_t)tap * CI + ci0 +
                                  half * 8) = v;
      } else {                                       // dgrad: [ci][tap'][co]
        const int cil = rest / T, tap = rest % T;
        const int tq = jb.flip ? T - 1 - tap : tap;
        const float* tp = tile + ((half * 8) * T + tap) * 17 + cil;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = pack_bf16x2(tp[(2 * q) * T * 17], tp[(2 * q + 1) * T * 17]);
        *reinterpret_cast<u32x4*>(wd + (int64_t)(ci0 + cil) * T * CO + (int64_t)tq * CO + co0 +
                                  half * 8) = v;
      }
    }
  }
  // step counter: every wave of every block has read *jb.step (its value fed the bias
  // corrections above) before its block arrives -- the barrier orders all of this block's
  // waves before thread 0's arrival on every branch; the last to arrive stores step + 1 and
  // re-arms the counter
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = atomicAdd(arrivals + lo, 1);
    if (prev == (int)jb.ntiles - 1) {
      *jb.step = step;
      atomicExch(arrivals + lo, 0);
    }
  }
}

}  // namespace

extern "C" {

int64_t mmad_adam_job_tiles(const mmad_adam_job* job) {
  if (job == nullptr || job->numel <= 0) return 0;
  if (job->w_fwd != nullptr && job->unf_kw > 0) return job->co;    // one block per row
  if (job->w_fwd != nullptr) return (int64_t)(job->co / 16) * (job->ci / 16);
  return (job->numel + FLAT - 1) / FLAT;
}

int mmad_adam_repack(int njobs, const mmad_adam_job* jobs_device, const int* block_job,
                     int64_t total_tiles, int* arrivals, void* stream) {
  if (njobs <= 0 || total_tiles <= 0) return MMAD_OK;
  if (jobs_device == nullptr || arrivals == nullptr || total_tiles > 0x7fffffff)
    return MMAD_ENULL;
  hipLaunchKernelGGL(adam_repack_kernel, dim3((unsigned)total_tiles), dim3(NT), 0,
                     as_stream(stream), jobs_device, njobs, block_job, arrivals);
  return launch_status();
}

}  // extern "C"
