// Classifier / late-fusion MLP head, losses, casts and dropout, gfx950.
//
// Replaces nn.Linear (+ReLU) of the conv_seg head (pkg/models/mri_models/anat_cnn.py:68-76),
// reduce_dim_mri / stage2out / cls2 and the feature concat of Anat_PET_CNN
// (pkg/models/fusion_models/anat_pet_fusion.py:42-51, :76), the focal loss
// (pkg/loss_functions/focalloss.py:19-39), the weighted cross entropy (anat_cnn.py:84-85),
// the fp32 input cast / fp64 logits cast of general_step (anat_cnn.py:102-104) and
// nn.Dropout of Small_PET_CNN (pkg/models/pet_models/pet_cnn.py:27-29, :38-39).
//
// The head is tiny (B <= 64 rows, <= 2048 features): one wave per output dot product
// with lane-strided coalesced reads and a shuffle reduction; no MFMA (a 16-row MFMA
// tile would be >= 75 % padding at these batch sizes).
#include "common.h"

namespace {

// y[b][o] = act(sum_i x[b][i] * w[o][i] + bias[o]); one wave per (b, o)
__global__ __launch_bounds__(256) void linear_fwd_kernel(int B, int IN, int OUT,
                                                         const float* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         int relu, float* __restrict__ y) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= B * OUT) return;
  const int b = wid / OUT, o = wid % OUT;
  float s = 0.f;
  for (int i = lane; i < IN; i += 64) s += x[(int64_t)b * IN + i] * w[(int64_t)o * IN + i];
  s = wave_sum(s);
  if (lane == 0) {
    if (bias) s += bias[o];
    y[(int64_t)b * OUT + o] = relu ? fmaxf(s, 0.f) : s;
  }
}

// Linear backward in one launch: blocks [0, nbx) compute dx, the rest dw / dbias.
//   dx[b][i] = sum_o g[b][o] w[o][i]   (thread per (b, i), coalesced over i)
//   dw[o][i] = sum_b g[b][o] x[b][i];  dbias[o] = sum_b g[b][o]
// g = dy, or with ymask (the forward's ReLU output) g = ymask > 0 ? dy : 0 -- the fused
// Linear+ReLU's backward, same values as a separate ReLU-backward pass
__global__ void linear_bwd_kernel(int B, int IN, int OUT, int nbx, const float* __restrict__ x,
                                  const float* __restrict__ w, const float* __restrict__ dy,
                                  const float* __restrict__ ymask, float* __restrict__ dx,
                                  float* __restrict__ dw, float* __restrict__ dbias) {
  auto gval = [&](int64_t k) {
    const float v = dy[k];
    return ymask == nullptr || ymask[k] > 0.f ? v : 0.f;
  };
  if ((int)blockIdx.x < nbx) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= (int64_t)B * IN) return;
    const int b = (int)(t / IN), i = (int)(t % IN);
    float s = 0.f;
    for (int o = 0; o < OUT; ++o) s += gval((int64_t)b * OUT + o) * w[(int64_t)o * IN + i];
    dx[t] = s;
    return;
  }
  const int64_t t = (blockIdx.x - nbx) * (int64_t)blockDim.x + threadIdx.x;
  if (dw != nullptr && t < (int64_t)OUT * IN) {
    const int o = (int)(t / IN), i = (int)(t % IN);
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += gval((int64_t)b * OUT + o) * x[(int64_t)b * IN + i];
    dw[t] = s;
  }
  if (dbias && t < OUT) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += gval((int64_t)b * OUT + t);
    dbias[t] = s;
  }
}

// AdaptiveAvgPool3d(1) -> Flatten -> Linear (-> ReLU) forward in one launch after the GAP's
// partial sums (mmad_gap_partial).  Block b: x[b][i] = (sum over p, in order, of
// ws[b][p][i]) / S -- gap_fold_kernel's arithmetic -- or ws[b][i] itself when P == 1, kept in
// LDS and in xs (the linear backward's input); then each wave takes outputs o = wave, wave +
// 8, ... with linear_fwd_kernel's dot product (lane-strided sum + wave_sum)
constexpr int GL_THREADS = 512, GL_MAX_IN = 4096;
__global__ __launch_bounds__(GL_THREADS) void gap_linear_fwd_kernel(
    int IN, int OUT, int P, float Sf, const float* __restrict__ ws, const float* __restrict__ w,
    const float* __restrict__ bias, int relu, float* __restrict__ xs, float* __restrict__ y) {
  __shared__ float xsh[GL_MAX_IN];
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < IN; i += GL_THREADS) {
    float xi;
    if (P > 1) {
      float acc = 0.f;
#pragma unroll 16
      for (int p = 0; p < P; ++p) acc += ws[((int64_t)b * P + p) * IN + i];
      xi = acc / Sf;
    } else {
      xi = ws[(int64_t)b * IN + i];
    }
    xsh[i] = xi;
    xs[(int64_t)b * IN + i] = xi;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int o = wave; o < OUT; o += GL_THREADS / 64) {
    float s = 0.f;
    for (int i = lane; i < IN; i += 64) s += xsh[i] * w[(int64_t)o * IN + i];
    s = wave_sum(s);
    if (lane == 0) {
      if (bias) s += bias[o];
      y[(int64_t)b * OUT + o] = relu ? fmaxf(s, 0.f) : s;
    }
  }
}

// its backward in one launch: linear_bwd_kernel with the input gradient leaving as the GAP's
// compact rows, rows[b][i] = T(dx[b][i] * inv) (gap_bwd_kernel's arithmetic, inv = 1 / S)
template <typename T>
__global__ void linear_gap_bwd_kernel(int B, int IN, int OUT, int nbx, float inv,
                                      const float* __restrict__ x, const float* __restrict__ w,
                                      const float* __restrict__ dy,
                                      const float* __restrict__ ymask, T* __restrict__ rows,
                                      float* __restrict__ dw, float* __restrict__ dbias) {
  auto gval = [&](int64_t k) {
    const float v = dy[k];
    return ymask == nullptr || ymask[k] > 0.f ? v : 0.f;
  };
  if ((int)blockIdx.x < nbx) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= (int64_t)B * IN) return;
    const int i = (int)(t % IN);
    const int b = (int)(t / IN);
    float s = 0.f;
    for (int o = 0; o < OUT; ++o) s += gval((int64_t)b * OUT + o) * w[(int64_t)o * IN + i];
    Elt<T>::st(rows, t, s * inv);
    return;
  }
  const int64_t t = (blockIdx.x - nbx) * (int64_t)blockDim.x + threadIdx.x;
  if (dw != nullptr && t < (int64_t)OUT * IN) {
    const int o = (int)(t / IN), i = (int)(t % IN);
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += gval((int64_t)b * OUT + o) * x[(int64_t)b * IN + i];
    dw[t] = s;
  }
  if (dbias && t < OUT) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += gval((int64_t)b * OUT + t);
    dbias[t] = s;
  }
}

struct ColList {
  const float* p[8];
  float* q[8];
  int w[8];
  int n;
};

__global__ void concat_kernel(int B, int total, ColList L, float* __restrict__ dst) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * total) return;
  const int b = (int)(t / total);
  int c = (int)(t % total);
  for (int k = 0; k < L.n; ++k) {
    if (c < L.w[k]) { dst[t] = L.p[k][(int64_t)b * L.w[k] + c]; return; }
    c -= L.w[k];
  }
}

__global__ void split_kernel(int B, int total, ColList L, const float* __restrict__ src) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * total) return;
  const int b = (int)(t / total);
  int c = (int)(t % total);
  for (int k = 0; k < L.n; ++k) {
    if (c < L.w[k]) { L.q[k][(int64_t)b * L.w[k] + c] = src[t]; return; }
    c -= L.w[k];
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(int64_t n, const TI* __restrict__ x, TO* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (sizeof(TO) == 2) {
      y[i] = f2bf((float)x[i]);                 // f64 -> f32 -> bf16, as torch does
    } else if constexpr (sizeof(TI) == 2) {
      y[i] = (TO)bf2f(x[i]);
    } else {
      y[i] = (TO)x[i];
    }
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__global__ void dropout_fwd_kernel(int64_t n, float p, uint64_t seed,
                                   const uint64_t* __restrict__ seed_dev, const T* __restrict__ x,
                                   T* __restrict__ y, uint8_t* __restrict__ keep) {
  const float sc = 1.f / (1.f - p);
  // a device-resident seed (drawn on the stream by the caller) keeps the mask fresh under
  // HIP-graph replay, where a host scalar would be frozen into the captured arguments
  if (seed_dev) seed = *seed_dev;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float u = (float)(mix64(seed * 0xD1342543DE82EF95ull + (uint64_t)i) >> 40) * 0x1p-24f;
    const bool k = u >= p;
    keep[i] = k;
    Elt<T>::st(y, i, k ? Elt<T>::ld(x, i) * sc : 0.f);
  }
}

template <typename T>
__global__ void dropout_bwd_kernel(int64_t n, float p, const T* __restrict__ g,
                                   const uint8_t* __restrict__ keep, T* __restrict__ dx) {
  const float sc = 1.f / (1.f - p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    Elt<T>::st(dx, i, keep[i] ? Elt<T>::ld(g, i) * sc : 0.f);
}

// mode 0: weighted CE (mean = sum w_y nll / sum w_y); mode 1: focal, pt detached.
// One block; thread per sample (loop), f64 throughout; block reduction in fixed order.
// TI = float: the logits arrive in fp32 and are widened on load (exactly, as the f64 cast
// general_step applies first); x64 (may be NULL) then receives that f64 copy.
template <typename TI>
__global__ __launch_bounds__(256) void loss_kernel(int B, int C, const TI* __restrict__ xin,
                                                   const int64_t* __restrict__ y,
                                                   const double* __restrict__ w, double gamma,
                                                   int mode, double* __restrict__ loss,
                                                   double* __restrict__ dx,
                                                   int* __restrict__ err,
                                                   double* __restrict__ x64) {
  __shared__ double red[2][256];
  struct Wide {
    const TI* p;
    __device__ double operator[](int64_t i) const { return (double)p[i]; }
  } x{xin};
  if (x64 != nullptr)
    for (int64_t i = threadIdx.x; i < (int64_t)B * C; i += blockDim.x) x64[i] = x[i];
  double num = 0.0, den = 0.0;
  const int igamma = (int)gamma;
  const bool int_gamma = (double)igamma == gamma && igamma >= 0 && igamma <= 16;
  double lse_first = 0.0;                        // this thread's first sample's lse, reused
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int64_t t = y[b];
    if (t < 0 || t >= C) { if (err) *err = 1; continue; }
    double mx = -__builtin_inf();
    for (int c = 0; c < C; ++c) mx = fmax(mx, x[(int64_t)b * C + c]);
    double se = 0.0;
    for (int c = 0; c < C; ++c) se += exp(x[(int64_t)b * C + c] - mx);
    const double lse = mx + log(se);
    if (b == (int)threadIdx.x) lse_first = lse;
    const double logpt = x[(int64_t)b * C + t] - lse;
    if (mode == 0) {
      const double wt = w ? w[t] : 1.0;
      num += wt * -logpt;
      den += wt;
    } else {
      const double pt = exp(logpt);
      double f;
      if (int_gamma) { f = 1.0; for (int k = 0; k < igamma; ++k) f *= (1.0 - pt); }
      else f = pow(1.0 - pt, gamma);
      num += -f * logpt;
      den += 1.0;
    }
  }
  red[0][threadIdx.x] = num;
  red[1][threadIdx.x] = den;
  __syncthreads();
  if (threadIdx.x == 0) {
    // threads >= B hold +0.0 partials: leaving them out changes no bit of the sums
    double a = 0.0, d = 0.0;
    const int nk = min((int)blockDim.x, B);
    for (int k = 0; k < nk; ++k) { a += red[0][k]; d += red[1][k]; }
    red[0][0] = a;
    red[1][0] = d;
    *loss = a / d;
  }
  __syncthreads();
  const double den_all = red[1][0];
  // d loss / d x[b][c] = coef_b * (softmax_bc - [c == t_b])
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const int64_t t = y[b];
    if (t < 0 || t >= C) continue;
    double lse = lse_first;
    if (b != (int)threadIdx.x) {
      double mx = -__builtin_inf();
      for (int c = 0; c < C; ++c) mx = fmax(mx, x[(int64_t)b * C + c]);
      double se = 0.0;
      for (int c = 0; c < C; ++c) se += exp(x[(int64_t)b * C + c] - mx);
      lse = mx + log(se);
    }
    double coef;
    if (mode == 0) {
      coef = (w ? w[t] : 1.0) / den_all;
    } else {
      const double pt = exp(x[(int64_t)b * C + t] - lse);
      double f;
      if (int_gamma) { f = 1.0; for (int k = 0; k < igamma; ++k) f *= (1.0 - pt); }
      else f = pow(1.0 - pt, gamma);
      coef = f / den_all;
    }
    for (int c = 0; c < C; ++c) {
      const double sm = exp(x[(int64_t)b * C + c] - lse);
      dx[(int64_t)b * C + c] = coef * (sm - (c == t ? 1.0 : 0.0));
    }
  }
}

// d logits = cast(dlogits * gloss (+ gout)): the loss's backward (autograd's f64 product with
// the incoming scalar gradient, plus the f64 logits' own gradient when they are used) and
// the f64 -> out_dtype cast's backward in one pass
__global__ void loss_bwd_kernel(int64_t n, const double* __restrict__ dl,
                                const double* __restrict__ gl, const double* __restrict__ go,
                                int out_dtype, void* __restrict__ dx) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = dl[i] * gl[0];
  if (go != nullptr) v = v + go[i];
  if (out_dtype == MMAD_F32) static_cast<float*>(dx)[i] = (float)v;
  else static_cast<double*>(dx)[i] = v;
}

// Bootstrap of the test-set classification metrics (pkg/models/base_model.py:219-239):
// one block per drawing; the drawing's confusion matrix is counted in LDS (integer adds, so
// the result does not depend on their order), then thread 0 evaluates torchmetrics-0.10
// macro F1 (classes with tp + fp + fn = 0 left out of the mean) and multiclass MCC (0 when
// a marginal is degenerate) in f64 and rounds to f32, as metric.compute() returns f32.
// pred = argmax of the f64 logits row, first index on ties (torch.argmax).
constexpr int BOOT_MAXC = 16;
__global__ __launch_bounds__(256) void bootstrap_kernel(int n, int C, const double* __restrict__ x,
                                                        const int64_t* __restrict__ y,
                                                        const int64_t* __restrict__ idx,
                                                        float* __restrict__ f1,
                                                        float* __restrict__ mcc) {
  __shared__ int cm[BOOT_MAXC * BOOT_MAXC];
  const int d = blockIdx.x;
  for (int i = threadIdx.x; i < C * C; i += blockDim.x) cm[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t s = idx[(int64_t)d * n + i];
    const double* row = x + s * C;
    int p = 0;
    double best = row[0];
    for (int c = 1; c < C; ++c)
      if (row[c] > best || (row[c] != row[c] && best == best)) { best = row[c]; p = c; }
    const int64_t t = y[s];
    if (t >= 0 && t < C) atomicAdd(&cm[t * C + p], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double f1sum = 0.0;
    int used = 0;
    double s = 0.0, tr = 0.0, tp_sum = 0.0, pp = 0.0, tt = 0.0;
    for (int c = 0; c < C; ++c) {
      double tk = 0.0, pk = 0.0;
      for (int j = 0; j < C; ++j) { tk += cm[c * C + j]; pk += cm[j * C + c]; }
      const double tp = cm[c * C + c], fp = pk - tp, fn = tk - tp;
      if (tp + fp + fn > 0) { f1sum += 2.0 * tp / (2.0 * tp + fp + fn); ++used; }
      s += tk; tr += tp; tp_sum += tk * pk; pp += pk * pk; tt += tk * tk;
    }
    f1[d] = (float)(used ? f1sum / used : 0.0);
    const double cov_tp = tr * s - tp_sum, cov_pp = s * s - pp, cov_tt = s * s - tt;
    mcc[d] = (float)(cov_pp * cov_tt == 0.0 ? 0.0 : cov_tp / sqrt(cov_tt * cov_pp));
  }
}

// out = (mean, unbiased std) of v[0..n) in f64, fixed-order block reduction
__global__ __launch_bounds__(256) void mean_std_kernel(int n, const float* __restrict__ v,
                                                       double* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += v[i];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int k = 0; k < (int)blockDim.x; ++k) a += red[k];
    red[0] = a / n;
  }
  __syncthreads();
  const double mu = red[0];
  __syncthreads();
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) q += (v[i] - mu) * (v[i] - mu);
  red[threadIdx.x] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0;
    for (int k = 0; k < (int)blockDim.x; ++k) a += red[k];
    out[0] = mu;
    out[1] = n > 1 ? sqrt(a / (n - 1)) : __builtin_nan("");
  }
}

unsigned grid_n(int64_t n, int block = 256) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, block), 256 * 16));
}

}  // namespace

extern "C" {

int mmad_linear_fwd(int b, int in, int out, const float* x, const float* w, const float* bias,
                    int relu, float* y, void* stream) {
  if (b <= 0 || in <= 0 || out <= 0) return MMAD_EBADSHAPE;
  if (!x || !w || !y) return MMAD_ENULL;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((unsigned)cdiv((int64_t)b * out, 4)), dim3(256), 0,
                     as_stream(stream), b, in, out, x, w, bias, relu, y);
  return launch_status();
}

int mmad_linear_bwd(int b, int in, int out, const float* x, const float* w, const float* dy,
                    float* dx, float* dw, float* dbias, void* stream) {
  return mmad_linear_bwd_ex(b, in, out, x, w, dy, nullptr, dx, dw, dbias, stream);
}

int mmad_linear_bwd_ex(int b, int in, int out, const float* x, const float* w, const float* dy,
                       const float* ymask, float* dx, float* dw, float* dbias, void* stream) {
  if (b <= 0 || in <= 0 || out <= 0) return MMAD_EBADSHAPE;
  if (!dy) return MMAD_ENULL;
  if (dx && !w) return MMAD_ENULL;
  if ((dw || dbias) && (!x || !dw)) return MMAD_ENULL;
  const int nbx = dx ? (int)cdiv((int64_t)b * in, 256) : 0;
  const int nbw = (dw || dbias) ? (int)cdiv(std::max<int64_t>((int64_t)out * in, out), 256) : 0;
  if (nbx + nbw == 0) return MMAD_OK;
  hipLaunchKernelGGL(linear_bwd_kernel, dim3((unsigned)(nbx + nbw)), dim3(256), 0,
                     as_stream(stream), b, in, out, nbx, x, w, dy, ymask, dx, dw, dbias);
  return launch_status();
}

int mmad_gap_linear_fwd(int b, int in, int out, int parts, int64_t s, const float* ws,
                        const float* w, const float* bias, int relu, float* xs, float* y,
                        void* stream) {
  if (b <= 0 || in <= 0 || out <= 0 || parts <= 0 || s <= 0) return MMAD_EBADSHAPE;
  if (in > GL_MAX_IN) return MMAD_EUNSUPPORTED;
  if (!ws || !w || !xs || !y) return MMAD_ENULL;
  hipLaunchKernelGGL(gap_linear_fwd_kernel, dim3((unsigned)b), dim3(GL_THREADS), 0,
                     as_stream(stream), in, out, parts, (float)s, ws, w, bias, relu, xs, y);
  return launch_status();
}

int mmad_linear_gap_bwd(int b, int in, int out, int64_t s, const float* x, const float* w,
                        const float* dy, const float* ymask, int rows_dtype, void* rows,
                        float* dw, float* dbias, void* stream) {
  if (b <= 0 || in <= 0 || out <= 0 || s <= 0) return MMAD_EBADSHAPE;
  if (!dy) return MMAD_ENULL;
  if (rows && !w) return MMAD_ENULL;
  if ((dw || dbias) && (!x || !dw)) return MMAD_ENULL;
  if (rows && rows_dtype != MMAD_BF16 && rows_dtype != MMAD_F32) return MMAD_EBADDTYPE;
  const int nbx = rows ? (int)cdiv((int64_t)b * in, 256) : 0;
  const int nbw = (dw || dbias) ? (int)cdiv(std::max<int64_t>((int64_t)out * in, out), 256) : 0;
  if (nbx + nbw == 0) return MMAD_OK;
  const float inv = 1.f / (float)s;
  if (rows_dtype == MMAD_BF16)
    hipLaunchKernelGGL(linear_gap_bwd_kernel<u16>, dim3((unsigned)(nbx + nbw)), dim3(256), 0,
                       as_stream(stream), b, in, out, nbx, inv, x, w, dy, ymask, (u16*)rows, dw,
                       dbias);
  else
    hipLaunchKernelGGL(linear_gap_bwd_kernel<float>, dim3((unsigned)(nbx + nbw)), dim3(256), 0,
                       as_stream(stream), b, in, out, nbx, inv, x, w, dy, ymask, (float*)rows, dw,
                       dbias);
  return launch_status();
}

int mmad_concat_cols(int b, int n_in, const float* const* srcs, const int* widths, float* dst,
                     void* stream) {
  if (b <= 0 || n_in <= 0 || n_in > 8) return MMAD_EBADSHAPE;
  if (!srcs || !widths || !dst) return MMAD_ENULL;
  ColList L{};
  int total = 0;
  for (int k = 0; k < n_in; ++k) {
    if (!srcs[k] || widths[k] <= 0) return MMAD_ENULL;
    L.p[k] = srcs[k]; L.w[k] = widths[k]; total += widths[k];
  }
  L.n = n_in;
  hipLaunchKernelGGL(concat_kernel, dim3((unsigned)cdiv((int64_t)b * total, 256)), dim3(256), 0,
                     as_stream(stream), b, total, L, dst);
  return launch_status();
}

int mmad_split_cols(int b, int n_out, const float* src, float* const* dsts, const int* widths,
                    void* stream) {
  if (b <= 0 || n_out <= 0 || n_out > 8) return MMAD_EBADSHAPE;
  if (!src || !dsts || !widths) return MMAD_ENULL;
  ColList L{};
  int total = 0;
  for (int k = 0; k < n_out; ++k) {
    if (!dsts[k] || widths[k] <= 0) return MMAD_ENULL;
    L.q[k] = dsts[k]; L.w[k] = widths[k]; total += widths[k];
  }
  L.n = n_out;
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)cdiv((int64_t)b * total, 256)), dim3(256), 0,
                     as_stream(stream), b, total, L, src);
  return launch_status();
}

int mmad_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!x || !y) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  const unsigned grid = grid_n(n);
#define CAST(TI, TO) \
  hipLaunchKernelGGL((cast_kernel<TI, TO>), dim3(grid), dim3(256), 0, st, n, (const TI*)x, (TO*)y)
  if (in_dtype == MMAD_F64 && out_dtype == MMAD_F32) CAST(double, float);
  else if (in_dtype == MMAD_F64 && out_dtype == MMAD_BF16) CAST(double, u16);
  else if (in_dtype == MMAD_F32 && out_dtype == MMAD_BF16) CAST(float, u16);
  else if (in_dtype == MMAD_F32 && out_dtype == MMAD_F64) CAST(float, double);
  else if (in_dtype == MMAD_BF16 && out_dtype == MMAD_F32) CAST(u16, float);
  else if (in_dtype == MMAD_BF16 && out_dtype == MMAD_F64) CAST(u16, double);
  else if (in_dtype == MMAD_F32 && out_dtype == MMAD_F32) CAST(float, float);
  else if (in_dtype == MMAD_F64 && out_dtype == MMAD_F64) CAST(double, double);
  else return MMAD_EBADDTYPE;
#undef CAST
  return launch_status();
}

static int dropout_fwd_launch(int dtype, int64_t n, float p, uint64_t seed,
                              const uint64_t* seed_dev, const void* x, void* y, uint8_t* keep,
                              void* stream) {
  if (n <= 0 || !(p >= 0.f && p < 1.f)) return MMAD_EBADSHAPE;
  if (!x || !y || !keep) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(dropout_fwd_kernel<u16>, dim3(grid_n(n)), dim3(256), 0, as_stream(stream),
                       n, p, seed, seed_dev, (const u16*)x, (u16*)y, keep);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(dropout_fwd_kernel<float>, dim3(grid_n(n)), dim3(256), 0,
                       as_stream(stream), n, p, seed, seed_dev, (const float*)x, (float*)y, keep);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_dropout_fwd(int dtype, int64_t n, float p, uint64_t seed, const void* x, void* y,
                     uint8_t* keep, void* stream) {
  return dropout_fwd_launch(dtype, n, p, seed, nullptr, x, y, keep, stream);
}

int mmad_dropout_fwd_dev(int dtype, int64_t n, float p, const uint64_t* seed, const void* x,
                         void* y, uint8_t* keep, void* stream) {
  if (!seed) return MMAD_ENULL;
  return dropout_fwd_launch(dtype, n, p, 0, seed, x, y, keep, stream);
}

int mmad_dropout_bwd(int dtype, int64_t n, float p, const void* g, const uint8_t* keep, void* dx,
                     void* stream) {
  if (n <= 0 || !(p >= 0.f && p < 1.f)) return MMAD_EBADSHAPE;
  if (!g || !dx || !keep) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(dropout_bwd_kernel<u16>, dim3(grid_n(n)), dim3(256), 0, as_stream(stream),
                       n, p, (const u16*)g, keep, (u16*)dx);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(dropout_bwd_kernel<float>, dim3(grid_n(n)), dim3(256), 0,
                       as_stream(stream), n, p, (const float*)g, keep, (float*)dx);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_loss_fwd(int b, int c, const double* logits, const int64_t* labels, const double* weight,
                  double gamma, int mode, double* loss, double* dlogits, void* stream) {
  return mmad_loss_fwd_ex(b, c, MMAD_F64, logits, labels, weight, gamma, mode, nullptr, loss,
                          dlogits, stream);
}

int mmad_loss_fwd_ex(int b, int c, int logits_dtype, const void* logits, const int64_t* labels,
                     const double* weight, double gamma, int mode, double* logits64,
                     double* loss, double* dlogits, void* stream) {
  if (b <= 0 || c <= 0 || (mode != 0 && mode != 1)) return MMAD_EBADSHAPE;
  if (!logits || !labels || !loss || !dlogits) return MMAD_ENULL;
  // one wave for small batches (the usual 8-16 samples), up to 256 threads beyond
  const unsigned nt = (unsigned)std::min(256, (int)cdiv(b, 64) * 64);
  hipStream_t st = as_stream(stream);
  if (logits_dtype == MMAD_F64)
    hipLaunchKernelGGL(loss_kernel<double>, dim3(1), dim3(nt), 0, st, b, c,
                       (const double*)logits, labels, weight, gamma, mode, loss, dlogits,
                       (int*)nullptr, logits64);
  else if (logits_dtype == MMAD_F32)
    hipLaunchKernelGGL(loss_kernel<float>, dim3(1), dim3(nt), 0, st, b, c, (const float*)logits,
                       labels, weight, gamma, mode, loss, dlogits, (int*)nullptr, logits64);
  else
    return MMAD_EBADDTYPE;
  return launch_status();
}

int mmad_loss_bwd(int64_t n, const double* dlogits, const double* gloss, const double* gout,
                  int out_dtype, void* dx, void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!dlogits || !gloss || !dx) return MMAD_ENULL;
  if (out_dtype != MMAD_F64 && out_dtype != MMAD_F32) return MMAD_EBADDTYPE;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                     as_stream(stream), n, dlogits, gloss, gout, out_dtype, dx);
  return launch_status();
}

int mmad_bootstrap_cls_metrics(int n, int c, const double* logits, const int64_t* labels,
                               int ndraw, const int64_t* idx, float* f1, float* mcc,
                               void* stream) {
  if (n <= 0 || c <= 0 || c > BOOT_MAXC || ndraw <= 0) return MMAD_EBADSHAPE;
  if (!logits || !labels || !idx || !f1 || !mcc) return MMAD_ENULL;
  hipLaunchKernelGGL(bootstrap_kernel, dim3((unsigned)ndraw), dim3(256), 0, as_stream(stream), n,
                     c, logits, labels, idx, f1, mcc);
  return launch_status();
}

int mmad_mean_std(int n, const float* v, double* out, void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!v || !out) return MMAD_ENULL;
  hipLaunchKernelGGL(mean_std_kernel, dim3(1), dim3(256), 0, as_stream(stream), n, v, out);
  return launch_status();
}

int mmad_abi_version(void) { return MMAD_ABI_VERSION; }

const char* mmad_strerror(int s) {
  switch (s) {
    case MMAD_OK: return "ok";
    case MMAD_EBADSHAPE: return "bad shape / descriptor / buffer alignment";
    case MMAD_EBADDTYPE: return "unsupported dtype";
    case MMAD_ENULL: return "null pointer argument";
    case MMAD_EUNSUPPORTED: return "unsupported configuration";
    default: break;
  }
  if (s >= MMAD_EHIP) return hipGetErrorString((hipError_t)(s - MMAD_EHIP));
  return "unknown status";
}

}  // extern "C"
