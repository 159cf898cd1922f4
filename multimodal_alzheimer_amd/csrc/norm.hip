// Input-pipeline normalisation on device, gfx950 (float64, as the reference loader).
//
// Replaces the per-sample CPU normalisation of MultiModalDataset.__getitem__
// (pkg/utils/dataloader.py:213-215 PET z-score with split statistics, :244-270 MRI per-scan
// normalisation over the brain mask, :272-277 MRI all-scan z-score), run by the reference in
// float64 on 32 loader workers, as batched kernels over (scans x voxels) float64 volumes:
//
//   min_max (:262-270): v = nonzero(x * mask);  lo = quantile(v, 1-q), hi = quantile(v, q)
//            (torch.quantile 'linear': sorted[r], r = q*(n-1), lerp with torch's formula);
//            out = clamp((x - lo) / (hi - lo), 0, 1) * mask   -- bit-exact with the reference;
//   zscore  (:253-260): out = (x - mean(v)) / std(v) * mask (unbiased std; fp64 sums in a
//            fixed order: matches torch.std_mean to rounding, not bitwise);
//   affine  (:213-215, :272-277): out = (x - mean) / std.
//
// The quantiles are exact order statistics found by radix SELECTION (no sort): the
// masked nonzero values are compacted once as order-preserving 64-bit keys, then six
// passes of 11/11/11/11/10/10-bit digits narrow the four wanted ranks (floor and floor+1 of
// both quantile positions) using LDS-privatised histograms; integer counts make every step
// order-independent, so the result is deterministic although the compaction order is not.
#include <cstdlib>

#include "common.h"

// torch's CPU quantile/normalise arithmetic rounds every multiply and add separately
// (r = q*(n-1); w = r - floor(r); lerp); a contracted fma(q, n-1, -floor) differs in the
// last bit, so contraction is off for this file.
#pragma clang fp contract(off)

namespace {

constexpr int NT = 4;              // targets per scan: hi_below, hi_above, lo_below, lo_above
constexpr int DBITS = 11, NBIN = 1 << DBITS;
__host__ __device__ constexpr int digit_shift(int pass) {   // 64 = 11+11+11+11+10+10
  return pass < 4 ? 64 - DBITS * (pass + 1) : (pass == 4 ? 10 : 0);
}
__host__ __device__ constexpr int digit_bits(int pass) { return pass < 4 ? DBITS : 10; }

__device__ __forceinline__ uint64_t okey(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// per-scan selection state (in the workspace)
struct Sel {
  uint64_t prefix[NT];     // key bits fixed so far (high bits)
  int64_t rank[NT];        // rank still to skip inside the current prefix bucket
  int64_t nnz;             // masked nonzero count
  double w_hi, w_lo;       // lerp weights
  double qmin, qmax;       // results
  int status;              // 0 ok, 1 empty
};

// pass 0: compact keys of v = x*mask != 0 per scan; count them
__global__ __launch_bounds__(256) void compact_kernel(int64_t vox, const double* __restrict__ x,
                                                      const double* __restrict__ m,
                                                      uint64_t* __restrict__ keys,
                                                      unsigned long long* __restrict__ cnt) {
  __shared__ unsigned int lcount, lbase;
  const int scan = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (threadIdx.x == 0) lcount = 0;
  __syncthreads();
  double v = 0.0;
  if (i < vox) v = x[(int64_t)scan * vox + i] * m[(int64_t)scan * vox + i];
  const bool keep = i < vox && v != 0.0;       // data_masked_mri[data_masked_mri.nonzero()]
  unsigned int slot = 0;
  if (keep) slot = atomicAdd(&lcount, 1u);
  __syncthreads();
  if (threadIdx.x == 0) lbase = (unsigned int)atomicAdd(&cnt[scan], (unsigned long long)lcount);
  __syncthreads();
  if (keep) keys[(int64_t)scan * vox + lbase + slot] = okey(v);
}

// ranks from counts (torch.quantile: r = q*(n-1), below = floor, above = ceil)
__global__ void ranks_kernel(int nscan, double q, const unsigned long long* __restrict__ cnt,
                             Sel* __restrict__ sel) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nscan) return;
  Sel st{};
  st.nnz = (int64_t)cnt[s];
  if (st.nnz == 0) {                       // torch.quantile raises; we emit NaN volumes
    st.status = 1;
    st.qmin = st.qmax = __longlong_as_double(0x7ff8000000000000ll);
    sel[s] = st;
    return;
  }
  const double n1 = (double)(st.nnz - 1);
  const double rh = q * n1, rl = (1.0 - q) * n1;
  const int64_t hb = (int64_t)rh, lb = (int64_t)rl;
  st.rank[0] = hb;
  st.rank[1] = (int64_t)ceil(rh);
  st.rank[2] = lb;
  st.rank[3] = (int64_t)ceil(rl);
  st.w_hi = rh - (double)hb;
  st.w_lo = rl - (double)lb;
  for (int t = 0; t < NT; ++t) st.prefix[t] = 0;
  sel[s] = st;
}

// one radix pass: LDS histograms of the next digit of every key that matches each target's
// prefix, added into the global histogram hist[scan][t][bin]
__global__ __launch_bounds__(256) void hist_kernel(int pass, int64_t vox,
                                                   const uint64_t* __restrict__ keys,
                                                   const unsigned long long* __restrict__ cnt,
                                                   const Sel* __restrict__ sel,
                                                   unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[NT][NBIN];
  const int scan = blockIdx.y;
  const Sel st = sel[scan];
  for (int b = threadIdx.x; b < NT * NBIN; b += 256) (&h[0][0])[b] = 0;
  __syncthreads();
  const int64_t n = (int64_t)cnt[scan];
  const int sh = digit_shift(pass), nb = digit_bits(pass);
  const int hs = sh + nb;                       // bits above the digit (already fixed)
  const uint64_t dmask = (1ull << nb) - 1;
  if (st.status == 0) {
    const uint64_t* k = keys + (int64_t)scan * vox;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
      const uint64_t key = k[i];
      const uint64_t hi = hs >= 64 ? 0 : (key >> hs);
      const unsigned d = (unsigned)((key >> sh) & dmask);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (hi == (hs >= 64 ? 0 : (st.prefix[t] >> hs))) atomicAdd(&h[t][d], 1u);
    }
  }
  __syncthreads();
  unsigned int* g = hist + (int64_t)scan * NT * NBIN;
  for (int b = threadIdx.x; b < NT * NBIN; b += 256) {
    const unsigned v = (&h[0][0])[b];
    if (v) atomicAdd(&g[b], v);
  }
}

// pick the bucket holding each target's rank; clear the histogram for the next pass;
// after the last pass the prefixes are the exact keys -> quantiles
__global__ __launch_bounds__(256) void select_kernel(int pass, int last, Sel* __restrict__ sel,
                                                     unsigned int* __restrict__ hist) {
  const int scan = blockIdx.x, tid = threadIdx.x;
  __shared__ int64_t scanbuf[2][256];
  __shared__ int64_t found[2];
  unsigned int* g = hist + (int64_t)scan * NT * NBIN;
  Sel st = sel[scan];
  const int nb = digit_bits(pass), sh = digit_shift(pass);
  constexpr int PER = NBIN / 256;                 // bins per thread
  for (int t = 0; t < NT; ++t) {
    // per-thread bin sums -> inclusive block scan (Hillis-Steele, double-buffered)
    int64_t loc[PER], mine = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int bin = tid * PER + j;
      loc[j] = bin < (1 << nb) ? (int64_t)g[t * NBIN + bin] : 0;
      mine += loc[j];
    }
    int cur = 0;
    scanbuf[0][tid] = mine;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const int64_t v = scanbuf[cur][tid] + (tid >= o ? scanbuf[cur][tid - o] : 0);
      scanbuf[cur ^ 1][tid] = v;
      cur ^= 1;
      __syncthreads();
    }
    const int64_t incl = scanbuf[cur][tid], excl = incl - mine, r = st.rank[t];
    if (r >= excl && r < incl) {                  // exactly one thread owns rank r
      int64_t c = excl;
      int dsel = tid * PER + PER - 1;
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (r < c + loc[j]) { dsel = tid * PER + j; break; }
        c += loc[j];
      }
      found[0] = dsel;
      found[1] = r - c;
    }
    __syncthreads();
    if (tid == 0 && st.status == 0) {
      st.prefix[t] |= (uint64_t)found[0] << sh;
      st.rank[t] = found[1];
    }
    __syncthreads();
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NT * NBIN; b += 256) g[b] = 0;
  if (threadIdx.x == 0) {
    if (last && st.status == 0) {
      // torch lerp(a, b, w): w < 0.5 ? a + w*(b-a) : b - (b-a)*(1-w)
      auto lerp = [](double a, double b, double w) {
        return w < 0.5 ? a + w * (b - a) : b - (b - a) * (1.0 - w);
      };
      st.qmax = lerp(unkey(st.prefix[0]), unkey(st.prefix[1]), st.w_hi);
      st.qmin = lerp(unkey(st.prefix[2]), unkey(st.prefix[3]), st.w_lo);
    }
    sel[scan] = st;
  }
}

// out = clamp((x - qmin) / (qmax - qmin), 0, 1) * mask   (dataloader.py:266-270)
__global__ void minmax_apply_kernel(int64_t vox, const double* __restrict__ x,
                                    const double* __restrict__ m, const Sel* __restrict__ sel,
                                    double* __restrict__ out) {
  const int scan = blockIdx.y;
  const double lo = sel[scan].qmin, hi = sel[scan].qmax;
  const double den = hi - lo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < vox;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = (int64_t)scan * vox + i;
    double v = (x[j] - lo) / den;
    if (v > 1.0) v = 1.0;
    if (v < 0.0) v = 0.0;
    out[j] = v * m[j];
  }
}

// per-scan z-score statistics over v = nonzero(x*mask): fixed-order two-level sums
__global__ __launch_bounds__(256) void zsum_kernel(int64_t vox, const double* __restrict__ x,
                                                   const double* __restrict__ m,
                                                   const double* __restrict__ mean, int pass,
                                                   double* __restrict__ part) {
  __shared__ double red[256];
  const int scan = blockIdx.y;
  double s = 0.0;
  const double mu = pass ? mean[scan] : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < vox; i += (int64_t)gridDim.x * 256) {
    const double v = x[(int64_t)scan * vox + i] * m[(int64_t)scan * vox + i];
    if (v != 0.0) s += pass ? (v - mu) * (v - mu) : v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)scan * gridDim.x + blockIdx.x] = red[0];
}

__global__ void zfin_kernel(int nscan, int nparts, int pass, const double* __restrict__ part,
                            const unsigned long long* __restrict__ cnt, double* __restrict__ mean,
                            double* __restrict__ stdv) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nscan) return;
  double acc = 0.0;
  for (int p = 0; p < nparts; ++p) acc += part[(int64_t)s * nparts + p];
  const double n = (double)cnt[s];
  if (pass == 0) mean[s] = acc / n;
  else stdv[s] = sqrt(acc / (n - 1.0));
}

__global__ void zcount_kernel(int64_t vox, const double* __restrict__ x,
                              const double* __restrict__ m, unsigned long long* __restrict__ cnt) {
  const int scan = blockIdx.y;
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < vox;
       i += (int64_t)gridDim.x * blockDim.x)
    c += (x[(int64_t)scan * vox + i] * m[(int64_t)scan * vox + i]) != 0.0;
  if (c) atomicAdd(&cnt[scan], c);
}

__global__ void zapply_kernel(int64_t vox, const double* __restrict__ x,
                              const double* __restrict__ m, const double* __restrict__ mean,
                              const double* __restrict__ stdv, double* __restrict__ out) {
  const int scan = blockIdx.y;
  const double mu = mean[scan], sd = stdv[scan];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < vox;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = (int64_t)scan * vox + i;
    out[j] = (x[j] - mu) / sd * m[j];
  }
}

__global__ void affine_kernel(int64_t n, const double* __restrict__ x, double mean, double sd,
                              double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (x[i] - mean) / sd;
}

unsigned blocks_for(int64_t n, int64_t cap = 4096) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), cap));
}

// workspace layout (bytes, 256-aligned pieces)
struct WsLayout {
  int64_t keys, cnt, sel, hist, part, stats, total;
};
WsLayout ws_layout(int nscan, int64_t vox) {
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  WsLayout w{};
  int64_t o = 0;
  w.keys = o; o += al((int64_t)nscan * vox * 8);
  w.cnt = o; o += al((int64_t)nscan * 8);
  w.sel = o; o += al((int64_t)nscan * sizeof(Sel));
  w.hist = o; o += al((int64_t)nscan * NT * NBIN * 4);
  w.part = o; o += al((int64_t)nscan * 1024 * 8);
  w.stats = o; o += al((int64_t)nscan * 2 * 8);
  w.total = o;
  return w;
}

}  // namespace

extern "C" {

int64_t mmad_norm_ws_bytes(int nscan, int64_t vox) {
  if (nscan <= 0 || vox <= 0) return -1;
  return ws_layout(nscan, vox).total;
}

int mmad_mri_minmax_norm(int nscan, int64_t vox, const double* x, const double* mask, double q,
                         double* out, void* ws, double* q_out, void* stream) {
  if (nscan <= 0 || vox <= 0 || nscan > 65535) return MMAD_EBADSHAPE;
  if (!(q >= 0.0 && q <= 1.0)) return MMAD_EBADSHAPE;
  if (!x || !mask || !out || !ws) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  const WsLayout w = ws_layout(nscan, vox);
  char* base = reinterpret_cast<char*>(ws);
  auto* keys = reinterpret_cast<uint64_t*>(base + w.keys);
  auto* cnt = reinterpret_cast<unsigned long long*>(base + w.cnt);
  auto* sel = reinterpret_cast<Sel*>(base + w.sel);
  auto* hist = reinterpret_cast<unsigned int*>(base + w.hist);
  int rc = hip_status(hipMemsetAsync(cnt, 0, (size_t)nscan * 8, st));
  if (rc) return rc;
  rc = hip_status(hipMemsetAsync(hist, 0, (size_t)nscan * NT * NBIN * 4, st));
  if (rc) return rc;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)cdiv(vox, 256), (unsigned)nscan), dim3(256), 0,
                     st, vox, x, mask, keys, cnt);
  hipLaunchKernelGGL(ranks_kernel, dim3((unsigned)cdiv(nscan, 64)), dim3(64), 0, st, nscan, q, cnt,
                     sel);
  const unsigned hb = blocks_for(vox, std::max<int64_t>(1, 1024 / nscan));
  for (int pass = 0; pass < 6; ++pass) {
    hipLaunchKernelGGL(hist_kernel, dim3(hb, (unsigned)nscan), dim3(256), 0, st, pass, vox, keys,
                       cnt, sel, hist);
    hipLaunchKernelGGL(select_kernel, dim3((unsigned)nscan), dim3(256), 0, st, pass,
                       (int)(pass == 5), sel, hist);
  }
  hipLaunchKernelGGL(minmax_apply_kernel, dim3(blocks_for(vox, std::max<int64_t>(1, 4096 / nscan)),
                                               (unsigned)nscan),
                     dim3(256), 0, st, vox, x, mask, sel, out);
  if (q_out) {
    // (qmin, qmax) per scan for inspection / tests: copy from the selection state
    for (int s = 0; s < nscan; ++s) {
      rc = hip_status(hipMemcpyAsync(q_out + 2 * s, &sel[s].qmin, 2 * sizeof(double),
                                     hipMemcpyDeviceToDevice, st));
      if (rc) return rc;
    }
  }
  return launch_status();
}

int mmad_mri_zscore_norm(int nscan, int64_t vox, const double* x, const double* mask,
                         double* out, void* ws, void* stream) {
  if (nscan <= 0 || vox <= 0 || nscan > 65535) return MMAD_EBADSHAPE;
  if (!x || !mask || !out || !ws) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  const WsLayout w = ws_layout(nscan, vox);
  char* base = reinterpret_cast<char*>(ws);
  auto* cnt = reinterpret_cast<unsigned long long*>(base + w.cnt);
  auto* part = reinterpret_cast<double*>(base + w.part);
  auto* mean = reinterpret_cast<double*>(base + w.stats);
  double* sd = mean + nscan;
  int rc = hip_status(hipMemsetAsync(cnt, 0, (size_t)nscan * 8, st));
  if (rc) return rc;
  const unsigned nb = blocks_for(vox, 1024);
  hipLaunchKernelGGL(zcount_kernel, dim3(nb, (unsigned)nscan), dim3(256), 0, st, vox, x, mask, cnt);
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(zsum_kernel, dim3(nb, (unsigned)nscan), dim3(256), 0, st, vox, x, mask,
                       mean, pass, part);
    hipLaunchKernelGGL(zfin_kernel, dim3((unsigned)cdiv(nscan, 64)), dim3(64), 0, st, nscan,
                       (int)nb, pass, part, cnt, mean, sd);
  }
  hipLaunchKernelGGL(zapply_kernel, dim3(blocks_for(vox, std::max<int64_t>(1, 4096 / nscan)),
                                         (unsigned)nscan),
                     dim3(256), 0, st, vox, x, mask, mean, sd, out);
  return launch_status();
}

int mmad_affine_norm(int64_t n, const double* x, double mean, double stdv, double* out,
                     void* stream) {
  if (n <= 0) return MMAD_EBADSHAPE;
  if (!x || !out) return MMAD_ENULL;
  hipLaunchKernelGGL(affine_kernel, dim3(blocks_for(n)), dim3(256), 0, as_stream(stream), n, x,
                     mean, stdv, out);
  return launch_status();
}

}  // extern "C"
