// 1x1x1 stride-1 convolutions (MedicalNet shortcut B downsample of layers 3 and 4, reached
// from pkg/models/mri_models/anat_cnn.py:29-31) are plain GEMMs over NDHWC rows, so their
// input gradient goes to hipBLASLt instead of the implicit-GEMM kernel (whose 32-deep K
// stages and row gathers are built for 27-tap convs: layer4's shortcut dgrad 25.6 -> 18.8 us,
// layer3's 14.2 -> 10.8 us).  The forward keeps conv.hip's implicit GEMM, whose epilogue
// produces the BN partial sums; the weight gradient (wgrad below) is kept for experiments
// but not routed: hipBLASLt returned no split-K algorithm for K = 32768 and its single-pass
// kernels took 140-165 us.  Internal to libmmad_hip.so; host code only.
//
// Row-major NDHWC tensors are column-major with the channel as the leading dimension:
//   dgrad  dX[M][ci] = dY[M][co] . Wd[ci][co]^T   ->  D(ci x M) = op_T(Wd: co x ci) . dY(co x M)
//   wgrad  dW[co][ci] = sum_m dY[m][co] X[m][ci]   ->  D(ci x co) = X(ci x M) . op_T(dY: co x M)
// (fp32 accumulation; dW written in fp32, the torch layout [co][ci][1][1][1]).
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <tuple>

#include "common.h"
#include "pointwise.h"

namespace {

bool pw_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PW_GEMM");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}

hipblasLtHandle_t handle() {
  static hipblasLtHandle_t h = [] {
    hipblasLtHandle_t x = nullptr;
    if (hipblasLtCreate(&x) != HIPBLAS_STATUS_SUCCESS) x = nullptr;
    return x;
  }();
  return h;
}

// one GEMM shape: descriptors and the heuristic's first algorithm, built on first use
// (eagerly, before any graph capture: warm-up steps run every shape first)
struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};

using Key = std::tuple<int, int, int, int, int, int, size_t>;   // ta, tb, m, n, k, dtype, ws

const Plan& plan_for(hipblasOperation_t ta, hipblasOperation_t tb, int m, int n, int k,
                     hipDataType dt, size_t ws_max) {
  static std::map<Key, Plan> cache;
  const Key key{(int)ta, (int)tb, m, n, k, (int)dt, ws_max};
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  Plan p;
  hipblasLtHandle_t h = handle();
  bool good = h != nullptr;
  good = good && hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) ==
                     HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta,
                                                 sizeof(ta)) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb,
                                                 sizeof(tb)) == HIPBLAS_STATUS_SUCCESS;
  const uint64_t ar = ta == HIPBLAS_OP_N ? m : k, ac = ta == HIPBLAS_OP_N ? k : m;
  const uint64_t br = tb == HIPBLAS_OP_N ? k : n, bc = tb == HIPBLAS_OP_N ? n : k;
  good = good && hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ar, ac, (int64_t)ar) ==
                     HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, br, bc, (int64_t)br) ==
                     HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.d, dt, m, n, m) == HIPBLAS_STATUS_SUCCESS;
  hipblasLtMatmulPreference_t pref = nullptr;
  good = good && hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS;
  uint64_t wmax = ws_max;
  good = good && hipblasLtMatmulPreferenceSetAttribute(
                     pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax, sizeof(wmax)) ==
                     HIPBLAS_STATUS_SUCCESS;
  if (good) {
    // a long-K product (the weight gradient: K = all voxels) wants a split-K algorithm; the
    // heuristic's first answer is not always one (measured: 165 us instead of ~25 us), so
    // take the first candidate that uses workspace when K dwarfs the output
    hipblasLtMatmulHeuristicResult_t res[8];
    int nres = 0;
    good = hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.a, p.b, p.d, p.d, pref, 8, res, &nres) ==
               HIPBLAS_STATUS_SUCCESS &&
           nres > 0;
    int pick = 0;
    if (good && ws_max > 0 && (int64_t)k > 16 * (int64_t)std::max(m, n))
      for (int i = 0; i < nres; ++i)
        if (res[i].workspaceSize > 0 && res[i].workspaceSize <= ws_max) { pick = i; break; }
    good = good && res[pick].workspaceSize <= ws_max;
    if (good) {
      p.algo = res[pick].algo;
      p.ws = res[pick].workspaceSize;
    }
  }
  if (pref) hipblasLtMatmulPreferenceDestroy(pref);
  p.ok = good;
  return cache.emplace(key, p).first->second;
}

int run(hipblasOperation_t ta, hipblasOperation_t tb, int m, int n, int k, const void* A,
        const void* B, void* D, hipDataType dt, void* ws, size_t ws_max, void* stream) {
  const Plan& p = plan_for(ta, tb, m, n, k, dt, ws_max);
  if (!p.ok) return MMAD_EUNSUPPORTED;
  const float alpha = 1.f, beta = 0.f;
  const hipblasStatus_t s = hipblasLtMatmul(handle(), p.op, &alpha, A, p.a, B, p.b, &beta, D,
                                            p.d, D, p.d, &p.algo, p.ws ? ws : nullptr, p.ws,
                                            as_stream(stream));
  return s == HIPBLAS_STATUS_SUCCESS ? launch_status() : MMAD_EUNSUPPORTED;
}

}  // namespace

namespace mmad_pw {

bool ok(const mmad_conv_desc* d, int dtype) {
  if (!pw_on() || dtype != MMAD_BF16) return false;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->sd != 1 || d->sh != 1 || d->sw != 1) return false;
  if (d->pd || d->ph || d->pw || d->ci % 64 || d->co % 64) return false;   // unpadded K
  if (d->di != d->do_ || d->hi != d->ho || d->wi != d->wo) return false;
  const int64_t m = (int64_t)d->n * d->di * d->hi * d->wi;
  return m < (int64_t(1) << 31);   // (the hipBLASLt handle is created on the first GEMM)
}

int64_t wgrad_workspace(const mmad_conv_desc* d) {
  (void)d;
  return WGRAD_WS;
}

int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream) {
  const int m = d->n * d->di * d->hi * d->wi;
  return run(HIPBLAS_OP_T, HIPBLAS_OP_N, d->ci, m, d->co, wpt, dy, dx, HIP_R_16BF, nullptr, 0,
             stream);
}

int wgrad(const mmad_conv_desc* d, const void* x, const void* dy, float* dw, void* ws,
          void* stream) {
  const int m = d->n * d->di * d->hi * d->wi;
  return run(HIPBLAS_OP_N, HIPBLAS_OP_T, d->ci, d->co, m, x, dy, dw, HIP_R_32F, ws, WGRAD_WS,
             stream);
}

}  // namespace mmad_pw
