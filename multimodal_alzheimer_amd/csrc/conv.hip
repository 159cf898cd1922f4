// 3D convolution as MFMA implicit GEMM on gfx950.
//
// Replaces torch.nn.Conv3d forward / backward for every conv of the reference hot path
// (MedicalNet stem + BasicBlock / Bottleneck / shortcut-B convs used at
// pkg/models/mri_models/anat_cnn.py:29-31, head convs anat_cnn.py:55-63, Small_PET_CNN
// convs pkg/models/pet_models/pet_cnn.py:20-22).
//
// Data layout: NDHWC activations ("voxel-major"), so the GEMM K dimension
// (tap, input channel) is channel-contiguous and every operand load is a 16-byte
// vector.  GEMM view of one conv:
//   forward : Y[m, co]   = sum_{tap, ci} X[src(m, tap), ci] * W[co, tap, ci]
//   dgrad   : dX[i, ci]  = sum_{tap, co} dY[src^T(i, tap), co] * W[co, tap, ci]
//   wgrad   : dW[co, k]  = sum_m dY[m, co] * X[src(m, tap(k)), ci(k)]   (split over m)
// Input-channel counts of 1 (the stem, PET conv 1) are handled by unfolding the input
// along W into 8 "channels" (j = kw tap, zero-padded), which turns the conv into a
// (kd, kh, 1) conv with Cin = 8 and keeps the vector path.
//
// Kernel structure: 256 threads = 4 waves in a 2x2 arrangement; block tile 128 (voxels)
// x BN (channels); register-staged, double-buffered LDS tiles (one barrier per K-step);
// bf16: v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32 (exact f32 fma chain).
// Forward epilogue also emits per-block BN partial sums (sum, sum of squares).
#include "common.h"

namespace {

constexpr int BM = 128;        // voxels per block tile
constexpr int KB = 64;         // bytes of K per K-step
constexpr int ROWB = KB + 16;  // LDS row stride (bytes), +16 pad breaks bank aliasing
constexpr int MAXTAPS = 344;
constexpr int TAPB = ((MAXTAPS * 4 + 15) / 16) * 16;

struct Geom {
  int M, Nd, Cs, K, Kpad, cs_shift, taps;
  int Ds, Hs, Ws, Dd, Hd, Wd;
  int KD, KH, KW;
  int sd, sh, sw, pd, ph, pw, dd, dh, dw;
};

template <typename T> constexpr int bk_elems() { return KB / (int)sizeof(T); }

__device__ __forceinline__ void fill_taps(const Geom& g, int* tapoff, bool trans) {
  for (int t = threadIdx.x; t < g.taps; t += blockDim.x) {
    int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
    tapoff[t] = (kd * g.dd) | ((kh * g.dh) << 8) | ((kw * g.dw) << 16);
  }
  (void)trans;
}

// Resolve the source voxel of (dst voxel base coords, tap offsets).  Returns false for
// padding / stride holes.
template <bool TRANS>
__device__ __forceinline__ bool src_voxel(const Geom& g, int bz, int by, int bx, int to,
                                          int& z, int& y, int& x) {
  const int oz = to & 255, oy = (to >> 8) & 255, ox = to >> 16;
  if (!TRANS) {
    z = bz + oz; y = by + oy; x = bx + ox;
  } else {
    z = bz - oz; y = by - oy; x = bx - ox;
    if (g.sd != 1) { if (z % g.sd) return false; z /= g.sd; }
    if (g.sh != 1) { if (y % g.sh) return false; y /= g.sh; }
    if (g.sw != 1) { if (x % g.sw) return false; x /= g.sw; }
  }
  return (unsigned)z < (unsigned)g.Ds && (unsigned)y < (unsigned)g.Hs &&
         (unsigned)x < (unsigned)g.Ws;
}

template <typename T, int BN, bool TRANS>
__global__ __launch_bounds__(256) void igemm_kernel(Geom g, const T* __restrict__ src,
                                                     const T* __restrict__ wgt,
                                                     const float* __restrict__ bias,
                                                     T* __restrict__ dst,
                                                     float* __restrict__ stats) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = bk_elems<T>();
  constexpr int TN = BN / 32;
  constexpr int BCH = BN / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  char* As = smem + TAPB;
  char* Bs = As + 2 * BM * ROWB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int ch = tid & 3;
  fill_taps(g, tapoff, TRANS);

  int rz[2], ry[2], rx[2];
  int64_t rbase[2];
  bool rok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int m = m0 + (tid >> 2) + 64 * h;
    rok[h] = m < g.M;
    const int mm = rok[h] ? m : 0;
    const int xw = mm % g.Wd;
    int t1 = mm / g.Wd;
    const int yh = t1 % g.Hd;
    t1 /= g.Hd;
    const int zd = t1 % g.Dd, nb = t1 / g.Dd;
    if (!TRANS) {
      rz[h] = zd * g.sd - g.pd; ry[h] = yh * g.sh - g.ph; rx[h] = xw * g.sw - g.pw;
    } else {
      rz[h] = zd + g.pd; ry[h] = yh + g.ph; rx[h] = xw + g.pw;
    }
    rbase[h] = (int64_t)nb * g.Ds;
  }
  __syncthreads();

  u32x4 ra[2], rb[BCH];
  auto load_tiles = [&](int k0) {
    const int k = k0 + ch * EPC;
    const bool kok = k < g.K;
    const int tap = k >> g.cs_shift, ci = k & (g.Cs - 1);
    const int to = kok ? tapoff[tap] : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int z, y, x;
      bool ok = rok[h] && kok && src_voxel<TRANS>(g, rz[h], ry[h], rx[h], to, z, y, x);
      if (ok) {
        const int64_t vox = ((rbase[h] + z) * g.Hs + y) * g.Ws + x;
        ra[h] = *reinterpret_cast<const u32x4*>(src + (vox << g.cs_shift) + ci);
      } else {
        ra[h] = u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int h = 0; h < BCH; ++h) {
      const int co = n0 + (tid >> 2) + 64 * h;
      rb[h] = co < g.Nd
                  ? *reinterpret_cast<const u32x4*>(wgt + (int64_t)co * g.Kpad + k0 + ch * EPC)
                  : u32x4{0, 0, 0, 0};
    }
  };
  auto store_tiles = [&](int buf) {
    char* a = As + buf * BM * ROWB;
    char* b = Bs + buf * BN * ROWB;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      *reinterpret_cast<u32x4*>(a + ((tid >> 2) + 64 * h) * ROWB + ch * 16) = ra[h];
#pragma unroll
    for (int h = 0; h < BCH; ++h)
      *reinterpret_cast<u32x4*>(b + ((tid >> 2) + 64 * h) * ROWB + ch * 16) = rb[h];
  };

  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  // fp32 mode sums K in two levels (a fresh partial per FLUSH K-steps, then acc += part):
  // one f32 MFMA chain over K = 27*512 terms would grow the rounding error ~K-fold.
  constexpr int FLUSH = 8;
  f32x4 acc[4][TN], part[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto flush = [&]() {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] += part[i][j];
          part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  };

  auto compute = [&](int buf) {
    const char* a = As + buf * BM * ROWB + (wm * 64 + lr) * ROWB;
    const char* b = Bs + buf * BN * ROWB + (wn * (BN / 2) + lr) * ROWB;
    if constexpr (sizeof(T) == 2) {
      bf16x8 fa[4], fb[TN];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(a + i * 16 * ROWB + lk * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * ROWB + lk * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        float fa[4], fb[TN];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = *reinterpret_cast<const float*>(a + i * 16 * ROWB + (s * 4 + lk) * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const float*>(b + j * 16 * ROWB + (s * 4 + lk) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], part[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = g.Kpad / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) load_tiles((ks + 1) * BK);
    compute(cur);
    if (ks % FLUSH == FLUSH - 1) flush();
    if (ks + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }
  flush();

  // epilogue: bias, store, BN partial sums over this block's valid rows
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    cs[j] = 0.f; cq[j] = 0.f;
    const int co = n0 + wn * (BN / 2) + j * 16 + lr;
    const float bv = (bias != nullptr && co < g.Nd) ? bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + lk * 4 + r;
        const float v = acc[i][j][r] + bv;
        if (m < g.M && co < g.Nd) {
          Elt<T>::st(dst, (int64_t)m * g.Nd + co, v);
          cs[j] += v;
          cq[j] += v * v;
        }
      }
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(As);   // staging LDS is free after the last barrier
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm == 1 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + lr;
        red[col] = cs[j];
        red[BN + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + lr;
        const int co = n0 + col;
        if (co < g.Nd) {
          stats[((int64_t)blockIdx.x * 2) * g.Nd + co] = cs[j] + red[col];
          stats[((int64_t)blockIdx.x * 2 + 1) * g.Nd + co] = cq[j] + red[BN + col];
        }
      }
    }
  }
}

// ---- implicit GEMM v2: LDS-DMA staging ----------------------------------------------
// Same GEMM view as igemm_kernel, restructured for gfx950:
//  * operands go global -> LDS directly with global_load_lds_dwordx4 (no VGPR staging):
//    one wave instruction fills 8 tile rows x 128 B; each lane supplies its own source
//    address, so the implicit-GEMM row gather and the zero padding (lanes pointed at a
//    128-B zero block in the code object) cost no extra LDS writes;
//  * 128-B K-slices per stage (64 bf16 / 32 f32) in a 2-stage ring, one barrier per stage;
//  * XOR-swizzled LDS rows (chunk c of row r lives in slot c ^ (r & 7)), applied on the
//    source address so the DMA image stays lane-linear, which spreads the fragment reads
//    of 16 consecutive rows over 8 slots;
//  * XCD-aware tile order: each XCD walks a contiguous range of (m, n) tiles with n
//    fastest, so the n-tiles that share an A panel (and neighbouring m-tiles that share
//    halo voxels) meet in the same L2.
__device__ const u32x4 g_zero_chunk[8] = {};

constexpr int RB2 = 128;   // K bytes per stage row

template <typename T, int BN, bool TRANS, int BM2, int NST>
__global__ __launch_bounds__(256, NST == 2 ? 2 : 1) void igemm2_kernel(
    Geom g, const T* __restrict__ src, const T* __restrict__ wgt, const float* __restrict__ bias,
    T* __restrict__ dst, float* __restrict__ stats, int nbm, int nbn) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = RB2 / (int)sizeof(T);
  constexpr int TM = BM2 / 32, TN = BN / 32;
  constexpr int A_BYTES = BM2 * RB2, B_BYTES = BN * RB2, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = A_BYTES / 4096, BI = B_BYTES / 4096;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  char* ring = smem + TAPB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = tile / nbn, nt = tile % nbn;
  const int m0 = mt * BM2, n0 = nt * BN;
  fill_taps(g, tapoff, TRANS);

  // this lane's A rows: one per DMA instruction, row = (wave*AI + i)*8 + lane/8
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;          // logical K chunk this lane fetches
  int rz[AI], ry[AI], rx[AI];
  int64_t rbase[AI];
  bool rok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (wave * AI + i) * 8 + lrow;
    rok[i] = m < g.M;
    const int mm = rok[i] ? m : 0;
    const int xw = mm % g.Wd;
    int t1 = mm / g.Wd;
    const int yh = t1 % g.Hd;
    t1 /= g.Hd;
    const int zd = t1 % g.Dd, nb = t1 / g.Dd;
    if (!TRANS) {
      rz[i] = zd * g.sd - g.pd; ry[i] = yh * g.sh - g.ph; rx[i] = xw * g.sw - g.pw;
    } else {
      rz[i] = zd + g.pd; ry[i] = yh + g.ph; rx[i] = xw + g.pw;
    }
    rbase[i] = (int64_t)nb * g.Ds;
  }
  __syncthreads();

  auto issue = [&](int stage, int k0) {
    char* sbase = ring + stage * STAGE;
    const int k = k0 + lchunk * EPC;
    const bool kok = k < g.K;
    const int tap = k >> g.cs_shift, ci = k & (g.Cs - 1);
    const int to = kok ? tapoff[tap] : 0;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const void* p = g_zero_chunk;
      int z, y, x;
      if (rok[i] && kok && src_voxel<TRANS>(g, rz[i], ry[i], rx[i], to, z, y, x)) {
        const int64_t vox = ((rbase[i] + z) * g.Hs + y) * g.Ws + x;
        p = src + (vox << g.cs_shift) + ci;
      }
      __builtin_amdgcn_global_load_lds(p, (LDS_AS void*)(sbase + (wave * AI + i) * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int co = n0 + (wave * BI + i) * 8 + lrow;
      const void* p = co < g.Nd ? (const void*)(wgt + (int64_t)co * g.Kpad + k0 + lchunk * EPC)
                                : (const void*)g_zero_chunk;
      __builtin_amdgcn_global_load_lds(
          p, (LDS_AS void*)(sbase + A_BYTES + (wave * BI + i) * 1024), 16, 0, 0);
    }
  };

  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  const int sw = lr & 7;                          // swizzle of every row this lane reads
  constexpr int FLUSH = 8;
  f32x4 acc[TM][TN], part[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* a = ring + stage * STAGE + (wm * (BM2 / 2) + lr) * RB2;
    const char* b = ring + stage * STAGE + A_BYTES + (wn * (BN / 2) + lr) * RB2;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        const int off = ((4 * s + lk) ^ sw) << 4;
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[i] = *reinterpret_cast<const bf16x8*>(a + i * 16 * RB2 + off);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * RB2 + off);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        const int off = ((s ^ sw) << 4) + lk * 4;
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[i] = *reinterpret_cast<const float*>(a + i * 16 * RB2 + off);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const float*>(b + j * 16 * RB2 + off);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], part[i][j], 0, 0, 0);
      }
    }
  };
  auto flush = [&]() {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] += part[i][j];
          part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  };

  const int nk = g.Kpad / BK;
  if constexpr (NST == 2) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nk) issue(cur ^ 1, (ks + 1) * BK);
      compute(cur);
      if (ks % FLUSH == FLUSH - 1) flush();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // 3-stage ring: stage ks+2 is issued while stage ks is consumed; the counted wait
    // vmcnt(AI+BI) at the end of an iteration retires stage ks+1 and leaves ks+2 in flight
    // across the raw barrier (a __syncthreads() would drain it: vmcnt(0)).
    constexpr int NI = AI + BI;
    issue(0, 0);
    if (nk > 1) {
      issue(1, BK);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    int cur = 0;
    for (int ks = 0; ks < nk; ++ks) {
      const int nxt2 = cur == 0 ? 2 : cur - 1;          // (ks + 2) % 3
      if (ks + 2 < nk) issue(nxt2, (ks + 2) * BK);
      compute(cur);
      if (ks % FLUSH == FLUSH - 1) flush();
      if (ks + 2 < nk)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NI) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      cur = cur == 2 ? 0 : cur + 1;
    }
  }
  flush();

  // epilogue: bias, store, BN partial sums over this tile's valid rows.  bf16 tiles are
  // transposed through LDS so the global stores are whole 16-byte channel vectors (the
  // MFMA C layout gives each lane 4 voxels x 1 channel).
  constexpr int CROW = BN * 2 + 16;
  const bool lds_out = sizeof(T) == 2 && (g.Nd & 7) == 0;
  u16* ctile = reinterpret_cast<u16*>(ring + 1024);
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    cs[j] = 0.f; cq[j] = 0.f;
    const int col = wn * (BN / 2) + j * 16 + lr;
    const int co = n0 + col;
    const float bv = (bias != nullptr && co < g.Nd) ? bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM2 / 2) + i * 16 + lk * 4 + r;
        const int m = m0 + row;
        const float v = acc[i][j][r] + bv;
        if (lds_out) ctile[row * (CROW / 2) + col] = f2bf(v);
        if (m < g.M && co < g.Nd) {
          if (!lds_out) Elt<T>::st(dst, (int64_t)m * g.Nd + co, v);
          cs[j] += v;
          cq[j] += v * v;
        }
      }
  }
  if (lds_out) {
    __syncthreads();
    constexpr int CPR = BN / 8;
#pragma unroll
    for (int h = 0; h < BM2 * CPR / 256; ++h) {
      const int q = tid + 256 * h;
      const int row = q / CPR, c8 = q % CPR;
      const int m = m0 + row, co = n0 + c8 * 8;
      if (m < g.M && co < g.Nd)
        *reinterpret_cast<u32x4*>(reinterpret_cast<u16*>(dst) + (int64_t)m * g.Nd + co) =
            *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) + row * CROW +
                                            c8 * 16);
    }
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(ring);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm == 1 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + lr;
        red[col] = cs[j];
        red[BN + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + j * 16 + lr;
        const int co = n0 + col;
        if (co < g.Nd) {
          stats[((int64_t)mt * 2) * g.Nd + co] = cs[j] + red[col];
          stats[((int64_t)mt * 2 + 1) * g.Nd + co] = cq[j] + red[BN + col];
        }
      }
    }
  }
}

// ---- weight gradient --------------------------------------------------------------
// dW[co][k] = sum_m dY[m][co] * X(m, k): block tile BMW (co) x 128 (k), K-step = 32
// voxels, split over m into `splits` slices -> fp32 partial slabs ws[s][co][k].
// Both operands are m-major in memory: bf16 fragments are read with the gfx950
// transposing LDS read (ds_read_b64_tr_b16), f32 fragments need no transpose.
constexpr int WBN = 128;
constexpr int WBK = 32;

template <typename T, int BMW>
__global__ __launch_bounds__(256) void wgrad_kernel(Geom g, const T* __restrict__ src,
                                                     const T* __restrict__ dy,
                                                     float* __restrict__ ws, int m_per_split) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int AROW = BMW * (int)sizeof(T) + 16;   // bytes per m-row of the dY tile
  constexpr int BROW = WBN * (int)sizeof(T) + 16;   // bytes per m-row of the X tile
  constexpr int ACPR = BMW * (int)sizeof(T) / 16;   // 16-B chunks per A row
  constexpr int BCPR = WBN * (int)sizeof(T) / 16;
  constexpr int ACH = WBK * ACPR / 256;             // A chunks per thread
  constexpr int BCH = WBK * BCPR / 256;
  constexpr int TI = BMW / 32, TJ = WBN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  char* As = smem + TAPB;
  char* Bs = As + 2 * WBK * AROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k0 = blockIdx.x * WBN, co0 = blockIdx.y * BMW;
  const int mbeg = blockIdx.z * m_per_split;
  const int mend = min(g.M, mbeg + m_per_split);
  fill_taps(g, tapoff, false);
  __syncthreads();

  // B chunks: fixed column (tap, ci) per thread, rows advance by WBK each K-step
  int bto[BCH], bci[BCH], brow[BCH], bx[BCH], by[BCH], bz[BCH], bn[BCH];
  bool bkok[BCH];
#pragma unroll
  for (int h = 0; h < BCH; ++h) {
    const int q = tid + 256 * h;
    brow[h] = q / BCPR;
    const int k = k0 + (q % BCPR) * EPC;
    bkok[h] = k < g.K;
    const int tap = bkok[h] ? (k >> g.cs_shift) : 0;
    bci[h] = k & (g.Cs - 1);
    bto[h] = tapoff[tap];
    int m = mbeg + brow[h];
    bx[h] = m % g.Wd; m /= g.Wd;
    by[h] = m % g.Hd; m /= g.Hd;
    bz[h] = m % g.Dd; bn[h] = m / g.Dd;
  }
  u32x4 ra[ACH], rb[BCH];
  auto load_tiles = [&](int mk) {   // mk = first voxel of this K-step
#pragma unroll
    for (int h = 0; h < ACH; ++h) {
      const int q = tid + 256 * h;
      const int m = mk + q / ACPR;
      const int co = co0 + (q % ACPR) * EPC;
      ra[h] = (m < mend && co < g.Nd)
                  ? *reinterpret_cast<const u32x4*>(dy + (int64_t)m * g.Nd + co)
                  : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int h = 0; h < BCH; ++h) {
      const int m = mk + brow[h];
      int z, y, x;
      bool ok = m < mend && bkok[h] &&
                src_voxel<false>(g, bz[h] * g.sd - g.pd, by[h] * g.sh - g.ph,
                                 bx[h] * g.sw - g.pw, bto[h], z, y, x);
      if (ok) {
        const int64_t vox = (((int64_t)bn[h] * g.Ds + z) * g.Hs + y) * g.Ws + x;
        rb[h] = *reinterpret_cast<const u32x4*>(src + (vox << g.cs_shift) + bci[h]);
      } else {
        rb[h] = u32x4{0, 0, 0, 0};
      }
      // advance this chunk's voxel by WBK
      bx[h] += WBK;
      while (bx[h] >= g.Wd) {
        bx[h] -= g.Wd;
        if (++by[h] == g.Hd) { by[h] = 0; if (++bz[h] == g.Dd) { bz[h] = 0; ++bn[h]; } }
      }
    }
  };
  auto store_tiles = [&](int buf) {
    char* a = As + buf * WBK * AROW;
    char* b = Bs + buf * WBK * BROW;
#pragma unroll
    for (int h = 0; h < ACH; ++h) {
      const int q = tid + 256 * h;
      *reinterpret_cast<u32x4*>(a + (q / ACPR) * AROW + (q % ACPR) * 16) = ra[h];
    }
#pragma unroll
    for (int h = 0; h < BCH; ++h) {
      const int q = tid + 256 * h;
      *reinterpret_cast<u32x4*>(b + (q / BCPR) * BROW + (q % BCPR) * 16) = rb[h];
    }
  };

  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  constexpr int FLUSH = 4;    // fp32: fresh partial every 4 K-steps (128 voxels)
  f32x4 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto flush = [&]() {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          acc[i][j] += part[i][j];
          part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  };

  auto compute = [&](int buf) {
    const char* a = As + buf * WBK * AROW;
    const char* b = Bs + buf * WBK * BROW;
    if constexpr (sizeof(T) == 2) {
      // tr16 read: lane 4q+p of each 16-lane group g addresses row 8g+q (+4), cols 4p..4p+3
      const int q = (lane & 15) >> 2, p = lane & 3;
      bf16x8 fa[TI], fb[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const char* base = a + (8 * lk + q) * AROW + (wm * (BMW / 2) + i * 16 + 4 * p) * 2;
        bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(base));
        bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(base + 4 * AROW));
        fa[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const char* base = b + (8 * lk + q) * BROW + (wn * (WBN / 2) + j * 16 + 4 * p) * 2;
        bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(base));
        bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(base + 4 * BROW));
        fb[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < WBK / 4; ++s) {
        float fa[TI], fb[TJ];
        const int row = s * 4 + lk;
#pragma unroll
        for (int i = 0; i < TI; ++i)
          fa[i] = *reinterpret_cast<const float*>(a + row * AROW + (wm * (BMW / 2) + i * 16 + lr) * 4);
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          fb[j] = *reinterpret_cast<const float*>(b + row * BROW + (wn * (WBN / 2) + j * 16 + lr) * 4);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], part[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = (mend - mbeg + WBK - 1) / WBK;
  if (nk > 0) {
    load_tiles(mbeg);
    store_tiles(0);
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nk) load_tiles(mbeg + (ks + 1) * WBK);
      compute(cur);
      if (ks % FLUSH == FLUSH - 1) flush();
      if (ks + 1 < nk) store_tiles(cur ^ 1);
      __syncthreads();
    }
  }
  flush();
  float* out = ws + (int64_t)blockIdx.z * g.Nd * g.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = k0 + wn * (WBN / 2) + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * (BMW / 2) + i * 16 + lk * 4 + r;
        if (co < g.Nd && k < g.K) out[(int64_t)co * g.K + k] = acc[i][j][r];
      }
    }
}

// ---- weight gradient v2: LDS-DMA staging ---------------------------------------------
// Same GEMM as wgrad_kernel.  Both tiles are m-major images ([m][co] of dY, [m][k] of the
// gathered X) filled by global_load_lds_dwordx4: a wave instruction writes 1 KB = RPI
// m-rows.  Rows are XOR-swizzled in 16-byte slots (swizzle applied to the source address,
// image stays lane-linear) so the transposing fragment reads of 8 m-rows x 16 columns
// (bf16: ds_read_b64_tr_b16) or 2 m-rows x 16 columns (f32: ds_read_b32) hit distinct
// banks.  2-stage ring, one barrier per 32-voxel stage.
template <typename T, int ROWB>
__device__ __forceinline__ int wswz(int r) {
  if constexpr (sizeof(T) == 4) return 4 * (r & 1);
  else if constexpr (ROWB >= 256) return 2 * (r & 3) + 8 * ((r >> 3) & 1);
  else return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1);
}

template <typename T, int BMW>
__global__ __launch_bounds__(256, 2) void wgrad2_kernel(Geom g, const T* __restrict__ src,
                                                        const T* __restrict__ dy,
                                                        float* __restrict__ ws, int m_per_split) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int AROWB = BMW * (int)sizeof(T), BROWB = WBN * (int)sizeof(T);
  constexpr int A_BYTES = WBK * AROWB, B_BYTES = WBK * BROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int ARPI = 1024 / AROWB, BRPI = 1024 / BROWB;      // rows per DMA instruction
  constexpr int ALPR = AROWB / 16, BLPR = BROWB / 16;         // lanes per row
  constexpr int AIPW = A_BYTES / 4096, BIPW = B_BYTES / 4096; // instructions per wave
  constexpr int TI = BMW / 32, TJ = WBN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  char* ring = smem + TAPB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k0 = blockIdx.x * WBN, co0 = blockIdx.y * BMW;
  const int mbeg = blockIdx.z * m_per_split;
  const int mend = min(g.M, mbeg + m_per_split);
  fill_taps(g, tapoff, false);
  __syncthreads();

  // A (dY) rows / chunks of this lane
  int arow[AIPW], aco[AIPW];
#pragma unroll
  for (int i = 0; i < AIPW; ++i) {
    arow[i] = (wave * AIPW + i) * ARPI + lane / ALPR;
    aco[i] = co0 + ((lane % ALPR) ^ wswz<T, AROWB>(arow[i])) * EPC;
  }
  // B (gathered X) rows / chunks of this lane: fixed (tap, ci) per instruction, rows advance
  int brow[BIPW], bto[BIPW], bci[BIPW], bx[BIPW], by[BIPW], bz[BIPW], bn[BIPW];
  bool bkok[BIPW];
#pragma unroll
  for (int i = 0; i < BIPW; ++i) {
    brow[i] = (wave * BIPW + i) * BRPI + lane / BLPR;
    const int k = k0 + ((lane % BLPR) ^ wswz<T, BROWB>(brow[i])) * EPC;
    bkok[i] = k < g.K;
    bci[i] = k & (g.Cs - 1);
    bto[i] = tapoff[bkok[i] ? (k >> g.cs_shift) : 0];
    int m = mbeg + brow[i];
    bx[i] = m % g.Wd; m /= g.Wd;
    by[i] = m % g.Hd; m /= g.Hd;
    bz[i] = m % g.Dd; bn[i] = m / g.Dd;
  }

  auto issue = [&](int stage, int mk) {
    char* sbase = ring + stage * STAGE;
#pragma unroll
    for (int i = 0; i < AIPW; ++i) {
      const int m = mk + arow[i];
      const void* p = (m < mend && aco[i] < g.Nd)
                          ? (const void*)(dy + (int64_t)m * g.Nd + aco[i])
                          : (const void*)g_zero_chunk;
      __builtin_amdgcn_global_load_lds(p, (LDS_AS void*)(sbase + (wave * AIPW + i) * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < BIPW; ++i) {
      const int m = mk + brow[i];
      const void* p = g_zero_chunk;
      int z, y, x;
      if (m < mend && bkok[i] &&
          src_voxel<false>(g, bz[i] * g.sd - g.pd, by[i] * g.sh - g.ph, bx[i] * g.sw - g.pw,
                           bto[i], z, y, x)) {
        const int64_t vox = (((int64_t)bn[i] * g.Ds + z) * g.Hs + y) * g.Ws + x;
        p = src + (vox << g.cs_shift) + bci[i];
      }
      __builtin_amdgcn_global_load_lds(
          p, (LDS_AS void*)(sbase + A_BYTES + (wave * BIPW + i) * 1024), 16, 0, 0);
      bx[i] += WBK;
      while (bx[i] >= g.Wd) {
        bx[i] -= g.Wd;
        if (++by[i] == g.Hd) { by[i] = 0; if (++bz[i] == g.Dd) { bz[i] = 0; ++bn[i]; } }
      }
    }
  };

  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  constexpr int FLUSH = 4;
  f32x4 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* a = ring + stage * STAGE;
    const char* b = a + A_BYTES;
    if constexpr (sizeof(T) == 2) {
      // lane 4q+p of each 16-lane group lk reads m-rows 8lk+q (+4), columns 4p..4p+3
      const int q = (lane & 15) >> 2, p = lane & 3;
      const int r0 = 8 * lk + q, r1 = r0 + 4;
      bf16x8 fa[TI], fb[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int col = wm * (BMW / 2) + i * 16 + 4 * p;          // element column
        const int ch = col >> 3, hb = (col & 7) * 2;
        const char* lo = a + r0 * AROWB + ((ch ^ wswz<T, AROWB>(r0)) << 4) + hb;
        const char* hi = a + r1 * AROWB + ((ch ^ wswz<T, AROWB>(r1)) << 4) + hb;
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)lo);
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)hi);
        fa[i] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = wn * (WBN / 2) + j * 16 + 4 * p;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const char* lo = b + r0 * BROWB + ((ch ^ wswz<T, BROWB>(r0)) << 4) + hb;
        const char* hi = b + r1 * BROWB + ((ch ^ wswz<T, BROWB>(r1)) << 4) + hb;
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)lo);
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)hi);
        fb[j] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < WBK / 4; ++s) {
        const int row = s * 4 + lk;
        float fa[TI], fb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int col = wm * (BMW / 2) + i * 16 + lr;
          fa[i] = *reinterpret_cast<const float*>(
              a + row * AROWB + (((col >> 2) ^ wswz<T, AROWB>(row)) << 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int col = wn * (WBN / 2) + j * 16 + lr;
          fb[j] = *reinterpret_cast<const float*>(
              b + row * BROWB + (((col >> 2) ^ wswz<T, BROWB>(row)) << 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], part[i][j], 0, 0, 0);
      }
    }
  };
  auto flush = [&]() {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          acc[i][j] += part[i][j];
          part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
  };

  const int nk = (mend - mbeg + WBK - 1) / WBK;
  if (nk > 0) {
    issue(0, mbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int ks = 0; ks < nk; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < nk) issue(cur ^ 1, mbeg + (ks + 1) * WBK);
      compute(cur);
      if (ks % FLUSH == FLUSH - 1) flush();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  flush();
  float* out = ws + (int64_t)blockIdx.z * g.Nd * g.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = k0 + wn * (WBN / 2) + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * (BMW / 2) + i * 16 + lk * 4 + r;
        if (co < g.Nd && k < g.K) out[(int64_t)co * g.K + k] = acc[i][j][r];
      }
    }
}

// sum the split-K slabs in fixed order and scatter into the torch [co][ci][kd][kh][kw]
// layout.  unf_kw > 0: the conv ran on a W-unfolded Cin=1 input (k = (kd,kh)*8 + j).
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                    int splits, int Nd, int K, int Cs, int cs_shift, int taps,
                                    int unf_kw) {
  const int64_t total = (int64_t)Nd * K;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int sp = 0; sp < splits; ++sp) s += ws[sp * total + idx];
    const int co = (int)(idx / K), k = (int)(idx % K);
    if (unf_kw > 0) {
      const int j = k & 7, tkh = k >> 3;   // tkh = kd*KH + kh
      if (j < unf_kw) dw[((int64_t)co * (taps) + tkh) * unf_kw + j] = s;
    } else {
      const int tap = k >> cs_shift, ci = k & (Cs - 1);
      dw[((int64_t)co * Cs + ci) * taps + tap] = s;
    }
  }
}

// ---- weight packing / input unfolding -------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ wp, int rows,
                                   int Kpad, int K, int Cs, int cs_shift, int taps, int mode,
                                   int Ci, int unf_kw) {
  const int64_t total = (int64_t)rows * Kpad;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(idx / Kpad), k = (int)(idx % Kpad);
    float v = 0.f;
    if (k < K) {
      const int tap = k >> cs_shift, c = k & (Cs - 1);
      if (mode == 0) {            // forward: row = co, c = ci
        v = w[((int64_t)r * Ci + c) * taps + tap];
      } else if (mode == 1) {     // dgrad: row = ci, c = co
        v = w[((int64_t)c * Ci + r) * taps + tap];
      } else {                    // unfolded Cin=1 forward: tap = kd*KH+kh, c = kw
        v = c < unf_kw ? w[((int64_t)r * taps + tap) * unf_kw + c] : 0.f;
      }
    }
    Elt<T>::st(wp, idx, v);
  }
}

template <typename TI, typename TO>
__global__ void unfold_w_kernel(const TI* __restrict__ x, TO* __restrict__ xu, int64_t rows,
                                int Wi, int Wo, int KW, int sw, int pw, int dw) {
  // rows = n*Di*Hi ; output [row][wo][8]
  const int64_t total = rows * Wo;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = idx / Wo;
    const int xo = (int)(idx % Wo);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int xi = xo * sw - pw + j * dw;
      v[j] = (j < KW && xi >= 0 && xi < Wi) ? (float)x[row * Wi + xi] : 0.f;
    }
    if constexpr (sizeof(TO) == 2) {
      Chunk<u16>::store(reinterpret_cast<u16*>(xu) + idx * 8, v);
    } else {
      Chunk<float>::store(reinterpret_cast<float*>(xu) + idx * 8, v);
      Chunk<float>::store(reinterpret_cast<float*>(xu) + idx * 8 + 4, v + 4);
    }
  }
}

// ---- host-side geometry -----------------------------------------------------------
// packed-weight row stride granule: one 128-byte K-slice (igemm2's stage row)
int bk_of(int dtype) { return dtype == MMAD_BF16 ? 64 : 32; }

bool desc_ok(const mmad_conv_desc* d) {
  if (!d) return false;
  const int v[] = {d->n, d->ci, d->di, d->hi, d->wi, d->co, d->do_, d->ho, d->wo, d->kd, d->kh,
                   d->kw, d->sd, d->sh, d->sw, d->dd, d->dh, d->dw};
  for (int x : v) if (x <= 0) return false;
  if (d->pd < 0 || d->ph < 0 || d->pw < 0) return false;
  if (d->kd * d->kh * d->kw > MAXTAPS - 1) return false;
  if ((d->kd - 1) * d->dd > 255 || (d->kh - 1) * d->dh > 255 || (d->kw - 1) * d->dw > 255) return false;
  // output extent must agree with torch's formula
  auto ext = [](int i, int k, int s, int p, int dl) { return (i + 2 * p - dl * (k - 1) - 1) / s + 1; };
  return ext(d->di, d->kd, d->sd, d->pd, d->dd) == d->do_ &&
         ext(d->hi, d->kh, d->sh, d->ph, d->dh) == d->ho &&
         ext(d->wi, d->kw, d->sw, d->pw, d->dw) == d->wo;
}

bool unfolded(const mmad_conv_desc* d) { return d->ci == 1; }

Geom fwd_geom(const mmad_conv_desc* d, int dtype) {
  Geom g{};
  const bool u = unfolded(d);
  g.Cs = u ? 8 : d->ci;
  g.Nd = d->co;
  g.Ds = d->di; g.Hs = d->hi; g.Ws = u ? d->wo : d->wi;
  g.Dd = d->do_; g.Hd = d->ho; g.Wd = d->wo;
  g.KD = d->kd; g.KH = d->kh; g.KW = u ? 1 : d->kw;
  g.sd = d->sd; g.sh = d->sh; g.sw = u ? 1 : d->sw;
  g.pd = d->pd; g.ph = d->ph; g.pw = u ? 0 : d->pw;
  g.dd = d->dd; g.dh = d->dh; g.dw = u ? 1 : d->dw;
  g.taps = g.KD * g.KH * g.KW;
  g.K = g.taps * g.Cs;
  g.Kpad = (int)cdiv(g.K, bk_of(dtype)) * bk_of(dtype);
  g.cs_shift = ilog2(g.Cs);
  g.M = d->n * d->do_ * d->ho * d->wo;
  return g;
}

Geom dgrad_geom(const mmad_conv_desc* d, int dtype) {
  Geom g{};
  g.Cs = d->co; g.Nd = d->ci;
  g.Ds = d->do_; g.Hs = d->ho; g.Ws = d->wo;
  g.Dd = d->di; g.Hd = d->hi; g.Wd = d->wi;
  g.KD = d->kd; g.KH = d->kh; g.KW = d->kw;
  g.sd = d->sd; g.sh = d->sh; g.sw = d->sw;
  g.pd = d->pd; g.ph = d->ph; g.pw = d->pw;
  g.dd = d->dd; g.dh = d->dh; g.dw = d->dw;
  g.taps = g.KD * g.KH * g.KW;
  g.K = g.taps * g.Cs;
  g.Kpad = (int)cdiv(g.K, bk_of(dtype)) * bk_of(dtype);
  g.cs_shift = ilog2(g.Cs);
  g.M = d->n * d->di * d->hi * d->wi;
  return g;
}

bool geom_ok(const Geom& g, int dtype) {
  const int epc = dtype == MMAD_BF16 ? 8 : 4;
  return is_pow2(g.Cs) && g.Cs % epc == 0 && (int64_t)g.M * g.Nd < (int64_t(1) << 40);
}

int bn_of(const Geom& g) { return g.Nd <= 64 ? 64 : 128; }

struct WSplit { int bmw, splits, m_per_split; };
WSplit wgrad_split(const Geom& g) {
  WSplit s{};
  s.bmw = g.Nd <= 64 ? 64 : 128;
  const int64_t tiles = cdiv(g.Nd, s.bmw) * cdiv(g.K, WBN);
  int64_t want = cdiv(1024, tiles);     // ~4 blocks per CU: 2 resident + a second wave
  const int64_t max_split = std::max<int64_t>(1, cdiv(g.M, WBK * 8));
  want = std::max<int64_t>(1, std::min(want, max_split));
  // keep the slab workspace bounded (<= 512 MiB)
  while (want > 1 && want * g.Nd * (int64_t)g.K * 4 > (int64_t(512) << 20)) --want;
  s.m_per_split = (int)(cdiv(cdiv(g.M, want), WBK) * WBK);
  s.splits = (int)cdiv(g.M, s.m_per_split);
  return s;
}

template <typename T, int BN, bool TRANS>
int launch_igemm(const Geom& g, const void* src, const void* w, const float* bias, void* dst,
                 float* stats, hipStream_t st) {
  const size_t lds = TAPB + 2 * BM * ROWB + 2 * BN * ROWB;
  dim3 grid((unsigned)cdiv(g.M, BM), (unsigned)cdiv(g.Nd, BN));
  hipLaunchKernelGGL((igemm_kernel<T, BN, TRANS>), grid, dim3(256), lds, st, g,
                     (const T*)src, (const T*)w, bias, (T*)dst, stats);
  return launch_status();
}

// tile rows: 64 when 128-row tiles would leave the 256 CUs under two blocks each
int igemm_bm(const Geom& g) {
  const int64_t tiles = cdiv(g.M, 128) * cdiv(g.Nd, bn_of(g));
  return tiles < 512 ? 64 : 128;
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

template <typename T, int BN, bool TRANS, int BMT, int NST>
int launch_igemm2_bm(const Geom& g, const void* src, const void* w, const float* bias,
                     void* dst, float* stats, hipStream_t st) {
  const size_t lds = TAPB + NST * (BMT + BN) * RB2;
  static const bool attr_ok =
      lds <= 65536 || hipFuncSetAttribute((const void*)igemm2_kernel<T, BN, TRANS, BMT, NST>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds) == hipSuccess;
  if (!attr_ok) return MMAD_EUNSUPPORTED;
  const int nbm = (int)cdiv(g.M, BMT), nbn = (int)cdiv(g.Nd, BN);
  hipLaunchKernelGGL((igemm2_kernel<T, BN, TRANS, BMT, NST>), dim3((unsigned)(nbm * nbn)),
                     dim3(256), lds, st, g, (const T*)src, (const T*)w, bias, (T*)dst, stats,
                     nbm, nbn);
  return launch_status();
}

template <typename T, int BN, bool TRANS>
int launch_igemm2(const Geom& g, const void* src, const void* w, const float* bias, void* dst,
                  float* stats, hipStream_t st) {
  // ring depth for 128-row tiles: 3 stages need 96 KB (1 block/CU) and measured 0.6x of
  // the 2-stage / 2-blocks-per-CU configuration, so 2 is the default
  static const int nst = env_int("MMAD_NST", 2);
  if (igemm_bm(g) == 64)
    return launch_igemm2_bm<T, BN, TRANS, 64, 2>(g, src, w, bias, dst, stats, st);
  if (nst == 3)
    return launch_igemm2_bm<T, BN, TRANS, 128, 3>(g, src, w, bias, dst, stats, st);
  return launch_igemm2_bm<T, BN, TRANS, 128, 2>(g, src, w, bias, dst, stats, st);
}

// MMAD_IGEMM=1 selects the register-staged v1 kernel (kept for A/B measurements)
bool use_v1() {
  static const bool v = [] {
    const char* e = getenv("MMAD_IGEMM");
    return e != nullptr && e[0] == '1';
  }();
  return v;
}

template <bool TRANS>
int run_igemm(const Geom& g, int dtype, const void* src, const void* w, const float* bias,
              void* dst, float* stats, hipStream_t st) {
  const int bn = bn_of(g);
  if (!use_v1()) {
    if (dtype == MMAD_BF16)
      return bn == 64 ? launch_igemm2<u16, 64, TRANS>(g, src, w, bias, dst, stats, st)
                      : launch_igemm2<u16, 128, TRANS>(g, src, w, bias, dst, stats, st);
    return bn == 64 ? launch_igemm2<float, 64, TRANS>(g, src, w, bias, dst, stats, st)
                    : launch_igemm2<float, 128, TRANS>(g, src, w, bias, dst, stats, st);
  }
  if (dtype == MMAD_BF16)
    return bn == 64 ? launch_igemm<u16, 64, TRANS>(g, src, w, bias, dst, stats, st)
                    : launch_igemm<u16, 128, TRANS>(g, src, w, bias, dst, stats, st);
  return bn == 64 ? launch_igemm<float, 64, TRANS>(g, src, w, bias, dst, stats, st)
                  : launch_igemm<float, 128, TRANS>(g, src, w, bias, dst, stats, st);
}

template <typename T, int BMW>
int launch_wgrad(const Geom& g, const WSplit& sp, const void* x, const void* dy, float* ws,
                 hipStream_t st) {
  if (!use_v1()) {
    const size_t lds2 = TAPB + 2 * WBK * (BMW + WBN) * sizeof(T);
    static const bool ok2 =
        lds2 <= 65536 || hipFuncSetAttribute((const void*)wgrad2_kernel<T, BMW>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds2) == hipSuccess;
    if (!ok2) return MMAD_EUNSUPPORTED;
    dim3 grid2((unsigned)cdiv(g.K, WBN), (unsigned)cdiv(g.Nd, BMW), (unsigned)sp.splits);
    hipLaunchKernelGGL((wgrad2_kernel<T, BMW>), grid2, dim3(256), lds2, st, g, (const T*)x,
                       (const T*)dy, ws, sp.m_per_split);
    return launch_status();
  }
  const size_t arow = BMW * sizeof(T) + 16, brow = WBN * sizeof(T) + 16;
  const size_t lds = TAPB + 2 * WBK * (arow + brow);
  if (lds > 65536) {
    static bool once = [&] {
      return hipFuncSetAttribute((const void*)wgrad_kernel<T, BMW>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    }();
    if (!once) return MMAD_EUNSUPPORTED;
  }
  dim3 grid((unsigned)cdiv(g.K, WBN), (unsigned)cdiv(g.Nd, BMW), (unsigned)sp.splits);
  hipLaunchKernelGGL((wgrad_kernel<T, BMW>), grid, dim3(256), lds, st, g, (const T*)x,
                     (const T*)dy, ws, sp.m_per_split);
  return launch_status();
}

unsigned grid_for(int64_t total, int block = 256) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(total, block), 65536));
}

}  // namespace

// =====================================================================================
extern "C" {

int64_t mmad_conv_packed_elems(const mmad_conv_desc* d, int dtype, int for_dgrad) {
  if (!desc_ok(d)) return -1;
  const Geom g = for_dgrad ? dgrad_geom(d, dtype) : fwd_geom(d, dtype);
  return (int64_t)g.Nd * g.Kpad;
}

int mmad_conv_pack_weight(const mmad_conv_desc* d, int dtype, const float* w, void* wp,
                          int for_dgrad, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!w || !wp) return MMAD_ENULL;
  if (for_dgrad && unfolded(d)) return MMAD_EUNSUPPORTED;
  const Geom g = for_dgrad ? dgrad_geom(d, dtype) : fwd_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  const int mode = for_dgrad ? 1 : (unfolded(d) ? 2 : 0);
  const int64_t total = (int64_t)g.Nd * g.Kpad;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<u16>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), w, (u16*)wp, g.Nd, g.Kpad, g.K, g.Cs, g.cs_shift,
                       g.taps, mode, d->ci, d->kw);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), w, (float*)wp, g.Nd, g.Kpad, g.K, g.Cs, g.cs_shift,
                       g.taps, mode, d->ci, d->kw);
  return launch_status();
}

int64_t mmad_conv_unfolded_elems(const mmad_conv_desc* d) {
  if (!desc_ok(d) || !unfolded(d)) return -1;
  return (int64_t)d->n * d->di * d->hi * d->wo * 8;
}

int mmad_conv_unfold_input(const mmad_conv_desc* d, int in_dtype, const void* x, int dtype,
                           void* xu, void* stream) {
  if (!desc_ok(d) || !unfolded(d)) return MMAD_EBADSHAPE;
  if (d->kw > 8) return MMAD_EUNSUPPORTED;
  if (!x || !xu) return MMAD_ENULL;
  const int64_t rows = (int64_t)d->n * d->di * d->hi;
  const unsigned grid = grid_for(rows * d->wo);
  hipStream_t st = as_stream(stream);
#define UNF(TI, TO)                                                                    \
  hipLaunchKernelGGL((unfold_w_kernel<TI, TO>), dim3(grid), dim3(256), 0, st, (const TI*)x, \
                     (TO*)xu, rows, d->wi, d->wo, d->kw, d->sw, d->pw, d->dw)
  if (dtype == MMAD_BF16) {
    if (in_dtype == MMAD_F64) UNF(double, u16);
    else if (in_dtype == MMAD_F32) UNF(float, u16);
    else return MMAD_EBADDTYPE;
  } else if (dtype == MMAD_F32) {
    if (in_dtype == MMAD_F64) UNF(double, float);
    else if (in_dtype == MMAD_F32) UNF(float, float);
    else return MMAD_EBADDTYPE;
  } else {
    return MMAD_EBADDTYPE;
  }
#undef UNF
  return launch_status();
}

int64_t mmad_conv3d_stats_rows(const mmad_conv_desc* d, int dtype) {
  if (!desc_ok(d)) return -1;
  const Geom g = fwd_geom(d, dtype);
  return cdiv(g.M, use_v1() ? BM : igemm_bm(g));
}

int mmad_conv3d_fwd(const mmad_conv_desc* d, int dtype, const void* x, const void* wp,
                    const float* bias, void* y, float* stats, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!x || !wp || !y) return MMAD_ENULL;
  const Geom g = fwd_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  return run_igemm<false>(g, dtype, x, wp, bias, y, stats, as_stream(stream));
}

int mmad_conv3d_dgrad(const mmad_conv_desc* d, int dtype, const void* dy, const void* wpt,
                      void* dx, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!dy || !wpt || !dx) return MMAD_ENULL;
  if (unfolded(d)) return MMAD_EUNSUPPORTED;   // the raw input never needs a gradient
  const Geom g = dgrad_geom(d, dtype);
  if (!geom_ok(g, dtype) || d->ci % (dtype == MMAD_BF16 ? 8 : 4)) return MMAD_EUNSUPPORTED;
  return run_igemm<true>(g, dtype, dy, wpt, nullptr, dx, nullptr, as_stream(stream));
}

int64_t mmad_conv3d_wgrad_workspace(const mmad_conv_desc* d, int dtype) {
  if (!desc_ok(d)) return -1;
  const Geom g = fwd_geom(d, dtype);
  const WSplit sp = wgrad_split(g);
  const int64_t slabs = (int64_t)sp.splits * g.Nd * g.K * 4;
  const int64_t parts = (int64_t)1024 * 2 * g.Nd * 4;   // bias-gradient column sums
  return std::max(slabs, parts);
}

int mmad_colsum_ws(int dtype, int64_t m, int c, const void* y, float* parts, float* out,
                   void* stream);

int mmad_conv3d_wgrad(const mmad_conv_desc* d, int dtype, const void* x, const void* dy,
                      float* dw, float* dbias, void* workspace, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!x || !dy || !dw || !workspace) return MMAD_ENULL;
  const Geom g = fwd_geom(d, dtype);
  if (!geom_ok(g, dtype) || g.Nd % (dtype == MMAD_BF16 ? 8 : 4)) return MMAD_EUNSUPPORTED;
  const WSplit sp = wgrad_split(g);
  hipStream_t st = as_stream(stream);
  int rc;
  if (dtype == MMAD_BF16)
    rc = sp.bmw == 64 ? launch_wgrad<u16, 64>(g, sp, x, dy, (float*)workspace, st)
                      : launch_wgrad<u16, 128>(g, sp, x, dy, (float*)workspace, st);
  else
    rc = sp.bmw == 64 ? launch_wgrad<float, 64>(g, sp, x, dy, (float*)workspace, st)
                      : launch_wgrad<float, 128>(g, sp, x, dy, (float*)workspace, st);
  if (rc) return rc;
  const int64_t total = (int64_t)g.Nd * g.K;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for(total)), dim3(256), 0, st,
                     (const float*)workspace, dw, sp.splits, g.Nd, g.K, g.Cs, g.cs_shift,
                     g.taps, unfolded(d) ? d->kw : 0);
  rc = launch_status();
  if (rc) return rc;
  if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, stream);
  return MMAD_OK;
}

}  // extern "C"
