// 3D convolution as MFMA implicit GEMM on gfx950.
//
// Replaces torch.nn.Conv3d forward / backward for every conv of the reference hot path
// (MedicalNet stem + BasicBlock / Bottleneck / shortcut-B convs used at
// pkg/models/mri_models/anat_cnn.py:29-31, head convs anat_cnn.py:55-63, Small_PET_CNN
// convs pkg/models/pet_models/pet_cnn.py:20-22).
//
// Data layout: NDHWC activations ("voxel-major"), so the GEMM K dimension
// (tap, input channel) is channel-contiguous and every operand load is a 16-byte vector.
// GEMM view of one conv:
//   forward : Y[m, co]  = sum_{tap, ci} X[m*s - p + tap*d, ci] * W[co, tap, ci]
//   dgrad   : dX[i, ci] = sum_{tap, co} dY[(i + p - tap*d) / s, co] * W[co, tap, ci]
//   wgrad   : dW[co, k] = sum_m dY[m, co] * X[m*s - p + tap(k)*d, ci(k)]   (split over m)
// dgrad is run per stride-parity class of the output voxels (s^3 classes): inside a class
// only the taps with (i + p - tap*d) divisible by s contribute and the division is exact,
// so every class is a dense stride-1 gather with its own tap list -- no MFMA is spent on
// stride holes (the naive transposed gather wastes 7/8 of them at stride 2).
// Input-channel counts of 1 (the stem, PET conv 1) are handled by unfolding the input
// along W into 8 "channels" (j = kw tap, zero-padded), which turns the conv into a
// (kd, kh, 1) conv with Cin = 8 and keeps the vector path.
//
// Kernel structure (igemm_kernel / wgrad_kernel):
//  * 256-thread blocks = 4 waves (2x2), MFMA 16x16x32 bf16 (16x16x4 f32, exact f32);
//  * operands move global -> LDS with global_load_lds_dwordx4 (no VGPR staging): a wave
//    instruction fills 1 KB of tile; each lane supplies its own source address, so the
//    implicit-GEMM gather, zero padding (lanes pointed at a 128-B zero block in the code
//    object) and stride holes cost no extra instructions;
//  * LDS rows XOR-swizzled in 16-byte slots (applied on the SOURCE address so the DMA image
//    stays lane-linear) -> conflict-free fragment reads;
//  * 2-stage ring, one barrier per stage, 2 blocks per CU (a 3-stage ring needs 96 KB = 1
//    block/CU and measured 0.6x);
//  * XCD-aware tile order: each XCD walks a contiguous range of (m, n) tiles, n fastest;
//  * epilogue: bias, BN partial sums (sum, sum of squares per channel) from the fp32
//    accumulators, bf16 tile transposed through LDS into 16-byte channel-vector stores.
#include "common.h"
#include "reduce.h"
#include "patchconv.h"
#include "pointwise.h"
#include "stem.h"

namespace {

constexpr int MAXTAPS = 344;
constexpr int TAPB = ((3 * MAXTAPS * 4 + 15) / 16) * 16;   // tap offsets, indices, deltas
constexpr int RB = 128;                                      // K bytes per stage row

struct Geom {
  int M, Nd, Cs, K, Kpad, cs_shift, taps, nb;
  int Ds, Hs, Ws, Dd, Hd, Wd;
  int KD, KH, KW;
  int sd, sh, sw, pd, ph, pw, dd, dh, dw;
  // forward epilogue extras (eval-mode fused conv+BN(+residual)+ReLU): residual tensor
  // shaped like the output (added after bias), ReLU flag
  const void* res;
  int relu;
};

enum { FWD = 0, DGRAD = 1 };

__device__ const u32x4 g_zero_chunk[8] = {};

__device__ __forceinline__ int pack_off(int oz, int oy, int ox) {
  return (oz + 128) | ((oy + 128) << 8) | ((ox + 128) << 16);
}

// Source voxel of (base coords, packed signed tap offsets); false = padding.
__device__ __forceinline__ bool src_voxel(const Geom& g, int bz, int by, int bx, int to, int& z,
                                          int& y, int& x) {
  z = bz + (to & 255) - 128;
  y = by + ((to >> 8) & 255) - 128;
  x = bx + ((to >> 16) & 255) - 128;
  return (unsigned)z < (unsigned)g.Ds && (unsigned)y < (unsigned)g.Hs &&
         (unsigned)x < (unsigned)g.Ws;
}

// forward tap table: offsets kd*d (base = out*s - p)
__device__ __forceinline__ void fill_taps_fwd(const Geom& g, int* tapoff) {
  for (int t = threadIdx.x; t < g.taps; t += blockDim.x) {
    const int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
    tapoff[t] = pack_off(kd * g.dd, kh * g.dh, kw * g.dw);
  }
}

// ---- implicit GEMM (forward / per-parity-class dgrad) --------------------------------
// Block = WGM x WGN waves, tile BM voxels x BN channels, NST-deep LDS ring with NST-1 stages
// of LDS-DMA in flight (asm DMA + counted vmcnt + raw barrier, see wgrad_kernel).
// RBT = K bytes per stage row: 128 (8 x 16-B chunks, XOR swizzle row & 7) or 64 (bf16 only:
// 4 chunks, swizzle 3 * ((row >> 3) & 1), which keeps every 16-lane ds_read_b128 group on 16
// distinct bank slots); 64-B rows halve the stage so the same LDS holds twice the stages
// in flight.
template <typename T, int BN, int MODE, int BM, int WGM = 2, int WGN = 2, int NST = 2,
          int RBT = RB>
__global__ __launch_bounds__(64 * WGM * WGN) void igemm_kernel(Geom g, const T* __restrict__ src,
                                                       const T* __restrict__ wgt,
                                                       const float* __restrict__ bias,
                                                       T* __restrict__ dst,
                                                       float* __restrict__ stats, int nbm,
                                                       int nbn) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = RBT / (int)sizeof(T);
  static_assert(RBT == 128 || (RBT == 64 && sizeof(T) == 2), "stage row bytes");
  constexpr int RPI = 1024 / RBT;                        // tile rows per DMA instruction
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;          // per-wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * RBT, B_BYTES = BN * RBT, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = A_BYTES / (1024 * NW), BI = B_BYTES / (1024 * NW);
  static_assert(AI * 1024 * NW == A_BYTES && BI * 1024 * NW == B_BYTES, "tile/wave split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  int* tapidx = tapoff + MAXTAPS;
  int* tapdelta = tapidx + MAXTAPS;
  char* ring = smem + TAPB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = tile / nbn, nt = tile % nbn;

  // dst lattice: the whole output grid (FWD) or one stride-parity class of dX (DGRAD)
  int pz = 0, py = 0, px = 0, Dc = g.Dd, Hc = g.Hd, Wc = g.Wd, Mc = g.M;
  if (MODE == DGRAD) {
    // classes dispatch in blockIdx.y order; the all-odd class (index sd*sh*sw - 1) has the
    // most taps (2^3 for a stride-2 3^3 conv vs 1 for all-even), so run it first: the light
    // classes then fill the tail instead of the heavy ones extending it
    const int cls = (int)gridDim.y - 1 - (int)blockIdx.y;
    px = cls % g.sw; py = (cls / g.sw) % g.sh; pz = cls / (g.sw * g.sh);
    Dc = (g.Dd - pz + g.sd - 1) / g.sd;
    Hc = (g.Hd - py + g.sh - 1) / g.sh;
    Wc = (g.Wd - px + g.sw - 1) / g.sw;
    Mc = g.nb * Dc * Hc * Wc;
  }
  if (mt * BM >= Mc) return;                      // uniform: class smaller than the grid
  const int m0 = mt * BM, n0 = nt * BN;

  int ntap = g.taps, Kc = g.K;
  if (MODE == FWD) {
    fill_taps_fwd(g, tapoff);
  } else {
    // (count kept in the unused last tap-index slot: a second __shared__ object beside
    // the LDS-DMA ring makes hipcc drain vmcnt before every ds_read)
    if (tid == 0) {
      int n = 0;
      for (int t = 0; t < g.taps; ++t) {
        const int kw = t % g.KW, kh = (t / g.KW) % g.KH, kd = t / (g.KW * g.KH);
        const int vz = pz + g.pd - kd * g.dd, vy = py + g.ph - kh * g.dh,
                  vx = px + g.pw - kw * g.dw;
        if (vz % g.sd || vy % g.sh || vx % g.sw) continue;
        tapoff[n] = pack_off(vz / g.sd, vy / g.sh, vx / g.sw);
        tapidx[n] = t;
        ++n;
      }
      tapidx[MAXTAPS - 1] = n;
    }
    __syncthreads();
    ntap = tapidx[MAXTAPS - 1];
    Kc = ntap * g.Cs;
  }

  // this lane's A rows: one per DMA instruction, row = (wave*AI + i)*RPI + lane/(RBT/16)
  const int lrow = RBT == 128 ? lane >> 3 : lane >> 2;
  const int lchunk = RBT == 128 ? (lane & 7) ^ lrow              // logical K chunk fetched
                                : (lane & 3) ^ (3 * ((lrow >> 3) & 1));
  int rz[AI], ry[AI], rx[AI];
  int64_t rbase[AI];
  bool rok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (wave * AI + i) * RPI + lrow;
    rok[i] = m < Mc;
    const int mm = rok[i] ? m : 0;
    const int xw = mm % Wc;
    int t1 = mm / Wc;
    const int yh = t1 % Hc;
    t1 /= Hc;
    const int zd = t1 % Dc, nbi = t1 / Dc;
    if (MODE == FWD) {
      rz[i] = zd * g.sd - g.pd; ry[i] = yh * g.sh - g.ph; rx[i] = xw * g.sw - g.pw;
    } else {
      rz[i] = zd; ry[i] = yh; rx[i] = xw;          // class lattice coords: src = j + offset
    }
    rbase[i] = (int64_t)nbi * g.Ds;
  }
  __syncthreads();

  // With <= 64 taps, resolve padding once per row: bit t of rmask = tap t lands inside the
  // source volume, and the source address is row voxel + a per-tap voxel delta, so a DMA
  // issue costs a bit test and one add instead of three bounds checks and a 3-D index.
  // Building the masks costs about one issue per tap, so it only pays when every tap spans
  // several K stages (wide channel slices).
  const bool use_mask = ntap <= 64 && g.Cs * (int)sizeof(T) >= 512;
  uint64_t rmask[AI];
  int64_t rvox[AI];
  if (use_mask) {
    for (int t = tid; t < ntap; t += NT) {
      const int to = tapoff[t];
      tapdelta[t] = (((to & 255) - 128) * g.Hs + (((to >> 8) & 255) - 128)) * g.Ws +
                    (((to >> 16) & 255) - 128);
    }
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      uint64_t msk = 0;
      if (rok[i])
        for (int t = 0; t < ntap; ++t) {
          int z, y, x;
          if (src_voxel(g, rz[i], ry[i], rx[i], tapoff[t], z, y, x)) msk |= uint64_t(1) << t;
        }
      rmask[i] = msk;
      rvox[i] = ((rbase[i] + rz[i]) * g.Hs + ry[i]) * g.Ws + rx[i];
    }
    __syncthreads();
  }

#ifndef MMAD_IGEMM_CULL
#define MMAD_IGEMM_CULL 1                  // (-DMMAD_IGEMM_CULL=0: variant build for A/B)
#endif
  // Tap culling (round 5, bf16 forward): a tap that lands in the padding for EVERY row of
  // the tile (e.g. the z-shifted taps of a tile inside the first / last d planes of a dilated
  // 'same' conv: config 5's 20^3 layer3 / layer4) is dropped from the tile's K loop -- no
  // DMA, no MFMA.  Its MACs were exact zeros, so the outputs are bit-identical.  The union of
  // the rows' masks decides; the tap tables are compacted in place and the weights addressed
  // through tapidx (as DGRAD does), each row's mask compressed to the kept taps.
  bool culled = false;
  if constexpr (MODE == FWD && sizeof(T) == 2 && MMAD_IGEMM_CULL) {
    if (use_mask && ntap > 1) {
      uint64_t u = 0;
#pragma unroll
      for (int i = 0; i < AI; ++i) u |= rmask[i];
      uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        lo |= __shfl_xor(lo, o, 64);
        hi |= __shfl_xor(hi, o, 64);
      }
      uint32_t* un = reinterpret_cast<uint32_t*>(tapidx + MAXTAPS - 2 * NW - 2);
      if (lane == 0) {
        un[2 * wave] = lo;
        un[2 * wave + 1] = hi;
      }
      __syncthreads();
      uint64_t full = 0;
      for (int w = 0; w < NW; ++w) full |= (uint64_t)un[2 * w] | ((uint64_t)un[2 * w + 1] << 32);
      const uint64_t all = ntap == 64 ? ~uint64_t(0) : (uint64_t(1) << ntap) - 1;
      if (full != all) {
        culled = true;
        __syncthreads();                       // every wave has read the union words
        if (tid == 0) {
          int n = 0;
          for (int t = 0; t < ntap; ++t) {
            if (!((full >> t) & 1)) continue;
            tapoff[n] = tapoff[t];
            tapdelta[n] = tapdelta[t];
            tapidx[n] = t;
            ++n;
          }
          tapidx[MAXTAPS - 1] = n;
        }
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          uint64_t c = 0;
          int j = 0;
          for (int t = 0; t < ntap; ++t) {
            if (!((full >> t) & 1)) continue;
            c |= ((rmask[i] >> t) & 1) << j;
            ++j;
          }
          rmask[i] = c;
        }
        __syncthreads();
        ntap = tapidx[MAXTAPS - 1];
        Kc = ntap * g.Cs;
      }
    }
  }

  auto issue = [&](int stage, int k0) {
    char* sbase = ring + stage * STAGE;
    const int k = k0 + lchunk * EPC;
    const bool kok = k < Kc;
    const int ti = k >> g.cs_shift, ci = k & (g.Cs - 1);
    if (use_mask) {
      const int td = kok ? tapdelta[ti] : 0;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const void* p = g_zero_chunk;
        if (kok && ((rmask[i] >> ti) & 1)) p = src + ((rvox[i] + td) << g.cs_shift) + ci;
        glds16_asm(p, lds_addr_of(sbase + (wave * AI + i) * 1024));
      }
    } else {
      const int to = kok ? tapoff[ti] : 0;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const void* p = g_zero_chunk;
        int z, y, x;
        if (rok[i] && kok && src_voxel(g, rz[i], ry[i], rx[i], to, z, y, x)) {
          const int64_t vox = ((rbase[i] + z) * g.Hs + y) * g.Ws + x;
          p = src + (vox << g.cs_shift) + ci;
        }
        glds16_asm(p, lds_addr_of(sbase + (wave * AI + i) * 1024));
      }
    }
    const int woff = MODE == FWD && !culled ? k : (kok ? (tapidx[ti] << g.cs_shift) + ci : 0);
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int co = n0 + (wave * BI + i) * RPI + lrow;
      const void* p = (co < g.Nd && kok) ? (const void*)(wgt + (int64_t)co * g.Kpad + woff)
                                         : (const void*)g_zero_chunk;
      glds16_asm(p, lds_addr_of(sbase + A_BYTES + (wave * BI + i) * 1024));
    }
  };

  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 15, lk = lane >> 4;
  const int sw8 = RBT == 128 ? lr & 7 : 3 * ((lr >> 3) & 1);   // swizzle of this lane's rows
  // fp32 mode sums K in two levels (fresh partial every FLUSH stages): one f32 MFMA chain
  // over K = 27*512 terms grows the rounding error ~K-fold and flips ReLU masks.
  constexpr int FLUSH = 8;
  f32x4 acc[TM][TN], part[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* a = ring + stage * STAGE + (wm * WTM + lr) * RBT;
    const char* b = ring + stage * STAGE + A_BYTES + (wn * WTN + lr) * RBT;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        const int off = ((4 * s + lk) ^ sw8) << 4;
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(a + i * 16 * RBT + off);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(b + j * 16 * RBT + off);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < BK / 4; ++s) {
        const int off = ((s ^ sw8) << 4) + lk * 4;
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const float*>(a + i * 16 * RBT + off);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const float*>(b + j * 16 * RBT + off);
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

  const int nk = (Kc + BK - 1) / BK;
  constexpr int LPS = AI + BI;                   // DMA instructions per stage per wave
  constexpr int PD = NST - 1;                    // stages in flight
  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < PD; ++s)
      if (s < nk) issue(s, s * BK);
    for (int ks = 0; ks < nk; ++ks) {
      const int younger = min(PD - 1, nk - 1 - ks);
      if constexpr (PD >= 3) {
        if (younger >= 2) wait_vm_lgkm0<2 * LPS>();
        else if (younger == 1) wait_vm_lgkm0<LPS>();
        else wait_vm_lgkm0<0>();
      } else if constexpr (PD == 2) {
        if (younger >= 1) wait_vm_lgkm0<LPS>();
        else wait_vm_lgkm0<0>();
      } else {
        wait_vm_lgkm0<0>();
      }
      raw_barrier();
      if (ks + PD < nk) issue((ks + PD) % NST, (ks + PD) * BK);
      compute(ks % NST);
      if (ks % FLUSH == FLUSH - 1) flush();
    }
  }
  flush();
  __syncthreads();                               // ring reused by the epilogue

  // dst voxel of a tile row
  auto dst_row = [&](int m) -> int64_t {
    if (MODE == FWD) return m;
    const int xw = m % Wc;
    int t1 = m / Wc;
    const int yh = t1 % Hc;
    t1 /= Hc;
    const int zd = t1 % Dc, nbi = t1 / Dc;
    return (((int64_t)nbi * g.Dd + zd * g.sd + pz) * g.Hd + yh * g.sh + py) * g.Wd +
           xw * g.sw + px;
  };

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
    const int col = wn * WTN + j * 16 + lr;
    const int co = n0 + col;
    const float bv = (bias != nullptr && co < g.Nd) ? bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + i * 16 + lk * 4 + r;
        const int m = m0 + row;
        const float v = acc[i][j][r] + bv;
        if (lds_out) ctile[row * (CROW / 2) + col] = f2bf(v);
        if (m < Mc && co < g.Nd) {
          if (!lds_out) {
            const int64_t o = dst_row(m) * g.Nd + co;
            float w = v;
            if (MODE == FWD && g.res != nullptr) w += Elt<T>::ld((const T*)g.res, o);
            if (MODE == FWD && g.relu) w = fmaxf(w, 0.f);
            Elt<T>::st(dst, o, w);
          }
          cs[j] += v;
          cq[j] += v * v;
        }
      }
  }
  if (lds_out) {
    __syncthreads();
    constexpr int CPR = BN / 8;
#pragma unroll
    for (int h = 0; h < BM * CPR / NT; ++h) {
      const int q = tid + NT * h;
      const int row = q / CPR, c8 = q % CPR;
      const int m = m0 + row, co = n0 + c8 * 8;
      if (m < Mc && co < g.Nd) {
        const int64_t o = dst_row(m) * g.Nd + co;
        u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                  row * CROW + c8 * 16);
        if (MODE == FWD && (g.res != nullptr || g.relu))
          v = epi_res_relu(v, g.res ? reinterpret_cast<const u16*>(g.res) + o : nullptr, g.relu);
        *reinterpret_cast<u32x4*>(reinterpret_cast<u16*>(dst) + o) = v;
      }
    }
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(ring + 1024 + BM * CROW);   // past the C tile
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm > 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + lr;
        red[(wm - 1) * 2 * BN + col] = cs[j];
        red[(wm - 1) * 2 * BN + BN + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + lr;
        const int co = n0 + col;
        float ss = cs[j], qs = cq[j];
        for (int w = 1; w < WGM; ++w) {        // fixed order: deterministic
          ss += red[(w - 1) * 2 * BN + col];
          qs += red[(w - 1) * 2 * BN + BN + col];
        }
        if (co < g.Nd) {
          stats[((int64_t)mt * 2) * g.Nd + co] = ss;
          stats[((int64_t)mt * 2 + 1) * g.Nd + co] = qs;
        }
      }
    }
  }
}

// ---- weight gradient -------------------------------------------------------------------
// dW[co][k] = sum_m dY[m][co] * X(m, k): block tile BMW (co) x 128 (k), 32 voxels per stage,
// split over m into `splits` slices -> fp32 partial slabs ws[s][co][k].  Both tiles are
// m-major images ([m][co] of dY, [m][k] of the gathered X); rows XOR-swizzled so the
// transposing fragment reads of 8 m-rows x 16 columns (bf16: ds_read_b64_tr_b16) or
// 2 m-rows x 16 columns (f32: ds_read_b32) hit distinct banks.
constexpr int WBN = 128;
template <typename T>
constexpr int wbk() { return 32; }
int wbk_of(int) { return 32; }   // 64 measured slower (fewer blocks per CU)

template <typename T, int ROWB>
__device__ __forceinline__ int wswz(int r) {
  if constexpr (sizeof(T) == 4) return 4 * (r & 1);
  else if constexpr (ROWB >= 256) return 2 * (r & 3) + 8 * ((r >> 3) & 1);
  else return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1);
}

// Operand DMA uses buffer_load ... lds with 32-bit byte offsets into one buffer resource
// per tensor: out-of-range offsets (padding taps, rows past the split, k past K) read as
// zeros in hardware, so no zero-block pointer select and no 64-bit address math.  Each B
// row's source voxel is tracked incrementally (32-bit, one add per stage plus carry
// corrections) instead of re-deriving ((n*D + z)*H + y)*W + x; with XFIX (the stage step
// is a whole number of output rows, WBK % Wd == 0) x never changes, so the x test is made
// once and only y/z carry.  (Index math was ~1/4 of the kernel's time: a build with the B
// addressing stubbed out ran 12-30 % faster.)
template <typename T, int BMW, int WBK, int NST, int WBNT = WBN, int WGM = 2, int WGN = 2,
          bool XFIX = false>
__global__ __launch_bounds__(64 * WGM * WGN) void wgrad_kernel(Geom g, const T* __restrict__ src,
                                                       const T* __restrict__ dy,
                                                       float* __restrict__ ws, int m_per_split,
                                                       uint32_t src_bytes, uint32_t dy_bytes,
                                                       int xcd_remap) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int NW = WGM * WGN;
  constexpr int AROWB = BMW * (int)sizeof(T), BROWB = WBNT * (int)sizeof(T);
  constexpr int A_BYTES = WBK * AROWB, B_BYTES = WBK * BROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int ARPI = 1024 / AROWB, BRPI = 1024 / BROWB;      // rows per DMA instruction
  constexpr int ALPR = AROWB / 16, BLPR = BROWB / 16;         // lanes per row
  constexpr int AIPW = A_BYTES / (1024 * NW), BIPW = B_BYTES / (1024 * NW);   // per wave
  static_assert(AIPW * 1024 * NW == A_BYTES && BIPW * 1024 * NW == B_BYTES, "wave split");
  constexpr int TI = BMW / WGM / 16, TJ = WBNT / WGN / 16;
  constexpr uint32_t OOB = 0x80000000u;                        // >= any buffer size used
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* tapoff = reinterpret_cast<int*>(smem);
  char* ring = smem + TAPB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware block order: the hardware deals workgroups round-robin over the 8 XCDs, so
  // in launch order the k-tiles of one m-split (which read the same dY rows and shifted
  // views of the same X rows) would land on 8 different L2s.  Each XCD instead walks a
  // contiguous range of (k-tile, co-tile, split) tiles, k fastest.
  int bxk = blockIdx.x, byc = blockIdx.y, bzs = blockIdx.z;
  if (xcd_remap) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int nwg = nx * ny * gridDim.z;
    const int bid = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
    const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
    const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    bxk = tile % nx;
    byc = (tile / nx) % ny;
    bzs = tile / (nx * ny);
  }
  const int k0 = bxk * WBNT, co0 = byc * BMW;
  const int mbeg = bzs * m_per_split;
  const int mend = min(g.M, mbeg + m_per_split);
  fill_taps_fwd(g, tapoff);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)src, 0, (int)__builtin_amdgcn_readfirstlane(src_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy, 0, (int)__builtin_amdgcn_readfirstlane(dy_bytes), 0x00020000);

  // A chunks (dY rows, fixed channel slice per lane): byte offset advances WBK rows a stage
  uint32_t aoff[AIPW];
  int arow[AIPW];
  bool acok[AIPW];
#pragma unroll
  for (int i = 0; i < AIPW; ++i) {
    arow[i] = (wave * AIPW + i) * ARPI + lane / ALPR;
    const int aco = co0 + ((lane % ALPR) ^ wswz<T, AROWB>(arow[i])) * EPC;
    acok[i] = aco < g.Nd;
    aoff[i] = (uint32_t)(((int64_t)(mbeg + arow[i]) * g.Nd + aco) * (int)sizeof(T));
  }
  const uint32_t astep = (uint32_t)WBK * g.Nd * (int)sizeof(T);

  // B chunks: fixed (tap, ci) per instruction; rows advance WBK voxels per stage as a
  // mixed-radix (x, y, z, n) add with at most one carry per digit (step digits < radix)
  const int sx = WBK % g.Wd;
  int qq = WBK / g.Wd;
  const int sy = qq % g.Hd;
  qq /= g.Hd;
  const int sz = qq % g.Dd, sn = qq / g.Dd;
  // source-voxel deltas: base step, and the corrections a carry out of x / y / z adds
  const int HW = g.Hs * g.Ws, DHW = g.Ds * HW;
  const int dstep = sx * g.sw + sy * g.sh * g.Ws + sz * g.sd * HW + sn * DHW;
  const int dcx = -g.Wd * g.sw + g.sh * g.Ws;
  const int dcy = -g.Hd * g.sh * g.Ws + g.sd * HW;
  const int dcz = -g.Dd * g.sd * HW + DHW;
  const int bshift = g.cs_shift + (sizeof(T) == 2 ? 1 : 2);
  int bci2[BIPW], bx[BIPW], by[BIPW], bz[BIPW], box[BIPW], boy[BIPW], boz[BIPW];
  int srow[BIPW], tdel[BIPW];
#pragma unroll
  for (int i = 0; i < BIPW; ++i) {
    const int brow = (wave * BIPW + i) * BRPI + lane / BLPR;
    const int k = k0 + ((lane % BLPR) ^ wswz<T, BROWB>(brow)) * EPC;
    const bool kok = k < g.K;
    bci2[i] = (k & (g.Cs - 1)) * (int)sizeof(T);
    const int to = tapoff[kok ? (k >> g.cs_shift) : 0];
    box[i] = ((to >> 16) & 255) - 128 - g.pw;
    boy[i] = ((to >> 8) & 255) - 128 - g.ph;
    boz[i] = (to & 255) - 128 - g.pd;
    if (!kok) boy[i] = -(1 << 20);              // k past K: the y test always fails
    tdel[i] = (boz[i] * g.Hs + boy[i]) * g.Ws + box[i];
    int m = mbeg + brow;
    bx[i] = m % g.Wd; m /= g.Wd;
    by[i] = m % g.Hd; m /= g.Hd;
    bz[i] = m % g.Dd;
    const int bn = m / g.Dd;
    srow[i] = bn * DHW + bz[i] * g.sd * HW + by[i] * g.sh * g.Ws + bx[i] * g.sw;
    if (XFIX && (unsigned)(bx[i] * g.sw + box[i]) >= (unsigned)g.Ws) boy[i] = -(1 << 20);
  }

  auto issue = [&](int stage, int mk) {
    char* sbase = ring + stage * STAGE;
#pragma unroll
    for (int i = 0; i < AIPW; ++i) {
      const bool ok = acok[i] && mk + arow[i] < mend;
      buf_lds16_asm(ok ? aoff[i] : OOB, rsy, lds_addr_of(sbase + (wave * AIPW + i) * 1024));
      aoff[i] += astep;
    }
#pragma unroll
    for (int i = 0; i < BIPW; ++i) {
      bool ok = (unsigned)(by[i] * g.sh + boy[i]) < (unsigned)g.Hs &&
                (unsigned)(bz[i] * g.sd + boz[i]) < (unsigned)g.Ds;
      if (!XFIX) ok = ok && (unsigned)(bx[i] * g.sw + box[i]) < (unsigned)g.Ws;
      const uint32_t off = ((uint32_t)(srow[i] + tdel[i]) << bshift) + bci2[i];
      buf_lds16_asm(ok ? off : OOB, rsx, lds_addr_of(sbase + A_BYTES + (wave * BIPW + i) * 1024));
      int d = dstep, cx = 0;
      if (!XFIX) {
        bx[i] += sx;
        cx = bx[i] >= g.Wd;
        bx[i] -= cx ? g.Wd : 0;
        d += cx ? dcx : 0;
      }
      by[i] += sy + cx;
      const int cy = by[i] >= g.Hd;
      by[i] -= cy ? g.Hd : 0;
      bz[i] += sz + cy;
      const int cz = bz[i] >= g.Dd;
      bz[i] -= cz ? g.Dd : 0;
      d += cy ? dcy : 0;
      d += cz ? dcz : 0;
      srow[i] += d;
    }
  };

  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 15, lk = lane >> 4;
  constexpr int FLUSH = 4;    // fp32: fresh partial every 4 stages (128 voxels)
  f32x4 acc[TI][TJ], part[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bf16: every fragment of a stage is read into registers first (the transposing LDS reads
  // make hipcc wait for all LDS-DMA in flight, so the next stage's DMA is issued after
  // them), then the MFMAs run while that DMA lands.
  constexpr int KH = WBK / 32;
  bf16x8 fa[KH][TI], fb[KH][TJ];
  auto read_frags = [&](int stage) {
    const char* a = ring + stage * STAGE;
    const char* b = a + A_BYTES;
    // lane 4q+p of each 16-lane group lk reads m-rows 8lk+q (+4), columns 4p..4p+3
    const int q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const int r0 = 32 * kh + 8 * lk + q, r1 = r0 + 4;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int col = wm * (BMW / WGM) + i * 16 + 4 * p;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const char* lo = a + r0 * AROWB + ((ch ^ wswz<T, AROWB>(r0)) << 4) + hb;
        const char* hi = a + r1 * AROWB + ((ch ^ wswz<T, AROWB>(r1)) << 4) + hb;
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)lo);
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)hi);
        fa[kh][i] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = wn * (WBNT / WGN) + j * 16 + 4 * p;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const char* lo = b + r0 * BROWB + ((ch ^ wswz<T, BROWB>(r0)) << 4) + hb;
        const char* hi = b + r1 * BROWB + ((ch ^ wswz<T, BROWB>(r1)) << 4) + hb;
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)lo);
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)hi);
        fb[kh][j] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
  };
  auto mma_frags = [&]() {
#pragma unroll
    for (int kh = 0; kh < KH; ++kh)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kh][i], fb[kh][j], acc[i][j],
                                                              0, 0, 0);
  };

  auto compute = [&](int stage) {
    const char* a = ring + stage * STAGE;
    const char* b = a + A_BYTES;
    if constexpr (sizeof(T) == 2) {
      (void)a; (void)b;
    } else {
#pragma unroll
      for (int s = 0; s < WBK / 4; ++s) {
        const int row = s * 4 + lk;
        float fa[TI], fb[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int col = wm * (BMW / WGM) + i * 16 + lr;
          fa[i] = *reinterpret_cast<const float*>(
              a + row * AROWB + (((col >> 2) ^ wswz<T, AROWB>(row)) << 4) + (col & 3) * 4);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int col = wn * (WBNT / WGN) + j * 16 + lr;
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

  // NST-deep ring, NST-1 stages of DMA in flight (asm DMA: hipcc adds no drains).  At the
  // top of step ks: wait until only the younger stages' DMA is outstanding, barrier (all
  // waves' DMA for ks landed; all waves done reading ks-1), refill buffer (ks-1) % NST.
  const int nk = (mend - mbeg + WBK - 1) / WBK;
  constexpr int LPS = AIPW + BIPW;          // DMA instructions per stage per wave
  constexpr int PD = NST - 1;
  if (nk > 0) {
#pragma unroll
    for (int s = 0; s < PD; ++s)
      if (s < nk) issue(s, mbeg + s * WBK);
    for (int ks = 0; ks < nk; ++ks) {
      const int younger = min(PD - 1, nk - 1 - ks);
      if constexpr (PD >= 3) {
        if (younger >= 2) wait_vm_lgkm0<2 * LPS>();
        else if (younger == 1) wait_vm_lgkm0<LPS>();
        else wait_vm_lgkm0<0>();
      } else if constexpr (PD == 2) {
        if (younger >= 1) wait_vm_lgkm0<LPS>();
        else wait_vm_lgkm0<0>();
      } else {
        wait_vm_lgkm0<0>();
      }
      raw_barrier();
      if (ks + PD < nk) issue((ks + PD) % NST, mbeg + (ks + PD) * WBK);
      if constexpr (sizeof(T) == 2) {
        read_frags(ks % NST);
        mma_frags();
      } else {
        compute(ks % NST);
        if (ks % FLUSH == FLUSH - 1) flush();
      }
    }
  }
  flush();
  float* out = ws + (int64_t)bzs * g.Nd * g.K;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int k = k0 + wn * (WBNT / WGN) + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * (BMW / WGM) + i * 16 + lk * 4 + r;
        if (co < g.Nd && k < g.K) out[(int64_t)co * g.K + k] = acc[i][j][r];
      }
    }
}

// sum the split-K slabs in fixed order and scatter into the torch [co][ci][kd][kh][kw]
// layout.  unf_kw > 0: the conv ran on a W-unfolded Cin=1 input (k = (kd,kh)*8 + j).
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                    int splits, int Nd, int K, int Cs, int cs_shift, int taps,
                                    int unf_kw, int stride) {
  const int64_t total = (int64_t)Nd * K;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int sp = 0; sp < splits; sp += stride) s += ws[sp * total + idx];
    const int co = (int)(idx / K), k = (int)(idx % K);
    if (unf_kw > 0) {
      const int j = k & 7, tkh = k >> 3;   // tkh = kd*KH + kh
      if (j < unf_kw) dw[((int64_t)co * taps + tkh) * unf_kw + j] = s;
    } else {
      const int tap = k >> cs_shift, ci = k & (Cs - 1);
      dw[((int64_t)co * Cs + ci) * taps + tap] = s;
    }
  }
}

// Same sum for many slabs: 4 groups of 64 lanes take every 4th slab of 256 consecutive
// elements, 16 bytes per lane per load (independent load streams instead of one serial
// chain of `splits` 4-byte loads per thread -- 128 slabs of a 1x1x1 conv took 32 us as a
// chain, and 4-byte loads left the slab pass TA-bound at ~2.5 TB/s), combined in fixed
// order.  total % 4 == 0 (Nd % 8 == 0 is a wgrad precondition).
__global__ __launch_bounds__(256) void wgrad_reduce_wide_kernel(
    const float* __restrict__ ws, float* __restrict__ dw, int splits, int Nd, int K, int Cs,
    int cs_shift, int taps, int unf_kw, int stride) {
  __shared__ f32x4 red[4][64];
  const int64_t total = (int64_t)Nd * K;
  const int e = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t idx = ((int64_t)blockIdx.x * 64 + e) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (idx < total) {
#pragma unroll 4
    for (int sp = grp * stride; sp < splits; sp += 4 * stride)
      s += *reinterpret_cast<const f32x4*>(ws + sp * total + idx);
  }
  red[grp][e] = s;
  __syncthreads();
  if (grp != 0 || idx >= total) return;
  s = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t id = idx + q;
    const int co = (int)(id / K), k = (int)(id % K);
    if (unf_kw > 0) {
      const int j = k & 7, tkh = k >> 3;
      if (j < unf_kw) dw[((int64_t)co * taps + tkh) * unf_kw + j] = s[q];
    } else {
      const int tap = k >> cs_shift, ci = k & (Cs - 1);
      dw[((int64_t)co * Cs + ci) * taps + tap] = s[q];
    }
  }
}

// First level of a two-level slab sum (many slabs): slab[g*G] += slabs g*G+1 .. g*G+G-1,
// in place and in fixed order; the second level sums every G-th slab.
__global__ void slab_group_sum_kernel(float* __restrict__ ws, int splits, int64_t total, int G) {
  const int ng = (splits + G - 1) / G;
  const int64_t n = total * ng;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int gi = (int)(t / total);
    const int64_t idx = t % total;
    float s = 0.f;
    const int s1 = min(splits, (gi + 1) * G);
#pragma unroll 16
    for (int sp = gi * G; sp < s1; ++sp) s += ws[sp * total + idx];
    ws[(int64_t)gi * G * total + idx] = s;
  }
}

// The transposing slab reductions (bodies in reduce.h)
__global__ __launch_bounds__(256) void wgrad_reduce_t_kernel(const float* __restrict__ ws,
                                                             float* __restrict__ dw, int splits,
                                                             int Nd, int K, int Cs, int taps) {
  __shared__ float sm[mmad_reduce::SMEM_FLOATS];
  mmad_reduce::t_body(ws, dw, splits, Nd, K, Cs, taps, blockIdx.x, blockIdx.y, sm);
}

__global__ __launch_bounds__(256) void wgrad_reduce_tz_kernel(const float* __restrict__ ws,
                                                              float* __restrict__ dw, int splits,
                                                              int Nd, int K, int Cs, int taps,
                                                              int tper) {
  __shared__ float sm[mmad_reduce::SMEM_FLOATS];
  mmad_reduce::tz_body(ws, dw, splits, Nd, K, Cs, taps, tper, blockIdx.x, blockIdx.y, blockIdx.z,
                       sm);
}

// Many pending reductions (mmad_wgrad_reduce_batch) in one launch: the jobs travel in the
// kernel arguments (a captured launch replays them as recorded); block b runs block
// b - start[j] of job j, the same body and per-element order as the job's own launch.
constexpr int kReduceBatch = 16;
struct ReduceBatch {
  int n, n_total;
  int start[kReduceBatch + 1];
  mmad_reduce::Job jobs[kReduceBatch];
};

__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(ReduceBatch b) {
  __shared__ float sm[mmad_reduce::SMEM_FLOATS];
  const int bid = blockIdx.x;
  int j = 0;
  while (j + 1 < b.n && bid >= b.start[j + 1]) ++j;
  mmad_reduce::run(b.jobs[j], bid - b.start[j], sm);
}

// the transposing reduce: wgrad_reduce_t_kernel when its (channel slice, co) grid fills the
// CUs, else wgrad_reduce_tz_kernel over tap groups (MMAD_REDUCE_TZ=0 keeps the former;
// r03tz: layer1 16.4 / 16.2 -> 10.6 / 10.3 us, layer2.0.conv1 13.9 -> 11.5)
mmad_reduce::Job plan_reduce_t(const float* ws, float* dw, int splits, int Nd, int K, int Cs,
                              int taps) {
  static const bool tz_on = [] {
    const char* e = getenv("MMAD_REDUCE_TZ");
    return e == nullptr || atoi(e) != 0;
  }();
  mmad_reduce::Job j{};
  j.ws = ws; j.dw = dw; j.splits = splits; j.nd = Nd; j.k = K; j.cs = Cs; j.taps = taps;
  const int64_t blocks = (int64_t)cdiv(Cs, 64) * Nd;
  const int ct = std::min(64, Cs);
  j.gx = (int)cdiv(Cs, 64);
  j.gy = Nd;
  if (tz_on && blocks < 256 && taps <= 32 && ct % 4 == 0) {
    int gz = (int)std::min<int64_t>(taps, cdiv(256, blocks));
    int tper = (int)cdiv(taps, gz);
    while (tper * (ct / 4) > 256) ++gz, tper = (int)cdiv(taps, gz);
    j.gz = (int)cdiv(taps, tper);
    j.tper = tper;
    j.kind = mmad_reduce::KIND_TZ;
  } else {
    j.gz = 1;
    j.kind = mmad_reduce::KIND_T;
  }
  return j;
}

int run_reduce_job(const mmad_reduce::Job& j, hipStream_t st) {
  if (j.kind == mmad_reduce::KIND_TZ)
    hipLaunchKernelGGL(wgrad_reduce_tz_kernel, dim3((unsigned)j.gx, (unsigned)j.gy, (unsigned)j.gz),
                       dim3(256), 0, st, j.ws, j.dw, j.splits, j.nd, j.k, j.cs, j.taps, j.tper);
  else if (j.kind == mmad_reduce::KIND_T)
    hipLaunchKernelGGL(wgrad_reduce_t_kernel, dim3((unsigned)j.gx, (unsigned)j.gy), dim3(256), 0,
                       st, j.ws, j.dw, j.splits, j.nd, j.k, j.cs, j.taps);
  else
    return MMAD_OK;
  return launch_status();
}

int launch_reduce_t(const float* ws, float* dw, int splits, int Nd, int K, int Cs, int taps,
                    hipStream_t st) {
  return run_reduce_job(plan_reduce_t(ws, dw, splits, Nd, K, Cs, taps), st);
}

// ---- weight packing / input unfolding -------------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, T* __restrict__ wp, int rows,
                                   int Kpad, int K, int Cs, int cs_shift, int taps, int mode,
                                   int Ci, int unf_kw, int flip) {
  const int64_t total = (int64_t)rows * Kpad;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(idx / Kpad), k = (int)(idx % Kpad);
    float v = 0.f;
    if (k < K) {
      const int tap = k >> cs_shift, c = k & (Cs - 1);
      if (mode == 0) {            // forward: row = co, c = ci
        v = w[((int64_t)r * Ci + c) * taps + tap];
      } else if (mode == 1) {     // dgrad: row = ci, c = co (flip: taps in reverse order)
        v = w[((int64_t)c * Ci + r) * taps + (flip ? taps - 1 - tap : tap)];
      } else {                    // unfolded Cin=1 forward: tap = kd*KH+kh, c = kw
        v = c < unf_kw ? w[((int64_t)r * taps + tap) * unf_kw + c] : 0.f;
      }
    }
    Elt<T>::st(wp, idx, v);
  }
}

// Coalesced packing for unpadded rows (Kpad == K): the input is read as [B][R][Cc]
// (contiguous along Cc) through a 64x64 LDS tile and element (b, i, j) is written to
// b*ob + (j / jd)*oj1 + (j % jd)*oj2 + i  (contiguous along i).
//   forward: B = Co, R = Ci, Cc = taps           -> [co][tap][ci]
//   dgrad:   B = 1,  R = Co, Cc = Ci*taps (jd = taps) -> [ci][tap][co]
template <typename T>
__global__ __launch_bounds__(256) void pack_transpose_kernel(const float* __restrict__ w,
                                                             T* __restrict__ wp, int R, int Cc,
                                                             int64_t ob, int jd, int64_t oj1,
                                                             int oj2, int flip,
                                                             const float* __restrict__ scale) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const float sb = scale != nullptr ? scale[b] : 1.f;    // per-output-channel (forward layout)
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const float* src = w + (int64_t)b * R * Cc;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int r = ty; r < 64; r += 4) {
    const int i = i0 + r, j = j0 + tx;
    tile[r][tx] = (i < R && j < Cc) ? src[(int64_t)i * Cc + j] * sb : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int c = ty; c < 64; c += 4) {
    const int j = j0 + c, i = i0 + tx;
    if (i < R && j < Cc)
      Elt<T>::st(wp, (int64_t)b * ob + (int64_t)(j / jd) * oj1 +
                         (int64_t)(flip ? jd - 1 - j % jd : j % jd) * oj2 + i,
                 tile[tx][c]);
  }
}

// Batched form: blockIdx.x walks the concatenated tile ranges of all jobs.  A tile is
// 64 x 64 (rows x cols), or 128 x 32 when cols <= 32 (the 27-tap forward jobs: 84 % of a
// tile's lanes carry data instead of 42 %); source reads run along cols, packed stores
// along rows, both through a padded LDS tile.
template <typename T>
__global__ __launch_bounds__(256) void pack_batch_kernel(const mmad_pack_job* __restrict__ jobs,
                                                         int njobs) {
  __shared__ float tile[128 * 33];            // >= 64 x 65 and 32 x 129 (column-major)
  // job lookup: last job with tile0 <= blockIdx.x (jobs sorted by tile0)
  int lo = 0, hi = njobs - 1;
  const int64_t bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
  }
  const mmad_pack_job& jb = jobs[lo];
  int64_t t = bid - jb.tile0;
  const int bx = (int)(t % jb.tiles_x);
  t /= jb.tiles_x;
  const int by = (int)(t % jb.tiles_y);
  const int b = (int)(t / jb.tiles_y);
  const int R = jb.rows, Cc = jb.cols, jd = jb.jdiv, oj2 = jb.ostride_j2, rdiv = jb.rdiv;
  const bool narrow = Cc <= 32;                       // job-uniform
  const int TR = narrow ? 128 : 64, TC = narrow ? 32 : 64, LD = TC + 1;
  const int i0 = by * TR, j0 = bx * TC;
  const float* src = jb.w + (int64_t)b * R * Cc;
  T* wp = reinterpret_cast<T*>(jb.w_packed);
  const int cl = threadIdx.x & (TC - 1), rl = threadIdx.x / TC, rstep = 256 / TC;
  // bf16 with 8-row groups inside one packed block: the tile is kept column-major and each
  // thread stores 8 consecutive rows as one 16-byte vector (2-byte stores made this kernel
  // store-issue bound)
  const bool vec = sizeof(T) == 2 && jb.rdiv % 8 == 0 && (jb.ostride_b | jb.ostride_j1 | oj2) % 8 == 0;
  if (vec) {
    const int LDT = TR + 1;
    for (int r = rl; r < TR; r += rstep) {
      const int i = i0 + r, j = j0 + cl;
      tile[cl * LDT + r] = (i < R && j < Cc) ? src[(int64_t)i * Cc + j] : 0.f;
    }
    __syncthreads();
    const int RG = TR / 8;
    for (int it = threadIdx.x; it < RG * TC; it += 256) {
      const int rg = it % RG, c = it / RG;
      const int i = i0 + rg * 8, j = j0 + c;
      if (i >= R || j >= Cc) continue;           // (R is a multiple of 8: rdiv % 8 == 0)
      const float* tp = tile + c * LDT + rg * 8;
      u32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = pack_bf16x2(tp[2 * e], tp[2 * e + 1]);
      const int64_t o = (int64_t)(b * (R / rdiv) + i / rdiv) * jb.ostride_b + i % rdiv +
                        (int64_t)(j / jd) * jb.ostride_j1 +
                        (int64_t)(jb.pad_ ? jd - 1 - j % jd : j % jd) * oj2;
      *reinterpret_cast<u32x4*>(wp + o) = v;
    }
    return;
  }
  for (int r = rl; r < TR; r += rstep) {
    const int i = i0 + r, j = j0 + cl;
    tile[r * LD + cl] = (i < R && j < Cc) ? src[(int64_t)i * Cc + j] : 0.f;
  }
  __syncthreads();
  const int rw = threadIdx.x & (TR - 1), cw = threadIdx.x / TR, cstep = 256 / TR;
  const int i = i0 + rw;
  if (i >= R) return;
  const int64_t obase = (int64_t)(b * (R / rdiv) + i / rdiv) * jb.ostride_b + i % rdiv;
  for (int c = cw; c < TC; c += cstep) {
    const int j = j0 + c;
    if (j < Cc)
      Elt<T>::st(wp, obase + (int64_t)(j / jd) * jb.ostride_j1 +
                         (int64_t)(jb.pad_ ? jd - 1 - j % jd : j % jd) * oj2,
                 tile[rw * LD + c]);
  }
}

// Dual-layout pack (mmad_conv_pack_dual_batch): one 16 co x 16 ci x taps tile per block,
// read once (rows of taps*16 contiguous floats per co) into LDS [co][tap][ci | pad], then
// written as 16-byte bf16 vectors of 8 ci (forward rows) and of 8 co (dgrad rows).
__global__ __launch_bounds__(256) void pack_dual_kernel(const mmad_pack_dual* __restrict__ jobs,
                                                        int njobs) {
  __shared__ float tile[16 * 27 * 17];
  int lo = 0, hi = njobs - 1;
  const int64_t bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].tile0 <= bid) lo = mid; else hi = mid - 1;
  }
  const mmad_pack_dual& jb = jobs[lo];
  const int T = jb.taps, CI = jb.ci, CO = jb.co;
  const int t = (int)(bid - jb.tile0), nci = CI / 16;
  const int co0 = (t / nci) * 16, ci0 = (t % nci) * 16;
  const int per_co = 16 * T, q4 = per_co / 4;    // a co's tile row: 16*T contiguous floats
  for (int e = threadIdx.x; e < 16 * q4; e += 256) {
    const int col = e / q4, rem0 = (e % q4) * 4;
    const f32x4 v =
        *reinterpret_cast<const f32x4*>(jb.w + ((int64_t)(co0 + col) * CI + ci0) * T + rem0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rem = rem0 + q, cil = rem / T, tap = rem % T;
      tile[(col * T + tap) * 17 + cil] = v[q];
    }
  }
  __syncthreads();
  u16* wf = reinterpret_cast<u16*>(jb.w_fwd);
  u16* wd = reinterpret_cast<u16*>(jb.w_dgrad);
  const int items = 16 * T * 2;
  for (int e = threadIdx.x; e < 2 * items; e += 256) {
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
      for (int q = 0; q < 4; ++q) v[q] = pack_bf16x2(tp[(2 * q) * T * 17], tp[(2 * q + 1) * T * 17]);
      *reinterpret_cast<u32x4*>(wd + (int64_t)(ci0 + cil) * T * CO + (int64_t)tq * CO + co0 +
                                half * 8) = v;
    }
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

// Same, UNF_RB input rows per block staged through LDS (Wi <= UNF_MAXW): the rows are one
// contiguous span, read with one coalesced load per element instead of one strided load
// per (output, tap); the taps then come from LDS.
#ifndef UNF_RB_V
#define UNF_RB_V 8
#endif
constexpr int UNF_RB = UNF_RB_V, UNF_MAXW = 256;
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void unfold_w_rows_kernel(const TI* __restrict__ x,
                                                            TO* __restrict__ xu, int64_t rows,
                                                            int Wi, int Wo, int KW, int sw,
                                                            int pw, int dw) {
  __shared__ float row[UNF_RB * UNF_MAXW];
  const int64_t r0 = (int64_t)blockIdx.x * UNF_RB;
  const int nr = (int)min((int64_t)UNF_RB, rows - r0);
  // all of a thread's loads issued before any is used (one memory round trip per block,
  // not one per loop trip: the rolled loop waited on each load, 55 us at 128^3 x 8)
  constexpr int PER = UNF_RB * UNF_MAXW / 256;
  const int nel = nr * Wi;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = threadIdx.x + 256 * i;
    v[i] = k < nel ? (float)x[r0 * Wi + k] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = threadIdx.x + 256 * i;
    if (k < nel) row[k] = v[i];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nr * Wo; k += 256) {
    const int r = k / Wo, xo = k - r * Wo;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int xi = xo * sw - pw + j * dw;
      v[j] = (j < KW && xi >= 0 && xi < Wi) ? row[r * Wi + xi] : 0.f;
    }
    const int64_t idx = r0 * Wo + k;
    if constexpr (sizeof(TO) == 2) {
      Chunk<u16>::store(reinterpret_cast<u16*>(xu) + idx * 8, v);
    } else {
      Chunk<float>::store(reinterpret_cast<float*>(xu) + idx * 8, v);
      Chunk<float>::store(reinterpret_cast<float*>(xu) + idx * 8 + 4, v + 4);
    }
  }
}

// ---- host-side geometry ---------------------------------------------------------------
// packed-weight row stride granule: one 128-byte K slice (a stage row)
int bk_of(int dtype) { return dtype == MMAD_BF16 ? 64 : 32; }

bool desc_ok(const mmad_conv_desc* d) {
  if (!d) return false;
  const int v[] = {d->n, d->ci, d->di, d->hi, d->wi, d->co, d->do_, d->ho, d->wo, d->kd, d->kh,
                   d->kw, d->sd, d->sh, d->sw, d->dd, d->dh, d->dw};
  for (int x : v) if (x <= 0) return false;
  if (d->pd < 0 || d->ph < 0 || d->pw < 0) return false;
  if (d->kd * d->kh * d->kw > MAXTAPS - 1) return false;
  if ((d->kd - 1) * d->dd > 100 || (d->kh - 1) * d->dh > 100 || (d->kw - 1) * d->dw > 100 ||
      d->pd > 100 || d->ph > 100 || d->pw > 100)
    return false;                                   // packed signed tap offsets
  auto ext = [](int i, int k, int s, int p, int dl) { return (i + 2 * p - dl * (k - 1) - 1) / s + 1; };
  return ext(d->di, d->kd, d->sd, d->pd, d->dd) == d->do_ &&
         ext(d->hi, d->kh, d->sh, d->ph, d->dh) == d->ho &&
         ext(d->wi, d->kw, d->sw, d->pw, d->dw) == d->wo;
}

bool unfolded(const mmad_conv_desc* d) { return d->ci == 1; }

Geom fwd_geom(const mmad_conv_desc* d, int dtype) {
  Geom g{};
  const bool u = unfolded(d);
  g.nb = d->n;
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

// dgrad: dst = dX grid, src = dY grid; the conv's strides become the parity-class count
Geom dgrad_geom(const mmad_conv_desc* d, int dtype) {
  Geom g{};
  g.nb = d->n;
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

// A stride-1 conv's input gradient is itself a forward conv: dY (Co channels) against the
// weights with the taps reversed, padding (k-1)*dil - pad.  It then runs on the forward
// kernels (tap masks, large tiles) instead of the parity-class path.
bool dgrad_as_fwd(const mmad_conv_desc* d) {
  return d->sd == 1 && d->sh == 1 && d->sw == 1 && !unfolded(d) &&
         (d->kd - 1) * d->dd - d->pd >= 0 && (d->kh - 1) * d->dh - d->ph >= 0 &&
         (d->kw - 1) * d->dw - d->pw >= 0;
}

Geom dgrad_fwd_geom(const mmad_conv_desc* d, int dtype) {
  Geom g = dgrad_geom(d, dtype);
  g.sd = g.sh = g.sw = 1;
  g.pd = (d->kd - 1) * d->dd - d->pd;
  g.ph = (d->kh - 1) * d->dh - d->ph;
  g.pw = (d->kw - 1) * d->dw - d->pw;
  return g;
}

bool geom_ok(const Geom& g, int dtype) {
  const int epc = dtype == MMAD_BF16 ? 8 : 4;
  const int64_t src_vox = (int64_t)g.nb * g.Ds * g.Hs * g.Ws;
  const int64_t dst_vox = (int64_t)g.nb * g.Dd * g.Hd * g.Wd;
  return is_pow2(g.Cs) && g.Cs % epc == 0 && (int64_t)g.M * g.Nd < (int64_t(1) << 40) &&
         src_vox < (int64_t(1) << 31) && dst_vox < (int64_t(1) << 31);   // 32-bit voxel ids
}

// the patch-resident kernel (patchconv.hip) for narrow stride-1 bf16 convs
mmad_patch::Geo patch_geo(const Geom& g) {
  return mmad_patch::Geo{g.nb, g.Cs, g.Nd, g.Kpad, g.Ds, g.Hs, g.Ws, g.Dd, g.Hd, g.Wd,
                         g.KD, g.KH, g.KW, g.pd, g.ph, g.pw, g.dd, g.dh, g.dw};
}
bool use_patch(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && g.sd == 1 && g.sh == 1 && g.sw == 1 &&
         mmad_patch::ok(patch_geo(g));
}
// the residue-class kernel (latticeconv.hip) for dilated stride-1 bf16 convs on 4d^3 grids
bool use_lattice(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && g.sd == 1 && g.sh == 1 && g.sw == 1 &&
         mmad_lattice::ok(patch_geo(g));
}
bool use_lattice8(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && g.sd == 1 && g.sh == 1 && g.sw == 1 &&
         mmad_lattice8::ok(patch_geo(g));
}
bool use_pwgrad(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && g.sd == 1 && g.sh == 1 && g.sw == 1 &&
         mmad_pwgrad::ok(patch_geo(g));
}
// the parity-sub-patch kernel (s2conv.hip) for the stride-2 3^3 forward (layer2.0.conv1)
bool use_s2(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && mmad_s2::ok(patch_geo(g), g.sd, g.sh, g.sw);
}
bool use_lattice_wgrad(const Geom& g, int dtype) {
  return dtype == MMAD_BF16 && g.sd == 1 && g.sh == 1 && g.sw == 1 &&
         mmad_lattice::wgrad_ok(patch_geo(g));
}

int bn_of(const Geom& g) { return g.Nd <= 64 ? 64 : 128; }

// tile rows: 64 when 128-row tiles would leave the 256 CUs with under two blocks each
int igemm_bm(int64_t m, const Geom& g) {
  return cdiv(m, 128) * cdiv(g.Nd, bn_of(g)) < 512 ? 64 : 128;
}

struct WSplit { int bmw, splits, m_per_split; };
// 256 x 256 wgrad tiles (8 waves, one block per CU): measured 10-15 % SLOWER than the
// 4-wave 128 x 128 tiles at config 2's 16^3 grids (M = 32768: more split-K slabs, less latency
// hiding) but faster at config 5's 20^3 grids (M = 64000 at batch 8: the config-5 step
// 158 -> 161 triples/s, r04q), so used from M = 49152 on.  MMAD_WGRAD_BIG: 0 never, 1
// wherever the tile fits, unset the M rule.
int wgrad_big(const Geom& g, int dtype) {
  static const int v = [] { const char* e = getenv("MMAD_WGRAD_BIG"); return e ? atoi(e) : -1; }();
  if (dtype != MMAD_BF16 || g.Nd % 256 || g.K < 256 * 8) return 0;
  if (v >= 0) return v;
  return g.M >= 49152 ? 1 : 0;
}

WSplit wgrad_split(const Geom& g, int dtype) {
  const int WBK = wbk_of(dtype);
  WSplit s{};
  const bool big = wgrad_big(g, dtype);
  s.bmw = big ? 256 : (g.Nd <= 64 ? 64 : 128);
  const int wbn = big ? 256 : WBN;
  const int64_t tiles = cdiv(g.Nd, s.bmw) * cdiv(g.K, wbn);
  // Split count from a small cost model (measured on MI355X, tools/exp_wgrad.sh):
  //   rounds(s) * stages_per_split(s) * c  +  s * slab_MB * r
  // rounds = ceil(blocks / resident slots): 4 blocks per CU for the 4-wave tiles (LDS
  // 36 KB, <128 VGPRs), 1 for the 8-wave ones.  A block count just past a multiple of the
  // slots costs a whole extra round (the old "cdiv(1024, tiles)" rule always landed there:
  // l4c1 1080 blocks ran 19 % slower than 864).  c ~ 0.93 us per 32-voxel stage of a
  // 128-wide tile, r ~ 0.2 us per MB of fp32 slab written and re-read by the reduce.
  const int64_t slots = big ? 256 : 1024;
  const int64_t max_split = std::max<int64_t>(1, std::min<int64_t>(cdiv(g.M, WBK * 8), 512));
  const double c = 0.93 * s.bmw / 128.0, r = 0.2;
  const double slab_mb = (double)g.Nd * g.K * 4 / 1e6;
  int64_t want = 1;
  double best = 1e30;
  for (int64_t sp = 1; sp <= max_split; ++sp) {
    if (sp > 1 && sp * g.Nd * (int64_t)g.K * 4 > (int64_t(512) << 20)) break;
    const int64_t stages = cdiv(cdiv(g.M, sp), WBK);
    const int64_t nsp = cdiv(g.M, stages * WBK);          // splits actually produced
    const double cost = (double)cdiv(tiles * nsp, slots) * stages * c + nsp * slab_mb * r;
    if (cost < best * 0.999) { best = cost; want = sp; }
  }
  static const int force = [] { const char* e = getenv("MMAD_WGRAD_SPLITS"); return e ? atoi(e) : 0; }();
  if (force > 0) want = std::min<int64_t>(force, max_split);
  // 1x1x1 convs (the shortcuts): MMAD_WGRAD_1X1_SPLITS overrides the model's count (A/B)
  static const int force1 = [] { const char* e = getenv("MMAD_WGRAD_1X1_SPLITS"); return e ? atoi(e) : 0; }();
  if (force1 > 0 && g.taps == 1) want = std::min<int64_t>(force1, max_split);
  s.m_per_split = (int)(cdiv(cdiv(g.M, want), WBK) * WBK);
  s.splits = (int)cdiv(g.M, s.m_per_split);
  return s;
}

template <typename F>
bool set_lds(F* kern, size_t lds) {
  return lds <= 65536 || hipFuncSetAttribute((const void*)kern,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)lds) == hipSuccess;
}

template <typename T, int BN, int MODE, int BMT, int WGM = 2, int WGN = 2, int NST = 2,
          int RBT = RB>
int launch_igemm_bm(const Geom& g, int64_t m_max, int classes, const void* src, const void* w,
                    const float* bias, void* dst, float* stats, hipStream_t st) {
  const size_t ring = (size_t)NST * (BMT + BN) * RBT;
  const size_t epi = 1024 + (size_t)BMT * (BN * 2 + 16) + (size_t)(WGM - 1) * 2 * BN * 4;
  const size_t lds = TAPB + std::max(ring, epi);
  static const bool ok = set_lds(igemm_kernel<T, BN, MODE, BMT, WGM, WGN, NST, RBT>, lds);
  if (!ok) return MMAD_EUNSUPPORTED;
  const int nbm = (int)cdiv(m_max, BMT), nbn = (int)cdiv(g.Nd, BN);
  hipLaunchKernelGGL((igemm_kernel<T, BN, MODE, BMT, WGM, WGN, NST, RBT>),
                     dim3((unsigned)(nbm * nbn), (unsigned)classes), dim3(64 * WGM * WGN), lds,
                     st, g, (const T*)src, (const T*)w, bias, (T*)dst, stats, nbm, nbn);
  return launch_status();
}

// experiment switch for the large-tile configurations (bf16, >= 256 output channels)
int big_cfg() {
  static const int v = [] { const char* e = getenv("MMAD_IGEMM_BIG"); return e ? atoi(e) : 0; }();
  return v;
}
int big_min_k() {
  static const int v = [] { const char* e = getenv("MMAD_IGEMM_BIG_MINK"); return e ? atoi(e) : 1024; }();
  return v;
}
// fewest 256 x 256 tiles for the default big-tile rule: 200, so config 5's 20^3 layer3
// (64000 x 256, 250 tiles: 6 CUs idle) takes them too -- config-5 step 160.1 -> 165.8
// triples/s (r04s); MMAD_IGEMM_BIG_MINBLK overrides (256: one tile per CU at least)
int big_min_blocks() {
  static const int v = [] { const char* e = getenv("MMAD_IGEMM_BIG_MINBLK"); return e ? atoi(e) : 200; }();
  return v;
}
// ring depth of the default (4-wave) tiles: 3 (two stages of LDS-DMA in flight, still two
// blocks per CU at 64 x 128 tiles) for strided forward convs with taps (those the stride-2
// sub-patch kernel does not take: fp32, ragged grids), 2 elsewhere.  Measured in the
// config-2 step (r03s): layer2.0.conv1 fwd 39.3 -> 33.1 us;
// every stride-1 launch and the parity-class dgrads were slower at 3 (e.g. 57.9 -> 71.6
// us).  MMAD_IGEMM_NST=2 / 3 forces one depth everywhere (A/B).
int igemm_nst(const Geom& g, int mode) {
  static const int v = [] { const char* e = getenv("MMAD_IGEMM_NST"); return e ? atoi(e) : 0; }();
  if (v) return v;
  return mode == FWD && g.taps > 1 && (g.sd > 1 || g.sh > 1 || g.sw > 1) ? 3 : 2;
}
int big_cfg_for(const Geom& g, int dtype, int64_t m_max, int classes) {
  if (dtype != MMAD_BF16) return 0;
  int cfg = big_cfg();
  if (cfg < 0) return 0;                        // MMAD_IGEMM_BIG=-1: 128 x 128 tiles only
  if (cfg == 0)   // default: 256 x 256 tiles (8 waves) when they give every CU a block and
                  // K is deep enough to amortise their epilogue (the 1x1x1 shortcut, K = 256,
                  // is epilogue-bound at one block per CU; MMAD_IGEMM_BIG_MINK=0 keeps them)
    return g.Nd % 256 == 0 && g.K >= big_min_k() &&
                   cdiv(m_max, 256) * classes * (g.Nd / 256) >= big_min_blocks() ? 2 : 0;
  if (cfg == 4) return g.Nd % 128 == 0 && cdiv(m_max, 256) * classes * (g.Nd / 128) >= 256 ? 4 : 0;
  if (cfg == 5 || cfg == 6)
    return g.Nd % 256 == 0 && cdiv(m_max, 256) * classes * (g.Nd / 256) >= 256 ? cfg : 0;
  return g.Nd % 256 == 0 && cdiv(m_max, 128) * classes * (g.Nd / 256) >= 256 ? cfg : 0;
}
// every activation / packed-weight operand is moved as 16-byte vectors (and LDS-DMA rows):
// a misaligned base pointer is refused up front (MMAD_EBADSHAPE) instead of faulting
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool al16(const void* a, const void* b, const void* c) {
  return al16(a) && al16(b) && al16(c);
}

// MMAD_STEM=0 routes the MedicalNet stem through the generic implicit GEMM (A/B switch)
bool stem_kernel_on() {
  static const bool v = [] { const char* e = getenv("MMAD_STEM"); return !e || atoi(e) != 0; }();
  return v;
}
// rows per M tile of a forward launch (= rows of the BN partial-sum buffer per tile)
int fwd_tile_rows(const Geom& g, int dtype) {
  const int cfg = big_cfg_for(g, dtype, g.M, 1);
  if (cfg == 2 || cfg == 4 || cfg == 5 || cfg == 6) return 256;
  if (cfg) return 128;
  return igemm_bm(g.M, g);
}

template <typename T, int MODE>
int run_igemm_t(const Geom& g, int64_t m_max, int classes, const void* src, const void* w,
                const float* bias, void* dst, float* stats, hipStream_t st) {
  if constexpr (sizeof(T) == 2 && MODE == FWD) {
    const int cfg = big_cfg_for(g, MMAD_BF16, m_max, classes);
    if (cfg) {
      if (cfg == 1)   // 128 x 256 tile, 8 waves (2 x 4), 3-deep ring, 1 block per CU
        return launch_igemm_bm<T, 256, MODE, 128, 2, 4, 3>(g, m_max, classes, src, w, bias,
                                                          dst, stats, st);
      if (cfg == 2)   // 256 x 256 tile, 8 waves (2 x 4) of 128 x 64, 2-deep ring
        return launch_igemm_bm<T, 256, MODE, 256, 2, 4, 2>(g, m_max, classes, src, w, bias,
                                                          dst, stats, st);
      if (cfg == 3)   // 128 x 128 tile, 4 waves, 3-deep ring (1 block per CU)
        return launch_igemm_bm<T, 128, MODE, 128, 2, 2, 3>(g, m_max, classes, src, w, bias,
                                                          dst, stats, st);
      if (cfg == 4)   // 256 x 128 tile, 8 waves (4 x 2), 2-deep ring
        return launch_igemm_bm<T, 128, MODE, 256, 4, 2, 2>(g, m_max, classes, src, w, bias,
                                                          dst, stats, st);
      if (cfg == 5)   // 256 x 256 tile, 64-B stage rows, 4-deep ring (3 stages in flight)
        return launch_igemm_bm<T, 256, MODE, 256, 2, 4, 4, 64>(g, m_max, classes, src, w, bias,
                                                              dst, stats, st);
      if (cfg == 6)   // 256 x 256 tile, 64-B stage rows, 3-deep ring
        return launch_igemm_bm<T, 256, MODE, 256, 2, 4, 3, 64>(g, m_max, classes, src, w, bias,
                                                              dst, stats, st);
    }
  }
  const bool small = igemm_bm(m_max * classes, g) == 64;
  if constexpr (sizeof(T) == 2) {
    if (igemm_nst(g, MODE) == 3) {
      if (bn_of(g) == 64)
        return small ? launch_igemm_bm<T, 64, MODE, 64, 2, 2, 3>(g, m_max, classes, src, w, bias, dst, stats, st)
                     : launch_igemm_bm<T, 64, MODE, 128, 2, 2, 3>(g, m_max, classes, src, w, bias, dst, stats, st);
      return small ? launch_igemm_bm<T, 128, MODE, 64, 2, 2, 3>(g, m_max, classes, src, w, bias, dst, stats, st)
                   : launch_igemm_bm<T, 128, MODE, 128, 2, 2, 3>(g, m_max, classes, src, w, bias, dst, stats, st);
    }
  }
  if (bn_of(g) == 64)
    return small ? launch_igemm_bm<T, 64, MODE, 64>(g, m_max, classes, src, w, bias, dst, stats, st)
                 : launch_igemm_bm<T, 64, MODE, 128>(g, m_max, classes, src, w, bias, dst, stats, st);
  return small ? launch_igemm_bm<T, 128, MODE, 64>(g, m_max, classes, src, w, bias, dst, stats, st)
               : launch_igemm_bm<T, 128, MODE, 128>(g, m_max, classes, src, w, bias, dst, stats, st);
}

template <int MODE>
int run_igemm(const Geom& g, int dtype, int64_t m_max, int classes, const void* src,
              const void* w, const float* bias, void* dst, float* stats, hipStream_t st) {
  if (dtype == MMAD_BF16)
    return run_igemm_t<u16, MODE>(g, m_max, classes, src, w, bias, dst, stats, st);
  return run_igemm_t<float, MODE>(g, m_max, classes, src, w, bias, dst, stats, st);
}

// MMAD_WGRAD_XCD=0 keeps launch-order block placement (A/B switch)
int wgrad_xcd() {
  static const int v = [] { const char* e = getenv("MMAD_WGRAD_XCD"); return e ? atoi(e) : 1; }();
  return v;
}

template <typename T, int BMW, int WBK, int NST, int WBNT, int WGM, int WGN, bool XFIX>
int launch_wgrad_x(const Geom& g, const WSplit& sp, const void* x, const void* dy, float* ws,
                   hipStream_t st) {
  const size_t lds = TAPB + NST * WBK * (BMW + WBNT) * sizeof(T);
  static const bool ok = set_lds(wgrad_kernel<T, BMW, WBK, NST, WBNT, WGM, WGN, XFIX>, lds);
  if (!ok) return MMAD_EUNSUPPORTED;
  const uint32_t xb = (uint32_t)((int64_t)g.nb * g.Ds * g.Hs * g.Ws * g.Cs * sizeof(T));
  const uint32_t yb = (uint32_t)((int64_t)g.M * g.Nd * sizeof(T));
  dim3 grid((unsigned)cdiv(g.K, WBNT), (unsigned)cdiv(g.Nd, BMW), (unsigned)sp.splits);
  hipLaunchKernelGGL((wgrad_kernel<T, BMW, WBK, NST, WBNT, WGM, WGN, XFIX>), grid,
                     dim3(64 * WGM * WGN), lds, st, g, (const T*)x, (const T*)dy, ws,
                     sp.m_per_split, xb, yb, wgrad_xcd());
  return launch_status();
}

template <typename T, int BMW, int WBK, int NST, int WBNT = WBN, int WGM = 2, int WGN = 2>
int launch_wgrad_k(const Geom& g, const WSplit& sp, const void* x, const void* dy, float* ws,
                   hipStream_t st) {
  // both tensors must be addressable by 32-bit buffer offsets (padding offsets use bit 31)
  if ((int64_t)g.nb * g.Ds * g.Hs * g.Ws * g.Cs * (int64_t)sizeof(T) >= (int64_t(1) << 31) ||
      (int64_t)g.M * g.Nd * (int64_t)sizeof(T) >= (int64_t(1) << 31))
    return MMAD_EUNSUPPORTED;
  if (WBK % g.Wd == 0)
    return launch_wgrad_x<T, BMW, WBK, NST, WBNT, WGM, WGN, true>(g, sp, x, dy, ws, st);
  return launch_wgrad_x<T, BMW, WBK, NST, WBNT, WGM, WGN, false>(g, sp, x, dy, ws, st);
}

// ring depth of the 1x1x1 (shortcut) weight gradients: 3 (two stages in flight; measured r03zf
// layer4 / 3 / 2 downsample wgrad 26.2 / 13.1 / 11.4 -> 26.0 / 12.1 / 10.1 us), or 2
// (MMAD_WGRAD_1X1_NST=2, the depth of every other wgrad)
int wgrad_1x1_nst() {
  static const int v = [] { const char* e = getenv("MMAD_WGRAD_1X1_NST"); return e ? atoi(e) : 3; }();
  return v;
}

template <typename T, int BMW>
int launch_wgrad(const Geom& g, const WSplit& sp, const void* x, const void* dy, float* ws,
                 hipStream_t st) {
  // ring depth 2: deeper rings (3, 4) cost blocks per CU and measured 10-30 % slower
  if (g.taps == 1 && wgrad_1x1_nst() == 3) return launch_wgrad_k<T, BMW, 32, 3>(g, sp, x, dy, ws, st);
  return launch_wgrad_k<T, BMW, 32, 2>(g, sp, x, dy, ws, st);
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

int mmad_conv_pack_weight_scaled(const mmad_conv_desc* d, int dtype, const float* w,
                                 const float* scale, void* wp, int for_dgrad, void* stream);

int mmad_conv_pack_weight(const mmad_conv_desc* d, int dtype, const float* w, void* wp,
                          int for_dgrad, void* stream) {
  return mmad_conv_pack_weight_scaled(d, dtype, w, nullptr, wp, for_dgrad, stream);
}

int mmad_conv_pack_weight_scaled(const mmad_conv_desc* d, int dtype, const float* w,
                                 const float* scale, void* wp, int for_dgrad, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!w || !wp) return MMAD_ENULL;
  if (for_dgrad && unfolded(d)) return MMAD_EUNSUPPORTED;
  const Geom g = for_dgrad ? dgrad_geom(d, dtype) : fwd_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  const int mode = for_dgrad ? 1 : (unfolded(d) ? 2 : 0);
  const int flip = for_dgrad && dgrad_as_fwd(d);
  const int64_t total = (int64_t)g.Nd * g.Kpad;
  if (scale != nullptr && (mode != 0 || g.Kpad != g.K)) return MMAD_EUNSUPPORTED;
  if (mode != 2 && g.Kpad == g.K) {
    // forward: per co, [Ci][taps] -> [taps][Ci]; dgrad: [Co][Ci*taps] -> [Ci][taps][Co]
    const int R = mode == 0 ? d->ci : d->co;
    const int Cc = mode == 0 ? g.taps : d->ci * g.taps;
    const int B = mode == 0 ? d->co : 1;
    const int64_t ob = mode == 0 ? g.Kpad : 0, oj1 = mode == 0 ? 0 : g.Kpad;
    const int jd = g.taps, oj2 = mode == 0 ? d->ci : d->co;
    dim3 grid((unsigned)cdiv(Cc, 64), (unsigned)cdiv(R, 64), (unsigned)B);
    if (dtype == MMAD_BF16)
      hipLaunchKernelGGL(pack_transpose_kernel<u16>, grid, dim3(256), 0, as_stream(stream), w,
                         (u16*)wp, R, Cc, ob, jd, oj1, oj2, flip, scale);
    else
      hipLaunchKernelGGL(pack_transpose_kernel<float>, grid, dim3(256), 0, as_stream(stream), w,
                         (float*)wp, R, Cc, ob, jd, oj1, oj2, flip, scale);
    return launch_status();
  }
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<u16>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), w, (u16*)wp, g.Nd, g.Kpad, g.K, g.Cs, g.cs_shift,
                       g.taps, mode, d->ci, d->kw, flip);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0,
                       as_stream(stream), w, (float*)wp, g.Nd, g.Kpad, g.K, g.Cs, g.cs_shift,
                       g.taps, mode, d->ci, d->kw, flip);
  return launch_status();
}

int mmad_conv_pack_job(const mmad_conv_desc* d, int dtype, int for_dgrad, const float* w,
                       void* wp, int64_t tile0, mmad_pack_job* job) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!w || !wp || !job) return MMAD_ENULL;
  if (unfolded(d)) return MMAD_EUNSUPPORTED;
  const Geom g = for_dgrad ? dgrad_geom(d, dtype) : fwd_geom(d, dtype);
  if (!geom_ok(g, dtype) || g.Kpad != g.K) return MMAD_EUNSUPPORTED;
  const bool fw = !for_dgrad;
  mmad_pack_job j{};
  j.w = w;
  j.w_packed = wp;
  // forward: [co][ci][tap] -> [co][tap][ci] with all co in one (co*ci) x taps matrix
  // (row i -> block i / ci, offset i % ci); dgrad: one co x (ci*taps) matrix
  j.rows = fw ? d->co * d->ci : d->co;
  j.rdiv = fw ? d->ci : d->co;
  j.cols = fw ? g.taps : d->ci * g.taps;
  j.batch = 1;
  j.jdiv = g.taps;
  j.ostride_j2 = fw ? d->ci : d->co;
  j.ostride_b = fw ? g.Kpad : 0;
  j.ostride_j1 = fw ? 0 : g.Kpad;
  const bool narrow = j.cols <= 32;      // pack_batch_kernel's 128 x 32 tile
  j.tiles_x = (int)cdiv(j.cols, narrow ? 32 : 64);
  j.tiles_y = (int)cdiv(j.rows, narrow ? 128 : 64);
  j.pad_ = for_dgrad && dgrad_as_fwd(d);       // reversed tap order (see dgrad_as_fwd)
  j.tile0 = tile0;
  *job = j;
  return MMAD_OK;
}

int mmad_conv_pack_dual_job(const mmad_conv_desc* d, int dtype, const float* w, void* w_fwd,
                            void* w_dgrad, int64_t tile0, mmad_pack_dual* job) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_BF16) return MMAD_EUNSUPPORTED;
  if (!w || !w_fwd || !w_dgrad || !job) return MMAD_ENULL;
  if (unfolded(d)) return MMAD_EUNSUPPORTED;
  const Geom gf = fwd_geom(d, dtype), gd = dgrad_geom(d, dtype);
  if (!geom_ok(gf, dtype) || !geom_ok(gd, dtype) || gf.Kpad != gf.K || gd.Kpad != gd.K)
    return MMAD_EUNSUPPORTED;
  if (d->ci % 16 || d->co % 16 || gf.taps > 27) return MMAD_EUNSUPPORTED;
  mmad_pack_dual j{};
  j.w = w;
  j.w_fwd = w_fwd;
  j.w_dgrad = w_dgrad;
  j.co = d->co;
  j.ci = d->ci;
  j.taps = gf.taps;
  j.flip = dgrad_as_fwd(d) ? 1 : 0;
  j.tile0 = tile0;
  *job = j;
  return MMAD_OK;
}

int64_t mmad_pack_dual_tiles(const mmad_pack_dual* job) {
  return job ? (int64_t)(job->co / 16) * (job->ci / 16) : -1;
}

int mmad_conv_pack_dual_batch(int dtype, int njobs, const mmad_pack_dual* jobs,
                              int64_t total_tiles, void* stream) {
  if (njobs <= 0 || total_tiles <= 0 || total_tiles > INT32_MAX) return MMAD_EBADSHAPE;
  if (!jobs) return MMAD_ENULL;
  if (dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  hipLaunchKernelGGL(pack_dual_kernel, dim3((unsigned)total_tiles), dim3(256), 0,
                     as_stream(stream), jobs, njobs);
  return launch_status();
}

int64_t mmad_pack_job_tiles(const mmad_pack_job* job) {
  return job ? (int64_t)job->tiles_x * job->tiles_y * job->batch : -1;
}

int mmad_conv_pack_batch(int dtype, int njobs, const mmad_pack_job* jobs, int64_t total_tiles,
                         void* stream) {
  if (njobs <= 0 || total_tiles <= 0 || total_tiles > INT32_MAX) return MMAD_EBADSHAPE;
  if (!jobs) return MMAD_ENULL;
  if (dtype == MMAD_BF16)
    hipLaunchKernelGGL(pack_batch_kernel<u16>, dim3((unsigned)total_tiles), dim3(256), 0,
                       as_stream(stream), jobs, njobs);
  else if (dtype == MMAD_F32)
    hipLaunchKernelGGL(pack_batch_kernel<float>, dim3((unsigned)total_tiles), dim3(256), 0,
                       as_stream(stream), jobs, njobs);
  else
    return MMAD_EBADDTYPE;
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
  const bool staged = d->wi <= UNF_MAXW && rows / UNF_RB < INT32_MAX;
  const unsigned sgrid = (unsigned)cdiv(rows, UNF_RB);
#define UNF(TI, TO)                                                                         \
  do {                                                                                      \
    if (staged)                                                                             \
      hipLaunchKernelGGL((unfold_w_rows_kernel<TI, TO>), dim3(sgrid), dim3(256), 0, st,     \
                         (const TI*)x, (TO*)xu, rows, d->wi, d->wo, d->kw, d->sw, d->pw, d->dw); \
    else                                                                                    \
      hipLaunchKernelGGL((unfold_w_kernel<TI, TO>), dim3(grid), dim3(256), 0, st,           \
                         (const TI*)x, (TO*)xu, rows, d->wi, d->wo, d->kw, d->sw, d->pw, d->dw); \
  } while (0)
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
  if (unfolded(d) && mmad_stem::fwd_ok(d, dtype) && stem_kernel_on())
    return mmad_stem::fwd_stats_rows(d);
  const Geom g = fwd_geom(d, dtype);
  if (!unfolded(d) && use_lattice(g, dtype)) return mmad_lattice::tiles(patch_geo(g));
  if (!unfolded(d) && use_lattice8(g, dtype)) return mmad_lattice8::tiles(patch_geo(g));
  if (!unfolded(d) && use_patch(g, dtype)) return mmad_patch::tiles(patch_geo(g));
  if (!unfolded(d) && use_s2(g, dtype)) return mmad_s2::tiles(patch_geo(g));
  if (mmad_pw::fwd_ok(d, dtype)) return mmad_pw::fwd_tiles(d);
  return cdiv(g.M, fwd_tile_rows(g, dtype));
}

int mmad_conv3d_fwd(const mmad_conv_desc* d, int dtype, const void* x, const void* wp,
                    const float* bias, void* y, float* stats, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!x || !wp || !y) return MMAD_ENULL;
  if (!al16(x, wp, y)) return MMAD_EBADSHAPE;
  if (unfolded(d) && mmad_stem::fwd_ok(d, dtype) && stem_kernel_on())
    return mmad_stem::fwd(d, x, wp, bias, y, stats, stream);
  const Geom g = fwd_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  if (!unfolded(d) && use_lattice(g, dtype))
    return mmad_lattice::fwd(patch_geo(g), x, wp, bias, y, stats, stream);
  if (!unfolded(d) && use_lattice8(g, dtype))
    return mmad_lattice8::fwd(patch_geo(g), x, wp, bias, y, stats, stream);
  if (!unfolded(d) && use_patch(g, dtype))
    return mmad_patch::fwd(patch_geo(g), x, wp, bias, y, stats, stream);
  if (!unfolded(d) && use_s2(g, dtype))
    return mmad_s2::fwd(patch_geo(g), g.sd, g.sh, g.sw, x, wp, bias, y, stats, stream);
  if (mmad_pw::fwd_ok(d, dtype)) return mmad_pw::fwd(d, x, wp, bias, y, stats, stream);
  return run_igemm<FWD>(g, dtype, g.M, 1, x, wp, bias, y, stats, as_stream(stream));
}

int mmad_conv3d_fwd_ex(const mmad_conv_desc* d, int dtype, const void* x, const void* wp,
                       const float* bias, const void* res, int relu, void* y, float* stats,
                       void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!x || !wp || !y) return MMAD_ENULL;
  if (!al16(x, wp, y) || !al16(res)) return MMAD_EBADSHAPE;
  if (res == nullptr && !relu) return mmad_conv3d_fwd(d, dtype, x, wp, bias, y, stats, stream);
  if (unfolded(d)) return MMAD_EUNSUPPORTED;     // the stem keeps its own epilogue
  Geom g = fwd_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  g.res = res;
  g.relu = relu ? 1 : 0;
  if (use_lattice(g, dtype) || use_lattice8(g, dtype)) {
    mmad_patch::Geo q = patch_geo(g);
    q.res = res;
    q.relu = g.relu;
    return use_lattice(g, dtype) ? mmad_lattice::fwd(q, x, wp, bias, y, stats, stream)
                                 : mmad_lattice8::fwd(q, x, wp, bias, y, stats, stream);
  }
  if (use_patch(g, dtype)) {
    mmad_patch::Geo q = patch_geo(g);
    q.res = res;
    q.relu = g.relu;
    return mmad_patch::fwd(q, x, wp, bias, y, stats, stream);
  }
  if (use_s2(g, dtype)) {
    mmad_patch::Geo q = patch_geo(g);
    q.res = res;
    q.relu = g.relu;
    return mmad_s2::fwd(q, g.sd, g.sh, g.sw, x, wp, bias, y, stats, stream);
  }
  return run_igemm<FWD>(g, dtype, g.M, 1, x, wp, bias, y, stats, as_stream(stream));
}

int mmad_conv3d_dgrad(const mmad_conv_desc* d, int dtype, const void* dy, const void* wpt,
                      void* dx, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!dy || !wpt || !dx) return MMAD_ENULL;
  if (!al16(dy, wpt, dx)) return MMAD_EBADSHAPE;
  if (unfolded(d)) return MMAD_EUNSUPPORTED;   // the raw input never needs a gradient
  if (mmad_pw::ok(d, dtype)) {
    const int rc = mmad_pw::dgrad(d, dy, wpt, dx, stream);
    if (rc != MMAD_EUNSUPPORTED) return rc;
  }
  if (dgrad_as_fwd(d)) {
    const Geom gf = dgrad_fwd_geom(d, dtype);
    if (!geom_ok(gf, dtype)) return MMAD_EUNSUPPORTED;
    if (use_lattice(gf, dtype))
      return mmad_lattice::fwd(patch_geo(gf), dy, wpt, nullptr, dx, nullptr, stream);
    if (use_lattice8(gf, dtype))
      return mmad_lattice8::fwd(patch_geo(gf), dy, wpt, nullptr, dx, nullptr, stream);
    if (use_patch(gf, dtype))
      return mmad_patch::fwd(patch_geo(gf), dy, wpt, nullptr, dx, nullptr, stream);
    return run_igemm<FWD>(gf, dtype, gf.M, 1, dy, wpt, nullptr, dx, nullptr,
                          as_stream(stream));
  }
  if (dtype == MMAD_BF16 && mmad_s2::dgrad_ok(d)) return mmad_s2::dgrad(d, dy, wpt, dx, stream);
  const Geom g = dgrad_geom(d, dtype);
  if (!geom_ok(g, dtype)) return MMAD_EUNSUPPORTED;
  // the largest parity class (0,0,0) sizes the grid
  const int64_t mmax = (int64_t)d->n * cdiv(d->di, d->sd) * cdiv(d->hi, d->sh) * cdiv(d->wi, d->sw);
  if (g.taps == 1 && d->pd == 0 && d->ph == 0 && d->pw == 0) {
    // strided 1^3 conv (shortcut B): only the all-even class has a tap, so dX is one fill
    // plus that class's GEMM (the 7 empty classes as igemm launches cost ~3x more)
    const int64_t bytes = (int64_t)d->n * d->di * d->hi * d->wi * d->ci *
                          (dtype == MMAD_BF16 ? 2 : 4);
    const int rc = zero_fill(dx, bytes, as_stream(stream));
    if (rc) return rc;
    return run_igemm<DGRAD>(g, dtype, mmax, 1, dy, wpt, nullptr, dx, nullptr, as_stream(stream));
  }
  return run_igemm<DGRAD>(g, dtype, mmax, d->sd * d->sh * d->sw, dy, wpt, nullptr, dx, nullptr,
                          as_stream(stream));
}

// dgrad routes whose epilogue also writes the BN-backward partial sums of the BN+ReLU that
// produced the conv's input (bnsum.h): 1 = the plane-pair residue-class kernel (layer4),
// 2 = the dilation-2 residue-class kernel (layer3), 3 = the patch conv (layer2's 128-channel
// stride-1 conv; not its persistent z-walking form)
static int bnsum_route(const mmad_conv_desc* d, int dtype, mmad_patch::Geo* qo) {
  if (dtype != MMAD_BF16 || !desc_ok(d) || unfolded(d) || !dgrad_as_fwd(d)) return 0;
  if (mmad_pw::ok(d, dtype)) return 0;
  const Geom gf = dgrad_fwd_geom(d, dtype);
  if (!geom_ok(gf, dtype)) return 0;
  const mmad_patch::Geo q = patch_geo(gf);
  int route = 0;
  if (use_lattice(gf, dtype)) {
    if (!mmad_lattice5::ok(q) && mmad_lattice_zp::ok(q)) route = 1;
  } else if (use_lattice8(gf, dtype)) {
    route = 2;
  } else if (use_patch(gf, dtype) && !mmad_patchz::ok(q)) {
    route = 3;
  }
  if (route) *qo = q;
  return route;
}

int64_t mmad_conv3d_dgrad_bnsum_rows(const mmad_conv_desc* d, int dtype) {
  mmad_patch::Geo q{};
  switch (bnsum_route(d, dtype, &q)) {
    case 1: return mmad_lattice_zp::tiles(q);
    case 2: return mmad_lattice8::tiles(q);
    case 3: return mmad_patch::tiles(q);
    default: return -1;
  }
}

int mmad_conv3d_dgrad_bnsum(const mmad_conv_desc* d, int dtype, const void* dy, const void* wpt,
                            void* dx, const void* y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, float* parts, void* stream) {
  if (!dy || !wpt || !dx || !y || !scale || !shift || !mean || !invstd || !parts)
    return MMAD_ENULL;
  mmad_patch::Geo q{};
  const int route = bnsum_route(d, dtype, &q);
  if (route == 0) return MMAD_EUNSUPPORTED;
  if (((uintptr_t)scale | (uintptr_t)shift | (uintptr_t)mean | (uintptr_t)invstd) & 15)
    return MMAD_EBADSHAPE;                        // (16-byte constant loads)
  if (!al16(dy, wpt, dx) || !al16(y)) return MMAD_EBADSHAPE;
  q.bny = y;
  q.bnsc = scale; q.bnsh = shift; q.bnmu = mean; q.bnis = invstd;
  q.bnparts = parts;
  switch (route) {
    case 1: return mmad_lattice_zp::fwd(q, dy, wpt, nullptr, dx, nullptr, stream);
    case 2: return mmad_lattice8::fwd(q, dy, wpt, nullptr, dx, nullptr, stream);
    default: return mmad_patch::fwd(q, dy, wpt, nullptr, dx, nullptr, stream);
  }
}

int64_t mmad_conv3d_wgrad_workspace(const mmad_conv_desc* d, int dtype) {
  if (!desc_ok(d)) return -1;
  const Geom g = fwd_geom(d, dtype);
  const WSplit sp = wgrad_split(g, dtype);
  int64_t slabs = (int64_t)sp.splits * g.Nd * g.K * 4;
  if (!unfolded(d) && use_lattice_wgrad(g, dtype))
    slabs = std::max<int64_t>(slabs, mmad_lattice::wgrad_workspace(patch_geo(g)));
  if (!unfolded(d) && use_pwgrad(g, dtype))
    slabs = std::max<int64_t>(slabs, mmad_pwgrad::workspace(patch_geo(g)));
  if (!unfolded(d) && mmad_pw::wgrad_ok(d, dtype))
    slabs = std::max<int64_t>(slabs, mmad_pw::wgrad_splits(d) * g.Nd * g.K * 4);
  if (unfolded(d) && mmad_stem::fwd_ok(d, dtype) && stem_kernel_on())
    slabs = std::max<int64_t>(slabs, mmad_stem::wgrad_blocks(d) * g.Nd * g.K * 4);
  const int64_t parts = (int64_t)1024 * 2 * g.Nd * 4;   // bias-gradient column sums
  return std::max(slabs, parts);
}

int mmad_colsum_ws(int dtype, int64_t m, int c, const void* y, float* parts, float* out,
                   void* stream);

}  // extern "C"

namespace {

// make `rst` wait for everything queued on `st` so far (one reusable event per device: a
// wait binds to the record made before it, also under stream capture)
int fork_stream(hipStream_t st, hipStream_t rst) {
  static hipEvent_t ev[16] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return MMAD_EHIP;
  if (!ev[dev]) {
    const int rc = hip_status(hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming));
    if (rc) return rc;
  }
  int rc = hip_status(hipEventRecord(ev[dev], st));
  if (rc) return rc;
  return hip_status(hipStreamWaitEvent(rst, ev[dev], 0));
}

// weight gradient: the split-K kernel on `st`, then the slab reduction (and the bias
// gradient) on `rst` -- a second stream lets the memory-bound reduction overlap the
// latency-bound BN backward kernels that follow on `st`
// defer (non-null, no bias): the slab reduction is recorded there instead of launched when
// the path has one (defer->kind = KIND_NONE: everything ran inline)
int conv3d_wgrad(const mmad_conv_desc* d, int dtype, const void* x, const void* dy, float* dw,
                 float* dbias, void* workspace, hipStream_t st, hipStream_t rst,
                 int raw_dtype = -1, mmad_reduce::Job* defer = nullptr) {
  if (defer != nullptr) {
    *defer = mmad_reduce::Job{};
    if (dbias != nullptr) return MMAD_EUNSUPPORTED;
  }
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (dtype != MMAD_F32 && dtype != MMAD_BF16) return MMAD_EBADDTYPE;
  if (!x || !dy || !dw || !workspace) return MMAD_ENULL;
  if (!al16(x, dy, workspace)) return MMAD_EBADSHAPE;
  const Geom g = fwd_geom(d, dtype);
  if (!geom_ok(g, dtype) || g.Nd % (dtype == MMAD_BF16 ? 8 : 4)) return MMAD_EUNSUPPORTED;
  void* const stream = st;
  void* const rstream = rst;
  int rc;
  // (the bf16 1x1x1 and stride-2 3^3 weight gradients leave below for pw_wgrad_kernel,
  // pointwise.hip; what stays on wgrad_kernel is fp32 and the geometries it declines)
  if (raw_dtype >= 0 && !(unfolded(d) && mmad_stem::fwd_ok(d, dtype) && g.K == 392))
    return MMAD_EUNSUPPORTED;                    // raw input: the stem kernel or nothing
  if (unfolded(d) && mmad_stem::fwd_ok(d, dtype) && (stem_kernel_on() || raw_dtype >= 0) &&
      g.K == 392) {
    rc = mmad_stem::wgrad(d, x, dy, (float*)workspace, stream, raw_dtype);
    if (rc) return rc;
    // (one slab per block: sum 16-slab groups in place first, so no thread walks them all)
    const int nb = (int)mmad_stem::wgrad_blocks(d);
    const int64_t total = (int64_t)g.Nd * g.K;
    constexpr int G = 16;
    static_assert(G == mmad_reduce::STEM_G, "the deferred stem reduction sums the same groups");
    if (defer != nullptr && cdiv(nb, G) <= 32) {
      mmad_reduce::Job& j = *defer;
      j.ws = (const float*)workspace; j.dw = dw; j.splits = nb; j.nd = g.Nd; j.k = g.K;
      j.cs = g.Cs; j.taps = g.taps; j.tper = d->kw; j.kind = mmad_reduce::KIND_STEM;
      j.gx = (int)cdiv(total, 64); j.gy = 1; j.gz = 1;
      return MMAD_OK;
    }
    if (rst != st && (rc = fork_stream(st, rst))) return rc;
    hipLaunchKernelGGL(slab_group_sum_kernel, dim3(grid_for(total * cdiv(nb, G))), dim3(256), 0,
                       rst, (float*)workspace, nb, total, G);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for(total)), dim3(256), 0, rst,
                       (const float*)workspace, dw, nb, g.Nd, g.K, g.Cs, g.cs_shift, g.taps,
                       d->kw, G);
    rc = launch_status();
    if (rc) return rc;
    if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, rstream);
    return MMAD_OK;
  }
  if (!unfolded(d) && (use_lattice_wgrad(g, dtype) || use_pwgrad(g, dtype))) {
    int splits = 0;
    rc = use_pwgrad(g, dtype)
             ? mmad_pwgrad::wgrad(patch_geo(g), x, dy, (float*)workspace, &splits, stream)
             : mmad_lattice::wgrad(patch_geo(g), x, dy, (float*)workspace, &splits, stream);
    if (rc) return rc;
    if (defer != nullptr) {
      *defer = plan_reduce_t((const float*)workspace, dw, splits, g.Nd, g.K, g.Cs, g.taps);
      return MMAD_OK;
    }
    if (rst != st && (rc = fork_stream(st, rst))) return rc;
    rc = launch_reduce_t((const float*)workspace, dw, splits, g.Nd, g.K, g.Cs, g.taps, rst);
    if (rc) return rc;
    if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, rstream);
    return MMAD_OK;
  }
  if (!unfolded(d) && mmad_pw::wgrad_ok(d, dtype)) {
    // 1x1x1 (the shortcuts) and the stride-2 3^3 conv: the pointwise split-K GEMM, then the
    // wide (1^3) or transposing (3^3) slab reduction
    rc = mmad_pw::wgrad(d, x, dy, (float*)workspace, st);
    if (rc) return rc;
    const int splits = (int)mmad_pw::wgrad_splits(d);
    const int64_t total = (int64_t)g.Nd * g.K;
    if (g.taps > 1) {
      if (defer != nullptr) {
        *defer = plan_reduce_t((const float*)workspace, dw, splits, g.Nd, g.K, g.Cs, g.taps);
        return MMAD_OK;
      }
      if (rst != st && (rc = fork_stream(st, rst))) return rc;
      rc = launch_reduce_t((const float*)workspace, dw, splits, g.Nd, g.K, g.Cs, g.taps, rst);
      if (rc) return rc;
      if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, rstream);
      return MMAD_OK;
    }
    if (defer != nullptr && ((uintptr_t)dw & 15) == 0) {
      mmad_reduce::Job& j = *defer;
      j.ws = (const float*)workspace; j.dw = dw; j.splits = splits; j.nd = g.Nd;
      j.k = g.K; j.cs = g.Cs; j.taps = 1; j.kind = mmad_reduce::KIND_WIDE;
      j.gx = (int)cdiv(total, 256); j.gy = 1; j.gz = 1;
      return MMAD_OK;
    }
    if (rst != st && (rc = fork_stream(st, rst))) return rc;
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       rst, (const float*)workspace, dw, splits, g.Nd, g.K, g.Cs, g.cs_shift,
                       g.taps, 0, 1);
    rc = launch_status();
    if (rc) return rc;
    if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, rstream);
    return MMAD_OK;
  }
  const WSplit sp = wgrad_split(g, dtype);
  if (dtype == MMAD_BF16)
    rc = sp.bmw == 256 ? (wgrad_big(g, dtype) == 3
                              ? launch_wgrad_k<u16, 256, 32, 3, 256, 2, 4>(g, sp, x, dy,
                                                                          (float*)workspace, st)
                              : launch_wgrad_k<u16, 256, 32, 2, 256, 2, 4>(g, sp, x, dy,
                                                                          (float*)workspace, st))
       : sp.bmw == 64 ? launch_wgrad<u16, 64>(g, sp, x, dy, (float*)workspace, st)
                      : launch_wgrad<u16, 128>(g, sp, x, dy, (float*)workspace, st);
  else
    rc = sp.bmw == 64 ? launch_wgrad<float, 64>(g, sp, x, dy, (float*)workspace, st)
                      : launch_wgrad<float, 128>(g, sp, x, dy, (float*)workspace, st);
  if (rc) return rc;
  const int64_t total = (int64_t)g.Nd * g.K;
  if (defer != nullptr && !unfolded(d)) {
    if (g.taps > 1 && g.taps <= 32) {
      *defer = plan_reduce_t((const float*)workspace, dw, sp.splits, g.Nd, g.K, g.Cs, g.taps);
      return MMAD_OK;
    }
    if (g.taps == 1 && sp.splits >= 8 && total % 4 == 0 && ((uintptr_t)dw & 15) == 0) {
      mmad_reduce::Job& j = *defer;
      j.ws = (const float*)workspace; j.dw = dw; j.splits = sp.splits; j.nd = g.Nd;
      j.k = g.K; j.cs = g.Cs; j.taps = 1; j.kind = mmad_reduce::KIND_WIDE;
      j.gx = (int)cdiv(total, 256); j.gy = 1; j.gz = 1;
      return MMAD_OK;
    }
  }
  if (rst != st && (rc = fork_stream(st, rst))) return rc;
  // (the transposing reduce writes whole [ci][taps] runs of dW; scattered 4-byte dW stores
  // from an element-wise reduce cost ~2x in partial-line writes)
  if (!unfolded(d) && g.taps > 1 && g.taps <= 32) {
    rc = launch_reduce_t((const float*)workspace, dw, sp.splits, g.Nd, g.K, g.Cs, g.taps, rst);
    if (rc) return rc;
  } else if (sp.splits >= 8)
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       rst, (const float*)workspace, dw, sp.splits, g.Nd, g.K, g.Cs, g.cs_shift,
                       g.taps, unfolded(d) ? d->kw : 0, 1);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for(total)), dim3(256), 0, rst,
                       (const float*)workspace, dw, sp.splits, g.Nd, g.K, g.Cs, g.cs_shift,
                       g.taps, unfolded(d) ? d->kw : 0, 1);
  rc = launch_status();
  if (rc) return rc;
  if (dbias) return mmad_colsum_ws(dtype, g.M, g.Nd, dy, (float*)workspace, dbias, rstream);
  return MMAD_OK;
}

}  // namespace

extern "C" {

int mmad_conv3d_wgrad(const mmad_conv_desc* d, int dtype, const void* x, const void* dy,
                      float* dw, float* dbias, void* workspace, void* stream) {
  return conv3d_wgrad(d, dtype, x, dy, dw, dbias, workspace, as_stream(stream),
                      as_stream(stream));
}

int mmad_conv3d_wgrad_deferred(const mmad_conv_desc* d, int dtype, const void* x,
                               const void* dy, float* dw, void* workspace, mmad_wgrad_job* job,
                               void* stream) {
  if (job == nullptr) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  return conv3d_wgrad(d, dtype, x, dy, dw, nullptr, workspace, st, st, -1, job);
}

int mmad_wgrad_reduce_batch(int njobs, const mmad_wgrad_job* jobs, void* stream) {
  if (njobs < 0 || (njobs > 0 && jobs == nullptr)) return MMAD_ENULL;
  hipStream_t st = as_stream(stream);
  ReduceBatch b{};
  auto flush = [&]() -> int {
    if (b.n == 0) return MMAD_OK;
    const int64_t blocks = b.start[b.n];
    b.n_total = (int)blocks;
    hipLaunchKernelGGL(wgrad_reduce_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b);
    b = ReduceBatch{};
    return launch_status();
  };
  for (int i = 0; i < njobs; ++i) {
    const mmad_reduce::Job& j = jobs[i];
    const int64_t nb = mmad_reduce::job_blocks(j);
    if (nb <= 0) continue;
    if (!j.ws || !j.dw) return MMAD_ENULL;
    if (b.n == kReduceBatch || (int64_t)b.start[b.n] + nb > 0x7fffffff) {
      const int rc = flush();
      if (rc) return rc;
    }
    b.jobs[b.n] = j;
    b.start[b.n + 1] = b.start[b.n] + (int)nb;
    ++b.n;
  }
  return flush();
}

int mmad_conv3d_wgrad_raw_deferred(const mmad_conv_desc* d, int in_dtype, const void* x,
                                   int dtype, const void* dy, float* dw, void* workspace,
                                   mmad_wgrad_job* job, void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (job == nullptr) return MMAD_ENULL;
  if (!mmad_stem_raw_ok(d, in_dtype, dtype)) return MMAD_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  return conv3d_wgrad(d, dtype, x, dy, dw, nullptr, workspace, st, st, in_dtype, job);
}

int mmad_conv3d_wgrad_split(const mmad_conv_desc* d, int dtype, const void* x, const void* dy,
                            float* dw, float* dbias, void* workspace, void* stream,
                            void* reduce_stream) {
  if (!reduce_stream) return MMAD_ENULL;
  return conv3d_wgrad(d, dtype, x, dy, dw, dbias, workspace, as_stream(stream),
                      as_stream(reduce_stream));
}

int mmad_stem_raw_ok(const mmad_conv_desc* d, int in_dtype, int dtype) {
  if (!desc_ok(d) || !unfolded(d) || dtype != MMAD_BF16 || !stem_kernel_on()) return 0;
  return mmad_stem::fwd_ok(d, dtype) && mmad_stem::raw_ok(d, in_dtype) ? 1 : 0;
}

int mmad_conv3d_fwd_raw(const mmad_conv_desc* d, int in_dtype, const void* x, int dtype,
                        const void* w_packed, const float* bias, void* y, float* stats,
                        void* stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (!x || !w_packed || !y) return MMAD_ENULL;
  if (!al16(x, w_packed, y)) return MMAD_EBADSHAPE;
  if (!mmad_stem_raw_ok(d, in_dtype, dtype)) return MMAD_EUNSUPPORTED;
  return mmad_stem::fwd(d, x, w_packed, bias, y, stats, stream, in_dtype);
}

int mmad_conv3d_wgrad_raw(const mmad_conv_desc* d, int in_dtype, const void* x, int dtype,
                          const void* dy, float* dw, float* dbias, void* workspace,
                          void* stream, void* reduce_stream) {
  if (!desc_ok(d)) return MMAD_EBADSHAPE;
  if (!mmad_stem_raw_ok(d, in_dtype, dtype)) return MMAD_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  return conv3d_wgrad(d, dtype, x, dy, dw, dbias, workspace, st,
                      reduce_stream ? as_stream(reduce_stream) : st, in_dtype);
}

}  // extern "C"

__global__ void zero_fill_kernel(uint32_t* __restrict__ p, int64_t words) {
  const int64_t n4 = words >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<u32x4*>(p)[i] = u32x4{0u, 0u, 0u, 0u};
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words;
       i += stride)
    p[i] = 0u;
}

int zero_fill(void* p, int64_t bytes, hipStream_t st) {
  if (bytes <= 0) return MMAD_OK;
  if (((uintptr_t)p & 15) || (bytes & 3)) return MMAD_EUNSUPPORTED;
  const int64_t words = bytes / 4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(cdiv(words / 4, 256), 4096));
  hipLaunchKernelGGL(zero_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (uint32_t*)p, words);
  return launch_status();
}
