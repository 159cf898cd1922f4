// Stride-2 3x3x3 convolution, forward, gfx950 bf16 with fp32 accumulation: the first conv
// of MedicalNet's layer2 (64 -> 128 channels, 32^3 -> 16^3 at a 128^3 input; BasicBlock
// conv1 with stride 2, reached from pkg/models/mri_models/anat_cnn.py:29-31).
//
// On the implicit GEMM (conv.hip) this conv ran at 10-15 % of the MFMA peak: 512 tiles of
// 64 voxels whose every K stage gathers 64 stride-2 rows through a two-deep LDS ring, so each
// stage waits out an L2 round trip.  Here a block owns a 2 x 8 x 8 box of output voxels (128
// GEMM rows) x 128 output channels and keeps its input in LDS as a patch, so every input
// voxel is fetched once per block instead of once per tap:
//  * the input box (5 x 17 x 17 voxels x 64 channels) is split by the parity of its
//    coordinates into 8 sub-patches ("chunks"); in each dimension the even inputs meet one
//    tap (k = 1, output o reads input 2o) and the odd ones two (k = 0 reads 2o - 1, k = 2 reads
//    2o + 1 = 2(o + 1) - 1), so a chunk of parity (bz, by, bx) carries (1+bz)(1+by)(1+bx) of the
//    27 taps and inside a chunk every tap is a dense, unit-stride shift of {0, 1} per
//    dimension -- the stride-2 gather disappears from the inner loop;
//  * chunks are walked in order of decreasing tap count (8, 4, 4, 4, 2, 2, 2, 1) through two
//    32 KiB patch slots: chunk c + 1's sub-patch (3 x 9 x 9 rows of 128 B) is DMA'd during
//    chunk c, so a patch reload never stalls the MFMAs;
//  * the weights (128 co x 64 ci = 16 KiB per tap) stream through a 5-slot LDS ring, four
//    taps ahead; the 27 stages are unrolled at compile time, and every stage's counted
//    vmcnt wait is a constant derived from the issue schedule (stage_wait below);
//  * 8 waves = 4 (32 voxels) x 2 (64 channels); fragments are read one K-half ahead of their
//    MFMAs (the next stage's first half right after the stage barrier);
//  * sub-patch rows are 16-byte-chunk swizzled by (2 * x) & 7, which keeps every
//    ds_read_b128 fragment read of every tap on distinct bank slots (checked exhaustively
//    over the 27 taps for the 3 x 9 x 9 layout);
//  * epilogue as the implicit GEMM: bias, BN partial sums (one row per tile), optional
//    residual + ReLU (eval-mode folded BN), bf16 tile transposed through LDS into 16-byte
//    channel-vector stores.
#include <cstdlib>
#include <utility>

#include "common.h"
#include "patchconv.h"

namespace {

constexpr int TZ = 2, TY = 8, TX = 8, TV = TZ * TY * TX;   // output box: 128 GEMM rows
constexpr int QZ = 3, QY = 9, QX = 9;                      // sub-patch extents (odd parity)
constexpr int QROWS = QZ * QY * QX;                        // 243 rows used
constexpr int RB = 128;                                    // 64 ci x bf16 per row
constexpr int PSLOT = 256 * RB;                            // 32 KiB (rows padded to 256)
constexpr int NTHR = 512, NW = NTHR / 64;
constexpr int NSL = 5;                                     // weight ring slots
constexpr int NSTAGE = 27;
constexpr int PI = 256 / 8 / NW;                           // patch DMA instructions per wave

template <int BN>
struct SC {
  static constexpr int WSLOT = BN * RB;
  static constexpr int BI = WSLOT / 1024 / NW;             // weight DMA instructions per wave
  static constexpr int WGN = BN / 64, WGM = NW / WGN;
  static constexpr int WTM = TV / WGM, TM = WTM / 16, TN = 4;
  static constexpr int RING = 2 * PSLOT;
  static constexpr int MAIN = RING + NSL * WSLOT;
  static constexpr int CROW = BN * 2 + 16;
  static constexpr int EPI = TV * CROW + (WGM - 1) * 2 * BN * 4;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static_assert(BI >= 1 && BI * NW * 1024 == WSLOT, "weight slot split");
};

// chunk walk order: parity codes (bz << 2 | by << 1 | bx) by decreasing tap count
__host__ __device__ constexpr int chunk_parity(int c) {
  return c == 0 ? 7 : c == 1 ? 6 : c == 2 ? 5 : c == 3 ? 3 : c == 4 ? 4 : c == 5 ? 2 : c == 6 ? 1 : 0;
}
__host__ __device__ constexpr int chunk_taps(int c) {
  const int p = chunk_parity(c);
  return (1 + ((p >> 2) & 1)) * (1 + ((p >> 1) & 1)) * (1 + (p & 1));
}
__host__ __device__ constexpr int chunk_first(int c) {
  int s = 0;
  for (int i = 0; i < c; ++i) s += chunk_taps(i);
  return s;
}
__host__ __device__ constexpr int stage_chunk(int s) {
  int c = 0;
  while (c + 1 < 8 && chunk_first(c + 1) <= s) ++c;
  return c;
}
struct StageInfo {
  int c, slot, tap, sz, sy, sx;   // chunk, its patch slot, torch tap index, sub-patch shift
};
__host__ __device__ constexpr StageInfo stage_info(int s) {
  const int c = stage_chunk(s), p = chunk_parity(c), j = s - chunk_first(c);
  const int bz = (p >> 2) & 1, by = (p >> 1) & 1, bx = p & 1;
  const int ny = 1 + by, nx = 1 + bx;
  const int jz = j / (ny * nx), jy = (j / nx) % ny, jx = j % nx;
  // odd parity: local index 0 -> k = 0 (shift 0), 1 -> k = 2 (shift 1); even: k = 1
  const int kz = bz ? 2 * jz : 1, ky = by ? 2 * jy : 1, kx = bx ? 2 * jx : 1;
  return StageInfo{c, c & 1, (kz * 3 + ky) * 3 + kx, kz == 2, ky == 2, kx == 2};
}

// The issue schedule (per wave; every wave issues the same counts):
//   prologue: patch(0), weights(0 .. NSL-2)
//   boundary before stage s (after its barrier): patch(c + 1) when s opens chunk c (c < 7),
//   then weights(s + NSL - 1) into the slot stage s - 1 just released.
// stage_wait(s) = DMA instructions issued after the later of weights(s) and patch(chunk(s))
// up to the wait before stage s: the vmcnt that guarantees both have landed.
template <int BN>
__host__ __device__ constexpr int stage_wait(int s) {
  constexpr int BI = SC<BN>::BI;
  // positions (running instruction counts at the END of each event) in issue order
  int pos = 0, need_end = 0;
  const int cs = stage_chunk(s);
  // prologue
  pos += PI;
  if (cs == 0) need_end = pos;                    // patch(0)
  for (int w = 0; w <= NSL - 2 && w < NSTAGE; ++w) {
    pos += BI;
    if (w == s && pos > need_end) need_end = pos;
  }
  for (int b = 0; b < s; ++b) {                   // boundaries before stages 0 .. s-1
    const int c = stage_chunk(b);
    if (b == chunk_first(c) && c + 1 < 8) {
      pos += PI;
      if (c + 1 == cs && pos > need_end) need_end = pos;
    }
    const int w = b + NSL - 1;
    if (w < NSTAGE) {
      pos += BI;
      if (w == s && pos > need_end) need_end = pos;
    }
  }
  return pos - need_end;
}

__device__ const u32x4 g_s2zero[8] = {};

struct S2G {
  int Ds, Hs, Ws, Dd, Hd, Wd, Nd, Kpad, nby, nbx, nbz, nbn;
  const u16* res;
  int relu;
};

template <int BN>
__global__ __launch_bounds__(NTHR) void s2conv_kernel(S2G g, const u16* __restrict__ src,
                                                      const u16* __restrict__ wgt,
                                                      const float* __restrict__ bias,
                                                      u16* __restrict__ dst,
                                                      float* __restrict__ stats) {
  using C = SC<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wring = smem + C::RING;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: each XCD walks a contiguous range of tiles (the N tiles of one box share
  // its patch; neighbouring boxes share halo voxels)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = tile / g.nbn, nt = tile % g.nbn;
  int t1 = mt;
  const int bx = t1 % g.nbx;
  t1 /= g.nbx;
  const int by = t1 % g.nby;
  t1 /= g.nby;
  const int bz = t1 % g.nbz, bn = t1 / g.nbz;
  const int oz0 = bz * TZ, oy0 = by * TY, ox0 = bx * TX, n0 = nt * BN;
  const u16* __restrict__ srcb = src + (int64_t)bn * g.Ds * g.Hs * g.Ws * 64;

  // ---- sub-patch DMA: row r = (qz, qy, qx) of chunk parity p holds input voxel
  // (2 (o0 + q) - b) per dimension (b = parity bit); rows past 243 and voxels outside the
  // volume (the conv's zero padding) read the zero block
  int prow[PI], pq[PI], pqx[PI];
#pragma unroll
  for (int k = 0; k < PI; ++k) {
    const int r = (wave * PI + k) * 8 + (lane >> 3);
    prow[k] = r;
    const int qz = r / (QY * QX), qy = (r / QX) % QY, qx = r % QX;
    pq[k] = (qz << 8) | qy;
    pqx[k] = qx;
  }
  auto issue_patch = [&](auto pc, int slot) {
    constexpr int P = decltype(pc)::value;
    constexpr int BZ = (P >> 2) & 1, BY = (P >> 1) & 1, BX = P & 1;
#pragma unroll
    for (int k = 0; k < PI; ++k) {
      const int qz = pq[k] >> 8, qy = pq[k] & 255, qx = pqx[k];
      const int z = 2 * (oz0 + qz) - BZ, y = 2 * (oy0 + qy) - BY, x = 2 * (ox0 + qx) - BX;
      const void* p = g_s2zero;
      if (prow[k] < QROWS && (unsigned)z < (unsigned)g.Ds && (unsigned)y < (unsigned)g.Hs &&
          (unsigned)x < (unsigned)g.Ws) {
        const int chunk = (lane & 7) ^ ((2 * qx) & 7);
        p = srcb + ((int64_t)((z * g.Hs + y) * g.Ws + x) * 64 + chunk * 8);
      }
      glds16_asm(p, lds_addr_of(smem + slot * PSLOT + (wave * PI + k) * 1024));
    }
  };
  // ---- weight DMA: stage s's tap into ring slot s % NSL; instruction q = wave * BI + i holds
  // co rows 8q .. 8q + 7 (chunk swizzle = row & 7 = lane >> 3)
  const u16* wrow[C::BI];
#pragma unroll
  for (int i = 0; i < C::BI; ++i) {
    const int co = n0 + (wave * C::BI + i) * 8 + (lane >> 3);
    wrow[i] = wgt + (int64_t)co * g.Kpad + (((lane & 7) ^ (lane >> 3)) * 8);
  }
  auto issue_w = [&](int tap, int slot) {
#pragma unroll
    for (int i = 0; i < C::BI; ++i)
      glds16_asm(wrow[i] + tap * 64, lds_addr_of(wring + slot * C::WSLOT + (wave * C::BI + i) * 1024));
  };

  const int wm = wave % C::WGM, wn = wave / C::WGM;
  const int lr = lane & 15, lk = lane >> 4;
  int arow[C::TM], atx[C::TM];
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    const int v = wm * C::WTM + i * 16 + lr;
    const int tz = v >> 6, ty = (v >> 3) & 7, tx = v & 7;
    arow[i] = (tz * QY + ty) * QX + tx;
    atx[i] = tx;
  }
  f32x4 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[C::TM], fb0[C::TN], fa1[C::TM], fb1[C::TN];

  auto read_frags = [&](auto sc, int h, bf16x8* A, bf16x8* B) {
    constexpr StageInfo I = stage_info(decltype(sc)::value);
    constexpr int dr = (I.sz * QY + I.sy) * QX + I.sx;
    const int c = 4 * h + lk;
    const char* pbase = smem + I.slot * PSLOT;
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
      A[i] = *reinterpret_cast<const bf16x8*>(pbase + (arow[i] + dr) * RB +
                                              ((c ^ ((2 * (atx[i] + I.sx)) & 7)) << 4));
    const char* wb = wring + (decltype(sc)::value % NSL) * C::WSLOT;
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const int row = wn * 64 + j * 16 + lr;
      B[j] = *reinterpret_cast<const bf16x8*>(wb + row * RB + ((c ^ (lr & 7)) << 4));
    }
  };
  auto mma = [&](const bf16x8* A, const bf16x8* B) {
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
  };
  // DMA issued at the boundary before stage S (after its barrier)
  auto boundary_issue = [&](auto sc) {
    constexpr int S = decltype(sc)::value;
    constexpr int CH = stage_chunk(S);
    if constexpr (S == chunk_first(CH) && CH + 1 < 8)
      issue_patch(std::integral_constant<int, chunk_parity(CH + 1)>{}, (CH + 1) & 1);
    if constexpr (S + NSL - 1 < NSTAGE)
      issue_w(stage_info(S + NSL - 1).tap, (S + NSL - 1) % NSL);
  };

  // prologue
  issue_patch(std::integral_constant<int, chunk_parity(0)>{}, 0);
#pragma unroll
  for (int w = 0; w <= NSL - 2; ++w) issue_w(stage_info(w).tap, w);
  wait_vm_lgkm0<stage_wait<BN>(0)>();
  raw_barrier();
  boundary_issue(std::integral_constant<int, 0>{});
  read_frags(std::integral_constant<int, 0>{}, 0, fa0, fb0);

  [&]<int... S>(std::integer_sequence<int, S...>) {
    (
        [&] {
          read_frags(std::integral_constant<int, S>{}, 1, fa1, fb1);
          mma(fa0, fb0);
          if constexpr (S + 1 < NSTAGE) {
            wait_vm_lgkm0<stage_wait<BN>(S + 1)>();
            raw_barrier();
            boundary_issue(std::integral_constant<int, S + 1>{});
            read_frags(std::integral_constant<int, S + 1>{}, 0, fa0, fb0);
          }
          mma(fa1, fb1);
        }(),
        ...);
  }(std::make_integer_sequence<int, NSTAGE>{});
  __syncthreads();                                  // patch / ring reused by the epilogue

  // ---- epilogue: tile row v = (tz, ty, tx); every box lies inside the output grid
  constexpr int CROW = C::CROW;
  u16* ctile = reinterpret_cast<u16*>(smem);
  float cs[C::TN], cq[C::TN];
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    cs[j] = 0.f;
    cq[j] = 0.f;
    const int col = wn * 64 + j * 16 + lr;
    const float bv = bias != nullptr ? bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * C::WTM + i * 16 + lk * 4 + r;
        const float v = acc[i][j][r] + bv;
        ctile[row * (CROW / 2) + col] = f2bf(v);
        cs[j] += v;
        cq[j] += v * v;
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  const int64_t vbase = (((int64_t)bn * g.Dd + oz0) * g.Hd + oy0) * g.Wd + ox0;
  u16* __restrict__ dstb = dst + vbase * g.Nd + n0;
  const u16* __restrict__ resb = g.res != nullptr ? g.res + vbase * g.Nd + n0 : nullptr;
#pragma unroll
  for (int hh = 0; hh < TV * CPR / NTHR; ++hh) {
    const int q = tid + NTHR * hh;
    const int row = q / CPR, c8 = q % CPR;
    const int o = (((row >> 6) * g.Hd + ((row >> 3) & 7)) * g.Wd + (row & 7)) * g.Nd + c8 * 8;
    u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                              row * CROW + c8 * 16);
    if (g.res != nullptr || g.relu) v = epi_res_relu(v, resb ? resb + o : nullptr, g.relu);
    *reinterpret_cast<u32x4*>(dstb + o) = v;
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(smem + TV * CROW);
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm > 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int col = wn * 64 + j * 16 + lr;
        red[(wm - 1) * 2 * BN + col] = cs[j];
        red[(wm - 1) * 2 * BN + BN + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int col = wn * 64 + j * 16 + lr;
        float ss = cs[j], qs = cq[j];
        for (int w = 1; w < C::WGM; ++w) {           // fixed order: deterministic
          ss += red[(w - 1) * 2 * BN + col];
          qs += red[(w - 1) * 2 * BN + BN + col];
        }
        stats[((int64_t)mt * 2) * g.Nd + n0 + col] = ss;
        stats[((int64_t)mt * 2 + 1) * g.Nd + n0 + col] = qs;
      }
    }
  }
}

// ---- input gradient ------------------------------------------------------------------
// dX[i] = sum over (o, k) with 2o - 1 + k = i of dY[o] W[k]^T, per dimension.  Split dX by
// the parity b of its coordinates (i = 2j + b): b = 0 meets only k = 1 (o = j), b = 1 meets
// k = 0 (o = j + 1) and k = 2 (o = j).  So for a box of class positions j, ALL 8 parity
// classes read dY only at j + {0, 1}^3: one dY patch (3 x 9 x 9 rows x 128 co = 64 KiB)
// serves the whole block, and class b is a dense GEMM over (1+bz)(1+by)(1+bx) taps x 128 co
// (27 taps over the 8 classes, none wasted).  The implicit GEMM ran the classes as 8 separate
// grids of 64-voxel tiles, at 10 % of the MFMA peak.
//  * block = one 2 x 8 x 8 box of class positions (128 rows) x all 64 input channels, for all
//    8 classes in turn (heaviest first); 8 waves = 4 (32 rows) x 2 (32 ci), a stage = one tap
//    (K = 128 co, two halves of 64);
//  * packed dgrad weights [ci][tap][co] (conv.hip's layout for strided dgrads): 16 KiB per
//    tap through a 4-slot ring, three taps ahead;
//  * a class's epilogue goes through its own LDS tile (the ring and the patch stay live): 16-B
//    channel-vector stores of 128 B dX rows; the accumulators restart for the next class.
//  * 256-B rows: patch chunks swizzled by (2 x) & 15, weight rows by row & 15 (conflict-free
//    ds_read_b128 fragments, checked exhaustively).
constexpr int DRB = 256;                                   // 128 co x bf16 per row
constexpr int DPATCH = 256 * DRB;                          // 64 KiB (243 rows used)
constexpr int DWSLOT = 64 * DRB;                           // 64 ci rows per tap: 16 KiB
constexpr int DNSL = 4;
constexpr int DPI = DPATCH / 1024 / NW;                    // 8 patch DMA instructions / wave
constexpr int DBI = DWSLOT / 1024 / NW;                    // 2 weight DMA instructions / wave
constexpr int DCROW = 64 * 2 + 16;
constexpr int D_WRING = DPATCH;
constexpr int D_CTILE = DPATCH + DNSL * DWSLOT;
constexpr int DLDS = D_CTILE + TV * DCROW;                 // 146 KiB

// class walk = chunk_parity order; stage s -> (class, tap, dY shift)
__host__ __device__ constexpr StageInfo dstage_info(int s) {
  const int c = stage_chunk(s), p = chunk_parity(c), j = s - chunk_first(c);
  const int bz = (p >> 2) & 1, by = (p >> 1) & 1, bx = p & 1;
  const int ny = 1 + by, nx = 1 + bx;
  const int jz = j / (ny * nx), jy = (j / nx) % ny, jx = j % nx;
  // odd parity: local 0 -> k = 0 (o = j + 1, shift 1), 1 -> k = 2 (shift 0); even: k = 1
  const int kz = bz ? 2 * jz : 1, ky = by ? 2 * jy : 1, kx = bx ? 2 * jx : 1;
  return StageInfo{c, 0, (kz * 3 + ky) * 3 + kx, bz && kz == 0, by && ky == 0, bx && kx == 0};
}
// prologue: patch, weights(0 .. DNSL-2); boundary before stage s: weights(s + DNSL - 1)
__host__ __device__ constexpr int dstage_wait(int s) {
  int pos = DPI, need_end = s == 0 ? DPI : 0;
  for (int w = 0; w <= DNSL - 2; ++w) {
    pos += DBI;
    if (w == s) need_end = pos;
  }
  for (int b = 0; b < s; ++b) {
    const int w = b + DNSL - 1;
    if (w < NSTAGE) {
      pos += DBI;
      if (w == s) need_end = pos;
    }
  }
  return pos - need_end;
}

struct S2D {
  int Do, Ho, Wo, Di, Hi, Wi, Kpad, nbz, nby, nbx;
};

__global__ __launch_bounds__(NTHR) void s2dgrad_kernel(S2D g, const u16* __restrict__ dy,
                                                       const u16* __restrict__ wgt,
                                                       u16* __restrict__ dx) {
  constexpr int TM = 2, TN = 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wring = smem + D_WRING;
  u16* ctile = reinterpret_cast<u16*>(smem + D_CTILE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  int t1 = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int bx = t1 % g.nbx;
  t1 /= g.nbx;
  const int by = t1 % g.nby;
  t1 /= g.nby;
  const int bz = t1 % g.nbz, bn = t1 / g.nbz;
  const int jz0 = bz * TZ, jy0 = by * TY, jx0 = bx * TX;
  const u16* __restrict__ dyb = dy + (int64_t)bn * g.Do * g.Ho * g.Wo * 128;

  // dY patch: instruction k of wave w = rows 4 (w * DPI + k) + lane / 16, chunk lane & 15
  {
#pragma unroll
    for (int k = 0; k < DPI; ++k) {
      const int r = (wave * DPI + k) * 4 + (lane >> 4);
      const int qz = r / (QY * QX), qy = (r / QX) % QY, qx = r % QX;
      const int z = jz0 + qz, y = jy0 + qy, x = jx0 + qx;
      const void* p = g_s2zero;
      if (r < QROWS && z < g.Do && y < g.Ho && x < g.Wo) {
        const int chunk = (lane & 15) ^ ((2 * qx) & 15);
        p = dyb + ((int64_t)((z * g.Ho + y) * g.Wo + x) * 128 + chunk * 8);
      }
      glds16_asm(p, lds_addr_of(smem + (wave * DPI + k) * 1024));
    }
  }
  // weights: tap t's rows ci = 4 (w * DBI + i) + lane / 16, chunk swizzle ci & 15
  const u16* wrow[DBI];
#pragma unroll
  for (int i = 0; i < DBI; ++i) {
    const int ci = (wave * DBI + i) * 4 + (lane >> 4);
    wrow[i] = wgt + (int64_t)ci * g.Kpad + (((lane & 15) ^ (ci & 15)) * 8);
  }
  auto issue_w = [&](int tap, int slot) {
#pragma unroll
    for (int i = 0; i < DBI; ++i)
      glds16_asm(wrow[i] + tap * 128, lds_addr_of(wring + slot * DWSLOT + (wave * DBI + i) * 1024));
  };

  const int wm = wave & 3, wn = wave >> 2;
  const int lr = lane & 15, lk = lane >> 4;
  int arow[TM], atx[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int v = wm * 32 + i * 16 + lr;
    const int tz = v >> 6, ty = (v >> 3) & 7, tx = v & 7;
    arow[i] = (tz * QY + ty) * QX + tx;
    atx[i] = tx;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[2][TM], fb0[2][TN], fa1[2][TM], fb1[2][TN];

  // fragments of half h (co 64h .. 64h + 63: two 32-deep K steps) of stage S
  auto read_frags = [&](auto sc, int h, bf16x8 (*A)[TM], bf16x8 (*B)[TN]) {
    constexpr StageInfo I = dstage_info(decltype(sc)::value);
    constexpr int dr = (I.sz * QY + I.sy) * QX + I.sx;
    const char* wb = wring + (decltype(sc)::value % DNSL) * DWSLOT;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 8 * h + 4 * ks + lk;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        A[ks][i] = *reinterpret_cast<const bf16x8*>(smem + (arow[i] + dr) * DRB +
                                                    ((c ^ ((2 * (atx[i] + I.sx)) & 15)) << 4));
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * 32 + j * 16 + lr;
        B[ks][j] = *reinterpret_cast<const bf16x8*>(wb + row * DRB + ((c ^ (row & 15)) << 4));
      }
    }
  };
  auto mma = [&](bf16x8 (*A)[TM], bf16x8 (*B)[TN]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[ks][i], B[ks][j], acc[i][j], 0, 0, 0);
  };
  // class epilogue: accumulators -> LDS tile -> 16-B stores of dX rows (2j + b)
  auto epilogue = [&](auto cc) {
    constexpr int P = chunk_parity(decltype(cc)::value);
    constexpr int BZ = (P >> 2) & 1, BY = (P >> 1) & 1, BX = P & 1;
    if constexpr (chunk_taps(decltype(cc)::value) == 1) {
      // a one-stage class has no stage barrier between the previous class's tile reads
      // and these writes
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * 32 + j * 16 + lr;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 32 + i * 16 + lk * 4 + r;
          ctile[row * (DCROW / 2) + col] = f2bf(acc[i][j][r]);
        }
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
#pragma unroll
    for (int hh = 0; hh < TV * 8 / NTHR; ++hh) {
      const int q = tid + NTHR * hh;
      const int row = q >> 3, c8 = q & 7;
      const int tz = row >> 6, ty = (row >> 3) & 7, tx = row & 7;
      const int z = 2 * (jz0 + tz) + BZ, y = 2 * (jy0 + ty) + BY, x = 2 * (jx0 + tx) + BX;
      const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                      row * DCROW + c8 * 16);
      *reinterpret_cast<u32x4*>(dx + ((((int64_t)bn * g.Di + z) * g.Hi + y) * g.Wi + x) * 64 +
                                c8 * 8) = v;
    }
    // (the tile is rewritten only after the next class's stage barriers)
  };

#pragma unroll
  for (int w = 0; w <= DNSL - 2; ++w) issue_w(dstage_info(w).tap, w);
  wait_vm_lgkm0<dstage_wait(0)>();
  raw_barrier();
  issue_w(dstage_info(DNSL - 1).tap, DNSL - 1);
  read_frags(std::integral_constant<int, 0>{}, 0, fa0, fb0);

  [&]<int... S>(std::integer_sequence<int, S...>) {
    (
        [&] {
          read_frags(std::integral_constant<int, S>{}, 1, fa1, fb1);
          mma(fa0, fb0);
          if constexpr (S + 1 < NSTAGE) {
            wait_vm_lgkm0<dstage_wait(S + 1)>();
            raw_barrier();
            if constexpr (S + DNSL < NSTAGE) issue_w(dstage_info(S + DNSL).tap, (S + DNSL) % DNSL);
            read_frags(std::integral_constant<int, S + 1>{}, 0, fa0, fb0);
          }
          mma(fa1, fb1);
          constexpr int CH = stage_chunk(S);
          if constexpr (S + 1 == NSTAGE || stage_chunk(S + 1) != CH)
            epilogue(std::integral_constant<int, CH>{});
        }(),
        ...);
  }(std::make_integer_sequence<int, NSTAGE>{});
}

int s2_mode() {
  static const int v = [] { const char* e = getenv("MMAD_S2CONV"); return e ? atoi(e) : 1; }();
  return v;
}

template <int BN>
int launch(const S2G& g, int64_t nblk, const void* src, const void* wp, const float* bias,
           void* dst, float* stats, hipStream_t st) {
  static const bool attr = hipFuncSetAttribute((const void*)s2conv_kernel<BN>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               SC<BN>::LDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  hipLaunchKernelGGL(s2conv_kernel<BN>, dim3((unsigned)nblk), dim3(NTHR), SC<BN>::LDS, st, g,
                     (const u16*)src, (const u16*)wp, bias, (u16*)dst, stats);
  return launch_status();
}

}  // namespace

namespace mmad_s2 {

bool ok(const mmad_patch::Geo& q, int sd, int sh, int sw) {
  if (s2_mode() <= 0) return false;
  if (sd != 2 || sh != 2 || sw != 2) return false;
  if (q.Cs != 64 || q.Nd % 64 || q.Kpad != 27 * 64) return false;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.pd != 1 || q.ph != 1 || q.pw != 1) return false;
  if (q.dd != 1 || q.dh != 1 || q.dw != 1) return false;
  if (q.Ds != 2 * q.Dd || q.Hs != 2 * q.Hd || q.Ws != 2 * q.Wd) return false;
  if (q.Dd % TZ || q.Hd % TY || q.Wd % TX) return false;   // whole boxes only
  const int64_t ivox = (int64_t)q.Ds * q.Hs * q.Ws;
  return ivox * 64 < (int64_t(1) << 31) && (int64_t)q.Dd * q.Hd * q.Wd * q.Nd < (int64_t(1) << 31);
}

int64_t tiles(const mmad_patch::Geo& q) {
  return (int64_t)q.nb * (q.Dd / TZ) * (q.Hd / TY) * (q.Wd / TX);
}

int fwd(const mmad_patch::Geo& q, int sd, int sh, int sw, const void* src, const void* wp,
        const float* bias, void* dst, float* stats, void* stream) {
  if (!ok(q, sd, sh, sw)) return MMAD_EUNSUPPORTED;
  const int bn = q.Nd % 128 == 0 ? 128 : 64;
  S2G g{};
  g.Ds = q.Ds; g.Hs = q.Hs; g.Ws = q.Ws; g.Dd = q.Dd; g.Hd = q.Hd; g.Wd = q.Wd;
  g.Nd = q.Nd; g.Kpad = q.Kpad;
  g.nbz = q.Dd / TZ; g.nby = q.Hd / TY; g.nbx = q.Wd / TX;
  g.nbn = q.Nd / bn;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  const int64_t nblk = mmad_s2::tiles(q) * g.nbn;
  if (nblk >= (int64_t(1) << 31)) return MMAD_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  if (bn == 128) return launch<128>(g, nblk, src, wp, bias, dst, stats, st);
  return launch<64>(g, nblk, src, wp, bias, dst, stats, st);
}

bool dgrad_ok(const mmad_conv_desc* d) {
  if (s2_mode() <= 0 || d == nullptr) return false;
  if (d->sd != 2 || d->sh != 2 || d->sw != 2 || d->ci != 64 || d->co != 128) return false;
  if (d->kd != 3 || d->kh != 3 || d->kw != 3 || d->pd != 1 || d->ph != 1 || d->pw != 1) return false;
  if (d->dd != 1 || d->dh != 1 || d->dw != 1) return false;
  if (d->di != 2 * d->do_ || d->hi != 2 * d->ho || d->wi != 2 * d->wo) return false;
  if (d->do_ % TZ || d->ho % TY || d->wo % TX) return false;
  return (int64_t)d->di * d->hi * d->wi * 64 < (int64_t(1) << 31) &&
         (int64_t)d->n * (d->do_ / TZ) * (d->ho / TY) * (d->wo / TX) < (int64_t(1) << 31);
}

int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream) {
  if (!dgrad_ok(d)) return MMAD_EUNSUPPORTED;
  static const bool attr = hipFuncSetAttribute((const void*)s2dgrad_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               DLDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  S2D g{};
  g.Do = d->do_; g.Ho = d->ho; g.Wo = d->wo; g.Di = d->di; g.Hi = d->hi; g.Wi = d->wi;
  g.Kpad = 27 * 128;
  g.nbz = d->do_ / TZ; g.nby = d->ho / TY; g.nbx = d->wo / TX;
  const int64_t nblk = (int64_t)d->n * g.nbz * g.nby * g.nbx;
  hipLaunchKernelGGL(s2dgrad_kernel, dim3((unsigned)nblk), dim3(NTHR), DLDS, as_stream(stream), g,
                     (const u16*)dy, (const u16*)wpt, (u16*)dx);
  return launch_status();
}

}  // namespace mmad_s2
