// Input gradient of the 1x1x1 stride-1 convolutions (MedicalNet shortcut B downsample of
// layers 3 and 4, reached from pkg/models/mri_models/anat_cnn.py:29-31) as a plain MFMA GEMM
// over NDHWC rows, gfx950 bf16 with fp32 accumulation.  Internal to libmmad_hip.so.
//
//   dX[m][ci] = sum_co dY[m][co] * Wd[ci][co]      (Wd: the dgrad-packed weights [ci][co])
//
// Both operands are K-contiguous rows (K = co), the layout the MFMA fragments read, so the
// kernel is the implicit GEMM without its gather: a block owns 128 voxel rows and ALL ci
// columns (128 or 256), so every dY byte is read once; K streams through a 3-slot LDS ring
// in 64-deep chunks (128-byte rows, 16-byte slots XOR-swizzled by row & 7 on the source
// address so the LDS-DMA image stays lane-linear and the fragment reads are conflict-free),
// two chunks in flight; 8 waves = 2 (64 rows) x 4 (ci quarters); the tile leaves through LDS
// as 16-byte channel vectors.  The step has two such launches (layer4: 32768 x 256 x 512,
// layer3: 32768 x 128 x 256 at batch 8): bandwidth-bound on the dY read (M x K x 2 bytes).
// Replaces the hipBLASLt GEMM used before round 3 (Cijk_* kernels, 18.8 / 10.8 us).
//
// The same GEMM form serves the shortcut's forward (round 3): Y[m][co] = sum_ci X[m][ci] *
// W[co][ci] with the forward-packed weights [co][ci] as the B rows, N tiles of 256 columns
// in blockIdx.y, and the BN partial sums of the fp32 accumulators written per 128-row tile
// (the implicit GEMM ran this K = 128 / 256 GEMM latency-bound: 31.4 / 17.6 us).
#include <atomic>
#include <cstdlib>

#include "common.h"
#include "pointwise.h"

namespace {

constexpr int TM = 128;                   // voxel rows per block
constexpr int KS = 64;                    // K elements per stage (128-byte rows)
constexpr int RB = KS * 2;
constexpr int NST = 3;                    // ring slots: two stages in flight
constexpr int NTHR = 512;
constexpr int NW = NTHR / 64;

template <int BN>
struct PC {
  static constexpr int TN = BN / 64;                // 16-column MFMA tiles per wave
  static constexpr int A_BYTES = TM * RB;
  static constexpr int SLOT = (TM + BN) * RB;
  static constexpr int NQ = SLOT / 1024;            // 1 KiB DMA instructions per stage
  static constexpr int WI = NQ / NW;
  static_assert(NQ % NW == 0, "DMA split over the waves");
  static constexpr int CROW = BN * 2 + 16;
  static constexpr int EPI = TM * CROW;
  static constexpr int MAIN = NST * SLOT;
  static constexpr int LDS = MAIN > EPI + 2 * BN * 4 ? MAIN : EPI + 2 * BN * 4;
};

__device__ __forceinline__ int swz8(int row) { return row & 7; }

// stride-2 1x1x1 geometry (the layer2 shortcut): output grid Do x Ho x Wo, input Di x Hi x Wi
struct PwS2 {
  int Do, Ho, Wo, Di, Hi, Wi;
};
// the input voxel a stride-2 1x1x1 conv's output row m reads
__device__ __forceinline__ int64_t s2_src(const PwS2& q, int64_t m) {
  const int ox = (int)(m % q.Wo);
  int64_t t = m / q.Wo;
  const int oy = (int)(t % q.Ho);
  t /= q.Ho;
  const int oz = (int)(t % q.Do);
  const int64_t n = t / q.Do;
  return ((n * q.Di + 2 * oz) * q.Hi + 2 * oy) * q.Wi + 2 * ox;
}

// C[m][n0 + n] = sum_k A[m][k] * B[n0 + n][k]; ldc = the output row length (all N tiles);
// stats (forward): [m tile][2][ldc] sums of C and C^2 over the tile's 128 rows.
// MODE 1 (stride-2 forward): A row m is the input voxel s2_src(m).  MODE 2 (stride-2 input
// gradient): C row m is dX voxel s2_src(m), and the block also writes the zeros of the other
// 7 voxels of each 2x2x2 cell (inside the volume), so dX needs no separate fill.
template <int BN, int MODE = 0>
__global__ __launch_bounds__(NTHR) void pw_dgrad_kernel(int K, const u16* __restrict__ dy,
                                                        const u16* __restrict__ wd,
                                                        u16* __restrict__ dx, int ldc,
                                                        float* __restrict__ stats,
                                                        const float* __restrict__ bias,
                                                        PwS2 s2) {
  using C = PC<BN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t m0 = (int64_t)blockIdx.x * TM;
  const int n0 = (int)blockIdx.y * BN;
  wd += (int64_t)n0 * K;
  const int nstage = K / KS;

  // DMA instruction q = wave + NW h: rows 8q .. 8q + 7 of the stage image (A rows first,
  // then B rows); lane -> row 8q + (lane >> 3), 16-byte slot lane & 7 (source slot swizzled)
  const u16* srcp[C::WI];
  uint32_t lofs[C::WI];
#pragma unroll
  for (int h = 0; h < C::WI; ++h) {
    const int q = wave + NW * h;
    const int row = q * 8 + (lane >> 3);
    const int ch = (lane & 7) ^ swz8(row);
    const int64_t arow = MODE == 1 ? s2_src(s2, m0 + row) : m0 + row;
    srcp[h] = row < TM ? dy + arow * K + ch * 8 : wd + (int64_t)(row - TM) * K + ch * 8;
    lofs[h] = q * 1024;
  }
  auto issue = [&](int s) {
    char* slot = smem + (s % NST) * C::SLOT;
#pragma unroll
    for (int h = 0; h < C::WI; ++h)
      glds16_asm(srcp[h] + s * KS, lds_addr_of(slot + lofs[h]));
  };

  const int wm = wave & 1, wn = wave >> 1;          // 64 rows x BN/4 columns per wave
  const int lr = lane & 15, lk = lane >> 4;
  f32x4 acc[4][C::TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nstage > 1) issue(1);
  for (int s = 0; s < nstage; ++s) {
    if (s + 1 < nstage) wait_vm_lgkm0<C::WI>();       // this stage landed, the next in flight
    else wait_vm_lgkm0<0>();
    raw_barrier();
    if (s + 2 < nstage) issue(s + 2);
    const char* slot = smem + (s % NST) * C::SLOT;
#pragma unroll
    for (int kk = 0; kk < KS / 32; ++kk) {          // two 32-deep MFMA k steps per stage
      bf16x8 a[4], b[C::TN];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + lr;
        a[i] = *reinterpret_cast<const bf16x8*>(slot + row * RB + (((kk * 4 + lk) ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int row = wn * 16 * C::TN + j * 16 + lr;
        b[j] = *reinterpret_cast<const bf16x8*>(slot + C::A_BYTES + row * RB +
                                                (((kk * 4 + lk) ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();                                  // ring reused by the epilogue

  // acc[i][j][e]: row wm*64 + i*16 + lk*4 + e, column wn*16*TN + j*16 + lr
  if (bias != nullptr) {
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      const float bv = bias[n0 + wn * 16 * C::TN + j * 16 + lr];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] += f32x4{bv, bv, bv, bv};
    }
  }
  u16* ctile = reinterpret_cast<u16*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * 64 + i * 16 + lk * 4 + e;
        const int col = wn * 16 * C::TN + j * 16 + lr;
        ctile[row * (C::CROW / 2) + col] = f2bf(acc[i][j][e]);
      }
  if (stats != nullptr) {
    // per column: this wave's 64 rows (i, e, then the 4 lk groups by shuffles), then the two
    // row halves (wm) in fixed order through LDS past the C tile: deterministic
    float* red = reinterpret_cast<float*>(smem + C::EPI);
    float cs[C::TN], cq[C::TN];
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
      cs[j] = 0.f;
      cq[j] = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cs[j] += acc[i][j][e];
          cq[j] += acc[i][j][e] * acc[i][j][e];
        }
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm == 1 && lk == 0) {
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int col = wn * 16 * C::TN + j * 16 + lr;
        red[col] = cs[j];
        red[BN + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < C::TN; ++j) {
        const int col = wn * 16 * C::TN + j * 16 + lr;
        stats[((int64_t)blockIdx.x * 2) * ldc + n0 + col] = cs[j] + red[col];
        stats[((int64_t)blockIdx.x * 2 + 1) * ldc + n0 + col] = cq[j] + red[BN + col];
      }
    }
  } else {
    __syncthreads();
  }
  constexpr int CPR = BN / 8;                       // 16-byte vectors per row
#pragma unroll
  for (int hh = 0; hh < TM * CPR / NTHR; ++hh) {
    const int qd = tid + NTHR * hh;
    const int row = qd / CPR, c8 = qd % CPR;
    const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                    row * C::CROW + c8 * 16);
    if constexpr (MODE == 2) {
      const int64_t dv = s2_src(s2, m0 + row);
      const int64_t m = m0 + row;
      const int ox = (int)(m % s2.Wo), oy = (int)((m / s2.Wo) % s2.Ho),
                oz = (int)((m / ((int64_t)s2.Wo * s2.Ho)) % s2.Do);
#pragma unroll
      for (int cell = 0; cell < 8; ++cell) {
        const int a = cell >> 2, b = (cell >> 1) & 1, c = cell & 1;
        if (2 * oz + a < s2.Di && 2 * oy + b < s2.Hi && 2 * ox + c < s2.Wi) {
          const int64_t o = dv + ((int64_t)a * s2.Hi + b) * s2.Wi + c;
          *reinterpret_cast<u32x4*>(dx + o * ldc + n0 + c8 * 8) =
              cell == 0 ? v : u32x4{0u, 0u, 0u, 0u};
        }
      }
    } else {
      *reinterpret_cast<u32x4*>(dx + (m0 + row) * ldc + n0 + c8 * 8) = v;
    }
  }
}

bool pw_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PW_GEMM");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}

// ---- weight gradient (round 5) ------------------------------------------------------
//   dW[co][ci] = sum_m dY[m][co] * X[src(m)][ci]      (src(m) = m, or s2_src for stride 2)
// K = the voxels, split over blocks: block = 128 co x CIT ci over one K range of a split;
// fp32 partial slabs [split][co][ci] (the torch layout of a 1x1x1 dW), summed by the wide
// slab reduction (deferred or not: conv.hip).  Both operands are K-strided in memory (NDHWC
// rows), so each stage DMAs 32 voxel rows of dY (128 co = 256 B) and of X (CIT ci) into LDS
// lane-linearly, and the MFMA fragments are read with transposing ds_read_b64_tr_b16: lane
// 4q + p of a 16-lane group supplies row q (a voxel), 4 channels; lane i receives channel i
// of 4 voxels.  The 16-byte chunks are XOR-swizzled per row on the DMA's source address so
// that the 8 rows x 2 chunks a 32-lane half reads hit 64 distinct banks (pw_tsw256 /
// pw_tsw128: rows {0-3, 8-11} + 16 t map to distinct chunk pairs).  4 waves = 2 (64 co) x 2
// (CIT / 2 ci); 4-slot ring, three 32-voxel stages in flight, one barrier per stage; two
// blocks per CU.  The row-gather wgrad_kernel (conv.hip) ran these GEMMs at 20-30 GB/s per
// CU of operand traffic (its 8-split run took 97 us per 4096-voxel block).
constexpr int WG_KS = 32;                 // voxels per stage (one MFMA k step)
// ring slots: every stage but one in flight (WGC<...>::NS: 8, or 7 for the 3^3 form's
// 20 KiB stages), one block per CU (round 5: 4 slots at two blocks per CU left the 16-stage
// blocks latency-bound at ~1.2 us per stage, with twice the slabs)
constexpr int WG_NTHR = 256;

__device__ __forceinline__ int pw_tsw256(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }
__device__ __forceinline__ int pw_tsw128(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

// NTAP = 3 (MODE 2, round 5): the stride-2 3^3 conv of layer2.0.conv1 (64 -> 128, pad 1):
// dW[co][tap][ci] = sum_m dY[m][co] * X[2 o(m) + tap - 1][ci].  A block takes one (kz, ky)
// and the three kx taps, so each stage's dY rows feed three X images (one gathered row set
// per kx: input voxel 2o + k - 1 per dimension, a zero block outside the volume) and three
// accumulator sets; slabs [split][co][tap * Ci + ci] for the transposing reduction.  The
// row-gather wgrad_kernel ran it with 69 splits (61 MB of slabs) at 0.13 of peak.
template <int CIT, int NTAP = 1>
struct WGC {
  static constexpr int NS = NTAP == 3 ? 7 : 8;
  static constexpr int YROW = 256;                    // 128 co x 2 B
  static constexpr int XROW = CIT * 2;
  static constexpr int YIMG = WG_KS * YROW;           // 8 KiB
  static constexpr int XIMG = WG_KS * XROW;           // 8 / 4 KiB per tap
  static constexpr int SLOT = YIMG + NTAP * XIMG;
  static constexpr int LDS = NS * SLOT;               // 128 / 96 / 140 KiB
  static constexpr int NQ = SLOT / 1024;              // DMA instructions per stage
  static constexpr int WI = NQ / 4;                   // per wave
  static_assert(WI * 4 == NQ, "stage DMA split over 4 waves");
  static constexpr int TJ = CIT / 32;                 // 16-column ci tiles per wave: 4 / 2
  static constexpr int XQ = XIMG / 1024;              // DMA instructions per X image
};

// MODE 0: stride 1, X row = m; 1: stride 2 1^3, X row = s2_src(m); 2: stride 2 3^3 (NTAP 3);
// 4: MODE 2 on 16-wide output rows (layer2.0.conv1 at 128^3) with de-duplicated X rows: a
// stage is exactly two output rows, and the kx = 0 and kx = 2 taps read the same odd input
// columns shifted by one (x = 2 ox - 1 and 2 ox + 1), so the stage's X image holds the even
// columns once (32 rows, kx = 1) and the 17 odd columns x = -1, 1, .., 31 of each of the two
// rows once (34 rows, read by kx = 0 at row 17 r + ox and by kx = 2 at row 17 r + ox + 1):
// 66 gathered rows instead of 96.  Same voxel pairs in the same K order: dW bit-identical
template <int CIT, int MODE, int NTAP = 1>
__global__ __launch_bounds__(WG_NTHR, 1) void pw_wgrad_kernel(
    const u16* __restrict__ x, const u16* __restrict__ dy, float* __restrict__ out, int Ci,
    int Co, int kper, int ntiles, PwS2 s2, uint32_t xbytes, uint32_t ybytes, int mrows) {
  using C = WGC<CIT, NTAP>;
  static_assert((MODE != 2 && MODE != 4) || NTAP == 3, "the 3^3 forms take the three kx taps");
  static_assert(MODE != 4 || (CIT == 64 && C::XQ == 4), "MODE 4: 128-byte X rows");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: the tiles of one split (the same voxel rows) on one XCD
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tile = lin % ntiles, split = lin / ntiles;
  const int nci = Ci / CIT, nco = Co / 128;
  const int ci0 = (tile % nci) * CIT, co0 = ((tile / nci) % nco) * 128;
  constexpr bool T3 = MODE == 2 || MODE == 4;                  // the 3^3 forms
  const int kzy = T3 ? tile / (nci * nco) : 0;                 // (kz, ky) of the 3^3 form
  const int kz = kzy / 3, ky = kzy % 3;
  const int64_t m0 = (int64_t)split * kper;
  const int nstage = (int)(min((int64_t)kper, (int64_t)mrows - m0) / WG_KS);   // last: ragged

  // DMA instruction q (= wave + 4 h) of a stage: q < 8 the dY image (rows 4q .. 4q + 3),
  // else X image (q - 8) / XQ (256-B rows: 4 per instruction; 128-B rows: 8).  Operands
  // move by buffer_load ... lds with 32-bit byte offsets (an offset past the buffer reads
  // zeros: the 3^3 form's padding); each row's offset advances incrementally per stage --
  // dY / stride-1 X by a constant, the strided X rows as a mixed-radix (x, y, z, n) add of
  // the 32-voxel step with at most one carry per digit (no divisions in the loop)
  constexpr uint32_t OOB = 0x80000000u;
  // MODE 4 (xbytes <= 2^30): a lane without a column carries OOB_L, a stage row outside the
  // volume gets OOB_S as its scalar part; every sum stays below 2^32 and every sum with
  // either part is past the buffer
  constexpr uint32_t OOB_L = 0x80000000u, OOB_S = 0x40000000u;
  // MODE 4: the stage's first output row (wave-uniform), advanced two rows a stage
  int soy = 0, soz = 0, son = 0;
  if constexpr (MODE == 4) {
    const int64_t t1 = m0 / s2.Wo;
    soy = (int)(t1 % s2.Ho);
    soz = (int)((t1 / s2.Ho) % s2.Do);
    son = (int)(t1 / s2.Ho / s2.Do);
  }
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy, 0, (int)__builtin_amdgcn_readfirstlane((int)ybytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)x, 0, (int)__builtin_amdgcn_readfirstlane((int)xbytes), 0x00020000);
  // the 32-voxel step in the output grid's (x, y, z, n) digits (MODE 1 / 2)
  const int stx = WG_KS % s2.Wo, st1 = WG_KS / s2.Wo;
  const int sty = MODE ? st1 % s2.Ho : 0, st2 = MODE ? st1 / s2.Ho : 0;
  const int stz = MODE ? st2 % s2.Do : 0, stn = MODE ? st2 / s2.Do : 0;
  uint32_t off[C::WI], lofs[C::WI], cix[C::WI];
  int ox[C::WI], oy[C::WI], oz[C::WI], on[C::WI], tapx[C::WI];
  int ixc[C::WI];                                   // MODE 4: the lane's output row of the stage
  bool isx[C::WI];
#pragma unroll
  for (int h = 0; h < C::WI; ++h) {
    const int q = wave + 4 * h;
    lofs[h] = (uint32_t)(q * 1024);
    ixc[h] = -1;
    int row, ch;
    if (MODE == 4 && q >= 8) {
      // pieces 8..11: even columns (row k = 16 r + ox -> x = 2 ox); 12..16: odd columns
      // (row j = 17 r + u, u < 17 -> x = 2 u - 1; rows 34.. of piece 16 unused); 17..19 unused.
      // The lane keeps its column's byte offset (OOB_L when it has none) and its output row
      // r of the stage; the stage's (n, z, y) part is a wave-uniform scalar (see issue)
      const bool even = q < 12;
      row = even ? 8 * (q - 8) + (lane >> 3) : 8 * (q - 12) + (lane >> 3);
      ch = (lane & 7) ^ pw_tsw128(row);
      isx[h] = true;
      tapx[h] = 0;
      int ix = -1, r = 0;
      if (even) {
        r = row >> 4;
        ix = 2 * (row & 15);
      } else if (q < 17 && row < 34) {
        r = row / 17;
        ix = 2 * (row % 17) - 1;                    // -1: the padding column
      }
      ixc[h] = r;
      off[h] = (unsigned)ix < (unsigned)s2.Wi ? (uint32_t)(ix * Ci + ci0 + ch * 8) * 2u : OOB_L;
      cix[h] = 0;
      ox[h] = oy[h] = oz[h] = on[h] = 0;
      continue;
    }
    if (q < 8) {
      row = 4 * q + (lane >> 4);
      ch = (lane & 15) ^ pw_tsw256(row);
      isx[h] = false;
      tapx[h] = 0;
      off[h] = (uint32_t)((m0 + row) * Co + co0 + ch * 8) * 2u;
    } else {
      const int qx = (q - 8) % C::XQ;
      row = CIT == 128 ? 4 * qx + (lane >> 4) : 8 * qx + (lane >> 3);
      ch = CIT == 128 ? (lane & 15) ^ pw_tsw256(row) : (lane & 7) ^ pw_tsw128(row);
      isx[h] = true;
      tapx[h] = (q - 8) / C::XQ;                                 // kx of this image
      off[h] = (uint32_t)((m0 + row) * Ci + ci0 + ch * 8) * 2u;   // (MODE 0)
    }
    cix[h] = (uint32_t)(ci0 + ch * 8) * 2u;
    const int64_t m = m0 + row;
    ox[h] = (int)(m % s2.Wo);
    const int64_t t1 = m / s2.Wo;
    oy[h] = (int)(t1 % s2.Ho);
    oz[h] = (int)((t1 / s2.Ho) % s2.Do);
    on[h] = (int)(t1 / s2.Ho / s2.Do);
  }
  const uint32_t ystep = (uint32_t)(WG_KS * Co) * 2u, xstep = (uint32_t)(WG_KS * Ci) * 2u;
  const uint32_t smem_l = lds_addr_of(smem);
  auto issue = [&](int s) {
    const uint32_t slot = smem_l + (uint32_t)((s % C::NS) * C::SLOT);
    // MODE 4: the stage's two output rows' input-row byte offsets (or OOB_S), scalar
    uint32_t srow0 = 0, srow1 = 0;
    if constexpr (MODE == 4) {
      const int iz = 2 * soz + kz - 1, iy0 = 2 * soy + ky - 1;
      const bool vz = (unsigned)iz < (unsigned)s2.Di;
      const int base = ((son * s2.Di + iz) * s2.Hi + iy0) * s2.Wi * Ci * 2;
      srow0 = vz && (unsigned)iy0 < (unsigned)s2.Hi ? (uint32_t)base : OOB_S;
      srow1 = vz && (unsigned)(iy0 + 2) < (unsigned)s2.Hi
                  ? (uint32_t)(base + 2 * s2.Wi * Ci * 2) : OOB_S;
      soy += 2;                                      // two output rows a stage (Wo = 16)
      const int cy = soy >= s2.Ho;
      soy -= cy ? s2.Ho : 0;
      soz += cy;
      const int cz = soz >= s2.Do;
      soz -= cz ? s2.Do : 0;
      son += cz;
    }
#pragma unroll
    for (int h = 0; h < C::WI; ++h) {
      if (!isx[h]) {
        buf_lds16_asm(off[h], rsy, slot + lofs[h]);
        off[h] += ystep;
      } else if (MODE == 0) {
        buf_lds16_asm(off[h], rsx, slot + lofs[h]);
        off[h] += xstep;
      } else if (MODE == 4) {
        uint32_t vo = off[h] + (ixc[h] ? srow1 : srow0);
        asm volatile("" : "+v"(vo));                // (a lane offset: keep it in a VGPR)
        buf_lds16_asm(vo, rsx, __builtin_amdgcn_readfirstlane(slot + lofs[h]));
      } else {
        const int dz = MODE == 2 ? kz - 1 : 0, dyy = MODE == 2 ? ky - 1 : 0;
        const int dx = MODE == 2 ? tapx[h] - 1 : 0;
        const int iz = 2 * oz[h] + dz, iy = 2 * oy[h] + dyy, ix = 2 * ox[h] + dx;
        const bool ok = (unsigned)iz < (unsigned)s2.Di && (unsigned)iy < (unsigned)s2.Hi &&
                        (unsigned)ix < (unsigned)s2.Wi;
        const uint32_t v = (uint32_t)(((on[h] * s2.Di + iz) * s2.Hi + iy) * s2.Wi + ix);
        buf_lds16_asm(ok ? v * (uint32_t)Ci * 2u + cix[h] : OOB, rsx, slot + lofs[h]);
        ox[h] += stx;
        const int cx = ox[h] >= s2.Wo;
        ox[h] -= cx ? s2.Wo : 0;
        oy[h] += sty + cx;
        const int cy = oy[h] >= s2.Ho;
        oy[h] -= cy ? s2.Ho : 0;
        oz[h] += stz + cy;
        const int cz = oz[h] >= s2.Do;
        oz[h] -= cz ? s2.Do : 0;
        on[h] += stn + cz;
      }
    }
  };

  const int wm = wave & 1, wn = wave >> 1;
  const int lk = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  // fragment byte offsets inside a slot: lo = voxel rows 8 lk + q4, hi = + 4
  uint32_t ya_lo[4], ya_hi[4], xb_lo[C::TJ], xb_hi[C::TJ];
  const int rlo = 8 * lk + q4, rhi = rlo + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = wm * 64 + i * 16 + 4 * p4;
    ya_lo[i] = (uint32_t)(rlo * C::YROW + (((col >> 3) ^ pw_tsw256(rlo)) << 4) + (col & 7) * 2);
    ya_hi[i] = (uint32_t)(rhi * C::YROW + (((col >> 3) ^ pw_tsw256(rhi)) << 4) + (col & 7) * 2);
  }
#pragma unroll
  for (int j = 0; j < C::TJ; ++j) {
    const int col = wn * (CIT / 2) + j * 16 + 4 * p4;
    const int slo = CIT == 128 ? pw_tsw256(rlo) : pw_tsw128(rlo);
    const int shi = CIT == 128 ? pw_tsw256(rhi) : pw_tsw128(rhi);
    xb_lo[j] = (uint32_t)(C::YIMG + rlo * C::XROW + (((col >> 3) ^ slo) << 4) + (col & 7) * 2);
    xb_hi[j] = (uint32_t)(C::YIMG + rhi * C::XROW + (((col >> 3) ^ shi) << 4) + (col & 7) * 2);
  }
  // MODE 4: per tap, the X rows of this lane's K rows rlo / rhi (k = 16 r + ox): kx = 1 the
  // even image's row k, kx = 0 / 2 the odd image's row 17 r + ox / + 1
  uint32_t xm_lo[3][C::TJ], xm_hi[3][C::TJ];
  if constexpr (MODE == 4) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int j = 0; j < C::TJ; ++j) {
        const int col = wn * (CIT / 2) + j * 16 + 4 * p4;
        auto at = [&](int k) {
          const int r = t == 1 ? k : 17 * (k >> 4) + (k & 15) + (t == 2 ? 1 : 0);
          const int img = C::YIMG + (t == 1 ? 0 : C::XIMG);
          return (uint32_t)(img + r * C::XROW + (((col >> 3) ^ pw_tsw128(r)) << 4) + (col & 7) * 2);
        };
        xm_lo[t][j] = at(rlo);
        xm_hi[t][j] = at(rhi);
      }
  }
  auto tr8 = [](const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)p);
  };
  f32x4 acc[NTAP][4][C::TJ];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::TJ; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int PD = C::NS - 1;                        // stages in flight
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < nstage) issue(p);
  for (int s = 0; s < nstage; ++s) {
    // stage s landed; the younger stages already issued stay in flight
    const int younger = min(PD - 1, nstage - 1 - s);
    [&]<int... Y>(std::integer_sequence<int, Y...>) {
      ((younger == Y ? wait_vm_lgkm0<Y * C::WI>() : void()), ...);
    }(std::make_integer_sequence<int, PD>{});
    raw_barrier();                                     // every wave's part of stage s; and
    if (s + PD < nstage) issue(s + PD);                // all are past stage s - 1's slot
    int so = (s % C::NS) * C::SLOT;
    asm volatile("" : "+s"(so));
    const char* slot = smem + so;
    bf16x8 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = __builtin_shufflevector(tr8(slot + ya_lo[i]), tr8(slot + ya_hi[i]), 0, 1, 2, 3, 4,
                                     5, 6, 7);
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      bf16x8 b[C::TJ];
#pragma unroll
      for (int j = 0; j < C::TJ; ++j) {
        if constexpr (MODE == 4)
          b[j] = __builtin_shufflevector(tr8(slot + xm_lo[t][j]), tr8(slot + xm_hi[t][j]), 0, 1,
                                         2, 3, 4, 5, 6, 7);
        else
          b[j] = __builtin_shufflevector(tr8(slot + t * C::XIMG + xb_lo[j]),
                                         tr8(slot + t * C::XIMG + xb_hi[j]), 0, 1, 2, 3, 4, 5, 6,
                                         7);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < C::TJ; ++j)
          acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[t][i][j], 0, 0, 0);
    }
  }

  // acc[t][i][j][r]: co = wm*64 + i*16 + 4 lk + r, ci = wn*CIT/2 + j*16 + (lane & 15);
  // slab column tap * Ci + ci (taps = 27 for the 3^3 form, tap = (kz*3 + ky)*3 + kx)
  const int K = T3 ? 27 * Ci : Ci;
  float* o = out + (int64_t)split * Co * K;
  const int lr = lane & 15;
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wm * 64 + i * 16 + 4 * lk + r;
          const int ci = ci0 + wn * (CIT / 2) + j * 16 + lr;
          const int col = T3 ? (kzy * 3 + t) * Ci + ci : ci;
          o[(int64_t)co * K + col] = acc[t][i][j][r];
        }
}

// MMAD_PW_WG3_DEDUP=0 keeps the three gathered X images per stage for 16-wide rows (A/B);
// mmad_set_kernel_variant("pw_wg3_dedup", v) overrides it at run time
std::atomic<int> g_wg3_dedup{-1};
bool wg3_dedup() {
  int v = g_wg3_dedup.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_PW_WG3_DEDUP");
    int expect = -1;
    g_wg3_dedup.compare_exchange_strong(expect, e == nullptr || atoi(e) != 0 ? 1 : 0);
    v = g_wg3_dedup.load(std::memory_order_relaxed);
  }
  return v != 0;
}

bool pw_wgrad_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PW_WGRAD");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}

}  // namespace

namespace mmad_pw {

namespace {
bool s2_geom(const mmad_conv_desc* d) {
  return d->sd == 2 && d->sh == 2 && d->sw == 2 &&
         (d->di == 2 * d->do_ || d->di == 2 * d->do_ - 1) &&
         (d->hi == 2 * d->ho || d->hi == 2 * d->ho - 1) &&
         (d->wi == 2 * d->wo || d->wi == 2 * d->wo - 1);
}
bool stride1_geom(const mmad_conv_desc* d) {
  return d->sd == 1 && d->sh == 1 && d->sw == 1 && d->di == d->do_ && d->hi == d->ho &&
         d->wi == d->wo;
}
PwS2 s2_of(const mmad_conv_desc* d) {
  return PwS2{d->do_, d->ho, d->wo, d->di, d->hi, d->wi};
}
template <int BN, int MODE>
int launch(dim3 grid, int K, const void* a, const void* b, void* c, int ldc, float* stats,
           const float* bias, PwS2 q, void* stream) {
  static const bool attr = hipFuncSetAttribute((const void*)pw_dgrad_kernel<BN, MODE>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               PC<BN>::LDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  hipLaunchKernelGGL((pw_dgrad_kernel<BN, MODE>), grid, dim3(NTHR), PC<BN>::LDS,
                     as_stream(stream), K, (const u16*)a, (const u16*)b, (u16*)c, ldc, stats, bias,
                     q);
  return launch_status();
}
}  // namespace

bool ok(const mmad_conv_desc* d, int dtype) {
  if (!pw_on() || dtype != MMAD_BF16) return false;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw) return false;
  if (!stride1_geom(d) && !s2_geom(d)) return false;
  if (d->co % KS || (d->ci != 64 && d->ci != 128 && d->ci != 256)) return false;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;       // dY rows
  const int64_t mi = (int64_t)d->n * d->di * d->hi * d->wi;
  return m % TM == 0 && mi * d->ci < (int64_t(1) << 40) && m * d->co < (int64_t(1) << 40);
}

int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream) {
  if (!ok(d, MMAD_BF16)) return MMAD_EUNSUPPORTED;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const dim3 grid((unsigned)(m / TM));
  const PwS2 q = s2_of(d);
  if (s2_geom(d)) {
    if (d->ci == 256) return launch<256, 2>(grid, d->co, dy, wpt, dx, 256, nullptr, nullptr, q, stream);
    if (d->ci == 128) return launch<128, 2>(grid, d->co, dy, wpt, dx, 128, nullptr, nullptr, q, stream);
    return launch<64, 2>(grid, d->co, dy, wpt, dx, 64, nullptr, nullptr, q, stream);
  }
  if (d->ci == 256) return launch<256, 0>(grid, d->co, dy, wpt, dx, 256, nullptr, nullptr, q, stream);
  if (d->ci == 128) return launch<128, 0>(grid, d->co, dy, wpt, dx, 128, nullptr, nullptr, q, stream);
  return launch<64, 0>(grid, d->co, dy, wpt, dx, 64, nullptr, nullptr, q, stream);
}

bool fwd_ok(const mmad_conv_desc* d, int dtype) {
  if (!pw_on() || dtype != MMAD_BF16) return false;
  if (d->kd != 1 || d->kh != 1 || d->kw != 1 || d->pd || d->ph || d->pw) return false;
  if (!stride1_geom(d) && !s2_geom(d)) return false;
  if (d->ci % KS || (d->co % 256 && d->co != 128)) return false;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const int64_t mi = (int64_t)d->n * d->di * d->hi * d->wi;
  return m % TM == 0 && m / TM < (int64_t(1) << 31) && m * d->co < (int64_t(1) << 40) &&
         mi * d->ci < (int64_t(1) << 40);
}

int64_t fwd_tiles(const mmad_conv_desc* d) {
  return (int64_t)d->n * d->do_ * d->ho * d->wo / TM;
}

int fwd(const mmad_conv_desc* d, const void* x, const void* wp, const float* bias, void* y,
        float* stats, void* stream) {
  if (!fwd_ok(d, MMAD_BF16)) return MMAD_EUNSUPPORTED;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const PwS2 q = s2_of(d);
  const bool s2 = s2_geom(d);
  if (d->co == 128) {
    const dim3 grid((unsigned)(m / TM), 1);
    return s2 ? launch<128, 1>(grid, d->ci, x, wp, y, 128, stats, bias, q, stream)
              : launch<128, 0>(grid, d->ci, x, wp, y, 128, stats, bias, q, stream);
  }
  const dim3 grid((unsigned)(m / TM), (unsigned)(d->co / 256));
  return s2 ? launch<256, 1>(grid, d->ci, x, wp, y, d->co, stats, bias, q, stream)
            : launch<256, 0>(grid, d->ci, x, wp, y, d->co, stats, bias, q, stream);
}

namespace {
int wg_cit(const mmad_conv_desc* d) { return d->ci % 128 == 0 && d->ci >= 256 ? 128 : 64; }
// the 3^3 stride-2 form (layer2.0.conv1): pad 1, dilation 1, the s2 grid relation
bool wg3_geom(const mmad_conv_desc* d) {
  return d->kd == 3 && d->kh == 3 && d->kw == 3 && d->pd == 1 && d->ph == 1 && d->pw == 1 &&
         d->dd == 1 && d->dh == 1 && d->dw == 1 && s2_geom(d);
}
int64_t wg_tiles(const mmad_conv_desc* d) {
  const int64_t t = (int64_t)(d->co / 128) * (d->ci / (wg3_geom(d) ? 64 : wg_cit(d)));
  return wg3_geom(d) ? 9 * t : t;
}
}  // namespace

int set_wg3_dedup(int v) {
  const int prev = wg3_dedup() ? 1 : 0;
  if (v >= 0) g_wg3_dedup.store(v ? 1 : 0, std::memory_order_relaxed);
  return prev;
}

bool wgrad_ok(const mmad_conv_desc* d, int dtype) {
  if (!pw_on() || !pw_wgrad_on() || dtype != MMAD_BF16) return false;
  const bool one = d->kd == 1 && d->kh == 1 && d->kw == 1 && !d->pd && !d->ph && !d->pw &&
                   (stride1_geom(d) || s2_geom(d));
  if (!one && !wg3_geom(d)) return false;
  if (d->co % 128 || d->ci % 64) return false;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const int64_t mi = (int64_t)d->n * d->di * d->hi * d->wi;
  // (32-bit byte offsets, bit 31 marking padding)
  return m % WG_KS == 0 && m * d->co * 2 < (int64_t(1) << 31) &&
         mi * d->ci * 2 < (int64_t(1) << 31);
}

// voxels per split: as many splits as give every CU one block (256 / tiles), each a whole
// number of 32-voxel stages (the last split takes the remainder)
int64_t wgrad_kper(const mmad_conv_desc* d) {
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const int64_t want = std::max<int64_t>(1, 256 / wg_tiles(d));
  return std::max<int64_t>(WG_KS, cdiv(cdiv(m, want), WG_KS) * WG_KS);
}

int64_t wgrad_splits(const mmad_conv_desc* d) {
  return cdiv((int64_t)d->n * d->do_ * d->ho * d->wo, wgrad_kper(d));
}

int wgrad(const mmad_conv_desc* d, const void* x, const void* dy, float* ws, void* stream) {
  if (!wgrad_ok(d, MMAD_BF16)) return MMAD_EUNSUPPORTED;
  const int64_t kper = wgrad_kper(d), sp = wgrad_splits(d);
  const int64_t ntiles = wg_tiles(d);
  const int64_t nblk = sp * ntiles;
  const int64_t m = (int64_t)d->n * d->do_ * d->ho * d->wo;
  const int64_t mi = (int64_t)d->n * d->di * d->hi * d->wi;
  // 32-bit byte offsets (bit 31 marks padding)
  if (nblk > 0x7fffffff || m * d->co * 2 >= (int64_t(1) << 31) ||
      mi * d->ci * 2 >= (int64_t(1) << 31))
    return MMAD_EUNSUPPORTED;
  const PwS2 q = s2_of(d);
  auto go = [&](auto kern, int lds) {
    static_cast<void>(hipFuncSetAttribute((const void*)kern,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(WG_NTHR), lds, as_stream(stream),
                       (const u16*)x, (const u16*)dy, ws, d->ci, d->co, (int)kper, (int)ntiles,
                       q, (uint32_t)(mi * d->ci * 2), (uint32_t)(m * d->co * 2), (int)m);
    return launch_status();
  };
  if (wg3_geom(d)) {
    // 16-wide output rows (and an even row count): every 32-voxel stage is two whole rows
    if (d->wo == 16 && d->ho % 2 == 0 && kper % 32 == 0 && mi * d->ci * 2 <= (int64_t(1) << 30) &&
        wg3_dedup())
      return go(pw_wgrad_kernel<64, 4, 3>, WGC<64, 3>::LDS);
    return go(pw_wgrad_kernel<64, 2, 3>, WGC<64, 3>::LDS);
  }
  const bool s2 = s2_geom(d);
  if (wg_cit(d) == 128)
    return s2 ? go(pw_wgrad_kernel<128, 1>, WGC<128>::LDS) : go(pw_wgrad_kernel<128, 0>, WGC<128>::LDS);
  return s2 ? go(pw_wgrad_kernel<64, 1>, WGC<64>::LDS) : go(pw_wgrad_kernel<64, 0>, WGC<64>::LDS);
}

}  // namespace mmad_pw
