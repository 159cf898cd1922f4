// Residue-class conv on 5d^3 grids: config 5's layer4 (dilation-4 3x3x3 convs, padding 4,
// 256 / 512 channels on the 20^3 grids a 160^3 input reaches; pet_resnet_cnn.py:12-138 and
// anat_cnn.py:29-31 via MedicalNet) forward and -- as a forward over reversed taps -- input
// gradient, gfx950 bf16 with fp32 accumulation.  Same operands as latticeconv.hip (NDHWC
// volumes, packed weights [Nd][27 * Cs] with k = tap * Cs + ci, BN partial sums one row per
// tile); what differs is the sub-lattice extent, 5 instead of 4:
//  * voxel (rz + d tz, ry + d ty, rx + d tx) only meets voxels of its own residue class, so
//    the conv is d^3 dense 3^3 convs (padding 1) over 5^3 sub-lattices; taps that leave the
//    sub-lattice land in the zero padding and are skipped outright (35 % of the dense MACs
//    at d = 4, which the row-gather implicit GEMM executes as zeros);
//  * a tile is one z-plane tz of 16 subs (sample x class): 25 positions x 16 subs = 400 GEMM
//    rows, position-major, so an MFMA fragment (16 rows) is the 16 subs at ONE position and
//    whether a tap is padding is the same for the whole fragment (a compile-time fact: wave,
//    tap and fragment are template constants in the stage body);
//  * 8 waves = 4 position groups x 2 channel halves (64 output channels, 4 MFMA columns);
//    the position groups (6, 6, 7, 6 positions) are chosen so that the two waves sharing a
//    SIMD (w and w + 4: groups 0 + 2, 1 + 3) carry exactly half of every tap's fragments --
//    85 of the 169 (position, ky, kx) pairs each, per stage as well as in total;
//  * A never goes through a per-tap gather: the input planes tz - 1 .. tz + 1 of the 16 subs
//    (32 input channels at a time, 25 KiB each) sit in LDS and each tap reads its fragments
//    at a shifted position; planes outside the sub-lattice (kz at tz = 0 or 4) are neither
//    loaded nor visited;
//  * a stage = (channel chunk, kz, ky): the three kx taps' weights (3 x 128 rows x 64 B)
//    through a 3-slot ring, two stages in flight; input planes through a 3-slot ring, each
//    issued six stages ahead of its first reader;
//  * edge planes (tz = 0, 4) carry 2/3 of the work of interior ones: one block runs tz = 0
//    and then tz = 4, the others one interior plane each, the pair blocks dispatched first
//    on every XCD (each XCD holds whole sub groups, so their input planes share one L2).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <utility>

#include "common.h"
#include "patchconv.h"

namespace {

constexpr int S = 5;                      // sub-lattice extent
constexpr int NP = S * S;                 // positions per plane
constexpr int NS = 16;                    // subs per tile
constexpr int PR = NP * NS;               // rows per plane: 400
constexpr int RBL = 64;                   // bytes per LDS row: 32 bf16 channels
constexpr int KC = RBL / 2;
constexpr int PLB = PR * RBL;             // 25 KiB per plane
constexpr int NPS = 3;                    // plane ring slots
constexpr int TPS = 3;                    // taps per stage
constexpr int TN = 4;                     // 16-column MFMA tiles per wave
constexpr int BW = 32 * TN;               // output channels per tile: 128
constexpr int BTAP = BW * RBL;
constexpr int BSLOT = TPS * BTAP;         // 24 KiB
constexpr int NSTL = 3;                   // weight ring slots
constexpr int RING_OFF = NPS * PLB;
constexpr int MAIN = RING_OFF + NSTL * BSLOT;
constexpr int CROW = BW * 2 + 16;
constexpr int EPI = PR * CROW + 3 * 2 * BW * 4;
constexpr int LDS = MAIN > EPI ? MAIN : EPI;
constexpr int NTHR = 512;
constexpr int NW = NTHR / 64;
constexpr int NQ = TPS * BW / 16;         // weight DMA instructions per stage: 24
constexpr int WI = NQ / NW;               // ... per wave: 3
constexpr int PI = (NP + NW - 1) / NW;    // plane DMA instructions per wave: 4
constexpr int NF = 7;                     // A fragments (positions) per wave, at most
static_assert(NQ % NW == 0, "weight DMAs split evenly over the waves");
static_assert(LDS <= 160 * 1024, "LDS");

struct G5 {
  int Cs, Nd, Kpad, nchunk, nbn;
  int d, E, G;                            // dilation, grid extent 5d, sub groups per sample
  int ngroups;                            // nb * G
  int xcd;                                // blocks walk the XCDs in whole sub groups
  const u16* res;
  int relu;
};

__device__ __forceinline__ int swz(int row) { return 3 * ((row >> 3) & 1); }

// position (y * 5 + x) of fragment F of position group WM; -1: none.  Found by exhaustive
// search: SIMD {0, 2} and SIMD {1, 3} hold 85 / 84 of the 169 valid (position, ky, kx) pairs,
// split evenly inside every ky stage
__host__ __device__ constexpr int pos_tab(int wm, int f) {
  constexpr int t[4][NF] = {{7, 9, 12, 18, 20, 21, -1},
                            {6, 11, 14, 15, 16, 23, -1},
                            {0, 2, 4, 8, 10, 17, 24},
                            {1, 3, 5, 13, 19, 22, -1}};
  return t[wm][f];
}
template <int WM, int KY, int KX, int F>
__device__ constexpr bool frag_ok() {
  constexpr int p = pos_tab(WM, F);
  if (p < 0) return false;
  constexpr int y = p / S + KY, x = p % S + KX;
  return y >= 0 && y < S && x >= 0 && x < S;
}
template <int WM, int KY, int KX, int F>
__device__ constexpr int frag_src() {
  constexpr int p = pos_tab(WM, F);
  return (p / S + KY) * S + p % S + KX;
}

template <int KX>
__device__ __forceinline__ void read_b(const char* bsl, bf16x8 (&b)[TN]) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
    b[j] = *reinterpret_cast<const bf16x8*>(bsl + (KX + 1) * BTAP + j * 16 * RBL);
}
template <int WM, int KY, int KX, int F>
__device__ __forceinline__ void read_a(const char* pl, bf16x8 (&a)[NF]) {
  if constexpr (frag_ok<WM, KY, KX, F>())
    a[F] = *reinterpret_cast<const bf16x8*>(pl + frag_src<WM, KY, KX, F>() * 16 * RBL);
}
template <int WM, int KY, int KX, int F>
__device__ __forceinline__ void mma_a(f32x4 (&acc)[NF][TN], const bf16x8 (&a)[NF],
                                      const bf16x8 (&b)[TN]) {
  if constexpr (frag_ok<WM, KY, KX, F>()) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      acc[F][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[F], b[j], acc[F][j], 0, 0, 0);
  }
}

// one stage (ky; kx = -1, 0, 1) with rolling registers: each A fragment register is refilled
// for the next tap right after the current tap's MFMAs have read it; a scheduling barrier
// after each (MFMAs, refill) pair keeps the compiler from hoisting refills (more live
// fragment registers, spills)
#define PIN() __builtin_amdgcn_sched_barrier(0)
template <int WM, int KY>
__device__ __forceinline__ void stage_body(f32x4 (&acc)[NF][TN], const char* bsl,
                                           const char* pl) {
  bf16x8 a[NF], b0[TN], b1[TN];
  read_b<-1>(bsl, b0);
  [&]<int... F>(std::integer_sequence<int, F...>) {
    (read_a<WM, KY, -1, F>(pl, a), ...);
  }(std::make_integer_sequence<int, NF>{});
  read_b<0>(bsl, b1);
  [&]<int... F>(std::integer_sequence<int, F...>) {
    ((mma_a<WM, KY, -1, F>(acc, a, b0), read_a<WM, KY, 0, F>(pl, a), PIN()), ...);
  }(std::make_integer_sequence<int, NF>{});
  read_b<1>(bsl, b0);
  [&]<int... F>(std::integer_sequence<int, F...>) {
    ((mma_a<WM, KY, 0, F>(acc, a, b1), read_a<WM, KY, 1, F>(pl, a), PIN()), ...);
  }(std::make_integer_sequence<int, NF>{});
  [&]<int... F>(std::integer_sequence<int, F...>) {
    (mma_a<WM, KY, 1, F>(acc, a, b0), ...);
  }(std::make_integer_sequence<int, NF>{});
}

// vmcnt wait for the counts a stage can see (0, WI, PI, WI + PI); lgkm drained too
__device__ __forceinline__ void wait_ops(int n) {
  if (n == WI + PI) wait_vm_lgkm0<WI + PI>();
  else if (n == PI) wait_vm_lgkm0<PI>();
  else if (n == WI) wait_vm_lgkm0<WI>();
  else wait_vm_lgkm0<0>();
}

__global__ __launch_bounds__(NTHR) void lattice5_conv_kernel(
    G5 g, const u16* __restrict__ src, const u16* __restrict__ wgt,
    const float* __restrict__ bias, u16* __restrict__ dst, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + RING_OFF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x;
  // unit (z block zb, sub group, channel tile): zb 0 = planes 0 and 4, zb 1..3 = plane zb
  int zb, grp, nt;
  {
    const int per = g.ngroups * g.nbn;
    if (g.xcd) {
      // XCD x takes sub groups [x gpx, (x + 1) gpx); on each XCD the pair blocks go first
      const int gpx = g.ngroups >> 3, xcd = bid & 7, li = bid >> 3;
      const int pz = gpx * g.nbn;
      zb = li / pz;
      const int rem = li % pz;
      grp = xcd * gpx + rem / g.nbn;
      nt = rem % g.nbn;
    } else {
      zb = bid / per;
      const int rem = bid % per;
      grp = rem / g.nbn;
      nt = rem % g.nbn;
    }
  }
  const int n = grp / g.G, gl = grp % g.G;
  const int d = g.d, E = g.E;
  const int n0 = nt * BW;
  const int64_t vol = (int64_t)E * E * E;
  // both operands through buffer resources with 32-bit byte offsets (a scalar plane / stage
  // part + a constant lane part; no 64-bit lane addresses, no generic-pointer casts per DMA)
  const __amdgpu_buffer_rsrc_t rss = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(src + (int64_t)n * vol * g.Cs), 0,
      (int)__builtin_amdgcn_readfirstlane((uint32_t)(vol * g.Cs * 2)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wgt, 0, (int)__builtin_amdgcn_readfirstlane((uint32_t)g.Nd * g.Kpad * 2),
      0x00020000);
  const uint32_t lds0 = lds_addr_of(smem);

  // ---- plane DMA: instruction k of wave w = position w + 8k (clamped: surplus slots repeat
  // the last position, the same bytes to the same place, so every wave issues PI); lane >> 2
  // = sub, lane & 3 = 16-byte chunk (swizzled)
  uint32_t pofs[PI];
  {
    const int s = lane >> 2;
    const int c = gl * NS + s;                      // class of sub s
    const int rz = c / (d * d), ry = (c / d) % d, rx = c % d;
#pragma unroll
    for (int k = 0; k < PI; ++k) {
      const int pos = min(wave + NW * k, NP - 1), ty = pos / S, tx = pos % S;
      const int row = pos * NS + s;
      const int vox = (rz * E + ry + d * ty) * E + rx + d * tx;
      pofs[k] = (uint32_t)(vox * g.Cs + ((lane & 3) ^ swz(row)) * 8) * 2u;
    }
  }
  // ---- weight DMA: instruction q = wave + NW h: tap q / 8, rows 16 (q % 8) ..
  uint32_t wofs[WI];
#pragma unroll
  for (int h = 0; h < WI; ++h) {
    const int q = wave + NW * h;
    const int tk = q / (BW / 16), rb = q % (BW / 16);
    const int row = rb * 16 + (lane >> 2);
    wofs[h] = (uint32_t)((n0 + row) * g.Kpad + (((lane & 3) ^ swz(row)) * 8) + tk * g.Cs) * 2u;
  }
  const uint32_t zstep = (uint32_t)(d * E * E * g.Cs * 2);   // bytes from plane tz to tz + 1

  const int wn = wave & 1, wm = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  const uint32_t a_lane = lr * RBL + ((lk ^ swz(lr)) << 4);
  const uint32_t b_lane = (wn * 16 * TN + lr) * RBL + ((lk ^ swz(lr)) << 4);
  const u16* ctile = reinterpret_cast<const u16*>(smem);
  float* red = reinterpret_cast<float*>(smem + PR * CROW);

  const int nrep = zb == 0 ? 2 : 1;
  for (int rep = 0; rep < nrep; ++rep) {
    const int tz = zb == 0 ? 4 * rep : zb;
    const int kz0 = tz == 0 ? 0 : -1;               // first kz inside the sub-lattice
    const int nz = (tz == 0 || tz == S - 1) ? 2 : 3;
    const int nplanes = g.nchunk * nz;
    // plane i = (chunk c, kz index kzi) -> ring slot i % 3; stage (i, ky) reads plane i and
    // the weights of taps 9 (kz + 1) + 3 (ky + 1) .. + 2 from weight slot ky + 1 (a plane's
    // three stages use the three slots in order, so the slot is a compile-time constant)
    auto issue_plane = [&](int c, int kzi, int slot) {
      const uint32_t zoff = (uint32_t)(tz + kz0 + kzi) * zstep + (uint32_t)(c * KC * 2);
      const uint32_t pb = lds0 + (uint32_t)(slot * PLB);
#pragma unroll
      for (int k = 0; k < PI; ++k) {
        const int pos = min(wave + NW * k, NP - 1);
        buf_lds16_asm(pofs[k] + zoff, rss, pb + (uint32_t)(pos * 1024));
      }
    };
    auto issue_w = [&](int c, int kzi, auto kyc) {
      constexpr int KY = decltype(kyc)::value;
      const uint32_t toff =
          (uint32_t)(((9 * (kz0 + kzi + 1) + 3 * (KY + 1)) * g.Cs + c * KC) * 2);
      constexpr uint32_t sb = (uint32_t)(RING_OFF + (KY + 1) * BSLOT);
#pragma unroll
      for (int h = 0; h < WI; ++h) {
        const int q = wave + NW * h;
        const uint32_t dst = (uint32_t)((q / (BW / 16)) * BTAP + (q % (BW / 16)) * 1024);
        buf_lds16_asm(wofs[h] + toff, rsw, lds0 + sb + dst);
      }
    };

    f32x4 acc[NF][TN];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: planes 0, 1 and the weights of plane 0's stages ky = -1, 0.  After stage
    // (i, ky)'s barrier: ky = -1 issues plane i + 2 (slot of plane i - 1, last read at stage
    // (i - 1, +1)) and the weights of (i, +1) (slot 2, last read at (i - 1, +1)); ky = 0 the
    // weights of (i + 1, -1) (slot 0); ky = +1 those of (i + 1, 0) (slot 1).  Each stage waits
    // for its weights; younger than them is the previous stage's group only.
    issue_plane(0, 0, 0);
    issue_plane(nz > 1 ? 0 : 1, nz > 1 ? 1 : 0, 1);
    issue_w(0, 0, std::integral_constant<int, -1>{});
    issue_w(0, 0, std::integral_constant<int, 0>{});
    auto run = [&](auto wmc) {
      constexpr int WM = decltype(wmc)::value;
      int c = 0, kzi = 0, ps = 0;                   // plane i = (c, kzi) in slot ps
      for (int i = 0; i < nplanes; ++i) {
        // planes i + 1 and i + 2
        const bool w1 = kzi + 1 == nz;
        const int c1 = w1 ? c + 1 : c, k1 = w1 ? 0 : kzi + 1;
        const bool w2 = k1 + 1 == nz;
        const int c2 = w2 ? c1 + 1 : c1, k2 = w2 ? 0 : k1 + 1;
        const int ps2 = ps == 0 ? 2 : ps - 1;       // (i + 2) % 3
        const bool more1 = i + 1 < nplanes, more2 = i + 2 < nplanes;
        const char* pl = smem + ps * PLB + a_lane;
        auto stage = [&](auto kyc) {
          constexpr int KY = decltype(kyc)::value;
          if constexpr (KY == -1) {
            wait_vm_lgkm0<WI>();
          } else if constexpr (KY == 0) {
            if (more2) wait_vm_lgkm0<WI + PI>();
            else wait_vm_lgkm0<WI>();
          } else {
            if (more1) wait_vm_lgkm0<WI>();
            else wait_vm_lgkm0<0>();
          }
          raw_barrier();
          if constexpr (KY == -1) {
            if (more2) issue_plane(c2, k2, ps2);
            issue_w(c, kzi, std::integral_constant<int, 1>{});
          } else if constexpr (KY == 0) {
            if (more1) issue_w(c1, k1, std::integral_constant<int, -1>{});
          } else {
            if (more1) issue_w(c1, k1, std::integral_constant<int, 0>{});
          }
          stage_body<WM, KY>(acc, smem + RING_OFF + (KY + 1) * BSLOT + b_lane, pl);
        };
        stage(std::integral_constant<int, -1>{});
        stage(std::integral_constant<int, 0>{});
        stage(std::integral_constant<int, 1>{});
        c = c1;
        kzi = k1;
        ps = ps == 2 ? 0 : ps + 1;
      }
    };
    switch (wm) {                                     // wave-uniform
      case 0: run(std::integral_constant<int, 0>{}); break;
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      default: run(std::integral_constant<int, 3>{}); break;
    }
    __syncthreads();                                  // planes / ring reused by the epilogue

    // ---- epilogue: acc[f][j][e] is row pos_tab(wm, f) * 16 + lk * 4 + e, column
    // wn * 64 + j * 16 + lr.  The LDS base is opaque so that none of the tile's addresses is
    // computed (and held live) ahead of the main loop
    float cs[TN], cq[TN];
    uint32_t eb = (uint32_t)(lk * 4 * CROW + (wn * 16 * TN + lr) * 2);
    asm volatile("" : "+v"(eb));
    auto epi = [&](auto wmc) {
      constexpr int WM = decltype(wmc)::value;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        cs[j] = 0.f;
        cq[j] = 0.f;
        const float bv = bias != nullptr ? bias[n0 + wn * 16 * TN + j * 16 + lr] : 0.f;
        [&]<int... F>(std::integer_sequence<int, F...>) {
          ([&] {
            constexpr int p = pos_tab(WM, F);
            if constexpr (p >= 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float v = acc[F][j][e] + bv;
                *reinterpret_cast<u16*>(smem + eb + (p * NS + e) * CROW + j * 32) = f2bf(v);
                cs[j] += v;
                cq[j] += v * v;
              }
            }
          }(), ...);
        }(std::make_integer_sequence<int, NF>{});
      }
    };
    switch (wm) {
      case 0: epi(std::integral_constant<int, 0>{}); break;
      case 1: epi(std::integral_constant<int, 1>{}); break;
      case 2: epi(std::integral_constant<int, 2>{}); break;
      default: epi(std::integral_constant<int, 3>{}); break;
    }
    __syncthreads();
    constexpr int CPR = BW / 8;
    for (int qd = tid; qd < PR * CPR; qd += NTHR) {
      const int row = qd / CPR, c8 = qd % CPR;
      const int p = row / NS, s = row % NS;
      const int c = gl * NS + s;
      const int rz = c / (d * d), ry = (c / d) % d, rx = c % d;
      const int vox = ((rz + d * tz) * E + ry + d * (p / S)) * E + rx + d * (p % S);
      const int64_t o = ((int64_t)n * vol + vox) * g.Nd + n0 + c8 * 8;
      u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                row * CROW + c8 * 16);
      if (g.res != nullptr || g.relu) v = epi_res_relu(v, g.res ? g.res + o : nullptr, g.relu);
      *reinterpret_cast<u32x4*>(dst + o) = v;
    }
    if (stats != nullptr) {
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
          const int col = wn * 16 * TN + j * 16 + lr;
          red[(wm - 1) * 2 * BW + col] = cs[j];
          red[(wm - 1) * 2 * BW + BW + col] = cq[j];
        }
      }
      __syncthreads();
      if (wm == 0 && lk == 0) {
        const int64_t mt = (int64_t)grp * S + tz;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * 16 * TN + j * 16 + lr;
          float ss = cs[j], qs = cq[j];
          for (int w = 1; w < 4; ++w) {               // fixed order: deterministic
            ss += red[(w - 1) * 2 * BW + col];
            qs += red[(w - 1) * 2 * BW + BW + col];
          }
          stats[(mt * 2) * g.Nd + n0 + col] = ss;
          stats[(mt * 2 + 1) * g.Nd + n0 + col] = qs;
        }
      }
    }
    __syncthreads();                                  // the next plane's DMA reuses the LDS
  }
}

// ---- weight gradient on the 5^3 sub-lattices ----------------------------------------------
// dW[co][tap][ci] = sum over output voxels v of dY[v][co] X[v + tap][ci], v walked as (sub
// group, plane tz, K step): a K step of 32 voxels is the 16 subs at TWO output positions
// (pa, pb), so a tap's X rows for it are the 16 subs at each shifted position of one input
// plane.  The pairs are chosen so that both positions see the same taps in the padding
// wherever possible (interior with interior, edge with edge of the same side; the four
// corners go with an edge neighbour and differ in one tap column or row): a tap whose shift
// leaves the sub-lattice for both has neither reads nor MFMAs (compile time: wave, plane,
// K step and tap are template constants), and one that leaves it for a single position reads
// that half's rows from a 1 KiB zero block (a per-lane select between two constants).  25
// positions make 12 pairs + (18, none) + an empty step: 7 stages of 2 K steps per plane.
//  * block = 64 output channels x 32 input channels x all 27 taps over a split of the sub
//    groups; 8 waves = 2 (16-channel ci halves) x 4 tap groups of 7 (6), 4 x 7 accumulator
//    tiles per wave (as latticeconv.hip's lattice_wgrad_kernel);
//  * X input planes (16 subs x 25 positions x 32 channels = 25 KiB) stream through a 4-slot
//    ring, each loaded once per sub group: output plane o reads planes o - 1 .. o + 1 of its
//    group, and plane o + 2 of the stream is issued when output plane o starts;
//  * dY (2 K steps x 32 rows x 64 channels = 8 KiB per stage) through a 3-slot ring;
//  * both operands are m-major images read with transposing ds_read_b64_tr_b16 fragment
//    reads; fp32 partial slabs [split][co][tap * Cs + ci] as latticeconv.hip's (summed and
//    transposed by conv.hip's slab reduction).
constexpr int WXROW = 64;                 // X rows: 32 ci x 2 B
constexpr int WYROW = 128;                // dY rows: 64 co x 2 B
constexpr int WXSLOTS = 4;
constexpr int WPLANE = PLB;               // one X plane: 25 KiB
constexpr int KSP = 14;                   // K steps per plane (13 + an empty one)
constexpr int WST = KSP / 2;              // stages per plane
constexpr int WYST = 2 * 32 * WYROW;      // 8 KiB per stage
constexpr int WYSLOTS = 3;
constexpr int WZERO_OFF = WXSLOTS * WPLANE;
constexpr int WY_OFF = WZERO_OFF + NS * WXROW;
constexpr int WLDS = WY_OFF + WYSLOTS * WYST;
static_assert(WLDS <= 160 * 1024, "LDS");

// position of half h of K step j (NP: none)
__host__ __device__ constexpr int kpos(int j, int h) {
  constexpr int t[KSP][2] = {{6, 7},   {8, 11},  {12, 13}, {16, 17}, {1, 2},
                             {21, 22}, {5, 10},  {9, 14},  {0, 3},   {24, 23},
                             {4, 19},  {20, 15}, {18, NP}, {NP, NP}};
  return t[j][h];
}
// the position whose dY rows half h of K step j loads: a real one everywhere (finite rows;
// a half without a position meets zero X rows)
__host__ __device__ constexpr int kpos_dma(int j, int h) {
  return kpos(j, h) < NP ? kpos(j, h) : kpos(j, 0) < NP ? kpos(j, 0) : 18;
}
// position p shifted by tap t's (ky, kx): inside the 5 x 5 plane?
__host__ __device__ constexpr bool yx_in(int p, int t) {
  if (p >= NP) return false;
  const int y = p / S + (t / 3) % 3 - 1, x = p % S + t % 3 - 1;
  return y >= 0 && y < S && x >= 0 && x < S;
}
__host__ __device__ constexpr bool z_in(int tz, int t) {
  const int z = tz + t / 9 - 1;
  return z >= 0 && z < S;
}

// tap K (of tap group TG: taps 7 TG ..) at half h of K step j, output plane tz: inside?
template <int TG>
__host__ __device__ constexpr bool w_on(int k, int j, int tz, int h) {
  const int t = TG * 7 + k;
  return k < (TG == 3 ? 6 : 7) && z_in(tz, t) && yx_in(kpos(j, h), t);
}
template <int TG>
__host__ __device__ constexpr bool w_any(int j, int tz) {
  for (int k = 0; k < 7; ++k)
    if (w_on<TG>(k, j, tz, 0) || w_on<TG>(k, j, tz, 1)) return true;
  return false;
}

__device__ __forceinline__ int wsz64(int r) { return 2 * ((r >> 3) & 1); }
__device__ __forceinline__ int wsz128(int r) { return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1); }

#ifndef L5W_SEQ
#define L5W_SEQ 1
#endif

struct LW5 {
  int Cs, Nd, d, E, G, K;
  int groups_per_split;
  uint32_t xbytes, ybytes;                // operand sizes (buffer-resource ranges)
};

// DD: the dilation as a template constant (4, 8; 0 = run time), so the per-sub-group class
// digits (grp_vox / grp_off, every 5 planes) divide by constants
template <int DD>
__global__ __launch_bounds__(NTHR) void lattice5_wgrad_kernel(LW5 g, const u16* __restrict__ src,
                                                              const u16* __restrict__ dy,
                                                              float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: the co tiles of one (ci chunk, split) read the same X planes
  const int nci = g.Cs / KC, nco = g.Nd / 64;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int cot = tile % nco;
  const int t2 = tile / nco;
  const int cit = t2 % nci, split = t2 / nci;
  const int co0 = cot * 64, ci0 = cit * KC;
  const int d = DD ? DD : g.d, E = DD ? S * DD : g.E;
  const int GG = DD ? DD * DD * DD / NS : g.G;        // sub groups per sample
  const int g0 = split * g.groups_per_split;
  const int nplane_out = g.groups_per_split * S;

  for (int i = tid; i < NS * WXROW / 16; i += NTHR)
    *reinterpret_cast<u32x4*>(smem + WZERO_OFF + i * 16) = u32x4{0u, 0u, 0u, 0u};

  // voxel of (sub group gi, plane z, position ty, tx) for the group's first class; a sub's
  // class digits never carry into the group's (16-aligned classes, d^2 >= 16), so sub s adds
  // a constant
  auto grp_vox = [&](int gi, int z, int ty, int tx) -> int64_t {
    const int n = gi / GG, q = (gi % GG) * NS;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    return (((int64_t)n * E + rz + d * z) * E + ry + d * ty) * E + rx + d * tx;
  };
  auto sub_part = [&](int s) -> int {
    return ((s / (d * d)) * E + (s / d) % d) * E + s % d;
  };
  // X plane: instruction k of wave w = position w + 8k (clamped, as the forward)
  uint32_t xl[PI];
#pragma unroll
  for (int k = 0; k < PI; ++k) {
    const int pos = min(wave + NW * k, NP - 1), s = lane >> 2;
    const int row = pos * NS + s;
    xl[k] = (uint32_t)((sub_part(s) + d * (pos / S) * E + d * (pos % S)) * g.Cs + ci0 +
                       (((lane & 3) ^ wsz64(row)) * 8)) * 2u;
  }
  // both operands through buffer resources: 32-bit byte offsets (wgrad_ok bounds the
  // tensors), a scalar plane part + a constant lane part, no 64-bit lane addresses
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)src, 0, (int)__builtin_amdgcn_readfirstlane(g.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy, 0, (int)__builtin_amdgcn_readfirstlane(g.ybytes), 0x00020000);
  const uint32_t lds0 = lds_addr_of(smem);
  const uint32_t zsx = (uint32_t)(d * E * E * g.Cs * 2), zsy = (uint32_t)(d * E * E * g.Nd * 2);
  // X plane z of a sub group whose first voxel is gx bytes into X, into ring slot `slot`
  auto issue_x = [&](uint32_t gx, int z, int slot) {
    const uint32_t zb = gx + (uint32_t)z * zsx;
    const uint32_t lb = lds0 + (uint32_t)(slot * WPLANE);
#pragma unroll
    for (int k = 0; k < PI; ++k) {
      const int pos = min(wave + NW * k, NP - 1);
      buf_lds16_asm(zb + xl[k], rsx, lb + (uint32_t)(pos * 1024));
    }
  };
  // dY of a stage: one instruction per wave, rows 8w .. 8w + 7 = K step q = w >> 2, half
  // h = (w >> 1) & 1, subs (w & 1) * 8 ..
  const int yrow = wave * 8 + (lane >> 3);
  const int yq = wave >> 2, yh = (wave >> 1) & 1;
  const uint32_t ylane = (uint32_t)(sub_part(yrow & 15) * g.Nd + co0 +
                                    (((lane & 7) ^ wsz128(yrow)) * 8)) * 2u;
  // this wave's dY position of stage M, as a byte offset inside a plane (wave-uniform)
  uint32_t py[WST];
#pragma unroll
  for (int m = 0; m < WST; ++m) {
    const int p = yq == 0 ? (yh == 0 ? kpos_dma(2 * m, 0) : kpos_dma(2 * m, 1))
                          : (yh == 0 ? kpos_dma(2 * m + 1, 0) : kpos_dma(2 * m + 1, 1));
    py[m] = (uint32_t)((d * (p / S) * E + d * (p % S)) * g.Nd * 2);
  }
  // dY of stage M of plane z of a sub group whose first voxel is gy bytes into dY
  auto issue_y = [&](uint32_t gy, int z, auto mc, int sl) {
    constexpr int M = decltype(mc)::value;
    buf_lds16_asm(gy + (uint32_t)z * zsy + py[M] + ylane, rsy,
                  lds0 + (uint32_t)(WY_OFF + sl * WYST + wave * 1024));
  };
  // first voxel of sub group gi (its first class), as byte offsets into X and dY
  auto grp_off = [&](int gi, uint32_t& gx, uint32_t& gy) {
    const int64_t v = grp_vox(gi, 0, 0, 0);
    gx = (uint32_t)(v * g.Cs * 2);
    gy = (uint32_t)(v * g.Nd * 2);
  };

  const int cf = wave & 1, tg = wave >> 1;          // ci half, tap group
  const int t0 = tg * 7, nt = tg == 3 ? 6 : 7;
  const int lk = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int rsel = 8 * lk + q4;                     // this lane's K rows r, r + 4 of a step
  const bool hb = (rsel >> 4) & 1;                  // ... in the step's second half
  auto tr_off = [&](int rowb, int r, int col, int sw) -> uint32_t {
    return (uint32_t)(r * rowb + (((col >> 3) ^ sw) << 4) + (col & 7) * 2);
  };
  uint32_t ya_lo[4], ya_hi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + 4 * p4;
    ya_lo[i] = tr_off(WYROW, rsel, col, wsz128(rsel));
    ya_hi[i] = tr_off(WYROW, rsel + 4, col, wsz128(rsel + 4));
  }
  const uint32_t xb_lo = tr_off(WXROW, rsel & 15, cf * 16 + 4 * p4, wsz64(rsel));
  const uint32_t xb_hi = tr_off(WXROW, (rsel + 4) & 15, cf * 16 + 4 * p4, wsz64(rsel + 4));
  auto tr8 = [](const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)p);
  };
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 7; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};

  {
    uint32_t gx0, gy0;
    grp_off(g0, gx0, gy0);
    issue_x(gx0, 0, 0);
    issue_x(gx0, 1, 1);                             // (nplane_out >= 5)
    issue_y(gy0, 0, std::integral_constant<int, 0>{}, 0);
    issue_y(gy0, 0, std::integral_constant<int, 1>{}, 1);
  }

  struct WFr { bf16x8 a[4], b[7]; };
  auto run = [&](auto tgc) {
    constexpr int TG = decltype(tgc)::value;
    uint32_t xp[3];                                 // X ring offsets of planes o - 1, o, o + 1
    uint32_t hsel = 0;                              // this lane reads the step's second half
    auto kread = [&](const char* yimg, auto qc, auto jc, auto tzc, WFr& f) {
      constexpr int Q = decltype(qc)::value, J = decltype(jc)::value;
      constexpr int TZ = decltype(tzc)::value;
      if constexpr (w_any<TG>(J, TZ)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          f.a[i] = __builtin_shufflevector(tr8(yimg + Q * 32 * WYROW + ya_lo[i]),
                                           tr8(yimg + Q * 32 * WYROW + ya_hi[i]), 0, 1, 2, 3, 4,
                                           5, 6, 7);
        auto one = [&](auto kc) {
          constexpr int K = decltype(kc)::value;
          constexpr bool va = w_on<TG>(K, J, TZ, 0), vb = w_on<TG>(K, J, TZ, 1);
          if constexpr (va || vb) {
            constexpr int t = TG * 7 + K;
            constexpr int dys = ((t / 3) % 3 - 1) * S + t % 3 - 1;
            constexpr int oa = (kpos(J, 0) + dys) * NS * WXROW;
            constexpr int ob = (kpos(J, 1) + dys) * NS * WXROW;
            const uint32_t pl = xp[t / 9];
            uint32_t off;
            if constexpr (va && vb) off = pl + oa + (hsel ? (uint32_t)(ob - oa) : 0u);
            else if constexpr (va) off = hsel ? (uint32_t)WZERO_OFF : pl + oa;
            else off = hsel ? pl + ob : (uint32_t)WZERO_OFF;
            f.b[K] = __builtin_shufflevector(tr8(smem + off + xb_lo), tr8(smem + off + xb_hi), 0,
                                             1, 2, 3, 4, 5, 6, 7);
          }
        };
        one(std::integral_constant<int, 0>{});
        one(std::integral_constant<int, 1>{});
        one(std::integral_constant<int, 2>{});
        one(std::integral_constant<int, 3>{});
        one(std::integral_constant<int, 4>{});
        one(std::integral_constant<int, 5>{});
        one(std::integral_constant<int, 6>{});
      }
    };
    auto kmma = [&](const WFr& f, auto jc, auto tzc) {
      constexpr int J = decltype(jc)::value, TZ = decltype(tzc)::value;
      auto one = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (w_on<TG>(K, J, TZ, 0) || w_on<TG>(K, J, TZ, 1)) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][K] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[K], acc[i][K], 0, 0,
                                                                0);
        }
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
      one(std::integral_constant<int, 4>{});
      one(std::integral_constant<int, 5>{});
      one(std::integral_constant<int, 6>{});
    };

    // sub group offsets: this one and the next (zero past the stream's end: never issued)
    uint32_t gxc = 0, gyc = 0, gxn = 0, gyn = 0;
    // output plane o of the block's stream, TZ = its z position in the sub group
    auto plane = [&](int o, auto tzc) {
      constexpr int TZ = decltype(tzc)::value;
      const bool xnow = o + 2 < nplane_out;         // X plane o + 2 issued at stage 0
      const bool lastp = o + 1 == nplane_out;
      const int o3 = o % WYSLOTS;                   // stage o * 7 + M sits in slot (o + M) % 3
      uint32_t xq[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) xq[k] = (uint32_t)(((o + k + 3) & 3) * WPLANE);
      auto stage = [&](auto mc) {
        constexpr int M = decltype(mc)::value;
        const int sl = (o3 + M) % WYSLOTS;
        const int sl2 = (o3 + M + 2) % WYSLOTS;
        // dY of this stage landed (issued two stages ago); younger: the next stage's dY and,
        // at stages 1 and 2, the X plane issued at stage 0 after stage 2's dY
        if ((M == 1 || M == 2) && xnow) wait_vm_lgkm0<PI + 1>();
        else if (lastp && M == WST - 1) wait_vm_lgkm0<0>();
        else wait_vm_lgkm0<1>();
        raw_barrier();
        if constexpr (M + 2 < WST) {
          issue_y(gyc, TZ, std::integral_constant<int, M + 2>{}, sl2);
        } else if (!lastp) {
          if constexpr (TZ + 1 < S) issue_y(gyc, TZ + 1, std::integral_constant<int, M + 2 - WST>{}, sl2);
          else issue_y(gyn, 0, std::integral_constant<int, M + 2 - WST>{}, sl2);
        }
        if (M == 0 && xnow) {
          if constexpr (TZ + 2 < S) issue_x(gxc, TZ + 2, (o + 2) % WXSLOTS);
          else issue_x(gxn, TZ + 2 - S, (o + 2) % WXSLOTS);
        }
        // (opaque after the barrier, so that no stage's fragment addresses are computed
        // early and held in VGPRs)
        int yoff = WY_OFF + sl * WYST;
        asm volatile("" : "+s"(yoff));
        const char* yimg = smem + yoff;
        xp[0] = xq[0]; xp[1] = xq[1]; xp[2] = xq[2];
        asm volatile("" : "+s"(xp[0]), "+s"(xp[1]), "+s"(xp[2]));
        hsel = hb ? 1u : 0u;
        asm volatile("" : "+v"(hsel));
#if L5W_SEQ
        // one fragment set: step 0's reads, MFMAs, then step 1's (the reads of step 1 overlap
        // step 0's MFMAs only as far as the compiler hoists them)
        WFr f0;
        kread(yimg, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * M>{}, tzc,
              f0);
        kmma(f0, std::integral_constant<int, 2 * M>{}, tzc);
        kread(yimg, std::integral_constant<int, 1>{}, std::integral_constant<int, 2 * M + 1>{},
              tzc, f0);
        kmma(f0, std::integral_constant<int, 2 * M + 1>{}, tzc);
#else
        WFr f0, f1;
        kread(yimg, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * M>{}, tzc,
              f0);
        kread(yimg, std::integral_constant<int, 1>{}, std::integral_constant<int, 2 * M + 1>{},
              tzc, f1);
        kmma(f0, std::integral_constant<int, 2 * M>{}, tzc);
        kmma(f1, std::integral_constant<int, 2 * M + 1>{}, tzc);
#endif
      };
      stage(std::integral_constant<int, 0>{});
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      stage(std::integral_constant<int, 4>{});
      stage(std::integral_constant<int, 5>{});
      stage(std::integral_constant<int, 6>{});
    };
    for (int og = 0, gi = g0; og < nplane_out; og += S, ++gi) {   // a sub group's 5 planes
      grp_off(gi, gxc, gyc);
      if (og + S < nplane_out) grp_off(gi + 1, gxn, gyn);
      plane(og + 0, std::integral_constant<int, 0>{});
      plane(og + 1, std::integral_constant<int, 1>{});
      plane(og + 2, std::integral_constant<int, 2>{});
      plane(og + 3, std::integral_constant<int, 3>{});
      plane(og + 4, std::integral_constant<int, 4>{});
    }
  };
  switch (tg) {                                     // wave-uniform
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }

  // partial slab [split][co][tap * Cs + ci]
  float* out = ws + (int64_t)split * g.Nd * g.K;
  const int lr = lane & 15;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    if (k < nt) {
      const int kcol = (t0 + k) * g.Cs + ci0 + cf * 16 + lr;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          out[(int64_t)(co0 + i * 16 + lk * 4 + r) * g.K + kcol] = acc[i][k][r];
    }
  }
}

// MMAD_LATTICE5: 1 (default) where the blocks fill the CUs, 2 at any size, 0 off;
// mmad_set_kernel_variant("lattice5", v) overrides it at run time
std::atomic<int> g_mode{-1};
int mode() {
  int v = g_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_LATTICE5");
    int expect = -1;
    g_mode.compare_exchange_strong(expect, e ? atoi(e) : 1);
    v = g_mode.load(std::memory_order_relaxed);
  }
  return v;
}

}  // namespace

namespace mmad_lattice5 {

int set_mode(int v) {
  const int prev = mode();
  if (v >= 0) g_mode.store(v, std::memory_order_relaxed);
  return prev;
}

static int64_t blocks(const mmad_patch::Geo& q) {
  return (int64_t)q.nb * (q.dd * q.dd * q.dd / NS) * 4 * (q.Nd / BW);
}

bool ok(const mmad_patch::Geo& q) {
  if (mode() <= 0) return false;
  const int d = q.dd;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dh != d || q.dw != d || d < 2) return false;
  if (q.pd != d || q.ph != d || q.pw != d || (d * d * d) % NS) return false;
  const int E = S * d;
  if (q.Ds != E || q.Hs != E || q.Ws != E || q.Dd != E || q.Hd != E || q.Wd != E) return false;
  if (q.Cs % KC || q.Nd % BW || q.Kpad != 27 * q.Cs) return false;
  // 32-bit per-lane DMA offsets: one sample's volume, the packed weights
  if ((int64_t)E * E * E * q.Cs >= (int64_t(1) << 31) ||
      (int64_t)q.Nd * q.Kpad >= (int64_t(1) << 31))
    return false;
  if (blocks(q) >= (int64_t(1) << 31)) return false;
  return mode() == 2 || blocks(q) >= 256;
}

// BN partial-sum rows: one per (sample, sub group, plane)
int64_t tiles(const mmad_patch::Geo& q) { return (int64_t)q.nb * (q.dd * q.dd * q.dd / NS) * S; }

int fwd(const mmad_patch::Geo& q, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream) {
  if (!mmad_lattice5::ok(q)) return MMAD_EUNSUPPORTED;
  static const bool attr = hipFuncSetAttribute((const void*)lattice5_conv_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               LDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  G5 g{};
  g.Cs = q.Cs; g.Nd = q.Nd; g.Kpad = q.Kpad;
  g.nchunk = q.Cs / KC;
  g.nbn = q.Nd / BW;
  g.d = q.dd; g.E = S * q.dd; g.G = q.dd * q.dd * q.dd / NS;
  g.ngroups = q.nb * g.G;
  g.xcd = g.ngroups % 8 == 0 ? 1 : 0;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  hipLaunchKernelGGL(lattice5_conv_kernel, dim3((unsigned)blocks(q)), dim3(NTHR), LDS,
                     as_stream(stream), g, (const u16*)src, (const u16*)wp, bias, (u16*)dst,
                     stats);
  return launch_status();
}

// weight gradient: splits of the sub groups until the (ci chunk, co tile) blocks fill the CUs
static bool wgrad_geom(const mmad_patch::Geo& q) {
  const int d = q.dd;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dh != d || q.dw != d || d < 2) return false;
  if (q.pd != d || q.ph != d || q.pw != d || (d * d * d) % NS) return false;
  const int E = S * d;
  if (q.Ds != E || q.Hs != E || q.Ws != E || q.Dd != E || q.Hd != E || q.Wd != E) return false;
  if (q.Cs % KC || q.Nd % 64) return false;
  // 32-bit byte offsets into X and dY (buffer resources)
  return (int64_t)q.nb * E * E * E * std::max(q.Cs, q.Nd) * 2 < (int64_t(1) << 31);
}
int wgrad_splits(const mmad_patch::Geo& q) {
  const int64_t tiles = (int64_t)(q.Cs / KC) * (q.Nd / 64);
  const int64_t ngroups = (int64_t)q.nb * (q.dd * q.dd * q.dd / NS);
  int sp = 1;
  while (tiles * sp < 256 && ngroups % (sp * 2) == 0) sp *= 2;
  return sp;
}
bool wgrad_ok(const mmad_patch::Geo& q) {
  if (mode() <= 0 || !wgrad_geom(q)) return false;
  const int64_t nblk = (int64_t)(q.Cs / KC) * (q.Nd / 64) * wgrad_splits(q);
  if (nblk >= (int64_t(1) << 31)) return false;
  return mode() == 2 || nblk >= 256;
}
int64_t wgrad_workspace(const mmad_patch::Geo& q) {
  return (int64_t)wgrad_splits(q) * q.Nd * 27 * q.Cs * 4;
}
int wgrad(const mmad_patch::Geo& q, const void* x, const void* dy, float* ws, int* splits,
          void* stream) {
  if (!wgrad_ok(q)) return MMAD_EUNSUPPORTED;
  auto at = [](const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, WLDS) == hipSuccess;
  };
  static const bool attr = at((const void*)lattice5_wgrad_kernel<4>) &&
                           at((const void*)lattice5_wgrad_kernel<8>) &&
                           at((const void*)lattice5_wgrad_kernel<0>);
  if (!attr) return MMAD_EUNSUPPORTED;
  const int sp = wgrad_splits(q);
  LW5 g{};
  g.Cs = q.Cs; g.Nd = q.Nd; g.d = q.dd; g.E = S * q.dd; g.G = q.dd * q.dd * q.dd / NS;
  g.K = 27 * q.Cs;
  g.groups_per_split = q.nb * g.G / sp;
  const int64_t vox = (int64_t)q.nb * g.E * g.E * g.E;
  g.xbytes = (uint32_t)(vox * q.Cs * 2);
  g.ybytes = (uint32_t)(vox * q.Nd * 2);
  const int64_t nblk = (int64_t)(q.Cs / KC) * (q.Nd / 64) * sp;
  if (q.dd == 4)
    hipLaunchKernelGGL(lattice5_wgrad_kernel<4>, dim3((unsigned)nblk), dim3(NTHR), WLDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else if (q.dd == 8)
    hipLaunchKernelGGL(lattice5_wgrad_kernel<8>, dim3((unsigned)nblk), dim3(NTHR), WLDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else
    hipLaunchKernelGGL(lattice5_wgrad_kernel<0>, dim3((unsigned)nblk), dim3(NTHR), WLDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  *splits = sp;
  return launch_status();
}

}  // namespace mmad_lattice5
