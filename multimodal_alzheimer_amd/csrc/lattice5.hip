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
  const u16* __restrict__ srcn = src + (int64_t)n * vol * g.Cs;

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
      pofs[k] = (uint32_t)(vox * g.Cs + ((lane & 3) ^ swz(row)) * 8);
    }
  }
  // ---- weight DMA: instruction q = wave + NW h: tap q / 8, rows 16 (q % 8) ..
  uint32_t wofs[WI];
  int wq_off[WI];
#pragma unroll
  for (int h = 0; h < WI; ++h) {
    const int q = wave + NW * h;
    const int tk = q / (BW / 16), rb = q % (BW / 16);
    const int row = rb * 16 + (lane >> 2);
    wofs[h] = (uint32_t)((n0 + row) * g.Kpad + (((lane & 3) ^ swz(row)) * 8) + tk * g.Cs);
    wq_off[h] = tk * BTAP + rb * 1024;
  }

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
    const int nplanes = g.nchunk * nz, nstage = 3 * nplanes;
    // plane i = (chunk i / nz, kz = kz0 + i % nz) -> ring slot i % 3
    auto issue_plane = [&](int i) {
      const int c = i / nz, z = tz + kz0 + i % nz;
      const u16* base = srcn + (int64_t)z * d * E * E * g.Cs + c * KC;
      char* pb = smem + (i % NPS) * PLB;
#pragma unroll
      for (int k = 0; k < PI; ++k) {
        const int pos = min(wave + NW * k, NP - 1);
        glds16_asm(base + pofs[k], lds_addr_of(pb + pos * 1024));
      }
    };
    // stage s = 3 i + (ky + 1) of plane i: taps t0 = 9 (kz + 1) + 3 (ky + 1) .. + 2
    auto issue_stage_b = [&](int s) {
      const int i = s / 3, c = i / nz, kz = kz0 + i % nz, ky = s % 3 - 1;
      const u16* base = wgt + (9 * (kz + 1) + 3 * (ky + 1)) * g.Cs + c * KC;
      char* sb = ring + (s % NSTL) * BSLOT;
#pragma unroll
      for (int h = 0; h < WI; ++h) glds16_asm(base + wofs[h], lds_addr_of(sb + wq_off[h]));
    };

    f32x4 acc[NF][TN];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: planes 0, 1 and the weights of stages 0, 1.  Group s (issued after stage
    // s's barrier): plane s / 3 + 2 when s % 3 == 0 (its slot's last reader, plane s / 3 - 1,
    // finished at stage s - 1) and the weights of stage s + 2 (into stage s - 1's slot)
    issue_plane(0);
    if (nplanes > 1) issue_plane(1);
    issue_stage_b(0);
    if (nstage > 1) issue_stage_b(1);
    auto group_ops = [&](int s) {
      return (s + 2 < nstage ? WI : 0) + ((s % 3 == 0 && s / 3 + 2 < nplanes) ? PI : 0);
    };
    auto run = [&](auto wmc) {
      constexpr int WM = decltype(wmc)::value;
      for (int i = 0; i < nplanes; ++i) {
        const char* pl = smem + (i % NPS) * PLB + a_lane;
        auto stage = [&](auto kyc) {
          constexpr int KY = decltype(kyc)::value;
          const int s = 3 * i + KY + 1;
          // younger than this stage's weights: group s - 1 (or, at s = 0, stage 1's weights);
          // a plane is issued six stages before its first reader, ahead of its weights
          wait_ops(s == 0 ? (nstage > 1 ? WI : 0) : group_ops(s - 1));
          raw_barrier();
          if (s % 3 == 0 && s / 3 + 2 < nplanes) issue_plane(s / 3 + 2);
          if (s + 2 < nstage) issue_stage_b(s + 2);
          int boff = RING_OFF + (s % NSTL) * BSLOT;
          asm volatile("" : "+s"(boff));
          stage_body<WM, KY>(acc, smem + boff + b_lane, pl);
        };
        stage(std::integral_constant<int, -1>{});
        stage(std::integral_constant<int, 0>{});
        stage(std::integral_constant<int, 1>{});
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

}  // namespace mmad_lattice5
