// Residue-class ("lattice") 3D convolution for the dilated MedicalNet convs, gfx950 (bf16,
// fp32 accumulate).
//
// Serves layer4's 3x3x3 convs (dilation 4, padding 4, stride 1; 256/512 channels at 16^3
// for a 128^3 input, reached from pkg/models/mri_models/anat_cnn.py:29-31) forward and --
// as a forward conv over reversed taps -- input gradient.
//
// A dilation-d 3^3 conv with padding d on a grid of 4d voxels per dimension splits into d^3
// independent dense 3^3 convs (padding 1) on the residue classes' 4^3 sub-lattices: voxel
// (rz + d*tz, ry + d*ty, rx + d*tx) only ever meets voxels of its own class (rz, ry, rx),
// and every tap that leaves the 4^3 sub-lattice lands in the zero padding.  So:
//  * a tile is one z-plane (4 x 4 positions) of 32 sub-lattices ("subs": sample x class):
//    512 GEMM rows = position-major, sub-minor, so an MFMA fragment (16 rows) is 16 subs at
//    ONE position and whether a tap is padding is the same for the whole fragment;
//  * padding taps are skipped outright (no zero MACs: per dimension 2 of the 12
//    (position, tap) pairs are padding, so 58 % of the dense MACs remain);
//  * the A operand never goes through the per-tap gather: the three z-planes a tile needs
//    (tz-1, tz, tz+1 of its 32 subs, 32 input channels at a time) sit in LDS as the
//    "patch", and each tap's fragments are read from it at a shifted row -- one LDS-DMA per
//    input voxel per channel chunk per tile instead of one per tap;
//  * only the weights stream per tap (128 output channels x 32 input channels = 8 KiB per
//    tap, 24 KiB per 3-tap stage, a 3-slot ring with two stages in flight): per wave three
//    1 KiB LDS-DMAs per stage;
//  * the loop walks (chunk, kz) groups of three stages that read ONE input plane each, so
//    the patch is a 2-slot plane ring: the next group's plane is loaded while the current
//    group runs (3 stages ahead);
//  * 8 waves = 4 x 2 wave tiles of 128 rows x 64 channels; wave wm takes the positions of
//    one diagonal of the 4 x 4 plane, (t, (t + wm) & 3), so every wave loses the same number
//    of fragments to padding on every tap (a row of the plane would idle the edge waves);
//  * 64-byte patch / weight rows (32 channels), 16-byte chunks swizzled by 3*((row>>3)&1)
//    (conflict-free ds_read_b128 fragment reads, as conv.hip's 64-byte variant);
//  * epilogue as the implicit GEMM: bias, BN partial sums (one row per tile), optional
//    residual + ReLU (eval-mode fused BN), bf16 tile transposed through LDS into 16-byte
//    channel-vector stores; tiles walk the XCDs in contiguous ranges (the 4 channel tiles
//    and neighbouring planes of one sub group share an L2).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "patchconv.h"

namespace {

constexpr int S = 4;                      // sub-lattice extent per dimension
constexpr int NS = 32;                    // subs per tile
constexpr int PL = S * S * NS;            // rows per plane (512)
constexpr int RBL = 64;                   // bytes per row: 32 bf16 channels
constexpr int KC = RBL / 2;               // channels per chunk
constexpr int PLANE = PL * RBL;           // 32 KiB
constexpr int BNL = 128;                  // output channels per tile
constexpr int TPS = 3;                    // taps per stage (one kx row)
constexpr int BTAP = BNL * RBL;           // one tap's weights: 8 KiB
constexpr int BSLOT = TPS * BTAP;         // one stage: 24 KiB
// weight ring slots: NSTL - 1 stages of weights in flight (an LDS-DMA lands ~1 us after
// issue, about one stage of MFMAs); the patch holds 2 plane slots, since a stage group
// (one kz plane of one chunk) reads a single plane and the next group's plane streams in
// during it
#ifndef LAT_NSTL
#define LAT_NSTL 3
#endif
constexpr int NSTL = LAT_NSTL;
constexpr int NPS = 2;                    // patch plane slots
constexpr int RING_OFF = NPS * PLANE;
constexpr int MAIN_LDS = RING_OFF + NSTL * BSLOT;
constexpr int CROW = BNL * 2 + 16;
constexpr int EPI_LDS = PL * CROW + 3 * 2 * BNL * 4;
constexpr int LDS_BYTES = MAIN_LDS > EPI_LDS ? MAIN_LDS : EPI_LDS;
constexpr int NTHR = 512;

struct LG {
  int nb, Cs, Nd, Kpad, d;
  int ngroups, nbn, nchunk;
  const u16* res;
  int relu;
  int prio;                                         // s_setprio 1 for waves 4-7 (A/B switch)
  int D, H, W, nz;                                  // ragged grids: extents, planes per class
};

__device__ __forceinline__ int swz(int row) { return 3 * ((row >> 3) & 1); }

template <int TN>
struct Frags {
  bf16x8 b[TN];
  bf16x8 a[4][2];
};

// position i of wave diagonal WM, shifted by tap (KY, KX), inside the 4 x 4 plane
template <int WM, int KY, int KX>
__device__ constexpr bool tap_ok(int i) {
  return i + KY >= 0 && i + KY < S && ((i + WM) & 3) + KX >= 0 && ((i + WM) & 3) + KX < S;
}

template <int TN, int WM, int KY, int KX>
__device__ __forceinline__ void read_tap(const char* bsl, const char* apl, Frags<TN>& f) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
    f.b[j] = *reinterpret_cast<const bf16x8*>(bsl + (KX + 1) * BTAP + j * 16 * RBL);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (tap_ok<WM, KY, KX>(i)) {
      constexpr int dummy = 0;
      const int ps = (i + KY) * S + ((i + WM) & 3) + KX + dummy;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        f.a[i][h] = *reinterpret_cast<const bf16x8*>(apl + (ps * 2 + h) * 16 * RBL);
    }
  }
}

template <int TN, int WM, int KY, int KX>
__device__ __forceinline__ void mma_tap(f32x4 (&acc)[8][TN], const Frags<TN>& f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (tap_ok<WM, KY, KX>(i)) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#ifndef LAT_NO_MFMA
          acc[i * 2 + h][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i][h], f.b[j], acc[i * 2 + h][j], 0, 0, 0);
#endif
        }
    }
  }
}

template <int TN, int WM, int KY>
__device__ __forceinline__ void stage_body(f32x4 (&acc)[8][TN], const char* bsl, const char* apl) {
  Frags<TN> f0, f1;
  read_tap<TN, WM, KY, -1>(bsl, apl, f0);
  read_tap<TN, WM, KY, 0>(bsl, apl, f1);
  mma_tap<TN, WM, KY, -1>(acc, f0);
  read_tap<TN, WM, KY, 1>(bsl, apl, f0);
  mma_tap<TN, WM, KY, 0>(acc, f1);
  mma_tap<TN, WM, KY, 1>(acc, f0);
}

// TN = 16-column MFMA tiles per wave: 4 (128-channel tiles) or 2 (64-channel tiles, for
// layers whose 128-channel tiling leaves CUs idle).
// RAG: ragged grids (any D x H x W with ceil(H / d), ceil(W / d) <= 4, e.g. the reference's
// 91 x 109 x 91 MNI volumes, 12 x 14 x 12 at layer4): a class's sub-lattice is then up to
// 4 x 4 positions per plane and nz planes deep, and the positions / planes it lacks are read
// as zeros (buffer-resource LDS-DMA past the resource's end, no branch) -- exactly the conv's
// zero padding -- and skipped in the epilogue (no store, no BN sum).  The tap skipping stays
// compile-time on the 4 x 4 plane.
template <int TN, bool RAG>
__global__ __launch_bounds__(NTHR) void lattice_conv_kernel(LG g, const u16* __restrict__ src,
                                                            const u16* __restrict__ wgt,
                                                            const float* __restrict__ bias,
                                                            u16* __restrict__ dst,
                                                            float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + RING_OFF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = tile % g.nbn;
  const int t2 = tile / g.nbn;
  const int NZ = RAG ? g.nz : S;                    // planes per class
  const int tz = t2 % NZ, gid = t2 / NZ;
  const int d = g.d, E = S * d;                     // grid extent per dimension (4d grids)
  const int gpn = d * d * d / NS;                   // sub groups per sample
  const int n = gid / gpn, q0 = (gid % gpn) * NS;   // sample, first class of the group
  constexpr int BW = 32 * TN;                      // output channels of this tile
  const int n0 = nt * BW;
  const int64_t plane_vox = (int64_t)d * E * E;     // voxel step between planes tz, tz+1

  // ---- patch DMA: plane slot p <- absolute plane tz - 1 + p of chunk cc (32 rows per
  // wave: 4 instructions of 16 rows x 64 B); every row is a real voxel (no halo rows)
  // (per-lane DMA offsets in 32 bits from uniform bases: this sample's volume and the
  // packed weights, both < 2^31 elements -- checked in ok(); fewer VGPRs than pointers)
  const int lrow = lane >> 2;
  const int64_t svox = RAG ? (int64_t)g.D * g.H * g.W : (int64_t)E * E * E;
  const u16* __restrict__ srcn = src + (int64_t)n * svox * g.Cs;
  uint32_t pofs[4];
  int rzk[4];                                       // RAG: the row's class z residue, or
#pragma unroll                                      // -huge when its (y, x) is outside
  for (int k = 0; k < 4; ++k) {
    const int row = (wave * 4 + k) * 16 + lrow;
    const int pos = row / NS, s = row % NS;
    const int q = q0 + s;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    const int ty = pos / S, tx = pos % S;
    if constexpr (RAG) {                            // byte offsets for the buffer DMA
      const int y = ry + d * ty, x = rx + d * tx;
      const int vox = (rz * g.H + y) * g.W + x;
      pofs[k] = (uint32_t)(vox * g.Cs + ((lane & 3) ^ swz(row)) * 8) * 2u;
      rzk[k] = (y < g.H && x < g.W) ? rz : -(1 << 20);
    } else {
      const int vox = (rz * E + ry + d * ty) * E + rx + d * tx;
      pofs[k] = (uint32_t)(vox * g.Cs + ((lane & 3) ^ swz(row)) * 8);
      rzk[k] = 0;
    }
  }
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)srcn, 0, RAG ? (int)__builtin_amdgcn_readfirstlane((uint32_t)(svox * g.Cs * 2)) : 0,
      0x00020000);
  auto issue_plane = [&](int kz, int cc, int slot) {
    char* pb = smem + slot * PLANE;
    if constexpr (RAG) {
      constexpr uint32_t OOB = 0x80000000u;         // >= any per-sample volume (ok())
      const int zp = d * (tz + kz);                 // plane's z offset from the class residue
      const uint32_t zoff = (uint32_t)(zp * g.H * g.W * g.Cs + cc * KC) * 2u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = rzk[k] >= 0 && rzk[k] + zp < g.D;
        buf_lds16_asm(ok ? pofs[k] + zoff : OOB, rsx, lds_addr_of(pb + (wave * 4 + k) * 1024));
      }
    } else {
      const u16* base = srcn + (int64_t)(tz + kz) * plane_vox * g.Cs + cc * KC;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        glds16_asm(base + pofs[k], lds_addr_of(pb + (wave * 4 + k) * 1024));
    }
  };
  // ---- weight DMA: stage (chunk cc, first tap t) into ring slot sl: 3 consecutive taps
  // (one kx row), 16 rows per wave per tap
  // 2*TN instructions of 16 rows per tap, 6*TN per stage: wave w issues q = w + 8h (the
  // same count WI on every wave -- surplus slots repeat the last row -- so the counted
  // vmcnt waits below hold on every wave)
  constexpr int NQ = TPS * 2 * TN, WI = (NQ + 7) / 8;
  uint32_t wofs[3];
  int wq_off[3];
#pragma unroll
  for (int h = 0; h < 3; ++h) {
    const int q = min(wave + 8 * h, NQ - 1);
    const int tk = q / (2 * TN), rb = q % (2 * TN);
    const int row = rb * 16 + lrow;
    wofs[h] = (uint32_t)((n0 + row) * g.Kpad + (((lane & 3) ^ swz(row)) * 8) + tk * g.Cs);
    wq_off[h] = tk * BTAP + rb * 1024;
  }
  auto issue_b = [&](int cc, int t, int sl) {
    const u16* base = wgt + t * g.Cs + cc * KC;
#pragma unroll
    for (int h = 0; h < WI; ++h)
      glds16_asm(base + wofs[h], lds_addr_of(ring + sl * BSLOT + wq_off[h]));
  };

  // stage list: chunk-major, then the valid kz planes, then ky; a stage runs kx = -1, 0, 1.
  // Group u = (chunk, kz) of 3 stages reads plane slot u % 2.
  const int kz0 = tz == 0 ? 0 : -1, kz1 = tz == NZ - 1 ? 0 : 1;
  const int nkz = kz1 - kz0 + 1;
  const int ngrp = g.nchunk * nkz;                  // (chunk, kz) groups
  const int nstage = ngrp * 3;
  auto issue_group_plane = [&](int u) {
    issue_plane(kz0 + u % nkz, u / nkz, u % NPS);
  };

  // wave tiles: wm -> diagonal positions (t, (t + wm) & 3), wn -> 64 output channels
  const int wm = wave & 3, wn = wave >> 2;
  const int lr = lane & 15, lk = lane >> 4;
  const uint32_t a_lane = lr * RBL + ((lk ^ swz(lr)) << 4);
  const uint32_t b_lane = (wn * 16 * TN + lr) * RBL + ((lk ^ swz(lr)) << 4);
  f32x4 acc[8][TN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue_stage_b = [&](int s) {                 // weights of stage s (kx = -1 .. 1)
    const int u = s / 3, ky = s % 3 - 1;
    const int cc = u / nkz, kz = kz0 + u % nkz;
    issue_b(cc, (kz + 1) * 9 + (ky + 1) * 3, s % NSTL);
  };
  // prologue: plane of group 0, weights of stage 0, plane of group 1, weights of stages
  // 1 .. NSTL-2; everything lands before stage 0 (one tile per CU: paid once)
  issue_group_plane(0);
  issue_stage_b(0);
  if (ngrp > 1) issue_group_plane(1);
#pragma unroll
  for (int s = 1; s < NSTL - 1; ++s)
    if (s < nstage) issue_stage_b(s);
  // Main loop, compiled once per wave diagonal WM with the three ky stages of a (chunk,
  // kz) group unrolled, so every padding test in the stage bodies is a compile-time
  // constant: no branch sits between a fragment read and its MFMA, and the next tap's reads
  // stay in flight during each tap's MFMAs.
  //
  // Stage s = 3u + r waits for its weights (issued at stage s - NSTL + 1); younger are the
  // weights of the next NSTL - 2 stages and, for 0 < r <= NSTL - 2, the plane of group
  // u + 1 (issued at stage 3u, before that stage's weights, so the wait at stage 3u + 3 --
  // its first use -- forces it).
  auto one_stage = [&](int s, auto rc, bool plane_young) {
    constexpr int R = decltype(rc)::value;
    constexpr int YW = (NSTL - 2) * WI;             // younger weight DMAs per wave
    constexpr bool PW = R != 0 && R <= NSTL - 2;    // group plane issued inside the window
    if (s == 0 || s + NSTL - 2 >= nstage) wait_vm_lgkm0<0>();
    else if (PW && plane_young) wait_vm_lgkm0<YW + 4>();
    else wait_vm_lgkm0<YW>();
    raw_barrier();
    if (R == 0 && s > 0 && s / 3 + 1 < ngrp) issue_group_plane(s / 3 + 1);
#ifndef LAT_NO_B
    if (s + NSTL - 1 < nstage) issue_stage_b(s + NSTL - 1);
#endif
  };
  auto run = [&](auto wmc) {
    constexpr int WM = decltype(wmc)::value;
    for (int u = 0; u < ngrp; ++u) {
      const char* apl = smem + (u % NPS) * PLANE + a_lane;
      const int s0 = u * 3;
      // the plane of group u + 1 was issued at stage s0 (u >= 1) and is younger than the
      // weights waited for at stages s0 + 1 .. s0 + NSTL - 2
      const bool py = u >= 1 && u + 1 < ngrp;
      one_stage(s0, std::integral_constant<int, 0>{}, py);
      stage_body<TN, WM, -1>(acc, ring + (s0 % NSTL) * BSLOT + b_lane, apl);
      one_stage(s0 + 1, std::integral_constant<int, 1>{}, py);
      stage_body<TN, WM, 0>(acc, ring + ((s0 + 1) % NSTL) * BSLOT + b_lane, apl);
      one_stage(s0 + 2, std::integral_constant<int, 2>{}, py);
      stage_body<TN, WM, 1>(acc, ring + ((s0 + 2) % NSTL) * BSLOT + b_lane, apl);
    }
  };
  // the second-dispatched half of the waves loses every issue arbitration at the stage
  // barrier; a static priority for it (MI355X_MICROARCH.md, "two waves per SIMD" item 4)
  if (g.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  switch (wm) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }
  __syncthreads();                                  // patch / ring reused by the epilogue

  // ---- epilogue: tile row r = pos * NS + sub; acc[i*2+h][j][e] is row
  // (pos_i * NS + h*16 + lk*4 + e), column wn*64 + j*16 + lr
  // (RAG: -1 for a row outside the grid)
  auto dst_vox = [&](int row) -> int64_t {
    const int pos = row / NS, s = row % NS;
    const int q = q0 + s;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    const int ty = pos / S, tx = pos % S;
    if constexpr (RAG) {
      const int z = rz + d * tz, y = ry + d * ty, x = rx + d * tx;
      if (z >= g.D || y >= g.H || x >= g.W) return -1;
      return (((int64_t)n * g.D + z) * g.H + y) * g.W + x;
    }
    return (((int64_t)n * E + rz + d * tz) * E + ry + d * ty) * E + rx + d * tx;
  };
  u16* ctile = reinterpret_cast<u16*>(smem);
  // RAG: which of this lane's 32 accumulator rows lie inside the grid (bit i*8 + h*4 + e),
  // computed once in a rolled loop (unrolled, the row tests were hoisted into ~100 VGPRs)
  uint32_t vmask = 0xffffffffu;
  if constexpr (RAG) {
    vmask = 0;
#pragma unroll 1
    for (int b = 0; b < 32; ++b) {
      const int i = b >> 3, h = (b >> 2) & 1, e = b & 3;
      const int row = (i * S + ((i + wm) & 3)) * NS + h * 16 + lk * 4 + e;
      if (dst_vox(row) >= 0) vmask |= 1u << b;
    }
  }
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    cs[j] = 0.f;
    cq[j] = 0.f;
    const int col = wn * 16 * TN + j * 16 + lr;
    const float bv = bias != nullptr ? bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pos = i * S + ((i + wm) & 3);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = pos * NS + h * 16 + lk * 4 + e;
          const float v = acc[i * 2 + h][j][e] + bv;
          ctile[row * (CROW / 2) + col] = f2bf(v);
          if ((vmask >> (i * 8 + h * 4 + e)) & 1u) {
            cs[j] += v;
            cq[j] += v * v;
          }
        }
    }
  }
  __syncthreads();
  constexpr int CPR = BW / 8;
#pragma unroll
  for (int hh = 0; hh < PL * CPR / NTHR; ++hh) {
    const int qd = tid + NTHR * hh;
    const int row = qd / CPR, c8 = qd % CPR;
    const int64_t dv = dst_vox(row);
    if (RAG && dv < 0) continue;
    const int64_t o = dv * g.Nd + n0 + c8 * 8;
    u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) + row * CROW +
                                              c8 * 16);
    if (g.res != nullptr || g.relu) v = epi_res_relu(v, g.res ? g.res + o : nullptr, g.relu);
    *reinterpret_cast<u32x4*>(dst + o) = v;
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(smem + PL * CROW);
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
      const int mt = gid * NZ + tz;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * 16 * TN + j * 16 + lr;
        float ss = cs[j], qs = cq[j];
        for (int w = 1; w < 4; ++w) {              // fixed order: deterministic
          ss += red[(w - 1) * 2 * BW + col];
          qs += red[(w - 1) * 2 * BW + BW + col];
        }
        stats[((int64_t)mt * 2) * g.Nd + n0 + col] = ss;
        stats[((int64_t)mt * 2 + 1) * g.Nd + n0 + col] = qs;
      }
    }
  }
}


// ---- weight gradient on the residue-class lattice ----------------------------------------
// dW[co][tap][ci] = sum over output voxels v of dY[v][co] * X[v + tap][ci], v walked as
// (sub group, plane tz, position, 32 subs): a K step of 32 voxels is 32 subs at ONE output
// position, so a tap's X rows for that step are the 32 subs at one shifted position of one
// input plane -- or, when the shift leaves the 4^3 sub-lattice, padding: those (tap, K step)
// pairs are skipped at compile time (position, tap group and plane are template constants).
//  * block = 64 output channels x 32 input channels x all 27 taps over a split of the sub
//    groups; 8 waves = 2 (16-channel ci halves) x 4 tap groups of 7 (6); per wave 4 x 7
//    accumulator tiles;
//  * X input planes (32 subs x 16 positions x 32 channels = 32 KiB) stream through a 4-slot
//    ring, each loaded once per sub group (the tile of output plane tz reads planes
//    tz-1..tz+1; plane o+2 of the stream is issued when output plane o starts);
//  * dY (2 positions x 32 subs x 64 channels = 8 KiB per stage) through a 3-slot ring;
//  * both operands are m-major images read with transposing ds_read_b64_tr_b16 fragment
//    reads (as conv.hip's wgrad_kernel); fp32 partial slabs [split][co][tap*Cs + ci] are
//    summed and transposed by conv.hip's wgrad_reduce_t_kernel.
// (A software-pipelined stage loop -- the barrier between a stage's two positions, as in
// latticezp.hip -- measured slower in the config-2 step, r03e: layer4.0.conv2 wgrad 266.5 us
// against 241.0 for this barrier-first loop, conv1 138.1 against 125.7; removed.)
constexpr int WXROW = 64;                 // X rows: 32 ci x 2 B
constexpr int WYROW = 128;                // dY rows: 64 co x 2 B
constexpr int WPLANE = PL * WXROW;        // 32 KiB
constexpr int WXSLOTS = 4;
constexpr int WYST = 2 * NS * WYROW;      // 8 KiB: 2 positions per stage
constexpr int WYSLOTS = 3;
constexpr int WZERO_OFF = WXSLOTS * WPLANE;  // 2 KiB spare (the former padding-row block)
constexpr int WY_OFF = WZERO_OFF + NS * WXROW;
constexpr int WLDS = WY_OFF + WYSLOTS * WYST;

// 16-byte chunk swizzles of bf16 m-major rows for the transposing fragment reads (a read
// covers rows {0-3, 8-11} (+4) x two chunks): 64-B rows (4 chunks) move rows 8-15 to the
// other 32-B half; 128-B rows as conv.hip's wgrad_kernel.  Both stay inside the row.
__device__ __forceinline__ int wsz64(int r) { return 2 * ((r >> 3) & 1); }
__device__ __forceinline__ int wsz128(int r) { return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1); }

// transposed fragment (8 consecutive K rows of one 16-column group) from an m-major image
template <int ROWB>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int r0, int col) {
  const int ch = col >> 3, hb = (col & 7) * 2;
  const int r1 = r0 + 4;
  const int s0 = ROWB == 64 ? wsz64(r0) : wsz128(r0);
  const int s1 = ROWB == 64 ? wsz64(r1) : wsz128(r1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (LDS_AS bf16x4*)(img + r0 * ROWB + ((ch ^ s0) << 4) + hb));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (LDS_AS bf16x4*)(img + r1 * ROWB + ((ch ^ s1) << 4) + hb));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

struct LWG {
  int nb, Cs, Nd, d, K;
  int groups_per_split;
  uint32_t xbytes, ybytes;                  // operand sizes (buffer-resource ranges)
};

// DD = the dilation (4 or 8), a template constant: the sub-group / class digit arithmetic of
// every plane's DMA bases then divides by constants (run-time divisions by d, d^2 and d^3 / 32
// were ~35 scalar instructions each, several per plane)
template <int DD>
__global__ __launch_bounds__(NTHR) void lattice_wgrad_kernel(LWG g, const u16* __restrict__ src,
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
  constexpr int d = DD, E = S * d;
  const int gpn = d * d * d / NS;
  const int g0 = split * g.groups_per_split;
  const int nplane_out = g.groups_per_split * S;    // output planes of this block
  const int nstage = nplane_out * 8;                // 2 positions per stage
  const int64_t plane_vox = (int64_t)d * E * E;

  // sub s of group gi -> voxel of (plane z, position ty, tx) = a group-uniform part
  // (scalar, recomputed per stage / plane) + a per-lane sub part (constant: a group holds
  // 32 consecutive classes, so for d = 4 or 8 the sub's class digits never carry into the
  // group's, and the lane part is the same in every group)
  auto grp_vox = [&](int gi, int z, int ty, int tx) -> int64_t {
    const int n = gi / gpn, q = (gi % gpn) * NS;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    return (((int64_t)n * E + rz + d * z) * E + ry + d * ty) * E + rx + d * tx;
  };
  auto sub_part = [&](int s) -> int64_t {
    const int q = s;                                 // classes 0..31 of a 32-aligned group
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    return ((int64_t)rz * E + ry) * E + rx;
  };
  // X stream entry e = (group g0 + e / 4, plane e % 4) into slot e % 4: 4 instructions per
  // wave of 16 rows x 64 B (row = pos * 32 + sub)
  const int xrow_l = lane >> 2;
  // (round 5) both operands through buffer resources with 32-bit byte offsets (wgrad_ok
  // bounds the tensors): a scalar plane / stage part plus a constant lane part -- no 64-bit
  // lane addresses or generic-to-LDS casts in the stage loop
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)src, 0, (int)__builtin_amdgcn_readfirstlane(g.xbytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dy, 0, (int)__builtin_amdgcn_readfirstlane(g.ybytes), 0x00020000);
  const uint32_t lds0 = lds_addr_of(smem);
  uint32_t xlane[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = (wave * 4 + k) * 16 + xrow_l;
    const int pos = row / NS, sb = row % NS;
    const int chunk = (lane & 3) ^ wsz64(row);
    xlane[k] = (uint32_t)(((sub_part(sb) + (int64_t)d * (pos / S) * E + d * (pos % S)) * g.Cs +
                           ci0 + chunk * 8) * 2);
  }
  auto issue_x = [&](int e) {
    const int gi = g0 + e / S, pz = e % S;
    const uint32_t slot = lds0 + (uint32_t)(((unsigned)e % WXSLOTS) * WPLANE);
    const uint32_t zb = (uint32_t)(grp_vox(gi, pz, 0, 0) * g.Cs * 2);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      buf_lds16_asm(zb + xlane[k], rsx, slot + (uint32_t)((wave * 4 + k) * 1024));
  };
  // dY stage s = (output plane s / 8, positions 2*(s%8), +1): one instruction per wave of
  // 8 rows x 128 B (row = q * 32 + sub; position 2m + q = (ty, tx) = (m / 2, 2 (m % 2) + q))
  const int yrow = wave * 8 + (lane >> 3);
  const int ychunk = (lane & 7) ^ wsz128(yrow);
  const uint32_t ylane = (uint32_t)(((sub_part(yrow % NS) + (int64_t)d * (yrow / NS)) * g.Nd +
                                     co0 + ychunk * 8) * 2);


  const int cf = wave & 1, tg = wave >> 1;          // ci half, tap group
  const int t0 = tg * 7, nt = tg == 3 ? 6 : 7;
  const int lk = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int rsel = 8 * lk + q4;                     // this lane's K rows r, r + 4 of a step
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 7; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Fragment addressing, hoisted out of the K loop.  Per lane: the byte offsets of its two
  // transposed 8-byte reads (rows rsel and rsel + 4) in a dY image (4 channel groups, two
  // positions) and in an X position block.  Per wave (scalar): each of its taps' offset in
  // the X ring relative to (plane tz, position) and the positions / planes where that tap
  // is inside the sub-lattice.  X entry e sits in slot e % 4 and a sub group's planes are
  // entries 4g..4g+3, so plane z of the current group is slot z.
  auto tr_off = [&](int rowb, int r, int col, int sw) -> uint32_t {
    return (uint32_t)(r * rowb + ((((col >> 3) ^ sw)) << 4) + (col & 7) * 2);
  };
  // (the second position's rows are NS further: same swizzle, a constant offset)
  uint32_t ya_lo[4], ya_hi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + 4 * p4;
    ya_lo[i] = tr_off(WYROW, rsel, col, wsz128(rsel));
    ya_hi[i] = tr_off(WYROW, rsel + 4, col, wsz128(rsel + 4));
  }
  const uint32_t xb_lo = tr_off(WXROW, rsel, cf * 16 + 4 * p4, wsz64(rsel));
  const uint32_t xb_hi = tr_off(WXROW, rsel + 4, cf * 16 + 4 * p4, wsz64(rsel + 4));
  auto tr8 = [](const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)p);
  };
  // dY of stage (plane o, pair m) into ring slot sl
  auto issue_y_at = [&](int64_t plane_vox0, int m, int sl) {
    const uint32_t base =
        (uint32_t)((plane_vox0 + (int64_t)d * (m / 2) * E + 2 * d * (m % 2)) * g.Nd * 2);
    buf_lds16_asm(base + ylane, rsy, lds0 + (uint32_t)(WY_OFF + sl * WYST + wave * 1024));
  };
  auto plane_y0 = [&](int o) -> int64_t { return grp_vox(g0 + o / S, o % S, 0, 0); };

  // prologue: X entries 0 and 1, dY stages 0 and 1
  issue_x(0);
  issue_x(1);
  issue_y_at(plane_y0(0), 0, 0);
  issue_y_at(plane_y0(0), 1, 1);

  // The wave's tap group TG is a compile-time constant of its code path, and so is each
  // K step's position: a tap whose (y, x) shift leaves the sub-lattice at that position has
  // neither fragment reads nor MFMAs (no branches in the MFMA stream, 31 % fewer X reads);
  // nor has a tap whose z shift leaves it (first / last plane of a sub group).
  struct WFr { bf16x8 a[4], b[7]; };
  auto run = [&](auto tgc) {
    constexpr int TG = decltype(tgc)::value;
    constexpr int NT = TG == 3 ? 6 : 7;
    auto yx_on = [](auto kc, auto posc) constexpr {
      constexpr int K = decltype(kc)::value, POS = decltype(posc)::value;
      constexpr int t = TG * 7 + K;
      constexpr int ky = (t / 3) % 3 - 1, kx = t % 3 - 1;
      constexpr int py = POS / S + ky, px = POS % S + kx;
      return K < NT && py >= 0 && py < S && px >= 0 && px < S;
    };
    // the plane's z position in its sub group is a compile-time constant too, so a tap
    // whose z shift leaves the sub-lattice has no reads and no MFMAs either (the plane loop
    // is unrolled by the 4 planes of a sub group)
    auto z_on = [](auto kc, auto tzc) constexpr {
      constexpr int K = decltype(kc)::value, TZ = decltype(tzc)::value;
      constexpr int kz = (TG * 7 + K) / 9 - 1;
      return TZ + kz >= 0 && TZ + kz < S;
    };
    auto kread = [&](const char* yimg, auto qc, auto posc, auto tzc, WFr& f) {
      constexpr int Q = decltype(qc)::value, POS = decltype(posc)::value;
      constexpr int TZ = decltype(tzc)::value;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f.a[i] = __builtin_shufflevector(tr8(yimg + Q * NS * WYROW + ya_lo[i]),
                                         tr8(yimg + Q * NS * WYROW + ya_hi[i]), 0, 1, 2, 3, 4,
                                         5, 6, 7);
      auto one = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (yx_on(kc, posc) && z_on(kc, tzc)) {
          constexpr int t = TG * 7 + K;
          constexpr int dk = (t / 9 - 1) * WPLANE + (((t / 3) % 3 - 1) * S + t % 3 - 1) * NS * WXROW +
                             POS * NS * WXROW;
          const char* img = smem + TZ * WPLANE + dk;
          f.b[K] = __builtin_shufflevector(tr8(img + xb_lo), tr8(img + xb_hi), 0, 1, 2, 3, 4, 5,
                                           6, 7);
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
    auto kmma = [&](const WFr& f, auto posc, auto tzc) {
      auto one = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (yx_on(kc, posc) && z_on(kc, tzc)) {
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

    // plane o of the block's stream; tzc = its z position in the sub group
    auto plane = [&](int o, auto tzc) {
      const bool xnow = o + 2 < nplane_out;         // X plane o + 2 issued at stage 0
      const int64_t y_here = plane_y0(o);
      const int64_t y_next = o + 1 < nplane_out ? plane_y0(o + 1) : y_here;
      const int sl0 = (int)((unsigned)(o * 8) % WYSLOTS);   // (unsigned: no signed fixup)
      auto stage = [&](auto mc) {
        constexpr int M = decltype(mc)::value;
        const int sl = (int)((unsigned)(sl0 + M) % WYSLOTS);
        // dY of this stage landed (issued two stages ago); younger: the next stage's dY and,
        // at stages 1 and 2, the X plane issued at stage 0 right after stage 2's dY
        const bool last = o + 1 == nplane_out && M == 7;
        if ((M == 1 || M == 2) && xnow) wait_vm_lgkm0<5>();
        else if (last) wait_vm_lgkm0<0>();
        else wait_vm_lgkm0<1>();
        raw_barrier();
        if (M < 6) issue_y_at(y_here, M + 2, (int)((unsigned)(sl + 2) % WYSLOTS));
        else if (o + 1 < nplane_out) issue_y_at(y_next, M - 6, (int)((unsigned)(sl + 2) % WYSLOTS));
        if (M == 0 && xnow) issue_x(o + 2);
        // (opaque, defined after the barrier, so the fragment addresses of later stages are
        // not computed early and held in VGPRs)
        int yoff = WY_OFF + sl * WYST;
        asm volatile("" : "+s"(yoff));
        const char* yimg = smem + yoff;
        WFr f0, f1;
        kread(yimg, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * M>{}, tzc,
              f0);
        kread(yimg, std::integral_constant<int, 1>{}, std::integral_constant<int, 2 * M + 1>{},
              tzc, f1);
        kmma(f0, std::integral_constant<int, 2 * M>{}, tzc);
        kmma(f1, std::integral_constant<int, 2 * M + 1>{}, tzc);
      };
      stage(std::integral_constant<int, 0>{});
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      stage(std::integral_constant<int, 4>{});
      stage(std::integral_constant<int, 5>{});
      stage(std::integral_constant<int, 6>{});
      stage(std::integral_constant<int, 7>{});
    };
    for (int og = 0; og < nplane_out; og += S) {    // a sub group's 4 planes
      plane(og + 0, std::integral_constant<int, 0>{});
      plane(og + 1, std::integral_constant<int, 1>{});
      plane(og + 2, std::integral_constant<int, 2>{});
      plane(og + 3, std::integral_constant<int, 3>{});
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

// MMAD_LATTICE: 1 (default) where the tiles fill the CUs, 2 at any size, 0 off;
// mmad_set_kernel_variant("lattice", v) overrides it at run time
std::atomic<int> g_lattice_mode{-1};
int lattice_mode() {
  int v = g_lattice_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_LATTICE");
    int expect = -1;
    g_lattice_mode.compare_exchange_strong(expect, e ? atoi(e) : 1);
    v = g_lattice_mode.load(std::memory_order_relaxed);
  }
  return v;
}

}  // namespace

namespace mmad_lattice {

int64_t tiles(const mmad_patch::Geo& q);

int set_mode(int v) {
  const int prev = lattice_mode();
  if (v >= 0) g_lattice_mode.store(v, std::memory_order_relaxed);
  return prev;
}

// a 4d^3 grid (every class a full 4^3 sub-lattice) or, with MMAD_LATTICE_RAGGED (default
// on), a ragged one: same extents in and out, up to 4 x 4 positions per class plane
static bool exact(const mmad_patch::Geo& q) {
  const int E = S * q.dd;
  return q.Ds == E && q.Hs == E && q.Ws == E && q.Dd == E && q.Hd == E && q.Wd == E;
}
static int ragged_mode() {
  static const int v = [] {
    const char* e = getenv("MMAD_LATTICE_RAGGED");
    return e ? atoi(e) : 1;
  }();
  return v;
}
static bool ragged(const mmad_patch::Geo& q) {
  const int d = q.dd;
  return !exact(q) && q.Ds == q.Dd && q.Hs == q.Hd && q.Ws == q.Wd &&
         (q.Hs + d - 1) / d <= S && (q.Ws + d - 1) / d <= S &&
         (int64_t)q.Ds * q.Hs * q.Ws * q.Cs * 2 < (int64_t(1) << 31);
}
static int planes(const mmad_patch::Geo& q) {
  return exact(q) ? S : (q.Ds + q.dd - 1) / q.dd;
}

bool ok(const mmad_patch::Geo& q) {
  if (mmad_lattice5::ok(q)) return true;          // 5d^3 grids (lattice5.hip)
  if (lattice_mode() <= 0) return false;
  const int d = q.dd;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dh != d || q.dw != d || d < 2) return false;
  if (q.pd != d || q.ph != d || q.pw != d) return false;
  const int E = S * d;
  if (!exact(q) && !(ragged_mode() > 0 && ragged(q))) return false;
  if ((d * d * d) % NS) return false;
  if (q.Cs % KC || q.Nd % 64 || q.Kpad != 27 * q.Cs) return false;
  // 32-bit per-lane DMA offsets (lattice_conv_kernel): one sample's volume, the packed weights
  if ((int64_t)E * E * E * q.Cs >= (int64_t(1) << 31) ||
      (int64_t)q.Nd * q.Kpad >= (int64_t(1) << 31))
    return false;
  // one 512-thread block per CU: tiles too few for the CUs even at 64 channels leave the
  // row-gather implicit GEMM (more, smaller blocks) ahead
  if (lattice_mode() == 1 && mmad_lattice::tiles(q) * (q.Nd / 64) < 256) return false;
  return (int64_t)q.nb * E * E * E * q.Cs < (int64_t(1) << 40);
}

int64_t tiles(const mmad_patch::Geo& q) {
  if (mmad_lattice5::ok(q)) return mmad_lattice5::tiles(q);
  if (exact(q) && mmad_lattice_zp::ok(q)) return mmad_lattice_zp::tiles(q);
  return (int64_t)q.nb * q.dd * q.dd * q.dd / NS * planes(q);
}


int wgrad_splits(const mmad_patch::Geo& q) {
  const int64_t tiles = (int64_t)(q.Cs / KC) * (q.Nd / 64);
  const int ngroups = q.nb * q.dd * q.dd * q.dd / NS;
  int sp = 1;
  while (tiles * sp < 256 && ngroups % (sp * 2) == 0) sp *= 2;
  return sp;
}

// MMAD_LATTICE_WGRAD=0 routes layer4's wgrad back to the row-gather wgrad_kernel (A/B).
// At 2 waves per SIMD the per-stage fragment reads and barrier are not hidden, so this
// kernel is only ~2 % ahead of wgrad_kernel (4 blocks of 4 waves per CU) in the step:
// 4.25-4.30 vs 4.32 ms (MI355X, batch 8, interleaved A/B); l4c2 380 + 20 us (isolated)
int lattice_wgrad_mode() {
  static const int v = [] {
    const char* e = getenv("MMAD_LATTICE_WGRAD");
    return e ? atoi(e) : 1;
  }();
  return v;
}

bool wgrad_ok(const mmad_patch::Geo& q) {
  if (mmad_lattice5::wgrad_ok(q)) return true;    // 5d^3 grids (lattice5.hip)
  if (lattice_mode() <= 0 || lattice_wgrad_mode() <= 0) return false;
  const int d = q.dd;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dh != d || q.dw != d || d < 2) return false;
  if (q.pd != d || q.ph != d || q.pw != d) return false;
  const int E = S * d;
  if (q.Ds != E || q.Hs != E || q.Ws != E || q.Dd != E || q.Hd != E || q.Wd != E) return false;
  if ((d * d * d) % NS || q.Cs % KC || q.Nd % 64 || (d != 4 && d != 8)) return false;
  const int64_t tiles = (int64_t)(q.Cs / KC) * (q.Nd / 64) * wgrad_splits(q);
  if (lattice_mode() == 1 && tiles < 256) return false;
  // 32-bit byte offsets into X and dY (buffer resources)
  return (int64_t)q.nb * E * E * E * std::max(q.Cs, q.Nd) * 2 < (int64_t(1) << 31);
}

int64_t wgrad_workspace(const mmad_patch::Geo& q) {
  if (mmad_lattice5::wgrad_ok(q)) return mmad_lattice5::wgrad_workspace(q);
  return (int64_t)wgrad_splits(q) * q.Nd * 27 * q.Cs * 4;
}

int wgrad(const mmad_patch::Geo& q, const void* x, const void* dy, float* ws, int* splits,
          void* stream) {
  if (mmad_lattice5::wgrad_ok(q)) return mmad_lattice5::wgrad(q, x, dy, ws, splits, stream);
  if (!wgrad_ok(q)) return MMAD_EUNSUPPORTED;
  static const bool attr =
      hipFuncSetAttribute((const void*)lattice_wgrad_kernel<4>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, WLDS) == hipSuccess &&
      hipFuncSetAttribute((const void*)lattice_wgrad_kernel<8>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, WLDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  const int sp = wgrad_splits(q);
  LWG g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.d = q.dd; g.K = 27 * q.Cs;
  g.groups_per_split = q.nb * q.dd * q.dd * q.dd / NS / sp;
  const int64_t vox = (int64_t)q.nb * S * q.dd * S * q.dd * S * q.dd;
  g.xbytes = (uint32_t)(vox * q.Cs * 2);
  g.ybytes = (uint32_t)(vox * q.Nd * 2);
  const int64_t nblk = (int64_t)(q.Cs / KC) * (q.Nd / 64) * sp;
  if (q.dd == 4)
    hipLaunchKernelGGL(lattice_wgrad_kernel<4>, dim3((unsigned)nblk), dim3(NTHR), WLDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else
    hipLaunchKernelGGL(lattice_wgrad_kernel<8>, dim3((unsigned)nblk), dim3(NTHR), WLDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  *splits = sp;
  return launch_status();
}

int fwd(const mmad_patch::Geo& q, const void* src, const void* wp, const float* bias,
        void* dst, float* stats, void* stream) {
  if (mmad_lattice5::ok(q)) return mmad_lattice5::fwd(q, src, wp, bias, dst, stats, stream);
  if (!mmad_lattice::ok(q)) return MMAD_EUNSUPPORTED;
  const bool rag = !exact(q);
  if (!rag && mmad_lattice_zp::ok(q))
    return mmad_lattice_zp::fwd(q, src, wp, bias, dst, stats, stream);
  static const bool attr =
      hipFuncSetAttribute((const void*)lattice_conv_kernel<4, false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
      hipFuncSetAttribute((const void*)lattice_conv_kernel<2, false>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
      hipFuncSetAttribute((const void*)lattice_conv_kernel<4, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess &&
      hipFuncSetAttribute((const void*)lattice_conv_kernel<2, true>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  // 128-channel tiles (4 MFMA columns per wave) when they give every CU a block, else 64
  const bool wide = q.Nd % BNL == 0 && mmad_lattice::tiles(q) * (q.Nd / BNL) >= 256;
  LG g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.Kpad = q.Kpad; g.d = q.dd;
  g.ngroups = q.nb * q.dd * q.dd * q.dd / NS;
  g.nbn = q.Nd / (wide ? BNL : 64);
  g.nchunk = q.Cs / KC;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  static const int prio = [] {
    const char* e = getenv("MMAD_SETPRIO");
    return e ? atoi(e) : 0;
  }();
  g.prio = prio;
  g.D = q.Ds; g.H = q.Hs; g.W = q.Ws;
  g.nz = planes(q);
  const int64_t nblk = (int64_t)g.ngroups * g.nz * g.nbn;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(NTHR), LDS_BYTES, as_stream(stream), g,
                       (const u16*)src, (const u16*)wp, bias, (u16*)dst, stats);
  };
  if (wide) rag ? go(lattice_conv_kernel<4, true>) : go(lattice_conv_kernel<4, false>);
  else rag ? go(lattice_conv_kernel<2, true>) : go(lattice_conv_kernel<2, false>);
  return launch_status();
}

}  // namespace mmad_lattice
