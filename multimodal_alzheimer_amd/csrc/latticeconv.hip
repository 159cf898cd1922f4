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
//    stage, 3-slot ring, two stages in flight): per wave one 1 KiB LDS-DMA per stage where
//    the row-gather implicit GEMM (conv.hip) issues eight;
//  * the plane the next channel chunk needs is loaded as soon as the current chunk's last
//    tap on that plane has run (the loop walks taps plane by plane), 18 stages ahead;
//  * 8 waves = 4 x 2 wave tiles of 128 rows x 64 channels; wave wm takes the positions of
//    one diagonal of the 4 x 4 plane, (t, (t + wm) & 3), so every wave loses the same number
//    of fragments to padding on every tap (a row of the plane would idle the edge waves);
//  * 64-byte patch / weight rows (32 channels), 16-byte chunks swizzled by 3*((row>>3)&1)
//    (conflict-free ds_read_b128 fragment reads, as conv.hip's 64-byte variant);
//  * epilogue as the implicit GEMM: bias, BN partial sums (one row per tile), optional
//    residual + ReLU (eval-mode fused BN), bf16 tile transposed through LDS into 16-byte
//    channel-vector stores; tiles walk the XCDs in contiguous ranges (the 4 channel tiles
//    and neighbouring planes of one sub group share an L2).
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
constexpr int NSTL = 2;                   // weight ring slots
constexpr int RING_OFF = 3 * PLANE;
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
};

__device__ __forceinline__ int swz(int row) { return 3 * ((row >> 3) & 1); }

struct Frags {
  bf16x8 b[4];
  bf16x8 a[4][2];
};

// position i of wave diagonal WM, shifted by tap (KY, KX), inside the 4 x 4 plane
template <int WM, int KY, int KX>
__device__ constexpr bool tap_ok(int i) {
  return i + KY >= 0 && i + KY < S && ((i + WM) & 3) + KX >= 0 && ((i + WM) & 3) + KX < S;
}

template <int WM, int KY, int KX>
__device__ __forceinline__ void read_tap(const char* bsl, const char* apl, Frags& f) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
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

template <int WM, int KY, int KX>
__device__ __forceinline__ void mma_tap(f32x4 (&acc)[8][4], const Frags& f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (tap_ok<WM, KY, KX>(i)) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#ifndef LAT_NO_MFMA
          acc[i * 2 + h][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i][h], f.b[j], acc[i * 2 + h][j], 0, 0, 0);
#endif
        }
    }
  }
}

template <int WM, int KY>
__device__ __forceinline__ void stage_body(f32x4 (&acc)[8][4], const char* bsl, const char* apl) {
  Frags f0, f1;
  read_tap<WM, KY, -1>(bsl, apl, f0);
  read_tap<WM, KY, 0>(bsl, apl, f1);
  mma_tap<WM, KY, -1>(acc, f0);
  read_tap<WM, KY, 1>(bsl, apl, f0);
  mma_tap<WM, KY, 0>(acc, f1);
  mma_tap<WM, KY, 1>(acc, f0);
}

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
  const int tz = t2 % S, gid = t2 / S;
  const int d = g.d, E = S * d;                     // grid extent per dimension
  const int gpn = d * d * d / NS;                   // sub groups per sample
  const int n = gid / gpn, q0 = (gid % gpn) * NS;   // sample, first class of the group
  const int n0 = nt * BNL;
  const int64_t plane_vox = (int64_t)d * E * E;     // voxel step between planes tz, tz+1

  // ---- patch DMA: plane slot p <- absolute plane tz - 1 + p of chunk cc (32 rows per
  // wave: 4 instructions of 16 rows x 64 B); every row is a real voxel (no halo rows)
  const int lrow = lane >> 2;
  int64_t pvox[4];
  int pchunk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = (wave * 4 + k) * 16 + lrow;
    const int pos = row / NS, s = row % NS;
    const int q = q0 + s;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    const int ty = pos / S, tx = pos % S;
    pvox[k] = (((int64_t)n * E + rz) * E + ry + d * ty) * E + rx + d * tx;
    pchunk[k] = (lane & 3) ^ swz(row);
  }
  auto issue_plane = [&](int p, int cc) {
    const int64_t zoff = (int64_t)(tz - 1 + p) * plane_vox;
    char* pb = smem + p * PLANE;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u16* a = src + (pvox[k] + zoff) * g.Cs + cc * KC + pchunk[k] * 8;
      glds16_asm(a, lds_addr_of(pb + (wave * 4 + k) * 1024));
    }
  };
  // ---- weight DMA: stage (chunk cc, first tap t) into ring slot sl: 3 consecutive taps
  // (one kx row), 16 rows per wave per tap
  const int brow = wave * 16 + lrow;
  const u16* wrow = wgt + (int64_t)(n0 + brow) * g.Kpad + (((lane & 3) ^ swz(brow)) * 8);
  auto issue_b = [&](int cc, int t, int sl) {
#pragma unroll
    for (int k = 0; k < TPS; ++k)
      glds16_asm(wrow + (t + k) * g.Cs + cc * KC,
                 lds_addr_of(ring + sl * BSLOT + k * BTAP + wave * 1024));
  };

  // stage list: chunk-major, then the valid kz planes, then ky; a stage runs kx = -1, 0, 1
  const int kz0 = tz == 0 ? 0 : -1, kz1 = tz == S - 1 ? 0 : 1;
  const int nspc = (kz1 - kz0 + 1) * 3;             // stages per chunk
  const int nstage = g.nchunk * nspc;
  auto stage_of = [&](int s, int& cc, int& kz, int& ky) {
    cc = s / nspc;
    const int r = s - cc * nspc;
    kz = kz0 + r / 3;
    ky = r % 3 - 1;
  };
  // a plane slot is reloaded (next chunk) at the stage after its last stage of this chunk
  auto plane_due = [&](int s, int& p, int& cc) -> bool {
    if (s < 1) return false;
    const int c = (s - 1) / nspc, r = (s - 1) - c * nspc;
    if (r % 3 != 2 || c + 1 >= g.nchunk) return false;
    p = kz0 + r / 3 + 1;
    cc = c + 1;
    return true;
  };

  // wave tiles: wm -> diagonal positions (t, (t + wm) & 3), wn -> 64 output channels
  const int wm = wave & 3, wn = wave >> 2;
  const int lr = lane & 15, lk = lane >> 4;
  const uint32_t a_lane = lr * RBL + ((lk ^ swz(lr)) << 4);
  const uint32_t b_lane = (wn * 64 + lr) * RBL + ((lk ^ swz(lr)) << 4);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage_w = [&](int s, int& cc, int& t) {       // packed-weight tap of stage s, kx = -1
    int kz, ky;
    stage_of(s, cc, kz, ky);
    t = (kz + 1) * 9 + (ky + 1) * 3;
  };
  // prologue: the chunk-0 planes, weights of stage 0
  for (int p = 0; p < 3; ++p) {
    const int kz = p - 1;
    if (kz >= kz0 && kz <= kz1) issue_plane(p, 0);
  }
  {
    int cc, t;
    stage_w(0, cc, t);
    issue_b(cc, t, 0);
  }
  // Main loop, compiled once per wave diagonal WM with the three ky stages of a (chunk,
  // kz) group unrolled, so every padding test in the stage bodies is a compile-time
  // constant: no branch sits between a fragment read and its MFMA, and the next tap's reads
  // stay in flight during each tap's MFMAs.
  bool plane_prev = false;                          // a plane was issued at stage s-1
  auto one_stage = [&](int s) {
    // B(s) (issued at stage s-1) must have landed; a plane issued after it may still fly
    if (plane_prev) wait_vm_lgkm0<4>();
    else wait_vm_lgkm0<0>();
    raw_barrier();
    plane_prev = false;
#ifndef LAT_NO_B
    if (s + 1 < nstage) {
      int cc, t;
      stage_w(s + 1, cc, t);
      issue_b(cc, t, (s + 1) % NSTL);
    }
#endif
    int p, pc;
    if (plane_due(s, p, pc)) {
      issue_plane(p, pc);
      plane_prev = true;
    }
  };
  auto run = [&](auto wmc) {
    constexpr int WM = decltype(wmc)::value;
    const int ngrp = nstage / 3;                    // (chunk, kz) groups
    for (int g2 = 0; g2 < ngrp; ++g2) {
      const int kz = kz0 + g2 % (kz1 - kz0 + 1);
      const char* apl = smem + (kz + 1) * PLANE + a_lane;
      const int s0 = g2 * 3;
      one_stage(s0);
      stage_body<WM, -1>(acc, ring + (s0 % NSTL) * BSLOT + b_lane, apl);
      one_stage(s0 + 1);
      stage_body<WM, 0>(acc, ring + ((s0 + 1) % NSTL) * BSLOT + b_lane, apl);
      one_stage(s0 + 2);
      stage_body<WM, 1>(acc, ring + ((s0 + 2) % NSTL) * BSLOT + b_lane, apl);
    }
  };
  switch (wm) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }
  __syncthreads();                                  // patch / ring reused by the epilogue

  // ---- epilogue: tile row r = pos * NS + sub; acc[i*2+h][j][e] is row
  // (pos_i * NS + h*16 + lk*4 + e), column wn*64 + j*16 + lr
  auto dst_vox = [&](int row) -> int64_t {
    const int pos = row / NS, s = row % NS;
    const int q = q0 + s;
    const int rz = q / (d * d), ry = (q / d) % d, rx = q % d;
    const int ty = pos / S, tx = pos % S;
    return (((int64_t)n * E + rz + d * tz) * E + ry + d * ty) * E + rx + d * tx;
  };
  u16* ctile = reinterpret_cast<u16*>(smem);
  float cs[4], cq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    cs[j] = 0.f;
    cq[j] = 0.f;
    const int col = wn * 64 + j * 16 + lr;
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
          cs[j] += v;
          cq[j] += v * v;
        }
    }
  }
  __syncthreads();
  constexpr int CPR = BNL / 8;
#pragma unroll
  for (int hh = 0; hh < PL * CPR / NTHR; ++hh) {
    const int qd = tid + NTHR * hh;
    const int row = qd / CPR, c8 = qd % CPR;
    const int64_t o = dst_vox(row) * g.Nd + n0 + c8 * 8;
    u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) + row * CROW +
                                              c8 * 16);
    if (g.res != nullptr || g.relu) v = epi_res_relu(v, g.res ? g.res + o : nullptr, g.relu);
    *reinterpret_cast<u32x4*>(dst + o) = v;
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(smem + PL * CROW);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] += __shfl_xor(cs[j], 16, 64);
      cs[j] += __shfl_xor(cs[j], 32, 64);
      cq[j] += __shfl_xor(cq[j], 16, 64);
      cq[j] += __shfl_xor(cq[j], 32, 64);
    }
    if (wm > 0 && lk == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + lr;
        red[(wm - 1) * 2 * BNL + col] = cs[j];
        red[(wm - 1) * 2 * BNL + BNL + col] = cq[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lk == 0) {
      const int mt = gid * S + tz;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + lr;
        float ss = cs[j], qs = cq[j];
        for (int w = 1; w < 4; ++w) {              // fixed order: deterministic
          ss += red[(w - 1) * 2 * BNL + col];
          qs += red[(w - 1) * 2 * BNL + BNL + col];
        }
        stats[((int64_t)mt * 2) * g.Nd + n0 + col] = ss;
        stats[((int64_t)mt * 2 + 1) * g.Nd + n0 + col] = qs;
      }
    }
  }
}

int lattice_mode() {
  static const int v = [] { const char* e = getenv("MMAD_LATTICE"); return e ? atoi(e) : 1; }();
  return v;
}

}  // namespace

namespace mmad_lattice {

int64_t tiles(const mmad_patch::Geo& q);

bool ok(const mmad_patch::Geo& q) {
  if (lattice_mode() <= 0) return false;
  const int d = q.dd;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dh != d || q.dw != d || d < 2) return false;
  if (q.pd != d || q.ph != d || q.pw != d) return false;
  const int E = S * d;
  if (q.Ds != E || q.Hs != E || q.Ws != E || q.Dd != E || q.Hd != E || q.Wd != E) return false;
  if ((d * d * d) % NS) return false;
  if (q.Cs % KC || q.Nd % BNL || q.Kpad != 27 * q.Cs) return false;
  // one 512-thread block per CU: below 256 tiles the row-gather implicit GEMM (more, smaller
  // blocks) is as fast (layer4.0.conv1 dgrad, 128 tiles: 237 vs 232 us)
  if (lattice_mode() == 1 && tiles(q) * (q.Nd / BNL) < 256) return false;
  return (int64_t)q.nb * E * E * E * q.Cs < (int64_t(1) << 40);
}

int64_t tiles(const mmad_patch::Geo& q) {
  return (int64_t)q.nb * q.dd * q.dd * q.dd / NS * S;
}

int fwd(const mmad_patch::Geo& q, const void* src, const void* wp, const float* bias,
        void* dst, float* stats, void* stream) {
  if (!mmad_lattice::ok(q)) return MMAD_EUNSUPPORTED;
  static const bool attr = hipFuncSetAttribute((const void*)lattice_conv_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               LDS_BYTES) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  LG g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.Kpad = q.Kpad; g.d = q.dd;
  g.ngroups = q.nb * q.dd * q.dd * q.dd / NS;
  g.nbn = q.Nd / BNL;
  g.nchunk = q.Cs / KC;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  const int64_t nblk = (int64_t)g.ngroups * S * g.nbn;
  hipLaunchKernelGGL(lattice_conv_kernel, dim3((unsigned)nblk), dim3(NTHR), LDS_BYTES,
                     as_stream(stream), g, (const u16*)src, (const u16*)wp, bias, (u16*)dst,
                     stats);
  return launch_status();
}

}  // namespace mmad_lattice
