// Residue-class convolution for MedicalNet's layer3 convs (3x3x3, dilation 2, padding 2,
// stride 1; 128/256 channels on the 16^3 grid of a 128^3 input, reached from
// pkg/models/mri_models/anat_cnn.py:29-31), forward and -- over reversed taps -- input
// gradient, gfx950 bf16.
//
// The dilation-2 conv on a 16^3 grid is 8 independent dense 3^3 convs (padding 1), one per
// residue class (rz, ry, rx) in {0,1}^3, each on an 8^3 sub-lattice (latticeconv.hip does
// the same for layer4's 4^3 sub-lattices).  Here a tile is one sample's 8 classes over one
// whole z-plane of the sub-lattice: 64 positions x 8 classes = 512 GEMM rows
// (position-major), so the tile needs no y/x halo -- a y or x shift that leaves the plane
// is padding.  A stage is one input plane tz+kz (32 input channels, 32 KiB) and its 9 taps'
// weights (64 output channels x 32 input channels = 4 KiB a tap), double-buffered: the next
// stage's plane and weights load during this stage's MFMAs.
//  * a 16-row MFMA fragment is 2 x-neighbouring positions x 8 classes: a y shift out of
//    the plane drops the whole fragment (compile-time per wave row, skipped); an x shift
//    out of the plane drops half the lanes, which then read a zero row (one select);
//  * 8 waves = 4 x 2 wave tiles of 128 rows (two y rows of the plane) x 32 channels;
//  * the loop walks (chunk, kz) stages with ky, kx = -1, 0, 1 inside, the next tap's
//    fragment reads in flight during each tap's MFMAs, one barrier per stage;
//  * epilogue as the implicit GEMM: bias, BN partial sums (one row per tile), optional
//    residual + ReLU, bf16 tile transposed through LDS into 16-byte channel stores.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "bnsum.h"
#include "common.h"
#include "patchconv.h"

namespace {

constexpr int S8 = 8;                      // sub-lattice extent
constexpr int NC = 8;                      // classes (d^3, d = 2)
constexpr int PL8 = S8 * S8 * NC;          // rows per plane (512)
constexpr int RB8 = 64;                    // bytes per row (32 channels)
constexpr int KC8 = RB8 / 2;
constexpr int PLANE8 = PL8 * RB8;          // 32 KiB
constexpr int BN8 = 64;                    // output channels per tile
constexpr int BTAP8 = BN8 * RB8;           // 4 KiB
// A stage is a whole kz plane of 9 taps (3 ky rows x 3 kx), streamed with its input plane
// through a 2-slot plane ring and a 2-slot weight ring (36 KiB a slot), so a tile runs
// nchunk * nkz stages with one barrier each.  Measured r03l8s9 in the config-2 step: the four
// layer3 launches 52.1 / 91.7 / 88.0 / 59.1 us with 3-tap stages -> 47.2 / 81.2 / 76.0 /
// 47.1 us; a software-pipelined 3-tap loop (the barrier between the kx = 0 and kx = +1 MFMAs,
// as latticezp.hip) measured 1-2 % slower than the 3-tap barrier-first loop (r03e); both
// removed.
constexpr int TPS8 = 9;
constexpr int BSLOT8 = TPS8 * BTAP8;       // 36 KiB
constexpr int NSL8 = 2;                    // weight slots
constexpr int NPL8 = 2;                    // plane slots
constexpr int RING8 = NPL8 * PLANE8;
constexpr int ZERO8 = RING8 + NSL8 * BSLOT8;
constexpr int MAIN8 = ZERO8 + RB8;
constexpr int CROW8 = BN8 * 2 + 16;
constexpr int EPI8 = PL8 * CROW8 + 7 * 2 * BN8 * 4;   // + partial sums of up to 7 wave rows
constexpr int LDS8 = MAIN8 > EPI8 ? MAIN8 : EPI8;
constexpr int NT8 = 512;

struct L8 {
  int nb, Cs, Nd, Kpad, nbn, nchunk;
  const u16* res;
  int relu;
  int D, H, W, nz;                         // ragged grids: extents, planes per class
  const u16* bny;                          // dgrad: BN-backward sums epilogue (bnsum.h)
  const float *bnsc, *bnsh, *bnmu, *bnis;
  float* bnparts;
};

__device__ __forceinline__ int swz8(int row) { return 3 * ((row >> 3) & 1); }

template <int TN, int NFR>
struct Fr8 {
  bf16x8 b[TN];
  bf16x8 a[NFR];
};

// fragment f of wave row WM (WR plane rows per wave): plane row ty = WR*WM + (f >> 2),
// x pair j = f & 3
template <int WM, int KY, int WR>
__device__ constexpr bool row_ok(int f) {
  return WR * WM + (f >> 2) + KY >= 0 && WR * WM + (f >> 2) + KY < S8;
}

// ao: this lane's row offset + chunk for an even (index 0) / odd (1) x shift; zlane: the
// lane's zero-row address; lhi: lane is the fragment's second x position
template <int TN, int WM, int KY, int KX, int WR>
__device__ __forceinline__ void read8(const char* bsl, const char* pl, const uint32_t (&ao)[2],
                                      const char* zp, bool lhi, Fr8<TN, 4 * WR>& f) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
    f.b[j] = *reinterpret_cast<const bf16x8*>(bsl + (KX + 1) * BTAP8 + j * 16 * RB8);
#pragma unroll
  for (int q = 0; q < 4 * WR; ++q) {
    if (row_ok<WM, KY, WR>(q)) {
      constexpr int dummy = 0;
      const int ty = WR * WM + (q >> 2) + KY + dummy, x0 = 2 * (q & 3) + KX;
      const int base = (ty * S8 + x0) * NC * RB8;       // may be -8 rows: lanes redirected
      const char* p = pl + base + ao[KX & 1];
      if (KX == -1 && (q & 3) == 0) p = lhi ? p : zp;
      if (KX == 1 && (q & 3) == 3) p = lhi ? zp : p;
      f.a[q] = *reinterpret_cast<const bf16x8*>(p);
    }
  }
}

template <int TN, int WM, int KY, int WR>
__device__ __forceinline__ void mma8(f32x4 (&acc)[4 * WR][TN], const Fr8<TN, 4 * WR>& f) {
#pragma unroll
  for (int q = 0; q < 4 * WR; ++q)
    if (row_ok<WM, KY, WR>(q)) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[q], f.b[j], acc[q][j], 0, 0, 0);
    }
}

template <int TN, int WM, int KY, int WR>
__device__ __forceinline__ void stage8(f32x4 (&acc)[4 * WR][TN], const char* bsl,
                                       const char* pl, const uint32_t (&ao)[2], const char* zp,
                                       bool lhi) {
  Fr8<TN, 4 * WR> f0, f1;
  read8<TN, WM, KY, -1, WR>(bsl, pl, ao, zp, lhi, f0);
  read8<TN, WM, KY, 0, WR>(bsl, pl, ao, zp, lhi, f1);
  mma8<TN, WM, KY, WR>(acc, f0);
  read8<TN, WM, KY, 1, WR>(bsl, pl, ao, zp, lhi, f0);
  mma8<TN, WM, KY, WR>(acc, f1);
  mma8<TN, WM, KY, WR>(acc, f0);
}

// TN = 16-column MFMA tiles per wave: 2 (64-channel tiles) or 1 (32 channels, for layers
// whose 64-channel tiling leaves CUs idle)
// RAG: ragged grids (any D x H x W with ceil(H / 2), ceil(W / 2) <= 8: the reference's
// 91 x 109 x 91 MNI volumes give 12 x 14 x 12 at layer3), as latticeconv.hip's RAG form:
// the positions / planes a class lacks are LDS-DMA'd as zeros (buffer resource, offset past
// its end) and skipped in the epilogue.
// WR = plane rows per wave: 2 (4 x 2 waves of 128 rows x 16 TN channels) or 1 (8 waves of
// 64 rows, one y row each, x 16 TN channels: the same tile width at TN doubled, 4 A + TN B
// fragment reads per tap instead of 8 + TN / 2 ... for the same MFMAs)
template <int TN, bool RAG, int WR>
__global__ __launch_bounds__(NT8) void lattice8_conv_kernel(L8 g, const u16* __restrict__ src,
                                                            const u16* __restrict__ wgt,
                                                            const float* __restrict__ bias,
                                                            u16* __restrict__ dst,
                                                            float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ring = smem + RING8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = tile % g.nbn;
  const int t2 = tile / g.nbn;
  const int NZ = RAG ? g.nz : S8;
  const int tz = t2 % NZ, n = t2 / NZ;
  constexpr int NFR = 4 * WR;                      // A fragments per wave
  constexpr int NWM = 8 / WR, NWN = WR;            // wave rows x wave columns
  constexpr int BW = 16 * TN * NWN;                // output channels of this tile
  const int n0 = nt * BW;
  constexpr int E = 2 * S8;                          // 16

  if (tid < RB8 / 16)
    *reinterpret_cast<u32x4*>(smem + ZERO8 + tid * 16) = u32x4{0u, 0u, 0u, 0u};

  // ---- patch DMA: plane slot p <- plane tz - 1 + p, chunk cc; 4 instructions per wave of
  // 16 rows x 64 B (row = pos * 8 + class)
  // (both grids through a per-sample buffer resource: a lane's 32-bit byte offset in the
  // sample, plus a wave-uniform plane / chunk part per stage -- no 64-bit lane addresses in
  // the stage loop)
  const int lrow = lane >> 2;
  int rzk[4];                                       // RAG: class z residue, -huge off-grid
  uint32_t pofs[4];                                 // byte offset in this sample
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = (wave * 4 + k) * 16 + lrow;
    const int pos = row >> 3, c = row & 7;
    const int ty = pos >> 3, tx = pos & 7;
    const int pch = (lane & 3) ^ swz8(row);
    if constexpr (RAG) {
      const int y = ((c >> 1) & 1) + 2 * ty, x = (c & 1) + 2 * tx;
      pofs[k] = (uint32_t)((((c >> 2) * g.H + y) * g.W + x) * g.Cs + pch * 8) * 2u;
      rzk[k] = (y < g.H && x < g.W) ? (c >> 2) : -(1 << 20);
    } else {
      const int v = ((c >> 2) * E + ((c >> 1) & 1) + 2 * ty) * E + (c & 1) + 2 * tx;
      pofs[k] = (uint32_t)(v * g.Cs + pch * 8) * 2u;
      rzk[k] = 0;
    }
  }
  const int64_t svox = RAG ? (int64_t)g.D * g.H * g.W : (int64_t)E * E * E;
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(src + (int64_t)n * svox * g.Cs), 0,
      (int)__builtin_amdgcn_readfirstlane((uint32_t)(svox * g.Cs * 2)), 0x00020000);
  // input plane tz - 1 + zr (zr = kz + 1) of channel chunk cc into plane slot p
  auto issue_plane_at = [&](int p, int zr, int cc) {
    char* pb = smem + p * PLANE8;
    if constexpr (RAG) {
      constexpr uint32_t OOB = 0x80000000u;         // >= any per-sample volume (ok())
      const int zp = 2 * (tz - 1 + zr);
      const uint32_t zoff = (uint32_t)(zp * g.H * g.W * g.Cs + cc * KC8) * 2u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = rzk[k] >= 0 && rzk[k] + zp >= 0 && rzk[k] + zp < g.D;
        buf_lds16_asm(ok ? pofs[k] + zoff : OOB, rsx, lds_addr_of(pb + (wave * 4 + k) * 1024));
      }
    } else {
      const uint32_t zoff = (uint32_t)(2 * (tz - 1 + zr) * E * E * g.Cs + cc * KC8) * 2u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t o = pofs[k];
        asm volatile("" : "+v"(o));                 // (opaque: no hoisted per-stage copies)
        buf_lds16_asm(o + zoff, rsx, lds_addr_of(pb + (wave * 4 + k) * 1024));
      }
    }
  };
  // ---- weight DMA, a stage's 9 taps: taps t0 .. t0 + 8 of chunk cc into slot sl; 9 * BW / 16
  // instructions of 16 rows x 64 B, WI9 per wave (surplus ones repeat the last: the same
  // bytes, same place); QB 16-row pieces per tap
  constexpr int QB = BW / 16;
  constexpr int NQ9 = 9 * BW / 16, WI9 = (NQ9 + 7) / 8;
  // (lane byte offsets into the packed weights, fixed; the stage adds (t0 Cs + cc KC8) * 2)
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)wgt, 0, (int)__builtin_amdgcn_readfirstlane((uint32_t)(g.Nd * g.Kpad * 2)),
      0x00020000);
  uint32_t wofs9[WI9];
#pragma unroll
  for (int h = 0; h < WI9; ++h) {
    const int q = min(wave + 8 * h, NQ9 - 1);
    const int row = (q % QB) * 16 + lrow;
    wofs9[h] = (uint32_t)((n0 + row) * g.Kpad + ((lane & 3) ^ swz8(row)) * 8 + (q / QB) * g.Cs) *
               2u;
  }
  auto issue_b9 = [&](int cc, int t0, int sl) {
    const uint32_t so = (uint32_t)(t0 * g.Cs + cc * KC8) * 2u;
#pragma unroll
    for (int h = 0; h < WI9; ++h) {
      const int q = min(wave + 8 * h, NQ9 - 1);
      uint32_t o = wofs9[h];
      asm volatile("" : "+v"(o));
      buf_lds16_asm(o + so, rsw, lds_addr_of(ring + sl * BSLOT8 + (q / QB) * BTAP8 + (q % QB) * 1024));
    }
  };
  const int kz0 = tz == 0 ? 0 : -1, kz1 = tz == NZ - 1 ? 0 : 1;
  const int nkz = kz1 - kz0 + 1;
  const int wm = wave % NWM, wn = wave / NWM;
  const int lr = lane & 15, lk = lane >> 4;
  const bool lhi = (lr >> 3) != 0;
  uint32_t ao[2];
  ao[0] = lr * RB8 + ((lk ^ swz8(lr)) << 4);
  ao[1] = lr * RB8 + ((lk ^ (3 - swz8(lr))) << 4);   // rows shifted by 8: the other swizzle
  const char* zp = smem + ZERO8 + (lk << 4);
  const uint32_t b_lane = (wn * 16 * TN + lr) * RB8 + ((lk ^ swz8(lr)) << 4);
  f32x4 acc[NFR][TN];
#pragma unroll
  for (int i = 0; i < NFR; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // stage e = (chunk c, kz): plane e and its 9 taps' weights land in slot e & 1,
  // issued at the top of stage e - 1 (after its barrier, when slot (e - 1) & 1 = (e + 1) & 1
  // has been read by every wave), so the top of stage e waits for everything issued
  auto run9 = [&](auto wmc) {
    constexpr int WM = decltype(wmc)::value;
    const int n9 = g.nchunk * nkz;
    issue_plane_at(0, kz0 + 1, 0);
    issue_b9(0, (kz0 + 1) * 9, 0);
    int e = 0;
    for (int c = 0; c < g.nchunk; ++c)
      for (int kzi = 0; kzi < nkz; ++kzi, ++e) {
        wait_vm_lgkm0<0>();
        raw_barrier();
        if (e + 1 < n9) {
          const int c1 = kzi + 1 < nkz ? c : c + 1, kz1 = kz0 + (kzi + 1 < nkz ? kzi + 1 : 0);
          issue_plane_at((e + 1) & 1, kz1 + 1, c1);
          issue_b9(c1, (kz1 + 1) * 9, (e + 1) & 1);
        }
        const char* pl = smem + (e & 1) * PLANE8;
        const char* bs = ring + (e & 1) * BSLOT8 + b_lane;
        stage8<TN, WM, -1, WR>(acc, bs, pl, ao, zp, lhi);
        stage8<TN, WM, 0, WR>(acc, bs + 3 * BTAP8, pl, ao, zp, lhi);
        stage8<TN, WM, 1, WR>(acc, bs + 6 * BTAP8, pl, ao, zp, lhi);
      }
  };
  auto dispatch = [&](auto wmc) {
    if constexpr (decltype(wmc)::value < NWM) run9(wmc);
  };
  switch (wm) {                                     // wave-uniform
    case 0: dispatch(std::integral_constant<int, 0>{}); break;
    case 1: dispatch(std::integral_constant<int, 1>{}); break;
    case 2: dispatch(std::integral_constant<int, 2>{}); break;
    case 3: dispatch(std::integral_constant<int, 3>{}); break;
    case 4: dispatch(std::integral_constant<int, 4>{}); break;
    case 5: dispatch(std::integral_constant<int, 5>{}); break;
    case 6: dispatch(std::integral_constant<int, 6>{}); break;
    default: dispatch(std::integral_constant<int, 7>{}); break;
  }
  __syncthreads();                                  // patch / ring reused by the epilogue

  // ---- epilogue: acc[q][j][e] is tile row (ty*8 + 2*(q&3))*8 + lk*4 + e with
  // ty = WR*wm + (q >> 2), column wn*16*TN + j*16 + lr
  // (RAG: -1 for a row outside the grid)
  auto dst_vox = [&](int row) -> int64_t {
    const int pos = row >> 3, c = row & 7;
    const int ty = pos >> 3, tx = pos & 7;
    if constexpr (RAG) {
      const int z = (c >> 2) + 2 * tz, y = ((c >> 1) & 1) + 2 * ty, x = (c & 1) + 2 * tx;
      if (z >= g.D || y >= g.H || x >= g.W) return -1;
      return (((int64_t)n * g.D + z) * g.H + y) * g.W + x;
    }
    return (((int64_t)n * E + (c >> 2) + 2 * tz) * E + ((c >> 1) & 1) + 2 * ty) * E + (c & 1) +
           2 * tx;
  };
  u16* ctile = reinterpret_cast<u16*>(smem);
  // RAG: which of this lane's 4 NFR accumulator rows lie inside the grid (bit q*4 + e)
  uint32_t vmask = 0xffffffffu;
  if constexpr (RAG) {
    vmask = 0;
#pragma unroll 1
    for (int b = 0; b < 4 * NFR; ++b) {
      const int q = b >> 2, e = b & 3;
      const int row = ((WR * wm + (q >> 2)) * S8 + 2 * (q & 3)) * NC + lk * 4 + e;
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
    for (int q = 0; q < NFR; ++q) {
      const int ty = WR * wm + (q >> 2);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = (ty * S8 + 2 * (q & 3)) * NC + lk * 4 + e;
        const float v = acc[q][j][e] + bv;
        ctile[row * (CROW8 / 2) + col] = f2bf(v);
        if ((vmask >> (q * 4 + e)) & 1u) {
          cs[j] += v;
          cq[j] += v * v;
        }
      }
    }
  }
  __syncthreads();
  constexpr int CPR = BW / 8;
  static_assert(NT8 % CPR == 0, "a thread keeps one channel vector in the store loop");
  if (g.bny != nullptr) {                           // (block-uniform) dgrad + BN-backward sums
    BnSum bs;
    bs.init(g.bnsc, g.bnsh, g.bnmu, g.bnis, n0 + (tid % CPR) * 8);
#pragma unroll
    for (int hh = 0; hh < PL8 * CPR / NT8; ++hh) {
      const int qd = tid + NT8 * hh;
      const int row = qd / CPR, c8 = qd % CPR;
      const int64_t dv = dst_vox(row);
      if (RAG && dv < 0) continue;
      const int64_t o = dv * g.Nd + n0 + c8 * 8;
      const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                      row * CROW8 + c8 * 16);
      const u32x4 yv = *reinterpret_cast<const u32x4*>(g.bny + o);
      *reinterpret_cast<u32x4*>(dst + o) = v;
      bs.add(v, yv);
    }
    __syncthreads();                                // ctile reads done: reuse it below
    bnsum_flush(bs, reinterpret_cast<float*>(smem), CPR, NT8, g.bnparts, n * NZ + tz, g.Nd, n0);
    return;
  }
#pragma unroll
  for (int hh = 0; hh < PL8 * CPR / NT8; ++hh) {
    const int qd = tid + NT8 * hh;
    const int row = qd / CPR, c8 = qd % CPR;
    const int64_t dv = dst_vox(row);
    if (RAG && dv < 0) continue;
    const int64_t o = dv * g.Nd + n0 + c8 * 8;
    u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                              row * CROW8 + c8 * 16);
    if (g.res != nullptr || g.relu) v = epi_res_relu(v, g.res ? g.res + o : nullptr, g.relu);
    *reinterpret_cast<u32x4*>(dst + o) = v;
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(smem + PL8 * CROW8);
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
      const int mt = n * NZ + tz;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * 16 * TN + j * 16 + lr;
        float ss = cs[j], qs = cq[j];
        for (int w = 1; w < NWM; ++w) {            // fixed order: deterministic
          ss += red[(w - 1) * 2 * BW + col];
          qs += red[(w - 1) * 2 * BW + BW + col];
        }
        stats[((int64_t)mt * 2) * g.Nd + n0 + col] = ss;
        stats[((int64_t)mt * 2 + 1) * g.Nd + n0 + col] = qs;
      }
    }
  }
}

// MMAD_LATTICE8: 1 (default) where the tiles fill the CUs, 2 at any size, 0 off;
// mmad_set_kernel_variant("lattice8", v) overrides it at run time
std::atomic<int> g_lattice8_mode{-1};
int lattice8_mode() {
  int v = g_lattice8_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_LATTICE8");
    int expect = -1;
    g_lattice8_mode.compare_exchange_strong(expect, e ? atoi(e) : 1);
    v = g_lattice8_mode.load(std::memory_order_relaxed);
  }
  return v;
}

// MMAD_L8_ROWS: plane rows per wave, 1 (default: 64-row wave tiles at twice the columns,
// fewer A-fragment reads per MFMA) or 2 (128-row wave tiles)
int l8_rows() {
  static const int v = [] {
    const char* e = getenv("MMAD_L8_ROWS");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  return v;
}

}  // namespace

namespace mmad_lattice8 {

int set_mode(int v) {
  const int prev = lattice8_mode();
  if (v >= 0) g_lattice8_mode.store(v, std::memory_order_relaxed);
  return prev;
}

static bool exact8(const mmad_patch::Geo& q) {
  constexpr int E = 2 * S8;
  return q.Ds == E && q.Hs == E && q.Ws == E && q.Dd == E && q.Hd == E && q.Wd == E;
}
// ragged grids (MMAD_LATTICE_RAGGED, default on): same extents in and out, at most 8 x 8
// positions per class plane, one sample's bytes addressable by a 32-bit buffer offset
static bool ragged8(const mmad_patch::Geo& q) {
  static const int mode = [] {
    const char* e = getenv("MMAD_LATTICE_RAGGED");
    return e ? atoi(e) : 1;
  }();
  return mode > 0 && !exact8(q) && q.Ds == q.Dd && q.Hs == q.Hd && q.Ws == q.Wd &&
         (q.Hs + 1) / 2 <= S8 && (q.Ws + 1) / 2 <= S8 &&
         (int64_t)q.Ds * q.Hs * q.Ws * q.Cs * 2 < (int64_t(1) << 31);
}
static int planes8(const mmad_patch::Geo& q) { return exact8(q) ? S8 : (q.Ds + 1) / 2; }

bool ok(const mmad_patch::Geo& q) {
  if (lattice8_mode() <= 0) return false;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3) return false;
  if (q.dd != 2 || q.dh != 2 || q.dw != 2 || q.pd != 2 || q.ph != 2 || q.pw != 2) return false;
  if (!exact8(q) && !ragged8(q)) return false;
  if (q.Cs % KC8 || q.Nd % 32 || q.Kpad != 27 * q.Cs) return false;
  // one 512-thread block per CU: with too few tiles even at 32 channels the row-gather
  // GEMM's more, smaller blocks win
  if (lattice8_mode() == 1 && (int64_t)q.nb * planes8(q) * (q.Nd / 32) < 256) return false;
  // 32-bit buffer offsets: one sample's input, the packed weights
  return (int64_t)q.Ds * q.Hs * q.Ws * q.Cs * 2 < (int64_t(1) << 31) &&
         (int64_t)q.Nd * q.Kpad * 2 < (int64_t(1) << 31);
}

int64_t tiles(const mmad_patch::Geo& q) { return (int64_t)q.nb * planes8(q); }

int fwd(const mmad_patch::Geo& q, const void* src, const void* wp, const float* bias,
        void* dst, float* stats, void* stream) {
  if (!mmad_lattice8::ok(q)) return MMAD_EUNSUPPORTED;
  auto attr1 = [](const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8) ==
           hipSuccess;
  };
  static const bool attr =
      attr1((const void*)lattice8_conv_kernel<2, false, 2>) &&
      attr1((const void*)lattice8_conv_kernel<1, false, 2>) &&
      attr1((const void*)lattice8_conv_kernel<2, true, 2>) &&
      attr1((const void*)lattice8_conv_kernel<1, true, 2>) &&
      attr1((const void*)lattice8_conv_kernel<4, false, 1>) &&
      attr1((const void*)lattice8_conv_kernel<2, false, 1>) &&
      attr1((const void*)lattice8_conv_kernel<4, true, 1>) &&
      attr1((const void*)lattice8_conv_kernel<2, true, 1>);
  if (!attr) return MMAD_EUNSUPPORTED;
  const bool rag = !exact8(q);
  const int nz = planes8(q);
  // 64-channel tiles when they give every CU a block, else 32
  const bool wide = q.Nd % BN8 == 0 && (int64_t)q.nb * nz * (q.Nd / BN8) >= 256;
  L8 g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.Kpad = q.Kpad;
  g.nbn = q.Nd / (wide ? BN8 : 32);
  g.nchunk = q.Cs / KC8;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  g.D = q.Ds; g.H = q.Hs; g.W = q.Ws; g.nz = nz;
  g.bny = reinterpret_cast<const u16*>(q.bny);
  g.bnsc = q.bnsc; g.bnsh = q.bnsh; g.bnmu = q.bnmu; g.bnis = q.bnis;
  g.bnparts = q.bnparts;
  if (g.bny != nullptr && (stats != nullptr || g.res != nullptr || g.relu || bias != nullptr))
    return MMAD_EUNSUPPORTED;                       // (one epilogue at a time)
  const int64_t nblk = (int64_t)q.nb * nz * g.nbn;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(NT8), LDS8, as_stream(stream), g,
                       (const u16*)src, (const u16*)wp, bias, (u16*)dst, stats);
  };
  if (l8_rows() == 1) {                             // one plane row per wave
    if (wide) rag ? go(lattice8_conv_kernel<4, true, 1>) : go(lattice8_conv_kernel<4, false, 1>);
    else rag ? go(lattice8_conv_kernel<2, true, 1>) : go(lattice8_conv_kernel<2, false, 1>);
  } else {                                          // two plane rows per wave
    if (wide) rag ? go(lattice8_conv_kernel<2, true, 2>) : go(lattice8_conv_kernel<2, false, 2>);
    else rag ? go(lattice8_conv_kernel<1, true, 2>) : go(lattice8_conv_kernel<1, false, 2>);
  }
  return launch_status();
}

}  // namespace mmad_lattice8
