// Persistent z-walking patch conv for MedicalNet's layer1 (64 -> 64 channels, 3x3x3,
// stride 1, padding 1 on the 32^3 grid of a 128^3 input; pkg/models/mri_models/
// anat_cnn.py:29-31 via MedicalNet's BasicBlock), forward and -- as a forward conv over
// reversed taps -- input gradient, gfx950 bf16 with fp32 accumulation.
//
// patchconv.hip runs one 2x8x8 output box per block and loads its 4x10x10-voxel patch in a
// prologue that nothing overlaps: the round-2 skeleton timings put 54 of its 73 us in that
// prologue, the epilogue and the per-tap barriers.  Here a block stays on one (sample, y
// box, x box) column and walks its z-range in 4x8x8 boxes (256 rows x 64 channels):
//  * the input arrives as 10x10-voxel z-planes (12.8 KiB) through an 8-slot plane ring:
//    consecutive boxes share two planes, so each box loads 4 new planes (not 6), and they
//    are loaded while the previous box computes -- planes 4i+6, 4i+7 at box i's first tap,
//    4i+8 once its last kz = -1 tap has run, 4i+9 after the last kz = 0 tap; the next box
//    finds them resident;
//  * the weights stream per tap (64 x 64 bf16 = 8 KiB) through a 4-slot ring, three taps
//    ahead, across box boundaries (every box uses the same 27 taps);
//  * 8 waves of 32 rows x 64 channels (wave w: z-plane w/2 of the box, y rows 4(w&1)..+3),
//    the K halves of each tap pipelined across one barrier per tap as in patchconv.hip;
//  * the epilogue stages the bf16 box through LDS in two halves (16-byte channel-vector
//    stores) and writes one BN partial-sum row per box.
// Same per-element K order as patchconv.hip (tap-major, channels ascending in 32-wide
// halves), so the conv outputs are bit-identical to it; only the BN partial sums are grouped
// into different rows (one per 4x8x8 box instead of per 2x8x8 box).
#include <atomic>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "patchconv.h"

namespace {

constexpr int PX = 10, PY = 10;                 // plane extent (8 + halo)
constexpr int RB = 128;                         // 64 channels x 2 B per row
constexpr int PROWS = PX * PY;                  // 100
constexpr int PSLOT = 104 * RB;                 // 13 x 1 KiB DMA pieces (rows 100..103 spare)
constexpr int NPS = 8;                          // plane ring slots
constexpr int WSLOT = 64 * RB;                  // one tap's weights: 64 co x 64 ci
constexpr int NST = 4;                          // weight ring slots (three taps in flight)
constexpr int RING_OFF = NPS * PSLOT;           // 106496
constexpr int STG_OFF = RING_OFF + NST * WSLOT; // 139264
constexpr int CROW = 64 * 2 + 16;               // staged output row (padded)
constexpr int STG_BYTES = 128 * CROW;           // half a box
constexpr int RED_OFF = STG_OFF + STG_BYTES;
constexpr int LDS = RED_OFF + (8 - 1) * 128 * 4;      // BN sums of waves 1..7
static_assert(LDS <= 160 * 1024, "LDS budget");
constexpr int NTHR = 512, NW = 8;
constexpr int TAPS = 27;

struct PZ {
  int nb, Nd, Kpad, D, H, W;
  int nty, ntx, nbn, nseg, tps;                 // y / x boxes, channel tiles, z segments,
                                                // boxes per segment
  const u16* res;
  int relu;
};

__device__ const u32x4 g_zero16z[8] = {};
constexpr int EPI_ST = 4;                       // epilogue data stores per wave
constexpr int STATS_ST = 8;                     // BN partial-sum stores (wave 0)

// counted global stores (see the epilogue): exactly one VMEM instruction each
__device__ __forceinline__ void st_u32x4(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_f32(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// LDS hand-over inside the epilogue: this wave's LDS ops done, then the barrier (no vmcnt
// drain, unlike __syncthreads)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// planes issued at tap r of a box that has a successor: 2 at r = 0, 1 at r = 9 and r = 18
__host__ __device__ constexpr int planes_at(int r) { return r == 0 ? 2 : (r == 9 || r == 18) ? 1 : 0; }
// VMEM instructions (per wave) younger than the weights of tap t + 1 at tap t's barrier:
// the DMA groups of taps t - 2 and t - 1 (weights 1 each while they exist, planes 2 each)
template <int T, bool NEXT, bool PREV_NEXT, bool LAST>
__host__ __device__ constexpr int younger() {
  int n = 0;
  for (int d = 1; d <= 2; ++d) {
    const int r = T - d;                        // group of tap r (< 0: the previous box)
    const bool next = r >= 0 ? NEXT : PREV_NEXT;
    const int rr = r >= 0 ? r : r + TAPS;
    n += 2 * (next ? planes_at(rr) : 0);
    // weights of tap r + 4 (relative to this box) were issued unless they run past the end
    const bool w = !(LAST && r + 4 >= TAPS);
    n += w ? 1 : 0;
  }
  return n;
}

__global__ __launch_bounds__(NTHR) void patchz_conv_kernel(PZ g, const u16* __restrict__ src,
                                                           const u16* __restrict__ wgt,
                                                           const float* __restrict__ bias,
                                                           u16* __restrict__ dst,
                                                           float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: each XCD walks a contiguous range of work items; neighbouring columns
  // (halo voxels) and the segments of one column meet in one L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int item = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  int t1 = item;
  const int seg = t1 % g.nseg;
  t1 /= g.nseg;
  const int nt = t1 % g.nbn;
  t1 /= g.nbn;
  const int bx = t1 % g.ntx;
  t1 /= g.ntx;
  const int by = t1 % g.nty;
  const int n = t1 / g.nty;
  const int y0 = by * 8, x0 = bx * 8, n0 = nt * 64;
  const int zs = seg * g.tps * 4;               // first output plane of the segment
  const int HW = g.H * g.W;

  // ---- plane DMA: plane q (input z = zs - 1 + q) into slot q % 8; piece p = wave + 8h
  // (13 pieces of 8 rows; surplus pieces repeat piece 12: the same bytes to the same place)
  const u16* __restrict__ srcn = src + (int64_t)n * g.D * HW * 64;
  int poff[2];                                  // lane's voxel offset in the plane (or -1)
  uint32_t pdst[2];
  {
    const int lrow = lane >> 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = min(wave + NW * h, 12);
      const int r = p * 8 + lrow;
      const int px = r % PX, py = r / PX;
      const int y = y0 - 1 + py, x = x0 - 1 + px;
      const bool in = r < PROWS && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
      const int chunk = (lane & 7) ^ (px & 7);
      poff[h] = in ? (y * g.W + x) * 64 + chunk * 8 : -1;
      pdst[h] = p * 1024;
    }
  }
  auto issue_plane = [&](int q) __attribute__((always_inline)) {
    const int z = zs - 1 + q;
    const bool zin = (unsigned)z < (unsigned)g.D;
    const u16* base = srcn + (int64_t)(zin ? z : 0) * HW * 64;
    char* slot = smem + (q & (NPS - 1)) * PSLOT;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const void* p = (zin && poff[h] >= 0) ? (const void*)(base + poff[h]) : (const void*)g_zero16z;
      glds16_asm(p, lds_addr_of(slot + pdst[h]));
    }
  };
  // ---- weight DMA: tap t's 64 x 64 slice, wave w rows 8w .. 8w + 7 (one instruction)
  const int lrow = lane >> 3;
  const u16* wrow = wgt + (int64_t)(n0 + wave * 8 + lrow) * g.Kpad + (((lane & 7) ^ lrow) * 8);
  // global tap counter gt -> slot gt % NST; wt = gt % TAPS, a compile-time constant at every
  // call (a run-time modulo by 27 per tap was ~20 scalar instructions in the tap loop)
  auto issue_w = [&](int gt, int wt) __attribute__((always_inline)) {
    glds16_asm(wrow + wt * 64,
               lds_addr_of(smem + RING_OFF + (gt & (NST - 1)) * WSLOT + wave * 1024));
  };

  // ---- fragment addressing: wave w = plane w >> 1 of the box, y rows 4 (w & 1) .. + 3
  const int wz = wave >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  const int tx = lr & 7, ty0 = 4 * (wave & 1) + (lr >> 3);
  uint32_t aoff[3][2];                          // [kx][K half] lane part of the A address
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int k = 0; k < 2; ++k)
      aoff[kx][k] = (uint32_t)((ty0 * PX + tx + kx) * RB + (((4 * k + lk) ^ ((tx + kx) & 7)) << 4));
  uint32_t boff[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) boff[k] = (uint32_t)(lr * RB + (((4 * k + lk) ^ (lr & 7)) << 4));

  f32x4 acc[2][4];
  bf16x8 fa0[2], fb0[4], fa1[2], fb1[4];
#if defined(PZ_NO_AREAD) || defined(PZ_NO_BREAD)
  // (skeletons: the skipped fragments start as opaque register contents, so the MFMAs stay)
#pragma unroll
  for (int i = 0; i < 2; ++i) { asm volatile("" : "=v"(fa0[i])); asm volatile("" : "=v"(fa1[i])); }
#pragma unroll
  for (int j = 0; j < 4; ++j) { asm volatile("" : "=v"(fb0[j])); asm volatile("" : "=v"(fb1[j])); }
#endif
  // fragments of K half K of tap T of the box whose first plane is q0
  auto read_frags = [&](auto tc, auto kc, int q0, int gt, bf16x8 (&A)[2], bf16x8 (&B)[4])
      __attribute__((always_inline)) {
    constexpr int T = decltype(tc)::value, K = decltype(kc)::value;
    constexpr int kz = T / 9, ky = (T / 3) % 3, kx = T % 3;
    int pbase = __builtin_amdgcn_readfirstlane(((q0 + wz + kz) & (NPS - 1)) * PSLOT);
    int wbase = __builtin_amdgcn_readfirstlane(RING_OFF + (gt & (NST - 1)) * WSLOT);
    asm volatile("" : "+s"(pbase), "+s"(wbase));
    const char* pa = smem + pbase + aoff[kx][K] + ky * PX * RB;
#ifndef PZ_NO_AREAD   // timing skeleton (tools): no A fragment reads (stale registers)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      A[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2 * PX * RB);
#endif
    const char* pb = smem + wbase + boff[K];
#ifndef PZ_NO_BREAD   // timing skeleton (tools): no B fragment reads (stale registers)
#pragma unroll
    for (int j = 0; j < 4; ++j) B[j] = *reinterpret_cast<const bf16x8*>(pb + j * 16 * RB);
#endif
  };
  auto mma = [&](const bf16x8 (&A)[2], const bf16x8 (&B)[4]) __attribute__((always_inline)) {
#ifdef PZ_NO_MMA   // timing skeleton (tools): fragments consumed, no MFMA
#pragma unroll
    for (int i = 0; i < 2; ++i) asm volatile("" ::"v"(A[i]));
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(B[j]));
#else
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
#endif
  };

  // ---- epilogue of box i (output planes zs + 4i .. + 3).  No vmcnt drain here: the next
  // box's planes and first weights stay in flight.  Its global stores are VMEM ops too
  // (counted in issue order with the LDS-DMA), so they are issued from asm -- an exact count
  // per wave (EPI_ST; + STATS_ST on wave 0 when BN sums are written) -- and the first three
  // counted waits of the next box add them to the younger ops they allow.
  float bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bv[j] = bias != nullptr ? bias[n0 + j * 16 + lr] : 0.f;
    asm volatile("" ::"v"(bv[j]));              // consumed here: its vmcnt wait comes before
  }                                             // any DMA, not in an epilogue
  const int64_t nbase = (int64_t)n * g.D;
  auto epilogue = [&](int i) __attribute__((always_inline)) {
#ifdef PZ_NO_EPI   // timing skeleton (tools): accumulators consumed, nothing stored
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[a][j]));
    return;
#endif
    const int z0 = zs + 4 * i;
    u16* ctile = reinterpret_cast<u16*>(smem + STG_OFF);
    float cs[4], cq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cs[j] = 0.f;
      cq[j] = 0.f;
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i2][j][r] + bv[j];
          cs[j] += v;
          cq[j] += v * v;
        }
    }
    // BN partial sums first (wave 0 stores them), then the box in two staged halves
    if (stats != nullptr) {
      float* red = reinterpret_cast<float*>(smem + RED_OFF);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs[j] += __shfl_xor(cs[j], 16, 64);
        cs[j] += __shfl_xor(cs[j], 32, 64);
        cq[j] += __shfl_xor(cq[j], 16, 64);
        cq[j] += __shfl_xor(cq[j], 32, 64);
      }
      if (wave > 0 && lk == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          red[(wave - 1) * 128 + j * 16 + lr] = cs[j];
          red[(wave - 1) * 128 + 64 + j * 16 + lr] = cq[j];
        }
      }
      lds_barrier();
      if (wave == 0) {
        const int64_t mt = (((int64_t)n * (g.D / 4) + z0 / 4) * g.nty + by) * g.ntx + bx;
        float* srow = stats + (mt * 2) * g.Nd + n0 + lr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float ss = cs[j], qs = cq[j];
          for (int w = 1; w < NW; ++w) {        // fixed order: deterministic
            ss += red[(w - 1) * 128 + j * 16 + lr];
            qs += red[(w - 1) * 128 + 64 + j * 16 + lr];
          }
          // lanes lk > 0 hold the same sums: all 64 lanes store, lanes of one lr the same
          // value to the same address (one instruction each, counted)
          st_f32(srow + j * 16, ss);
          st_f32(srow + g.Nd + j * 16, qs);
        }
      }
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if ((wave >> 2) == hh) {                  // waves 4 hh .. 4 hh + 3 own rows 128 hh ..
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = j * 16 + lr;
#pragma unroll
          for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = (wave & 3) * 32 + i2 * 16 + lk * 4 + r;   // within the half
              ctile[row * (CROW / 2) + col] = f2bf(acc[i2][j][r] + bv[j]);
            }
        }
      }
      lds_barrier();
#pragma unroll
      for (int h = 0; h < 2; ++h) {             // 128 rows x 8 chunks / 512 threads
        const int qd = tid + NTHR * h;
        const int row = qd >> 3, c8 = qd & 7;
        const int v = hh * 128 + row;           // box row: z (v >> 6), y, x
        const int64_t vox = ((nbase + z0 + (v >> 6)) * g.H + y0 + ((v >> 3) & 7)) * g.W + x0 + (v & 7);
        const int64_t o = vox * g.Nd + n0 + c8 * 8;
        u32x4 val = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                    row * CROW + c8 * 16);
        if (g.res != nullptr || g.relu) val = epi_res_relu(val, g.res ? g.res + o : nullptr, g.relu);
        st_u32x4(dst + o, val);
      }
      lds_barrier();                            // staging reused by the second half
    }
  };

  // ---- prologue: the first box's six planes, weights of taps 0..3
  for (int q = 0; q < 6; ++q) issue_plane(q);
#pragma unroll
  for (int t = 0; t < NST; ++t) issue_w(t, t);
  wait_vm_lgkm0<NST - 1>();
  raw_barrier();
  read_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0, 0, fa0, fb0);

  // box i: taps unrolled; NEXT = a box follows (its planes are issued here), PREV_NEXT =
  // this box had a predecessor that issued planes for it (its last taps' groups count)
  auto box = [&](int i, auto nextc, auto lastc) __attribute__((always_inline)) {
    constexpr bool NEXT = decltype(nextc)::value, LAST = decltype(lastc)::value;
    const int q0 = 4 * i, gt0 = TAPS * i;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto tap = [&](auto tc) __attribute__((always_inline)) {
      constexpr int T = decltype(tc)::value;
      const int gt = gt0 + T;
      read_frags(tc, std::integral_constant<int, 1>{}, q0, gt, fa1, fb1);
      mma(fa0, fb0);
      // barrier of tap T: the weights of tap gt + 1 landed (the planes it reads are older)
      if constexpr (!(LAST && T == TAPS - 1)) {
        constexpr int Y = younger<T, NEXT, true, LAST>();
        if constexpr (T <= 2) {                 // the previous box's epilogue stores are
          if (i == 0) {                         // younger than the awaited weights
            wait_vm_lgkm0<Y>();
          } else if (wave == 0 && stats != nullptr) {
            wait_vm_lgkm0<Y + EPI_ST + STATS_ST>();
          } else {
            wait_vm_lgkm0<Y + EPI_ST>();
          }
        } else {
          wait_vm_lgkm0<Y>();
        }
#ifndef PZ_NO_BAR   // timing skeleton (tools): no per-tap barrier (races; timing only)
        raw_barrier();
#endif
        if constexpr (NEXT && planes_at(T) == 2) {
          issue_plane(q0 + 6);
          issue_plane(q0 + 7);
        } else if constexpr (NEXT && T == 9) {
          issue_plane(q0 + 8);
        } else if constexpr (NEXT && T == 18) {
          issue_plane(q0 + 9);
        }
        if constexpr (!(LAST && T + 4 >= TAPS)) issue_w(gt + 4, (T + 4) % TAPS);
        if constexpr (T + 1 < TAPS)
          read_frags(std::integral_constant<int, T + 1>{}, std::integral_constant<int, 0>{}, q0,
                     gt + 1, fa0, fb0);
        else
          read_frags(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, q0 + 4,
                     gt + 1, fa0, fb0);
      }
      mma(fa1, fb1);
    };
    [&]<int... T>(std::integer_sequence<int, T...>) {
      (tap(std::integral_constant<int, T>{}), ...);
    }(std::make_integer_sequence<int, TAPS>{});
    epilogue(i);
  };
  for (int i = 0; i + 1 < g.tps; ++i) box(i, std::true_type{}, std::false_type{});
  box(g.tps - 1, std::false_type{}, std::true_type{});
}

std::atomic<int> g_patchz_mode{-1};
int patchz_mode() {
  int v = g_patchz_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("MMAD_PATCHZ");
    int expect = -1;
    g_patchz_mode.compare_exchange_strong(expect, e ? atoi(e) : 1);
    v = g_patchz_mode.load(std::memory_order_relaxed);
  }
  return v;
}

// z segments per column: the fewest that give every CU a work item, each >= 2 boxes
int segments(const mmad_patch::Geo& q) {
  const int64_t cols = (int64_t)q.nb * (q.Hd / 8) * (q.Wd / 8) * (q.Nd / 64);
  const int boxes = q.Dd / 4;
  int s = 1;
  while (cols * s < 256 && boxes % (2 * s) == 0 && boxes / (2 * s) >= 2) s *= 2;
  return s;
}

}  // namespace

namespace mmad_patchz {

int set_mode(int v) {
  const int prev = patchz_mode();
  if (v >= 0) g_patchz_mode.store(v, std::memory_order_relaxed);
  return prev;
}

bool ok(const mmad_patch::Geo& q) {
  if (patchz_mode() <= 0) return false;
  if (q.Cs != 64 || q.Nd % 64 || q.Kpad < 27 * 64) return false;
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dd != 1 || q.dh != 1 || q.dw != 1) return false;
  if (q.pd != 1 || q.ph != 1 || q.pw != 1) return false;
  if (q.Ds != q.Dd || q.Hs != q.Hd || q.Ws != q.Wd) return false;
  if (q.Dd % 4 || q.Hd % 8 || q.Wd % 8) return false;
  const int s = segments(q);
  if (q.Dd / 4 / s < 2) return false;           // nothing to walk
  const int64_t cols = (int64_t)q.nb * (q.Hd / 8) * (q.Wd / 8) * (q.Nd / 64);
  if (patchz_mode() == 1 && cols * s < 256) return false;   // fewer items than CUs
  // per-sample offsets in 32 bits (plane DMA lane offsets, epilogue)
  return (int64_t)q.Ds * q.Hs * q.Ws * 64 < (int64_t(1) << 31) &&
         (int64_t)q.nb * q.Dd * q.Hd * q.Wd * q.Nd < (int64_t(1) << 40);
}

int64_t tiles(const mmad_patch::Geo& q) {
  return (int64_t)q.nb * (q.Dd / 4) * (q.Hd / 8) * (q.Wd / 8);
}

int fwd(const mmad_patch::Geo& q, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream) {
  if (!mmad_patchz::ok(q)) return MMAD_EUNSUPPORTED;
  static const bool attr =
      hipFuncSetAttribute((const void*)patchz_conv_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, LDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  PZ g{};
  g.nb = q.nb; g.Nd = q.Nd; g.Kpad = q.Kpad; g.D = q.Dd; g.H = q.Hd; g.W = q.Wd;
  g.nty = q.Hd / 8; g.ntx = q.Wd / 8; g.nbn = q.Nd / 64;
  g.nseg = segments(q);
  g.tps = q.Dd / 4 / g.nseg;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  const int64_t items = (int64_t)q.nb * g.nty * g.ntx * g.nbn * g.nseg;
  hipLaunchKernelGGL(patchz_conv_kernel, dim3((unsigned)items), dim3(NTHR), LDS,
                     as_stream(stream), g, (const u16*)src, (const u16*)wp, bias, (u16*)dst,
                     stats);
  return launch_status();
}

}  // namespace mmad_patchz
