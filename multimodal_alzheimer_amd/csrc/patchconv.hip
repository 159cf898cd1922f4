// Patch-resident stride-1 3D convolution for narrow layers, gfx950 (bf16, fp32 accumulate).
//
// Serves the MedicalNet layer1 BasicBlock convs (64 -> 64, 3x3x3, 32^3 at a 128^3 input,
// reached from pkg/models/mri_models/anat_cnn.py:29-31) and the other stride-1 convs with
// at most 128 channels per side, forward and -- as a forward conv over reversed taps --
// input gradient.
//
// Why a second conv kernel: the implicit GEMM (conv.hip) stages the A operand row by row,
// so every input voxel is fetched from L2 into LDS once per tap (27x) and, with only 64
// output channels to amortise it over, the 64-channel layers ran L2->LDS-bound at ~500
// TFLOP/s.  Here a block owns a TZ x 8 x 8 box of output voxels (TZ = 2: 128 GEMM rows) x
// 64 output channels, DMAs the input box plus its halo (the "patch": 4 x 10 x 10 voxels x
// 64 channels = 50 KiB for a 3^3 conv) into LDS ONCE, and builds each tap's A fragments
// from it by address offset: ~3 fetches per input voxel instead of 27.  Per tap only the
// weights (64 x 64 bf16, 8 KiB) stream through a 3-deep LDS ring by LDS-DMA.  The tap
// loop is compiled for the 3x3x3 dilation-1 stencil, so all tap offsets are constants.
//
//  * 8 (4) waves of 32 x 64 wave tiles (MFMA 16x16x32), each fragment read once
//    per wave with ds_read_b128; wider layers run one block per 64-channel N slice;
//  * patch rows are 128-byte voxel slices; 16-byte chunks XOR-swizzled by (patch x & 7),
//    which makes every fragment read of every tap conflict-free (rows of a fragment are
//    8 consecutive x of two patch rows; checked exhaustively over the 27 taps);
//  * software pipeline: the second K-half's fragment reads are in flight during the first
//    half's MFMAs, and the next tap's first-half reads during the second half's MFMAs, with
//    one barrier per tap (weight slot hand-over); weight DMA runs two taps ahead;
//  * input channels beyond 64 are walked as 64-channel chunks (patch reloaded per chunk);
//  * epilogue as the implicit GEMM: bias, BN partial sums (one row per tile), bf16 tile
//    transposed through LDS into 16-byte channel-vector stores.
#include <algorithm>
#include <cstdlib>

#include "bnsum.h"
#include "common.h"
#include "patchconv.h"

namespace {

// 2 x 8 x 8 output boxes: the patch (4 x 10 x 10 voxels x 128 B = 50 KB) plus the weight
// ring fit twice in the 160 KB LDS, so two blocks share a CU and one's per-tap barrier no
// longer idles the MFMA pipes; measured against 4 x 8 x 8 boxes (one block per CU, twice
// the tap reuse): layer1 fwd 90 -> 77 us, dgrad 85 -> 80 us, layer2.conv2 fwd 43 -> 37 us
// Output boxes TZ x 8 x 8.  TZ = 2 (two 4-wave blocks per CU) is the default; TZ = 4
// (MMAD_PATCH_TZ4=1: one 8-wave block per CU, half the weight LDS-DMA per MAC, a 5-tap
// weight lead) measured slower (layer1 fwd 77 vs 73 us).  Timing skeletons of the TZ = 2
// form (the PATCH_NO_* build flags below, layer1 fwd): no MFMA 54 us, no MFMA and no
// fragment reads 50 us, no MFMA and no weight DMA 42 us, no weight DMA 64 us -- the
// per-tile patch prologue and epilogue, not the DMA bandwidth or the MFMAs, set the time.
constexpr int TY = 8, TX = 8;
constexpr int RB = 128;                                    // bytes per patch row / K slice
// weight ring depth: NST - 1 taps of weights in flight (an LDS-DMA lands ~1 us after issue)
constexpr int nst_for(int tz) { return tz == 4 ? 6 : 3; }
constexpr int LDS_MAX = 160 * 1024;

struct PG {
  int nb, Cs, Nd, Kpad, Ds, Hs, Ws, Dd, Hd, Wd;
  int KD, KH, KW, pd, ph, pw, dd, dh, dw;
  int PZ, PY, PX, prow8;     // patch extents; patch DMA instructions (8 rows each)
  int ntz, nty, ntx, nbn, taps, nchunk;
  int ring_off;              // LDS byte offset of the weight ring
  const u16* res;            // eval-mode epilogue extras (see patchconv.h)
  int relu;
  const u16* bny;            // dgrad: BN-backward sums epilogue (bnsum.h)
  const float *bnsc, *bnsh, *bnmu, *bnis;
  float* bnparts;
};

__device__ const u32x4 g_zero16[8] = {};

template <int BN, int WGM, int WGN, int KS, int TZ>
__global__ __launch_bounds__(WGM * WGN * 64) void patch_conv_kernel(PG g, const u16* __restrict__ src,
                                                         const u16* __restrict__ wgt,
                                                         const float* __restrict__ bias,
                                                         u16* __restrict__ dst,
                                                         float* __restrict__ stats) {
  constexpr int NW = WGM * WGN, NTHR = NW * 64, TV = TZ * TY * TX, NST = nst_for(TZ);
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int WTM = TV / WGM, WTN = BN / WGN, TM = WTM / 16, TN = WTN / 16;
  constexpr int BSLOT = BN * RB;          // one tap's weights for the N tile
  constexpr int BI = BN * RB / 1024 / NW; // weight DMA instructions per wave per tap
  static_assert(BI >= 1 && BI * NW * 1024 == BSLOT, "weight slot split over the waves");
  // compile-time patch geometry (cubic KS^3 stencil, dilation 1): every tap offset and
  // swizzle below folds to a constant, so the unrolled tap loop carries no index math
  constexpr int PX = TX + KS - 1, PY = TY + KS - 1, PZ = TZ + KS - 1;
  constexpr int TAPS = KS * KS * KS, PROWS = PZ * PY * PX, PROW8 = (PROWS + 7) / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* patch = smem;
  char* ring = smem + g.ring_off;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: each XCD walks a contiguous range of tiles (neighbouring boxes share
  // halo voxels, the N tiles of one box share the whole patch) so they meet in one L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = tile / g.nbn, nt = tile % g.nbn;
  int t1 = mt;
  const int bx = t1 % g.ntx;
  t1 /= g.ntx;
  const int by = t1 % g.nty;
  t1 /= g.nty;
  const int bz = t1 % g.ntz, bn = t1 / g.ntz;
  const int z0 = bz * TZ, y0 = by * TY, x0 = bx * TX, n0 = nt * BN;
  const int lrow = lane >> 3;

  // this sample's input (per-sample offsets fit 32 bits: checked in ok())
  const u16* __restrict__ srcb = src + (int64_t)bn * g.Ds * g.Hs * g.Ws * g.Cs;
  auto issue_patch = [&](int cc) {
    for (int q = wave; q < PROW8; q += NW) {
      const int r = q * 8 + lrow;
      const int px = r % PX, t2 = r / PX;          // constant divisors: mul-shift
      const int py = t2 % PY, pz = t2 / PY;
      const int z = z0 - g.pd + pz, y = y0 - g.ph + py, x = x0 - g.pw + px;
      const void* p = g_zero16;
      if (r < PROWS && (unsigned)z < (unsigned)g.Ds && (unsigned)y < (unsigned)g.Hs &&
          (unsigned)x < (unsigned)g.Ws) {
        const int chunk = (lane & 7) ^ (px & 7);
        p = srcb + (((z * g.Hs + y) * g.Ws + x) * g.Cs + cc * 64 + chunk * 8);
      }
      glds16_asm(p, lds_addr_of(patch + q * 1024));
    }
  };
  const int bchunk = (lane & 7) ^ lrow;          // weight row & 7 == lrow
  const u16* wrow[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int co = n0 + (wave * BI + i) * 8 + lrow;
    wrow[i] = co < g.Nd ? wgt + (int64_t)co * g.Kpad + bchunk * 8 : nullptr;
  }
  // weights of stage (chunk cc, tap t) into ring slot `slot`
  auto issue_b = [&](int cc, int t, int slot) {
#ifdef PATCH_NO_WDMA
    return;
#endif
    char* sb = ring + slot * BSLOT;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const void* p = wrow[i] ? (const void*)(wrow[i] + t * g.Cs + cc * 64)
                              : (const void*)g_zero16;
      glds16_asm(p, lds_addr_of(sb + (wave * BI + i) * 1024));
    }
  };
  const int wm = wave % WGM, wn = wave / WGM;
  const int lr = lane & 15, lk = lane >> 4;
  int pb[TM], ptx[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int v = wm * WTM + i * 16 + lr;
    const int tx = v & 7, ty = (v >> 3) & 7, tz = v >> 6;
    pb[i] = (tz * PY + ty) * PX + tx;
    ptx[i] = tx;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  // fragments of K-half k of tap t (weights in ring slot `slot`)
  auto read_frags = [&](int t, int slot, int k, bf16x8* A, bf16x8* B) {
    const int kx = t % KS, ky = (t / KS) % KS, kz = t / (KS * KS);
    const int delta = (kz * PY + ky) * PX + kx;
    const int c = 4 * k + lk;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int p = pb[i] + delta;
#ifdef PATCH_NO_AREAD                           // timing experiments (skeleton breakdown)
      A[i] = bf16x8{};
      asm volatile("" : "+v"(A[i]));
#else
      A[i] = *reinterpret_cast<const bf16x8*>(patch + p * RB + ((c ^ ((ptx[i] + kx) & 7)) << 4));
#endif
    }
    const char* sb = ring + slot * BSLOT;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * WTN + j * 16 + lr;
#ifdef PATCH_NO_BREAD
      B[j] = bf16x8{};
      asm volatile("" : "+v"(B[j]));
#else
      B[j] = *reinterpret_cast<const bf16x8*>(sb + row * RB + ((c ^ (lr & 7)) << 4));
#endif
    }
  };
  auto mma = [&](const bf16x8* A, const bf16x8* B) {
#ifdef PATCH_NO_MFMA                            // timing experiment: memory/sync skeleton
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(A[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(B[j]));
    return;
#endif
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j], acc[i][j], 0, 0, 0);
  };

  // stage s = (chunk cc, tap t) lives in ring slot s % NST; weights run NST - 1 taps ahead
  const int S = g.nchunk * TAPS;
  issue_patch(0);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < S) issue_b(s / TAPS, s % TAPS, s);
  if (S >= NST - 1) wait_vm_lgkm0<(NST - 2) * BI>();   // the patch and stage 0 landed
  else wait_vm_lgkm0<0>();
  raw_barrier();
  if (S > NST - 1) issue_b((NST - 1) / TAPS, (NST - 1) % TAPS, NST - 1);
  read_frags(0, 0, 0, fa0, fb0);
  for (int cc = 0; cc < g.nchunk; ++cc) {
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int s = cc * TAPS + t;
      const int slot = (cc * (TAPS % NST) + t) % NST;     // == s % NST
      read_frags(t, slot, 1, fa1, fb1);
      mma(fa0, fb0);
      if (s + 1 < S) {
        // weights of stage s+1 landed (s+2 .. s+NST-1 may still fly); every fragment read
        // of stage s is done -> after the barrier its slot is free
        if (s + NST - 1 < S) wait_vm_lgkm0<(NST - 2) * BI>();
        else wait_vm_lgkm0<0>();
        raw_barrier();
        const int s3 = s + NST;
        if (t == TAPS - 1) {                   // next 64-channel chunk: reload the patch
          issue_patch(cc + 1);
          if (s3 < S) issue_b(s3 / TAPS, s3 % TAPS, slot);
          wait_vm_lgkm0<0>();
          raw_barrier();
        } else if (s3 < S) {
          issue_b(t + NST < TAPS ? cc : cc + 1, (t + NST) % TAPS, slot);
        }
        read_frags((t + 1) % TAPS, (slot + 1) % NST, 0, fa0, fb0);
      }
      mma(fa1, fb1);
    }
  }
  __syncthreads();                             // patch / ring reused by the epilogue

  // output rows: box-relative voxel offsets in 32 bits from one 64-bit tile base; a box
  // wholly inside the volume (every box of a 32^3 / 16^3 layer) skips the per-row checks
  const bool full = z0 + TZ <= g.Dd && y0 + TY <= g.Hd && x0 + TX <= g.Wd;
  const int64_t vbase = (((int64_t)bn * g.Dd + z0) * g.Hd + y0) * g.Wd + x0;
  auto row_ok = [&](int row) {
    return full || (z0 + (row >> 6) < g.Dd && y0 + ((row >> 3) & 7) < g.Hd && x0 + (row & 7) < g.Wd);
  };
  auto row_off = [&](int row) { return ((row >> 6) * g.Hd + ((row >> 3) & 7)) * g.Wd + (row & 7); };
  constexpr int CROW = BN * 2 + 16;
  u16* ctile = reinterpret_cast<u16*>(smem);
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    cs[j] = 0.f;
    cq[j] = 0.f;
    const int col = wn * WTN + j * 16 + lr;
    const int co = n0 + col;                   // < Nd: Nd % 64 == 0 (ok())
    const float bv = bias != nullptr ? bias[co] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * WTM + i * 16 + lk * 4 + r;
        const float v = acc[i][j][r] + bv;
        ctile[row * (CROW / 2) + col] = f2bf(v);
        if (row_ok(row)) {
          cs[j] += v;
          cq[j] += v * v;
        }
      }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  u16* __restrict__ dstb = dst + vbase * g.Nd + n0;
  const u16* __restrict__ resb = g.res != nullptr ? g.res + vbase * g.Nd + n0 : nullptr;
  static_assert(NTHR % CPR == 0, "a thread keeps one channel vector in the store loop");
  if (g.bny != nullptr) {                      // (block-uniform) dgrad + BN-backward sums
    BnSum bs;
    bs.init(g.bnsc, g.bnsh, g.bnmu, g.bnis, n0 + (tid % CPR) * 8);
    const u16* __restrict__ yb = g.bny + vbase * g.Nd + n0;
#pragma unroll
    for (int h = 0; h < TV * CPR / NTHR; ++h) {
      const int q = tid + NTHR * h;
      const int row = q / CPR, c8 = q % CPR;
      if (row_ok(row)) {
        const int o = row_off(row) * g.Nd + c8 * 8;
        const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                        row * CROW + c8 * 16);
        const u32x4 yv = *reinterpret_cast<const u32x4*>(yb + o);
        *reinterpret_cast<u32x4*>(dstb + o) = v;
        bs.add(v, yv);
      }
    }
    __syncthreads();                           // ctile reads done: reuse it below
    bnsum_flush(bs, reinterpret_cast<float*>(smem), CPR, NTHR, g.bnparts, mt, g.Nd, n0);
    return;
  }
#pragma unroll
  for (int h = 0; h < TV * CPR / NTHR; ++h) {
    const int q = tid + NTHR * h;
    const int row = q / CPR, c8 = q % CPR;
    if (row_ok(row)) {
      const int o = row_off(row) * g.Nd + c8 * 8;
      u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(ctile) +
                                                row * CROW + c8 * 16);
      if (g.res != nullptr || g.relu) v = epi_res_relu(v, resb ? resb + o : nullptr, g.relu);
      *reinterpret_cast<u32x4*>(dstb + o) = v;
    }
  }
  if (stats != nullptr) {
    float* red = reinterpret_cast<float*>(smem + TV * CROW);
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
        stats[((int64_t)mt * 2) * g.Nd + co] = ss;
        stats[((int64_t)mt * 2 + 1) * g.Nd + co] = qs;
      }
    }
  }
}

int patch_mode() {
  static const int v = [] { const char* e = getenv("MMAD_PATCH"); return e ? atoi(e) : 1; }();
  return v;
}

// 64-channel N tiles only: the 128-wide variant (128 x 64 wave tiles) spills with the
// fully unrolled tap loop; wider layers run one block per 64-channel slice of the same box
int bn_for(const mmad_patch::Geo&) { return 64; }

// output-box depth: 2 (two 4-wave blocks per CU) unless MMAD_PATCH_TZ4=1 (4: one 8-wave block)
int tz_for(const mmad_patch::Geo&) {
  static const int v = [] { const char* e = getenv("MMAD_PATCH_TZ4"); return e && atoi(e) ? 4 : 2; }();
  return v;
}

PG make_pg(const mmad_patch::Geo& q, int TZ) {
  PG g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.Kpad = q.Kpad;
  g.Ds = q.Ds; g.Hs = q.Hs; g.Ws = q.Ws; g.Dd = q.Dd; g.Hd = q.Hd; g.Wd = q.Wd;
  g.KD = q.KD; g.KH = q.KH; g.KW = q.KW; g.pd = q.pd; g.ph = q.ph; g.pw = q.pw;
  g.dd = q.dd; g.dh = q.dh; g.dw = q.dw;
  g.PZ = TZ + (q.KD - 1) * q.dd;
  g.PY = TY + (q.KH - 1) * q.dh;
  g.PX = TX + (q.KW - 1) * q.dw;
  g.prow8 = (int)cdiv((int64_t)g.PZ * g.PY * g.PX, 8);
  g.ntz = (int)cdiv(q.Dd, TZ); g.nty = (int)cdiv(q.Hd, TY); g.ntx = (int)cdiv(q.Wd, TX);
  g.nbn = (int)cdiv(q.Nd, bn_for(q));
  g.taps = q.KD * q.KH * q.KW;
  g.nchunk = q.Cs / 64;
  g.ring_off = g.prow8 * 1024;
  g.res = reinterpret_cast<const u16*>(q.res);
  g.relu = q.relu;
  g.bny = reinterpret_cast<const u16*>(q.bny);
  g.bnsc = q.bnsc; g.bnsh = q.bnsh; g.bnmu = q.bnmu; g.bnis = q.bnis;
  g.bnparts = q.bnparts;
  return g;
}

size_t lds_bytes(const PG& g, int bn, int wgm, int TZ) {
  const size_t main = (size_t)g.ring_off + (size_t)nst_for(TZ) * bn * RB;
  const size_t epi = (size_t)TZ * TY * TX * (bn * 2 + 16) + (size_t)(wgm - 1) * 2 * bn * 4;
  return std::max(main, epi);
}

template <int BN, int WGM, int WGN, int KS, int TZ>
int launch(const PG& g, const void* src, const void* wp, const float* bias, void* dst,
           float* stats, hipStream_t st) {
  const size_t lds = lds_bytes(g, BN, WGM, TZ);
  static const bool ok = hipFuncSetAttribute(
                             (const void*)patch_conv_kernel<BN, WGM, WGN, KS, TZ>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX) == hipSuccess;
  if (!ok || lds > (size_t)LDS_MAX) return MMAD_EUNSUPPORTED;
  const int64_t nblk = (int64_t)g.nb * g.ntz * g.nty * g.ntx * g.nbn;
  hipLaunchKernelGGL((patch_conv_kernel<BN, WGM, WGN, KS, TZ>), dim3((unsigned)nblk),
                     dim3(WGM * WGN * 64), lds, st, g, (const u16*)src, (const u16*)wp, bias,
                     (u16*)dst, stats);
  return launch_status();
}

}  // namespace

namespace mmad_patch {

bool ok(const Geo& q) {
  const int mode = patch_mode();
  if (mode <= 0) return false;
  if (q.Cs % 64 || q.Nd % 64 || q.Kpad < q.KD * q.KH * q.KW * q.Cs) return false;
  if (mode == 1 && (q.Cs > 128 || q.Nd > 128)) return false;   // narrow layers only
  // compiled stencil: 3x3x3, dilation 1 (MedicalNet layer1/layer2 convs and their dgrads)
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dd != 1 || q.dh != 1 || q.dw != 1) return false;
  const int tz = tz_for(q);
  const PG g = make_pg(q, tz);
  if (lds_bytes(g, bn_for(q), tz == 4 ? 8 : 4, tz) > (size_t)LDS_MAX) return false;
  // per-sample input / output offsets in 32 bits (the patch DMA and epilogue index math)
  const int64_t ivox = (int64_t)q.Ds * q.Hs * q.Ws, ovox = (int64_t)q.Dd * q.Hd * q.Wd;
  return ivox * q.Cs < (int64_t(1) << 31) && ovox * q.Nd < (int64_t(1) << 31) &&
         (int64_t)q.nb * g.ntz * g.nty * g.ntx * g.nbn < (int64_t(1) << 31);
}

int64_t tiles(const Geo& q) {
  if (mmad_patchz::ok(q)) return mmad_patchz::tiles(q);
  const PG g = make_pg(q, tz_for(q));
  return (int64_t)q.nb * g.ntz * g.nty * g.ntx;
}

int fwd(const Geo& q, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream) {
  if (!ok(q)) return MMAD_EUNSUPPORTED;
  if (mmad_patchz::ok(q)) return mmad_patchz::fwd(q, src, wp, bias, dst, stats, stream);
  const int tz = tz_for(q);
  const PG g = make_pg(q, tz);
  if (g.bny != nullptr && (stats != nullptr || g.res != nullptr || g.relu || bias != nullptr))
    return MMAD_EUNSUPPORTED;                  // (one epilogue at a time)
  hipStream_t st = as_stream(stream);
  if (tz == 4) return launch<64, 8, 1, 3, 4>(g, src, wp, bias, dst, stats, st);
  return launch<64, 4, 1, 3, 2>(g, src, wp, bias, dst, stats, st);
}

}  // namespace mmad_patch
