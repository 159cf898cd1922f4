// Dedicated MedicalNet stem convolution, gfx950.
//
// conv1 of MedicalNet's ResNet (nn.Conv3d(1, 64, 7, stride 2, padding 3), reached from
// pkg/models/mri_models/anat_cnn.py:29-31 and pet_resnet_cnn.py:33-35) runs on the
// W-unfolded input U[n][z][y][xo][8] (8 = the kw taps of output column xo, see
// mmad_conv_unfold_input), so the conv is a (7, 7, 1) stencil over 16-byte rows of U.
//
// The generic implicit GEMM gathers 49 x 16 B per output voxel from L2 and runs only 7
// K-stages per tile, which leaves it latency-bound (~250 TFLOP/s).  Here a block owns two
// output rows (y, y+1) x all 64 output columns x all 64 channels and walks the whole z
// range: the (kd) input planes it needs sit in an LDS ring of KD + sd planes (each plane
// = the 9 input rows those two output rows touch, 1 KiB each), so each input row is
// fetched from memory about once per block instead of ~12 times, and the next z-step's
// sd new planes are DMA'd (asm LDS-DMA) while the MFMAs of the current step run.  The
// weights (64 x 448 bf16) stay in LDS for the block's lifetime.  Per z-step the epilogue
// writes the 128 x 64 bf16 output tile as 16-byte vectors and one row of BN partial sums,
// exactly like the implicit-GEMM epilogue, so the BN that follows is unchanged.  The MFMA
// runs transposed (channels x voxels) so each lane stores 4 adjacent channels directly.
#include <type_traits>

#include "common.h"
#include "stem.h"

namespace {

constexpr int CO = 64;            // output channels
constexpr int YT = 2;             // output rows per block
constexpr int XW = 64;            // output columns per row (max)
constexpr int ROWB = XW * 16;     // one unfolded input row in LDS (1 KiB)
// wgrad ring rows are padded by 64 B: its transposing U reads put lanes two taps (= two
// rows) apart in one 32-lane group, and 1088-byte rows move those onto the other 16 banks
// (at 1024 B every such pair was a 2-way conflict)
constexpr int ROWB_W = ROWB + 64;
constexpr int CROW = CO * 2 + 16; // C tile row (bf16, padded)

__device__ const u32x4 g_zero_kb[64] = {};   // 1 KiB of zeros: DMA source for padding rows

struct StemG {
  int n, di, hi, wo, do_, ho;
  int sd, sh, pd, ph;
  int kpad, wrow;                 // packed weight row (elements), LDS weight row (bytes)
  int rz, yin, nks;               // ring planes (wgrad), rows per plane, K-steps of 32
  int rzf;                        // forward ring planes: KD + 2*SD (two z-steps ahead)
  int nyb, nzc, zsteps;           // y-pairs, z-chunks, z-steps per block
  int ring_off, c_off, red_off;   // LDS offsets (bytes)
  int wi;                         // raw input width (raw-input forms)
  int nxt, tw;                    // output column tiles (wo > 64: config 5's 80) and width
};

// ---- raw-input rows (round 4) -----------------------------------------------------------
// The stem kernels below can read the sample's raw volume (f64 as the DataLoader delivers it,
// or f32) instead of the W-unfolded copy mmad_conv_unfold_input writes: a row of 2*64 input
// values is one 16-byte (f64) / 8-byte (f32) load per lane (lane l holds x[2l], x[2l+1]), and
// the unfolded 16-byte row of output column l -- taps kw 0..6 at x[2l-3 .. 2l+3] and a zero
// eighth -- is assembled from lanes l-2 .. l+1 with three DPP wave shifts, then written to the
// same LDS row the DMA would have filled.  Same bf16 values (f64 -> f32 -> bf16, as the
// unfold kernel rounds), so the results are bit-identical; the unfold kernel's 134 MB write
// and the kernels' re-read of it disappear.  Needs stride 2, pad 3, kw 7 along W, even Wi.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <typename TI>
using RawV = std::conditional_t<sizeof(TI) == 8, u32x4, u32x2>;

template <typename TI>
__device__ __forceinline__ RawV<TI> raw_row_load(__amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  if constexpr (sizeof(TI) == 8) return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
  else return __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, 0);
}

// the unfolded row of output column `lane` (zero past wo) into LDS at `dst` + lane * 16;
// every lane of the wave must run it (cross-lane reads)
template <typename TI>
__device__ __forceinline__ void raw_row_commit(RawV<TI> v, int lane, int wo, char* dst) {
  float a, b;
  if constexpr (sizeof(TI) == 8) {
    a = (float)__builtin_bit_cast(double, ((uint64_t)v[1] << 32) | v[0]);
    b = (float)__builtin_bit_cast(double, ((uint64_t)v[3] << 32) | v[2]);
  } else {
    a = __uint_as_float(v[0]);
    b = __uint_as_float(v[1]);
  }
  // neighbours by DPP wave shifts (VALU: no LDS-queue traffic, so no lgkmcnt wait that would
  // drain the MFMA fragment reads in flight); lanes shifted in from outside the wave read 0
  const int me = (int)pack_bf16x2(a, b);                      // x[2l], x[2l+1]
  const uint32_t l1 = (uint32_t)__builtin_amdgcn_update_dpp(0, me, 0x138, 0xf, 0xf, true);
  const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)l1, 0x138, 0xf, 0xf, true);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_update_dpp(0, me, 0x130, 0xf, 0xf, true);
  const uint32_t m = (uint32_t)me;
  u32x4 w{(l2 >> 16) | (l1 << 16), (l1 >> 16) | (m << 16), (m >> 16) | (r1 << 16), r1 >> 16};
  if (lane >= wo) w = u32x4{0u, 0u, 0u, 0u};
  *reinterpret_cast<u32x4*>(dst + lane * 16) = w;
}

template <int KD, int KH, int SD, int SH>
__global__ __launch_bounds__(320) void stem_fwd_kernel(StemG g, const u16* __restrict__ U,
                                                       const u16* __restrict__ wp,
                                                       const float* __restrict__ bias,
                                                       u16* __restrict__ y,
                                                       float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wimg = smem;
  char* ring = smem + g.ring_off;
  float* red = reinterpret_cast<float*>(smem + g.red_off);
  constexpr int NTAP = KD * KH, NKS = (NTAP + 3) / 4;   // K-steps of 4 taps (32)
  constexpr int NTHR = 320;                               // 4 compute waves + 1 loader

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware block order: neighbouring y-pairs (sharing input rows) meet in one L2
  const int nwg = gridDim.x, bid0 = blockIdx.x;
  const int xcd = bid0 & 7, qq = nwg >> 3, rr = nwg & 7;
  const int bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid0 >> 3);
  const int zc = bid % g.nzc;
  const int yb = (bid / g.nzc) % g.nyb;
  const int nb = bid / (g.nzc * g.nyb);
  const int oz0 = zc * g.zsteps;
  const int oz1 = min(g.do_, oz0 + g.zsteps);

  // weights -> LDS once: 64 rows of kpad bf16, row stride wrow bytes (bank-spread pad)
  {
    const int cpr = g.kpad / 8;                   // 16-byte chunks per row
    for (int q = tid; q < CO * cpr; q += NTHR) {
      const int r = q / cpr, c = q % cpr;
      *reinterpret_cast<u32x4*>(wimg + r * g.wrow + c * 16) =
          *reinterpret_cast<const u32x4*>(wp + (int64_t)r * g.kpad + c * 8);
    }
  }

  // Wave 4 is the loader: it alone issues the plane DMAs, so its vmcnt counts nothing but
  // them (the compute waves' output stores would otherwise sit in the same counter and
  // turn every counted wait into a full drain).
  constexpr int YIN = (YT - 1) * SH + KH, RSTEP = SD * YIN;
  const int ybase = yb * YT * SH - g.ph;
  const bool loader = wave == 4;
  auto load_row = [&](int zi, int slot, int t) __attribute__((always_inline)) {
    const int yi = ybase + t;
    const bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi &&
                    lane < g.wo;
    const void* p = ok ? (const void*)(U + ((((int64_t)nb * g.di + zi) * g.hi + yi) * g.wo +
                                            lane) * 8)
                       : (const void*)(g_zero_kb + lane);
    glds16_asm(p, lds_addr_of(ring + (slot * YIN + t) * ROWB));
  };
  // the SD new planes of z-step ozn (RSTEP row DMAs)
  auto load_step = [&](int ozn) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < RSTEP; ++f) {
      const int kd = KD - SD + f / YIN;
      load_row(ozn * SD - g.pd + kd, (ozn * SD + kd) % g.rzf, f % YIN);
    }
  };
  if (loader) {
    // prologue: all KD planes of the first z-step, then the next step's SD new planes (the
    // ring holds KD + 2*SD planes, so the loader always runs two z-steps ahead)
#pragma unroll 1
    for (int kd = 0; kd < KD; ++kd)
#pragma unroll 1
      for (int t = 0; t < YIN; ++t) load_row(oz0 * SD - g.pd + kd, (oz0 * SD + kd) % g.rzf, t);
    if (oz0 + 1 < oz1) load_step(oz0 + 1);
  }

  const int yl = (wave >> 1) & 1, xh = wave & 1;  // compute wave: output row yl, cols xh*32..
  const int lr = lane & 15, lk = lane >> 4;
  // per K-step s, this lane's A tap (kd, kh) and B k offset
  int a_kd[NKS], a_kh[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int t = min(4 * s + lk, NTAP - 1);     // taps past NTAP have zero weights
    a_kd[s] = t / KH;
    a_kh[s] = t % KH;
  }

  // BN partial sums accumulate in registers over the block's whole z range (one partial
  // row per block, written at the end): per-z-step reductions cost more than the MFMAs
  float cs[4][4], cq[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = bias != nullptr ? bias[j * 16 + lk * 4 + r] : 0.f;
  const int oy = yb * YT + yl;
  const bool yok = oy < g.ho;

#pragma unroll 1
  for (int oz = oz0; oz < oz1; ++oz) {
    // planes of oz landed (step oz+1's RSTEP DMAs may still fly); every wave done with the
    // fragment reads of step oz-1, so its planes' slots are free for step oz+2
    if (loader) {
      if (oz + 1 < oz1) wait_vm_lgkm0<RSTEP>();
      else wait_vm_lgkm0<0>();
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    raw_barrier();
    if (loader) {
      if (oz + 2 < oz1) load_step(oz + 2);      // lands during steps oz and oz+1
      continue;
    }
    const int sbase = (oz * SD) % g.rzf;
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      int slot = sbase + a_kd[s];
      slot -= slot >= g.rzf ? g.rzf : 0;
      const char* arow = ring + (slot * YIN + yl * SH + a_kh[s]) * ROWB + (xh * 32 + lr) * 16;
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(arow + i * 256);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(wimg + (j * 16 + lr) * g.wrow +
                                                 (32 * s + 8 * lk) * 2);
      // transposed product (channels x voxels): each lane ends with 4 consecutive output
      // channels of one voxel
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }

    // epilogue straight from the accumulators: each lane owns 4 consecutive channels of
    // one voxel (8-byte stores; the 4 j-stores of a voxel fill its 128-byte line in L2), no
    // LDS C tile and no second barrier per z-step
    u16* yrow = y + (((int64_t)nb * g.do_ + oz) * g.ho + oy) * g.wo * CO;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = xh * 32 + i * 16 + lr;
      const bool ok = yok && x < g.wo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][j][r] + bv[j][r];
          if (ok) {                              // (fp32 values, as the igemm epilogue)
            cs[j][r] += v[r];
            cq[j][r] += v[r] * v[r];
          }
        }
        uint2 pk;
        pk.x = pack_bf16x2(v[0], v[1]);
        pk.y = pack_bf16x2(v[2], v[3]);
        if (ok) *reinterpret_cast<uint2*>(yrow + (int64_t)x * CO + j * 16 + lk * 4) = pk;
      }
    }
  }

  // one partial row per block: sum the 16 voxel lanes, then the 4 compute waves
  if (stats != nullptr) {
    if (!loader) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            cs[j][r] += __shfl_xor(cs[j][r], o, 64);
            cq[j][r] += __shfl_xor(cq[j][r], o, 64);
          }
          if (lr == 0) {
            red[(wave * 2) * CO + j * 16 + lk * 4 + r] = cs[j][r];
            red[(wave * 2 + 1) * CO + j * 16 + lk * 4 + r] = cq[j][r];
          }
        }
    }
    __syncthreads();
    if (tid < CO) {
      float ss = 0.f, sq = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {              // fixed order: deterministic
        ss += red[(w * 2) * CO + tid];
        sq += red[(w * 2 + 1) * CO + tid];
      }
      stats[((int64_t)bid * 2) * CO + tid] = ss;
      stats[((int64_t)bid * 2 + 1) * CO + tid] = sq;
    }
  }
}

// ---- forward, y-quad form ------------------------------------------------------------------
// Two compute waves per SIMD and no loader wave: a block owns FOUR output rows x all 64
// columns x 64 channels and walks its z range; wave w computes row w & 3, channels
// 32 (w >> 2) .. +32.  Each wave keeps its 32 x 416 weight slice in registers (26 B
// fragments), so the only LDS reads are the input rows (4 per 8 MFMAs), and the epilogue of
// z-step oz-1 (bias, BN partial sums, bf16 stores) is spread over the MFMAs of z-step oz
// (two accumulator sets).  (One wave per row with all 64 channels needs 208 VGPRs of
// weights: the compiler then serialises every input read behind its MFMAs.)  The ring holds KD + 2*SD planes of 13 rows; every
// wave issues the same number of plane DMAs (padding ones into a dummy row) and output
// stores (buffer stores whose masked lanes fall outside the resource and are dropped) per
// z-step, so one counted vmcnt wait covers "this step's planes have landed".
constexpr int YQ = 4;                      // output rows per block (one per wave)
constexpr int YINQ = (YQ - 1) * 2 + 7;     // input rows per plane
constexpr int RZQ = 7 + 2 * 2;             // ring planes
constexpr int PLQ = YINQ * ROWB;           // one plane in LDS
constexpr int NKSQ = 13;                   // K-steps of 4 taps
constexpr int NWQ = 8;                     // waves
constexpr int DMAQ = 4;                    // plane-row DMAs per wave per z-step: 26 = 2x4 + 6x3
constexpr int PROQ = 12;                   // prologue DMAs per wave (91 rows)
constexpr int STQ = 4;                     // output stores (16 B) per wave per z-step
constexpr uint32_t OOBQ = 0x40000000u;     // masked-lane store offset (past any resource)
constexpr size_t LDSQ = (size_t)RZQ * PLQ + ROWB + 4 * 2 * CO * sizeof(float);

template <bool BIAS, typename TI>
__global__ __launch_bounds__(512) void stem_fwdq_kernel(StemG g, const TI* __restrict__ U,
                                                        const u16* __restrict__ wp,
                                                        const float* __restrict__ bias,
                                                        u16* __restrict__ y,
                                                        float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool RAW = sizeof(TI) != 2;          // raw volume rows (else the unfolded U)
  constexpr int RZ = RZQ;                        // ring planes
  char* ring = smem;
  float* red = reinterpret_cast<float*>(smem + RZQ * PLQ + ROWB);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid0 = blockIdx.x;
  const int xcd = bid0 & 7, qq = nwg >> 3, rr = nwg & 7;
  const int bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid0 >> 3);
  const int zc = bid % g.nzc;
  const int yb = (bid / g.nzc) % g.nyb;
  const int xt = (bid / (g.nzc * g.nyb)) % g.nxt;  // column tile (U form only; raw: nxt 1)
  const int nb = bid / (g.nzc * g.nyb * g.nxt);
  const int x0 = xt * g.tw;
  const int oz0 = zc * g.zsteps;
  const int oz1 = min(g.do_, oz0 + g.zsteps);
  const int ybase = yb * YQ * 2 - g.ph;

  // Padding rows read past the end of a buffer resource over this sample's U
  // (the range check returns zeros without touching memory: a shared zero buffer would put
  // every block's padding reads on one L2 channel)
  const int64_t srow = RAW ? g.wi : (int64_t)g.wo * 8;         // elements per input row
  const __amdgpu_buffer_rsrc_t rsu = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(U + (int64_t)nb * g.di * g.hi * srow), 0,
      (int)__builtin_amdgcn_readfirstlane((int)(g.di * g.hi * srow * (int64_t)sizeof(TI))),
      0x00020000);
  // raw form: this lane's offset of row (zi, t), OOBQ for padding rows / lanes past Wi
  auto raw_off = [&](int zi, int t) __attribute__((always_inline)) {
    const int yi = ybase + t;
    const bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi &&
                    2 * lane < g.wi;
    return ok ? (uint32_t)(((zi * g.hi + yi) * g.wi + 2 * lane) * (int)sizeof(TI)) : OOBQ;
  };
  // raw form: the 2 new planes of z-step ozn (26 rows, <= DMAQ per wave) into registers, and
  // later into their ring rows
  auto raw_step_load = [&](int ozn, RawV<TI> (&r)[DMAQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < DMAQ; ++h) {
      const int f = wave + NWQ * h;
      if (f < 2 * YINQ)
        r[h] = raw_row_load<TI>(rsu, raw_off(ozn * 2 - g.pd + 5 + f / YINQ, f % YINQ));
    }
  };
  auto raw_step_commit = [&](int ozn, const RawV<TI> (&r)[DMAQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < DMAQ; ++h) {
      const int f = wave + NWQ * h;
      if (f < 2 * YINQ)
        raw_row_commit<TI>(r[h], lane, g.wo,
                           smem + ((ozn * 2 + 5 + f / YINQ) % RZ) * PLQ + (f % YINQ) * ROWB);
    }
  };
  auto load_row = [&](int zi, int slot, int t) __attribute__((always_inline)) {
    const int yi = ybase + t;
    bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi && lane < g.tw &&
              x0 + lane < g.wo;
#ifdef STEMQ_NO_DMA
    ok = false;                                   // (experiment: no input traffic)
#endif
    const uint32_t voff = ok ? (uint32_t)(((zi * g.hi + yi) * g.wo + x0 + lane) * 16) : OOBQ;
    buf_lds16_asm(voff, rsu, lds_addr_of(smem) + (uint32_t)(slot * PLQ + t * ROWB));
  };
  // the 2 new planes of z-step ozn: 26 rows over the 8 waves (waves 0-1: 4, others 3)
  auto load_step = [&](int ozn) __attribute__((always_inline)) {
    if (ozn >= oz1) return;
#pragma unroll
    for (int h = 0; h < DMAQ; ++h) {
      const int f = wave + NWQ * h;
      const int kd = 5 + f / YINQ;
      if (f < 2 * YINQ) load_row(ozn * 2 - g.pd + kd, (ozn * 2 + kd) % RZQ, f % YINQ);
    }
  };
  const size_t plane_out = (size_t)g.ho * g.wo * CO * 2;      // bytes of one output z-plane
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(y + (int64_t)nb * g.do_ * g.ho * g.wo * CO), 0,
      (int)__builtin_amdgcn_readfirstlane((int)(plane_out * g.do_)), 0x00020000);
  auto dummy_stores = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int e = 0; e < STQ; ++e)
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, rsy, 2 * OOBQ + e * 16, 0, 0);
  };
  // vm ops this wave issues after the DMAs of step oz: the STQ stores of step oz-2's loop,
  // step oz+1's DMAs (if that step exists), the STQ stores of step oz-1's loop.  The
  // prologue mimics that sequence with dropped stores.
  const int ndma = wave < 2 ? 4 : 3;
  auto wait_planes = [&](int oz) __attribute__((always_inline)) {
    if (oz + 1 >= oz1) wait_vm_lgkm0<2 * STQ>();
    else if (ndma == 4) wait_vm_lgkm0<2 * STQ + 4>();
    else wait_vm_lgkm0<2 * STQ + 3>();
  };

  // prologue: the 7 planes of the first z-step, then the next step's 2
  if constexpr (RAW) {
    // (registers, once, 4 rows at a time) the first step's planes; the next step's raw rows
    // into staging
#pragma unroll
    for (int h0 = 0; h0 < PROQ; h0 += 4) {
      RawV<TI> pr[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int f = wave + NWQ * (h0 + h);
        if (f < 7 * YINQ) pr[h] = raw_row_load<TI>(rsu, raw_off(oz0 * 2 - g.pd + f / YINQ, f % YINQ));
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int f = wave + NWQ * (h0 + h);
        if (f < 7 * YINQ)
          raw_row_commit<TI>(pr[h], lane, g.wo,
                             smem + ((oz0 * 2 + f / YINQ) % RZ) * PLQ + (f % YINQ) * ROWB);
      }
    }
    if (oz0 + 1 < oz1) {
      RawV<TI> r1[DMAQ];
      raw_step_load(oz0 + 1, r1);
      raw_step_commit(oz0 + 1, r1);
    }
    __builtin_amdgcn_sched_barrier(0);
  } else {
#pragma unroll 1
    for (int h = 0; h < PROQ; ++h) {
      const int f = wave + NWQ * h, kd = f / YINQ;
      if (f < 7 * YINQ) load_row(oz0 * 2 - g.pd + kd, (oz0 * 2 + kd) % RZQ, f % YINQ);
    }
    dummy_stores();
    load_step(oz0 + 1);
    dummy_stores();
  }

  const int lr = lane & 15, lk = lane >> 4;
  const int yl = wave & 3, ch = wave >> 2;
  // weights: this wave's fragments for all 13 K-steps and its 2 channel tiles (104 VGPRs).
  // Row m of tile j is channel ch*32 + (m >> 2)*8 + j*4 + (m & 3), so a lane's 4 + 4 results
  // are 8 consecutive channels (one 16-byte store per voxel)
  auto chan = [&](int j, int m) { return ch * 32 + (m >> 2) * 8 + j * 4 + (m & 3); };
  bf16x8 fb[NKSQ][2];
#pragma unroll
  for (int s = 0; s < NKSQ; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      fb[s][j] = *reinterpret_cast<const bf16x8*>(wp + (int64_t)chan(j, lr) * g.kpad + 32 * s +
                                                  8 * lk);
  // A row of this lane at K-step s: tap t = 4s + lk = 7 kd + kh; kd is the step's first plane
  // (4s / 7) or the next one, kh = (4s % 7) + lk - (next ? 7 : 0).  The last step's taps
  // 48..51 all read tap 48 (weights past tap 49 are zero; a wrapped read could hit a plane
  // still in flight or never written)
  const uint32_t lane_a = (uint32_t)((yl * 2 + lk) * ROWB + lr * 16);
  const uint32_t lane_l = (uint32_t)((yl * 2 + 6) * ROWB + lr * 16);
  float bv[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = BIAS ? bias[chan(j, lk * 4 + r)] : 0.f;
  const int oy = yb * YQ + yl;
  const bool yok = oy < g.ho;
  uint32_t so[4];
  bool xok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int x = i * 16 + lr;
    xok[i] = x < g.tw && x0 + x < g.wo;
    so[i] = yok && xok[i] ? (uint32_t)(((oy * g.wo + x0 + x) * CO + ch * 32 + lk * 8) * 2)
                          : OOBQ;
  }
  float cs[2][4], cq[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) { cs[j][r] = 0.f; cq[j][r] = 0.f; }

  // epilogue of voxel group i of the previous step's accumulators (both channel tiles).
  // Without bias the partial sums need no masking: the first step's P is zero, columns
  // x >= wo read zero input rows, and a wave whose row is past ho never writes its sums.
  // (Branch-free: a uniform branch here would split the MFMA schedule into small blocks.)
  auto epi = [&](f32x4 (&P)[4][2], int i, bool live, uint32_t soff) __attribute__((always_inline)) {
    float v[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[j][r] = P[i][j][r] + bv[j][r];
        const float vs = BIAS ? (live && xok[i] ? v[j][r] : 0.f) : v[j][r];
        cs[j][r] += vs;
        cq[j][r] = fmaf(vs, vs, cq[j][r]);
      }
    const u32x4 pk{pack_bf16x2(v[0][0], v[0][1]), pack_bf16x2(v[0][2], v[0][3]),
                   pack_bf16x2(v[1][0], v[1][1]), pack_bf16x2(v[1][2], v[1][3])};
#ifdef STEMQ_NO_STORE
    soff = OOBQ;                                  // (experiment: every store dropped)
#endif
    // (offset folded into the VGPR, soffset a literal 0: for a >8-byte MUBUF store with an
    // SGPR soffset the compiler inserts no wait state before the data registers are
    // rewritten, and on gfx950 the last lanes of the store then read the new values)
    __builtin_amdgcn_raw_buffer_store_b128(pk, rsy, so[i] + soff, 0, 0);
  };

  // z-step oz into C while the epilogue of step oz-1 (P) drains
  auto zstep = [&](f32x4 (&C)[4][2], f32x4 (&P)[4][2], int oz) __attribute__((always_inline)) {
    RawV<TI> rn[DMAQ];
    if constexpr (RAW) {
      // this wave's ring writes of step oz-1 (the planes of oz + 1) are done; the barrier
      // makes everyone's visible.  Then the raw rows of oz + 2 (two steps ahead, as the DMA
      // form) into registers: they land while the MFMAs of oz run
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
      if (oz + 2 < oz1) raw_step_load(oz + 2, rn);
    } else {
      wait_planes(oz);                             // planes of oz landed (all waves' ...)
      raw_barrier();                               // ... and step oz-1's reads are done
      load_step(oz + 2);
    }
    const bool plive = oz > oz0;
    const uint32_t psoff = plive ? (uint32_t)((oz - 1) * plane_out) : OOBQ;
    const int sb = (oz * 2) % RZ;
    auto pbk = [&](int k) __attribute__((always_inline)) {
      const int sl = sb + k;
      return (uint32_t)((sl >= RZ ? sl - RZ : sl) * PLQ);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) C[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // input fragments of K-step s (4 x 16 voxels), read one K-step ahead of their MFMAs
    auto read_a = [&](int s, bf16x8 (&fa)[4]) __attribute__((always_inline)) {
      const int kl = (4 * s) / 7, c = 7 * (kl + 1) - 4 * s;   // lanes lk >= c: next plane
      uint32_t aoff;
      if (s == NKSQ - 1) {
        aoff = pbk(6) + lane_l;
      } else if (c >= 4) {
        aoff = pbk(kl) + lane_a + (uint32_t)((4 * s) % 7) * ROWB;
      } else {
        const uint32_t lo = pbk(kl) + (uint32_t)((4 * s) % 7) * ROWB;
        const uint32_t hi = pbk(kl + 1) + (uint32_t)((4 * s) % 7) * ROWB - 7 * ROWB;
        aoff = (lk >= c ? hi : lo) + lane_a;
      }
      const char* ap = ring + aoff;
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(ap + i * 256);
    };
    bf16x8 fa[2][4];
    read_a(0, fa[0]);
#pragma unroll
    for (int s = 0; s < NKSQ; ++s) {
      if (s + 1 < NKSQ) read_a(s + 1, fa[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#ifdef STEMQ_NO_MFMA
      if (s == 0)                                 // (experiment: one K-step of MFMAs)
#endif
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          C[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][j], fa[s & 1][i], C[i][j], 0,
                                                            0, 0);
      if (s >= 2 && s < 10 && (s & 1) == 0) epi(P, (s - 2) >> 1, plive, psoff);
      // scheduling fence: the next step's reads stay ahead of this step's MFMAs (left
      // alone, the scheduler serialises every read behind the MFMAs that consume it)
      __builtin_amdgcn_sched_barrier(0);
    }
    // raw form: staging is free again (this wave's reads of it are done): the raw rows of
    // oz + 2, unfolded into the ring during the next step
    // raw form: the planes of oz + 2 into their ring slots (last read by step oz - 1, next
    // by step oz + 2)
    if constexpr (RAW)
      if (oz + 2 < oz1) raw_step_commit(oz + 2, rn);
  };
  f32x4 acc0[4][2], acc1[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int oz = oz0;
#pragma unroll 1
  for (; oz + 1 < oz1; oz += 2) {
    zstep(acc0, acc1, oz);
    zstep(acc1, acc0, oz + 1);
  }
  // the last step's epilogue (a plain tail: nothing waits on these stores)
  if (oz < oz1) {
    zstep(acc0, acc1, oz);
#pragma unroll
    for (int i = 0; i < 4; ++i) epi(acc0, i, true, (uint32_t)(oz * plane_out));
  } else if (oz > oz0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) epi(acc1, i, true, (uint32_t)((oz - 1) * plane_out));
  }
  wait_vm_lgkm0<0>();                              // (dummy DMAs into LDS before exit)

  if (stats != nullptr) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          cs[j][r] += __shfl_xor(cs[j][r], o, 64);
          cq[j][r] += __shfl_xor(cq[j][r], o, 64);
        }
        if (lr == 0) {
          red[(yl * 2) * CO + chan(j, lk * 4 + r)] = yok ? cs[j][r] : 0.f;
          red[(yl * 2 + 1) * CO + chan(j, lk * 4 + r)] = yok ? cq[j][r] : 0.f;
        }
      }
    __syncthreads();
    if (tid < CO) {
      float ss = 0.f, sq = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        ss += red[(w * 2) * CO + tid];
        sq += red[(w * 2 + 1) * CO + tid];
      }
      stats[((int64_t)bid * 2) * CO + tid] = ss;
      stats[((int64_t)bid * 2 + 1) * CO + tid] = sq;
    }
  }
}

// ---- stem weight gradient ----------------------------------------------------------------
// dW[co][k] = sum over output voxels m of dY[m][co] * U(m, k), k = (kd*7 + kh)*8 + kw.
// Same block walk as the forward (n, y-pair, z range; the U planes in an LDS ring), plus
// the block's 128 x 64 dY tile per z-step DMA'd into a 2-deep LDS ring (rows XOR-swizzled
// for the transposing reads).  8 waves; each keeps a 32 (co) x 112 (k) slice of dW in
// registers for the whole z range and issues 1/8 of the next step's DMAs (these waves
// store nothing inside the loop, so a plain vmcnt(0) waits only for DMA).  The only output
// is one fp32 partial slab per block, summed by wgrad_reduce_kernel.
constexpr int WK = 392;            // 49 taps x 8 (unfolded kw)
constexpr int WKW = 112;           // k columns per compute wave (7 MFMA tiles)

__device__ __forceinline__ int dswz(int r) { return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1); }

template <int KD, int KH, int SD, int SH>
__global__ __launch_bounds__(512) void stem_wgrad_kernel(StemG g, const u16* __restrict__ U,
                                                         const u16* __restrict__ dy,
                                                         float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int YIN = (YT - 1) * SH + KH, RSTEP = SD * YIN;
  constexpr int DYB = YT * XW * CO * 2;            // one dY tile: 128 rows x 128 B
  char* ring = smem;                               // U planes
  char* dyr = smem + g.ring_off;                   // 2 dY tiles (ring_off reused as offset)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid0 = blockIdx.x;
  const int xcd = bid0 & 7, qq = nwg >> 3, rr = nwg & 7;
  const int bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid0 >> 3);
  const int zc = bid % g.nzc;
  const int yb = (bid / g.nzc) % g.nyb;
  const int nb = bid / (g.nzc * g.nyb);
  const int oz0 = zc * g.zsteps;
  const int oz1 = min(g.do_, oz0 + g.zsteps);
  const int ybase = yb * YT * SH - g.ph;

  auto load_row = [&](int zi, int slot, int t) __attribute__((always_inline)) {
    const int yi = ybase + t;
    const bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi &&
                    lane < g.wo;
    const void* p = ok ? (const void*)(U + ((((int64_t)nb * g.di + zi) * g.hi + yi) * g.wo +
                                            lane) * 8)
                       : (const void*)(g_zero_kb + lane);
    glds16_asm(p, lds_addr_of(ring + (slot * YIN + t) * ROWB_W));
  };
  // dY tile of z-step oz: 128 rows (voxel m = yl*64 + x) of 64 channels; one DMA
  // instruction = 8 rows; lane chunk swizzled so the transposing reads are conflict-free
  auto load_dy = [&](int oz, int buf, int q) __attribute__((always_inline)) {
    {
      const int row = q * 8 + (lane >> 3);
      const int ry = row >> 6, x = row & 63, yy = yb * YT + ry;
      const int ch = (lane & 7) ^ dswz(row);
      const bool ok = x < g.wo && yy < g.ho;
      const void* p = ok ? (const void*)(dy + ((((int64_t)nb * g.do_ + oz) * g.ho + yy) * g.wo +
                                              x) * CO + ch * 8)
                         : (const void*)(g_zero_kb + lane);
      glds16_asm(p, lds_addr_of(dyr + buf * DYB + q * 1024));
    }
  };
  // the new planes + dY tile of z-step ozn: RSTEP + 16 DMAs spread over the 8 waves
  auto load_step = [&](int ozn) __attribute__((always_inline)) {
#pragma unroll 1
    for (int f = wave; f < RSTEP + 16; f += 8) {
      if (f < RSTEP) {
        const int kd = KD - SD + f / YIN;
        load_row(ozn * SD - g.pd + kd, (ozn * SD + kd) % g.rz, f % YIN);
      } else {
        load_dy(ozn, ozn & 1, f - RSTEP);
      }
    }
  };
  if (oz0 < oz1) {
#pragma unroll 1
    for (int f = wave; f < (KD - SD) * YIN; f += 8) {
      const int kd = f / YIN;
      load_row(oz0 * SD - g.pd + kd, (oz0 * SD + kd) % g.rz, f % YIN);
    }
    load_step(oz0);
  }

  // compute wave w: channels [32*(w&1), +32), k columns [112*(w>>1), +112) = 14 taps
  const int q = (lane & 15) >> 2, p = lane & 3, lk = lane >> 4;
  const int wc = wave & 1, wk = wave >> 1;
  f32x4 acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's B columns: k-tile j covers taps 2*(7w + j) + (p >> 1), kw 4*(p & 1)..+3
  // packed per k-tile: plane kd in bits 20+, byte offset (kh row + kw half) below
  int b_off[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int t = min(2 * (7 * wk + j) + (p >> 1), KD * KH - 1);
    b_off[j] = ((t / KH) << 20) | ((t % KH) * ROWB_W + (p & 1) * 8);
  }

#pragma unroll 1
  for (int oz = oz0; oz < oz1; ++oz) {
    wait_vm_lgkm0<0>();                            // this wave's DMAs for oz landed
    raw_barrier();                                 // ... and everyone's; step oz-1 done
    if (oz + 1 < oz1) load_step(oz + 1);          // lands while the MFMAs of oz run
    const int sbase = (oz * SD) % g.rz;
    const char* dyt = dyr + (oz & 1) * DYB;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {               // 32 voxels per K-step
      const int yl = ks >> 1;
      const int r0 = 32 * ks + 8 * lk + q, r1 = r0 + 4;
      bf16x8 fa[2], fb[7];
#pragma unroll
      for (int i = 0; i < 2; ++i) {                // dY^T: co tile i of this wave's half
        const int col = wc * 32 + i * 16 + 4 * p;
        const int ch = col >> 3, cb = (col & 7) * 2;
        const char* lo = dyt + r0 * 128 + ((ch ^ dswz(r0)) << 4) + cb;
        const char* hi = dyt + r1 * 128 + ((ch ^ dswz(r1)) << 4) + cb;
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)lo);
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)hi);
        fa[i] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      const int x0 = (r0 & 63), x1 = (r1 & 63);
#pragma unroll
      for (int j = 0; j < 7; ++j) {                // U: k tile j
        int slot = sbase + (b_off[j] >> 20);
        slot -= slot >= g.rz ? g.rz : 0;
        const char* rowp = ring + (slot * YIN + yl * SH) * ROWB_W + (b_off[j] & 0xfffff);
        bf16x4 vlo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(rowp + x0 * 16));
        bf16x4 vhi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(rowp + x1 * 16));
        fb[j] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  // this block's partial slab: ws[bid][co][k], k < 392
  float* out = ws + (int64_t)bid * CO * WK;
  const int lr = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int k = wk * WKW + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = wc * 32 + i * 16 + lk * 4 + r;
        if (k < WK) out[(int64_t)co * WK + k] = acc[i][j][r];
      }
    }
}

// Same walk and output as stem_wgrad_kernel with the per-step address arithmetic hoisted:
// every DMA of a wave has a fixed lane offset into a per-sample buffer resource that only
// moves by a constant per z-step (padding rows fall past the resource and read zeros, so no
// shared zero buffer and no per-row range checks), and every LDS fragment read is a
// per-z-step base register plus an immediate.  The next K-step's fragments are read ahead
// of the current MFMAs (fenced, so the scheduler keeps them there).
template <int KD, int KH, int SD, int SH, typename TI>
__global__ __launch_bounds__(512) void stem_wgrad2_kernel(StemG g, const TI* __restrict__ U,
                                                          const u16* __restrict__ dy,
                                                          float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int YIN = (YT - 1) * SH + KH, RSTEP = SD * YIN;
  // ring planes (geom_for's g.rz = kd + sd) as a compile-time constant: the per-z-step slot
  // arithmetic (mod RZW) then needs no run-time scalar division
  constexpr int RZW = KD + SD;
  constexpr int DYB = YT * XW * CO * 2;
  constexpr int NH = (RSTEP + 16 + 7) / 8;          // DMA slots per wave per step
  constexpr uint32_t OOB = 0x80000000u;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = gridDim.x, bid0 = blockIdx.x;
  const int xcd = bid0 & 7, qq = nwg >> 3, rr = nwg & 7;
  const int bid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid0 >> 3);
  const int zc = bid % g.nzc;
  const int yb = (bid / g.nzc) % g.nyb;
  const int xt = (bid / (g.nzc * g.nyb)) % g.nxt;  // column tile (U form only; raw: nxt 1)
  const int nb = bid / (g.nzc * g.nyb * g.nxt);
  const int x0 = xt * g.tw;
  const int oz0 = zc * g.zsteps;
  const int oz1 = min(g.do_, oz0 + g.zsteps);
  const int ybase = yb * YT * SH - g.ph;
  const uint32_t ring_l = lds_addr_of(smem), dyr_l = ring_l + (uint32_t)g.ring_off;
  constexpr bool RAW = sizeof(TI) != 2;          // raw volume rows (else the unfolded U)

  const int64_t srow = RAW ? g.wi : (int64_t)g.wo * 8;         // elements per input row
  const __amdgpu_buffer_rsrc_t rsu = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(U + (int64_t)nb * g.di * g.hi * srow), 0,
      (int)__builtin_amdgcn_readfirstlane((int)(g.di * g.hi * srow * (int64_t)sizeof(TI))),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dy + (int64_t)nb * g.do_ * g.ho * g.wo * CO), 0,
      (int)__builtin_amdgcn_readfirstlane(g.do_ * g.ho * g.wo * CO * 2), 0x00020000);
  const uint32_t ustep = (uint32_t)(SD * g.hi * srow * (int64_t)sizeof(TI));
  const uint32_t dstep = (uint32_t)(g.ho * g.wo * CO * 2);

  // this wave's DMA slots h: f = wave + 8h; U rows of the step's SD new planes (f < RSTEP),
  // then the 16 dY pieces (8 rows x 128 B each, chunk-swizzled for the transposing reads)
  uint32_t voff[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int f = wave + 8 * h;
    voff[h] = OOB;
    if (f < RSTEP) {
      const int kd = KD - SD + f / YIN, yi = ybase + f % YIN;
      if (RAW && (unsigned)yi < (unsigned)g.hi && 2 * lane < g.wi)
        voff[h] = (uint32_t)((((kd - g.pd) * g.hi + yi) * g.wi + 2 * lane) * (int)sizeof(TI));
      else if (!RAW && (unsigned)yi < (unsigned)g.hi && lane < g.tw && x0 + lane < g.wo)
        voff[h] = (uint32_t)((((kd - g.pd) * g.hi + yi) * g.wo + x0 + lane) * 16);
    } else if (f < RSTEP + 16) {
      const int row = (f - RSTEP) * 8 + (lane >> 3);
      const int x = row & 63, yy = yb * YT + (row >> 6);
      const int ch = (lane & 7) ^ dswz(row);
      if (x < g.tw && x0 + x < g.wo && yy < g.ho)
        voff[h] = (uint32_t)(((yy * g.wo + x0 + x) * CO + ch * 8) * 2);
    }
  }
  // raw form: this wave's U rows of the next step in registers (issued with its dY DMAs),
  // unfolded into the ring at the end of the current step
  RawV<TI> rv[NH];
  auto raw_commit_step = [&](int ozn) __attribute__((always_inline)) {
    int sbn = (ozn * SD) % RZW;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int f = wave + 8 * h;
      if (f < RSTEP) {
        int slot = sbn + KD - SD + f / YIN;
        slot -= slot >= RZW ? RZW : 0;
        raw_row_commit<TI>(rv[h], lane, g.wo, smem + (slot * YIN + f % YIN) * ROWB_W);
      }
    }
  };
  auto load_step = [&](int ozn, bool urows = true) __attribute__((always_inline)) {
    int sbn = (ozn * SD) % RZW;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int f = wave + 8 * h;
      if (f < RSTEP) {
        int slot = sbn + KD - SD + f / YIN;
        slot -= slot >= RZW ? RZW : 0;
        if constexpr (RAW) {
          if (urows) rv[h] = raw_row_load<TI>(rsu, voff[h] + (uint32_t)ozn * ustep);
        } else {
          buf_lds16_asm(voff[h] + (uint32_t)ozn * ustep, rsu,
                        ring_l + (uint32_t)((slot * YIN + f % YIN) * ROWB_W));
        }
      } else if (f < RSTEP + 16) {
        buf_lds16_asm(voff[h] + (uint32_t)ozn * dstep, rsd,
                      dyr_l + (uint32_t)((ozn & 1) * DYB + (f - RSTEP) * 1024));
      }
    }
  };
  if (oz0 < oz1) {
    // prologue: the first step's KD - SD older planes (generic addressing, once)
    if constexpr (RAW) {
      // (registers, once) all KD planes of the first step; then its dY tile and the next
      // step's raw rows into staging
      constexpr int NPR = (KD * YIN + 7) / 8;
      RawV<TI> pr[NPR];
#pragma unroll
      for (int h = 0; h < NPR; ++h) {
        const int f = wave + 8 * h;
        if (f < KD * YIN) {
          const int kd = f / YIN, zi = oz0 * SD - g.pd + kd, yi = ybase + f % YIN;
          const bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi &&
                          2 * lane < g.wi;
          pr[h] = raw_row_load<TI>(
              rsu, ok ? (uint32_t)(((zi * g.hi + yi) * g.wi + 2 * lane) * (int)sizeof(TI)) : OOB);
        }
      }
#pragma unroll
      for (int h = 0; h < NPR; ++h) {
        const int f = wave + 8 * h;
        if (f < KD * YIN)
          raw_row_commit<TI>(pr[h], lane, g.wo,
                             smem + (((oz0 * SD + f / YIN) % RZW) * YIN + f % YIN) * ROWB_W);
      }
      load_step(oz0, false);                     // (its dY tile; its U rows are in)
    } else {
#pragma unroll 1
      for (int f = wave; f < (KD - SD) * YIN; f += 8) {
        const int kd = f / YIN, zi = oz0 * SD - g.pd + kd, yi = ybase + f % YIN;
        const bool ok = (unsigned)zi < (unsigned)g.di && (unsigned)yi < (unsigned)g.hi &&
                        lane < g.tw && x0 + lane < g.wo;
        buf_lds16_asm(ok ? (uint32_t)(((zi * g.hi + yi) * g.wo + x0 + lane) * 16) : OOB, rsu,
                      ring_l + (uint32_t)((((oz0 * SD + kd) % RZW) * YIN + f % YIN) * ROWB_W));
      }
      load_step(oz0);
    }
  }

  // compute wave w: channels [32*(w&1), +32), k columns [112*(w>>1), +112) = 14 taps
  const int q = (lane & 15) >> 2, p = lane & 3, lk = lane >> 4;
  const int wc = wave & 1, wk = wave >> 1;
  // U fragment of k-tile j: tap t_j = 2*(7 wk + j) + (p >> 1) = 7 kd_j + kh_j; the lane's
  // row offset in its plane (kh_j row, kw half, voxel x = 8 lk + q of the K-step's 32)
  int kdj[7];
  uint32_t rowj[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int t = min(2 * (7 * wk + j) + (p >> 1), KD * KH - 1);
    kdj[j] = t / KH;
    rowj[j] = (uint32_t)((t % KH) * ROWB_W + (p & 1) * 8 + (8 * lk + q) * 16);
  }
  // dY^T fragment of co tile i: rows r0 = 32 ks + 8 lk + q (and r0 + 4), swizzled chunk
  uint32_t dlo[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int col = wc * 32 + i * 16 + 4 * p, r0 = 8 * lk + q;
    dlo[i] = (uint32_t)(r0 * 128 + (((col >> 3) ^ dswz(r0)) << 4) + (col & 7) * 2);
  }
  f32x4 acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int oz = oz0; oz < oz1; ++oz) {
    // this wave's DMAs for oz landed.  (Raw form: as the builtin, which the compiler's wait
    // bookkeeping sees -- after the opaque asm form it still counted the previous step's
    // register loads as pending and put a vmcnt(0) before every new one.)
    if constexpr (RAW) __builtin_amdgcn_s_waitcnt(0);
    else wait_vm_lgkm0<0>();
    raw_barrier();                                 // ... and everyone's; step oz-1 done
#ifndef STEMW_NO_DMA
    if (oz + 1 < oz1) load_step(oz + 1);          // lands while the MFMAs of oz run
#endif

    const int sbase = (oz * SD) % RZW;
    const char* dyt = smem + g.ring_off + (oz & 1) * DYB;
    const char* pl[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      int slot = sbase + kdj[j];
      slot -= slot >= RZW ? RZW : 0;
      pl[j] = smem + slot * YIN * ROWB_W + rowj[j];
    }
    auto rd = [&](const char* a) __attribute__((always_inline)) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)a);
    };
    auto read_k = [&](int ks, bf16x8 (&fa)[2], bf16x8 (&fb)[7]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const char* a = dyt + dlo[i] + ks * 32 * 128;
        fa[i] = __builtin_shufflevector(rd(a), rd(a + 4 * 128), 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const char* b = pl[j] + (ks >> 1) * SH * ROWB_W + (ks & 1) * 32 * 16;
        fb[j] = __builtin_shufflevector(rd(b), rd(b + 4 * 16), 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    bf16x8 fa[2][2], fb[2][7];
    read_k(0, fa[0], fb[0]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks + 1 < 4) read_k(ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#ifdef STEMW_NO_MFMA
      if (ks == 0)                                // (experiment: one K-step of MFMAs)
#endif
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks & 1][i], fb[ks & 1][j],
                                                              acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // raw form: the next step's U rows into their ring slots (free during step oz; read
    // after the loop-top wait + barrier)
    if constexpr (RAW)
      if (oz + 1 < oz1) raw_commit_step(oz + 1);
  }
  // this block's partial slab: ws[bid][co][k], k < 392
  float* out = ws + (int64_t)bid * CO * WK;
  const int lr = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int k = wk * WKW + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = wc * 32 + i * 16 + lk * 4 + r;
        if (k < WK) out[(int64_t)co * WK + k] = acc[i][j][r];
      }
    }
}

// MMAD_STEM_WG2=0 keeps the first stem weight-gradient kernel (A/B switch)
bool wg2_on() {
  static const bool on = [] {
    const char* e = getenv("MMAD_STEM_WG2");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

// MMAD_STEM_QUAD=0 keeps the y-pair forward kernel (A/B switch)
bool quad_on() {
  static const bool on = [] {
    const char* e = getenv("MMAD_STEM_QUAD");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

bool geom_for(const mmad_conv_desc* d, StemG& g, int& blocks, size_t& lds, bool quad = false) {
  if (d->ci != 1 || d->co != CO || d->kd != 7 || d->kh != 7 || d->kw > 8) return false;
  if (d->sd != 2 || d->sh != 2) return false;     // the instantiated form (MedicalNet)
  if (d->dd != 1 || d->dh != 1 || d->dw != 1 || d->wo < 1) return false;
  g = StemG{};
  // rows wider than the 64 lanes (config 5's 160^3: wo 80) split into equal column tiles,
  // one per block; the tiled forms read the W-unfolded U (the raw forms need wi <= 128)
  g.nxt = (int)cdiv(d->wo, XW);
  g.tw = (int)cdiv(d->wo, g.nxt);
  g.n = d->n; g.di = d->di; g.hi = d->hi; g.wo = d->wo; g.do_ = d->do_; g.ho = d->ho;
  g.wi = d->wi;
  g.sd = d->sd; g.sh = d->sh; g.pd = d->pd; g.ph = d->ph;
  const int ntap = d->kd * d->kh;
  g.kpad = (int)cdiv(ntap * 8, 64) * 64;        // as mmad_conv_pack_weight (mode 2)
  // weight row stride: (wrow / 16) % 16 == 10 makes the B-fragment reads (16 rows x 4 tap
  // groups per 16-lane ds_read_b128 group) hit 16 distinct 16-byte bank slots; the former
  // +16-byte pad (57 slots: % 16 == 9) put up to 8 lanes of a group on one slot
  g.wrow = g.kpad * 2 + 16 * (int)(((10 - (g.kpad * 2 / 16)) % 16 + 16) % 16);
  g.rz = d->kd + g.sd;                           // planes of this and the next z-step
  g.rzf = d->kd + 2 * g.sd;                      // forward: and the one after
  const int yt = quad ? YQ : YT;
  g.yin = (yt - 1) * g.sh + d->kh;
  g.nks = (int)cdiv(ntap, 4);
  if (g.nks > 16 || g.kpad < g.nks * 32) return false;
  if (quad && ((int64_t)g.ho * g.wo * CO * 2 * g.do_ >= (int64_t(1) << 30) ||
               (int64_t)g.di * g.hi * g.wo * 16 >= (int64_t(1) << 30) || g.rzf != RZQ ||
               g.yin != YINQ || g.nks != NKSQ))
    return false;
  g.nyb = (int)cdiv(g.ho, yt);
  const int64_t base = (int64_t)g.n * g.nyb * g.nxt;
  g.nzc = (int)std::max<int64_t>(1, std::min<int64_t>(g.do_, cdiv(256, base)));
  g.zsteps = (int)cdiv(g.do_, g.nzc);
  g.nzc = (int)cdiv(g.do_, g.zsteps);
  g.ring_off = CO * g.wrow;
  g.c_off = g.ring_off + g.rzf * g.yin * ROWB;   // (no C tile: the epilogue stores directly)
  g.red_off = g.c_off;
  lds = quad ? LDSQ : (size_t)g.red_off + 4 * 2 * CO * sizeof(float);
  blocks = (int)(base * g.nzc);
  return lds <= 160 * 1024 && base * g.nzc < (int64_t(1) << 31);
}

}  // namespace

namespace mmad_stem {

bool raw_ok(const mmad_conv_desc* d, int in_dtype) {
  StemG g;
  int blocks;
  size_t lds;
  if (in_dtype != MMAD_F64) return false;         // (16-byte raw rows: f64 only)
  if (d->kw != 7 || d->sw != 2 || d->pw != 3 || d->dw != 1 || d->wi % 2 || d->wi > 2 * XW)
    return false;
  if (!quad_on() || !geom_for(d, g, blocks, lds, true)) return false;
  // 32-bit buffer offsets over one sample's volume
  return (int64_t)d->di * d->hi * d->wi * 8 < (int64_t(1) << 30) &&
         (int64_t)d->do_ * d->ho * d->wo * CO * 2 < (int64_t(1) << 30);
}

// the hoisted weight gradient's buffer offsets are 32-bit
static bool wg2_small(const StemG& g) {
  return (int64_t)g.di * g.hi * g.wo * 16 < (int64_t(1) << 30) &&
         (int64_t)g.do_ * g.ho * g.wo * CO * 2 < (int64_t(1) << 30);
}

bool fwd_ok(const mmad_conv_desc* d, int dtype) {
  StemG g;
  int blocks;
  size_t lds;
  if (dtype != MMAD_BF16 || !geom_for(d, g, blocks, lds)) return false;
  if (g.nxt == 1) return true;
  // column tiles: the y-quad forward and the hoisted weight gradient only -- and the
  // weight gradient's 32-bit offsets must hold, or the backward would have no stem route
  // (so the whole conv takes the generic unfold path from the forward on)
  return quad_on() && wg2_on() && wg2_small(g) && geom_for(d, g, blocks, lds, true);
}

int64_t fwd_stats_rows(const mmad_conv_desc* d) {
  StemG g;
  int blocks;
  size_t lds;
  if (!(quad_on() && geom_for(d, g, blocks, lds, true)) && !geom_for(d, g, blocks, lds))
    return -1;
  return blocks;                                 // one BN partial row per block
}

int64_t wgrad_blocks(const mmad_conv_desc* d) {
  StemG g;
  int blocks;
  size_t lds;
  if (!geom_for(d, g, blocks, lds)) return -1;
  return blocks;
}

int wgrad(const mmad_conv_desc* d, const void* x_unf, const void* dy, float* ws, void* stream,
          int in_dtype) {
  StemG g;
  int blocks;
  size_t lds;
  if (!geom_for(d, g, blocks, lds)) return MMAD_EUNSUPPORTED;
  if (in_dtype >= 0 && !raw_ok(d, in_dtype)) return MMAD_EUNSUPPORTED;
  if (g.nxt > 1 && in_dtype >= 0) return MMAD_EUNSUPPORTED;
  // LDS: U plane ring, then two dY tiles
  g.ring_off = g.rz * g.yin * ROWB_W;
  const size_t wl = (size_t)g.ring_off + 2 * YT * XW * CO * 2;
  auto attr = [](const void* k) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
           hipSuccess;
  };
  static const bool ok = attr((const void*)stem_wgrad_kernel<7, 7, 2, 2>) &&
                         attr((const void*)stem_wgrad2_kernel<7, 7, 2, 2, u16>) &&
                         attr((const void*)stem_wgrad2_kernel<7, 7, 2, 2, double>);
  if (!ok || wl > 160 * 1024) return MMAD_EUNSUPPORTED;
  const bool small = wg2_small(g);
  if (in_dtype == MMAD_F64)
    hipLaunchKernelGGL((stem_wgrad2_kernel<7, 7, 2, 2, double>), dim3((unsigned)blocks),
                       dim3(512), wl, as_stream(stream), g, (const double*)x_unf, (const u16*)dy,
                       ws);
  else if (wg2_on() && small)
    hipLaunchKernelGGL((stem_wgrad2_kernel<7, 7, 2, 2, u16>), dim3((unsigned)blocks), dim3(512), wl,
                       as_stream(stream), g, (const u16*)x_unf, (const u16*)dy, ws);
  else if (g.nxt > 1)
    return MMAD_EUNSUPPORTED;                     // (the first kernel has no column tiles)
  else
    hipLaunchKernelGGL((stem_wgrad_kernel<7, 7, 2, 2>), dim3((unsigned)blocks), dim3(512), wl,
                       as_stream(stream), g, (const u16*)x_unf, (const u16*)dy, ws);
  return launch_status();
}

template <typename TI>
int launch_fwdq(const StemG& g, int blocks, const void* x, const void* w_packed,
                const float* bias, void* y, float* stats, void* stream) {
  constexpr size_t lds = LDSQ;
  static const bool okq =
      hipFuncSetAttribute((const void*)stem_fwdq_kernel<false, TI>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
      hipFuncSetAttribute((const void*)stem_fwdq_kernel<true, TI>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!okq) return MMAD_EUNSUPPORTED;
  if (bias != nullptr)
    hipLaunchKernelGGL((stem_fwdq_kernel<true, TI>), dim3((unsigned)blocks), dim3(512), lds,
                       as_stream(stream), g, (const TI*)x, (const u16*)w_packed, bias, (u16*)y,
                       stats);
  else
    hipLaunchKernelGGL((stem_fwdq_kernel<false, TI>), dim3((unsigned)blocks), dim3(512), lds,
                       as_stream(stream), g, (const TI*)x, (const u16*)w_packed, bias, (u16*)y,
                       stats);
  return launch_status();
}

int fwd(const mmad_conv_desc* d, const void* x_unf, const void* w_packed, const float* bias,
        void* y, float* stats, void* stream, int in_dtype) {
  StemG g;
  int blocks;
  size_t lds;
  if (in_dtype >= 0) {
    if (!raw_ok(d, in_dtype) || !geom_for(d, g, blocks, lds, true)) return MMAD_EUNSUPPORTED;
    return launch_fwdq<double>(g, blocks, x_unf, w_packed, bias, y, stats, stream);
  }
  if (quad_on() && geom_for(d, g, blocks, lds, true))
    return launch_fwdq<u16>(g, blocks, x_unf, w_packed, bias, y, stats, stream);
  if (!geom_for(d, g, blocks, lds) || g.nxt > 1) return MMAD_EUNSUPPORTED;
  static const bool ok = hipFuncSetAttribute((const void*)stem_fwd_kernel<7, 7, 2, 2>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024) == hipSuccess;
  if (!ok) return MMAD_EUNSUPPORTED;
  hipLaunchKernelGGL((stem_fwd_kernel<7, 7, 2, 2>), dim3((unsigned)blocks), dim3(320), lds,
                     as_stream(stream), g, (const u16*)x_unf, (const u16*)w_packed, bias, (u16*)y,
                     stats);
  return launch_status();
}

}  // namespace mmad_stem
