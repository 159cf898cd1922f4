// Patch-resident weight gradient for dense stride-1 3^3 convolutions (dilation 1, padding 1)
// on volumes 32 voxels wide, gfx950 (bf16 operands, fp32 accumulate): the MedicalNet layer1
// convs (64 -> 64 at 32^3, reached from pkg/models/mri_models/anat_cnn.py:29-31).
//
// dW[co][tap][ci] = sum over output voxels v of dY[v][co] * X[v + tap - 1][ci].  The
// row-gather wgrad (conv.hip wgrad_kernel) DMAs one gathered 32-voxel K row per tap, so
// at 64 channels it issues three LDS-DMA instructions per eight MFMAs per wave and runs
// issue-bound.  Here, as in the residue-class lattice wgrad (latticeconv.hip), a block keeps
// the input planes it needs resident and builds every tap's fragments from them:
//  * block = 64 output channels x 32 input channels x all 27 taps over a split
//    (sample, 8-row y tile, z range); 8 waves = 2 (16-channel ci halves) x 4 tap groups of
//    7 (6); per wave 4 x 7 accumulator tiles;
//  * a K step is one output row (32 voxels): the dY rows are 32 consecutive x, and a tap's
//    X rows are the 32 x of row (y + ky, z + kz) shifted by kx.  X plane images hold the
//    tile's 10 rows x 34 x positions (the x = -1 / 32 padding as zero rows, and the
//    padding rows / planes read past a buffer resource, i.e. zeros), so every tap's block
//    of 32 rows is contiguous and no tap needs a validity test;
//  * input planes stream through a 4-slot ring (plane o + 3 issued when output plane o
//    starts); dY (2 output rows x 64 channels = 8 KiB per stage) through a 3-slot ring;
//  * both operands are read with transposing ds_read_b64_tr_b16 fragment reads; the dY
//    image is chunk-swizzled (conflict-free), the X image is not (its taps shift the row
//    by kx, which a row-keyed swizzle cannot follow without per-read address math), so the
//    X reads run 2-way bank-conflicted;
//  * fp32 partial slabs [split][co][tap * Cs + ci], summed and transposed by conv.hip's
//    wgrad_reduce_t_kernel.
#include "common.h"
#include "patchconv.h"

namespace {

constexpr int PW_KC = 32;                        // input channels per block
constexpr int PW_TY = 8;                         // output rows per y tile
constexpr int PW_XW = 32;                        // voxels per row (one K step)
constexpr int PW_YR = PW_TY + 2;                 // y rows per plane image
constexpr int PW_XSLOTS = 4;
constexpr int PW_YROW = 128;                     // dY rows: 64 co x 2 B
constexpr int PW_YST = 2 * PW_XW * PW_YROW;      // 8 KiB: 2 K steps per stage
constexpr int PW_YSLOTS = 4;                     // (4: the slot of stage s is s & 3, no run-time mod 3)
constexpr int PW_NTHR = 512;
constexpr uint32_t PW_OOB = 0x80000000u;
// LAT = false: the 32-wide volume (layer1); a K step is one 32-voxel row and an image row
// group holds its 34 x positions (x = -1 .. 32).
// LAT = true: the residue-class form for layer3's dilation-2 convs (16^3 grid, 8 classes of
// 8^3 sub-lattices, pkg/models/mri_models/anat_cnn.py:29-31): a K step is one sub-lattice
// row (z', y') of the 4 classes (ry, rx) of one rz, as 4 segments of 8 voxels (x' = 0..7),
// and an image row group holds 4 x 10 positions (x' = -1 .. 8 per segment, the pads zero
// rows).  The transposing fragment reads cover 8 K rows per 16-lane group, i.e. exactly one
// segment, so a tap's kx shift stays a per-lane constant plus an immediate and the layer1
// loop runs unchanged; a split is (sample, rz, z range) -- or (sample, z range) with both rz
// groups walked as one plane stream (g.ng = 2) -- and taps whose y shift leaves the
// sub-lattice are skipped at compile time (the y tile is the whole 8-row sub-lattice).
// W16 (MODE 2): 16-wide volumes (layer2's stride-1 conv on the 16^3 grid): a K step is two
// consecutive 16-voxel rows (y, y + 1) of one plane, as 2 segments of 16 (the 16-lane groups
// lk = 0, 1 read segment 0, lk = 2, 3 segment 1); the y tile is the whole 16-row plane and an
// image row group holds 18 x positions (x = -1 .. 16), 18 rows of them.
// W40 (MODE 3, round 5): 40-wide volumes (config 5's layer1 at 40^3, 160^3 input): a row is
// 5 segments of 8 voxels and a K step is 4 consecutive segments of the y tile in row-major
// order (every 4 rows = 20 segments = 5 K steps, none wasted); an image row group holds the
// 5 segments with their own x halos (x' = -1 .. 8 per segment, 50 positions; the halos
// between segments are real voxels, the row ends zero), so lane group lk reads its segment
// at a per-K-step lane offset (5 of them, the pattern's period) plus the tap's immediate.
// MODE: 0 the 32-wide form, 1 LAT, 2 W16, 3 W40
template <int MODE>
struct PWC {
  static constexpr bool LAT = MODE == 1, W16 = MODE == 2, W40 = MODE == 3;
  static constexpr int XR = LAT ? 40 : W16 ? 18 : W40 ? 50 : PW_XW + 2;  // positions per y row
  static constexpr int SPP = W40 ? 5 : 4;                    // dY stages per output plane
  static constexpr int YRI = W16 ? 18 : PW_YR;               // image y rows
  static constexpr int XROWS = YRI * XR;                     // 400 / 324 / 340 / 500 rows
  static constexpr int XDMA = (XROWS + 15) / 16;             // 25 / 21 / 22 / 32 DMAs
  static constexpr int XSLOT = XDMA * 1024;
  static constexpr int Y_OFF = PW_XSLOTS * XSLOT;
  static constexpr int LDS = Y_OFF + PW_YSLOTS * PW_YST;
  static constexpr int NXMAX = (XDMA + 7) / 8;               // X DMA instructions per wave
};

struct PWG {
  int nb, Cs, Nd, D, H, K;
  int zr;                                        // output planes per split
  int ng;                                        // LAT: class groups (rz) per block, 1 or 2
};

__device__ __forceinline__ int pw_wsz128(int r) { return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1); }

template <int MODE>
__global__ __launch_bounds__(PW_NTHR) void pwgrad_kernel(PWG g, const u16* __restrict__ x,
                                                         const u16* __restrict__ dy,
                                                         float* __restrict__ ws) {
  using C = PWC<MODE>;
  constexpr bool LAT = C::LAT, W16 = C::W16, W40 = C::W40;
  constexpr int XR = C::XR, SPP = C::SPP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware order: the co tiles and ci chunks of one split (same planes) stay together
  const int nci = g.Cs / PW_KC, nco = g.Nd / 64;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int cot = tile % nco, t2 = tile / nco;
  const int cit = t2 % nci, split = t2 / nci;
  // split = (n, y tile, z range); LAT: (n, rz, z range), rz the class group (or, with
  // g.ng = 2, (n, z range): the block walks both groups as one stream)
  const int nyt = LAT ? 2 / g.ng : W16 ? 1 : g.H / PW_TY, nzr = (LAT ? 8 : g.D) / g.zr;
  const int zi = split % nzr, yt = (split / nzr) % nyt, n = split / (nzr * nyt);
  const int rz = LAT ? yt : 0;                    // (first) class group
  const int co0 = cot * 64, ci0 = cit * PW_KC, y0 = LAT || W16 ? 0 : yt * PW_TY, z0 = zi * g.zr;
  constexpr int VW = LAT || W16 ? 16 : W40 ? 40 : PW_XW;   // voxels per volume row

  const int64_t vox = LAT ? (int64_t)16 * 16 * 16 : (int64_t)g.D * g.H * VW;
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + n * vox * g.Cs), 0, (int)__builtin_amdgcn_readfirstlane((int)(vox * g.Cs * 2)),
      0x00020000);
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dy + n * vox * g.Nd), 0, (int)__builtin_amdgcn_readfirstlane((int)(vox * g.Nd * 2)),
      0x00020000);
  const uint32_t smem_l = lds_addr_of(smem);

  // X plane image DMA: instruction q of a plane = image rows 16q..16q+15 (row = yy*34 + xx);
  // wave w issues q = w, w + 8, w + 16 (< 22).  Input plane iz adds iz * plane bytes (iz = -1
  // wraps past the resource; iz = D lands past it: zeros either way)
  // (the lane offsets are recomputed per plane: a few VALU per DMA; held in registers they
  // were spilled by the MFMA loop and reloaded behind a full vmcnt drain)
  const int nx = wave + 8 * (C::NXMAX - 1) < C::XDMA ? C::NXMAX : C::NXMAX - 1;
  auto xoff = [&](int h) -> uint32_t {
    const int q = wave + 8 * h, row = 16 * q + (lane >> 2);
    if constexpr (LAT) {
      // image row = (y' + 1) * 40 + segment * 10 + x' + 1; segment = class (ry, rx)
      const int yv = row / XR - 1, ps = row % XR, sg = ps / 10, xv = ps % 10 - 1;
      const bool ok = row < C::XROWS && (unsigned)yv < 8u && (unsigned)xv < 8u;
      const int vy = (sg >> 1) + 2 * yv, vx = (sg & 1) + 2 * xv;
      return ok ? (uint32_t)(((vy * 16 + vx) * g.Cs + ci0 + (lane & 3) * 8) * 2) : PW_OOB;
    } else if constexpr (W16) {
      const int yv = row / XR - 1, xv = row % XR - 1;
      const bool ok = row < C::XROWS && (unsigned)yv < (unsigned)g.H && (unsigned)xv < 16u;
      return ok ? (uint32_t)(((yv * 16 + xv) * g.Cs + ci0 + (lane & 3) * 8) * 2) : PW_OOB;
    } else if constexpr (W40) {
      // image row = (y - y0 + 1) * 50 + segment * 10 + x' + 1, voxel x = 8 segment + x'
      const int yv = y0 - 1 + row / XR, ps = row % XR, xv = 8 * (ps / 10) + ps % 10 - 1;
      const bool ok = row < C::XROWS && (unsigned)yv < (unsigned)g.H && (unsigned)xv < 40u;
      return ok ? (uint32_t)(((yv * 40 + xv) * g.Cs + ci0 + (lane & 3) * 8) * 2) : PW_OOB;
    } else {
      const int yv = y0 - 1 + row / XR, xv = row % XR - 1;
      const bool ok = row < C::XROWS && (unsigned)yv < (unsigned)g.H &&
                      (unsigned)xv < (unsigned)PW_XW;
      return ok ? (uint32_t)(((yv * PW_XW + xv) * g.Cs + ci0 + (lane & 3) * 8) * 2) : PW_OOB;
    }
  };
  const uint32_t xplane = LAT ? (uint32_t)(16 * 16 * g.Cs * 2) : (uint32_t)(g.H * VW * g.Cs * 2);
  // (rz: LAT's class group, 0 or 1).  With two groups per block the stream is both groups'
  // entries back to back: entry e = g (zr + 2) + e', e' = input plane z0 - 1 + e' of group g
  const int gstride = g.zr + 2;
  auto issue_x = [&](int e, int rz) {            // stream entry e = input plane z0 - 1 + e
    const uint32_t slot = smem_l + (uint32_t)(((unsigned)e % PW_XSLOTS) * C::XSLOT);
    if (LAT && e >= gstride) {
      e -= gstride;
      rz += 1;
    }
    const int zp = z0 - 1 + e;
    // LAT: sub-lattice plane z' -> grid plane rz + 2 z'; planes outside it read as zeros
    const bool zin = !LAT || (unsigned)zp < 8u;
    const uint32_t pz = LAT ? (uint32_t)(rz + 2 * zp) * xplane : (uint32_t)zp * xplane;
#pragma unroll
    for (int h = 0; h < C::NXMAX; ++h)
      if (h < nx)
        buf_lds16_asm(zin ? xoff(h) + pz : PW_OOB, rsx, slot + (uint32_t)((wave + 8 * h) * 1024));
  };
  // dY stage (output plane o, rows 2M, 2M + 1): image row r = q * 32 + x, one instruction
  // per wave of 8 rows x 128 B, chunk-swizzled for the transposing reads
  const int yr = wave * 8 + (lane >> 3);
  // LAT: image row q * 32 + segment * 8 + x' = voxel (ry + 2 (y' + q), rx + 2 x') of the plane
  const int yvox = LAT ? ((((yr >> 3) & 3) >> 1) + 2 * (yr >> 5)) * 16 + (((yr >> 3) & 3) & 1) +
                             2 * (yr & 7)
                       : yr;
  const uint32_t ylane = (uint32_t)(((W40 ? (lane >> 3) : yvox) * g.Nd + co0 +
                                     ((lane & 7) ^ pw_wsz128(yr)) * 8) * 2);
  auto issue_y = [&](int o, int m, int sl, int rz) {
    uint32_t base;
    if constexpr (W40) {
      // wave w: segment j = 4 (2m + w / 4) + w % 4 of the y tile (row j / 5, x 8 (j % 5))
      const int j = 4 * (2 * m + (wave >> 2)) + (wave & 3);
      base = (uint32_t)((((z0 + o) * g.H + y0 + j / 5) * 40 + 8 * (j % 5)) * g.Nd * 2);
    } else {
      base = LAT ? (uint32_t)(((rz + 2 * (z0 + o)) * 16 + 4 * m) * 16) * (uint32_t)g.Nd * 2
             : W16 ? (uint32_t)(((z0 + o) * g.H + 4 * m) * 16) * (uint32_t)g.Nd * 2
                   : (uint32_t)(((z0 + o) * g.H + y0 + 2 * m) * PW_XW) * (uint32_t)g.Nd * 2;
    }
    buf_lds16_asm(base + ylane, rsy, smem_l + (uint32_t)(C::Y_OFF + sl * PW_YST + wave * 1024));
  };

  const int cf = wave & 1, tg = wave >> 1;
  const int t0 = tg * 7, nt = tg == 3 ? 6 : 7;
  const int lk = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int rsel = 8 * lk + q4;
  uint32_t ya_lo[4], ya_hi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 16 + 4 * p4;
    ya_lo[i] = (uint32_t)(rsel * PW_YROW + (((col >> 3) ^ pw_wsz128(rsel)) << 4) + (col & 7) * 2);
    ya_hi[i] = (uint32_t)((rsel + 4) * PW_YROW + (((col >> 3) ^ pw_wsz128(rsel + 4)) << 4) +
                          (col & 7) * 2);
  }
  // (LAT: the 16-lane group lk reads segment lk, whose image positions start at 10 lk)
  // (W16: groups lk = 0, 1 read x 0-7, 8-15 of segment 0 -- image row y -- and lk = 2, 3 those
  // of segment 1, one image row group (18 positions) further)
  const uint32_t xb = (uint32_t)((LAT ? 10 * lk + q4 : W16 ? 18 * (lk >> 1) + 8 * (lk & 1) + q4
                                  : W40 ? q4 : rsel) *
                                     64 + cf * 32 + 8 * p4);
  // W40: lane group lk's segment of K step kt (of the 5-step period): image position of its
  // first voxel (segment 4 kt + lk of the period's 4 rows)
  uint32_t xk[W40 ? 5 : 1];
#pragma unroll
  for (int kt = 0; kt < (W40 ? 5 : 1); ++kt) {
    const int j = 4 * kt + lk;
    xk[kt] = W40 ? (uint32_t)(((j / 5) * XR + (j % 5) * 10) * 64) : 0u;
  }
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 7; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto tr8 = [](const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)p);
  };
  // prologue (per rz group): stream entries 0..2 (planes z0-1..z0+1), dY stages 0 and 1
  auto prologue = [&](int rz) {
    issue_x(0, rz);
    issue_x(1, rz);
    issue_x(2, rz);
    issue_y(0, 0, 0, rz);
    issue_y(0, 1, 1, rz);
  };
  prologue(rz);
  const int ng = LAT ? g.ng : 1;
  const int nstage = ng * g.zr * SPP;

  struct PFr { bf16x8 a[4], b[7]; };
  auto run = [&](auto tgc) {
    constexpr int TG = decltype(tgc)::value;
    constexpr int NT = TG == 3 ? 6 : 7;
    // per plane: this lane's fragment base in the slots of planes z-1, z, z+1.  Made opaque
    // (asm move) so the compiler cannot hoist one base per (tap, row) out of the plane loop
    // (30 live VGPRs, spilled); every read is then base + an immediate offset
    const char* xbase[3];
    // LAT: tap t at output row YL reads sub-lattice row YL + ky - 1: inside it?
    auto y_on = [](int t, int yl) constexpr {
      return !LAT || ((unsigned)(yl + (t / 3) % 3 - 1) < 8u);
    };
    // one K step = output row YL of the current plane (compile time); W40: K step YL of the
    // plane's 10
    auto kread = [&](const char* yimg, auto qc, auto ylc, PFr& f) {
      constexpr int Q = decltype(qc)::value, YL = decltype(ylc)::value;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f.a[i] = __builtin_shufflevector(tr8(yimg + Q * PW_XW * PW_YROW + ya_lo[i]),
                                         tr8(yimg + Q * PW_XW * PW_YROW + ya_hi[i]), 0, 1, 2, 3,
                                         4, 5, 6, 7);
      auto one = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (K < NT && y_on(TG * 7 + K, YL)) {
          constexpr int t = TG * 7 + K;
          constexpr int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;   // 0..2 (shift + 1)
          const char* img;
          if constexpr (W40) {
            constexpr int r0 = ((YL / 5) * 4 + ky) * XR + kx;
            img = xbase[kz] + xk[YL % 5] + r0 * 64;
          } else {
            constexpr int r0 = ((W16 ? 2 : 1) * YL + ky) * XR + kx;
            img = xbase[kz] + r0 * 64;
          }
          f.b[K] = __builtin_shufflevector(tr8(img), tr8(img + 4 * 64), 0, 1, 2, 3, 4, 5, 6, 7);
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
    auto kmma = [&](const PFr& f, auto ylc) {
      constexpr int YL = decltype(ylc)::value;
      auto one = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (K < NT && y_on(TG * 7 + K, YL)) {
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
#pragma unroll 1
    for (int o = 0; o < ng * g.zr; ++o) {
      // v: this plane's stream position (the second group's planes sit 2 entries on)
      const bool second = o >= g.zr;
      const int v = o + (second ? 2 : 0);
      if (LAT && o == g.zr) {
        // between the groups: every wave is done with the first group's last plane, whose
        // slots take the second group's entries 1 and 2 (entry 0 went out a plane earlier)
        raw_barrier();
        issue_x(v + 1, rz);
        issue_x(v + 2, rz);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        uint32_t b = (uint32_t)(((unsigned)(v + j) % PW_XSLOTS) * C::XSLOT) + xb;
        asm volatile("v_mov_b32 %0, %1" : "=v"(b) : "v"(b));
        xbase[j] = smem + b;
      }
      const bool xnext = v + 3 < ng * gstride;   // stream entry v + 3 exists
      auto stage = [&](auto mc) {
        constexpr int M = decltype(mc)::value;
        const int s = o * SPP + M;
        // dY(s) landed (and at M = 0 the planes of o, issued a plane earlier); younger: dY(s+1)
        // and, at stages 1 and 2, the X plane issued at stage 0 right after stage 2's dY
        // (the second group's first stage: everything, its entries 1 and 2 included)
        if (s + 1 >= nstage || (LAT && M == 0 && o == g.zr)) {
          wait_vm_lgkm0<0>();
        } else if ((M == 1 || M == 2) && xnext) {
          if (nx == 4) wait_vm_lgkm0<5>();
          else if (nx == 3) wait_vm_lgkm0<4>();
          else wait_vm_lgkm0<3>();
        } else {
          wait_vm_lgkm0<1>();
        }
        raw_barrier();
        if (s + 2 < nstage) {
          const int p2 = (int)((unsigned)(s + 2) / SPP), g2 = p2 >= g.zr ? 1 : 0;
          issue_y(p2 - g2 * g.zr, (int)((unsigned)(s + 2) % SPP), (int)((unsigned)(s + 2) % PW_YSLOTS), rz + g2);
        }
        if (M == 0 && xnext) issue_x(v + 3, rz);
        // (opaque, defined after the barrier: otherwise the dY fragment addresses of all four
        // stages are computed at the plane start and held -- 64 VGPRs, spilled)
        int yoff = C::Y_OFF + (int)((unsigned)s % PW_YSLOTS) * PW_YST;
        asm volatile("" : "+s"(yoff));
        const char* yimg = smem + yoff;
        PFr f0, f1;
        kread(yimg, std::integral_constant<int, 0>{}, std::integral_constant<int, 2 * M>{}, f0);
        kread(yimg, std::integral_constant<int, 1>{}, std::integral_constant<int, 2 * M + 1>{},
              f1);
        kmma(f0, std::integral_constant<int, 2 * M>{});
        kmma(f1, std::integral_constant<int, 2 * M + 1>{});
      };
      stage(std::integral_constant<int, 0>{});
      stage(std::integral_constant<int, 1>{});
      stage(std::integral_constant<int, 2>{});
      stage(std::integral_constant<int, 3>{});
      if constexpr (SPP == 5) stage(std::integral_constant<int, 4>{});
    }
  };
  switch (tg) {                                  // wave-uniform
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

// MMAD_PWGRAD=0 routes these convs back to the row-gather wgrad_kernel (A/B switch);
// MMAD_PWGRAD_LAT=0 keeps layer3's dilation-2 convs there
bool pw_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PWGRAD");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}
bool lat_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PWGRAD_LAT");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}

// MMAD_PWGRAD_W16=0 keeps the 16-wide stride-1 convs on the row-gather wgrad_kernel
// (measured r03w16: layer2.0.conv2 wgrad 40.0 + 13.4 us reduce -> 29.9 + 10.6)
bool w16_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PWGRAD_W16");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}
// the 16-wide form: dense 3^3, padding 1, stride 1 on volumes 16 voxels wide and high
bool w16_geo(const mmad_patch::Geo& q) {
  return q.KD == 3 && q.KH == 3 && q.KW == 3 && q.dd == 1 && q.dh == 1 && q.dw == 1 &&
         q.pd == 1 && q.ph == 1 && q.pw == 1 && q.Ds == q.Dd && q.Hs == q.Hd && q.Ws == q.Wd &&
         q.Wd == 16 && q.Hd == 16 && q.Dd >= 4;
}
// MMAD_PWGRAD_W40=0 keeps the 40-wide convs on the row-gather wgrad_kernel (A/B switch)
bool w40_on() {
  static const bool v = [] {
    const char* e = getenv("MMAD_PWGRAD_W40");
    return e == nullptr || atoi(e) != 0;
  }();
  return v;
}
// the 40-wide form: dense 3^3, padding 1, stride 1 on volumes 40 voxels wide, H % 8 == 0
bool w40_geo(const mmad_patch::Geo& q) {
  return q.KD == 3 && q.KH == 3 && q.KW == 3 && q.dd == 1 && q.dh == 1 && q.dw == 1 &&
         q.pd == 1 && q.ph == 1 && q.pw == 1 && q.Ds == q.Dd && q.Hs == q.Hd && q.Ws == q.Wd &&
         q.Wd == 40 && q.Hd % PW_TY == 0 && q.Dd >= 4;
}
// the residue-class form: 3^3 dilation 2, padding 2, stride 1 on a 16^3 grid (8^3 classes)
bool lat_geo(const mmad_patch::Geo& q) {
  return q.KD == 3 && q.KH == 3 && q.KW == 3 && q.dd == 2 && q.dh == 2 && q.dw == 2 &&
         q.pd == 2 && q.ph == 2 && q.pw == 2 && q.Ds == 16 && q.Hs == 16 && q.Ws == 16 &&
         q.Dd == 16 && q.Hd == 16 && q.Wd == 16;
}

// LAT: both class groups in one block (half the partial slabs) when that still gives >= 256
// blocks over whole sub-lattices (MMAD_PWGRAD_LAT_NG=1 keeps one group per block; r03ng:
// layer3.0.conv2 wgrad 90.5 + 20.0 us reduce -> 84.5 + 11.5)
int lat_ng(const mmad_patch::Geo& q) {
  static const int force1 = [] {
    const char* e = getenv("MMAD_PWGRAD_LAT_NG");
    return e != nullptr && atoi(e) == 1;
  }();
  if (!lat_geo(q) || force1) return 1;
  return (int64_t)q.nb * (q.Cs / PW_KC) * (q.Nd / 64) >= 256 ? 2 : 1;
}

// output planes per split: the largest divisor of D (>= 4) that still gives >= 256 blocks
// (LAT: of the 8-plane sub-lattice, down to 2)
int pw_zr(const mmad_patch::Geo& q) {
  if (lat_geo(q)) {
    const int64_t base = (int64_t)q.nb * (2 / lat_ng(q)) * (q.Cs / PW_KC) * (q.Nd / 64);
    int zr = 8;
    while (zr > 2 && base * (8 / zr) < 256) zr /= 2;
    return zr;
  }
  const int64_t base =
      (int64_t)q.nb * (w16_geo(q) ? 1 : q.Hd / PW_TY) * (q.Cs / PW_KC) * (q.Nd / 64);
  int zr = q.Dd;
  while (zr > 4 && zr % 2 == 0 && base * (q.Dd / zr) < 256) zr /= 2;
  return zr;
}

}  // namespace

namespace mmad_pwgrad {

bool ok(const mmad_patch::Geo& q) {
  if (!pw_on()) return false;
  if (q.Cs % PW_KC || q.Nd % 64 || q.Kpad != 27 * q.Cs) return false;
  if (lat_geo(q)) return lat_on() && (int64_t)4096 * std::max(q.Cs, q.Nd) * 2 < (int64_t(1) << 30);
  if (w16_geo(q)) {
    if (!w16_on() || (int64_t)q.Dd * 256 * std::max(q.Cs, q.Nd) * 2 >= (int64_t(1) << 30))
      return false;
    const int zr = pw_zr(q);
    return q.Dd % zr == 0 && zr >= 2;
  }
  if (w40_geo(q)) {
    if (!w40_on() || (int64_t)q.Dd * q.Hd * 40 * std::max(q.Cs, q.Nd) * 2 >= (int64_t(1) << 30))
      return false;
    const int zr = pw_zr(q);
    return q.Dd % zr == 0 && zr >= 2;
  }
  if (q.KD != 3 || q.KH != 3 || q.KW != 3 || q.dd != 1 || q.dh != 1 || q.dw != 1) return false;
  if (q.pd != 1 || q.ph != 1 || q.pw != 1) return false;
  if (q.Ds != q.Dd || q.Hs != q.Hd || q.Ws != q.Wd || q.Wd != PW_XW) return false;
  if (q.Hd % PW_TY || q.Dd < 4) return false;
  if ((int64_t)q.Dd * q.Hd * PW_XW * std::max(q.Cs, q.Nd) * 2 >= (int64_t(1) << 30)) return false;
  const int zr = pw_zr(q);
  return q.Dd % zr == 0 && zr >= 2;
}

int64_t splits(const mmad_patch::Geo& q) {
  if (lat_geo(q)) return (int64_t)q.nb * (2 / lat_ng(q)) * (8 / pw_zr(q));
  if (w16_geo(q)) return (int64_t)q.nb * (q.Dd / pw_zr(q));
  return (int64_t)q.nb * (q.Hd / PW_TY) * (q.Dd / pw_zr(q));
}

int64_t workspace(const mmad_patch::Geo& q) {
  return mmad_pwgrad::splits(q) * q.Nd * 27 * q.Cs * 4;
}

int wgrad(const mmad_patch::Geo& q, const void* x, const void* dy, float* ws, int* nsplit,
          void* stream) {
  if (!mmad_pwgrad::ok(q)) return MMAD_EUNSUPPORTED;
  static const bool attr =
      hipFuncSetAttribute((const void*)pwgrad_kernel<0>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, PWC<0>::LDS) == hipSuccess &&
      hipFuncSetAttribute((const void*)pwgrad_kernel<1>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, PWC<1>::LDS) == hipSuccess &&
      hipFuncSetAttribute((const void*)pwgrad_kernel<2>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, PWC<2>::LDS) == hipSuccess &&
      hipFuncSetAttribute((const void*)pwgrad_kernel<3>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, PWC<3>::LDS) == hipSuccess;
  if (!attr) return MMAD_EUNSUPPORTED;
  const int mode = lat_geo(q) ? 1 : w16_geo(q) ? 2 : w40_geo(q) ? 3 : 0;
  PWG g{};
  g.nb = q.nb; g.Cs = q.Cs; g.Nd = q.Nd; g.D = q.Dd; g.H = q.Hd; g.K = 27 * q.Cs;
  g.zr = pw_zr(q);
  g.ng = lat_ng(q);
  const int64_t sp = mmad_pwgrad::splits(q);
  const int64_t nblk = sp * (q.Cs / PW_KC) * (q.Nd / 64);
  if (mode == 1)
    hipLaunchKernelGGL(pwgrad_kernel<1>, dim3((unsigned)nblk), dim3(PW_NTHR), PWC<1>::LDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else if (mode == 2)
    hipLaunchKernelGGL(pwgrad_kernel<2>, dim3((unsigned)nblk), dim3(PW_NTHR), PWC<2>::LDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else if (mode == 3)
    hipLaunchKernelGGL(pwgrad_kernel<3>, dim3((unsigned)nblk), dim3(PW_NTHR), PWC<3>::LDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  else
    hipLaunchKernelGGL(pwgrad_kernel<0>, dim3((unsigned)nblk), dim3(PW_NTHR), PWC<0>::LDS,
                       as_stream(stream), g, (const u16*)x, (const u16*)dy, ws);
  *nsplit = (int)sp;
  return launch_status();
}

}  // namespace mmad_pwgrad
