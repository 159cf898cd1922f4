// Patch-resident stride-1 3D convolution for narrow layers (bf16), internal to
// libmmad_hip.so: mmad_conv3d_fwd / mmad_conv3d_dgrad route matching geometries here
// (see patchconv.hip for the design).
#pragma once
#include <stdint.h>

#include "../../include/mmad.h"

namespace mmad_patch {
// stride-1 conv over NDHWC bf16 volumes; weights packed [Nd][Kpad] with k = tap*Cs + ci
struct Geo {
  int nb, Cs, Nd, Kpad;           // input channels, output channels, packed weight row
  int Ds, Hs, Ws, Dd, Hd, Wd;     // source / destination extents
  int KD, KH, KW, pd, ph, pw, dd, dh, dw;
  const void* res = nullptr;      // eval-mode epilogue: residual (output-shaped) and ReLU
  int relu = 0;
  // dgrad epilogue (bnsum.h): the BN-backward partial sums of the BN+ReLU whose output was
  // this conv's input -- its input y (output-shaped), scale / shift (the ReLU mask), mean /
  // invstd, and the partial rows [tiles][2][Nd] to write (bny == nullptr: off)
  const void* bny = nullptr;
  const float* bnsc = nullptr;
  const float* bnsh = nullptr;
  const float* bnmu = nullptr;
  const float* bnis = nullptr;
  float* bnparts = nullptr;
};
// true when the geometry is handled (and the kernel is switched on, MMAD_PATCH)
bool ok(const Geo& g);
// M tiles of one launch = rows of the BN partial-sum buffer it writes ([rows][2][Nd])
int64_t tiles(const Geo& g);
int fwd(const Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
}  // namespace mmad_patch

// Persistent z-walking form of the patch conv for 64-channel inputs on grids of 4 x 8 x 8
// boxes (patchz.hip, layer1): mmad_patch::fwd / tiles route to it when ok().
namespace mmad_patchz {
int set_mode(int v);              // MMAD_PATCHZ at run time; returns the previous mode
bool ok(const mmad_patch::Geo& g);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
}  // namespace mmad_patchz

// Residue-class conv for dilated 3^3 convs on a 4d^3 grid (latticeconv.hip): same geometry
// record, packed weights and partial-sum layout as the patch kernel.
namespace mmad_lattice {
int set_mode(int v);              // MMAD_LATTICE at run time; returns the previous mode
bool ok(const mmad_patch::Geo& g);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
// weight gradient: fp32 partial slabs [splits][Nd][27 * Cs] into ws (wgrad_workspace bytes),
// *splits set; the caller sums / transposes them into the torch layout
bool wgrad_ok(const mmad_patch::Geo& g);
int64_t wgrad_workspace(const mmad_patch::Geo& g);
int wgrad(const mmad_patch::Geo& g, const void* x, const void* dy, float* ws, int* splits,
          void* stream);
}  // namespace mmad_lattice

// Stride-2 3^3 conv forward on parity sub-patches (s2conv.hip, layer2.0.conv1: 64 input
// channels, even input extents, whole 2 x 8 x 8 output boxes); strides passed separately
// (Geo has none).  One BN partial-sum row per output box.
namespace mmad_s2 {
bool ok(const mmad_patch::Geo& g, int sd, int sh, int sw);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, int sd, int sh, int sw, const void* src, const void* wp,
        const float* bias, void* dst, float* stats, void* stream);
// its input gradient (64 ci, 128 co, bf16; dgrad-packed weights [ci][tap][co]): all 8
// stride-parity classes of dX from one dY patch per block
bool dgrad_ok(const mmad_conv_desc* d);
int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream);
}  // namespace mmad_s2

// Plane-pair form of the residue-class conv for d = 4 (latticezp.hip): two z-planes of 16
// subs per tile, one wave per SIMD; mmad_lattice::fwd / tiles route to it when ok().
namespace mmad_lattice_zp {
bool ok(const mmad_patch::Geo& g);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
}  // namespace mmad_lattice_zp

// Residue-class conv on 5d^3 grids (lattice5.hip: config 5's 20^3 layer4, 5^3 sub-lattices):
// mmad_lattice::ok / tiles / fwd route to it first.
namespace mmad_lattice5 {
int set_mode(int v);              // MMAD_LATTICE5 at run time; returns the previous mode
bool ok(const mmad_patch::Geo& g);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
// weight gradient (mmad_lattice::wgrad_ok / wgrad_workspace / wgrad route to it first):
// fp32 partial slabs [splits][Nd][27 * Cs]
bool wgrad_ok(const mmad_patch::Geo& g);
int64_t wgrad_workspace(const mmad_patch::Geo& g);
int wgrad(const mmad_patch::Geo& g, const void* x, const void* dy, float* ws, int* splits,
          void* stream);
}  // namespace mmad_lattice5

// Residue-class conv for dilation-2 3^3 convs on a 16^3 grid (lattice8.hip, layer3).
namespace mmad_lattice8 {
int set_mode(int v);              // MMAD_LATTICE8 at run time; returns the previous mode
bool ok(const mmad_patch::Geo& g);
int64_t tiles(const mmad_patch::Geo& g);
int fwd(const mmad_patch::Geo& g, const void* src, const void* wp, const float* bias, void* dst,
        float* stats, void* stream);
}  // namespace mmad_lattice8

// Patch-resident weight gradient for dense stride-1 3^3 convs on 32-wide volumes
// (pwgrad.hip, layer1): fp32 partial slabs [splits][Nd][27 * Cs] as mmad_lattice::wgrad.
namespace mmad_pwgrad {
bool ok(const mmad_patch::Geo& g);
int64_t workspace(const mmad_patch::Geo& g);
int wgrad(const mmad_patch::Geo& g, const void* x, const void* dy, float* ws, int* splits,
          void* stream);
}  // namespace mmad_pwgrad

namespace mmad_pool {
// MMAD_POOL_RUN run-time override (mmad_set_kernel_variant("pool_run", v)); returns the old mode
int set_run_mode(int v);
}  // namespace mmad_pool
