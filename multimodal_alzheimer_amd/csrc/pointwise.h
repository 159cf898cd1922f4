// 1x1x1 stride-1 conv input gradient as a hand-written MFMA GEMM (pointwise.hip), internal to
// libmmad_hip.so.
#pragma once
#include <stdint.h>

#include "../../include/mmad.h"

namespace mmad_pw {
// true for bf16 1x1x1 unpadded convs of stride 1 or 2 with ci in {64, 128, 256}, co % 64 == 0
// and an output voxel count that is a multiple of 128 (the layer2 / 3 / 4 shortcuts at batch 8)
bool ok(const mmad_conv_desc* d, int dtype);
// dX = dY . W over the dgrad-packed weights [ci][co]; stride 2: the GEMM rows land on the
// all-even voxels and the block writes the zeros of the rest of each 2x2x2 cell
int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream);
// the same GEMM as the forward of a bf16 1x1x1 conv of stride 1 or 2 with co % 256 == 0 or
// co == 128, ci % 64 == 0 (the layer2 / 3 / 4 shortcuts): Y = X . W^T over the forward-packed
// weights [co][ci] (stride 2: the A rows gathered from the all-even input voxels), BN partial
// sums one row per 128 output voxels (fwd_tiles rows)
bool fwd_ok(const mmad_conv_desc* d, int dtype);
int64_t fwd_tiles(const mmad_conv_desc* d);
int fwd(const mmad_conv_desc* d, const void* x, const void* wp, const float* bias, void* y,
        float* stats, void* stream);
// the weight gradient of a bf16 1x1x1 conv of stride 1 or 2 (the shortcuts), or of a 3^3
// stride-2 pad-1 conv (layer2.0.conv1), with co % 128 == 0, ci % 64 == 0: split-K MFMA GEMM
// over the voxels into fp32 slabs [split][co][tap * ci + ci'] (wgrad_splits slabs), summed by
// the caller's slab reduction (wide for 1^3, transposing for 3^3)
bool wgrad_ok(const mmad_conv_desc* d, int dtype);
int64_t wgrad_splits(const mmad_conv_desc* d);
int wgrad(const mmad_conv_desc* d, const void* x, const void* dy, float* ws, void* stream);
// the de-duplicated X rows of the 16-wide stride-2 3^3 weight gradient: 1 on (default), 0 off
// (mmad_set_kernel_variant("pw_wg3_dedup", v)); returns the previous setting
int set_wg3_dedup(int v);
}  // namespace mmad_pw
