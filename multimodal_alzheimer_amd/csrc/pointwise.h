// 1x1x1 stride-1 conv input gradient as a hand-written MFMA GEMM (pointwise.hip), internal to
// libmmad_hip.so.
#pragma once
#include <stdint.h>

#include "../../include/mmad.h"

namespace mmad_pw {
// true for bf16 1x1x1 stride-1 unpadded convs with ci in {128, 256}, co % 64 == 0 and a
// voxel count that is a multiple of 128 (layer3 / layer4 shortcuts at batch 8)
bool ok(const mmad_conv_desc* d, int dtype);
// dX = dY . W over the dgrad-packed weights [ci][co]
int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream);
// the same GEMM as the forward of a bf16 1x1x1 stride-1 conv with co % 256 == 0 and ci % 64
// == 0 (layer3 / layer4 shortcuts): Y = X . W^T over the forward-packed weights [co][ci], BN
// partial sums one row per 128 voxels (fwd_tiles rows)
bool fwd_ok(const mmad_conv_desc* d, int dtype);
int64_t fwd_tiles(const mmad_conv_desc* d);
int fwd(const mmad_conv_desc* d, const void* x, const void* wp, const float* bias, void* y,
        float* stats, void* stream);
}  // namespace mmad_pw
