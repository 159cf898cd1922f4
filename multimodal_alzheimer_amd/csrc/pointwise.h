// 1x1x1 stride-1 conv gradients through hipBLASLt (pointwise.hip), internal to libmmad_hip.so.
#pragma once
#include <stdint.h>

#include "../../include/mmad.h"

namespace mmad_pw {
constexpr int64_t WGRAD_WS = int64_t(32) << 20;   // hipBLASLt split-K workspace bound
// true for bf16 1x1x1 stride-1 unpadded convs with channel counts that are multiples of 64
bool ok(const mmad_conv_desc* d, int dtype);
int64_t wgrad_workspace(const mmad_conv_desc* d);
// dX = dY . W over the dgrad-packed weights [ci][co]
int dgrad(const mmad_conv_desc* d, const void* dy, const void* wpt, void* dx, void* stream);
// dW (fp32, [co][ci]) = dY^T . X; ws: wgrad_workspace bytes
int wgrad(const mmad_conv_desc* d, const void* x, const void* dy, float* dw, void* ws,
          void* stream);
}  // namespace mmad_pw
