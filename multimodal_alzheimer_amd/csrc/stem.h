// Dedicated MedicalNet stem convolution (conv1: Cin 1 -> 64, 7x7x7, stride 2, pad 3) on the
// W-unfolded input (layout [n][di][hi][wo][8], see mmad_conv_unfold_input).  Internal to
// libmmad_hip.so: mmad_conv3d_fwd routes a matching descriptor here.
#pragma once
#include <stdint.h>

#include "../../include/mmad.h"

namespace mmad_stem {
// true when the descriptor/dtype is handled by the stem kernel
bool fwd_ok(const mmad_conv_desc* d, int dtype);
// rows of the BN partial-sum buffer the stem kernel writes ([rows][2][64])
int64_t fwd_stats_rows(const mmad_conv_desc* d);
// in_dtype -1: x is the unfolded U; MMAD_F64 / MMAD_F32: x is the raw (n, 1, D, H, W) volume
// (raw_ok must hold), read and unfolded inside the kernel
int fwd(const mmad_conv_desc* d, const void* x_unf, const void* w_packed, const float* bias,
        void* y, float* stats, void* stream, int in_dtype = -1);
bool raw_ok(const mmad_conv_desc* d, int in_dtype);
// weight gradient: one fp32 partial slab [64][392] per block into ws (see wgrad_blocks)
int64_t wgrad_blocks(const mmad_conv_desc* d);
int wgrad(const mmad_conv_desc* d, const void* x_unf, const void* dy, float* ws, void* stream,
          int in_dtype = -1);
}  // namespace mmad_stem
