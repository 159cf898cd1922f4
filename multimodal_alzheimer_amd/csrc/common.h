// Shared device helpers for libmmad_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmad.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))

// Wait until at most N vector-memory ops (incl. LDS-DMA) of this wave are outstanding and
// all LDS ops have completed; N must be a compile-time constant (it is an immediate).
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate (6 bits)");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(N) : "memory");
}

// Workgroup barrier that does NOT drain in-flight LDS-DMA (unlike __syncthreads, whose
// fence waits vmcnt(0)); pair it with wait_vm_lgkm0<N>() for the stage being consumed.
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16-byte LDS-DMA (global_load_lds_dwordx4) issued from inline asm: hipcc does not count it,
// so it never inserts its own vmcnt(0) drain before a later LDS read (which it does for
// the builtin ahead of ds_read_*_tr reads); the caller waits with wait_vm_lgkm0<N>().
// lds_addr = wave-uniform LDS byte address of this wave's 1 KiB destination.
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_addr)
      : "memory");
}
// Same through a buffer resource: lane byte offset `voff` (32-bit); an offset past the
// resource's size reads 16 zero bytes (hardware range check), which is how padding and
// out-of-range rows are fed without a pointer select.
__device__ __forceinline__ void buf_lds16_asm(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc,
                                              uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_addr)
      : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const LDS_AS void*)p);
}

// bf16 <-> f32 (round to nearest even; NaN stays NaN) --------------------------------
__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
__device__ __forceinline__ u16 f2bf(float f) { return (u16)(pack_bf16x2(f, 0.f) & 0xffffu); }

// element access by compute dtype: T = float or u16 (bf16 bits) ----------------------
template <typename T> struct Elt;
template <> struct Elt<float> {
  static __device__ __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }
  static constexpr int VEC = 4;   // elements per 16-byte chunk
};
template <> struct Elt<u16> {
  static __device__ __forceinline__ float ld(const u16* p, int64_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(u16* p, int64_t i, float v) { p[i] = f2bf(v); }
  static constexpr int VEC = 8;
};

// 16-byte chunk <-> 8 (or 4) floats
template <typename T> struct Chunk;
template <> struct Chunk<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void load(const float* p, float* v) {
    f32x4 c = *reinterpret_cast<const f32x4*>(p);
    v[0] = c[0]; v[1] = c[1]; v[2] = c[2]; v[3] = c[3];
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    f32x4 c; c[0] = v[0]; c[1] = v[1]; c[2] = v[2]; c[3] = v[3];
    *reinterpret_cast<f32x4*>(p) = c;
  }
};
template <> struct Chunk<u16> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const u16* p, float* v) {
    u16x8 c = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bf2f(c[i]);
  }
  static __device__ __forceinline__ void store(u16* p, const float* v) {
    u32x4 c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
    *reinterpret_cast<u32x4*>(p) = c;
  }
};

// epilogue of a fused eval-mode conv: 8 bf16 outputs (+ 8 bf16 residuals) (-> ReLU)
__device__ __forceinline__ u32x4 epi_res_relu(u32x4 v, const u16* res, int relu) {
  float f[8];
  Chunk<u16>::load(reinterpret_cast<const u16*>(&v), f);
  if (res != nullptr) {
    float r[8];
    Chunk<u16>::load(res, r);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += r[e];
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
  }
  u32x4 o;
  Chunk<u16>::store(reinterpret_cast<u16*>(&o), f);
  return o;
}

// BN affine (+ReLU) of one value, shared by every kernel that applies a BN so the fused and
// unfused paths round identically: o = fma(y, scale, shift), relu -> max(o, 0).
__device__ __forceinline__ float bn_affine(float y, float scale, float shift) {
  return __builtin_fmaf(y, scale, shift);
}
// value as stored in dtype T (bf16 rounding for u16)
template <typename T>
__device__ __forceinline__ float as_stored(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v));
  else return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static inline int hip_status(hipError_t e) { return e == hipSuccess ? MMAD_OK : MMAD_EHIP + (int)e; }
static inline int launch_status() { return hip_status(hipGetLastError()); }
static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Zero-fill as a kernel (16-byte stores, any 4-byte-aligned size): used instead of
// hipMemsetAsync on paths that run inside captured HIP graphs -- a captured memset node was
// not re-executed on replays after the first on this ROCm stack (tools/diag_replay.py),
// while kernel nodes are.
__global__ void zero_fill_kernel(uint32_t* __restrict__ p, int64_t words);
int zero_fill(void* p, int64_t bytes, hipStream_t st);
static inline bool is_pow2(int64_t v) { return v > 0 && (v & (v - 1)) == 0; }
static inline int ilog2(int64_t v) { int r = 0; while ((int64_t(1) << r) < v) ++r; return r; }
