// Contention probe (tools/spin_contention.py): k blocks that each hold 64 KiB of LDS and a
// CU's wave slots busy for a given number of microseconds, standing in for the RCCL ring
// kernels that share the CUs with the backward when all-reduces overlap it.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void spin_kernel(long long cycles, int* sink) {
  extern __shared__ int lds[];
  const long long t0 = wall_clock64();
  int v = threadIdx.x;
  while (wall_clock64() - t0 < cycles) {
    lds[threadIdx.x] = v;
    v = lds[(threadIdx.x + 1) & 255] + 1;
  }
  if (v == -12345) sink[0] = v;
}

extern "C" int spin_launch(int blocks, double usec, void* stream, int* sink) {
  // wall_clock64 runs at 100 MHz on gfx9 parts
  const long long cycles = (long long)(usec * 100.0);
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(256), 64 * 1024,
                     reinterpret_cast<hipStream_t>(stream), cycles, sink);
  return (int)hipGetLastError();
}
