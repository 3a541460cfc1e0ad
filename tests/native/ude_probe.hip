// Arithmetic probes for the kernel-order oracle (tests/test_kernel_order.py) -- TEST INFRASTRUCTURE.
// Built by __graft_entry__.build() into tests/native/_build/libude_probe.so; never linked into the
// product library.  Two questions the restatement in oracle/ude_korder.c depends on:
//  * what one v_mfma_f32_16x16x4_f32 computes per output element (which fmaf chain over its 4 K lanes);
//  * what the device expm1f (ROCm's __ocml_expm1_f32, the ELU of csrc/ude_kernels.h elu1) returns.
// Compiled with the product library's flags (-O3 -ffp-contract=off).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

// case c: A [16][4], B [4][16], C / D [16][16] row-major; lane l holds A[l & 15][l >> 4],
// B[l >> 4][l & 15] and D[4 (l >> 4) + i][l & 15] (the operand layout the solve kernels use)
__global__ void __launch_bounds__(64) probe_mfma_kernel(const float* A, const float* B, const float* C, float* D,
                                                        int n_case) {
  const int cs = blockIdx.x;
  if (cs >= n_case) return;
  const int l = threadIdx.x, row = l & 15, g = l >> 4;
  const float a = A[cs * 64 + row * 4 + g];
  const float b = B[cs * 64 + g * 16 + row];
  f4 c;
  for (int i = 0; i < 4; ++i) c[i] = C[cs * 256 + (4 * g + i) * 16 + row];
  const f4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[cs * 256 + (4 * g + i) * 16 + row] = d[i];
}

// y[i] = expm1f(x) for the float with bit pattern start + i
__global__ void probe_expm1_kernel(uint32_t start, long n, float* y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = __uint_as_float(start + (uint32_t)i);
  y[i] = expm1f(x);
}

extern "C" int ude_probe_mfma(const float* A, const float* B, const float* C, float* D, int n_case,
                              hipStream_t s) {
  if (n_case <= 0) return 0;
  hipLaunchKernelGGL(probe_mfma_kernel, dim3(n_case), dim3(64), 0, s, A, B, C, D, n_case);
  return (int)hipGetLastError();
}

extern "C" int ude_probe_expm1_bits(uint32_t start, long n, float* y, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(probe_expm1_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, start, n, y);
  return (int)hipGetLastError();
}
