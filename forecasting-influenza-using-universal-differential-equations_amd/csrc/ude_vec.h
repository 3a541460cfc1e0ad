// Dense vector kernels of the adaptive step controllers (no model): the stage / solution / error
// combinations of torchdiffeq's Dormand-Prince step (``y + sum_j beta_j k_j``, a `stack(k) @ c`
// GEMV in torchdiffeq, a chain of multiply-adds in ude_amd/adaptive.py) as ONE pass over the state,
// and the error-ratio numerator sum((err / (atol + rtol max(|y0|, |y1|)))^2).  odeint_adjoint's
// augmented state (y, a_y: 2 N R L floats, plus the parameter adjoint) makes these passes the
// bulk of an augmented step's memory traffic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ude {

constexpr int LC_MAXK = 8;
struct LcArgs {
  const float* base;            // nullable: 0
  const float* k[LC_MAXK];
  const float* coef;            // device, nk floats (null: the by-value copy cv)
  float* out;
  int64_t n;
  int nk;
  float cv[LC_MAXK];            // coefficients passed by value (ude_lincomb_hc)
};

// out = base + sum_j coef[j] k_j; every term accumulated in the fixed order j = 0.. (k_0 first),
// as the multiply-add chain it replaces: acc = k_0 c_0; acc = fma-free acc + k_j c_j; out = base + acc.
__global__ __launch_bounds__(256) void ude_lincomb_kernel(LcArgs a) {
  float c[LC_MAXK];
#pragma unroll
  for (int j = 0; j < LC_MAXK; ++j) c[j] = j < a.nk ? (a.coef ? a.coef[j] : a.cv[j]) : 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
    float acc = a.k[0][i] * c[0];
#pragma unroll
    for (int j = 1; j < LC_MAXK; ++j)
      if (j < a.nk) acc = acc + a.k[j][i] * c[j];
    a.out[i] = a.base ? a.base[i] + acc : acc;
  }
}

// The same combination 16 bytes per lane (every pointer 16-byte aligned): four independent elements
// per lane, each with the scalar kernel's per-element operation order; the n % 4 tail by block 0.
__global__ __launch_bounds__(256) void ude_lincomb4_kernel(LcArgs a) {
  typedef float v4 __attribute__((ext_vector_type(4)));
  float c[LC_MAXK];
#pragma unroll
  for (int j = 0; j < LC_MAXK; ++j) c[j] = j < a.nk ? (a.coef ? a.coef[j] : a.cv[j]) : 0.f;
  const int64_t n4 = a.n >> 2, stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
    v4 acc = reinterpret_cast<const v4*>(a.k[0])[i] * c[0];
#pragma unroll
    for (int j = 1; j < LC_MAXK; ++j)
      if (j < a.nk) acc = acc + reinterpret_cast<const v4*>(a.k[j])[i] * c[j];
    reinterpret_cast<v4*>(a.out)[i] = a.base ? reinterpret_cast<const v4*>(a.base)[i] + acc : acc;
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
    const int64_t i = n4 * 4 + threadIdx.x;
    float acc = a.k[0][i] * c[0];
#pragma unroll
    for (int j = 1; j < LC_MAXK; ++j)
      if (j < a.nk) acc = acc + a.k[j][i] * c[j];
    a.out[i] = a.base ? a.base[i] + acc : acc;
  }
}

// Per-block partial sums (fp64) of ((err / tol)^2), tol = atol + rtol * max(|y0|, |y1|) in fp32 as
// torchdiffeq forms it; out[1 + block] = partial, then ude_sumsq_finish sums them in order into out[0].
constexpr int SSQ_BLOCKS = 1024;
__global__ __launch_bounds__(256) void ude_scaled_sumsq_kernel(const float* __restrict__ err,
                                                               const float* __restrict__ y0,
                                                               const float* __restrict__ y1, float atol,
                                                               float rtol, int64_t n, double* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float tol = atol + rtol * fmaxf(fabsf(y0[i]), fabsf(y1[i]));
    const float r = err[i] / tol;
    s += (double)r * (double)r;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[1 + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(64) void ude_sumsq_finish_kernel(double* __restrict__ out, int nb) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 64) s += out[1 + i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (threadIdx.x == 0) out[0] = s;
}

// coef: device array (coef_host null) or host array copied into the launch (coef null)
inline int lincomb(int64_t n, const float* base, const float* const* k, int nk, const float* coef, float* out,
                   hipStream_t s, const float* coef_host = nullptr) {
  if (n < 0 || nk < 1 || nk > LC_MAXK || !k || (!coef && !coef_host) || !out) return -2;
  if (n == 0) return 0;
  LcArgs a;
  a.base = base;
  for (int j = 0; j < LC_MAXK; ++j) a.cv[j] = (coef_host && j < nk) ? coef_host[j] : 0.f;
  if (coef_host) coef = nullptr;
  for (int j = 0; j < LC_MAXK; ++j) a.k[j] = j < nk ? k[j] : nullptr;
  for (int j = 0; j < nk; ++j)
    if (!k[j]) return -2;
  a.coef = coef; a.out = out; a.n = n; a.nk = nk;
  uintptr_t any = (uintptr_t)out | (uintptr_t)base;
  for (int j = 0; j < nk; ++j) any |= (uintptr_t)k[j];
  if ((any & 15) == 0) {
    int64_t blocks = (n / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(ude_lincomb4_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
  }
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ude_lincomb_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// One Dormand-Prince attempt's error ratio and next step size (torchdiffeq's mixed error norm and
// _optimal_step_size, in PyTorch's own operation order so the controller's decisions match the operator
// chain it replaces bit for bit: the fp32 tolerance of element 0, sqrt of each piece's fp64 sum times the
// reciprocal of its count, NaN-propagating max, 0.9 * reciprocal(ratio^0.2) clamped to [dfac, 10]).
struct RatioArgs {
  const float* err;
  const float* y0;
  const float* y1;
  const double* ssq;            // n_pieces sums at ssq + i * SSQ_STRIDE (ude_scaled_sumsq outputs)
  const double* extra;          // nullable: n_extra more norm parts (fp64, device)
  const unsigned char* flag;    // nullable: copied to status[2]
  double* status;               // [ratio, next dt, flag]
  double inv_n[4];
  double dt;
  float atol, rtol;
  int n_pieces, n_extra;
};
constexpr int SSQ_STRIDE = SSQ_BLOCKS + 1;
__device__ __forceinline__ double nanmax(double a, double b) { return (a != a || b != b) ? NAN : fmax(a, b); }
__global__ void ude_dopri_ratio_kernel(RatioArgs a) {
  if (threadIdx.x != 0) return;
  const float u = fabsf(a.y0[0]), v = fabsf(a.y1[0]);
  const float m = (u != u || v != v) ? NAN : fmaxf(u, v);
  const float tol0 = __fadd_rn(a.atol, __fmul_rn(a.rtol, m));
  double r = (double)fabsf(__fdiv_rn(a.err[0], tol0));
  for (int i = 0; i < a.n_pieces; ++i) r = nanmax(r, sqrt(__dmul_rn(a.ssq[(size_t)i * SSQ_STRIDE], a.inv_n[i])));
  for (int i = 0; i < a.n_extra; ++i) r = nanmax(r, a.extra[i]);
  double dt;
  if (r == 0.0) {
    dt = __dmul_rn(a.dt, 10.0);
  } else {
    const double dfac = r < 1.0 ? 1.0 : 0.2;
    double f = __dmul_rn(__ddiv_rn(1.0, pow(r, 0.2)), 0.9);
    f = (f != f) ? f : fmin(fmax(f, dfac), 10.0);
    dt = __dmul_rn(a.dt, f);
  }
  a.status[0] = r;
  a.status[1] = dt;
  a.status[2] = a.flag ? (double)a.flag[0] : 0.0;
}

inline int dopri_ratio(const float* err, const float* y0, const float* y1, double atol, double rtol, const double* ssq,
                       const int64_t* n, int n_pieces, const double* extra, int n_extra, double dt,
                       const unsigned char* flag, double* status, hipStream_t s) {
  if (!err || !y0 || !y1 || !status || n_pieces < 0 || n_pieces > 4 || (n_pieces > 0 && (!ssq || !n)) ||
      n_extra < 0 || (n_extra > 0 && !extra))
    return -2;
  RatioArgs a;
  a.err = err; a.y0 = y0; a.y1 = y1; a.ssq = ssq; a.extra = extra; a.flag = flag; a.status = status;
  for (int i = 0; i < 4; ++i) a.inv_n[i] = i < n_pieces ? 1.0 / (double)n[i] : 0.0;
  a.dt = dt; a.atol = (float)atol; a.rtol = (float)rtol; a.n_pieces = n_pieces; a.n_extra = n_extra;
  hipLaunchKernelGGL(ude_dopri_ratio_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

inline int scaled_sumsq(int64_t n, const float* err, const float* y0, const float* y1, double atol, double rtol,
                        double* out, hipStream_t s) {
  if (n < 0 || !err || !y0 || !y1 || !out) return -2;
  int64_t blocks = (n + 255) / 256;
  if (blocks > SSQ_BLOCKS) blocks = SSQ_BLOCKS;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ude_scaled_sumsq_kernel, dim3((unsigned)blocks), dim3(256), 0, s, err, y0, y1, (float)atol,
                     (float)rtol, n, out);
  hipLaunchKernelGGL(ude_sumsq_finish_kernel, dim3(1), dim3(64), 0, s, out, (int)blocks);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace ude
