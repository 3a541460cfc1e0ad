// A/B probe: the R = 1 forward solve with ONE WAVEFRONT PER TRAJECTORY on the VALU
// (no MFMA, no workgroup barrier), against the product's 16-trajectory MFMA tiles.  Development tool,
// not linked into the product library.  Fp [H0, H1] (lib/models.py:109-146), R = 1, L = 8, 3/8-rule RK4,
// fp64 state (as the product kernel), outputs at every grid point, fp64 rate sums.
//   lane o of layer i computes output o (weights of row o in VGPRs); the layer input goes through a
//   per-wave LDS row read back as wave-uniform ds_read_b128 broadcasts; the 2-row output layer is a
//   per-lane product + a cross-lane sum (DPP row sums + 4 readlanes).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float elu1(float x) {
  const float e = expm1f(fminf(x, 0.f));
  return x > 0.f ? x : e;
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  const float a = __builtin_amdgcn_readlane(__float_as_int(v), 0) , b = 0;
  (void)b;
  float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  (void)a;
  return (r0 + r1) + (r2 + r3);
}

template <int H0, int H1, int WPB>
__global__ __launch_bounds__(64 * WPB) void valu_fp_fwd(const float* __restrict__ W0, const float* __restrict__ b0,
                                                       const float* __restrict__ W1, const float* __restrict__ b1,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       const float* __restrict__ y0, int N, int n_steps,
                                                       const float* __restrict__ dts, float* __restrict__ latent,
                                                       double* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) float hb[WPB][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * WPB + w;
  if (n >= N) return;                                   // wave-uniform
  const float* y = y0 + (size_t)n * 8;
  // layer 0: dynamic columns in registers, static columns hoisted
  float w0[3], c1 = 0.f;
  if (lane < H0) {
    c1 = b0[lane];
#pragma unroll
    for (int s = 3; s < 8; ++s) c1 = fmaf(W0[lane * 8 + s], y[s], c1);
#pragma unroll
    for (int c = 0; c < 3; ++c) w0[c] = W0[lane * 8 + c];
  } else {
    w0[0] = w0[1] = w0[2] = 0.f;
  }
  float w1[H0], bb1 = 0.f;
#pragma unroll
  for (int k = 0; k < H0; ++k) w1[k] = lane < H1 ? W1[lane * H0 + k] : 0.f;
  if (lane < H1) bb1 = b1[lane];
  const float w2a = lane < H1 ? W2[lane] : 0.f, w2b = lane < H1 ? W2[H1 + lane] : 0.f;
  const float bq0 = b2[0], bq1 = b2[1];
  double ys[3] = {y[0], y[1], y[2]};
  float Y[3] = {y[0], y[1], y[2]};
  float k1[3], k2[3], k3[3];
  double sb = 0, sg = 0, sbb = 0, sgg = 0;
  const size_t NRL = (size_t)N * 8;
  if (lane < 8) latent[(size_t)n * 8 + lane] = y[lane];
  for (int step = 0; step < n_steps; ++step) {
    const float dt = dts[step];
    const double dd = dt;
    for (int j = 0; j < 4; ++j) {
      float z0 = fmaf(w0[2], Y[2], fmaf(w0[1], Y[1], fmaf(w0[0], Y[0], c1)));
      hb[w][lane] = elu1(z0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
      float z1a = bb1, z1b = 0.f;
#pragma unroll
      for (int k = 0; k < H0; k += 8) {
        const f4 h = *reinterpret_cast<const f4*>(&hb[w][k]);
        const f4 g = *reinterpret_cast<const f4*>(&hb[w][k + 4]);
        z1a = fmaf(w1[k], h[0], z1a); z1b = fmaf(w1[k + 4], g[0], z1b);
        z1a = fmaf(w1[k + 1], h[1], z1a); z1b = fmaf(w1[k + 5], g[1], z1b);
        z1a = fmaf(w1[k + 2], h[2], z1a); z1b = fmaf(w1[k + 6], g[2], z1b);
        z1a = fmaf(w1[k + 3], h[3], z1a); z1b = fmaf(w1[k + 7], g[3], z1b);
      }
      const float a1 = z1a + z1b;
      const float q0 = wave_sum(w2a * a1) + bq0, q1 = wave_sum(w2b * a1) + bq1;
      const float b = fabsf(q0), gm = fabsf(q1);
      sb += b; sg += gm; sbb += (double)b * b; sgg += (double)gm * gm;
      const float plus = (b * Y[0]) * Y[1], minus = gm * Y[1];
      float f[3] = {-plus, plus - minus, minus};
#pragma unroll
      for (int c = 0; c < 3; ++c) f[c] = (Y[c] > 2.f || Y[c] < -1.f) ? 0.f : f[c];
      if (j == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { k1[c] = f[c]; Y[c] = (float)(ys[c] + (dd * f[c]) * (1.0 / 3.0)); }
      } else if (j == 1) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { k2[c] = f[c]; Y[c] = (float)(ys[c] + dd * ((double)f[c] - (double)k1[c] * (1.0 / 3.0))); }
      } else if (j == 2) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { k3[c] = f[c]; Y[c] = (float)(ys[c] + dd * (((double)k1[c] - (double)k2[c]) + (double)f[c])); }
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          ys[c] += ((((double)k1[c] + 3.0 * ((double)k2[c] + (double)k3[c])) + (double)f[c]) * dd) * 0.125;
          Y[c] = (float)ys[c];
        }
        float* dst = latent + (size_t)(step + 1) * NRL + (size_t)n * 8;
        if (lane < 3) dst[lane] = lane == 0 ? Y[0] : (lane == 1 ? Y[1] : Y[2]);
        else if (lane < 8) dst[lane] = y[lane];
      }
    }
  }
  if (lane == 0) {
    double* st = stats + (size_t)n * 4;
    st[0] = sb; st[1] = sg; st[2] = sbb; st[3] = sgg;
  }
}

extern "C" int valu_fp32x32_fwd(const float* W0, const float* b0, const float* W1, const float* b1, const float* W2,
                                const float* b2, const float* y0, int N, int n_steps, const float* dts, float* latent,
                                double* stats, int wpb, hipStream_t s) {
  if (wpb == 4) hipLaunchKernelGGL((valu_fp_fwd<32, 32, 4>), dim3((N + 3) / 4), dim3(256), 0, s, W0, b0, W1, b1, W2, b2, y0, N, n_steps, dts, latent, stats);
  else if (wpb == 2) hipLaunchKernelGGL((valu_fp_fwd<32, 32, 2>), dim3((N + 1) / 2), dim3(128), 0, s, W0, b0, W1, b1, W2, b2, y0, N, n_steps, dts, latent, stats);
  else hipLaunchKernelGGL((valu_fp_fwd<32, 32, 1>), dim3(N), dim3(64), 0, s, W0, b0, W1, b1, W2, b2, y0, N, n_steps, dts, latent, stats);
  return (int)hipGetLastError();
}
