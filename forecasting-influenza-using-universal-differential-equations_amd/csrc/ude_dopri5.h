// gfx950 kernels for the adaptive Dormand-Prince (dopri5) solve of the UDE RHS:
// torchdiffeq.odeint(func, y0, t, rtol, atol, method='dopri5') -- the default method
// of the solver API the reference imports (lib/VAE.py:5) and BASELINE configs[2].
//
// torchdiffeq semantics (restated in oracle/ude_oracle_dopri5.py): ONE step size for
// the whole batch, chosen from the RMS error norm over every element of the
// (N, R, L) state; FSAL stages; accept iff error_ratio <= 1; dense output by the
// DPS 4th-order interpolant of the last accepted step; Hairer's initial step.
//
// Execution model: the per-trajectory work (6 RHS evaluations of a step attempt on
// MFMA, exactly the RK4 kernels' mlp_forward) runs in a persistent kernel over
// trajectory tiles; the batch-global decisions (error norm, accept / reject, next
// step size, which outputs the accepted step covers) are made by a one-workgroup
// control kernel that reads the per-workgroup partial sums.  Both are queued back
// to back on the stream, so the host only checks a "done" flag every few steps.
// The accepted state (y, f) is double-buffered in HBM ([tile][y|f][F][16], the
// checkpoint layout of the RK4 kernels); the control kernel flips the buffer index.
#pragma once
#include "ude_kernels.h"

namespace ude {

namespace dp {
constexpr double BETA[6][6] = {
    {1.0 / 5, 0, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656, 0},
    {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84},
};
constexpr double C_ERR[7] = {35.0 / 384 - 1951.0 / 21600, 0, 500.0 / 1113 - 22642.0 / 50085,
                             125.0 / 192 - 451.0 / 720, -2187.0 / 6784 - -12231.0 / 42400,
                             11.0 / 84 - 649.0 / 6300, -1.0 / 60.0};
constexpr double C_MID[7] = {6025192743.0 / 30085553152.0 / 2, 0, 51252292925.0 / 65400821598.0 / 2,
                             -2691868925.0 / 45128329728.0 / 2, 187940372067.0 / 1594534317056.0 / 2,
                             -1776094331.0 / 19743644256.0 / 2, 11237099.0 / 235043384.0 / 2};
enum : int { MODE_F0 = 0, MODE_TRIAL = 1, MODE_STEP = 2 };
}  // namespace dp

// Solver state shared by the kernels of one solve (device memory, ws head).
struct DopriCtl {
  double t0;              // start of the next attempt (end of the last accepted step)
  double dt;              // size of the next attempt (float64 time arithmetic)
  double acc_t0, acc_t1;  // last accepted step: dense-output interval
  float bdt[6][6];        // fp32(beta_ij) * fp32(dt)  (torchdiffeq: tableau in y's dtype)
  float edt[7];           // fp32(c_err_j) * fp32(dt)
  float mdt[7];           // fp32(c_mid_j) * fp32(dt)
  float acc_dt32;         // fp32 dt of the last accepted step (interp fit)
  float h0;               // start-up trial step
  float d0, d1;
  int cur;                // state buffer holding the accepted (y, f)
  int out_lo, out_hi;     // outputs [lo, hi) to write from the last accepted step
  int next_out;           // first output not yet covered
  int done, err;          // err: 1 dt underflow, 2 max steps, 3 non-finite
  int n_steps, n_accepted, n_evals;
};

struct DArgs {
  const float* pack;
  const float* y0;
  const double* t_out;    // T output times, float64
  float* latent;          // (T, N, R, L)
  float* S;               // [2][tile][2][F][16]  accepted (y, f), double-buffered
  float* Cm;              // [tile][F][16]        y_mid of the last attempt
  double* part;           // [grid][4]            per-workgroup partial sums
  double* stats_slab;     // [grid][5]            side statistics, summed over launches
  DopriCtl* ctl;
  int n_traj, n_tiles, n_times;
  float fa_w, rtol32, atol32;
};

__device__ __forceinline__ size_t dp_sidx(int n_tiles, int buf, int tile, int which, int F, int f, int t) {
  return (((((size_t)buf * n_tiles + tile) * 2 + which) * F + f) * TT) + t;
}

// Flux of one (trajectory, region) pair from the record's final-layer outputs
// (lib/models.py:130-150: |rates| -> SIR flux, + fa_w * Fa, masked outside [-1, 2]);
// accumulates the tracked side statistics (params / tracker) of this evaluation.
template <class M>
__device__ __forceinline__ void dp_flux(const float* rec, int r, bool valid, float fa_w, const float (&Y)[3],
                                        float (&f)[3], double (&st)[5]) {
  f[0] = f[1] = f[2] = 0.f;
  if constexpr (M::HAS_P) {
    const float q0 = rec[M::act_off(0, M::nl(0) - 1) + 2 * r];
    const float q1 = rec[M::act_off(0, M::nl(0) - 1) + 2 * r + 1];
    const float b = fabsf(q0), gm = fabsf(q1);
    const float plus = (b * Y[0]) * Y[1];
    const float minus = gm * Y[1];
    f[0] = -plus; f[1] = plus - minus; f[2] = minus;
    if (valid) {
      st[0] += (double)b; st[1] += (double)gm;
      st[2] += (double)b * (double)b; st[3] += (double)gm * (double)gm;
    }
  }
  if constexpr (M::HAS_A) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float fa = rec[M::act_off(1, M::nl(1) - 1) + 3 * r + c];
      if constexpr (M::HAS_P) f[c] = f[c] + fa_w * fa;
      else f[c] = fa;
      if (valid) st[4] += (double)fa * (double)fa;
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) f[c] = (Y[c] > 2.f || Y[c] < -1.f) ? 0.f : f[c];
}

// torchdiffeq _interp_fit + _interp_evaluate for one element (fp32, its op order)
__device__ __forceinline__ float dp_interp(float y0, float y1, float ym, float f0, float f1, float dt, float x) {
  const float a = ((2.f * dt) * (f1 - f0) - 8.f * (y1 + y0)) + 16.f * ym;
  const float b = (((dt * (5.f * f0 - 3.f * f1)) + 18.f * y0) + 14.f * y1) - 32.f * ym;
  const float c = (((dt * (f1 - 4.f * f0)) - 11.f * y0) - 5.f * y1) + 16.f * ym;
  const float d = dt * f0;
  float total = y0 + x * d;
  float xp = x * x;
  total = total + xp * c;
  xp = xp * x;
  total = total + xp * b;
  xp = xp * x;
  total = total + xp * a;
  return total;
}

template <class M, int MODE, int W>
__device__ void dopri_body(const DArgs& A, float* lds) {
  constexpr int SR = M::SR_F;
  constexpr int SL = M::SLOTS;
  int tid = threadIdx.x;
  const int lane = tid & 63;
  const Rsrc rs = make_rsrc(A.pack, M::PACK_TOTAL * 4);
  const size_t NRL = (size_t)A.n_traj * M::R * M::L;
  const DopriCtl* C = A.ctl;
  const int cur = C->cur;
  const bool done = MODE == dp::MODE_STEP && C->done != 0;
  const int out_lo = MODE == dp::MODE_STEP ? C->out_lo : 0, out_hi = MODE == dp::MODE_STEP ? C->out_hi : 0;
  double st[5] = {0, 0, 0, 0, 0};
  double ps0 = 0, ps1 = 0;

  #pragma unroll 1
  for (int i = tid; i < TT * SR; i += NTHREADS) lds[i] = 0.f;
  __syncthreads();

  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    // ---- dense output of the last accepted step (outputs out_lo .. out_hi-1) ----
    if (MODE == dp::MODE_STEP && out_hi > out_lo) {
      const double t0 = C->acc_t0, span = C->acc_t1 - C->acc_t0;
      const float dts = C->acc_dt32;
      #pragma unroll 1
      for (int p = tid; p < M::PAIRS; p += NTHREADS) {
        const int r = p / TT, t = p - r * TT, n = n0 + t;
        if (n >= A.n_traj) continue;
        float y0v[3], f0v[3], y1v[3], f1v[3], ym[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int f = 3 * r + c;
          y0v[c] = A.S[dp_sidx(A.n_tiles, cur ^ 1, tile, 0, M::F, f, t)];
          f0v[c] = A.S[dp_sidx(A.n_tiles, cur ^ 1, tile, 1, M::F, f, t)];
          y1v[c] = A.S[dp_sidx(A.n_tiles, cur, tile, 0, M::F, f, t)];
          f1v[c] = A.S[dp_sidx(A.n_tiles, cur, tile, 1, M::F, f, t)];
          ym[c] = A.Cm[((size_t)tile * M::F + f) * TT + t];
        }
        const float* src = A.y0 + ((size_t)n * M::R + r) * M::L;
        #pragma unroll 1
        for (int j = out_lo; j < out_hi; ++j) {
          const float x = (float)((A.t_out[j] - t0) / span);
          float* dst = A.latent + (size_t)j * NRL + ((size_t)n * M::R + r) * M::L;
#pragma unroll
          for (int c = 0; c < 3; ++c) dst[c] = dp_interp(y0v[c], y1v[c], ym[c], f0v[c], f1v[c], dts, x);
          for (int c = 3; c < M::L; ++c) dst[c] = src[c];
        }
      }
    }
    if (done) continue;

    // ---- stage 0 input ----------------------------------------------------------
    float ys[SL][3], k[7][SL][3];
    load_static<M, SR, M::XSF_OFF>(A.y0, lds, n0, A.n_traj);
    sfor<SL>([&](auto ss) {
      constexpr int sl = decltype(ss)::value;
      const int p = tid + sl * NTHREADS;
      if (p < M::PAIRS) {
        const int r = p / TT, t = p - r * TT, n = n0 + t;
        const bool valid = n < A.n_traj;
        float Y[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int f = 3 * r + c;
          if constexpr (MODE == dp::MODE_F0) {
            ys[sl][c] = valid ? A.y0[((size_t)n * M::R + r) * M::L + c] : 0.f;
            A.S[dp_sidx(A.n_tiles, 0, tile, 0, M::F, f, t)] = ys[sl][c];
            Y[c] = ys[sl][c];
            if (valid) {
              const float sc = A.atol32 + fabsf(ys[sl][c]) * A.rtol32;
              const float q = ys[sl][c] / sc;
              ps0 += (double)(q * q);
            }
          } else {
            const int b = MODE == dp::MODE_TRIAL ? 0 : cur;
            ys[sl][c] = A.S[dp_sidx(A.n_tiles, b, tile, 0, M::F, f, t)];
            k[0][sl][c] = A.S[dp_sidx(A.n_tiles, b, tile, 1, M::F, f, t)];
            if constexpr (MODE == dp::MODE_TRIAL) Y[c] = ys[sl][c] + C->h0 * k[0][sl][c];
            else Y[c] = ys[sl][c] + k[0][sl][c] * C->bdt[0][0];
          }
          lds[t * SR + M::Y_OFF + f] = Y[c];
        }
        if (MODE == dp::MODE_F0 && valid) {
          // latent[0] = y0 (all dims)
          const float* src = A.y0 + ((size_t)n * M::R + r) * M::L;
          float* dst = A.latent + ((size_t)n * M::R + r) * M::L;
          for (int c = 0; c < M::L; ++c) dst[c] = src[c];
        }
      }
    });
    if constexpr (MODE == dp::MODE_F0) {
      // the RMS norms run over every element of y, the constant dims included
      #pragma unroll 1
      for (int i = tid; i < TT * M::S; i += NTHREADS) {
        const int t = i / M::S, s = i - t * M::S, n = n0 + t;
        if (n < A.n_traj) {
          const int r = s / (M::L - 3), c = 3 + s - r * (M::L - 3);
          const float v = A.y0[((size_t)n * M::R + r) * M::L + c];
          const float q = v / (A.atol32 + fabsf(v) * A.rtol32);
          ps0 += (double)(q * q);
        }
      }
    }
    __syncthreads();
    f4 c1[M::NZ(W) > 0 ? M::NZ(W) : 1];
    static_hoist<M, W, SR, M::XSF_OFF>(rs, lds, c1, lane);
    __syncthreads();

    constexpr int NST = MODE == dp::MODE_STEP ? 6 : 1;
    #pragma unroll 1
    for (int s = 0; s < NST; ++s) {
      asm volatile("" : "+v"(tid));
      mlp_forward<M, W, SR>(rs, lds, c1, lane);
      sfor<SL>([&](auto ss) {
        constexpr int sl = decltype(ss)::value;
        const int p = tid + sl * NTHREADS;
        if (p < M::PAIRS) {
          const int r = p / TT, t = p - r * TT, n = n0 + t;
          const bool valid = n < A.n_traj;
          float* rec = lds + t * SR;
          float Y[3], f[3];
#pragma unroll
          for (int c = 0; c < 3; ++c) Y[c] = rec[M::Y_OFF + 3 * r + c];
          dp_flux<M>(rec, r, valid, A.fa_w, Y, f, st);
          if constexpr (MODE == dp::MODE_F0) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              A.S[dp_sidx(A.n_tiles, 0, tile, 1, M::F, 3 * r + c, t)] = f[c];
              if (valid) {
                const float q = f[c] / (A.atol32 + fabsf(ys[sl][c]) * A.rtol32);
                ps1 += (double)(q * q);
              }
            }
          } else if constexpr (MODE == dp::MODE_TRIAL) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
              if (valid) {
                const float q = (f[c] - k[0][sl][c]) / (A.atol32 + fabsf(ys[sl][c]) * A.rtol32);
                ps0 += (double)(q * q);
              }
          } else {
            // k_{s+1}; the next stage input y + sum_{j<=s+1} k_j beta_{s+1,j} dt
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              float kn = f[c];
#pragma unroll
              for (int q = 1; q < 7; ++q)
                if (q == s + 1) k[q][sl][c] = kn;
            }
            if (s < 5) {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                float acc = k[0][sl][c] * C->bdt[s + 1][0];
#pragma unroll
                for (int j = 1; j < 6; ++j)
                  if (j <= s + 1) acc = acc + k[j][sl][c] * C->bdt[s + 1][j];
                rec[M::Y_OFF + 3 * r + c] = ys[sl][c] + acc;
              }
            }
          }
        }
      });
      __syncthreads();
    }

    if constexpr (MODE == dp::MODE_STEP) {
      // y1 (5th order, = the last stage input), f1 = k7, error estimate, y_mid
      sfor<SL>([&](auto ss) {
        constexpr int sl = decltype(ss)::value;
        const int p = tid + sl * NTHREADS;
        if (p < M::PAIRS) {
          const int r = p / TT, t = p - r * TT, n = n0 + t;
          const bool valid = n < A.n_traj;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const int f = 3 * r + c;
            float acc = k[0][sl][c] * C->bdt[5][0];
#pragma unroll
            for (int j = 1; j < 6; ++j) acc = acc + k[j][sl][c] * C->bdt[5][j];
            const float y1 = ys[sl][c] + acc;
            float e = k[0][sl][c] * C->edt[0];
            float m = k[0][sl][c] * C->mdt[0];
#pragma unroll
            for (int j = 1; j < 7; ++j) {
              e = e + k[j][sl][c] * C->edt[j];
              m = m + k[j][sl][c] * C->mdt[j];
            }
            if (valid) {
              const float tol = A.atol32 + A.rtol32 * fmaxf(fabsf(ys[sl][c]), fabsf(y1));
              const float q = e / tol;
              ps0 += (double)(q * q);
              if (!isfinite(ys[sl][c])) ps1 += 1.0;
            }
            A.S[dp_sidx(A.n_tiles, cur ^ 1, tile, 0, M::F, f, t)] = y1;
            A.S[dp_sidx(A.n_tiles, cur ^ 1, tile, 1, M::F, f, t)] = k[6][sl][c];
            A.Cm[((size_t)tile * M::F + f) * TT + t] = ys[sl][c] + m;
          }
        }
      });
    }
    __syncthreads();
  }

  // deterministic per-workgroup partials: [ps0, ps1] and the side statistics
  double* red = reinterpret_cast<double*>(lds);
  double v[7] = {wave_sum(ps0), wave_sum(ps1), wave_sum(st[0]), wave_sum(st[1]), wave_sum(st[2]),
                 wave_sum(st[3]), wave_sum(st[4])};
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 7; ++c) red[(tid >> 6) * 7 + c] = v[c];
  }
  __syncthreads();
  if (tid < 7) {
    double s = 0;
    for (int w = 0; w < WAVES; ++w) s += red[w * 7 + tid];
    if (tid < 2) A.part[(size_t)blockIdx.x * 4 + tid] = s;
    else if (MODE == dp::MODE_F0) A.stats_slab[(size_t)blockIdx.x * 5 + tid - 2] = s;
    else if (!done) A.stats_slab[(size_t)blockIdx.x * 5 + tid - 2] += s;
  }
}

template <class M, int MODE>
__global__ __launch_bounds__(NTHREADS, 2) void ude_dopri_kernel(DArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w == 0) dopri_body<M, MODE, 0>(a, lds);
  else if (w == 1) dopri_body<M, MODE, 1>(a, lds);
  else if (w == 2) dopri_body<M, MODE, 2>(a, lds);
  else dopri_body<M, MODE, 3>(a, lds);
}

// fp32 coefficient tables of the next attempt (torchdiffeq casts the tableau and dt
// to y's dtype before the products)
__device__ inline void dp_set_tables(DopriCtl* C) {
  const float d = (float)C->dt;
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) C->bdt[i][j] = (float)dp::BETA[i][j] * d;
  for (int j = 0; j < 7; ++j) {
    C->edt[j] = (float)dp::C_ERR[j] * d;
    C->mdt[j] = (float)dp::C_MID[j] * d;
  }
}

// torchdiffeq _optimal_step_size (float64; safety 0.9, ifactor 10, dfactor 0.2, order 5)
__device__ inline double dp_optimal_step(double last, float er32) {
  if (er32 == 0.f) return last * 10.0;
  const double dfactor = er32 < 1.f ? 1.0 : 0.2;
  const double er = (double)er32;
  const double f = fmin(10.0, fmax(0.9 / pow(er, 0.2), dfactor));
  return last * f;
}

// One-workgroup control step.  MODE_F0: d0, d1, h0 of _select_initial_step;
// MODE_TRIAL: d2, first step; MODE_STEP: error norm, accept / reject, next dt,
// the outputs the accepted step covers.
template <int V_ = 0>
__global__ __launch_bounds__(64) void ude_dopri_ctl_kernel(int mode, const double* __restrict__ part, int grid,
                                                           DopriCtl* C, const double* __restrict__ t_out,
                                                           int n_times, double count, int max_steps,
                                                           double first_step) {
  __shared__ double sum[2];
  const int ln = threadIdx.x;
  double a = 0, b = 0;
  for (int g = ln; g < grid; g += 64) {
    a += part[(size_t)g * 4];
    b += part[(size_t)g * 4 + 1];
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    a += __shfl_xor(a, m, 64);
    b += __shfl_xor(b, m, 64);
  }
  if (ln == 0) { sum[0] = a; sum[1] = b; }
  __syncthreads();
  if (ln != 0) return;
  if (mode == dp::MODE_F0) {
    // rms in y's dtype: mean of the squares, then sqrt (fp32)
    const float d0 = sqrtf((float)(sum[0] / count)), d1 = sqrtf((float)(sum[1] / count));
    float h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : (0.01f * d0) / d1;
    C->h0 = fabsf(h0);
    C->d0 = d0;
    C->d1 = d1;
    C->n_evals = 1;
    return;
  }
  if (mode == dp::MODE_TRIAL) {
    if (first_step > 0.0) {
      C->dt = first_step;                        // options['first_step']: no start-up trial
    } else {
      const float h0 = C->h0, d1 = C->d1;
      const float d2 = fabsf(sqrtf((float)(sum[0] / count)) / h0);
      float h1 = (d1 <= 1e-15f && d2 <= 1e-15f) ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / fmaxf(d1, d2), 1.0f / 5.0f);
      h1 = fabsf(h1);
      C->dt = (double)fminf(100.f * h0, h1);
    }
    C->t0 = t_out[0];
    C->acc_t0 = C->acc_t1 = t_out[0];
    C->cur = 0;
    C->out_lo = C->out_hi = 0;
    C->next_out = 1;
    C->done = n_times <= 1;
    C->err = 0;
    C->n_steps = C->n_accepted = 0;
    C->n_evals = first_step > 0.0 ? 1 : 2;
    if (!C->done && !(C->t0 + C->dt > C->t0)) C->err = 1;
    dp_set_tables(C);
    return;
  }
  // MODE_STEP
  if (C->done || C->err) return;
  C->n_steps += 1;
  C->n_evals += 6;
  if (sum[1] > 0.0) { C->err = 3; return; }      // non-finite state (torchdiffeq asserts isfinite(y))
  const float er = sqrtf((float)(sum[0] / count));
  if (!(er == er)) { C->err = 3; return; }
  const bool accept = er <= 1.f;
  if (accept) {
    C->acc_t0 = C->t0;
    C->acc_t1 = C->t0 + C->dt;
    C->acc_dt32 = (float)C->dt;
    C->cur ^= 1;
    C->n_accepted += 1;
    int j = C->next_out;
    C->out_lo = j;
    while (j < n_times && t_out[j] <= C->acc_t1) ++j;
    C->out_hi = j;
    C->next_out = j;
    C->t0 = C->acc_t1;
    if (j >= n_times) C->done = 1;
  } else {
    C->out_lo = C->out_hi = 0;
  }
  C->dt = dp_optimal_step(C->dt, er);
  if (!C->done) {
    if (!(C->t0 + C->dt > C->t0)) C->err = 1;
    else if (C->n_steps >= max_steps) C->err = 2;
  }
  dp_set_tables(C);
}

}  // namespace ude
