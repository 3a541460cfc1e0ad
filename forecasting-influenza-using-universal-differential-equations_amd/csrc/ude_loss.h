// gfx950 kernels for the training loss head that consumes the solve's latent:
//   y_pred = Decoder(latent[..., :3])            lib/models.py:27-51 (Flatten -> Linear(3R -> R))
//            .reshape(T, S, B, R).permute(2, 1, 0, 3)                       lib/VAE.py:138
//   nll    = nll_loss(y_pred, y)                  lib/train_functions.py:81-90
//            (mean / unbiased std over the S samples, -Normal.log_prob, masked y == -1, mean)
//   reg    = latent_init_loss(latent[..., :3])    lib/train_functions.py:116-126
//            (sum of |x| where x < 0 and |1 - x| where x > 1; the VAE adds 0.1 * reg)
// Forward and backward are one pass each over the latent (no (T,N,R,3) slice copies,
// no permuted reductions): a workgroup takes one (t, window b) group at a time -- its S
// sample rows n = s*B + b -- and runs the decoder GEMM, its transposed GEMM and the
// decoder-weight gradient GEMM on v_mfma_f32_16x16x4_f32 with the group in LDS.
#pragma once
#include "ude_kernels.h"

namespace ude {

constexpr int SP_MAX = 128;                  // samples per group the loss head holds (LDS)

template <int R_>
struct LossDims {
  static constexpr int R = R_;
  static constexpr int K = 3 * R;            // decoder inputs (S, I, R of every region)
  static constexpr int KP = pad16(K);
  static constexpr int NP = pad16(R);        // decoder outputs, padded
  static constexpr int KT = KP / 16, NT = NP / 16;
  static constexpr int XS = KP + 4;          // LDS row strides (== 4 mod 64 floats where possible)
  static constexpr int PS = NP + 4;
  static constexpr int NTILE = NT * KT;      // dW tiles (16 x 16)
  static constexpr int tiles_of(int w) { return (NTILE + WAVES - 1 - w) / WAVES; }
  static constexpr int SLAB = NP * KP + NP;  // per-workgroup dW | db partials
  static int lds_bytes(int S) {
    const int SP = pad16(S);
    return (SP * XS + NP * XS + 2 * SP * PS + 2 * NP) * 4;
  }
};

struct LArgs {
  const float* latent;   // (T, S*B, R, L)
  const float* W;        // (R, 3R)   decoder weight
  const float* bias;     // (R)
  const float* y;        // (B, T, R) targets, -1 = missing
  float* musd;           // (T, B, R, 2)   per-group mean / std of the predictions
  double* part;          // [grid][2]     nll / reg partial sums
  float* slab;           // [grid][SLAB]  dW / db partials (backward)
  float* dlatent;        // (T, S*B, R, L) (backward)
  const float* grad;     // device [g_nll, g_reg] (backward)
  int T, S, B;
};

// LDS layout: X [SP][XS] | Wl [NP][XS] | P [SP][PS] | Q [SP][PS] | bias [NP] | aux [NP]
template <class D, int L, bool BWD, int W>
__device__ void loss_body(const LArgs& A, float* lds) {
  const int tid = threadIdx.x, lane = tid & 63, t16 = lane & 15, g = lane >> 4;
  const int S = A.S, SP = pad16(S), N = A.S * A.B;
  float* X = lds;
  float* Wl = X + SP * D::XS;
  float* P = Wl + D::NP * D::XS;
  float* Q = P + SP * D::PS;
  float* bl = Q + SP * D::PS;
  const size_t NRL = (size_t)N * D::R * L;
  const double M = (double)A.B * A.T * D::R;    // nll.mean() over (B, T, R)
  const float g_nll = BWD ? A.grad[0] : 0.f, g_reg = BWD ? A.grad[1] : 0.f;

  // decoder weight / bias -> LDS (zero padded), once per workgroup
  #pragma unroll 1
  for (int i = tid; i < D::NP * D::XS; i += NTHREADS) {
    const int o = i / D::XS, k = i - o * D::XS;
    Wl[i] = (o < D::R && k < D::K) ? A.W[o * D::K + k] : 0.f;
  }
  for (int i = tid; i < D::NP; i += NTHREADS) {
    bl[i] = i < D::R ? A.bias[i] : 0.f;
    bl[D::NP + i] = 0.f;                         // db partial (backward)
  }
  f4 dw[D::tiles_of(W) > 0 ? D::tiles_of(W) : 1];
  if constexpr (BWD) {
#pragma unroll
    for (int i = 0; i < D::tiles_of(W); ++i) dw[i] = f4zero();
  }
  double nll_acc = 0.0, reg_acc = 0.0;
  __syncthreads();

  for (int grp = blockIdx.x; grp < A.T * A.B; grp += gridDim.x) {
    const int t = grp / A.B, b = grp - t * A.B;
    // ---- the group's S sample rows (dims 0..2 of every region) -> X ----------------
    // zero the padding (rows >= S, columns >= 3R), then stream whole rows (R*L floats,
    // contiguous) with 16-B loads and keep the dynamic dims
    #pragma unroll 1
    for (int i = tid; i < SP * D::XS; i += NTHREADS) {
      const int s = i / D::XS, k = i - s * D::XS;
      if (s >= S || k >= D::K) X[i] = 0.f;
    }
    if constexpr ((D::R * L) % 4 == 0) {
      constexpr int RL4 = D::R * L / 4;
      const int n4 = S * RL4;
#pragma unroll 4
      for (int i = tid; i < n4; i += NTHREADS) {
        const int s = i / RL4, j = i - s * RL4;
        const f4 v = *reinterpret_cast<const f4*>(A.latent + (size_t)t * NRL + (size_t)(s * A.B + b) * D::R * L + 4 * j);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = 4 * j + q, r = e / L, c = e - r * L;
          if (c < 3) {
            X[s * D::XS + 3 * r + c] = v[q];
            if (!BWD) reg_acc += (double)((v[q] < 0.f ? fabsf(v[q]) : 0.f) + (v[q] > 1.f ? fabsf(1.f - v[q]) : 0.f));
          }
        }
      }
    } else {
      #pragma unroll 4
      for (int i = tid; i < S * D::K; i += NTHREADS) {
        const int s = i / D::K, k = i - s * D::K, r = k / 3, c = k - 3 * r;
        const float v = A.latent[(size_t)t * NRL + ((size_t)(s * A.B + b) * D::R + r) * L + c];
        if (!BWD) reg_acc += (double)((v < 0.f ? fabsf(v) : 0.f) + (v > 1.f ? fabsf(1.f - v) : 0.f));
        X[s * D::XS + k] = v;
      }
    }
    __syncthreads();
    // ---- P = X W^T + b  (S x R) ----------------------------------------------------
    for (int mt = W; mt < SP / 16; mt += WAVES) {
      f4 acc[D::NT];
#pragma unroll
      for (int nt = 0; nt < D::NT; ++nt) acc[nt] = f4zero();
#pragma unroll 4
      for (int kq = 0; kq < D::KP / 4; ++kq) {
        const float a = X[(mt * 16 + t16) * D::XS + 4 * kq + g];
#pragma unroll
        for (int nt = 0; nt < D::NT; ++nt) acc[nt] = mfma4(a, Wl[(nt * 16 + t16) * D::XS + 4 * kq + g], acc[nt]);
      }
#pragma unroll
      for (int nt = 0; nt < D::NT; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) P[(mt * 16 + 4 * g + e) * D::PS + nt * 16 + t16] = acc[nt][e] + bl[nt * 16 + t16];
    }
    __syncthreads();
    // ---- per region: mean / unbiased std over the samples; nll or d nll / d pred ---
    for (int r = tid; r < D::R; r += NTHREADS) {
      float mu, sd;
      if (!BWD) {
        float s1 = 0.f;
        for (int s = 0; s < S; ++s) s1 += P[s * D::PS + r];
        mu = s1 / (float)S;
        float s2 = 0.f;
        for (int s = 0; s < S; ++s) { const float d = P[s * D::PS + r] - mu; s2 += d * d; }
        sd = sqrtf(s2 / (float)(S - 1));
        A.musd[(((size_t)t * A.B + b) * D::R + r) * 2] = mu;
        A.musd[(((size_t)t * A.B + b) * D::R + r) * 2 + 1] = sd;
      } else {
        mu = A.musd[(((size_t)t * A.B + b) * D::R + r) * 2];
        sd = A.musd[(((size_t)t * A.B + b) * D::R + r) * 2 + 1];
      }
      const float yv = A.y[((size_t)b * A.T + t) * D::R + r];
      const bool live = yv != -1.f;
      if (!BWD) {
        if (live) {
          const float z = (yv - mu) / sd;
          nll_acc += (double)(0.5f * z * z + logf(sd) + 0.9189385332046727f);
        }
      } else {
        // d/d pred_s of mean_{b,t,r}(mask * (-log N(y | mu, sd)))
        float cm = 0.f, cs = 0.f;
        if (live) {
          const float iv = 1.f / sd, dy = yv - mu;
          const float dmu = -dy * iv * iv;                          // d nll / d mu
          const float dsd = iv - dy * dy * iv * iv * iv;            // d nll / d sd
          const float sc = (float)((double)g_nll / M);
          cm = sc * dmu / (float)S;
          cs = sc * dsd * iv / (float)(S - 1);
        }
        for (int s = 0; s < SP; ++s) Q[s * D::PS + r] = s < S ? cm + cs * (P[s * D::PS + r] - mu) : 0.f;
      }
    }
    if constexpr (BWD) {
      for (int i = tid; i < SP * (D::NP - D::R); i += NTHREADS) {
        const int s = i / (D::NP - D::R), r = D::R + i - s * (D::NP - D::R);
        Q[s * D::PS + r] = 0.f;
      }
      __syncthreads();
      // ---- dW += Q^T X (R x 3R) ----------------------------------------------------
#pragma unroll
      for (int i = 0; i < D::tiles_of(W); ++i) {
        const int id = W + WAVES * i, nt = id / D::KT, kt = id - nt * D::KT;
        f4 acc = dw[i];
        for (int sq = 0; sq < SP / 4; ++sq)
          acc = mfma4(Q[(4 * sq + g) * D::PS + nt * 16 + t16], X[(4 * sq + g) * D::XS + kt * 16 + t16], acc);
        dw[i] = acc;
      }
      // ---- d X = Q W  (S x 3R), + g_reg * latent_init_loss'(x), in place of X ----------
      // (every wave first finishes reading X / Q; each M tile is owned by one wave)
      constexpr int MI = (SP_MAX / 16 + WAVES - 1) / WAVES;
      f4 dx[MI][D::KT];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int mt = W + WAVES * mi;
        if (mt < SP / 16) {
#pragma unroll
          for (int kt = 0; kt < D::KT; ++kt) dx[mi][kt] = f4zero();
#pragma unroll 4
          for (int rq = 0; rq < D::NP / 4; ++rq) {
            const float a = Q[(mt * 16 + t16) * D::PS + 4 * rq + g];
#pragma unroll
            for (int kt = 0; kt < D::KT; ++kt) dx[mi][kt] = mfma4(a, Wl[(4 * rq + g) * D::XS + kt * 16 + t16], dx[mi][kt]);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int mt = W + WAVES * mi;
        if (mt < SP / 16)
#pragma unroll
          for (int kt = 0; kt < D::KT; ++kt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float* xp = X + (mt * 16 + 4 * g + e) * D::XS + kt * 16 + t16;
              const float x = *xp;
              const float dr = x < 0.f ? -1.f : (x > 1.f ? 1.f : 0.f);
              *xp = dx[mi][kt][e] + g_reg * dr;
            }
      }
      __syncthreads();
      // ---- whole rows of d latent (static dims 0) with 16-B stores ---------------------
      if constexpr ((D::R * L) % 4 == 0) {
        constexpr int RL4 = D::R * L / 4;
#pragma unroll 4
        for (int i = tid; i < S * RL4; i += NTHREADS) {
          const int s = i / RL4, j = i - s * RL4;
          f4 v;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = 4 * j + q, r = e / L, c = e - r * L;
            v[q] = c < 3 ? X[s * D::XS + 3 * r + c] : 0.f;
          }
          *reinterpret_cast<f4*>(A.dlatent + (size_t)t * NRL + (size_t)(s * A.B + b) * D::R * L + 4 * j) = v;
        }
      } else {
        #pragma unroll 4
        for (int i = tid; i < S * D::R * L; i += NTHREADS) {
          const int s = i / (D::R * L), e = i - s * D::R * L, r = e / L, c = e - r * L;
          A.dlatent[(size_t)t * NRL + (size_t)(s * A.B + b) * D::R * L + e] = c < 3 ? X[s * D::XS + 3 * r + c] : 0.f;
        }
      }
      for (int r = tid; r < D::NP; r += NTHREADS) {
        float s1 = 0.f;
        for (int s = 0; s < S; ++s) s1 += Q[s * D::PS + r];
        bl[D::NP + r] += s1;      // aux row: db partial
      }
    }
    __syncthreads();
  }

  if constexpr (BWD) {
    float* my = A.slab + (size_t)blockIdx.x * D::SLAB;
#pragma unroll
    for (int i = 0; i < D::tiles_of(W); ++i) {
      const int id = W + WAVES * i, nt = id / D::KT, kt = id - nt * D::KT;
#pragma unroll
      for (int e = 0; e < 4; ++e) my[(nt * 16 + 4 * g + e) * D::KP + kt * 16 + t16] = dw[i][e];
    }
    for (int r = tid; r < D::NP; r += NTHREADS) my[D::NP * D::KP + r] = bl[D::NP + r];
  } else {
    double* red = reinterpret_cast<double*>(lds);
    const double v0 = wave_sum(nll_acc), v1 = wave_sum(reg_acc);
    if (lane == 0) { red[(tid >> 6) * 2] = v0; red[(tid >> 6) * 2 + 1] = v1; }
    __syncthreads();
    if (tid < 2) {
      double s = 0;
      for (int w = 0; w < WAVES; ++w) s += red[w * 2 + tid];
      A.part[(size_t)blockIdx.x * 2 + tid] = s;
    }
  }
}

template <class D, int L, bool BWD>
__global__ __launch_bounds__(NTHREADS) void ude_loss_kernel(LArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w == 0) loss_body<D, L, BWD, 0>(a, lds);
  else if (w == 1) loss_body<D, L, BWD, 1>(a, lds);
  else if (w == 2) loss_body<D, L, BWD, 2>(a, lds);
  else loss_body<D, L, BWD, 3>(a, lds);
}

// nll = sum / (B T R), reg = sum (fixed-order sums over the workgroup partials)
template <int V_ = 0>
__global__ void ude_loss_finalize_kernel(const double* __restrict__ part, int grid, double M, float* __restrict__ out) {
  __shared__ double tot[2];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (wv < 2) {
    double s = 0;
    for (int i = ln; i < grid; i += 64) s += part[(size_t)i * 2 + wv];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (ln == 0) tot[wv] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) { out[0] = (float)(tot[0] / M); out[1] = (float)tot[1]; }
}

// sum of the per-workgroup dW / db slabs -> (R, 3R) weight gradient and (R) bias gradient
template <class D>
__global__ __launch_bounds__(256) void ude_loss_grad_finalize_kernel(const float* __restrict__ slab, int grid,
                                                                     float* __restrict__ dW, float* __restrict__ db) {
  const int off = blockIdx.x * 256 + threadIdx.x;
  if (off >= D::SLAB) return;
  float v = 0.f;
  for (int i = 0; i < grid; ++i) v += slab[(size_t)i * D::SLAB + off];
  if (off < D::NP * D::KP) {
    const int o = off / D::KP, k = off - o * D::KP;
    if (o < D::R && k < D::K) dW[o * D::K + k] = v;
  } else {
    const int o = off - D::NP * D::KP;
    if (o < D::R) db[o] = v;
  }
}

}  // namespace ude
