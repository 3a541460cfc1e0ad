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
constexpr int LWAVES = 8;                    // loss-head waves per workgroup (two per SIMD)
constexpr int LTHREADS = LWAVES * 64;

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
  static constexpr int tiles_of(int w) { return (NTILE + LWAVES - 1 - w) / LWAVES; }
  static constexpr int SLAB = NP * KP + NP;  // per-workgroup dW | db partials
  static constexpr int LPR = 8;              // lanes per decoder output in the statistics pass
  static_assert(NP <= LTHREADS / LPR, "one lane octet per decoder output");
  // forward: each wave's GEMM tiles share one output-column tile (LWAVES % NT == 0), whose
  // decoder-weight fragment (KP/4 floats per lane) stays in registers -- no weight copy in LDS,
  // so two workgroups fit a CU
  static constexpr bool FWD_WREG = LWAVES % NT == 0;
  static int lds_bytes(int S, bool bwd = true) {
    const int SP = pad16(S);
    return (SP * XS + ((bwd || !FWD_WREG) ? NP * XS : 0) + SP * PS + 2 * NP) * 4;
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
  float* dlatent;        // (T, S*B, R, L) (backward), or (T, S*B, R, 3) when dl_sir
  const float* grad;     // device [g_nll, g_reg] (backward)
  int T, S, B;
  int dl_sir;            // backward writes only the S, I, R cotangents (the rest are zero)
};

// barrier for LDS hand-offs only: in-flight global loads (the next group's prefetch)
// stay in flight across it
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ float reg_term(float v) {
  return (v < 0.f ? fabsf(v) : 0.f) + (v > 1.f ? fabsf(1.f - v) : 0.f);
}

// LDS layout: X [SP][XS] | Wl [NP][XS] | P [SP][PS] (Q in place, backward) | bias [NP] | aux [NP]
// A group's rows are read once: when L % 4 == 0 the dims 0..3 of every (sample, region)
// are one 16-B load, and the next group's loads are issued into registers before the
// current group's GEMMs run (software pipelined across the group loop).
template <class D, int L, bool BWD, int W>
__device__ void loss_body(const LArgs& A, float* lds) {
  const int tid = threadIdx.x, lane = tid & 63, t16 = lane & 15, g = lane >> 4;
  const int S = A.S, SP = pad16(S), N = A.S * A.B;
  constexpr bool WF = !BWD && D::FWD_WREG;       // decoder weight in registers (forward)
  float* X = lds;
  float* Wl = X + SP * D::XS;
  float* P = WF ? Wl : Wl + D::NP * D::XS;
  float* bl = P + SP * D::PS;
  const size_t NRL = (size_t)N * D::R * L;
  const double M = (double)A.B * A.T * D::R;    // nll.mean() over (B, T, R)
  const float g_nll = BWD ? A.grad[0] : 0.f, g_reg = BWD ? A.grad[1] : 0.f;
  const int ngroups = A.T * A.B;

  // decoder weight -> LDS (backward) or this wave's fragment -> registers (forward), bias ->
  // LDS (zero padded), X padding zeroed, once per workgroup
  constexpr int NTF = WF ? D::NT : 1, WQ = WF ? D::KP / 4 : 1;
  const int ntw = W % NTF;                       // the forward GEMM's output-column tile of this wave
  float wq[WQ];
  if constexpr (WF) {
    const int o = ntw * 16 + t16;
#pragma unroll
    for (int kq = 0; kq < WQ; ++kq) {
      const int k = 4 * kq + g;
      wq[kq] = (o < D::R && k < D::K) ? A.W[o * D::K + k] : 0.f;
    }
  } else {
    #pragma unroll 1
    for (int i = tid; i < D::NP * D::XS; i += LTHREADS) {
      const int o = i / D::XS, k = i - o * D::XS;
      Wl[i] = (o < D::R && k < D::K) ? A.W[o * D::K + k] : 0.f;
    }
  }
  #pragma unroll 1
  for (int i = tid; i < SP * D::XS; i += LTHREADS) X[i] = 0.f;
  for (int i = tid; i < D::NP; i += LTHREADS) {
    bl[i] = i < D::R ? A.bias[i] : 0.f;
    bl[D::NP + i] = 0.f;                         // db partial (backward)
  }
  f4 dw[D::tiles_of(W) > 0 ? D::tiles_of(W) : 1];
  if constexpr (BWD) {
#pragma unroll
    for (int i = 0; i < D::tiles_of(W); ++i) dw[i] = f4zero();
  }
  double nll_acc = 0.0, reg_acc = 0.0;

  constexpr bool VEC = (L % 4) == 0;
  constexpr int PF = VEC ? (SP_MAX * D::R + LTHREADS - 1) / LTHREADS : 1;
  const int nreg = S * D::R;                     // (sample, region) pairs of a group
  f4 pf[PF];
  auto prefetch = [&](int grp) {
    const int t = grp / A.B, b = grp - t * A.B;
    const float* base = A.latent + (size_t)t * NRL;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      if (j * LTHREADS < nreg) {
        int i = tid + j * LTHREADS;
        i = i < nreg ? i : nreg - 1;
        const int s = i / D::R, r = i - s * D::R;
        pf[j] = *reinterpret_cast<const f4*>(base + ((size_t)(s * A.B + b) * D::R + r) * L);
      }
    }
  };
  if constexpr (VEC) {
    if ((int)blockIdx.x < ngroups) prefetch(blockIdx.x);
  }
  __syncthreads();

  #pragma unroll 1
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int t = grp / A.B, b = grp - t * A.B;
    // ---- the group's S sample rows (dims 0..2 of every region) -> X ----------------
    if constexpr (VEC) {
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int i = tid + j * LTHREADS;
        if (j * LTHREADS < nreg && i < nreg) {
          const int s = i / D::R, r = i - s * D::R;
          float* xp = X + s * D::XS + 3 * r;
          xp[0] = pf[j][0]; xp[1] = pf[j][1]; xp[2] = pf[j][2];
          if (!BWD) reg_acc += (double)(reg_term(pf[j][0]) + reg_term(pf[j][1]) + reg_term(pf[j][2]));
        }
      }
    } else {
      #pragma unroll 4
      for (int i = tid; i < S * D::K; i += LTHREADS) {
        const int s = i / D::K, k = i - s * D::K, r = k / 3, c = k - 3 * r;
        const float v = A.latent[(size_t)t * NRL + ((size_t)(s * A.B + b) * D::R + r) * L + c];
        if (!BWD) reg_acc += (double)reg_term(v);
        X[s * D::XS + k] = v;
      }
    }
    // per-region inputs of this group, loaded before the next group's prefetch
    float yv = -1.f, mu_in = 0.f, sd_in = 1.f;
    constexpr int LPR = D::LPR;
    const int rq = tid / LPR, part = tid % LPR;  // LPR lanes per region
    if (rq < D::R) {
      yv = A.y[((size_t)b * A.T + t) * D::R + rq];
      if (BWD) {
        mu_in = A.musd[(((size_t)t * A.B + b) * D::R + rq) * 2];
        sd_in = A.musd[(((size_t)t * A.B + b) * D::R + rq) * 2 + 1];
      }
    }
    if constexpr (VEC) {
      if (grp + (int)gridDim.x < ngroups) prefetch(grp + gridDim.x);
    }
    lds_barrier();
    // ---- P = X W^T + b  (S x R), one (M, N) tile per wave step ----------------------
    if constexpr (WF) {
      // this wave's tiles all have column tile ntw: two at a time (independent MFMA chains),
      // B operand from registers, A operands read in batches ahead of their MFMAs
      const int ntl = (SP / 16) * D::NT;
      const float bv = bl[ntw * 16 + t16];
      for (int id = W; id < ntl; id += 2 * LWAVES) {
        const int mt0 = id / D::NT, id1 = id + LWAVES;
        const bool two = id1 < ntl;
        const int mt1 = two ? id1 / D::NT : mt0;
        const float* x0 = X + (mt0 * 16 + t16) * D::XS + g;
        const float* x1 = X + (mt1 * 16 + t16) * D::XS + g;
        f4 acc0 = f4zero(), acc1 = f4zero();
        constexpr int QB = 8;
#pragma unroll
        for (int q0 = 0; q0 < WQ; q0 += QB) {
          float a0[QB], a1[QB];
#pragma unroll
          for (int q = 0; q < QB; ++q)
            if (q0 + q < WQ) { a0[q] = x0[4 * (q0 + q)]; a1[q] = x1[4 * (q0 + q)]; }
#pragma unroll
          for (int q = 0; q < QB; ++q)
            if (q0 + q < WQ) {
              acc0 = mfma4(a0[q], wq[q0 + q], acc0);
              acc1 = mfma4(a1[q], wq[q0 + q], acc1);
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) P[(mt0 * 16 + 4 * g + e) * D::PS + ntw * 16 + t16] = acc0[e] + bv;
        if (two) {
#pragma unroll
          for (int e = 0; e < 4; ++e) P[(mt1 * 16 + 4 * g + e) * D::PS + ntw * 16 + t16] = acc1[e] + bv;
        }
      }
    } else {
      for (int id = W; id < (SP / 16) * D::NT; id += LWAVES) {
        const int mt = id / D::NT, nt = id - mt * D::NT;
        f4 acc = f4zero();
#pragma unroll 8
        for (int kq = 0; kq < D::KP / 4; ++kq)
          acc = mfma4(X[(mt * 16 + t16) * D::XS + 4 * kq + g], Wl[(nt * 16 + t16) * D::XS + 4 * kq + g], acc);
        const float bv = bl[nt * 16 + t16];
#pragma unroll
        for (int e = 0; e < 4; ++e) P[(mt * 16 + 4 * g + e) * D::PS + nt * 16 + t16] = acc[e] + bv;
      }
    }
    lds_barrier();
    // ---- per region (4 lanes each): mean / unbiased std over the samples; nll or
    //      d nll / d pred (in place of P) and its column sum (db) ---------------------
    for (int r = rq; r < D::NP; r += LTHREADS / LPR) {
      const bool real = r < D::R;
      float mu = mu_in, sd = sd_in;
      if (!BWD) {
        // the lane's samples s = part + LPR j read at once (one LDS latency), then two passes
        constexpr int NV = SP_MAX / LPR;
        float v[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int s = part + LPR * j;
          v[j] = s < S ? P[s * D::PS + r] : 0.f;
        }
        // fp64 sums: the mean is (nearly) correctly rounded, so the cancellation in the
        // backward's sum_s (pred_s - mean) (the decoder-bias gradient) stays at rounding level
        double s1 = 0.0;
#pragma unroll
        for (int j = 0; j < NV; ++j) s1 += (double)v[j];
        s1 += __shfl_xor(s1, 1, 64);
        s1 += __shfl_xor(s1, 2, 64);
        s1 += __shfl_xor(s1, 4, 64);
        mu = (float)(s1 / (double)S);
        double s2 = 0.0;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const float d = v[j] - mu;
          s2 += part + LPR * j < S ? (double)(d * d) : 0.0;
        }
        s2 += __shfl_xor(s2, 1, 64);
        s2 += __shfl_xor(s2, 2, 64);
        s2 += __shfl_xor(s2, 4, 64);
        sd = sqrtf((float)(s2 / (double)(S - 1)));
        if (real && part == 0) {
          A.musd[(((size_t)t * A.B + b) * D::R + r) * 2] = mu;
          A.musd[(((size_t)t * A.B + b) * D::R + r) * 2 + 1] = sd;
          if (yv != -1.f) {
            const float z = (yv - mu) / sd;
            nll_acc += (double)(0.5f * z * z + logf(sd) + 0.9189385332046727f);
          }
        }
      } else {
        // d/d pred_s of mean_{b,t,r}(mask * (-log N(y | mu, sd)))
        float cm = 0.f, cs = 0.f;
        if (real && yv != -1.f) {
          const float iv = 1.f / sd, dy = yv - mu;
          const float dmu = -dy * iv * iv;                          // d nll / d mu
          const float dsd = iv - dy * dy * iv * iv * iv;            // d nll / d sd
          const float sc = (float)((double)g_nll / M);
          cm = sc * dmu / (float)S;
          cs = sc * dsd * iv / (float)(S - 1);
        }
        double s1 = 0.0;
        for (int s = part; s < SP; s += LPR) {
          const float q = s < S ? cm + cs * (P[s * D::PS + r] - mu) : 0.f;
          P[s * D::PS + r] = q;
          s1 += (double)q;
        }
        s1 += __shfl_xor(s1, 1, 64);
        s1 += __shfl_xor(s1, 2, 64);
        s1 += __shfl_xor(s1, 4, 64);
        if (part == 0) bl[D::NP + r] += (float)s1;     // aux row: db partial
      }
    }
    if constexpr (BWD) {
      lds_barrier();
      // ---- dW += Q^T X (R x 3R) ----------------------------------------------------
#pragma unroll 1
      for (int sq = 0; sq < SP / 4; ++sq) {
#pragma unroll
        for (int i = 0; i < D::tiles_of(W); ++i) {   // independent chains, one per tile
          const int id = W + LWAVES * i, nt = id / D::KT, kt = id - nt * D::KT;
          dw[i] = mfma4(P[(4 * sq + g) * D::PS + nt * 16 + t16], X[(4 * sq + g) * D::XS + kt * 16 + t16], dw[i]);
        }
      }
      // ---- d X = Q W  (S x 3R), + g_reg * latent_init_loss'(x), in place of X ----------
      // (after every wave has finished reading X for dW; each tile is one wave's)
      lds_barrier();
      // tiles of this wave in chunks of CH independent MFMA chains
      constexpr int DXT = ((SP_MAX / 16) * D::KT + LWAVES - 1) / LWAVES, CH = DXT < 3 ? DXT : 3;
      const int ndx = (SP / 16) * D::KT;
#pragma unroll 1
      for (int c0 = 0; c0 < DXT && W + LWAVES * c0 < ndx; c0 += CH) {
        f4 dx[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) dx[i] = f4zero();
#pragma unroll 2
        for (int rq4 = 0; rq4 < D::NP / 4; ++rq4) {
#pragma unroll
          for (int i = 0; i < CH; ++i) {
            const int id = W + LWAVES * (c0 + i), mt = id / D::KT, kt = id - mt * D::KT;
            if (id < ndx)
              dx[i] = mfma4(P[(mt * 16 + t16) * D::PS + 4 * rq4 + g], Wl[(4 * rq4 + g) * D::XS + kt * 16 + t16], dx[i]);
          }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int id = W + LWAVES * (c0 + i), mt = id / D::KT, kt = id - mt * D::KT;
          if (id < ndx)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float* xp = X + (mt * 16 + 4 * g + e) * D::XS + kt * 16 + t16;
              const float x = *xp;
              const float dr = x < 0.f ? -1.f : (x > 1.f ? 1.f : 0.f);
              *xp = dx[i][e] + g_reg * dr;
            }
        }
      }
      lds_barrier();
      // ---- d latent rows: compact S, I, R cotangents (handed to the solve's backward) ----
      if (A.dl_sir) {
        constexpr int R3 = 3 * D::R;
        #pragma unroll 4
        for (int i = tid; i < S * R3; i += LTHREADS) {
          const int s = i / R3, e = i - s * R3;
          A.dlatent[((size_t)t * N + (size_t)(s * A.B + b)) * R3 + e] = X[s * D::XS + e];
        }
      // ---- or whole rows of d latent (static dims 0) with 16-B stores -------------------
      } else if constexpr ((D::R * L) % 4 == 0) {
        constexpr int RL4 = D::R * L / 4;
#pragma unroll 4
        for (int i = tid; i < S * RL4; i += LTHREADS) {
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
        for (int i = tid; i < S * D::R * L; i += LTHREADS) {
          const int s = i / (D::R * L), e = i - s * D::R * L, r = e / L, c = e - r * L;
          A.dlatent[(size_t)t * NRL + (size_t)(s * A.B + b) * D::R * L + e] = c < 3 ? X[s * D::XS + 3 * r + c] : 0.f;
        }
      }
      // (X padding stays zero: Q rows s >= S and W's padding columns are zero, so dX is 0
      // there, and the next group overwrites every real entry)
    }
    lds_barrier();
  }

  if constexpr (BWD) {
    float* my = A.slab + (size_t)blockIdx.x * D::SLAB;
#pragma unroll
    for (int i = 0; i < D::tiles_of(W); ++i) {
      const int id = W + LWAVES * i, nt = id / D::KT, kt = id - nt * D::KT;
#pragma unroll
      for (int e = 0; e < 4; ++e) my[(nt * 16 + 4 * g + e) * D::KP + kt * 16 + t16] = dw[i][e];
    }
    __syncthreads();
    for (int r = tid; r < D::NP; r += LTHREADS) my[D::NP * D::KP + r] = bl[D::NP + r];
  } else {
    double* red = reinterpret_cast<double*>(lds);
    const double v0 = wave_sum(nll_acc), v1 = wave_sum(reg_acc);
    __syncthreads();
    if (lane == 0) { red[(tid >> 6) * 2] = v0; red[(tid >> 6) * 2 + 1] = v1; }
    __syncthreads();
    if (tid < 2) {
      double s = 0;
      for (int w = 0; w < LWAVES; ++w) s += red[w * 2 + tid];
      A.part[(size_t)blockIdx.x * 2 + tid] = s;
    }
  }
}

template <class D, int L, bool BWD>
__global__ __launch_bounds__(LTHREADS) void ude_loss_kernel(LArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  switch (w) {
    case 0: loss_body<D, L, BWD, 0>(a, lds); break;
    case 1: loss_body<D, L, BWD, 1>(a, lds); break;
    case 2: loss_body<D, L, BWD, 2>(a, lds); break;
    case 3: loss_body<D, L, BWD, 3>(a, lds); break;
    case 4: loss_body<D, L, BWD, 4>(a, lds); break;
    case 5: loss_body<D, L, BWD, 5>(a, lds); break;
    case 6: loss_body<D, L, BWD, 6>(a, lds); break;
    default: loss_body<D, L, BWD, 7>(a, lds); break;
  }
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

// sum of the per-workgroup dW / db slabs -> (R, 3R) weight gradient and (R) bias gradient:
// a block owns 64 slab columns; its 4 waves sum interleaved quarters of the slabs with 8
// independent accumulators each, then a fixed-order combine in LDS (deterministic)
template <class D>
__global__ __launch_bounds__(256) void ude_loss_grad_finalize_kernel(const float* __restrict__ slab, int grid,
                                                                     float* __restrict__ dW, float* __restrict__ db) {
  __shared__ float red[4][64];
  const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int off = blockIdx.x * 64 + ln;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (off < D::SLAB) {
    int i = wv;
    for (; i + 28 < grid; i += 32)
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += slab[(size_t)(i + 4 * u) * D::SLAB + off];
    for (; i < grid; i += 4) acc[0] += slab[(size_t)i * D::SLAB + off];
  }
  red[wv][ln] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (wv == 0 && off < D::SLAB) {
    const float v = (red[0][ln] + red[1][ln]) + (red[2][ln] + red[3][ln]);
    if (off < D::NP * D::KP) {
      const int o = off / D::KP, k = off - o * D::KP;
      if (o < D::R && k < D::K) dW[o * D::K + k] = v;
    } else {
      const int o = off - D::NP * D::KP;
      if (o < D::R) db[o] = v;
    }
  }
}

}  // namespace ude
