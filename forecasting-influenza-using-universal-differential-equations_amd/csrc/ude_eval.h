// gfx950 kernels for ONE evaluation of the UDE right-hand side and its VJP:
//   forward  f = RHS(x), rates = |net(x)|, Fa = aug_net(x)     (lib/models.py:129-146, :177-188,
//            :230-254 -- the tensors forward() returns and appends to params / tracker)
//   VJP      dx, dW given the cotangents of f, rates and Fa
// for every trajectory of a batch, one tile of 16 trajectories per workgroup, on the same MFMA
// layer machinery as the fused RK4 kernels (mlp_forward / mlp_backward, register-resident
// weights, static-feature hoist).
//
// These serve every solve that is not the fused fixed-grid RK4: the RHS module's forward on
// a HIP device (so eager solvers -- dopri5 with autograd, torchdiffeq's odeint_adjoint
// backward, euler / midpoint -- call one kernel per evaluation instead of ~40 PyTorch ops),
// and the Bayesian RHS at sizes whose two dW accumulator sets do not fit the fused kernel's
// registers (models_bayes.py:43-48: each evaluation's sampled weights are a deterministic
// RHS for that evaluation; d mean / d std follow from dW on the host).
#pragma once
#include "ude_kernels.h"

namespace ude {

struct EArgs {
  const float* pack;
  const float* x;          // (N, R, L) evaluation point
  float* f;                // forward: (N, R, L) RHS value (dims >= 3 zero, masked)
  float* rates;            // forward: (N, R, 2) |net(x)| (nullable)
  float* fa;               // forward: (N, R, 3) aug_net(x) (nullable)
  const float* cot_f;      // VJP: (N, R, L) cotangent of f (dims >= 3 ignored: f is 0 there)
  const float* cot_rates;  // VJP: (N, R, 2) (nullable: zero)
  const float* cot_fa;     // VJP: (N, R, 3) (nullable: zero)
  float* dx;               // VJP: (N, R, L); static dims written by ude_dy0_static_kernel (HOIST)
  float* slab;             // VJP: per-workgroup dW partials [grid][SLAB_STRIDE]
  float* g0buf;            // VJP: per-trajectory layer-0 output gradients [tile][K0][16] (HOIST)
  int n_traj, n_tiles;
  float fa_w;
  float* fout;             // VJP (nullable): f_scale * f(x) (N, R, L) from the same launch
  float f_scale;
  unsigned int* ctl;       // VJP (HOIST): the tail's ticket words, zeroed here for the launch behind
  int n_ctl;
};

// f = RHS(x) of pair p from the record after mlp_forward (lib/models.py:130-150), scaled by `scale`
// (dims >= 3 zero, masked outside [-1, 2]).
template <class M, int SR>
__device__ __forceinline__ void eval_f_pairs(const float* lds, const EArgs& A, int n0, float* out, float scale) {
  // row-mapped: consecutive lanes write consecutive (n, r) rows
  const int nvalid = min(TT, A.n_traj - n0) * M::R;
  #pragma unroll 1
  for (int i = threadIdx.x; i < nvalid; i += NTHREADS) {
    const int t = i / M::R, r = i - t * M::R;
    const float* rec = lds + t * SR;
    float Y[3], f[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) Y[c] = rec[M::Y_OFF + 3 * r + c];
    if constexpr (M::HAS_P) {
      const float b = fabsf(rec[M::act_off(0, M::nl(0) - 1) + 2 * r]);
      const float gm = fabsf(rec[M::act_off(0, M::nl(0) - 1) + 2 * r + 1]);
      const float plus = (b * Y[0]) * Y[1];
      const float minus = gm * Y[1];
      f[0] = -plus; f[1] = plus - minus; f[2] = minus;
    }
    if constexpr (M::HAS_A) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v = rec[M::act_off(1, M::nl(1) - 1) + 3 * r + c];
        if constexpr (M::HAS_P) f[c] = f[c] + A.fa_w * v;
        else f[c] = v;
      }
    }
    float* dst = out + ((size_t)n0 * M::R + i) * M::L;
#pragma unroll
    for (int c = 0; c < 3; ++c) dst[c] = scale * ((Y[c] > 2.f || Y[c] < -1.f) ? 0.f : f[c]);
    for (int c = 3; c < M::L; ++c) dst[c] = 0.f;
  }
}

// ---- forward --------------------------------------------------------------------------
template <class M, int W>
__device__ void eval_fwd_body(const EArgs& A, float* lds) {
  constexpr int SR = M::SR_F;
  const int tid = threadIdx.x, lane = tid & 63;
  const Rsrc rs = make_rsrc(A.pack, M::PACK_TOTAL * 4);
  WRegs<M, W, false> wr;
  wr.load(rs, lane);
  #pragma unroll 1
  for (int i = tid; i < TT * SR; i += NTHREADS) lds[i] = 0.f;
  __syncthreads();
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    #pragma unroll 1
    for (int p = tid; p < M::PAIRS; p += NTHREADS) {
      const int r = p / TT, t = p - r * TT, n = n0 + t;
      const float* src = A.x + ((size_t)n * M::R + r) * M::L;
#pragma unroll
      for (int c = 0; c < 3; ++c) lds[t * SR + M::Y_OFF + 3 * r + c] = n < A.n_traj ? src[c] : 0.f;
    }
    load_static<M, SR, M::XSF_OFF>(A.x, lds, n0, A.n_traj);
    __syncthreads();
    f4 c1[M::NZ(W) > 0 ? M::NZ(W) : 1];
    static_hoist<M, W, SR, M::XSF_OFF>(rs, lds, c1, lane);
    __syncthreads();
    mlp_forward<M, W, SR>(rs, lds, c1, lane, wr);
    #pragma unroll 1
    for (int p = tid; p < M::PAIRS; p += NTHREADS) {
      const int r = p / TT, t = p - r * TT, n = n0 + t;
      if (n >= A.n_traj) continue;
      const float* rec = lds + t * SR;
      float Y[3], f[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) Y[c] = rec[M::Y_OFF + 3 * r + c];
      if constexpr (M::HAS_P) {
        const float b = fabsf(rec[M::act_off(0, M::nl(0) - 1) + 2 * r]);
        const float gm = fabsf(rec[M::act_off(0, M::nl(0) - 1) + 2 * r + 1]);
        const float plus = (b * Y[0]) * Y[1];
        const float minus = gm * Y[1];
        f[0] = -plus; f[1] = plus - minus; f[2] = minus;
        if (A.rates) {
          A.rates[((size_t)n * M::R + r) * 2] = b;
          A.rates[((size_t)n * M::R + r) * 2 + 1] = gm;
        }
      }
      if constexpr (M::HAS_A) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float v = rec[M::act_off(1, M::nl(1) - 1) + 3 * r + c];
          if constexpr (M::HAS_P) f[c] = f[c] + A.fa_w * v;
          else f[c] = v;
          if (A.fa) A.fa[((size_t)n * M::R + r) * 3 + c] = v;
        }
      }
      float* dst = A.f + ((size_t)n * M::R + r) * M::L;
#pragma unroll
      for (int c = 0; c < 3; ++c) dst[c] = (Y[c] > 2.f || Y[c] < -1.f) ? 0.f : f[c];
      for (int c = 3; c < M::L; ++c) dst[c] = 0.f;
    }
    __syncthreads();
  }
}

template <class M>
__global__ __launch_bounds__(NTHREADS, 2) void ude_eval_fwd_kernel(EArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w == 0) eval_fwd_body<M, 0>(a, lds);
  else if (w == 1) eval_fwd_body<M, 1>(a, lds);
  else if (w == 2) eval_fwd_body<M, 2>(a, lds);
  else eval_fwd_body<M, 3>(a, lds);
}

// ---- VJP --------------------------------------------------------------------------------
// Layer-0 input gradient epilogue: accumulates into the per-trajectory dx record (the RK_ACCY
// slot of the backward record; dynamic rows only -- static rows go through G0, HOIST).
template <class M, int SR>
struct EvalEp {
  float* rec;
  __device__ __forceinline__ void operator()(int f0, f4 dY) const {
    if (f0 >= M::F4) return;
    *reinterpret_cast<f4*>(rec + M::RK_ACCY + f0) += dY;
  }
};

// Flux backward of one evaluation: the cotangents of f (masked outside [-1, 2]), of rates
// (through |.|) and of Fa -> final-layer gradients, and the direct d f / d (S, I) part of dx.
// The tile's cotangents were staged in the record: f in RK_DK1, rates in RK_DK2 ([r][2]),
// Fa in RK_DK3 ([r][3]).
template <class M, int SR>
__device__ __forceinline__ void eval_flux_backward(float* lds, const EArgs& A, int n0) {
  constexpr int RG = (M::R + 3) / 4, ITEMS = TT * RG;
  constexpr int QO = M::HAS_P ? M::act_off(0, M::nl(0) - 1) : 0, QG = M::HAS_P ? M::gbuf(0, M::nl(0) - 1) : 0;
  constexpr int FO = M::HAS_A ? M::act_off(1, M::nl(1) - 1) : 0, FG = M::HAS_A ? M::gbuf(1, M::nl(1) - 1) : 0;
  #pragma unroll 1
  for (int it = threadIdx.x; it < ITEMS; it += NTHREADS) {
    const int t = it & (TT - 1), rg = it >> 4;
    const bool valid = n0 + t < A.n_traj;
    float* rec = lds + t * SR;
    float dyf[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) dyf[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * rg + j;
      if (r >= M::R) break;
      const bool live = valid;
      float Y[3], dres[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Y[c] = rec[M::Y_OFF + 3 * r + c];
        const float dk = rec[M::RK_DK1 + 3 * r + c];
        dres[c] = (!live || Y[c] > 2.f || Y[c] < -1.f) ? 0.f : dk;
      }
      if constexpr (M::HAS_A) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float d = M::HAS_P ? A.fa_w * dres[c] : dres[c];
          rec[FG + 3 * r + c] = live ? d + rec[M::RK_DK3 + 3 * r + c] : 0.f;
        }
      }
      if constexpr (M::HAS_P) {
        const float q0 = rec[QO + 2 * r], q1 = rec[QO + 2 * r + 1];
        const float b = fabsf(q0), gm = fabsf(q1);
        const float dplus = dres[1] - dres[0];
        const float dminus = dres[2] - dres[1];
        const float dpi = dplus * Y[1];
        float dbeta = dpi * Y[0];
        float dgam = dminus * Y[1];
        dyf[3 * j] = dpi * b;
        dyf[3 * j + 1] = dplus * (b * Y[0]) + dminus * gm;
        if (live) {
          dbeta += rec[M::RK_DK2 + 2 * r];
          dgam += rec[M::RK_DK2 + 2 * r + 1];
        } else {
          dbeta = 0.f; dgam = 0.f;
        }
        rec[QG + 2 * r] = q0 > 0.f ? dbeta : (q0 < 0.f ? -dbeta : 0.f);
        rec[QG + 2 * r + 1] = q1 > 0.f ? dgam : (q1 < 0.f ? -dgam : 0.f);
      }
    }
    // direct part of dx (the MLP part is added by the layer-0 epilogue)
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const f4 dY = {dyf[4 * v], dyf[4 * v + 1], dyf[4 * v + 2], dyf[4 * v + 3]};
      *reinterpret_cast<f4*>(rec + M::RK_ACCY + 12 * rg + 4 * v) = dY;
    }
  }
}

// Tile start of the evaluation + VJP: the evaluation point (dynamic dims -> Y slot, static dims ->
// the static-feature columns) and the three cotangents -> record.  Row-mapped (consecutive lanes,
// consecutive (n, r) rows of the tile's contiguous (16, R, L) block) with every load of the thread in
// flight before the first LDS write: one HBM round trip per tile instead of one per row pass.
template <class M, int SR>
__device__ __forceinline__ void eval_tile_load(const EArgs& A, float* lds, int n0) {
  constexpr int NROW = TT * M::R, PR = (NROW + NTHREADS - 1) / NTHREADS, LS = M::L - 3;
  const int tid = threadIdx.x;
  const int nvalid = min(TT, A.n_traj - n0) * M::R;
  float xv[PR][M::L], cf[PR][3], cfa[PR][3], cr[PR][2];
#pragma unroll
  for (int u = 0; u < PR; ++u) {
    const int i = tid + u * NTHREADS;
    const bool ok = i < nvalid;
    const size_t row = (size_t)n0 * M::R + (ok ? i : 0);
#pragma unroll
    for (int c = 0; c < M::L; ++c) xv[u][c] = ok ? A.x[row * M::L + c] : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      cf[u][c] = ok ? A.cot_f[row * M::L + c] : 0.f;
      cfa[u][c] = (ok && A.cot_fa) ? A.cot_fa[row * 3 + c] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) cr[u][c] = (ok && A.cot_rates) ? A.cot_rates[row * 2 + c] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < PR; ++u) {
    const int i = tid + u * NTHREADS;
    if (i < NROW) {
      const int t = i / M::R, r = i - t * M::R;
      float* rec = lds + t * SR;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        rec[M::Y_OFF + 3 * r + c] = xv[u][c];
        rec[M::RK_DK1 + 3 * r + c] = cf[u][c];
        rec[M::RK_DK3 + 3 * r + c] = cfa[u][c];
      }
#pragma unroll
      for (int c = 0; c < 2; ++c) rec[M::RK_DK2 + 2 * r + c] = cr[u][c];
      if constexpr (M::S > 0) {
#pragma unroll
        for (int c = 0; c < LS; ++c) rec[M::XSB_OFF + LS * r + c] = xv[u][3 + c];
      }
    }
  }
  // the static columns' padding (the activation region aliases them in the recomputed forward)
  if constexpr (M::S > 0 && M::S16 > M::S) {
    constexpr int NP = M::S16 - M::S;
    for (int i = tid; i < TT * NP; i += NTHREADS) lds[(i / NP) * SR + M::XSB_OFF + M::S + i % NP] = 0.f;
  }
}

// SPLIT (eval_split<M>): waves 0-3 run this critical path without weight-gradient accumulators
// (input gradients only, each phase's input-gradient fragments one phase ahead); waves 4-7
// (eval_wbody) accumulate dW, the bias row sums and G0 from the same LDS operands on the same
// barrier sequence -- the RK4 backward's SPLIT_BWD_L arrangement for one evaluation.
template <class M, int W, bool SPLIT>
__device__ void eval_vjp_body(const EArgs& A, float* lds) {
  constexpr int SR = M::SR_B;
  constexpr int NDWn = M::NDW(W) > 0 ? M::NDW(W) : 1;
  constexpr int NZn = M::NZ(W) > 0 ? M::NZ(W) : 1;
  constexpr bool PFX = SPLIT && M::PF_X && !WRegs<M, W, true, true>::ON;
  const int tid = threadIdx.x, lane = tid & 63;
  const int t16 = lane & 15, g = lane >> 4;
  float* myslab = A.slab + (size_t)blockIdx.x * M::SLAB_STRIDE;
  const Rsrc rs = make_rsrc(A.pack, M::PACK_TOTAL * 4);
  f4 dw[SPLIT ? 1 : NDWn], dws[1], g0t[NZn], c1[NZn];
  f4 fxp[(PFX && M::WX_Q(W) > 0) ? M::WX_Q(W) : 1];
#pragma unroll
  for (int i = 0; i < (SPLIT ? 1 : NDWn); ++i) dw[i] = f4zero();
  WRegs<M, W, true, true> wr;                      // recomputes the forward: all fragments
  wr.load(rs, lane);
  #pragma unroll 1
  for (int i = tid; i < M::LDS_B / 4; i += NTHREADS) lds[i] = 0.f;
  __syncthreads();

  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    eval_tile_load<M, SR>(A, lds, n0);
    __syncthreads();
    static_hoist<M, W, SR, M::XSB_OFF>(rs, lds, c1, lane);
#pragma unroll
    for (int i = 0; i < NZn; ++i) g0t[i] = f4zero();
    __syncthreads();
    mlp_forward<M, W, SR>(rs, lds, c1, lane, wr);
    if constexpr (PFX) load_x_frags<M, W, M::D - 1>(rs, lane, fxp + M::xq_base(W, M::D - 1));
    if (A.fout) eval_f_pairs<M, SR>(lds, A, n0, A.fout, A.f_scale);
    eval_flux_backward<M, SR>(lds, A, n0);
    // zero the padded rows of the final-layer gradient slots
    if constexpr (M::HAS_P) {
      constexpr int lo = 2 * M::R, hi = M::kout(0, M::nl(0) - 1);
      #pragma unroll 1
      for (int i = tid; i < TT * (hi - lo); i += NTHREADS) {
        const int t = i / (hi - lo), o = lo + i - t * (hi - lo);
        lds[t * SR + M::gbuf(0, M::nl(0) - 1) + o] = 0.f;
      }
    }
    if constexpr (M::HAS_A) {
      constexpr int lo = 3 * M::R, hi = M::kout(1, M::nl(1) - 1);
      #pragma unroll 1
      for (int i = tid; i < TT * (hi - lo); i += NTHREADS) {
        const int t = i / (hi - lo), o = lo + i - t * (hi - lo);
        lds[t * SR + M::gbuf(1, M::nl(1) - 1) + o] = 0.f;
      }
    }
    __syncthreads();
    mlp_backward<M, W, SR, SPLIT, PFX>(rs, rs, lds, dw, dws, g0t, lane, nullptr, EvalEp<M, SR>{lds + t16 * SR}, wr,
                                       nullptr, fxp);
    if constexpr (M::SPLITX0) {
      constexpr int NVX = cmin(M::F4, M::F16) / 4;
      #pragma unroll 1
      for (int i = tid; i < TT * NVX; i += NTHREADS) {
        const int t = i / NVX, v = i - t * NVX, f0 = 4 * v;
        const int m = f0 >> 4, li = ((f0 >> 2) & 3) * 16 + t;
        f4 s = f4zero();
#pragma unroll
        for (int w = 0; w < WAVES; ++w)
          s += *reinterpret_cast<const f4*>(lds + M::X0P_LDS + ((w * M::XT(0) + m) * 64 + li) * 4);
        EvalEp<M, SR>{lds + t * SR}(f0, s);
      }
    }
    __syncthreads();
    // dx (dynamic dims; static dims: ude_dy0_static_kernel from the G0 sums below)
    {
      const int nvalid = min(TT, A.n_traj - n0) * M::R;    // row-mapped, as the tile start
      #pragma unroll 1
      for (int i = tid; i < nvalid; i += NTHREADS) {
        const int t = i / M::R, r = i - t * M::R;
#pragma unroll
        for (int c = 0; c < 3; ++c) A.dx[((size_t)n0 * M::R + i) * M::L + c] = lds[t * SR + M::RK_ACCY + 3 * r + c];
      }
    }
    // per-trajectory layer-0 output gradients -> G0 (static-feature gradients) + bias row sums
    // (SPLIT: the partner waves')
    if constexpr (!SPLIT) g0_tile_end<M, W>(A, lds, g0t, tile, lane);
    __syncthreads();
  }

  if constexpr (SPLIT) lds_sync();                 // the partner waves' last bias row sums have landed
  else dw_to_slab<M, W>(dw, dws, myslab, lane);
  #pragma unroll 1
  for (int i = tid; i < M::NDB; i += NTHREADS) myslab[M::SLAB_DB + i] = lds[M::DB_LDS + i];
}

// eval_vjp_body's partner wave W + 4 (SPLIT): one barrier for each of the critical path's, the weight
// gradients of the backward phases (mlp_backward_dw_l, no data movement) and the tile's G0 rows.
template <class M, int W>
__device__ void eval_wbody(const EArgs& A, float* lds) {
  constexpr int SR = M::SR_B;
  constexpr int NDWn = M::NDW(W) > 0 ? M::NDW(W) : 1;
  constexpr int NZn = M::NZ(W) > 0 ? M::NZ(W) : 1;
  int lane = threadIdx.x & 63;
  float* myslab = A.slab + (size_t)blockIdx.x * M::SLAB_STRIDE;
  f4 dw[NDWn], g0t[NZn];
#pragma unroll
  for (int i = 0; i < NDWn; ++i) dw[i] = f4zero();
  __builtin_amdgcn_s_setprio(1);                  // as bwd_wbody_l
  lds_sync();                                     // record zeroed
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    asm volatile("" : "+v"(lane));                // lane-derived addresses per tile (bwd_wbody_l)
    lds_sync();                                   // evaluation point and cotangents in the record
#pragma unroll
    for (int i = 0; i < NZn; ++i) g0t[i] = f4zero();
    lds_sync();                                   // static hoist
    sfor<M::D>([&](auto) { lds_sync(); });        // the forward's layer phases
    lds_sync();                                   // flux backward: final-layer gradients written
    mlp_backward_dw_l<M, W, SR>(lds, dw, g0t, lane, [](auto) {});
    lds_sync();                                   // layer-0 input-gradient epilogue
    g0_tile_end<M, W>(A, lds, g0t, tile, lane);
    lds_sync();                                   // dx written
  }
  f4 none[1];
  dw_to_slab<M, W>(dw, none, myslab, lane);
  lds_sync();                                     // bias row sums complete -> eval_vjp_body copies them
}

// the split evaluation + VJP where the RK4 backward is split the same way (large records)
template <class M>
constexpr bool eval_split() { return M::SPLIT_BWD_L; }
template <class M>
constexpr int eval_vjp_threads() { return eval_split<M>() ? 2 * NTHREADS : NTHREADS; }

template <class M>
__global__ __launch_bounds__(eval_vjp_threads<M>()) void ude_eval_vjp_kernel(EArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // the workspace's ticket words start at zero for ude_bwd_tail_kernel (same stream, next launch)
  if (blockIdx.x == 0 && (int)threadIdx.x < a.n_ctl) a.ctl[threadIdx.x] = 0u;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr bool SPLIT = eval_split<M>();
  if constexpr (SPLIT) {
    if (w >= WAVES) {
      if (w == 4) eval_wbody<M, 0>(a, lds);
      else if (w == 5) eval_wbody<M, 1>(a, lds);
      else if (w == 6) eval_wbody<M, 2>(a, lds);
      else eval_wbody<M, 3>(a, lds);
      return;
    }
  }
  if (w == 0) eval_vjp_body<M, 0, SPLIT>(a, lds);
  else if (w == 1) eval_vjp_body<M, 1, SPLIT>(a, lds);
  else if (w == 2) eval_vjp_body<M, 2, SPLIT>(a, lds);
  else eval_vjp_body<M, 3, SPLIT>(a, lds);
}

}  // namespace ude
