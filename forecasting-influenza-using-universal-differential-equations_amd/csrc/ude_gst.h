// Weight gradients of the large Bayesian RHS (Model::GST: R >= 10 Bayes_Fp / Bayes_Fa / Bayes_FaFp,
// lib/in_development/models_bayes.py:69-265).
//
// Every RHS evaluation e draws its own weight sample w_e = mean + eps_e * |std| (Dense_Variational
// .forward, models_bayes.py:43-48), so the reference's gradients are
//   d mean = sum_e dW_e,   d |std| = sum_e eps_e * dW_e,   dW_e = sum_traj G_e^T X_e (per layer),
// with G_e the layer-output gradients and X_e the layer inputs of evaluation e.  Two register sets
// of dW accumulators (plain and eps-weighted) fit the R = 1 models only; for the rest the training
// forward stores X (the stage input in front of every stage's activation rows, Model::XST_W), the
// backward stores G (mlp_backward's GST rows, [tile][step][stage][16][ACT_A4]) and this kernel forms
// each evaluation's dW_e as one MFMA GEMM with K = the whole batch of trajectories:
//
//  * workgroup (ks, e): evaluation e over the ks-th contiguous chunk of tiles, 8 waves; every dW tile
//    of the evaluation belongs to one wave (whole row tiles, balanced greedily over the waves) and is
//    accumulated in registers over the chunk, then written once to the partial slab [e][ks] (the
//    backward slab layout: dW tiles in MFMA C order, then the bias rows = trajectory sums of G);
//  * half-tiles of 8 trajectories are triple-buffered in LDS ([t][Y | static | activations | G] rows,
//    the backward record's column order, row stride = 4 mod 64): the next two half-tiles' rows arrive
//    by LDS-DMA (buffer loads with the LDS destination, no data registers; the static features from
//    the per-tile block the training forward wrote) while the waves multiply the current one
//    (v_mfma_f32_16x16x4_f32, MFMA step s over trajectories 4 s + lane group);
//  * ude_gst_reduce_kernel sums the chunks in fixed order per evaluation, weights each evaluation's
//    sum by its eps (slab order, ude_eps_slab_kernel) and scatters d mean / d |std| to torch order.
// Bandwidth-balanced at R = 49: ~98 KB of rows per 16 trajectories and evaluation against 1208
// MFMAs (4 per dW tile).
#pragma once
#include "ude_kernels.h"

namespace ude {

template <class M>
struct Gst {
  static constexpr int NW = 8, NT = NW * 64;
  static constexpr int GOFF = M::ACT0 + M::ACT_A4;          // output-gradient rows in the record
  static constexpr int SRG = M::stride(GOFF + M::ACT_A4);
  static constexpr int HT = 8;                               // trajectories per half-tile
  static constexpr int BUF = HT * SRG;                       // floats per LDS buffer
  // three buffers when they fit (two half-tiles in flight while one is multiplied), else two
  static constexpr int NBUF = 3 * BUF * 4 <= 160 * 1024 ? 3 : 2;
  static constexpr int LDS = NBUF * BUF * 4;
  static_assert(LDS <= 160 * 1024, "GST half-tile buffers do not fit the 160 KiB LDS");
  // row tiles r = FTbase(d) + k of every layer, in slab order
  static constexpr int NRT = M::FTbase(M::D);
  static constexpr int rt_d(int r) {
    int d = 0;
    while (d + 1 < M::D && M::FTbase(d + 1) <= r) ++d;
    return d;
  }
  static constexpr int rt_k(int r) { return r - M::FTbase(rt_d(r)); }
  static constexpr int width(int r) { return M::rti(M::fnet(rt_d(r), rt_k(r)), rt_d(r)); }
  // greedy balance: each row tile (layer 0 first, the widest) to the least loaded wave; tabulated
  // once with the per-wave accumulator / bias-row offsets
  struct Tab {
    int own[64], acc[64], row[64], nacc[NW], nrow[NW];
  };
  static constexpr Tab make_tab() {
    Tab T{};
    int load[NW] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int q = 0; q < NRT; ++q) {
      int best = 0;
      for (int w = 1; w < NW; ++w)
        if (load[w] < load[best]) best = w;
      load[best] += width(q);
      T.own[q] = best;
      T.acc[q] = T.nacc[best];
      T.row[q] = T.nrow[best];
      T.nacc[best] += width(q);
      T.nrow[best] += 1;
    }
    return T;
  }
  static constexpr Tab TAB = make_tab();
  static_assert(NRT <= 64, "too many row tiles");
  static constexpr int owner(int r) { return TAB.own[r]; }
  static constexpr int acc_before(int, int r) { return TAB.acc[r]; }
  static constexpr int rows_before(int, int r) { return TAB.row[r]; }
  static constexpr int NACC(int w) { return TAB.nacc[w]; }
  static constexpr int NROW(int w) { return TAB.nrow[w]; }
  // LDS-DMA jobs of one half-tile: per row, the stage input (F16 floats), the static features (S16,
  // the tile's block the training forward wrote), the activation rows and the output-gradient rows
  // (ACT_A4 each), up to 256 floats (64 lanes x 16 B) per job
  static constexpr int NJY = (M::F16 + 255) / 256, NJS = (M::S16 + 255) / 256, NJA = (M::ACT_A4 + 255) / 256;
  static constexpr int NJR = NJY + NJS + 2 * NJA;
  static constexpr int NJ = HT * NJR;
  // LDS-DMA instructions wave w issues per half-tile
  static constexpr int ndma(int w) {
    int s = 0;
    for (int j = 0; j < NJ; ++j)
      if (j % NW == w) s += 1;
    return s;
  }
};

// s_waitcnt vmcnt(n) (expcnt / lgkmcnt untouched)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt out of range");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
  __builtin_amdgcn_sched_barrier(0);
}

struct GstArgs {
  const float* ckpt;     // training store (stage inputs + [16][XST_W] stored rows)
  const float* gst;      // [tile][step][stage][16][ACT_A4] layer-output gradient rows
  const float* y0;
  float* part;           // [eval][ks][SLAB_TOTAL] partial slabs
  int n_traj, n_steps, n_tiles, n_ks;
};

template <class M, int W>
__device__ void gst_body(const GstArgs& A, float* lds) {
  using P = Gst<M>;
  constexpr int SRG = P::SRG, HT = P::HT;
  constexpr int NA = P::NACC(W) > 0 ? P::NACC(W) : 1, NB = P::NROW(W) > 0 ? P::NROW(W) : 1;
  const int tid = threadIdx.x, lane = tid & 63, t = lane & 15, g = lane >> 4;
  const int e = blockIdx.y, ks = blockIdx.x;
  const int step = e >> 2, jj = e & 3;
  const int tb = (int)(((long)A.n_tiles * ks) / A.n_ks), te = (int)(((long)A.n_tiles * (ks + 1)) / A.n_ks);
  const int hb = 2 * tb, he = 2 * te;

  f4 acc[NA];
  float bacc[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = f4zero();
#pragma unroll
  for (int i = 0; i < NB; ++i) bacc[i] = 0.f;

  // the buffers zeroed once: the static pads [F16 + S, F16 + S16) are never written
  #pragma unroll 1
  for (int i = tid; i < P::NBUF * P::BUF; i += P::NT) lds[i] = 0.f;
  lds_sync();
  auto bufp = [&](int h) { return lds + (h % P::NBUF) * P::BUF; };

  auto issue = [&](int h) {                     // LDS-DMA of half-tile h's rows into its buffer
    const int tile = h >> 1, r0 = (h & 1) * HT;
    float* buf = bufp(h);
    const Rsrc xs = make_rsrc(act_block<M>(const_cast<float*>(A.ckpt), A.n_tiles, A.n_steps, tile, step, jj),
                              TT * M::XST_W * 4);
    const Rsrc gs = make_rsrc(A.gst + (((size_t)tile * A.n_steps + step) * 4 + jj) * TT * M::ACT_A4,
                              TT * M::ACT_A4 * 4);
    const Rsrc ss = make_rsrc(A.ckpt + gst_static_off<M>(A.n_tiles, A.n_steps) + (size_t)tile * TT * M::S16,
                              TT * M::S16 * 4);
    sfor<P::NJ>([&](auto jb) {
      constexpr int j = decltype(jb)::value;
      if constexpr (j % P::NW == W) {
        constexpr int row = j / P::NJR, sj = j % P::NJR;
        // kind: 0 stage input, 1 static features, 2 activation rows, 3 output-gradient rows
        constexpr int kind = sj < P::NJY ? 0 : sj < P::NJY + P::NJS ? 1 : sj < P::NJY + P::NJS + P::NJA ? 2 : 3;
        constexpr int c = kind == 0 ? sj : kind == 1 ? sj - P::NJY : kind == 2 ? sj - P::NJY - P::NJS
                                                                                : sj - P::NJY - P::NJS - P::NJA;
        constexpr int segw = kind == 0 ? M::F16 : kind == 1 ? M::S16 : M::ACT_A4;
        constexpr int nq = cmin(64, (segw - 256 * c) / 4);                        // quads of this job
        constexpr int dst = (kind == 0 ? 0 : kind == 1 ? M::F16 : kind == 2 ? M::ACT0 : P::GOFF) + 256 * c;
        constexpr int src = (kind == 2 ? M::ACT_IN : 0) + 256 * c;
        constexpr int rs = kind <= 2 ? (kind == 1 ? M::S16 : M::XST_W) : M::ACT_A4;
#if defined(__HIP_DEVICE_COMPILE__)
        if (lane < nq)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(kind == 0 || kind == 2 ? xs : kind == 1 ? ss : gs,
                                                   (LdsPtr)(buf + row * SRG + dst), 16, 16 * lane,
                                                   ((r0 + row) * rs + src) * 4, 0, 0);
#endif
      }
    });
  };

  // pipeline: NBUF - 1 half-tiles in flight; the only vector-memory operations of the loop are the
  // DMAs, so the wait for the next half-tile at an iteration's end leaves the newest one in flight
  // (vmcnt(ndma)).
  constexpr int AHEAD = P::NBUF - 1;
  #pragma unroll 1
  for (int h = hb; h < hb + AHEAD && h < he; ++h) issue(h);
  wait_dma();
  lds_sync();
  #pragma unroll 1
  for (int h = hb; h < he; ++h) {
    const bool more = h + AHEAD < he;
    if (more) issue(h + AHEAD);
    const float* buf = bufp(h);
    sfor<P::NRT>([&](auto rr) {
      constexpr int r = decltype(rr)::value;
      if constexpr (P::owner(r) == W) {
        constexpr int d = P::rt_d(r), k = P::rt_k(r), net = M::fnet(d, k), rt = M::frt(d, k);
        constexpr int NC = M::rti(net, d);
        constexpr int goff = P::GOFF + (M::act_off(net, d) - M::ACT0) + rt * 16;
        constexpr int inoff = d == 0 ? 0 : M::act_off(net, d - 1);
        constexpr int a0 = P::acc_before(W, r), bi = P::rows_before(W, r);
        float ga[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) ga[s] = buf[(4 * s + g) * SRG + goff + t];
        bacc[bi] += ga[0] + ga[1];
        constexpr int XC = 8;
        sfor<(NC + XC - 1) / XC>([&](auto cc0) {
          constexpr int c0 = decltype(cc0)::value * XC, NCC = cmin(XC, NC - c0);
          float bv[2][NCC];
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ct = 0; ct < NCC; ++ct) bv[s][ct] = buf[(4 * s + g) * SRG + inoff + (c0 + ct) * 16 + t];
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int ct = 0; ct < NCC; ++ct) acc[a0 + c0 + ct] = mfma4(ga[s], bv[s][ct], acc[a0 + c0 + ct]);
        });
      }
    });
    if (AHEAD > 1 && more) wait_vm<P::ndma(W)>();   // half-tile h + 1 has landed, h + AHEAD may not have
    else wait_dma();
    lds_sync();
  }

  // partial slab of (e, ks): dW tiles (MFMA C order) and the bias rows (trajectory sums of G)
  float* slab = A.part + ((size_t)e * A.n_ks + ks) * M::SLAB_TOTAL;
  sfor<P::NRT>([&](auto rr) {
    constexpr int r = decltype(rr)::value;
    if constexpr (P::owner(r) == W) {
      constexpr int d = P::rt_d(r), k = P::rt_k(r), net = M::fnet(d, k);
      constexpr int a0 = P::acc_before(W, r), bi = P::rows_before(W, r);
      sfor<M::rti(net, d)>([&](auto cc) {
        constexpr int ct = decltype(cc)::value;
        reinterpret_cast<f4*>(slab + (M::dyn_tiles_before(d, k) + ct) * 256)[lane] = acc[a0 + ct];
      });
      float b = bacc[bi];
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if (g == 0) slab[M::SLAB_DB + r * 16 + t] = b;
    }
  });
}

template <class M>
__global__ __launch_bounds__(Gst<M>::NT) void ude_gst_dw_kernel(GstArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w == 0) gst_body<M, 0>(a, lds);
  else if (w == 1) gst_body<M, 1>(a, lds);
  else if (w == 2) gst_body<M, 2>(a, lds);
  else if (w == 3) gst_body<M, 3>(a, lds);
  else if (w == 4) gst_body<M, 4>(a, lds);
  else if (w == 5) gst_body<M, 5>(a, lds);
  else if (w == 6) gst_body<M, 6>(a, lds);
  else gst_body<M, 7>(a, lds);
}

// d mean[p] = sum_e sum_ks part[e][ks][off],  d |std|[p] = sum_e eps_e[off] * sum_ks part[e][ks][off]
// (p = slab_to_param(off)).  A block owns 64 consecutive slab offsets x 4 groups of evaluations, each
// summed in order, combined in a fixed order: deterministic.
template <class M>
__global__ __launch_bounds__(256) void ude_gst_reduce_kernel(const float* __restrict__ part,
                                                             const float* __restrict__ eslab, int n_ev, int n_ks,
                                                             float* __restrict__ dparams) {
  __shared__ float pm[4][64], ps[4][64];
  const int lo = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int off = blockIdx.x * 64 + lo;
  float sm = 0.f, ss = 0.f;
  if (off < M::SLAB_TOTAL) {
    const int per = (n_ev + 3) / 4, e0 = grp * per, e1 = min(n_ev, e0 + per);
    for (int e = e0; e < e1; ++e) {
      const float* p = part + (size_t)e * n_ks * M::SLAB_TOTAL + off;
      float v = 0.f;
#pragma unroll 8
      for (int k = 0; k < n_ks; ++k) v += p[(size_t)k * M::SLAB_TOTAL];
      sm += v;
      ss += eslab[(size_t)e * M::SLAB_TOTAL + off] * v;
    }
  }
  pm[grp][lo] = sm;
  ps[grp][lo] = ss;
  __syncthreads();
  if (grp == 0 && off < M::SLAB_TOTAL) {
    const int p = slab_to_param<M>(off);
    if (p >= 0) {
      dparams[p] = (pm[0][lo] + pm[1][lo]) + (pm[2][lo] + pm[3][lo]);
      dparams[M::N_PARAMS + p] = (ps[0][lo] + ps[1][lo]) + (ps[2][lo] + ps[3][lo]);
    }
  }
}

}  // namespace ude
