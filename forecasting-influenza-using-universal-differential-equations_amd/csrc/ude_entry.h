// Host-side launch logic for one compiled model configuration (Ops<M>) and
// the type-erased registry entry the C-ABI (ude_rk4.hip) dispatches on.
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include "ude_rk4.h"
#include "ude_kernels.h"
#include "ude_dopri5.h"
#include "ude_loss.h"
#include "ude_eval.h"
#include "ude_gst.h"

namespace ude {

#ifdef UDE_PROFILE
extern unsigned long long* g_prof_buffer;   // diagnostic builds: set by ude_debug_set_prof()
#endif

template <class M>
bool matches(const UdeModelDesc* d) {
  if (!M::FITS) return false;
  if (d->kind != M::KIND || d->n_regions != M::R || d->latent_dim != M::L) return false;
  if (M::HAS_P) {
    if (d->n_p_hidden != M::NPH) return false;
    for (int i = 0; i < M::NPH; ++i) if (d->p_hidden[i] != M::hid(0, i)) return false;
  }
  if (M::HAS_A) {
    if (d->n_a_hidden != M::NAH) return false;
    for (int i = 0; i < M::NAH; ++i) if (d->a_hidden[i] != M::hid(1, i)) return false;
  }
  return true;
}

#define HIPCHK(x) do { if ((x) != hipSuccess) return UDE_E_HIP; } while (0)

template <class M>
struct Ops {
  static constexpr int DY0_STATIC_LDS = TT * M::R * M::L * 4;
  static constexpr int LDS_MAX = 160 * 1024;
  static int64_t sched_bytes(const UdeProblem* p) {
    return (int64_t)p->n_steps * 4 + (int64_t)(p->n_steps + 1) * 4 + (int64_t)p->n_out * 12;
  }
  static_assert(!M::HOIST || DY0_STATIC_LDS <= 160 * 1024, "dy0 static time sums do not fit the 160 KiB LDS");
  static int ensure_attrs() {
    static bool done = false;
    if (done) return UDE_OK;
    // record + (when it fits) the schedule: up to the full 160 KiB
    HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true, M::SPLIT_FWD>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_bwd_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true, false, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true, M::SPLIT_FWD, true>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_dec_bwd_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               DecBwdDims<M>::LDS));
    // the static-feature dy0 kernel stages one tile's (16, R, L) time sums of d latent in LDS
    if (M::HOIST)
      HIPCHK(hipFuncSetAttribute((const void*)&ude_dy0_static_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 DY0_STATIC_LDS));
    if constexpr (M::GST)
      HIPCHK(hipFuncSetAttribute((const void*)&ude_gst_dw_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 Gst<M>::LDS));
    HIPCHK(hipFuncSetAttribute((const void*)&ude_bwd_tail_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               Tail<M>::LDS));
    if constexpr (M::FWD_RES) {
      HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true, false, false, true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, false, false, false, true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_fwd_kernel<M, true, false, true, true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX));
    }
    done = true;
    return UDE_OK;
  }

  static int grids(int device, int n_tiles, int* gf, int* gb) {
    int rc = ensure_attrs();
    if (rc) return rc;
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    int of = 0, ob = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&of, (const void*)&ude_fwd_kernel<M, true>, NTHREADS, M::LDS_F));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&ob, (const void*)&ude_bwd_kernel<M>, M::BWD_THREADS, M::LDS_B));
    if (of < 1) of = 1;
    if (ob < 1) ob = 1;
    const long mf = (long)cus * of, mb = (long)cus * ob;
    *gf = (int)(n_tiles < mf ? n_tiles : mf);
    *gb = (int)(n_tiles < mb ? n_tiles : mb);
    if (*gf < 1) *gf = 1;
    if (*gb < 1) *gb = 1;
    return UDE_OK;
  }

  // grad-slab workspace tail (HOIST): G0 [tile][K0][16] + split-K partials [chunks][K0][S16]
  static int64_t static_ws_floats(int n_tiles) {
    if (!M::HOIST) return 0;
    const int64_t legacy = (int64_t)M::STATIC_CHUNKS * M::K0 * M::S16, tail = Tail<M>::part_floats();
    return (int64_t)n_tiles * M::K0 * TT + (legacy > tail ? legacy : tail);
  }
  // control words of the *_ex calls: [0] the forward's arrival counter, [1 + st] the tail's static
  // column tiles (include/ude_rk4.h)
  static constexpr int64_t CTL_WORDS = 1 + Tail<M>::NST;

  // the resident-weight forward (one workgroup per CU) when every tile has a CU of its own;
  // UDE_FWD_RES=0 turns it off, =2 forces it at any batch (A/B measurement)
  static bool fwd_res(int n_tiles, int cus) {
    if constexpr (!M::FWD_RES) return false;
    static const int env = [] { const char* e = getenv("UDE_FWD_RES"); return e ? atoi(e) : 1; }();
    return env == 2 || (env != 0 && n_tiles <= cus);
  }

  // BAYES: one weight sample per RHS evaluation (4 per RK4 step)
  static int64_t n_evals(const UdeProblem* p) { return M::BAYES ? 4 * (int64_t)p->n_steps : 1; }

  // GST weight-gradient GEMM: tile chunks per evaluation (at least one workgroup per CU over the
  // evaluations) and the backward workspace [G rows | partial slabs [eval][ks][SLAB_TOTAL]]
  static int gst_ks(int cus, int64_t ne, int n_tiles) {
    int64_t ks = ne > 0 ? (cus + ne - 1) / ne : 1;
    if (ks > n_tiles) ks = n_tiles;
    return ks < 1 ? 1 : (int)ks;
  }
  static int64_t gst_rows_floats(int n_tiles, int n_steps) { return (int64_t)n_tiles * n_steps * 4 * TT * M::ACT_A4; }

  // FULL0: the output cotangents of the static latent dims, summed over the output times into dy0
  static hipError_t static_tsum(const UdeProblem* p, const float* dlatent, float* dy0, hipStream_t s) {
    if constexpr (M::FULL0) {
      if (dlatent) {
        if constexpr (M::L == 8) {
          if (((reinterpret_cast<uintptr_t>(dlatent) | reinterpret_cast<uintptr_t>(dy0)) & 15) == 0) {
            const long rows = (long)p->n_traj * M::R;
            long blocks = (rows + 255) / 256;
            if (blocks > 8192) blocks = 8192;
            if (blocks < 1) blocks = 1;
            hipLaunchKernelGGL((ude_static_tsum_rows_kernel<M>), dim3((unsigned)blocks), dim3(256), 0, s, dlatent,
                               p->n_traj, p->n_out + 1, dy0);
            return hipGetLastError();
          }
        }
        const long total = (long)p->n_traj * M::R * (M::L - 3);
        long blocks = (total + 255) / 256;
        if (blocks > 4096) blocks = 4096;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL((ude_static_tsum_kernel<M>), dim3((unsigned)blocks), dim3(256), 0, s, dlatent, p->n_traj,
                           p->n_out + 1, dy0);
        return hipGetLastError();
      }
    }
    return hipSuccess;
  }

  // UdeProblem.recompute: the Recompute<M> view of the model (no stored activations; GST needs them)
  static constexpr bool RC_VIEW = M::ACT_STORED && !M::GST;
  static bool rc(const UdeProblem* p) { return RC_VIEW && p->recompute; }

  static int query(const UdeProblem* p, int device, UdeSizes* o) {
    if constexpr (RC_VIEW) {
      if (p->recompute) return Ops<Recompute<M>>::query(p, device, o);
    }
    if (p->n_traj < 1 || p->n_steps < 0 || p->n_out < 0) return UDE_E_INVALID;
    if (M::BAYES && 4 * (int64_t)p->n_steps > 65535) return UDE_E_INVALID;   // grid.y / grid.z of the packers
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(device, n_tiles, &gf, &gb);
    if (rc) return rc;
    const int64_t ne = n_evals(p) > 0 ? n_evals(p) : 1;
    // BAYES: [eval][PACK_TOTAL] weight samples, then [eval][SLAB_TOTAL] eps in slab order
    o->pack_bytes = M::BAYES ? ne * (int64_t)(M::PACK_TOTAL + M::SLAB_TOTAL) * 4 : (int64_t)M::PACK_TOTAL * 4;
    o->sched_bytes = sched_bytes(p);
    // stage inputs [tile][step][stage][F][16] (+ STORE_ACT / STORE_ACT_D: activations [tile][step][stage][16][ACT_A4])
    o->ckpt_bytes = (int64_t)n_tiles * p->n_steps * 4 * (M::F * TT + (M::ACT_STORED ? TT * M::XST_W : 0)) * 4;
    // GST: + the tiles' static features [tile][16][S16] (the weight-gradient GEMM's layer-0 input)
    if (M::GST) o->ckpt_bytes += (int64_t)n_tiles * TT * M::S16 * 4;
    o->stats_slab_bytes = (int64_t)gf * 5 * 8;
    o->grad_slab_bytes = (int64_t)gb * M::SLAB_STRIDE * 4 + static_ws_floats(n_tiles) * 4;
    if constexpr (M::GST) {
      int cus = 0;
      HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
      o->grad_slab_bytes = (gst_rows_floats(n_tiles, p->n_steps) +
                            n_evals(p) * gst_ks(cus, n_evals(p), n_tiles) * (int64_t)M::SLAB_TOTAL) * 4;
    }
    o->n_params = M::N_GRAD;
    o->grid_fwd = gf;
    o->grid_bwd = gb;
    o->lds_fwd = M::LDS_F;
    o->lds_bwd = M::LDS_B;
    // decoder epilogue (ude_rk4_forward_dec / ude_decoder_backward)
    int gd = 1;
    rc = dec_grid(device, n_tiles, &gd);
    if (rc) return rc;
    o->dec_pack_bytes = (int64_t)M::DEC_PACK * 4;
    o->ckpt_final_bytes = (int64_t)n_tiles * M::F * TT * 4;
    o->dec_ws_bytes = (int64_t)gd * LossDims<M::R>::SLAB * 4;
    o->act_bytes = M::ACT_STORED ? (int64_t)n_tiles * p->n_steps * 4 * TT * M::XST_W * 4 : 0;
    o->ctl_bytes = ((CTL_WORDS * 4 + 63) / 64) * 64;
    return UDE_OK;
  }

  static int dec_grid(int device, int n_tiles, int* g) {
    int rc = ensure_attrs();
    if (rc) return rc;
    int cus = 0, occ = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&ude_dec_bwd_kernel<M>, NTHREADS,
                                                        DecBwdDims<M>::LDS));
    if (occ < 1) occ = 1;
    const long mx = (long)cus * occ;
    *g = (int)(n_tiles < mx ? n_tiles : mx);
    if (*g < 1) *g = 1;
    return UDE_OK;
  }

  static int dec_pack(const float* W, const float* b, float* out, hipStream_t s) {
    if (!W || !b || !out) return UDE_E_INVALID;
    hipLaunchKernelGGL(ude_dec_pack_kernel<M>, dim3((M::DEC_PACK + 255) / 256), dim3(256), 0, s, W, b, out);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }

  // Training forward with the decoder epilogue: y_hat (T, N, R) and latent_init_loss instead of the
  // latent; ckpt (ckpt_bytes + ckpt_final_bytes) also receives the final state.
  // stats: mean / std / fa_norm outputs (sums nullable); ctl: null = the separate finalize launches
  static int forward_dec(const UdeProblem* p, const float* pack, const void* sched, const float* y0,
                         const float* dec_pack, float* yhat, float* ckpt, double* stats_slab, double* reg_slab,
                         const UdeSideStats* st, unsigned* ctl, float* reg_out, hipStream_t s) {
    if constexpr (RC_VIEW) {
      if (p->recompute)
        return Ops<Recompute<M>>::forward_dec(p, pack, sched, y0, dec_pack, yhat, ckpt, stats_slab, reg_slab,
                                              st, ctl, reg_out, s);
    }
    if (!pack || !sched || !y0 || !dec_pack || !yhat || !ckpt || !stats_slab || !reg_slab || !reg_out ||
        !stats_ok(st))
      return UDE_E_INVALID;
    if (p->n_steps < 1) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(dev, n_tiles, &gf, &gb);
    if (rc) return rc;
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.y0 = y0; a.sched = (const unsigned char*)sched;
    a.ckpt = ckpt; a.stats_slab = stats_slab;
    a.dec_pack = dec_pack; a.yhat = yhat; a.reg_slab = reg_slab;
    a.ckpt_final = ckpt + ckpt_final_off<M>(n_tiles, p->n_steps);
    a.n_traj = p->n_traj; a.n_steps = p->n_steps; a.n_out = p->n_out; a.n_tiles = n_tiles;
    a.fa_w = p->fa_w;
    const double n_eval = 4.0 * (double)p->n_steps * (double)p->n_traj * (double)M::R;
    set_stats_out(a, st, ctl, n_eval);
    a.o_reg = reg_out;
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // the resident-weight forward runs one workgroup per CU (min(n_tiles, cus) <= gf slabs)
    const bool res = !(M::SPLIT_FWD && n_tiles <= cus) && fwd_res(n_tiles, cus);
    if (res) gf = n_tiles < cus ? n_tiles : cus;
    if (M::SPLIT_FWD && n_tiles <= cus)
      hipLaunchKernelGGL((ude_fwd_kernel<M, true, M::SPLIT_FWD, true>), dim3(gf), dim3(2 * NTHREADS), M::LDS_F_DEC, s, a);
    else if (res)
      hipLaunchKernelGGL((ude_fwd_kernel<M, true, false, true, M::FWD_RES>), dim3(gf), dim3(NTHREADS), M::LDS_F_DEC, s, a);
    else hipLaunchKernelGGL((ude_fwd_kernel<M, true, false, true>), dim3(gf), dim3(NTHREADS), M::LDS_F_DEC, s, a);
    HIPCHK(hipGetLastError());
    if (!ctl) {
      hipLaunchKernelGGL(ude_stats_finalize_kernel<0>, dim3(1), dim3(320), 0, s, stats_slab, gf, n_eval, a.o_mean,
                         a.o_std, a.o_norm);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL(ude_sum_finalize_kernel<0>, dim3(1), dim3(64), 0, s, (const double*)reg_slab, gf, reg_out);
      HIPCHK(hipGetLastError());
    }
    return UDE_OK;
  }

  // Backward of the decoder epilogue: dl3 (T, N, R, 3) for ude_rk4_backward_sir, d W_dec, d b_dec.
  static int dec_backward(const UdeProblem* p, const void* sched, const float* ckpt, const float* dyhat,
                          const float* W, const float* grad_reg, void* ws, float* dl3, float* dW, float* db,
                          hipStream_t s) {
    if constexpr (RC_VIEW) {
      if (p->recompute) return Ops<Recompute<M>>::dec_backward(p, sched, ckpt, dyhat, W, grad_reg, ws, dl3, dW, db, s);
    }
    if (!sched || !ckpt || !dyhat || !W || !grad_reg || !ws || !dl3 || !dW || !db) return UDE_E_INVALID;
    if (p->n_steps < 1 || p->n_out + 1 > DecBwdDims<M>::MAX_T) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gd = 1;
    int rc = dec_grid(dev, n_tiles, &gd);
    if (rc) return rc;
    DecBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.sched = (const unsigned char*)sched; a.ckpt = ckpt; a.dyhat = dyhat; a.W = W; a.grad_reg = grad_reg;
    a.dl3 = dl3; a.slab = (float*)ws;
    a.n_traj = p->n_traj; a.n_steps = p->n_steps; a.n_out = p->n_out; a.n_tiles = n_tiles;
    hipLaunchKernelGGL((ude_dec_bwd_kernel<M>), dim3(gd), dim3(NTHREADS), DecBwdDims<M>::LDS, s, a);
    HIPCHK(hipGetLastError());
    using D = LossDims<M::R>;
    hipLaunchKernelGGL((ude_loss_grad_finalize_kernel<D>), dim3((D::SLAB + 63) / 64), dim3(256), 0, s,
                       (const float*)ws, gd, dW, db);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }

  // nll_loss over y_hat: ws = musd (T, B, R, 2) floats | per-block fp64 partials
  static int64_t nll_blocks(int T, int B) { return ((int64_t)T * B * M::R + 255) / 256; }
  static int64_t nll_part_off(int T, int B) { return (((int64_t)T * B * M::R * 2 * 4) + 255) & ~(int64_t)255; }
  static int nll_workspace(int T, int S, int B, int64_t* bytes) {
    if (T < 1 || S < 2 || B < 1) return UDE_E_INVALID;
    *bytes = nll_part_off(T, B) + nll_blocks(T, B) * 8;
    return UDE_OK;
  }
  static int nll_forward(int T, int S, int B, const float* yhat, const float* y, void* ws, float* out, hipStream_t s) {
    if (!yhat || !y || !ws || !out || T < 1 || S < 2 || B < 1) return UDE_E_INVALID;
    const int nb = (int)nll_blocks(T, B);
    float* musd = (float*)ws;
    double* part = (double*)((unsigned char*)ws + nll_part_off(T, B));
    hipLaunchKernelGGL(ude_nll_fwd_kernel<0>, dim3(nb), dim3(256), 0, s, yhat, y, T, S, B, M::R, musd, part);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(ude_nll_finalize_kernel<0>, dim3(1), dim3(64), 0, s, (const double*)part, nb,
                       (double)B * T * M::R, out);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }
  static int nll_backward(int T, int S, int B, const float* yhat, const float* y, const float* grad, const void* ws,
                          float* dyhat, hipStream_t s) {
    if (!yhat || !y || !grad || !ws || !dyhat || T < 1 || S < 2 || B < 1) return UDE_E_INVALID;
    hipLaunchKernelGGL(ude_nll_bwd_kernel<0>, dim3((int)nll_blocks(T, B)), dim3(256), 0, s, yhat, y,
                       (const float*)ws, grad, T, S, B, M::R, dyhat);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }

  static int launch_pack(const PackPtrs& P, float* out, int n_ev, hipStream_t s) {
    int mx = M::W0SP_SIZE;
    for (int net = 0; net < 2; ++net) {
      if (M::wsf_size(net) > mx) mx = M::wsf_size(net);
      for (int i = 0; i < M::nl(net); ++i) {
        if (M::wf_size(net, i) > mx) mx = M::wf_size(net, i);
        if (M::wt_size(net, i) > mx) mx = M::wt_size(net, i);
        if (M::b_size(net, i) > mx) mx = M::b_size(net, i);
      }
    }
    dim3 grid((mx + 255) / 256, 33, n_ev);
    hipLaunchKernelGGL(ude_pack_kernel<M>, grid, dim3(256), 0, s, P, out);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }

  static int pack(const float* const* W, const float* const* b, float* out, hipStream_t s) {
    if (M::BAYES) return UDE_E_INVALID;          // ude_pack_weights_bayes
    PackPtrs P;
    memset(&P, 0, sizeof(P));
    int li = 0;
    for (int net = 0; net < 2; ++net)
      for (int i = 0; i < M::nl(net); ++i, ++li) {
        if (!W[li] || !b[li]) return UDE_E_INVALID;
        P.W[net][i] = W[li];
        P.b[net][i] = b[li];
      }
    return launch_pack(P, out, 1, s);
  }

  static int pack_bayes(const UdeProblem* p, const float* const* W, const float* const* b, const float* const* Ws,
                        const float* const* bs, const float* eps, float* out, hipStream_t s) {
    if (!M::BAYES) return UDE_E_INVALID;         // ude_pack_weights
    if (!eps || p->n_steps < 0 || 4 * (int64_t)p->n_steps > 65535) return UDE_E_INVALID;
    const int ne = (int)n_evals(p);
    if (ne == 0) return UDE_OK;                  // no evaluation, nothing to pack
    PackPtrs P;
    memset(&P, 0, sizeof(P));
    int li = 0;
    for (int net = 0; net < 2; ++net)
      for (int i = 0; i < M::nl(net); ++i, ++li) {
        if (!W[li] || !b[li] || !Ws[li] || !bs[li]) return UDE_E_INVALID;
        P.W[net][i] = W[li];
        P.b[net][i] = b[li];
        P.Ws[net][i] = Ws[li];
        P.bs[net][i] = bs[li];
      }
    P.eps = eps;
    int rc = launch_pack(P, out, ne, s);
    if (rc) return rc;
    float* eslab = out + (size_t)ne * M::PACK_TOTAL;
    hipLaunchKernelGGL(ude_eps_slab_kernel<M>, dim3((M::SLAB_TOTAL + 255) / 256, ne), dim3(256), 0, s, eps, eslab);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }

  // every statistic of the model's nets needs a buffer (an absent net's may be null)
  static bool stats_ok(const UdeSideStats* st) {
    return st && (!M::HAS_P || (st->mean && st->std)) && (!M::HAS_A || st->fa_norm);
  }
  static void set_stats_out(KArgs& a, const UdeSideStats* st, unsigned* ctl, double n_eval) {
    a.o_mean = st->mean;                  // an absent net's buffers may be null: not written
    a.o_std = st->std;
    a.o_norm = st->fa_norm;
    a.o_sums = st->sums;
    a.ctl = ctl;
    a.n_eval = n_eval;
  }

  static int forward(const UdeProblem* p, const float* pack, const void* sched, const float* y0,
                     float* latent, float* ckpt, double* stats_slab, const UdeSideStats* st, unsigned* ctl,
                     hipStream_t s) {
    if constexpr (RC_VIEW) {
      if (p->recompute && ckpt) return Ops<Recompute<M>>::forward(p, pack, sched, y0, latent, ckpt, stats_slab,
                                                                  st, ctl, s);
    }
    if (!pack || !sched || !y0 || !latent || !stats_slab || !stats_ok(st)) return UDE_E_INVALID;
    if (M::L == 8 && (reinterpret_cast<uintptr_t>(latent) & 15))
      return UDE_E_INVALID;                          // the row-mapped tile start writes 16-B latent rows
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(dev, n_tiles, &gf, &gb);
    if (rc) return rc;
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.y0 = y0; a.sched = (const unsigned char*)sched;
    a.latent = latent; a.ckpt = ckpt; a.stats_slab = stats_slab;
    a.n_traj = p->n_traj; a.n_steps = p->n_steps; a.n_out = p->n_out; a.n_tiles = n_tiles;
    a.fa_w = p->fa_w;
    const double n_eval = 4.0 * (double)p->n_steps * (double)p->n_traj * (double)M::R;
    set_stats_out(a, st, ctl, n_eval);
#ifdef UDE_PROFILE
    a.prof = g_prof_buffer ? g_prof_buffer + (size_t)PROF_FWD_SLOT * NPROF : nullptr;   // behind the backward's
#endif
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const bool res = !(ckpt && M::SPLIT_FWD && n_tiles <= cus) && fwd_res(n_tiles, cus);
    if (res) gf = n_tiles < cus ? n_tiles : cus;
    if (ckpt && M::SPLIT_FWD && n_tiles <= cus)
      hipLaunchKernelGGL((ude_fwd_kernel<M, true, M::SPLIT_FWD>), dim3(gf), dim3(2 * NTHREADS), M::LDS_F, s, a);
    else if (res && ckpt)
      hipLaunchKernelGGL((ude_fwd_kernel<M, true, false, false, M::FWD_RES>), dim3(gf), dim3(NTHREADS), M::LDS_F, s, a);
    else if (res)
      hipLaunchKernelGGL((ude_fwd_kernel<M, false, false, false, M::FWD_RES>), dim3(gf), dim3(NTHREADS), M::LDS_F, s, a);
    else if (ckpt) hipLaunchKernelGGL((ude_fwd_kernel<M, true>), dim3(gf), dim3(NTHREADS), M::LDS_F, s, a);
    else hipLaunchKernelGGL((ude_fwd_kernel<M, false>), dim3(gf), dim3(NTHREADS), M::LDS_F, s, a);
    HIPCHK(hipGetLastError());
    if (!ctl) {
      hipLaunchKernelGGL(ude_stats_finalize_kernel<0>, dim3(1), dim3(320), 0, s, stats_slab, gf, n_eval, a.o_mean,
                         a.o_std, a.o_norm);
      HIPCHK(hipGetLastError());
    }
    return UDE_OK;
  }

  // st: the forward's statistics (read); dst: their cotangents (nullable); ctl: null = the separate
  // tail launches (grad finalize, static partial / reduce, dy0 static), else the one tail kernel
  static int backward(const UdeProblem* p, const float* pack, const void* sched, const float* y0,
                      const float* ckpt, const float* dlatent, const float* dlat_sir, const UdeSideStats* st,
                      const UdeSideStatsGrad* dst, float* dy0, float* slab, unsigned* ctl, float* dparams,
                      hipStream_t s) {
    if constexpr (RC_VIEW) {
      if (p->recompute) return Ops<Recompute<M>>::backward(p, pack, sched, y0, ckpt, dlatent, dlat_sir, st, dst,
                                                           dy0, slab, ctl, dparams, s);
    }
    if (!pack || !sched || !y0 || !stats_ok(st) || !dy0 || !slab || !dparams) return UDE_E_INVALID;
    if (p->n_steps > 0 && !ckpt) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(dev, n_tiles, &gf, &gb);
    if (rc) return rc;
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.y0 = y0; a.sched = (const unsigned char*)sched;
    a.ckpt = (float*)ckpt; a.dlatent = dlatent; a.dlat_sir = dlat_sir;
    a.st_mean = st->mean; a.st_std = st->std; a.st_norm = st->fa_norm;
    if (dst) { a.d_mean = dst->d_mean; a.d_std = dst->d_std; a.d_norm = dst->d_fa_norm; }
    a.dy0 = dy0; a.slab = slab;
    if (M::BAYES) a.eslab = pack + (size_t)n_evals(p) * M::PACK_TOTAL;
    float* g0buf = slab + (size_t)gb * M::SLAB_STRIDE;
    float* part = g0buf + (size_t)n_tiles * M::K0 * TT;
    a.g0buf = g0buf;
#ifdef UDE_PROFILE
    a.prof = g_prof_buffer;
#endif
    a.n_traj = p->n_traj; a.n_steps = p->n_steps; a.n_out = p->n_out; a.n_tiles = n_tiles;
    a.fa_w = p->fa_w;
    if constexpr (M::GST) {
      // the backward stores the layer-output gradient rows; ude_gst_dw_kernel forms every evaluation's
      // weight gradient from them and the stored rows, ude_gst_reduce_kernel sums / eps-weights them
      int cus = 0;
      HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      const int64_t ne = n_evals(p);
      const int ks = gst_ks(cus, ne, n_tiles);
      a.gst = slab;
      float* part = slab + gst_rows_floats(n_tiles, p->n_steps);
      hipLaunchKernelGGL((ude_bwd_kernel<M>), dim3(gb), dim3(M::BWD_THREADS), M::LDS_B, s, a);
      HIPCHK(hipGetLastError());
      HIPCHK(static_tsum(p, dlatent, dy0, s));
      if (ne > 0) {
        GstArgs ga;
        ga.ckpt = ckpt; ga.gst = slab; ga.y0 = y0; ga.part = part;
        ga.n_traj = p->n_traj; ga.n_steps = p->n_steps; ga.n_tiles = n_tiles; ga.n_ks = ks;
        hipLaunchKernelGGL((ude_gst_dw_kernel<M>), dim3(ks, (unsigned)ne), dim3(Gst<M>::NT), Gst<M>::LDS, s, ga);
        HIPCHK(hipGetLastError());
      }
      hipLaunchKernelGGL((ude_gst_reduce_kernel<M>), dim3((M::SLAB_TOTAL + 63) / 64), dim3(256), 0, s,
                         (const float*)part, (const float*)a.eslab, (int)ne, ks, dparams);
      HIPCHK(hipGetLastError());
      return UDE_OK;
    }
    hipLaunchKernelGGL((ude_bwd_kernel<M>), dim3(gb), dim3(M::BWD_THREADS), M::LDS_B, s, a);
    HIPCHK(hipGetLastError());
    HIPCHK(static_tsum(p, dlatent, dy0, s));
    if (ctl) {
      hipLaunchKernelGGL((ude_bwd_tail_kernel<M>), dim3(Tail<M>::blocks(n_tiles)), dim3(256), Tail<M>::LDS, s,
                         (const float*)slab, gb, (const float*)g0buf, pack, y0, dlatent, p->n_traj, n_tiles,
                         p->n_out + 1, part, ctl, dy0, dparams);
      HIPCHK(hipGetLastError());
      return UDE_OK;
    }
    hipLaunchKernelGGL((ude_grad_finalize_kernel<M>), dim3((M::SLAB_TOTAL + 63) / 64), dim3(256), 0, s,
                       (const float*)slab, gb, dparams);
    HIPCHK(hipGetLastError());
    if (M::BAYES) {
      // d |std|: the eps-weighted half of every workgroup slab
      hipLaunchKernelGGL((ude_grad_finalize_kernel<M>), dim3((M::SLAB_TOTAL + 63) / 64), dim3(256), 0, s,
                         (const float*)(slab + M::SLAB_TOTAL), gb, dparams + M::N_PARAMS);
      HIPCHK(hipGetLastError());
    }
    if (M::HOIST) {
      hipLaunchKernelGGL((ude_static_partial_kernel<M>), dim3(M::STATIC_CHUNKS, M::STATIC_GROUPS), dim3(256), 0, s,
                         (const float*)g0buf, y0, p->n_traj, n_tiles, part);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL((ude_static_reduce_kernel<M>), dim3((M::K0 * M::S + 255) / 256), dim3(256), 0, s,
                         (const float*)part, dparams);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL((ude_dy0_static_kernel<M>), dim3(n_tiles), dim3(256), TT * M::R * M::L * 4, s,
                         (const float*)g0buf, pack, dlatent, p->n_traj, p->n_out + 1, dy0);
      HIPCHK(hipGetLastError());
    }
    return UDE_OK;
  }
};

// ---- adaptive dopri5 solve (ude_dopri5.h) ------------------------------------
template <class M>
struct DopriOps {
  struct Layout {
    size_t ctl, part, stats, S, Cm, total;
  };
  static constexpr int CHUNK = 8;      // step attempts queued between host checks

  static int attrs_grid(int device, int n_tiles, int* grid) {
    static bool done = false;
    if (!done) {
      HIPCHK(hipFuncSetAttribute((const void*)&ude_dopri_kernel<M, dp::MODE_F0>, hipFuncAttributeMaxDynamicSharedMemorySize, M::LDS_F));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_dopri_kernel<M, dp::MODE_TRIAL>, hipFuncAttributeMaxDynamicSharedMemorySize, M::LDS_F));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_dopri_kernel<M, dp::MODE_STEP>, hipFuncAttributeMaxDynamicSharedMemorySize, M::LDS_F));
      done = true;
    }
    int cus = 0, occ = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&ude_dopri_kernel<M, dp::MODE_STEP>, NTHREADS, M::LDS_F));
    if (occ < 1) occ = 1;
    const long mx = (long)cus * occ;
    *grid = (int)(n_tiles < mx ? n_tiles : mx);
    if (*grid < 1) *grid = 1;
    return UDE_OK;
  }

  static Layout layout(int n_tiles, int grid) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    Layout L;
    L.ctl = 0;
    L.part = al(sizeof(DopriCtl));
    L.stats = L.part + al((size_t)grid * 4 * 8);
    L.S = L.stats + al((size_t)grid * 5 * 8);
    L.Cm = L.S + al((size_t)2 * n_tiles * 2 * M::F * TT * 4);
    L.total = L.Cm + al((size_t)n_tiles * M::F * TT * 4);
    return L;
  }

  static int workspace(const UdeProblem* p, int device, int64_t* bytes) {
    if (M::BAYES) return UDE_E_UNSUPPORTED;
    if (p->n_traj < 1 || p->n_out < 0) return UDE_E_INVALID;
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int grid = 1;
    int rc = attrs_grid(device, n_tiles, &grid);
    if (rc) return rc;
    *bytes = (int64_t)layout(n_tiles, grid).total;
    return UDE_OK;
  }

  static int forward(const UdeProblem* p, const float* pack, const double* t_out, double rtol, double atol,
                     double first_step, int max_steps, const float* y0, float* latent, void* ws, float* stats_out,
                     UdeDopriInfo* info, hipStream_t s) {
    if (M::BAYES) return UDE_E_UNSUPPORTED;
    if (!pack || !t_out || !y0 || !latent || !ws || !stats_out || p->n_traj < 1 || p->n_out < 0) return UDE_E_INVALID;
    if (max_steps < 1) max_steps = 1;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int grid = 1;
    int rc = attrs_grid(dev, n_tiles, &grid);
    if (rc) return rc;
    const Layout L = layout(n_tiles, grid);
    unsigned char* base = (unsigned char*)ws;
    DArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.y0 = y0; a.t_out = t_out; a.latent = latent;
    a.S = (float*)(base + L.S); a.Cm = (float*)(base + L.Cm);
    a.part = (double*)(base + L.part); a.stats_slab = (double*)(base + L.stats);
    a.ctl = (DopriCtl*)(base + L.ctl);
    a.n_traj = p->n_traj; a.n_tiles = n_tiles; a.n_times = p->n_out + 1;
    a.fa_w = p->fa_w; a.rtol32 = (float)rtol; a.atol32 = (float)atol;
    const double count = (double)p->n_traj * M::R * M::L;
    const dim3 g(grid), b(NTHREADS);
    hipLaunchKernelGGL((ude_dopri_kernel<M, dp::MODE_F0>), g, b, M::LDS_F, s, a);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(ude_dopri_ctl_kernel<0>, dim3(1), dim3(64), 0, s, (int)dp::MODE_F0, (const double*)a.part, grid,
                       a.ctl, t_out, a.n_times, count, max_steps, first_step);
    if (!(first_step > 0.0)) {
      hipLaunchKernelGGL((ude_dopri_kernel<M, dp::MODE_TRIAL>), g, b, M::LDS_F, s, a);
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(ude_dopri_ctl_kernel<0>, dim3(1), dim3(64), 0, s, (int)dp::MODE_TRIAL, (const double*)a.part,
                       grid, a.ctl, t_out, a.n_times, count, max_steps, first_step);
    HIPCHK(hipGetLastError());
    DopriCtl h;
    memset(&h, 0, sizeof(h));
    for (long it = 0;; it += CHUNK) {
      HIPCHK(hipMemcpyAsync(&h, a.ctl, sizeof(h), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      if (h.done || h.err) break;
      for (int i = 0; i < CHUNK; ++i) {
        hipLaunchKernelGGL((ude_dopri_kernel<M, dp::MODE_STEP>), g, b, M::LDS_F, s, a);
        hipLaunchKernelGGL(ude_dopri_ctl_kernel<0>, dim3(1), dim3(64), 0, s, (int)dp::MODE_STEP, (const double*)a.part,
                           grid, a.ctl, t_out, a.n_times, count, max_steps, first_step);
      }
      HIPCHK(hipGetLastError());
    }
    if (info) {
      info->n_steps = h.n_steps; info->n_accepted = h.n_accepted; info->n_evals = h.n_evals; info->status = h.err;
    }
    if (h.err) return UDE_E_SOLVER;
    // the last accepted step's outputs (idempotent if a queued step kernel already wrote them)
    hipLaunchKernelGGL((ude_dopri_kernel<M, dp::MODE_STEP>), g, b, M::LDS_F, s, a);
    HIPCHK(hipGetLastError());
    const double n_eval = (double)h.n_evals * (double)p->n_traj * (double)M::R;
    hipLaunchKernelGGL(ude_stats_finalize_kernel<0>, dim3(1), dim3(320), 0, s, a.stats_slab, grid,
                       n_eval, stats_out, stats_out + 2, stats_out + 4);
    HIPCHK(hipGetLastError());
    return UDE_OK;
  }
};

// ---- fused loss head (ude_loss.h): decoder + nll_loss + latent_init_loss ----------
template <class M>
struct LossOps {
  using D = LossDims<M::R>;
  struct Layout {
    size_t musd, part, slab, total;
  };
  // forward and backward grids differ (the forward needs no decoder-weight copy in LDS: two
  // workgroups per CU); the workspace holds the forward's partials and the backward's slabs
  static int grid(int device, int T, int S, int B, bool bwd, int* g) {
    if (T < 1 || S < 2 || B < 1) return UDE_E_INVALID;
    const int lds = D::lds_bytes(S, bwd);
    if (lds > 160 * 1024 || pad16(S) > SP_MAX) return UDE_E_UNSUPPORTED;
    static bool done = false;
    if (!done) {
      HIPCHK(hipFuncSetAttribute((const void*)&ude_loss_kernel<D, M::L, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_loss_kernel<D, M::L, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      done = true;
    }
    int cus = 0, occ = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    if (bwd)
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&ude_loss_kernel<D, M::L, true>, LTHREADS, lds));
    else
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)&ude_loss_kernel<D, M::L, false>, LTHREADS, lds));
    if (occ < 1) occ = 1;
    const long mx = (long)cus * occ, groups = (long)T * B;
    *g = (int)(groups < mx ? groups : mx);
    return UDE_OK;
  }
  static Layout layout(int T, int B, int gf, int gb) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    Layout L;
    L.musd = 0;
    L.part = al((size_t)T * B * M::R * 2 * 4);
    L.slab = L.part + al((size_t)gf * 2 * 8);
    L.total = L.slab + al((size_t)gb * D::SLAB * 4);
    return L;
  }
  static int grids(int device, int T, int S, int B, int* gf, int* gb) {
    int rc = grid(device, T, S, B, false, gf);
    if (rc) return rc;
    return grid(device, T, S, B, true, gb);
  }
  static int workspace(int T, int S, int B, int device, int64_t* bytes) {
    int gf = 1, gb = 1;
    int rc = grids(device, T, S, B, &gf, &gb);
    if (rc) return rc;
    *bytes = (int64_t)layout(T, B, gf, gb).total;
    return UDE_OK;
  }
  static int run(bool bwd, int T, int S, int B, const float* latent, const float* W, const float* b, const float* y,
                 const float* grad, void* ws, float* out, float* dlatent, float* dW, float* db, hipStream_t s,
                 int dl_sir = 0) {
    if (!latent || !W || !b || !y || !ws) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    int gf = 1, gb = 1;
    int rc = grids(dev, T, S, B, &gf, &gb);
    if (rc) return rc;
    const Layout Lo = layout(T, B, gf, gb);
    unsigned char* base = (unsigned char*)ws;
    LArgs a;
    memset(&a, 0, sizeof(a));
    a.latent = latent; a.W = W; a.bias = b; a.y = y;
    a.musd = (float*)(base + Lo.musd); a.part = (double*)(base + Lo.part); a.slab = (float*)(base + Lo.slab);
    a.dlatent = dlatent; a.grad = grad;
    a.T = T; a.S = S; a.B = B; a.dl_sir = dl_sir;
    if (!bwd) {
      if (!out) return UDE_E_INVALID;
      hipLaunchKernelGGL((ude_loss_kernel<D, M::L, false>), dim3(gf), dim3(LTHREADS), D::lds_bytes(S, false), s, a);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL(ude_loss_finalize_kernel<0>, dim3(1), dim3(128), 0, s, (const double*)a.part, gf,
                         (double)B * T * M::R, out);
      HIPCHK(hipGetLastError());
    } else {
      if (!grad || !dlatent || !dW || !db) return UDE_E_INVALID;
      hipLaunchKernelGGL((ude_loss_kernel<D, M::L, true>), dim3(gb), dim3(LTHREADS), D::lds_bytes(S, true), s, a);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL((ude_loss_grad_finalize_kernel<D>), dim3((D::SLAB + 63) / 64), dim3(256), 0, s,
                         (const float*)a.slab, gb, dW, db);
      HIPCHK(hipGetLastError());
    }
    return UDE_OK;
  }
  static int forward(int T, int S, int B, const float* latent, const float* W, const float* b, const float* y,
                     void* ws, float* out, hipStream_t s) {
    return run(false, T, S, B, latent, W, b, y, nullptr, ws, out, nullptr, nullptr, nullptr, s);
  }
  static int backward(int T, int S, int B, const float* latent, const float* W, const float* b, const float* y,
                      const float* grad, void* ws, float* dlatent, float* dW, float* db, hipStream_t s) {
    return run(true, T, S, B, latent, W, b, y, grad, ws, nullptr, dlatent, dW, db, s);
  }
  static int backward_sir(int T, int S, int B, const float* latent, const float* W, const float* b, const float* y,
                          const float* grad, void* ws, float* dlat_sir, float* dW, float* db, hipStream_t s) {
    return run(true, T, S, B, latent, W, b, y, grad, ws, nullptr, dlat_sir, dW, db, s, 1);
  }
};

// ---- one RHS evaluation + its VJP (ude_eval.h) -------------------------------------------
template <class M>
struct EvalOps {
  static int grids(int device, int n_tiles, int* gf, int* gb) {
    if constexpr (M::BAYES) {
      return UDE_E_UNSUPPORTED;
    } else {
    static bool done = false;
    if (!done) {
      HIPCHK(hipFuncSetAttribute((const void*)&ude_eval_fwd_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize, M::LDS_F));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_eval_vjp_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize, M::LDS_B));
      HIPCHK(hipFuncSetAttribute((const void*)&ude_bwd_tail_kernel<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 Tail<M>::LDS));
      done = true;
    }
    int cus = 0, of = 0, ob = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&of, (const void*)&ude_eval_fwd_kernel<M>, NTHREADS, M::LDS_F));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&ob, (const void*)&ude_eval_vjp_kernel<M>, eval_vjp_threads<M>(),
                                                           M::LDS_B));
    const long mf = (long)cus * (of < 1 ? 1 : of), mb = (long)cus * (ob < 1 ? 1 : ob);
    *gf = (int)(n_tiles < mf ? n_tiles : mf);
    *gb = (int)(n_tiles < mb ? n_tiles : mb);
    return UDE_OK;
    }
  }
  // workspace: dW slab [gb][SLAB_STRIDE], G0 + static partials (HOIST), the tail's ticket words
  static int64_t ctl_off(int gb, int n_tiles) {
    return ((int64_t)gb * M::SLAB_STRIDE + Ops<M>::static_ws_floats(n_tiles) + 3) & ~(int64_t)3;
  }
  static int workspace(const UdeProblem* p, int device, int64_t* bytes) {
    if (M::BAYES) return UDE_E_UNSUPPORTED;      // each evaluation's sample is a deterministic RHS
    if (p->n_traj < 1) return UDE_E_INVALID;
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(device, n_tiles, &gf, &gb);
    if (rc) return rc;
    *bytes = (ctl_off(gb, n_tiles) + Ops<M>::CTL_WORDS) * 4;
    return UDE_OK;
  }
  static int forward(const UdeProblem* p, const float* pack, const float* x, float* f, float* rates, float* fa,
                     hipStream_t s) {
    if constexpr (M::BAYES) {
      return UDE_E_UNSUPPORTED;
    } else {
    if (!pack || !x || !f || p->n_traj < 1) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(dev, n_tiles, &gf, &gb);
    if (rc) return rc;
    EArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.x = x; a.f = f; a.rates = rates; a.fa = fa;
    a.n_traj = p->n_traj; a.n_tiles = n_tiles; a.fa_w = p->fa_w;
    hipLaunchKernelGGL((ude_eval_fwd_kernel<M>), dim3(gf), dim3(NTHREADS), M::LDS_F, s, a);
    HIPCHK(hipGetLastError());
    return UDE_OK;
    }
  }
  static int vjp(const UdeProblem* p, const float* pack, const float* x, const float* cot_f, const float* cot_rates,
                 const float* cot_fa, float* dx, void* ws, float* dparams, hipStream_t s) {
    return eval_vjp(p, pack, x, cot_f, cot_rates, cot_fa, nullptr, 1.f, dx, ws, dparams, s);
  }
  // odeint_adjoint's augmented evaluation: f (scaled) and the VJP in one launch
  static int fused(const UdeProblem* p, const float* pack, const float* x, const float* cot_f, float* fout,
                   float f_scale, float* dx, void* ws, float* dparams, hipStream_t s) {
    if (!fout) return UDE_E_INVALID;
    return eval_vjp(p, pack, x, cot_f, nullptr, nullptr, fout, f_scale, dx, ws, dparams, s);
  }
  static int eval_vjp(const UdeProblem* p, const float* pack, const float* x, const float* cot_f,
                      const float* cot_rates, const float* cot_fa, float* fout, float f_scale, float* dx, void* ws,
                      float* dparams, hipStream_t s) {
    if constexpr (M::BAYES) {
      return UDE_E_UNSUPPORTED;
    } else {
    if (!pack || !x || !cot_f || !dx || !ws || !dparams || p->n_traj < 1) return UDE_E_INVALID;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const int n_tiles = (p->n_traj + TT - 1) / TT;
    int gf = 1, gb = 1;
    int rc = grids(dev, n_tiles, &gf, &gb);
    if (rc) return rc;
    float* slab = (float*)ws;
    float* g0buf = slab + (size_t)gb * M::SLAB_STRIDE;
    float* part = g0buf + (size_t)n_tiles * M::K0 * TT;
    EArgs a;
    memset(&a, 0, sizeof(a));
    a.pack = pack; a.x = x; a.cot_f = cot_f; a.cot_rates = cot_rates; a.cot_fa = cot_fa;
    a.dx = dx; a.slab = slab; a.g0buf = g0buf;
    a.n_traj = p->n_traj; a.n_tiles = n_tiles; a.fa_w = p->fa_w;
    a.fout = fout; a.f_scale = f_scale;
    unsigned int* ctl = reinterpret_cast<unsigned int*>(slab + ctl_off(gb, n_tiles));
    a.ctl = ctl; a.n_ctl = (int)Ops<M>::CTL_WORDS;
    hipLaunchKernelGGL((ude_eval_vjp_kernel<M>), dim3(gb), dim3(eval_vjp_threads<M>()), M::LDS_B, s, a);
    HIPCHK(hipGetLastError());
    // gradient finalize, static-column dW and dx's static dims: one launch (no time sums here)
    hipLaunchKernelGGL((ude_bwd_tail_kernel<M>), dim3(Tail<M>::blocks(n_tiles)), dim3(256), Tail<M>::LDS, s,
                       (const float*)slab, gb, (const float*)g0buf, pack, x, (const float*)nullptr, p->n_traj,
                       n_tiles, 0, part, ctl, dx, dparams);
    HIPCHK(hipGetLastError());
    return UDE_OK;
    }
  }
};

struct Entry {
  bool (*match)(const UdeModelDesc*);
  int (*query)(const UdeProblem*, int, UdeSizes*);
  int (*pack)(const float* const*, const float* const*, float*, hipStream_t);
  int (*pack_bayes)(const UdeProblem*, const float* const*, const float* const*, const float* const*,
                    const float* const*, const float*, float*, hipStream_t);
  int (*forward)(const UdeProblem*, const float*, const void*, const float*, float*, float*, double*,
                 const UdeSideStats*, unsigned*, hipStream_t);
  int (*backward)(const UdeProblem*, const float*, const void*, const float*, const float*, const float*,
                  const float*, const UdeSideStats*, const UdeSideStatsGrad*, float*, float*, unsigned*, float*,
                  hipStream_t);
  int (*dopri5_workspace)(const UdeProblem*, int, int64_t*);
  int (*dopri5_forward)(const UdeProblem*, const float*, const double*, double, double, double, int, const float*,
                        float*, void*, float*, UdeDopriInfo*, hipStream_t);
  int (*loss_workspace)(int, int, int, int, int64_t*);
  int (*loss_forward)(int, int, int, const float*, const float*, const float*, const float*, void*, float*,
                      hipStream_t);
  int (*loss_backward)(int, int, int, const float*, const float*, const float*, const float*, const float*, void*,
                       float*, float*, float*, hipStream_t);
  int (*loss_backward_sir)(int, int, int, const float*, const float*, const float*, const float*, const float*,
                           void*, float*, float*, float*, hipStream_t);
  int (*rhs_workspace)(const UdeProblem*, int, int64_t*);
  int (*rhs_forward)(const UdeProblem*, const float*, const float*, float*, float*, float*, hipStream_t);
  int (*rhs_vjp)(const UdeProblem*, const float*, const float*, const float*, const float*, const float*, float*,
                 void*, float*, hipStream_t);
  int (*dec_pack)(const float*, const float*, float*, hipStream_t);
  int (*forward_dec)(const UdeProblem*, const float*, const void*, const float*, const float*, float*, float*, double*,
                     double*, const UdeSideStats*, unsigned*, float*, hipStream_t);
  int (*dec_backward)(const UdeProblem*, const void*, const float*, const float*, const float*, const float*, void*,
                      float*, float*, float*, hipStream_t);
  int (*nll_workspace)(int, int, int, int64_t*);
  int (*nll_forward)(int, int, int, const float*, const float*, void*, float*, hipStream_t);
  int (*nll_backward)(int, int, int, const float*, const float*, const float*, const void*, float*, hipStream_t);
  int (*rhs_eval_vjp)(const UdeProblem*, const float*, const float*, const float*, float*, float, float*, void*,
                      float*, hipStream_t);
};

template <class M>
constexpr Entry make_entry() {
  return Entry{&matches<M>, &Ops<M>::query, &Ops<M>::pack, &Ops<M>::pack_bayes, &Ops<M>::forward, &Ops<M>::backward,
               &DopriOps<M>::workspace, &DopriOps<M>::forward, &LossOps<M>::workspace, &LossOps<M>::forward,
               &LossOps<M>::backward, &LossOps<M>::backward_sir, &EvalOps<M>::workspace, &EvalOps<M>::forward,
               &EvalOps<M>::vjp, &Ops<M>::dec_pack, &Ops<M>::forward_dec, &Ops<M>::dec_backward,
               &Ops<M>::nll_workspace, &Ops<M>::nll_forward, &Ops<M>::nll_backward, &EvalOps<M>::fused};
}


}  // namespace ude
