// C-ABI entry points (include/ude_rk4.h) over the compiled model configurations.
// The registry (ude_registry.inc, generated at build time) lists one
// ude::Entry per configuration object linked into this library.
#include <hip/hip_runtime.h>
#include "ude_rk4.h"
#include "ude_entry.h"
#include "ude_vec.h"      // model-independent vector kernels (compiled in both passes)

// This translation unit is host code only (no kernels are instantiated here).
#if !defined(__HIP_DEVICE_COMPILE__)
#include "ude_registry.inc"   // extern const ude::Entry ude_entry_N; + kEntries[] / kNumEntries

using ude::Entry;

namespace {
// the legacy contiguous statistics vectors ({mean[2], std[2], |Fa|}) as UdeSideStats / UdeSideStatsGrad
UdeSideStats stats_of(float* stats_out) {
  UdeSideStats st = {stats_out, stats_out ? stats_out + 2 : nullptr, stats_out ? stats_out + 4 : nullptr, nullptr};
  return st;
}
UdeSideStatsGrad dstats_of(const float* d) {
  UdeSideStatsGrad g = {d, d ? d + 2 : nullptr, d ? d + 4 : nullptr};
  return g;
}
const ude::Entry* find(const UdeModelDesc* m) {
  if (!m) return nullptr;
  for (int i = 0; i < ude::kNumEntries; ++i)
    if (ude::kEntries[i]->match(m)) return ude::kEntries[i];
  return nullptr;
}
}  // namespace

#ifdef UDE_PROFILE
namespace ude { unsigned long long* g_prof_buffer = nullptr; }
#endif

extern "C" {

int ude_supported(const UdeModelDesc* m) { return find(m) ? 1 : 0; }

int ude_query(const UdeModelDesc* m, const UdeProblem* p, int device, UdeSizes* out) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || !out) return UDE_E_INVALID;
  return e->query(p, device, out);
}

int ude_pack_weights(const UdeModelDesc* m, const float* const* W, const float* const* b, float* pack,
                     ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!W || !b || !pack) return UDE_E_INVALID;
  return e->pack(W, b, pack, (hipStream_t)stream);
}

int ude_pack_weights_bayes(const UdeModelDesc* m, const UdeProblem* p, const float* const* W_mean,
                           const float* const* b_mean, const float* const* W_std, const float* const* b_std,
                           const float* eps, float* pack, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || !W_mean || !b_mean || !W_std || !b_std || !eps || !pack) return UDE_E_INVALID;
  return e->pack_bayes(p, W_mean, b_mean, W_std, b_std, eps, pack, (hipStream_t)stream);
}

int ude_rk4_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                    const float* y0, float* latent, float* ckpt, double* stats_slab, float* stats_out,
                    ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 0 || !stats_out) return UDE_E_INVALID;
  const UdeSideStats st = stats_of(stats_out);
  return e->forward(p, pack, sched, y0, latent, ckpt, stats_slab, &st, nullptr, (hipStream_t)stream);
}

int ude_rk4_forward_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                       const float* y0, float* latent, float* ckpt, double* stats_slab, uint32_t* ctl,
                       const UdeSideStats* stats, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 0 || !ctl || !stats) return UDE_E_INVALID;
  return e->forward(p, pack, sched, y0, latent, ckpt, stats_slab, stats, ctl, (hipStream_t)stream);
}

int ude_rk4_backward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                     const float* y0, const float* ckpt, const float* dlatent, const float* stats_out,
                     const float* dstats, float* dy0, float* grad_slab, float* dparams, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 0 || !dlatent || !stats_out || !dstats) return UDE_E_INVALID;
  const UdeSideStats st = stats_of(const_cast<float*>(stats_out));
  const UdeSideStatsGrad dst = dstats_of(dstats);
  return e->backward(p, pack, sched, y0, ckpt, dlatent, nullptr, &st, &dst, dy0, grad_slab, nullptr, dparams,
                     (hipStream_t)stream);
}

int ude_rk4_backward_sir(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                         const float* y0, const float* ckpt, const float* dlatent, const float* dlatent_sir,
                         const float* stats_out, const float* dstats, float* dy0, float* grad_slab, float* dparams,
                         ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 0 || (!dlatent) == (!dlatent_sir) || !stats_out || !dstats)
    return UDE_E_INVALID;
  const UdeSideStats st = stats_of(const_cast<float*>(stats_out));
  const UdeSideStatsGrad dst = dstats_of(dstats);
  return e->backward(p, pack, sched, y0, ckpt, dlatent, dlatent_sir, &st, &dst, dy0, grad_slab, nullptr, dparams,
                     (hipStream_t)stream);
}

int ude_rk4_backward_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                        const float* y0, const float* ckpt, const float* dlatent, const float* dlatent_sir,
                        const UdeSideStats* stats, const UdeSideStatsGrad* dstats, float* dy0, float* grad_slab,
                        uint32_t* ctl, float* dparams, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 0 || (!dlatent) == (!dlatent_sir) || !stats || !ctl)
    return UDE_E_INVALID;
  return e->backward(p, pack, sched, y0, ckpt, dlatent, dlatent_sir, stats, dstats, dy0, grad_slab, ctl, dparams,
                     (hipStream_t)stream);
}

int ude_dopri5_workspace(const UdeModelDesc* m, const UdeProblem* p, int device, int64_t* ws_bytes) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || !ws_bytes) return UDE_E_INVALID;
  return e->dopri5_workspace(p, device, ws_bytes);
}

int ude_dopri5_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const double* t_out,
                       double rtol, double atol, double first_step, int32_t max_steps, const float* y0,
                       float* latent, void* ws, float* stats_out, UdeDopriInfo* info, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || !(rtol >= 0.0) || !(atol >= 0.0)) return UDE_E_INVALID;
  return e->dopri5_forward(p, pack, t_out, rtol, atol, first_step, max_steps, y0, latent, ws, stats_out, info,
                           (hipStream_t)stream);
}

int ude_loss_head_workspace(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, int device, int64_t* ws_bytes) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!ws_bytes) return UDE_E_INVALID;
  return e->loss_workspace(T, S, B, device, ws_bytes);
}

int ude_loss_head_forward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                          const float* W, const float* b, const float* y, void* ws, float* out, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  return e->loss_forward(T, S, B, latent, W, b, y, ws, out, (hipStream_t)stream);
}

int ude_loss_head_backward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                           const float* W, const float* b, const float* y, const float* grad, void* ws,
                           float* dlatent, float* dW, float* db, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  return e->loss_backward(T, S, B, latent, W, b, y, grad, ws, dlatent, dW, db, (hipStream_t)stream);
}

int ude_loss_head_backward_sir(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                               const float* W, const float* b, const float* y, const float* grad, void* ws,
                               float* dlatent_sir, float* dW, float* db, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!dlatent_sir) return UDE_E_INVALID;
  return e->loss_backward_sir(T, S, B, latent, W, b, y, grad, ws, dlatent_sir, dW, db, (hipStream_t)stream);
}

int ude_rhs_workspace(const UdeModelDesc* m, const UdeProblem* p, int device, int64_t* ws_bytes) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || !ws_bytes) return UDE_E_INVALID;
  return e->rhs_workspace(p, device, ws_bytes);
}

int ude_rhs_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x, float* f,
                    float* rates, float* fa, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p) return UDE_E_INVALID;
  return e->rhs_forward(p, pack, x, f, rates, fa, (hipStream_t)stream);
}

int ude_rhs_vjp(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x, const float* cot_f,
                const float* cot_rates, const float* cot_fa, float* dx, void* ws, float* dparams,
                ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p) return UDE_E_INVALID;
  return e->rhs_vjp(p, pack, x, cot_f, cot_rates, cot_fa, dx, ws, dparams, (hipStream_t)stream);
}

int ude_rhs_eval_vjp(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x,
                     const float* cot_f, float* f_out, float f_scale, float* dx, void* ws, float* dparams,
                     ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p) return UDE_E_INVALID;
  return e->rhs_eval_vjp(p, pack, x, cot_f, f_out, f_scale, dx, ws, dparams, (hipStream_t)stream);
}

int ude_lincomb(int64_t n, const float* base, const float* const* k, int32_t nk, const float* coef, float* out,
                ude_stream_t stream) {
  return ude::lincomb(n, base, k, nk, coef, out, (hipStream_t)stream);
}

int ude_scaled_sumsq(int64_t n, const float* err, const float* y0, const float* y1, double atol, double rtol,
                     double* out, ude_stream_t stream) {
  return ude::scaled_sumsq(n, err, y0, y1, atol, rtol, out, (hipStream_t)stream);
}

int ude_lincomb_hc(int64_t n, const float* base, const float* const* k, int32_t nk, const float* coef_host,
                   float* out, ude_stream_t stream) {
  if (!coef_host) return UDE_E_INVALID;
  return ude::lincomb(n, base, k, nk, nullptr, out, (hipStream_t)stream, coef_host);
}

int ude_dopri_ratio(const float* err, const float* y0, const float* y1, double atol, double rtol, const double* ssq,
                    const int64_t* n, int32_t n_pieces, const double* extra, int32_t n_extra, double dt,
                    const unsigned char* flag, double* status, ude_stream_t stream) {
  return ude::dopri_ratio(err, y0, y1, atol, rtol, ssq, n, n_pieces, extra, n_extra, dt, flag, status,
                          (hipStream_t)stream);
}

int ude_pack_decoder(const UdeModelDesc* m, const float* W_dec, const float* b_dec, float* dec_pack,
                     ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  return e->dec_pack(W_dec, b_dec, dec_pack, (hipStream_t)stream);
}

int ude_rk4_forward_dec(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                        const float* y0, const float* dec_pack, float* yhat, float* ckpt, double* stats_slab,
                        double* reg_slab, float* stats_out, float* reg_out, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 1 || !stats_out) return UDE_E_INVALID;
  const UdeSideStats st = stats_of(stats_out);
  return e->forward_dec(p, pack, sched, y0, dec_pack, yhat, ckpt, stats_slab, reg_slab, &st, nullptr, reg_out,
                        (hipStream_t)stream);
}

int ude_rk4_forward_dec_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                           const float* y0, const float* dec_pack, float* yhat, float* ckpt, double* stats_slab,
                           double* reg_slab, uint32_t* ctl, const UdeSideStats* stats, float* reg_out,
                           ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 1 || !stats || !ctl) return UDE_E_INVALID;
  return e->forward_dec(p, pack, sched, y0, dec_pack, yhat, ckpt, stats_slab, reg_slab, stats, ctl, reg_out,
                        (hipStream_t)stream);
}

int ude_decoder_backward(const UdeModelDesc* m, const UdeProblem* p, const void* sched, const float* ckpt,
                         const float* dyhat, const float* W_dec, const float* grad_reg, void* ws, float* dl3,
                         float* dW_dec, float* db_dec, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!p || p->n_traj < 1 || p->n_steps < 1) return UDE_E_INVALID;
  return e->dec_backward(p, sched, ckpt, dyhat, W_dec, grad_reg, ws, dl3, dW_dec, db_dec, (hipStream_t)stream);
}

int ude_nll_workspace(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, int64_t* ws_bytes) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  if (!ws_bytes) return UDE_E_INVALID;
  return e->nll_workspace(T, S, B, ws_bytes);
}

int ude_nll_forward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* yhat, const float* y,
                    void* ws, float* out, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  return e->nll_forward(T, S, B, yhat, y, ws, out, (hipStream_t)stream);
}

int ude_nll_backward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* yhat, const float* y,
                     const float* grad, const void* ws, float* dyhat, ude_stream_t stream) {
  const Entry* e = find(m);
  if (!e) return UDE_E_UNSUPPORTED;
  return e->nll_backward(T, S, B, yhat, y, grad, ws, dyhat, (hipStream_t)stream);
}

#ifdef UDE_PROFILE
void ude_debug_set_prof(unsigned long long* p) { ude::g_prof_buffer = p; }
#endif

const char* ude_build_info(void) {
  return "ude_rk4 gfx950: v_mfma_f32_16x16x4_f32, TT=16, 4 waves/WG, registry=" UDE_REGISTRY_TAG
         " src=" UDE_SRC_HASH " extra_flags=[" UDE_EXTRA_FLAGS "]";
}

}  // extern "C"
#endif  // !__HIP_DEVICE_COMPILE__
