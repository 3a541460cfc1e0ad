/*
 * ude_rk4.h -- C-ABI of the MI355X (gfx950) UDE RK4 solver library.
 *
 * Drop-in boundary for the reference's hot path:
 *   torchdiffeq.odeint(ode, z, t, method='rk4', options=dict(step_size=h))
 *   called at lib/VAE.py:137 (and tuning/tune_encoders.py:221,
 *   tuning/tune_node.py:204, tuning/tune_Fp.py:93), with `ode` one of the
 *   right-hand sides Fp / Fa / FaFp of lib/models.py:109-265, plus the
 *   autograd backward through that solve that lib/VAE.py:203
 *   (`loss.backward()`) triggers, and the side statistics the loss reads:
 *   ode.posterior() (lib/models.py:152-156, lib/VAE.py:173) and
 *   torch.norm(torch.stack(ode.tracker)) (lib/VAE.py:180).
 *
 * Conventions
 *   - every pointer is a device pointer (HBM) unless stated; the caller owns
 *     every buffer, sized by ude_query(); the library never allocates and
 *     keeps no state between calls (re-entrant, stream ordered);
 *   - y0 / latent / dlatent / dy0 are row-major (..., N, R, L) fp32 exactly as
 *     a contiguous torch tensor; weights are nn.Linear layout (out, in);
 *   - return value 0 = ok, < 0 = error (UDE_E_*); the Python layer raises.
 */
#ifndef UDE_RK4_H
#define UDE_RK4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* ude_stream_t; /* == hipStream_t */

enum {
  UDE_OK = 0,
  UDE_E_UNSUPPORTED = -1, /* no compiled kernel for this model description */
  UDE_E_INVALID = -2,     /* bad argument (sizes, null pointers)            */
  UDE_E_HIP = -3,         /* a HIP runtime call failed                      */
  UDE_E_SOLVER = -4       /* adaptive solve failed (see UdeDopriInfo.status) */
};

/* kind: Fp / Fa / FaFp, optionally | UDE_KIND_BAYES for the Bayesian right-hand
 * sides Bayes_Fp / Bayes_Fa / Bayes_FaFp of lib/in_development/models_bayes.py
 * (:69-265), whose Dense_Variational layers (:12-48) draw a fresh weight sample
 * w = w_mean + eps * |w_std| at every evaluation. */
enum { UDE_KIND_FP = 1, UDE_KIND_FA = 2, UDE_KIND_FAFP = 3, UDE_KIND_BAYES = 4 };

/* The RHS module: lib/models.py FaFp(n_regions, latent_dim, net_sizes,
 * aug_net_sizes) etc.  Hidden-size lists of up to 4 entries. */
typedef struct UdeModelDesc {
  int32_t kind;          /* UDE_KIND_*                                   */
  int32_t n_regions;     /* R                                            */
  int32_t latent_dim;    /* L (>= 3)                                     */
  int32_t n_p_hidden;    /* len(net_sizes), 0 if no P-net                */
  int32_t p_hidden[4];
  int32_t n_a_hidden;    /* len(aug_net_sizes), 0 if no A-net            */
  int32_t a_hidden[4];
} UdeModelDesc;

/* One solve: N trajectories, `n_steps` RK4 grid steps, `n_out` output times. */
typedef struct UdeProblem {
  int32_t n_traj;
  int32_t n_steps;
  int32_t n_out;
  float fa_w;            /* FaFp.Fa_w (lib/models.py:225)                */
  int32_t recompute;     /* 0: the training forward stores every stage's activation rows
                            (UdeSizes.act_bytes of the checkpoint) and the backward reads
                            them; 1: memory fallback -- only the 3R stage inputs are stored
                            and the backward re-runs each stage's layers from them (same
                            results, bit for bit).  Forward and backward must agree. */
} UdeProblem;

/* Buffer sizes in bytes for one (model, problem). */
typedef struct UdeSizes {
  int64_t pack_bytes;       /* packed weights                                  */
  int64_t sched_bytes;      /* step/output schedule (layout below)              */
  int64_t ckpt_bytes;       /* stage states saved by a training forward          */
  int64_t stats_slab_bytes; /* per-workgroup fp64 partial sums                   */
  int64_t grad_slab_bytes;  /* per-workgroup gradient partials                   */
  int64_t n_params;         /* floats in the flat parameter-gradient output      */
  int32_t grid_fwd;         /* workgroups launched by the forward                */
  int32_t grid_bwd;         /* workgroups launched by the backward               */
  int32_t lds_fwd;          /* bytes of LDS per workgroup                        */
  int32_t lds_bwd;
  int64_t dec_pack_bytes;   /* packed decoder (ude_pack_decoder)                  */
  int64_t ckpt_final_bytes; /* final-state block a decoder-epilogue training forward
                               stores behind ckpt_bytes                          */
  int64_t dec_ws_bytes;     /* ude_decoder_backward workspace                     */
  int64_t act_bytes;        /* part of ckpt_bytes holding stored activation rows
                               (0 with UdeProblem.recompute = 1)                 */
  int64_t ctl_bytes;        /* control words of the *_ex calls (see below)         */
} UdeSizes;

/*
 * Schedule buffer (host-built, copied to the device), little-endian, packed:
 *   float   dt[n_steps]            grid[n+1]-grid[n] in fp32 (torchdiffeq)
 *   int32   out_start[n_steps+1]   CSR: outputs written after step n
 *   int32   out_j[n_out]           output index (1..T-1; output 0 is y0)
 *   int32   out_mode[n_out]        0: y(t0)  1: y(t1)  2: linear interpolation
 *   float   out_slope[n_out]       (t_j - t0)/(t1 - t0) in fp32
 * n_out here counts outputs 1..T-1 (T-1 entries).
 */

/* 1 if a kernel for this model is compiled into this library. */
int ude_supported(const UdeModelDesc* m);

/* Fill *out.  `device` is the HIP device ordinal used to size the grid. */
int ude_query(const UdeModelDesc* m, const UdeProblem* p, int device, UdeSizes* out);

/* Pack nn.Linear weights into the fragment layouts the kernels read.
 * W[i] / b[i]: P-net layers first (i = 0..n_p_hidden), then A-net layers. */
int ude_pack_weights(const UdeModelDesc* m, const float* const* W, const float* const* b,
                     float* pack, ude_stream_t stream);

/* Bayesian models (kind & UDE_KIND_BAYES): the per-evaluation weight samples of
 * one solve.  Replaces Dense_Variational.make_z + forward (models_bayes.py:30-48),
 * called 4 * n_steps times per solve by the reference: eps (device) is that draw
 * stream, [4 * n_steps][n_params / 2] floats, row e feeding evaluation e (stage
 * e % 4 of step e / 4), each row in torch parameter order (per layer: weight
 * (out, in) then bias; rate net first) -- the order the reference's layers call
 * make_z within one evaluation.  W_* / b_*: the layers' w_mean / b_mean /
 * w_std / b_std (|std| is taken here).  pack is sized by ude_query
 * (pack_bytes) and holds every sample plus the eps stream the backward needs.
 * For Bayesian models ude_query's n_params is 2 x the parameter count and
 * ude_rk4_backward's dparams = [d mean (torch order) | d |std| (torch order)]. */
int ude_pack_weights_bayes(const UdeModelDesc* m, const UdeProblem* p, const float* const* W_mean,
                           const float* const* b_mean, const float* const* W_std, const float* const* b_std,
                           const float* eps, float* pack, ude_stream_t stream);

/* Forward solve.  latent: (T, N, R, L) with T = n_out + 1.  If ckpt != NULL
 * the stage states are saved for ude_rk4_backward.  stats_out (device, 5
 * floats) receives {mean_beta, mean_gamma, std_beta, std_gamma, |Fa|}
 * (entries of an absent net are 0); on return stats_slab[0..4] holds the fp64
 * totals {sum beta, sum gamma, sum beta^2, sum gamma^2, sum Fa^2} those are
 * formed from (the data-parallel statistics exchange all-reduces them; the
 * same holds for ude_rk4_forward_dec and ude_dopri5_forward's workspace).
 * With L = 8, latent must be 16-byte aligned (the tile start writes its 32-B
 * (n, r) rows with 16-B stores): UDE_E_INVALID otherwise. */
int ude_rk4_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack,
                    const void* sched, const float* y0, float* latent, float* ckpt,
                    double* stats_slab, float* stats_out, ude_stream_t stream);

/* Backward (VJP) through the same solve.
 *   dlatent: (T, N, R, L) cotangent of latent
 *   dstats (device, 5 floats): d/dmean[2], d/dstd[2], d/d|Fa|
 *   dy0: (N, R, L) written;  dparams: n_params floats, torch parameter order
 *   (for each net: weight (out,in) then bias, layer by layer; P-net first). */
int ude_rk4_backward(const UdeModelDesc* m, const UdeProblem* p, const float* pack,
                     const void* sched, const float* y0, const float* ckpt,
                     const float* dlatent, const float* stats_out, const float* dstats,
                     float* dy0, float* grad_slab, float* dparams, ude_stream_t stream);

/* Backward with the S, I, R output cotangents handed over compactly: the
 * training loss terms read only latent[..., :3] (lib/VAE.py:138, :189 -- Decoder and
 * latent_init_loss), so their cotangent has zeros in every dim >= 3.  Exactly one of dlatent
 * (T, N, R, L) and dlatent_sir (T, N, R, 3) is given (the other NULL); with dlatent_sir the
 * dims >= 3 are zero.  With the fused loss head (ude_loss_head_backward_sir) neither the zero
 * dims nor a full-size cotangent are written or read.  Replaces the same autograd backward as
 * ude_rk4_backward (lib/VAE.py:203). */
int ude_rk4_backward_sir(const UdeModelDesc* m, const UdeProblem* p, const float* pack,
                         const void* sched, const float* y0, const float* ckpt,
                         const float* dlatent, const float* dlatent_sir, const float* stats_out,
                         const float* dstats, float* dy0, float* grad_slab, float* dparams,
                         ude_stream_t stream);

/* ---- side statistics as separate buffers, statistics and gradients finalised in-kernel --------
 * The reference reads a solve's statistics as three tensors: posterior() = Normal(mean, std) of every
 * recorded rate (lib/models.py:152-156, lib/VAE.py:173) and torch.norm(torch.stack(tracker)) = |Fa|
 * (lib/VAE.py:180).  The *_ex calls take them as separate device buffers (what the autograd layer
 * hands over as three outputs / three cotangents: no split, concatenation or zero-fill between the
 * solve and the loss), and finalise in the solve's own launches:
 *   ude_rk4_forward_ex / ude_rk4_forward_dec_ex: the last workgroup of the forward kernel turns the
 *     per-workgroup fp64 partials (stats_slab) into mean / std / |Fa| (and reg_out), in the fixed
 *     order of the separate finalize kernel of ude_rk4_forward (same bits);
 *   ude_rk4_backward_ex: the per-workgroup gradient slabs, the static-feature weight gradient and
 *     dy0's static dims are formed by ONE trailing kernel (instead of four).
 * ctl: ude_query's ctl_bytes of device memory, zeroed by the caller ONCE (e.g. at allocation) and
 * left zero by every call; calls that share a ctl buffer must be stream ordered (one ctl per stream
 * that runs solves concurrently).  Any UdeSideStats pointer of an absent net may be NULL; every
 * UdeSideStatsGrad pointer is nullable (zero cotangent).  Results equal ude_rk4_forward /
 * ude_rk4_backward_sir (statistics bitwise; the static-feature weight gradient within fp32 summation
 * order). */
typedef struct UdeSideStats {
  float* mean;      /* 2 floats: mean beta, mean gamma        (posterior().loc)   */
  float* std;       /* 2 floats: unbiased std of beta, gamma  (posterior().scale) */
  float* fa_norm;   /* 1 float: |Fa| over every evaluation                         */
  double* sums;     /* 5 doubles, nullable: sum beta, sum gamma, sum beta^2, sum gamma^2, sum Fa^2 */
} UdeSideStats;

typedef struct UdeSideStatsGrad {
  const float* d_mean;     /* 2 floats, nullable */
  const float* d_std;      /* 2 floats, nullable */
  const float* d_fa_norm;  /* 1 float, nullable  */
} UdeSideStatsGrad;

int ude_rk4_forward_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                       const float* y0, float* latent, float* ckpt, double* stats_slab, uint32_t* ctl,
                       const UdeSideStats* stats, ude_stream_t stream);

int ude_rk4_forward_dec_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                           const float* y0, const float* dec_pack, float* yhat, float* ckpt, double* stats_slab,
                           double* reg_slab, uint32_t* ctl, const UdeSideStats* stats, float* reg_out,
                           ude_stream_t stream);

/* stats: the forward's mean / std / fa_norm (read; sums unused). */
int ude_rk4_backward_ex(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                        const float* y0, const float* ckpt, const float* dlatent, const float* dlatent_sir,
                        const UdeSideStats* stats, const UdeSideStatsGrad* dstats, float* dy0, float* grad_slab,
                        uint32_t* ctl, float* dparams, ude_stream_t stream);

/* ---- adaptive Dormand-Prince solve (forward) ---------------------------------
 * Replaces torchdiffeq.odeint(func, y0, t, rtol, atol, method='dopri5',
 * options={'first_step': h?}) -- the default method of the solver API the
 * reference imports (lib/VAE.py:5, run_ode.py:24) -- for the UDE right-hand
 * sides (deterministic kinds only).  torchdiffeq semantics: one step size for
 * the whole batch from the RMS error norm over all N*R*L state elements, accept
 * iff error_ratio <= 1, torchdiffeq's initial-step heuristic, dense output (DPS
 * interpolant of the last accepted step) at every t_out, float64 time
 * arithmetic.  Stats are taken over every RHS evaluation (rejected steps and the
 * start-up evaluations included), as the reference's params / tracker lists.
 *   p->n_out = T - 1 (p->n_steps is ignored); t_out: T increasing float64 times
 *   (device); latent: (T, N, R, L); ws: ude_dopri5_workspace() bytes; info
 *   (host, may be NULL): step / evaluation counts and the failure reason
 *   (status 1: dt underflow, 2: max_steps reached, 3: non-finite state).
 * first_step <= 0 selects the initial step automatically.  This call waits for
 * the device (the number of steps is data dependent): it checks the device's
 * "done" flag every 8 step attempts. */
typedef struct UdeDopriInfo {
  int32_t n_steps, n_accepted, n_evals, status;
} UdeDopriInfo;

int ude_dopri5_workspace(const UdeModelDesc* m, const UdeProblem* p, int device, int64_t* ws_bytes);

int ude_dopri5_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const double* t_out,
                       double rtol, double atol, double first_step, int32_t max_steps, const float* y0,
                       float* latent, void* ws, float* stats_out, UdeDopriInfo* info, ude_stream_t stream);

/* ---- fused loss head ----------------------------------------------------------
 * The training loss terms that read the solve's latent, forward and backward in one
 * pass each over it (replaces, for one model's R and L):
 *   y_pred = Decoder(latent[..., :3])  (lib/models.py:27-51, Linear(3R -> R); lib/VAE.py:138)
 *            reshaped (T, S, B, R) -> permuted (B, S, T, R), sample n = s * B + b
 *   out[0] = nll_loss(y_pred, y)       (lib/train_functions.py:81-90: mean / unbiased std
 *            over the S samples, -Normal.log_prob(y), zero where y == -1, mean over B*T*R)
 *   out[1] = latent_init_loss(latent[..., :3])  (lib/train_functions.py:116-126, a sum)
 * latent (T, S*B, R, L), W (R, 3R), b (R), y (B, T, R); S >= 2.  ws: workspace bytes
 * from ude_loss_head_workspace, kept from forward to backward (per-group mean / std).
 * backward: grad (device, 2 floats) = d loss / d out; writes dlatent (T, S*B, R, L)
 * (dims >= 3: zero), dW (R, 3R), db (R). */
int ude_loss_head_workspace(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, int device, int64_t* ws_bytes);

int ude_loss_head_forward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                          const float* W, const float* b, const float* y, void* ws, float* out, ude_stream_t stream);

int ude_loss_head_backward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                           const float* W, const float* b, const float* y, const float* grad, void* ws,
                           float* dlatent, float* dW, float* db, ude_stream_t stream);

/* As ude_loss_head_backward, but d latent is written compactly: dlatent_sir (T, S*B, R, 3) =
 * the S, I, R cotangents (the loss terms do not read dims >= 3), to be handed to
 * ude_rk4_backward_sir. */
int ude_loss_head_backward_sir(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* latent,
                               const float* W, const float* b, const float* y, const float* grad, void* ws,
                               float* dlatent_sir, float* dW, float* db, ude_stream_t stream);

/* ---- one evaluation of the right-hand side and its VJP ---------------------------------
 * Fp / Fa / FaFp.forward(t, x) (lib/models.py:129-146, :177-188, :230-254) for every trajectory
 * of a batch: f (N, R, L) = the returned derivative (dims >= 3 zero, masked outside [-1, 2]),
 * rates (N, R, 2) = |net(x)| (what params.append records, :137 / :238; nullable) and
 * fa (N, R, 3) = aug_net(x) (tracker.append, :187 / :252; nullable).  ude_rhs_vjp: given the
 * cotangents of f (dims >= 3 ignored), rates and fa (both nullable: zero) writes dx (N, R, L)
 * and dparams (torch parameter order, ude_query's n_params) -- what autograd computes through
 * one forward() call.  These serve the solves that are not the fused RK4 kernel (adaptive
 * solves with autograd, odeint_adjoint, euler / midpoint) and, with each evaluation's sampled
 * weights packed by ude_pack_weights as a deterministic model, the Bayesian RHS
 * (models_bayes.py:43-48).  Deterministic kinds only; p->n_traj = N, p->fa_w = FaFp.Fa_w;
 * ws: ude_rhs_workspace() bytes. */
int ude_rhs_workspace(const UdeModelDesc* m, const UdeProblem* p, int device, int64_t* ws_bytes);

int ude_rhs_forward(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x, float* f,
                    float* rates, float* fa, ude_stream_t stream);

int ude_rhs_vjp(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x, const float* cot_f,
                const float* cot_rates, const float* cot_fa, float* dx, void* ws, float* dparams,
                ude_stream_t stream);

/* ---- decoder epilogue: the training solve without a latent ----------
 * The VAE's training loss reads the latent only through y_pred = Decoder(latent[..., :3])
 * (lib/models.py:27-51 Linear(3R -> R); lib/VAE.py:138) and latent_init_loss(latent[..., :3])
 * (lib/train_functions.py:116-126, lib/VAE.py:186).  ude_rk4_forward_dec runs the training forward
 * of ude_rk4_forward but emits, at every output time, y_hat (T, N, R) = W_dec . y[:3R] + b_dec
 * (y_pred = y_hat.reshape(T, S, B, R).permute(2, 1, 0, 3)) and reg_out (device float) =
 * latent_init_loss over every output's S, I, R, and writes no (T, N, R, L) latent.  Every output
 * time must be a grid point (torchdiffeq exact hit: schedule mode 1), n_steps >= 1 and
 * T <= 2048 (ude_decoder_backward returns UDE_E_INVALID otherwise).
 *   dec_pack: ude_query's dec_pack_bytes, filled by ude_pack_decoder(W_dec (R, 3R), b_dec (R));
 *   ckpt: ckpt_bytes + ckpt_final_bytes (the final state is stored behind the checkpoints);
 *   stats_slab: stats_slab_bytes; reg_slab: grid_fwd doubles.
 * ude_decoder_backward: given d y_hat (T, N, R) and grad_reg (device float, d loss / d reg_out)
 * writes the compact S, I, R cotangent dl3 (T, N, R, 3) for ude_rk4_backward_sir (every output
 * state read back from ckpt), d W_dec (R, 3R) and d b_dec (R); ws: dec_ws_bytes.
 * ude_nll_*: nll_loss(y_pred, y) (lib/train_functions.py:81-90) over y_hat (T, S*B, R) with targets
 * y (B, T, R), -1 = missing: out[0] = the mean nll; ws (ude_nll_workspace) keeps the per-group
 * sample mean / std (T, B, R, 2) for the backward, which writes d y_hat given grad (device float,
 * d loss / d nll). */
int ude_pack_decoder(const UdeModelDesc* m, const float* W_dec, const float* b_dec, float* dec_pack,
                     ude_stream_t stream);

int ude_rk4_forward_dec(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const void* sched,
                        const float* y0, const float* dec_pack, float* yhat, float* ckpt, double* stats_slab,
                        double* reg_slab, float* stats_out, float* reg_out, ude_stream_t stream);

int ude_decoder_backward(const UdeModelDesc* m, const UdeProblem* p, const void* sched, const float* ckpt,
                         const float* dyhat, const float* W_dec, const float* grad_reg, void* ws, float* dl3,
                         float* dW_dec, float* db_dec, ude_stream_t stream);

int ude_nll_workspace(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, int64_t* ws_bytes);

int ude_nll_forward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* yhat, const float* y,
                    void* ws, float* out, ude_stream_t stream);

int ude_nll_backward(const UdeModelDesc* m, int32_t T, int32_t S, int32_t B, const float* yhat, const float* y,
                     const float* grad, const void* ws, float* dyhat, ude_stream_t stream);

/* ---- odeint_adjoint's augmented dynamics (torchdiffeq adjoint; the solver API lib/VAE.py:5 imports) --
 * One evaluation of the right-hand side and its VJP in ONE launch: f_out = f_scale * f(x) (N, R, L),
 * dx = cot_f^T df/dx (N, R, L) and dparams = cot_f^T df/dtheta (torch parameter order).  The reversed
 * augmented dynamics of odeint_adjoint's backward, (-f, a^T df/dy, a^T df/dtheta), are f_scale = -1,
 * cot_f = a; replaces the module call + torch.autograd.grad per augmented evaluation.  Deterministic
 * kinds; ws: ude_rhs_workspace() bytes. */
int ude_rhs_eval_vjp(const UdeModelDesc* m, const UdeProblem* p, const float* pack, const float* x,
                     const float* cot_f, float* f_out, float f_scale, float* dx, void* ws, float* dparams,
                     ude_stream_t stream);

/* Dense passes of the adaptive step controllers (torchdiffeq's Dormand-Prince step; no model).
 * ude_lincomb: out[i] = base[i] + sum_j coef[j] * k[j][i] over n floats (base nullable: 0; coef a
 * DEVICE array of nk <= 8 floats; k a host array of nk device pointers), one pass.
 * ude_scaled_sumsq: out[0] (device fp64) = sum_i (err_i / (atol + rtol * max(|y0_i|, |y1_i|)))^2
 * (the error ratio's numerator, tolerance formed in fp32); out must hold UDE_SUMSQ_WS doubles. */
#define UDE_SUMSQ_WS 1025
int ude_lincomb(int64_t n, const float* base, const float* const* k, int32_t nk, const float* coef, float* out,
                ude_stream_t stream);
int ude_scaled_sumsq(int64_t n, const float* err, const float* y0, const float* y1, double atol, double rtol,
                     double* out, ude_stream_t stream);
/* ude_lincomb_hc: ude_lincomb with the nk coefficients in a HOST array, copied into the launch (the
 * controller forms them from its exact host mirror of dt: no device scalar arithmetic per stage).
 * ude_dopri_ratio: one attempt's error ratio and next step size on the device, status[0..2] (device fp64)
 * = [ratio, next dt, *flag (nullable: 0)]: ratio = max(|err[0] / (atol + rtol max(|y0[0]|, |y1[0]|))| (fp32
 * tolerance), sqrt(ssq[i * UDE_SUMSQ_WS] / n[i]) for the n_pieces <= 4 sums of ude_scaled_sumsq, extra[0 ..
 * n_extra)) (NaN-propagating), next dt = dt * 10 at ratio 0, else dt * clamp(0.9 / ratio^0.2, ratio < 1 ? 1 :
 * 0.2, 10) -- torchdiffeq's mixed norm and _optimal_step_size (torchdiffeq/_impl/rk_common.py), in
 * PyTorch's operation order; one host read per attempt.  Replace the per-attempt operator chains of the
 * adaptive controller (odeint_adjoint's fused backward). */
int ude_lincomb_hc(int64_t n, const float* base, const float* const* k, int32_t nk, const float* coef_host,
                   float* out, ude_stream_t stream);
int ude_dopri_ratio(const float* err, const float* y0, const float* y1, double atol, double rtol, const double* ssq,
                    const int64_t* n, int32_t n_pieces, const double* extra, int32_t n_extra, double dt,
                    const unsigned char* flag, double* status, ude_stream_t stream);

/* Library build tag (for logs / tests). */
const char* ude_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* UDE_RK4_H */
