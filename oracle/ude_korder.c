/* Kernel-order oracle for the fused RK4 solve -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/ (through oracle/ude_korder.py) load this library, as a checker.  The product path never
 * does.  Build: oracle/Makefile (gcc, -ffp-contract=off: every fused multiply-add below is an explicit
 * fmaf, every other operation is rounded on its own, as on the GPU).
 *
 * What it restates.  The reference arithmetic is lib/models.py:109-265 (Fp / Fa / FaFp .forward)
 * under torchdiffeq's rk4 / rk4_alt_step_func, at lib/VAE.py:137.  oracle/ude_oracle.py restates it
 * in torch's operation order.  This file restates the SAME mathematics in the operation order that
 * the gfx950 kernels claim for their training forward (csrc/ude_kernels.h fwd_body / mlp_forward /
 * static_hoist).
 *
 *  - Every Linear is a chain of fp32 fused multiply-adds.  v_mfma_f32_16x16x4_f32 is an fmaf chain
 *    over its 4 K lanes, bitwise (MI355X_MICROARCH.md "exact f32 (== fmaf chain, bitwise)"; the lane
 *    order is checked on the GPU by tests/test_kernel_order.py).  Lane group g of the wave reads
 *    input feature g * KP/4 + 4q + e at quad q, element e.  So output o's chain visits, for q
 *    ascending, e ascending, g = 0..3, the feature k = g*KP/4 + 4q + e, with KP = pad16(in).
 *  - Layer 0 with static features (latent dims >= 3 have zero derivative, lib/models.py:144, :249)
 *    is the per-trajectory hoist c1 = b0 + W0[:, static] . x_static (chain over the static features
 *    in the record order s = r (L-3) + (c-3), K = pad16(R (L-3))), and per evaluation the chain over
 *    the dynamic features f = 3r + c (K = pad16(3R)) starting from c1.
 *  - ELU (lib/models.py:121-124): x > 0 ? x : expm1f(min(x, 0)), with expm1f = ROCm device-libs'
 *    __ocml_expm1_f32 restated operation by operation (ko_expm1f).
 *  - Flux (lib/models.py:138-146): plus = (|q0| S) I, minus = |q1| I, [-plus, plus - minus, minus];
 *    FaFp: f + fa_w Fa (lib/models.py:247); masked where a stage input leaves [-1, 2] (:130).
 *  - RK4 3/8 rule (torchdiffeq rk4_alt_step_func) with the state and the combinations in fp64 and
 *    every stage input rounded to fp32 (the kernel's fp64 state).
 *
 * The forward (ko_solve) is meant to be BITWISE equal to the kernel's: latent, every stage input and
 * so every mask decision.  The backward (ko_vjp) is the exact (fp64) vector-Jacobian product of that
 * fp32 forward at its own fp32 linearisation points -- every stage input, pre-activation, rate and
 * mask decision is the forward's fp32 value; every derivative and sum is formed in fp64.  The kernel's
 * fp32 backward must agree with it up to its own fp32 rounding: no mask flip, no different branch.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define MAXLIN 5

typedef struct {
  int kind;                    /* 1 Fp, 2 Fa, 3 FaFp (lib/models.py ode_type) */
  int R, L;
  float fa_w;
  int nl[2];                   /* Linears per net: [0] rate net ("net" / "Fp_net"), [1] aug_net */
  int in_dim[2][MAXLIN], out_dim[2][MAXLIN], act[2][MAXLIN];
  const float* w[2][MAXLIN];   /* nn.Linear layout (out, in), row-major; layer 0's in = R * L */
  const float* b[2][MAXLIN];
} KoModel;

typedef struct {
  int n_steps, n_out, n_times;
  const float* dt;             /* [n_steps] */
  const int* out_start;        /* [n_steps + 1] */
  const int* out_j;            /* [n_out] */
  const int* out_mode;         /* [n_out]: 0 y_n, 1 y_{n+1}, 2 linear interpolation */
  const float* out_slope;      /* [n_out] */
} KoSched;

static int pad16(int x) { return (x + 15) & ~15; }

static float fbits(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return (float)d;
}

/* __ocml_expm1_f32 (ROCm device libs, ocml.bc), operation by operation: range reduction by
 * rint(x log2 e), two-piece ln 2, a degree-7 polynomial on fmaf (llvm.fmuladd is an fma on gfx950),
 * reconstruction 2^k (1 + p) - 1 as one fmaf. */
float ko_expm1f(float x) {
  const float z = rintf(x * fbits(0x3FF7154760000000ull));
  const float nz = -z;
  float r = fmaf(nz, fbits(0x3FE62E4300000000ull), x);
  r = fmaf(nz, fbits(0xBE205C6100000000ull), r);
  float p = fmaf(r, fbits(0x3F2A267620000000ull), fbits(0x3F56D2E000000000ull));
  p = fmaf(r, p, fbits(0x3F8110FF20000000ull));
  p = fmaf(r, p, fbits(0x3FA5555020000000ull));
  p = fmaf(r, p, fbits(0x3FC5555560000000ull));
  p = fmaf(r, p, 0.5f);
  const float q = r * p;
  const float m = fmaf(r, q, r);
  const int big = z == 128.0f;
  const float s = big ? fbits(0x47E0000000000000ull) : ldexpf(1.0f, (int)z);
  const float sm1 = s + -1.0f;
  float v = fmaf(s, m, sm1);
  v = big ? v * 2.0f : v;
  v = x > fbits(0x40562E42E0000000ull) ? INFINITY : v;
  return x < -17.0f ? -1.0f : v;
}

static float elu1(float x) {
  const float e = ko_expm1f(fminf(x, 0.0f));
  return x > 0.0f ? x : e;
}

/* one v_mfma_f32_16x16x4_f32 output element: acc + sum_g a[g] b[g] as fmaf chain in lane-group order
 * perm[0..3] (the GPU probe test checks which order the hardware uses) */
void ko_mfma_elem(const float* a, const float* b, const int* perm, float* acc) {
  float c = *acc;
  for (int i = 0; i < 4; ++i) c = fmaf(a[perm[i]], b[perm[i]], c);
  *acc = c;
}

/* ------------------------------------------------------------------------------------------------ */
/* prepared model: per layer the chain order and the weights transposed into it                      */

typedef struct {
  int O, n;                    /* outputs, chain length (valid inputs only) */
  int* idx;                    /* [n] input index (record order) visited at chain position p */
  float* wc;                   /* [n][O] W[o][col(idx[p])] */
  double* wd;                  /* [O][In] W as double, torch layout (backward) */
  float* bias;                 /* [O] */
  int In;                      /* torch input width (layer 0: R L) */
} Layer;

typedef struct {
  KoModel m;
  int F, S, has[2];
  Layer dyn[2][MAXLIN];        /* layer 0: dynamic-feature chain; i > 0: the layer */
  Layer stat[2];               /* layer 0: static-feature chain (hoist) */
  int n_params, poff[2][MAXLIN];   /* torch order: w then b per layer, net 0 first */
  int maxw;
} Prep;

static int col_dyn(const KoModel* m, int f) { return (f / 3) * m->L + (f % 3); }
static int col_stat(const KoModel* m, int s) { return (s / (m->L - 3)) * m->L + 3 + s % (m->L - 3); }

/* chain over K = KP (padded) inputs with `valid` of them live, in the MFMA order (q, e, g) */
static void build_chain(Layer* ly, const KoModel* m, int net, int i, int valid, int KP, int kind) {
  const int KQ = KP / 4;
  const float* W = m->w[net][i];
  const int In = m->in_dim[net][i];
  ly->O = m->out_dim[net][i];
  ly->In = In;
  ly->idx = (int*)malloc(sizeof(int) * (valid > 0 ? valid : 1));
  ly->wc = (float*)malloc(sizeof(float) * (size_t)(valid > 0 ? valid : 1) * ly->O);
  int n = 0;
  for (int q = 0; q < KP / 16; ++q)
    for (int e = 0; e < 4; ++e)
      for (int g = 0; g < 4; ++g) {
        const int k = g * KQ + 4 * q + e;
        if (k >= valid) continue;
        const int col = kind == 0 ? k : (kind == 1 ? col_dyn(m, k) : col_stat(m, k));
        ly->idx[n] = k;
        for (int o = 0; o < ly->O; ++o) ly->wc[(size_t)n * ly->O + o] = W[(size_t)o * In + col];
        ++n;
      }
  ly->n = n;
  ly->wd = (double*)malloc(sizeof(double) * (size_t)ly->O * In);
  for (size_t j = 0; j < (size_t)ly->O * In; ++j) ly->wd[j] = (double)W[j];
  ly->bias = (float*)malloc(sizeof(float) * ly->O);
  for (int o = 0; o < ly->O; ++o) ly->bias[o] = m->b[net][i][o];
}

static void prep_init(Prep* P, const KoModel* m) {
  memset(P, 0, sizeof(*P));
  P->m = *m;
  P->F = 3 * m->R;
  P->S = m->R * (m->L - 3);
  int off = 0;
  for (int net = 0; net < 2; ++net) {
    P->has[net] = m->nl[net] > 0;
    for (int i = 0; i < m->nl[net]; ++i) {
      P->poff[net][i] = off;
      off += m->out_dim[net][i] * m->in_dim[net][i] + m->out_dim[net][i];
      if (m->out_dim[net][i] > P->maxw) P->maxw = m->out_dim[net][i];
      if (m->in_dim[net][i] > P->maxw) P->maxw = m->in_dim[net][i];
      if (i == 0) {
        build_chain(&P->dyn[net][0], m, net, 0, P->F, pad16(P->F), 1);
        build_chain(&P->stat[net], m, net, 0, P->S, pad16(P->S), 2);
      } else {
        build_chain(&P->dyn[net][i], m, net, i, m->in_dim[net][i], pad16(m->in_dim[net][i]), 0);
      }
    }
  }
  P->n_params = off;
}

static void layer_free(Layer* l) { free(l->idx); free(l->wc); free(l->wd); free(l->bias); }

static void prep_free(Prep* P) {
  for (int net = 0; net < 2; ++net) {
    for (int i = 0; i < P->m.nl[net]; ++i) layer_free(&P->dyn[net][i]);
    if (P->has[net]) layer_free(&P->stat[net]);
  }
}

/* out[o] = acc0[o] + chain  (fmaf, chain order) */
static void chain_apply(const Layer* ly, const float* x, float* acc) {
  const int O = ly->O;
  for (int p = 0; p < ly->n; ++p) {
    const float xv = x[ly->idx[p]];
    const float* wr = ly->wc + (size_t)p * O;
    for (int o = 0; o < O; ++o) acc[o] = fmaf(wr[o], xv, acc[o]);
  }
}

/* per-trajectory scratch of one evaluation: every layer's pre-activation z and output a (fp32) */
typedef struct {
  float* z[2][MAXLIN];
  float* a[2][MAXLIN];
  float* c1[2];                /* hoisted layer-0 start values */
  float* xs;                   /* static features, record order [S] */
  double* g[2];                /* backward work vectors */
  double* gin[2];
} Work;

static void work_init(Work* w, const Prep* P) {
  memset(w, 0, sizeof(*w));
  for (int net = 0; net < 2; ++net) {
    for (int i = 0; i < P->m.nl[net]; ++i) {
      w->z[net][i] = (float*)calloc(P->m.out_dim[net][i], sizeof(float));
      w->a[net][i] = (float*)calloc(P->m.out_dim[net][i], sizeof(float));
    }
    if (P->has[net]) w->c1[net] = (float*)calloc(P->m.out_dim[net][0], sizeof(float));
    /* g: a layer's output cotangent; gin: its input cotangent, then the input itself (2 x In) */
    w->g[net] = (double*)calloc(P->maxw + P->m.R * P->m.L, sizeof(double));
    w->gin[net] = (double*)calloc(2 * (P->maxw + P->m.R * P->m.L), sizeof(double));
  }
  w->xs = (float*)calloc(P->S > 0 ? P->S : 1, sizeof(float));
}

static void work_free(Work* w, const Prep* P) {
  for (int net = 0; net < 2; ++net) {
    for (int i = 0; i < P->m.nl[net]; ++i) { free(w->z[net][i]); free(w->a[net][i]); }
    free(w->c1[net]); free(w->g[net]); free(w->gin[net]);
  }
  free(w->xs);
}

/* the tile-start hoist of one trajectory: c1 = b0 + W0[:, static] . x_static */
static void hoist(const Prep* P, Work* w, const float* y0n) {
  const KoModel* m = &P->m;
  for (int s = 0; s < P->S; ++s) w->xs[s] = y0n[(s / (m->L - 3)) * m->L + 3 + s % (m->L - 3)];
  for (int net = 0; net < 2; ++net) {
    if (!P->has[net]) continue;
    const Layer* ly = &P->stat[net];
    memcpy(w->c1[net], ly->bias, sizeof(float) * ly->O);
    chain_apply(ly, w->xs, w->c1[net]);
  }
}

/* both MLPs on the stage input x (record order [F]) */
static void mlp(const Prep* P, Work* w, const float* x) {
  const KoModel* m = &P->m;
  for (int net = 0; net < 2; ++net) {
    if (!P->has[net]) continue;
    for (int i = 0; i < m->nl[net]; ++i) {
      const Layer* ly = &P->dyn[net][i];
      float* z = w->z[net][i];
      memcpy(z, i == 0 ? w->c1[net] : ly->bias, sizeof(float) * ly->O);
      chain_apply(ly, i == 0 ? x : w->a[net][i - 1], z);
      float* a = w->a[net][i];
      if (m->act[net][i])
        for (int o = 0; o < ly->O; ++o) a[o] = elu1(z[o]);
      else
        memcpy(a, z, sizeof(float) * ly->O);
    }
  }
}

static int masked(float v) { return v > 2.0f || v < -1.0f; }

/* the flux of one evaluation (fp32, the kernel's operation order); st: fp64 side sums */
static void flux(const Prep* P, Work* w, const float* Y, float* f, double* st, int valid) {
  const KoModel* m = &P->m;
  const int R = m->R;
  for (int r = 0; r < R; ++r) {
    float fr[3] = {0.f, 0.f, 0.f};
    if (P->has[0]) {
      const float* q = w->a[0][m->nl[0] - 1];
      const float b = fabsf(q[2 * r]), gm = fabsf(q[2 * r + 1]);
      const float plus = (b * Y[3 * r]) * Y[3 * r + 1];
      const float minus = gm * Y[3 * r + 1];
      fr[0] = -plus; fr[1] = plus - minus; fr[2] = minus;
      if (valid) {
        st[0] += (double)b; st[1] += (double)gm;
        st[2] += (double)b * (double)b; st[3] += (double)gm * (double)gm;
      }
    }
    if (P->has[1]) {
      const float* fa = w->a[1][m->nl[1] - 1];
      for (int c = 0; c < 3; ++c) {
        const float v = fa[3 * r + c];
        if (P->has[0]) {
          const float t = m->fa_w * v;
          fr[c] = fr[c] + t;
        } else {
          fr[c] = v;
        }
        if (valid) st[4] += (double)v * (double)v;
      }
    }
    for (int c = 0; c < 3; ++c) f[3 * r + c] = masked(Y[3 * r + c]) ? 0.0f : fr[c];
  }
}

/* ko_state32: the RK4 state and the 3/8-rule combinations in fp32, in torchdiffeq's operation order
 * (rk4_alt_step_func: y0 + dt * k1 * 1/3, y0 + dt * (k2 - k1 * 1/3), y0 + dt * (k1 - k2 + k3),
 * y0 + (k1 + 3 * (k2 + k3) + k4) * dt * 0.125, the python scalars applied as fp32) -- the reference's
 * integrator arithmetic around the kernel's MLP order (a sample of the fp32 reference arithmetic that
 * differs from the kernel only in the state precision) */
static int ko_state32 = 0;
void ko_set_state32(int v) { ko_state32 = v; }

/* one trajectory's forward: stage inputs X [n_steps * 4][F] (fp32), states ys [(n_steps + 1)][F]
 * (fp64), outputs written into lat (stride NRL per output time), side sums into st */
static void traj_forward(const Prep* P, Work* w, const KoSched* sc, const float* y0n, float* X, double* ys,
                         float* lat, size_t NRL, double* st) {
  const KoModel* m = &P->m;
  const int F = P->F, R = m->R, L = m->L;
  float* k1 = (float*)alloca(sizeof(float) * F);
  float* k2 = (float*)alloca(sizeof(float) * F);
  float* k3 = (float*)alloca(sizeof(float) * F);
  float* f = (float*)alloca(sizeof(float) * F);
  float* Yc = (float*)alloca(sizeof(float) * F);
  float* yold = (float*)alloca(sizeof(float) * F);
  double* y = (double*)alloca(sizeof(double) * F);
  hoist(P, w, y0n);
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < 3; ++c) { Yc[3 * r + c] = y0n[r * L + c]; y[3 * r + c] = (double)y0n[r * L + c]; }
  if (ys) memcpy(ys, y, sizeof(double) * F);
  if (lat) {
    for (int j = 0; j < sc->n_times; ++j)
      for (int r = 0; r < R; ++r)
        for (int c = (j == 0 ? 0 : 3); c < L; ++c) lat[(size_t)j * NRL + r * L + c] = y0n[r * L + c];
  }
  for (int n = 0; n < sc->n_steps; ++n) {
    const double dd = (double)sc->dt[n];
    for (int j = 0; j < 4; ++j) {
      if (X) memcpy(X + ((size_t)n * 4 + j) * F, Yc, sizeof(float) * F);
      mlp(P, w, Yc);
      flux(P, w, Yc, f, st, 1);
      if (ko_state32) {
        const float dtf = sc->dt[n], third = (float)(1.0 / 3.0);
        for (int i = 0; i < F; ++i) {
          const float yf = (float)y[i];                /* exact: the fp32 state */
          if (j == 0) { k1[i] = f[i]; Yc[i] = yf + (dtf * f[i]) * third; }
          else if (j == 1) { k2[i] = f[i]; Yc[i] = yf + dtf * (f[i] - k1[i] * third); }
          else if (j == 2) { k3[i] = f[i]; Yc[i] = yf + dtf * ((k1[i] - k2[i]) + f[i]); }
        }
      } else
      for (int i = 0; i < F; ++i) {
        if (j == 0) {
          k1[i] = f[i];
          Yc[i] = (float)(y[i] + (dd * (double)f[i]) * (1.0 / 3.0));
        } else if (j == 1) {
          k2[i] = f[i];
          Yc[i] = (float)(y[i] + dd * ((double)f[i] - (double)k1[i] * (1.0 / 3.0)));
        } else if (j == 2) {
          k3[i] = f[i];
          Yc[i] = (float)(y[i] + dd * (((double)k1[i] - (double)k2[i]) + (double)f[i]));
        }
      }
      if (j == 3) {
        for (int i = 0; i < F; ++i) {
          yold[i] = (float)y[i];
          if (ko_state32) {
            const float y1 = yold[i] + (((k1[i] + 3.0f * (k2[i] + k3[i])) + f[i]) * sc->dt[n]) * 0.125f;
            y[i] = (double)y1;
          } else {
            const double dy = ((((double)k1[i] + 3.0 * ((double)k2[i] + (double)k3[i])) + (double)f[i]) * dd) * 0.125;
            y[i] = y[i] + dy;
          }
          Yc[i] = (float)y[i];
        }
        if (ys) memcpy(ys + (size_t)(n + 1) * F, y, sizeof(double) * F);
        if (lat) {
          for (int o = sc->out_start[n]; o < sc->out_start[n + 1]; ++o) {
            const int jo = sc->out_j[o], mode = sc->out_mode[o];
            const float slope = sc->out_slope[o];
            for (int r = 0; r < R; ++r)
              for (int c = 0; c < 3; ++c) {
                const int i = 3 * r + c;
                float v;
                if (mode == 0) v = yold[i];
                else if (mode == 1) v = Yc[i];
                else v = yold[i] + slope * (Yc[i] - yold[i]);
                lat[(size_t)jo * NRL + r * L + c] = v;
              }
          }
        }
      }
    }
  }
}

/* Forward solve of N trajectories (y0 (N, R, L) fp32): latent (T, N, R, L) fp32 (nullable), every
 * stage input X (n_steps * 4, N, 3R) fp32 (nullable) and the fp64 side sums [sum b, sum g, sum b^2,
 * sum g^2, sum Fa^2] (summed per trajectory, then over trajectories in order). */
int ko_solve(const KoModel* m, const KoSched* sc, int N, const float* y0, float* latent, float* stage_in,
             double* sums, int nthreads) {
  Prep P;
  prep_init(&P, m);
  const int F = P.F, RL = m->R * m->L;
  const size_t NRL = (size_t)N * RL;
  double* part = (double*)calloc((size_t)N * 5, sizeof(double));
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
    Work w;
    work_init(&w, &P);
    float* X = (float*)malloc(sizeof(float) * ((size_t)sc->n_steps * 4 + 1) * F);
#pragma omp for schedule(dynamic, 8)
    for (int n = 0; n < N; ++n) {
      traj_forward(&P, &w, sc, y0 + (size_t)n * RL, stage_in ? X : NULL, NULL,
                   latent ? latent + (size_t)n * RL : NULL, NRL, part + (size_t)n * 5);
      if (stage_in)
        for (int e = 0; e < sc->n_steps * 4; ++e)
          memcpy(stage_in + ((size_t)e * N + n) * F, X + (size_t)e * F, sizeof(float) * F);
    }
    free(X);
    work_free(&w, &P);
  }
  for (int c = 0; c < 5; ++c) {
    double s = 0.0;
    for (int n = 0; n < N; ++n) s += part[(size_t)n * 5 + c];
    sums[c] = s;
  }
  free(part);
  prep_free(&P);
  return 0;
}

/* association variant of the fp32 VJP's RK adjoint (0: the oracle's, 1: the kernel's bwd_body) */
static int ko_assoc = 0;
void ko_set_assoc(int v) { ko_assoc = v; }
/* development knob: the backward's 1/3 as the fp32 constant (the kernel's 1.0f / 3.0f) */
static int ko_third32 = 0;
void ko_set_third32(int v) { ko_third32 = v; }

/* ---- backward ------------------------------------------------------------------------------------ */
/* ude_korder_vjp.h, twice: REAL = double -- the exact VJP (ko_vjp) -- and REAL = float -- the same VJP
 * executed in fp32 (ko_vjp32): trajectories grouped in tiles of 16 whose weight-gradient terms are
 * summed in fp32 per tile, then the tiles in fp32, like the kernel's per-workgroup register
 * accumulators and slab reduction (not its exact order).  Its distance to the exact VJP is the size
 * of fp32 backward rounding on the very same forward. */
#define REAL double
#define FN(x) x##_d
#define ELU_D(z, a) exp((double)(z))   /* the exact derivative at the fp32 pre-activation */
#define KO_VJP_NAME ko_vjp
#include "ude_korder_vjp.h"
#undef REAL
#undef FN
#undef ELU_D
#undef KO_VJP_NAME
#define REAL float
#define FN(x) x##_f
#define ELU_D(z, a) ((a) + 1.0f)     /* torch's elu_backward on the result (nn.ELU(inplace=True),
                                        lib/models.py:121), and the kernel's: out + alpha, in fp32 */
#define KO_VJP_NAME ko_vjp32
#include "ude_korder_vjp.h"
#undef REAL
#undef FN
#undef ELU_D
#undef KO_VJP_NAME

int ko_n_params(const KoModel* m) {
  int off = 0;
  for (int net = 0; net < 2; ++net)
    for (int i = 0; i < m->nl[net]; ++i) off += m->out_dim[net][i] * m->in_dim[net][i] + m->out_dim[net][i];
  return off;
}

void ko_expm1f_array(const float* x, float* y, long n) {
  for (long i = 0; i < n; ++i) y[i] = ko_expm1f(x[i]);
}

/* compare y[i] against ko_expm1f of the float with bit pattern start + i: number of bitwise
 * mismatches, the first one's index in *first (-1 if none) */
long ko_expm1f_compare_bits(uint32_t start, long n, const float* y, long* first) {
  long bad = 0, fb = -1;
#pragma omp parallel for reduction(+ : bad) schedule(static)
  for (long i = 0; i < n; ++i) {
    uint32_t u = start + (uint32_t)i;
    float x;
    memcpy(&x, &u, 4);
    const float v = ko_expm1f(x);
    if (memcmp(&v, y + i, 4) != 0) {
      ++bad;
#pragma omp critical
      if (fb < 0 || i < fb) fb = i;
    }
  }
  *first = fb;
  return bad;
}
