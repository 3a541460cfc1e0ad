/* The VJP of the kernel-order forward, in REAL arithmetic -- TEST INFRASTRUCTURE ONLY (included by
 * oracle/ude_korder.c; see there).  Every linearisation point (stage input, pre-activation, rate, mask
 * decision) is the fp32 forward's own value. */

/* one evaluation (mlp() must have run on Y): df (3R, the cotangent of f) -> dY (3R, added), dstat
 * (R (L-3), added), the parameter gradients (added into gp, torch order; |terms| into ga when given) */
static void FN(eval_vjp)(const Prep* P, Work* w, const float* Y, const float* y0n, const REAL* df_in,
                         const REAL* ct, REAL* dY, REAL* dstat, REAL* gp, double* ga, REAL* xfull, REAL* const* gb,
                         REAL* const* gib, REAL* dYflux) {
  REAL* dYf = dYflux ? dYflux : dY;
  const KoModel* m = &P->m;
  const int R = m->R, L = m->L;
  for (int r = 0; r < R; ++r) {
    REAL df[3];
    for (int c = 0; c < 3; ++c) df[c] = masked(Y[3 * r + c]) ? (REAL)0 : df_in[3 * r + c];
    const REAL S = (REAL)Y[3 * r], I = (REAL)Y[3 * r + 1];
    if (P->has[0]) {
      const float* q = w->a[0][m->nl[0] - 1];
      const REAL b = (REAL)fabsf(q[2 * r]), gm = (REAL)fabsf(q[2 * r + 1]);
      const REAL dplus = -df[0] + df[1], dminus = -df[1] + df[2];
      const REAL db = dplus * S * I + ct[0] + ct[2] * (b - ct[4]);
      const REAL dg = dminus * I + ct[1] + ct[3] * (gm - ct[5]);
      dYf[3 * r] += dplus * b * I;
      dYf[3 * r + 1] += dplus * b * S + dminus * gm;
      const float q0 = q[2 * r], q1 = q[2 * r + 1];
      gb[0][2 * r] = db * (q0 > 0.f ? (REAL)1 : (q0 < 0.f ? (REAL)-1 : (REAL)0));     /* torch: sign(0) = 0 */
      gb[0][2 * r + 1] = dg * (q1 > 0.f ? (REAL)1 : (q1 < 0.f ? (REAL)-1 : (REAL)0));
    }
    if (P->has[1]) {
      const float* fa = w->a[1][m->nl[1] - 1];
      for (int c = 0; c < 3; ++c)
        gb[1][3 * r + c] = (P->has[0] ? (REAL)m->fa_w * df[c] : df[c]) + ct[6] * (REAL)fa[3 * r + c];
    }
  }
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < L; ++c) xfull[r * L + c] = c < 3 ? (REAL)Y[3 * r + c] : (REAL)y0n[r * L + c];
  for (int net = 0; net < 2; ++net) {
    if (!P->has[net]) continue;
    REAL* g = gb[net];
    REAL* gin = gib[net];
    for (int i = m->nl[net] - 1; i >= 0; --i) {
      const Layer* ly = &P->dyn[net][i];
      const int O = ly->O, In = ly->In;
      if (m->act[net][i]) {
        const float* z = w->z[net][i];
        const float* av = w->a[net][i];
        (void)av;
        for (int o = 0; o < O; ++o) g[o] *= z[o] > 0.f ? (REAL)1 : ELU_D(z[o], av[o]);
      }
      const float* ain = i > 0 ? w->a[net][i - 1] : NULL;
      REAL* xin = gin + In;                   /* this layer's input */
      for (int k = 0; k < In; ++k) xin[k] = ain ? (REAL)ain[k] : xfull[k];
      REAL* gw = gp + P->poff[net][i];
      REAL* gbias = gw + (size_t)O * In;
      double* aw = ga ? ga + P->poff[net][i] : NULL;
      for (int k = 0; k < In; ++k) gin[k] = 0;
      for (int o = 0; o < O; ++o) {
        const REAL go = g[o];
        gbias[o] += go;
        const double* wr = ly->wd + (size_t)o * In;   /* the fp32 weights (exact in double) */
        REAL* gr = gw + (size_t)o * In;
        for (int k = 0; k < In; ++k) {
          const REAL t = go * xin[k];
          gr[k] += t;
          gin[k] += (REAL)wr[k] * go;
        }
        if (aw) {
          double* ar = aw + (size_t)o * In;
          aw[(size_t)O * In + o] += fabs((double)go);
          for (int k = 0; k < In; ++k) ar[k] += fabs((double)go * (double)xin[k]);
        }
      }
      if (i > 0) {
        for (int k = 0; k < In; ++k) g[k] = gin[k];
      } else {
        for (int r = 0; r < R; ++r)
          for (int c = 0; c < L; ++c) {
            const REAL v = gin[r * L + c];
            if (c < 3) dY[3 * r + c] += v;
            else dstat[r * (L - 3) + c - 3] += v;
          }
      }
    }
  }
}

/* VJP of the kernel-order forward of N trajectories (REAL arithmetic).
 *   dlatent (T, N, R, L) fp64: the latent's cotangent (rounded to REAL);
 *   cot [7] = {dmean_0 / n, dmean_1 / n, dstd_0 / ((n-1) std_0), dstd_1 / ((n-1) std_1), mean_0, mean_1,
 *              d|Fa| / |Fa|} (the kernel's bwd_body coefficients, from the solve's own fp32 statistics);
 *   -> dy0 (N, R, L) fp64, the parameter gradient (torch order, fp64) and, when gabs is given, per
 *      parameter the sum of its terms' magnitudes (in fp64). */
int KO_VJP_NAME(const KoModel* m, const KoSched* sc, int N, const float* y0, const double* dlatent,
                const double* cot_in, double* dy0, double* gparams, double* gabs, int nthreads) {
  Prep P;
  prep_init(&P, m);
  const int F = P.F, RL = m->R * m->L, S = P.S, L = m->L, R = m->R;
  const size_t NRL = (size_t)N * RL;
  REAL cot[7];
  for (int c = 0; c < 7; ++c) cot[c] = (REAL)cot_in[c];
  if (nthreads > 0) omp_set_num_threads(nthreads);
  const int NT = omp_get_max_threads();
  const int n_tiles = (N + 15) / 16;
  REAL* tgp = (REAL*)calloc((size_t)NT * P.n_params, sizeof(REAL));
  double* tga = gabs ? (double*)calloc((size_t)NT * P.n_params, sizeof(double)) : NULL;
#pragma omp parallel
  {
    const int tn = omp_get_thread_num();
    REAL* gacc = tgp + (size_t)tn * P.n_params;
    double* ga = tga ? tga + (size_t)tn * P.n_params : NULL;
    REAL* gtile = (REAL*)calloc(P.n_params, sizeof(REAL));
    Work w;
    work_init(&w, &P);
    const int E = sc->n_steps * 4;
    float* X = (float*)malloc(sizeof(float) * ((size_t)E + 1) * F);
    double st[5];
    REAL* a = (REAL*)calloc(F, sizeof(REAL));
    REAL* pend = (REAL*)calloc(F, sizeof(REAL));
    REAL* dy = (REAL*)calloc(F, sizeof(REAL));
    REAL* dk[4];
    for (int j = 0; j < 4; ++j) dk[j] = (REAL*)calloc(F, sizeof(REAL));
    REAL* dYs = (REAL*)calloc(F, sizeof(REAL));
    REAL* dYf = (REAL*)calloc(F, sizeof(REAL));
    REAL* dstat = (REAL*)calloc(S > 0 ? S : 1, sizeof(REAL));
    REAL* xfull = (REAL*)calloc(RL, sizeof(REAL));
    REAL* gb[2];
    REAL* gib[2];
    for (int net = 0; net < 2; ++net) {
      gb[net] = (REAL*)calloc(P.maxw + RL, sizeof(REAL));
      gib[net] = (REAL*)calloc(2 * (P.maxw + RL), sizeof(REAL));
    }
#pragma omp for schedule(dynamic, 1)
    for (int tile = 0; tile < n_tiles; ++tile) {
      memset(gtile, 0, sizeof(REAL) * P.n_params);
      for (int n = tile * 16; n < N && n < tile * 16 + 16; ++n) {
        const float* y0n = y0 + (size_t)n * RL;
        traj_forward(&P, &w, sc, y0n, X, NULL, NULL, NRL, st);
        for (int i = 0; i < F; ++i) a[i] = 0;
        for (int s = 0; s < S; ++s) dstat[s] = 0;
        for (int st_ = sc->n_steps - 1; st_ >= 0; --st_) {
          const REAL dd = (REAL)sc->dt[st_];
        const REAL third = ko_third32 ? (REAL)(float)(1.0 / 3.0) : (REAL)(1.0 / 3.0);
          for (int i = 0; i < F; ++i) pend[i] = 0;
          for (int o = sc->out_start[st_]; o < sc->out_start[st_ + 1]; ++o) {
            const double* dl = dlatent + (size_t)sc->out_j[o] * NRL + (size_t)n * RL;
            const int mode = sc->out_mode[o];
            const REAL sl = (REAL)sc->out_slope[o];
            for (int r = 0; r < R; ++r)
              for (int c = 0; c < 3; ++c) {
                const REAL v = (REAL)dl[r * L + c];
                if (mode == 1) a[3 * r + c] += v;
                else if (mode == 0) pend[3 * r + c] += v;
                else { const REAL u = sl * v; a[3 * r + c] += u; pend[3 * r + c] += v - u; }
              }
          }
          for (int i = 0; i < F; ++i) {
            if (ko_assoc >= 1) {
              /* the kernel's association (bwd_body step start): accy = a, + pend at the step end */
              dy[i] = a[i];
              const REAL sdk = (a[i] * (REAL)0.125) * dd;
              dk[0][i] = sdk; dk[1][i] = (REAL)3 * sdk; dk[2][i] = (REAL)3 * sdk; dk[3][i] = sdk;
            } else {
              dy[i] = a[i] + pend[i];
              dk[0][i] = a[i] * dd * (REAL)0.125;
              dk[1][i] = (REAL)3 * a[i] * dd * (REAL)0.125;
              dk[2][i] = dk[1][i];
              dk[3][i] = dk[0][i];
            }
          }
          for (int j = 3; j >= 0; --j) {
            const float* Y = X + ((size_t)st_ * 4 + j) * F;
            mlp(&P, &w, Y);
            for (int i = 0; i < F; ++i) { dYs[i] = 0; dYf[i] = 0; }
            FN(eval_vjp)(&P, &w, Y, y0n, dk[j], cot, dYs, dstat, gtile, ga, xfull, gb, gib,
                         ko_assoc == 2 ? dYf : NULL);
            if (ko_assoc == 2) {
              /* the kernel's two updates per stage: the flux part (flux pass), then the MLP part */
              for (int i = 0; i < F; ++i) {
                const REAL v = dYf[i];
                dy[i] += v;
                if (j == 3) { const REAL u = dd * v; dk[0][i] += u; dk[1][i] -= u; dk[2][i] += u; }
                else if (j == 2) { const REAL u = dd * v; dk[1][i] += u; dk[0][i] -= u * third; }
                else if (j == 1) { dk[0][i] += (v * third) * dd; }
              }
            }
            for (int i = 0; i < F; ++i) {
              const REAL v = dYs[i];
              dy[i] += v;
              if (j == 3) { const REAL u = dd * v; dk[0][i] += u; dk[1][i] -= u; dk[2][i] += u; }
              else if (j == 2) { const REAL u = dd * v; dk[1][i] += u; dk[0][i] -= u * third; }
              else if (j == 1) { dk[0][i] += (v * third) * dd; }
            }
          }
          for (int i = 0; i < F; ++i) a[i] = ko_assoc >= 1 ? dy[i] + pend[i] : dy[i];
        }
        /* y0: the solve's adjoint, output 0 (= y0) and every output's static dims (carried unchanged) */
        double* d = dy0 + (size_t)n * RL;
        for (int r = 0; r < R; ++r)
          for (int c = 0; c < L; ++c) {
            REAL v = c < 3 ? a[3 * r + c] : dstat[r * (L - 3) + c - 3];
            v += (REAL)dlatent[(size_t)n * RL + r * L + c];
            if (c >= 3)
              for (int j = 1; j < sc->n_times; ++j) v += (REAL)dlatent[(size_t)j * NRL + (size_t)n * RL + r * L + c];
            d[r * L + c] = (double)v;
          }
      }
      for (int k = 0; k < P.n_params; ++k) gacc[k] += gtile[k];
    }
    free(X); free(a); free(pend); free(dy); free(dYs); free(dYf); free(dstat); free(xfull); free(gtile);
    for (int j = 0; j < 4; ++j) free(dk[j]);
    for (int net = 0; net < 2; ++net) { free(gb[net]); free(gib[net]); }
    work_free(&w, &P);
  }
  for (int k = 0; k < P.n_params; ++k) {
    REAL s = 0;
    double sa = 0.0;
    for (int t = 0; t < NT; ++t) {
      s += tgp[(size_t)t * P.n_params + k];
      if (tga) sa += tga[(size_t)t * P.n_params + k];
    }
    gparams[k] = (double)s;
    if (gabs) gabs[k] = sa;
  }
  free(tgp);
  free(tga);
  prep_free(&P);
  return 0;
}
