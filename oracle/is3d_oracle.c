/*
 * is3d_oracle.c -- TEST INFRASTRUCTURE ONLY (see is3d_oracle.h).
 *
 * A plain-C, race-free restatement of iS3D2's continuous-spectra path, kept
 * deliberately close to the reference loop structure and expression order so
 * that it reproduces the reference numbers to rounding.  Every function cites
 * the reference file:line it follows.  Never linked by the product.
 */
#include "is3d_oracle.h"
#include "../include/is3d_gl16.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* iS3D.h:14-17 */
#define HBARC 0.197327053
static double two_pi2_hbarC3(void) { return 2.0 * pow(M_PI, 2) * pow(HBARC, 3); }
static double four_pi2_hbarC3(void) { return 4.0 * pow(M_PI, 2) * pow(HBARC, 3); }

static void seterr(char *err, int n, const char *msg) {
  if (err && n > 0) { strncpy(err, msg, (size_t)n - 1); err[n - 1] = 0; }
}

/* ------------------------------------------------------------------------- */
/* GSL natural cubic spline (gsl_interp_cspline), restated.                   */
/* cspline.c cspline_init + linalg/tridiag.c solve_tridiag (symmetric case).  */
/* ------------------------------------------------------------------------- */
typedef struct { int n; const double *x; const double *y; double *c; } cspline;

static int cspline_init(cspline *s, const double *x, const double *y, int n) {
  s->n = n; s->x = x; s->y = y;
  s->c = (double *)calloc((size_t)n, sizeof(double));
  for (int i = 0; i + 1 < n; i++) if (!(x[i] < x[i + 1])) return -1; /* gsl_interp_init EINVAL */
  int sys = n - 2;
  s->c[0] = 0.0; s->c[n - 1] = 0.0;
  if (sys <= 0) return 0;
  double *g = (double *)malloc(sizeof(double) * sys), *diag = (double *)malloc(sizeof(double) * sys);
  double *off = (double *)malloc(sizeof(double) * sys);
  for (int i = 0; i < sys; i++) {
    const double h_i = x[i + 1] - x[i], h_ip1 = x[i + 2] - x[i + 1];
    const double yd_i = y[i + 1] - y[i], yd_ip1 = y[i + 2] - y[i + 1];
    const double g_i = (h_i != 0.0) ? 1.0 / h_i : 0.0;
    const double g_ip1 = (h_ip1 != 0.0) ? 1.0 / h_ip1 : 0.0;
    off[i] = h_ip1;
    diag[i] = 2.0 * (h_ip1 + h_i);
    g[i] = 3.0 * (yd_ip1 * g_ip1 - yd_i * g_i);
  }
  if (sys == 1) {
    s->c[1] = g[0] / diag[0];
  } else {
    /* symmetric tridiagonal: A = L D L^T (gamma = sub-diag of L, alpha = D) */
    int N = sys;
    double *gamma = (double *)malloc(sizeof(double) * N), *alpha = (double *)malloc(sizeof(double) * N);
    double *cc = (double *)malloc(sizeof(double) * N), *z = (double *)malloc(sizeof(double) * N);
    alpha[0] = diag[0];
    gamma[0] = off[0] / alpha[0];
    for (int i = 1; i < N - 1; i++) {
      alpha[i] = diag[i] - off[i - 1] * gamma[i - 1];
      gamma[i] = off[i] / alpha[i];
    }
    alpha[N - 1] = diag[N - 1] - off[N - 2] * gamma[N - 2];
    z[0] = g[0];
    for (int i = 1; i < N; i++) z[i] = g[i] - gamma[i - 1] * z[i - 1];
    for (int i = 0; i < N; i++) cc[i] = z[i] / alpha[i];
    double *xs = s->c + 1;
    xs[N - 1] = cc[N - 1];
    for (int i = N - 2; i >= 0; i--) xs[i] = cc[i] - gamma[i] * xs[i + 1];
    free(gamma); free(alpha); free(cc); free(z);
  }
  free(g); free(diag); free(off);
  return 0;
}

static size_t bsearch_idx(const double *xa, double x, size_t lo, size_t hi) {
  while (hi > lo + 1) { size_t i = (hi + lo) / 2; if (xa[i] > x) hi = i; else lo = i; }
  return lo;
}

/* gsl_spline_eval: range check (interp.c) + cspline_eval/coeff_calc (cspline.c) */
static double cspline_eval(const cspline *s, double x, int *bad) {
  if (x < s->x[0] || x > s->x[s->n - 1]) { *bad = 1; return NAN; }
  size_t i = bsearch_idx(s->x, x, 0, (size_t)s->n - 1);
  const double x_hi = s->x[i + 1], x_lo = s->x[i], dx = x_hi - x_lo;
  if (!(dx > 0.0)) return 0.0;
  const double y_lo = s->y[i], y_hi = s->y[i + 1], dy = y_hi - y_lo, delx = x - x_lo;
  const double c_i = s->c[i], c_ip1 = s->c[i + 1];
  const double b_i = (dy / dx) - dx * (c_ip1 + 2.0 * c_i) / 3.0;
  const double d_i = (c_ip1 - c_i) / (3.0 * dx);
  return y_lo + delx * (b_i + delx * (c_i + delx * d_i));
}

/* ------------------------------------------------------------------------- */
/* GaussThermal.cpp:7-130                                                     */
/* ------------------------------------------------------------------------- */
enum { GT_NEQ = 0, GT_J10, GT_J11, GT_J20, GT_J30, GT_J31 };
enum { GM_E = 0, GM_P };

static double thermal_integrand(int kind, double pbar, double mbar, double alphaB, double baryon, double sign) {
  double Ebar = sqrt(pbar * pbar + mbar * mbar);
  switch (kind) {
    case GT_NEQ: return pbar * exp(pbar) / (exp(Ebar - baryon * alphaB) + sign);
    case GT_J10: { double q = exp(Ebar - baryon * alphaB) + sign;
                   return pbar * exp(pbar + Ebar - baryon * alphaB) / (q * q); }
    case GT_J11: { double q = exp(Ebar - baryon * alphaB) + sign;
                   return pbar * pbar * pbar / (Ebar * Ebar) * exp(pbar + Ebar - baryon * alphaB) / (q * q); }
    case GT_J20: { double q = exp(Ebar - baryon * alphaB) + sign;
                   return Ebar * exp(pbar + Ebar - baryon * alphaB) / (q * q); }
    case GT_J30: { double q = exp(Ebar - baryon * alphaB) + sign;
                   return Ebar * Ebar / pbar * exp(pbar + Ebar - baryon * alphaB) / (q * q); }
    default:     { double q = exp(Ebar - baryon * alphaB) + sign;
                   return pbar * exp(pbar + Ebar - baryon * alphaB) / (q * q); }
  }
}

double orc_gauss_thermal(int kind, const double *root, const double *weight, int pts,
                         double mbar, double alphaB, double baryon, double sign) {
  double integral = 0.0;
  for (int k = 0; k < pts; k++) integral += weight[k] * thermal_integrand(kind, root[k], mbar, alphaB, baryon, sign);
  return integral;
}

static double mod_integrand(int kind, double pbar, double mbar, double lambda, double sign) {
  double scale2 = (1.0 + lambda) * (1.0 + lambda);
  double Ebar = sqrt(pbar * pbar + mbar * mbar);
  if (kind == GM_E) return sqrt(pbar * pbar * scale2 + mbar * mbar) * exp(pbar) / (exp(Ebar) + sign);
  return pbar * pbar * scale2 / sqrt(pbar * pbar * scale2 + mbar * mbar) * exp(pbar) / (exp(Ebar) + sign);
}

double orc_gauss1d_mod(int kind, const double *root, const double *weight, int pts,
                       double mbar, double lambda, double sign) {
  double sum = 0.0;
  for (int k = 0; k < pts; k++) sum += weight[k] * mod_integrand(kind, root[k], mbar, lambda, sign);
  return sum;
}

/* ------------------------------------------------------------------------- */
/* LocalRestFrame.cpp:12-41, 133-154, 173-185                                 */
/* ------------------------------------------------------------------------- */
typedef struct { double Xt, Xx, Xy, Xn, Yx, Yy, Zt, Zn; } milne;

static milne milne_basis(double ut, double ux, double uy, double un, double uperp, double utperp, double tau) {
  milne b;
  double sinhL = tau * un / utperp, coshL = ut / utperp;
  b.Xt = uperp * coshL; b.Xx = 1; b.Xy = 0; b.Xn = uperp * sinhL / tau;
  b.Yx = 0; b.Yy = 1;
  b.Zt = sinhL; b.Zn = coshL / tau;
  if (uperp > 1.e-5) {
    b.Xx = utperp * ux / uperp; b.Xy = utperp * uy / uperp;
    b.Yx = -uy / uperp; b.Yy = ux / uperp;
  }
  return b;
}

typedef struct { double xx, xy, xz, yy, yz, zz; } pilrf;

static pilrf boost_pimunu(milne b, double tau2, double pitt, double pitx, double pity, double pitn,
                          double pixx, double pixy, double pixn, double piyy, double piyn, double pinn) {
  pilrf r;
  double Xt = b.Xt, Xx = b.Xx, Xy = b.Xy, Xn = b.Xn, Yx = b.Yx, Yy = b.Yy, Zt = b.Zt, Zn = b.Zn;
  r.xx = pitt * Xt * Xt + pixx * Xx * Xx + piyy * Xy * Xy + tau2 * tau2 * pinn * Xn * Xn
       + 2.0 * (-Xt * (pitx * Xx + pity * Xy) + pixy * Xx * Xy + tau2 * Xn * (pixn * Xx + piyn * Xy - pitn * Xt));
  r.xy = Yx * (-pitx * Xt + pixx * Xx + pixy * Xy + tau2 * pixn * Xn) + Yy * (-pity * Xt + pixy * Xx + piyy * Xy + tau2 * piyn * Xn);
  r.xz = Zt * (pitt * Xt - pitx * Xx - pity * Xy - tau2 * pitn * Xn) - tau2 * Zn * (pitn * Xt - pixn * Xx - piyn * Xy - tau2 * pinn * Xn);
  r.yy = pixx * Yx * Yx + 2.0 * pixy * Yx * Yy + piyy * Yy * Yy;
  r.yz = -Zt * (pitx * Yx + pity * Yy) + tau2 * Zn * (pixn * Yx + piyn * Yy);
  r.zz = -(r.xx + r.yy);
  return r;
}

/* in[15]: ut ux uy un tau pitt pitx pity pitn pixx pixy pixn piyy piyn pinn
 * out[14]: Xt Xx Xy Xn Yx Yy Zt Zn pixx_LRF pixy_LRF pixz_LRF piyy_LRF piyz_LRF pizz_LRF */
void orc_milne_lrf(const double *in, double *out) {
  double ut = in[0], ux = in[1], uy = in[2], un = in[3], tau = in[4];
  double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
  milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  pilrf r = boost_pimunu(b, tau * tau, in[5], in[6], in[7], in[8], in[9], in[10], in[11], in[12], in[13], in[14]);
  double o[14] = {b.Xt, b.Xx, b.Xy, b.Xn, b.Yx, b.Yy, b.Zt, b.Zn, r.xx, r.xy, r.xz, r.yy, r.yz, r.zz};
  memcpy(out, o, sizeof(o));
}

/* ------------------------------------------------------------------------- */
/* 3x3 LU with partial pivoting (gsl_linalg_LU_decomp / _solve / _invert)     */
/* ------------------------------------------------------------------------- */
static void lu3_decomp(double A[9], int perm[3]) {
  for (int i = 0; i < 3; i++) perm[i] = i;
  for (int j = 0; j < 3; j++) {
    int piv = j; double mx = fabs(A[3 * j + j]);
    for (int i = j + 1; i < 3; i++) if (fabs(A[3 * i + j]) > mx) { mx = fabs(A[3 * i + j]); piv = i; }
    if (piv != j) {
      for (int k = 0; k < 3; k++) { double t = A[3 * j + k]; A[3 * j + k] = A[3 * piv + k]; A[3 * piv + k] = t; }
      int t = perm[j]; perm[j] = perm[piv]; perm[piv] = t;
    }
    double ajj = A[3 * j + j];
    if (ajj != 0.0) {
      for (int i = j + 1; i < 3; i++) {
        double aij = A[3 * i + j] / ajj;
        A[3 * i + j] = aij;
        for (int k = j + 1; k < 3; k++) A[3 * i + k] -= aij * A[3 * j + k];
      }
    }
  }
}

static void lu3_solve(const double LU[9], const int perm[3], const double b[3], double x[3]) {
  double y[3];
  for (int i = 0; i < 3; i++) y[i] = b[perm[i]];
  for (int i = 0; i < 3; i++) { double s = y[i]; for (int k = 0; k < i; k++) s -= LU[3 * i + k] * y[k]; y[i] = s; }
  for (int i = 2; i >= 0; i--) { double s = y[i]; for (int k = i + 1; k < 3; k++) s -= LU[3 * i + k] * x[k]; x[i] = s / LU[3 * i + i]; }
}

static void inverse3(const double A[9], double Ainv[3][3]) {
  double LU[9]; int perm[3];
  memcpy(LU, A, sizeof(LU));
  lu3_decomp(LU, perm);
  for (int j = 0; j < 3; j++) {
    double e[3] = {0, 0, 0}, col[3];
    e[j] = 1.0;
    lu3_solve(LU, perm, e, col);
    for (int i = 0; i < 3; i++) Ainv[i][j] = col[i];
  }
}

/* test hook (tests/test_oracle_gsl_pins.py): the restated gsl_linalg_LU_decomp + gsl_linalg_LU_solve on one 3x3
   system A x = b (A row-major); perm = the row permutation the decomposition chose */
void orc_lu3_solve(const double *A, const double *b, double *x, int *perm) {
  double LU[9];
  memcpy(LU, A, sizeof(LU));
  lu3_decomp(LU, perm);
  lu3_solve(LU, perm, b, x);
}

/* Arsenal.cpp:167-208 */
static void matvec3(double M[3][3], const double x[3], double y[3]) {
  for (int i = 0; i < 3; i++) { y[i] = 0; for (int j = 0; j < 3; j++) y[i] += M[i][j] * x[j]; }
}

/* ------------------------------------------------------------------------- */
/* Deltaf_Data (DeltafData.cpp)                                               */
/* ------------------------------------------------------------------------- */
typedef struct {
  double c0, c1, c2, c3, c4, shear14, F, G, betabulk, betaV, betapi, lambda, z, delta_lambda, delta_z;
} dfcoef;

typedef struct {
  int df_mode, include_baryon;
  int nT, nmuB;
  const double *T, *muB, *tab;
  double T_min, muB_min, dT, dmuB;
  cspline c0, c2, c3, F, betabulk, betaV, betapi, lambda2, z;
  double *jl2, *jz, *jx;
  double bulkPi_over_Peq_max;
  int have_splines, have_jonah;
} dfdata;

#define TAB(d, k, iB, iT) ((d)->tab[((size_t)(k) * (d)->nmuB + (iB)) * (d)->nT + (iT)])
enum { K_C0 = 0, K_C1, K_C2, K_C3, K_C4, K_F, K_G, K_BB, K_BV, K_BP };

/* DeltafData.cpp:220-295 compute_jonah_coefficients */
static int jonah(dfdata *d, const orc_setup *s) {
  const int pts = 301;
  const double lmin = -1.0, lmax = 2.0, dl = (lmax - lmin) / ((double)pts - 1.0);
  d->jl2 = (double *)calloc(pts, sizeof(double));
  d->jz = (double *)calloc(pts, sizeof(double));
  d->jx = (double *)calloc(pts, sizeof(double));
  d->bulkPi_over_Peq_max = -1.0;
  const double T = s->T_avg;
  const double *r2 = s->gla_root + 2 * s->gla_points, *w2 = s->gla_weight + 2 * s->gla_points;
  for (int i = 0; i < pts; i++) {
    double lambda = lmin + (double)i * dl;
    double E = 0.0, P = 0.0, Em = 0.0, Pm = 0.0;
    for (int n = 0; n < s->npdg; n++) {
      double g = s->pdg_degen[n], mass = s->pdg_mass[n], sign = s->pdg_sign[n];
      double mbar = mass / T;
      if (mass == 0.0) continue;
      E += g * orc_gauss1d_mod(GM_E, r2, w2, s->gla_points, mbar, 0.0, sign);
      P += (1.0 / 3.0) * g * orc_gauss1d_mod(GM_P, r2, w2, s->gla_points, mbar, 0.0, sign);
      Em += g * orc_gauss1d_mod(GM_E, r2, w2, s->gla_points, mbar, lambda, sign);
      Pm += (1.0 / 3.0) * g * orc_gauss1d_mod(GM_P, r2, w2, s->gla_points, mbar, lambda, sign);
    }
    double z = E / Em;
    double bp = (Pm / P) * z - 1.0;
    d->jl2[i] = lambda * lambda; d->jz[i] = z; d->jx[i] = bp;
    if (bp > d->bulkPi_over_Peq_max) d->bulkPi_over_Peq_max = bp;
  }
  if (cspline_init(&d->lambda2, d->jx, d->jl2, pts)) return -1;
  if (cspline_init(&d->z, d->jx, d->jz, pts)) return -1;
  d->have_jonah = 1;
  return 0;
}

static int df_setup(dfdata *d, const orc_params *p, const orc_setup *s, int need_jonah) {
  memset(d, 0, sizeof(*d));
  d->df_mode = p->df_mode; d->include_baryon = p->include_baryon;
  d->nT = s->nT; d->nmuB = s->nmuB; d->T = s->Tarr; d->muB = s->muBarr; d->tab = s->dftab;
  d->T_min = s->Tarr[0]; d->muB_min = s->muBarr[0];
  d->dT = fabs(s->Tarr[1] - s->Tarr[0]);
  d->dmuB = s->nmuB > 1 ? fabs(s->muBarr[1] - s->muBarr[0]) : 0.0;
  if (!p->include_baryon) {   /* iS3D.cpp:242-246 */
    const double *T = s->Tarr; int n = s->nT;
    cspline_init(&d->c0, T, &TAB(d, K_C0, 0, 0), n);
    cspline_init(&d->c2, T, &TAB(d, K_C2, 0, 0), n);
    cspline_init(&d->c3, T, &TAB(d, K_C3, 0, 0), n);
    cspline_init(&d->F, T, &TAB(d, K_F, 0, 0), n);
    cspline_init(&d->betabulk, T, &TAB(d, K_BB, 0, 0), n);
    cspline_init(&d->betaV, T, &TAB(d, K_BV, 0, 0), n);
    cspline_init(&d->betapi, T, &TAB(d, K_BP, 0, 0), n);
    d->have_splines = 1;
    if (need_jonah && jonah(d, s)) return -1;
  }
  return 0;
}

static void df_free(dfdata *d) {
  free(d->c0.c); free(d->c2.c); free(d->c3.c); free(d->F.c); free(d->betabulk.c); free(d->betaV.c);
  free(d->betapi.c); free(d->lambda2.c); free(d->z.c); free(d->jl2); free(d->jz); free(d->jx);
}

/* DeltafData.cpp:324-402 cubic_spline; returns nonzero on GSL range error */
static int df_cubic(const dfdata *d, double T, double E, double P, double bulkPi, dfcoef *df) {
  int bad = 0;
  memset(df, 0, sizeof(*df));
  switch (d->df_mode) {
    case 1: {
      double T4 = T * T * T * T;
      df->c0 = cspline_eval(&d->c0, T, &bad) / T4;
      df->c1 = 0.0;
      df->c2 = cspline_eval(&d->c2, T, &bad) / T4;
      df->c3 = 0.0; df->c4 = 0.0;
      df->shear14 = 2.0 * T * T * (E + P);
      break;
    }
    case 2: case 3: case 5: {
      double T4 = T * T * T * T;
      df->F = cspline_eval(&d->F, T, &bad) * T;
      df->G = 0.0;
      df->betabulk = cspline_eval(&d->betabulk, T, &bad) * T4;
      df->betaV = 1.0;
      df->betapi = cspline_eval(&d->betapi, T, &bad) * T4;
      break;
    }
    case 4: {
      double T4 = T * T * T * T;
      double l2 = cspline_eval(&d->lambda2, bulkPi / P, &bad);
      /* reference leaves lambda uninitialized for bulkPi == 0 (DeltafData.cpp:369-376); we use 0 */
      df->lambda = 0.0;
      if (bulkPi < 0.0) df->lambda = -sqrt(l2);
      else if (bulkPi > 0.0) df->lambda = sqrt(l2);
      df->z = cspline_eval(&d->z, bulkPi / P, &bad);
      df->betapi = cspline_eval(&d->betapi, T, &bad) * T4;
      df->delta_lambda = bulkPi / (5.0 * df->betapi - 3.0 * P * (E + P) / E);
      df->delta_z = -3.0 * df->delta_lambda * P / E;
      break;
    }
    default: return 2;
  }
  return bad ? 1 : 0;
}

/* DeltafData.cpp:404-499 bilinear_interpolation */
static double bilin(const dfdata *d, int k, double T, double muB, double TL, double TR, double mL, double mR,
                    int iTL, int iTR, int imL, int imR) {
  double f_LL = TAB(d, k, imL, iTL), f_LR = TAB(d, k, imR, iTL), f_RL = TAB(d, k, imL, iTR), f_RR = TAB(d, k, imR, iTR);
  return ((f_LL * (TR - T) + f_RL * (T - TL)) * (mR - muB) + (f_LR * (TR - T) + f_RR * (T - TL)) * (muB - mL)) / (d->dT * d->dmuB);
}

static int df_bilinear(const dfdata *d, double T, double muB, double E, double P, double bulkPi, dfcoef *df) {
  (void)bulkPi;
  memset(df, 0, sizeof(*df));
  int iTL = (int)floor((T - d->T_min) / d->dT), iTR = iTL + 1;
  int imL = (int)floor((muB - d->muB_min) / d->dmuB), imR = imL + 1;
  if (!(iTL >= 0 && iTR < d->nT) || !(imL >= 0 && imR < d->nmuB)) return 3;
  double TL = d->T[iTL], TR = d->T[iTR], mL = d->muB[imL], mR = d->muB[imR];
  switch (d->df_mode) {
    case 1: {
      double T3 = T * T * T, T4 = T3 * T, T5 = T4 * T;
      df->c0 = bilin(d, K_C0, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df->c1 = bilin(d, K_C1, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T3;
      df->c2 = bilin(d, K_C2, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df->c3 = bilin(d, K_C3, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T4;
      df->c4 = bilin(d, K_C4, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) / T5;
      df->shear14 = 2.0 * T * T * (E + P);
      break;
    }
    case 2: case 3: case 5: {
      double T3 = T * T * T, T4 = T3 * T;
      df->F = bilin(d, K_F, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T;
      df->G = bilin(d, K_G, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR);
      df->betabulk = bilin(d, K_BB, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T4;
      df->betaV = bilin(d, K_BV, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T3;
      df->betapi = bilin(d, K_BP, T, muB, TL, TR, mL, mR, iTL, iTR, imL, imR) * T4;
      break;
    }
    case 4: return 4;   /* PTB with baryon exits (DeltafData.cpp:480-483) */
    default: return 2;
  }
  return 0;
}

/* DeltafData.cpp:501-519 */
static int df_eval(const dfdata *d, double T, double muB, double E, double P, double bulkPi, dfcoef *df) {
  if (!d->include_baryon) return df_cubic(d, T, E, P, bulkPi, df);
  return df_bilinear(d, T, muB, E, P, bulkPi, df);
}

static const char *df_errmsg(int rc) {
  switch (rc) {
    case 1: return "gsl: interpolation error (df coefficient spline evaluated out of range)";
    case 2: return "bad df_mode";
    case 3: return "Error: (T,muB) outside df coefficient table";
    case 4: return "Bilinear interpolation error: Jonah df doesn't work for nonzero muB";
    default: return "df coefficient error";
  }
}

/* ------------------------------------------------------------------------- */
/* EmissionFunction.cpp:52-109 does_feqmod_breakdown                           */
/* ------------------------------------------------------------------------- */
static int feqmod_breaks_down(double mass_pion0, double T, double F, double bulkPi, double betabulk,
                              double detA, double detA_min, double z, const orc_setup *s, int df_mode) {
  if (df_mode == 3) {
    const int pts = s->gla_points;
    const double *r1 = s->gla_root + pts, *r2 = s->gla_root + 2 * pts;
    const double *w1 = s->gla_weight + pts, *w2 = s->gla_weight + 2 * pts;
    double mbar = mass_pion0 / T;
    double neq_fact = T * T * T / two_pi2_hbarC3();
    double J20_fact = T * neq_fact;
    double neq = neq_fact * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar, 0., 0., -1.);
    double J20 = J20_fact * orc_gauss_thermal(GT_J20, r2, w2, pts, mbar, 0., 0., -1.);
    double dn = bulkPi * (neq + J20 * F / T / T) / betabulk;
    int negative = (neq + dn < 0.0);
    if (detA <= detA_min || negative) return 1;
  } else if (df_mode == 4) {
    if (detA <= detA_min || z < 0.0) return 1;
  }
  return 0;
}

/* ------------------------------------------------------------------------- */
/* Common per-run grid setup (MomentumSpectra.cpp:49-91)                      */
/* ------------------------------------------------------------------------- */
typedef struct {
  long npT, nphi, ny, neta;
  double *cosphi, *sinphi, *pT, *yv, *etav, *etaw;
} grid;

static void grid_setup(grid *g, const orc_params *p, const orc_setup *s) {
  g->npT = s->npT; g->nphi = s->nphi;
  g->ny = (p->dimension == 2) ? 1 : s->ny;          /* EmissionFunction.cpp:146-153 */
  g->neta = (p->dimension == 3) ? 1 : s->neta;
  g->cosphi = (double *)malloc(sizeof(double) * g->nphi);
  g->sinphi = (double *)malloc(sizeof(double) * g->nphi);
  g->pT = (double *)malloc(sizeof(double) * g->npT);
  g->yv = (double *)malloc(sizeof(double) * g->ny);
  g->etav = (double *)malloc(sizeof(double) * g->neta);
  g->etaw = (double *)malloc(sizeof(double) * g->neta);
  for (long j = 0; j < g->nphi; j++) { g->cosphi[j] = cos(s->phi[j]); g->sinphi[j] = sin(s->phi[j]); }
  for (long i = 0; i < g->npT; i++) g->pT[i] = s->pT[i];
  if (p->dimension == 2) {
    g->yv[0] = 0.0;
    for (long l = 0; l < g->neta; l++) { g->etav[l] = s->eta[l]; g->etaw[l] = s->eta_w[l]; }
  } else {
    g->etav[0] = 0.0; g->etaw[0] = 1.0;
    for (long k = 0; k < g->ny; k++) g->yv[k] = s->y[k];
  }
}

static void grid_free(grid *g) { free(g->cosphi); free(g->sinphi); free(g->pT); free(g->yv); free(g->etav); free(g->etaw); }

/* The reference's cell striding: thread n handles cells n + icell*C (MomentumSpectra.cpp:40-47, 98-107). */
#define CELL_LOOP_BEGIN(n, C, FO_length, icell_glb)                               \
  {                                                                               \
    long FO_chunk_ = (FO_length) / (C);                                           \
    long rem_ = (FO_length) - (C) * FO_chunk_;                                    \
    if (rem_ != 0) FO_chunk_++;                                                   \
    for (long icell_ = 0; icell_ < FO_chunk_; icell_++) {                         \
      if ((icell_ == FO_chunk_ - 1) && (rem_ != 0) && ((n) > rem_ - 1)) continue; \
      long icell_glb = (n) + icell_ * (C);
#define CELL_LOOP_END }}

typedef struct { long breakdown, pl_negative, recon_fail, iterations, skipped; int err; } tstats;

/* ------------------------------------------------------------------------- */
/* calculate_dN_pTdpTdphidy  (MomentumSpectra.cpp:32-415)                     */
/* ------------------------------------------------------------------------- */
static void spectra_grad_ce(const orc_params *p, const orc_setup *s, const orc_surface *S, const dfdata *df_data,
                            const grid *g, long n, long C, double *slice, tstats *st) {
  const double prefactor = pow(2.0 * M_PI * HBARC, -3);
  const long npart = s->npart, npT = g->npT, nphi = g->nphi, ny = g->ny, neta = g->neta;
  const int DF_MODE = p->df_mode;
  CELL_LOOP_BEGIN(n, C, S->n, ic)
    double etaValues0 = g->etav[0];
    double tau = S->tau[ic];
    double tau2 = tau * tau;
    if (p->dimension == 3) etaValues0 = S->eta[ic];   /* thread-local (race fix) */
    double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
    double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
    double ux2 = ux * ux, uy2 = uy * uy;
    double utperp = sqrt(1.0 + ux2 + uy2);
    double tau2_un = tau2 * un;
    double ut = sqrt(utperp * utperp + tau2_un * un);
    double ut2 = ut * ut;
    if (ut * dat + ux * dax + uy * day + un * dan <= 0.0) continue;
    double T = S->T[ic], P = S->P[ic], E = S->E[ic];
    double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
    if (p->include_shear_deltaf) {
      pixx = S->pixx[ic]; pixy = S->pixy[ic]; pixn = S->pixn[ic]; piyy = S->piyy[ic]; piyn = S->piyn[ic];
      pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2_un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
      pitn = (pixn * ux + piyn * uy + tau2_un * pinn) / ut;
      pity = (pixy * ux + piyy * uy + tau2_un * piyn) / ut;
      pitx = (pixx * ux + pixy * uy + tau2_un * pixn) / ut;
      pitt = (pitx * ux + pity * uy + tau2_un * pitn) / ut;
    }
    double bulkPi = 0.0;
    if (p->include_bulk_deltaf) bulkPi = S->bulkPi[ic];
    double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
    if (p->include_baryon && p->include_baryondiff_deltaf) {
      muB = S->muB[ic]; nB = S->nB[ic]; Vx = S->Vx[ic]; Vy = S->Vy[ic]; Vn = S->Vn[ic];
      Vt = (Vx * ux + Vy * uy + Vn * tau2_un) / ut;
      alphaB = muB / T;
      ber = nB / (E + P);
    }
    double tau2_pitn = tau2 * pitn, tau2_pixn = tau2 * pixn, tau2_piyn = tau2 * piyn;
    double tau4_pinn = tau2 * tau2 * pinn, tau2_Vn = tau2 * Vn;
    dfcoef df;
    int rc = df_eval(df_data, T, muB, E, P, bulkPi, &df);
    if (rc) { st->err = rc; return; }
    double shear_coeff = 0, bulk0 = 0, bulk1 = 0, bulk2 = 0, diff0 = 0, diff1 = 0;
    if (DF_MODE == 1) {
      shear_coeff = 1.0 / df.shear14;
      bulk0 = (df.c0 - df.c2) * bulkPi; bulk1 = df.c1 * bulkPi; bulk2 = (4. * df.c2 - df.c0) * bulkPi;
      diff0 = df.c3; diff1 = df.c4;
    } else {
      shear_coeff = 0.5 / (df.betapi * T);
      bulk0 = df.F / (T * T * df.betabulk) * bulkPi;
      bulk1 = df.G / df.betabulk * bulkPi;
      bulk2 = bulkPi / (3.0 * T * df.betabulk);
      diff0 = ber / df.betaV;
      diff1 = 1.0 / df.betaV;
    }
    for (long ipart = 0; ipart < npart; ipart++) {
      long iS0D = npT * ipart;
      double mass = s->mass[ipart], mass_squared = mass * mass, sign = s->sign[ipart];
      double degeneracy = s->degen[ipart], baryon = s->baryon[ipart], chem = baryon * alphaB;
      for (long ipT = 0; ipT < npT; ipT++) {
        long iS1D = nphi * (ipT + iS0D);
        double pT = g->pT[ipT], mT = sqrt(mass_squared + pT * pT), mT_over_tau = mT / tau;
        for (long iphip = 0; iphip < nphi; iphip++) {
          long iS2D = ny * (iphip + iS1D);
          double px = pT * g->cosphi[iphip], py = pT * g->sinphi[iphip];
          double px_dax = px * dax, py_day = py * day, px_ux = px * ux, py_uy = py * uy;
          double pixx_px_px = pixx * px * px, piyy_py_py = piyy * py * py;
          double pitx_px = pitx * px, pity_py = pity * py, pixy_px_py = pixy * px * py;
          double tau2_pixn_px = tau2_pixn * px, tau2_piyn_py = tau2_piyn * py;
          double Vx_px = Vx * px, Vy_py = Vy * py;
          for (long iy = 0; iy < ny; iy++) {
            long iS3D = iy + iS2D;
            double y = g->yv[iy];
            double eta_integral = 0.0;
            for (long ieta = 0; ieta < neta; ieta++) {
              double eta = (p->dimension == 3) ? etaValues0 : g->etav[ieta];
              double eta_weight = g->etaw[ieta];
              double sinhyeta = sinh(y - eta);
              double coshyeta = sqrt(1.0 + sinhyeta * sinhyeta);
              double pt = mT * coshyeta, pn = mT_over_tau * sinhyeta;
              double pdotdsigma = pt * dat + px_dax + py_day + pn * dan;
              if (p->outflow && pdotdsigma <= 0.0) continue;
              double Eu = pt * ut - px_ux - py_uy - pn * tau2_un;
              double feq = 1.0 / (exp(Eu / T - chem) + sign);
              double feqbar = 1.0 - sign * feq;
              double pimunu_pmu_pnu = pitt * pt * pt + pixx_px_px + piyy_py_py + tau4_pinn * pn * pn
                  + 2.0 * (-(pitx_px + pity_py) * pt + pixy_px_py + pn * (tau2_pixn_px + tau2_piyn_py - tau2_pitn * pt));
              double Vmu_pmu = Vt * pt - Vx_px - Vy_py - tau2_Vn * pn;
              double dfv;
              if (DF_MODE == 1) {
                double df_shear = shear_coeff * pimunu_pmu_pnu;
                double df_bulk = bulk0 * mass_squared + (bulk1 * baryon + bulk2 * Eu) * Eu;
                double df_diff = (diff0 * baryon + diff1 * Eu) * Vmu_pmu;
                dfv = feqbar * (df_shear + df_bulk + df_diff);
              } else {
                double df_shear = shear_coeff * pimunu_pmu_pnu / Eu;
                double df_bulk = bulk0 * Eu + bulk1 * baryon + bulk2 * (Eu - mass_squared / Eu);
                double df_diff = (diff0 - diff1 * baryon / Eu) * Vmu_pmu;
                dfv = feqbar * (df_shear + df_bulk + df_diff);
              }
              if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
              double f = feq * (1.0 + dfv);
              eta_integral += eta_weight * pdotdsigma * f;
            }
            slice[iS3D] += (prefactor * degeneracy * eta_integral);
          }
        }
      }
    }
  CELL_LOOP_END
}

/* ------------------------------------------------------------------------- */
/* calculate_dN_pTdpTdphidy_feqmod  (MomentumSpectra.cpp:419-1044)            */
/* ------------------------------------------------------------------------- */
static void spectra_feqmod(const orc_params *p, const orc_setup *s, const orc_surface *S, const dfdata *df_data,
                           const grid *g, long n, long C, double *slice, tstats *st) {
  const double prefactor = pow(2.0 * M_PI * HBARC, -3);
  const long npart = s->npart, npT = g->npT, nphi = g->nphi, ny = g->ny, neta = g->neta;
  const int DF_MODE = p->df_mode, DIMENSION = p->dimension;
  const double detA_min = p->deta_min;
  const int pts = s->gla_points;
  const double *r1 = s->gla_root + pts, *r2 = s->gla_root + 2 * pts;
  const double *w1 = s->gla_weight + pts, *w2 = s->gla_weight + 2 * pts;
  double A_copy[3][3], A_inv[3][3];
  CELL_LOOP_BEGIN(n, C, S->n, ic)
    double tau = S->tau[ic], tau2 = tau * tau;
    double eta0 = (DIMENSION == 3) ? S->eta[ic] : 0.0;
    double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
    double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
    double ut = sqrt(1.0 + ux * ux + uy * uy + tau2 * un * un);
    if (ut * dat + ux * dax + uy * day + un * dan <= 0.0) continue;
    double ut2 = ut * ut, ux2 = ux * ux, uy2 = uy * uy;
    double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
    double T = S->T[ic], P = S->P[ic], E = S->E[ic];
    double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
    if (p->include_shear_deltaf) {
      pixx = S->pixx[ic]; pixy = S->pixy[ic]; pixn = S->pixn[ic]; piyy = S->piyy[ic]; piyn = S->piyn[ic];
      pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
      pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
      pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
      pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
      pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
    }
    double bulkPi = 0.0;
    if (p->include_bulk_deltaf) bulkPi = S->bulkPi[ic];
    double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
    if (p->include_baryon && p->include_baryondiff_deltaf) {
      muB = S->muB[ic]; nB = S->nB[ic]; Vx = S->Vx[ic]; Vy = S->Vy[ic]; Vn = S->Vn[ic];
      Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
      alphaB = muB / T;
      ber = nB / (E + P);
    }
    if (DF_MODE == 4) {  /* :603-615 */
      if (bulkPi < -P) bulkPi = -(1.0 - 1.e-5) * P;
      else if (bulkPi / P > df_data->bulkPi_over_Peq_max) bulkPi = P * (df_data->bulkPi_over_Peq_max - 1.e-5);
    }
    double zt = tau * un / utperp, zn = ut / (tau * utperp);
    double pl = P + bulkPi + zt * zt * pitt + tau2 * tau2 * zn * zn * pinn + 2. * tau2 * zt * zn * pitn;
    if (pl < 0) st->pl_negative++;
    dfcoef df;
    int rc = df_eval(df_data, T, muB, E, P, bulkPi, &df);
    if (rc) { st->err = rc; return; }
    double F = df.F, G = df.G, betabulk = df.betabulk, betaV = df.betaV, betapi = df.betapi;
    double lambda = df.lambda, z = df.z, delta_lambda = df.delta_lambda, delta_z = df.delta_z;
    milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
    pilrf pl_ = boost_pimunu(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
    double T_mod = T, alphaB_mod = alphaB;
    if (DF_MODE == 3) { T_mod = T + bulkPi * F / betabulk; alphaB_mod = alphaB + bulkPi * G / betabulk; }
    double shear_coeff = 0.5 / (betapi * T);
    double bulk0 = F / (T * T * betabulk), bulk1 = G / betabulk, bulk2 = 1.0 / (3.0 * T * betabulk);
    double shear_mod = 0.5 / betapi, bulk_mod = bulkPi / (3.0 * betabulk);
    if (DF_MODE == 4) bulk_mod = lambda;
    double Axx = 1.0 + pl_.xx * shear_mod + bulk_mod, Axy = pl_.xy * shear_mod, Axz = pl_.xz * shear_mod;
    double Ayy = 1.0 + pl_.yy * shear_mod + bulk_mod, Ayz = pl_.yz * shear_mod, Azz = 1.0 + pl_.zz * shear_mod + bulk_mod;
    double detA = Axx * (Ayy * Azz - Ayz * Ayz) - Axy * (Axy * Azz - Ayz * Axz) + Axz * (Axy * Ayz - Ayy * Axz);
    double detA_b23 = pow(1.0 + bulk_mod, 2);
    double A[9] = {Axx, Axy, Axz, Axy, Ayy, Ayz, Axz, Ayz, Azz};
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) A_copy[i][j] = A[3 * i + j];
    inverse3(A, A_inv);
    double neq_fact = T * T * T / two_pi2_hbarC3();
    double dn_fact = bulkPi / betabulk, J20_fact = T * neq_fact, N10_fact = neq_fact;
    double nmod_fact = T_mod * T_mod * T_mod / two_pi2_hbarC3();
    int breaks = feqmod_breaks_down(p->mass_pion0, T, F, bulkPi, betabulk, detA, detA_min, z, s, DF_MODE);
    if (breaks) st->breakdown++;
    double eta_scale = 1.0;
    if (detA > detA_min && DIMENSION == 2) eta_scale = detA / detA_b23;
    for (long ipart = 0; ipart < npart; ipart++) {
      long iS0D = npT * ipart;
      double mass = s->mass[ipart], mass2 = mass * mass, sign = s->sign[ipart];
      double degeneracy = s->degen[ipart], baryon = s->baryon[ipart];
      double chem = baryon * alphaB, chem_mod = baryon * alphaB_mod;
      double renorm = 1.0;
      if (p->include_bulk_deltaf) {
        if (DF_MODE == 3) {
          double mbar = mass / T, mbar_mod = mass / T_mod;
          double neq = neq_fact * degeneracy * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar, alphaB, baryon, sign);
          double N10 = baryon * N10_fact * degeneracy * orc_gauss_thermal(GT_J10, r1, w1, pts, mbar, alphaB, baryon, sign);
          double J20 = J20_fact * degeneracy * orc_gauss_thermal(GT_J20, r2, w2, pts, mbar, alphaB, baryon, sign);
          double n_linear = neq + dn_fact * (neq + N10 * G + J20 * F / T / T);
          double n_mod = nmod_fact * degeneracy * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar_mod, alphaB_mod, baryon, sign);
          renorm = n_linear / n_mod;
        } else if (DF_MODE == 4) {
          renorm = z;
        }
      }
      if (DIMENSION == 2) renorm /= detA_b23; else renorm /= detA;
      if (isnan(renorm) || isinf(renorm)) { st->skipped++; continue; }
      for (long ipT = 0; ipT < npT; ipT++) {
        long iS1D = nphi * (ipT + iS0D);
        double pT = g->pT[ipT], mT = sqrt(mass2 + pT * pT), mT_over_tau = mT / tau;
        for (long iphip = 0; iphip < nphi; iphip++) {
          long iS2D = ny * (iphip + iS1D);
          double px = pT * g->cosphi[iphip], py = pT * g->sinphi[iphip];
          for (long iy = 0; iy < ny; iy++) {
            long iS3D = iy + iS2D;
            double y = g->yv[iy];
            double eta_integral = 0.0;
            for (long ieta = 0; ieta < neta; ieta++) {
              double eta = (DIMENSION == 3) ? eta0 : g->etav[ieta];
              double eta_weight = g->etaw[ieta];
              int narrow = 0;
              if (DIMENSION == 3 && !breaks) { if (detA < 0.01 && fabs(y - eta) < detA) narrow = 1; }
              double pdotdsigma, f;
              if (breaks || narrow) {
                double pt = mT * cosh(y - eta), pn = mT_over_tau * sinh(y - eta), tau2_pn = tau2 * pn;
                pdotdsigma = eta_weight * (pt * dat + px * dax + py * day) + pn * dan;
                if (p->outflow && pdotdsigma <= 0.0) continue;
                if (DF_MODE == 3) {
                  double pdotu = pt * ut - px * ux - py * uy - tau2_pn * un;
                  double feq = 1.0 / (exp(pdotu / T - chem) + sign);
                  double feqbar = 1.0 - sign * feq;
                  double ppp = pitt * pt * pt + pixx * px * px + piyy * py * py + pinn * tau2_pn * tau2_pn
                      + 2.0 * (-(pitx * px + pity * py) * pt + pixy * px * py + tau2_pn * (pixn * px + piyn * py - pitn * pt));
                  double Vp = Vt * pt - Vx * px - Vy * py - Vn * tau2_pn;
                  double df_shear = shear_coeff * ppp / pdotu;
                  double df_bulk = (bulk0 * pdotu + bulk1 * baryon + bulk2 * (pdotu - mass2 / pdotu)) * bulkPi;
                  double df_diff = (ber - baryon / pdotu) * Vp / betaV;
                  double dfv = feqbar * (df_shear + df_bulk + df_diff);
                  if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
                  f = feq * (1.0 + dfv);
                } else {
                  double pdotu = pt * ut - px * ux - py * uy - tau2_pn * un;
                  double feq = 1.0 / (exp(pdotu / T) + sign);
                  double feqbar = 1.0 - sign * feq;
                  double ppp = pitt * pt * pt + pixx * px * px + piyy * py * py + pinn * tau2_pn * tau2_pn
                      + 2.0 * (-(pitx * px + pity * py) * pt + pixy * px * py + tau2_pn * (pixn * px + piyn * py - pitn * pt));
                  double df_shear = feqbar * shear_coeff * ppp / pdotu;
                  double df_bulk = delta_z - 3.0 * delta_lambda + feqbar * delta_lambda * (pdotu - mass2 / pdotu) / T;
                  double dfv = df_shear + df_bulk;
                  if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
                  f = feq * (1.0 + dfv);
                }
              } else {
                double pt = mT * cosh(y - eta_scale * eta), pn = mT_over_tau * sinh(y - eta_scale * eta), tau2_pn = tau2 * pn;
                pdotdsigma = eta_weight * (pt * dat + px * dax + py * day) + pn * dan;
                if (p->outflow && pdotdsigma <= 0.0) continue;
                double pLRF[3] = {-b.Xt * pt + b.Xx * px + b.Xy * py + b.Xn * tau2_pn, b.Yx * px + b.Yy * py, -b.Zt * pt + b.Zn * tau2_pn};
                double pm[3], pmp[3], pp[3], dpv[3], dpm[3];
                matvec3(A_inv, pLRF, pm);
                for (int it = 0; it < 5; it++) {
                  for (int q = 0; q < 3; q++) pmp[q] = pm[q];
                  matvec3(A_copy, pmp, pp);
                  for (int q = 0; q < 3; q++) dpv[q] = pLRF[q] - pp[q];
                  double dp = sqrt(dpv[0] * dpv[0] + dpv[1] * dpv[1] + dpv[2] * dpv[2]);
                  if (dp <= 1.e-16) break;
                  matvec3(A_inv, dpv, dpm);
                  for (int q = 0; q < 3; q++) pm[q] = pmp[q] + dpm[q];
                }
                double E_mod = sqrt(mass2 + pm[0] * pm[0] + pm[1] * pm[1] + pm[2] * pm[2]);
                f = fabs(renorm) / (exp(E_mod / T_mod - chem_mod) + sign);
              }
              eta_integral += (pdotdsigma * f);
            }
            slice[iS3D] += (prefactor * degeneracy * eta_integral);
          }
        }
      }
    }
  CELL_LOOP_END
}

/* ------------------------------------------------------------------------- */
/* AnisoVariables.cpp:15-643                                                  */
/* ------------------------------------------------------------------------- */
static const double gl_r2[16] = IS3D_GL16_ROOT_A2, gl_w2[16] = IS3D_GL16_WEIGHT_A2;
static const double gl_r3[16] = IS3D_GL16_ROOT_A3, gl_w3[16] = IS3D_GL16_WEIGHT_A3;
#define ANISO_DELTA 0.01

static void hyper_t(double z, double *t200, double *t220, double *t201) {
  if (z > ANISO_DELTA) {
    double sqrtz = sqrt(z), t = atan(sqrtz) / sqrtz;
    *t200 = 1. + (1. + z) * t; *t220 = (-1. + (1. + z) * t) / z; *t201 = (1. + (z - 1.) * t) / z;
  } else if (z < -ANISO_DELTA && z > -1.) {
    double sqrtmz = sqrt(-z), t = atanh(sqrtmz) / sqrtmz;
    *t200 = 1. + (1. + z) * t; *t220 = (-1. + (1. + z) * t) / z; *t201 = (1. + (z - 1.) * t) / z;
  } else if (fabs(z) <= ANISO_DELTA) {
    double z2 = z * z, z3 = z2 * z, z4 = z3 * z, z5 = z4 * z, z6 = z5 * z;
    *t200 = 2. + 0.6666666666666667 * z - 0.1333333333333333 * z2 + 0.05714285714285716 * z3 - 0.031746031746031744 * z4 + 0.020202020202020193 * z5 - 0.013986013986013984 * z6;
    *t220 = 0.6666666666666667 - 0.1333333333333333 * z + 0.05714285714285716 * z2 - 0.031746031746031744 * z3 + 0.020202020202020193 * z4 - 0.013986013986013984 * z5 + 0.010256410256410262 * z6;
    *t201 = 1.3333333333333333 - 0.5333333333333333 * z + 0.34285714285714286 * z2 - 0.25396825396825395 * z3 + 0.20202020202020202 * z4 - 0.16783216783216784 * z5 + 0.14358974358974358 * z6;
  } else { *t200 = *t220 = *t201 = 0.0; }   /* reference: uninitialized (unreachable for z > -1) */
}

static void hyper_t4(double z, double *t402, double *t421, double *t440) {
  double z2 = z * z;
  if (z > ANISO_DELTA) {
    double sqrtz = sqrt(z), t = atan(sqrtz) / sqrtz;
    *t402 = (3. * (z - 1.) + (z * (3. * z - 2.) + 3.) * t) / (4. * z2);
    *t421 = (3. + z + (1. + z) * (z - 3.) * t) / (4. * z2);
    *t440 = (-(3. + 5. * z) + 3. * (z + 1.) * (z + 1.) * t) / (4. * z2);
  } else if (z < -ANISO_DELTA && z > -1.) {
    double sqrtmz = sqrt(-z), t = atanh(sqrtmz) / sqrtmz;
    *t402 = (3. * (z - 1.) + (z * (3. * z - 2.) + 3.) * t) / (4. * z2);
    *t421 = (3. + z + (1. + z) * (z - 3.) * t) / (4. * z2);
    *t440 = (-(3. + 5. * z) + 3. * (z + 1.) * (z + 1.) * t) / (4. * z2);
  } else if (fabs(z) <= ANISO_DELTA) {
    double z3 = z2 * z, z4 = z3 * z, z5 = z4 * z, z6 = z5 * z;
    *t402 = 1.0666666666666667 - 0.4571428571428572 * z + 0.3047619047619048 * z2 - 0.23088023088023088 * z3 + 0.1864801864801865 * z4 - 0.15664335664335666 * z5 + 0.13514328808446457 * z6;
    *t421 = 0.2666666666666666 - 0.0761904761904762 * z + 0.0380952380952381 * z2 - 0.023088023088023088 * z3 + 0.015540015540015537 * z4 - 0.011188811188811189 * z5 + 0.00844645550527904 * z6;
    *t440 = 0.4 - 0.057142857142857106 * z + 0.019047619047619063 * z2 - 0.008658008658008663 * z3 + 0.004662004662004657 * z4 - 0.002797202797202792 * z5 + 0.0018099547511312257 * z6;
  } else { *t402 = *t421 = *t440 = 0.0; }
}

typedef struct { int n; const double *mass, *sign, *degen; } hadrons;

static void compute_F(double Ea, double PTa, double PLa, const hadrons *h, const double X[3], double F[3]) {
  double lambda = X[0], aT = X[1], aL = X[2];
  double aT2 = aT * aT, aL2 = aL * aL, d = aT2 - aL2;
  double cf = aT2 * aL * lambda * lambda * lambda * lambda / four_pi2_hbarC3();
  double I200 = 0, I220 = 0, I201 = 0;
  for (int n = 0; n < h->n; n++) {
    double mass = h->mass[n], sign = h->sign[n], g = h->degen[n];
    if (mass == 0) continue;
    double mbar = mass / lambda, mbar2 = mbar * mbar;
    double a = 0, b = 0, c = 0;
    for (int i = 0; i < 16; i++) {
      double pbar = gl_r2[i], weight = gl_w2[i];
      double Ebar = sqrt(pbar * pbar + mbar2);
      double w = sqrt(aL2 + mbar2 / (pbar * pbar));
      double z = d / (w * w);
      double t200, t220, t201;
      hyper_t(z, &t200, &t220, &t201);
      double cw = pbar * weight * exp(pbar) / (exp(Ebar + 0) + sign);
      a += cw * t200 * w; b += cw * t220 / w; c += cw * t201 / w;
    }
    a *= g; b *= g; c *= g;
    I200 += a; I220 += b; I201 += c;
  }
  I200 *= cf; I220 *= cf * aL2; I201 *= cf * aT2 / 2.;
  F[0] = I200 - Ea; F[1] = I201 - PTa; F[2] = I220 - PLa;
}

static void compute_J(double Ea, double PTa, double PLa, const hadrons *h, const double X[3], const double F[3], double J[3][3]) {
  double lambda = X[0], aT = X[1], aL = X[2];
  double aT2 = aT * aT, aL2 = aL * aL, d = aT2 - aL2;
  double lambda2 = lambda * lambda, lambda3 = lambda2 * lambda;
  double lambda_aT3 = lambda * aT2 * aT, lambda_aL3 = lambda * aL2 * aL;
  double cf = aT2 * aL * lambda2 * lambda3 / four_pi2_hbarC3();
  double J2001 = 0, J2011 = 0, J2201 = 0, J402 = 0, J421 = 0, J440 = 0;
  for (int n = 0; n < h->n; n++) {
    double mass = h->mass[n], sign = h->sign[n], g = h->degen[n];
    if (mass == 0) continue;
    double mbar = mass / lambda, mbar2 = mbar * mbar;
    double a = 0, b = 0, c = 0, e = 0, f = 0, k = 0;
    for (int i = 0; i < 16; i++) {
      double pbar = gl_r3[i], weight = gl_w3[i], pbar2 = pbar * pbar;
      double Ebar = sqrt(pbar2 + mbar2);
      double w = sqrt(aL2 + mbar2 / pbar2);
      double z = d / (w * w);
      double t200, t220, t201, t402, t421, t440;
      hyper_t(z, &t200, &t220, &t201);
      hyper_t4(z, &t402, &t421, &t440);
      double qs = exp(Ebar + 0) + sign;
      double cw = weight * exp(pbar + Ebar) / (qs * qs);
      a += Ebar * cw * t200 * w; b += Ebar * cw * t201 / w; c += Ebar * cw * t220 / w;
      e += pbar2 / Ebar * cw * t402 / w; f += pbar2 / Ebar * cw * t421 / w; k += pbar2 / Ebar * cw * t440 / w;
    }
    a *= g; b *= g; c *= g; e *= g; f *= g; k *= g;
    J2001 += a; J2011 += b; J2201 += c; J402 += e; J421 += f; J440 += k;
  }
  J2001 *= cf; J2011 *= cf * aT2 / 2.; J2201 *= cf * aL2;
  J402 *= cf * aT2 * aT2 / 8.; J421 *= cf * aT2 * aL2 / 2.; J440 *= cf * aL2 * aL2;
  double Eai = F[0] + Ea, PTai = F[1] + PTa, PLai = F[2] + PLa;
  J[0][0] = J2001 / lambda2; J[0][1] = 2. * (Eai + PTai) / aT; J[0][2] = (Eai + PLai) / aL;
  J[1][0] = J2011 / lambda2; J[1][1] = 4. * J402 / lambda_aT3; J[1][2] = J421 / lambda_aL3;
  J[2][0] = J2201 / lambda2; J[2][1] = 2. * J421 / lambda_aT3; J[2][2] = J440 / lambda_aL3;
}

#define TOL_DX 1.e-4
#define TOL_F 1.e-4

/* AnisoVariables.cpp:302-390 (Numerical Recipes line search) */
static double line_backtrack(double Ea, double PTa, double PLa, const hadrons *h, const double Xc[3],
                             const double dX[3], double dX_abs, double g0, double F[3]) {
  double X[3];
  for (int i = 0; i < 3; i++) X[i] = Xc[i] + dX[i];
  compute_F(Ea, PTa, PLa, h, X, F);
  double f = (F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) / 2.;
  double gprime0 = -2. * g0;
  double l = 1, alpha = 0.0001, lroot = 0, lprev = 0, fprev = 0;
  for (int n = 0; n < 20; n++) {
    if ((l * dX_abs) <= TOL_DX) return l;
    else if (f <= (g0 + l * alpha * gprime0)) return l;
    else if (n == 0) lroot = -gprime0 / (2. * (f - g0 - gprime0));
    else {
      double a = ((f - g0 - l * gprime0) / (l * l) - (fprev - g0 - lprev * gprime0) / (lprev * lprev)) / (l - lprev);
      double b = (-lprev * (f - g0 - l * gprime0) / (l * l) + l * (fprev - g0 - lprev * gprime0) / (lprev * lprev)) / (l - lprev);
      if (a == 0) lroot = -gprime0 / (2. * b);
      else {
        double z = b * b - 3. * a * gprime0;
        if (z < 0) lroot = 0.5 * l;
        else if (b <= 0) lroot = (-b + sqrt(z)) / (3. * a);
        else lroot = -gprime0 / (b + sqrt(z));
      }
      lroot = fmin(lroot, 0.5 * l);
    }
    lprev = l; fprev = f;
    l = fmax(lroot, 0.5 * l);
    for (int i = 0; i < 3; i++) X[i] = Xc[i] + l * dX[i];
    compute_F(Ea, PTa, PLa, h, X, F);
    f = (F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) / 2.;
  }
  return l;
}

typedef struct { double lambda, aT, aL; int fail, iters; } aniso;

/* AnisoVariables.cpp:393-538 */
static aniso find_aniso(double E, double pl, double pt, double l0, double aT0, double aL0, const hadrons *h) {
  aniso r = {l0, aT0, aL0, 1, 0};
  double Ea = E, PTa = pt, PLa = pl;
  if (Ea < 0 || PTa < 0 || PLa < 0) return r;
  double X[3] = {l0, aT0, aL0}, dX[3], F[3], J[3][3];
  compute_F(Ea, PTa, PLa, h, X, F);
  double stepmax = 100. * fmax(sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]), 3.);
  for (int n = 0; n < 30; n++) {
    compute_J(Ea, PTa, PLa, h, X, F, J);
    double f = (F[0] * F[0] + F[1] * F[1] + F[2] * F[2]) / 2.;
    double Jm[9] = {J[0][0], J[0][1], J[0][2], J[1][0], J[1][1], J[1][2], J[2][0], J[2][1], J[2][2]};
    for (int i = 0; i < 3; i++) F[i] *= -1.;
    int perm[3];
    lu3_decomp(Jm, perm);
    lu3_solve(Jm, perm, F, dX);
    double dX_abs = sqrt(dX[0] * dX[0] + dX[1] * dX[1] + dX[2] * dX[2]);
    if (dX_abs > stepmax) { for (int i = 0; i < 3; i++) dX[i] *= stepmax / dX_abs; dX_abs = stepmax; }
    double l = line_backtrack(Ea, PTa, PLa, h, X, dX, dX_abs, f, F);
    for (int i = 0; i < 3; i++) X[i] += (l * dX[i]);
    double F_abs = sqrt(F[0] * F[0] + F[1] * F[1] + F[2] * F[2]);
    dX_abs *= l;
    if (X[0] < 0 || X[1] < 0 || X[2] < 0) { r.iters = n + 1; return r; }
    else if (dX_abs <= TOL_DX && F_abs <= TOL_F) {
      r.lambda = X[0]; r.aT = X[1]; r.aL = X[2]; r.fail = 0; r.iters = n + 1; return r;
    }
  }
  r.iters = 30;
  return r;
}

/* AnisoVariables.cpp:541-643 */
static void famod_coefficient(double lambda, double aT, double aL, const hadrons *h, double *bpi, double *bW) {
  double lambda2 = lambda * lambda, aT2 = aT * aT, aL2 = aL * aL, d = aT2 - aL2;
  double cf = aT2 * aL * lambda * lambda2 * lambda2 / four_pi2_hbarC3();
  double J402 = 0, J421 = 0;
  for (int n = 0; n < h->n; n++) {
    double mass = h->mass[n], sign = h->sign[n], g = h->degen[n];
    if (mass == 0) continue;
    double mbar = mass / lambda, mbar2 = mbar * mbar;
    double e = 0, f = 0;
    for (int i = 0; i < 16; i++) {
      double pbar = gl_r3[i], weight = gl_w3[i], pbar2 = pbar * pbar;
      double Ebar = sqrt(pbar2 + mbar2);
      double w = sqrt(aL2 + mbar2 / pbar2);
      double z = d / (w * w);
      double t402, t421, t440;
      hyper_t4(z, &t402, &t421, &t440);
      double qs = exp(Ebar + 0) + sign;
      double cw = weight * exp(pbar + Ebar) / (qs * qs);
      e += pbar2 / Ebar * cw * t402 / w; f += pbar2 / Ebar * cw * t421 / w;
    }
    e *= g; f *= g;
    J402 += e; J421 += f;
  }
  J402 *= cf * aT2 * aT2 / 8.; J421 *= cf * aT2 * aL2 / 2.;
  *bpi = J402 / (aT2 * lambda);
  *bW = J421 / (aT * aL * lambda);
}

int orc_aniso_solve(const orc_setup *s, double E, double pl, double pt, double l0, double aT0, double aL0, double *out) {
  hadrons h = {s->npdg < 320 ? s->npdg : 320, s->pdg_mass, s->pdg_sign, s->pdg_degen};
  aniso r = find_aniso(E, pl, pt, l0, aT0, aL0, &h);
  double bpi, bW;
  famod_coefficient(r.lambda, r.aT, r.aL, &h, &bpi, &bW);
  out[0] = r.lambda; out[1] = r.aT; out[2] = r.aL; out[3] = r.fail; out[4] = r.iters; out[5] = bpi;
  (void)bW;
  return 0;
}

/* PTMA warm-start chain state of one OpenMP thread (MomentumSpectra.cpp:1132-1135): the previous successful
 * cell's (lambda, aT, aL) */
typedef struct { double lambda_prev, aT_prev, aL_prev; int prev_ok; } chain_state;

/* one cell's warm-started Newton solve and the chain update (MomentumSpectra.cpp:1288-1368): p_L or p_T < 0 passes
 * the state through (breakdown), a failed warm start retries from (T, 1, 1), a failed retry resets the chain.
 * Returns 1 when the cell breaks down; lambda / aT / aL hold the cell's solution (or its (T, 1, 1) fallback). */
static int famod_chain_step(chain_state *cs, double T, double E, double pl, double pt, const hadrons *h,
                            double *lambda, double *aT, double *aL, tstats *st) {
  int broken = 0;
  *lambda = T; *aT = 1; *aL = 1;
  if (pl < 0 || pt < 0) { st->pl_negative++; broken = 1; }
  else {
    if (cs->prev_ok) { *lambda = cs->lambda_prev; *aT = cs->aT_prev; *aL = cs->aL_prev; }
    aniso X = find_aniso(E, pl, pt, *lambda, *aT, *aL, h);
    if (X.fail && cs->prev_ok) {
      *lambda = T; *aT = 1; *aL = 1;
      X = find_aniso(E, pl, pt, *lambda, *aT, *aL, h);
      if (X.fail) { broken = 1; st->recon_fail++; cs->prev_ok = 0; }
      else {
        *lambda = X.lambda; *aT = X.aT; *aL = X.aL;
        cs->lambda_prev = *lambda; cs->aT_prev = *aT; cs->aL_prev = *aL; cs->prev_ok = 1;
      }
    } else {
      *lambda = X.lambda; *aT = X.aT; *aL = X.aL;
      cs->lambda_prev = *lambda; cs->aT_prev = *aT; cs->aL_prev = *aL; cs->prev_ok = 1;
    }
    st->iterations += X.iters;
  }
  return broken;
}

/* PTMA warm-start chain over an explicit cell list (test hook for the distributed chain hand-off): the cells are
 * solved in list order from state[4] = (prev_ok, lambda_prev, aT_prev, aL_prev), with the prologue of
 * spectra_famod below (MomentumSpectra.cpp:1155-1268) and its chain step; cells with u.dsigma <= 0 are not in the
 * chain (:1146).  states[4 i + f] = the chain state after cell i, iters[i] = its Newton iterations (-1: skipped);
 * state returns the state after the last cell.  Returns the sum of iters over the solved cells. */
long orc_famod_chain(const orc_params *p, const orc_setup *s, const orc_surface *S, const long *cells, long ncells,
                     double *state, double *states, int *iters) {
  hadrons h = {s->npdg < 320 ? s->npdg : 320, s->pdg_mass, s->pdg_sign, s->pdg_degen};
  chain_state cs = {state[1], state[2], state[3], state[0] != 0.0};
  long total = 0;
  for (long i = 0; i < ncells; i++) {
    const long ic = cells[i];
    double tau = S->tau[ic], tau2 = tau * tau;
    double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
    double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
    double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
    iters[i] = -1;
    if (ut * dat + ux * dax + uy * day + un * dan > 0) {
      double ut2 = ut * ut, ux2 = ux * ux, uy2 = uy * uy;
      double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1. + ux * ux + uy * uy);
      double T = S->T[ic], P = S->P[ic], E = S->E[ic];
      double pixx = S->pixx[ic], pixy = S->pixy[ic], pixn = S->pixn[ic], piyy = S->piyy[ic], piyn = S->piyn[ic];
      double pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2. * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
      double pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
      double pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
      double pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
      double pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
      double bulkPi = S->bulkPi[ic];
      milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
      pilrf pl_ = boost_pimunu(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
      double pl = P + bulkPi + pl_.zz, pt = P + bulkPi - pl_.zz / 2.;
      tstats st = {0, 0, 0, 0, 0, 0};
      double lambda, aT, aL;
      famod_chain_step(&cs, T, E, pl, pt, &h, &lambda, &aT, &aL, &st);
      iters[i] = (int)st.iterations;
      total += st.iterations;
    }
    states[4 * i] = cs.prev_ok; states[4 * i + 1] = cs.lambda_prev; states[4 * i + 2] = cs.aT_prev; states[4 * i + 3] = cs.aL_prev;
  }
  (void)p;
  state[0] = cs.prev_ok; state[1] = cs.lambda_prev; state[2] = cs.aT_prev; state[3] = cs.aL_prev;
  return total;
}


/* ------------------------------------------------------------------------- */
/* calculate_dN_pTdpTdphidy_famod  (MomentumSpectra.cpp:1049-1682)            */
/* ------------------------------------------------------------------------- */
static void spectra_famod(const orc_params *p, const orc_setup *s, const orc_surface *S,
                          const grid *g, long n, long C, double *slice, tstats *st) {
  const double prefactor = pow(2.0 * M_PI * HBARC, -3);
  const long npart = s->npart, npT = g->npT, nphi = g->nphi, ny = g->ny, neta = g->neta;
  const int DIMENSION = p->dimension;
  const double detB_min = p->deta_min;
  hadrons h = {s->npdg < 320 ? s->npdg : 320, s->pdg_mass, s->pdg_sign, s->pdg_degen};  /* :1295 */
  chain_state cs = {0, 0, 0, 0};
  double B_copy[3][3], B_inv[3][3];
  CELL_LOOP_BEGIN(n, C, S->n, ic)
    double tau = S->tau[ic], tau2 = tau * tau;
    double eta0 = (DIMENSION == 3) ? S->eta[ic] : 0.0;
    double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
    double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
    double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
    if (ut * dat + ux * dax + uy * day + un * dan <= 0) continue;
    double ut2 = ut * ut, ux2 = ux * ux, uy2 = uy * uy;
    double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1. + ux * ux + uy * uy);
    double T = S->T[ic], P = S->P[ic], E = S->E[ic];
    double pixx = S->pixx[ic], pixy = S->pixy[ic], pixn = S->pixn[ic], piyy = S->piyy[ic], piyn = S->piyn[ic];
    double pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2. * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    double pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
    double pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
    double pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
    double pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
    double bulkPi = S->bulkPi[ic];
    double muB = 0;
    if (p->include_baryon) muB = S->muB[ic];   /* V^mu read but unused (:1216-1222) */
    double alphaB = muB / T;
    milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
    pilrf pl_ = boost_pimunu(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
    double pl = P + bulkPi + pl_.zz, pt = P + bulkPi - pl_.zz / 2.;
    double piTxx = 0, piTxy = 0, piTyy = 0, WTzx = 0, WTzy = 0;
    if (p->include_shear_deltaf) {
      piTxx = (pl_.xx - pl_.yy) / 2.; piTxy = pl_.xy; piTyy = -(piTxx);
      WTzx = pl_.xz; WTzy = pl_.yz;
    }
    double lambda = T, aT = 1, aL = 1, upsilonB = alphaB;
    int broken = famod_chain_step(&cs, T, E, pl, pt, &h, &lambda, &aT, &aL, st);
    double bpi, bW;
    famod_coefficient(lambda, aT, aL, &h, &bpi, &bW);
    double shear_coeff = 0.5 / bpi, diff_coeff = 1. / bW;
    double Axx = aT, Ayy = aT, Azz = aL, detA = Axx * Ayy * Azz;
    double Cxx = 1. + shear_coeff * piTxx, Cxy = shear_coeff * piTxy, Cxz = diff_coeff * WTzx * aT / (aT + aL);
    double Cyx = Cxy, Cyy = 1. + shear_coeff * piTyy, Cyz = diff_coeff * WTzy * aT / (aT + aL);
    double Czx = diff_coeff * WTzx * aL / (aT + aL), Czy = diff_coeff * WTzy * aL / (aT + aL), Czz = 1.;
    double detC = Cxx * (Cyy * Czz - Cyz * Czy) - Cxy * (Cyx * Czz - Cyz * Czx) + Cxz * (Cyx * Czy - Cyy * Czx);
    double Bxx = Axx + aT * shear_coeff * piTxx, Bxy = aT * shear_coeff * piTxy, Bxz = diff_coeff * WTzx * aT * aL / (aT + aL);
    double Byy = Ayy + aT * shear_coeff * piTyy, Byz = diff_coeff * WTzy * aT * aL / (aT + aL), Bzz = Azz;
    double detB = detC * detA;
    double detB_b23 = (2. * aT + aL) * (2. * aT + aL) / 9.;
    double B[9] = {Bxx, Bxy, Bxz, Bxy, Byy, Byz, Bxz, Byz, Bzz};
    for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) B_copy[i][j] = B[3 * i + j];
    inverse3(B, B_inv);
    if (detB <= detB_min) broken = 1;
    double eta_scale = 1;
    if (detB > detB_min && DIMENSION == 2) eta_scale = detB / detB_b23;
    double renorm = eta_scale / detC;
    if (isnan(renorm) || isinf(renorm)) broken = 1;
    if (broken) st->breakdown++;
    for (long ipart = 0; ipart < npart; ipart++) {
      long iS0D = npT * ipart;
      double mass = s->mass[ipart], mass2 = mass * mass, sign = s->sign[ipart];
      double degeneracy = s->degen[ipart], baryon = s->baryon[ipart];
      double chem = baryon * alphaB, chem_effect = baryon * upsilonB;
      for (long ipT = 0; ipT < npT; ipT++) {
        long iS1D = nphi * (ipT + iS0D);
        double pT = g->pT[ipT], mT = sqrt(mass2 + pT * pT), mT_over_tau = mT / tau;
        for (long iphip = 0; iphip < nphi; iphip++) {
          long iS2D = ny * (iphip + iS1D);
          double px = pT * g->cosphi[iphip], py = pT * g->sinphi[iphip];
          for (long iy = 0; iy < ny; iy++) {
            long iS3D = iy + iS2D;
            double y = g->yv[iy];
            double eta_integral = 0;
            for (long ieta = 0; ieta < neta; ieta++) {
              double eta = (DIMENSION == 3) ? eta0 : g->etav[ieta];
              double eta_weight = g->etaw[ieta];
              int narrow = 0;
              if (DIMENSION == 3 && !broken) { if (detB < 0.01 && fabs(y - eta) < detB) narrow = 1; }
              double p_dsigma, f;
              if (broken || narrow) {
                double ptau = mT * cosh(y - eta), pn = mT_over_tau * sinh(y - eta), tau2_pn = tau2 * pn;
                p_dsigma = ptau * dat + px * dax + py * day + pn * dan;
                if (p->outflow && p_dsigma <= 0) continue;
                double u_p = ptau * ut - px * ux - py * uy - tau2_pn * un;
                f = 1. / (exp(u_p / T - chem) + sign);
              } else {
                double ptau = mT * cosh(y - eta_scale * eta), pn = mT_over_tau * sinh(y - eta_scale * eta), tau2_pn = tau2 * pn;
                p_dsigma = ptau * dat + px * dax + py * day + pn * dan;
                if (p->outflow && p_dsigma <= 0.0) continue;
                double pLRF[3] = {-b.Xt * ptau + b.Xx * px + b.Xy * py + b.Xn * tau2_pn, b.Yx * px + b.Yy * py, -b.Zt * ptau + b.Zn * tau2_pn};
                double pm[3], pmp[3], pp[3], dpv[3], dpm[3];
                matvec3(B_inv, pLRF, pm);
                for (int it = 0; it < 5; it++) {
                  for (int q = 0; q < 3; q++) pmp[q] = pm[q];
                  matvec3(B_copy, pmp, pp);
                  for (int q = 0; q < 3; q++) dpv[q] = pLRF[q] - pp[q];
                  double dp = sqrt(dpv[0] * dpv[0] + dpv[1] * dpv[1] + dpv[2] * dpv[2]);
                  if (dp <= 1.e-16) break;
                  matvec3(B_inv, dpv, dpm);
                  for (int q = 0; q < 3; q++) pm[q] = pmp[q] + dpm[q];
                }
                double E_mod = sqrt(mass2 + pm[0] * pm[0] + pm[1] * pm[1] + pm[2] * pm[2]);
                f = fabs(renorm) / (exp(E_mod / lambda - chem_effect) + sign);
              }
              eta_integral += (eta_weight * p_dsigma * f);
            }
            slice[iS3D] += (prefactor * degeneracy * eta_integral);
          }
        }
      }
    }
  CELL_LOOP_END
}

/* ------------------------------------------------------------------------- */
/* operation = 0: spacetime distributions dN/dX                               */
/* SpacetimeDistribution.cpp:31-518 (calculate_dN_dX, df_mode 1/2) and        */
/* :520-1250 (calculate_dN_dX_feqmod, df_mode 3/4).  The reference loops       */
/* species -> threads -> cells and recomputes the (species-independent) cell   */
/* prologue for every species; here the prologue is computed once per cell and */
/* the species loop is inside -- same arithmetic, same values.  Output: the    */
/* per-(species, cell) dN/dy of the cell (dN_dy_cell, :374 / :1131), 0 for     */
/* skipped cells.                                                              */
/* ------------------------------------------------------------------------- */
static void dndx_cell_grad_ce(const orc_params *p, const orc_setup *s, const orc_surface *S, const dfdata *df_data,
                              const grid *g, const double *pTw, const double *phiw, long ic, long ncell,
                              double *cy, char *valid, int *err) {
  const double prefactor = pow(2.0 * M_PI * HBARC, -3);
  const long npart = s->npart, npT = g->npT, nphi = g->nphi, ny = g->ny, neta = g->neta;
  const int DF_MODE = p->df_mode;
  double tau = S->tau[ic], tau2 = tau * tau;
  double eta0 = (p->dimension == 3) ? S->eta[ic] : 0.0;     /* :181-184, thread-local (race fix) */
  double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
  double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
  double ut = sqrt(1.0 + ux * ux + uy * uy + tau2 * un * un);
  if (ut * dat + ux * dax + uy * day + un * dan <= 0.0) return;   /* :197 */
  double ux2 = ux * ux, uy2 = uy * uy, ut2 = ut * ut, utperp = sqrt(1.0 + ux * ux + uy * uy);
  double T = S->T[ic], P = S->P[ic], E = S->E[ic];
  double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
  if (p->include_shear_deltaf) {
    pixx = S->pixx[ic]; pixy = S->pixy[ic]; pixn = S->pixn[ic]; piyy = S->piyy[ic]; piyn = S->piyn[ic];
    pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
    pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
    pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
    pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
  }
  double bulkPi = 0.0;
  if (p->include_bulk_deltaf) bulkPi = S->bulkPi[ic];
  double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
  if (p->include_baryon && p->include_baryondiff_deltaf) {
    muB = S->muB[ic]; nB = S->nB[ic]; Vx = S->Vx[ic]; Vy = S->Vy[ic]; Vn = S->Vn[ic];
    Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
    alphaB = muB / T;
    ber = nB / (E + P);
  }
  dfcoef df;
  int rc = df_eval(df_data, T, muB, E, P, bulkPi, &df);
  if (rc) { *err = rc; return; }
  double c3 = df.c3, c4 = df.c4, betaV = df.betaV;
  double shear_coeff = 0, bulk0 = 0, bulk1 = 0, bulk2 = 0;       /* :266-290 */
  if (DF_MODE == 1) {
    shear_coeff = 0.5 / (T * T * (E + P));
    bulk0 = df.c0 - df.c2; bulk1 = df.c1; bulk2 = 4.0 * df.c2 - df.c0;
  } else {
    shear_coeff = 0.5 / (df.betapi * T);
    bulk0 = df.F / (T * T * df.betabulk); bulk1 = df.G / df.betabulk; bulk2 = 1.0 / (3.0 * T * df.betabulk);
  }
  for (long ipart = 0; ipart < npart; ipart++) {
    double mass = s->mass[ipart], mass2 = mass * mass, sign = s->sign[ipart];
    double degeneracy = s->degen[ipart], baryon = s->baryon[ipart];
    double chem = baryon * alphaB;
    double dN_dy_cell = 0.0;
    for (long ipT = 0; ipT < npT; ipT++) {                         /* :296-378 */
      double pT = g->pT[ipT], mT = sqrt(mass2 + pT * pT), mT_over_tau = mT / tau;
      double pT_weight = pTw[ipT];
      for (long iphip = 0; iphip < nphi; iphip++) {
        double px = pT * g->cosphi[iphip], py = pT * g->sinphi[iphip];
        double phi_weight = phiw[iphip];
        for (long iy = 0; iy < ny; iy++) {
          double y = g->yv[iy];
          double eta_integral = 0.0;
          for (long ieta = 0; ieta < neta; ieta++) {
            double eta = (p->dimension == 3) ? eta0 : g->etav[ieta];
            double eta_weight = g->etaw[ieta];
            double pt = mT * cosh(y - eta), pn = mT_over_tau * sinh(y - eta), tau2_pn = tau2 * pn;
            double pdotdsigma = eta_weight * (pt * dat + px * dax + py * day + pn * dan);
            if (p->outflow && pdotdsigma <= 0.0) continue;
            double pdotu = pt * ut - px * ux - py * uy - tau2_pn * un;
            double feq = 1.0 / (exp(pdotu / T - chem) + sign);
            double feqbar = 1.0 - sign * feq;
            double pimunu_pmu_pnu = pitt * pt * pt + pixx * px * px + piyy * py * py + pinn * tau2_pn * tau2_pn
                + 2.0 * (-(pitx * px + pity * py) * pt + pixy * px * py + tau2_pn * (pixn * px + piyn * py - pitn * pt));
            double Vmu_pmu = Vt * pt - Vx * px - Vy * py - Vn * tau2_pn;
            double dfv;
            if (DF_MODE == 1) {
              double df_shear = shear_coeff * pimunu_pmu_pnu;
              double df_bulk = (bulk0 * mass2 + (bulk1 * baryon + bulk2 * pdotu) * pdotu) * bulkPi;
              double df_diff = (c3 * baryon + c4 * pdotu) * Vmu_pmu;
              dfv = feqbar * (df_shear + df_bulk + df_diff);
            } else {
              double df_shear = shear_coeff * pimunu_pmu_pnu / pdotu;
              double df_bulk = (bulk0 * pdotu + bulk1 * baryon + bulk2 * (pdotu - mass2 / pdotu)) * bulkPi;
              double df_diff = (ber - baryon / pdotu) * Vmu_pmu / betaV;
              dfv = feqbar * (df_shear + df_bulk + df_diff);
            }
            if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
            double f = feq * (1.0 + dfv);
            eta_integral += (pdotdsigma * f);
          }
          dN_dy_cell += (pT_weight * phi_weight * prefactor * degeneracy * eta_integral);
        }
      }
    }
    cy[ipart * ncell + ic] = dN_dy_cell;
    valid[ipart * ncell + ic] = 1;
  }
}

static void dndx_cell_feqmod(const orc_params *p, const orc_setup *s, const orc_surface *S, const dfdata *df_data,
                             const grid *g, const double *pTw, const double *phiw, long ic, long ncell,
                             double *cy, char *valid, long *skipped, int *err) {
  const double prefactor = pow(2.0 * M_PI * HBARC, -3);
  const long npart = s->npart, npT = g->npT, nphi = g->nphi, ny = g->ny, neta = g->neta;
  const int DF_MODE = p->df_mode, DIMENSION = p->dimension;
  const double detA_min = p->deta_min;
  const int pts = s->gla_points;
  const double *r1 = s->gla_root + pts, *r2 = s->gla_root + 2 * pts;
  const double *w1 = s->gla_weight + pts, *w2 = s->gla_weight + 2 * pts;
  double A_copy[3][3], A_inv[3][3];
  double tau = S->tau[ic], tau2 = tau * tau;
  double eta0 = (DIMENSION == 3) ? S->eta[ic] : 0.0;
  double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
  double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
  double ut = sqrt(1.0 + ux * ux + uy * uy + tau2 * un * un);
  double udsigma = ut * dat + ux * dax + uy * day + un * dan;
  if (udsigma <= 0.0) return;                                      /* :695 */
  double ux2 = ux * ux, uy2 = uy * uy, ut2 = ut * ut;
  double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
  double T = S->T[ic], P = S->P[ic], E = S->E[ic];
  double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
  if (p->include_shear_deltaf) {
    pixx = S->pixx[ic]; pixy = S->pixy[ic]; pixn = S->pixn[ic]; piyy = S->piyy[ic]; piyn = S->piyn[ic];
    pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2.0 * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
    pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
    pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
    pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
    pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
  }
  double bulkPi = 0.0;
  if (p->include_bulk_deltaf) bulkPi = S->bulkPi[ic];
  double muB = 0, alphaB = 0, nB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0, ber = 0;
  if (p->include_baryon && p->include_baryondiff_deltaf) {
    muB = S->muB[ic]; nB = S->nB[ic]; Vx = S->Vx[ic]; Vy = S->Vy[ic]; Vn = S->Vn[ic];
    Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
    alphaB = muB / T;
    ber = nB / (E + P);
  }
  if (DF_MODE == 4) {   /* :766-772 (note <= / >=, the spectra path uses < / >) */
    double bulkPi_over_Peq_max = df_data->bulkPi_over_Peq_max;
    if (bulkPi <= -P) bulkPi = -(1.0 - 1.e-5) * P;
    else if (bulkPi / P >= bulkPi_over_Peq_max) bulkPi = P * (bulkPi_over_Peq_max - 1.e-5);
  }
  dfcoef df;
  int rc = df_eval(df_data, T, muB, E, P, bulkPi, &df);
  if (rc) { *err = rc; return; }
  double F = df.F, G = df.G, betabulk = df.betabulk, betaV = df.betaV, betapi = df.betapi;
  double lambda = df.lambda, z = df.z, delta_lambda = df.delta_lambda, delta_z = df.delta_z;
  milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  pilrf pl_ = boost_pimunu(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
  double T_mod = T, alphaB_mod = alphaB;
  if (DF_MODE == 3) { T_mod = T + bulkPi * F / betabulk; alphaB_mod = alphaB + bulkPi * G / betabulk; }
  double shear_coeff = 0.5 / (betapi * T);
  double bulk0 = F / (T * T * betabulk), bulk1 = G / betabulk, bulk2 = 1.0 / (3.0 * T * betabulk);
  double shear_mod = 0.5 / betapi, bulk_mod = bulkPi / (3.0 * betabulk);
  if (DF_MODE == 4) bulk_mod = lambda;
  double Axx = 1.0 + pl_.xx * shear_mod + bulk_mod, Axy = pl_.xy * shear_mod, Axz = pl_.xz * shear_mod;
  double Ayy = 1.0 + pl_.yy * shear_mod + bulk_mod, Ayz = pl_.yz * shear_mod, Azz = 1.0 + pl_.zz * shear_mod + bulk_mod;
  double detA = Axx * (Ayy * Azz - Ayz * Ayz) - Axy * (Axy * Azz - Ayz * Axz) + Axz * (Axy * Ayz - Ayy * Axz);
  double detA_b23 = pow(1.0 + bulk_mod, 2);
  int breaks = feqmod_breaks_down(p->mass_pion0, T, F, bulkPi, betabulk, detA, detA_min, z, s, DF_MODE);
  double A[9] = {Axx, Axy, Axz, Axy, Ayy, Ayz, Axz, Ayz, Azz};
  for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) A_copy[i][j] = A[3 * i + j];
  inverse3(A, A_inv);
  double neq_fact = T * T * T / two_pi2_hbarC3();
  double dn_fact = bulkPi / betabulk, J20_fact = T * neq_fact, N10_fact = neq_fact;
  double nmod_fact = T_mod * T_mod * T_mod / two_pi2_hbarC3();
  double eta_scale = 1.0;
  if (detA > detA_min && DIMENSION == 2) eta_scale = detA / detA_b23;
  for (long ipart = 0; ipart < npart; ipart++) {
    double mass = s->mass[ipart], mass2 = mass * mass, sign = s->sign[ipart];
    double degeneracy = s->degen[ipart], baryon = s->baryon[ipart];
    double chem = baryon * alphaB, chem_mod = baryon * alphaB_mod;
    double renorm = 1.0;                                            /* :932-970 */
    if (p->include_bulk_deltaf) {
      if (DF_MODE == 3) {
        double mbar = mass / T, mbar_mod = mass / T_mod;
        double neq = neq_fact * degeneracy * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar, alphaB, baryon, sign);
        double N10 = baryon * N10_fact * degeneracy * orc_gauss_thermal(GT_J10, r1, w1, pts, mbar, alphaB, baryon, sign);
        double J20 = J20_fact * degeneracy * orc_gauss_thermal(GT_J20, r2, w2, pts, mbar, alphaB, baryon, sign);
        double n_linear = neq + dn_fact * (neq + N10 * G + J20 * F / T / T);
        double n_mod = nmod_fact * degeneracy * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar_mod, alphaB_mod, baryon, sign);
        renorm = n_linear / n_mod;
      } else if (DF_MODE == 4) {
        renorm = z;
      }
    }
    if (DIMENSION == 2) renorm /= detA_b23; else renorm /= detA;
    if (isnan(renorm) || isinf(renorm)) { (*skipped)++; continue; }   /* :972-976: cell not binned */
    double dN_dy_cell = 0.0;
    for (long ipT = 0; ipT < npT; ipT++) {
      double pT = g->pT[ipT], mT = sqrt(mass2 + pT * pT), mT_over_tau = mT / tau;
      double pT_weight = pTw[ipT];
      for (long iphip = 0; iphip < nphi; iphip++) {
        double px = pT * g->cosphi[iphip], py = pT * g->sinphi[iphip];
        double phi_weight = phiw[iphip];
        for (long iy = 0; iy < ny; iy++) {
          double y = g->yv[iy];
          double eta_integral = 0.0;
          for (long ieta = 0; ieta < neta; ieta++) {
            double eta = (DIMENSION == 3) ? eta0 : g->etav[ieta];
            double eta_weight = g->etaw[ieta];
            int narrow = 0;
            if (DIMENSION == 3 && !breaks) { if (detA < 0.01 && fabs(y - eta) < detA) narrow = 1; }
            double pdotdsigma, f;
            if (breaks || narrow) {                                 /* :1015-1071 */
              double pt = mT * cosh(y - eta), pn = mT_over_tau * sinh(y - eta), tau2_pn = tau2 * pn;
              pdotdsigma = eta_weight * (pt * dat + px * dax + py * day + pn * dan);
              if (p->outflow && pdotdsigma <= 0.0) continue;
              double pdotu = pt * ut - px * ux - py * uy - tau2_pn * un;
              double ppp = pitt * pt * pt + pixx * px * px + piyy * py * py + pinn * tau2_pn * tau2_pn
                  + 2.0 * (-(pitx * px + pity * py) * pt + pixy * px * py + tau2_pn * (pixn * px + piyn * py - pitn * pt));
              if (DF_MODE == 3) {
                double feq = 1.0 / (exp(pdotu / T - chem) + sign);
                double feqbar = 1.0 - sign * feq;
                double Vp = Vt * pt - Vx * px - Vy * py - Vn * tau2_pn;
                double df_shear = shear_coeff * ppp / pdotu;
                double df_bulk = (bulk0 * pdotu + bulk1 * baryon + bulk2 * (pdotu - mass2 / pdotu)) * bulkPi;
                double df_diff = (ber - baryon / pdotu) * Vp / betaV;
                double dfv = feqbar * (df_shear + df_bulk + df_diff);
                if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
                f = feq * (1.0 + dfv);
              } else {
                double feq = 1.0 / (exp(pdotu / T) + sign);
                double feqbar = 1.0 - sign * feq;
                double df_shear = feqbar * shear_coeff * ppp / pdotu;
                double df_bulk = delta_z - 3.0 * delta_lambda + feqbar * delta_lambda * (pdotu - mass2 / pdotu) / T;
                double dfv = df_shear + df_bulk;
                if (p->regulate_deltaf) dfv = fmax(-1.0, fmin(dfv, 1.0));
                f = feq * (1.0 + dfv);
              }
            } else {                                                /* :1073-1122 */
              double pt = mT * cosh(y - eta_scale * eta), pn = mT_over_tau * sinh(y - eta_scale * eta), tau2_pn = tau2 * pn;
              pdotdsigma = eta_weight * (pt * dat + px * dax + py * day + pn * dan);
              if (p->outflow && pdotdsigma <= 0.0) continue;
              double pLRF[3] = {-b.Xt * pt + b.Xx * px + b.Xy * py + b.Xn * tau2_pn, b.Yx * px + b.Yy * py, -b.Zt * pt + b.Zn * tau2_pn};
              double pm[3], pmp[3], pp[3], dpv[3], dpm[3];
              matvec3(A_inv, pLRF, pm);
              for (int it = 0; it < 5; it++) {
                for (int q = 0; q < 3; q++) pmp[q] = pm[q];
                matvec3(A_copy, pmp, pp);
                for (int q = 0; q < 3; q++) dpv[q] = pLRF[q] - pp[q];
                double dp = sqrt(dpv[0] * dpv[0] + dpv[1] * dpv[1] + dpv[2] * dpv[2]);
                if (dp <= 1.e-16) break;
                matvec3(A_inv, dpv, dpm);
                for (int q = 0; q < 3; q++) pm[q] = pmp[q] + dpm[q];
              }
              double E_mod = sqrt(mass2 + pm[0] * pm[0] + pm[1] * pm[1] + pm[2] * pm[2]);
              f = fabs(renorm) / (exp(E_mod / T_mod - chem_mod) + sign);
            }
            eta_integral += (pdotdsigma * f);
          }
          dN_dy_cell += (pT_weight * phi_weight * prefactor * degeneracy * eta_integral);
        }
      }
    }
    cy[ipart * ncell + ic] = dN_dy_cell;
    valid[ipart * ncell + ic] = 1;
  }
}

/* The reference's per-species binning (:380-404 / :1136-1160) into thread slices all[i + n*bins],
 * the per-species reset memset(all, 0, C*bins) -- a BYTE count, so only the first C*bins/8 doubles
 * (and the low bytes of the next one) are cleared and the rest carries over from the previous
 * species when carry != 0 -- and the per-bin sum over threads + bin-width normalisation written to
 * the files (:407-440 / :1163-1194). */
static void dndx_bin(const orc_surface *S, const orc_bins *B, long C, int carry, long npart, const double *cy,
                     const char *valid, double *tau_out, double *r_out, double *phi_out) {
  const double two_pi = 2.0 * M_PI;
  const long taubins = B->tau_bins, rbins = B->r_bins, phibins = B->phip_bins;
  const double TAU_WIDTH = (B->tau_max - B->tau_min) / (double)B->tau_bins;
  const double R_WIDTH = (B->r_max - B->r_min) / (double)B->r_bins;
  const double PHIP_WIDTH = two_pi / (double)B->phip_bins;
  double *at = (double *)calloc((size_t)C * taubins, sizeof(double));
  double *ar = (double *)calloc((size_t)C * rbins, sizeof(double));
  double *ap = (double *)calloc((size_t)C * phibins, sizeof(double));
  const long n_cells = S->n;
  for (long ipart = 0; ipart < npart; ipart++) {
    if (carry) {
      memset(at, 0, (size_t)(C * taubins)); memset(ar, 0, (size_t)(C * rbins)); memset(ap, 0, (size_t)(C * phibins));
    } else {
      memset(at, 0, sizeof(double) * C * taubins); memset(ar, 0, sizeof(double) * C * rbins);
      memset(ap, 0, sizeof(double) * C * phibins);
    }
    for (long n = 0; n < C; n++) {
      CELL_LOOP_BEGIN(n, C, n_cells, ic)
        if (!valid[ipart * n_cells + ic]) continue;
        double dN_dy_cell = cy[ipart * n_cells + ic];
        double x_pos = S->x[ic], y_pos = S->y[ic], tau = S->tau[ic];
        double r = sqrt(x_pos * x_pos + y_pos * y_pos);
        double phi = atan2(y_pos, x_pos);
        if (phi < 0.0) phi += two_pi;
        long itau = (int)floor((tau - B->tau_min) / TAU_WIDTH);
        long ir = (int)floor((r - B->r_min) / R_WIDTH);
        long iphi = (int)floor(phi / PHIP_WIDTH);
        if (itau >= 0 && itau < taubins) at[itau + n * taubins] += dN_dy_cell;
        if (ir >= 0 && ir < rbins) ar[ir + n * rbins] += dN_dy_cell;
        if (iphi >= 0 && iphi < phibins) ap[iphi + n * phibins] += dN_dy_cell;
      CELL_LOOP_END
    }
    for (long ir = 0; ir < rbins; ir++) {
      double acc = 0.0;
      for (long n = 0; n < C; n++) acc += ar[ir + n * rbins];
      double r_mid = B->r_min + R_WIDTH * ((double)ir + 0.5);
      r_out[ipart * rbins + ir] = acc / (two_pi * r_mid * R_WIDTH);
    }
    for (long itau = 0; itau < taubins; itau++) {
      double acc = 0.0;
      for (long n = 0; n < C; n++) acc += at[itau + n * taubins];
      double tau_mid = B->tau_min + TAU_WIDTH * ((double)itau + 0.5);
      tau_out[ipart * taubins + itau] = acc / (tau_mid * TAU_WIDTH);
    }
    for (long iphi = 0; iphi < phibins; iphi++) {
      double acc = 0.0;
      for (long n = 0; n < C; n++) acc += ap[iphi + n * phibins];
      phi_out[ipart * phibins + iphi] = acc / PHIP_WIDTH;
    }
  }
  free(at); free(ar); free(ap);
}

int orc_dndx(const orc_params *p, const orc_setup *s, const orc_surface *surf, const orc_bins *B,
             double *cell_yield, double *tau_out, double *r_out, double *phi_out, long *stats, char *err, int errlen) {
  if (p->dimension != 2 && p->dimension != 3) { seterr(err, errlen, "EmissionFunctionArray error: need to set dimension = (2,3)"); return 1; }
  if (p->df_mode == 5) { seterr(err, errlen, "calculate_spectra error: no spacetime distribution routine for famod yet"); return 1; }
  if (p->df_mode < 1 || p->df_mode > 5) { seterr(err, errlen, "calculate_spectra error: need to set df_mode = (1, 2, 3, 4, 5)"); return 1; }
  if (B->tau_bins <= 0 || B->r_bins <= 0 || B->phip_bins <= 0) { seterr(err, errlen, "spacetime bins must be positive"); return 1; }
  dfdata d;
  if (df_setup(&d, p, s, 1)) { seterr(err, errlen, "gsl: x values must be strictly increasing (Jonah table)"); df_free(&d); return 1; }
  grid g;
  grid_setup(&g, p, s);
  const long n_cells = surf->n, npart = s->npart;
  const long C = p->threads > 0 ? p->threads : 1;
  double *pTw = (double *)malloc(sizeof(double) * (g.npT + 1)), *phiw = (double *)malloc(sizeof(double) * (g.nphi + 1));
  for (long i = 0; i < g.npT; i++) pTw[i] = s->pT_w ? s->pT_w[i] : 0.0;
  for (long j = 0; j < g.nphi; j++) phiw[j] = s->phi_w ? s->phi_w[j] : 0.0;
  double *cy = (double *)calloc((size_t)npart * (n_cells > 0 ? n_cells : 1), sizeof(double));
  int *cerr = (int *)calloc((size_t)(n_cells > 0 ? n_cells : 1), sizeof(int));
  long *cskip = (long *)calloc((size_t)(n_cells > 0 ? n_cells : 1), sizeof(long));
  /* valid[ipart][cell]: the cell passed u.dsigma > 0 (and a finite renorm); skipped cells are never binned */
  char *valid = (char *)calloc((size_t)npart * (n_cells > 0 ? n_cells : 1), 1);
#ifdef _OPENMP
  int nthr = p->omp_threads > 0 ? p->omp_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthr)
#endif
  for (long ic = 0; ic < n_cells; ic++) {
    if (p->df_mode <= 2) dndx_cell_grad_ce(p, s, surf, &d, &g, pTw, phiw, ic, n_cells, cy, valid, &cerr[ic]);
    else dndx_cell_feqmod(p, s, surf, &d, &g, pTw, phiw, ic, n_cells, cy, valid, &cskip[ic], &cerr[ic]);
  }
  int rc = 0;
  long skipped = 0;
  for (long ic = 0; ic < n_cells; ic++) { if (cerr[ic] && !rc) rc = cerr[ic]; skipped += cskip[ic]; }
  if (rc) seterr(err, errlen, df_errmsg(rc));
  else dndx_bin(surf, B, C, B->carry, npart, cy, valid, tau_out, r_out, phi_out);
  if (cell_yield) memcpy(cell_yield, cy, sizeof(double) * npart * n_cells);
  if (stats) { for (int i = 0; i < ORC_NSTATS; i++) stats[i] = 0; stats[4] = skipped; }
  free(pTw); free(phiw); free(cy); free(cerr); free(cskip); free(valid);
  grid_free(&g); df_free(&d);
  return rc ? 1 : 0;
}

/* ------------------------------------------------------------------------- */
/* drivers                                                                    */
/* ------------------------------------------------------------------------- */
int orc_spectra(const orc_params *p, const orc_setup *s, const orc_surface *surf,
                double *out, long *stats, char *err, int errlen) {
  if (p->dimension != 2 && p->dimension != 3) { seterr(err, errlen, "EmissionFunctionArray error: need to set dimension = (2,3)"); return 1; }
  if (p->df_mode < 1 || p->df_mode > 5) { seterr(err, errlen, "EmissionFunctionArray error: need to set df_mode = (1,2,3,4,5)"); return 1; }
  dfdata d;
  if (df_setup(&d, p, s, 1)) { seterr(err, errlen, "gsl: x values must be strictly increasing (Jonah table)"); df_free(&d); return 1; }
  grid g;
  grid_setup(&g, p, s);
  const long C = p->threads > 0 ? p->threads : 1;
  const size_t N = (size_t)s->npart * g.npT * g.nphi * g.ny;
  double *all = (double *)calloc((size_t)C * N, sizeof(double));
  tstats *ts = (tstats *)calloc((size_t)C, sizeof(tstats));
#ifdef _OPENMP
  int nthr = p->omp_threads > 0 ? p->omp_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthr)
#endif
  for (long n = 0; n < C; n++) {
    double *slice = all + (size_t)n * N;
    if (p->df_mode <= 2) spectra_grad_ce(p, s, surf, &d, &g, n, C, slice, &ts[n]);
    else if (p->df_mode <= 4) spectra_feqmod(p, s, surf, &d, &g, n, C, slice, &ts[n]);
    else spectra_famod(p, s, surf, &g, n, C, slice, &ts[n]);
  }
  int rc = 0;
  long st[ORC_NSTATS] = {0};
  for (long n = 0; n < C; n++) {
    if (ts[n].err && !rc) rc = ts[n].err;
    st[0] += ts[n].breakdown; st[1] += ts[n].pl_negative; st[2] += ts[n].recon_fail;
    st[3] += ts[n].iterations; st[4] += ts[n].skipped;
  }
  if (rc) seterr(err, errlen, df_errmsg(rc));
  /* reduction over threads (MomentumSpectra.cpp:383-411) */
  for (size_t i = 0; i < N; i++) {
    double acc = 0.0;
    for (long n = 0; n < C; n++) acc += all[(size_t)n * N + i];
    out[i] = acc;
  }
  if (stats) for (int i = 0; i < ORC_NSTATS; i++) stats[i] = st[i];
  free(all); free(ts); grid_free(&g); df_free(&d);
  return rc ? 1 : 0;
}

int orc_df_coefficients(const orc_params *p, const orc_setup *s, double T, double muB, double E, double P,
                        double bulkPi, double *out, char *err, int errlen) {
  dfdata d;
  int need_jonah = (p->df_mode == 4);
  if (df_setup(&d, p, s, need_jonah)) { seterr(err, errlen, "jonah table not monotonic"); df_free(&d); return 1; }
  dfcoef df;
  int rc = df_eval(&d, T, muB, E, P, bulkPi, &df);
  double o[15] = {df.c0, df.c1, df.c2, df.c3, df.c4, df.shear14, df.F, df.G, df.betabulk, df.betaV, df.betapi,
                  df.lambda, df.z, df.delta_lambda, df.delta_z};
  memcpy(out, o, sizeof(o));
  if (rc) seterr(err, errlen, df_errmsg(rc));
  df_free(&d);
  return rc;
}

int orc_jonah_table(const orc_setup *s, double *lambda2, double *z, double *bp, double *bpmax) {
  dfdata d;
  memset(&d, 0, sizeof(d));
  int rc = jonah(&d, s);
  if (d.jl2) { memcpy(lambda2, d.jl2, 301 * sizeof(double)); memcpy(z, d.jz, 301 * sizeof(double)); memcpy(bp, d.jx, 301 * sizeof(double)); }
  *bpmax = d.bulkPi_over_Peq_max;
  df_free(&d);
  return rc;
}

/* readindata.cpp:316-366: ds_max-weighted averages, then the 15-digit file round trip */
void orc_surface_averages(const orc_surface *S, double *out) {
  double T_avg = 0, E_avg = 0, P_avg = 0, muB_avg = 0, nB_avg = 0, vol = 0;
  for (long i = 0; i < S->n; i++) {
    double tau = S->tau[i], tau2 = tau * tau, ux = S->ux[i], uy = S->uy[i], un = S->un[i];
    double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
    double dat = S->dat[i], dax = S->dax[i], day = S->day[i], dan = S->dan[i];
    double uds = ut * dat + ux * dax + uy * day + un * dan;
    double ds_ds = dat * dat - dax * dax - day * day - dan * dan / tau2;
    double ds_max = fabs(uds) + sqrt(fabs(uds * uds - ds_ds));
    double muB = S->muB ? S->muB[i] : 0.0, nB = S->nB ? S->nB[i] : 0.0;
    vol += ds_max; E_avg += (S->E[i] * ds_max); T_avg += (S->T[i] * ds_max); P_avg += (S->P[i] * ds_max);
    muB_avg += (muB * ds_max); nB_avg += (nB * ds_max);
  }
  double v[5] = {T_avg / vol, E_avg / vol, P_avg / vol, muB_avg / vol, nB_avg / vol};
  for (int k = 0; k < 5; k++) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.15g", v[k]);
    out[k] = strtod(buf, NULL);
  }
}

/* ------------------------------------------------------------------------- */
/* operation = 2 oversampling estimate                                        */
/* DeltafData.cpp:555-690 compute_particle_densities (Plasma averages, bulkPi = 0 coefficients)  */
/* ParticleSampler.cpp:447-636 calculate_total_yield, :75-119 estimate_mean_particle_number      */
/* ------------------------------------------------------------------------- */
static void orc_particle_densities(const orc_params *p, const orc_setup *s, const dfcoef *df, const double *plasma,
                            double *neq_out, double *bulk_out, double *diff_out) {
  const double T = plasma[0], E = plasma[1], P = plasma[2], muB = plasma[3], nB = plasma[4];
  const double alphaB = muB / T, ber = nB / (E + P);
  const int pts = s->gla_points;
  const double *r1 = s->gla_root + pts, *r2 = s->gla_root + 2 * pts, *r3 = s->gla_root + 3 * pts;
  const double *w1 = s->gla_weight + pts, *w2 = s->gla_weight + 2 * pts, *w3 = s->gla_weight + 3 * pts;
  for (int i = 0; i < s->npart; i++) {
    double mass = s->mass[i], degeneracy = s->degen[i], baryon = s->baryon[i], sign = s->sign[i];
    double mbar = mass / T;
    double neq_fact = degeneracy * pow(T, 3) / two_pi2_hbarC3();
    double neq = neq_fact * orc_gauss_thermal(GT_NEQ, r1, w1, pts, mbar, alphaB, baryon, sign);
    double dn_bulk = 0.0, dn_diff = 0.0;
    if (p->df_mode == 1) {                                   /* :614-638 */
      double J10_fact = degeneracy * pow(T, 3) / two_pi2_hbarC3();
      double J20_fact = degeneracy * pow(T, 4) / two_pi2_hbarC3();
      double J30_fact = degeneracy * pow(T, 5) / two_pi2_hbarC3();
      double J31_fact = degeneracy * pow(T, 5) / two_pi2_hbarC3() / 3.0;
      double J10 = J10_fact * orc_gauss_thermal(GT_J10, r1, w1, pts, mbar, alphaB, baryon, sign);
      double J20 = J20_fact * orc_gauss_thermal(GT_J20, r2, w2, pts, mbar, alphaB, baryon, sign);
      double J30 = J30_fact * orc_gauss_thermal(GT_J30, r3, w3, pts, mbar, alphaB, baryon, sign);
      double J31 = J31_fact * orc_gauss_thermal(GT_J31, r3, w3, pts, mbar, alphaB, baryon, sign);
      dn_bulk = ((df->c0 - df->c2) * mass * mass * J10 + df->c1 * baryon * J20 + (4.0 * df->c2 - df->c0) * J30);
      dn_diff = baryon * df->c3 * neq * T + df->c4 * J31;
    } else if (p->df_mode == 2 || p->df_mode == 3 || p->df_mode == 5) {   /* :639-661, 666-669 */
      double J10_fact = degeneracy * pow(T, 3) / two_pi2_hbarC3();
      double J11_fact = degeneracy * pow(T, 3) / two_pi2_hbarC3() / 3.0;
      double J20_fact = degeneracy * pow(T, 4) / two_pi2_hbarC3();
      double J10 = J10_fact * orc_gauss_thermal(GT_J10, r1, w1, pts, mbar, alphaB, baryon, sign);
      double J11 = J11_fact * orc_gauss_thermal(GT_J11, r1, w1, pts, mbar, alphaB, baryon, sign);
      double J20 = J20_fact * orc_gauss_thermal(GT_J20, r2, w2, pts, mbar, alphaB, baryon, sign);
      dn_bulk = (neq + (baryon * J10 * df->G) + (J20 * df->F / pow(T, 2))) / df->betabulk;
      dn_diff = (neq * T * ber - baryon * J11) / df->betaV;
    }
    neq_out[i] = neq; bulk_out[i] = dn_bulk; diff_out[i] = dn_diff;
  }
}

/* Surface_Element_Vector::boost_dsigma_to_lrf + compute_dsigma_magnitude (LocalRestFrame.cpp:81-98).
 * in[9] = ut ux uy un tau dat dax day dan; out[5] = u.dsigma, dsigma_{x,y,z} LRF, dsigma_space */
void orc_dsigma_lrf(const double *in, double *out) {
  double ut = in[0], ux = in[1], uy = in[2], un = in[3], tau = in[4];
  double dat = in[5], dax = in[6], day = in[7], dan = in[8];
  double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
  milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
  out[0] = dat * ut + dax * ux + day * uy + dan * un;
  out[1] = -(dat * b.Xt + dax * b.Xx + day * b.Xy + dan * b.Xn);
  out[2] = -(dax * b.Yx + day * b.Yy);
  out[3] = -(dat * b.Zt + dan * b.Zn);
  out[4] = sqrt(out[1] * out[1] + out[2] * out[2] + out[3] * out[3]);
}

/* Reference loop is serial (its OpenMP pragma is commented out, :456): cells in order, species inner.
 * ds_space follows Surface_Element_Vector::compute_dsigma_magnitude (LocalRestFrame.cpp:94-98); the
 * reference reads the member without calling it (:582-583), i.e. an uninitialised value, which only
 * enters through ds_space * Vdsigma * diffusion_density (baryon diffusion on). */
int orc_total_yield(const orc_params *p, const orc_setup *s, const orc_surface *S, const double *plasma, double y_cut,
                    double *n_total, double *densities, char *err, int errlen) {
  if (p->df_mode < 1 || p->df_mode > 5) { seterr(err, errlen, "Estimate particle yield error: please set df_mode = (1,2,3,4,5)"); return 1; }
  dfdata d;
  if (df_setup(&d, p, s, 1)) { seterr(err, errlen, "gsl: x values must be strictly increasing (Jonah table)"); df_free(&d); return 1; }
  const int npart = s->npart;
  double *neq = (double *)malloc(sizeof(double) * (3 * npart + 1)), *bulk = neq + npart, *diff = bulk + npart;
  dfcoef dfa;
  int rc = df_eval(&d, plasma[0], plasma[3], plasma[1], plasma[2], 0.0, &dfa);   /* DeltafData.cpp:574 */
  if (rc) { seterr(err, errlen, df_errmsg(rc)); free(neq); df_free(&d); return 1; }
  orc_particle_densities(p, s, &dfa, plasma, neq, bulk, diff);
  if (densities) memcpy(densities, neq, sizeof(double) * 3 * npart);
  const int DF_MODE = p->df_mode;
  double Ntot = 0.0;
  for (long ic = 0; ic < S->n; ic++) {
    double tau = S->tau[ic], tau2 = tau * tau;
    double dat = S->dat[ic], dax = S->dax[ic], day = S->day[ic], dan = S->dan[ic];
    double ux = S->ux[ic], uy = S->uy[ic], un = S->un[ic];
    double ut = sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
    double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1. + ux * ux + uy * uy);
    double ux2 = ux * ux, uy2 = uy * uy, ut2 = ut * ut;
    double udsigma = ut * dat + ux * dax + uy * day + un * dan;
    if (udsigma <= 0) continue;
    double T = S->T[ic], P = S->P[ic], E = S->E[ic];
    double pitt = 0, pitx = 0, pity = 0, pitn = 0, pixx = 0, pixy = 0, pixn = 0, piyy = 0, piyn = 0, pinn = 0;
    if (p->include_shear_deltaf) {
      pixx = S->pixx[ic]; pixy = S->pixy[ic]; pixn = S->pixn[ic]; piyy = S->piyy[ic]; piyn = S->piyn[ic];
      pinn = (pixx * (ux2 - ut2) + piyy * (uy2 - ut2) + 2. * (pixy * ux * uy + tau2 * un * (pixn * ux + piyn * uy))) / (tau2 * utperp * utperp);
      pitn = (pixn * ux + piyn * uy + tau2 * pinn * un) / ut;
      pity = (pixy * ux + piyy * uy + tau2 * piyn * un) / ut;
      pitx = (pixx * ux + pixy * uy + tau2 * pixn * un) / ut;
      pitt = (pitx * ux + pity * uy + tau2 * pitn * un) / ut;
    }
    double bulkPi = p->include_bulk_deltaf ? S->bulkPi[ic] : 0.0;
    double muB = 0, Vt = 0, Vx = 0, Vy = 0, Vn = 0;
    if (p->include_baryon && p->include_baryondiff_deltaf) {
      muB = S->muB[ic];
      Vx = S->Vx[ic]; Vy = S->Vy[ic]; Vn = S->Vn[ic];
      Vt = (Vx * ux + Vy * uy + tau2 * Vn * un) / ut;
    }
    double Vdsigma = Vt * dat + Vx * dax + Vy * day + Vn * dan;
    if (DF_MODE == 4) {                                        /* :548-560 */
      if (bulkPi <= -P) bulkPi = -(1.0 - 1.e-5) * P;
      else if (bulkPi / P >= d.bulkPi_over_Peq_max) bulkPi = P * (d.bulkPi_over_Peq_max - 1.e-5);
    }
    dfcoef df;
    rc = df_eval(&d, T, muB, E, P, bulkPi, &df);
    if (rc) break;
    milne b = milne_basis(ut, ux, uy, un, uperp, utperp, tau);
    double dsin[9] = {ut, ux, uy, un, tau, dat, dax, day, dan}, dso[5];
    orc_dsigma_lrf(dsin, dso);
    double ds_time = dso[0], ds_space = dso[4];
    int breaks = 0;
    if (DF_MODE == 4) {          /* the only mode whose estimate depends on the breakdown (:91-104) */
      pilrf pl_ = boost_pimunu(b, tau2, pitt, pitx, pity, pitn, pixx, pixy, pixn, piyy, piyn, pinn);
      double shear_mod = 0.5 / df.betapi, bulk_mod = df.lambda;
      double Axx = 1.0 + pl_.xx * shear_mod + bulk_mod, Axy = pl_.xy * shear_mod, Axz = pl_.xz * shear_mod;
      double Ayy = 1.0 + pl_.yy * shear_mod + bulk_mod, Ayz = pl_.yz * shear_mod, Azz = 1.0 + pl_.zz * shear_mod + bulk_mod;
      double detA = Axx * (Ayy * Azz - Ayz * Ayz) - Axy * (Axy * Azz - Ayz * Axz) + Axz * (Axy * Ayz - Ayy * Axz);
      breaks = feqmod_breaks_down(p->mass_pion0, T, df.F, bulkPi, df.betabulk, detA, p->deta_min, df.z, s, 4);
    }
    for (int ipart = 0; ipart < npart; ipart++) {
      if (DF_MODE == 4) Ntot += breaks ? ds_time * (1.0 + df.delta_z) * neq[ipart] : ds_time * df.z * neq[ipart];
      else Ntot += ds_time * (neq[ipart] + bulkPi * bulk[ipart]) - ds_space * Vdsigma * diff[ipart];
    }
  }
  if (!rc && p->dimension == 2) Ntot *= (2.0 * y_cut);
  if (rc) seterr(err, errlen, df_errmsg(rc));
  *n_total = Ntot;
  free(neq); df_free(&d);
  return rc ? 1 : 0;
}
