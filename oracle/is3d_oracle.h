/*
 * is3d_oracle.h -- CPU restatement of iS3D2's continuous-spectra path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X engine
 * (libis3d_amd.so) and the "port" CPU baseline timed by bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * path never links or calls it.
 *
 * What it restates (reference = xyw2016/iS3D2 @ 2025-01-17, src/cpp/):
 *   SpacetimeDistribution.cpp:31-1250 calculate_dN_dX(_feqmod)   (operation 0, df_mode 1-4)
 *   MomentumSpectra.cpp:32-415    calculate_dN_pTdpTdphidy        (df_mode 1 Grad, 2 RTA-CE)
 *   MomentumSpectra.cpp:419-1044  calculate_dN_pTdpTdphidy_feqmod (df_mode 3 PTM, 4 PTB)
 *   MomentumSpectra.cpp:1049-1682 calculate_dN_pTdpTdphidy_famod  (df_mode 5 PTMA)
 *   DeltafData.cpp:220-519        Jonah table, natural cubic splines, bilinear tables
 *   GaussThermal.cpp:7-130        Gauss-Laguerre thermal integrals
 *   LocalRestFrame.cpp:12-185     Milne basis, pi^{mu nu} / V^mu LRF boosts
 *   AnisoVariables.cpp:15-643     (lambda, aT, aL) Newton solve + famod coefficients
 *   EmissionFunction.cpp:33-109   feqmod breakdown tests
 *   ParticleSampler.cpp:75-119, 447-636 + DeltafData.cpp:555-690   operation 2 yield estimate
 * The OpenMP cell striding of the reference (thread n takes cells n, n+C, ...,
 * MomentumSpectra.cpp:98-107) is emulated with `threads` = C virtual threads, so
 * the summation order and the PTMA warm-start chains follow the reference run
 * with OMP_NUM_THREADS=C.  Race fix: the 3+1D eta value is per-cell local
 * (the reference writes a shared stack array, MomentumSpectra.cpp:111-114).
 *
 * GSL (unpinned version; absent from this image, so the reference cannot be
 * built here -- see DESIGN.md) is restated: natural cubic spline = GSL cspline
 * (tridiagonal Cholesky solve, coefficient formulas of cspline.c), LU with
 * partial pivoting (gsl_linalg_LU_decomp/solve/invert).
 *
 * Parity pinning: the GSL-free reference sources (readers, GaussThermal,
 * LocalRestFrame) are compiled from /root/reference into oracle/_ref by
 * oracle/ref/build_ref.sh and pin the pieces they cover; the spectra loops
 * themselves depend on GSL and are "parity partially pinned" (DESIGN.md §3).
 */
#ifndef IS3D_ORACLE_H
#define IS3D_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int dimension;                 /* 2 or 3 */
  int df_mode;                   /* 1..5 */
  int include_baryon;
  int include_bulk_deltaf;
  int include_shear_deltaf;
  int include_baryondiff_deltaf;
  int regulate_deltaf;
  int outflow;
  int threads;                   /* emulated OpenMP thread count C (>=1) */
  int omp_threads;               /* real OpenMP threads (0 = runtime default) */
  double deta_min;
  double mass_pion0;
} orc_params;

typedef struct {
  int npart;                     /* chosen species */
  const double *mass, *sign, *degen, *baryon;
  int npdg;                      /* full PDG list (Jonah table, PTMA Newton) */
  const double *pdg_mass, *pdg_sign, *pdg_degen, *pdg_baryon;
  int npT, nphi, ny, neta;
  const double *pT, *phi, *y, *eta, *eta_w;
  int gla_alpha, gla_points;     /* tables/gauss/gla_roots_weights.txt: [alpha][points] */
  const double *gla_root, *gla_weight;
  int nT, nmuB;                  /* df coefficient grid */
  const double *Tarr, *muBarr;
  const double *dftab;           /* [10][nmuB][nT]: c0 c1 c2 c3 c4 F G betabulk betaV betapi */
  double T_avg;                  /* Plasma::temperature (15-digit file round trip) */
  const double *pT_w, *phi_w;    /* pT / phi quadrature weights (operation 0 only; may be NULL otherwise) */
} orc_setup;

/* operation = 0 spacetime bins (EmissionFunction.cpp:232-247, iS3D_parameters.dat tau_* r_* phip_bins) */
typedef struct {
  double tau_min, tau_max;
  int tau_bins;
  double r_min, r_max;
  int r_bins;
  int phip_bins;
  int carry;                     /* 1 = the reference's byte-count memset (values carry over between
                                    species in all but the first C*bins/8 thread-slice entries);
                                    0 = every species binned from zero */
} orc_bins;

/* canonical surface field order (shared with include/is3d_amd.h) */
typedef struct {
  long n;
  const double *tau, *x, *y, *eta;
  const double *dat, *dax, *day, *dan;
  const double *ux, *uy, *un;
  const double *E, *T, *P;
  const double *pixx, *pixy, *pixn, *piyy, *piyn;
  const double *bulkPi;
  const double *muB, *nB, *Vx, *Vy, *Vn;
} orc_surface;

/* stats[0] breakdown cells, [1] pl<0 cells, [2] PTMA reconstruction failures,
 * [3] PTMA total Newton iterations, [4] skipped species (NaN/Inf renorm) */
#define ORC_NSTATS 8

/* dN/(pT dpT dphi dy) in the reference layout [species][pT][phi][y].
 * Returns 0 on success, nonzero (and a message in err) where the reference
 * would abort (GSL range error, bad df_mode, table out of range). */
int orc_spectra(const orc_params *p, const orc_setup *s, const orc_surface *surf,
                double *out, long *stats, char *err, int errlen);

/* operation = 0: dN/dX (SpacetimeDistribution.cpp:31-1250).  Outputs are the values the
 * reference writes to results/continuous/dN_taudtaudy_<MCID>.dat, dN_2pirdrdy_, dN_dphidy_
 * ([species][bins], already divided by the bin measure); cell_yield (optional, [species][cell])
 * is dN_dy_cell, 0 for skipped cells.  p->threads = the reference's CORES (cell striding and
 * thread slices of the binning). */
int orc_dndx(const orc_params *p, const orc_setup *s, const orc_surface *surf, const orc_bins *bins,
             double *cell_yield, double *tau_out, double *r_out, double *phi_out, long *stats,
             char *err, int errlen);

/* operation = 2 oversampling estimate (ParticleSampler.cpp:447-636 calculate_total_yield with the
 * DeltafData.cpp:555-690 densities).  plasma = (T, E, P, muB, nB) Plasma averages; the Gauss-Laguerre
 * table must be tables/gauss/gla_roots_weights.txt (32 points), as compute_particle_densities loads it.
 * n_total = the reference's Ntotal (x 2 y_cut in 2+1D); densities (optional) = [3][npart] equilibrium,
 * bulk and diffusion densities of the chosen species. */
int orc_total_yield(const orc_params *p, const orc_setup *s, const orc_surface *surf, const double *plasma,
                    double y_cut, double *n_total, double *densities, char *err, int errlen);

/* --- pieces exposed for pinning tests --- */
double orc_gauss_thermal(int kind, const double *root, const double *weight, int pts,
                         double mbar, double alphaB, double baryon, double sign);
double orc_gauss1d_mod(int kind, const double *root, const double *weight, int pts,
                       double mbar, double lambda, double sign);
void orc_milne_lrf(const double *in15, double *out14);
void orc_dsigma_lrf(const double *in9, double *out5);
void orc_lu3_solve(const double *A9, const double *b3, double *x3, int *perm3);
int orc_df_coefficients(const orc_params *p, const orc_setup *s, double T, double muB,
                        double E, double P, double bulkPi, double *out15, char *err, int errlen);
int orc_jonah_table(const orc_setup *s, double *lambda2, double *z, double *bulk_over_P,
                    double *bulk_over_P_max);
void orc_surface_averages(const orc_surface *surf, double *out5);
int orc_aniso_solve(const orc_setup *s, double E, double pl, double pt, double l0,
                    double aT0, double aL0, double *out6);
/* PTMA warm-start chain over an explicit cell list from state[4] = (prev_ok, lambda, aT, aL) (MomentumSpectra.cpp:
 * 1288-1368): states[4 i ..] = chain state after cell i, iters[i] = Newton iterations (-1: u.dsigma <= 0, not in the
 * chain); state is updated to the last cell's; returns the total iterations. */
long orc_famod_chain(const orc_params *p, const orc_setup *s, const orc_surface *surf, const long *cells,
                     long ncells, double *state, double *states, int *iters);

#ifdef __cplusplus
}
#endif
#endif
