/*
 * is3d_amd.h -- C ABI of the MI355X Cooper-Frye continuous-spectra engine
 * (libis3d_amd.so).  Plain pointers and sizes only; no torch / HIP types.
 *
 * This is the drop-in boundary for iS3D2's operation = 1 hot path.  Each entry
 * point replaces one piece of the reference's EmissionFunctionArray /
 * Deltaf_Data / IS3D plug-in surface (reference = xyw2016/iS3D2 @ 2025-01-17):
 *
 *   is3d_create / is3d_destroy        EmissionFunctionArray ctor / dtor        (EmissionFunction.cpp:114-399)
 *   is3d_set_params                   ParameterReader flags read by the ctor   (EmissionFunction.cpp:140-205)
 *   is3d_set_species                  chosen particle arrays                    (EmissionFunction.cpp:997-1021, 339-390)
 *   is3d_set_pdg                      full PDG arrays (PTMA, PTB Jonah table)   (EmissionFunction.cpp:1025-1036)
 *   is3d_set_momentum_grid            pT/phi/y/eta Tables                      (iS3D.cpp:254-257, MomentumSpectra.cpp:49-91)
 *   is3d_set_gauss_laguerre           Gauss_Laguerre::load_roots_and_weights   (readindata.cpp:26-61)
 *   is3d_set_df_tables                Deltaf_Data::load_df_coefficient_data +  (DeltafData.cpp:65-321)
 *                                     construct_cubic_splines + compute_jonah_coefficients
 *   is3d_set_surface                  FO_surf[] -> SoA unpack                  (EmissionFunction.cpp:1049-1161)
 *   is3d_calculate_spectra            calculate_spectra, operation = 1         (EmissionFunction.cpp:1198-1226)
 *   is3d_set_momentum_weights         pT/phi Table weight columns              (SpacetimeDistribution.cpp:57-79)
 *   is3d_set_spacetime_bins           tau/r/phip bin parameters                (EmissionFunction.cpp:232-247)
 *   is3d_calculate_dN_dX              calculate_spectra, operation = 0         (EmissionFunction.cpp:1165-1196)
 *   is3d_get_cell_yields              dN_dy_cell of each freeze-out cell       (SpacetimeDistribution.cpp:374)
 *   is3d_evaluate_df_coefficients     Deltaf_Data::evaluate_df_coefficients    (DeltafData.cpp:501-519)
 *   is3d_surface_averages             ds_max-weighted averages (Plasma)        (readindata.cpp:316-366, iS3D.cpp:184-219)
 *   is3d_total_yield                  calculate_total_yield (operation 2       (ParticleSampler.cpp:447-636,
 *                                     oversampling) + particle densities        DeltafData.cpp:555-690)
 *
 * Conventions: caller-owned host buffers in and out; the engine owns its HBM
 * buffers.  Errors are return codes (never exit()); is3d_last_error() gives the
 * message the reference would have printed before aborting.  One engine per
 * host thread per GPU; an engine is not re-entrant.  Output layout is the
 * reference's dN_pTdpTdphidy[ipart][ipT][iphi][iy] (MomentumSpectra.cpp:252-295).
 */
#ifndef IS3D_AMD_H
#define IS3D_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define IS3D_ABI_VERSION 5

enum {
  IS3D_OK = 0,
  IS3D_ERR_ARG = 1,          /* bad argument / inconsistent setup */
  IS3D_ERR_STATE = 2,        /* missing setup step */
  IS3D_ERR_DEVICE = 3,       /* HIP runtime error */
  IS3D_ERR_DF_RANGE = 4,     /* df coefficient spline/table evaluated out of range (reference: GSL abort / exit) */
  IS3D_ERR_UNSUPPORTED = 5   /* combination the reference rejects (e.g. PTB + baryon) */
};

typedef struct is3d_engine is3d_engine;

typedef struct {
  int operation;                  /* 1 continuous spectra, 0 spacetime distributions, 2 the sampler's yield estimate;
                                     informs the host facade -- each compute entry point fixes its own semantics */
  int dimension;                  /* 2 = boost-invariant (eta quadrature), 3 = 3+1d (y grid) */
  int df_mode;                    /* 1 Grad, 2 RTA-CE, 3 PTM, 4 PTB, 5 PTMA */
  int include_baryon;
  int include_bulk_deltaf;
  int include_shear_deltaf;
  int include_baryondiff_deltaf;
  int regulate_deltaf;
  int outflow;
  int famod_chains;               /* PTMA warm-start chains (= reference OpenMP thread count);
                                     0 = every cell solved independently (= threads >= cells) */
  double deta_min;
  double mass_pion0;
} is3d_params;

/* Freeze-out surface as structure-of-arrays, reference units after the reader's
 * conversion (GeV, fm): tau x y eta | dsigma_mu (covariant) | u^x u^y u^eta |
 * E T P | pi^xx pi^xy pi^xeta pi^yy pi^yeta | Pi | muB nB V^x V^y V^eta.
 * The baryon arrays may be NULL when include_baryon = 0.  (readindata.h:79-91) */
typedef struct {
  const double *tau, *x, *y, *eta;
  const double *dat, *dax, *day, *dan;
  const double *ux, *uy, *un;
  const double *E, *T, *P;
  const double *pixx, *pixy, *pixn, *piyy, *piyn;
  const double *bulkPi;
  const double *muB, *nB, *Vx, *Vy, *Vn;
} is3d_surface;

/* operation = 0 binning (iS3D_parameters.dat tau_min/tau_max/tau_bins, r_min/r_max/r_bins, phip_bins;
 * EmissionFunction.cpp:232-247).  threads = the reference's OpenMP thread count CORES:
 *   0      every species is binned from zero (the evident intent of the reference);
 *   C >= 1 reproduce a reference run with OMP_NUM_THREADS = C, whose per-species reset
 *          memset(all, 0, CORES * bins) clears BYTES, so thread-slice entries past the first
 *          CORES*bins/8 doubles carry the previous species' sums (SpacetimeDistribution.cpp:165-167). */
typedef struct {
  double tau_min, tau_max;
  int tau_bins;
  double r_min, r_max;
  int r_bins;
  int phip_bins;
  int threads;
} is3d_spacetime_bins;

typedef struct {
  long cells;                     /* cells processed in the last call */
  long breakdown;                 /* feqmod / famod breakdown cells */
  long pl_negative;               /* cells with p_L < 0 (p_L or p_T < 0 for PTMA) */
  long recon_fail;                /* PTMA reconstruction failures */
  long iterations;                /* PTMA total Newton iterations */
  double ms_prepass, ms_spectra, ms_total;   /* device time of the last call (HIP events) */
} is3d_stats;

int is3d_abi_version(void);
/* Build identity: a hash of the sources and compiler flags this library was built from (Makefile SRC_ID).
 * The committed rocprofv3 counter summaries (profiles/pmc_*.json) record it; bench.py reports their
 * roofline figures only for the identical build. */
const char *is3d_build_id(void);
is3d_engine *is3d_create(int device);
/* One engine over several GPUs of this process (the multi-GPU fan-out inside the compute
 * call).  Every setter goes to one engine per listed device; is3d_set_surface splits the cells into
 * contiguous windows of ~equal estimated cost (cells with u.dsigma <= 0 are nearly free); one
 * is3d_calculate_spectra / is3d_launch runs all devices concurrently and sums their spectra with one
 * RCCL ncclAllReduce (float64, sum) of the device-resident outputs -- or, when the list repeats a device,
 * with peer copies and a fixed-order add on devices[0].  is3d_launch's dev_out and stream belong to
 * devices[0].  PTMA with warm-start chains (famod_chains > 0): every device holds the whole surface and
 * walks the chains (set the params before the surface).  Replaces the reference's OpenMP fan-out
 * (MomentumSpectra.cpp:98-107) and its thread reduction (:383-411). */
is3d_engine *is3d_create_devices(int n_devices, const int *devices);
void is3d_destroy(is3d_engine *e);
const char *is3d_last_error(const is3d_engine *e);

int is3d_set_params(is3d_engine *e, const is3d_params *p);
/* Engine tuning knobs (no reference counterpart; a device-list engine forwards them to every shard).
 *   "phitab_one_bytes"    F_TS scalar tables (Grad / RTA-CE, one phi block) of the whole window up to this size are
 *                         written and integrated in one chunk (default 8 GiB)
 *   "phitab_chunk_bytes"  larger ones in chunks of whole cell splits of about this size, alternating over two streams
 *                         (default 2 GiB; BASELINE config 4 runs 29 chunks)
 *   "max_splits"          cap on k_spectra's cell splits, one output-sized partial slab each (default 1024)
 *   "slab_bytes"          cap on those slabs' memory (default 48 GiB; also at most half the device's free memory)
 *   "split_bytes"         record bytes per cell split the plan aims for (default 512 KiB: a split stays in an XCD's L2)
 * A negative value restores the default.  is3d_get_tuning also reads "phitab_chunks": the F_TS chunks of the last
 * launch (0: not an F_TS launch), "splits": the cell splits of the last launch, and "slabs": the output-sized partial
 * slabs it held (several 3+1D F_TS chunks fold theirs into one accumulator as they finish: 1 + 2 x splits per chunk);
 * -1 = unknown key. */
int is3d_set_tuning(is3d_engine *e, const char *key, long value);
long is3d_get_tuning(const is3d_engine *e, const char *key);
int is3d_set_species(is3d_engine *e, int n, const double *mass, const double *sign,
                     const double *degeneracy, const double *baryon);
/* Integrand classes (no reference counterpart: an engine option, default on).  The momentum integrals see a
 * species only through its (mass, sign, baryon) -- and, for PTM, its degeneracy, which enters the
 * renormalisation (MomentumSpectra.cpp:800-808) -- while the degeneracy multiplies the result
 * (MomentumSpectra.cpp:365).  With classes on, chosen species with identical keys are integrated once and the
 * reduction writes every member (prefactor x its degeneracy x the shared cell sum): the spectra are
 * bit-identical to integrating each species separately (on = 0) when both take the same launch plan (at the
 * BASELINE sizes), otherwise equal to rounding (the class count can change the cell-split grouping).
 * is3d_species_integrated returns the number of species the kernels integrate (SMASH 444 -> 193), or minus an
 * IS3D_ERR_* code when the tables cannot be finalised (is3d_last_error says why). */
int is3d_set_species_classes(is3d_engine *e, int on);
int is3d_species_integrated(is3d_engine *e);
int is3d_set_pdg(is3d_engine *e, int n, const double *mass, const double *sign,
                 const double *degeneracy, const double *baryon);
int is3d_set_momentum_grid(is3d_engine *e, int npT, const double *pT, int nphi, const double *phi,
                           int ny, const double *y, int neta, const double *eta, const double *eta_weight);
/* roots/weights[alpha][points], as in tables/gauss/gla_roots_weights.txt */
int is3d_set_gauss_laguerre(is3d_engine *e, int alpha, int points, const double *roots, const double *weights);
/* tables[10][nmuB][nT] in file order c0 c1 c2 c3 c4 F G betabulk betaV betapi;
 * T_avg = Plasma::temperature (surface average after the 15-digit file round trip),
 * used only for the PTB (Jonah) table. */
int is3d_set_df_tables(is3d_engine *e, int nT, int nmuB, const double *T, const double *muB,
                       const double *tables, double T_avg);

/* Copies n_cells cells (host pointers) into engine-owned HBM. */
int is3d_set_surface(is3d_engine *e, long n_cells, const is3d_surface *s);
/* Same, but the 25 field arrays are already in device memory on the engine's GPU
 * (field-major: dev[f * n_cells + c], f in is3d_surface order).  Not copied. */
int is3d_set_surface_device(is3d_engine *e, long n_cells, const double *dev_fields);

/* Integrate only cells [lo, hi) of the surface set last (lo = hi = -1: every cell; setting a surface clears
 * it).  For one process per GPU: every rank holds the whole surface and integrates its window; the PTMA
 * warm-start chains (famod_chains > 0) still walk every cell, so each window sees the serial chain's
 * solutions (MomentumSpectra.cpp:1308-1364), which cell shards could not. */
int is3d_set_cell_window(is3d_engine *e, long lo, long hi);

/* Estimated k_spectra cost of every cell of the surface set last, relative to a live cell of the mode's main
 * launch (no reference counterpart: the shard cost model of SURVEY.md 8(e), used by is3d_create_devices' windows
 * and by one-process-per-GPU callers): 0.02 for u.dsigma <= 0 (skipped by every kernel,
 * MomentumSpectra.cpp:132; its record prep only); PTM / PTB cells that break down or have narrow rapidity
 * windows take the separable fallback launch (MomentumSpectra.cpp:863-929) at 1.4 / 1.8 (measured on MI355X,
 * tools/fb_cost_probe.py); every other cell 1 (PTMA's breakdowns are only known after its Newton solves).
 * Runs the record prepass on the engine's GPU (synchronous); cost holds n_cells doubles. */
int is3d_cell_costs(is3d_engine *e, double *cost);

/* PTMA warm-start chains split over processes (one process per GPU; SURVEY.md 8(e) "partition by chain and keep
 * chain order").  The reference warm-starts each Newton solve from the previous successful cell of its OpenMP thread
 * (MomentumSpectra.cpp:1132-1135, 1308-1364): chain c = cells c, c + C, c + 2C, ... with C = famod_chains.  Every
 * process holds the whole surface; is3d_set_chain_range(e, q0, q1) makes this engine solve chain positions
 * [q0, q1) of every chain and integrate cells [q0 C, min(n, q1 C)) (q0 = q1 = -1: off; setting a surface or a cell
 * window clears it).  The staged launch then lets the caller move the boundary states between processes:
 *   is3d_launch_begin                        prepass of the range (on `stream`)
 *   for pass j < is3d_chain_passes(e):
 *     [q0 > 0, j > 0]  is3d_chain_boundary_put(e, (j - 1) & 1, buf)   the predecessor's pass j - 1 end states
 *     is3d_chain_pass(e, j)
 *     [successor]      is3d_chain_boundary_get(e, j & 1, buf)         this range's pass j end states, to send
 *   [q0 > 0]  is3d_chain_boundary_put(e, 2, buf)   the predecessor's final states (after its is3d_chain_end)
 *   is3d_chain_end(e)
 *   [successor]  is3d_chain_boundary_get(e, 2, buf)
 *   is3d_launch_end(e)   ...   is3d_finish(e)
 * Buffers hold is3d_chain_boundary_size(e) doubles, in device memory (or host memory: the copies are asynchronous
 * on the launch stream, so the caller synchronises it before reading a host buffer it got).
 * At the fixed point each range's solutions are the one-chain solutions bit for bit (engine.hip k_chain_pass), so
 * the per-process Newton iteration counts (is3d_get_stats) add up to the serial chain's.  is3d_launch refuses an
 * engine with a chain range. */
int is3d_set_chain_range(is3d_engine *e, long q0, long q1);
int is3d_launch_begin(is3d_engine *e, double *dev_out, void *stream);
int is3d_chain_passes(const is3d_engine *e);
int is3d_chain_pass(is3d_engine *e, int pass);
int is3d_chain_end(is3d_engine *e);
int is3d_launch_end(is3d_engine *e);
long is3d_chain_boundary_size(const is3d_engine *e);
int is3d_chain_boundary_get(is3d_engine *e, int slot, double *dev_buf);
int is3d_chain_boundary_put(is3d_engine *e, int slot, const double *dev_buf);

/* Full call: kernels + device->host copy of dN/(pT dpT dphi dy) into dN_out. */
int is3d_calculate_spectra(is3d_engine *e, double *dN_out);

/* Split call for resident benchmarking / multi-GPU reduction: launch the whole
 * hot path on `stream` (a hipStream_t, NULL = default) writing the spectra into
 * the device buffer dev_out (npart*npT*nphi*ny doubles on the engine's GPU);
 * is3d_finish() synchronises and reports device-side errors. */
int is3d_launch(is3d_engine *e, double *dev_out, void *stream);
int is3d_finish(is3d_engine *e);
int is3d_get_stats(const is3d_engine *e, is3d_stats *out);
long is3d_output_size(const is3d_engine *e);

/* operation = 0, spacetime distributions dN/dX (EmissionFunction.cpp:1165-1196 ->
 * calculate_dN_dX / calculate_dN_dX_feqmod, SpacetimeDistribution.cpp:31-1250; df_mode 1-4, PTMA is
 * rejected as in the reference).  Needs the pT / phi quadrature weights (Table column 2) and the bins.
 * Outputs [species][bins] are the values the reference writes to results/continuous/dN_taudtaudy_<MCID>.dat,
 * dN_2pirdrdy_<MCID>.dat and dN_dphidy_<MCID>.dat (already divided by tau dtau, 2 pi r dr, dphi). */
int is3d_set_momentum_weights(is3d_engine *e, const double *pT_weight, const double *phi_weight);
int is3d_set_spacetime_bins(is3d_engine *e, const is3d_spacetime_bins *bins);
int is3d_calculate_dN_dX(is3d_engine *e, double *dN_taudtaudy, double *dN_2pirdrdy, double *dN_dphidy);
/* dN_dy_cell[species][cell] of the last is3d_calculate_dN_dX call (SpacetimeDistribution.cpp:374). */
int is3d_get_cell_yields(const is3d_engine *e, double *dN_dy_cell);

/* Test hooks mirroring reference services. out[15] = c0 c1 c2 c3 c4 shear14 F G
 * betabulk betaV betapi lambda z delta_lambda delta_z (evaluated on the GPU). */
int is3d_evaluate_df_coefficients(is3d_engine *e, double T, double muB, double E, double P,
                                  double bulkPi, double *out15);
/* out[5] = T, E, P, muB, nB averages (after the setprecision(15) round trip). */
int is3d_surface_averages(long n_cells, const is3d_surface *s, int include_baryon, double *out5);
/* Jonah table the engine built: lambda^2, z, bulkPi/P (301 each) and the max. */
/* operation = 2 oversampling estimate: the reference's Ntotal (ParticleSampler.cpp:447-636
 * calculate_total_yield, EmissionFunction.cpp:1237-1242), with the per-species densities of
 * Deltaf_Data::compute_particle_densities (DeltafData.cpp:555-690) evaluated on the device at the
 * Plasma averages plasma = (T, E, P, muB, nB) (is3d_surface_averages).  Like the reference, the
 * densities use the alpha = 1, 2, 3 rows of tables/gauss/gla_roots_weights.txt: set that 32-point
 * table with is3d_set_gauss_laguerre.  2+1D: multiplied by 2 y_cut.  densities (optional, [3][npart]):
 * equilibrium, bulk and diffusion densities of the chosen species.  Nevents =
 * min(ceil(min_num_hadrons / Ntotal), max_num_samples) is the caller's (EmissionFunction.cpp:1242). */
int is3d_total_yield(is3d_engine *e, const double *plasma, double y_cut, double *n_total, double *densities);

int is3d_get_jonah_table(const is3d_engine *e, double *lambda2, double *z, double *bulk_over_P,
                         double *bulk_over_P_max);

#ifdef __cplusplus
}
#endif
#endif
