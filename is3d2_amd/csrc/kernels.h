// kernels.h -- the momentum-integral kernels (k_spectra: operation 1, k_dndx: operation 0), their
// argument blocks and launchers.  The kernels and launchers are compiled one delta-f mode per
// translation unit (spectra_tu.hip, built five times in parallel: 5 modes x 4 flag sets x 4 phi-block
// sizes of each kernel no longer serialise the build); engine.hip (host side) sees declarations.
#pragma once
#include <hip/hip_runtime.h>

#include "cf_math.h"

namespace is3d {
namespace kern {

constexpr int kBlock = 256;
#ifndef IS3D_KTILE
#define IS3D_KTILE 8
#endif
constexpr int kTile = IS3D_KTILE;   // cells per LDS tile
#ifndef IS3D_KTILE_MOD
#define IS3D_KTILE_MOD 8    // modified path: 8 cells per tile since it runs 3 waves/SIMD (3 workgroups' LDS per CU;
                            // 16 paid at 2 waves: 1279 -> 1245 ms, r2t A/B)
#endif
// cells per k_spectra tile of one delta-f mode and launch (8 for Grad / RTA-CE: 16 costs them 18% / 11%,
// r2t; the modified path's F_T8 and F_LY launches keep 8 where 16 cells' q-row tables would not fit:
// config 1's shape in F_LY ran 11.2 ms with 8-cell tiles, 13.6 ms with 16)
#ifndef IS3D_KTILE_TS
#define IS3D_KTILE_TS 12      // F_TS launches (LDS: records, y-terms and T1 rows only). Each k_phitab row a
                              // wave reads through the scalar cache serves the tile's cells: config 2 Grad
                              // 155.5 ms at 8 cells, 154.2 at 10, 151.5 at 12 and 14, 188.5 at 16 (LDS
                              // occupancy); RTA-CE 241.6 / 239.0 / 237.8 / 240.3; config 4 flat at 8-14
                              // (profiles/round5_r5h_ab_ts_tile.log)
#endif
template <int MODE, int FLAGS>
constexpr int spectra_tile() {
  return (MODE >= PTM && !(FLAGS & (32 | 16 | 8))) ? IS3D_KTILE_MOD : ((FLAGS & 128) && (FLAGS & 4)) ? IS3D_KTILE_TS : kTile;
}
// waves per SIMD the spectra kernel is register-allocated for (measured on MI355X, config2):
// Grad and RTA-CE run best at 3 (168 VGPRs), the modified-momentum modes at 2
#ifndef IS3D_SPECTRA_WAVES_SEP
#define IS3D_SPECTRA_WAVES_SEP 3
#endif
#ifndef IS3D_SPECTRA_WAVES_MOD
#define IS3D_SPECTRA_WAVES_MOD 3   // without the separable code (F_FB launch): 164 VGPRs; config2 PTM 1242 -> 1044 ms (r3 A/B)
#endif
#ifndef IS3D_SPECTRA_WAVES_CE
#define IS3D_SPECTRA_WAVES_CE 3      // RTA-CE: 3 (16 spilled VGPRs, 3 scratch accesses per 32 points) beat 2 by 4.3% once
                                     // the lane setup shrank (profiles/round1_r1z_ab_ce3.log; 2 won before, r1n)
#endif
// waves per SIMD of one spectra / dN/dX instantiation
template <int MODE>
constexpr int spectra_waves() {
  return MODE >= PTM ? IS3D_SPECTRA_WAVES_MOD : MODE == CE ? IS3D_SPECTRA_WAVES_CE : IS3D_SPECTRA_WAVES_SEP;
}
#ifndef IS3D_SPECTRA_WAVES_KJ16
#define IS3D_SPECTRA_WAVES_KJ16 4     // Grad with 16-point phi blocks (acc in 32 VGPRs)
#endif
template <int MODE, int KJ>
constexpr int spectra_waves_kj() { return (KJ == 16 && MODE == GRAD) ? IS3D_SPECTRA_WAVES_KJ16 : spectra_waves<MODE>(); }
#ifndef IS3D_WAVES_TS
#define IS3D_WAVES_TS 0       // F_TS launches: waves per SIMD (0: as the mode's other launches)
#endif
// the F_FB launch (separable lanes of a modified mode: per-point exp, RTA-CE-like lane setup) stays at 2
template <int MODE, int FLAGS, int KJ>
constexpr int spectra_waves_f() {
  return (MODE >= PTM && (FLAGS & 32)) ? 2 : (IS3D_WAVES_TS && (FLAGS & 128)) ? IS3D_WAVES_TS : spectra_waves_kj<MODE, KJ>();
}
// k_dndx keeps RTA-CE and the modified modes at 2 (its pT loop holds more live state: 215 VGPRs; it keeps
// the separable fallback inline)
template <int MODE>
constexpr int dndx_waves() { return (MODE == CE || MODE >= PTM) ? 2 : spectra_waves<MODE>(); }
#ifndef IS3D_DNDX_WAVES_MOD
#define IS3D_DNDX_WAVES_MOD 2      // k_dndx's modified-lane launch (the separable fallback in its own F_FB launch)
#endif
#ifndef IS3D_DNDX_MOD_UNROLL
#define IS3D_DNDX_MOD_UNROLL 2     // k_dndx modified lanes: phi pairs per loop trip (fully unrolled, 16 at 32 points, the
                                   // PTM / PTB launch held 256 VGPRs + 95 spilled; two: 129 VGPRs, 3 waves per SIMD)
#endif
#ifndef IS3D_DNDX_QUAD
#define IS3D_DNDX_QUAD 1           // k_dndx lanes in fours (one reciprocal per four points; modified lanes: staged exp).
                                   // Config 2 operation 0 against pairs: Grad 345 -> 322 ms (168 VGPRs with 15-37
                                   // spilled -> 124), RTA-CE 506 -> 480, PTM 834 -> 741, PTB 732 -> 660 ms
                                   // (profiles/round5_r5m_ab_dndx_quad.log)
#endif
template <int MODE, int FLAGS>
constexpr int dndx_waves_f() { return (MODE >= PTM && !(FLAGS & 32)) ? IS3D_DNDX_WAVES_MOD : dndx_waves<MODE>(); }
#ifndef IS3D_DNDX_TILE_MOD
#define IS3D_DNDX_TILE_MOD 4       // k_dndx's modified launch: cells per record tile (engine.hip sizes its LDS the same way).
                                   // 4: ~28 KB of LDS and 126-128 VGPRs, 4 workgroups per CU; config 2 operation 0 against
                                   // 8-cell tiles (53 KB, 3 per CU): PTM 661 -> 645 ms, PTB 661 -> 640 ms
                                   // (profiles/round6_r6q_ab_dndx_tile.log)
#endif
#ifndef IS3D_DNDX_TILE
#define IS3D_DNDX_TILE 8           // k_dndx's Grad / RTA-CE launches: cells per record tile
#endif
#ifndef IS3D_DNDX_PD
#define IS3D_DNDX_PD 2             // k_dndx's separable launches with per-(cell, phi) PD = p.dsigma_perp b' rows (k_spectra's
                                   // PD-table fours: w p.dsigma f_eq = fma(D0, b', escw PD), one op fewer per point); bit 1
                                   // Grad, bit 2 RTA-CE.  Config 2 operation 0 (profiles/round6_r6v_ab_dndx_pd.log): RTA-CE
                                   // 485.2 -> 474.7 ms; Grad 317.6 -> 330.3 ms (its Boltzmann-tail pairs become fours): off
#endif
template <int MODE>
constexpr bool dndx_pd() { return (MODE == GRAD && (IS3D_DNDX_PD & 1)) || (MODE == CE && (IS3D_DNDX_PD & 2)); }
#ifndef IS3D_DNDX_PDM
#define IS3D_DNDX_PDM 1            // k_dndx's modified launch: per-(cell, phi) {PDm, Qv} rows, p.dsigma = fma(Dw, PDm, D0)
#endif
// cells per record tile of a k_dndx launch (the F_FB launch keeps kTile)
template <int MODE, int FLAGS>
constexpr int dndx_tile() { return (FLAGS & 32) ? kTile : (MODE >= PTM ? IS3D_DNDX_TILE_MOD : IS3D_DNDX_TILE); }

// LDS row stride of the y-terms (doubles): NYT | 1 is odd, so the 8-byte stores of one y-term field
// by consecutive lanes (rows 152 B apart) spread over the 64 banks instead of hitting two of them
// (a 128-B stride put every lane of a wave on the same bank pair: a 32-way conflict)
constexpr int kYRow = NYT | 1;
// per-lane y-term rows of the F_LY / F_FB launches: without the Y_MU2 / Y_MU slots (17 doubles, odd): the
// 256 rows are LDS the launch's occupancy depends on, and each lane's row serves one lane only
constexpr int kYRowLY = Y_MU2 | 1;

// ------------------------------------------------------------------------------------------
// spectra kernel
// ------------------------------------------------------------------------------------------
struct SpecArgs {
  const double* rec; long n;
  int* err;                   // DF_TS_SLOW: a F_TS lane off the fast path (engine.hip routes such surfaces to F_TB)
  const double* renorm;       // PTM: [c][renorm class]
  const int* rcls; int nrcls; // renorm class of each sorted species (engine.hip), number of classes
  double* slab; long outsize;
  const double *smass, *ssign, *sbaryon; const int* sorig;
  const double *pT, *cphi, *sphi, *yv, *etav, *etaw;
  const double* csg;          // [npT][nphp] {pT cos, pT sin} (read by scalar loads when njb == 1)
  int npart, npT, nphi, ny_out, nk, nl, nq, njb;
  int nqmax;                  // q rows a workgroup's lanes can span (LDS rows of the y-term / q tables)
  long ntask;                 // npart * nq * njb lanes per pT: (species, q = y x eta node, phi block)
  long cells_per_split;
  int nbx, nsplit;            // lane groups per pT, cell splits (1-D grid of nbx * npT * nsplit)
  int npw;                    // F_MP: pT values per workgroup (1-D grid of ceil(npT / npw) * nsplit)
  long sstride;               // doubles per slab: npT * nbx * KJ * kBlock
  int regulate, outflow, dim;
  int op;                     // 1 spectra / 0 spacetime (yterms variants)
  const int* fbcells;         // F_FB launch: ascending indices of the cells with separable-fallback lanes
  const int* fbcount;         //   (k_fbcount / k_fbwrite, device-side) and their number
  int split0;                 // first cell split of this launch (F_TS launches cover the splits chunk by chunk)
  int slab0;                  // split whose slab `slab` points at (folded F_TS chunks: a chunk's own slab buffer)
  // F_TS: the per-(cell, pT, phi) tables k_phitab wrote for this chunk of cells, rows [pT][cell - phc0][phrow]
  const double* phtab; long phn, phc0; int phrow;
  // device-side choice between two enqueued plans (engine.hip launch_end): the workgroups return at once unless
  // (*gate != 0) == gate_want; gate = nullptr: always run
  const unsigned long long* gate; int gate_want;
};

__device__ __forceinline__ bool gate_closed(const unsigned long long* gate, int want) {
  return gate && ((*gate != 0ULL) != (want != 0));
}

// flag bits of the spectra kernel instantiation
// F_TB (Grad / RTA-CE, include_baryon = 0, one phi block, KJ % 4 == 0): linear delta-f part from the
// (cell, q, phi) {PD, T1} table (sep_quad_tb_t); a workgroup then uses at most kTbQ q values
// F_LY (grids whose q rows do not fit in LDS: large y / eta tables with few species, KJ = 8 only): every
// lane builds its own y-term row in LDS and the modified lanes use their linear forms, no q-row tables
// F_T8 (modified path): 8-cell tiles instead of IS3D_KTILE_MOD (q-row tables of many rows, config 1's shape)
// F_FB (modified path): the separable-fallback launch -- only the lanes the modified launch leaves out (breakdown
// cells, narrow rapidity windows), over the cells listed by k_fbwrite, per-lane y-term rows as F_LY.  Keeping
// the separable code out of the modified launch takes its k_spectra from 241 to 164 VGPRs (3 waves per SIMD
// instead of 2) and removes the 32-64 v_mov_b64 per lane and cell that merged two register assignments of acc
// F_MP (Grad / RTA-CE with few lane tasks per pT: np x nq <= 128, e.g. pikp 2+1D = 72): a lane owns a whole
// phi row (one block of KJ >= nphi) and a workgroup holds npw = 256 / (np nq) pT values, whose {b', Phi} /
// PD / {pc, ps} tables it builds side by side; the lane setup is amortised over every phi point instead of
// an 8-point block
// F_TS (with F_TB, one phi block): the wave-uniform per-(cell, phi) operands {b', Phi}, PD (and RTA-CE's {TE, T2})
// come by scalar loads from a per-(cell, pT) global table that k_phitab writes before the launch, straight into
// SGPRs, instead of broadcast ds_read_b128s from LDS tables the workgroup builds; LDS keeps only the per-(cell, q
// row, phi) T1 rows (one ds_read_b128 per two points).  The F_TB tail loop read two ds_read_b128 (8 LDS-array
// cycles) per 5 VALU ops, so four SIMDs in it were bound by the CU's LDS array, not by the FP64 pipe
// F_BY (with F_TS, include_baryon = 1): the lanes' baryon part of the linear delta-f coefficients,
// b (SCB pc + SSB ps) per (cell, phi) (R_SCB / R_SSB: c1 / c3 and V^mu terms, prep_grad_ce), comes as one more table
// operand T3: a S = fma(a, fma(b, T3, fma(mT, T1, Phi)), S0') -- the F_TB factorisation needed R_SCB = R_SSB = 0
constexpr int F_REG = 1, F_OUT = 2, F_TB = 4, F_LY = 8, F_T8 = 16, F_FB = 32, F_MP = 64, F_TS = 128, F_BY = 256;
constexpr int kTbQ = 4;
// doubles per F_TS table row of one (cell, pT): {b', Phi}[nphp] | PD[nphp] | RTA-CE {TE, T2}[nphp] | F_BY T3[nphp]
__host__ __device__ constexpr int phitab_row(int mode, int nphp, bool by = false) { return ((mode == CE ? 5 : 3) + (by ? 1 : 0)) * nphp; }
#ifndef IS3D_TS
#define IS3D_TS 1             // F_TB launches with one phi block take the scalar-table form (F_TS)
#endif
#ifndef IS3D_TS_BY
#define IS3D_TS_BY 1          // ... with include_baryon too (F_BY); otherwise the per-lane launch
#endif
#ifndef IS3D_PHITAB_ONE
#define IS3D_PHITAB_ONE (8L << 30)     // F_TS tables up to this size are written and integrated in one chunk
#endif
#ifndef IS3D_PHITAB_BYTES
#define IS3D_PHITAB_BYTES (2L << 30)   // larger ones in chunks of whole cell splits of about this size, alternating
                                       // over two streams (config 4: 2 GB chunks 2738 ms, 6 GB 2770 ms, one 61 GB
                                       // chunk 2734 ms; config 2 RTA-CE in one 6.1 GB chunk 249 ms, 2 GB chunks 254 ms)
#endif

#ifndef IS3D_SPLIT_BYTES
#define IS3D_SPLIT_BYTES (512L << 10) // record bytes per cell split (k_spectra grid sizing): 0.5 MB (2 MB before round 3:
                                      // config2 PTM 467 -> 461 ms, PTB 437 -> 431, config4 3194 -> 3180 ms, Grad unchanged;
                                      // profiles/round3_r3j_ab_split.log; 2 MB for Grad / RTA-CE alone -- a quarter
                                      // of the slabs -- measured again on the round-3 final kernels: Grad 195 -> 196 ms,
                                      // RTA-CE 313 -> 321 ms, config4 3153 -> 3175 ms, round3_r3x_ab_split_dndx_tail.log)
#endif
#ifndef IS3D_NOPF_MODES
#define IS3D_NOPF_MODES 0     // bit m: mode m's fours skip the one-quad-ahead prefetch (register-starved builds)
#endif
#ifndef IS3D_QUAD_RCP
#define IS3D_QUAD_RCP 1       // fast path: four phi points per reciprocal where sep_quads() says so
#endif
#ifndef IS3D_MOD_PF
#define IS3D_MOD_PF 0         // modified table fours: one-quad-ahead prefetch of the {PDm, Qv} / T2 rows (helped at
                              // 2 waves/SIMD; at 3 it does not fit the 168-VGPR budget)
#endif
#ifndef IS3D_MOD_QUAD
#define IS3D_MOD_QUAD 1       // modified path: four phi points per reciprocal when KJ % 4 == 0
#endif
#ifndef IS3D_PD_TABLE
#define IS3D_PD_TABLE 1       // Grad / RTA-CE fast lanes: p.dsigma b' from the per-(cell, phi) PD table (sep_quad_pd_t)
#endif
#ifndef IS3D_PD_PREFETCH
#define IS3D_PD_PREFETCH 0    // PD fours without the one-quad-ahead prefetch (with it Grad spilled 64 VGPRs)
#endif
#ifndef IS3D_CS_SCALAR
#define IS3D_CS_SCALAR 1      // PD fours with one phi block: {pc, ps} by scalar loads (SGPR operands)
#endif
#ifndef IS3D_GRAD_TB
#define IS3D_GRAD_TB 1        // Grad without baryon: the F_TB {PD, T1} table launch (engine.hip)
#endif
#ifndef IS3D_CE_TB
#define IS3D_CE_TB 1          // RTA-CE without baryon also takes the F_TB launch ({PD, T1} + {TE, T2} tables)
#endif
#ifndef IS3D_TAIL
#define IS3D_TAIL 1           // Boltzmann-tail lanes skip the per-point reciprocal (kTailX): Grad F_TB 497 -> 481 ms (r2d)
#endif
#ifndef IS3D_TAIL_WAVE
#define IS3D_TAIL_WAVE 1      // the tail decision per wavefront: a wave mixing tail and other lanes runs one loop
#endif
#ifndef IS3D_TAIL_PDL
#define IS3D_TAIL_PDL 1       // Boltzmann-tail lanes in the per-lane Grad / RTA-CE launches too (sep_quad_pd_tail_t)
#endif
#ifndef IS3D_CE_PE
#define IS3D_CE_PE 1          // RTA-CE per-lane launch: E and the linear delta-f part from a {TE, T2} table (sep_quad_pde_t)
#endif
#ifndef IS3D_TAIL_DNDX
#define IS3D_TAIL_DNDX 1      // operation 0 (k_dndx): Boltzmann-tail Grad lanes in pairs (sep_pair_tail_t)
#endif
#ifndef IS3D_TS_PF
#define IS3D_TS_PF 1          // F_TS: the table rows of tile i + PFD are touched into L2 (LDS-DMA of one dword per 128 B)
#endif
// F_TS prefetch distance in tiles (Grad / RTA-CE): one tile of lane work covers the HBM latency, and the nearer tile
// keeps fewer rows in L2 (12-cell tiles, distance 1 vs 2: config 2 Grad 152.4 / 152.7 ms, RTA-CE 239.4 / 240.6,
// config 3 RTA-CE 258.4 / 261.5, config 4 2399 / 2435; 3 slower still; profiles/round5_r5j_ab_ts_prefetch.log)
#ifndef IS3D_TS_PF_DIST_GRAD
#define IS3D_TS_PF_DIST_GRAD 1
#endif
#ifndef IS3D_TS_PF_DIST_CE
#define IS3D_TS_PF_DIST_CE 1
#endif
// F_TS: the operands of the next four loaded before this four's arithmetic (bit 1 tail lanes, bit 2 other
// lanes), per mode: RTA-CE 260.8 -> 250.8 ms (config 2), 2663 -> 2511 ms (config 4); Grad 167.5 -> 168.9 ms (r4d)
#ifndef IS3D_TS_AHEAD_CE
#define IS3D_TS_AHEAD_CE 1
#endif
// Grad without baryon terms ahead on every four since round 5 (12-cell tiles, prefetch distance 1: config 2 Grad
// 151.9 -> 150.6 ms; the same for RTA-CE and F_BY Grad lost 1-4%: profiles/round5_r5k_ab_tiles_ahead.log)
#ifndef IS3D_TS_AHEAD_GRAD
#define IS3D_TS_AHEAD_GRAD 3
#endif
#ifndef IS3D_TS_AHEAD_GRAD_BY
#define IS3D_TS_AHEAD_GRAD_BY 1
#endif
#ifndef IS3D_TS_SLOW
#define IS3D_TS_SLOW 0        // F_TS kernels with the slow-path loop (0: such surfaces take F_TB, sep_slow_cell)
#endif
#ifndef IS3D_NEAR
#define IS3D_NEAR 1           // F_TS Grad: near-tail lanes (sep_quad_tb_near_t, kNearX), no reciprocal per point
#endif
#ifndef IS3D_TAIL_PD
#define IS3D_TAIL_PD 0        // Grad tail lanes: PD table + scalar {pc, ps} instead of {PD, T1}: 2.2% slower (r2d A/B)
#endif
#ifndef IS3D_TAIL_CE
#define IS3D_TAIL_CE 0        // RTA-CE tail lanes (sep_quad_tb_tail_t): 3% slower on MI355X (r2d A/B: 697 vs 675 ms)
#endif
// (a modified-path tail loop, mod_quad_tail_t, ran 2.5% fewer VALU ops but 11% slower: r2d, 1445 vs 1297 ms)
#ifndef IS3D_PIPE
#define IS3D_PIPE 1           // k_spectra: tables of tile i + 1 built between the lane work of tile i (2 barriers per tile)
#endif
#ifndef IS3D_EARLY_SKIP
// k_spectra tests a lane's overflow skip before its setup, so a wavefront whose lanes all skip a cell branches
// past the setup: bit 1 separable lanes (sep_skips; config 2 Grad 222.0 -> 215.4 ms, RTA-CE 320.4 -> 317.5 ms),
// bit 2 modified lanes (mod_skips; round 3: PTM 465.1 -> 471.8 ms, PTMA unchanged, profiles/round3_r3i_ab_skip.log;
// round 6, on the g-free classes and the table-only modified tiles: PTM 405.9 -> 397.3 ms, PTMA 397.5 -> 391.2 ms,
// profiles/round6_r6d_ab_tables.log -- on)
#define IS3D_EARLY_SKIP 3
#endif
#ifndef IS3D_PAIR_RCP
#define IS3D_PAIR_RCP 1       // fast path: two phi points per reciprocal (sep_pair_t)
#endif
// timing ablations of k_spectra (wrong results; tools/ab.sh variants only, never a product build): 1 = lanes stop
// after their setup (no phi loop), 2 = lanes stop before their setup, 3 = modified lanes run the tail fours,
// 4 = no per-lane cell work at all (tiles, tables, barriers only), 5 = 4 without the per-tile tables
#ifndef IS3D_ABLATE
#define IS3D_ABLATE 0
#endif
// IS3D_MOD_TABLES (cf_math.h): the modified launch builds only the per-tile tables its lanes read
// per-tile table loops split their flat index into (cell, row, phi) with a float reciprocal of the runtime row count
// instead of integer divisions
#ifndef IS3D_TAB_FDIV
#define IS3D_TAB_FDIV 1
#endif

// q = r / d, m = r % d for 0 <= r < 2^24, d >= 1 (rd = 1 / d in float): float(r) is exact and the float quotient is
// within (r / d) 2^-23 < 1 of the true one, so one correction step makes it exact
__device__ __forceinline__ void fdivmod(int r, int d, float rd, int& q, int& m) {
  q = (int)((float)r * rd);
  m = r - q * d;
  if (m < 0) { q--; m += d; }
  if (m >= d) { q++; m -= d; }
}


struct DndxArgs {
  const double* rec; long n;
  const double* renorm;       // PTM: [c][renorm class]
  const int* rcls; int nrcls; // renorm class of each sorted species (engine.hip), number of classes
  double* ycell;              // [npart (sorted)][n]: sum over (pT, phi, y, eta) of w_pT w_phi w_eta p.dsigma f
  const double *smass, *ssign, *sbaryon;
  const double *pT, *pTw, *cphi, *sphi, *phiw, *yv, *etav, *etaw;
  int npart, npT, nphi, nk, nl, nq, njb;
  int Sl, Yl, ntask, nbx;     // species per wavefront, task slots per wavefront, tasks per species
                              // (y x phi block x eta node), species groups
  long cells_per_wg, nchunk;
  int dim;
  const int* fbcells;         // F_FB launch (modified modes): ascending indices of the cells with separable-fallback
  const int* fbcount;         //   lanes (k_fbwrite) and their number; the launch adds those lanes' sums to ycell
};

// k_phitab: the F_TS tables of one chunk of cells (every pT), rows [pT][cell - c0][phitab_row]
struct PhiTabArgs {
  const double* rec; long c0, nc;           // records of the launch window, first cell and cells of the chunk
  const double *pT, *cphi, *sphi;
  int npT, nphi, nphp;
  double* tab; long phn;                    // rows per pT plane (>= nc)
  int by;                                   // F_BY: rows carry T3
  const unsigned long long* gate; int gate_want;   // as SpecArgs
};

template <int MODE>
void launch_spectra(dim3 grid, size_t shmem, hipStream_t st, const SpecArgs& a, int flags, int kj);
template <int MODE>
void launch_dndx(dim3 grid, size_t shmem, hipStream_t st, const DndxArgs& a, int flags, int kj);
template <int MODE>
void launch_phitab(hipStream_t st, const PhiTabArgs& a);

// phi blocks launch_spectra has an instantiation for (the host plan must pick one of these)
__host__ __device__ constexpr bool spectra_kj_supported(int kj) {
#ifdef IS3D_KJ16
  if (kj == 16) return true;
#endif
  return kj == 32 || kj == 24 || kj == 8 || kj == 2;
}

#ifdef IS3D_KERNEL_DEFS
// The kernels and their helpers have internal linkage (unnamed namespace): with external linkage the
// AMDGPU backend must keep them callable from elsewhere and allocated Grad's k_spectra 35 spilled
// VGPRs + 60 spilled SGPRs (11% slower on MI355X) where the internal-linkage build spills nothing.
namespace {
// 32 phi points of one lane; the next points' LDS pairs are loaded before the current ones are
// evaluated so the LDS latency overlaps the FP64 chain
template <int MODE, int FLAGS, bool FAST, int KJ, typename ACC>
__device__ __forceinline__ void sep_phi_loop(const SepLane& L, const dbl2* CS, const dbl2* BP, ACC acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : (MODE == CE || MODE == PTM) ? SEP_CE : (MODE == PTB) ? SEP_PTB : SEP_FEQ;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  if (FAST && IS3D_QUAD_RCP && ((IS3D_NOPF_MODES >> MODE) & 1) && sep_quads(MODE, KJ)) {
    // fours without the one-quad-ahead prefetch (for register-starved builds)
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      dbl2 c[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; i++) { c[i] = CS[jj + i]; b[i] = BP[jj + i]; }
      double v[4];
      sep_quad_t<FL, REG, OUT>(L, c, b, v);
#pragma unroll
      for (int i = 0; i < 4; i++) acc[jj + i] += v[i];
    }
    return;
  }
  if (FAST && IS3D_QUAD_RCP && sep_quads(MODE, KJ)) {
    dbl2 c[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { c[i] = CS[i]; b[i] = BP[i]; }
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      dbl2 nc[4], nb[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        nc[i] = c[i]; nb[i] = b[i];
        if (jj + 4 < KJ) { nc[i] = CS[jj + 4 + i]; nb[i] = BP[jj + 4 + i]; }
      }
      double v[4];
      sep_quad_t<FL, REG, OUT>(L, c, b, v);
#pragma unroll
      for (int i = 0; i < 4; i++) { acc[jj + i] += v[i]; c[i] = nc[i]; b[i] = nb[i]; }
    }
    return;
  }
  if (FAST && IS3D_PAIR_RCP) {
    dbl2 c0 = CS[0], b0 = BP[0], c1 = CS[1], b1 = BP[1];
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 2) {   // phi rows are padded to a multiple of KJ
      dbl2 n0 = c0, m0 = b0, n1 = c1, m1 = b1;
      if (jj + 2 < KJ) { n0 = CS[jj + 2]; m0 = BP[jj + 2]; n1 = CS[jj + 3]; m1 = BP[jj + 3]; }
      double v0, v1;
      sep_pair_t<FL, REG, OUT>(L, c0, b0, c1, b1, v0, v1);
      acc[jj] += v0; acc[jj + 1] += v1;
      c0 = n0; b0 = m0; c1 = n1; b1 = m1;
    }
    return;
  }
  dbl2 c = CS[0], b = BP[0];
#pragma unroll
  for (int jj = 0; jj < KJ; jj++) {
    dbl2 cn = c, bn = b;
    if (jj + 1 < KJ) { cn = CS[jj + 1]; bn = BP[jj + 1]; }
    acc[jj] += sep_point_t<FL, REG, OUT, FAST>(L, c, b);
    c = cn; b = bn;
  }
}

// {pc, ps} of phi slot k from LDS or, wave-uniform, from the constant address space (scalar loads)
typedef const __attribute__((address_space(4))) double* cs_sptr;
__device__ __forceinline__ dbl2 cs_at(const dbl2* p, int k) { return p[k]; }
__device__ __forceinline__ dbl2 cs_at(cs_sptr p, int k) {
  dbl2 v;
  v.x = p[2 * k]; v.y = p[2 * k + 1];
  return v;
}

// sep_phi_loop's fours for fast Grad / RTA-CE lanes with p.dsigma b' from the PD table (sep_quad_pd_t)
template <int MODE, int FLAGS, int KJ, bool SC, typename CSP>
__device__ __forceinline__ void sep_phi_loop_pd(const SepLane& L, CSP CS, const dbl2* BP, const double* PD,
                                                double* acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : (MODE == CE || MODE == PTM) ? SEP_CE : (MODE == PTB) ? SEP_PTB : SEP_FEQ;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  if (!IS3D_PD_PREFETCH) {
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      dbl2 c[4], b[4];
      double pd[4], v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) { c[i] = cs_at(CS, jj + i); b[i] = BP[jj + i]; pd[i] = PD[jj + i]; }
      sep_quad_pd_t<FL, REG, OUT, SC>(L, c, b, pd, v);
#pragma unroll
      for (int i = 0; i < 4; i++) acc[jj + i] += v[i];
    }
    return;
  }
  dbl2 c[4], b[4];
  double pd[4];
#pragma unroll
  for (int i = 0; i < 4; i++) { c[i] = cs_at(CS, i); b[i] = BP[i]; pd[i] = PD[i]; }
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    dbl2 nc[4], nb[4];
    double np[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      nc[i] = c[i]; nb[i] = b[i]; np[i] = pd[i];
      if (jj + 4 < KJ) { nc[i] = cs_at(CS, jj + 4 + i); nb[i] = BP[jj + 4 + i]; np[i] = PD[jj + 4 + i]; }
    }
    double v[4];
    sep_quad_pd_t<FL, REG, OUT, SC>(L, c, b, pd, v);
#pragma unroll
    for (int i = 0; i < 4; i++) { acc[jj + i] += v[i]; c[i] = nc[i]; b[i] = nb[i]; pd[i] = np[i]; }
  }
}

// RTA-CE lanes of the per-lane launch with the {TE, T2} table (sep_quad_pde_t; TAIL: Boltzmann-tail lanes)
template <int FLAGS, int KJ, bool TAIL, typename CSP>
__device__ __forceinline__ void sep_phi_loop_pde(const SepLane& L, CSP CS, const dbl2* BP, const double* PD,
                                                 const dbl2* PE, double* acc) {
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    dbl2 c[4], b[4], pe[4];
    double pd[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { c[i] = cs_at(CS, jj + i); b[i] = BP[jj + i]; pd[i] = PD[jj + i]; pe[i] = PE[jj + i]; }
    sep_quad_pde_t<REG, OUT, TAIL>(L, c, b, pd, pe, acc + jj);
  }
}

// fast Grad lanes of an F_TB launch: fours from the {b', Phi} and {PD, T1} tables (sep_quad_tb_t)
template <int MODE, int FLAGS, int KJ>
__device__ __forceinline__ void sep_phi_loop_tb(const SepLane& L, double mT, const dbl2* BP, const dbl2* PT,
                                                const dbl2* PE, double* acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  static_assert(KJ % 4 == 0, "F_TB needs phi blocks of fours");
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    dbl2 b[4], pt[4], pe[4];
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      b[i] = BP[jj + i]; pt[i] = PT[jj + i];
      if (FL == SEP_CE) pe[i] = PE[jj + i];
    }
    sep_quad_tb_t<FL, REG, OUT>(L, mT, b, pt, pe, v);
#pragma unroll
    for (int i = 0; i < 4; i++) acc[jj + i] += v[i];
  }
}

// Boltzmann-tail lanes of an F_TB launch (sep_setup allow_tail): sep_quad_tb_tail_t, no reciprocal per point
template <int MODE, int FLAGS, int KJ>
__device__ __forceinline__ void sep_phi_loop_tb_tail(const SepLane& L, double mT, const dbl2* BP, const dbl2* PT,
                                                     const dbl2* PE, double* acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  static_assert(KJ % 4 == 0, "F_TB needs phi blocks of fours");
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    dbl2 b[4], pt[4], pe[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      b[i] = BP[jj + i]; pt[i] = PT[jj + i];
      if (FL == SEP_CE) pe[i] = PE[jj + i];
    }
    sep_quad_tb_tail_t<FL, REG, OUT>(L, mT, b, pt, pe, acc + jj);
  }
}

// F_TS lanes: the F_TB fours (sep_quad_tb_t / sep_quad_tb_tail_t, the same arithmetic) with {b', Phi}, PD and
// RTA-CE's {TE, T2} by scalar loads from the cell's k_phitab row G (wave-uniform address: SGPR operands) and T1
// from the lane's LDS row (16-byte aligned pairs: one ds_read_b128 per two points)
template <int MODE, int FLAGS, int KJ, bool TAIL, bool NEAR = false>
__device__ __forceinline__ void sep_phi_loop_ts(const SepLane& L, double mT, double bary, cs_sptr G, const dbl2* T1,
                                                double* acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0, BY = (FLAGS & F_BY) != 0;
  static_assert(KJ % 4 == 0, "F_TS needs phi blocks of fours");
  constexpr int O3 = (MODE == CE ? 5 : 3) * KJ;        // T3 slot of the row (F_BY)
  // operands of one four: scalar loads from G and the T1 pairs from LDS (both counted by lgkmcnt, the scalar
  // ones out of order: a wait for either is a wait for all, so the next four's loads go out before this four's
  // arithmetic -- AHEAD -- instead of just before their use)
  struct Four { dbl2 b[4], pt[4], pe[4]; double t3[4]; };
  auto load = [&](int jj, Four& f) {
    const dbl2 t01 = T1[jj >> 1], t23 = T1[(jj >> 1) + 1];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      f.b[i].x = G[2 * (jj + i)]; f.b[i].y = G[2 * (jj + i) + 1];
      f.pt[i].x = G[2 * KJ + jj + i];
      if (FL == SEP_CE) { f.pe[i].x = G[3 * KJ + 2 * (jj + i)]; f.pe[i].y = G[3 * KJ + 2 * (jj + i) + 1]; }
      f.t3[i] = BY ? G[O3 + jj + i] : 0.0;
    }
    f.pt[0].y = t01.x; f.pt[1].y = t01.y; f.pt[2].y = t23.x; f.pt[3].y = t23.y;
  };
  constexpr int AH = (MODE == GRAD) ? (BY ? IS3D_TS_AHEAD_GRAD_BY : IS3D_TS_AHEAD_GRAD) : IS3D_TS_AHEAD_CE;
  constexpr bool AHEAD = (AH >> (TAIL || NEAR ? 0 : 1)) & 1;
  Four fq[2];
  if (AHEAD) load(0, fq[0]);
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    Four& cur = fq[AHEAD ? (jj >> 2) & 1 : 0];
    if (AHEAD) {
      // wait for this four's operands (lgkmcnt(0)) before the next four's loads go out, and keep the compiler
      // from moving them (left alone, it issued the loads of two fours before one wait)
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
      if (jj + 4 < KJ) load(jj + 4, fq[((jj >> 2) + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      load(jj, cur);
    }
    const dbl2* b = cur.b; const dbl2* pt = cur.pt; const dbl2* pe = cur.pe; const double* t3 = cur.t3;
    if constexpr (NEAR) {
      static_assert(FL == SEP_GRAD && !REG, "near-tail fours: Grad without regulate");
      sep_quad_tb_near_t<OUT, true, BY>(L, mT, b, pt, acc + jj, bary, t3);
    } else if (TAIL) {
      sep_quad_tb_tail_t<FL, REG, OUT, true, BY>(L, mT, b, pt, pe, acc + jj, bary, t3);
    } else {
      double v[4];
      sep_quad_tb_t<FL, REG, OUT, true, BY>(L, mT, b, pt, pe, v, bary, t3);
#pragma unroll
      for (int i = 0; i < 4; i++) acc[jj + i] += v[i];
    }
  }
}

// Boltzmann-tail Grad lanes of an F_TB launch, PD-table form: {b', Phi} and PD from LDS, {pc, ps} by scalar
// loads (sep_quad_pd_tail_t; 6 LDS-array cycles per point instead of 8)
template <int MODE, int FLAGS, int KJ, typename CSP>
__device__ __forceinline__ void sep_phi_loop_pd_tail(const SepLane& L, CSP CS, const dbl2* BP, const double* PD,
                                                     double* acc) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    dbl2 c[4], b[4];
    double pd[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { c[i] = cs_at(CS, jj + i); b[i] = BP[jj + i]; pd[i] = PD[jj + i]; }
    sep_quad_pd_tail_t<FL, REG, OUT>(L, c, b, pd, acc + jj);
  }
}

// modified lanes of k_spectra, table form: {PDm, Qv} (MW) and T2 (MT) rows, four points per reciprocal
template <int FLAGS, bool CLAMP, int KJ, typename ACC>
__device__ __forceinline__ void mod_phi_loop_tab(const ModLane& M, const dbl2* MW, const double* MT, ACC acc) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
  if (IS3D_MOD_QUAD && !IS3D_MOD_PF && KJ % 4 == 0) {
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) mod_quad_tab_t<OUT, CLAMP>(M, MW + jj, MT + jj, acc + jj);
    return;
  }
  if (IS3D_MOD_QUAD && KJ % 4 == 0) {
    // the next four points' table rows are loaded before the current four are evaluated (at 2 waves per
    // SIMD the LDS latency is not hidden by other waves)
    dbl2 mw[4];
    double mt[4];
#pragma unroll
    for (int i = 0; i < 4; i++) { mw[i] = MW[i]; mt[i] = MT[i]; }
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      dbl2 nw[4];
      double nt[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        nw[i] = mw[i]; nt[i] = mt[i];
        if (jj + 4 < KJ) { nw[i] = MW[jj + 4 + i]; nt[i] = MT[jj + 4 + i]; }
      }
      mod_quad_tab_t<OUT, CLAMP>(M, mw, mt, acc + jj);
#pragma unroll
      for (int i = 0; i < 4; i++) { mw[i] = nw[i]; mt[i] = nt[i]; }
    }
    return;
  }
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 2) {
    double v0, v1;
    mod_pair_tab_t<OUT, CLAMP>(M, MW[jj], MW[jj + 1], MT[jj], MT[jj + 1], v0, v1);
    acc[jj] += v0; acc[jj + 1] += v1;
  }
}

// Boltzmann-tail modified lanes, table form (mod_quad_tab_tail_t; KJ % 4 == 0 only: mod_setup's allow_tail)
template <int FLAGS, int KJ, typename ACC>
__device__ __forceinline__ void mod_phi_loop_tab_tail(const ModLane& M, const dbl2* MW, const double* MT, ACC acc) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
  if constexpr (KJ % 4 == 0) {
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) mod_quad_tab_tail_t<OUT>(M, MW + jj, MT + jj, acc + jj);
  }
}

// modified lanes without q-row tables (lane_y launches): {pc, ps} and the {PDm, Qv} rows, the lane's
// linear forms for E_mod^2 and p.dsigma (mod_quad_lane_t), pairs of points per reciprocal
template <int FLAGS, bool CLAMP, int KJ, typename ACC>
__device__ __forceinline__ void mod_phi_loop_lane(const ModLane& M, const dbl2* CS, const dbl2* MW, ACC acc) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 2) {
    double v0, v1;
    mod_pair_lane_t<OUT, CLAMP>(M, CS[jj], CS[jj + 1], MW[jj].y, MW[jj + 1].y, v0, v1);
    acc[jj] += v0; acc[jj + 1] += v1;
  }
}

template <int FLAGS, bool CLAMP, int KJ>
__device__ __forceinline__ void mod_phi_loop(const ModLane& M, const dbl2* CS, const dbl2* QV, double* acc) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
  if (IS3D_MOD_QUAD && KJ % 4 == 0) {
    dbl2 c[4], qa = QV[0], qb = QV[1];
#pragma unroll
    for (int i = 0; i < 4; i++) c[i] = CS[i];
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      dbl2 nc[4], na = qa, nb = qb;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        nc[i] = c[i];
        if (jj + 4 < KJ) nc[i] = CS[jj + 4 + i];
      }
      if (jj + 4 < KJ) { na = QV[(jj >> 1) + 2]; nb = QV[(jj >> 1) + 3]; }
      double v[4];
      mod_quad_t<OUT, CLAMP>(M, c, qa, qb, v);
#pragma unroll
      for (int i = 0; i < 4; i++) { acc[jj + i] += v[i]; c[i] = nc[i]; }
      qa = na; qb = nb;
    }
    return;
  }
  dbl2 c0 = CS[0], c1 = CS[1], q = QV[0];
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 2) {
    dbl2 n0 = c0, n1 = c1, nq = q;
    if (jj + 2 < KJ) { n0 = CS[jj + 2]; n1 = CS[jj + 3]; nq = QV[(jj >> 1) + 1]; }
    double v0, v1;
    mod_pair_t<OUT, CLAMP>(M, c0, c1, q, v0, v1);
    acc[jj] += v0; acc[jj + 1] += v1;
    c0 = n0; c1 = n1; q = nq;
  }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations (lgkmcnt) but
// not for its outstanding global loads -- a __syncthreads() (or a workgroup release fence) would
// also wait for vmcnt(0) and drain the next tile's record copy.  The empty asm statements with a
// memory clobber keep the compiler from moving LDS accesses across the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}


// Async copy of the record tile starting at cell cb into LDS (global_load_lds_dwordx4: no VGPR
// staging; the LDS destination of a wave-instruction is base + 16 * lane, so the tile lands
// in the same linear order as the records in HBM).  Completion is tracked by vmcnt.
// With an index list (F_FB) tile slot k holds the record of cell idx[cb + k]: each lane names its own
// source pair, so the same LDS-DMA instruction gathers.
template <int KT>
__device__ __forceinline__ void fetch_tile(const double* rec, long cb, long c_end, double* dst, const int* idx = nullptr) {
  constexpr int kTilePairs = KT * NREC / 2;   // dbl2 pairs of one record tile (KT records of NREC doubles)
  const int tid = threadIdx.x;
  const long lim = (min(c_end, cb + KT) - cb) * (NREC / 2);
  for (int base = 0; base < kTilePairs; base += kBlock) {
    const int e = base + tid;
    const int wave0 = base + (tid & ~63);
    if (e < lim) {     // the index list is read only for slots of this tile (it holds just the listed cells)
      const long src = idx ? ((long)idx[cb + e / (NREC / 2)] * (NREC / 2) + e % (NREC / 2)) : cb * (NREC / 2) + e;
      __builtin_amdgcn_global_load_lds((const void*)(rec + src * 2),
                                       (__attribute__((address_space(3))) void*)(dst + 2 * wave0), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ void wait_fetch() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// KJ = phi points per lane (an even divisor-friendly block: 32, 24, 8 or 2, spectra_kj); a lane owns one
// (species, q, phi block) with q = (y, eta node): in 2+1D the eta nodes are spread over lanes and
// summed by k_reduce, so a few species still fill the wavefronts
template <int MODE, int FLAGS, int KJ>
__global__ __launch_bounds__(kBlock, (spectra_waves_f<MODE, FLAGS, KJ>())) void k_spectra(SpecArgs A) {
  if (gate_closed(A.gate, A.gate_want)) return;
  constexpr int kTile = spectra_tile<MODE, FLAGS>();      // cells per LDS tile for this mode / launch
  extern __shared__ double smem[];
  const int nphp = A.njb * KJ;                            // phi rows padded to KJ multiples
  constexpr bool TB = (MODE == GRAD || MODE == CE) && (FLAGS & F_TB) != 0 && KJ % 4 == 0;
  // F_TS: per-(cell, phi) operands from the k_phitab rows by scalar loads; LDS holds the T1 rows only
  constexpr bool TS = TB && (FLAGS & F_TS) != 0;
  constexpr bool FB = MODE >= PTM && (FLAGS & F_FB) != 0;   // separable-fallback launch of a modified mode
  constexpr bool MODMAIN = MODE >= PTM && !FB;              // modified launch: separable lanes left to F_FB
  constexpr bool LY = (FLAGS & F_LY) != 0 || FB;
  // Boltzmann-tail lanes of the per-lane Grad / RTA-CE launches (PD-table fours, sep_quad_pd_tail_t)
  constexpr bool PDT = IS3D_TAIL_PDL && !TB && MODE <= CE && IS3D_PD_TABLE && KJ % 4 == 0;
  // RTA-CE per-lane launch with the per-(cell, phi) {TE, T2} table (one pT per workgroup, workgroup y-term rows)
  constexpr bool PDE = IS3D_CE_PE && MODE == CE && !TB && (FLAGS & F_MP) == 0 && !LY && IS3D_PD_TABLE && KJ % 4 == 0;
  constexpr bool MP = (FLAGS & F_MP) != 0;                  // several pT per workgroup, one phi block per lane
  const int npw = MP ? A.npw : 1;                           // pT values of this launch's workgroups
  // per-(cell, q, phi) tables built from the per-tile tables (phase C below): Grad / RTA-CE {PD, T1},
  // modified path T2
  constexpr bool HAS_C = TB || (MODE >= PTM && !LY);
  // pipelined tile schedule (see the tile loop): record tiles triple-buffered, per-tile tables
  // double-buffered.  Only the launches whose tables are small (F_TB: <= kTbQ rows per cell; the modified
  // path's 16-cell tiles, which fall back to F_T8 when they do not fit): double y-term rows of many q
  // values would cost a workgroup per CU (config 1's shape: 4.8 -> 5.7 ms, r2z)
  constexpr bool PIPE = IS3D_PIPE && (TB || (MODE >= PTM && !(FLAGS & (F_LY | F_T8 | F_FB))));
  constexpr int kRecBufs = PIPE ? 3 : 2, kTabBufs = PIPE ? 2 : 1;
  constexpr int kQvF = (MODE >= PTM || !PIPE) ? 2 : 1;    // doubles per (cell, phi) of s_qv
  const int nqm = A.nqmax;                                // rows per cell (>= every workgroup's nqw)
  const long recsz = (long)kTile * NREC, bpsz = TS ? 0L : (long)npw * kTile * nphp, qvsz = kQvF * bpsz;
  // the {b', Phi} rows: none in F_TS launches, nor in modified launches that build only the tables their lanes read
  const long bpa = (MODMAIN && IS3D_MOD_TABLES) ? 0L : bpsz;
  // exp table entries at LDS offset 0: the modified lanes' own table in the modified launches (IS3D_MOD_TAB_BITS)
  constexpr int kET = MODMAIN ? kModTabN : kExpTabN;
  // y-term rows per cell: per row, or per q once the rows cover every q (nyr below): min(nqm, nq);
  // LY launches: one y-term row per lane instead ([kBlock][kYRowLY], single; odd row stride: no conflicts)
  const long ysz = LY ? (long)kBlock * kYRowLY : (long)kTile * min(nqm, A.nq) * kYRow;
  // the exp table first: at LDS offset 0 its address is the table index alone (no base register, which
  // the modified loop otherwise re-read from an SGPR spill lane at every point)
  double* s_etab = smem;                                  // [kET] 2^(j/kET)
  double* s_recb = smem + kET;                            // [kRecBufs][kTile][NREC]
  dbl2* s_trig = (dbl2*)(s_recb + kRecBufs * recsz);      // [nphp]        {cos, sin}
  dbl2* s_cs = s_trig + nphp;                             // [npw][nphp]   {pT cos, pT sin}
  dbl2* s_bp = s_cs + npw * nphp;                         // [kTabBufs][npw][kTile][nphp] {b', Phi}
  // Grad / RTA-CE: [kTabBufs][kTile][nphp] PD table; modified path: {PDm, Qv} pairs (s_mw)
  double* s_qv = (double*)(s_bp + kTabBufs * bpa);
  double* s_grid = s_qv + kTabBufs * qvsz;                // y[nk] | eta[nl] | eta_w[nl]
  double* s_y = s_grid + A.nk + 2 * A.nl;                 // [kTabBufs (LY: 1)][kTile][min(nqm, nq)][kYRow]
  // TB: [kTile][nqm][prow] {PD, T1}, 16-byte aligned for ds_read_b128 (s_grid's nk + 2 nl doubles
  // can leave the y-term rows' end at an odd double; misaligned dbl2 reads ran the kernel 3.5x slower)
  dbl2* s_pt = (dbl2*)(smem + (((s_y + (LY ? 1 : kTabBufs) * ysz) - smem + 1) & ~1L));
  // row tables hold the KJ phi points of their row's phi block plus one padding entry, so two rows read
  // at the same phi by the two halves of a wavefront that straddles a row boundary land in different
  // banks (a 512-B row stride is 128 dwords: the same bank, a 2-way conflict in every straddling wave)
  constexpr int prow = KJ + 1;
  dbl2* s_pe = s_pt + (TB && !TS ? kTile * nqm * prow : 0);   // TB / PDE, RTA-CE: [kTabBufs][kTile][nphp] {TE, T2}
  double* s_mt = (double*)s_pt;                           // modified path: [kTile][nqm][prow] T2 = 2 U_q . W
  // F_TS: [kTile][nqm][prow2] T1 rows; an even stride keeps every row 16-byte aligned for the ds_read_b128 pairs,
  // and 2 (KJ + 2) dwords put the same phi of two rows of a straddling wavefront 4 banks apart
  constexpr int prow2 = KJ + 2;
  double* s_t1 = (double*)s_pt;

  const int tid = threadIdx.x;
  for (int i = tid; i < kET; i += kBlock) s_etab[i] = MODMAIN ? kModExp2Tab[i] : kExp2Tab[i];
  // XCD-aware block order (cdna_hip_programming.md T1): blocks that share an XCD (same
  // blockIdx % 8) take one contiguous range of logical ids, and logical ids run split-major, so
  // each XCD's L2 sees only its own cell splits (sized to fit) instead of every split
  // F_MP: the workgroup's pT group pg holds pT values pg npw .. pg npw + npw - 1; lane tid is task tid % ntask
  // of pT lp = tid / ntask
  const long npg = MP ? (A.npT + npw - 1) / npw : A.npT;
  const long nwg = (long)A.nbx * npg * A.nsplit;
  const long bid = blockIdx.x, q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const long lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int lane_group = (int)(lid % A.nbx);
  const int pg = (int)((lid / A.nbx) % npg);
  const int split = A.split0 + (int)(lid / ((long)A.nbx * npg));
  const int lp = MP ? tid / (int)A.ntask : 0;
  const int ipt = MP ? min(pg * npw + lp, A.npT - 1) : pg;
  const double pT = A.pT[ipt];
  const long task = MP ? (long)(tid % (int)A.ntask) : (long)lane_group * kBlock + tid;
  const bool active = MP ? (lp < npw && pg * npw + lp < A.npT) : task < A.ntask;
  int s = 0, q = 0, jb = 0;
  if (active) {
    s = (int)(task % A.npart);
    const long r = task / A.npart;
    q = (int)(r % A.nq);
    jb = (int)(r / A.nq);
  }
  const int j0 = jb * KJ;
  // rows r = task / npart = q + nq jb this workgroup's 256 consecutive tasks use: the contiguous range
  // r0 .. r0 + nqw - 1, at most (kBlock - 1) / npart + 2 of them (the host's nqmax).  The y-terms and
  // the q tables are built per row (row r holds the (cell, q) y-terms and its own phi block's points),
  // so a workgroup never builds rows its lanes do not read, whatever the number of phi blocks
  long r0 = 0;
  int nqw = 1;
  {
    const long t0 = (long)lane_group * kBlock, t1 = min(A.ntask, t0 + kBlock) - 1;
    r0 = t0 / A.npart;
    nqw = (int)(t1 / A.npart - r0) + 1;
  }
  const int row = active ? (int)(task / A.npart - r0) : 0;
  // the LDS row tables are sized for nqmax rows (host, spectra_plan): a launch whose workgroup spans more
  // would write past them, so it computes nothing and returns NaN spectra instead (never on a host plan)
  const bool rows_ok = LY || nqw <= A.nqmax;
  // y-term rows: per row, or per q when the rows cover every q (several phi blocks, few species: the
  // y-terms depend on q only)
  const bool allq = nqw >= A.nq;
  const int nyr = allq ? A.nq : nqw;
  const int yrow = allq ? q : row;
  const double mass = A.smass[s], m2 = mass * mass, sign = A.ssign[s], baryon = A.sbaryon[s];
  const double mT = sqrt(m2 + pT * pT), mT2 = mT * mT, mTb = mT * baryon;

  // per-workgroup constants into LDS: inside the cell loop the only global loads are the
  // record prefetch (and PTM's renormalisation factor)
  for (int i = tid; i < npw * nphp; i += kBlock) {
    const int j = i % nphp;
    const bool in = j < A.nphi;
    const double c = in ? A.cphi[j] : 0.0, sn = in ? A.sphi[j] : 0.0;
    dbl2 v; v.x = c; v.y = sn;
    if (i < nphp) s_trig[j] = v;
    const double pTi = MP ? A.pT[min(pg * npw + i / nphp, A.npT - 1)] : pT;
    v.x = pTi * c; v.y = pTi * sn;
    s_cs[i] = v;
  }
  for (int i = tid; i < A.nk; i += kBlock) s_grid[i] = (A.dim == 3) ? A.yv[i] : 0.0;
  for (int i = tid; i < A.nl; i += kBlock) {
    s_grid[A.nk + i] = (A.dim == 3) ? 0.0 : A.etav[i];
    s_grid[A.nk + A.nl + i] = (A.dim == 3) ? 1.0 : A.etaw[i];
  }

  double acc[KJ];
#pragma unroll
  for (int jj = 0; jj < KJ; jj++) acc[jj] = 0.0;

  // F_FB: positions in the fallback cell list (its length is known on the device only), split evenly
  long c_begin, c_end;
  if constexpr (FB) {
    const long nfb = *A.fbcount, cps = ((nfb + A.nsplit - 1) / A.nsplit + kTile - 1) / kTile * kTile;
    c_begin = (long)split * cps;
    c_end = min(nfb, c_begin + cps);
  } else {
    c_begin = (long)split * A.cells_per_split;
    c_end = min(A.n, c_begin + A.cells_per_split);
  }
  const int* const fbl = FB ? A.fbcells : nullptr;
  // this thread's slab entries, layout [split][pT][lane group][phi slot][lane] (see the stores at the end); F_MP:
  // lane group 0 of the lane's own pT, slot = its task
  double* const out = A.slab + (long)(split - A.slab0) * A.sstride + ((long)ipt * A.nbx + lane_group) * (KJ * kBlock) +
                      (MP ? task : (long)tid);

  // ---- phase A / B of one tile (records s_rec, ntx cells) into table buffer tb: {b', Phi} and PD (or
  // the modified path's {PDm, Qv}) per (cell, phi), {TE, T2} for RTA-CE's table launch, y-terms per
  // (cell, row)
  auto tables_ab = [&](const double* s_rec, int ntx, int tb) __attribute__((always_inline)) {
    if (IS3D_ABLATE >= 5) return;
    dbl2* bp = s_bp + tb * bpsz;
    double* qvt = s_qv + tb * qvsz;
    dbl2* mw = (dbl2*)qvt;
    dbl2* pe = s_pe + tb * bpsz;
    double* yb = s_y + tb * ysz;
    // F_MP: npw pT blocks of [kTile][nphp]; o = the entry's offset in its block, csj = its {pc, ps}
    for (int idx = tid; idx < (TS ? 0 : npw * ntx * nphp); idx += kBlock) {
      const int l2 = MP ? idx / (ntx * nphp) : 0, ix = MP ? idx % (ntx * nphp) : idx;
      const int t = ix / nphp, j = ix % nphp;
      const int o = (l2 * kTile + t) * nphp + j;
      const dbl2 csj = s_cs[l2 * nphp + j];
      const double pTl = MP ? A.pT[min(pg * npw + l2, A.npT - 1)] : pT;
      const double* R = s_rec + t * NREC;
      dbl2 v; v.x = 0.0; v.y = 0.0;                        // padding: finite, never written out
      double qv = 0.0;
      if (j < A.nphi && R[R_KIND] != 0.0) {
        const dbl2 tr = s_trig[j];
        // the modified launch reads only {PDm, Qv}: {b', Phi} serve the separable lanes (the F_FB launch)
        if constexpr (!(MODMAIN && IS3D_MOD_TABLES)) v = phiterms(MODE, R, pTl, tr.x, tr.y, s_etab);
        if (MODE >= PTM && R[R_KIND] == 2.0) qv = modqv(R, csj);
      }
      if constexpr (!(MODMAIN && IS3D_MOD_TABLES)) bp[o] = v;
      if constexpr (MODE >= PTM) {
        dbl2 m; m.x = modpdm(R, csj); m.y = qv;           // zero rows / padding give 0
        mw[o] = m;
      } else {
        qvt[o] = sep_pd(R, csj, v.x);                     // PD table (sep_pd)
      }
      if constexpr ((TB || PDE) && MODE == CE && !TS) {
        const dbl2 c = s_cs[j];
        dbl2 e;
        e.x = -fma(R[R_UX], c.x, R[R_UY] * c.y);
        e.y = fma(R[R_LC], c.x, R[R_LS] * c.y);
        pe[t * nphp + j] = e;
      }
    }
    for (int idx = tid; idx < (LY ? 0 : ntx * nyr); idx += kBlock) {
      const int t = idx / nyr, qq = idx % nyr, q = allq ? qq : (int)((r0 + qq) % A.nq);
      const double* R = s_rec + t * NREC;
      if (R[R_KIND] != 0.0) {
        const int kk = q / A.nl, l = q % A.nl;
        const double y = s_grid[kk];
        const double eta = (A.dim == 3) ? R[R_ETA] : s_grid[A.nk + l];
        yterms(MODE, A.op, R, y, eta, s_grid[A.nk + A.nl + l], yb + ((long)t * nyr + qq) * kYRow, true,
               MODMAIN && IS3D_MOD_TABLES);
      }
    }
  };
  // ---- phase C: the per-(cell, row, phi) tables of one tile from its buffer-tb tables (single buffer)
  // flat per-tile table index -> phi slot jj, (cell t, row qq), phi block jb and q = (r0 + qq) % nq
  const float rnqw = MODMAIN ? 1.0f / (float)nqw : 0.0f, rnq = MODMAIN ? 1.0f / (float)A.nq : 0.0f;
  auto tab_index = [&](int idx, int& jj, int& t, int& qq, int& jb, int& qm) __attribute__((always_inline)) {
    jj = idx % KJ;
    const int r = idx / KJ;
    if (IS3D_TAB_FDIV) {
      fdivmod(r, nqw, rnqw, t, qq);
      fdivmod((int)r0 + qq, A.nq, rnq, jb, qm);
    } else {
      qq = r % nqw; t = r / nqw;
      jb = (int)((r0 + qq) / A.nq); qm = (int)((r0 + qq) % A.nq);
    }
  };
  auto tables_c = [&](const double* s_rec, int ntx, int tb) __attribute__((always_inline)) {
    if (IS3D_ABLATE >= 5) return;
    const double* qvt = s_qv + tb * qvsz;
    const double* yb = s_y + tb * ysz;
    if constexpr (MODE >= PTM && !LY) {
      // T2 = 2 U_q . W per (cell, q, phi) of the modified cells (mod_quad_tab_t)
      for (int idx = tid; idx < ntx * nqw * KJ; idx += kBlock) {
        int jj, t, qq, jb, qm;
        tab_index(idx, jj, t, qq, jb, qm);
        const int j = jb * KJ + jj;
        const double* R = s_rec + t * NREC;
        if (R[R_KIND] != 2.0) continue;
        const int yr = allq ? qm : qq;
        s_mt[((long)t * nqw + qq) * prow + jj] = modt2(R, yb + ((long)t * nyr + yr) * kYRow, s_cs[j]);
      }
    }
    // the separable launches keep their round-5 index arithmetic (integer divisions): with tab_index the F_TS kernels
    // compiled to the same loops but ran 1-1.5% slower (profiles/round6_r6j_ab_bisect.log)
    if constexpr (TS) {
      // T1 = SC1 pc + SS1 ps per (cell, q row, phi) (one phi block: phi slot jj)
      for (int idx = tid; idx < ntx * nqw * KJ; idx += kBlock) {
        const int jj = idx % KJ, r = idx / KJ, qq = r % nqw, t = r / nqw;
        const double* Y = yb + ((long)t * nyr + (allq ? (int)((r0 + qq) % A.nq) : qq)) * kYRow;
        const dbl2 c = s_cs[jj];
        s_t1[((long)t * nqw + qq) * prow2 + jj] = fma(Y[Y_SC1], c.x, Y[Y_SS1] * c.y);
      }
    } else if constexpr (TB) {
      // {PD, T1 = SC1 pc + SS1 ps} per (cell, q, phi) (rows of skipped cells are never read)
      for (int idx = tid; idx < ntx * nqw * KJ; idx += kBlock) {
        const int jj = idx % KJ, r = idx / KJ, qq = r % nqw, t = r / nqw;
        const int j = (int)((r0 + qq) / A.nq) * KJ + jj;
        const double* Y = yb + ((long)t * nyr + (allq ? (int)((r0 + qq) % A.nq) : qq)) * kYRow;
        const dbl2 c = s_cs[j];
        dbl2 v;
        v.x = qvt[t * nphp + j];
        v.y = fma(Y[Y_SC1], c.x, Y[Y_SS1] * c.y);
        s_pt[((long)t * nqw + qq) * prow + jj] = v;
      }
    }
  };
  // Tile schedule.  PIPE: a software pipeline over the split's record tiles (2 workgroup
  // barriers per tile instead of 3); iteration i:
  //   [records of tile i + 1 landed]  barrier X
  //   copy the records of tile i + 2 (buffer (i + 2) % 3, last read by iteration i - 1)
  //   phase C of tile i (from tables buffer i & 1)                          barrier Y (if phase C)
  //   phases A / B of tile i + 1 into tables buffer (i + 1) & 1
  //   lane work of tile i
  // so the y-term wave's work and the tables of tile i + 1 overlap other waves' lane work of tile i instead
  // of idling every wave at a barrier, and each record copy has a full tile of lead time.
  // otherwise: two record buffers, one table buffer, A / B -> barrier -> C -> barrier -> lanes.
  const int ntiles = (rows_ok && c_begin < c_end) ? (int)((c_end - c_begin + kTile - 1) / kTile) : 0;
  auto tile_cb = [&](int i) { return c_begin + (long)i * kTile; };
  auto tile_nt = [&](int i) { return (int)min((long)kTile, c_end - tile_cb(i)); };
  auto recbuf = [&](int i) { return s_recb + (i % kRecBufs) * recsz; };
  for (int i = 0; i < min(ntiles, kRecBufs - 1); i++) fetch_tile<kTile>(A.rec, tile_cb(i), c_end, recbuf(i), fbl);
  if (PIPE && ntiles > 0) {
    wait_fetch();
    lds_barrier();     // tiles 0 and 1, the trig / grid / exp tables visible
    tables_ab(recbuf(0), tile_nt(0), 0);
  }
  for (int i = 0; i < ntiles; i++) {
    const double* s_rec = recbuf(i);
    const long cbx = tile_cb(i);
    const int ntx = tile_nt(i), tb = PIPE ? (i & 1) : 0;
    wait_fetch();
    lds_barrier();     // X: this tile's records (and, pipelined, its A / B tables) visible; the last tile is done
    if (i + kRecBufs - 1 < ntiles) fetch_tile<kTile>(A.rec, tile_cb(i + kRecBufs - 1), c_end, recbuf(i + kRecBufs - 1), fbl);
    constexpr int PFD = (MODE == GRAD) ? IS3D_TS_PF_DIST_GRAD : IS3D_TS_PF_DIST_CE;
    if (i + PFD < ntiles) {
      if constexpr (TS && IS3D_TS_PF) {
        // the k_phitab rows of tile i + PFD (contiguous: cells x RW doubles of this pT) into L2, so the scalar loads of
        // its first points miss the K$ into L2 instead of HBM; one dword per 128-byte line, landing in a dummy LDS row
        constexpr int RW = phitab_row(MODE, KJ, (FLAGS & F_BY) != 0);
        const long cbp = tile_cb(i + PFD);
        const long nb = (min(c_end, cbp + kTile) - cbp) * RW * 8;
        const char* src = (const char*)(A.phtab + ((long)ipt * A.phn + (cbp - A.phc0)) * RW);
        double* pfd = s_t1 + (long)kTile * nqm * prow2;
        for (long off = (long)tid * 128; off < nb; off += (long)kBlock * 128)
          __builtin_amdgcn_global_load_lds((const void*)(src + off),
                                           (__attribute__((address_space(3))) void*)(pfd + 32 * (tid >> 6)), 4, 0, 0);
      }
    }
    if (!PIPE) {
      tables_ab(s_rec, ntx, 0);
      lds_barrier();
    }
    if constexpr (HAS_C) {
      tables_c(s_rec, ntx, tb);
      lds_barrier();   // Y
    }
    if (PIPE && i + 1 < ntiles) tables_ab(recbuf(i + 1), tile_nt(i + 1), (i + 1) & 1);
    if (active) {
      // the lane's phi points over the ntx cells of tile i
      const dbl2* bpt = s_bp + tb * bpsz;
      const double* qvt = s_qv + tb * qvsz;
      const dbl2* mwt = (const dbl2*)qvt;
      const dbl2* pet = s_pe + tb * bpsz;
      const double* yb = s_y + tb * ysz;
      // PTM: the lane's renormalisation factor of cell t + 1 is loaded while cell t is integrated (a
      // per-cell load used at once left every cell waiting for the HBM / MALL latency)
      const int rc = (MODE == PTM) ? A.rcls[s] : 0;
      auto rn_load = [&](int t) { return A.renorm[(FB ? (long)fbl[cbx + t] : cbx + t) * A.nrcls + rc]; };
      double rn_next = (MODE == PTM && ntx > 0) ? rn_load(0) : 0.0;
      for (int t = 0; t < ntx; t++) {
        const double rn_cell = rn_next;
        if (IS3D_ABLATE >= 4) { acc[0] += s_rec[t * NREC]; continue; }
        if (MODE == PTM && t + 1 < ntx) rn_next = rn_load(t + 1);
        const double* R = s_rec + t * NREC;
        const double kind = R[R_KIND];
        if (kind == 0.0) continue;
        double rn_abs = R[R_RENORM];
        if (MODE == PTM || MODE == PTB) {
          const double rn = (MODE == PTM) ? rn_cell : R[R_RENORM];
          if (!isfinite(rn)) continue;    // species skipped (MomentumSpectra.cpp:828-832)
          rn_abs = fabs(rn);
        }
        // this lane's (pT block, cell) row of the per-(cell, phi) tables (F_MP: block lp, else 0) and {pc, ps}
        const long tro = ((long)lp * kTile + t) * nphp + j0;
        const dbl2* BP = bpt + tro;
        const dbl2* CSl = s_cs + lp * nphp + j0;
        const double* Y = yb + ((long)t * nyr + yrow) * kYRow;
        if constexpr (LY) {        // this lane's own y-terms, in its LDS row
          double* Yl = s_y + (long)tid * kYRowLY;
          const int kk = q / A.nl, l = q % A.nl;
          yterms(MODE, A.op, R, s_grid[kk], (A.dim == 3) ? R[R_ETA] : s_grid[A.nk + l], s_grid[A.nk + A.nl + l], Yl, false);
          Y = Yl;
        }
        const bool sep = (MODE <= CE) || kind == 1.0 || Y[Y_NARROW] != 0.0;
        // the modified launch leaves its separable lanes to the F_FB launch and vice versa (if constexpr:
        // neither kernel carries the other's code)
        if (MODMAIN && sep) continue;
        if (FB && !sep) continue;
        if constexpr (!MODMAIN) {     // Grad / RTA-CE lanes (sep throughout), the F_FB launch's separable lanes
          if ((IS3D_EARLY_SKIP & 1) && sep_skips(R, Y, mT, pT, baryon)) continue;
          if (IS3D_ABLATE == 2) { acc[0] += R[R_KIND] * Y[0]; continue; }
          SepLane L;
          // near-tail lanes: F_TS Grad launches without regulate or baryon (IS3D_NEAR: config 2 166.2 -> 162.7 ms;
          // the F_BY launch, config 3, 176.8 -> 179.5 ms: off there)
          constexpr bool NEAR = TS && MODE == GRAD && !(FLAGS & (F_REG | F_BY)) && IS3D_NEAR && IS3D_TAIL && IS3D_TAIL_WAVE;
          sep_setup(sep_flavor(MODE), R, Y, mT, mT2, m2, mTb, pT, sign, baryon, s_etab, L,
                    ((TB && IS3D_TAIL && (MODE == GRAD || IS3D_TAIL_CE || TS)) || PDT) ? (IS3D_TAIL_WAVE ? 2 : 1) : 0,
                    NEAR ? 2 : 0);
          if (L.skip) continue;
          if (IS3D_ABLATE == 1) { acc[0] += L.a + L.D0 + L.S0 + L.Sc + L.Ss + L.E0 + L.L0 + L.escw + L.ssc + L.Dc + L.Ds; continue; }
          if constexpr (TS) {
            // this cell's k_phitab row (wave-uniform: ipt, the tile and t are) and the lane's T1 row
            constexpr int RW = phitab_row(MODE, KJ, (FLAGS & F_BY) != 0);   // one phi block: nphp = KJ
            const long go = ((long)ipt * A.phn + (cbx - A.phc0)) * RW + t * RW;
            const dbl2* T1 = (const dbl2*)(s_t1 + ((long)t * nqw + row) * prow2);
            if (IS3D_TAIL && L.tail) sep_phi_loop_ts<MODE, FLAGS, KJ, true>(L, mT, baryon, (cs_sptr)A.phtab + go, T1, acc);
            else if (NEAR && L.near) sep_phi_loop_ts<MODE, FLAGS, KJ, false, NEAR>(L, mT, baryon, (cs_sptr)A.phtab + go, T1, acc);
            else if (L.fast) sep_phi_loop_ts<MODE, FLAGS, KJ, false>(L, mT, baryon, (cs_sptr)A.phtab + go, T1, acc);
            // lanes off the fast path never reach F_TS (sep_slow_cell, engine.hip launch_end): their loop, inlined
            // here, was the kernels' register peak (IS3D_TS_SLOW = 1 keeps it)
            else if constexpr (IS3D_TS_SLOW) sep_phi_loop<MODE, FLAGS, false, KJ>(L, CSl, (const dbl2*)(A.phtab + go), acc);
            else atomicMax(A.err, (int)DF_TS_SLOW);
          } else if constexpr (TB) {
            const dbl2* PT = s_pt + ((long)t * nqw + row) * prow;
            if (IS3D_TAIL && L.tail) {
              if (MODE == GRAD && IS3D_TAIL_PD)
                sep_phi_loop_pd_tail<MODE, FLAGS, KJ>(L, (cs_sptr)A.csg + 2L * (ipt * nphp + j0), BP, qvt + t * nphp + j0, acc);
              else
                sep_phi_loop_tb_tail<MODE, FLAGS, KJ>(L, mT, BP, PT, pet + t * nphp + j0, acc);
            }
            else if (L.fast) sep_phi_loop_tb<MODE, FLAGS, KJ>(L, mT, BP, PT, pet + t * nphp + j0, acc);
            else sep_phi_loop<MODE, FLAGS, false, KJ>(L, CSl, BP, acc);
          } else if (IS3D_PD_TABLE && IS3D_CS_SCALAR && !MP && MODE <= CE && KJ % 4 == 0 && L.fast && A.njb == 1) {
            // one phi block: every lane reads the same {pc, ps}, so they come by scalar loads into SGPRs
            // (VALU operands) instead of LDS (not F_MP: a wavefront can straddle two pT blocks)
            if constexpr (PDE) {
              if (PDT && L.tail) sep_phi_loop_pde<FLAGS, KJ, true>(L, (cs_sptr)A.csg + 2L * ipt * nphp, BP, qvt + t * nphp, pet + t * nphp, acc);
              else sep_phi_loop_pde<FLAGS, KJ, false>(L, (cs_sptr)A.csg + 2L * ipt * nphp, BP, qvt + t * nphp, pet + t * nphp, acc);
            } else {
              if (PDT && L.tail) sep_phi_loop_pd_tail<MODE, FLAGS, KJ>(L, (cs_sptr)A.csg + 2L * ipt * nphp, BP, qvt + t * nphp, acc);
              else sep_phi_loop_pd<MODE, FLAGS, KJ, true>(L, (cs_sptr)A.csg + 2L * ipt * nphp, BP, qvt + t * nphp, acc);
            }
          } else if (IS3D_PD_TABLE && MODE <= CE && KJ % 4 == 0 && L.fast) {
            if constexpr (PDE) {
              if (PDT && L.tail) sep_phi_loop_pde<FLAGS, KJ, true>(L, CSl, BP, qvt + tro, pet + tro, acc);
              else sep_phi_loop_pde<FLAGS, KJ, false>(L, CSl, BP, qvt + tro, pet + tro, acc);
            } else {
              if (PDT && L.tail) sep_phi_loop_pd_tail<MODE, FLAGS, KJ>(L, CSl, BP, qvt + tro, acc);
              else sep_phi_loop_pd<MODE, FLAGS, KJ, true>(L, CSl, BP, qvt + tro, acc);
            }
          }
          else if (L.fast) sep_phi_loop<MODE, FLAGS, true, KJ>(L, CSl, BP, acc);
          else sep_phi_loop<MODE, FLAGS, false, KJ>(L, CSl, BP, acc);
        }
        if constexpr (MODMAIN) {
          if ((IS3D_EARLY_SKIP & 2) && IS3D_MOD_SQ_BOUNDS && mod_skips(R, Y, mT, m2, pT, baryon, !LY)) continue;
          if (IS3D_ABLATE == 2) { acc[0] += R[R_KIND] * Y[0]; continue; }
          ModLane M;
          const dbl2* MW = mwt + t * nphp + j0;
          const double* MT = s_mt + ((long)t * nqw + row) * prow;
          if constexpr (!LY && KJ % 4 == 0) mod_setup<KJ>(R, Y, mT, m2, pT, sign, baryon, rn_abs, s_etab, M, true, true, MW, MT);
          else mod_setup(R, Y, mT, m2, pT, sign, baryon, rn_abs, s_etab, M, !LY, false);
          if (M.skip) continue;
          if (IS3D_ABLATE == 1) { acc[0] += M.E0 + M.D0 + M.Dw + M.mT + M.shiftk + M.sign + M.tail + M.clamp; continue; }
          if constexpr (IS3D_ABLATE == 3 && !LY && KJ % 4 == 0) {
            if (!M.clamp) { mod_phi_loop_tab_tail<FLAGS, KJ>(M, MW, MT, acc); continue; }
          }
          if constexpr (LY) {        // no T2 rows: the lane's linear forms (mod_pair_lane_t)
            if (M.clamp) mod_phi_loop_lane<FLAGS, true, KJ>(M, CSl, MW, acc);
            else mod_phi_loop_lane<FLAGS, false, KJ>(M, CSl, MW, acc);
            continue;
          }
          if (M.clamp) mod_phi_loop_tab<FLAGS, true, KJ>(M, MW, MT, acc);
          else if (IS3D_MOD_TAIL && M.tail) mod_phi_loop_tab_tail<FLAGS, KJ>(M, MW, MT, acc);
          else mod_phi_loop_tab<FLAGS, false, KJ>(M, MW, MT, acc);
        }
      }
    }
  }
  // partial sums, slab layout [split][pT][lane group][phi slot][lane]: every store of the wave is
  // one contiguous 512-byte row; non-temporal so the stream does not evict the cell records the
  // XCD's other workgroups are still reading from L2.  k_reduce scatters into the reference layout.
  if (MP && !active) return;    // lanes past the workgroup's pT blocks own no slab entries
#pragma unroll
  for (int jj = 0; jj < KJ; jj++) __builtin_nontemporal_store(rows_ok ? acc[jj] : __builtin_nan(""), out + jj * kBlock);
}

// ------------------------------------------------------------------------------------------
// operation = 0: spacetime distributions dN/dX (SpacetimeDistribution.cpp:31-1250)
// ------------------------------------------------------------------------------------------
// Weighted phi sums: sum_j w_phi[j] x (w_eta p.dsigma f)(phi_j) for one lane and cell, with the
// same per-point arithmetic as k_spectra (W = phi weights as {w_j, w_j+1} pairs, 0 in the padding).
template <int MODE, int FLAGS, bool FAST, int KJ>
__device__ __forceinline__ double sep_phi_wsum(const SepLane& L, const dbl2* CS, const dbl2* BP, const dbl2* W) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : (MODE == CE || MODE == PTM) ? SEP_CE : (MODE == PTB) ? SEP_PTB : SEP_FEQ;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  double a0 = 0.0, a1 = 0.0;
  if constexpr (FAST && IS3D_PAIR_RCP && IS3D_DNDX_QUAD && KJ % 4 == 0) {
    // fours with one reciprocal (sep_quad_t, as k_spectra's lane-form launches)
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 4) {
      const dbl2 c[4] = {CS[jj], CS[jj + 1], CS[jj + 2], CS[jj + 3]}, b[4] = {BP[jj], BP[jj + 1], BP[jj + 2], BP[jj + 3]};
      const dbl2 wa = W[jj >> 1], wb = W[(jj >> 1) + 1];
      double v[4];
      sep_quad_t<FL, REG, OUT>(L, c, b, v);
      a0 = fma(wa.x, v[0], a0); a1 = fma(wa.y, v[1], a1);
      a0 = fma(wb.x, v[2], a0); a1 = fma(wb.y, v[3], a1);
    }
    return a0 + a1;
  }
  if (FAST && IS3D_PAIR_RCP) {
    dbl2 c0 = CS[0], b0 = BP[0], c1 = CS[1], b1 = BP[1];
#pragma unroll
    for (int jj = 0; jj < KJ; jj += 2) {
      dbl2 n0 = c0, m0 = b0, n1 = c1, m1 = b1;
      if (jj + 2 < KJ) { n0 = CS[jj + 2]; m0 = BP[jj + 2]; n1 = CS[jj + 3]; m1 = BP[jj + 3]; }
      const dbl2 w = W[jj >> 1];
      double v0, v1;
      sep_pair_t<FL, REG, OUT>(L, c0, b0, c1, b1, v0, v1);
      a0 = fma(w.x, v0, a0); a1 = fma(w.y, v1, a1);
      c0 = n0; b0 = m0; c1 = n1; b1 = m1;
    }
    return a0 + a1;
  }
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 2) {
    const dbl2 w = W[jj >> 1];
    a0 = fma(w.x, sep_point_t<FL, REG, OUT, FAST>(L, CS[jj], BP[jj]), a0);
    a1 = fma(w.y, sep_point_t<FL, REG, OUT, FAST>(L, CS[jj + 1], BP[jj + 1]), a1);
  }
  return a0 + a1;
}

// sep_phi_wsum for a Boltzmann-tail lane (Grad / RTA-CE, sep_setup allow_tail): sep_pair_tail_t
template <int MODE, int FLAGS, int KJ>
__device__ __forceinline__ double sep_phi_wsum_tail(const SepLane& L, const dbl2* CS, const dbl2* BP, const dbl2* W) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 2) {
    const dbl2 w = W[jj >> 1];
    double v0, v1;
    sep_pair_tail_t<FL, REG, OUT>(L, CS[jj], BP[jj], CS[jj + 1], BP[jj + 1], v0, v1);
    a0 = fma(w.x, v0, a0); a1 = fma(w.y, v1, a1);
  }
  return a0 + a1;
}

// sep_phi_wsum for fast lanes with the per-(cell, phi) PD rows (IS3D_DNDX_PD): sep_quad_pd_t's fours
template <int MODE, int FLAGS, int KJ>
__device__ __forceinline__ double sep_phi_wsum_pd(const SepLane& L, const dbl2* CS, const dbl2* BP, const double* PD,
                                                  const dbl2* W) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  static_assert(KJ % 4 == 0, "fours");
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    const dbl2 c[4] = {CS[jj], CS[jj + 1], CS[jj + 2], CS[jj + 3]}, b[4] = {BP[jj], BP[jj + 1], BP[jj + 2], BP[jj + 3]};
    const double pd[4] = {PD[jj], PD[jj + 1], PD[jj + 2], PD[jj + 3]};
    const dbl2 wa = W[jj >> 1], wb = W[(jj >> 1) + 1];
    double v[4];
    sep_quad_pd_t<FL, REG, OUT, true>(L, c, b, pd, v);
    a0 = fma(wa.x, v[0], a0); a1 = fma(wa.y, v[1], a1);
    a0 = fma(wb.x, v[2], a0); a1 = fma(wb.y, v[3], a1);
  }
  return a0 + a1;
}

// Boltzmann-tail Grad lanes with the PD rows: sep_quad_pd_tail_t's fours (w p.dsigma f_eq in two ops)
template <int MODE, int FLAGS, int KJ>
__device__ __forceinline__ double sep_phi_wsum_pd_tail(const SepLane& L, const dbl2* CS, const dbl2* BP, const double* PD,
                                                       const dbl2* W) {
  constexpr int FL = (MODE == GRAD) ? SEP_GRAD : SEP_CE;
  constexpr bool REG = (FLAGS & F_REG) != 0, OUT = (FLAGS & F_OUT) != 0;
  static_assert(KJ % 4 == 0, "fours");
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int jj = 0; jj < KJ; jj += 4) {
    const dbl2 c[4] = {CS[jj], CS[jj + 1], CS[jj + 2], CS[jj + 3]}, b[4] = {BP[jj], BP[jj + 1], BP[jj + 2], BP[jj + 3]};
    const double pd[4] = {PD[jj], PD[jj + 1], PD[jj + 2], PD[jj + 3]};
    const dbl2 wa = W[jj >> 1], wb = W[(jj >> 1) + 1];
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    sep_quad_pd_tail_t<FL, REG, OUT>(L, c, b, pd, v);
    a0 = fma(wa.x, v[0], a0); a1 = fma(wa.y, v[1], a1);
    a0 = fma(wb.x, v[2], a0); a1 = fma(wb.y, v[3], a1);
  }
  return a0 + a1;
}

// mod_phi_wsum with the per-(cell, phi) {PDm, Qv} rows (IS3D_DNDX_PDM): p.dsigma |renorm| = fma(Dw, PDm, D0), one op
// where the lane's linear form took two (the k_spectra table launch's form; Dw PDm = Dc pc + Ds ps to rounding)
template <int FLAGS, bool CLAMP, int KJ>
__device__ __forceinline__ double mod_phi_wsum_mw(const ModLane& M, const dbl2* CS, const dbl2* MW, const dbl2* W) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
  static_assert(KJ % 4 == 0, "fours");
  double a0 = 0.0, a1 = 0.0;
#pragma unroll IS3D_DNDX_MOD_UNROLL
  for (int jj = 0; jj < KJ; jj += 4) {
    const dbl2 c[4] = {CS[jj], CS[jj + 1], CS[jj + 2], CS[jj + 3]};
    const dbl2 mw[4] = {MW[jj], MW[jj + 1], MW[jj + 2], MW[jj + 3]};
    const dbl2 wa = W[jj >> 1], wb = W[(jj >> 1) + 1];
    double X[4], num[4], q[4], rq[4];
#pragma unroll
    for (int i = 0; i < 4; i++) X[i] = fma(M.Ec, c[i].x, fma(M.Es, c[i].y, M.E0 + mw[i].y));
    mod_nq4<CLAMP>(M, X, num, q);
    mod_quad_rq(q, rq);
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const double pds = fma(M.Dw, mw[i].x, M.D0);
      const double g = pds * (num[i] * rq[i]);
      v[i] = (OUT && pds <= 0.0) ? 0.0 : g;
    }
    a0 = fma(wa.x, v[0], a0); a1 = fma(wa.y, v[1], a1);
    a0 = fma(wb.x, v[2], a0); a1 = fma(wb.y, v[3], a1);
  }
  return a0 + a1;
}

template <int FLAGS, bool CLAMP, int KJ>
__device__ __forceinline__ double mod_phi_wsum(const ModLane& M, const dbl2* CS, const dbl2* QV, const dbl2* W) {
  constexpr bool OUT = (FLAGS & F_OUT) != 0;
  double a0 = 0.0, a1 = 0.0;
  if constexpr (IS3D_DNDX_QUAD && KJ % 4 == 0) {
    // fours: the staged table exp of mod_nq4 (four LDS reads per wait) and one reciprocal per four points
#pragma unroll IS3D_DNDX_MOD_UNROLL
    for (int jj = 0; jj < KJ; jj += 4) {
      const dbl2 c[4] = {CS[jj], CS[jj + 1], CS[jj + 2], CS[jj + 3]};
      const dbl2 qa = QV[jj >> 1], qb = QV[(jj >> 1) + 1], wa = W[jj >> 1], wb = W[(jj >> 1) + 1];
      const double qv[4] = {qa.x, qa.y, qb.x, qb.y};
      double X[4], num[4], q[4], rq[4];
#pragma unroll
      for (int i = 0; i < 4; i++) X[i] = fma(M.Ec, c[i].x, fma(M.Es, c[i].y, M.E0 + qv[i]));
      mod_nq4<CLAMP>(M, X, num, q);
      mod_quad_rq(q, rq);
      double v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const double pds = lin(M.D0, M.Dc, M.Ds, c[i]);
        const double g = pds * (num[i] * rq[i]);
        v[i] = (OUT && pds <= 0.0) ? 0.0 : g;
      }
      a0 = fma(wa.x, v[0], a0); a1 = fma(wa.y, v[1], a1);
      a0 = fma(wb.x, v[2], a0); a1 = fma(wb.y, v[3], a1);
    }
    return a0 + a1;
  }
  dbl2 c0 = CS[0], c1 = CS[1], q = QV[0];
#pragma unroll IS3D_DNDX_MOD_UNROLL
  for (int jj = 0; jj < KJ; jj += 2) {
    dbl2 n0 = c0, n1 = c1, nq = q;
    if (jj + 2 < KJ) { n0 = CS[jj + 2]; n1 = CS[jj + 3]; nq = QV[(jj >> 1) + 1]; }
    const dbl2 w = W[jj >> 1];
    double v0, v1;
    mod_pair_t<OUT, CLAMP>(M, c0, c1, q, v0, v1);
    a0 = fma(w.x, v0, a0); a1 = fma(w.y, v1, a1);
    c0 = n0; c1 = n1; q = nq;
  }
  return a0 + a1;
}



// One workgroup = (species group of Sl mass-sorted species, cell chunk).  Lane = (species s_l, slot); the
// 4 Yl slots of a workgroup stride over the species' tasks (y, phi block, eta node), so every wavefront
// evaluates one task for Sl neighbouring species at a time -- the exp-underflow skip stays coherent as in
// k_spectra.  The momentum loop (pT) is inside: per (cell tile, pT) the {b', Phi} phi-terms are rebuilt
// in LDS and every lane adds w_pT x sum_phi w_phi (point) into its column of s_red; after the pT loop a
// species' slot columns are summed in slot order.  No atomics: bit-reproducible.
// Modified modes (PTM / PTB) run two launches, as k_spectra does: the main one integrates the modified lanes only
// and writes ycell, the F_FB one integrates the separable-fallback lanes (breakdown cells, narrow rapidity windows:
// MomentumSpectra.cpp:863-929) of the cells k_fbwrite lists and adds them to ycell.  With both in one kernel the
// PTM / PTB instances spilled 147 VGPRs at 2 waves per SIMD (5.6e11 B of scratch traffic per config-2 pass).
template <int MODE, int FLAGS, int KJ>
__global__ __launch_bounds__(kBlock, (dndx_waves_f<MODE, FLAGS>())) void k_dndx(DndxArgs A) {
  constexpr bool FB = MODE >= PTM && (FLAGS & F_FB) != 0;   // separable-fallback launch of a modified mode
  constexpr bool MODMAIN = MODE >= PTM && !FB;              // modified launch: separable lanes left to F_FB
  extern __shared__ double smem[];
  constexpr int kTile = dndx_tile<MODE, FLAGS>();         // cells per record tile of this launch
  const int nphp = A.njb * KJ;
  double* s_rec = smem;                                   // [kTile][NREC]
  dbl2* s_trig = (dbl2*)(s_rec + kTile * NREC);           // [nphp] {cos, sin}
  dbl2* s_cs = s_trig + nphp;                             // [nphp] {pT cos, pT sin} of the current pT
  double* s_w = (double*)(s_cs + nphp);                   // [nphp] phi weights (0 in the padding)
  dbl2* s_bp = (dbl2*)(s_w + nphp);                       // [kTile][nphp] {b', Phi} of the current pT
  // (none in the modified launch, which builds only the tables its lanes read: IS3D_MOD_TABLES)
  double* s_qv = (double*)(s_bp + ((MODMAIN && IS3D_MOD_TABLES) ? 0 : kTile * nphp));   // [kTile][nphp] Qv (modified path)
  // the modified launch's rows are {PDm, Qv} pairs with IS3D_DNDX_PDM
  constexpr bool MW = MODMAIN && IS3D_DNDX_PDM && KJ % 4 == 0;
  double* s_red = s_qv + (MW ? 2 : 1) * kTile * nphp;     // [kTile][kBlock] per-lane cell sums
  double* s_grid = s_red + kTile * kBlock;                // y[nk] | eta[nl] | eta_w[nl]
  // y-term rows without the Y_MU2 / Y_MU slots (kYRowLY): two more doubles per row took config 2's Grad
  // launch past the LDS of three workgroups per CU (k_dndx 647 -> 784 ms)
  double* s_y = s_grid + A.nk + 2 * A.nl;                 // [kTile][nq][kYRowLY]
  constexpr int kET = MODMAIN ? kModTabN : kExpTabN;      // the modified lanes' own table (IS3D_MOD_TAB_BITS)
  double* s_etab = s_y + (long)kTile * A.nq * kYRowLY;    // [kET] 2^(j/kET)
  // PTM: the renormalisation factor of the tile's cells for the workgroup's Sl species, loaded once per tile instead of
  // once per pT (the per-pT loads re-read the [cell][class] array 48 times: 7.3e11 B per config-2 pass); one entry
  // per species, not per lane (the lanes of a species share it): 4 KB instead of 16 KB, which takes PTM's launch to
  // the LDS of three workgroups per CU, as PTB's
  double* s_rn = s_etab + kET;                             // [kTile][Sl]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kET; i += kBlock) s_etab[i] = MODMAIN ? kModExp2Tab[i] : kExp2Tab[i];
  const long nwg = (long)A.nbx * A.nchunk;
  const long bid = blockIdx.x, q8 = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
  const long lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int grp = (int)(lid % A.nbx);
  const long ch = lid / A.nbx;
  const int s_l = lane % A.Sl, y_l = lane / A.Sl;
  const int slot = wave * A.Yl + y_l, nslot = 4 * A.Yl;
  const bool active = y_l < A.Yl && grp * A.Sl + s_l < A.npart;
  const int s = active ? grp * A.Sl + s_l : 0;
  const double mass = A.smass[s], m2 = mass * mass, sign = A.ssign[s], baryon = A.sbaryon[s];

  for (int j = tid; j < nphp; j += kBlock) {
    const bool in = j < A.nphi;
    dbl2 v; v.x = in ? A.cphi[j] : 0.0; v.y = in ? A.sphi[j] : 0.0;
    s_trig[j] = v;
    s_w[j] = in ? A.phiw[j] : 0.0;
  }
  for (int i = tid; i < A.nk; i += kBlock) s_grid[i] = (A.dim == 3) ? A.yv[i] : 0.0;
  for (int i = tid; i < A.nl; i += kBlock) {
    s_grid[A.nk + i] = (A.dim == 3) ? 0.0 : A.etav[i];
    s_grid[A.nk + A.nl + i] = (A.dim == 3) ? 1.0 : A.etaw[i];
  }

  // F_FB: positions in the fallback cell list (its length is known on the device only), split evenly
  long c_begin, c_end;
  if constexpr (FB) {
    const long nfb = *A.fbcount, cpw = ((nfb + A.nchunk - 1) / A.nchunk + kTile - 1) / kTile * kTile;
    c_begin = ch * cpw;
    c_end = min(nfb, c_begin + cpw);
  } else {
    c_begin = ch * A.cells_per_wg;
    c_end = min(A.n, c_begin + A.cells_per_wg);
  }
  auto cell_of = [&](long pos) -> long { return FB ? (long)A.fbcells[pos] : pos; };
  for (long cb = c_begin; cb < c_end; cb += kTile) {
    const int nt = (int)min((long)kTile, c_end - cb);
    __syncthreads();                                       // previous tile fully consumed
    for (int i = tid; i < nt * NREC; i += kBlock) s_rec[i] = A.rec[cell_of(cb + i / NREC) * NREC + i % NREC];
#pragma unroll
    for (int t = 0; t < kTile; t++) s_red[t * kBlock + tid] = 0.0;
    if (MODE == PTM) {
      for (int idx = tid; idx < nt * A.Sl; idx += kBlock) {
        const int t = idx / A.Sl, sl = idx % A.Sl, s2 = grp * A.Sl + sl;
        if (s2 < A.npart) s_rn[idx] = A.renorm[cell_of(cb + t) * A.nrcls + A.rcls[s2]];
      }
    }
    __syncthreads();
    for (int idx = tid; idx < nt * A.nq; idx += kBlock) {
      const int t = idx / A.nq, q = idx % A.nq;
      const double* R = s_rec + t * NREC;
      if (R[R_KIND] != 0.0) {
        const int ky = q / A.nl, l = q % A.nl;
        const double y = s_grid[ky];
        const double eta = (A.dim == 3) ? R[R_ETA] : s_grid[A.nk + l];
        const double w = s_grid[A.nk + A.nl + l];
        yterms(MODE, 0, R, y, eta, w, s_y + ((long)t * A.nq + q) * kYRowLY, false, MODMAIN && IS3D_MOD_TABLES);
      }
    }
    for (int ipt = 0; ipt < A.npT; ipt++) {
      const double pT = A.pT[ipt], wpT = A.pTw[ipt];
      const double mT = sqrt(m2 + pT * pT), mT2 = mT * mT, mTb = mT * baryon;
      __syncthreads();                                     // y-terms ready / previous pT's phi-terms consumed
      for (int j = tid; j < nphp; j += kBlock) {
        const dbl2 tr = s_trig[j];
        dbl2 v; v.x = pT * tr.x; v.y = pT * tr.y;
        s_cs[j] = v;
      }
      for (int idx = tid; idx < nt * nphp; idx += kBlock) {
        const int t = idx / nphp, j = idx % nphp;
        const double* R = s_rec + t * NREC;
        dbl2 v; v.x = 0.0; v.y = 0.0;
        double qv = 0.0;
        if (j < A.nphi && R[R_KIND] != 0.0) {
          const dbl2 tr = s_trig[j];
          // the modified launch reads Qv only ({b', Phi} serve the separable lanes of the F_FB launch)
          if constexpr (!(MODMAIN && IS3D_MOD_TABLES)) v = phiterms(MODE, R, pT, tr.x, tr.y, s_etab);
          if (MODE >= PTM && R[R_KIND] == 2.0) {
            dbl2 c; c.x = pT * tr.x; c.y = pT * tr.y;
            qv = modqv(R, c);
          }
        }
        if constexpr (!(MODMAIN && IS3D_MOD_TABLES)) s_bp[t * nphp + j] = v;
        if constexpr (dndx_pd<MODE>() && KJ % 4 == 0) {
          dbl2 c; c.x = pT * s_trig[j].x; c.y = pT * s_trig[j].y;
          s_qv[t * nphp + j] = (j < A.nphi && R[R_KIND] != 0.0) ? sep_pd(R, c, v.x) : 0.0;   // PD rows (sep_pd)
        } else if constexpr (MW) {
          dbl2 m; m.x = 0.0; m.y = qv;
          if (j < A.nphi && R[R_KIND] == 2.0) { dbl2 c; c.x = pT * s_trig[j].x; c.y = pT * s_trig[j].y; m.x = modpdm(R, c); }
          ((dbl2*)s_qv)[t * nphp + j] = m;
        } else if (MODE >= PTM) {
          s_qv[t * nphp + j] = qv;
        }
      }
      __syncthreads();
      if (!active) continue;
      for (int t = 0; t < nt; t++) {
        const double* R = s_rec + t * NREC;
        const double kind = R[R_KIND];
        if (kind == 0.0) continue;
        double rn_abs = R[R_RENORM];
        if (MODE == PTM || MODE == PTB) {
          const double rn = (MODE == PTM) ? s_rn[t * A.Sl + s_l] : R[R_RENORM];
          if (!isfinite(rn)) continue;    // cell skipped for this species (SpacetimeDistribution.cpp:972-976)
          rn_abs = fabs(rn);
        }
        double cell = 0.0;
        for (int task = slot; task < A.ntask; task += nslot) {
          const int kk = task / A.nl, l = task % A.nl;
          const int k = kk % A.nk, jb = kk / A.nk, j0 = jb * KJ;
          const double* Y = s_y + ((long)t * A.nq + k * A.nl + l) * kYRowLY;
          const dbl2* BP = s_bp + t * nphp + j0;
          const dbl2* W = (const dbl2*)(s_w + j0);
          const bool sep = (MODE <= CE) || kind == 1.0 || Y[Y_NARROW] != 0.0;
          if (MODMAIN && sep) continue;
          if (FB && !sep) continue;
          if constexpr (!MODMAIN) {
            SepLane L;
            // Boltzmann-tail lanes of Grad / RTA-CE (decided per wavefront, as in k_spectra)
            // (Grad only: RTA-CE's tail pairs, one 1/E per pair, were slower -- 508 -> 560 ms at config 2 against
            // Grad's 404 -> 333 ms, profiles/round3_r3x_ab_split_dndx_tail.log)
            constexpr bool TL = IS3D_TAIL_DNDX && MODE == GRAD;
            sep_setup(sep_flavor(MODE), R, Y, mT, mT2, m2, mTb, pT, sign, baryon, s_etab, L, TL ? 2 : 0, 0, true);
            if (L.skip) continue;
            constexpr bool PDL = dndx_pd<MODE>() && KJ % 4 == 0;
            const double* PDr = s_qv + t * nphp + j0;
            if constexpr (PDL) {
              if (TL && L.tail) cell += sep_phi_wsum_pd_tail<MODE, FLAGS, KJ>(L, s_cs + j0, BP, PDr, W);
              else if (L.fast) cell += sep_phi_wsum_pd<MODE, FLAGS, KJ>(L, s_cs + j0, BP, PDr, W);
              else cell += sep_phi_wsum<MODE, FLAGS, false, KJ>(L, s_cs + j0, BP, W);
            } else
            if (TL && L.tail) cell += sep_phi_wsum_tail<MODE, FLAGS, KJ>(L, s_cs + j0, BP, W);
            else cell += L.fast ? sep_phi_wsum<MODE, FLAGS, true, KJ>(L, s_cs + j0, BP, W)
                                : sep_phi_wsum<MODE, FLAGS, false, KJ>(L, s_cs + j0, BP, W);
          }
          if constexpr (MODMAIN) {
            ModLane M;
            mod_setup(R, Y, mT, m2, pT, sign, baryon, rn_abs, s_etab, M, false);
            if (M.skip) continue;
            if constexpr (MW) {
              const dbl2* MWr = (const dbl2*)s_qv + t * nphp + j0;
              cell += M.clamp ? mod_phi_wsum_mw<FLAGS, true, KJ>(M, s_cs + j0, MWr, W)
                              : mod_phi_wsum_mw<FLAGS, false, KJ>(M, s_cs + j0, MWr, W);
            } else {
              const dbl2* QV = (const dbl2*)(s_qv + t * nphp + j0);
              cell += M.clamp ? mod_phi_wsum<FLAGS, true, KJ>(M, s_cs + j0, QV, W)
                              : mod_phi_wsum<FLAGS, false, KJ>(M, s_cs + j0, QV, W);
            }
          }
        }
        s_red[t * kBlock + tid] = fma(wpT, cell, s_red[t * kBlock + tid]);
      }
    }
    __syncthreads();
    // per (species, cell): sum of the species' slot columns in slot order (idle slots hold 0)
    for (int idx = tid; idx < A.Sl * nt; idx += kBlock) {
      const int sl = idx % A.Sl, t = idx / A.Sl;
      const int s2 = grp * A.Sl + sl;
      if (s2 >= A.npart) continue;
      double acc = 0.0;
      for (int w = 0; w < 4; w++)
        for (int yl = 0; yl < A.Yl; yl++) acc += s_red[t * kBlock + w * 64 + yl * A.Sl + sl];
      double* y = A.ycell + (long)s2 * A.n + cell_of(cb + t);
      *y = FB ? *y + acc : acc;          // F_FB runs after the main launch on the same stream
    }
  }
}

// F_TS tables of one chunk of cells: per (pT, cell, phi slot) the values k_spectra's F_TB launch builds per tile
// in LDS -- {b', Phi} (phiterms), PD (sep_pd) and RTA-CE's {TE, T2} -- by the same expressions, so the F_TS lanes
// see the same operands.  One thread per entry, phi slot fastest (a cell's row is written by consecutive lanes);
// padding slots and cells with u.dsigma <= 0 get zeros, as in the LDS tables.
template <int MODE>
__global__ __launch_bounds__(256) void k_phitab(PhiTabArgs A) {
  if (gate_closed(A.gate, A.gate_want)) return;
  __shared__ double s_etab[kExpTabN];
  for (int i = threadIdx.x; i < kExpTabN; i += 256) s_etab[i] = kExp2Tab[i];
  __syncthreads();
  const int rw = phitab_row(MODE, A.nphp, A.by != 0);
  const long total = (long)A.npT * A.nc * A.nphp;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int j = (int)(idx % A.nphp);
    const long r = idx / A.nphp, c = r % A.nc;
    const int ipt = (int)(r / A.nc);
    const double* R = A.rec + (A.c0 + c) * NREC;
    double* row = A.tab + ((long)ipt * A.phn + c) * rw;
    const bool in = j < A.nphi;
    const double pT = A.pT[ipt], co = in ? A.cphi[j] : 0.0, sn = in ? A.sphi[j] : 0.0;
    dbl2 cs; cs.x = pT * co; cs.y = pT * sn;
    dbl2 v; v.x = 0.0; v.y = 0.0;
    if (in && R[R_KIND] != 0.0) v = phiterms(MODE, R, pT, co, sn, s_etab);
    row[2 * j] = v.x;
    row[2 * j + 1] = v.y;
    row[2 * A.nphp + j] = sep_pd(R, cs, v.x);
    if constexpr (MODE == CE) {
      row[3 * A.nphp + 2 * j] = -fma(R[R_UX], cs.x, R[R_UY] * cs.y);
      row[3 * A.nphp + 2 * j + 1] = fma(R[R_LC], cs.x, R[R_LS] * cs.y);
    }
    if (A.by) row[(MODE == CE ? 5 : 3) * A.nphp + j] = fma(R[R_SCB], cs.x, R[R_SSB] * cs.y);   // T3 (F_BY)
  }
}

}  // namespace

template <int MODE>
void launch_phitab(hipStream_t st, const PhiTabArgs& a) {
  const long total = (long)a.npT * a.nc * a.nphp;
  const long blocks = std::max(1L, std::min((total + 255) / 256, 256L * 32));
  hipLaunchKernelGGL((k_phitab<MODE>), dim3((unsigned)blocks), dim3(256), 0, st, a);
}

template <int MODE, int KJ>
void launch_spectra_kj(dim3 grid, size_t shmem, hipStream_t st, const SpecArgs& a, int flags) {
  if constexpr (MODE >= PTM) {
    if (flags & F_FB) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 32, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 33, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 34, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 35, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
    if (flags & F_T8) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 16, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 17, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 18, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 19, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  if constexpr (KJ == 8) {
    if (flags & F_LY) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 8, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 9, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 10, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 11, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  if constexpr ((MODE == GRAD || MODE == CE) && (KJ == 24 || KJ == 32)) {
    if (flags & F_MP) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 64, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 65, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 66, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 67, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  if constexpr ((MODE == GRAD || MODE == CE) && (KJ == 24 || KJ == 32)) {
    if ((flags & F_TS) && (flags & F_TB) && (flags & F_BY)) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 388, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 389, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 390, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 391, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
    if ((flags & F_TS) && (flags & F_TB)) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 132, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 133, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 134, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 135, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  if constexpr ((MODE == GRAD || MODE == CE) && KJ % 4 == 0) {
    if (flags & F_TB) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_spectra<MODE, 4, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_spectra<MODE, 5, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_spectra<MODE, 6, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_spectra<MODE, 7, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  switch (flags & 3) {
    case 0: hipLaunchKernelGGL((k_spectra<MODE, 0, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    case 1: hipLaunchKernelGGL((k_spectra<MODE, 1, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    case 2: hipLaunchKernelGGL((k_spectra<MODE, 2, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    default: hipLaunchKernelGGL((k_spectra<MODE, 3, KJ>), grid, dim3(kBlock), shmem, st, a); break;
  }
}

template <int MODE>
void launch_spectra(dim3 grid, size_t shmem, hipStream_t st, const SpecArgs& a, int flags, int kj) {
  switch (kj) {
#ifdef IS3D_KJ16
    case 16: launch_spectra_kj<MODE, 16>(grid, shmem, st, a, flags); break;
#endif
    case 32: launch_spectra_kj<MODE, 32>(grid, shmem, st, a, flags); break;
    case 24: launch_spectra_kj<MODE, 24>(grid, shmem, st, a, flags); break;
    case 8: launch_spectra_kj<MODE, 8>(grid, shmem, st, a, flags); break;
    case 2: launch_spectra_kj<MODE, 2>(grid, shmem, st, a, flags); break;
    default: break;     // no instantiation for this phi block: engine.hip checks kj against spectra_kj_supported
  }
}


template <int MODE, int KJ>
void launch_dndx_kj(dim3 grid, size_t shmem, hipStream_t st, const DndxArgs& a, int flags) {
  if constexpr (MODE >= PTM) {
    if (flags & F_FB) {
      switch (flags & 3) {
        case 0: hipLaunchKernelGGL((k_dndx<MODE, 32, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 1: hipLaunchKernelGGL((k_dndx<MODE, 33, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        case 2: hipLaunchKernelGGL((k_dndx<MODE, 34, KJ>), grid, dim3(kBlock), shmem, st, a); break;
        default: hipLaunchKernelGGL((k_dndx<MODE, 35, KJ>), grid, dim3(kBlock), shmem, st, a); break;
      }
      return;
    }
  }
  switch (flags & 3) {
    case 0: hipLaunchKernelGGL((k_dndx<MODE, 0, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    case 1: hipLaunchKernelGGL((k_dndx<MODE, 1, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    case 2: hipLaunchKernelGGL((k_dndx<MODE, 2, KJ>), grid, dim3(kBlock), shmem, st, a); break;
    default: hipLaunchKernelGGL((k_dndx<MODE, 3, KJ>), grid, dim3(kBlock), shmem, st, a); break;
  }
}

template <int MODE>
void launch_dndx(dim3 grid, size_t shmem, hipStream_t st, const DndxArgs& a, int flags, int kj) {
  switch (kj) {
    case 32: launch_dndx_kj<MODE, 32>(grid, shmem, st, a, flags); break;
    case 24: launch_dndx_kj<MODE, 24>(grid, shmem, st, a, flags); break;
    case 8: launch_dndx_kj<MODE, 8>(grid, shmem, st, a, flags); break;
    default: launch_dndx_kj<MODE, 2>(grid, shmem, st, a, flags); break;
  }
}

#endif  // IS3D_KERNEL_DEFS

}  // namespace kern
}  // namespace is3d
