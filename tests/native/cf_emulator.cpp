#include <cstdlib>
#include <cstdio>
// cf_emulator.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Runs the engine's device math (is3d2_amd/csrc/cf_math.h, aniso_math.h) serially on
// the host, in the same order of operations per lane as k_spectra, so the
// factorised integrand can be checked against the oracle in the CPU test tier.
// It is never linked into the product and is not a fallback: the product path
// (libis3d_amd.so) has no host implementation of the kernels.
#include <cmath>
#include <cstring>
#include <vector>

// the modified path's Boltzmann-tail lanes are compiled in (taken only under variant 16)
#define IS3D_MOD_TAIL 1
#include "../../is3d2_amd/csrc/aniso_math.h"
#include "../../is3d2_amd/csrc/cf_math.h"
#include "../../is3d2_amd/csrc/spline_host.h"
#include "../../oracle/is3d_oracle.h"

using namespace is3d;

// delta-f tables and prepass constants on the host (as finalize_tables / make_consts)
struct EmuTables {
  DfTables tb{};
  PrepConsts k{};
  std::vector<std::vector<double>> sy, sc;
  std::vector<double> jl2, jz, jx, jl2c, jzc;
  EmuTables(const orc_params* p, const orc_setup* su, int op) : sy(NSPL), sc(NSPL) {
    const int mode = p->df_mode, dim = p->dimension;
    tb.df_mode = mode; tb.include_baryon = p->include_baryon;
    tb.nT = su->nT; tb.nmuB = p->include_baryon ? su->nmuB : 1;
    tb.T = su->Tarr; tb.muB = su->muBarr; tb.tab = su->dftab;
    tb.T_min = su->Tarr[0]; tb.muB_min = su->muBarr[0];
    tb.dT = fabs(su->Tarr[1] - su->Tarr[0]);
    tb.dmuB = su->nmuB > 1 ? fabs(su->muBarr[1] - su->muBarr[0]) : 0.0;
    const int col[NSPL] = {0, 2, 3, 5, 7, 8, 9};
    if (!p->include_baryon) {
      for (int i = 0; i < NSPL; i++) {
        const double* yv = su->dftab + (size_t)col[i] * su->nmuB * su->nT;
        sy[i].assign(yv, yv + su->nT);
        cspline_coeffs(su->Tarr, yv, su->nT, sc[i]);
        tb.sy[i] = sy[i].data(); tb.sc[i] = sc[i].data();
      }
    }
    double bpmax = -1.0;
    if (!p->include_baryon && mode == PTB) {
      jonah_table(su->T_avg, su->npdg, su->pdg_mass, su->pdg_degen, su->pdg_sign, su->gla_root + 2 * su->gla_points,
                  su->gla_weight + 2 * su->gla_points, su->gla_points, jl2, jz, jx, bpmax);
      cspline_coeffs(jx.data(), jl2.data(), 301, jl2c);
      cspline_coeffs(jx.data(), jz.data(), 301, jzc);
      tb.nj = 301; tb.jx = jx.data(); tb.jl2 = jl2.data(); tb.jl2c = jl2c.data(); tb.jz = jz.data(); tb.jzc = jzc.data();
    }
    tb.bulk_over_P_max = bpmax;
    k.operation = op;
    k.df_mode = mode; k.dim = dim; k.include_baryon = p->include_baryon; k.include_bulk = p->include_bulk_deltaf;
    k.include_shear = p->include_shear_deltaf; k.include_diff = p->include_baryondiff_deltaf;
    k.deta_min = p->deta_min; k.mass_pion0 = p->mass_pion0; k.gla_pts = su->gla_points;
    k.gla_r1 = su->gla_root + su->gla_points; k.gla_r2 = su->gla_root + 2 * su->gla_points;
    k.gla_w1 = su->gla_weight + su->gla_points; k.gla_w2 = su->gla_weight + 2 * su->gla_points;
    k.two_pi2_hbarC3 = 2.0 * pow(M_PI, 2) * pow(kHbarC, 3);
  }
};

// op = 1: out = dN/(pT dpT dphi dy)[species][pT][phi][y];  op = 0: out = dN_dy_cell[species][cell]
// (sum over pT, phi, y of w_pT w_phi (w_eta p.dsigma f) x prefactor g, as k_dndx)
// variant bits (k_spectra's launch variants, checked on the CPU): 1 = the F_TB table algebra for Grad /
// RTA-CE fast lanes without baryon terms (sep_quad_tb_t, phi counts that are multiples of 4), 2 = the
// Boltzmann-tail lanes (sep_setup allow_tail + sep_quad_tb_tail_t under bit 1),
// 4 = the modified path's table form (mod_quad_tab_t / mod_pair_tab_t), 8 = PTMA Newton sums over hadrons
// merged by identical (mass, sign) with summed degeneracies, first-occurrence order (engine.hip
// finalize_tables, IS3D_ANISO_MERGE); without it the sums run per hadron in PDG order as the reference
// optional lane census of the separable lanes (tools/lane_census.py): [pT][3] counts of skipped, Boltzmann-tail
// and other lanes per (cell, species, q)
static long* g_census = nullptr;
extern "C" void emu_set_census(long* counts) { g_census = counts; }
// optional per-lane record (tools/lane_census.py --waves): [pT][cell][species][q] = 1 + (skip 0 / tail 1 / other 2)
static signed char* g_census_lane = nullptr;
// optional census of the modified (non-separable) lanes: counts of skipped, clamped, Boltzmann-tail and other lanes
static long* g_census_mod = nullptr;
extern "C" void emu_set_census_mod(long* counts) { g_census_mod = counts; }
extern "C" void emu_set_census_lanes(signed char* buf) { g_census_lane = buf; }
// optional per-lane margin of the modified table lanes (tools/mod_census.py), same indexing as g_census_lane
static unsigned char* g_census_margin = nullptr;
extern "C" void emu_set_census_margin(unsigned char* buf) { g_census_margin = buf; }
// lanes whose smallest exponent exceeds g_near_x (not tail) are recorded as 4 (tools/lane_census.py --near)
static double g_near_x = 1e300;
// optional check of sep_slow_cell (k_prep's per-cell bound, engine.hip launch_end): [0] separable lanes off the fast
// path (smallest exponent below kExpFast), [1] such lanes in cells the bound did NOT flag (must stay 0), [2] cells
// flagged, [3] live cells, [4] (as double bits) the smallest lane exponent x - zb seen in an unflagged cell
static long* g_slow_check = nullptr;
extern "C" void emu_set_slow_check(long* out) { g_slow_check = out; }
extern "C" void emu_set_near_x(double x) { g_near_x = x; }

extern "C" int emu_spectra_v(const orc_params* p, const orc_setup* su, const orc_surface* S, int chains, int op,
                             double* out, long* stats, int variant) {
  const int mode = p->df_mode, dim = p->dimension;
  const long n = S->n;
  const int np = su->npart, npT = su->npT, nphi = su->nphi;
  const int ny_out = (dim == 3) ? su->ny : 1, nk = ny_out, nl = (dim == 3) ? 1 : su->neta;
  EmuTables et(p, su, op);
  const DfTables& tb = et.tb;
  const PrepConsts& k = et.k;
  // --- prepass
  std::vector<double> rec((size_t)n * NREC), aux((size_t)n * 9), sol((size_t)n * 6);
  const double* fields[NSURF] = {S->tau, S->x, S->y, S->eta, S->dat, S->dax, S->day, S->dan, S->ux, S->uy, S->un,
                                 S->E, S->T, S->P, S->pixx, S->pixy, S->pixn, S->piyy, S->piyn, S->bulkPi,
                                 S->muB, S->nB, S->Vx, S->Vy, S->Vn};
  long st_break = 0, st_pl = 0, st_fail = 0, st_it = 0;
  for (long c = 0; c < n; c++) {
    double s[NSURF];
    for (int f = 0; f < NSURF; f++) s[f] = fields[f] ? fields[f][c] : 0.0;
    double* R = &rec[(size_t)c * NREC];
    int err = 0;
    if (mode <= CE) err = prep_grad_ce(k, tb, s, R);
    else if (mode <= PTB) {
      int flags[2];
      err = prep_feqmod(k, tb, s, R, &aux[(size_t)c * 9], flags);
      if (!err) { st_break += (flags[0] && R[R_KIND] != 0.0); st_pl += flags[1]; }
    } else prep_famod_a(k, s, R, &aux[(size_t)c * 9]);
    if (err) return 100 + err;
    if (R[R_KIND] != 0.0) sep_cell_consts(mode, R);
  }
  if (mode == PTMA) {
    const int nh = su->npdg < 320 ? su->npdg : 320;
    std::vector<double> am, as, ag;
    for (int i = 0; i < nh; i++) {
      int u = -1;
      if (variant & 8)
        for (size_t v = 0; v < am.size(); v++)
          if (am[v] == su->pdg_mass[i] && as[v] == su->pdg_sign[i]) { u = (int)v; break; }
      if (u < 0) { am.push_back(su->pdg_mass[i]); as.push_back(su->pdg_sign[i]); ag.push_back(su->pdg_degen[i]); }
      else ag[u] += su->pdg_degen[i];
    }
    Hadrons h{(int)am.size(), am.data(), as.data(), ag.data()};
    const double fp2 = 4.0 * pow(M_PI, 2) * pow(kHbarC, 3);
    auto id = [](double v) { return v; };
    const long C = (chains > 0) ? (chains < n ? chains : n) : n;
    for (long ch = 0; ch < C; ch++) {
      double state[4] = {0, 0, 0, 0};
      long cnt[3] = {0, 0, 0};
      for (long c = ch; c < n; c += C) {
        if (rec[(size_t)c * NREC + R_KIND] == 0.0) continue;
        aniso_cell(&aux[(size_t)c * 9], h, 0, 1, id, fp2, state, &sol[(size_t)c * 6], cnt);
      }
      st_pl += cnt[0]; st_fail += cnt[1]; st_it += cnt[2];
    }
    for (long c = 0; c < n; c++) {
      double* R = &rec[(size_t)c * NREC];
      if (R[R_KIND] == 0.0) continue;
      int broken = 0;
      prep_famod_b(k, R, &aux[(size_t)c * 9], &sol[(size_t)c * 6], &broken);
      st_break += broken;
    }
  }
  std::vector<char> slow_cell;
  double slow_min_ok = 1e300;
  if (g_slow_check && mode <= CE) {
    double pmax = 0.0, bmax = 0.0;
    for (int i = 0; i < npT; i++) pmax = fmax(pmax, su->pT[i]);
    for (int s2 = 0; s2 < np; s2++) bmax = fmax(bmax, fabs(su->baryon[s2]));
    slow_cell.assign(n, 0);
    for (long c = 0; c < n; c++) {
      const double* R = &rec[(size_t)c * NREC];
      if (R[R_KIND] == 0.0) continue;
      g_slow_check[3]++;
      slow_cell[c] = sep_slow_cell(R, pmax, bmax) ? 1 : 0;
      g_slow_check[2] += slow_cell[c];
    }
  }
  // --- spectra (same per-lane order as k_spectra: cells ascending, then l, then phi)
  const double prefactor = pow(2.0 * M_PI * kHbarC, -3);
  std::vector<double> cph(nphi), sph(nphi);
  for (int j = 0; j < nphi; j++) { cph[j] = cos(su->phi[j]); sph[j] = sin(su->phi[j]); }
  const int nq = nk * nl;
  std::vector<double> Yall((size_t)nq * NYT);
  std::vector<dbl2> CS(nphi), BP(nphi);
  std::vector<double> QV(nphi + 1);
  std::vector<dbl2> PE(nphi), PTq((size_t)nq * nphi);
  const bool use_tb = (variant & 1) && op != 0 && mode <= CE && !p->include_baryon && nphi % 4 == 0;
  const bool tail = (variant & 2) != 0;
  std::vector<double> acc((size_t)np * nk * nphi);
  for (int i = 0; i < npT; i++) {
    const double pT = su->pT[i];
    std::fill(acc.begin(), acc.end(), 0.0);
    for (long c = 0; c < n; c++) {
      const double* R = &rec[(size_t)c * NREC];
      const double kind = R[R_KIND];
      if (kind == 0.0) continue;
      for (int j = 0; j < nphi; j++) {
        CS[j].x = pT * cph[j]; CS[j].y = pT * sph[j];
        BP[j] = phiterms(mode, R, pT, cph[j], sph[j], kExp2Tab);
        QV[j] = (mode >= PTM && kind == 2.0) ? modqv(R, CS[j]) : 0.0;
      }
      for (int q = 0; q < nq; q++) {
        const int kk = q / nl, l = q % nl;
        const double y = (dim == 3) ? su->y[kk] : 0.0;
        const double eta = (dim == 3) ? R[R_ETA] : su->eta[l];
        const double w = (dim == 3) ? 1.0 : su->eta_w[l];
        yterms(mode, op, R, y, eta, w, &Yall[(size_t)q * NYT]);
        if (use_tb) {   // k_spectra's {PD, T1} rows
          const double* Yq = &Yall[(size_t)q * NYT];
          for (int j = 0; j < nphi; j++) {
            PTq[(size_t)q * nphi + j].x = sep_pd(R, CS[j], BP[j].x);
            PTq[(size_t)q * nphi + j].y = fma(Yq[Y_SC1], CS[j].x, Yq[Y_SS1] * CS[j].y);
          }
        }
      }
      if ((use_tb || (variant & 64)) && mode == CE)   // {TE, T2} (F_TB launch; variant 64: the per-lane launch's)
        for (int j = 0; j < nphi; j++) {
          PE[j].x = -fma(R[R_UX], CS[j].x, R[R_UY] * CS[j].y);
          PE[j].y = fma(R[R_LC], CS[j].x, R[R_LS] * CS[j].y);
        }
      if (op == 0) std::fill(acc.begin(), acc.end(), 0.0);
      for (int s = 0; s < np; s++) {
        const double mass = su->mass[s], m2 = mass * mass, sign = su->sign[s], baryon = su->baryon[s];
        const double mT = sqrt(m2 + pT * pT);
        double rn_abs = R[R_RENORM];
        if (mode == PTM || mode == PTB) {
          const double rn = (mode == PTM) ? ptm_renorm(k, &aux[(size_t)c * 9], mass, sign, su->degen[s], baryon) : R[R_RENORM];
          if (!std::isfinite(rn)) continue;
          rn_abs = fabs(rn);
        }
        for (int kk = 0; kk < nk; kk++) {
          double* a = &acc[((size_t)s * nk + kk) * nphi];
          for (int l = 0; l < nl; l++) {
            const double* Y = &Yall[(size_t)(kk * nl + l) * NYT];
            const bool sep = (mode <= CE) || kind == 1.0 || Y[Y_NARROW] != 0.0;
            if (sep) {
              SepLane L;
              // tail lanes: the F_TB fours, or k_spectra's per-lane PD-table fours (Grad / RTA-CE, phi blocks of fours)
              // (operation 0: k_dndx's tail pairs, any phi block)
              const bool pd_tail = tail && !use_tb && mode <= CE && (op == 0 || spectra_kj(nphi) % 4 == 0);
              // near-tail lanes: the F_TS Grad launch without regulate (sep_quad_tb_near_t)
              const bool near = use_tb && tail && mode == GRAD && !p->regulate_deltaf;
              sep_setup(sep_flavor(mode), R, Y, mT, mT * mT, m2, mT * baryon, pT, sign, baryon, kExp2Tab, L,
                        (use_tb || pd_tail) && tail, near);
              if (g_census) g_census[i * 3 + (L.skip ? 0 : (L.tail ? 1 : 2))]++;
              if (!slow_cell.empty() && !L.skip) {
                if (!L.fast) { g_slow_check[0]++; if (!slow_cell[c]) g_slow_check[1]++; }
                if (!slow_cell[c]) slow_min_ok = fmin(slow_min_ok, L.x - pT * R[R_ZB]);
              }
              if (g_census_lane)
                g_census_lane[(((size_t)i * n + c) * np + s) * nq + kk * nl + l] =
                    (signed char)(1 + (L.skip ? 0 : (L.tail ? 1 : (L.near || L.x - pT * R[R_ZB] > g_near_x ? 3 : 2))));
              if (L.skip) continue;
              if (use_tb && L.fast) {   // k_spectra's F_TB fours (normal or Boltzmann-tail lanes)
                const dbl2* PT = &PTq[(size_t)(kk * nl + l) * nphi];
                for (int j4 = 0; j4 < nphi; j4 += 4) {
                  const int rg = p->regulate_deltaf, of = p->outflow;
                  if (L.near) {
                    if (of) sep_quad_tb_near_t<true>(L, mT, &BP[j4], &PT[j4], &a[j4]);
                    else sep_quad_tb_near_t<false>(L, mT, &BP[j4], &PT[j4], &a[j4]);
                  } else if (L.tail) {
#define EMU_TAIL(FLV, RG, OF) sep_quad_tb_tail_t<FLV, RG, OF>(L, mT, &BP[j4], &PT[j4], &PE[j4], &a[j4])
                    if (mode == GRAD) { if (rg) { if (of) EMU_TAIL(SEP_GRAD, true, true); else EMU_TAIL(SEP_GRAD, true, false); }
                                        else { if (of) EMU_TAIL(SEP_GRAD, false, true); else EMU_TAIL(SEP_GRAD, false, false); } }
                    else { if (rg) { if (of) EMU_TAIL(SEP_CE, true, true); else EMU_TAIL(SEP_CE, true, false); }
                           else { if (of) EMU_TAIL(SEP_CE, false, true); else EMU_TAIL(SEP_CE, false, false); } }
#undef EMU_TAIL
                  } else {
                    double v[4];
#define EMU_TB(FLV, RG, OF) sep_quad_tb_t<FLV, RG, OF>(L, mT, &BP[j4], &PT[j4], &PE[j4], v)
                    if (mode == GRAD) { if (rg) { if (of) EMU_TB(SEP_GRAD, true, true); else EMU_TB(SEP_GRAD, true, false); }
                                        else { if (of) EMU_TB(SEP_GRAD, false, true); else EMU_TB(SEP_GRAD, false, false); } }
                    else { if (rg) { if (of) EMU_TB(SEP_CE, true, true); else EMU_TB(SEP_CE, true, false); }
                           else { if (of) EMU_TB(SEP_CE, false, true); else EMU_TB(SEP_CE, false, false); } }
#undef EMU_TB
                    for (int i = 0; i < 4; i++) a[j4 + i] += v[i];
                  }
                }
                continue;
              }
              // k_dndx's tail pairs (phi rows padded to even length); variant 32: the same pairs for operation 1, whose
              // per-y outputs show the pair arithmetic (in operation 0 the tail lanes' share of a cell yield is ~e^-24)
              if (L.fast && L.tail && (op == 0 || (variant & 32))) {
                const int rg = p->regulate_deltaf, of = p->outflow;
                for (int j2 = 0; j2 < nphi; j2 += 2) {
                  dbl2 z; z.x = 0.0; z.y = 0.0;
                  const dbl2 c1 = (j2 + 1 < nphi) ? CS[j2 + 1] : z, b1 = (j2 + 1 < nphi) ? BP[j2 + 1] : z;
                  double v0, v1;
#define EMU_PRT(FLV, RG, OF) sep_pair_tail_t<FLV, RG, OF>(L, CS[j2], BP[j2], c1, b1, v0, v1)
                  if (mode == GRAD) { if (rg) { if (of) EMU_PRT(SEP_GRAD, true, true); else EMU_PRT(SEP_GRAD, true, false); }
                                      else { if (of) EMU_PRT(SEP_GRAD, false, true); else EMU_PRT(SEP_GRAD, false, false); } }
                  else { if (rg) { if (of) EMU_PRT(SEP_CE, true, true); else EMU_PRT(SEP_CE, true, false); }
                         else { if (of) EMU_PRT(SEP_CE, false, true); else EMU_PRT(SEP_CE, false, false); } }
#undef EMU_PRT
                  a[j2] += v0;
                  if (j2 + 1 < nphi) a[j2 + 1] += v1;
                }
                continue;
              }
              // variant 64: the per-lane RTA-CE launch's fours with the {TE, T2} table (sep_quad_pde_t), tail or not
              if (L.fast && (variant & 64) && op != 0 && !use_tb && mode == CE && spectra_kj(nphi) % 4 == 0) {
                const int rg = p->regulate_deltaf, of = p->outflow;
                for (int j4 = 0; j4 < nphi; j4 += 4) {
                  dbl2 c4[4], b4[4], e4[4];
                  double P[4], a4[4];
                  for (int i = 0; i < 4; i++) {
                    const int jj = j4 + i;
                    const bool in = jj < nphi;
                    dbl2 z; z.x = 0.0; z.y = 0.0;
                    c4[i] = in ? CS[jj] : z; b4[i] = in ? BP[jj] : z; e4[i] = in ? PE[jj] : z;
                    P[i] = in ? sep_pd(R, CS[jj], BP[jj].x) : 0.0;
                    a4[i] = in ? a[jj] : 0.0;
                  }
#define EMU_PDE(RG, OF) (L.tail ? sep_quad_pde_t<RG, OF, true>(L, c4, b4, P, e4, a4) : sep_quad_pde_t<RG, OF, false>(L, c4, b4, P, e4, a4))
                  if (rg) { if (of) EMU_PDE(true, true); else EMU_PDE(true, false); }
                  else { if (of) EMU_PDE(false, true); else EMU_PDE(false, false); }
#undef EMU_PDE
                  for (int i = 0; i < 4 && j4 + i < nphi; i++) a[j4 + i] = a4[i];
                }
                continue;
              }
              if (L.fast && L.tail) {   // pd_tail: k_spectra's per-lane Boltzmann-tail fours over the padded phi row
                const int rg = p->regulate_deltaf, of = p->outflow;
                for (int j4 = 0; j4 < nphi; j4 += 4) {
                  dbl2 c4[4], b4[4];
                  double P[4], a4[4];
                  for (int i = 0; i < 4; i++) {
                    const int jj = j4 + i;
                    const bool in = jj < nphi;
                    c4[i].x = in ? CS[jj].x : 0.0; c4[i].y = in ? CS[jj].y : 0.0;
                    b4[i].x = in ? BP[jj].x : 0.0; b4[i].y = in ? BP[jj].y : 0.0;
                    P[i] = in ? sep_pd(R, CS[jj], BP[jj].x) : 0.0;
                    a4[i] = in ? a[jj] : 0.0;
                  }
#define EMU_PDT(FLV, RG, OF) sep_quad_pd_tail_t<FLV, RG, OF>(L, c4, b4, P, a4)
                  if (mode == GRAD) { if (rg) { if (of) EMU_PDT(SEP_GRAD, true, true); else EMU_PDT(SEP_GRAD, true, false); }
                                      else { if (of) EMU_PDT(SEP_GRAD, false, true); else EMU_PDT(SEP_GRAD, false, false); } }
                  else { if (rg) { if (of) EMU_PDT(SEP_CE, true, true); else EMU_PDT(SEP_CE, true, false); }
                         else { if (of) EMU_PDT(SEP_CE, false, true); else EMU_PDT(SEP_CE, false, false); } }
#undef EMU_PDT
                  for (int i = 0; i < 4 && j4 + i < nphi; i++) a[j4 + i] = a4[i];
                }
                continue;
              }
              // same arithmetic as k_spectra: fast lanes evaluate phi points in fours (phi blocks that
              // are multiples of 4) or pairs sharing one reciprocal (an odd tail point alone)
              int j = 0;
              if (L.fast) {
                // k_spectra's PD-table fours (Grad / RTA-CE)
                const bool pd = op != 0 && mode <= CE && spectra_kj(nphi) % 4 == 0;
                if (op != 0 && sep_quads(mode, spectra_kj(nphi)))   // k_spectra; k_dndx pairs
                  for (; j + 3 < nphi; j += 4) {
                    double v[4];
                    if (pd) {
                      double P[4];
                      for (int i = 0; i < 4; i++) P[i] = sep_pd(R, CS[j + i], BP[j + i].x);
                      sep_quad_pd(sep_flavor(mode), L, &CS[j], &BP[j], P, p->regulate_deltaf, p->outflow, v);
                    } else {
                      sep_quad(sep_flavor(mode), L, &CS[j], &BP[j], p->regulate_deltaf, p->outflow, v);
                    }
                    for (int i = 0; i < 4; i++) a[j + i] += v[i];
                  }
                for (; j + 1 < nphi; j += 2) {
                  double v0, v1;
                  sep_pair(sep_flavor(mode), L, CS[j], BP[j], CS[j + 1], BP[j + 1], p->regulate_deltaf, p->outflow, v0, v1);
                  a[j] += v0; a[j + 1] += v1;
                }
              }
              for (; j < nphi; j++)
                a[j] += sep_point(sep_flavor(mode), L, CS[j], BP[j], p->regulate_deltaf, p->outflow);
            } else {
              ModLane M;
              // variant 16 (with 4): k_spectra's Boltzmann-tail table lanes (IS3D_MOD_TAIL builds; per lane here)
              const bool mtail = (variant & 20) == 20 && op != 0 && nphi % 4 == 0;
              // k_spectra's table lanes (variant 4) take the exact range of a wide lane's points (IS3D_MOD_EXACT)
              std::vector<dbl2> MW(nphi);
              std::vector<double> MT(nphi);
              if ((variant & 4) && op != 0) {
                for (int jj = 0; jj < nphi; jj++) {
                  MW[jj].x = modpdm(R, CS[jj]); MW[jj].y = QV[jj];
                  MT[jj] = modt2(R, Y, CS[jj]);
                }
                mod_setup<-1>(R, Y, mT, m2, pT, sign, baryon, rn_abs, kModExp2Tab, M, true, mtail, MW.data(), MT.data(), nphi);
              } else {
                mod_setup(R, Y, mT, m2, pT, sign, baryon, rn_abs, kModExp2Tab, M, true, mtail);
              }
              if (g_census_mod) g_census_mod[M.skip ? 0 : M.clamp ? 1 : M.tail ? 2 : 3]++;
              if (g_census_mod && g_census_lane)
                g_census_lane[(((size_t)i * n + c) * np + s) * nq + kk * nl + l] =
                    (signed char)(11 + (M.skip ? 0 : M.clamp ? 1 : M.tail ? 2 : 3));
              // margin record (tools/mod_census.py): binades between the lane's smallest E = e^x 2^-k and |s| =
              // e^chem 2^-k, i.e. k - chem log2(e), clipped to [0, 120]; 255 for skipped / clamped lanes
              if (g_census_mod && g_census_margin) {
                const double kk2 = (6755399441055744.0 - M.shiftk) / kModTabN;
                const double mg = M.tail ? 120.0 : (kk2 - M.chemm * 1.4426950408889634);
                g_census_margin[(((size_t)i * n + c) * np + s) * nq + kk * nl + l] =
                    (M.skip || M.clamp) ? 255 : (unsigned char)std::max(0.0, std::min(120.0, std::floor(mg)));
              }
              if (M.skip) continue;
              int j = 0;
              if ((variant & 4) && op != 0) {   // k_spectra's table form: {PDm, Qv} and T2 rows (MW, MT above)
                const bool of = p->outflow != 0;
                if (g_census_mod && M.clamp && getenv("EMU_SPAN")) {
                  double xmn = 1e300, xmx = 0;
                  for (int jj = 0; jj < nphi; jj++) { double X = fma(M.mT, MT[jj], M.E0 + MW[jj].y); xmn = fmin(xmn, sqrt(X)); xmx = fmax(xmx, sqrt(X)); }
                  printf("SPAN %g %g %g chem %g\n", xmn / kModTabN, xmx / kModTabN, (xmx - xmn) / kModTabN, M.chemm);
                }
                if (spectra_kj(nphi) % 4 == 0)
                  for (; j + 3 < nphi; j += 4) {
                    if (M.tail) { if (of) mod_quad_tab_tail_t<true>(M, &MW[j], &MT[j], &a[j]); else mod_quad_tab_tail_t<false>(M, &MW[j], &MT[j], &a[j]); }
                    else if (M.clamp) { if (of) mod_quad_tab_t<true, true>(M, &MW[j], &MT[j], &a[j]); else mod_quad_tab_t<false, true>(M, &MW[j], &MT[j], &a[j]); }
                    else { if (of) mod_quad_tab_t<true, false>(M, &MW[j], &MT[j], &a[j]); else mod_quad_tab_t<false, false>(M, &MW[j], &MT[j], &a[j]); }
                  }
                for (; j + 1 < nphi; j += 2) {
                  double v0, v1;
                  if (M.clamp) { if (of) mod_pair_tab_t<true, true>(M, MW[j], MW[j + 1], MT[j], MT[j + 1], v0, v1); else mod_pair_tab_t<false, true>(M, MW[j], MW[j + 1], MT[j], MT[j + 1], v0, v1); }
                  else { if (of) mod_pair_tab_t<true, false>(M, MW[j], MW[j + 1], MT[j], MT[j + 1], v0, v1); else mod_pair_tab_t<false, false>(M, MW[j], MW[j + 1], MT[j], MT[j + 1], v0, v1); }
                  a[j] += v0; a[j + 1] += v1;
                }
                // an odd last point: k_spectra pads the phi row (zero {PDm, Qv, T2} rows contribute 0)
                if (j < nphi) {
                  dbl2 z; z.x = 0.0; z.y = 0.0;
                  double v0, v1;
                  if (M.clamp) mod_pair_tab_t<false, true>(M, MW[j], z, MT[j], 0.0, v0, v1);
                  else mod_pair_tab_t<false, false>(M, MW[j], z, MT[j], 0.0, v0, v1);
                  if (of && fma(M.Dw, MW[j].x, M.D0) <= 0.0) v0 = 0.0;
                  a[j] += v0;
                  j++;
                }
              }
              if (op != 0 && spectra_kj(nphi) % 4 == 0)       // k_spectra's fours; k_dndx pairs
                for (; j + 3 < nphi; j += 4) {
                  double v[4];
                  dbl2 qa, qb; qa.x = QV[j]; qa.y = QV[j + 1]; qb.x = QV[j + 2]; qb.y = QV[j + 3];
                  mod_quad(M, &CS[j], qa, qb, p->outflow, v);
                  for (int i = 0; i < 4; i++) a[j + i] += v[i];
                }
              for (; j + 1 < nphi; j += 2) {
                double v0, v1;
                dbl2 q; q.x = QV[j]; q.y = QV[j + 1];
                mod_pair(M, CS[j], CS[j + 1], q, p->outflow, v0, v1);
                a[j] += v0; a[j + 1] += v1;
              }
              for (; j < nphi; j++) a[j] += mod_point(M, CS[j], QV[j], p->outflow);
            }
          }
        }
      }
      if (op == 0) {   // fold this cell's points with the pT / phi weights (k_dndx order: phi, then y, then pT)
        for (int s = 0; s < np; s++) {
          double cell = 0.0;
          for (int kk = 0; kk < nk; kk++) {
            double sj = 0.0;
            for (int j = 0; j < nphi; j++) sj += su->phi_w[j] * acc[((size_t)s * nk + kk) * nphi + j];
            cell += sj;
          }
          out[(size_t)s * n + c] += su->pT_w[i] * cell;
        }
      }
    }
    if (op != 0) {
      for (int s = 0; s < np; s++)
        for (int kk = 0; kk < nk; kk++)
          for (int j = 0; j < nphi; j++)
            out[(((size_t)s * npT + i) * nphi + j) * ny_out + kk] = prefactor * su->degen[s] * acc[((size_t)s * nk + kk) * nphi + j];
    }
  }
  if (op == 0) {
    for (int s = 0; s < np; s++)
      for (long c = 0; c < n; c++) out[(size_t)s * n + c] *= prefactor * su->degen[s];
  }
  if (stats) { stats[0] = st_break; stats[1] = st_pl; stats[2] = st_fail; stats[3] = st_it; }
  if (g_slow_check) std::memcpy(&g_slow_check[4], &slow_min_ok, sizeof(double));
  return 0;
}

extern "C" int emu_spectra(const orc_params* p, const orc_setup* su, const orc_surface* S, int chains, int op,
                           double* out, long* stats) {
  return emu_spectra_v(p, su, S, chains, op, out, stats, 0);
}

// the device exp used by the spectra kernel (exp_dom690 / exp_clamped), evaluated on the host
extern "C" void emu_exp(const double* x, long n, double* out) {
  const ExpCoef E = exp_coef();
  for (long i = 0; i < n; i++) out[i] = exp_clamped(E, x[i]);
}

// the y-terms' sinh / cosh (sinh_cosh)
extern "C" void emu_sinh_cosh(const double* x, long n, double* sh, double* ch) {
  for (long i = 0; i < n; i++) sinh_cosh(x[i], sh + i, ch + i);
}

// PTB Jonah table from the cf_math.h pieces, serially (the device builds it in parallel, same order)
extern "C" void emu_jonah_table(const orc_setup* su, double* l2, double* z, double* bp, double* bpmax) {
  std::vector<double> a, b, c;
  jonah_table(su->T_avg, su->npdg, su->pdg_mass, su->pdg_degen, su->pdg_sign, su->gla_root + 2 * su->gla_points,
              su->gla_weight + 2 * su->gla_points, su->gla_points, a, b, c, *bpmax);
  for (int i = 0; i < kJonahN; i++) { l2[i] = a[i]; z[i] = b[i]; bp[i] = c[i]; }
}

// the modified path's table exp (exp_tab) on x: the caller's scaling x 64/ln2 included
extern "C" int emu_exp_tab_n() { return kExpTabN; }

extern "C" void emu_exp_tab(const double* x, long n, double* out) {
  const ExpTabCoef E = exp_tab_coef();
  for (long i = 0; i < n; i++) out[i] = exp_tab(E, kExp2Tab, x[i] * kInvLn2xN);
}

// operation 2 yield estimate with the device math (k_densities + k_yield, sequential sums)
extern "C" int emu_total_yield(const orc_params* p, const orc_setup* su, const orc_surface* S, const double* plasma,
                               double y_cut, double* n_total, double* dens) {
  EmuTables et(p, su, 1);
  const int np = su->npart, pts = su->gla_points;
  DfCoef df;
  int err = df_eval(et.tb, plasma[0], plasma[3], plasma[1], plasma[2], 0.0, df);
  if (err) return 100 + err;
  static const int kAlpha[6] = {1, 1, 1, 2, 3, 3};
  double dsum[3] = {0, 0, 0};
  for (int s = 0; s < np; s++) {
    const double T = plasma[0], mbar = su->mass[s] / T, chem = su->baryon[s] * (plasma[3] / T);
    double J[6];
    for (int q = 0; q < 6; q++) {
      double v = 0.0;
      for (int i = 0; i < pts; i++) {
        const long o = (long)kAlpha[q] * pts + i;
        v += su->gla_weight[o] * gt_term(q, su->gla_root[o], mbar, chem, su->sign[s]);
      }
      J[q] = v;
    }
    double d3[3];
    species_densities(p->df_mode, df, T, plasma[4] / (plasma[1] + plasma[2]), su->mass[s], su->degen[s], su->baryon[s],
                      J, et.k.two_pi2_hbarC3, d3);
    for (int i = 0; i < 3; i++) { dens[(long)i * np + s] = d3[i]; }
  }
  for (int i = 0; i < 3; i++) for (int s = 0; s < np; s++) dsum[i] += dens[(long)i * np + s];
  const double* fields[NSURF] = {S->tau, S->x, S->y, S->eta, S->dat, S->dax, S->day, S->dan, S->ux, S->uy, S->un,
                                 S->E, S->T, S->P, S->pixx, S->pixy, S->pixn, S->piyy, S->piyn, S->bulkPi,
                                 S->muB, S->nB, S->Vx, S->Vy, S->Vn};
  double Ntot = 0.0;
  for (long c = 0; c < S->n; c++) {
    double sv[NSURF];
    for (int f = 0; f < NSURF; f++) sv[f] = fields[f] ? fields[f][c] : 0.0;
    double v;
    err = yield_cell(et.k, et.tb, sv, dsum, &v);
    if (err) return 100 + err;
    Ntot += v;
  }
  if (p->dimension == 2) Ntot *= 2.0 * y_cut;
  *n_total = Ntot;
  return 0;
}

// PTMA warm-start chain (one chain, MomentumSpectra.cpp:1308-1364) solved by parallel sweeps: sweep 0 solves
// every cell from its cold start, sweep m solves cell i from the chain state sweep m - 1 left after cell i - 1.
// The serial chain is the recurrence's unique fixed point, so once a sweep changes nothing the sweeps equal
// the serial solve bit for bit.  changed[m] = cells whose chain state after sweep m differs (bitwise) from
// sweep m - 1; wrong[m] = cells whose output differs from the serial chain's.  Returns the sweeps run.
extern "C" int emu_chain_sweeps(const orc_params* p, const orc_setup* su, const orc_surface* S, int max_sweeps,
                                long* changed, long* wrong) {
  const long n = S->n;
  EmuTables et(p, su, 1);
  const PrepConsts& k = et.k;
  std::vector<double> rec((size_t)n * NREC), aux((size_t)n * 9);
  const double* fields[NSURF] = {S->tau, S->x, S->y, S->eta, S->dat, S->dax, S->day, S->dan, S->ux, S->uy, S->un,
                                 S->E, S->T, S->P, S->pixx, S->pixy, S->pixn, S->piyy, S->piyn, S->bulkPi,
                                 S->muB, S->nB, S->Vx, S->Vy, S->Vn};
  for (long c = 0; c < n; c++) {
    double s[NSURF];
    for (int f = 0; f < NSURF; f++) s[f] = fields[f] ? fields[f][c] : 0.0;
    prep_famod_a(k, s, &rec[(size_t)c * NREC], &aux[(size_t)c * 9]);
  }
  const int nh = su->npdg < 320 ? su->npdg : 320;
  std::vector<double> am, as, ag;
  for (int i = 0; i < nh; i++) {
    int u = -1;
    for (size_t v = 0; v < am.size(); v++)
      if (am[v] == su->pdg_mass[i] && as[v] == su->pdg_sign[i]) { u = (int)v; break; }
    if (u < 0) { am.push_back(su->pdg_mass[i]); as.push_back(su->pdg_sign[i]); ag.push_back(su->pdg_degen[i]); }
    else ag[u] += su->pdg_degen[i];
  }
  Hadrons h{(int)am.size(), am.data(), as.data(), ag.data()};
  const double fp2 = 4.0 * pow(M_PI, 2) * pow(kHbarC, 3);
  auto id = [](double v) { return v; };
  // serial reference: state after each cell
  std::vector<double> sst((size_t)n * 4), sout((size_t)n * 6);
  {
    double state[4] = {0, 0, 0, 0};
    long cnt[3] = {0, 0, 0};
    for (long c = 0; c < n; c++) {
      if (rec[(size_t)c * NREC + R_KIND] != 0.0) aniso_cell(&aux[(size_t)c * 9], h, 0, 1, id, fp2, state, &sout[(size_t)c * 6], cnt);
      std::memcpy(&sst[(size_t)c * 4], state, sizeof(state));
    }
  }
  std::vector<double> prev((size_t)n * 4, 0.0), cur((size_t)n * 4), out((size_t)n * 6, 0.0);
  int m = 0;
  for (; m < max_sweeps; m++) {
    long ch = 0, wr = 0;
    for (long c = 0; c < n; c++) {
      double state[4] = {0, 0, 0, 0};
      if (m > 0 && c > 0) std::memcpy(state, &prev[(size_t)(c - 1) * 4], sizeof(state));
      long cnt[3] = {0, 0, 0};
      if (rec[(size_t)c * NREC + R_KIND] != 0.0) aniso_cell(&aux[(size_t)c * 9], h, 0, 1, id, fp2, state, &out[(size_t)c * 6], cnt);
      std::memcpy(&cur[(size_t)c * 4], state, sizeof(state));
      if (m == 0 || std::memcmp(&cur[(size_t)c * 4], &prev[(size_t)c * 4], sizeof(state))) ch++;
      if (rec[(size_t)c * NREC + R_KIND] != 0.0 && std::memcmp(&out[(size_t)c * 6], &sout[(size_t)c * 6], 6 * sizeof(double))) wr++;
    }
    changed[m] = ch; wrong[m] = wr;
    prev.swap(cur);
    if (m > 0 && ch == 0) { m++; break; }
  }
  return m;
}
