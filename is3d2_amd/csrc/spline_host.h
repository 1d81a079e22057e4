// spline_host.h -- host-side construction of the natural cubic splines the
// engine evaluates on the GPU (gsl_interp_cspline semantics, DeltafData.cpp:298-321
// and :290-294), plus a serial PTB "Jonah" table for the test emulator (DeltafData.cpp:220-295).
#pragma once
#include <cmath>
#include <vector>

#include "cf_math.h"

namespace is3d {

// Second-derivative/2 coefficients c[i] of GSL's cspline_init (natural boundary),
// via the symmetric tridiagonal L D L^T solve of linalg/tridiag.c.
// Returns false if x is not strictly increasing (gsl_interp_init EINVAL).
inline bool cspline_coeffs(const double* x, const double* y, int n, std::vector<double>& c) {
  c.assign(n, 0.0);
  for (int i = 0; i + 1 < n; i++) if (!(x[i] < x[i + 1])) return false;
  const int sys = n - 2;
  if (sys <= 0) return true;
  std::vector<double> g(sys), diag(sys), off(sys);
  for (int i = 0; i < sys; i++) {
    const double h_i = x[i + 1] - x[i], h_ip1 = x[i + 2] - x[i + 1];
    const double yd_i = y[i + 1] - y[i], yd_ip1 = y[i + 2] - y[i + 1];
    const double g_i = (h_i != 0.0) ? 1.0 / h_i : 0.0, g_ip1 = (h_ip1 != 0.0) ? 1.0 / h_ip1 : 0.0;
    off[i] = h_ip1;
    diag[i] = 2.0 * (h_ip1 + h_i);
    g[i] = 3.0 * (yd_ip1 * g_ip1 - yd_i * g_i);
  }
  if (sys == 1) { c[1] = g[0] / diag[0]; return true; }
  const int N = sys;
  std::vector<double> gamma(N), alpha(N), cc(N), z(N);
  alpha[0] = diag[0];
  gamma[0] = off[0] / alpha[0];
  for (int i = 1; i < N - 1; i++) { alpha[i] = diag[i] - off[i - 1] * gamma[i - 1]; gamma[i] = off[i] / alpha[i]; }
  alpha[N - 1] = diag[N - 1] - off[N - 2] * gamma[N - 2];
  z[0] = g[0];
  for (int i = 1; i < N; i++) z[i] = g[i] - gamma[i - 1] * z[i - 1];
  for (int i = 0; i < N; i++) cc[i] = z[i] / alpha[i];
  c[N] = cc[N - 1];
  for (int i = N - 2; i >= 0; i--) c[i + 1] = cc[i] - gamma[i] * c[i + 2];
  return true;
}

// compute_jonah_coefficients serially on the host (test emulator only; the engine builds the table
// on the device from the same cf_math.h pieces, summing every row over the PDG in the same order)
inline void jonah_table(double T, int npdg, const double* mass, const double* degen, const double* sign, const double* r2,
                        const double* w2, int pts, std::vector<double>& l2, std::vector<double>& z,
                        std::vector<double>& bp, double& bpmax) {
  l2.assign(kJonahN, 0.0); z.assign(kJonahN, 0.0); bp.assign(kJonahN, 0.0);
  bpmax = -1.0;
  std::vector<double> e0(npdg), p0(npdg);
  for (int n = 0; n < npdg; n++) jonah_terms(T, mass[n], degen[n], sign[n], r2, w2, pts, 0.0, &e0[n], &p0[n]);
  for (int i = 0; i < kJonahN; i++) {
    double E = 0.0, P = 0.0, Em = 0.0, Pm = 0.0;
    for (int n = 0; n < npdg; n++) {
      if (mass[n] == 0.0) continue;
      double em, pm;
      jonah_terms(T, mass[n], degen[n], sign[n], r2, w2, pts, jonah_lambda(i), &em, &pm);
      E += e0[n]; P += p0[n]; Em += em; Pm += pm;
    }
    jonah_row(i, E, P, Em, Pm, l2.data(), z.data(), bp.data());
    bpmax = std::fmax(bpmax, bp[i]);
  }
}

}  // namespace is3d
