// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A small driver around the GSL-free reference sources (compiled in place from
// /root/reference/src/cpp by oracle/ref/build_ref.sh into oracle/_ref/ref_harness):
//   readindata.cpp (FO_data_reader, PDG_Data, read_mcid, Gauss_Laguerre, Plasma),
//   GaussThermal.cpp, LocalRestFrame.cpp, Table.cpp, ParameterReader.cpp, Arsenal.cpp.
// The spectra loops (MomentumSpectra.cpp), Deltaf_Data and AnisoVariables need GSL,
// which this image lacks, so they cannot be built here.
//
// Every command runs in the current directory (the reference hard-codes relative
// paths) and prints numbers with %.17g.
//   ref_harness surface            -> reads iS3D_parameters.dat + input/surface.dat
//   ref_harness pdg                -> reads iS3D_parameters.dat + PDG/<hrg file>
//   ref_harness gauss <file>       -> GaussThermal integrals for stdin lines "kind mbar alphaB baryon sign"
//   ref_harness gaussmod <file>    -> Gauss1D_mod for stdin lines "kind mbar lambda sign"
//   ref_harness lrf                -> Milne basis + pi LRF + V LRF for stdin lines of 19 numbers
//   ref_harness dslrf              -> Surface_Element_Vector LRF boost + magnitude for stdin lines
//                                     "ut ux uy un tau dat dax day dan"
//   ref_harness table <file>       -> Table dimensions and contents
//   ref_harness params <file> k... -> ParameterReader::getVal for each key
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "GaussThermal.h"
#include "LocalRestFrame.h"
#include "ParameterReader.h"
#include "Table.h"
#include "iS3D.h"
#include "readindata.h"

static void surface() {
  ParameterReader* pr = new ParameterReader;
  pr->readFromFile("iS3D_parameters.dat");
  FO_data_reader rd(pr, "input");
  long n = rd.get_number_cells();
  FO_surf* s = new FO_surf[n];
  memset((void*)s, 0, sizeof(FO_surf) * n);
  rd.read_freezeout_surface(s);
  printf("\n@@BEGIN\n%ld\n", n);
  for (long i = 0; i < n; i++) {
    const FO_surf& c = s[i];
    double v[] = {c.tau, c.x, c.y, c.eta, c.dat, c.dax, c.day, c.dan, c.ux, c.uy, c.un, c.E, c.T, c.P,
                  c.pixx, c.pixy, c.pixn, c.piyy, c.piyn, c.bulkPi, c.muB, c.nB, c.Vx, c.Vy, c.Vn};
    for (double x : v) printf("%.17g ", x);
    printf("\n");
  }
  Plasma q;
  q.load_thermodynamic_averages();
  printf("%.17g %.17g %.17g %.17g %.17g\n", q.temperature, q.energy_density, q.pressure, q.baryon_chemical_potential,
         q.net_baryon_density);
}

static void pdg() {
  ParameterReader* pr = new ParameterReader;
  pr->readFromFile("iS3D_parameters.dat");
  particle_info* p = new particle_info[Maxparticle];
  PDG_Data d(pr);
  int n = d.read_resonances(p);
  printf("\n@@BEGIN\n%d\n", n);
  for (int i = 0; i < n; i++) printf("%ld %.17g %d %d %d\n", p[i].mc_id, p[i].mass, p[i].gspin, p[i].baryon, p[i].sign);
}

static void gauss(const char* file, bool mod) {
  Gauss_Laguerre g;
  g.load_roots_and_weights(file);
  char line[512];
  while (fgets(line, sizeof(line), stdin)) {
    int kind, alpha;
    double a, b, c, d;
    if (!mod) {
      if (sscanf(line, "%d %d %lf %lf %lf %lf", &kind, &alpha, &a, &b, &c, &d) != 6) continue;
      double (*f)(double, double, double, double, double) = neq_int;
      switch (kind) { case 0: f = neq_int; break; case 1: f = J10_int; break; case 2: f = J11_int; break;
                      case 3: f = J20_int; break; case 4: f = J30_int; break; default: f = J31_int; }
      printf("%.17g\n", GaussThermal(f, g.root[alpha], g.weight[alpha], g.points, a, b, c, d));
    } else {
      if (sscanf(line, "%d %d %lf %lf %lf", &kind, &alpha, &a, &b, &c) != 5) continue;
      printf("%.17g\n", Gauss1D_mod(kind == 0 ? E_mod_int : P_mod_int, g.root[alpha], g.weight[alpha], g.points, a, b, c));
    }
  }
}

// stdin: ut ux uy un tau pitt pitx pity pitn pixx pixy pixn piyy piyn pinn Vt Vx Vy Vn
static void lrf() {
  double v[19];
  while (true) {
    for (int i = 0; i < 19; i++) if (scanf("%lf", &v[i]) != 1) return;
    double ut = v[0], ux = v[1], uy = v[2], un = v[3], tau = v[4];
    double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
    Milne_Basis b(ut, ux, uy, un, uperp, utperp, tau);
    Shear_Stress pi(v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12], v[13], v[14]);
    pi.boost_pimunu_to_lrf(b, tau * tau);
    Baryon_Diffusion V(v[15], v[16], v[17], v[18]);
    V.boost_Vmu_to_lrf(b, tau * tau);
    double o[] = {b.Xt, b.Xx, b.Xy, b.Xn, b.Yx, b.Yy, b.Zt, b.Zn, pi.pixx_LRF, pi.pixy_LRF, pi.pixz_LRF, pi.piyy_LRF,
                  pi.piyz_LRF, pi.pizz_LRF, V.Vx_LRF, V.Vy_LRF, V.Vz_LRF};
    for (double x : o) printf("%.17g ", x);
    printf("\n");
  }
}

// stdin: ut ux uy un tau dat dax day dan
static void dslrf() {
  double v[9];
  while (true) {
    for (int i = 0; i < 9; i++) if (scanf("%lf", &v[i]) != 1) return;
    double ut = v[0], ux = v[1], uy = v[2], un = v[3], tau = v[4];
    double uperp = sqrt(ux * ux + uy * uy), utperp = sqrt(1.0 + ux * ux + uy * uy);
    Milne_Basis b(ut, ux, uy, un, uperp, utperp, tau);
    Surface_Element_Vector ds(v[5], v[6], v[7], v[8]);
    ds.boost_dsigma_to_lrf(b, ut, ux, uy, un);
    ds.compute_dsigma_magnitude();
    double o[] = {ds.dsigmat_LRF, ds.dsigmax_LRF, ds.dsigmay_LRF, ds.dsigmaz_LRF, ds.dsigma_space};
    for (double x : o) printf("%.17g ", x);
    printf("\n");
  }
}

static void table(const char* file) {
  Table t(file);
  printf("%ld %ld\n", t.getNumberOfCols(), t.getNumberOfRows());
  for (long j = 1; j <= t.getNumberOfRows(); j++) {
    for (long i = 1; i <= t.getNumberOfCols(); i++) printf("%.17g ", t.get(i, j));
    printf("\n");
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::string cmd = argv[1];
  if (cmd == "surface") surface();
  else if (cmd == "pdg") pdg();
  else if (cmd == "gauss" && argc > 2) gauss(argv[2], false);
  else if (cmd == "gaussmod" && argc > 2) gauss(argv[2], true);
  else if (cmd == "lrf") lrf();
  else if (cmd == "dslrf") dslrf();
  else if (cmd == "table" && argc > 2) table(argv[2]);
  else if (cmd == "params" && argc > 2) {
    ParameterReader pr;
    pr.readFromFile(argv[2]);
    for (int i = 3; i < argc; i++) printf("%.17g\n", pr.getVal(argv[i]));
  } else return 2;
  return 0;
}
