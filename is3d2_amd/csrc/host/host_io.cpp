// host_io.cpp -- readers / writers of the iS3D2 file formats (see host_io.h).
#include "host_io.h"

#include <cctype>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

namespace is3d {
namespace host {

static const double kHbarC = 0.197327053;   // iS3D.h:14

static std::string join(const std::string& dir, const std::string& rel) {
  if (dir.empty() || dir == ".") return rel;
  return dir.back() == '/' ? dir + rel : dir + "/" + rel;
}

static bool read_all(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

// ---------------------------------------------------------------------------------------------
// ParameterReader
// ---------------------------------------------------------------------------------------------
// Arsenal.cpp trim(): removes EVERY blank and tab (not only the ends); toLower()
static std::string squeeze_lower(const std::string& s) {
  std::string t;
  for (char c : s)
    if (c != ' ' && c != '\t') t.push_back((char)std::tolower((unsigned char)c));
  return t;
}

long ParameterReader::find(const std::string& key) const {
  const std::string k = squeeze_lower(key);
  for (size_t i = 0; i < names_.size(); i++) if (names_[i] == k) return (long)i;
  return -1;
}

void ParameterReader::set(const std::string& key, double v) {
  const long i = find(key);
  if (i < 0) { names_.push_back(squeeze_lower(key)); values_.push_back(v); }
  else values_[i] = v;
}

bool ParameterReader::read_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) return false;
  std::string line;
  while (std::getline(f, line)) {
    const std::string body = line.substr(0, line.find('#'));
    std::string compact;
    for (char c : body) if (c != ' ' && c != '\t') compact.push_back(c);
    if (compact.empty() || compact == "\r") continue;
    const size_t eq = body.find('=');
    if (eq == std::string::npos) throw std::runtime_error("ParameterReader: \"=\" symbol not found in equation assignment " + line);
    std::stringstream ss(squeeze_lower(body.substr(eq + 1)) + " ");
    double v = 0.0;
    ss >> v;
    set(body.substr(0, eq), v);
  }
  return true;
}

bool ParameterReader::has(const std::string& key) const { return find(key) >= 0; }

double ParameterReader::get(const std::string& key) const {
  const long i = find(key);
  if (i < 0) throw std::runtime_error("ParameterReader::getVal error: parameter with name " + key + " not found.");
  return values_[i];
}

double ParameterReader::get(const std::string& key, double fallback) const {
  const long i = find(key);
  return i < 0 ? fallback : values_[i];
}

// ---------------------------------------------------------------------------------------------
// Table
// ---------------------------------------------------------------------------------------------
bool load_table(const std::string& path, Table& t) {
  std::string txt;
  if (!read_all(path, txt)) return false;
  t.cols.clear();
  size_t pos = 0;
  while (true) {
    const size_t nl = txt.find('\n', pos);
    if (nl == std::string::npos) break;   // unterminated last line is not read (readBlockData)
    std::stringstream ss(txt.substr(pos, nl - pos));
    pos = nl + 1;
    std::vector<double> row;
    double v;
    while (ss >> v) row.push_back(v);
    if (row.empty()) continue;
    if (t.cols.empty()) t.cols.resize(row.size());
    for (size_t c = 0; c < t.cols.size() && c < row.size(); c++) t.cols[c].push_back(row[c]);
  }
  return !t.cols.empty();
}

// ---------------------------------------------------------------------------------------------
// surfaces
// ---------------------------------------------------------------------------------------------
void Surface::resize(long n) {
  for (auto* v : {&tau, &x, &y, &eta, &dat, &dax, &day, &dan, &ux, &uy, &un, &E, &T, &P, &pixx, &pixy, &pixn, &piyy,
                  &piyn, &bulkPi, &muB, &nB, &Vx, &Vy, &Vn})
    v->assign(n, 0.0);
}

static double round15(double v) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.15g", v);   // ofstream << setprecision(15), read back with %lf
  return std::strtod(buf, nullptr);
}

struct AvgAcc {
  double vol = 0, T = 0, E = 0, P = 0, muB = 0, nB = 0;
  void add(double ut, double tau, double ux, double uy, double un, double dat, double dax, double day, double dan,
           double E_, double T_, double P_, double muB_, double nB_) {
    const double tau2 = tau * tau;
    const double uds = ut * dat + ux * dax + uy * day + un * dan;
    const double ds_ds = dat * dat - dax * dax - day * day - dan * dan / tau2;
    const double ds_max = std::fabs(uds) + std::sqrt(std::fabs(uds * uds - ds_ds));
    vol += ds_max; E += (E_ * ds_max); T += (T_ * ds_max); P += (P_ * ds_max); muB += (muB_ * ds_max); nB += (nB_ * ds_max);
  }
  Averages finish() const {
    return Averages{round15(T / vol), round15(E / vol), round15(P / vol), round15(muB / vol), round15(nB / vol)};
  }
};

Averages surface_averages(const Surface& s, int include_baryon) {
  AvgAcc a;
  for (long i = 0; i < s.size(); i++) {
    const double tau = s.tau[i];
    const double ut = std::sqrt(1. + s.ux[i] * s.ux[i] + s.uy[i] * s.uy[i] + tau * tau * s.un[i] * s.un[i]);
    a.add(ut, tau, s.ux[i], s.uy[i], s.un[i], s.dat[i], s.dax[i], s.day[i], s.dan[i], s.E[i], s.T[i], s.P[i],
          include_baryon ? s.muB[i] : 0.0, include_baryon ? s.nB[i] : 0.0);
  }
  return a.finish();
}

std::string write_averages_file(const std::string& dir, const Averages& a) {
  std::ofstream f(join(dir, "tables/thermodynamic/average_thermodynamic_quantities.dat"));
  if (!f) return "cannot write tables/thermodynamic/average_thermodynamic_quantities.dat";
  f << std::setprecision(15) << a.T << "\n" << a.E << "\n" << a.P << "\n" << a.muB << "\n" << a.nB;
  return "";
}

std::string read_surface(const std::string& dir, int mode, int dimension, int include_baryon, Surface& s,
                         Averages& avg, bool write_avg) {
  const std::string path = join(dir, "input/surface.dat");
  Table rows;
  if (!load_table(path, rows)) return "cannot read " + path;
  const long n = rows.rows();           // FO_data_reader::get_number_cells (readindata.cpp:137-146)
  std::ifstream f(path);
  s.resize(n);
  AvgAcc acc;
  double d;
  auto rd = [&]() { double v = 0.0; f >> v; return v; };
  if (mode == 1 || mode == 5) {
    for (long i = 0; i < n; i++) {
      s.tau[i] = rd(); s.x[i] = rd(); s.y[i] = rd(); s.eta[i] = rd();
      s.dat[i] = rd(); s.dax[i] = rd(); s.day[i] = rd(); s.dan[i] = rd();
      s.ux[i] = rd(); s.uy[i] = rd(); s.un[i] = rd();
      d = rd(); s.E[i] = d * kHbarC;
      d = rd(); s.T[i] = d * kHbarC;
      d = rd(); s.P[i] = d * kHbarC;
      d = rd(); s.pixx[i] = d * kHbarC;
      d = rd(); s.pixy[i] = d * kHbarC;
      d = rd(); s.pixn[i] = d * kHbarC;
      d = rd(); s.piyy[i] = d * kHbarC;
      d = rd(); s.piyn[i] = d * kHbarC;
      d = rd(); s.bulkPi[i] = d * kHbarC;
      double muB = 0, nB = 0;
      if (include_baryon) {
        d = rd(); muB = d * kHbarC; s.muB[i] = muB;
        nB = rd(); s.nB[i] = nB;
        s.Vx[i] = rd(); s.Vy[i] = rd(); s.Vn[i] = rd();
      }
      if (mode == 5) for (int k = 0; k < 6; k++) rd();   // thermal vorticity (polarization, out of scope)
      if (dimension == 2) s.eta[i] = 0;
      const double tau = s.tau[i];
      const double ut = std::sqrt(1. + s.ux[i] * s.ux[i] + s.uy[i] * s.uy[i] + tau * tau * s.un[i] * s.un[i]);
      acc.add(ut, tau, s.ux[i], s.uy[i], s.un[i], s.dat[i], s.dax[i], s.day[i], s.dan[i], s.E[i], s.T[i], s.P[i], muB, nB);
    }
  } else if (mode == 6) {
    for (long i = 0; i < n; i++) {
      const double tau = rd();
      s.tau[i] = tau; s.x[i] = rd(); s.y[i] = rd(); s.eta[i] = rd();
      d = rd(); s.dat[i] = d * tau;
      d = rd(); s.dax[i] = d * tau;
      d = rd(); s.day[i] = d * tau;
      d = rd(); s.dan[i] = d * tau;
      rd();                                   // u^tau
      s.ux[i] = rd(); s.uy[i] = rd();
      d = rd(); s.un[i] = d / tau;
      d = rd(); const double E = d * kHbarC; s.E[i] = E;
      d = rd(); const double T = d * kHbarC; s.T[i] = T;
      d = rd(); const double muB = d * kHbarC; s.muB[i] = muB;
      rd(); rd();                             // muS, muC
      d = rd(); s.P[i] = d * T - E;
      rd(); rd(); rd(); rd();                 // pi^tt pi^tx pi^ty tau pi^teta
      d = rd(); s.pixx[i] = d * kHbarC;
      d = rd(); s.pixy[i] = d * kHbarC;
      d = rd(); s.pixn[i] = d * kHbarC / tau;
      d = rd(); s.piyy[i] = d * kHbarC;
      d = rd(); s.piyn[i] = d * kHbarC / tau;
      rd();                                   // tau^2 pi^etaeta
      d = rd(); s.bulkPi[i] = d * kHbarC;
      double nB = 0.0;
      if (include_baryon) {
        nB = rd(); s.nB[i] = nB;
        rd();                                 // V^tau
        s.Vx[i] = rd(); s.Vy[i] = rd();
        d = rd(); s.Vn[i] = d / tau;
      }
      if (dimension == 2) s.eta[i] = 0;
      const double ut = std::sqrt(1. + s.ux[i] * s.ux[i] + s.uy[i] * s.uy[i] + tau * tau * s.un[i] * s.un[i]);
      acc.add(ut, tau, s.ux[i], s.uy[i], s.un[i], s.dat[i], s.dax[i], s.day[i], s.dan[i], s.E[i], s.T[i], s.P[i], muB, nB);
    }
  } else if (mode == 7) {
    if (dimension != 2) return "read_surface_hic_eventgen error: HIC-EventGen is boost-invariant (need to set dimension = 2)";
    if (include_baryon) return "read_surface_hic_eventgen error: HIC-EventGen does not consider baryon chemical potential (need to set include_baryon = 0)";
    for (long i = 0; i < n; i++) {
      const double tau = rd();
      s.tau[i] = tau; s.x[i] = rd(); s.y[i] = rd(); rd(); s.eta[i] = 0;
      d = rd(); s.dat[i] = d * tau;
      d = rd(); s.dax[i] = d * tau;
      d = rd(); s.day[i] = d * tau;
      rd(); s.dan[i] = 0;
      const double vx = rd(), vy = rd();
      rd();
      const double ut = 1. / std::sqrt(std::fabs(1. - vx * vx - vy * vy));
      s.ux[i] = ut * vx; s.uy[i] = ut * vy; s.un[i] = 0;
      rd(); rd(); rd(); rd();
      s.pixx[i] = rd(); s.pixy[i] = rd(); rd(); s.pixn[i] = 0;
      s.piyy[i] = rd(); rd(); s.piyn[i] = 0; rd();
      s.bulkPi[i] = rd();
      s.T[i] = rd(); s.E[i] = rd(); s.P[i] = rd();
      const double muB = rd(); s.muB[i] = muB;
      acc.add(ut, tau, s.ux[i], s.uy[i], 0.0, s.dat[i], s.dax[i], s.day[i], 0.0, s.E[i], s.T[i], s.P[i], muB, 0.0);
    }
  } else {
    return "read_freezeout_surface: mode must be 1, 5, 6 or 7";
  }
  avg = acc.finish();
  if (write_avg) return write_averages_file(dir, avg);
  return "";
}

// ---------------------------------------------------------------------------------------------
// PDG
// ---------------------------------------------------------------------------------------------
void decode_mcid(long mcid, int& gspin, int& baryon, int& sign, bool& has_anti) {
  long x = std::labs(mcid);
  int dg[10];
  for (int i = 0; i < 10; i++) { dg[i] = (int)(x % 10); x /= 10; }
  const unsigned nJ = (unsigned)(dg[0] + dg[7]) & 0xFu;    // 4-bit field, n8 adds to nJ
  const int nq3 = dg[1], nq2 = dg[2], nq1 = dg[3];
  const bool is_deuteron = (mcid == 1000010020);
  const bool is_hadron = !is_deuteron && nq3 != 0 && nq2 != 0;
  const bool is_meson = is_hadron && nq1 == 0, is_baryon = is_hadron && nq1 != 0;
  int spin;
  if (is_hadron) spin = (nJ == 0) ? 0 : (int)nJ - 1;
  else if (is_deuteron) spin = 2;
  else spin = nq3;
  if (is_hadron && nJ > 0) gspin = (int)nJ;
  else if (is_deuteron) gspin = 3;
  else gspin = spin + 1;
  if (is_deuteron) baryon = 2;
  else if (is_hadron) baryon = is_meson ? 0 : (is_baryon ? 1 : 0);
  else baryon = 0;
  if (is_deuteron) sign = -1;
  else if (is_hadron) sign = is_meson ? -1 : 1;
  else sign = spin % 2;
  if (is_hadron) has_anti = (baryon != 0) || (nq2 != nq3);
  else if (is_deuteron) has_anti = true;
  else has_anti = (nq3 == 1);
}

std::string read_pdg(const std::string& dir, int hrg_eos, std::vector<Particle>& out) {
  out.clear();
  if (hrg_eos == 1 || hrg_eos == 2) {
    const std::string path = join(dir, hrg_eos == 1 ? "PDG/pdg-urqmd_v3.3+.dat" : "PDG/pdg_smash.dat");
    std::ifstream f(path);
    if (!f) return "cannot read " + path;
    while (true) {
      Particle p{};
      int strange, charm, bottom, giso, charge, ndec;
      if (!(f >> p.mcid)) break;
      f >> p.name >> p.mass >> p.width >> p.gspin >> p.baryon >> strange >> charm >> bottom >> giso >> charge >> ndec;
      for (int j = 0; j < ndec; j++) { std::string tok; for (int k = 0; k < 8; k++) f >> tok; }
      out.push_back(p);
      if (p.baryon > 0) {                       // antibaryon entry (readindata.cpp:1023-1063)
        Particle a = p;
        a.mcid = -p.mcid; a.name = "Anti-baryon-" + p.name; a.baryon = -p.baryon;
        out.push_back(a);
      }
    }
    for (auto& p : out) p.sign = (p.baryon % 2 == 0) ? -1 : 1;
    return "";
  }
  if (hrg_eos == 3) {
    const std::string path = join(dir, "PDG/pdg_box.dat");
    std::ifstream f(path);
    if (!f) return "cannot read " + path;
    std::string line;
    while (std::getline(f, line)) {
      if (line.empty() || line[0] == '#') continue;
      std::istringstream ls(line);
      std::string name; double mass = 0, width = 0; char parity;
      long ids[4] = {0, 0, 0, 0};
      ls >> name >> mass >> width >> parity;
      for (int k = 0; k < 4; k++) if (!(ls >> ids[k])) { ids[k] = 0; break; }
      for (int k = 0; k < 4; k++) {
        if (ids[k] == 0) continue;
        int gs, b, sg; bool anti;
        decode_mcid(ids[k], gs, b, sg, anti);
        out.push_back(Particle{ids[k], name, mass, width, gs, b, sg});
        if (anti) out.push_back(Particle{-ids[k], "Anti-" + name, mass, width, gs, -b, sg});
      }
    }
    return "";
  }
  return "read_resonances error: need to set hrg_eos = (1,2,3)";
}

// ---------------------------------------------------------------------------------------------
// delta-f tables, Gauss-Laguerre
// ---------------------------------------------------------------------------------------------
std::string read_df_tables(const std::string& dir, int hrg_eos, DfTablesData& d) {
  const char* sub = hrg_eos == 1 ? "urqmd" : hrg_eos == 2 ? "smash" : hrg_eos == 3 ? "smash_box" : nullptr;
  if (!sub) return "Error: please choose hrg_eos = (1,2,3)";
  static const char* names[10] = {"c0", "c1", "c2", "c3", "c4", "F", "G", "betabulk", "betaV", "betapi"};
  for (int k = 0; k < 10; k++) {
    const std::string path = join(dir, std::string("deltaf_coefficients/vh/") + sub + "/" + names[k] + ".dat");
    std::ifstream f(path);
    if (!f) return "Couldn't open " + path;
    int nT = 0, nmuB = 0;
    f >> nT >> nmuB;
    std::string header;
    std::getline(f, header);
    std::getline(f, header);             // label line
    if (k == 0) { d.nT = nT; d.nmuB = nmuB; d.T.assign(nT, 0.0); d.muB.assign(nmuB, 0.0); d.tab.assign((size_t)10 * nmuB * nT, 0.0); }
    if (nT != d.nT || nmuB != d.nmuB) return "df coefficient tables have different (T, muB) grids";
    for (int iB = 0; iB < nmuB; iB++)
      for (int iT = 0; iT < nT; iT++) {
        double t, m, v;
        if (!(f >> t >> m >> v)) return "truncated " + path;
        d.T[iT] = t; d.muB[iB] = m;
        d.tab[((size_t)k * nmuB + iB) * nT + iT] = v;
      }
  }
  return "";
}

std::string read_gauss_laguerre(const std::string& path, int& alpha, int& points, std::vector<double>& roots,
                                std::vector<double>& weights) {
  std::ifstream f(path);
  if (!f) return "load_roots_and_weights flag: couldn't open gauss laguerre file " + path;
  f >> alpha >> points;
  roots.assign((size_t)alpha * points, 0.0);
  weights.assign((size_t)alpha * points, 0.0);
  for (int i = 0; i < alpha; i++)
    for (int j = 0; j < points; j++) {
      int dummy;
      f >> dummy >> roots[(size_t)i * points + j] >> weights[(size_t)i * points + j];
    }
  return f ? "" : "truncated " + path;
}

// ---------------------------------------------------------------------------------------------
// writers (EmissionFunction.cpp:406-558, 804-878)
// ---------------------------------------------------------------------------------------------
static void mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); i++) {
    cur.push_back(path[i]);
    if (path[i] == '/' && cur.size() > 1) mkdir(cur.c_str(), 0755);
  }
  mkdir(path.c_str(), 0755);
}

std::string write_spectra_files(const std::string& dir, const SpectraView& v) {
  const std::string out = join(dir, "results/continuous");
  mkdirs(out);
  const long npT = v.npT, nphi = v.nphi, ny = v.ny;
  auto idx = [&](long ipart, long ipT, long iphip, long iy) { return iy + ny * (iphip + nphi * (ipT + npT * ipart)); };
  const double two_pi = 2.0 * M_PI;
  for (long ipart = 0; ipart < v.npart; ipart++) {
    const long mc = (*v.mcid)[ipart];
    char fn[512];
    {   // dN_pTdpTdphidy
      std::snprintf(fn, sizeof(fn), "%s/dN_pTdpTdphidy_%ld.dat", out.c_str(), mc);
      std::ofstream s(fn);
      if (!s) return std::string("cannot write ") + fn;
      s << "y" << "\t" << "phip" << "\t" << "pT" << "\t" << "dN_pTdpTdphidy" << "\n";
      for (long iy = 0; iy < ny; iy++) {
        double y = 0.0;
        if (v.dimension == 3) y = v.y->get(1, iy + 1);
        for (long iphip = 0; iphip < nphi; iphip++) {
          const double phip = v.phi->get(1, iphip + 1);
          for (long ipT = 0; ipT < npT; ipT++) {
            const double pT = v.pT->get(1, ipT + 1);
            s << std::scientific << std::setw(5) << std::setprecision(8) << y << "\t" << phip << "\t" << pT << "\t"
              << v.dN[idx(ipart, ipT, iphip, iy)] << "\n";
          }
          s << "\n";
        }
      }
    }
    {   // vn (k = 1..7)
      std::snprintf(fn, sizeof(fn), "%s/vn_%ld.dat", out.c_str(), mc);
      std::ofstream s(fn);
      if (!s) return std::string("cannot write ") + fn;
      const std::complex<double> I(0.0, 1.0);
      for (long iy = 0; iy < ny; iy++) {
        double y = 0.0;
        if (v.dimension == 3) y = v.y->get(1, iy + 1);
        for (long ipT = 0; ipT < npT; ipT++) {
          const double pT = v.pT->get(1, ipT + 1);
          double re[7] = {0}, im[7] = {0}, den = 0.0;
          for (long iphip = 0; iphip < nphi; iphip++) {
            const double phip = v.phi->get(1, iphip + 1), w = v.phi->get(2, iphip + 1);
            const double dn = v.dN[idx(ipart, ipT, iphip, iy)];
            for (int k = 0; k < 7; k++) {
              re[k] += std::cos(((double)k + 1.0) * phip) * w * dn;
              im[k] += std::sin(((double)k + 1.0) * phip) * w * dn;
            }
            den += w * dn;
          }
          s << std::scientific << std::setw(5) << std::setprecision(8) << y << "\t" << pT;
          for (int k = 0; k < 7; k++) {
            double vn = std::abs(re[k] + I * im[k]) / den;
            if (den < 1.e-15) vn = 0.0;
            s << "\t" << vn;
          }
          s << "\n";
        }
        s << "\n";
      }
    }
    {   // dN_2pipTdpTdy
      std::snprintf(fn, sizeof(fn), "%s/dN_2pipTdpTdy_%ld.dat", out.c_str(), mc);
      std::ofstream s(fn);
      if (!s) return std::string("cannot write ") + fn;
      for (long iy = 0; iy < ny; iy++) {
        double y = 0.0;
        if (v.dimension == 3) y = v.y->get(1, iy + 1);
        for (long ipT = 0; ipT < npT; ipT++) {
          const double pT = v.pT->get(1, ipT + 1);
          double acc = 0.0;
          for (long iphip = 0; iphip < nphi; iphip++) acc += v.phi->get(2, iphip + 1) * v.dN[idx(ipart, ipT, iphip, iy)] / two_pi;
          s << std::scientific << std::setw(5) << std::setprecision(8) << y << "\t" << pT << "\t" << acc << "\n";
        }
        if (iy < ny - 1) s << "\n";
      }
    }
    {   // dN_dphidy
      std::snprintf(fn, sizeof(fn), "%s/dN_dphidy_%ld.dat", out.c_str(), mc);
      std::ofstream s(fn);
      if (!s) return std::string("cannot write ") + fn;
      for (long iy = 0; iy < ny; iy++) {
        double y = 0.0;
        if (v.dimension == 3) y = v.y->get(1, iy + 1);
        for (long iphip = 0; iphip < nphi; iphip++) {
          const double phip = v.phi->get(1, iphip + 1);
          double acc = 0.0;
          for (long ipT = 0; ipT < npT; ipT++) acc += v.pT->get(2, ipT + 1) * v.dN[idx(ipart, ipT, iphip, iy)];
          s << std::scientific << std::setw(5) << std::setprecision(8) << y << "\t" << phip << "\t" << acc << "\n";
        }
        if (iy < ny - 1) s << "\n";
      }
    }
    {   // dN_dy
      std::snprintf(fn, sizeof(fn), "%s/dN_dy_%ld.dat", out.c_str(), mc);
      std::ofstream s(fn);
      if (!s) return std::string("cannot write ") + fn;
      for (long iy = 0; iy < ny; iy++) {
        double y = 0.0;
        if (v.dimension == 3) y = v.y->get(1, iy + 1);
        double acc = 0.0;
        for (long iphip = 0; iphip < nphi; iphip++) {
          const double wphi = v.phi->get(2, iphip + 1);
          for (long ipT = 0; ipT < npT; ipT++) acc += wphi * v.pT->get(2, ipT + 1) * v.dN[idx(ipart, ipT, iphip, iy)];
        }
        s << std::setw(5) << std::setprecision(8) << y << "\t" << acc << std::endl;
      }
    }
  }
  return "";
}

std::string write_spacetime_files(const std::string& dir, const SpacetimeView& v) {
  const std::string out = join(dir, "results/continuous");
  mkdirs(out);
  const double two_pi = 2.0 * M_PI;
  const double tau_w = (v.tau_max - v.tau_min) / (double)v.tau_bins, r_w = (v.r_max - v.r_min) / (double)v.r_bins;
  const double phi_w = two_pi / (double)v.phip_bins;
  for (long ipart = 0; ipart < v.npart; ipart++) {
    const long mc = (*v.mcid)[ipart];
    char ft[512], fr[512], fp[512];
    std::snprintf(ft, sizeof(ft), "%s/dN_taudtaudy_%ld.dat", out.c_str(), mc);
    std::snprintf(fr, sizeof(fr), "%s/dN_2pirdrdy_%ld.dat", out.c_str(), mc);
    std::snprintf(fp, sizeof(fp), "%s/dN_dphidy_%ld.dat", out.c_str(), mc);
    std::ofstream t(ft, std::ios_base::app), r(fr, std::ios_base::app), a(fp, std::ios_base::app);   // appended, as the reference
    if (!t || !r || !a) return std::string("cannot write spacetime distributions of ") + std::to_string(mc);
    for (long ir = 0; ir < v.r_bins; ir++)
      r << std::setprecision(6) << std::scientific << v.r_min + r_w * ((double)ir + 0.5) << "\t"
        << v.dN_2pirdrdy[ipart * v.r_bins + ir] << "\n";
    for (long it = 0; it < v.tau_bins; it++)
      t << std::setprecision(6) << std::scientific << v.tau_min + tau_w * ((double)it + 0.5) << "\t"
        << v.dN_taudtaudy[ipart * v.tau_bins + it] << "\n";
    for (long ip = 0; ip < v.phip_bins; ip++)
      a << std::setprecision(6) << std::scientific << phi_w * ((double)ip + 0.5) << "\t"
        << v.dN_dphidy[ipart * v.phip_bins + ip] << "\n";
  }
  return "";
}

}  // namespace host
}  // namespace is3d
