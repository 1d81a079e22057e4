// host_io.h -- C++ host services for the iS3D2 drop-in workflow (reference file
// formats on both sides of the continuous-spectra hot path).  Clean-room
// implementations of the reference's readers/writers; each function cites the
// reference code whose behaviour it reproduces.
#pragma once
#include <string>
#include <vector>

namespace is3d {
namespace host {

// ParameterReader (ParameterReader.cpp:28-155): "key = value # comment", keys
// lower-cased and trimmed, values parsed as double, later keys overwrite earlier.
class ParameterReader {
 public:
  bool read_file(const std::string& path);            // false if the file cannot be opened
  bool has(const std::string& key) const;
  double get(const std::string& key) const;           // throws std::runtime_error if missing
  double get(const std::string& key, double fallback) const;
  void set(const std::string& key, double v);
 private:
  std::vector<std::string> names_;
  std::vector<double> values_;
  long find(const std::string& key) const;
};

// Table (Table.cpp:141-162 + Arsenal.cpp:86-121): whitespace columns; a row is a line
// terminated by '\n' (a final unterminated line is not read, as in readBlockData).
struct Table {
  std::vector<std::vector<double>> cols;              // cols[c][r]
  long rows() const { return cols.empty() ? 0 : (long)cols[0].size(); }
  long ncols() const { return (long)cols.size(); }
  double get(long col1, long row1) const { return cols[col1 - 1][row1 - 1]; }   // 1-based like the reference
};
bool load_table(const std::string& path, Table& t);

// Freeze-out surface, SoA in reader units (GeV, fm), field order of include/is3d_amd.h.
struct Surface {
  std::vector<double> tau, x, y, eta, dat, dax, day, dan, ux, uy, un, E, T, P, pixx, pixy, pixn, piyy, piyn, bulkPi,
      muB, nB, Vx, Vy, Vn;
  long size() const { return (long)tau.size(); }
  void resize(long n);
};

// Plasma averages (readindata.cpp:316-366): ds_max-weighted T, E, P, muB, nB.
struct Averages { double T, E, P, muB, nB; };

// FO_data_reader::read_freezeout_surface for mode 1/5 (CPU VH, readindata.cpp:167-367),
// 6 (MUSIC, :372-567) and 7 (HIC-EventGen, :570-731).  Reads <dir>/input/surface.dat,
// returns the averages after the reference's setprecision(15) text round trip and (like the
// reference) writes them to <dir>/tables/thermodynamic/average_thermodynamic_quantities.dat
// when write_averages is set.  Returns an empty string on success, else an error message.
std::string read_surface(const std::string& dir, int mode, int dimension, int include_baryon, Surface& s,
                         Averages& avg, bool write_averages);
// averages for a surface handed over in memory (iS3D.cpp:126-220)
Averages surface_averages(const Surface& s, int include_baryon);
std::string write_averages_file(const std::string& dir, const Averages& a);

// PDG_Data::read_resonances (readindata.cpp:973-1252): hrg_eos 1 UrQMD, 2 SMASH
// (conventional format, antibaryons inserted), 3 SMASH box (mcid-decoded).
struct Particle { long mcid; std::string name; double mass, width; int gspin, baryon, sign; };
std::string read_pdg(const std::string& dir, int hrg_eos, std::vector<Particle>& out);
void decode_mcid(long mcid, int& gspin, int& baryon, int& sign, bool& has_antiparticle);   // read_mcid

// Deltaf_Data::load_df_coefficient_data (DeltafData.cpp:65-217): 10 tables
// c0 c1 c2 c3 c4 F G betabulk betaV betapi from <dir>/deltaf_coefficients/vh/<hrg>/.
struct DfTablesData { int nT = 0, nmuB = 0; std::vector<double> T, muB, tab; };   // tab[10][nmuB][nT]
std::string read_df_tables(const std::string& dir, int hrg_eos, DfTablesData& d);

// Gauss_Laguerre::load_roots_and_weights (readindata.cpp:26-61)
std::string read_gauss_laguerre(const std::string& path, int& alpha, int& points, std::vector<double>& roots,
                                std::vector<double>& weights);

// EmissionFunctionArray writers (EmissionFunction.cpp:406-558, 804-878): dN_pTdpTdphidy_<mcid>.dat,
// vn_, dN_2pipTdpTdy_, dN_dphidy_, dN_dy_ under <dir>/results/continuous/.
struct SpectraView {
  const double* dN;                 // [species][pT][phi][y]
  int npart, npT, nphi, ny, dimension;
  const Table *pT, *phi, *y;
  const std::vector<long>* mcid;
};
std::string write_spectra_files(const std::string& dir, const SpectraView& v);

// operation = 0 writers (SpacetimeDistribution.cpp:138-145, 407-440): dN_taudtaudy_<mcid>.dat,
// dN_2pirdrdy_<mcid>.dat, dN_dphidy_<mcid>.dat under <dir>/results/continuous/, opened in append mode,
// "bin midpoint \t value" with setprecision(6) scientific.
struct SpacetimeView {
  const double *dN_taudtaudy, *dN_2pirdrdy, *dN_dphidy;   // [species][bins], bin-normalised
  int npart;
  double tau_min, tau_max; int tau_bins;
  double r_min, r_max; int r_bins;
  int phip_bins;
  const std::vector<long>* mcid;
};
std::string write_spacetime_files(const std::string& dir, const SpacetimeView& v);

}  // namespace host
}  // namespace is3d
