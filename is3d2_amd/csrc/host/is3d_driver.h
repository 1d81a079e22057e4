// is3d_driver.h -- drop-in C++ facade of iS3D2's particlization plug-in surface for
// operations 1 (continuous spectra) and 0 (spacetime distributions), running the MI355X engine
// (libis3d_amd.so) underneath.
//
//   class IS3D                (iS3D.h:25-104)   read_fo_surf_from_memory + run_particlization
//   class EmissionFunctionArray (EmissionFunction.h:135-140) ctor + calculate_spectra
//
// Same inputs (iS3D_parameters.dat, input/surface.dat, PDG/, deltaf_coefficients/, tables/
// relative to a working directory) and the same outputs (results/continuous/*.dat).
// Differences from the reference: errors are returned / thrown instead of exit(); of operation = 2
// only the oversampling estimate (Ntotal, Nevents) is on this path, not the particle sampler itself;
// cells may be sharded over several GPUs in one process.
#pragma once
#include <string>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/is3d_amd.h"
#include "host_io.h"

namespace is3d {
namespace host {

// engine failure with the is3d_amd.h return code (IS3D_ERR_DF_RANGE for the reference's GSL abort, ...)
struct EngineError : std::runtime_error {
  int code;
  EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct RunOptions {
  int device = 0;          // first HIP device
  int num_devices = 1;     // cells sharded over devices [device, device + num_devices)
  std::vector<int> devices;  // if not empty: shard k runs on devices[k] (an index may repeat)
  bool write_files = true;
  bool quiet = false;
};

// EmissionFunctionArray(paraRdr, chosen, pT, phi, y, eta, particles, Nparticles, surface, FO_length, df tables)
class EmissionFunctionArray {
 public:
  EmissionFunctionArray(const ParameterReader& params, const Table& chosen, const Table& pT, const Table& phi,
                        const Table& y, const Table& eta, const std::vector<Particle>& particles, const Surface& surf,
                        const DfTablesData& df, const Averages& plasma, const std::vector<double>& gla_roots,
                        const std::vector<double>& gla_weights, int gla_alpha, int gla_points);
  // operation = 1: dN/(pT dpT dphi dy) [species][pT][phi][y]; throws std::runtime_error on failure
  void calculate_spectra(const RunOptions& opt);
  void write_files(const std::string& dir) const;
  const std::vector<double>& spectra() const { return dN_; }
  // operation = 0 (SpacetimeDistribution.cpp): dN/(tau dtau dy), dN/(2 pi r dr dy), dN/(dphi dy) [species][bins]
  void calculate_dN_dX(const RunOptions& opt);
  void write_spacetime_files(const std::string& dir) const;
  const std::vector<double>& dN_taudtaudy() const { return dNtau_; }
  const std::vector<double>& dN_2pirdrdy() const { return dNr_; }
  const std::vector<double>& dN_dphidy() const { return dNphi_; }
  is3d_spacetime_bins bins() const { return bins_; }
  const std::vector<long>& mcid() const { return mcid_; }
  // operation = 2 oversampling estimate (ParticleSampler.cpp:447-636): the reference's Ntotal
  double estimate_total_yield(const RunOptions& opt);
  double seconds() const { return seconds_; }

 private:
  const ParameterReader& p_;
  const Table &pT_, &phi_, &y_, &eta_;
  const Surface& surf_;
  const DfTablesData& df_;
  Averages plasma_;
  const std::vector<double>&gr_, &gw_;
  int galpha_, gpts_;
  int dimension_ = 2;
  std::vector<double> mass_, sign_, degen_, baryon_;
  std::vector<double> pdg_mass_, pdg_sign_, pdg_degen_, pdg_baryon_;
  std::vector<long> mcid_;
  std::vector<double> dN_;
  std::vector<double> dNtau_, dNr_, dNphi_;
  is3d_spacetime_bins bins_{};
  double seconds_ = 0.0;
  double ntotal_ = 0.0;
  void run_sharded(const RunOptions& opt, int operation);   // operation 2: the yield estimate
};

class IS3D {
 public:
  explicit IS3D(std::string workdir = ".") : dir_(std::move(workdir)) {}
  // iS3D.cpp:33-78 (units: reader-converted, GeV / fm)
  void read_fo_surf_from_memory(std::vector<double> tau, std::vector<double> x, std::vector<double> y,
                                std::vector<double> eta, std::vector<double> dsigma_tau, std::vector<double> dsigma_x,
                                std::vector<double> dsigma_y, std::vector<double> dsigma_eta, std::vector<double> E,
                                std::vector<double> T, std::vector<double> P, std::vector<double> ux,
                                std::vector<double> uy, std::vector<double> un, std::vector<double> pixx,
                                std::vector<double> pixy, std::vector<double> pixn, std::vector<double> piyy,
                                std::vector<double> piyn, std::vector<double> pinn, std::vector<double> Pi);
  // iS3D.cpp:81-282 for operation = 1, 0 and the estimate of 2; throws std::runtime_error.  spectra() = the momentum
  // spectra (operation 1) or, per species, [dN_taudtaudy | dN_2pirdrdy | dN_dphidy] bins (operation 0)
  void run_particlization(int fo_from_file, const RunOptions& opt = RunOptions());
  const std::vector<double>& spectra() const { return dN_; }
  // operation = 2: Ntotal and Nevents = min(ceil(min_num_hadrons / Ntotal), max_num_samples) if
  // oversample, else 1 (EmissionFunction.cpp:1237-1249); the sampling itself is not on this path
  double total_yield() const { return ntotal_; }
  long events() const { return nevents_; }

 private:
  std::string dir_;
  double ntotal_ = 0.0;
  long nevents_ = 0;
  Surface mem_;
  std::vector<double> dN_;
};

}  // namespace host
}  // namespace is3d
