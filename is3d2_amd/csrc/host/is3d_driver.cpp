// is3d_driver.cpp -- IS3D / EmissionFunctionArray facades over the engine's C ABI.
#include "is3d_driver.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "../../../include/is3d_amd.h"
#include "../../../include/is3d_host.h"

namespace is3d {
namespace host {

static void check(bool ok, const std::string& msg) {
  if (!ok) throw std::runtime_error(msg);
}

EmissionFunctionArray::EmissionFunctionArray(const ParameterReader& params, const Table& chosen, const Table& pT,
                                             const Table& phi, const Table& y, const Table& eta,
                                             const std::vector<Particle>& particles, const Surface& surf,
                                             const DfTablesData& df, const Averages& plasma,
                                             const std::vector<double>& gla_roots, const std::vector<double>& gla_weights,
                                             int gla_alpha, int gla_points)
    : p_(params), pT_(pT), phi_(phi), y_(y), eta_(eta), surf_(surf), df_(df), plasma_(plasma), gr_(gla_roots),
      gw_(gla_weights), galpha_(gla_alpha), gpts_(gla_points) {
  dimension_ = (int)p_.get("dimension");
  check(dimension_ == 2 || dimension_ == 3, "EmissionFunctionArray error: need to set dimension = (2,3)");
  const int df_mode = (int)p_.get("df_mode");
  check(df_mode >= 1 && df_mode <= 5, "EmissionFunctionArray error: need to set df_mode = (1,2,3,4,5)");
  // chosen particles -> PDG indices, first match (EmissionFunction.cpp:356-372)
  std::vector<int> idx;
  for (long m = 0; m < chosen.rows(); m++) {
    const long mc = (long)chosen.get(1, m + 1);
    int hit = -1;
    for (size_t n = 0; n < particles.size(); n++)
      if (particles[n].mcid == mc) { hit = (int)n; break; }
    check(hit >= 0, "chosen particle " + std::to_string(mc) + " is not in the PDG list");
    idx.push_back(hit);
  }
  if ((int)p_.get("group_particles", 0.0) == 1) {   // bubble sort by mass (:375-390)
    const int nc = (int)idx.size();
    for (int m = 0; m < nc; m++)
      for (int n = 0; n < nc - m - 1; n++)
        if (particles[idx[n]].mass > particles[idx[n + 1]].mass) std::swap(idx[n], idx[n + 1]);
  }
  for (int i : idx) {
    mass_.push_back(particles[i].mass); sign_.push_back(particles[i].sign); degen_.push_back(particles[i].gspin);
    baryon_.push_back(particles[i].baryon); mcid_.push_back(particles[i].mcid);
  }
  for (const auto& q : particles) {
    pdg_mass_.push_back(q.mass); pdg_sign_.push_back(q.sign); pdg_degen_.push_back(q.gspin); pdg_baryon_.push_back(q.baryon);
  }
}

static void set_or_throw(is3d_engine* e, int rc) {
  if (rc != IS3D_OK) throw EngineError(rc, std::string("is3d engine: ") + is3d_last_error(e));
}

static is3d_params engine_params(const ParameterReader& p, int operation, int dimension) {
  is3d_params prm{};
  prm.operation = operation;
  prm.dimension = dimension;
  prm.df_mode = (int)p.get("df_mode");
  prm.include_baryon = (int)p.get("include_baryon");
  prm.include_bulk_deltaf = (int)p.get("include_bulk_deltaf");
  prm.include_shear_deltaf = (int)p.get("include_shear_deltaf");
  prm.include_baryondiff_deltaf = (int)p.get("include_baryondiff_deltaf");
  prm.regulate_deltaf = (int)p.get("regulate_deltaf");
  prm.outflow = (int)p.get("outflow");
  prm.deta_min = p.get("deta_min");
  prm.mass_pion0 = p.get("mass_pion0");
  // PTMA warm-start chains: the reference as shipped is serial (CORES = 1, EmissionFunction.cpp:131-135), one
  // chain over every cell (MomentumSpectra.cpp:1308-1364); iS3D_parameters.dat has no such key, so the drop-in
  // default is 1.  famod_chains = C reproduces an OpenMP build with C threads, 0 solves every cell cold.
  prm.famod_chains = (int)p.get("famod_chains", 1.0);
  return prm;
}

// operation = 0 binning from the parameter file (EmissionFunction.cpp:232-247); spacetime_threads (ours,
// default 0) = the reference run's OpenMP thread count to reproduce its memset carry (is3d_amd.h)
static is3d_spacetime_bins spacetime_bins(const ParameterReader& p) {
  is3d_spacetime_bins b{};
  b.tau_min = p.get("tau_min", 0.0); b.tau_max = p.get("tau_max", 12.0); b.tau_bins = (int)p.get("tau_bins", 120.0);
  b.r_min = p.get("r_min", 0.0); b.r_max = p.get("r_max", 12.0); b.r_bins = (int)p.get("r_bins", 60.0);
  b.phip_bins = (int)p.get("phip_bins", 100.0);
  b.threads = (int)p.get("spacetime_threads", 0.0);
  return b;
}

// One engine over every requested device (is3d_create_devices): the library splits the cells into
// cost-balanced windows, runs the devices concurrently and sums their spectra on the devices (RCCL
// all-reduce over distinct GPUs), replacing the reference's OpenMP fan-out and thread reduction
// (MomentumSpectra.cpp:98-107, 383-411).
void EmissionFunctionArray::run_sharded(const RunOptions& opt, int operation) {
  const is3d_params prm = engine_params(p_, operation, dimension_);
  const is3d_spacetime_bins bins = spacetime_bins(p_);
  const int ndev = opt.devices.empty() ? std::max(1, opt.num_devices) : (int)opt.devices.size();
  std::vector<int> devs(ndev);
  for (int k = 0; k < ndev; k++) devs[k] = opt.devices.empty() ? opt.device + k : opt.devices[k];
  std::vector<double> pTv(pT_.cols[0]), phiv(phi_.cols[0]), yv(y_.cols[0]), etav(eta_.cols[0]), etaw(eta_.cols[1]);
  std::vector<double> pTw(pT_.ncols() > 1 ? pT_.cols[1] : std::vector<double>(pTv.size(), 0.0));
  std::vector<double> phiw(phi_.ncols() > 1 ? phi_.cols[1] : std::vector<double>(phiv.size(), 0.0));
  const long n = surf_.size();
  const int np = (int)mass_.size();
  auto t0 = std::chrono::steady_clock::now();
  is3d_engine* e = ndev == 1 ? is3d_create(devs[0]) : is3d_create_devices(ndev, devs.data());
  if (!e) throw EngineError(IS3D_ERR_DEVICE, "is3d_create on device " + std::to_string(devs[0]) + " failed");
  try {
    set_or_throw(e, is3d_set_params(e, &prm));
    set_or_throw(e, is3d_set_species(e, np, mass_.data(), sign_.data(), degen_.data(), baryon_.data()));
    set_or_throw(e, is3d_set_pdg(e, (int)pdg_mass_.size(), pdg_mass_.data(), pdg_sign_.data(), pdg_degen_.data(), pdg_baryon_.data()));
    set_or_throw(e, is3d_set_momentum_grid(e, (int)pTv.size(), pTv.data(), (int)phiv.size(), phiv.data(), (int)yv.size(),
                                           yv.data(), (int)etav.size(), etav.data(), etaw.data()));
    set_or_throw(e, is3d_set_gauss_laguerre(e, galpha_, gpts_, gr_.data(), gw_.data()));
    set_or_throw(e, is3d_set_df_tables(e, df_.nT, df_.nmuB, df_.T.data(), df_.muB.data(), df_.tab.data(), plasma_.T));
    auto fp = [&](const std::vector<double>& v) { return v.empty() ? nullptr : v.data(); };
    is3d_surface s{fp(surf_.tau), fp(surf_.x), fp(surf_.y), fp(surf_.eta), fp(surf_.dat), fp(surf_.dax), fp(surf_.day),
                   fp(surf_.dan), fp(surf_.ux), fp(surf_.uy), fp(surf_.un), fp(surf_.E), fp(surf_.T), fp(surf_.P),
                   fp(surf_.pixx), fp(surf_.pixy), fp(surf_.pixn), fp(surf_.piyy), fp(surf_.piyn), fp(surf_.bulkPi),
                   fp(surf_.muB), fp(surf_.nB), fp(surf_.Vx), fp(surf_.Vy), fp(surf_.Vn)};
    set_or_throw(e, is3d_set_surface(e, n, &s));
    if (operation == 1) {
      dN_.assign(is3d_output_size(e), 0.0);
      set_or_throw(e, is3d_calculate_spectra(e, dN_.data()));
    } else if (operation == 2) {
      const double plasma[5] = {plasma_.T, plasma_.E, plasma_.P, plasma_.muB, plasma_.nB};
      set_or_throw(e, is3d_total_yield(e, plasma, p_.get("y_cut", 0.5), &ntotal_, nullptr));
    } else {
      set_or_throw(e, is3d_set_momentum_weights(e, pTw.data(), phiw.data()));
      set_or_throw(e, is3d_set_spacetime_bins(e, &bins));
      bins_ = bins;
      dNtau_.assign((size_t)np * bins.tau_bins, 0.0);
      dNr_.assign((size_t)np * bins.r_bins, 0.0);
      dNphi_.assign((size_t)np * bins.phip_bins, 0.0);
      set_or_throw(e, is3d_calculate_dN_dX(e, dNtau_.data(), dNr_.data(), dNphi_.data()));
    }
  } catch (...) {
    is3d_destroy(e);
    throw;
  }
  is3d_destroy(e);
  seconds_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void EmissionFunctionArray::calculate_spectra(const RunOptions& opt) { run_sharded(opt, 1); }

void EmissionFunctionArray::calculate_dN_dX(const RunOptions& opt) { run_sharded(opt, 0); }

double EmissionFunctionArray::estimate_total_yield(const RunOptions& opt) {
  run_sharded(opt, 2);
  return ntotal_;
}

void EmissionFunctionArray::write_spacetime_files(const std::string& dir) const {
  SpacetimeView v{dNtau_.data(), dNr_.data(), dNphi_.data(), (int)mass_.size(), bins_.tau_min, bins_.tau_max,
                  bins_.tau_bins, bins_.r_min, bins_.r_max, bins_.r_bins, bins_.phip_bins, &mcid_};
  const std::string err = host::write_spacetime_files(dir, v);
  if (!err.empty()) throw std::runtime_error(err);
}

void EmissionFunctionArray::write_files(const std::string& dir) const {
  const int ny = (dimension_ == 3) ? (int)y_.rows() : 1;
  SpectraView v{dN_.data(), (int)mass_.size(), (int)pT_.rows(), (int)phi_.rows(), ny, dimension_, &pT_, &phi_, &y_, &mcid_};
  const std::string err = write_spectra_files(dir, v);
  if (!err.empty()) throw std::runtime_error(err);
}

void IS3D::read_fo_surf_from_memory(std::vector<double> tau, std::vector<double> x, std::vector<double> y,
                                   std::vector<double> eta, std::vector<double> dsigma_tau,
                                   std::vector<double> dsigma_x, std::vector<double> dsigma_y,
                                   std::vector<double> dsigma_eta, std::vector<double> E, std::vector<double> T,
                                   std::vector<double> P, std::vector<double> ux, std::vector<double> uy,
                                   std::vector<double> un, std::vector<double> pixx, std::vector<double> pixy,
                                   std::vector<double> pixn, std::vector<double> piyy, std::vector<double> piyn,
                                   std::vector<double> pinn, std::vector<double> Pi) {
  (void)pinn;   // reconstructed from orthogonality/tracelessness, as in the reference
  const long n = (long)tau.size();
  mem_.resize(n);
  mem_.tau = tau; mem_.x = x; mem_.y = y; mem_.eta = eta; mem_.dat = dsigma_tau; mem_.dax = dsigma_x;
  mem_.day = dsigma_y; mem_.dan = dsigma_eta; mem_.E = E; mem_.T = T; mem_.P = P; mem_.ux = ux; mem_.uy = uy;
  mem_.un = un; mem_.pixx = pixx; mem_.pixy = pixy; mem_.pixn = pixn; mem_.piyy = piyy; mem_.piyn = piyn;
  mem_.bulkPi = Pi;
}

static std::string path_in(const std::string& dir, const std::string& rel) {
  return (dir.empty() || dir == ".") ? rel : dir + "/" + rel;
}

void IS3D::run_particlization(int fo_from_file, const RunOptions& opt) {
  ParameterReader prm;
  check(prm.read_file(path_in(dir_, "iS3D_parameters.dat")), "ParameterReader::readFromFile error: file iS3D_parameters.dat does not exist.");
  const int operation = (int)prm.get("operation");
  check(operation == 0 || operation == 1 || operation == 2, "calculate_spectra error: need to set operation = (0, 1, 2)");
  const int mode = (int)prm.get("mode"), dimension = (int)prm.get("dimension"), hrg = (int)prm.get("hrg_eos");
  const int include_baryon = (int)prm.get("include_baryon");
  Surface file_surf;
  Averages avg{};
  const Surface* surf = &mem_;
  if (fo_from_file == 1) {
    const std::string err = read_surface(dir_, mode, dimension, include_baryon, file_surf, avg, true);
    check(err.empty(), err);
    surf = &file_surf;
  } else {
    avg = surface_averages(mem_, 0);            // JETSCAPE path: muB, nB not considered (iS3D.cpp:174-176)
    const std::string err = write_averages_file(dir_, avg);
    check(err.empty(), err);
  }
  if (!opt.quiet) std::printf("Number of freezeout cells = %ld\n", surf->size());
  std::vector<Particle> parts;
  std::string err = read_pdg(dir_, hrg, parts);
  check(err.empty(), err);
  Table chosen, pT, phi, y, eta;
  check(load_table(path_in(dir_, "PDG/chosen_particles.dat"), chosen), "cannot read PDG/chosen_particles.dat");
  DfTablesData df;
  err = read_df_tables(dir_, hrg, df);
  check(err.empty(), err);
  check(load_table(path_in(dir_, "tables/momentum/pT_table.dat"), pT), "cannot read tables/momentum/pT_table.dat");
  check(load_table(path_in(dir_, "tables/momentum/phi_table.dat"), phi), "cannot read tables/momentum/phi_table.dat");
  check(load_table(path_in(dir_, "tables/momentum/y_table.dat"), y), "cannot read tables/momentum/y_table.dat");
  check(load_table(path_in(dir_, "tables/spacetime_rapidity/eta_table.dat"), eta),
        "cannot read tables/spacetime_rapidity/eta_table.dat");
  int galpha = 0, gpts = 0;
  std::vector<double> gr, gw;
  err = read_gauss_laguerre(path_in(dir_, "tables/gauss/gla_roots_weights.txt"), galpha, gpts, gr, gw);
  check(err.empty(), err);
  EmissionFunctionArray efa(prm, chosen, pT, phi, y, eta, parts, *surf, df, avg, gr, gw, galpha, gpts);
  if (operation == 2) {        // EmissionFunction.cpp:1235-1249: the oversampling estimate
    nevents_ = 1;
    if ((int)prm.get("oversample", 0.0)) {
      ntotal_ = efa.estimate_total_yield(opt);
      if (!opt.quiet) std::printf("\nEstimated total particle yield = %ld particles\n", (long)ntotal_);
      nevents_ = (long)std::min(std::ceil(prm.get("min_num_hadrons", 1.0e5) / ntotal_), prm.get("max_num_samples", 1.0e3));
      if (!opt.quiet) std::printf("\nSampling %ld particlization events...\n\n", nevents_);
    } else if (!opt.quiet) {
      std::printf("\nSampling 1 particlization event...\n\n");
    }
    dN_.clear();
    return;
  }
  if (operation == 1) {
    efa.calculate_spectra(opt);
    if (opt.write_files) efa.write_files(dir_);
    if (!opt.quiet) std::printf("\nSpectra calculation took %g seconds\n\n", efa.seconds());
    dN_ = efa.spectra();
  } else {
    efa.calculate_dN_dX(opt);
    if (opt.write_files) efa.write_spacetime_files(dir_);
    if (!opt.quiet) std::printf("\nSpacetime distributions took %g seconds\n\n", efa.seconds());
    const int np = (int)efa.mcid().size();
    const is3d_spacetime_bins b = efa.bins();
    dN_.clear();
    for (int k = 0; k < np; k++) {   // per species [tau bins | r bins | phip bins]
      dN_.insert(dN_.end(), efa.dN_taudtaudy().begin() + (long)k * b.tau_bins, efa.dN_taudtaudy().begin() + (long)(k + 1) * b.tau_bins);
      dN_.insert(dN_.end(), efa.dN_2pirdrdy().begin() + (long)k * b.r_bins, efa.dN_2pirdrdy().begin() + (long)(k + 1) * b.r_bins);
      dN_.insert(dN_.end(), efa.dN_dphidy().begin() + (long)k * b.phip_bins, efa.dN_dphidy().begin() + (long)(k + 1) * b.phip_bins);
    }
  }
}

}  // namespace host
}  // namespace is3d

// ------------------------------------------------------------------------------------------------
// C ABI of the host layer (include/is3d_host.h)
// ------------------------------------------------------------------------------------------------
using namespace is3d::host;

static void put_err(char* buf, int len, const std::string& msg) {
  if (buf && len > 0) { std::strncpy(buf, msg.c_str(), (size_t)len - 1); buf[len - 1] = 0; }
}

static int run_particlization_opt(const char* workdir, RunOptions opt, double* dN_out, long out_capacity, char* err,
                                  int errlen) {
  try {
    IS3D run(workdir ? workdir : ".");
    opt.quiet = true;
    run.run_particlization(1, opt);
    const auto& dN = run.spectra();
    if (dN_out) {
      if ((long)dN.size() > out_capacity) { put_err(err, errlen, "output buffer too small"); return IS3D_ERR_ARG; }
      std::copy(dN.begin(), dN.end(), dN_out);
    }
    return IS3D_OK;
  } catch (const EngineError& ex) {
    put_err(err, errlen, ex.what());
    return ex.code;
  } catch (const std::exception& ex) {
    put_err(err, errlen, ex.what());
    return IS3D_ERR_ARG;
  }
}

extern "C" int is3d_host_run_particlization(const char* workdir, int device, int num_devices, double* dN_out,
                                            long out_capacity, char* err, int errlen) {
  RunOptions opt;
  opt.device = device;
  opt.num_devices = num_devices;
  return run_particlization_opt(workdir, opt, dN_out, out_capacity, err, errlen);
}

extern "C" int is3d_host_run_particlization_devices(const char* workdir, const int* devices, int num_devices,
                                                    double* dN_out, long out_capacity, char* err, int errlen) {
  if (!devices || num_devices <= 0) { put_err(err, errlen, "empty device list"); return IS3D_ERR_ARG; }
  RunOptions opt;
  opt.devices.assign(devices, devices + num_devices);
  return run_particlization_opt(workdir, opt, dN_out, out_capacity, err, errlen);
}

extern "C" int is3d_host_total_yield(const char* workdir, int device, int num_devices, double* n_total,
                                     long* n_events, char* err, int errlen) {
  try {
    IS3D run(workdir ? workdir : ".");
    RunOptions opt;
    opt.device = device;
    opt.num_devices = num_devices;
    opt.quiet = true;
    run.run_particlization(1, opt);
    if (n_total) *n_total = run.total_yield();
    if (n_events) *n_events = run.events();
    return IS3D_OK;
  } catch (const std::exception& ex) {
    put_err(err, errlen, ex.what());
    return IS3D_ERR_ARG;
  }
}

extern "C" long is3d_host_read_surface(const char* workdir, int mode, int dimension, int include_baryon, double* fields,
                                       double* avg5) {
  Surface s;
  Averages a{};
  if (!read_surface(workdir ? workdir : ".", mode, dimension, include_baryon, s, a, false).empty()) return -1;
  const long n = s.size();
  if (fields) {
    const std::vector<double>* f[25] = {&s.tau, &s.x, &s.y, &s.eta, &s.dat, &s.dax, &s.day, &s.dan, &s.ux, &s.uy, &s.un,
                                        &s.E, &s.T, &s.P, &s.pixx, &s.pixy, &s.pixn, &s.piyy, &s.piyn, &s.bulkPi,
                                        &s.muB, &s.nB, &s.Vx, &s.Vy, &s.Vn};
    for (int k = 0; k < 25; k++) std::copy(f[k]->begin(), f[k]->end(), fields + (size_t)k * n);
  }
  if (avg5) { avg5[0] = a.T; avg5[1] = a.E; avg5[2] = a.P; avg5[3] = a.muB; avg5[4] = a.nB; }
  return n;
}

extern "C" int is3d_host_read_pdg(const char* workdir, int hrg_eos, int capacity, long* mcid, double* mass, int* gspin,
                                  int* baryon, int* sign) {
  std::vector<Particle> p;
  if (!read_pdg(workdir ? workdir : ".", hrg_eos, p).empty()) return -1;
  const int n = (int)p.size();
  if (mcid) {
    if (n > capacity) return -2;
    for (int i = 0; i < n; i++) { mcid[i] = p[i].mcid; mass[i] = p[i].mass; gspin[i] = p[i].gspin; baryon[i] = p[i].baryon; sign[i] = p[i].sign; }
  }
  return n;
}

extern "C" int is3d_host_param(const char* path, const char* key, double* value) {
  ParameterReader r;
  if (!r.read_file(path) || !r.has(key)) return -1;
  *value = r.get(key);
  return 0;
}
