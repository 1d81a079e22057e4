// group.h -- private interface between engine.hip's C ABI and the multi-device engine (group.hip).
//
// is3d_create_devices(n, devices) returns an is3d_engine whose `grp` holds one engine per device
// (the multi-GPU fan-out happens inside the compute call).  Every setter is forwarded to
// the shard engines; the surface is split into contiguous cell windows balanced by estimated cost; one
// compute call launches every shard on its own device and stream, then sums the per-device spectra with
// one RCCL ncclAllReduce (ncclFloat64, ncclSum) over the device-resident outputs (xGMI), or -- when the
// device list repeats a GPU, which one RCCL communicator cannot hold -- with peer copies and a fixed-order
// add on the first device.
#pragma once
#include <string>

#include "../../include/is3d_amd.h"

namespace is3d {
struct Group;
// shard cost of a cell with u.dsigma <= 0 (skipped by every kernel, MomentumSpectra.cpp:132): its record prep only
constexpr double kSkipCost = 0.02;

Group* group_create(int n, const int* devices, std::string& err);
void group_destroy(Group* g);
const char* group_error(const Group* g);

int group_set_params(Group* g, const is3d_params* p);
int group_set_tuning(Group* g, const char* key, long value);
long group_get_tuning(const Group* g, const char* key);   // shard 0's value; "phitab_chunks": the max over shards
int group_set_species(Group* g, int n, const double* mass, const double* sign, const double* degen, const double* baryon);
int group_set_species_classes(Group* g, int on);
int group_species_integrated(Group* g);
// record an error on the group (is3d_last_error of a device-list engine reads the group's message)
int group_fail(Group* g, int code, const char* msg);
int group_set_pdg(Group* g, int n, const double* mass, const double* sign, const double* degen, const double* baryon);
int group_set_momentum_grid(Group* g, int npT, const double* pT, int nphi, const double* phi, int ny, const double* y,
                            int neta, const double* eta, const double* eta_w);
int group_set_momentum_weights(Group* g, const double* pT_w, const double* phi_w);
int group_set_spacetime_bins(Group* g, const is3d_spacetime_bins* b);
int group_set_gauss_laguerre(Group* g, int alpha, int points, const double* roots, const double* weights);
int group_set_df_tables(Group* g, int nT, int nmuB, const double* T, const double* muB, const double* tables, double T_avg);
int group_set_surface(Group* g, long n, const is3d_surface* s);
int group_set_surface_device(Group* g, long n, const double* dev_fields);
int group_launch(Group* g, double* dev_out, void* stream);
int group_finish(Group* g);
int group_calculate_spectra(Group* g, double* dN_out);
int group_calculate_dN_dX(Group* g, double* tau, double* r, double* phi);
int group_get_cell_yields(const Group* g, double* dN_dy_cell);
int group_get_stats(const Group* g, is3d_stats* out);
long group_output_size(const Group* g);
int group_evaluate_df_coefficients(Group* g, double T, double muB, double E, double P, double bulkPi, double* out15);
int group_total_yield(Group* g, const double* plasma, double y_cut, double* n_total, double* densities);
int group_get_jonah_table(const Group* g, double* l2, double* z, double* bp, double* bpmax);
}  // namespace is3d

// engine.hip internals the group uses on its shard engines (not part of the public ABI)
// staged launch (engine.hip launch_begin / chain_pass / chain_end / launch_end): a shard solves positions
// [q0, q1) of PTMA's warm-start chains (q1 < 0: the whole chains), its first segments starting from the end
// states the previous shard pushes into its boundary slots (has_pred)
int is3d_internal_launch_begin(is3d_engine* e, double* dev_out, void* stream, long q0, long q1, int has_pred);
int is3d_internal_chain_pass(is3d_engine* e, int pass);
int is3d_internal_chain_end(is3d_engine* e);
int is3d_internal_launch_end(is3d_engine* e);
int is3d_internal_chain_npass(const is3d_engine* e);
double* is3d_internal_chain_bnd(is3d_engine* e, int out, int slot);
long is3d_internal_chain_bnd_bytes(const is3d_engine* e);
extern "C" {
// engine-owned copy of cells [lo, lo + n) of a field-major device surface (25 x src_n doubles) on src_device
int is3d_internal_copy_surface(is3d_engine* e, long n, const double* src, long src_n, int src_device, long lo);
}
