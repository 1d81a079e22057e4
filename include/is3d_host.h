/*
 * is3d_host.h -- C ABI of the C++ host layer (libis3d_host.so): the iS3D2 drop-in
 * workflow around the engine (include/is3d_amd.h).
 *
 *   is3d_host_run_particlization   IS3D::run_particlization(1) for operation = 1 or 0 (iS3D.cpp:81-282)
 *                                  reading <workdir>/iS3D_parameters.dat, input/surface.dat, PDG/,
 *                                  deltaf_coefficients/, tables/ and writing results/continuous/
 *   is3d_host_run_particlization_devices   the same with an explicit device per cell shard
 *   is3d_host_total_yield          IS3D::run_particlization(1) for operation = 2: the oversampling
 *                                  estimate Ntotal / Nevents (EmissionFunction.cpp:1235-1249)
 *   is3d_host_read_surface         FO_data_reader::read_freezeout_surface modes 1/5/6/7 (readindata.cpp:149-731)
 *   is3d_host_read_pdg             PDG_Data::read_resonances                            (readindata.cpp:1217-1252)
 *   is3d_host_param                ParameterReader::getVal                              (ParameterReader.cpp:142-155)
 */
#ifndef IS3D_HOST_H
#define IS3D_HOST_H
#ifdef __cplusplus
extern "C" {
#endif

/* Runs the whole workflow on HIP devices [device, device + num_devices) (cells sharded);
 * dN_out (optional, capacity doubles) receives dN/(pT dpT dphi dy)[species][pT][phi][y] (operation 1)
 * or, per species, [dN_taudtaudy (tau_bins) | dN_2pirdrdy (r_bins) | dN_dphidy (phip_bins)] (operation 0). */
int is3d_host_run_particlization(const char *workdir, int device, int num_devices, double *dN_out,
                                 long out_capacity, char *err, int errlen);
/* As is3d_host_run_particlization with cell shard k on HIP device devices[k] (an index may repeat:
 * several engines on one GPU, e.g. to exercise the sharded path on a one-GPU box).  Returns the
 * engine's is3d_amd.h code (IS3D_ERR_DF_RANGE for the reference's GSL spline abort, ...). */
int is3d_host_run_particlization_devices(const char *workdir, const int *devices, int num_devices, double *dN_out,
                                         long out_capacity, char *err, int errlen);
/* operation = 2 in <workdir>/iS3D_parameters.dat: n_total = the estimated total yield (0 unless
 * oversample = 1), n_events = min(ceil(min_num_hadrons / Ntotal), max_num_samples) (1 without
 * oversampling).  The particle sampler itself is not on this engine's path. */
int is3d_host_total_yield(const char *workdir, int device, int num_devices, double *n_total, long *n_events,
                          char *err, int errlen);
/* Returns the number of cells (or < 0); fields (optional) receives [25][n] in is3d_surface order,
 * avg5 the Plasma averages T, E, P, muB, nB after the 15-digit round trip. */
long is3d_host_read_surface(const char *workdir, int mode, int dimension, int include_baryon, double *fields,
                            double *avg5);
/* Returns the number of particles (or < 0); arrays optional (capacity entries). */
int is3d_host_read_pdg(const char *workdir, int hrg_eos, int capacity, long *mcid, double *mass, int *gspin,
                       int *baryon, int *sign);
int is3d_host_param(const char *path, const char *key, double *value);

#ifdef __cplusplus
}
#endif
#endif
