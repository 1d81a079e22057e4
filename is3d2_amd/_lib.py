"""ctypes binding of libis3d_amd.so (include/is3d_amd.h).

The library is built in-tree by is3d2_amd/csrc/Makefile (or __graft_entry__.build()).
There is no fallback: if the HIP library is missing, importing the engine fails.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IS3D_LIB") or os.path.join(_HERE, "libis3d_amd.so")   # IS3D_LIB: A/B builds only

SURFACE_FIELDS = ["tau", "x", "y", "eta", "dat", "dax", "day", "dan", "ux", "uy", "un", "E", "T", "P",
                  "pixx", "pixy", "pixn", "piyy", "piyn", "bulkPi", "muB", "nB", "Vx", "Vy", "Vn"]

IS3D_OK, IS3D_ERR_ARG, IS3D_ERR_STATE, IS3D_ERR_DEVICE, IS3D_ERR_DF_RANGE, IS3D_ERR_UNSUPPORTED = range(6)

# every symbol include/is3d_amd.h declares
EXPORTS = ["is3d_abi_version", "is3d_build_id", "is3d_create", "is3d_create_devices", "is3d_destroy", "is3d_last_error", "is3d_set_params", "is3d_set_tuning", "is3d_get_tuning",
           "is3d_set_species", "is3d_set_species_classes", "is3d_species_integrated", "is3d_set_pdg", "is3d_set_momentum_grid", "is3d_set_gauss_laguerre",
           "is3d_set_df_tables", "is3d_set_surface", "is3d_set_surface_device", "is3d_set_cell_window", "is3d_cell_costs", "is3d_calculate_spectra",
           "is3d_launch", "is3d_finish", "is3d_get_stats", "is3d_output_size", "is3d_evaluate_df_coefficients",
           "is3d_surface_averages", "is3d_get_jonah_table", "is3d_set_momentum_weights", "is3d_set_spacetime_bins",
           "is3d_calculate_dN_dX", "is3d_get_cell_yields", "is3d_total_yield", "is3d_set_chain_range",
           "is3d_launch_begin", "is3d_chain_passes", "is3d_chain_pass", "is3d_chain_end", "is3d_launch_end",
           "is3d_chain_boundary_size", "is3d_chain_boundary_get", "is3d_chain_boundary_put"]


class Params(C.Structure):
    _fields_ = [("operation", C.c_int), ("dimension", C.c_int), ("df_mode", C.c_int), ("include_baryon", C.c_int),
                ("include_bulk_deltaf", C.c_int), ("include_shear_deltaf", C.c_int),
                ("include_baryondiff_deltaf", C.c_int), ("regulate_deltaf", C.c_int), ("outflow", C.c_int),
                ("famod_chains", C.c_int), ("deta_min", C.c_double), ("mass_pion0", C.c_double)]


class SpacetimeBins(C.Structure):
    _fields_ = [("tau_min", C.c_double), ("tau_max", C.c_double), ("tau_bins", C.c_int),
                ("r_min", C.c_double), ("r_max", C.c_double), ("r_bins", C.c_int), ("phip_bins", C.c_int),
                ("threads", C.c_int)]


class Surface(C.Structure):
    _fields_ = [(k, C.POINTER(C.c_double)) for k in SURFACE_FIELDS]


class Stats(C.Structure):
    _fields_ = [("cells", C.c_long), ("breakdown", C.c_long), ("pl_negative", C.c_long), ("recon_fail", C.c_long),
                ("iterations", C.c_long), ("ms_prepass", C.c_double), ("ms_spectra", C.c_double),
                ("ms_total", C.c_double)]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libis3d_amd.so not built (run `make -C is3d2_amd/csrc` or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    P = C.POINTER
    d = C.c_double
    pd = P(C.c_double)
    lib.is3d_abi_version.restype = C.c_int
    lib.is3d_build_id.restype = C.c_char_p
    lib.is3d_create.restype = C.c_void_p
    lib.is3d_create.argtypes = [C.c_int]
    lib.is3d_create_devices.restype = C.c_void_p
    lib.is3d_create_devices.argtypes = [C.c_int, P(C.c_int)]
    lib.is3d_destroy.argtypes = [C.c_void_p]
    lib.is3d_last_error.restype = C.c_char_p
    lib.is3d_last_error.argtypes = [C.c_void_p]
    lib.is3d_set_params.argtypes = [C.c_void_p, P(Params)]
    lib.is3d_set_tuning.argtypes = [C.c_void_p, C.c_char_p, C.c_long]
    lib.is3d_get_tuning.restype = C.c_long
    lib.is3d_get_tuning.argtypes = [C.c_void_p, C.c_char_p]
    lib.is3d_set_species.argtypes = [C.c_void_p, C.c_int, pd, pd, pd, pd]
    lib.is3d_set_species_classes.argtypes = [C.c_void_p, C.c_int]
    lib.is3d_species_integrated.argtypes = [C.c_void_p]
    lib.is3d_set_pdg.argtypes = [C.c_void_p, C.c_int, pd, pd, pd, pd]
    lib.is3d_set_momentum_grid.argtypes = [C.c_void_p, C.c_int, pd, C.c_int, pd, C.c_int, pd, C.c_int, pd, pd]
    lib.is3d_set_gauss_laguerre.argtypes = [C.c_void_p, C.c_int, C.c_int, pd, pd]
    lib.is3d_set_df_tables.argtypes = [C.c_void_p, C.c_int, C.c_int, pd, pd, pd, d]
    lib.is3d_set_surface.argtypes = [C.c_void_p, C.c_long, P(Surface)]
    lib.is3d_set_surface_device.argtypes = [C.c_void_p, C.c_long, C.c_void_p]
    lib.is3d_set_cell_window.argtypes = [C.c_void_p, C.c_long, C.c_long]
    lib.is3d_cell_costs.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    lib.is3d_calculate_spectra.argtypes = [C.c_void_p, pd]
    lib.is3d_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.is3d_finish.argtypes = [C.c_void_p]
    lib.is3d_get_stats.argtypes = [C.c_void_p, P(Stats)]
    lib.is3d_output_size.restype = C.c_long
    lib.is3d_output_size.argtypes = [C.c_void_p]
    lib.is3d_evaluate_df_coefficients.argtypes = [C.c_void_p, d, d, d, d, d, pd]
    lib.is3d_surface_averages.argtypes = [C.c_long, P(Surface), C.c_int, pd]
    lib.is3d_get_jonah_table.argtypes = [C.c_void_p, pd, pd, pd, pd]
    lib.is3d_set_momentum_weights.argtypes = [C.c_void_p, pd, pd]
    lib.is3d_set_spacetime_bins.argtypes = [C.c_void_p, P(SpacetimeBins)]
    lib.is3d_calculate_dN_dX.argtypes = [C.c_void_p, pd, pd, pd]
    lib.is3d_get_cell_yields.argtypes = [C.c_void_p, pd]
    lib.is3d_total_yield.argtypes = [C.c_void_p, pd, d, pd, pd]
    lib.is3d_set_chain_range.argtypes = [C.c_void_p, C.c_long, C.c_long]
    lib.is3d_launch_begin.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.is3d_chain_passes.argtypes = [C.c_void_p]
    lib.is3d_chain_pass.argtypes = [C.c_void_p, C.c_int]
    lib.is3d_chain_end.argtypes = [C.c_void_p]
    lib.is3d_launch_end.argtypes = [C.c_void_p]
    lib.is3d_chain_boundary_size.restype = C.c_long
    lib.is3d_chain_boundary_size.argtypes = [C.c_void_p]
    lib.is3d_chain_boundary_get.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lib.is3d_chain_boundary_put.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    _lib = lib
    return lib


def build_id():
    """Identity of the loaded libis3d_amd.so (hash of its sources and flags, is3d_build_id())."""
    return load().is3d_build_id().decode()
