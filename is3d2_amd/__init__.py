"""is3d2_amd -- MI355X-native Cooper-Frye continuous-spectra engine (iS3D2 operation = 1).

Product: libis3d_amd.so (HIP kernels for gfx950 + C ABI, include/is3d_amd.h).  This
package is the Python host binding used by tests and bench.py; the C++ host layer
(iS3D driver, readers, writers) lives in is3d2_amd/csrc/host.
"""
from . import data, hrg, synth  # noqa: F401
from .engine import Engine, IS3DError, build_engine, make_spec, output_shape, surface_averages  # noqa: F401
