"""ctypes binding of the C++ host layer (libis3d_host.so, include/is3d_host.h)."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libis3d_host.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libis3d_host.so not built (make -C is3d2_amd/csrc/host)")
        lib = C.CDLL(LIB_PATH)
        PD, PL, PI = C.POINTER(C.c_double), C.POINTER(C.c_long), C.POINTER(C.c_int)
        lib.is3d_host_run_particlization.argtypes = [C.c_char_p, C.c_int, C.c_int, PD, C.c_long, C.c_char_p, C.c_int]
        lib.is3d_host_run_particlization_devices.argtypes = [C.c_char_p, PI, C.c_int, PD, C.c_long, C.c_char_p,
                                                             C.c_int]
        lib.is3d_host_read_surface.restype = C.c_long
        lib.is3d_host_read_surface.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, PD, PD]
        lib.is3d_host_read_pdg.argtypes = [C.c_char_p, C.c_int, C.c_int, PL, PD, PI, PI, PI]
        lib.is3d_host_param.argtypes = [C.c_char_p, C.c_char_p, PD]
        lib.is3d_host_total_yield.argtypes = [C.c_char_p, C.c_int, C.c_int, PD, PL, C.c_char_p, C.c_int]
        _lib = lib
    return _lib


def read_surface(workdir, mode, dimension, include_baryon):
    lib = load()
    n = lib.is3d_host_read_surface(workdir.encode(), mode, dimension, include_baryon, None, None)
    if n < 0:
        raise RuntimeError("surface read failed")
    f = np.zeros(25 * n)
    avg = np.zeros(5)
    lib.is3d_host_read_surface(workdir.encode(), mode, dimension, include_baryon,
                               f.ctypes.data_as(C.POINTER(C.c_double)), avg.ctypes.data_as(C.POINTER(C.c_double)))
    return f.reshape(25, n), avg


def read_pdg(workdir, hrg_eos):
    lib = load()
    n = lib.is3d_host_read_pdg(workdir.encode(), hrg_eos, 0, None, None, None, None, None)
    if n < 0:
        raise RuntimeError("pdg read failed")
    mc = np.zeros(n, dtype=np.int64); m = np.zeros(n); g = np.zeros(n, dtype=np.int32)
    b = np.zeros(n, dtype=np.int32); s = np.zeros(n, dtype=np.int32)
    lib.is3d_host_read_pdg(workdir.encode(), hrg_eos, n, mc.ctypes.data_as(C.POINTER(C.c_long)),
                           m.ctypes.data_as(C.POINTER(C.c_double)), g.ctypes.data_as(C.POINTER(C.c_int)),
                           b.ctypes.data_as(C.POINTER(C.c_int)), s.ctypes.data_as(C.POINTER(C.c_int)))
    return dict(mcid=mc, mass=m, gspin=g, baryon=b, sign=s)


def param(path, key):
    v = C.c_double()
    if load().is3d_host_param(path.encode(), key.encode(), C.byref(v)):
        raise KeyError(key)
    return v.value


class HostError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


def run_particlization(workdir, out_size, device=0, num_devices=1):
    """IS3D::run_particlization on devices [device, device + num_devices); returns the spectra."""
    lib = load()
    out = np.zeros(out_size)
    err = C.create_string_buffer(512)
    rc = lib.is3d_host_run_particlization(workdir.encode(), device, num_devices,
                                          out.ctypes.data_as(C.POINTER(C.c_double)), out_size, err, 512)
    if rc:
        raise HostError(rc, err.value.decode())
    return out


def run_particlization_devices(workdir, out_size, devices):
    """The same with cell shard k on devices[k] (indices may repeat)."""
    lib = load()
    out = np.zeros(out_size)
    err = C.create_string_buffer(512)
    dv = np.ascontiguousarray(devices, dtype=np.int32)
    rc = lib.is3d_host_run_particlization_devices(workdir.encode(), dv.ctypes.data_as(C.POINTER(C.c_int)), len(dv),
                                                  out.ctypes.data_as(C.POINTER(C.c_double)), out_size, err, 512)
    if rc:
        raise HostError(rc, err.value.decode())
    return out


def total_yield(workdir, device=0, num_devices=1):
    """operation = 2 in the run directory: (Ntotal, Nevents) of the oversampling estimate."""
    lib = load()
    nt, ne = C.c_double(), C.c_long()
    err = C.create_string_buffer(512)
    rc = lib.is3d_host_total_yield(workdir.encode(), device, num_devices, C.byref(nt), C.byref(ne), err, 512)
    if rc:
        raise RuntimeError(err.value.decode())
    return nt.value, ne.value
