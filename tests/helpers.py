"""Shared test helpers: oracle/emulator bindings and parity metrics."""
import ctypes as C
import os
import subprocess

import numpy as np

from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_SRC = os.path.join(HERE, "native", "cf_emulator.cpp")
EMU_LIB = os.path.join(HERE, "native", "libcf_emulator.so")


def emulator():
    """Host build of the kernels' math (test-only), see tests/native/cf_emulator.cpp."""
    srcs = [EMU_SRC] + [os.path.join(HERE, "..", p) for p in (
        "is3d2_amd/csrc/cf_math.h", "is3d2_amd/csrc/aniso_math.h", "is3d2_amd/csrc/spline_host.h")]
    if not os.path.exists(EMU_LIB) or any(os.path.getmtime(s) > os.path.getmtime(EMU_LIB) for s in srcs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", EMU_LIB, EMU_SRC])
    lib = C.CDLL(EMU_LIB)
    return lib


def emu_spectra(spec, surf, chains=1, T_avg=None, op=1, variant=0):
    """op = 1: spectra [species][pT][phi][y]; op = 0: dN_dy_cell [species][cell].  variant bits: 1 = the
    F_TB table algebra (Grad / RTA-CE without baryon), 2 = Boltzmann-tail lanes (cf_emulator.cpp)."""
    lib = emulator()
    inp = O._Inputs(spec, surf, T_avg, 1)
    p = spec["params"]
    ny = len(spec["y"]) if p["dimension"] == 3 else 1
    if op == 0:
        out = np.zeros(len(spec["species"]["mass"]) * len(surf["tau"]))
    else:
        out = np.zeros(len(spec["species"]["mass"]) * len(spec["pT"]) * len(spec["phi"]) * ny)
    st = (C.c_long * 4)()
    rc = lib.emu_spectra_v(C.byref(inp.params), C.byref(inp.setup), C.byref(inp.surf), int(chains), int(op),
                           O._p(out), st, int(variant))
    if rc:
        raise RuntimeError("emulator rc=%d" % rc)
    return out, list(st)


def parity(got, ref, floor=1e-300):
    """max |got-ref|/|ref| over |ref| > floor, and the underflow-zone counts."""
    got = np.asarray(got); ref = np.asarray(ref)
    m = np.abs(ref) > floor
    rel = np.abs(got[m] - ref[m]) / np.abs(ref[m]) if m.any() else np.zeros(1)
    return float(rel.max()), int((~m).sum()), int((np.abs(got) <= floor).sum())


def rel_quantile(got, ref, q=0.99, floor=1e-300):
    """q-quantile of |got-ref|/|ref| over |ref| > floor: a drift guard far below the max-error bar (typical
    errors are ~1e-13, the 1e-8 bar sits 1e4-1e5x above them)."""
    got = np.asarray(got); ref = np.asarray(ref)
    m = np.abs(ref) > floor
    if not m.any():
        return 0.0
    return float(np.quantile(np.abs(got[m] - ref[m]) / np.abs(ref[m]), q))
