"""CPU tier: the C-ABI library loads and exports every symbol include/is3d_amd.h declares
(no compute calls without a GPU)."""
import ctypes as C
import re

from is3d2_amd import _lib


def declared_symbols():
    hdr = open("include/is3d_amd.h").read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(is3d_[A-Za-z_0-9]+)\s*\(", hdr)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_lib.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version():
    lib = _lib.load()
    assert lib.is3d_abi_version() == 5


def test_build_id_names_the_sources():
    """is3d_build_id() = the Makefile's SRC_ID: a hash of the sources + flags the library was built from."""
    bid = _lib.build_id()
    assert re.fullmatch(r"[0-9a-f]{12}-[0-9a-f]{4}", bid), bid
