"""CPU tests of the drop-in boundary: the C-ABI library loads and exports every symbol the header
declares; no compute calls (there is no GPU here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "accord_amd.h")
LIB = os.path.join(ROOT, "cassandra-accord_amd", "accord_amd", "libaccord_amd.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(acc_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libaccord_amd.so not built (run __graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    names = declared_functions()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_lists_all_exports():
    from accord_amd import _lib
    assert sorted(_lib.EXPORTS) == declared_functions()


def test_version_string():
    lib = ctypes.CDLL(LIB)
    lib.acc_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.acc_version()


def test_library_has_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_create_without_gpu_fails_cleanly():
    """No HIP device here: acc_create must return an error code, not crash."""
    from accord_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    rc = L.acc_create(0, None, ctypes.byref(h))
    if rc == 0:  # a GPU is visible (running on the box): clean up
        L.acc_destroy(h)
    else:
        assert rc in (_lib.ACC_E_ARG, _lib.ACC_E_DEVICE)
