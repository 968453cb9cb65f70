"""CPU-side checks of the C-ABI library: it builds, loads, exports every symbol the header
declares, and fails cleanly (an error code, no crash) when no GPU is present."""
import ctypes
import os
import re

import pytest

from wavernn_amd import _native as nat
from wavernn_amd import build as hbuild

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "wavernn_amd.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(wrnn_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    hbuild.build(verbose=False)
    return nat.lib()


def test_header_declares_expected_api():
    assert declared_functions() == sorted(nat.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name


def _header_fields(struct_name):
    """(type, name) of the fields of `typedef struct {...} struct_name;` in include/wavernn_amd.h"""
    import re
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                             "wavernn_amd.h")).read()
    body = re.search(r"typedef struct \{([^{}]*)\}\s*" + struct_name + ";", text).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"(\w+)\s*\*?\s*(\w+);", body)


def test_struct_layouts_match_header():
    for struct, ct in (("wrnn_config", nat.Config), ("wrnn_info", nat.Info)):
        fields = _header_fields(struct)
        assert [n for _, n in fields] == [n for n, _ in ct._fields_], struct
        assert all(t == "int32_t" for t, _ in fields)
        assert ctypes.sizeof(ct) == 4 * len(fields)
    assert ctypes.sizeof(nat.Tensor) == 8 + 8 + 8 + 8


def test_bad_arguments_are_rejected_without_gpu(lib):
    h = ctypes.c_void_p()
    cfg = nat.Config(999, nat.MODE_MOL, 512, 512, 32, 80, 30, 0, 0)   # wrong ABI version
    assert lib.wrnn_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1
    assert lib.wrnn_create(None, 0, ctypes.byref(h)) == -1
    assert lib.wrnn_last_error(None) == b"null handle"
    lib.wrnn_destroy(None)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_create_reports_missing_gpu(lib):
    from wavernn_amd.loop import FatchordLoop
    with pytest.raises(nat.WrnnError) as e:
        FatchordLoop("MOL", 512, 512, 32, 80, 30)
    assert e.value.code in (-2, -6)


def test_unsupported_dims_fail_loudly(lib):
    h = ctypes.c_void_p()
    cfg = nat.Config(nat.ABI_VERSION, nat.MODE_MOL, 510, 512, 32, 80, 30, 0, 0)   # rnn_dims % 4 != 0
    rc = lib.wrnn_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc == -6 and b"multiples of 4" in lib.wrnn_last_error(h)
    lib.wrnn_destroy(h)
