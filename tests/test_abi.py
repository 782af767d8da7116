"""CPU: the C-ABI library builds, loads without a GPU and exports every entry point
declared in include/eg_hip.h; argument validation needs no device."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def header_functions():
    src = (ROOT / "include" / "eg_hip.h").read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(eg_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__
    __graft_entry__.build_hip()
    from electionguard.core import native
    return native.load()


def test_exports_every_declared_symbol(lib):
    from electionguard.core import native
    declared = header_functions()
    assert declared == sorted(native.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name


def test_version_and_errors_without_gpu(lib):
    buf = ctypes.create_string_buffer(128)
    assert lib.eg_version(buf, 128) == 0
    assert b"gfx950" in buf.value and b"limbs=144" in buf.value and b"radix2^29" in buf.value
    out = ctypes.c_void_p()
    even_p = bytes(511) + b"\x02"
    rc = lib.eg_ctx_create(even_p, bytes(32), bytes(512), 0, ctypes.byref(out))
    assert rc == 4 and b"odd" in lib.eg_last_error()          # EG_ERR_MODULUS before any HIP call
    small_p = bytes(511) + b"\x03"
    assert lib.eg_ctx_create(small_p, bytes(32), bytes(512), 0, ctypes.byref(out)) == 4
    assert lib.eg_powp_batch(None, None, None, None, 0) == 1   # EG_ERR_ARG
    assert lib.eg_ctx_destroy(None) == 0


def test_product_path_fails_loudly_without_library(tmp_path):
    from electionguard.core import native
    with pytest.raises(native.NativeUnavailable):
        native.load(tmp_path / "missing.so")
