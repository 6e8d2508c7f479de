"""C-ABI checks that need no GPU: the kernel library builds for gfx950, loads, and exports
every entry point include/ducosy_hip.h declares; the ctypes mirrors (lib.SIGNATURES,
lib.ConvDesc) agree with the header as compiled by the C compiler."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ducosy_hip.h")
PKG = os.path.join(ROOT, "ducosy-gan_amd")


def _header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dcs_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def libso():
    from modules.hip import lib
    if not os.path.isfile(lib.LIB_PATH):
        subprocess.run(["make", "-C", PKG, f"-j{min(8, os.cpu_count() or 1)}"], check=True,
                       stdout=subprocess.DEVNULL, timeout=1200)
    return lib


def test_header_declares_the_bound_functions():
    from modules.hip import lib
    assert _header_functions() == lib.exported_symbols()


def test_library_exports_every_header_symbol(libso):
    so = ctypes.CDLL(libso.LIB_PATH)
    missing = [f for f in _header_functions() if not hasattr(so, f)]
    assert not missing, missing
    libso.load()  # binds restype/argtypes for every symbol
    assert libso.load().dcs_version() >= 1


def test_library_is_gfx950_code():
    """The shared object's offload bundle holds a gfx950 code object (and only that target)."""
    from modules.hip import lib
    if not os.path.isfile(lib.LIB_PATH):
        pytest.skip("library not built")
    blob = open(lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_conv_desc_layout_matches_c(tmp_path):
    """offsetof/sizeof of dcs_conv_desc from gcc == the ctypes Structure used by the host."""
    from modules.hip.lib import ConvDesc
    names = [f for f, _ in ConvDesc._fields_]
    src = tmp_path / "layout.c"
    body = "\n".join(f'  printf("{n} %zu\\n", offsetof(dcs_conv_desc, {n}));' for n in names)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ducosy_hip.h"\nint main(void){\n'
                   + body + '\n  printf("sizeof %zu\\n", sizeof(dcs_conv_desc));\n  return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if line)
    for n in names:
        assert int(got[n]) == getattr(ConvDesc, n).offset, n
    assert int(got["sizeof"]) == ctypes.sizeof(ConvDesc)


def test_missing_library_fails_loudly(monkeypatch):
    """No CPU fallback: a missing kernel library raises HipLibraryError on first use."""
    from modules.hip import lib
    monkeypatch.setattr(lib, "_lib", None)
    monkeypatch.setattr(lib, "LIB_PATH", "/nonexistent/libducosy_hip.so")
    with pytest.raises(lib.HipLibraryError):
        lib.load()


def test_gl_job_layout_matches_c(tmp_path):
    """offsetof/sizeof of dcs_gl_job (the fused loss kernel's job record) == lib.GLJob."""
    from modules.hip.lib import GLJob
    names = [f for f, _ in GLJob._fields_]
    src = tmp_path / "gl.c"
    body = "\n".join(f'  printf("{n} %zu\\n", offsetof(dcs_gl_job, {n}));' for n in names)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "ducosy_hip.h"\nint main(void){\n'
                   + body + '\n  printf("sizeof %zu\\n", sizeof(dcs_gl_job));\n  return 0;\n}\n')
    exe = tmp_path / "gl"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.split("\n") if line)
    for n in names:
        assert int(got[n]) == getattr(GLJob, n).offset, n
    assert int(got["sizeof"]) == ctypes.sizeof(GLJob)


def test_integration_md_export_count():
    """INTEGRATION.md states the number of extern "C" entry points the library exports."""
    from modules.hip import lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"The library exports (\d+) `extern \"C\"` functions", text)
    assert m, "INTEGRATION.md: export count sentence missing"
    assert int(m.group(1)) == len(lib.exported_symbols())
