"""The reference-side binding (integration/AnisoWrapperMI355X.c, the MEX plugin a
maintainer builds in place of AnisoWrapper.mexa64) compiles against the C ABI
header, and calls only entry points the library exports.  MATLAB is absent, so the
MEX API comes from a declaration-only stub (tests/mex_stub/mex.h)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "AnisoWrapperMI355X.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_mex_shim_compiles_against_header():
    subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "tests", "mex_stub"),
                           SHIM])


def test_mex_shim_ops_and_symbols():
    import aniso_amd

    src = open(SHIM).read()
    ops = set(re.findall(r'!strcmp\(op, "(\w+)"\)', src))
    # the six MEX ops of AnisoWrapper.cpp:10-136 plus aniso.m's block operator
    assert {"new", "delete", "getNodes", "setCoeff", "cache", "mapping"} <= ops
    assert {"forward", "mforward", "blockMatvec"} <= ops
    called = set(re.findall(r"\b(aniso_\w+)\(", src))
    exported = set(aniso_amd.exported_symbols())
    assert called <= exported, called - exported
    lib = aniso_amd.lib()
    for name in called:
        assert hasattr(lib, name), name
