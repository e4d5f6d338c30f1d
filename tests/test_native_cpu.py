"""CPU-side checks of the native boundary: the C-ABI library exists, loads
and exports every symbol include/dccrgx.h declares (no compute calls)."""
import ctypes
import os

import pytest

import dccrg_amd
from dccrg_amd import build as B


def test_library_is_built_for_gfx950():
    path = B.build()
    assert os.path.exists(path)
    data = open(path, "rb").read()
    assert b"gfx950" in data


def test_every_declared_symbol_is_exported():
    L = dccrg_amd.lib()
    syms = dccrg_amd.header_symbols()
    assert len(syms) > 50
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version_and_error_string():
    L = dccrg_amd.lib()
    assert L.dccrgx_abi_version() == 10
    assert isinstance(L.dccrgx_last_error(), bytes)


def test_null_grid_is_rejected_without_gpu():
    L = dccrg_amd.lib()
    assert L.dccrgx_initialize(None) == dccrg_amd._lib.EINVAL
    assert b"null grid" in L.dccrgx_last_error()


def test_no_oracle_in_product():
    """The product never imports or links the oracle."""
    root = os.path.dirname(os.path.abspath(dccrg_amd.__file__))
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(dp, f), errors="ignore").read()
                assert "oracle" not in txt.replace("oracle's", ""), f
