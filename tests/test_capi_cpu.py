"""C-ABI library checks that need no GPU: it loads, exports every symbol the public
headers declare, and the host-side argument/error paths behave like the reference
(acestep_ggml.cpp:108-194, :230-236, :1318-1329)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from acestep_mi355x import LIB_PATH
from acestep_mi355x import capi


def header_symbols(headers=("acestep_ggml.h", "acestep_mi355x.h")):
    syms = set()
    for h in headers:
        text = open(os.path.join(ROOT, "include", h), encoding="utf-8").read()
        syms |= set(re.findall(r"ACE_GGML_API\s+[\w\s\*]*?\b(ace_\w+)\s*\(", text))
    return syms


def test_library_exists_and_exports_header_symbols():
    """The product library exports exactly the public headers' symbols and none of the kernel self-tests; the
    test library (product objects + self-tests) exports both."""
    assert os.path.exists(LIB_PATH), "build the library first (__graft_entry__.build())"
    lib = ctypes.CDLL(LIB_PATH)
    declared = header_symbols()
    assert declared == set(capi.EXPORTED_SYMBOLS)
    for s in declared:
        assert hasattr(lib, s), s
    tests_only = header_symbols(("acestep_mi355x_selftest.h",))
    assert tests_only == set(capi.SELFTEST_SYMBOLS) and not (tests_only & declared)
    for s in tests_only:
        assert not hasattr(lib, s), f"{s}: self-test entry in the product library"
    st = capi.load_selftest_library()
    for s in declared | tests_only:
        assert hasattr(st, s), s


def test_reference_abi_signatures_present():
    declared = header_symbols()
    for s in ("ace_ggml_create", "ace_ggml_destroy", "ace_ggml_last_error", "ace_ggml_load_dit",
              "ace_ggml_dit_forward"):
        assert s in declared


def test_init_params_layout_matches_reference():
    # {int32 n_threads; int32 use_metal; size_t compute_buffer_bytes} = 16 B on x86-64 (acestep_ggml.h:31-35)
    assert ctypes.sizeof(capi.AceInitParams) == 16


def test_create_destroy_and_error_paths_without_gpu():
    lib = capi.load_library()
    ctx = ctypes.c_void_p()
    p = capi.AceInitParams(4, 0, 0)
    assert lib.ace_ggml_create(ctypes.byref(p), ctypes.byref(ctx)) == capi.ACE_GGML_OK
    assert ctx.value
    assert lib.ace_ggml_create(ctypes.byref(p), None) == capi.ACE_GGML_ERR_INVALID_ARG
    assert lib.ace_ggml_last_error(None) == b"ace_ggml_last_error: null context"
    out = np.zeros(64 * 4, np.float32)
    fp = out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    # (!ctx || !out || seq_len <= 0) -> INVALID_ARG without message
    assert lib.ace_ggml_dit_forward(None, None, None, None, None, None, 4, 0, 0.5, 0.5, fp, out.nbytes) == 2
    assert lib.ace_ggml_dit_forward(ctx, None, None, None, None, None, 0, 0, 0.5, 0.5, fp, out.nbytes) == 2
    assert lib.ace_ggml_dit_forward(ctx, None, None, None, None, None, 4, 0, 0.5, 0.5, None, out.nbytes) == 2
    # not loaded -> ERR "dit not loaded"
    assert lib.ace_ggml_dit_forward(ctx, None, None, None, None, None, 4, 0, 0.5, 0.5, fp, out.nbytes) == 1
    assert lib.ace_ggml_last_error(ctx) == b"dit not loaded"
    assert lib.ace_ggml_load_dit(ctx, None) == capi.ACE_GGML_ERR_INVALID_ARG
    assert lib.ace_mi_dit_get_info(ctx, None) == capi.ACE_GGML_ERR_INVALID_ARG
    lib.ace_ggml_destroy(ctx)
    lib.ace_ggml_destroy(None)
