"""ctypes binding of libmmre_base.so, the Base.so-compatible C ABI (include/mmre_base.h).

`load()` returns the library with the argtypes/restypes the reference's Tester declares
(OpenKE/openke/config/Tester.py:20-36) plus those its data loaders need for `sampling`
(Base.cpp:161-174). The reference's own Tester runs against it by pointing `base_file` at
BASE_PATH instead of release/Base.so.
"""
from __future__ import annotations

import ctypes
import os

from ._lib import LIB_DIR, MMREError

BASE_PATH = os.environ.get("MMRE_BASE_LIB") or os.path.join(LIB_DIR, "libmmre_base.so")

_P, _I, _F, _B = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_bool
SIGNATURES = {
    "setInPath": (None, [ctypes.c_char_p]), "setOutPath": (None, [ctypes.c_char_p]),
    "setTrainPath": (None, [ctypes.c_char_p]), "setValidPath": (None, [ctypes.c_char_p]),
    "setTestPath": (None, [ctypes.c_char_p]), "setEntPath": (None, [ctypes.c_char_p]),
    "setRelPath": (None, [ctypes.c_char_p]),
    "setWorkThreads": (None, [_I]), "getWorkThreads": (_I, []), "setBern": (None, [_I]),
    "getEntityTotal": (_I, []), "getRelationTotal": (_I, []), "getTripleTotal": (_I, []),
    "getTrainTotal": (_I, []), "getTestTotal": (_I, []), "getValidTotal": (_I, []),
    "randReset": (None, []), "importTrainFiles": (None, []), "importTestFiles": (None, []),
    "importTypeFiles": (None, []), "importProb": (None, [_F]),
    "sampling": (None, [_P, _P, _P, _P, _I, _I, _I, _I, _B, _B, _B]),
    "initTest": (None, []), "getHeadBatch": (None, [_P, _P, _P]), "getTailBatch": (None, [_P, _P, _P]),
    "testHead": (None, [_P, _I, _I]), "testTail": (None, [_P, _I, _I]),
    "test_link_prediction": (None, [_I]),
    "getTestLinkHit10": (_F, [_I]), "getTestLinkHit3": (_F, [_I]), "getTestLinkHit1": (_F, [_I]),
    "getTestLinkMR": (_F, [_I]), "getTestLinkMRR": (_F, [_I]),
    "mmre_base_last_error": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]), "mmre_base_clear_error": (None, []),
    "mmre_base_set_error_mode": (None, [ctypes.c_int]),
}

_base = None


def load(latch_errors: bool | None = None):
    """Load libmmre_base.so once (after libmmre_hip.so, which it links). This binding checks
    for errors (check()), so its FIRST load switches the library to the latched error mode; later
    calls leave the mode alone unless latch_errors is given explicitly. The mode is global to the
    process: a reference Tester that opens the same libmmre_base.so over ctypes.CDLL in a process
    where mmre.base was loaded sees latched errors too -- load(latch_errors=False) restores abort
    (INTEGRATION.md §C)."""
    global _base
    first = _base is None
    if first:
        if not os.path.exists(BASE_PATH):
            raise MMREError(f"{BASE_PATH} is missing: build it with __graft_entry__.build()")
        from ._lib import lib
        lib()  # resolve libmmre_hip.so first
        L = ctypes.CDLL(BASE_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _base = L
    if latch_errors is not None or first:
        _base.mmre_base_set_error_mode(1 if (latch_errors is None or latch_errors) else 0)
    return _base


def last_error():
    """(code, message) of the latched error (0, '' when none)."""
    buf = ctypes.create_string_buffer(512)
    code = int(load().mmre_base_last_error(buf, len(buf)))
    return code, buf.value.decode(errors="replace")


def check():
    """Raise MMREError for a latched error (and clear the latch)."""
    code, msg = last_error()
    if code:
        load().mmre_base_clear_error()
        raise MMREError(f"libmmre_base: {msg} (code {code})")
