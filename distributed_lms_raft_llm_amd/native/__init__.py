"""Native (C++) host runtime pieces, built in-tree into ``native/_lib/libdlms_native.so``:
the GPT-2 byte-level BPE and BERT WordPiece tokenizers (``csrc/tokenizers.cpp``).
Loaded with ctypes; no Python fallback."""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from pathlib import Path

_HERE = Path(__file__).resolve().parent
CSRC = _HERE / "csrc"
LIB_DIR = _HERE / "_lib"
LIB_PATH = LIB_DIR / "libdlms_native.so"
SOURCES = ["tokenizers.cpp"]

_lock = threading.Lock()
_lib = None


def needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    return any((CSRC / s).stat().st_mtime > t for s in SOURCES)


def build(force: bool = False, verbose: bool = False) -> Path:
    if not force and not needs_build():
        return LIB_PATH
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = LIB_PATH.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-o", str(tmp)] + [str(CSRC / s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if needs_build():
                build()
            L = ctypes.CDLL(str(LIB_PATH))
            P, I, C = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
            IP = ctypes.POINTER(ctypes.c_int)
            for name, args, res in [
                ("dlms_bpe_create", [C, C], P), ("dlms_bpe_is_synthetic", [P], I), ("dlms_bpe_vocab_size", [P], I),
                ("dlms_bpe_set_synthetic_words", [P, I], I),
                ("dlms_bpe_encode", [P, C, I, IP, I], I), ("dlms_bpe_decode", [P, IP, I, C, I], I),
                ("dlms_bpe_destroy", [P], None), ("dlms_wp_create", [C, I], P),
                ("dlms_wp_encode", [P, C, I, I, I, IP, I], I), ("dlms_wp_special", [P, I], I),
                ("dlms_wp_destroy", [P], None),
            ]:
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            _lib = L
    return _lib
