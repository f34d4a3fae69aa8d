"""Loader for the in-tree native extension ``_C`` (HIP kernels + C++ runtime).

The extension is built by ``build.py`` (hipcc, ``--offload-arch=gfx950``) into
``distributed-deep-learning_amd/_C.so`` and loaded from there directly — never from a
JIT cache — so the same binary travels to the GPU box.

Policy: on a machine with a GPU the HIP path is mandatory; if the extension is missing
or fails to load, GPU code paths raise instead of silently falling back to eager
PyTorch.  CPU-only code paths (tests, the gloo protocol rehearsal) use the torch oracle.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# DDL_SO: an alternative in-tree build of the same extension (same-box A/B of compile-time
# knobs, e.g. `_C_ab.so` built with DDL_EXTRA_CFLAGS); default the one build.py writes
SO_PATH = os.path.join(_PKG_DIR, os.environ.get("DDL_SO", "_C.so"))

_mod = None
_err: str | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    if not os.path.exists(SO_PATH):
        _err = f"native extension not built: {SO_PATH} missing (run `python build.py`)"
        return None
    try:
        import torch  # noqa: F401  (libtorch symbols must be loaded first)
        loader = importlib.machinery.ExtensionFileLoader("ddl_amd._C", SO_PATH)
        spec = importlib.util.spec_from_file_location("ddl_amd._C", SO_PATH, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        sys.modules["ddl_amd._C"] = mod
        _mod = mod
    except Exception as e:  # pragma: no cover - depends on build state
        _err = f"failed to load {SO_PATH}: {e!r}"
    return _mod


def available() -> bool:
    return _load() is not None


def ops():
    """The loaded extension module; raises if it is unavailable."""
    m = _load()
    if m is None:
        raise RuntimeError(_err)
    return m


def error() -> str | None:
    _load()
    return _err
