"""Import name for the framework package.

The source tree lives in ``distributed-deep-learning_amd/`` (a directory name that is
not a valid Python identifier).  This shim makes it importable as ``ddl_amd``: it
points the package search path at that directory and runs its ``__init__``.
"""
import os as _os

_SRC = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                     "distributed-deep-learning_amd")
__path__ = [_SRC]  # noqa: F811 - submodules resolve inside the real source dir
__file__ = _os.path.join(_SRC, "__init__.py")
with open(__file__, "r") as _f:
    exec(compile(_f.read(), __file__, "exec"))
