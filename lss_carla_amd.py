"""Import shim: exposes the ``lss-carla_amd/`` directory as the package ``lss_carla_amd``.

A hyphen is not legal in a Python module name, so this file loads the
directory's ``__init__.py`` as a package and replaces itself in
``sys.modules``; submodules (``lss_carla_amd.models`` ...) then resolve through
the package ``__path__`` as usual.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "lss-carla_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
