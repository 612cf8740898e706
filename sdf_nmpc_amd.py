"""Import shim.

The package source lives in ``./sdf-nmpc_amd/`` (hyphenated directory name, which Python cannot
import by name). ``import sdf_nmpc_amd`` resolves to this file, which loads that directory as the
package ``sdf_nmpc_amd`` and replaces itself in ``sys.modules``.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "sdf-nmpc_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
