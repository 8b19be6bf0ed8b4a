"""Import alias for the package directory ``depth-aware-shader-effects-for-nerf_amd/``.

The directory name carries hyphens (the repo layout fixes it), so it cannot be
imported by name.  ``import nerfmi`` executes this file, which loads that
directory as the package ``nerfmi`` and replaces itself in ``sys.modules``;
``from nerfmi.render import volume_render`` and friends then resolve through
the package's ``__path__`` as usual.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "depth-aware-shader-effects-for-nerf_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"),
    submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
