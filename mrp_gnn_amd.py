"""Import alias: ``import mrp_gnn_amd`` loads the package in ``multi-robot-perception-gnn-1_amd/``
(a directory name with hyphens cannot be imported directly).  The alias replaces itself in
``sys.modules`` with the real package, so ``mrp_gnn_amd.graph`` etc. resolve normally."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "multi-robot-perception-gnn-1_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_PKG_DIR, "__init__.py"),
                                               submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
