"""Import alias: ``import mfl_amd`` loads the package in
``mobile-federated-learning_amd/`` (a directory name that is not a valid
Python identifier) and registers it under this module's name."""
import importlib.util as _ilu
import pathlib as _pl
import sys as _sys

_PKG_DIR = _pl.Path(__file__).resolve().parent / "mobile-federated-learning_amd"
_spec = _ilu.spec_from_file_location(__name__, _PKG_DIR / "__init__.py",
                                     submodule_search_locations=[str(_PKG_DIR)])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
