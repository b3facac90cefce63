"""Import alias for the ``distributed-learning_amd/`` package directory.

The package directory name carries a hyphen (it mirrors the upstream repository name), which
Python cannot import directly.  Importing this module loads that directory as the package
``distributed_learning_amd`` and replaces itself in ``sys.modules``, so

    from distributed_learning_amd.utils.consensus_simple import Mixer

works from the repository root exactly like an ordinary package import.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "distributed-learning_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
