"""Drop-in replacement for the reference's ``attention.py`` (MI355X HIP backend).

``import attention`` from main_mp.py / test_model.py (or any caller of the
reference module) resolves here when this repo root is on ``sys.path``.  The
implementation lives in the package directory
``towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd/``
whose name is not a Python identifier, so it is registered as ``aaa_amd``.
"""
import importlib.util
import os
import sys

_DIR = os.path.join(
    os.path.dirname(os.path.abspath(__file__)),
    "towards-interpretable-reinforcement-learning-using-attention-augmented-agents-replication_amd",
)


def _load():
    mod = sys.modules.get("aaa_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "aaa_amd", os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["aaa_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


_pkg = _load()

from aaa_amd.attention import *  # noqa: E402,F401,F403
from aaa_amd.attention import __all__  # noqa: E402,F401
