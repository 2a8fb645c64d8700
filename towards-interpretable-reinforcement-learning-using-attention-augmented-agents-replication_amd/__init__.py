"""MI355X-native attention-augmented agent learner (package ``aaa_amd``).

Registered under the import name ``aaa_amd`` by the repo-root ``attention.py``
shim (the directory name is not a Python identifier).
"""
from . import detinit  # noqa: F401

__version__ = "0.1.0"
