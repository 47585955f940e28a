"""MI355X-native low-rank SDP inner solver (drop-in for the LoRADS path of
muhd-umer/ltr-lowrank-sdp).  See DESIGN.md.

Import with ``importlib.import_module("ltr-lowrank-sdp_amd")`` (the directory
name is the project's package name; it is not a Python identifier).
"""
from . import instances  # noqa: F401

__all__ = ["instances", "solver"]


def __getattr__(name):
    if name == "solver":
        from . import solver
        return solver
    raise AttributeError(name)
