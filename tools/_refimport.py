"""Import helper for the upstream reference (runs ONLY in the build container).

The reference's `modelling/` package needs `yacs.config.CfgNode` (through
`utils/config.py`) and `utils.Registry`.  `yacs` is not installed here, so an
in-memory stand-in for the CfgNode *container type* (a dict with attribute
access and `clone`) is registered before import.  Nothing under
/root/reference is modified; it is only put on `sys.path`.

This module is test/fixture tooling: nothing in the product package imports
it, and it is never shipped to or run on the GPU box (tests skip it when
/root/reference is absent).
"""
import copy
import os
import sys
import types

REF_ROOT = "/root/reference"


class _CfgNode(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def clone(self):
        return copy.deepcopy(self)


def available() -> bool:
    return os.path.isdir(os.path.join(REF_ROOT, "modelling"))


def import_reference():
    """Return (modelling, get_cfg_defaults) from the reference tree."""
    if not available():
        raise RuntimeError("reference tree not present")
    if "yacs" not in sys.modules:
        m = types.ModuleType("yacs")
        mc = types.ModuleType("yacs.config")
        mc.CfgNode = _CfgNode
        m.config = mc
        sys.modules["yacs"] = m
        sys.modules["yacs.config"] = mc
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import modelling  # noqa: E402  (reference package)
    from utils.config import get_cfg_defaults  # noqa: E402
    return modelling, get_cfg_defaults
