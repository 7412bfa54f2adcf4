"""Top-level `modelling` alias of image_compression_amd.modelling, so code written
against the reference (`from modelling import build_model`, engine/trainer.py:248-261;
`from modelling.layers import GDN`, test/test_gdn.py) imports this package unchanged.

The alias installs the real package and each of its submodules under the
`modelling.*` names in sys.modules, so both import paths yield the same module
objects (one set of registries, one class per layer)."""
import importlib
import pkgutil
import sys

import image_compression_amd.modelling as _pkg


def _alias(pkg, name):
    sys.modules[name] = pkg
    for info in pkgutil.iter_modules(pkg.__path__):
        mod = importlib.import_module(f"{pkg.__name__}.{info.name}")
        if info.ispkg:
            _alias(mod, f"{name}.{info.name}")
        else:
            sys.modules[f"{name}.{info.name}"] = mod


_alias(_pkg, __name__)
