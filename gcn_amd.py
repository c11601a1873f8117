"""Import shim for the package directory
``graph-convolutional-networks-for-text-classification_amd/`` (its name is not
a Python identifier).  ``import gcn_amd`` registers it as the module
``graph_convolutional_networks_for_text_classification_amd`` and re-exports
its public API.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "graph-convolutional-networks-for-text-classification_amd")
PKG_NAME = "graph_convolutional_networks_for_text_classification_amd"


def _load():
    mod = sys.modules.get(PKG_NAME)
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(PKG_NAME, os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[PKG_NAME]
        raise
    return mod


pkg = _load()
from graph_convolutional_networks_for_text_classification_amd import *  # noqa: E402,F401,F403
from graph_convolutional_networks_for_text_classification_amd import __all__  # noqa: E402,F401
