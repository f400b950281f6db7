"""Importer for the package directory ``cs566-project-lightglue_amd/``.

The directory name is not a Python identifier, so it cannot be imported with a
plain ``import``.  This module registers it in ``sys.modules`` as
``lightglue_amd``; afterwards ``import lightglue_amd`` (and its submodules)
works normally::

    import lgamd                      # side effect: registers the package
    from lightglue_amd import LightGlue
"""
import importlib.util
import os
import sys

PKG_NAME = "lightglue_amd"
PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cs566-project-lightglue_amd")


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules[PKG_NAME]
        raise
    return mod


lightglue_amd = load()
