"""kopia_amd — MI355X-native content-defined-chunking splitter for Kopia.

The hot path (Kopia's ``repo/splitter``) runs as hand-written gfx950 HIP
kernels in ``libkcdc.so``; see DESIGN.md.  Public Python surface:

* :mod:`kopia_amd.splitter` — mirror of the reference package
  (``SupportedAlgorithms``, ``GetFactory``, ``DefaultAlgorithm``, ``Splitter``).
* :mod:`kopia_amd.batch` — batch entry points (device-resident and host).
"""
from . import _lib  # noqa: F401
from .splitter import DefaultAlgorithm, GetFactory, Splitter, SupportedAlgorithms  # noqa: F401

__all__ = ["DefaultAlgorithm", "GetFactory", "Splitter", "SupportedAlgorithms"]
