"""kopia_amd — MI355X-native content-defined-chunking splitter for Kopia.

The hot path (Kopia's ``repo/splitter``) runs as hand-written gfx950 HIP
kernels in ``libkcdc.so``; see DESIGN.md.  Public Python surface:

* :mod:`kopia_amd.splitter` — mirror of the reference package
  (``SupportedAlgorithms``, ``GetFactory``, ``DefaultAlgorithm``, ``Splitter``).
* :mod:`kopia_amd.batch` — batch entry points (device-resident and host).
* :mod:`kopia_amd.hashing` — keyed BLAKE2 content hashes of many chunks on the device
  (``repo/hashing``; ``DefaultAlgorithm`` = ``BLAKE2B-256-128``).
* :mod:`kopia_amd.encryption` — ``AES256-GCM-HMAC-SHA256`` (the default) and
  ``CHACHA20-POLY1305-HMAC-SHA256`` seal/open of many chunks (``repo/encryption``;
  ``Encryptor``, ``SupportedAlgorithms``, ``derive_key``).
* :mod:`kopia_amd.compression` — ``deflate-*``, ``gzip*`` and ``pgzip*`` compression of many
  chunks with the content manager's keep-or-drop rule (``repo/compression``; ``Compressor``).
"""
from . import _lib  # noqa: F401
from . import compression, encryption, hashing  # noqa: F401
from .splitter import DefaultAlgorithm, GetFactory, Splitter, SupportedAlgorithms  # noqa: F401

__all__ = ["DefaultAlgorithm", "GetFactory", "Splitter", "SupportedAlgorithms", "compression", "encryption", "hashing"]
