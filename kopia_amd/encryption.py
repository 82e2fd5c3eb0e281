"""Content encryption of chunks on the GPU (C ABI: include/kcdc.h, kcdc_encrypt/decrypt_*),
mirroring Kopia's encryption package for AES256-GCM-HMAC-SHA256 (the default) and
CHACHA20-POLY1305-HMAC-SHA256 (repo/encryption/encryption.go: Encryptor, CreateEncryptor,
SupportedAlgorithms, deriveKey; aes256_gcm_hmac_sha256_encryptor.go;
chacha20_poly1305_hmac_sha256_encryptor.go; aead_helpers.go).  Many chunks per launch; the
content ID's last 16 bytes are the per-content IV (content_manager_lock_free.go:178-182).
No CPU fallback for the byte path: the library must be loaded."""
from __future__ import annotations

import ctypes as C
import hashlib
import hmac
import os

import numpy as np

from . import _lib

ChaCha20Poly1305 = "CHACHA20-POLY1305-HMAC-SHA256"
Aes256Gcm = "AES256-GCM-HMAC-SHA256"
DefaultAlgorithm = Aes256Gcm  # encryption.go DefaultAlgorithm
PurposeEncryptionKey = b"encryption"  # encryption.go purposeEncryptionKey
KeyDerivationSecretSize = 32  # chacha20KeyDerivationSecretSize
NonceSize = 12


def SupportedAlgorithms() -> list[str]:
    arr = (C.c_char_p * 8)()
    n = _lib.lib().kcdc_encryption_algorithms(arr, 8)
    return [arr[i].decode() for i in range(n)]


def overhead(name: str) -> int:
    return _lib.check(_lib.lib().kcdc_encryption_overhead(name.encode()))


def derive_key(master_key: bytes, purpose: bytes = PurposeEncryptionKey, length: int = KeyDerivationSecretSize) -> bytes:
    """deriveKey (encryption.go:80-92): hkdf.Key(sha256.New, masterKey, purpose, "", length).
    Once per repository, on the host, as in the reference."""
    if length < 32:
        raise ValueError(f"derived key must be at least 32 bytes, was {length}")  # minDerivedKeyLength
    prk = hmac.new(purpose, master_key, hashlib.sha256).digest()
    out, t, i = b"", b"", 1
    while len(out) < length:
        t = hmac.new(prk, t + bytes([i]), hashlib.sha256).digest()
        out += t
        i += 1
    return out[:length]


def sealed_layout(lengths, name: str = ChaCha20Poly1305):
    """Offsets (multiples of 4) and total size of a buffer holding every sealed chunk."""
    ov = overhead(name)
    sizes = np.asarray(lengths, dtype=np.int64) + ov
    slots = (sizes + 3) & ~3
    offs = np.concatenate(([0], np.cumsum(slots)[:-1])).astype(np.int64) if len(slots) else np.zeros(0, np.int64)
    return offs, int(slots.sum())


def plain_layout(sealed_lengths, name: str = ChaCha20Poly1305):
    """Offsets (multiples of 4, room for the 4-byte padding) for the opened plaintexts."""
    lens = np.maximum(np.asarray(sealed_lengths, dtype=np.int64) - overhead(name), 0)
    slots = (lens + 3) & ~3
    offs = np.concatenate(([0], np.cumsum(slots)[:-1])).astype(np.int64) if len(slots) else np.zeros(0, np.int64)
    return offs, max(int(slots.sum()), 4)


class Encryptor:
    """CreateEncryptor(Parameters) for the GPU: the batch forms of Encrypt / Decrypt."""

    def __init__(self, name: str, master_key: bytes):
        if name not in SupportedAlgorithms():
            raise _lib.KcdcError(_lib.KCDC_ENOENT, f"unknown encryption algorithm: {name}")
        self.name = name
        self.secret = derive_key(master_key)

    def Overhead(self) -> int:
        return overhead(self.name)

    def _work(self, n, device):
        import torch
        return torch.empty(max(int(_lib.lib().kcdc_crypt_workspace_size(n)), 1), dtype=torch.uint8, device=device)

    def encrypt_chunks_device(self, data_ptr: int, offsets, lengths, d_ivs, iv_stride: int, d_out, out_offsets,
                              device, nonces: bytes | None = None, stream=None, iv_len: int = 16):
        """Seal chunk i = [offsets[i], +lengths[i]) of the device bytes at data_ptr into d_out
        (a device uint8 tensor) at out_offsets[i].  d_ivs: a device tensor holding the content
        IDs, iv_len bytes each at stride iv_stride (the content manager's 16-byte packed IV).
        nonces: 12 bytes per chunk (default os.urandom, as crypto/rand).
        Returns the device int32 status tensor (asynchronous on `stream`)."""
        import torch
        n = len(offsets)
        if stream is None:
            stream = torch.cuda.current_stream(device)
        if nonces is None:
            nonces = os.urandom(NonceSize * n)
        if len(nonces) != NonceSize * n:
            raise ValueError("need 12 nonce bytes per chunk")
        # Every temporary is allocated and filled on `stream` itself, so the kernels below are
        # ordered after those fills whatever the caller's current stream is.  The status words
        # need no fill: the prep kernel writes every status[i].
        with torch.cuda.stream(stream):
            status = torch.empty(max(n, 1), dtype=torch.int32, device=device)
            if n == 0:
                return status[:0]
            d_offs = torch.as_tensor(np.asarray(offsets, dtype=np.int64)).to(device)
            d_lens = torch.as_tensor(np.asarray(lengths, dtype=np.int64)).to(device)
            d_oo = torch.as_tensor(np.asarray(out_offsets, dtype=np.int64)).to(device)
            d_nonce = torch.frombuffer(bytearray(nonces), dtype=torch.uint8).to(device)
            work = self._work(n, device)
        _lib.check(_lib.lib().kcdc_encrypt_chunks_device(
            self.name.encode(), self.secret, len(self.secret), C.c_void_p(data_ptr), d_offs.data_ptr(),
            d_lens.data_ptr(), n, C.c_void_p(d_ivs.data_ptr()), iv_len, iv_stride, d_nonce.data_ptr(), d_out.data_ptr(),
            d_oo.data_ptr(), status.data_ptr(), work.data_ptr(), work.numel(), C.c_void_p(stream.cuda_stream)))
        status._kcdc_keep = (d_offs, d_lens, d_oo, d_nonce, work, d_ivs)  # alive until the caller syncs
        return status[:n]

    def decrypt_chunks_device(self, sealed_ptr: int, offsets, sealed_lengths, d_ivs, iv_stride: int, d_out,
                              out_offsets, device, stream=None, iv_len: int = 16):
        """Open sealed chunk i = [offsets[i], +sealed_lengths[i]) into d_out at out_offsets[i].
        Returns the device int32 status tensor: 0, KCDC_EBADMSG, KCDC_EINVAL or KCDC_EFBIG.

        A chunk whose status is not 0 hands back no plaintext: its d_out slot (sealed length
        - 28 bytes) is zeroed on the device after the tag check, as Go's AEAD.Open returns nil
        on failure (aeadOpenPrefixedWithNonce).  raise_on_status(status) syncs and raises on any
        failed chunk."""
        import torch
        n = len(offsets)
        if stream is None:
            stream = torch.cuda.current_stream(device)
        with torch.cuda.stream(stream):  # temporaries ordered on the kernels' stream (encrypt_chunks_device)
            status = torch.empty(max(n, 1), dtype=torch.int32, device=device)
            if n == 0:
                return status[:0]
            d_offs = torch.as_tensor(np.asarray(offsets, dtype=np.int64)).to(device)
            d_lens = torch.as_tensor(np.asarray(sealed_lengths, dtype=np.int64)).to(device)
            d_oo = torch.as_tensor(np.asarray(out_offsets, dtype=np.int64)).to(device)
            work = self._work(n, device)
        _lib.check(_lib.lib().kcdc_decrypt_chunks_device(
            self.name.encode(), self.secret, len(self.secret), C.c_void_p(sealed_ptr), d_offs.data_ptr(),
            d_lens.data_ptr(), n, C.c_void_p(d_ivs.data_ptr()), iv_len, iv_stride, d_out.data_ptr(), d_oo.data_ptr(),
            status.data_ptr(), work.data_ptr(), work.numel(), C.c_void_p(stream.cuda_stream)))
        status._kcdc_keep = (d_offs, d_lens, d_oo, work, d_ivs)
        return status[:n]


def raise_on_status(status) -> None:
    """Synchronise on a seal/open status tensor and raise KcdcError for the first chunk that
    failed (KCDC_EBADMSG: authentication failed; its output slot must not be used)."""
    st = status.cpu().numpy()
    bad = np.nonzero(st)[0]
    if len(bad):
        i = int(bad[0])
        raise _lib.KcdcError(int(st[i]), f"chunk {i} of {len(st)} failed ({len(bad)} failed in all)")
