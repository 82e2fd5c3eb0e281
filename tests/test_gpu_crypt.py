"""GPU: content encryption of many chunks (kcdc_encrypt/decrypt_chunks_device) with both device
encryptors, CHACHA20-POLY1305-HMAC-SHA256 and AES256-GCM-HMAC-SHA256 (Kopia's default), bit-exact
against the oracles (oracle/aead.py, pinned by RFC 8439 / RFC 5869 vectors in
tests/test_aead_oracle.py; oracle/aesgcm.py, pinned by FIPS-197 / GCM vectors in
tests/test_aesgcm_oracle.py): random lengths across the 16-byte,
64-byte and 4 KiB unit boundaries, misaligned plaintext offsets, empty chunks, the chunks the
splitter cuts and hashes on config-2 streams (IV = the content hash), round trips, and the
authentication-failure / short-input / error contract; the reference's own ciphertext samples
(encryption_test.go:97-127) open and re-seal byte for byte, with 32-byte content IDs."""
import numpy as np
import pytest

from kopia_amd import _lib, batch
from kopia_amd import encryption as ke
from kopia_amd import hashing as kh
from oracle import aead, aesgcm, coracle

pytestmark = pytest.mark.gpu
SEED = 0x6B6F706961
ALGS = [ke.ChaCha20Poly1305, ke.Aes256Gcm]
ORACLE = {ke.ChaCha20Poly1305: aead, ke.Aes256Gcm: aesgcm}


@pytest.fixture(params=ALGS)
def alg(request):
    return request.param
MASTER = bytes(range(100, 132))


def _seal(enc, host, offs, lens, ivs, nonces, dev):
    import torch
    d = torch.from_numpy(host).to(dev)
    d_ivs = torch.from_numpy(np.frombuffer(b"".join(ivs), np.uint8).copy()).to(dev)
    oo, total = ke.sealed_layout(lens)
    out = torch.full((max(total, 1),), 0xAB, dtype=torch.uint8, device=dev)
    st = enc.encrypt_chunks_device(d.data_ptr(), offs, lens, d_ivs, 16, out, oo, dev, nonces=nonces)
    torch.cuda.synchronize()
    return out.cpu().numpy(), oo, st.cpu().numpy()


def _open(enc, sealed, soffs, slens, ivs, dev):
    import torch
    d = torch.from_numpy(np.ascontiguousarray(sealed)).to(dev)
    d_ivs = torch.from_numpy(np.frombuffer(b"".join(ivs), np.uint8).copy()).to(dev)
    po, total = ke.plain_layout(slens)
    out = torch.zeros(total, dtype=torch.uint8, device=dev)
    st = enc.decrypt_chunks_device(d.data_ptr(), soffs, slens, d_ivs, 16, out, po, dev)
    torch.cuda.synchronize()
    return out.cpu().numpy(), po, st.cpu().numpy()


def test_rfc_shaped_single(alg, gpu):
    """One chunk, fixed secret / IV / nonce, equals the oracle's Encrypt."""
    enc = ke.Encryptor(alg, MASTER)
    pt = b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, sunscreen would be it."
    host = np.frombuffer(pt, np.uint8).copy()
    iv = bytes(range(16))
    nonce = bytes(range(40, 52))
    out, oo, st = _seal(enc, host, [0], [len(pt)], [iv], nonce, gpu)
    assert st.tolist() == [0]
    want = ORACLE[alg].kopia_encrypt(aead.derive_key(MASTER), iv, nonce, pt)
    assert out[:len(want)].tobytes() == want


def test_random_chunks(alg, gpu):
    rng = np.random.default_rng(7)
    host = coracle.gen_stream(SEED, 3, 3 << 20)
    lens = list(rng.integers(0, 70000, 300))
    lens[:24] = [0, 1, 3, 4, 15, 16, 17, 63, 64, 65, 127, 1000, 4095, 4096, 4097, 8191, 8192, 8193,
                 12287, 16400, 65536, 65536 + 3, 1 << 20, (1 << 20) + 13]
    lens = np.array(lens, dtype=np.int64)
    offs = np.array([int(rng.integers(0, host.size - int(L))) for L in lens], dtype=np.int64)
    ivs = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in lens]
    nonces = bytes(rng.integers(0, 256, 12 * len(lens), dtype=np.uint8))
    enc = ke.Encryptor(alg, MASTER)
    secret = aead.derive_key(MASTER)
    out, oo, st = _seal(enc, host, offs, lens, ivs, nonces, gpu)
    assert not st.any()
    bad = []
    for i in range(len(lens)):
        want = ORACLE[alg].kopia_encrypt(secret, ivs[i], nonces[12 * i:12 * i + 12], host[offs[i]:offs[i] + lens[i]].tobytes())
        if out[oo[i]:oo[i] + len(want)].tobytes() != want:
            bad.append((i, int(lens[i])))
    assert not bad, bad[:10]
    # round trip through the device decryptor, sealed chunks at odd offsets
    slens = lens + 28
    soffs = np.concatenate(([5], 5 + np.cumsum(slens)[:-1] + np.arange(1, len(slens)))).astype(np.int64)
    sealed = np.zeros(int(soffs[-1] + slens[-1] + 8), np.uint8)
    for i in range(len(lens)):
        sealed[soffs[i]:soffs[i] + slens[i]] = out[oo[i]:oo[i] + slens[i]]
    plain, po, st2 = _open(enc, sealed, soffs, slens, ivs, gpu)
    assert not st2.any()
    for i in range(len(lens)):
        assert plain[po[i]:po[i] + lens[i]].tobytes() == host[offs[i]:offs[i] + lens[i]].tobytes(), i


def test_open_rejects(alg, gpu):
    """A flipped ciphertext, tag or nonce byte, a wrong IV, and a too-short input fail
    (aeadOpenPrefixedWithNonce: "unable to decrypt content" / "ciphertext too short"); the
    untouched chunks of the same call still open."""
    rng = np.random.default_rng(11)
    n, L = 8, 5000
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    ivs = [bytes([i]) * 16 for i in range(n)]
    enc = ke.Encryptor(alg, MASTER)
    out, oo, st = _seal(enc, host, np.arange(n) * L, [L] * n, ivs, None, gpu)
    assert not st.any()
    slens = np.full(n, L + 28, np.int64)
    sealed = out.copy()
    sealed[oo[1] + 100] ^= 1          # ciphertext
    sealed[oo[2] + 12 + L + 5] ^= 0x80  # tag
    sealed[oo[3] + 2] ^= 4             # nonce
    ivs2 = list(ivs)
    ivs2[4] = bytes(16)                # wrong content ID
    slens[5] = 27                      # too short
    plain, po, st2 = _open(enc, sealed, oo, slens, ivs2, gpu)
    assert st2.tolist() == [0, _lib.KCDC_EBADMSG, _lib.KCDC_EBADMSG, _lib.KCDC_EBADMSG, _lib.KCDC_EBADMSG,
                            _lib.KCDC_EINVAL, 0, 0]
    for i in (0, 6, 7):
        assert plain[po[i]:po[i] + L].tobytes() == host[i * L:(i + 1) * L].tobytes()


def test_failed_open_leaves_no_plaintext(alg, gpu):
    """A forged chunk's output slot is all zero after the call and its neighbours are intact (Go's
    Open returns no plaintext on a bad tag: aes256_gcm_hmac_sha256_encryptor.go:49-56).  The output
    buffer starts as 0xAB fill, so a slot the byte pass wrote and the mask missed would show."""
    import torch
    rng = np.random.default_rng(12)
    lens = [5000, 4096, 1, 70001, 33, 65536, 0, 777]
    offs = np.concatenate(([0], np.cumsum(lens)[:-1])).astype(np.int64)
    host = rng.integers(0, 256, int(sum(lens)) + 16, dtype=np.uint8)
    ivs = [bytes([i + 1]) * 16 for i in range(len(lens))]
    enc = ke.Encryptor(alg, MASTER)
    out, oo, st = _seal(enc, host, offs, lens, ivs, None, gpu)
    assert not st.any()
    slens = np.asarray(lens, np.int64) + 28
    sealed = out.copy()
    forged = [1, 3, 4, 7]
    for i in forged:
        sealed[oo[i] + 12 + lens[i]] ^= 0x40  # first tag byte
    d = torch.from_numpy(np.ascontiguousarray(sealed)).to(gpu)
    d_ivs = torch.from_numpy(np.frombuffer(b"".join(ivs), np.uint8).copy()).to(gpu)
    po, total = ke.plain_layout(slens)
    dout = torch.full((total + 64,), 0xAB, dtype=torch.uint8, device=gpu)
    st2 = enc.decrypt_chunks_device(d.data_ptr(), oo, slens, d_ivs, 16, dout, po, gpu).cpu().numpy()
    plain = dout.cpu().numpy()
    assert [i for i in range(len(lens)) if st2[i]] == forged
    assert all(st2[i] == _lib.KCDC_EBADMSG for i in forged)
    for i in range(len(lens)):
        got = plain[po[i]:po[i] + lens[i]]
        if i in forged:
            assert not got.any(), f"chunk {i}: {int(np.count_nonzero(got))} unauthenticated bytes left"
        else:
            assert got.tobytes() == host[offs[i]:offs[i] + lens[i]].tobytes(), i
    assert (plain[total:] == 0xAB).all()  # nothing written past the layout


def test_nonces_differ_by_default(alg, gpu):
    """Without caller nonces, two seals of the same chunk differ (random nonce prefix) and
    both open."""
    enc = ke.Encryptor(alg, MASTER)
    host = np.arange(3000, dtype=np.uint8)
    a, oo, _ = _seal(enc, host, [0], [3000], [bytes(16)], None, gpu)
    b, _, _ = _seal(enc, host, [0], [3000], [bytes(16)], None, gpu)
    assert a[:12].tobytes() != b[:12].tobytes()
    for s in (a, b):
        plain, po, st = _open(enc, s[:3028], [0], [3028], [bytes(16)], gpu)
        assert st.tolist() == [0] and plain[:3000].tobytes() == host.tobytes()


def test_config2_pipeline(alg, gpu):
    """split -> hash (BLAKE2B-256-128, content ID) -> encrypt with IV = content ID, all on the
    device, on 64 x 4 MiB config-2 streams; every sealed chunk equals the oracle's Encrypt of
    the same bytes with the same nonce, and the device decryptor round-trips the batch."""
    import torch
    name, ns, L = "DYNAMIC-4M-BUZHASH", 64, 4 << 20
    dev = gpu
    data = torch.empty(ns * L, dtype=torch.uint8, device=dev)
    batch.fill_prng(data, L, ns, L, SEED, 0)
    b = batch.make_device_batch(name, [data.data_ptr() + i * L for i in range(ns)], [L] * ns, dev)
    batch.split_batch_device(name, b)
    offs, lens = kh.chunk_table([i * L for i in range(ns)], batch.read_cuts(b))
    hkey = bytes(range(32))
    ids = kh.hash_chunks_device(kh.DefaultAlgorithm, data.data_ptr(), offs, lens, hkey, dev)
    ids = ids.contiguous()
    n = len(offs)
    nonces = bytes(np.random.default_rng(3).integers(0, 256, 12 * n, dtype=np.uint8))
    enc = ke.Encryptor(alg, MASTER)
    oo, total = ke.sealed_layout(lens)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    st = enc.encrypt_chunks_device(data.data_ptr(), offs, lens, ids, 16, out, oo, dev, nonces=nonces)
    torch.cuda.synchronize()
    assert not st.cpu().numpy().any()
    host, got, idh = data.cpu().numpy(), out.cpu().numpy(), ids.cpu().numpy()
    secret = aead.derive_key(MASTER)
    for i in range(0, n, max(1, n // (24 if alg == ke.ChaCha20Poly1305 else 8))):  # oracles run ~3-25 MB/s: a spread sample
        want = ORACLE[alg].kopia_encrypt(secret, idh[i].tobytes(), nonces[12 * i:12 * i + 12],
                                  host[offs[i]:offs[i] + lens[i]].tobytes())
        assert got[oo[i]:oo[i] + lens[i] + 28].tobytes() == want, i
    plain = torch.zeros(ke.plain_layout(lens + 28)[1], dtype=torch.uint8, device=dev)
    po, _ = ke.plain_layout(lens + 28)
    st2 = enc.decrypt_chunks_device(out.data_ptr(), oo, lens + 28, ids, 16, plain, po, dev)
    torch.cuda.synchronize()
    assert not st2.cpu().numpy().any()
    p = plain.cpu().numpy()
    assert all(p[po[i]:po[i] + lens[i]].tobytes() == host[offs[i]:offs[i] + lens[i]].tobytes() for i in range(n))


def test_reference_samples(alg, gpu):
    """The reference's TestCiphertextSamples (encryption_test.go:97-127) on the device: each
    CHACHA20-POLY1305-HMAC-SHA256 sample (32-byte content IDs) opens to its payload, and sealing
    the payload with the sample's nonce reproduces the sample byte for byte."""
    from conftest import golden
    import torch
    for c in golden("kopia_encryption_samples.json")["cases"]:
        enc = ke.Encryptor(alg, c["master_key"].encode())
        cid, payload = c["content_id"].encode(), c["payload"].encode()
        sample = bytes.fromhex(c["samples"][alg])
        d_id = torch.frombuffer(bytearray(cid), dtype=torch.uint8).to(gpu)
        d_in = torch.frombuffer(bytearray(sample), dtype=torch.uint8).to(gpu)
        plain = torch.zeros(len(payload) + 8, dtype=torch.uint8, device=gpu)
        st = enc.decrypt_chunks_device(d_in.data_ptr(), [0], [len(sample)], d_id, len(cid), plain, [0], gpu,
                                       iv_len=len(cid))
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [0]
        assert plain.cpu().numpy()[:len(payload)].tobytes() == payload
        d_pl = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(gpu)
        out = torch.zeros(len(sample) + 4, dtype=torch.uint8, device=gpu)
        st = enc.encrypt_chunks_device(d_pl.data_ptr(), [0], [len(payload)], d_id, len(cid), out, [0], gpu,
                                       nonces=sample[:12], iv_len=len(cid))
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [0]
        assert out.cpu().numpy()[:len(sample)].tobytes() == sample


@pytest.mark.parametrize("iv_len", [1, 15, 17, 32, 55, 56, 63, 64])
def test_content_id_lengths(alg, gpu, iv_len):
    """Content IDs of 1..64 bytes (HMAC message of one or two SHA-256 blocks, AAD of 1..4
    Poly1305 blocks) against the oracle."""
    import torch
    rng = np.random.default_rng(iv_len)
    n = 20
    lens = rng.integers(0, 9000, n)
    host = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    offs = np.concatenate(([1], 1 + np.cumsum(lens)[:-1])).astype(np.int64)
    ids = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    nonces = bytes(rng.integers(0, 256, 12 * n, dtype=np.uint8))
    enc = ke.Encryptor(alg, MASTER)
    d = torch.from_numpy(host).to(gpu)
    d_ids = torch.from_numpy(ids).to(gpu)
    oo, total = ke.sealed_layout(lens)
    out = torch.zeros(total, dtype=torch.uint8, device=gpu)
    st = enc.encrypt_chunks_device(d.data_ptr(), offs, lens, d_ids, 64, out, oo, gpu, nonces=nonces, iv_len=iv_len)
    torch.cuda.synchronize()
    assert not st.cpu().numpy().any()
    got = out.cpu().numpy()
    secret = aead.derive_key(MASTER)
    for i in range(n):
        want = ORACLE[alg].kopia_encrypt(secret, ids[i, :iv_len].tobytes(), nonces[12 * i:12 * i + 12],
                                  host[offs[i]:offs[i] + lens[i]].tobytes())
        assert got[oo[i]:oo[i] + lens[i] + 28].tobytes() == want, i


def test_errors(alg, gpu):
    import torch
    enc = ke.Encryptor(alg, MASTER)
    d = torch.zeros(64, dtype=torch.uint8, device=gpu)
    with pytest.raises(_lib.KcdcError):
        ke.Encryptor("AES128-GCM", MASTER)
    L = _lib.lib()
    def call(secret_len, iv_len, work):
        return L.kcdc_encrypt_chunks_device(alg.encode(), enc.secret, secret_len, d.data_ptr(), d.data_ptr(),
                                            d.data_ptr(), 1, d.data_ptr(), iv_len, 16, d.data_ptr(), d.data_ptr(),
                                            d.data_ptr(), d.data_ptr(), d.data_ptr(), work, None)
    assert call(65, 16, 1 << 20) == _lib.KCDC_EINVAL  # secret > 64 bytes
    assert call(32, 16, 64) == _lib.KCDC_EINVAL       # workspace too small
    assert call(32, 0, 1 << 20) == _lib.KCDC_EINVAL   # empty content ID
    assert call(32, 65, 1 << 20) == _lib.KCDC_EINVAL  # content ID > 64 bytes
    assert ke.overhead(alg) == 28


def test_large_chunk_power_table(alg, gpu):
    """An 80 MiB chunk: 5.2 M Poly1305 blocks, so the unit exponents reach the table's top level
    (r^(2^20 d)); sealed bytes and tag equal the oracle's, and the device opens it."""
    import torch
    n = 80 << 20 if alg == ke.ChaCha20Poly1305 else (24 << 20) + 5  # AES: 97 GHASH segments, numpy oracle
    host = coracle.gen_stream(SEED, 40, n + 3)
    iv = bytes(range(200, 216))
    nonce = bytes(range(12))
    enc = ke.Encryptor(alg, MASTER)
    out, oo, st = _seal(enc, host, [3], [n], [iv], nonce, gpu)
    assert st.tolist() == [0]
    want = ORACLE[alg].kopia_encrypt(aead.derive_key(MASTER), iv, nonce, host[3:3 + n].tobytes())
    assert out[:n + 28].tobytes() == want
    plain, po, st2 = _open(enc, out[:n + 28], [0], [n + 28], [iv], gpu)
    assert st2.tolist() == [0] and plain[:n].tobytes() == host[3:3 + n].tobytes()
    del torch


def test_too_long_chunk_and_empty_call(alg, gpu):
    """A chunk of 1 GiB + 1 byte reports KCDC_EFBIG (exponents stay below 2^26) while its
    neighbour seals normally; an empty call does nothing."""
    import torch
    enc = ke.Encryptor(alg, MASTER)
    big = (1 << 30) + 1
    d = torch.zeros(big + 64, dtype=torch.uint8, device=gpu)
    ids = torch.zeros((2, 16), dtype=torch.uint8, device=gpu)
    lens = np.array([big, 100], np.int64)
    oo = np.array([0, 256], np.int64)
    out = torch.zeros(512, dtype=torch.uint8, device=gpu)
    st = enc.encrypt_chunks_device(d.data_ptr(), [0, 64], lens, ids, 16, out, oo, gpu, nonces=bytes(24))
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [_lib.KCDC_EFBIG, 0]
    want = ORACLE[alg].kopia_encrypt(aead.derive_key(MASTER), bytes(16), bytes(12), bytes(100))
    assert out.cpu().numpy()[256:256 + 128].tobytes() == want
    st0 = enc.encrypt_chunks_device(d.data_ptr(), [], [], ids, 16, out, [], gpu)
    assert st0.numel() == 0


def test_side_stream_status(alg, gpu):
    """A caller's non-current stream (advisor, round 2): every temporary and the status words are
    ordered on that stream, so a tampered chunk's KCDC_EBADMSG survives and a good one reads 0;
    raise_on_status names the failed chunk."""
    import torch
    enc = ke.Encryptor(alg, MASTER)
    host = coracle.gen_stream(SEED, 5, 1 << 16)
    lens, offs = [1000, 5000, 77], [0, 2000, 9000]
    ivs = [bytes([i]) * 16 for i in range(3)]
    nonces = bytes(range(36))
    side = torch.cuda.Stream(device=gpu)
    d = torch.from_numpy(host).to(gpu)
    d_ivs = torch.from_numpy(np.frombuffer(b"".join(ivs), np.uint8).copy()).to(gpu)
    oo, total = ke.sealed_layout(lens)
    sealed = torch.zeros(total, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    st = enc.encrypt_chunks_device(d.data_ptr(), offs, lens, d_ivs, 16, sealed, oo, gpu, nonces=nonces, stream=side)
    side.synchronize()
    assert st.cpu().tolist() == [0, 0, 0]
    with torch.cuda.stream(side):
        sealed[int(oo[1]) + 20] ^= 1  # tamper chunk 1's ciphertext, on the side stream
    slens = [L + ke.overhead(alg) for L in lens]
    po, ptotal = ke.plain_layout(slens, alg)
    out = torch.zeros(ptotal, dtype=torch.uint8, device=gpu)
    st = enc.decrypt_chunks_device(sealed.data_ptr(), oo, slens, d_ivs, 16, out, po, gpu, stream=side)
    side.synchronize()
    assert st.cpu().tolist() == [0, _lib.KCDC_EBADMSG, 0]
    with pytest.raises(_lib.KcdcError, match="chunk 1 of 3"):
        ke.raise_on_status(st)
    got = out.cpu().numpy()
    assert got[po[0]:po[0] + lens[0]].tobytes() == host[0:1000].tobytes()
    assert got[po[2]:po[2] + lens[2]].tobytes() == host[9000:9077].tobytes()
