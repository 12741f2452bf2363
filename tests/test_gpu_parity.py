"""GPU parity tests: the HIP path (through the C ABI) against the reference's
own vectors, the reference library's outputs (tests/golden/ref_*.json) and
the CPU oracle, bit for bit.

Mirrors the reference's test strategy (crypto/cipher/aead_test.cc):
TestVector (188-281), truncated tags (963-1066), in-place / unaligned
(1068-1185), Wycheproof (1493-1564); plus batch-level checks at BASELINE
sizes through digests of the reference outputs (checksum of checksums) and
open(seal(x)) round trips.
"""
import hashlib
import os
import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import boringssl_amd as ba  # noqa: E402
import oracle_lib as o  # noqa: E402
from golden_util import AEAD_KEYLEN, batch_digests, load  # noqa: E402
import tls_util  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
ORACLE_ID = {"aes-128-gcm": o.AES_GCM, "aes-192-gcm": o.AES_GCM, "aes-256-gcm": o.AES_GCM,
             "chacha20-poly1305": o.CHACHA20_POLY1305, "xchacha20-poly1305": o.XCHACHA20_POLY1305,
             "aes-128-gcm-siv": o.AES_GCM_SIV, "aes-256-gcm-siv": o.AES_GCM_SIV}


def _nl(aead):
    """Nonce length of the AEAD (EVP_AEAD_nonce_length)."""
    return 24 if aead == "xchacha20-poly1305" else 12


def _h(s):
    return bytes.fromhex(s)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    ba.lib.ERR_clear_error()
    yield
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------
# helpers

def _pack(chunks, align=16, odd=0):
    """Concatenate byte strings into one uint8 array; returns (array, offsets)."""
    offs, pos = [], odd
    for c in chunks:
        offs.append(pos)
        pos += len(c)
        pos = (pos + align - 1) // align * align + odd
    buf = np.zeros(max(pos, 1) + 16, dtype=np.uint8)
    for off, c in zip(offs, chunks):
        if c:
            buf[off:off + len(c)] = np.frombuffer(c, dtype=np.uint8)
    return buf, np.array(offs, dtype=np.uint64)


def _t(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def run_batch(aead, keys, key_index, ins, nonces, ads, tag_len, open_=False, tags=None,
              align=16, odd=0, inplace=False):
    """Seal (or open) records given as Python bytes through the device batch
    API.  `keys` is a list; records select keys with key_index (None = ctx of
    keys[0]).  Returns (outs, tags, status)."""
    n = len(ins)
    nonce_len = len(nonces[0])
    assert all(len(x) == nonce_len for x in nonces)
    inbuf, offs = _pack(ins, align, odd)
    adbuf, ad_offs = _pack(ads, 1)
    d_in = _t(inbuf)
    d_out = d_in if inplace else torch.zeros_like(d_in)
    d_nonce = _t(np.frombuffer(b"".join(nonces), dtype=np.uint8).copy() if nonce_len else
                 np.zeros(1, np.uint8))
    d_ad = _t(adbuf)
    lens = np.array([len(x) for x in ins], dtype=np.int64)
    ad_lens = np.array([len(x) for x in ads], dtype=np.int64)
    d_tags = torch.zeros(max(1, n * tag_len), dtype=torch.uint8, device=DEV)
    if tags is not None:
        d_tags = _t(np.frombuffer(b"".join(tags), dtype=np.uint8).copy())
    d_status = torch.full((max(n, 1),), 7, dtype=torch.uint8, device=DEV)
    d_ki = _t(np.array(key_index, dtype=np.int32)) if key_index is not None else None
    b = ba.make_batch(n, d_in, d_out, d_tags, d_nonce, nonce_len, d_ad,
                      offsets=_t(offs.astype(np.int64)), lengths=_t(lens),
                      ad_offsets=_t(ad_offs.astype(np.int64)), ad_lengths=_t(ad_lens),
                      status=d_status, key_index=d_ki)
    if key_index is None:
        ctx = ba.AEADCtx(aead, keys[0], tag_len)
        (ctx.open_batch_device if open_ else ctx.seal_batch_device)(b)
    else:
        ks = ba.Keyset(aead, b"".join(keys), len(keys), tag_len)
        (ks.open_batch_device if open_ else ks.seal_batch_device)(b)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    tg = d_tags.cpu().numpy().tobytes()
    st = d_status.cpu().numpy()[:n]
    outs = [out[int(offs[i]):int(offs[i]) + len(ins[i])].tobytes() for i in range(n)]
    return outs, [tg[i * tag_len:(i + 1) * tag_len] for i in range(n)], st


# ---------------------------------------------------------------------------
# reference known-answer files through the single-record host API

@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-192-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
def test_kat_single_record(aead):
    cases = [c for c in load("kat_aead.json") if c["aead"] == aead]
    ctxs = {}
    for c in cases:
        key, nonce, ad, pt, ct, tag = (_h(c[k]) for k in ("key", "nonce", "ad", "pt", "ct", "tag"))
        tag_len = c.get("tag_len", len(tag))
        k = (key, tag_len)
        if k not in ctxs:
            ctxs[k] = ba.AEADCtx(aead, key, tag_len)
        ctx = ctxs[k]
        if c["valid"]:
            assert ctx.seal(nonce, pt, ad) == ct + tag, c["source"]
            assert ctx.open(nonce, ct + tag, ad) == pt, c["source"]
            if tag:
                bad = bytearray(ct + tag)
                bad[-1] ^= 0x80
                with pytest.raises(ba.AEADError) as e:
                    ctx.open(nonce, bytes(bad), ad)
                assert e.value.lib == ba.ERR_LIB_CIPHER
        else:
            with pytest.raises(ba.AEADError) as e:
                ctx.open(nonce, ct + tag, ad)
            assert e.value.lib == ba.ERR_LIB_CIPHER, c["source"]


def test_ref_edge_single_record():
    for c in load("ref_edge.json"):
        key, nonce, ad, pt, ct, tag = (_h(c[k]) for k in ("key", "nonce", "ad", "pt", "ct", "tag"))
        ctx = ba.AEADCtx(c["aead"], key, len(tag))
        assert ctx.seal(nonce, pt, ad) == ct + tag, (c["aead"], len(pt), len(nonce), len(ad))
        # (the one-record kernels' open: tag checked before the plaintext is written)
        assert ctx.open(nonce, ct + tag, ad) == pt, (c["aead"], len(pt), len(nonce), len(ad))


# ---------------------------------------------------------------------------
# batches

def _groups(cases):
    g = {}
    for c in cases:
        tag_len = c.get("tag_len", len(_h(c["tag"])))
        g.setdefault((c["aead"], len(_h(c["nonce"])), tag_len), []).append(c)
    return g


@pytest.mark.parametrize("source", ["ref_edge.json", "kat_aead.json"])
def test_batch_multikey_vectors(source):
    """Every record with its own key (keyset + key_index), seal then open."""
    cases = [c for c in load(source) if c.get("valid", True)]
    for (aead, nl, tag_len), grp in _groups(cases).items():
        if ("chacha" in aead or "siv" in aead) and nl != _nl(aead):
            continue
        if nl == 0:
            continue
        keys = [_h(c["key"]) for c in grp]
        ins = [_h(c["pt"]) for c in grp]
        nonces = [_h(c["nonce"]) for c in grp]
        ads = [_h(c["ad"]) for c in grp]
        outs, tags, st = run_batch(aead, keys, list(range(len(grp))), ins, nonces, ads, tag_len)
        assert st.tolist() == [1] * len(grp)
        for c, out, tag in zip(grp, outs, tags):
            assert out == _h(c["ct"]) and tag == _h(c["tag"]), (aead, c.get("source"), len(ins))
        back, _, st = run_batch(aead, keys, list(range(len(grp))), outs, nonces, ads, tag_len,
                                open_=True, tags=tags)
        assert st.tolist() == [1] * len(grp)
        assert back == ins


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
@pytest.mark.parametrize("layout", ["aligned", "unaligned", "inplace"])
def test_batch_ragged_vs_oracle(aead, layout):
    rng = random.Random(hash((aead, layout)) & 0xffff)
    key = bytes(rng.getrandbits(8) for _ in range(AEAD_KEYLEN[aead]))
    n = 300
    lens = [rng.choice([0, 1, 15, 16, 17, 63, 64, 65, 255, 256, 1000, 1350, 4097, 16384])
            for _ in range(n)]
    ins = [bytes(rng.getrandbits(8) for _ in range(l)) for l in lens]
    nonces = [bytes(rng.getrandbits(8) for _ in range(_nl(aead))) for _ in range(n)]
    ads = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 13, 16, 40, 300])))
           for _ in range(n)]
    outs, tags, st = run_batch(aead, [key], None, ins, nonces, ads, 16,
                               odd=3 if layout == "unaligned" else 0,
                               inplace=layout == "inplace")
    assert st.all()
    for i in range(n):
        ok, ct, tag = o.seal(ORACLE_ID[aead], key, nonces[i], ins[i], ads[i])
        assert ok and outs[i] == ct and tags[i] == tag, (i, lens[i], len(ads[i]))


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
@pytest.mark.parametrize("multikey", [False, True])
def test_batch_large_ragged_reordered(aead, multikey):
    """>= 4096 ragged records: the launcher processes them in length-class
    order (sched.hip); outputs must still land per record, as the oracle's."""
    rng = np.random.default_rng(11 + multikey)
    n = 5000
    lens = rng.choice([0, 1, 16, 17, 200, 1350, 4096, 9000, 16384, 16400], size=n).tolist()
    ins = [rng.integers(0, 256, size=l, dtype=np.uint8).tobytes() for l in lens]
    nonces = [rng.integers(0, 256, size=_nl(aead), dtype=np.uint8).tobytes() for _ in range(n)]
    ads = [rng.integers(0, 256, size=13, dtype=np.uint8).tobytes() for _ in range(n)]
    nkeys = 7 if multikey else 1
    keys = [rng.integers(0, 256, size=AEAD_KEYLEN[aead], dtype=np.uint8).tobytes()
            for _ in range(nkeys)]
    ki = rng.integers(0, nkeys, size=n).tolist() if multikey else None
    outs, tags, st = run_batch(aead, keys, ki, ins, nonces, ads, 16, odd=5)
    assert st.all()
    for i in range(n):
        k = keys[ki[i]] if multikey else keys[0]
        ok, ct, tag = o.seal(ORACLE_ID[aead], k, nonces[i], ins[i], ads[i])
        assert ok and outs[i] == ct and tags[i] == tag, (i, lens[i])
    back, _, st = run_batch(aead, keys, ki, outs, nonces, ads, 16, open_=True, tags=tags, odd=5)
    assert st.all() and back == ins


@pytest.mark.parametrize("mode", ["bs"])
@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-192-gcm", "aes-256-gcm"])
@pytest.mark.parametrize("rlen", [4096, 16384, 17408, 32768])
def test_bitsliced_gcm_path(aead, rlen, mode, aes_engine):
    """The table-free engine (gcm_bs.hip, BSSL_AMD_set_aes_gcm_engine) on
    uniform, 16-byte-multiple records: full and partial 256-block chunks,
    seal and open (tags verified, one tampered record)."""
    aes_engine(mode)
    rng = np.random.default_rng(rlen + len(mode))
    n = 50
    key = rng.integers(0, 256, size=AEAD_KEYLEN[aead], dtype=np.uint8).tobytes()
    pt = rng.integers(0, 256, size=n * rlen, dtype=np.uint8)
    nonces = rng.integers(0, 256, size=n * 12, dtype=np.uint8)
    ad = rng.integers(0, 256, size=n * 13, dtype=np.uint8)
    d_pt, d_ct = _t(pt), torch.zeros(n * rlen, dtype=torch.uint8, device=DEV)
    d_tags = torch.zeros(n * 16, dtype=torch.uint8, device=DEV)
    d_st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ctx = ba.AEADCtx(aead, key, 16)
    b = ba.make_batch(n, d_pt, d_ct, d_tags, _t(nonces), 12, _t(ad), record_stride=rlen,
                      record_len=rlen, ad_stride=13, ad_len=13, status=d_st)
    ctx.seal_batch_device(b)
    torch.cuda.synchronize()
    assert bool(d_st.all())
    ct, tg = d_ct.cpu().numpy(), d_tags.cpu().numpy()
    for i in range(n):
        ok, c, t = o.seal(ORACLE_ID[aead], key, nonces[12 * i:12 * i + 12].tobytes(),
                          pt[rlen * i:rlen * (i + 1)].tobytes(), ad[13 * i:13 * i + 13].tobytes())
        assert ok and ct[rlen * i:rlen * (i + 1)].tobytes() == c and tg[16 * i:16 * i + 16].tobytes() == t, i
    d_back = torch.zeros_like(d_pt)
    bad_tags = d_tags.clone()
    bad_tags[16 * 7] ^= 1
    b2 = ba.make_batch(n, d_ct, d_back, bad_tags, _t(nonces), 12, _t(ad), record_stride=rlen,
                       record_len=rlen, ad_stride=13, ad_len=13, status=d_st)
    ctx.open_batch_device(b2)
    torch.cuda.synchronize()
    stv = d_st.cpu().numpy()
    assert stv[7] == 0 and stv.sum() == n - 1
    back = d_back.cpu().numpy()
    assert not back[7 * rlen:8 * rlen].any()
    assert np.array_equal(np.delete(back.reshape(n, rlen), 7, 0), np.delete(pt.reshape(n, rlen), 7, 0))


@pytest.mark.parametrize("mode", ["bs"])
@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm"])
def test_mix_kernel_ragged(aead, mode, aes_engine):
    """The table-free kernel (gcm_bs_kernel) on a ragged one-key batch:
    16-byte-multiple records of 4-19 KiB mixed with records of any length,
    at two alignments -- every record must match the oracle, sealed and
    opened."""
    aes_engine(mode)
    rng = random.Random(len(mode) * 7 + len(aead))
    key = bytes(rng.getrandbits(8) for _ in range(AEAD_KEYLEN[aead]))
    n = 600
    lens = []
    for i in range(n):
        k = rng.randrange(4)
        lens.append(16 * rng.randrange(256, 1200) if k < 3 else rng.randrange(0, 9000))
    ins = [rng.randbytes(L) for L in lens]
    nonces = [rng.randbytes(12) for _ in range(n)]
    ads = [rng.randbytes(rng.randrange(0, 40)) for _ in range(n)]
    for odd in (0, 4):
        outs, tags, st = run_batch(aead, [key], None, ins, nonces, ads, 16, odd=odd)
        assert st.all()
        for i in range(n):
            ok, ct, tag = o.seal(ORACLE_ID[aead], key, nonces[i], ins[i], ads[i])
            assert ok and outs[i] == ct and tags[i] == tag, (odd, i, lens[i])
        back, _, st = run_batch(aead, [key], None, outs, nonces, ads, 16, open_=True, tags=tags,
                                odd=odd)
        assert st.all() and back == ins


def test_batch_gcm_nonce_lengths_and_truncated_tags():
    rng = random.Random(7)
    for nl in (1, 8, 12, 16, 17, 60, 128):
        for tag_len in (16, 12, 4, 1):
            key = bytes(rng.getrandbits(8) for _ in range(16))
            n = 40
            ins = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 700))) for _ in range(n)]
            nonces = [bytes(rng.getrandbits(8) for _ in range(nl)) for _ in range(n)]
            ads = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 40))) for _ in range(n)]
            outs, tags, st = run_batch("aes-128-gcm", [key], None, ins, nonces, ads, tag_len)
            assert st.all()
            for i in range(n):
                ok, ct, tag = o.seal(o.AES_GCM, key, nonces[i], ins[i], ads[i], tag_len)
                assert outs[i] == ct and tags[i] == tag, (nl, tag_len, i)


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
def test_open_rejects_tampering_and_zeroes_output(aead):
    rng = random.Random(11)
    key = bytes(rng.getrandbits(8) for _ in range(AEAD_KEYLEN[aead]))
    n = 64
    ins = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 3000))) for _ in range(n)]
    nonces = [bytes(rng.getrandbits(8) for _ in range(_nl(aead))) for _ in range(n)]
    ads = [bytes(rng.getrandbits(8) for _ in range(13)) for _ in range(n)]
    cts, tags, st = run_batch(aead, [key], None, ins, nonces, ads, 16)
    assert st.all()
    bad = set(range(0, n, 3))
    cts2, tags2, ads2 = list(cts), list(tags), list(ads)
    for i in bad:
        what = i % 4
        if what == 0:
            b = bytearray(cts2[i]); b[rng.randrange(len(b))] ^= 1 << rng.randrange(8); cts2[i] = bytes(b)
        elif what == 1:
            b = bytearray(tags2[i]); b[rng.randrange(16)] ^= 0x40; tags2[i] = bytes(b)
        elif what == 2:
            b = bytearray(ads2[i]); b[0] ^= 0x01; ads2[i] = bytes(b)
        else:
            tags2[i] = bytes(16)
    pts, _, st = run_batch(aead, [key], None, cts2, nonces, ads2, 16, open_=True, tags=tags2)
    for i in range(n):
        if i in bad:
            assert st[i] == 0 and pts[i] == bytes(len(ins[i])), i
        else:
            assert st[i] == 1 and pts[i] == ins[i], i


def test_device_synth_matches_host_definition():
    lens = np.array([16384, 1350, 1, 0, 77, 4096], dtype=np.uint64)
    pt, offs, nonces, ads = o.synth_batch(1000, lens)
    d_pt = torch.zeros(len(pt), dtype=torch.uint8, device=DEV)
    d_n = torch.zeros(12 * len(lens), dtype=torch.uint8, device=DEV)
    d_a = torch.zeros(13 * len(lens), dtype=torch.uint8, device=DEV)
    ba.synth_fill_device(1000, len(lens), _t(offs.astype(np.int64)), _t(lens.astype(np.int64)),
                         d_pt, d_n, d_a)
    torch.cuda.synchronize()
    assert np.array_equal(d_pt.cpu().numpy(), pt)
    assert np.array_equal(d_n.cpu().numpy(), nonces)
    assert np.array_equal(d_a.cpu().numpy(), ads)


# ---------------------------------------------------------------------------
# synthetic workloads vs the reference library's digests

def synth_device_batch(aead, nkeys, rpk, length, first=0, align=16):
    n = nkeys * rpk
    if length == "mixed":
        lens = np.array([o.synth_mixed_len(first + i) for i in range(n)], dtype=np.uint64)
    else:
        lens = np.full(n, int(length), dtype=np.uint64)
    a = np.uint64(align)
    padded = (lens + a - np.uint64(1)) // a * a
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(padded[:-1])
    total = int(padded.sum())
    d_offs, d_lens = _t(offs.astype(np.int64)), _t(lens.astype(np.int64))
    # zero-filled so the padding between records is defined (the kernels must
    # never write it; the in-place round trip below compares whole buffers)
    d_pt = torch.zeros(total, dtype=torch.uint8, device=DEV)
    d_n = torch.empty(12 * n, dtype=torch.uint8, device=DEV)
    d_a = torch.empty(13 * n, dtype=torch.uint8, device=DEV)
    ba.synth_fill_device(first, n, d_offs, d_lens, d_pt, d_n, d_a)
    return lens, offs, d_offs, d_lens, d_pt, d_n, d_a


def _device_digests(d_out, offs, lens, d_tags, chunk=1024):
    """tags_sha256 and the checksum-of-checksums ct digest, streamed from the
    device chunk by chunk."""
    n = len(lens)
    parts = []
    for c in range(0, n, chunk):
        hi = min(n, c + chunk)
        lo_b, hi_b = int(offs[c]), int(offs[hi - 1] + lens[hi - 1])
        host = d_out[lo_b:hi_b].cpu().numpy()
        h = hashlib.sha256()
        for i in range(c, hi):
            s = int(offs[i]) - lo_b
            h.update(host[s:s + int(lens[i])].data)
        parts.append(h.digest())
    tags = d_tags.cpu().numpy().tobytes()
    return hashlib.sha256(tags).hexdigest(), hashlib.sha256(b"".join(parts)).hexdigest()


def xchacha_nonces_device(d_n12):
    a = d_n12.view(-1, 12)
    b = a.clone()
    b[:, 4:] ^= 0xff
    return torch.cat([a, b], dim=1).contiguous().view(-1)


def _run_synth_digest(name, align=16):
    g = load("ref_digests.json")[name]
    aead, nkeys, rpk, length = g["aead"], g["nkeys"], g["records_per_key"], g["len"]
    n = nkeys * rpk
    lens, offs, d_offs, d_lens, d_pt, d_n, d_a = synth_device_batch(aead, nkeys, rpk, length,
                                                                    align=align)
    d_out = torch.zeros_like(d_pt)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=DEV)
    d_st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    keys = [o.synth_key(k, AEAD_KEYLEN[aead]) for k in range(nkeys)]
    nl = _nl(aead)
    if nl == 24:  # ref_tool.cc make_nonce: n_i || (n_i with bytes 4..11 XOR 0xff)
        d_n = xchacha_nonces_device(d_n)
    b = ba.make_batch(n, d_pt, d_out, d_tags, d_n, nl, d_a, offsets=d_offs, lengths=d_lens,
                      ad_stride=13, ad_len=13, status=d_st,
                      key_index=_t((np.arange(n) // rpk).astype(np.int32)) if nkeys > 1 else None)
    if nkeys > 1:
        obj = ba.Keyset(aead, b"".join(keys), nkeys, 16)
    else:
        obj = ba.AEADCtx(aead, keys[0], 16)
    obj.seal_batch_device(b)
    torch.cuda.synchronize()
    assert bool(d_st.all())
    tags_d, ct_d = _device_digests(d_out, offs, lens, d_tags)
    assert tags_d == g["tags_sha256"], name
    assert ct_d == g["ct_sha256"], name
    # open(seal(x)) == x, in place, all tags verify
    d_st.zero_()
    b2 = ba.make_batch(n, d_out, d_out, d_tags, d_n, nl, d_a, offsets=d_offs, lengths=d_lens,
                       ad_stride=13, ad_len=13, status=d_st, key_index=b._refs[-1])
    obj.open_batch_device(b2)
    torch.cuda.synchronize()
    assert bool(d_st.all())
    assert torch.equal(d_out, d_pt)
    del d_out, d_pt, d_tags, d_st, b, b2
    torch.cuda.empty_cache()  # the full-size configs hold up to 128 GiB


@pytest.mark.parametrize("name", ["parity_aes128_16k", "parity_aes256_mixed", "parity_chacha_1350",
                                  "parity_multikey_aes128", "parity_xchacha_1350",
                                  "parity_siv128_1350", "parity_siv256_mixed",
                                  "parity_siv128_multikey"])
def test_synth_parity_digest(name):
    _run_synth_digest(name)


@pytest.mark.parametrize("name", ["parity_chacha_1350", "parity_xchacha_1350",
                                  "parity_aes256_mixed", "config3_chacha_1350"])
def test_synth_parity_digest_align128(name):
    """The same digests with records 128-byte aligned (bench.py's alignment;
    per-record offsets/lengths arrays): ChaCha's 128-byte slot shift (sh = 1)
    with the per-record metadata path."""
    _run_synth_digest(name, align=128)


@pytest.mark.parametrize("name", ["config2_aes128_16k", "config3_chacha_1350",
                                  "config3x_xchacha_1350", "configs_siv128_16k"])
def test_baseline_config_digest(name):
    """BASELINE.json configs 2 and 3 at full size (16 GiB / 1.3 GiB)."""
    _run_synth_digest(name)


@pytest.mark.parametrize("name", ["config4_aes256_mixed", "config5_multikey_aes128"])
def test_baseline_config_digest_large(name):
    """BASELINE.json configs 4 (4M mixed-length AES-256-GCM records, 32 GiB) and
    5 (64K keys x 64 x 16 KiB, 64 GiB) at full size vs the reference digests.
    Part of the default GPU suite (about 70 s for both)."""
    _run_synth_digest(name)


def test_plain_c_caller_on_gpu(tmp_path):
    """examples/seal_one.c (a C program written against the reference API)
    reproduces the reference's bench/aead.cc all-zero 16 KiB tag."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    libdir = os.path.dirname(ba.LIB_PATH)
    exe = tmp_path / "seal_one"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(root, "include"),
                           os.path.join(root, "examples", "seal_one.c"), "-L", libdir,
                           "-lbssl_amd", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True, timeout=120).strip()
    assert out == "f9ff3fa1f8bade711aa97c0f652d67fe"  # SURVEY.md 8(c), reference output


# ---------------------------------------------------------------------------
# tls12 / tls13 AEADs: the stateful monotonic-nonce check, single records and
# batches (a batch = N sealv calls in record order).

U64_MAX = (1 << 64) - 1


def _tls_rule(kind, nonces, state):
    """Restatement of aead_aes_gcm_tls12_sealv (e_aes.cc.inc:1071-1100) and
    aead_aes_gcm_tls13_sealv (:1162-1202): which calls pass the nonce check;
    `state` (min_next, mask) is advanced in place."""
    ok = []
    for nz in nonces:
        given = int.from_bytes(nz[4:12], "big")
        if kind == 12:
            good = given != U64_MAX and given >= state["min_next"]
            if good:
                state["min_next"] = given + 1
        elif state["min_next"] == 0:
            state["mask"], state["min_next"], good = given, 1, True
        else:
            c = given ^ state["mask"]
            good = c != U64_MAX and c >= state["min_next"]
            if good:
                state["min_next"] = c + 1
        ok.append(good)
    return ok


def _tls_nonces(kind, rng, n):
    """Mostly increasing sequence numbers with repeats, steps back, gaps and
    the all-ones counter, in the record nonce layout of each variant
    (ssl/ssl_aead_ctx.cc:326-365: TLS 1.2 GCM fixed 4 B || explicit 8 B,
    TLS 1.3 fixed_iv XOR (0^4 || be64(seq)))."""
    seqs, s = [], 0
    for i in range(n):
        r = rng.random()
        if r < 0.1:
            s = max(0, s - rng.randint(1, 3))
        elif r < 0.2:
            pass
        elif r < 0.25:
            s += rng.randint(2, 50)
        else:
            s += 1
        seqs.append(s)
    seqs[n // 2] = U64_MAX
    if kind == 13:
        seqs[0] = 0  # the first record sets the mask
        iv = bytes(rng.getrandbits(8) for _ in range(12))
        return [bytes(a ^ b for a, b in zip(iv, bytes(4) + q.to_bytes(8, "big"))) for q in seqs]
    fixed = bytes(rng.getrandbits(8) for _ in range(4))
    return [fixed + q.to_bytes(8, "big") for q in seqs]


def _tls_batch(ctx, ins, nonces, ads):
    inbuf, offs = _pack(ins)
    adbuf, ad_offs = _pack(ads, 1)
    n = len(ins)
    d_in = _t(inbuf)
    d_out = torch.full_like(d_in, 0x5a)
    d_tags = torch.full((16 * n,), 0x5a, dtype=torch.uint8, device=DEV)
    d_status = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    b = ba.make_batch(n, d_in, d_out, d_tags, _t(np.frombuffer(b"".join(nonces), np.uint8).copy()),
                      12, _t(adbuf), offsets=_t(offs.astype(np.int64)),
                      lengths=_t(np.array([len(x) for x in ins], np.int64)),
                      ad_offsets=_t(ad_offs.astype(np.int64)),
                      ad_lengths=_t(np.array([len(x) for x in ads], np.int64)), status=d_status)
    ctx.seal_batch_device(b)
    torch.cuda.synchronize()
    out, tg, st = d_out.cpu().numpy(), d_tags.cpu().numpy().tobytes(), d_status.cpu().numpy()
    return ([out[int(offs[i]):int(offs[i]) + len(ins[i])].tobytes() for i in range(n)],
            [tg[16 * i:16 * i + 16] for i in range(n)], st)


@pytest.mark.parametrize("aead", ["aes-128-gcm-tls12", "aes-256-gcm-tls12", "aes-128-gcm-tls13",
                                  "aes-256-gcm-tls13"])
def test_tls_nonce_check_batches(aead):
    kind = 12 if "tls12" in aead else 13
    rng = random.Random(kind * 7 + len(aead))
    key = bytes(rng.getrandbits(8) for _ in range(32 if "256" in aead else 16))
    n = 700
    nonces = _tls_nonces(kind, rng, n)
    ins = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 15, 16, 17, 100, 1350])))
           for _ in range(n)]
    ads = [bytes(rng.getrandbits(8) for _ in range(13)) for _ in range(n)]
    state = {"min_next": 0, "mask": 0}
    expect = _tls_rule(kind, nonces, state)
    assert 0 < sum(expect) < n
    # The same calls as two device batches on one context, then one more
    # single-record call: the nonce state carries across them.
    ctx = ba.AEADCtx(aead, key, 16)
    half = n // 2
    outs, tags, st = _tls_batch(ctx, ins[:half], nonces[:half], ads[:half])
    outs2, tags2, st2 = _tls_batch(ctx, ins[half:], nonces[half:], ads[half:])
    outs, tags, st = outs + outs2, tags + tags2, list(st) + list(st2)
    for i in range(n):
        if expect[i]:
            ok, ct, tag = o.seal(o.AES_GCM, key, nonces[i], ins[i], ads[i])
            assert ok and st[i] == 1 and outs[i] == ct and tags[i] == tag, i
        else:
            assert st[i] == 0 and outs[i] == bytes(len(ins[i])) and tags[i] == bytes(16), i
    # Next call: a nonce one below the state must fail, the state's own must pass.
    nxt = state["min_next"]
    for delta, good in ((-1, False), (0, True)):
        c = nxt + delta
        if kind == 13:
            c ^= state["mask"]
        nonce = nonces[0][:4] + c.to_bytes(8, "big")
        if good:
            ok, ct, tag = o.seal(o.AES_GCM, key, nonce, b"abc", b"")
            assert ctx.seal(nonce, b"abc") == ct + tag
        else:
            with pytest.raises(ba.AEADError) as e:
                ctx.seal(nonce, b"abc")
            assert e.value.reason == ba.CIPHER_R_INVALID_NONCE
    # Sequential single-record calls on a fresh context agree with the batch.
    ctx1 = ba.AEADCtx(aead, key, 16)
    seq_ok = []
    for i in range(n):
        try:
            r = ctx1.seal(nonces[i], ins[i], ads[i])
            seq_ok.append(True)
            assert r == outs[i] + tags[i], i
        except ba.AEADError as e:
            assert e.reason == ba.CIPHER_R_INVALID_NONCE
            seq_ok.append(False)
    assert seq_ok == expect


def test_tls_batch_rejections():
    """Keysets reject the stateful variants; tls seal batches need 12-byte
    nonces (open batches accept any, as aead_aes_gcm_openv_detached)."""
    key = bytes(range(16))
    with pytest.raises(ba.AEADError) as e:
        ks = ba.Keyset("aes-128-gcm-tls13", key, 1, 16)
        d = torch.zeros(64, dtype=torch.uint8, device=DEV)
        ks.seal_batch_device(ba.make_batch(1, d, d, d, d, 12, d, record_len=16, record_stride=16))
    assert e.value.reason == ba.CIPHER_R_CTRL_NOT_IMPLEMENTED
    ctx = ba.AEADCtx("aes-128-gcm-tls12", key, 16)
    d = torch.zeros(64, dtype=torch.uint8, device=DEV)
    with pytest.raises(ba.AEADError) as e:
        ctx.seal_batch_device(ba.make_batch(1, d, d, d, d, 8, d, record_len=16, record_stride=16))
    assert e.value.reason == ba.CIPHER_R_UNSUPPORTED_NONCE_SIZE


# ---------------------------------------------------------------------------
# TLS record layer (include/bssl_amd/tls.h) against a restatement of the
# reference's do_seal_record (ssl/tls_record.cc:266-317) and
# SSLAEADContext::SealScatter / GetAdditionalData (ssl/ssl_aead_ctx.cc:207-380)
# on top of the oracle's AEAD.

def _tls_seal_oracle(version, aead, key, fixed_iv, seq0, records, types):
    return tls_util.tls_seal_restated(version, aead, key, fixed_iv, seq0, records, types)


@pytest.mark.parametrize("version,aead", [(0x0303, "aes-128-gcm"), (0x0303, "aes-256-gcm"),
                                          (0x0303, "chacha20-poly1305"), (0x0304, "aes-128-gcm"),
                                          (0x0304, "aes-256-gcm"),
                                          (0x0304, "chacha20-poly1305")])
def test_tls_record_layer(version, aead):
    rng = random.Random(version * 31 + len(aead))
    key = bytes(rng.getrandbits(8) for _ in range(16 if "128" in aead else 32))
    xor = version == 0x0304 or aead == "chacha20-poly1305"
    fixed_iv = bytes(rng.getrandbits(8) for _ in range(12 if xor else 4))
    # TLS 1.3 traffic keys start at sequence number 0 (RFC 8446 5.3) and the
    # tls13 AEAD takes its nonce mask from the first nonce on that basis
    # (e_aes.cc.inc:1181-1185); a writer created mid-stream starts from the
    # state the AEAD has after records 0 .. seq0-1.  Both starts are covered.
    seq0 = 0 if (version == 0x0304 and aead == "aes-128-gcm") else rng.getrandbits(40)
    n = 300
    lens = [rng.choice([0, 1, 15, 16, 17, 31, 64, 100, 1350, 4096, 16384]) for _ in range(n)]
    lens[7] = 16385  # over SSL3_RT_MAX_PLAIN_LENGTH: that record fails
    records = [bytes(rng.getrandbits(8) for _ in range(L)) for L in lens]
    types = [rng.choice([21, 22, 23]) for _ in range(n)]
    expect = _tls_seal_oracle(version, aead, key, fixed_iv, seq0, records, types)

    sealer = ba.TlsAead(ba.evp_aead_seal, version, aead, key, fixed_iv, seq0)
    pl, sl = sealer.prefix_len, sealer.suffix_len
    assert pl == (5 if xor else 13) and sl == (17 if version == 0x0304 else 16)
    inbuf, offs = _pack(records)
    d_in = _t(inbuf)
    d_body = torch.full_like(d_in, 0x5a)
    d_pre = torch.full((n * pl,), 0x5a, dtype=torch.uint8, device=DEV)
    d_suf = torch.full((n * sl,), 0x5a, dtype=torch.uint8, device=DEV)
    d_types = _t(np.array(types, np.uint8))
    d_st = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    d_offs, d_lens = _t(offs.astype(np.int64)), _t(np.array(lens, np.int64))
    # Two batches on one context: the sequence number carries over.
    h = n // 2
    for lo, hi in ((0, h), (h, n)):
        r = ba.make_tls_records(hi - lo, d_in, d_body, d_pre[lo * pl:], d_suf[lo * sl:],
                                offsets=d_offs[lo:], lengths=d_lens[lo:], types=d_types[lo:],
                                status=d_st[lo:])
        sealer.seal_records_device(r)
    torch.cuda.synchronize()
    assert sealer.sequence == seq0 + n
    body, pre, suf = d_body.cpu().numpy(), d_pre.cpu().numpy(), d_suf.cpu().numpy()
    st = d_st.cpu().numpy()
    for i in range(n):
        b = body[int(offs[i]):int(offs[i]) + lens[i]].tobytes()
        if expect[i] is None:
            assert st[i] == 0 and b == bytes(lens[i]), i
            continue
        e_pre, e_body, e_suf = expect[i]
        assert st[i] == 1, i
        assert pre[i * pl:(i + 1) * pl].tobytes() == e_pre, i
        assert b == e_body, i
        assert suf[i * sl:(i + 1) * sl].tobytes() == e_suf, i

    # Open the wire records (in place) with a reader at the same sequence.
    d_suf_bad = d_suf.clone()
    d_suf_bad[3 * sl] ^= 1  # record 3: corrupted (TLS 1.3: its sealed inner type)
    opener = ba.TlsAead(ba.evp_aead_open, version, aead, key, fixed_iv, seq0)
    d_otypes = torch.zeros(n, dtype=torch.uint8, device=DEV)
    d_st2 = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    r = ba.make_tls_records(n, d_body, d_body, d_pre, d_suf_bad, offsets=d_offs, lengths=d_lens,
                            types=d_otypes, status=d_st2)
    opener.open_records_device(r)
    torch.cuda.synchronize()
    body2, st2, ot = d_body.cpu().numpy(), d_st2.cpu().numpy(), d_otypes.cpu().numpy()
    for i in range(n):
        b = body2[int(offs[i]):int(offs[i]) + lens[i]].tobytes()
        if expect[i] is None or i == 3:
            assert st2[i] == 0 and b == bytes(lens[i]), i
            continue
        assert st2[i] == 1 and b == records[i] and ot[i] == types[i], i


def test_tls_record_layer_errors():
    key, iv = bytes(16), bytes(12)
    with pytest.raises(ba.AEADError) as e:  # TLS 1.2 AES-GCM wants a 4-byte fixed IV
        ba.TlsAead(ba.evp_aead_seal, 0x0303, "aes-128-gcm", key, iv)
    assert e.value.reason == ba.CIPHER_R_INVALID_NONCE_SIZE
    t = ba.TlsAead(ba.evp_aead_seal, 0x0304, "aes-128-gcm", key, iv, seq=(1 << 64) - 2)
    d = torch.zeros(64, dtype=torch.uint8, device=DEV)
    r = ba.make_tls_records(2, d, d, d, d, record_len=0, record_stride=16)
    with pytest.raises(ba.AEADError):  # the sequence number would wrap (tls_record.cc:305)
        t.seal_records_device(r)
    assert t.sequence == (1 << 64) - 2
    with pytest.raises(ba.AEADError) as e:
        t.open_records_device(r)
    assert e.value.reason == ba.CIPHER_R_INVALID_OPERATION


# ---------------------------------------------------------------------------
# iovec batches: N EVP_AEAD_CTX_sealv / _openv_detached calls over device
# chunks (aead.cc.inc:316-361, 531-584).

def _split(rng, data, max_parts):
    k = rng.randint(1, max_parts)
    cuts = sorted(rng.randint(0, len(data)) for _ in range(k - 1))
    parts, prev = [], 0
    for c in cuts + [len(data)]:
        parts.append(data[prev:c])
        prev = c
    return parts


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
def test_iovec_batch_vs_oracle(aead):
    rng = random.Random(hash(aead) & 0xffff)
    key = bytes(rng.getrandbits(8) for _ in range(AEAD_KEYLEN[aead]))
    nl = _nl(aead)
    n = 150
    pts = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 15, 16, 17, 100, 1350,
                                                                   5000, 16384])))
           for _ in range(n)]
    ads = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 5, 13, 40]))) for _ in range(n)]
    nonces = [bytes(rng.getrandbits(8) for _ in range(nl)) for _ in range(n)]
    inplace = [rng.random() < 0.3 for _ in range(n)]
    # Chunks at random (often odd) offsets of one input arena; outputs at the
    # same offsets of an output arena, or in place.
    chunks, starts, ad_chunks, ad_starts = [], [0], [], [0]
    pos, apos = 0, 0
    for i in range(n):
        for part in _split(rng, pts[i], 5):
            pos += rng.randint(0, 7)
            chunks.append((pos, part, inplace[i]))
            pos += len(part)
        starts.append(len(chunks))
        for part in _split(rng, ads[i], 3):
            apos += rng.randint(0, 3)
            ad_chunks.append((apos, part))
            apos += len(part)
        ad_starts.append(len(ad_chunks))
    src = np.zeros(pos + 16, dtype=np.uint8)
    for off, part, _ in chunks:
        src[off:off + len(part)] = np.frombuffer(part, dtype=np.uint8)
    adbuf = np.zeros(apos + 16, dtype=np.uint8)
    for off, part in ad_chunks:
        adbuf[off:off + len(part)] = np.frombuffer(part, dtype=np.uint8)
    d_src, d_ad = _t(src), _t(adbuf)
    d_dst = torch.zeros_like(d_src)
    sb, db, ab = d_src.data_ptr(), d_dst.data_ptr(), d_ad.data_ptr()
    iov = np.array([(sb + off if ip else db + off, sb + off, len(part)) for off, part, ip in chunks],
                   dtype=np.int64).reshape(-1, 3)
    aiv = np.array([(ab + off, len(part)) for off, part in ad_chunks], dtype=np.int64).reshape(-1, 2)
    d_iov, d_aiv = _t(iov), _t(aiv)
    d_starts, d_astarts = _t(np.array(starts, np.int64)), _t(np.array(ad_starts, np.int64))
    d_nonce = _t(np.frombuffer(b"".join(nonces), dtype=np.uint8).copy())
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=DEV)
    d_st = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    ctx = ba.AEADCtx(aead, key, 16)
    b = ba.make_iov_batch(n, d_iov, d_starts, d_tags, d_nonce, nl, aadvecs=d_aiv,
                          aadvec_start=d_astarts, status=d_st)
    ctx.sealv_batch_device(b)
    torch.cuda.synchronize()
    assert d_st.cpu().tolist() == [1] * n
    out_src, out_dst, tags = d_src.cpu().numpy(), d_dst.cpu().numpy(), d_tags.cpu().numpy()

    def gather(i, a, b_):
        return b"".join((a if chunks[c][2] else b_)[chunks[c][0]:chunks[c][0] + len(chunks[c][1])]
                        .tobytes() for c in range(starts[i], starts[i + 1]))

    cts = []
    for i in range(n):
        ok, ct, tag = o.seal(ORACLE_ID[aead], key, nonces[i], pts[i], ads[i])
        got = gather(i, out_src, out_dst)
        assert ok and got == ct and tags[16 * i:16 * i + 16].tobytes() == tag, (i, len(pts[i]))
        cts.append(ct)
    # Open the ciphertext chunks (where the seal left them) into a third arena;
    # corrupt every 7th tag: those records fail and their chunks are zeroed.
    d_back = torch.full_like(d_src, 0xAA)
    kb = d_back.data_ptr()
    iov2 = np.array([(kb + off, (sb if ip else db) + off, len(part)) for off, part, ip in chunks],
                    dtype=np.int64).reshape(-1, 3)
    bad = set(range(0, n, 7))
    tg = tags.copy()
    for i in bad:
        tg[16 * i] ^= 1
    d_st.fill_(7)
    b2 = ba.make_iov_batch(n, _t(iov2), d_starts, _t(tg), d_nonce, nl, aadvecs=d_aiv,
                           aadvec_start=d_astarts, status=d_st)
    ctx.openv_detached_batch_device(b2)
    torch.cuda.synchronize()
    st, back = d_st.cpu().numpy(), d_back.cpu().numpy()
    for i in range(n):
        got = b"".join(back[chunks[c][0]:chunks[c][0] + len(chunks[c][1])].tobytes()
                       for c in range(starts[i], starts[i + 1]))
        if i in bad:
            assert st[i] == 0 and got == bytes(len(pts[i])), i
        else:
            assert st[i] == 1 and got == pts[i], i


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
@pytest.mark.parametrize("n", [300, 4500])
def test_iovec_in_place_walk(aead, n):
    """Every AEAD's kernels walk iovec chunks in place
    (BatchDesc::iovecs): chunks of 0..4097 bytes incl. empty and 1-byte
    chunks, input and output at independent alignments 0..15 (so the loads
    and the stores shift by different amounts), blocks straddling several
    chunks, records up to 32 KiB, AD of up to 100 bytes in one or two
    chunks, and >= 4096 records (length-ordered schedule; AES-GCM runs the
    records below 2 KiB, of 2-4 KiB and of 4 KiB or more as three launches);
    seal vs the oracle, then open with a corrupted tag zeroing that record's chunks."""
    rng = random.Random(n * 31 + len(aead))
    key = bytes(rng.getrandbits(8) for _ in range(AEAD_KEYLEN[aead]))
    nl = _nl(aead)
    lens = [rng.choice([0, 1, 15, 16, 17, 31, 63, 64, 65, 255, 1350, 2047, 2048, 3000, 4095, 4096,
                        16384, 16397, 32768])
            for _ in range(n)]
    pts = [rng.randbytes(L) for L in lens]
    ads = [rng.randbytes(rng.choice([0, 5, 13, 29, 64, 100])) for _ in range(n)]
    nonces = [rng.randbytes(nl) for _ in range(n)]
    chunks, starts = [], [0]  # (in_off, out_off, bytes)
    ipos, opos = 0, 0
    for i in range(n):
        data, k = pts[i], 0
        while k < len(data) or (k == 0 and rng.random() < 0.5):
            size = rng.choice([0, 1, 2, 3, 15, 16, 17, 64, 255, 1000, 4097, 1 << 20])
            part = data[k:k + size]
            ipos += rng.randint(0, 15)
            opos += rng.randint(0, 15)
            chunks.append((ipos, opos, part))
            ipos += len(part)
            opos += len(part)
            k += len(part)
            if size == 0 and k >= len(data):
                break
        starts.append(len(chunks))
    src = np.zeros(ipos + 32, dtype=np.uint8)
    for io, _, part in chunks:
        src[io:io + len(part)] = np.frombuffer(part, dtype=np.uint8)
    adbuf, ad_offs = _pack(ads, 1)
    d_src, d_ad = _t(src), _t(adbuf)
    d_dst = torch.zeros(opos + 32, dtype=torch.uint8, device=DEV)
    sb, db, ab = d_src.data_ptr(), d_dst.data_ptr(), d_ad.data_ptr()
    iov = np.array([(db + oo, sb + io, len(p)) for io, oo, p in chunks], dtype=np.int64)
    # AD longer than 10 bytes in two chunks (cut at a random point).
    aiv_l, astarts = [], [0]
    for i in range(n):
        a0, la = int(ad_offs[i]), len(ads[i])
        if la > 10:
            cut = rng.randint(1, la - 1)
            aiv_l += [(ab + a0, cut), (ab + a0 + cut, la - cut)]
        else:
            aiv_l.append((ab + a0, la))
        astarts.append(len(aiv_l))
    aiv = np.array(aiv_l, dtype=np.int64)
    d_starts = _t(np.array(starts, np.int64))
    d_astarts = _t(np.array(astarts, np.int64))
    d_nonce = _t(np.frombuffer(b"".join(nonces), dtype=np.uint8).copy())
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=DEV)
    d_st = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    ctx = ba.AEADCtx(aead, key, 16)
    b = ba.make_iov_batch(n, _t(iov.reshape(-1, 3)), d_starts, d_tags, d_nonce, nl,
                          aadvecs=_t(aiv.reshape(-1, 2)), aadvec_start=d_astarts, status=d_st)
    ctx.sealv_batch_device(b)
    torch.cuda.synchronize()
    assert d_st.cpu().tolist() == [1] * n
    out, tags = d_dst.cpu().numpy(), d_tags.cpu().numpy()
    cts = []
    for i in range(n):
        ok, ct, tag = o.seal(ORACLE_ID[aead], key, nonces[i], pts[i], ads[i])
        got = b"".join(out[oo:oo + len(p)].tobytes() for _, oo, p in chunks[starts[i]:starts[i + 1]])
        assert ok and got == ct and tags[16 * i:16 * i + 16].tobytes() == tag, (i, lens[i])
        cts.append(ct)
    # Open in place (out == in on the ciphertext arena), one corrupted tag.
    bad = {3, n // 2}
    tg = tags.copy()
    for i in bad:
        tg[16 * i + 5] ^= 0x10
    iov2 = np.array([(db + oo, db + oo, len(p)) for _, oo, p in chunks], dtype=np.int64)
    d_st.fill_(7)
    b2 = ba.make_iov_batch(n, _t(iov2.reshape(-1, 3)), d_starts, _t(tg), d_nonce, nl,
                           aadvecs=_t(aiv.reshape(-1, 2)), aadvec_start=d_astarts, status=d_st)
    ctx.openv_detached_batch_device(b2)
    torch.cuda.synchronize()
    st, back = d_st.cpu().numpy(), d_dst.cpu().numpy()
    for i in range(n):
        got = b"".join(back[oo:oo + len(p)].tobytes() for _, oo, p in chunks[starts[i]:starts[i + 1]])
        if i in bad:
            assert st[i] == 0 and got == bytes(lens[i]), i
        else:
            assert st[i] == 1 and got == pts[i], i


@pytest.mark.multigpu
def test_context_used_from_another_device():
    """A context created on GPU 0 and used after the thread switched to GPU 1:
    host-buffer calls run on the key's device (and restore the caller's
    device); device-batch calls on the wrong device fail cleanly instead of
    launching kernels against another GPU's key memory.  Needs two GPUs
    (deselected elsewhere, tests/conftest.py)."""
    key, nonce = bytes(range(16)), bytes(12)
    ctx = ba.AEADCtx("aes-128-gcm", key, 16)
    ok, ct, tag = o.seal(o.AES_GCM, key, nonce, b"hello", b"ad")
    try:
        ba.set_device(1)
        torch.cuda.set_device(1)
        assert ctx.seal(nonce, b"hello", b"ad") == ct + tag
        assert ctx.open(nonce, ct + tag, b"ad") == b"hello"
        assert torch.cuda.current_device() == 1
        d = torch.zeros(64, dtype=torch.uint8, device="cuda:1")
        with pytest.raises(ba.AEADError) as e:
            ctx.seal_batch_device(ba.make_batch(1, d, d, d, d, 12, d, record_len=16,
                                                record_stride=16))
        assert e.value.reason == 66  # ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED
    finally:
        ba.set_device(0)
        torch.cuda.set_device(0)
