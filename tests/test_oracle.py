"""CPU tests: the oracle (oracle/aead_oracle.c) against the reference's own
known-answer data and against the reference library's outputs.

Pins the checker before it is trusted by the GPU parity tests
(crypto/cipher/aead_test.cc:188-281 TestVector, :1493-1564 Wycheproof;
crypto/fipsmodule/aes/aes_test.cc:154-166; crypto/poly1305/poly1305_test.cc:75).
"""
import numpy as np
import pytest

import oracle_lib as o
from golden_util import AEAD_KEYLEN, batch_digests, load

AEAD_ID = {"aes-128-gcm": o.AES_GCM, "aes-192-gcm": o.AES_GCM, "aes-256-gcm": o.AES_GCM,
           "chacha20-poly1305": o.CHACHA20_POLY1305, "xchacha20-poly1305": o.XCHACHA20_POLY1305,
           "aes-128-gcm-siv": o.AES_GCM_SIV, "aes-256-gcm-siv": o.AES_GCM_SIV}


def _h(s):
    return bytes.fromhex(s)


def test_aes_raw_kat():
    # Only the "Raw" blocks are on the AEAD path; KeyWrap modes are out of scope.
    cases = [c for c in load("kat_aes.json") if c["mode"] == "Raw"]
    assert len(cases) == 3
    for c in cases:
        assert o.aes_block(_h(c["key"]), _h(c["pt"])).hex() == c["ct"], c["source"]


def test_poly1305_kat():
    cases = load("kat_poly1305.json")
    assert len(cases) >= 30
    for c in cases:
        assert o.poly1305(_h(c["key"]), _h(c["input"])).hex() == c["mac"], c["source"]


@pytest.mark.parametrize("aead", ["aes-128-gcm", "aes-192-gcm", "aes-256-gcm", "chacha20-poly1305",
                                  "xchacha20-poly1305", "aes-128-gcm-siv", "aes-256-gcm-siv"])
def test_aead_kat_files(aead):
    cases = [c for c in load("kat_aead.json") if c["aead"] == aead]
    assert cases
    aid = AEAD_ID[aead]
    for c in cases:
        key, nonce, ad, pt, ct, tag = (_h(c[k]) for k in ("key", "nonce", "ad", "pt", "ct", "tag"))
        tag_len = c.get("tag_len", len(tag))
        if c["valid"]:
            ok, got_ct, got_tag = o.seal(aid, key, nonce, pt, ad, tag_len)
            assert ok and got_ct == ct and got_tag == tag, c["source"]
            ok, got_pt = o.open_(aid, key, nonce, ct, ad, tag)
            assert ok and got_pt == pt, c["source"]
            # bit flip in the tag must be rejected (aead_test.cc:262-281)
            if tag:
                bad = bytearray(tag)
                bad[0] ^= 1
                ok, got_pt = o.open_(aid, key, nonce, ct, ad, bytes(bad))
                assert not ok and got_pt == bytes(len(ct)), c["source"]
        else:
            if len(tag) != tag_len:
                continue  # truncated-tag files: rejected by the API length check
            ok, got_pt = o.open_(aid, key, nonce, ct, ad, tag)
            assert not ok, c["source"]


def test_hchacha20_kat():
    # draft-irtf-cfrg-xchacha-03 section 2.2.1 test vector (the construction of
    # CRYPTO_hchacha20, crypto/chacha/chacha.cc:43-63).
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a0000000031415927")
    assert o.hchacha20(key, nonce).hex() == (
        "82413b4227b27bfed30e42508a877d73a0f9e4d58a74a853c12ec41326d3ecdc")


def test_ref_edge_cases():
    cases = load("ref_edge.json")
    assert len(cases) > 200
    for c in cases:
        aid = AEAD_ID[c["aead"]]
        key, nonce, ad, pt, ct, tag = (_h(c[k]) for k in ("key", "nonce", "ad", "pt", "ct", "tag"))
        ok, got_ct, got_tag = o.seal(aid, key, nonce, pt, ad, len(tag))
        assert ok and got_ct == ct and got_tag == tag, (c["aead"], len(pt), len(nonce), len(ad))


def _parity_batch(aead, nkeys, rpk, length):
    n = nkeys * rpk
    lens = [o.synth_mixed_len(i) for i in range(n)] if length == "mixed" else [int(length)] * n
    lens = np.array(lens, dtype=np.uint64)
    pt, offsets, nonces, ads = o.synth_batch(0, lens)
    key_len = AEAD_KEYLEN[aead]
    keys = o.synth_keys(nkeys, key_len)
    key_index = (np.arange(n, dtype=np.uint32) // np.uint32(rpk)).astype(np.uint32)
    return lens, pt, offsets, nonces, ads, keys, key_index, key_len


@pytest.mark.parametrize("name", ["parity_aes128_16k", "parity_aes256_mixed", "parity_chacha_1350",
                                  "parity_multikey_aes128", "parity_xchacha_1350",
                                  "parity_siv128_1350", "parity_siv256_mixed",
                                  "parity_siv128_multikey"])
def test_oracle_batch_matches_reference_digest(name):
    g = load("ref_digests.json")[name]
    aead = g["aead"]
    lens, pt, offsets, nonces, ads, keys, key_index, key_len = _parity_batch(
        aead, g["nkeys"], g["records_per_key"], g["len"])
    n = len(lens)
    out = np.zeros_like(pt)
    tags = np.zeros(16 * n, dtype=np.uint8)
    ad_off = (np.arange(n, dtype=np.uint64) * np.uint64(13))
    ad_len = np.full(n, 13, dtype=np.uint64)
    nl = 12
    if aead == "xchacha20-poly1305":
        nonces, nl = o.xchacha_nonces(nonces), 24
    failed = o.batch(AEAD_ID[aead], 1, keys, key_len, key_index, pt, out, offsets, lens, nonces, nl,
                     ads, ad_off, ad_len, tags, 16)
    assert failed == 0
    tags_d, ct_d = batch_digests(out, offsets, lens, tags)
    assert tags_d == g["tags_sha256"]
    assert ct_d == g["ct_sha256"]
    # round trip through open
    back = np.zeros_like(pt)
    status = np.zeros(n, dtype=np.uint8)
    failed = o.batch(AEAD_ID[aead], 0, keys, key_len, key_index, out, back, offsets, lens, nonces,
                     nl, ads, ad_off, ad_len, tags, 16, status)
    assert failed == 0 and status.all()
    assert np.array_equal(back, pt)
