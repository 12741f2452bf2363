"""Per-key AES-GCM setup (key_sched.h): the tables the kernels read, built on
the host (EVP_AEAD_CTX_init) and by the device key-setup kernel (keysets).

The reference's CRYPTO_gcm128_init_aes_key (crypto/fipsmodule/aes/
gcm.cc.inc:253-296) derives the AES schedule (aes_nohw.cc.inc:935-1114) and H
= E_K(0^128).  CPU tests pin the host tables three ways: byte for byte to the
round-4 host implementation (tests/golden/gcm_key_tables.json, made by
tools/golden/gen_key_tables.py), the schedule to a FIPS-197 restatement here,
and H, H^k and the H^16 nibble table to the oracle's AES and GHASH multiply.
The GPU test requires the device kernel's tables to equal the host's."""
import hashlib
import json
import os
import random
import struct

import pytest

import oracle_lib as ol

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gcm_key_tables.json")
SIZE = 12816
# GcmKeyDev field offsets (boringssl_amd/csrc/internal.h)
O_RK, O_NR, O_RKP, O_HPOW, O_HTAB, O_BSM = 0, 240, 256, 496, 784, 8976


def _sbox():
    def mul(a, b):
        p = 0
        while b:
            if b & 1:
                p ^= a
            a = ((a << 1) ^ (0x11b if a & 0x80 else 0)) & 0x1ff
            b >>= 1
        return p
    s = []
    for x in range(256):
        inv = 0 if x == 0 else next(y for y in range(1, 256) if mul(x, y) == 1)
        r = v = inv
        for _ in range(4):
            v = ((v << 1) | (v >> 7)) & 0xff
            r ^= v
        s.append(r ^ 0x63)
    return s


S = _sbox()


def fips197_schedule(key):
    """FIPS-197 5.2 KeyExpansion as little-endian words."""
    nk = len(key) // 4
    nr = nk + 6
    w = [list(key[4 * i:4 * i + 4]) for i in range(nk)]
    rcon = 1
    for i in range(nk, 4 * (nr + 1)):
        t = list(w[i - 1])
        if i % nk == 0:
            t = [S[t[1]] ^ rcon, S[t[2]], S[t[3]], S[t[0]]]
            rcon = ((rcon << 1) ^ (0x1b if rcon & 0x80 else 0)) & 0xff
        elif nk == 8 and i % nk == 4:
            t = [S[b] for b in t]
        w.append([a ^ b for a, b in zip(w[i - nk], t)])
    return nr, [struct.unpack("<I", bytes(x))[0] for x in w]


def gf_prep(v):
    """gf128_ct.h gf_prep on the big-endian integer of a block."""
    top = v >> 127
    r = (v << 1) & ((1 << 128) - 1)
    if top:
        r ^= 1 | (0xc2 << 120)
    return r


def words_le(b, off, n):
    return list(struct.unpack_from("<%dI" % n, b, off))


def golden():
    return json.load(open(GOLDEN))


def test_golden_fixture_shape():
    g = golden()
    assert g["struct_bytes"] == SIZE
    assert sorted({len(r["key"]) // 2 for r in g["tables"]}) == [16, 24, 32]


@pytest.mark.parametrize("key_len", [16, 24, 32])
def test_host_tables_match_round4_digests(key_len):
    import boringssl_amd as ba
    rows = [r for r in golden()["tables"] if len(r["key"]) == 2 * key_len]
    keys = b"".join(bytes.fromhex(r["key"]) for r in rows)
    tabs = ba.gcm_key_tables(keys, key_len, on_device=False)
    assert [hashlib.sha256(t).hexdigest() for t in tabs] == [r["sha256"] for r in rows]


@pytest.mark.parametrize("key_len", [16, 24, 32])
def test_host_tables_vs_fips197_and_oracle(key_len):
    import boringssl_amd as ba
    rng = random.Random(key_len)
    keys = [bytes(rng.randrange(256) for _ in range(key_len)) for _ in range(6)]
    tabs = ba.gcm_key_tables(b"".join(keys), key_len, on_device=False)
    for key, t in zip(keys, tabs):
        assert len(t) == SIZE
        nr, w = fips197_schedule(key)
        assert words_le(t, O_NR, 2) == [nr, key_len]
        rkp = words_le(t, O_RKP, 60)
        rk = words_le(t, O_RK, 60)
        for r in range(15):
            for c in range(4):
                v = w[4 * r + c] if r <= nr else 0
                assert rkp[4 * r + c] == v
                rot = v if r in (0, nr) else ((v << 16) | (v >> 16)) & 0xffffffff
                assert rk[4 * r + c] == rot
        bsm = words_le(t, O_BSM, 15 * 64)
        for r in range(15):
            for i in range(64):
                h, bit = i >> 5, i & 31
                lo = (w[4 * r + h] >> bit) & 1 if r <= nr else 0
                hi = (w[4 * r + h + 2] >> bit) & 1 if r <= nr else 0
                assert bsm[64 * r + i] == lo * 0xffff | hi * 0xffff0000
        # H = E_K(0), its powers as prepared multipliers, H^16 in the nibble table
        H = ol.aes_block(key, bytes(16))
        hk = H
        hp = words_le(t, O_HPOW, 72)
        assert hp[0:4] == [0, 0, 0, 0]
        for k in range(1, 18):
            v = gf_prep(int.from_bytes(hk, "big"))
            assert hp[4 * k:4 * k + 4] == [(v >> (32 * j)) & 0xffffffff for j in range(4)], k
            if k == 16:
                h16 = hk
            hk = ol.gf128_mul(hk, H)
        # htab16[0][8]: nibble 8 in the high nibble of byte 0 = x^0, i.e. H^16
        assert t[O_HTAB + 8 * 16:O_HTAB + 9 * 16] == h16
        # htab16[pos][val] is linear in val
        for pos in (0, 7, 31):
            base = O_HTAB + pos * 256
            ent = [int.from_bytes(t[base + 16 * v:base + 16 * v + 16], "little") for v in range(16)]
            assert ent[0] == 0
            for v in range(16):
                assert ent[v] == ent[v & 8] ^ ent[v & 4] ^ ent[v & 2] ^ ent[v & 1]


def test_bad_key_length_rejected():
    import boringssl_amd as ba
    with pytest.raises(RuntimeError):
        ba.gcm_key_tables(bytes(20), 20, on_device=False)


@pytest.mark.gpu
@pytest.mark.parametrize("key_len", [16, 24, 32])
def test_device_key_setup_matches_host(key_len):
    """The keyset path (device kernel, one lane per key) and the single-key path
    (host) give byte-identical tables: the golden keys plus 1,000 random keys
    (not a multiple of the 64-lane block)."""
    import boringssl_amd as ba
    rows = [r for r in golden()["tables"] if len(r["key"]) == 2 * key_len]
    rng = random.Random(1000 + key_len)
    keys = b"".join(bytes.fromhex(r["key"]) for r in rows)
    keys += bytes(rng.randrange(256) for _ in range(1000 * key_len))
    dev = ba.gcm_key_tables(keys, key_len, on_device=True)
    host = ba.gcm_key_tables(keys, key_len, on_device=False)
    assert len(dev) == len(host) == len(rows) + 1000
    bad = [i for i in range(len(dev)) if dev[i] != host[i]]
    assert not bad, bad[:8]
    assert [hashlib.sha256(t).hexdigest() for t in dev[:len(rows)]] == [r["sha256"] for r in rows]
