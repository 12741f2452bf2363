"""Uniform keyset batches through the T-table keyset kernel (gcm.hip
gcm_keyset_kernel): tiles of one key's 64 records beside a tile of two keys
(two passes) and a partial last tile in one launch, AES-128/256, 12- and
16-byte nonces (J0 by GHASH), seal, open in place and one tampered record
per tile (status 0, plaintext zero-filled), every record and tag against the
CPU oracle (oracle/aead_oracle.c, following gcm.cc.inc:298-604).  Round 6
ran these records through record segments of the tiles (one key's records
split into 16 x nseg units claimed from an LDS counter); the
segments measured slower and were reverted, the test stays as the keyset
kernel's uniform-layout parity check.  The reference handles each key's
records independently (gcm.cc.inc:253-296, aead.cc.inc:70-106).
"""
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import boringssl_amd as ba  # noqa: E402
import oracle_lib as o  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KEYLEN = {"aes-128-gcm": 16, "aes-256-gcm": 32}


def _key_index(n):
    """Tile t (64 records) uses key t, except tile 2, whose records alternate
    between two keys (a two-pass tile: whole records)."""
    ki = np.arange(n, dtype=np.int64) // 64
    tile2 = np.arange(n) // 64 == 2
    ki[tile2] = 2 + (np.arange(n)[tile2] & 1) * 10
    return ki.astype(np.int32)


@pytest.mark.parametrize("aead,rlen,nl", [("aes-128-gcm", 8192, 12), ("aes-256-gcm", 16384, 12),
                                          ("aes-128-gcm", 12288, 16)])
def test_keyset_tiles_vs_oracle(aead, rlen, nl, aes_engine):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    aes_engine("table")
    rng = np.random.default_rng(zlib.crc32(repr((aead, rlen, nl)).encode()))
    n = 64 * 5 + 37
    nkeys = 13
    kl = KEYLEN[aead]
    keys = rng.integers(0, 256, size=nkeys * kl, dtype=np.uint8)
    ki = _key_index(n)
    recs = rng.integers(0, 256, size=(n, rlen), dtype=np.uint8)
    nonces = rng.integers(0, 256, size=n * nl, dtype=np.uint8)
    ad_len = 13
    ad = rng.integers(0, 256, size=n * ad_len, dtype=np.uint8)

    d_pt = torch.from_numpy(recs.reshape(-1).copy()).to(DEV)
    d_ct = torch.zeros_like(d_pt)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=DEV)
    d_st = torch.zeros(n, dtype=torch.uint8, device=DEV)
    d_n = torch.from_numpy(nonces).to(DEV)
    d_ad = torch.from_numpy(ad).to(DEV)
    d_ki = torch.from_numpy(ki).to(DEV)
    ks = ba.Keyset(aead, keys.tobytes(), nkeys, 16)
    b = ba.make_batch(n, d_pt, d_ct, d_tags, d_n, nl, d_ad, record_stride=rlen, record_len=rlen,
                      ad_stride=ad_len, ad_len=ad_len, status=d_st, key_index=d_ki)
    ks.seal_batch_device(b)
    torch.cuda.synchronize()
    assert bool(d_st.all())

    flat = recs.reshape(-1)
    ref = np.zeros_like(flat)
    ref_tags = np.zeros(16 * n, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(rlen)
    lens = np.full(n, rlen, dtype=np.uint64)
    adoff = np.arange(n, dtype=np.uint64) * np.uint64(ad_len)
    adl = np.full(n, ad_len, dtype=np.uint64)
    assert o.batch(o.AES_GCM, 1, keys, kl, ki.astype(np.uint32), flat, ref, offs, lens, nonces, nl,
                   ad, adoff, adl, ref_tags, 16) == 0
    got = d_ct.cpu().numpy()
    bad = np.nonzero((got.reshape(n, rlen) != ref.reshape(n, rlen)).any(axis=1))[0]
    assert bad.size == 0, f"records differ from the oracle: {bad[:8].tolist()}"
    gt = d_tags.cpu().numpy().reshape(n, 16)
    badt = np.nonzero((gt != ref_tags.reshape(n, 16)).any(axis=1))[0]
    assert badt.size == 0, f"tags differ from the oracle: {badt[:8].tolist()}"

    # Open in place with one tampered record per segmented tile: status 0 and
    # its plaintext zero-filled; every other record opens to its plaintext.
    bad_recs = [5, 64 + 63, 3 * 64 + 17]
    ct = d_ct.clone()
    for r in bad_recs:
        ct[r * rlen + rlen // 2] ^= 1
    d_st.zero_()
    b2 = ba.make_batch(n, ct, ct, d_tags, d_n, nl, d_ad, record_stride=rlen, record_len=rlen,
                       ad_stride=ad_len, ad_len=ad_len, status=d_st, key_index=d_ki)
    ks.open_batch_device(b2)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    assert [i for i in range(n) if not st[i]] == bad_recs
    back = ct.cpu().numpy().reshape(n, rlen)
    good = np.ones(n, dtype=bool)
    good[bad_recs] = False
    assert np.array_equal(back[good], recs[good])
    assert not back[bad_recs].any()
