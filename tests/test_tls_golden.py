"""TLS record framing pinned to the reference (missing #2).

tests/golden/ref_tls.json holds TLS 1.2 / 1.3 records sealed by the
reference's own record-protection code -- SSLAEADContext::Create and
SealScatter (ssl/ssl_aead_ctx.cc:44-123, 299-381) compiled from
/root/reference by oracle/ref/Makefile into oracle/_ref/ref_tls, framed as
do_seal_record frames them (ssl/tls_record.cc:266-317) -- for AES-128-GCM,
AES-256-GCM and ChaCha20-Poly1305, record types 21/22/23, lengths 0..16384,
sequence numbers from 0 and from 0x1234567890 (TLS 1.3 AES-GCM from 0 only:
its tls13 AEAD requires it, e_aes.cc.inc:1180-1185).

* CPU: the Python restatement the other TLS tests use (tls_util) reproduces
  every golden record.
* GPU: BSSL_AMD_TLS_AEAD (include/bssl_amd/tls.h) seals the same records in
  two device batches and reproduces every prefix (header || explicit nonce),
  body and suffix (sealed inner type || tag); a reader opens them back.
"""
import hashlib

import numpy as np
import pytest

import tls_util
from golden_util import load

CASES = load("ref_tls.json")
IDS = [f"v{c['version']:x}-{c['aead']}-seq{c['seq0']:x}" for c in CASES]


def _records(case):
    recs = [tls_util.fill_bytes(r["len"], r["pt_seed"]) for r in case["records"]]
    types = [r["type"] for r in case["records"]]
    return recs, types


def _body_matches(golden, body):
    if golden.startswith("sha256:"):
        return hashlib.sha256(body).hexdigest() == golden[7:]
    return body.hex() == golden


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_restatement_matches_reference(case):
    key, iv = bytes.fromhex(case["key"]), bytes.fromhex(case["fixed_iv"])
    recs, types = _records(case)
    got = tls_util.tls_seal_restated(case["version"], case["aead"], key, iv, case["seq0"], recs,
                                     types)
    for r, g in zip(case["records"], got):
        pre, body, suf = g
        assert pre.hex() == r["prefix"], r["seq"]
        assert _body_matches(r["body"], body), r["seq"]
        assert suf.hex() == r["suffix"], r["seq"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_tls_shim_matches_reference(case):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import boringssl_amd as ba
    dev = "cuda:0"
    key, iv = bytes.fromhex(case["key"]), bytes.fromhex(case["fixed_iv"])
    recs, types = _records(case)
    n = len(recs)
    lens = [len(x) for x in recs]
    offs = np.zeros(n, dtype=np.int64)
    pos = 0
    for i, L in enumerate(lens):
        offs[i] = pos
        pos += (L + 15) // 16 * 16
    buf = np.zeros(max(pos, 16), dtype=np.uint8)
    for i, x in enumerate(recs):
        buf[offs[i]:offs[i] + len(x)] = np.frombuffer(x, dtype=np.uint8)
    sealer = ba.TlsAead(ba.evp_aead_seal, case["version"], case["aead"], key, iv, case["seq0"])
    pl, sl = sealer.prefix_len, sealer.suffix_len
    d_in = torch.from_numpy(buf).to(dev)
    d_body = torch.zeros_like(d_in)
    d_pre = torch.zeros(n * pl, dtype=torch.uint8, device=dev)
    d_suf = torch.zeros(n * sl, dtype=torch.uint8, device=dev)
    d_types = torch.tensor(types, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_offs = torch.from_numpy(offs).to(dev)
    d_lens = torch.tensor(lens, dtype=torch.int64, device=dev)
    h = n // 3  # two batches on one context: the sequence number carries over
    for lo, hi in ((0, h), (h, n)):
        r = ba.make_tls_records(hi - lo, d_in, d_body, d_pre[lo * pl:], d_suf[lo * sl:],
                                offsets=d_offs[lo:], lengths=d_lens[lo:], types=d_types[lo:],
                                status=d_st[lo:])
        sealer.seal_records_device(r)
    torch.cuda.synchronize()
    assert sealer.sequence == case["seq0"] + n
    assert bool(d_st.all())
    body, pre, suf = d_body.cpu().numpy(), d_pre.cpu().numpy(), d_suf.cpu().numpy()
    for i, r in enumerate(case["records"]):
        assert pre[i * pl:(i + 1) * pl].tobytes().hex() == r["prefix"], r["seq"]
        assert _body_matches(r["body"], body[offs[i]:offs[i] + lens[i]].tobytes()), r["seq"]
        assert suf[i * sl:(i + 1) * sl].tobytes().hex() == r["suffix"], r["seq"]
    opener = ba.TlsAead(ba.evp_aead_open, case["version"], case["aead"], key, iv, case["seq0"])
    d_ot = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_st.zero_()
    r = ba.make_tls_records(n, d_body, d_body, d_pre, d_suf, offsets=d_offs, lengths=d_lens,
                            types=d_ot, status=d_st)
    opener.open_records_device(r)
    torch.cuda.synchronize()
    assert bool(d_st.all())
    assert torch.equal(d_body, d_in) and d_ot.cpu().tolist() == types
