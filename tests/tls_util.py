"""TLS record-layer helpers shared by the CPU and GPU tests.

tls_seal_restated: a Python restatement, over the CPU oracle's AEAD, of the
reference's record sealing -- SSLAEADContext::Create / SealScatter
(ssl/ssl_aead_ctx.cc:44-123, 207-224, 299-381) framed by do_seal_record
(ssl/tls_record.cc:266-317).  Pinned to the reference itself by
tests/golden/ref_tls.json (records sealed by the reference's own
SSLAEADContext, oracle/ref/ref_tls.cc) in tests/test_tls_golden.py.
"""
import oracle_lib as o

TLS1_2_VERSION, TLS1_3_VERSION = 0x0303, 0x0304


def tls_seal_restated(version, aead, key, fixed_iv, seq0, records, types):
    """[(prefix, body, suffix) or None for a record over 16384 bytes]."""
    tls13 = version == TLS1_3_VERSION
    chacha = aead == "chacha20-poly1305"
    aid = o.CHACHA20_POLY1305 if chacha else o.AES_GCM
    out = []
    for i, (pt, typ) in enumerate(zip(records, types)):
        seq = (seq0 + i).to_bytes(8, "big")
        if tls13 or chacha:  # ssl_aead_ctx.cc:96-103, 326-336, 367-373
            nonce, explicit = bytes(a ^ b for a, b in zip(fixed_iv, bytes(4) + seq)), b""
        else:                # fixed IV || explicit nonce in the record (:104-110, 355-365)
            nonce, explicit = fixed_iv + seq, seq
        extra = bytes([typ]) if tls13 else b""  # tls_record.cc:272-276
        ctlen = len(explicit) + len(pt) + len(extra) + 16
        hdr = bytes([23 if tls13 else typ, 3, 3, ctlen >> 8, ctlen & 0xff])  # :287-298
        ad = hdr if tls13 else seq + bytes([typ, 3, 3]) + len(pt).to_bytes(2, "big")  # :207-224
        if len(pt) > 16384:
            out.append(None)
            continue
        ok, ct, tag = o.seal(aid, key, nonce, pt + extra, ad)
        assert ok
        out.append((hdr + explicit, ct[:len(pt)], ct[len(pt):] + tag))
    return out


def fill_bytes(n, seed):
    """The deterministic record bytes of oracle/ref/ref_tls.cc fill()."""
    x = (seed * 2654435761 + 12345) & 0xffffffff
    out = bytearray(n)
    for i in range(n):
        x ^= (x << 13) & 0xffffffff
        x ^= x >> 17
        x ^= (x << 5) & 0xffffffff
        out[i] = (x >> 7) & 0xff
    return bytes(out)
