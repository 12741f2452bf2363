"""The single-record EVP_AEAD host surface, through the C ABI, on the GPU.

A restatement of the reference's PerAEADTest suite (crypto/cipher/aead_test.cc)
over the reference's own vector files (crypto/cipher/test/*_tests.txt, carried
as data in tests/golden/kat_aead.json).  Every call goes through
libbssl_amd.so with plain host pointers (ctypes), exactly as a C caller of the
reference API would make it; every record is sealed/opened by the HIP kernels.

  TestVector              aead_test.cc:188-281
  TestExtraInput          :283-360  (seal_scatter, every extra_in split)
  TestVectorScatterGather :362-478  (seal_scatter / open_gather)
  Sealv / Openv / OpenvDetached, in place and not, over the "interesting
  splits" of the input and of the AD       :480-937
  CleanupAfterInitFailure :940-961
  TruncatedTags           :963-1066 (sentinel bytes past the output)
  AliasedBuffers          :1068-1143
  UnalignedInput          :1145-1185
  Overflow                :1187-1210
  InvalidNonceLength      :1212-1265
plus the zero-on-error contract of EVP_AEAD_CTX_seal_scatter
(crypto/fipsmodule/cipher/aead.cc.inc:170-186) and a latency figure for
unbatched callers.
"""
import ctypes
import time

import pytest

torch = pytest.importorskip("torch")
import boringssl_amd as ba  # noqa: E402
from golden_util import load  # noqa: E402

pytestmark = pytest.mark.gpu

L = ba.lib
_S = ctypes.c_size_t

# kAEADs (aead_test.cc:76-168) restricted to the AEADs this engine provides.
CAN_TRUNCATE, VARIABLE_NONCE = 1, 2
AEADS = {
    "aes-128-gcm": ("aes_128_gcm_tests.txt", CAN_TRUNCATE | VARIABLE_NONCE),
    "aes-192-gcm": ("aes_192_gcm_tests.txt", CAN_TRUNCATE | VARIABLE_NONCE),
    "aes-256-gcm": ("aes_256_gcm_tests.txt", CAN_TRUNCATE | VARIABLE_NONCE),
    "aes-128-gcm-siv": ("aes_128_gcm_siv_tests.txt", 0),
    "aes-256-gcm-siv": ("aes_256_gcm_siv_tests.txt", 0),
    "chacha20-poly1305": ("chacha20_poly1305_tests.txt", CAN_TRUNCATE),
    "xchacha20-poly1305": ("xchacha20_poly1305_tests.txt", CAN_TRUNCATE),
}
NAMES = list(AEADS)
EVP_AEAD_MAX_KEY_LENGTH, EVP_AEAD_MAX_NONCE_LENGTH, EVP_AEAD_MAX_OVERHEAD = 80, 24, 64
SIZE_MAX = (1 << 64) - 1


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    L.ERR_clear_error()
    yield


def kat(aead):
    """The reference vector file of `aead` (PerAEADTest::TestVectorPath)."""
    f = AEADS[aead][0]
    out = []
    for c in load("kat_aead.json"):
        if c["aead"] == aead and c["source"].startswith("crypto/cipher/test/" + f):
            out.append({k: bytes.fromhex(c[k]) for k in ("key", "nonce", "ad", "pt", "ct", "tag")})
    assert out, aead
    return out


# ---------------------------------------------------------------------------
# ctypes plumbing: host buffers with stable addresses

class Buf:
    """A host buffer; `.p(off)` is the address of byte `off`."""

    def __init__(self, data_or_len, fill=0):
        if isinstance(data_or_len, int):
            self.b = ctypes.create_string_buffer(bytes([fill]) * max(1, data_or_len),
                                                 max(1, data_or_len))
            self.n = data_or_len
        else:
            d = bytes(data_or_len)
            self.b = ctypes.create_string_buffer(d if d else b"\0", max(1, len(d)))
            self.n = len(d)

    def p(self, off=0):
        return ctypes.addressof(self.b) + off

    def get(self, off=0, n=None):
        n = self.n - off if n is None else n
        return self.b.raw[off:off + n]


def errors():
    """Drain the error queue: list of (lib, reason)."""
    out = []
    while True:
        e = L.ERR_get_error()
        if not e:
            return out
        out.append(((e >> 24) & 0xff, e & 0xfff))


def errors_are(*reasons):
    return errors() == [(ba.ERR_LIB_CIPHER, r) for r in reasons]


def new_ctx(aead, key, tag_len, direction):
    ctx = ba.EVP_AEAD_CTX()
    L.EVP_AEAD_CTX_zero(ctypes.byref(ctx))
    k = Buf(key)
    if direction is None:  # EVP_AEAD_CTX_init
        ok = L.EVP_AEAD_CTX_init(ctypes.byref(ctx), ba.EVP_aead(aead), k.p(), len(key), tag_len,
                                 None)
    else:
        ok = L.EVP_AEAD_CTX_init_with_direction(ctypes.byref(ctx), ba.EVP_aead(aead), k.p(),
                                                len(key), tag_len, direction)
    assert ok, errors()
    return ctx


class Ctx:
    def __init__(self, aead, key, tag_len=0, direction=ba.evp_aead_seal):
        self.c = new_ctx(aead, key, tag_len, direction)

    def __del__(self):
        L.EVP_AEAD_CTX_cleanup(ctypes.byref(self.c))

    @property
    def ref(self):
        return ctypes.byref(self.c)


def seal(ctx, out_addr, max_out, nonce, in_addr, in_len, ad):
    n, a = Buf(nonce), Buf(ad)
    out_len = _S(12345)
    ok = L.EVP_AEAD_CTX_seal(ctx.ref, out_addr, ctypes.byref(out_len), max_out, n.p(), len(nonce),
                             in_addr, in_len, a.p(), len(ad))
    return ok, out_len.value


def open_(ctx, out_addr, max_out, nonce, in_addr, in_len, ad):
    n, a = Buf(nonce), Buf(ad)
    out_len = _S(12345)
    ok = L.EVP_AEAD_CTX_open(ctx.ref, out_addr, ctypes.byref(out_len), max_out, n.p(), len(nonce),
                             in_addr, in_len, a.p(), len(ad))
    return ok, out_len.value


def seal_scatter(ctx, out, out_tag, max_tag, nonce, inp, extra, ad):
    n, a = Buf(nonce), Buf(ad)
    i, x = Buf(inp), Buf(extra)
    tl = _S(12345)
    ok = L.EVP_AEAD_CTX_seal_scatter(ctx.ref, out.p(), out_tag.p(), ctypes.byref(tl), max_tag,
                                     n.p(), len(nonce), i.p(), len(inp), x.p(), len(extra), a.p(),
                                     len(ad))
    return ok, tl.value


# ---------------------------------------------------------------------------
# TestIOVecs / InterestingSplitsForLength (aead_test.cc:480-598)

class IOVecs:
    def __init__(self, data, splits, in_place):
        self.bufs, self.pieces = [], []
        cuts = [0] + list(splits) + [len(data)]
        for s, e in zip(cuts, cuts[1:]):
            piece = data[s:e]
            bi = Buf(piece)
            bo = bi if in_place else Buf(len(piece), ord("X"))
            self.bufs += [bi, bo]
            self.pieces.append((bo, bi, len(piece)))
        self.iov = (ba.CRYPTO_IOVEC * max(1, len(self.pieces)))()
        self.ivec = (ba.CRYPTO_IVEC * max(1, len(self.pieces)))()
        for k, (bo, bi, n) in enumerate(self.pieces):
            self.iov[k].out, self.iov[k].in_, self.iov[k].len = bo.p(), bi.p(), n
            self.ivec[k].in_, self.ivec[k].len = bi.p(), n
        self.count = len(self.pieces)

    def output(self):
        return b"".join(bo.get(0, n) for bo, _, n in self.pieces)


def interesting_splits(length, block=16):
    w = lambda v: v % (1 << 64)  # noqa: E731 (size_t arithmetic)
    second = block
    un_start = 1
    un_end = w(length - 2) if length % block == 1 else w(length - 1)
    last = w(length - 1) // block * block
    ideas = {(), (0,), (un_start,), (second,), (last,), (un_end,), (length,),
             (un_start, un_start), (un_start, last), (second, last), (un_start, un_end),
             (second, un_end)}
    out = []
    for idea in ideas:
        idea = tuple(sorted(set(idea)))
        if all(p <= length for p in idea) and list(idea) not in out:
            out.append(list(idea))
    return sorted(out)


def sealv(ctx, iov, nonce, ad_iov, max_tag):
    tag = Buf(max_tag)
    n = Buf(nonce)
    tl = _S(12345)
    ok = L.EVP_AEAD_CTX_sealv(ctx.ref, iov.iov, iov.count, tag.p(), ctypes.byref(tl), max_tag,
                              n.p(), len(nonce), ad_iov.ivec, ad_iov.count)
    return ok, tag.get(0, tl.value)


def openv_detached(ctx, iov, nonce, tag, ad_iov):
    n, t = Buf(nonce), Buf(tag or b"")
    return L.EVP_AEAD_CTX_openv_detached(ctx.ref, iov.iov, iov.count, n.p(), len(nonce),
                                         t.p() if tag is not None else None,
                                         len(tag or b""), ad_iov.ivec, ad_iov.count)


def openv(ctx, iov, nonce, ad_iov):
    n = Buf(nonce)
    total = _S(12345)
    ok = L.EVP_AEAD_CTX_openv(ctx.ref, iov.iov, iov.count, ctypes.byref(total), n.p(),
                              len(nonce), ad_iov.ivec, ad_iov.count)
    return ok, total.value


# ---------------------------------------------------------------------------

@pytest.mark.parametrize("aead", NAMES)
def test_vector(aead):
    """TestVector (aead_test.cc:188-281)."""
    for c in kat(aead):
        tag_len = len(c["tag"])
        ctx = Ctx(aead, c["key"], tag_len, ba.evp_aead_seal)
        out = Buf(len(c["pt"]) + L.EVP_AEAD_max_overhead(ba.EVP_aead(aead)))
        pt = Buf(c["pt"])
        ok, n = seal(ctx, out.p(), out.n, c["nonce"], pt.p(), pt.n, c["ad"])
        assert ok and n == len(c["ct"]) + tag_len
        sealed = out.get(0, n)
        assert sealed == c["ct"] + c["tag"]
        ctx = Ctx(aead, c["key"], tag_len, ba.evp_aead_open)
        src, dst = Buf(sealed), Buf(len(sealed))
        ok, n2 = open_(ctx, dst.p(), dst.n, c["nonce"], src.p(), src.n, c["ad"])
        assert ok and dst.get(0, n2) == c["pt"]
        # Garbage at the end isn't ignored.
        src = Buf(sealed + b"\0")
        dst = Buf(src.n)
        ok, _ = open_(ctx, dst.p(), dst.n, c["nonce"], src.p(), src.n, c["ad"])
        assert not ok
        errors()
        # Integrity is checked.
        bad = bytearray(sealed)
        bad[0] ^= 0x80
        src = Buf(bytes(bad))
        dst = Buf(src.n)
        ok, _ = open_(ctx, dst.p(), dst.n, c["nonce"], src.p(), src.n, c["ad"])
        assert not ok
        errors()


@pytest.mark.parametrize("aead", NAMES)
def test_extra_input(aead):
    """TestExtraInput (aead_test.cc:283-360): seal_scatter with every split of
    the input into `in` and `extra_in`, and the tag-buffer bounds."""
    overhead = L.EVP_AEAD_max_overhead(ba.EVP_aead(aead))
    cases = kat(aead)
    if "siv" in aead:  # 1 KiB inputs: every 8th split keeps the call count bounded
        stride = 8
    else:
        stride = 1
    for c in cases:
        tag_len, pt = len(c["tag"]), c["pt"]
        ctx = Ctx(aead, c["key"], tag_len, ba.evp_aead_seal)
        for extra in list(range(0, len(pt), stride)) + ([len(pt) - 1] if pt else []):
            out_tag = Buf(overhead + len(pt), 0x5a)
            out = Buf(len(pt), 0x5a)
            ok, written = seal_scatter(ctx, out, out_tag, out_tag.n, c["nonce"],
                                       pt[:len(pt) - extra], pt[len(pt) - extra:], c["ad"])
            assert ok and written == extra + tag_len, (extra, errors())
            got = out.get(0, len(pt) - extra) + out_tag.get(0, extra)
            assert got == c["ct"], extra
            assert out_tag.get(extra, tag_len) == c["tag"], extra
            # Bounds on the tag output are checked.
            for size in ((extra - 1) if extra else 0, extra + tag_len - 1):
                tb = Buf(size, 0x77)
                ok, written = seal_scatter(ctx, out, tb, size, c["nonce"], pt[:len(pt) - extra],
                                           pt[len(pt) - extra:], c["ad"])
                assert not ok and written == 0
                assert errors_are(ba.CIPHER_R_BUFFER_TOO_SMALL), (extra, size)


@pytest.mark.parametrize("aead", NAMES)
def test_vector_scatter_gather(aead):
    """TestVectorScatterGather (aead_test.cc:362-478)."""
    overhead = L.EVP_AEAD_max_overhead(ba.EVP_aead(aead))
    for c in kat(aead):
        tag_len, pt = len(c["tag"]), c["pt"]
        ctx = Ctx(aead, c["key"], tag_len, ba.evp_aead_seal)
        out, out_tag = Buf(len(pt)), Buf(overhead)
        ok, tl = seal_scatter(ctx, out, out_tag, overhead, c["nonce"], pt, b"", c["ad"])
        assert ok and tl == tag_len
        assert out.get(0, len(pt)) == c["ct"] and out_tag.get(0, tl) == c["tag"]
        octx = Ctx(aead, c["key"], tag_len, ba.evp_aead_open)
        n, a = Buf(c["nonce"]), Buf(c["ad"])

        def gather(tag):
            dst = Buf(len(pt), 0x33)
            t = Buf(tag)
            ok = L.EVP_AEAD_CTX_open_gather(octx.ref, dst.p(), n.p(), n.n, out.p(), len(pt),
                                            t.p(), len(tag), a.p(), a.n)
            return ok, dst.get(0, len(pt))

        ok, back = gather(c["tag"])
        assert ok and back == pt
        ok, back = gather(c["tag"] + b"\0")  # trailing garbage
        assert not ok and back == bytes(len(pt))
        errors()
        bad = bytearray(c["tag"])
        bad[0] ^= 0x80
        ok, back = gather(bytes(bad[:-1]))  # corrupted and short
        assert not ok and back == bytes(len(pt))
        errors()
        ok, back = gather(b"")  # zero-length tag
        assert not ok
        errors()


def _splits_for(c, pt_len):
    for adsplits in interesting_splits(len(c["ad"])):
        for splits in interesting_splits(pt_len):
            if adsplits and splits:
                continue
            yield adsplits, splits


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("aead", NAMES)
def test_sealv(aead, in_place):
    """RunSealvTests (aead_test.cc:611-670)."""
    overhead = L.EVP_AEAD_max_overhead(ba.EVP_aead(aead))
    for c in kat(aead):
        ctx = Ctx(aead, c["key"], len(c["tag"]), ba.evp_aead_seal)
        for adsplits, splits in _splits_for(c, len(c["pt"])):
            adv = IOVecs(c["ad"], adsplits, in_place)
            iov = IOVecs(c["pt"], splits, in_place)
            ok, tag = sealv(ctx, iov, c["nonce"], adv, overhead)
            assert ok, (adsplits, splits, errors())
            assert iov.output() == c["ct"] and tag == c["tag"], (adsplits, splits)


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("aead", NAMES)
def test_openv_detached(aead, in_place):
    """RunOpenvDetachedTests (aead_test.cc:672-786)."""
    for c in kat(aead):
        ctx = Ctx(aead, c["key"], len(c["tag"]), ba.evp_aead_open)
        for adsplits, splits in _splits_for(c, len(c["ct"])):
            adv = IOVecs(c["ad"], adsplits, in_place)
            iov = IOVecs(c["ct"], splits, in_place)
            assert openv_detached(ctx, iov, c["nonce"], c["tag"], adv), (adsplits, splits)
            assert iov.output() == c["pt"]
            iov = IOVecs(c["ct"], splits, in_place)  # trailing garbage on the tag
            assert not openv_detached(ctx, iov, c["nonce"], c["tag"] + b"\0", adv)
            assert iov.output() == bytes(len(c["ct"]))  # zeroed on failure
            errors()
            bad = bytearray(c["tag"])
            bad[0] ^= 0x80
            iov = IOVecs(c["ct"], splits, in_place)
            assert not openv_detached(ctx, iov, c["nonce"], bytes(bad), adv)
            assert iov.output() == bytes(len(c["ct"]))
            errors()
            iov = IOVecs(c["ct"], splits, in_place)  # zero-length tag
            assert not openv_detached(ctx, iov, c["nonce"], None, adv)
            errors()


@pytest.mark.parametrize("in_place", [False, True])
@pytest.mark.parametrize("aead", NAMES)
def test_openv(aead, in_place):
    """RunOpenvTests (aead_test.cc:788-913): the tag as a suffix of the iovecs."""
    for c in kat(aead):
        ctx = Ctx(aead, c["key"], len(c["tag"]), ba.evp_aead_open)
        combined = c["ct"] + c["tag"]
        for adsplits, splits in _splits_for(c, len(combined)):
            adv = IOVecs(c["ad"], adsplits, in_place)
            iov = IOVecs(combined, splits, in_place)
            ok, n = openv(ctx, iov, c["nonce"], adv)
            assert ok and n == len(c["pt"]), (adsplits, splits, errors())
            assert iov.output()[:n] == c["pt"]
            for wrecked in (combined + b"\0", combined[:-1] + bytes([combined[-1] ^ 0x80]),
                            combined[:-1]):
                sp = [min(s, len(wrecked)) for s in splits]
                iov = IOVecs(wrecked, sp, in_place)
                ok, n = openv(ctx, iov, c["nonce"], adv)
                assert not ok and n == 0
                assert iov.output() == bytes(len(wrecked))
                errors()


@pytest.mark.parametrize("aead", NAMES)
def test_cleanup_after_init_failure(aead):
    """CleanupAfterInitFailure (aead_test.cc:940-961)."""
    ctx = ba.EVP_AEAD_CTX()
    key = Buf(EVP_AEAD_MAX_KEY_LENGTH)
    a = ba.EVP_aead(aead)
    for _ in range(2):
        assert not L.EVP_AEAD_CTX_init(ctypes.byref(ctx), a, key.p(), L.EVP_AEAD_key_length(a),
                                       9999, None)
        errors()
    L.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))  # a no-op


@pytest.mark.parametrize("aead", NAMES)
def test_truncated_tags(aead):
    """TruncatedTags (aead_test.cc:963-1066): sealing and opening never write
    past the length they report (sentinel bytes)."""
    a = ba.EVP_aead(aead)
    key = bytes(L.EVP_AEAD_key_length(a))
    nonce = bytes(L.EVP_AEAD_nonce_length(a))
    ad = bytes(16)
    tag_len = 1 if AEADS[aead][1] & CAN_TRUNCATE else L.EVP_AEAD_max_tag_len(a)
    plaintext = b"A"
    sentinel = 42
    overhead = tag_len + L.EVP_AEAD_max_overhead(a) - L.EVP_AEAD_max_tag_len(a)
    expected = len(plaintext) + overhead
    pt = Buf(plaintext)
    ct = Buf(128, sentinel)
    ctx = Ctx(aead, key, tag_len, ba.evp_aead_seal)
    ok, _ = seal(ctx, ct.p(), expected - 1, nonce, pt.p(), 1, ad)
    assert not ok  # a full-featured AEAD respects the tag length exactly
    errors()
    ct = Buf(128, sentinel)
    ok, clen = seal(ctx, ct.p(), expected, nonce, pt.p(), 1, ad)
    assert ok and clen == expected
    assert ct.get(clen) == bytes([sentinel]) * (128 - clen)
    pt2 = Buf(1 + 64, sentinel)
    octx = Ctx(aead, key, tag_len, ba.evp_aead_open)
    ok, plen = open_(octx, pt2.p(), pt2.n, nonce, ct.p(), clen, ad)
    assert ok and pt2.get(0, plen) == plaintext
    assert pt2.get(plen) == bytes([sentinel]) * (pt2.n - plen)


@pytest.mark.parametrize("aead", NAMES)
def test_aliased_buffers(aead):
    """AliasedBuffers (aead_test.cc:1068-1143): out == in works, any other
    overlap fails with OUTPUT_ALIASES_INPUT."""
    a = ba.EVP_aead(aead)
    nl, overhead = L.EVP_AEAD_nonce_length(a), L.EVP_AEAD_max_overhead(a)
    ctx = Ctx(aead, b"a" * L.EVP_AEAD_key_length(a), 0, None)
    text = (b"testing123456" * 20)[:259] + b"\0"  # kPlaintext[260]
    nonce = b"b" * nl
    ptb = Buf(text)
    valid = Buf(len(text) + overhead)
    ok, vlen = seal(ctx, valid.p(), valid.n, nonce, ptb.p(), len(text), b"")
    assert ok
    buf = Buf(2 + vlen)
    inp, out1, out2 = buf.p(1), buf.p(0), buf.p(2)
    ctypes.memmove(inp, text, len(text))
    for o in (out1, out2):
        ok, _ = seal(ctx, o, len(text) + overhead, nonce, inp, len(text), b"")
        assert not ok
        assert errors_are(ba.CIPHER_R_OUTPUT_ALIASES_INPUT)
    ctypes.memmove(inp, valid.get(0, vlen), vlen)
    for o in (out1, out2):
        ok, _ = open_(ctx, o, vlen, nonce, inp, vlen, b"")
        assert not ok
        assert errors_are(ba.CIPHER_R_OUTPUT_ALIASES_INPUT)
    # out == in works
    ctypes.memmove(inp, text, len(text))
    ok, n = seal(ctx, inp, len(text) + overhead, nonce, inp, len(text), b"")
    assert ok and buf.get(1, n) == valid.get(0, vlen)
    ctypes.memmove(inp, valid.get(0, vlen), vlen)
    ok, n = open_(ctx, inp, vlen, nonce, inp, vlen, b"")
    assert ok and buf.get(1, n) == text


@pytest.mark.parametrize("aead", NAMES)
def test_unaligned_input(aead):
    """UnalignedInput (aead_test.cc:1145-1185)."""
    a = ba.EVP_aead(aead)
    kl, nl = L.EVP_AEAD_key_length(a), L.EVP_AEAD_nonce_length(a)
    key = Buf(b"K" * (EVP_AEAD_MAX_KEY_LENGTH + 1))
    nonce = Buf(b"N" * (EVP_AEAD_MAX_NONCE_LENGTH + 1))
    pt = Buf(b"P" * 33)
    ad = Buf(b"A" * 33)
    c = ba.EVP_AEAD_CTX()
    assert L.EVP_AEAD_CTX_init_with_direction(ctypes.byref(c), a, key.p(1), kl, 0,
                                              ba.evp_aead_seal)
    ct = Buf(33 + EVP_AEAD_MAX_OVERHEAD)
    clen = _S(0)
    assert L.EVP_AEAD_CTX_seal(ctypes.byref(c), ct.p(1), ctypes.byref(clen), ct.n - 1, nonce.p(1),
                               nl, pt.p(1), 32, ad.p(1), 32)
    L.EVP_AEAD_CTX_cleanup(ctypes.byref(c))
    c = ba.EVP_AEAD_CTX()
    assert L.EVP_AEAD_CTX_init_with_direction(ctypes.byref(c), a, key.p(1), kl, 0,
                                              ba.evp_aead_open)
    out = Buf(ct.n)
    olen = _S(0)
    assert L.EVP_AEAD_CTX_open(ctypes.byref(c), out.p(1), ctypes.byref(olen), out.n - 1,
                               nonce.p(1), nl, ct.p(1), clen.value, ad.p(1), 32)
    assert out.get(1, olen.value) == b"P" * 32
    L.EVP_AEAD_CTX_cleanup(ctypes.byref(c))


@pytest.mark.parametrize("aead", NAMES)
def test_overflow(aead):
    """Overflow (aead_test.cc:1187-1210): no size_t overflow computing the
    ciphertext length."""
    a = ba.EVP_aead(aead)
    max_tag = L.EVP_AEAD_max_tag_len(a)
    ctx = Ctx(aead, b"K" * L.EVP_AEAD_key_length(a), max_tag, ba.evp_aead_seal)
    pt, ct = Buf(1), Buf(1024)
    clen = _S(0)
    assert not L.EVP_AEAD_CTX_seal(ctx.ref, ct.p(), ctypes.byref(clen), 1024, None, 0, pt.p(),
                                   SIZE_MAX - max_tag + 1, None, 0)
    errors()


@pytest.mark.parametrize("aead", NAMES)
def test_invalid_nonce_length(aead):
    """InvalidNonceLength (aead_test.cc:1212-1265)."""
    a = ba.EVP_aead(aead)
    valid = L.EVP_AEAD_nonce_length(a)
    lens = [0]
    if not AEADS[aead][1] & VARIABLE_NONCE:
        lens += [valid + 1, valid - 1]
    zeros = Buf(EVP_AEAD_MAX_KEY_LENGTH)
    ok_codes = {(ba.ERR_LIB_CIPHER, ba.CIPHER_R_UNSUPPORTED_NONCE_SIZE),
                (ba.ERR_LIB_CIPHER, ba.CIPHER_R_INVALID_NONCE_SIZE)}
    for nl in lens:
        nonce = Buf(nl)
        for direction in (ba.evp_aead_seal, ba.evp_aead_open):
            ctx = Ctx(aead, bytes(L.EVP_AEAD_key_length(a)), 0, direction)
            out = Buf(256)
            n = _S(0)
            if direction == ba.evp_aead_seal:
                ok = L.EVP_AEAD_CTX_seal(ctx.ref, out.p(), ctypes.byref(n), 256, nonce.p(), nl,
                                         None, 0, zeros.p(), 16)
            else:
                ok = L.EVP_AEAD_CTX_open(ctx.ref, out.p(), ctypes.byref(n), 256, nonce.p(), nl,
                                         zeros.p(), EVP_AEAD_MAX_KEY_LENGTH, zeros.p(), 16)
            assert not ok
            e = errors()
            assert e and e[0] in ok_codes, (nl, direction, e)


@pytest.mark.parametrize("aead", ["aes-128-gcm", "chacha20-poly1305"])
def test_seal_scatter_zeroes_outputs_on_error(aead):
    """EVP_AEAD_CTX_seal_scatter's cleanup (aead.cc.inc:170-186): on any error
    the first in_len bytes of `out` and all max_out_tag_len bytes of `out_tag`
    are zeroed and *out_tag_len = 0."""
    a = ba.EVP_aead(aead)
    ctx = Ctx(aead, bytes(range(L.EVP_AEAD_key_length(a))), 0, ba.evp_aead_seal)
    nonce = bytes(12)
    pt, extra = b"x" * 40, b"yz"
    # (1) out_tag smaller than extra_in: BUFFER_TOO_SMALL
    out, tag = Buf(64, 0x5a), Buf(64, 0x5a)
    ok, tl = seal_scatter(ctx, out, tag, 1, nonce, pt, extra, b"")
    assert not ok and tl == 0 and errors_are(ba.CIPHER_R_BUFFER_TOO_SMALL)
    assert out.get(0, 40) == bytes(40) and out.get(40) == b"\x5a" * 24
    assert tag.get(0, 1) == b"\0" and tag.get(1) == b"\x5a" * 63
    # (2) room for extra_in but not for the tag: BUFFER_TOO_SMALL, all zeroed
    out, tag = Buf(64, 0x5a), Buf(64, 0x5a)
    ok, tl = seal_scatter(ctx, out, tag, len(extra) + 15, nonce, pt, extra, b"")
    assert not ok and tl == 0 and errors_are(ba.CIPHER_R_BUFFER_TOO_SMALL)
    assert out.get(0, 40) == bytes(40) and tag.get(0, 17) == bytes(17)
    assert tag.get(17) == b"\x5a" * 47
    # (3) bad nonce length: the same zeroing
    out, tag = Buf(64, 0x5a), Buf(64, 0x5a)
    ok, tl = seal_scatter(ctx, out, tag, 64, b"" if "gcm" in aead else bytes(11), pt, extra, b"")
    assert not ok and tl == 0
    assert errors()[0][1] in (ba.CIPHER_R_INVALID_NONCE_SIZE, ba.CIPHER_R_UNSUPPORTED_NONCE_SIZE)
    assert out.get(0, 40) == bytes(40) and tag.get(0, 64) == bytes(64)


def test_single_record_latency(record_property):
    """The cost an unbatched caller (SSLAEADContext::SealScatter,
    ssl/ssl_aead_ctx.cc:299-409) pays per EVP_AEAD_CTX_seal_scatter call:
    host buffers -> device -> kernels -> host, synchronised.  Reported, not
    asserted beyond a sanity bound."""
    res = {}
    for aead, size in (("aes-128-gcm", 1350), ("aes-128-gcm", 16384),
                       ("chacha20-poly1305", 1350), ("chacha20-poly1305", 16384)):
        a = ba.EVP_aead(aead)
        ctx = Ctx(aead, bytes(L.EVP_AEAD_key_length(a)), 0, ba.evp_aead_seal)
        out, tag = Buf(size), Buf(16)
        pt, ad = bytes(size), bytes(13)
        for _ in range(20):
            assert seal_scatter(ctx, out, tag, 16, bytes(12), pt, b"", ad)[0]
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            seal_scatter(ctx, out, tag, 16, bytes(12), pt, b"", ad)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        res[f"{aead}/{size}"] = {"median_us": round(ts[100] * 1e6, 1),
                                 "p90_us": round(ts[180] * 1e6, 1)}
        assert ts[100] < 0.05
    print("single-record seal_scatter latency:", res)
    record_property("latency", res)


def test_keyset_tag_len_rules():
    """BSSL_AMD_KEYSET_new applies EVP_AEAD_CTX_init's per-AEAD tag-length
    rule (AES-GCM-SIV takes only 16-byte tags, e_aesgcmsiv.cc:542-548)."""
    key = bytes(16)
    with pytest.raises(ba.AEADError) as e:
        ba.Keyset("aes-128-gcm-siv", key, 1, 8)
    assert e.value.reason == ba.CIPHER_R_TAG_TOO_LARGE
    with pytest.raises(ba.AEADError) as e:
        ba.Keyset("aes-128-gcm", key, 1, 17)
    assert e.value.reason == ba.CIPHER_R_TAG_TOO_LARGE
    ba.Keyset("aes-128-gcm-siv", key, 1, 16).close()
    ba.Keyset("aes-128-gcm", key, 1, 8).close()


@pytest.mark.parametrize("which", ["ctx", "keyset"])
def test_cleanup_while_batch_in_flight(which):
    """EVP_AEAD_CTX_cleanup / BSSL_AMD_KEYSET_free right after enqueueing a
    large device batch on a NON-BLOCKING stream (seal_batch_device is
    asynchronous to the host): the key wipe must not land while the kernel
    still reads the round keys (the null-stream memset does not
    order against such streams).  Sampled records and every status must
    match the oracle after the stream completes."""
    import numpy as np
    import oracle_lib as o
    n, rlen = 1 << 17, 16384  # 2 GiB: several ms of kernel time
    key = bytes(range(7, 23))
    dev = torch.device("cuda:0")
    d_pt = torch.randint(0, 256, (n * rlen,), dtype=torch.uint8, device=dev)
    d_ct = torch.zeros_like(d_pt)
    d_tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
    d_st = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_n = torch.randint(0, 256, (12 * n,), dtype=torch.uint8, device=dev)
    d_ad = torch.randint(0, 256, (13 * n,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()  # pool stream: created non-blocking by PyTorch
    b = ba.make_batch(n, d_pt, d_ct, d_tags, d_n, 12, d_ad, record_stride=rlen, record_len=rlen,
                      ad_stride=13, ad_len=13, status=d_st)
    if which == "ctx":
        obj = ba.AEADCtx("aes-128-gcm", key, 16)
    else:
        obj = ba.Keyset("aes-128-gcm", key, 1, 16)
    obj.seal_batch_device(b, s)
    obj.close()  # cleanup with the batch in flight
    s.synchronize()
    assert bool(d_st.all())
    pt, ct, tags = d_pt.cpu().numpy(), d_ct.cpu().numpy(), d_tags.cpu().numpy()
    nn, aa = d_n.cpu().numpy(), d_ad.cpu().numpy()
    for i in list(range(0, 32)) + list(range(n - 32, n)) + list(range(n // 2, n // 2 + 8)):
        ok, c, t = o.seal(o.AES_GCM, key, nn[12 * i:12 * i + 12].tobytes(),
                          pt[rlen * i:rlen * (i + 1)].tobytes(), aa[13 * i:13 * i + 13].tobytes())
        assert ok and ct[rlen * i:rlen * (i + 1)].tobytes() == c and \
            tags[16 * i:16 * i + 16].tobytes() == t, i


def test_device_guard_one_gpu():
    """Single-GPU check of the device guard (the two-GPU test is deselected on
    one-GPU boxes): host-buffer calls leave the caller's current device as
    it was, and a rejected device-batch call reports the same error every
    time and leaves the context usable."""
    key, nonce = bytes(range(16)), bytes(12)
    ctx = ba.AEADCtx("aes-128-gcm", key, 16)
    before = torch.cuda.current_device()
    sealed = ctx.seal(nonce, b"hello", b"ad")
    assert ctx.open(nonce, sealed, b"ad") == b"hello"
    assert torch.cuda.current_device() == before
    d = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    reasons = []
    for _ in range(3):
        with pytest.raises(ba.AEADError) as e:  # no nonces: rejected before any launch
            ctx.seal_batch_device(ba.make_batch(1, d, d, d, None, 12, d, record_len=16,
                                                record_stride=16))
        reasons.append(e.value.reason)
    assert len(set(reasons)) == 1 and reasons[0] == 66  # ERR_R_SHOULD_NOT_HAVE_BEEN_CALLED
    assert ctx.seal(nonce, b"hello", b"ad") == sealed
    assert torch.cuda.current_device() == before
