"""boringssl_amd -- MI355X-native bulk AEAD record engine.

Python host mirror of the C ABI in include/bssl_amd/aead.h, which itself keeps
BoringSSL's EVP_AEAD surface (reference include/openssl/aead.h).  The compute
runs only in the HIP kernels of libbssl_amd.so (built from boringssl_amd/csrc
for gfx950); there is no CPU implementation behind any call, and importing
this package fails loudly when the shared object is missing.

PyTorch, when present, is imported first so that the library binds to the
same HIP runtime as torch tensors; it is used only for device buffers,
streams and torch.distributed.
"""
import ctypes
import os

try:  # share one HIP runtime with torch (same SONAME libamdhip64.so.7)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# BSSL_AMD_LIB may point at a diagnostic build (csrc/Makefile `ablate`).
LIB_PATH = os.environ.get("BSSL_AMD_LIB", os.path.join(_HERE, "libbssl_amd.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C boringssl_amd/csrc` "
        "(or __graft_entry__.build()); there is no fallback implementation")

_lib = ctypes.CDLL(LIB_PATH)

_P = ctypes.c_void_p
_S = ctypes.c_size_t
_U32 = ctypes.c_uint32
_I = ctypes.c_int

# include/bssl_amd/aead.h constants (reference include/openssl/cipher.h:792-817)
ERR_LIB_CIPHER = 30
CIPHER_R_BAD_DECRYPT = 101
CIPHER_R_BAD_KEY_LENGTH = 102
CIPHER_R_BUFFER_TOO_SMALL = 103
CIPHER_R_CTRL_NOT_IMPLEMENTED = 104
CIPHER_R_INVALID_NONCE_SIZE = 111
CIPHER_R_INVALID_OPERATION = 112
CIPHER_R_OUTPUT_ALIASES_INPUT = 115
CIPHER_R_TAG_TOO_LARGE = 116
CIPHER_R_TOO_LARGE = 117
CIPHER_R_UNSUPPORTED_KEY_SIZE = 120
CIPHER_R_UNSUPPORTED_NONCE_SIZE = 121
CIPHER_R_UNSUPPORTED_TAG_SIZE = 122
CIPHER_R_INVALID_NONCE = 125
EVP_AEAD_DEFAULT_TAG_LENGTH = 0
evp_aead_open = 0
evp_aead_seal = 1

# Every symbol include/bssl_amd/*.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = [
    "EVP_aead_aes_128_gcm", "EVP_aead_aes_192_gcm", "EVP_aead_aes_256_gcm",
    "EVP_aead_chacha20_poly1305", "EVP_aead_xchacha20_poly1305",
    "EVP_aead_aes_128_gcm_siv", "EVP_aead_aes_256_gcm_siv", "EVP_aead_aes_128_gcm_tls12", "EVP_aead_aes_256_gcm_tls12",
    "EVP_aead_aes_128_gcm_tls13", "EVP_aead_aes_256_gcm_tls13",
    "EVP_AEAD_key_length", "EVP_AEAD_nonce_length", "EVP_AEAD_max_overhead",
    "EVP_AEAD_max_tag_len", "EVP_AEAD_CTX_zero", "EVP_AEAD_CTX_new", "EVP_AEAD_CTX_free",
    "EVP_AEAD_CTX_init", "EVP_AEAD_CTX_init_with_direction", "EVP_AEAD_CTX_cleanup",
    "EVP_AEAD_CTX_aead", "EVP_AEAD_CTX_seal", "EVP_AEAD_CTX_open", "EVP_AEAD_CTX_seal_scatter",
    "EVP_AEAD_CTX_open_gather", "EVP_AEAD_CTX_sealv", "EVP_AEAD_CTX_openv",
    "EVP_AEAD_CTX_openv_detached", "EVP_AEAD_CTX_tag_len", "EVP_AEAD_CTX_get_iv",
    "ERR_get_error", "ERR_peek_error", "ERR_peek_last_error", "ERR_clear_error",
    "EVP_AEAD_CTX_seal_batch_device", "EVP_AEAD_CTX_open_batch_device",
    "EVP_AEAD_CTX_sealv_batch_device", "EVP_AEAD_CTX_openv_detached_batch_device",
    "BSSL_AMD_KEYSET_new", "BSSL_AMD_KEYSET_free", "BSSL_AMD_KEYSET_num_keys",
    "BSSL_AMD_KEYSET_seal_batch_device", "BSSL_AMD_KEYSET_open_batch_device",
    "BSSL_AMD_set_device", "BSSL_AMD_device_count", "BSSL_AMD_synth_fill_device",
    "BSSL_AMD_set_kernel_timing", "BSSL_AMD_collect_kernel_times", "BSSL_AMD_last_kernel_ms",
    "BSSL_AMD_last_kernel_name", "BSSL_AMD_set_aes_gcm_engine", "BSSL_AMD_aes_gcm_engine",
    # include/bssl_amd/test_hooks.h (test support, not part of the EVP surface)
    "BSSL_AMD_gcm_key_tables", "BSSL_AMD_test_set_bs_ek0_producers", "BSSL_AMD_test_set_gcm_mix",
    # include/bssl_amd/tls.h
    "BSSL_AMD_TLS_AEAD_new", "BSSL_AMD_TLS_AEAD_free", "BSSL_AMD_TLS_AEAD_prefix_len",
    "BSSL_AMD_TLS_AEAD_suffix_len", "BSSL_AMD_TLS_AEAD_sequence",
    "BSSL_AMD_TLS_AEAD_seal_records_device", "BSSL_AMD_TLS_AEAD_open_records_device",
]
TLS1_2_VERSION = 0x0303
TLS1_3_VERSION = 0x0304


class EVP_AEAD_CTX(ctypes.Structure):
    """struct evp_aead_ctx_st (reference aead.h:229-237)."""
    _fields_ = [("aead", _P), ("state", ctypes.c_uint8 * 560), ("tag_len", ctypes.c_uint8)]


class CRYPTO_IVEC(ctypes.Structure):
    _fields_ = [("in_", _P), ("len", _S)]


class CRYPTO_IOVEC(ctypes.Structure):
    _fields_ = [("out", _P), ("in_", _P), ("len", _S)]


class BSSL_AMD_BATCH(ctypes.Structure):
    _fields_ = [
        ("num_records", _S), ("in_", _P), ("out", _P), ("offsets", _P), ("lengths", _P),
        ("record_stride", ctypes.c_uint64), ("record_len", ctypes.c_uint64),
        ("nonces", _P), ("nonce_len", _S), ("ad", _P), ("ad_offsets", _P), ("ad_lengths", _P),
        ("ad_stride", ctypes.c_uint64), ("ad_len", ctypes.c_uint64), ("tags", _P),
        ("status", _P), ("key_index", _P),
    ]


class BSSL_AMD_IOV_BATCH(ctypes.Structure):
    _fields_ = [
        ("num_records", _S), ("iovecs", _P), ("iovec_start", _P), ("aadvecs", _P),
        ("aadvec_start", _P), ("nonces", _P), ("nonce_len", _S), ("tags", _P), ("status", _P),
    ]


class BSSL_AMD_TLS_RECORDS(ctypes.Structure):
    _fields_ = [
        ("num_records", _S), ("in_", _P), ("out", _P), ("offsets", _P), ("lengths", _P),
        ("record_stride", ctypes.c_uint64), ("record_len", ctypes.c_uint64), ("types", _P),
        ("type", ctypes.c_uint8), ("prefix", _P), ("suffix", _P), ("status", _P),
    ]


_CTXP = ctypes.POINTER(EVP_AEAD_CTX)
_SIGS = {
    "EVP_AEAD_key_length": (_S, [_P]),
    "EVP_AEAD_nonce_length": (_S, [_P]),
    "EVP_AEAD_max_overhead": (_S, [_P]),
    "EVP_AEAD_max_tag_len": (_S, [_P]),
    "EVP_AEAD_CTX_zero": (None, [_CTXP]),
    "EVP_AEAD_CTX_new": (_CTXP, [_P, _P, _S, _S]),
    "EVP_AEAD_CTX_free": (None, [_CTXP]),
    "EVP_AEAD_CTX_init": (_I, [_CTXP, _P, _P, _S, _S, _P]),
    "EVP_AEAD_CTX_init_with_direction": (_I, [_CTXP, _P, _P, _S, _S, _I]),
    "EVP_AEAD_CTX_cleanup": (None, [_CTXP]),
    "EVP_AEAD_CTX_aead": (_P, [_CTXP]),
    "EVP_AEAD_CTX_seal": (_I, [_CTXP, _P, ctypes.POINTER(_S), _S, _P, _S, _P, _S, _P, _S]),
    "EVP_AEAD_CTX_open": (_I, [_CTXP, _P, ctypes.POINTER(_S), _S, _P, _S, _P, _S, _P, _S]),
    "EVP_AEAD_CTX_seal_scatter": (_I, [_CTXP, _P, _P, ctypes.POINTER(_S), _S, _P, _S, _P, _S,
                                       _P, _S, _P, _S]),
    "EVP_AEAD_CTX_open_gather": (_I, [_CTXP, _P, _P, _S, _P, _S, _P, _S, _P, _S]),
    "EVP_AEAD_CTX_sealv": (_I, [_CTXP, _P, _S, _P, ctypes.POINTER(_S), _S, _P, _S, _P, _S]),
    "EVP_AEAD_CTX_openv": (_I, [_CTXP, _P, _S, ctypes.POINTER(_S), _P, _S, _P, _S]),
    "EVP_AEAD_CTX_openv_detached": (_I, [_CTXP, _P, _S, _P, _S, _P, _S, _P, _S]),
    "EVP_AEAD_CTX_tag_len": (_I, [_CTXP, ctypes.POINTER(_S), _S, _S]),
    "ERR_get_error": (_U32, []),
    "ERR_peek_error": (_U32, []),
    "ERR_peek_last_error": (_U32, []),
    "ERR_clear_error": (None, []),
    "EVP_AEAD_CTX_seal_batch_device": (_I, [_CTXP, ctypes.POINTER(BSSL_AMD_BATCH), _P]),
    "EVP_AEAD_CTX_open_batch_device": (_I, [_CTXP, ctypes.POINTER(BSSL_AMD_BATCH), _P]),
    "EVP_AEAD_CTX_sealv_batch_device": (_I, [_CTXP, ctypes.POINTER(BSSL_AMD_IOV_BATCH), _P]),
    "EVP_AEAD_CTX_openv_detached_batch_device": (_I, [_CTXP, ctypes.POINTER(BSSL_AMD_IOV_BATCH),
                                                      _P]),
    "BSSL_AMD_KEYSET_new": (_P, [_P, _P, _S, _S]),
    "BSSL_AMD_KEYSET_free": (None, [_P]),
    "BSSL_AMD_KEYSET_num_keys": (_S, [_P]),
    "BSSL_AMD_KEYSET_seal_batch_device": (_I, [_P, ctypes.POINTER(BSSL_AMD_BATCH), _P]),
    "BSSL_AMD_KEYSET_open_batch_device": (_I, [_P, ctypes.POINTER(BSSL_AMD_BATCH), _P]),
    "BSSL_AMD_set_device": (_I, [_I]),
    "BSSL_AMD_device_count": (_I, []),
    "BSSL_AMD_synth_fill_device": (_I, [ctypes.c_uint64, _S, _P, _P, _P, _P, _P, _P]),
    "BSSL_AMD_set_kernel_timing": (None, [_I]),
    "BSSL_AMD_collect_kernel_times": (_S, [ctypes.POINTER(ctypes.c_double), _S]),
    "BSSL_AMD_last_kernel_ms": (ctypes.c_double, []),
    "BSSL_AMD_last_kernel_name": (ctypes.c_char_p, []),
    "BSSL_AMD_set_aes_gcm_engine": (_I, [_I]),
    "BSSL_AMD_aes_gcm_engine": (_I, []),
    "BSSL_AMD_gcm_key_tables": (_S, [_P, _S, _S, _I, _P]),
    "BSSL_AMD_test_set_bs_ek0_producers": (_I, [_I]),
    "BSSL_AMD_test_set_gcm_mix": (_I, [_I]),
    "BSSL_AMD_TLS_AEAD_new": (_P, [_I, ctypes.c_uint16, _P, _P, _S, _P, _S, ctypes.c_uint64]),
    "BSSL_AMD_TLS_AEAD_free": (None, [_P]),
    "BSSL_AMD_TLS_AEAD_prefix_len": (_S, [_P]),
    "BSSL_AMD_TLS_AEAD_suffix_len": (_S, [_P]),
    "BSSL_AMD_TLS_AEAD_sequence": (ctypes.c_uint64, [_P]),
    "BSSL_AMD_TLS_AEAD_seal_records_device": (_I, [_P, ctypes.POINTER(BSSL_AMD_TLS_RECORDS), _P]),
    "BSSL_AMD_TLS_AEAD_open_records_device": (_I, [_P, ctypes.POINTER(BSSL_AMD_TLS_RECORDS), _P]),
}
for _name in EXPORTED_SYMBOLS:
    _f = getattr(_lib, _name)
    if _name in _SIGS:
        _f.restype, _f.argtypes = _SIGS[_name]
    else:  # the EVP_aead_* getters
        _f.restype, _f.argtypes = _P, []

lib = _lib

AEADS = {
    "aes-128-gcm": _lib.EVP_aead_aes_128_gcm,
    "aes-192-gcm": _lib.EVP_aead_aes_192_gcm,
    "aes-256-gcm": _lib.EVP_aead_aes_256_gcm,
    "chacha20-poly1305": _lib.EVP_aead_chacha20_poly1305,
    "xchacha20-poly1305": _lib.EVP_aead_xchacha20_poly1305,
    "aes-128-gcm-siv": _lib.EVP_aead_aes_128_gcm_siv,
    "aes-256-gcm-siv": _lib.EVP_aead_aes_256_gcm_siv,
    "aes-128-gcm-tls12": _lib.EVP_aead_aes_128_gcm_tls12,
    "aes-256-gcm-tls12": _lib.EVP_aead_aes_256_gcm_tls12,
    "aes-128-gcm-tls13": _lib.EVP_aead_aes_128_gcm_tls13,
    "aes-256-gcm-tls13": _lib.EVP_aead_aes_256_gcm_tls13,
}


def EVP_aead(name):
    return AEADS[name]()


class AEADError(Exception):
    """A failed EVP_AEAD call; `.reason` is the CIPHER_R_* code."""

    def __init__(self, what, packed):
        self.packed = packed
        self.lib = (packed >> 24) & 0xff
        self.reason = packed & 0xfff
        super().__init__(f"{what} failed (lib {self.lib}, reason {self.reason})")


def _fail(what):
    e = _lib.ERR_get_error()
    # drain the rest of the queue (the reference pushes one entry per failure)
    while _lib.ERR_get_error():
        pass
    raise AEADError(what, e)


def _ptr(b):
    if b is None:
        return None
    if isinstance(b, (bytes, bytearray)):
        return ctypes.cast(ctypes.c_char_p(bytes(b)), _P) if isinstance(b, bytes) else \
            ctypes.addressof((ctypes.c_char * len(b)).from_buffer(b))
    raise TypeError(type(b))


class AEADCtx:
    """EVP_AEAD_CTX wrapper: init / seal / open / batch (host + device)."""

    def __init__(self, aead, key, tag_len=EVP_AEAD_DEFAULT_TAG_LENGTH, direction=None):
        if isinstance(aead, str):
            aead = EVP_aead(aead)
        self.aead = aead
        self.ctx = EVP_AEAD_CTX()
        _lib.EVP_AEAD_CTX_zero(ctypes.byref(self.ctx))
        key = bytes(key)
        if direction is None:
            ok = _lib.EVP_AEAD_CTX_init(ctypes.byref(self.ctx), aead, key, len(key), tag_len, None)
        else:
            ok = _lib.EVP_AEAD_CTX_init_with_direction(ctypes.byref(self.ctx), aead, key,
                                                      len(key), tag_len, direction)
        if not ok:
            _fail("EVP_AEAD_CTX_init")

    @property
    def tag_len(self):
        return self.ctx.tag_len

    def close(self):
        if self.ctx is not None:
            _lib.EVP_AEAD_CTX_cleanup(ctypes.byref(self.ctx))
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass

    # --- single record, host buffers (EVP_AEAD_CTX_seal / _open) ----------
    def seal(self, nonce, pt, ad=b""):
        pt, nonce, ad = bytes(pt), bytes(nonce), bytes(ad)
        max_out = len(pt) + _lib.EVP_AEAD_max_overhead(self.aead)
        out = ctypes.create_string_buffer(max(1, max_out))
        out_len = _S(0)
        if not _lib.EVP_AEAD_CTX_seal(ctypes.byref(self.ctx), out, ctypes.byref(out_len), max_out,
                                      nonce, len(nonce), pt, len(pt), ad, len(ad)):
            _fail("EVP_AEAD_CTX_seal")
        return out.raw[:out_len.value]

    def open(self, nonce, ct_and_tag, ad=b""):
        ct, nonce, ad = bytes(ct_and_tag), bytes(nonce), bytes(ad)
        out = ctypes.create_string_buffer(max(1, len(ct)))
        out_len = _S(0)
        if not _lib.EVP_AEAD_CTX_open(ctypes.byref(self.ctx), out, ctypes.byref(out_len), len(ct),
                                      nonce, len(nonce), ct, len(ct), ad, len(ad)):
            _fail("EVP_AEAD_CTX_open")
        return out.raw[:out_len.value]

    # --- device batches (torch tensors or raw device pointers) ------------
    def seal_batch_device(self, batch, stream=None):
        if not _lib.EVP_AEAD_CTX_seal_batch_device(ctypes.byref(self.ctx), ctypes.byref(batch),
                                                   _stream_ptr(stream)):
            _fail("EVP_AEAD_CTX_seal_batch_device")

    def open_batch_device(self, batch, stream=None):
        if not _lib.EVP_AEAD_CTX_open_batch_device(ctypes.byref(self.ctx), ctypes.byref(batch),
                                                   _stream_ptr(stream)):
            _fail("EVP_AEAD_CTX_open_batch_device")

    def sealv_batch_device(self, batch, stream=None):
        """N sealv calls over device iovec records (BSSL_AMD_IOV_BATCH)."""
        if not _lib.EVP_AEAD_CTX_sealv_batch_device(ctypes.byref(self.ctx), ctypes.byref(batch),
                                                    _stream_ptr(stream)):
            _fail("EVP_AEAD_CTX_sealv_batch_device")

    def openv_detached_batch_device(self, batch, stream=None):
        if not _lib.EVP_AEAD_CTX_openv_detached_batch_device(
                ctypes.byref(self.ctx), ctypes.byref(batch), _stream_ptr(stream)):
            _fail("EVP_AEAD_CTX_openv_detached_batch_device")


class Keyset:
    """BSSL_AMD_KEYSET: many keys of one AEAD resident on the device."""

    def __init__(self, aead, keys, num_keys, tag_len=EVP_AEAD_DEFAULT_TAG_LENGTH):
        if isinstance(aead, str):
            aead = EVP_aead(aead)
        keys = bytes(keys)
        self.h = _lib.BSSL_AMD_KEYSET_new(aead, keys, num_keys, tag_len)
        if not self.h:
            _fail("BSSL_AMD_KEYSET_new")

    def seal_batch_device(self, batch, stream=None):
        if not _lib.BSSL_AMD_KEYSET_seal_batch_device(self.h, ctypes.byref(batch),
                                                      _stream_ptr(stream)):
            _fail("BSSL_AMD_KEYSET_seal_batch_device")

    def open_batch_device(self, batch, stream=None):
        if not _lib.BSSL_AMD_KEYSET_open_batch_device(self.h, ctypes.byref(batch),
                                                      _stream_ptr(stream)):
            _fail("BSSL_AMD_KEYSET_open_batch_device")

    def close(self):
        if self.h:
            _lib.BSSL_AMD_KEYSET_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass


def _stream_ptr(stream):
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _dptr(t):
    return None if t is None else t.data_ptr()


class TlsAead:
    """BSSL_AMD_TLS_AEAD: one direction of a TLS 1.2 / 1.3 connection (the
    reference's SSLAEADContext) sealing / opening device batches of records."""

    def __init__(self, direction, version, aead, key, fixed_iv, seq=0):
        if isinstance(aead, str):
            aead = EVP_aead(aead)
        key, fixed_iv = bytes(key), bytes(fixed_iv)
        self.h = _lib.BSSL_AMD_TLS_AEAD_new(direction, version, aead, key, len(key), fixed_iv,
                                            len(fixed_iv), seq)
        if not self.h:
            _fail("BSSL_AMD_TLS_AEAD_new")

    @property
    def prefix_len(self):
        return _lib.BSSL_AMD_TLS_AEAD_prefix_len(self.h)

    @property
    def suffix_len(self):
        return _lib.BSSL_AMD_TLS_AEAD_suffix_len(self.h)

    @property
    def sequence(self):
        return _lib.BSSL_AMD_TLS_AEAD_sequence(self.h)

    def seal_records_device(self, recs, stream=None):
        if not _lib.BSSL_AMD_TLS_AEAD_seal_records_device(self.h, ctypes.byref(recs),
                                                          _stream_ptr(stream)):
            _fail("BSSL_AMD_TLS_AEAD_seal_records_device")

    def open_records_device(self, recs, stream=None):
        if not _lib.BSSL_AMD_TLS_AEAD_open_records_device(self.h, ctypes.byref(recs),
                                                          _stream_ptr(stream)):
            _fail("BSSL_AMD_TLS_AEAD_open_records_device")

    def close(self):
        if self.h:
            _lib.BSSL_AMD_TLS_AEAD_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover
            pass


def make_tls_records(num_records, inp, out, prefix, suffix, *, offsets=None, lengths=None,
                     record_stride=0, record_len=0, types=None, type_=23, status=None):
    """BSSL_AMD_TLS_RECORDS from torch device tensors (keeps references)."""
    r = BSSL_AMD_TLS_RECORDS()
    r.num_records = num_records
    r.in_, r.out = _dptr(inp), _dptr(out)
    r.offsets, r.lengths = _dptr(offsets), _dptr(lengths)
    r.record_stride, r.record_len = record_stride, record_len
    r.types, r.type = _dptr(types), type_
    r.prefix, r.suffix, r.status = _dptr(prefix), _dptr(suffix), _dptr(status)
    r._refs = (inp, out, offsets, lengths, types, prefix, suffix, status)
    return r


def make_batch(num_records, inp, out, tags, nonces, nonce_len, ad=None, *, offsets=None,
               lengths=None, record_stride=0, record_len=0, ad_offsets=None, ad_lengths=None,
               ad_stride=0, ad_len=0, status=None, key_index=None):
    """Builds a BSSL_AMD_BATCH from torch device tensors (uint8 / int64 /
    int32).  The returned structure keeps references to the tensors."""
    b = BSSL_AMD_BATCH()
    b.num_records = num_records
    b.in_ = _dptr(inp)
    b.out = _dptr(out)
    b.offsets = _dptr(offsets)
    b.lengths = _dptr(lengths)
    b.record_stride = record_stride
    b.record_len = record_len
    b.nonces = _dptr(nonces)
    b.nonce_len = nonce_len
    b.ad = _dptr(ad)
    b.ad_offsets = _dptr(ad_offsets)
    b.ad_lengths = _dptr(ad_lengths)
    b.ad_stride = ad_stride
    b.ad_len = ad_len
    b.tags = _dptr(tags)
    b.status = _dptr(status)
    b.key_index = _dptr(key_index)
    b._refs = (inp, out, tags, nonces, ad, offsets, lengths, ad_offsets, ad_lengths, status,
               key_index)
    return b


def make_iov_batch(num_records, iovecs, iovec_start, tags, nonces, nonce_len, *, aadvecs=None,
                   aadvec_start=None, status=None):
    """Builds a BSSL_AMD_IOV_BATCH.  `iovecs`: device int64 tensor [m, 3] of
    CRYPTO_IOVEC {out, in, len} (device addresses); `aadvecs`: [k, 2] of
    CRYPTO_IVEC {in, len}; `*_start`: device int64 [num_records + 1]."""
    b = BSSL_AMD_IOV_BATCH()
    b.num_records = num_records
    b.iovecs = _dptr(iovecs)
    b.iovec_start = _dptr(iovec_start)
    b.aadvecs = _dptr(aadvecs)
    b.aadvec_start = _dptr(aadvec_start)
    b.nonces = _dptr(nonces)
    b.nonce_len = nonce_len
    b.tags = _dptr(tags)
    b.status = _dptr(status)
    b._refs = (iovecs, iovec_start, aadvecs, aadvec_start, nonces, tags, status)
    return b


def synth_fill_device(first_record, n, offsets, lengths, pt, nonces, ads, stream=None):
    """Device-side synthetic workload (definition: oracle/synth.h)."""
    if not _lib.BSSL_AMD_synth_fill_device(first_record, n, _dptr(offsets), _dptr(lengths),
                                           _dptr(pt), _dptr(nonces), _dptr(ads),
                                           _stream_ptr(stream)):
        raise RuntimeError("BSSL_AMD_synth_fill_device failed")


def set_kernel_timing(enable):
    """Record HIP events around every batch's bulk kernel (see aead.h)."""
    _lib.BSSL_AMD_set_kernel_timing(1 if enable else 0)


def collect_kernel_times(max_n=4096):
    """Durations (ms) of the bulk kernels launched since the last call."""
    buf = (ctypes.c_double * max_n)()
    n = _lib.BSSL_AMD_collect_kernel_times(buf, max_n)
    return [buf[i] for i in range(min(n, max_n))]


AES_GCM_ENGINES = {"table": 0, "bs": 1}
# (2: the experimental mixed engine, selected only by BSSL_AMD_GCM_MODE=mixN)
_ENGINE_NAMES = {0: "table", 1: "bs", 2: "mix"}


def gcm_key_tables(keys, key_len, on_device):
    """The per-key AES-GCM device tables (GcmKeyDev bytes, one entry per key)
    of the concatenated `keys`, from the host key setup (on_device False) or
    the device key-setup kernel (True)."""
    size = lib.BSSL_AMD_gcm_key_tables(None, 0, 0, 0, None)
    n = len(keys) // key_len
    out = ctypes.create_string_buffer(size * n)
    kb = ctypes.create_string_buffer(bytes(keys), max(len(keys), 1))
    if lib.BSSL_AMD_gcm_key_tables(kb, key_len, n, 1 if on_device else 0, out) != n:
        raise RuntimeError("BSSL_AMD_gcm_key_tables failed")
    raw = out.raw
    return [raw[i * size:(i + 1) * size] for i in range(n)]


def set_aes_gcm_engine(engine):
    """Selects the AES-GCM engine ("bs": bitsliced, table-free; "table": LDS
    T-tables) for every later batch of this process; returns the previous one."""
    if engine not in AES_GCM_ENGINES:
        raise ValueError(f"unknown AES-GCM engine {engine!r} (one of {sorted(AES_GCM_ENGINES)})")
    prev = _lib.BSSL_AMD_set_aes_gcm_engine(AES_GCM_ENGINES[engine])
    if prev < 0:
        raise RuntimeError(f"BSSL_AMD_set_aes_gcm_engine refused {engine!r}")
    return _ENGINE_NAMES[prev]


def test_set_bs_ek0_producers(on):
    """Test support (include/bssl_amd/test_hooks.h): with False, the table-free
    engine's launches skip the batched E_K(J0) production, so every record end
    takes the bounded-wait fallback and computes its own E_K(J0).  Returns the
    previous setting."""
    return bool(_lib.BSSL_AMD_test_set_bs_ek0_producers(1 if on else 0))


def test_set_gcm_mix(bitsliced_waves):
    """Test support: selects the experimental mixed-role engine
    (include/bssl_amd/test_hooks.h); returns the previous engine's name."""
    prev = _lib.BSSL_AMD_test_set_gcm_mix(bitsliced_waves)
    if prev < 0:
        raise ValueError(bitsliced_waves)
    return _ENGINE_NAMES[prev]


def aes_gcm_engine():
    return _ENGINE_NAMES[_lib.BSSL_AMD_aes_gcm_engine()]


def last_kernel_name():
    return _lib.BSSL_AMD_last_kernel_name().decode()


def set_device(dev):
    if not _lib.BSSL_AMD_set_device(dev):
        raise RuntimeError(f"BSSL_AMD_set_device({dev}) failed")


def device_count():
    return _lib.BSSL_AMD_device_count()
