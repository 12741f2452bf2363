"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the checker for the HIP path; the
product package (boringssl_amd) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

AES_GCM = 0
CHACHA20_POLY1305 = 1
XCHACHA20_POLY1305 = 2
AES_GCM_SIV = 3

_P = ctypes.c_void_p
_S = ctypes.c_size_t


def _load():
    if not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(_LIB_PATH)
    sig = {
        "oracle_aes_encrypt_block": (None, [_P, _S, _P, _P]),
        "oracle_gf128_mul": (None, [_P, _P]),
        "oracle_aes_gcm_seal": (ctypes.c_int, [_P, _S, _P, _S, _P, _S, _P, _S, _P, _P, _S]),
        "oracle_aes_gcm_open": (ctypes.c_int, [_P, _S, _P, _S, _P, _S, _P, _S, _P, _S, _P]),
        "oracle_chacha20": (None, [_P, _P, _S, _P, _P, ctypes.c_uint32]),
        "oracle_poly1305": (None, [_P, _P, _S, _P]),
        "oracle_chacha20_poly1305_seal": (ctypes.c_int, [_P, _P, _S, _P, _S, _P, _S, _P, _P, _S]),
        "oracle_chacha20_poly1305_open": (ctypes.c_int, [_P, _P, _S, _P, _S, _P, _S, _P, _S, _P]),
        "oracle_hchacha20": (None, [_P, _P, _P]),
        "oracle_aes_gcm_siv_seal": (ctypes.c_int, [_P, _S, _P, _S, _P, _S, _P, _S, _P, _P, _S]),
        "oracle_aes_gcm_siv_open": (ctypes.c_int, [_P, _S, _P, _S, _P, _S, _P, _S, _P, _S, _P]),
        "oracle_xchacha20_poly1305_seal": (ctypes.c_int, [_P, _P, _S, _P, _S, _P, _S, _P, _P, _S]),
        "oracle_xchacha20_poly1305_open": (ctypes.c_int, [_P, _P, _S, _P, _S, _P, _S, _P, _S, _P]),
        "oracle_batch": (_S, [ctypes.c_int, ctypes.c_int, _P, _S, _P, _S, _P, _P, _P, _P, _P, _S,
                              _P, _P, _P, _P, _S, _P, ctypes.c_int]),
        "synth_key": (None, [ctypes.c_uint64, _S, _P]),
        "synth_nonce": (None, [ctypes.c_uint64, _P]),
        "synth_ad": (None, [ctypes.c_uint64, ctypes.c_uint64, _P]),
        "synth_pt": (None, [ctypes.c_uint64, ctypes.c_uint64, _P]),
        "synth_mixed_len": (ctypes.c_uint64, [ctypes.c_uint64]),
        "synth_fill": (None, [ctypes.c_uint64, _S, _P, _P, _P, _P, _P, ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _buf(b):
    if b is None:
        return None
    if isinstance(b, (bytes, bytearray)):
        return ctypes.c_char_p(bytes(b)) if isinstance(b, bytes) else (ctypes.c_char * len(b)).from_buffer(b)
    return b


def aes_block(key, block):
    out = ctypes.create_string_buffer(16)
    lib().oracle_aes_encrypt_block(bytes(key), len(key), bytes(block), out)
    return out.raw


def gf128_mul(x, h):
    xb = ctypes.create_string_buffer(bytes(x), 16)
    lib().oracle_gf128_mul(xb, bytes(h))
    return xb.raw[:16]


def seal(aead, key, nonce, pt, ad, tag_len=16):
    """Returns (ok, ct, tag)."""
    out = ctypes.create_string_buffer(max(1, len(pt)))
    tag = ctypes.create_string_buffer(16)
    if aead == AES_GCM:
        ok = lib().oracle_aes_gcm_seal(bytes(key), len(key), bytes(nonce), len(nonce), bytes(pt),
                                       len(pt), bytes(ad), len(ad), out, tag, tag_len)
    elif aead == AES_GCM_SIV:
        ok = lib().oracle_aes_gcm_siv_seal(bytes(key), len(key), bytes(nonce), len(nonce),
                                           bytes(pt), len(pt), bytes(ad), len(ad), out, tag,
                                           tag_len)
    elif aead == XCHACHA20_POLY1305:
        ok = lib().oracle_xchacha20_poly1305_seal(bytes(key), bytes(nonce), len(nonce), bytes(pt),
                                                  len(pt), bytes(ad), len(ad), out, tag, tag_len)
    else:
        ok = lib().oracle_chacha20_poly1305_seal(bytes(key), bytes(nonce), len(nonce), bytes(pt),
                                                 len(pt), bytes(ad), len(ad), out, tag, tag_len)
    return bool(ok), out.raw[:len(pt)], tag.raw[:tag_len]


def open_(aead, key, nonce, ct, ad, tag):
    """Returns (ok, pt)."""
    out = ctypes.create_string_buffer(max(1, len(ct)))
    if aead == AES_GCM:
        ok = lib().oracle_aes_gcm_open(bytes(key), len(key), bytes(nonce), len(nonce), bytes(ct),
                                       len(ct), bytes(ad), len(ad), bytes(tag), len(tag), out)
    elif aead == AES_GCM_SIV:
        ok = lib().oracle_aes_gcm_siv_open(bytes(key), len(key), bytes(nonce), len(nonce),
                                           bytes(ct), len(ct), bytes(ad), len(ad), bytes(tag),
                                           len(tag), out)
    elif aead == XCHACHA20_POLY1305:
        ok = lib().oracle_xchacha20_poly1305_open(bytes(key), bytes(nonce), len(nonce), bytes(ct),
                                                  len(ct), bytes(ad), len(ad), bytes(tag), len(tag),
                                                  out)
    else:
        ok = lib().oracle_chacha20_poly1305_open(bytes(key), bytes(nonce), len(nonce), bytes(ct),
                                                 len(ct), bytes(ad), len(ad), bytes(tag), len(tag), out)
    return bool(ok), out.raw[:len(ct)]


def chacha20(key, nonce, counter, data):
    out = ctypes.create_string_buffer(max(1, len(data)))
    lib().oracle_chacha20(out, bytes(data), len(data), bytes(key), bytes(nonce), counter)
    return out.raw[:len(data)]


def hchacha20(key, nonce16):
    out = ctypes.create_string_buffer(32)
    lib().oracle_hchacha20(out, bytes(key), bytes(nonce16))
    return out.raw


def poly1305(key, msg):
    tag = ctypes.create_string_buffer(16)
    lib().oracle_poly1305(tag, bytes(msg), len(msg), bytes(key))
    return tag.raw


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def batch(aead, seal_, keys, key_len, key_index, inp, out, offsets, lens, nonces, nonce_len,
          ad, ad_offsets, ad_lens, tags, tag_len, status=None, threads=8):
    """numpy-array batch front end; returns number of failed records."""
    n = len(lens)
    return lib().oracle_batch(aead, int(seal_), _ptr(keys), key_len, _ptr(key_index), n,
                              _ptr(inp), _ptr(out), _ptr(offsets), _ptr(lens), _ptr(nonces),
                              nonce_len, _ptr(ad), _ptr(ad_offsets), _ptr(ad_lens), _ptr(tags),
                              tag_len, _ptr(status), threads)


def synth_key(k, key_len):
    out = ctypes.create_string_buffer(key_len)
    lib().synth_key(k, key_len, out)
    return out.raw


def synth_keys(nkeys, key_len, first=0):
    arr = np.zeros(nkeys * key_len, dtype=np.uint8)
    for k in range(nkeys):
        lib().synth_key(first + k, key_len, arr[k * key_len:].ctypes.data_as(ctypes.c_void_p))
    return arr


def synth_mixed_len(i):
    return lib().synth_mixed_len(i)


def synth_batch(first, lens, align=16, threads=8):
    """Returns (pt, offsets, nonces, ads) numpy arrays for records first..first+n-1."""
    lens = np.asarray(lens, dtype=np.uint64)
    padded = (lens + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offsets = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offsets[1:] = np.cumsum(padded[:-1])
    total = int(padded.sum()) if len(lens) else 0
    pt = np.zeros(max(total, 1), dtype=np.uint8)
    nonces = np.zeros(12 * len(lens), dtype=np.uint8)
    ads = np.zeros(13 * len(lens), dtype=np.uint8)
    lib().synth_fill(first, len(lens), _ptr(offsets), _ptr(lens), _ptr(pt), _ptr(nonces),
                     _ptr(ads), threads)
    return pt, offsets, nonces, ads


def xchacha_nonces(nonces12):
    """24-byte synthetic nonces (ref_tool.cc make_nonce): synth_nonce(i) then
    synth_nonce(i) with bytes 4..11 XOR 0xff (= synth_nonce(~i))."""
    a = np.asarray(nonces12, dtype=np.uint8).reshape(-1, 12)
    b = a.copy()
    b[:, 4:] ^= 0xff
    return np.ascontiguousarray(np.concatenate([a, b], axis=1)).reshape(-1)
