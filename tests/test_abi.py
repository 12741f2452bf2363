"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
symbol include/bssl_amd/aead.h declares, and the host-side (no-GPU) parts of
the EVP_AEAD surface behave like the reference (aead.cc.inc:82-106 key-length
check, e_aes.cc.inc:742-749 tag length, err.h packing, aead.h:204-217 sizes)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "bssl_amd", h) for h in ("aead.h", "tls.h", "test_hooks.h")]


def header_functions():
    text = "\n".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = "\n".join(l for l in text.splitlines() if not l.lstrip().startswith("#"))
    names = re.findall(r"BSSL_AMD_EXPORT[^;(]*?\b(\w+)\s*\(", text, flags=re.S)
    return sorted(set(names))


def test_header_declares_expected_surface():
    names = header_functions()
    for must in ("EVP_AEAD_CTX_seal", "EVP_AEAD_CTX_open", "EVP_AEAD_CTX_seal_scatter",
                 "EVP_AEAD_CTX_sealv", "EVP_AEAD_CTX_openv_detached",
                 "EVP_AEAD_CTX_seal_batch_device", "BSSL_AMD_KEYSET_seal_batch_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import boringssl_amd as ba
    names = header_functions()
    assert sorted(ba.EXPORTED_SYMBOLS) == names
    out = subprocess.check_output(["nm", "-D", "--defined-only", ba.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    # nothing else leaks out of the library except the declared ABI
    extra = sorted(n for n in exported if not n.startswith("_") and n not in names)
    assert not extra, extra


def test_aead_parameters():
    import boringssl_amd as ba
    L = ba.lib
    for name, key_len, nonce_len in [
            ("aes-128-gcm", 16, 12), ("aes-192-gcm", 24, 12), ("aes-256-gcm", 32, 12),
            ("chacha20-poly1305", 32, 12), ("aes-128-gcm-tls13", 16, 12),
            ("xchacha20-poly1305", 32, 24),  # e_chacha20poly1305.cc:385-399
            ("aes-128-gcm-siv", 16, 12), ("aes-256-gcm-siv", 32, 12)]:  # e_aesgcmsiv.cc:869-899
        a = ba.EVP_aead(name)
        assert L.EVP_AEAD_key_length(a) == key_len
        assert L.EVP_AEAD_nonce_length(a) == nonce_len
        assert L.EVP_AEAD_max_overhead(a) == 16
        assert L.EVP_AEAD_max_tag_len(a) == 16


def test_init_rejects_bad_key_and_tag_length_without_gpu():
    import boringssl_amd as ba
    with pytest.raises(ba.AEADError) as e:
        ba.AEADCtx("aes-128-gcm", bytes(15))
    assert e.value.lib == ba.ERR_LIB_CIPHER and e.value.reason == ba.CIPHER_R_UNSUPPORTED_KEY_SIZE
    with pytest.raises(ba.AEADError) as e:
        ba.AEADCtx("aes-256-gcm", bytes(32), tag_len=17)
    assert e.value.reason == ba.CIPHER_R_TAG_TOO_LARGE
    with pytest.raises(ba.AEADError) as e:
        ba.AEADCtx("chacha20-poly1305", bytes(32), tag_len=17)
    assert e.value.reason == ba.CIPHER_R_TOO_LARGE
    # GCM-SIV takes 16-byte tags only (e_aesgcmsiv.cc:542-548)
    with pytest.raises(ba.AEADError) as e:
        ba.AEADCtx("aes-128-gcm-siv", bytes(16), tag_len=12)
    assert e.value.reason == ba.CIPHER_R_TAG_TOO_LARGE
    with pytest.raises(ba.AEADError) as e:
        ba.AEADCtx("xchacha20-poly1305", bytes(16))
    assert e.value.reason == ba.CIPHER_R_UNSUPPORTED_KEY_SIZE
    assert ba.lib.ERR_get_error() == 0


def test_struct_layouts_match_the_header(tmp_path):
    """The ctypes mirror's structures have the C header's sizes and field
    offsets (a C probe compiled against include/bssl_amd/*.h)."""
    import boringssl_amd as ba
    structs = {
        "EVP_AEAD_CTX": (ba.EVP_AEAD_CTX, {"aead": "aead", "state": "state", "tag_len": "tag_len"}),
        "CRYPTO_IOVEC": (ba.CRYPTO_IOVEC, {"out": "out", "in": "in_", "len": "len"}),
        "CRYPTO_IVEC": (ba.CRYPTO_IVEC, {"in": "in_", "len": "len"}),
        "BSSL_AMD_BATCH": (ba.BSSL_AMD_BATCH, {f: f for f in (
            "num_records", "out", "offsets", "lengths", "record_stride", "record_len", "nonces",
            "nonce_len", "ad", "ad_offsets", "ad_lengths", "ad_stride", "ad_len", "tags",
            "status", "key_index")} | {"in": "in_"}),
        "BSSL_AMD_IOV_BATCH": (ba.BSSL_AMD_IOV_BATCH, {f: f for f in (
            "num_records", "iovecs", "iovec_start", "aadvecs", "aadvec_start", "nonces",
            "nonce_len", "tags", "status")}),
    }
    lines = ["#include <stdio.h>", "#include <stddef.h>", "#include <bssl_amd/aead.h>",
             "int main(void) {"]
    for cname, (_, fields) in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for cf in fields:
            lines.append(f'  printf("{cname} {cf} %zu\\n", offsetof({cname}, {cf}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src),
                           "-o", str(exe)])
    got = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        name, key, val = line.split()
        got[(name, key)] = int(val)
    for cname, (cls, fields) in structs.items():
        assert ctypes.sizeof(cls) == got[(cname, "size")], cname
        for cf, pf in fields.items():
            assert getattr(cls, pf).offset == got[(cname, cf)], (cname, cf)


def test_error_queue_is_bounded_fifo():
    import boringssl_amd as ba
    L = ba.lib
    L.ERR_clear_error()
    ctx = ba.EVP_AEAD_CTX()
    for _ in range(20):
        assert not L.EVP_AEAD_CTX_init(ctypes.byref(ctx), ba.EVP_aead("aes-128-gcm"), bytes(3), 3,
                                       0, None)
    n = 0
    while True:
        e = L.ERR_get_error()
        if not e:
            break
        assert (e >> 24) == 30 and (e & 0xfff) == ba.CIPHER_R_UNSUPPORTED_KEY_SIZE
        n += 1
    assert n == 15  # ERR_NUM_ERRORS - 1 entries retained, as the reference queue


def test_zeroed_ctx_cleanup_is_safe():
    import boringssl_amd as ba
    ctx = ba.EVP_AEAD_CTX()
    ba.lib.EVP_AEAD_CTX_zero(ctypes.byref(ctx))
    ba.lib.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))
    ba.lib.EVP_AEAD_CTX_cleanup(ctypes.byref(ctx))


def test_plain_c_caller_compiles_and_links(tmp_path):
    """A C program written against the reference API links to the library."""
    import boringssl_amd as ba
    exe = tmp_path / "seal_one"
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "examples", "seal_one.c"),
                           "-L", os.path.dirname(ba.LIB_PATH), "-lbssl_amd",
                           f"-Wl,-rpath,{os.path.dirname(ba.LIB_PATH)}", "-o", str(exe)])
    assert exe.exists()
